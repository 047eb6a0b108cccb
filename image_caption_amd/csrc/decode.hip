// Fused decode-step kernels for the KV-cached decoder loop (one new token per sequence).
//
// The decode step of torch's post-LN TransformerDecoderLayer (transformer.py:1144-1153) is a chain of
// small dependent products at M = batch rows; as separate launches every product pays a launch plus a
// memory round trip (profiles/r02: QKV GEMM 9.7 us, self-attention 5.8, out-projection 4.8, FFN-1 10.4,
// FFN-2 10.3 at 256 rows).  These kernels fuse what is row-local:
//
//   dec_sa_kernel   block = (16 rows, head h):  q|k|v_h = a Wqkv_h^T + b   (12 column tiles, K = 512)
//                   -> append k, v to the fp32 KV cache at position t0 -> causal attention over the
//                   t0 + 1 cached keys (one wave per row) -> slab h = ctx_h Wo[:, 64h:64h+64]^T
//                   (the out-projection as a split-K over heads; residual_layernorm sums the 8 slabs
//                   with the bias and the residual: x = LN1(x + SA(x)))
//   dec_ffn_kernel  block = (16 rows, hidden slice j of 128): h_j = relu(a W1_j^T + b1_j), then
//                   slab j = h_j W2[:, 128j:128j+128]^T (split-K over the 16 slices of dim_ff = 2048)
//
// Every weight fragment a wave multiplies is loaded straight into its VGPRs at kernel start (one
// global_load_dwordx4 per fragment, all in flight at once; no LDS ring, no barrier in the k-loop);
// the activation rows (a bf16 planes, 16 rows x 512) are DMA'd to LDS once and shared.  So a launch
// is one memory round trip plus the MFMA chain.  Block order puts the 16 row tiles of one head (SA)
// or of one slice pair (FFN) on one XCD (blocks b, b + 8, ... share an XCD under round-robin dispatch),
// so each XCD's L2 serves that weight slice to all of them (speed only; correctness does not depend
// on placement).
//
// MFMA convention (as gemm_dec_kernel): D = W . X^T with W as the A operand, so lane l holds output
// row m = l & 15 and the four consecutive output columns n = 4 (l >> 4) + r -> 16-byte stores.
// LDS image of X per 32-deep k-step and plane: 16 rows x 64 B, 16-byte chunk c of row r at
// c ^ ((r >> 2) & 3) (conflict-free fragment reads).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int DEC_D = 512, DEC_H = 8, DEC_HD = 64, DEC_F = 2048;
constexpr int DEC_ROWS = 16;    // rows per block
constexpr int DEC_KS = DEC_D / 32;  // k-steps of the D-wide products

// X (16 rows x 512, ns planes at plane stride aL) -> LDS [ks][plane][16 rows][64 B], by all 16 waves
__device__ __forceinline__ void stage_rows(const bf16_t* A, long aL, int ns, int row0, int rows, char* sx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lrow = lane >> 2, lchunk = (lane & 3) ^ ((lrow >> 2) & 3);
  const int r = min(row0 + lrow, rows - 1);
  for (int q = wave; q < DEC_KS * ns; q += 16) {
    const int ks = q / ns, pl = q - ks * ns;
    const bf16_t* src = A + pl * aL + (long)r * DEC_D + ks * 32 + lchunk * 8;
    __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src, (LDS_AS void*)(sx + q * 1024), 16, 0, 0);
  }
}

// B-operand fragment (row m = l & 15, 8 k values of chunk l >> 4) of k-step ks, plane pl
__device__ __forceinline__ bf16x8 x_frag(const char* sx, int ns, int ks, int pl) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  return *(const bf16x8*)(sx + (ks * ns + pl) * 1024 + fr * 64 + ((fq ^ ((fr >> 2) & 3)) << 4));
}

// write v (this lane's 4 consecutive columns n0..n0+3 of row m) as bf16 planes into an LDS operand
// image with k = column: [ks][plane][16 rows][64 B] (same layout as x_frag reads)
__device__ __forceinline__ void put_planes(char* img, int ns, int m, int n0, f32x4 v) {
  bf16_t h[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) split_bf(v[r], h[r], l[r]);
  const int ks = n0 >> 5, c = (n0 & 31) >> 3;
  char* dst = img + ks * ns * 1024 + m * 64 + ((c ^ ((m >> 2) & 3)) << 4) + (n0 & 7) * 2;
  *(u32x2*)dst = (u32x2){(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
  if (ns == 2)
    *(u32x2*)(dst + 1024) = (u32x2){(uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16)};
}

// ------------------------------------------------------------------------------------------------
// Self-attention block of one decode step.  LDS: X image 32 KiB (reused for the q|k|v rows after
// the projection), ctx image 4 KiB.
__global__ __launch_bounds__(1024) void dec_sa_kernel(DecSaArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sx = smem;                                  // X image, then qkv fp32 [16][192]
  float* qkv = (float*)smem;
  char* sc = smem + DEC_KS * 2 * 1024;              // ctx image [2 ks][ns][16][64 B]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int h = blockIdx.x & (DEC_H - 1), row0 = (blockIdx.x >> 3) * DEC_ROWS;
  const int ns = p.nsplit;

  stage_rows(p.A, p.aL, ns, row0, p.rows, sx);
  // weight fragments: waves 0..11 -> q|k|v column tile (wave >> 2) x 16 + ..., all 16 k-steps
  bf16x8 wf[DEC_KS];
  if (wave < 12) {
    const int which = wave >> 2;  // 0 q, 1 k, 2 v
    const bf16_t* wr = p.Wqkv + (long)(which * DEC_D + h * DEC_HD + (wave & 3) * 16 + fr) * DEC_D + fq * 8;
#pragma unroll
    for (int ks = 0; ks < DEC_KS; ++ks) wf[ks] = *(const bf16x8*)(wr + ks * 32);
  }
  // out-projection fragments: output columns 32 wave + 16 i + (lane & 15), k = this head's 64
  bf16x8 of[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      of[i][ks] = *(const bf16x8*)(p.Wo + (long)(wave * 32 + i * 16 + fr) * DEC_D + h * DEC_HD + ks * 32 + fq * 8);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- q | k | v projection (16 rows x 192 columns of head h)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (wave < 12) {
#pragma unroll
    for (int ks = 0; ks < DEC_KS; ++ks) {
      acc = mfma16(wf[ks], x_frag(sx, ns, ks, 0), acc);
      if (ns == 2) acc = mfma16(wf[ks], x_frag(sx, ns, ks, 1), acc);
    }
    const int which = wave >> 2, n = (wave & 3) * 16 + 4 * fq;
    acc += *(const f32x4*)(p.bqkv + which * DEC_D + h * DEC_HD + n);
  }
  __syncthreads();  // X image no longer read: it becomes the q|k|v rows
  if (wave < 12) *(f32x4*)(qkv + fr * 192 + wave * 16 + 4 * fq) = acc;
  __syncthreads();

  // ---- attention, one wave per row (torch's causal SDPA of the new position over positions 0..t0)
  {
    const int r = wave, b = row0 + r;
    const int t0 = p.t0, nkeys = t0 + 1;
    const float* qr = qkv + r * 192;
    float ctx = 0.f, l = 1.f;
    if (b < p.rows) {
      const long cache = ((long)b * DEC_H + h) * p.Lmax * DEC_HD;
      p.kc[cache + (long)t0 * DEC_HD + lane] = qr[64 + lane];   // this step's key / value
      p.vc[cache + (long)t0 * DEC_HD + lane] = qr[128 + lane];
      float s = -INFINITY;
      if (lane < nkeys) {
        const float* kr;
        if (lane == t0) kr = qr + 64;
        else if (p.anc) kr = p.kc + ((long)p.anc[(long)b * p.Lmax + lane] * DEC_H + h) * p.Lmax * DEC_HD + (long)lane * DEC_HD;
        else kr = p.kc + cache + (long)lane * DEC_HD;
        float a = 0.f;
#pragma unroll
        for (int d = 0; d < DEC_HD; d += 4) {
          const f32x4 kv = *(const f32x4*)(kr + d);
          a = fmaf(qr[d], kv[0], a);
          a = fmaf(qr[d + 1], kv[1], a);
          a = fmaf(qr[d + 2], kv[2], a);
          a = fmaf(qr[d + 3], kv[3], a);
        }
        s = a * p.scale;
      }
      const float m = wave_max(s);
      const float e = lane < nkeys ? __expf(s - m) : 0.f;
      l = wave_sum(e);
      // context (lane = d): sum_j p_j v_j[d] (p_j from lane j); v of position t0 from LDS, older from the cache
      for (int j = 0; j < nkeys; ++j) {
        float v;
        if (j == t0) v = qr[128 + lane];
        else if (p.anc) v = p.vc[((long)p.anc[(long)b * p.Lmax + j] * DEC_H + h) * p.Lmax * DEC_HD + (long)j * DEC_HD + lane];
        else v = p.vc[cache + (long)j * DEC_HD + lane];
        ctx = fmaf(__shfl(e, j, 64), v, ctx);
      }
      ctx /= l;
    }
    // ctx row r (lane = d) -> operand image (k = d); lanes 4g..4g+3 gather 4 consecutive d
    f32x4 c4;
#pragma unroll
    for (int i = 0; i < 4; ++i) c4[i] = __shfl(ctx, (lane & ~3) + i, 64);
    if ((lane & 3) == 0) put_planes(sc, ns, r, lane, c4);
  }
  __syncthreads();

  // ---- out-projection slab of head h: 16 rows x 512 columns, K = 64
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      o = mfma16(of[i][ks], x_frag(sc, ns, ks, 0), o);
      if (ns == 2) o = mfma16(of[i][ks], x_frag(sc, ns, ks, 1), o);
    }
    const int row = row0 + fr;
    if (row < p.rows)
      *(f32x4*)(p.part + (long)h * p.part_stride + (long)row * DEC_D + wave * 32 + i * 16 + 4 * fq) = o;
  }
}

// ------------------------------------------------------------------------------------------------
// Feed-forward block of one decode step.  LDS: X image 32 KiB, k-half reduction 8 KiB, h image 8 KiB.
__global__ __launch_bounds__(1024) void dec_ffn_kernel(DecFfnArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sx = smem;
  f32x4* red = (f32x4*)(smem + DEC_KS * 2 * 1024);   // [8 tiles][64 lanes]
  char* sh = (char*)(red + 8 * 64);                  // h image [4 ks][ns][16][64 B]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int nslice = DEC_F / 128;
  const int j = blockIdx.x % nslice, row0 = (blockIdx.x / nslice) * DEC_ROWS;
  const int ns = p.nsplit;

  stage_rows(p.A, p.aL, ns, row0, p.rows, sx);
  // FFN-1 fragments: tile t = wave & 7 (hidden units 128 j + 16 t ..), k-half kh = wave >> 3
  const int t = wave & 7, kh = wave >> 3;
  bf16x8 w1[8];
  {
    const bf16_t* wr = p.W1 + (long)(j * 128 + t * 16 + fr) * DEC_D + kh * 256 + fq * 8;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) w1[ks] = *(const bf16x8*)(wr + ks * 32);
  }
  // FFN-2 fragments: output columns 32 wave + 16 i + (lane & 15), k = hidden units of slice j
  bf16x8 w2[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      w2[i][ks] = *(const bf16x8*)(p.W2 + (long)(wave * 32 + i * 16 + fr) * DEC_F + j * 128 + ks * 32 + fq * 8);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    acc = mfma16(w1[ks], x_frag(sx, ns, kh * 8 + ks, 0), acc);
    if (ns == 2) acc = mfma16(w1[ks], x_frag(sx, ns, kh * 8 + ks, 1), acc);
  }
  if (kh) red[t * 64 + lane] = acc;
  __syncthreads();
  if (!kh) {
    acc += red[t * 64 + lane];
    const int n = t * 16 + 4 * fq;
    acc += *(const f32x4*)(p.b1 + j * 128 + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = fmaxf(acc[r], 0.f);
    put_planes(sh, ns, fr, n, acc);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      o = mfma16(w2[i][ks], x_frag(sh, ns, ks, 0), o);
      if (ns == 2) o = mfma16(w2[i][ks], x_frag(sh, ns, ks, 1), o);
    }
    const int row = row0 + fr;
    if (row < p.rows)
      *(f32x4*)(p.part + (long)j * p.part_stride + (long)row * DEC_D + wave * 32 + i * 16 + 4 * fq) = o;
  }
}

}  // namespace

hipError_t launch_dec_sa(const DecSaArgs& a, hipStream_t s) {
  if (a.rows <= 0 || a.t0 < 0 || a.t0 >= a.Lmax || a.t0 >= 64 || (a.nsplit != 1 && a.nsplit != 2))
    return hipErrorInvalidValue;
  const int lds = DEC_KS * 2 * 1024 + 2 * 2 * 1024;
  const int blocks = (a.rows + DEC_ROWS - 1) / DEC_ROWS * DEC_H;
  hipLaunchKernelGGL(dec_sa_kernel, dim3(blocks), dim3(1024), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_dec_ffn(const DecFfnArgs& a, hipStream_t s) {
  if (a.rows <= 0 || (a.nsplit != 1 && a.nsplit != 2)) return hipErrorInvalidValue;
  const int lds = DEC_KS * 2 * 1024 + 8 * 64 * 16 + 4 * 2 * 1024;
  const int blocks = (a.rows + DEC_ROWS - 1) / DEC_ROWS * (DEC_F / 128);
  hipLaunchKernelGGL(dec_ffn_kernel, dim3(blocks), dim3(1024), lds, s, a);
  return hipGetLastError();
}
