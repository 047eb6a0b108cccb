// Fused decode-step kernels for the KV-cached decoder loop (one new token per sequence).
//
// The decode step of torch's post-LN TransformerDecoderLayer (transformer.py:1144-1153) is a chain of
// small dependent products at M = batch rows; as separate launches every product pays a launch plus a
// memory round trip (profiles/r02: QKV GEMM 9.7 us, self-attention 5.8, out-projection 4.8, FFN-1 10.4,
// FFN-2 10.3 at 256 rows).  These kernels fuse what is row-local:
//
//   dec_sa_kernel   block = (16 rows, head h):  q|k|v_h = a Wqkv_h^T + b   (K = 512)
//                   -> append k, v to the fp32 KV cache at position t0 -> causal attention over the
//                   t0 + 1 cached keys (one wave per row) -> slab h = ctx_h Wo[:, 64h:64h+64]^T
//                   (the out-projection as a split-K over heads; residual_layernorm sums the 8 slabs
//                   with the bias and the residual: x = LN1(x + SA(x)))
//   dec_ffn_kernel  block = (16 rows, hidden slice j of 128): h_j = relu(a W1_j^T + b1_j), then
//                   slab j = h_j W2[:, 128j:128j+128]^T (split-K over the 16 slices of dim_ff = 2048)
//
// Staging (tools/probe_ingest.hip, profiles/r02/probe_ingest.txt): with every CU loading at once, load
// instructions that each cover 16 rows x 64 B (the MFMA fragment shape) move 8 TB/s chip-wide, ones that
// cover whole 128-B lines 18-19 TB/s.  So every operand is LDS-DMA'd in 64-deep k-steps as 128-B row
// images (one instruction = 8 rows x 128 B; 16-byte chunk c of row r stored at c ^ ((r >> 1) & 7), the
// conflict-free swizzle of the int8 encoder GEMM) and fragments are read from LDS.  A block does two DMA
// rounds (the weights of a head / slice do not fit 160 KiB next to the activation rows at once).
// Block order puts the 16 row tiles of one head (SA) or slice pair (FFN) on one XCD (blocks b, b + 8,
// ... share an XCD under round-robin dispatch) so its L2 serves that slice (speed only).
//
// MFMA convention (as gemm_dec_kernel): D = W . X^T with W as the A operand, so lane l holds output
// row m = l & 15 and the four consecutive output columns n = 4 (l >> 4) + r -> 16-byte stores.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int DEC_D = 512, DEC_H = 8, DEC_HD = 64, DEC_F = 2048;
constexpr int DEC_ROWS = 16;           // rows per block
#ifdef ICAP_TOOLS
constexpr bool DEC_XCD_TILES = true;  // the XCD-aligned tile mapping (ICAP_DEC_XCD, measured neutral: tools build only;
#else                                 // its runtime test delayed every block's first loads behind a kernarg wait)
constexpr bool DEC_XCD_TILES = false;
#endif
constexpr int DEC_K64 = DEC_D / 64;    // 64-deep k-steps of the D-wide products
constexpr int DEC_LDS = 160 * 1024;    // both kernels: 128 KiB weight region + 32 KiB row region

// One DMA instruction: rows 8i .. 8i + 7 x 128 B of src (row stride ld bytes) into the LDS image
// dst[rows][128 B] (chunk swizzle c ^ ((r >> 1) & 7)).
__device__ __forceinline__ void dma_8rows(const char* src, long ld, int i, char* dst) {
  const int lane = threadIdx.x & 63;
  const int r = i * 8 + (lane >> 3), pos = lane & 7;
  const char* s = src + (long)r * ld + ((pos ^ ((r >> 1) & 7)) << 4);
  lds_dma16(s, (LDS_AS void*)(dst + i * 1024));
}
// nrows x 128 B, instructions spread over the 16 waves starting at wave `first` (balance across calls)
__device__ __forceinline__ void dma_rows(const char* src, long ld, int nrows, char* dst, int first = 0) {
  const int wave = threadIdx.x >> 6;
  for (int i = (wave - first) & 15; i < nrows / 8; i += 16) dma_8rows(src, ld, i, dst);
}

// MFMA operand fragment of a 128-B-row image: rows r0 + (l & 15), 32-deep half hf of the 64-deep step
__device__ __forceinline__ bf16x8 frag(const char* img, int r0, int hf) {
  const int lane = threadIdx.x & 63, r = r0 + (lane & 15), c = hf * 4 + (lane >> 4);
  return *(const bf16x8*)(img + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
}

// The a rows (16 x 512, row stride ld elements, ns planes at plane stride aL) -> X image [8 k64][ns][16][128 B]
__device__ __forceinline__ void dma_x(const bf16_t* A, long aL, int ns, int row0, int rows, char* sx,
                                      long ld = DEC_D) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane >> 3, pos = lane & 7;
  for (int i = wave; i < DEC_K64 * ns * 2; i += 16) {  // 2 instructions (16 rows) per (k64, plane)
    const int kp = i >> 1, half = i & 1, k64 = kp / ns, pl = kp - k64 * ns;
    const int r = half * 8 + lr, gr = min(row0 + r, rows - 1);
    const char* s = (const char*)(A + pl * aL + (long)gr * ld + k64 * 64) + ((pos ^ ((r >> 1) & 7)) << 4);
    lds_dma16(s, (LDS_AS void*)(sx + kp * 2048 + half * 1024));
  }
}

// write v (this lane's 4 consecutive columns n0..n0+3 of row m) as bf16 planes into a 128-B-row operand
// image with k = column: [k64][ns][16 rows][128 B]
__device__ __forceinline__ void put_planes(char* img, int ns, int m, int n0, f32x4 v) {
  bf16_t h[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) split_bf(v[r], h[r], l[r]);
  const int k64 = n0 >> 6, c = (n0 & 63) >> 3;
  char* dst = img + k64 * ns * 2048 + m * 128 + ((c ^ ((m >> 1) & 7)) << 4) + (n0 & 7) * 2;
  *(u32x2*)dst = (u32x2){(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
  if (ns == 2)
    *(u32x2*)(dst + 2048) = (u32x2){(uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16)};
}

// acc += W-image tile (rows w0.., k64 range) x X-image (16 rows), both planes of X
__device__ __forceinline__ f32x4 mma_rows(f32x4 acc, const char* wimg, int wrows, int w0, const char* ximg, int ns,
                                          int k0, int k1) {
#pragma unroll 2
  for (int k = k0; k < k1; ++k) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const bf16x8 b = frag(wimg + k * wrows * 128, w0, hf);
      acc = mfma16(b, frag(ximg + k * ns * 2048, 0, hf), acc);
      if (ns == 2) acc = mfma16(b, frag(ximg + k * ns * 2048 + 2048, 0, hf), acc);
    }
  }
  return acc;
}

// acc += register-held W fragments (frag_pack image, fragment 2 k + hf of k64-step k) x X-image (16 rows) over NK
// k64-steps of ximg; the same MFMA order as mma_rows (bit-identical sums)
// The X fragments of half-step j + 1 are read before the MFMAs of half-step j (with ns a compile-time constant in the
// kernels' NSC forms), so each MFMA pair waits for reads issued one pair earlier instead of its own.
// Hi/lo decoder weights (round 5): lo(j) is fragment j of the W_lo image and acc also takes W_lo . X_hi
// (every operand of the product then carries 16 significand bits); the lo fragment is fetched one pair ahead with X.
struct NoLo {
  __device__ __forceinline__ bf16x8 operator()(int) const { return bf16x8{}; }
};
template <int NK, class LoF = NoLo>
__device__ __forceinline__ f32x4 mma_frag(f32x4 acc, const bf16x8* wf, const char* ximg, int ns, LoF lo = LoF{}) {
  constexpr bool LO = !__is_same(LoF, NoLo);
  auto xf = [&](int j, int pl) { return frag(ximg + (j >> 1) * ns * 2048 + pl * 2048, 0, j & 1); };
  bf16x8 xh = xf(0, 0), xl = ns == 2 ? xf(0, 1) : xh, wl = LO ? lo(0) : xh;
#pragma unroll
  for (int j = 0; j < 2 * NK; ++j) {
    bf16x8 nh = xh, nl = xl, nw = wl;
    if (j + 1 < 2 * NK) {
      nh = xf(j + 1, 0);
      if (ns == 2) nl = xf(j + 1, 1);
      if (LO) nw = lo(j + 1);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the next pair's reads issued ahead of this pair's MFMAs
    acc = mfma16(wf[j], xh, acc);
    if (ns == 2) acc = mfma16(wf[j], xl, acc);
    if (LO) acc = mfma16(wl, xh, acc);
    xh = nh, xl = nl, wl = nw;
  }
  return acc;
}
// acc += W_lo . X_hi alone (a two-plane X image): the second pass of a block whose lo fragments reuse the hi registers
template <int NK>
__device__ __forceinline__ f32x4 mma_frag_lo(f32x4 acc, const bf16x8* wl, const char* ximg) {
  auto xf = [&](int j) { return frag(ximg + (j >> 1) * 2 * 2048, 0, j & 1); };
  bf16x8 xh = xf(0);
#pragma unroll
  for (int j = 0; j < 2 * NK; ++j) {
    const bf16x8 nh = j + 1 < 2 * NK ? xf(j + 1) : xh;
    __builtin_amdgcn_sched_barrier(0);
    acc = mfma16(wl[j], xh, acc);
    xh = nh;
  }
  return acc;
}
// Opening of an FR block: the X image DMA is this wave's OLDEST VMEM work and its weight fragments (`younger`
// loads, always issued) follow, so waiting for vmcnt(younger) lands the X image while the fragments stay in flight -
// the MFMAs then wait for each fragment through the compiler's own counted waits instead of for all of them here.
// (VMEM operations retire in issue order; a plain s_barrier: the X image is DMA'd, no store needs a fence.)
// YOUNGER = the fragment loads the caller issued after its X DMA (load_frags<N>: N one-instruction 16-byte loads),
// written as the sum of the load_frags template arguments at each call
template <int YOUNGER>
__device__ __forceinline__ void x_landed() {
  static_assert(YOUNGER == 24 || YOUNGER == 16 || YOUNGER == 8 || YOUNGER == 0,
                "x_landed: add the s_waitcnt form for this count");
  if constexpr (YOUNGER == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if constexpr (YOUNGER == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (YOUNGER == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void open_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int YOUNGER>
__device__ __forceinline__ void open_x() {
  x_landed<YOUNGER>();
  open_barrier();
}
// this wave's LDS stores done, then the barrier (no vmcnt wait: weight fragments stay in flight)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  open_barrier();
}
// this wave's n fragments first .. first + n - 1 of a frag_pack image: each one 1 KiB contiguous (full lines)
template <int N>
__device__ __forceinline__ void load_frags(bf16x8* w, const bf16_t* img, long first) {
  const bf16x8* src = (const bf16x8*)(img + first * 512) + (threadIdx.x & 63);
#pragma unroll
  for (int i = 0; i < N; ++i) w[i] = src[i * 64];
}

// ---- residual LayerNorm folded into the consuming block (round 5; RlnArgs fold, kernels.h) ----
// The block's X image is y = LN(x + drop(bias + sum_p slab_p)) of its 16 rows instead of the DMA of the a planes the
// separate residual_layernorm launch used to write: wave w normalises row row0 + w, lane l columns 8 l .. 8 l + 7.
// Step 1 (fold_issue) is the block's oldest VMEM work: waves 0-5 DMA one 1-KiB piece each of the LN parameters
// (bias | weight | bias of the norm, 2 KiB each) into LDS at prm, every wave loads its row's x and NP slab columns into
// registers; the caller then issues its weight fragments, so the compiler's counted wait for the slab data (step 2)
// leaves them in flight - and, VMEM retiring in issue order, covers the older parameter DMA, which one barrier then
// publishes to every wave.  Step 2 (fold_finish) sums, normalises, writes the bf16 hi / lo planes into the X image in
// dma_x's layout, and the tile's writer block stores y to x_out (x_out != x: the tile's other blocks still read x).
constexpr int FOLD_PRM = 32 * 1024;                    // LN parameters after the 32 KiB X image
constexpr int DEC_LDS_FOLD = FOLD_PRM + 6 * 1024;

template <int NP>
struct FoldIn {
  f32x4 x[2], s[NP][2];
};

template <int NP>
__device__ __forceinline__ void fold_issue(const RlnArgs& f, int row0, int rows, char* prm, FoldIn<NP>& in) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave < 6) {  // (a wave-uniform select of the three pointers: no indexed kernel-argument load)
    const float* src = wave < 2 ? f.bias : wave < 4 ? f.w : f.b;
    lds_dma16(src + (wave & 1) * 256 + lane * 4, (LDS_AS void*)(prm + wave * 1024));
  }
  const long off = (long)min(row0 + wave, rows - 1) * DEC_D + lane * 8;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    in.s[p][0] = *(const f32x4*)(f.parts + p * f.part_stride + off);
    in.s[p][1] = *(const f32x4*)(f.parts + p * f.part_stride + off + 4);
  }
  in.x[0] = *(const f32x4*)(f.x + off);
  in.x[1] = *(const f32x4*)(f.x + off + 4);
}

template <int NP, int NSC>
__device__ __forceinline__ void fold_finish(const RlnArgs& f, const FoldIn<NP>& in, int row0, int rows, const char* prm,
                                            char* sx, bool writer) {
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6, c = lane * 8;
  f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = o0;
#pragma unroll
  for (int p = 0; p < NP; ++p) o0 += in.s[p][0], o1 += in.s[p][1];
  asm volatile("" ::"v"(o0), "v"(o1));  // the slab sums (so the wait for their loads) stay before the barrier
  open_barrier();  // every wave's parameter piece landed (its wait for the slabs above retired it)
  const f32x4* pr = (const f32x4*)prm;
  o0 += pr[2 * lane], o1 += pr[2 * lane + 1];  // + bias
  if (f.drop.thr) {  // train mode: x + dropout(sublayer output)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o0[k] *= drop_mul(f.drop, f.site, row0 + r, f.drop.pos, c + k);
      o1[k] *= drop_mul(f.drop, f.site, row0 + r, f.drop.pos, c + 4 + k);
    }
  }
  float v[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = in.x[0][k] + o0[k], v[4 + k] = in.x[1][k] + o1[k];
  float sm = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) sm += v[k];
  const float mean = wave_sum(sm) / (float)DEC_D;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] -= mean;
    q += v[k] * v[k];
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)DEC_D + f.eps);
  const f32x4 w0 = pr[128 + 2 * lane], w1 = pr[128 + 2 * lane + 1];
  const f32x4 b0 = pr[256 + 2 * lane], b1 = pr[256 + 2 * lane + 1];
  f32x4 y0, y1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    y0[k] = v[k] * rstd * w0[k] + b0[k];
    y1[k] = v[4 + k] * rstd * w1[k] + b1[k];
  }
  bf16_t hv[8], lv[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) split_bf(y0[k], hv[k], lv[k]), split_bf(y1[k], hv[4 + k], lv[4 + k]);
  u32x4 hw, lw;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    hw[k] = (uint32_t)hv[2 * k] | ((uint32_t)hv[2 * k + 1] << 16);
    lw[k] = (uint32_t)lv[2 * k] | ((uint32_t)lv[2 * k + 1] << 16);
  }
  // X image [k64][NSC][16 rows][128 B]: columns 8 l .. 8 l + 7 are 16-byte chunk l & 7 of k64-step l >> 3
  char* dst = sx + (lane >> 3) * NSC * 2048 + r * 128 + (((lane & 7) ^ ((r >> 1) & 7)) << 4);
  *(u32x4*)dst = hw;
  if (NSC == 2) *(u32x4*)(dst + 2048) = lw;
  if (writer && row0 + r < rows) {
    *(f32x4*)(f.x_out + (long)(row0 + r) * DEC_D + c) = y0;
    *(f32x4*)(f.x_out + (long)(row0 + r) * DEC_D + c + 4) = y1;
  }
}

// A slab tile store: 16 bytes at byte offset off of a wave-uniform base; write-through (the sc1 bit of agent-scope
// relaxed atomics, as one vector store) when the block's SlabMerge follows.  (Per-dword agent atomics instead:
// dec_sa 12 -> 45 us, profiles/r04/merge_ab.txt.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
}
// Product (round 5): the slabs are stored non-temporal (cache policy nt, aux bit 2).  The split-K slabs are the bulk
// of what a decode node writes (4-8 MB per launch at B = 256) and the next node reads them once; written nt they
// leave the kernel-end L2 write-back little to do: decode 11.06-11.14 -> 10.79-10.94 ms, same box (sc1 write-through
// the same; nt on every decode output - LayerNorm rows, q~ / context planes, KV appends, next-token rows - only
// 11.01-11.03: those are read right back; profiles/r05/slab_nt_ab.txt).
__device__ __forceinline__ void slab_store(float* base, uint32_t off, f32x4 v, bool wt) {
#ifdef ICAP_TOOLS
  if (wt) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), slab_rsrc(base), off, 0, 16);
    return;
  }
#endif
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), slab_rsrc(base), off, 0, 2);
}

// SlabMerge (kernels.h) after this block's slab stores: the last of the NP blocks of the 16-row tile row0 merges the
// tile - wave w normalises row row0 + w, lane l columns 8 l .. 8 l + 7 (slabs read agent-scope, in index order, eight
// at a time).  flag: an LDS word nothing reads any more.
template <int NP>
__device__ void slab_merge(const SlabMerge& m, const float* part, long ps, int row0, int rows, int ns, int* flag) {
  const DropCfg& drop = m.drop;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's slab stores are complete
  __syncthreads();                                   // ... and every thread's
  const int tile = row0 >> 4;
  if (threadIdx.x == 0) *flag = __hip_atomic_fetch_add(m.tick + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (*flag != NP - 1) return;
  if (threadIdx.x == 0) __hip_atomic_store(m.tick + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = row0 + wave;
  if (wave >= 16 || row >= rows) return;
  const int c = lane * 8;
  float v[8], o[8];
  {
    const f32x4 x0 = *(const f32x4*)(m.x + (long)row * DEC_D + c), x1 = *(const f32x4*)(m.x + (long)row * DEC_D + c + 4);
    const f32x4 b0 = *(const f32x4*)(m.bias + c), b1 = *(const f32x4*)(m.bias + c + 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = x0[k], v[4 + k] = x1[k], o[k] = b0[k], o[4 + k] = b1[k];
  }
  // v = x + bias + sum_p slab_p in residual_layernorm_kernel's order; under dropout x + drop(bias + sum_p slab_p)
  float* const acc = drop.thr ? o : v;
  if (!drop.thr)
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += o[k];
  const uint32_t off = (uint32_t)(row * DEC_D + c) * 4;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const __amdgpu_buffer_rsrc_t r = slab_rsrc(part + (long)p * ps);  // sc1 loads (agent-coherent)
    const f32x4 a0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
    const f32x4 a1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 16));
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += a0[k], acc[4 + k] += a1[k];
  }
  if (drop.thr)  // x + dropout(sublayer output)
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += o[k] * drop_mul(drop, m.site, row, drop.pos, c + k);
  float sm = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) sm += v[k];
  const float mean = wave_sum(sm) / (float)DEC_D;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] -= mean;
    q += v[k] * v[k];
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)DEC_D + m.eps);
  const f32x4 w0 = *(const f32x4*)(m.w + c), w1 = *(const f32x4*)(m.w + c + 4);
  const f32x4 c0 = *(const f32x4*)(m.b + c), c1 = *(const f32x4*)(m.b + c + 4);
  f32x4 y0, y1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    y0[k] = v[k] * rstd * w0[k] + c0[k];
    y1[k] = v[4 + k] * rstd * w1[k] + c1[k];
  }
  *(f32x4*)(m.x + (long)row * DEC_D + c) = y0;
  *(f32x4*)(m.x + (long)row * DEC_D + c + 4) = y1;
  bf16_t hv[8], lv[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) split_bf(y0[k], hv[k], lv[k]), split_bf(y1[k], hv[4 + k], lv[4 + k]);
  u32x4 hw, lw;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    hw[k] = (uint32_t)hv[2 * k] | ((uint32_t)hv[2 * k + 1] << 16);
    lw[k] = (uint32_t)lv[2 * k] | ((uint32_t)lv[2 * k + 1] << 16);
  }
  *(u32x4*)(m.a + (long)row * DEC_D + c) = hw;
  if (ns == 2) *(u32x4*)(m.a + m.aL + (long)row * DEC_D + c) = lw;
}

// Fragment images of the decode weights (launch_frag_pack, kernels.h): one thread per 16-byte lane piece.
__global__ void frag_pack_kernel(const bf16_t* __restrict__ W, long ldw, int ntiles, int nk, int mode, int tps,
                                 int ksl, bf16_t* __restrict__ out) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)ntiles * nk * 64) return;
  const int l = (int)(idx & 63), s = (int)((idx >> 6) % nk), t = (int)((idx >> 6) / nk);
  int row0 = 16 * t, k0 = 0;
  if (mode == 1) {
    const int hh = t / 12, i = t - hh * 12;
    row0 = (i >> 2) * DEC_D + hh * DEC_HD + (i & 3) * 16;
  } else if (mode == 2) {
    const int j = t / tps, n = t - j * tps;
    row0 = 16 * n;
    k0 = ksl * j;
  }
  *(bf16x8*)(out + idx * 8) = *(const bf16x8*)(W + (long)(row0 + (l & 15)) * ldw + k0 + 32 * s + 8 * (l >> 4));
}

// ------------------------------------------------------------------------------------------------
// Self-attention block of one decode step.
//   round 1: X image (32 KiB, region B) + Wq_h, Wk_h images [8 k64][128 rows][128 B] (region A)
//   round 2: Wv_h [8 k64][64 rows][128 B] + Wo[:, 64h:64h+64] [512 rows][128 B] (region A)
//   then q|k|v rows fp32 [16][192] + ctx image in region B
// FR (DecSaArgs::Wqkv_f / Wo_f, round 4): no weight region - waves 0-11 load their q|k|v tile's 16 KiB of fragments
// straight into registers in the same burst as the X image, and every wave its 4 KiB of Wo fragments after its QKV
// MFMAs (behind the attention): one memory round instead of two, 32 KiB of LDS instead of 160.
// WLO (round 5, FR with two planes): hi/lo decoder weights - after its hi MFMAs a wave reloads the same registers with
// its lo q|k|v fragments (one more memory round: the hi and lo images of a tile, 32 KiB per wave, do not fit beside
// each other) and adds W_lo . X_hi; the Wo lo fragments ride with the hi ones behind the attention.
template <bool FR, int NSC = 0, bool WLO = false>
__global__ __launch_bounds__(1024) void dec_sa_kernel(DecSaArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ra = smem;                        // 128 KiB weight region (FR: none)
  char* sx = smem + (FR ? 0 : 128 * 1024);  // 32 KiB row region
  float* qkv = (float*)sx;                // after the v projection: [16][192]
  char* sc = sx + 16 * 192 * 4;           // ctx image [1 k64][ns][16][128 B]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int bid = blockIdx.x;  // xcd_tiles: tile = bid % 8 + 8 (bid / 64), head = (bid / 8) % 8 (a tile on one XCD)
  const bool xt = DEC_XCD_TILES && p.xcd_tiles;
  const int h = xt ? (bid >> 3) & 7 : bid & (DEC_H - 1);
  const int row0 = (xt ? (bid & 7) + 8 * (bid >> 6) : bid >> 3) * DEC_ROWS;
  const int ns = NSC ? NSC : p.nsplit;  // NSC: the plane count as a constant (no per-MFMA branches)
  const char* wq = (const char*)(p.Wqkv + (long)(h * DEC_HD) * DEC_D);
  const char* wk = (const char*)(p.Wqkv + (long)(DEC_D + h * DEC_HD) * DEC_D);
  const char* wv = (const char*)(p.Wqkv + (long)(2 * DEC_D + h * DEC_HD) * DEC_D);

  // this wave's bias columns first (the oldest load: the opening waits cover it, so the epilogue after the MFMAs
  // waits for no load - a late bias load's vmcnt(0) also drained the Wo fragments issued behind the attention)
  // (waves 12-15 load wave 0's columns and never use them: an unconditional load, see dec_chain_kernel)
  const int bc = (wave < 12 ? wave : 0) * 16 + 4 * fq;
  const f32x4 bias = *(const f32x4*)(p.bqkv + (bc >> 6) * DEC_D + h * DEC_HD + (bc & 63));
  dma_x(p.A, p.aL, ns, row0, p.rows, sx);
  constexpr int NWQ = 2 * DEC_K64;  // fragments per wave (the opening's vmcnt counts them)
  bf16x8 wf[FR ? NWQ : 1];  // FR: this wave's q|k|v tile (waves 0-11), all 16 k32-steps
  if (FR) {
    if (wave < 12) load_frags<NWQ>(wf, p.Wqkv_f, (long)(h * 12 + wave) * 2 * DEC_K64);
  } else {
    for (int k = 0; k < DEC_K64; ++k) {  // Wq_h, Wk_h: image [k64][128 rows] (q rows 0..63, k rows 64..127)
      dma_rows(wq + k * 128, DEC_D * 2, 64, ra + k * 128 * 128, 8 * (2 * k) + 2);
      dma_rows(wk + k * 128, DEC_D * 2, 64, ra + k * 128 * 128 + 64 * 128, 8 * (2 * k + 1) + 2);
    }
  }
  // the cached keys / values of positions < t0 of this wave's row (it attends for row row0 + wave below) do
  // not depend on this step: fetch the first 32 positions now, while the projections are staged.  Lane l
  // holds key / value j = 4 i + (l >> 4), dims 4 (l & 15) ..; 16 lanes read one 256-B row.
  constexpr int PRE = FR ? 3 : 8;  // FR: 12 cached positions in registers (no spill next to the W fragments, the prefetched X fragments and the bias)
  const int dq = (lane & 15) * 4, jg = lane >> 4;
  const int brow = row0 + wave, t0 = p.t0;
  f32x4 kpre[PRE], vpre[PRE];
  const long own = ((long)brow * DEC_H + h) * p.Lmax * DEC_HD;
  auto hist = [&](const float* cache, int j) -> f32x4 {  // cached row of position j < t0 (lane's 4 dims)
    const long rb = p.anc ? ((long)p.anc[(long)brow * p.Lmax + j] * DEC_H + h) * p.Lmax * DEC_HD : own;
    return *(const f32x4*)(cache + rb + (long)j * DEC_HD + dq);
  };
#pragma unroll
  for (int i = 0; i < PRE; ++i) {  // keys now, values at the start of the attention (register budget)
    const int j = 4 * i + jg;
    kpre[i] = brow < p.rows && j < t0 ? hist(p.kc, j) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  if (FR && NSC == 2) {  // X landed, the 16 q|k|v fragments of waves 0-11 may still fly (the cached keys behind them)
    if (wave < 12) x_landed<NWQ>();
    else x_landed<0>();
    open_barrier();  // one barrier on every wave's path
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  bf16x8 wo[FR ? 4 : 1], wol[WLO ? 4 : 1];  // FR: Wo fragments of output column tiles 2 wave, 2 wave + 1 (2 k32-steps each)
  if (FR) {
    if (wave < 12) acc = mma_frag<DEC_K64>(acc, wf, sx, ns);  // q tiles 0..3, k tiles 4..7, v tiles 8..11
    if (WLO && wave < 12) {
      __builtin_amdgcn_sched_barrier(0);  // the hi fragments consumed: their registers take the lo image
      load_frags<NWQ>(wf, p.Wqkv_fl, (long)(h * 12 + wave) * 2 * DEC_K64);
      acc = mma_frag_lo<DEC_K64>(acc, wf, sx);
    }
  } else {
    if (wave < 8) acc = mma_rows(acc, ra, 128, wave * 16, sx, ns, 0, DEC_K64);  // q tiles 0..3, k tiles 4..7
    __syncthreads();  // Wq / Wk no longer read
    for (int k = 0; k < DEC_K64; ++k) dma_rows(wv + k * 128, DEC_D * 2, 64, ra + k * 64 * 128, 8 * k);
    dma_rows((const char*)(p.Wo + h * DEC_HD), DEC_D * 2, DEC_D, ra + DEC_K64 * 64 * 128);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave >= 8 && wave < 12) acc = mma_rows(acc, ra, 64, (wave - 8) * 16, sx, ns, 0, DEC_K64);  // v tiles
  }
  __syncthreads();  // X image no longer read: it becomes the q|k|v rows
  if (FR) load_frags<4>(wo, p.Wo_f, (long)(h * 32 + 2 * wave) * 2);  // needed after the attention
  if (WLO) load_frags<4>(wol, p.Wo_fl, (long)(h * 32 + 2 * wave) * 2);
  if (wave < 12) {
    const int c = wave * 16 + 4 * fq;  // column in [q | k | v] of this head
    acc += bias;
    *(f32x4*)(qkv + fr * 192 + c) = acc;
  }
  __syncthreads();

  // ---- attention, one wave per row (torch's causal SDPA of the new position over positions 0..t0).
  // The cached keys / values of a (row, head) are [t0][64] fp32 rows: lane l reads 16-byte chunk
  // c = l + 64 i, i.e. key j = c >> 4, dims 4 (c & 15) ..; 16 lanes hold one key (1 KiB per instruction).
  {
    const int r = wave, b = brow, nkeys = t0 + 1;
    const float* qr = qkv + r * 192;
    f32x4 ctx = {0.f, 0.f, 0.f, 0.f};
    float l = 1.f;
    if (b < p.rows) {
      if (lane < 16) {  // this step's key / value into the cache
        *(f32x4*)(p.kc + own + (long)t0 * DEC_HD + dq) = *(const f32x4*)(qr + 64 + dq);
        *(f32x4*)(p.vc + own + (long)t0 * DEC_HD + dq) = *(const f32x4*)(qr + 128 + dq);
      }
#pragma unroll
      for (int i = 0; i < PRE; ++i) {
        const int j = 4 * i + jg;
        vpre[i] = j < t0 ? hist(p.vc, j) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      // keys 4 PRE .. 31 in one batch beside the values (their values behind the scores), so no score or context step
      // waits for its own cache load; positions >= 32 (max_len > 33) load in their loop
      constexpr int LATE = 8 - PRE;
      f32x4 klate[LATE > 0 ? LATE : 1], vlate[LATE > 0 ? LATE : 1];
#pragma unroll
      for (int i = 0; i < LATE; ++i) {
        const int j = 4 * (PRE + i) + jg;
        klate[i] = j < t0 ? hist(p.kc, j) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      const f32x4 q4 = *(const f32x4*)(qr + dq);
      const f32x4 kcur = *(const f32x4*)(qr + 64 + dq), vcur = *(const f32x4*)(qr + 128 + dq);
      // scores: lane j of the wave ends up holding score j.  Keys j = 4 i + jg: the first PRE x 4 from the
      // prefetched registers (unrolled, so they stay in VGPRs), any later ones straight from the cache
      float s_mine = -INFINITY;
      auto score = [&](int i, f32x4 k4) {
        float part = q4[0] * k4[0];
        part = fmaf(q4[1], k4[1], part);
        part = fmaf(q4[2], k4[2], part);
        part = fmaf(q4[3], k4[3], part);
        part = row16_sum(part);  // sum over the key's 16 lanes (DPP: no LDS round trip)
        // scores of keys 4i..4i+3 sit in rows 0..3: lane j takes key j's (lane broadcasts of the row leaders)
        const float p0 = lane_bcast(part, 0), p1 = lane_bcast(part, 16), p2 = lane_bcast(part, 32), p3 = lane_bcast(part, 48);
        const int kr = (lane - 4 * i) & 3;
        const float sc = kr == 0 ? p0 : kr == 1 ? p1 : kr == 2 ? p2 : p3;
        if (lane >= 4 * i && lane < 4 * i + 4) s_mine = lane < nkeys ? sc * p.scale : -INFINITY;
      };
      auto pick = [&](int j, f32x4 cur, f32x4 pre) -> f32x4 {
        return j == t0 ? cur : (j > t0 ? (f32x4){0.f, 0.f, 0.f, 0.f} : pre);
      };
#pragma unroll
      for (int i = 0; i < PRE; ++i)
        if (4 * i < nkeys) score(i, pick(4 * i + jg, kcur, kpre[i]));
#pragma unroll
      for (int i = 0; i < LATE; ++i)
        if (4 * (PRE + i) < nkeys) score(PRE + i, pick(4 * (PRE + i) + jg, kcur, klate[i]));
      for (int i = 8; 4 * i < nkeys; ++i) {
        const int j = 4 * i + jg;
        const f32x4 k4 = j < t0 ? hist(p.kc, j) : kcur;
        score(i, pick(j, kcur, k4));
      }
#pragma unroll
      for (int i = 0; i < LATE; ++i) {  // the late values, in flight behind the softmax
        const int j = 4 * (PRE + i) + jg;
        vlate[i] = j < t0 ? hist(p.vc, j) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      const float m = wave_max(s_mine);
      const float e = lane < nkeys ? __expf(s_mine - m) : 0.f;
      l = wave_sum(e);
      // train mode: dropout on the attention probabilities (key = lane), the normaliser stays undropped
      const float ed = p.drop.thr && lane < nkeys ? e * drop_mul(p.drop, 1, b, t0, h * 128 + lane) : e;
      // context: lane accumulates dims dq..dq+3 over keys j = 4 i + jg, then the 4 key groups are summed.  The
      // probability of key j (held by lane j) reaches row jg through four lane broadcasts (no LDS round trip)
      auto prob = [&](int i) {
        const float e0 = lane_bcast(ed, min(4 * i, 63)), e1 = lane_bcast(ed, min(4 * i + 1, 63));
        const float e2 = lane_bcast(ed, min(4 * i + 2, 63)), e3 = lane_bcast(ed, min(4 * i + 3, 63));
        return jg == 0 ? e0 : jg == 1 ? e1 : jg == 2 ? e2 : e3;
      };
#pragma unroll
      for (int i = 0; i < PRE; ++i)
        if (4 * i < nkeys) {
          const int j = 4 * i + jg;
          ctx += prob(i) * pick(j, vcur, vpre[i]);
        }
#pragma unroll
      for (int i = 0; i < LATE; ++i)
        if (4 * (PRE + i) < nkeys) ctx += prob(PRE + i) * pick(4 * (PRE + i) + jg, vcur, vlate[i]);
      for (int i = 8; 4 * i < nkeys; ++i) {
        const int j = 4 * i + jg;
        const f32x4 v4 = j < t0 ? hist(p.vc, j) : vcur;
        ctx += prob(i) * pick(j, vcur, v4);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) ctx[k] = rows4_sum(ctx[k]);
      ctx /= l;
    }
    if (lane < 16) put_planes(sc, ns, r, dq, ctx);
  }
  __syncthreads();

  // ---- out-projection slab of head h: 16 rows x 512 columns, K = 64 (one k64 step)
  const char* woi = ra + DEC_K64 * 64 * 128;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
    if (WLO) o = mma_frag<1>(o, wo + 2 * i, sc, ns, [&](int j) { return wol[2 * i + j]; });
    else if (FR) o = mma_frag<1>(o, wo + 2 * i, sc, ns);
    else o = mma_rows(o, woi, DEC_D, wave * 32 + i * 16, sc, ns, 0, 1);
    const int row = row0 + fr;
    if (row < p.rows)
      slab_store(p.part + (long)h * p.part_stride, (uint32_t)(row * DEC_D + wave * 32 + i * 16 + 4 * fq) * 4, o,
                 p.mg.tick);
  }
#ifdef ICAP_TOOLS  // (measured slower: tools build only, icap.cpp decoder_layers)
  if (p.mg.tick) slab_merge<DEC_H>(p.mg, p.part, p.part_stride, row0, p.rows, ns, (int*)smem);
#endif
}

// ------------------------------------------------------------------------------------------------
// Feed-forward block of one decode step.
//   round 1: X image (region B) + W1 slice [8 k64][128 rows][128 B] (region A)
//   round 2: W2 slice [2 k64][512 rows][128 B] (region A); h image + k-half reduction in region B
// FR (DecFfnArgs::W1f / W2f, round 4): each wave loads its W1 fragments (tile t, k-half kh: 8 KiB) and its W2
// fragments (column tiles 2 wave, 2 wave + 1 of the slice: 8 KiB) into registers with the X image - one memory round.
// FOLD (round 5, FR with two planes): X = the residual LN2 of the cross-attention chain's FOLD slabs, written by the
// block of slice 0; the W2 fragments are then issued after the fold (register budget) and fly behind FFN-1.
// WLO (round 5, FR with two planes, no fold): hi/lo decoder weights - each wave DMAs its W1 lo fragments (8 KiB) into
// its own LDS slot behind its W1 hi loads (the 128 KiB the FR form leaves free), and loads its W2 lo fragments into the
// registers the W1 fragments free after FFN-1.
template <bool FR, int NSC = 0, int FOLD = 0, bool WLO = false>
__global__ __launch_bounds__(1024) void dec_ffn_kernel(DecFfnArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ra = smem;
  char* sx = smem + (FR ? 0 : 128 * 1024);
  f32x4* red = (f32x4*)sx;                 // after FFN-1: [8 tiles][64 lanes]
  char* sh = sx + 8 * 64 * 16;             // h image [2 k64][ns][16][128 B]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int nslice = DEC_F / 128;
  const int bid = blockIdx.x;
  const bool xt = DEC_XCD_TILES && FOLD && p.xcd_tiles;  // tile = bid % 8 + 8 (bid / 128), slice = (bid / 8) % 16: a tile on one XCD
  const int j = xt ? (bid >> 3) & 15 : bid % nslice;
  const int row0 = (xt ? (bid & 7) + 8 * (bid >> 7) : bid / nslice) * DEC_ROWS;
  const int ns = NSC ? NSC : p.nsplit;  // NSC: the plane count as a constant (no per-MFMA branches)

  const int t = wave & 7, kh = wave >> 3;  // FFN-1 tile, k half (4 of the 8 k64 steps)
  const f32x4 bias = *(const f32x4*)(p.b1 + j * 128 + t * 16 + 4 * fq);  // oldest load (as dec_sa_kernel)
  FoldIn<FOLD ? FOLD : 1> fi;
  if constexpr (FOLD) fold_issue<FOLD>(p.fold, row0, p.rows, smem + FOLD_PRM, fi);
  else dma_x(p.A, p.aL, ns, row0, p.rows, sx);
  constexpr int NW1 = DEC_K64, NW2 = 8;  // fragments per wave (the opening's vmcnt counts them)
  // the counted waits below, by what this wave issues after dma_x, in order (no other VMEM operation may go between):
  // load_frags<NW1> (W1), WLO: NW1 lds_dma16 (W1 lo slot), load_frags<NW2> (W2)
  constexpr int YNG_X = NW1 + (WLO ? NW1 : 0) + NW2;  // younger than the X image at the opening
  constexpr int YNG_LO = NW2;                         // younger than the W1 lo slot (WLO's first FFN-1 wait)
  bf16x8 w1f[FR ? NW1 : 1], w2f[FR ? NW2 : 1];
  const long w1i = (long)(j * 8 + t) * 2 * DEC_K64 + kh * DEC_K64, w2i = (long)(j * 32 + 2 * wave) * 4;
  char* const lo1 = smem + 32 * 1024 + wave * NW1 * 1024;  // WLO: this wave's W1 lo fragments (its own slot)
  if (FR) {
    load_frags<NW1>(w1f, p.W1f, w1i);
    if (WLO) {
#pragma unroll
      for (int i = 0; i < NW1; ++i)
        lds_dma16(p.W1fl + (w1i + i) * 512 + lane * 8, (LDS_AS void*)(lo1 + i * 1024));
    }
    if (!FOLD) load_frags<NW2>(w2f, p.W2f, w2i);
    if (FOLD) __builtin_amdgcn_sched_barrier(0);  // every W1 fragment load issued before the fold's first wait
  } else {
    const char* w1 = (const char*)(p.W1 + (long)j * 128 * DEC_D);
    for (int k = 0; k < DEC_K64; ++k) dma_rows(w1 + k * 128, DEC_D * 2, 128, ra + k * 128 * 128);
  }
  if constexpr (FOLD) {
    fold_finish<FOLD, 2>(p.fold, fi, row0, p.rows, smem + FOLD_PRM, sx, j == 0);
    load_frags<NW2>(w2f, p.W2f, (long)(j * 32 + 2 * wave) * 4);
    lds_barrier();  // the X image written
  } else if (FR && NSC == 2) {
    open_x<YNG_X>();  // X landed; W1 / W1 lo / W2 fragments may still fly
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (WLO) {
    static_assert(!WLO || YNG_LO == NW2, "W2 fragments are the only loads after the W1 lo slot");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(YNG_LO) : "memory");  // this wave's W1 lo slot landed (W2 may fly)
    const bf16x8* l1 = (const bf16x8*)lo1 + lane;
    acc = mma_frag<4>(acc, w1f, sx + kh * 4 * ns * 2048, ns, [&](int i) { return l1[i * 64]; });
  } else if (FR) {
    acc = mma_frag<4>(acc, w1f, sx + kh * 4 * ns * 2048, ns);
  } else {
    acc = mma_rows(acc, ra, 128, t * 16, sx, ns, kh * 4, kh * 4 + 4);
  }
  bf16x8 w2l[WLO ? NW2 : 1];
  if (WLO) {
    __builtin_amdgcn_sched_barrier(0);  // after FFN-1: the W1 registers are free
    load_frags<NW2>(w2l, p.W2fl, w2i);
  }
  __syncthreads();  // W1 and X no longer read
  if (!FR) {
    const char* w2 = (const char*)(p.W2 + (long)j * 128);
    for (int k = 0; k < 2; ++k) dma_rows(w2 + k * 128, DEC_F * 2, DEC_D, ra + k * DEC_D * 128);
  }
  if (kh) red[t * 64 + lane] = acc;
  __syncthreads();
  if (!kh) {
    acc += red[t * 64 + lane];
    const int n = t * 16 + 4 * fq;
    acc += bias;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = fmaxf(acc[r], 0.f);
    if (p.drop.thr)  // train mode: dropout on the hidden activations
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] *= drop_mul(p.drop, 5, row0 + fr, p.drop.pos, j * 128 + n + r);
    put_planes(sh, ns, fr, n, acc);
  }
  if (!FR) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
    if (WLO) o = mma_frag<2>(o, w2f + 4 * i, sh, ns, [&](int q) { return w2l[4 * i + q]; });
    else if (FR) o = mma_frag<2>(o, w2f + 4 * i, sh, ns);
    else o = mma_rows(o, ra, DEC_D, wave * 32 + i * 16, sh, ns, 0, 2);
    const int row = row0 + fr;
    if (row < p.rows)
      slab_store(p.part + (long)j * p.part_stride, (uint32_t)(row * DEC_D + wave * 32 + i * 16 + 4 * fq) * 4, o,
                 p.mg.tick);
  }
#ifdef ICAP_TOOLS  // (measured slower: tools build only, icap.cpp decoder_layers)
  if (p.mg.tick) slab_merge<DEC_F / 128>(p.mg, p.part, p.part_stride, row0, p.rows, ns, (int*)smem);
#endif
}

// ------------------------------------------------------------------------------------------------
// Chained per-head products of the cross-attention block (replaces chain_dec_kernel on the decode path):
//   Y_h = X_h W1_h^T + b1_h (16 x 64, K = 512), O_h = Y_h W2_h^T (16 x 512, K = 64)
// block = (16 rows, head h), one DMA round: X image 32 KiB + W1_h [8 k64][64][128 B] 64 KiB +
// W2_h [512 rows][128 B] 64 KiB.  out = OUT_SPLIT (q~ planes of head h) or OUT_PARTIAL (slab h).
// FR (ChainArgs::W1f / W2f, round 4): W1 (tile t, k-quarter kq: 4 KiB) and W2 (column tiles 2 wave, 2 wave + 1: 4 KiB)
// fragments per wave in registers, 32 KiB of LDS (the X image) instead of 160.
// FOLD (round 5, FR with two planes, X shared by the heads): X = the residual LN1 of dec_sa's FOLD slabs (fold_issue /
// fold_finish), written by the block of head 0; the 8 head blocks of a row tile then run on one XCD (xcd_tiles) so
// the tile's slabs are read from that XCD's L2 after the first block's miss.
// WLO (round 5, FR with two planes, no fold): hi/lo decoder weights, the lo fragments in registers beside the hi ones.
template <bool FR, int NSC = 0, int FOLD = 0, bool WLO = false>
__global__ __launch_bounds__(1024) void dec_chain_kernel(ChainArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* w1i = smem;                       // 64 KiB (FR: none)
  char* w2i = smem + 64 * 1024;           // 64 KiB (FR: none)
  char* sx = smem + (FR ? 0 : 128 * 1024);  // 32 KiB: X image, then the k-quarter reduction + Y image
  f32x4* red = (f32x4*)sx;                // [3 quarters][4 tiles][64 lanes]
  char* sy = sx + 12 * 64 * 16;           // Y image [1 k64][ns][16][128 B]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int bid = blockIdx.x;
  const bool xt = DEC_XCD_TILES && p.xcd_tiles;  // tile = bid % 8 + 8 (bid / 64), head = (bid / 8) % 8 (one XCD)
  const int H = FR ? DEC_H : p.H;  // (the FR forms run DEC_H heads: launch_dec_chain checks it)
  const int h = xt ? (bid >> 3) & 7 : bid % H;
  const int row0 = (xt ? (bid & 7) + 8 * (bid >> 6) : bid / H) * DEC_ROWS;
  const int ns = NSC ? NSC : p.nsplit;  // NSC: the plane count as a constant (no per-MFMA branches)
  const int t = wave & 3, kq = wave >> 2;  // Y tile, k quarter (2 of the 8 k64 steps)
  const f32x4 bv = *(const f32x4*)(p.b1 + h * 64 + t * 16 + 4 * fq);  // oldest loads (as dec_sa_kernel)
  // (unconditional, from b1 when there is no scale: a load under a branch made hipcc wait for it at the join)
  const float bsc = *(p.b1_scale ? p.b1_scale + (long)min(row0 + fr, p.M - 1) * p.H + h : p.b1);
  FoldIn<FOLD ? FOLD : 1> fi;
  if constexpr (FOLD) fold_issue<FOLD>(p.fold, row0, p.M, smem + FOLD_PRM, fi);
  else dma_x(p.X + (long)h * p.x_hstride, p.x_lo, ns, row0, p.M, sx, p.ldx);
  constexpr int NW1 = 4, NW2 = 4;  // fragments per wave (the opening's vmcnt counts them)
  bf16x8 w1f[FR ? NW1 : 1], w2f[FR ? NW2 : 1], w1l[WLO ? NW1 : 1], w2l[WLO ? NW2 : 1];
  if (FR) {
    load_frags<NW1>(w1f, p.W1f, (long)(h * 4 + t) * 2 * DEC_K64 + kq * 4);
    load_frags<NW2>(w2f, p.W2f, (long)(h * 32 + 2 * wave) * 2);
    if (WLO) {
      load_frags<NW1>(w1l, p.W1fl, (long)(h * 4 + t) * 2 * DEC_K64 + kq * 4);
      load_frags<NW2>(w2l, p.W2fl, (long)(h * 32 + 2 * wave) * 2);
    }
    if (FOLD) __builtin_amdgcn_sched_barrier(0);  // every fragment load issued before the fold's first wait
  } else {
    const char* w1 = (const char*)(p.W1 + (long)h * 64 * DEC_D);
    for (int k = 0; k < DEC_K64; ++k) dma_rows(w1 + k * 128, DEC_D * 2, 64, w1i + k * 64 * 128, 8 * k + 2);
    dma_rows((const char*)(p.W2 + (long)h * p.w2_hstride), p.ldw2 * 2, DEC_D, w2i, 2);
  }
  if constexpr (FOLD) {
    fold_finish<FOLD, 2>(p.fold, fi, row0, p.M, smem + FOLD_PRM, sx, h == 0);
    lds_barrier();  // the X image written
  } else if (FR && NSC == 2) {
    open_x<(WLO ? 2 : 1) * (NW1 + NW2)>();  // X landed; the W1 / W2 (hi, lo) fragments may still fly
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (WLO) acc = mma_frag<2>(acc, w1f, sx + kq * 2 * ns * 2048, ns, [&](int i) { return w1l[i]; });
  else if (FR) acc = mma_frag<2>(acc, w1f, sx + kq * 2 * ns * 2048, ns);
  else acc = mma_rows(acc, w1i, 64, t * 16, sx, ns, kq * 2, kq * 2 + 2);
  __syncthreads();  // X no longer read
  if (kq) red[((kq - 1) * 4 + t) * 64 + lane] = acc;
  __syncthreads();
  if (!kq) {
#pragma unroll
    for (int q = 0; q < 3; ++q) acc += red[(q * 4 + t) * 64 + lane];
    const int n = t * 16 + 4 * fq;
    if (p.b1_scale) acc += bv * bsc;
    else acc += bv;
    put_planes(sy, ns, fr, n, acc);
  }
  __syncthreads();
  const int row = row0 + fr;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
    if (WLO) o = mma_frag<1>(o, w2f + 2 * i, sy, ns, [&](int q) { return w2l[2 * i + q]; });
    else if (FR) o = mma_frag<1>(o, w2f + 2 * i, sy, ns);
    else o = mma_rows(o, w2i, DEC_D, wave * 32 + i * 16, sy, ns, 0, 1);
    const int col = wave * 32 + i * 16 + 4 * fq;
    if (row >= p.M) continue;
    if (p.out == OUT_PARTIAL) {
      slab_store((float*)p.C + (long)h * p.part_stride, (uint32_t)(row * p.ldc + col) * 4, o, p.mg.tick);
    } else {
      bf16_t hv[4], lv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) split_bf(o[r], hv[r], lv[r]);
      bf16_t* dst = (bf16_t*)p.C + (long)row * p.ldc + (long)h * p.c_hstride + col;
      *(u32x2*)dst = (u32x2){(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16)};
      if (ns == 2)
        *(u32x2*)(dst + p.c_lo) =
            (u32x2){(uint32_t)lv[0] | ((uint32_t)lv[1] << 16), (uint32_t)lv[2] | ((uint32_t)lv[3] << 16)};
    }
  }
#ifdef ICAP_TOOLS  // (measured slower: tools build only, icap.cpp decoder_layers)
  if (p.out == OUT_PARTIAL && p.mg.tick)
    slab_merge<DEC_H>(p.mg, (const float*)p.C, p.part_stride, row0, p.M, ns, (int*)smem);
#endif
}

}  // namespace

namespace {
constexpr int DEC_LDS_FR = 32 * 1024;  // the FR forms: the X image region only
hipError_t dec_lds_attr() {
  static bool attr = false;
  if (attr) return hipSuccess;
  for (const void* f : {(const void*)dec_sa_kernel<false>, (const void*)dec_ffn_kernel<false>,
                        (const void*)dec_chain_kernel<false>}) {
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, DEC_LDS);
    if (e != hipSuccess) return e;
  }
  attr = true;
  return hipSuccess;
}
// a fold's arguments: the 8 producer slabs of d_model-wide rows, the LN parameters, x_out apart from x
bool fold_ok(const RlnArgs& f, int nparts) {
  return f.parts && f.x && f.x_out && f.x_out != f.x && f.bias && f.w && f.b && f.nparts == nparts &&
         f.part_stride > 0;
}
}  // namespace

hipError_t launch_dec_chain(const ChainArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N2 != DEC_D || a.H <= 0 || (a.nsplit != 1 && a.nsplit != 2)) return hipErrorInvalidValue;
  if (a.out != OUT_PARTIAL && a.out != OUT_SPLIT) return hipErrorInvalidValue;
  if (!a.W1f != !a.W2f || (a.W1f && a.H != DEC_H)) return hipErrorInvalidValue;
  if (a.mg.tick && (a.out != OUT_PARTIAL || a.H != DEC_H || a.ldc != DEC_D)) return hipErrorInvalidValue;
  const hipError_t e = dec_lds_attr();
  if (e != hipSuccess) return e;
  const int blocks = (a.M + DEC_ROWS - 1) / DEC_ROWS * a.H;
  if (a.fold.parts) {  // the residual LN1 folded in: X from dec_sa's 8 slabs (measured slower: tools build only)
#ifndef ICAP_TOOLS
    return hipErrorInvalidValue;
#else
    if (!a.W1f || a.W1fl || a.nsplit != 2 || a.x_hstride != 0 || a.H != DEC_H || a.out != OUT_SPLIT || a.mg.tick ||
        !fold_ok(a.fold, DEC_H))
      return hipErrorInvalidValue;
    ChainArgs b = a;
    b.xcd_tiles = a.xcd_tiles && ((a.M + DEC_ROWS - 1) / DEC_ROWS) % 8 == 0;
    hipLaunchKernelGGL((dec_chain_kernel<true, 2, DEC_H>), dim3(blocks), dim3(1024), DEC_LDS_FOLD, s, b);
    return hipGetLastError();
#endif
  }
  ChainArgs c = a;
  c.xcd_tiles = a.xcd_tiles && a.H == DEC_H && ((a.M + DEC_ROWS - 1) / DEC_ROWS) % 8 == 0;
  if (!a.W1fl != !a.W2fl || (a.W1fl && (!a.W1f || a.nsplit != 2 || a.mg.tick))) return hipErrorInvalidValue;
  if (a.W1fl) hipLaunchKernelGGL((dec_chain_kernel<true, 2, 0, true>), dim3(blocks), dim3(1024), DEC_LDS_FR, s, c);
  else if (a.W1f && a.nsplit == 2) hipLaunchKernelGGL((dec_chain_kernel<true, 2>), dim3(blocks), dim3(1024), DEC_LDS_FR, s, c);
  else if (a.W1f) hipLaunchKernelGGL(dec_chain_kernel<true>, dim3(blocks), dim3(1024), DEC_LDS_FR, s, c);
  else hipLaunchKernelGGL(dec_chain_kernel<false>, dim3(blocks), dim3(1024), DEC_LDS, s, c);
  return hipGetLastError();
}

hipError_t launch_dec_sa(const DecSaArgs& a, hipStream_t s) {
  if (a.rows <= 0 || a.t0 < 0 || a.t0 >= a.Lmax || a.t0 >= 64 || (a.nsplit != 1 && a.nsplit != 2))
    return hipErrorInvalidValue;
  if (!a.Wqkv_f != !a.Wo_f) return hipErrorInvalidValue;
  const hipError_t e = dec_lds_attr();
  if (e != hipSuccess) return e;
  const int blocks = (a.rows + DEC_ROWS - 1) / DEC_ROWS * DEC_H;
  DecSaArgs b = a;
  b.xcd_tiles = a.xcd_tiles && ((a.rows + DEC_ROWS - 1) / DEC_ROWS) % 8 == 0;
  if (!a.Wqkv_fl != !a.Wo_fl || (a.Wqkv_fl && (!a.Wqkv_f || a.nsplit != 2 || a.mg.tick))) return hipErrorInvalidValue;
  if (a.Wqkv_fl) hipLaunchKernelGGL((dec_sa_kernel<true, 2, true>), dim3(blocks), dim3(1024), DEC_LDS_FR, s, b);
  else if (a.Wqkv_f && a.nsplit == 2) hipLaunchKernelGGL((dec_sa_kernel<true, 2>), dim3(blocks), dim3(1024), DEC_LDS_FR, s, b);
  else if (a.Wqkv_f) hipLaunchKernelGGL(dec_sa_kernel<true>, dim3(blocks), dim3(1024), DEC_LDS_FR, s, b);
  else hipLaunchKernelGGL(dec_sa_kernel<false>, dim3(blocks), dim3(1024), DEC_LDS, s, b);
  return hipGetLastError();
}

hipError_t launch_dec_ffn(const DecFfnArgs& a, hipStream_t s) {
  if (a.rows <= 0 || (a.nsplit != 1 && a.nsplit != 2)) return hipErrorInvalidValue;
  if (!a.W1f != !a.W2f) return hipErrorInvalidValue;
  const hipError_t e = dec_lds_attr();
  if (e != hipSuccess) return e;
  const int blocks = (a.rows + DEC_ROWS - 1) / DEC_ROWS * (DEC_F / 128);
  if (a.fold.parts) {  // the residual LN2 folded in: X from the cross-attention chain's 8 slabs (tools build only)
#ifndef ICAP_TOOLS
    return hipErrorInvalidValue;
#else
    if (!a.W1f || a.W1fl || a.nsplit != 2 || a.mg.tick || !fold_ok(a.fold, DEC_H)) return hipErrorInvalidValue;
    DecFfnArgs b = a;
    b.xcd_tiles = a.xcd_tiles && ((a.rows + DEC_ROWS - 1) / DEC_ROWS) % 8 == 0;
    hipLaunchKernelGGL((dec_ffn_kernel<true, 2, DEC_H>), dim3(blocks), dim3(1024), DEC_LDS_FOLD, s, b);
    return hipGetLastError();
#endif
  }
  if (!a.W1fl != !a.W2fl || (a.W1fl && (!a.W1f || a.nsplit != 2 || a.mg.tick))) return hipErrorInvalidValue;
  if (a.W1fl) {  // hi/lo weights: the W1 lo slots after the X image
    static bool lattr = false;
    if (!lattr) {
      const hipError_t e2 = hipFuncSetAttribute((const void*)dec_ffn_kernel<true, 2, 0, true>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, DEC_LDS);
      if (e2 != hipSuccess) return e2;
      lattr = true;
    }
    hipLaunchKernelGGL((dec_ffn_kernel<true, 2, 0, true>), dim3(blocks), dim3(1024), DEC_LDS, s, a);
  } else if (a.W1f && a.nsplit == 2) hipLaunchKernelGGL((dec_ffn_kernel<true, 2>), dim3(blocks), dim3(1024), DEC_LDS_FR, s, a);
  else if (a.W1f) hipLaunchKernelGGL(dec_ffn_kernel<true>, dim3(blocks), dim3(1024), DEC_LDS_FR, s, a);
  else hipLaunchKernelGGL(dec_ffn_kernel<false>, dim3(blocks), dim3(1024), DEC_LDS, s, a);
  return hipGetLastError();
}

hipError_t launch_frag_pack(const bf16_t* W, long ldw, int ntiles, int nk, int mode, int tps, int ksl, bf16_t* out,
                            hipStream_t s) {
  if (!W || !out || ntiles <= 0 || nk <= 0 || mode < 0 || mode > 2 || (mode == 2 && (tps <= 0 || ksl <= 0)))
    return hipErrorInvalidValue;
  const long n = (long)ntiles * nk * 64;
  hipLaunchKernelGGL(frag_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, W, ldw, ntiles, nk, mode,
                     tps, ksl, out);
  return hipGetLastError();
}
