// Row-wise kernels: LayerNorm (SURVEY.md §2.1 K3 and the decoder/grid post-LNs), patch
// unfolding for the ViT patch-embed GEMM (K1), class-token rows (K2), grid feature-map
// transposition (K14), token embedding + sinusoidal PE (K7), weight packing helpers.
//
// All are HBM-streaming kernels: 16-byte vector accesses, one wave per row where a row
// reduction is needed (wave64 shuffles), fp32 arithmetic throughout.
#include "common.h"
#include "kernels.h"

namespace {

__device__ __forceinline__ void store_planes(bf16_t* base, long idx, long lo, int nsplit, float v) {
  if (nsplit == NS_F16) {
    base[idx] = f2h(v);
    return;
  }
  bf16_t hi, l;
  split_bf(v, hi, l);
  base[idx] = hi;
  if (nsplit == 2) base[idx + lo] = l;
}

// One wave per row, PER = D / 64 values per lane (D = 512 -> 8, 768 -> 12).
template <int PER>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, long ldx, int rows,
                                                        int in_group, long in_stride, long in_off,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ b, float eps,
                                                        float* out_f32, long ld_f32, bf16_t* out_bf,
                                                        long ld_bf, long bf_lo, int nsplit, unsigned* range_flag) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = PER * 64;
  const long irow = in_group ? (long)(row / in_group) * in_stride + in_off + row % in_group : (long)row;
  const float* xr = x + irow * ldx;
  float v[PER];
  // lane owns columns [4*lane + 256*c, +4)
#pragma unroll
  for (int c = 0; c < PER / 4; ++c) {
    f32x4 t = *(const f32x4*)(xr + c * 256 + lane * 4);
    v[c * 4 + 0] = t[0]; v[c * 4 + 1] = t[1]; v[c * 4 + 2] = t[2]; v[c * 4 + 3] = t[3];
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) s += v[i];
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) { const float d = v[i] - mean; q += d * d; }
  const float var = wave_sum(q) / (float)D;
  const float rstd = 1.0f / sqrtf(var + eps);
  bool bad = false;  // fp16 outputs: a value that is not finite in fp16 (a non-finite residual row included)
#pragma unroll
  for (int c = 0; c < PER / 4; ++c) {
    const int col = c * 256 + lane * 4;
    f32x4 wv = *(const f32x4*)(w + col), bv = *(const f32x4*)(b + col), y;
#pragma unroll
    for (int k = 0; k < 4; ++k) y[k] = (v[c * 4 + k] - mean) * rstd * wv[k] + bv[k];
    if (out_f32) *(f32x4*)(out_f32 + (long)row * ld_f32 + col) = y;
    if (out_bf && nsplit == NS_F16) {
      const u32x2 pk = pack16x4<true>(y);
      bad |= f16_pair_nonfinite(pk[0]) || f16_pair_nonfinite(pk[1]);
      *(u32x2*)(out_bf + (long)row * ld_bf + col) = pk;
    } else if (out_bf) {
      bf16_t h[4], l[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) split_bf(y[k], h[k], l[k]);
      bf16_t* o = out_bf + (long)row * ld_bf + col;
      *(u32x2*)o = (u32x2){(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
      if (nsplit == 2)
        *(u32x2*)(o + bf_lo) = (u32x2){(uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16)};
    }
  }
  if (range_flag && __any(bad) && lane == 0) range_flag_set(range_flag);
}

// layernorm_kernel's row statistics, output as int8 two-slice planes + the row scale (one wave per row)
template <int PER>
__global__ __launch_bounds__(256) void layernorm_i8_kernel(const float* __restrict__ x, long ldx, int rows,
                                                           int in_group, long in_stride, long in_off,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           float eps, int8_t* out,
                                                           float* __restrict__ scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = PER * 64;
  const long irow = in_group ? (long)(row / in_group) * in_stride + in_off + row % in_group : (long)row;
  const float* xr = x + irow * ldx;
  float v[PER];
#pragma unroll
  for (int c = 0; c < PER / 4; ++c) {
    f32x4 t = *(const f32x4*)(xr + c * 256 + lane * 4);
    v[c * 4 + 0] = t[0]; v[c * 4 + 1] = t[1]; v[c * 4 + 2] = t[2]; v[c * 4 + 3] = t[3];
  }
  float sm = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) sm += v[i];
  const float mean = wave_sum(sm) / (float)D;
  float qs = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) { const float d = v[i] - mean; qs += d * d; }
  const float var = wave_sum(qs) / (float)D;
  const float rstd = 1.0f / sqrtf(var + eps);
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < PER / 4; ++c) {
    const int col = c * 256 + lane * 4;
    f32x4 wv = *(const f32x4*)(w + col), bv = *(const f32x4*)(b + col);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[c * 4 + k] = (v[c * 4 + k] - mean) * rstd * wv[k] + bv[k];
      amax = fmaxf(amax, fabsf(v[c * 4 + k]));
    }
  }
  amax = wave_max(amax);
  const float inv = amax > 0.f ? 32639.f / amax : 0.f;
  if (lane == 0) scale[row] = amax / 32639.f;
  int8_t* o = out + (long)row * 2 * D;
#pragma unroll
  for (int c = 0; c < PER / 4; ++c) {
    uint32_t hi, lw;
    q2_pack4(v + c * 4, inv, hi, lw);
    const int k = c * 256 + lane * 4, off = (k >> 6) * 128 + (k & 63);  // [K/64][2][64] row image
    *(uint32_t*)(o + off) = hi;
    *(uint32_t*)(o + off + 64) = lw;
  }
}

// weight rows fp32 [N][K] -> int8 two-slice planes [N][K] + per-row scale (one wave per row, once at pack time)
__global__ __launch_bounds__(256) void pack_i8_rows_kernel(const float* __restrict__ w, int N, int K, int8_t* out,
                                                           float* __restrict__ scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const float* wr = w + (long)row * K;
  float amax = 0.f;
  for (int k = lane * 4; k < K; k += 256) {
    const f32x4 t = *(const f32x4*)(wr + k);
    amax = fmaxf(amax, fmaxf(fmaxf(fabsf(t[0]), fabsf(t[1])), fmaxf(fabsf(t[2]), fabsf(t[3]))));
  }
  amax = wave_max(amax);
  const float inv = amax > 0.f ? 32639.f / amax : 0.f;
  if (lane == 0) scale[row] = amax / 32639.f;
  for (int k = lane * 4; k < K; k += 256) {
    const f32x4 t = *(const f32x4*)(wr + k);
    const float y[4] = {t[0], t[1], t[2], t[3]};
    uint32_t hi, lw;
    q2_pack4(y, inv, hi, lw);
    int8_t* o = out + (long)row * 2 * K + (k >> 6) * 128 + (k & 63);  // [K/64][2][64] row image
    *(uint32_t*)o = hi;
    *(uint32_t*)(o + 64) = lw;
  }
}

// Post-LN residual block tail: x = LN(x + sum_s parts[s] + bias) in place, plus bf16 planes of
// the result.  Reduces the split-K partial slabs of the preceding decode GEMM (no atomics).
// x = LN(x + sum_s parts[s] + bias) in place, plus the bf16 planes of the result.  One block of
// D / 4 threads per row (each thread owns 4 consecutive columns), so a decode step's few hundred
// rows spread over every CU and each lane issues all its loads (x, bias, up to 8 partial slabs) at
// once: the kernel costs one memory latency, not one per slab.
constexpr int RLN_MAX_PARTS = 16;

template <int NT>
__global__ __launch_bounds__(NT) void residual_layernorm_kernel(const float* xin, float* x, int rows,
                                                                const float* __restrict__ parts, int nparts,
                                                                long part_stride, const float* __restrict__ bias,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ b, float eps,
                                                                bf16_t* out_bf, long bf_lo, int nsplit,
                                                                DropCfg drop, int site) {
  constexpr int D = NT * 4, NW = NT / 64;
  __shared__ float red[2][NW];
  const int row = blockIdx.x, col = threadIdx.x * 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* xr = x + (long)row * D;  // (xin: the residual input when it is not x itself)
  f32x4 pp[RLN_MAX_PARTS];
#pragma unroll
  for (int s = 0; s < RLN_MAX_PARTS; ++s)
    // (non-temporal, round 5: the slabs are read once - with the producers' nt slab stores, decode 10.93-10.95 ->
    // 10.70-10.86 ms on one box, profiles/r05/slab_nt_ab.txt)
    pp[s] = s < nparts ? __builtin_nontemporal_load((const f32x4*)(parts + s * part_stride + (long)row * D + col))
                       : (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 v = *(const f32x4*)(xin + (long)row * D + col);
  const f32x4 bb = bias ? *(const f32x4*)(bias + col) : (f32x4){0.f, 0.f, 0.f, 0.f};
  const f32x4 wv = *(const f32x4*)(w + col), bv = *(const f32x4*)(b + col);
  if (drop.thr == 0) {
    v += bb;
#pragma unroll
    for (int s = 0; s < RLN_MAX_PARTS; ++s) v += pp[s];
  } else {  // x + dropout(sublayer output) (TransformerDecoderLayer dropout1 / 2 / 3)
    f32x4 o = bb;
#pragma unroll
    for (int s = 0; s < RLN_MAX_PARTS; ++s) o += pp[s];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] += o[k] * drop_mul(drop, site, row, drop.pos, col + k);
  }
  float sm = wave_sum(v[0] + v[1] + v[2] + v[3]);
  if (lane == 0) red[0][wave] = sm;
  __syncthreads();
  sm = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) sm += red[0][i];
  const float mean = sm / (float)D;
  f32x4 d = v - mean;
  float q = wave_sum(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]);
  if (lane == 0) red[1][wave] = q;
  __syncthreads();
  q = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) q += red[1][i];
  const float rstd = 1.0f / sqrtf(q / (float)D + eps);
  f32x4 y;
  bf16_t h[4], l[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    y[k] = d[k] * rstd * wv[k] + bv[k];
    split_bf(y[k], h[k], l[k]);
  }
  *(f32x4*)(xr + col) = y;
  bf16_t* o = out_bf + (long)row * D + col;
  *(u32x2*)o = (u32x2){(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
  if (nsplit == 2)
    *(u32x2*)(o + bf_lo) = (u32x2){(uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16)};
}

// img (B,C,HW,HW) -> rows (B*np, C*P*P) in (c, kh, kw) order == torchvision conv_proj weight order.
__global__ void im2col_kernel(const float* __restrict__ img, int B, int C, int HW, int P, bf16_t* out,
                              long lo, int nsplit) {
  const int g = HW / P, np = g * g, K = C * P * P, chunks = K / 8;
  const long total = (long)B * np * chunks;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % chunks);
    const long r = i / chunks;
    const int p = (int)(r % np), b = (int)(r / np);
    const int k0 = ch * 8, c = k0 / (P * P), kh = (k0 / P) % P, kw = k0 % P;
    const int y = (p / g) * P + kh, xx = (p % g) * P + kw;
    const float* src = img + (((long)b * C + c) * HW + y) * HW + xx;
    f32x4 a = *(const f32x4*)src, bq = *(const f32x4*)(src + 4);
    float v[8] = {a[0], a[1], a[2], a[3], bq[0], bq[1], bq[2], bq[3]};
    if (nsplit == NS_F16) {
      const u32x2 x0 = pack16x4<true>(a), x1 = pack16x4<true>(bq);
      *(u32x4*)(out + r * K + k0) = (u32x4){x0[0], x0[1], x1[0], x1[1]};
      continue;
    }
    bf16_t h[8], l[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) split_bf(v[k], h[k], l[k]);
    u32x4 H, L;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      H[k] = (uint32_t)h[2 * k] | ((uint32_t)h[2 * k + 1] << 16);
      L[k] = (uint32_t)l[2 * k] | ((uint32_t)l[2 * k + 1] << 16);
    }
    *(u32x4*)(out + r * K + k0) = H;
    if (nsplit == 2) *(u32x4*)(out + lo + r * K + k0) = L;
  }
}

__global__ void cls_rows_kernel(const float* cls, const float* pos, float* x, int B, int tokens, int D) {
  const long total = (long)B * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int d = (int)(i % D), b = (int)(i / D);
    x[(long)b * tokens * D + d] = cls[d] + pos[d];
  }
}

// feats (B, C, S) -> rows (B*S, C) as bf16 planes
__global__ void nchw_to_rows_kernel(const float* __restrict__ f, int B, int C, int S, bf16_t* out, long lo,
                                    int nsplit) {
  const long total = (long)B * S * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long r = i / C;
    const int s = (int)(r % S), b = (int)(r / S);
    store_planes(out, i, lo, nsplit, f[((long)b * C + c) * S + s]);
  }
}

// x[r] = emb[tok[r]] * scale + pe[t0 + r % T]  (TransformerDecoder.forward, vit:166-169)
__global__ void embed_kernel(const int32_t* tok, long tok_ld, int fixed_tok, int rows, int T, int t0,
                             const float* emb, const float* pe, int D, float scale, float* x, bf16_t* a, long lo,
                             int nsplit, DropCfg drop) {
  const long total = (long)rows * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int d = (int)(i % D), r = (int)(i / D);
    const int t = tok ? tok[(long)(r / T) * tok_ld + r % T] : fixed_tok;
    float v = emb[(long)t * D + d] * scale + pe[(long)(t0 + r % T) * D + d];
    if (drop.thr) v *= drop_mul(drop, 0, r / T, t0 + r % T, d);  // PositionalEncoding's dropout
    x[i] = v;
    store_planes(a, i, lo, nsplit, v);
  }
}

__global__ void fill_u8_kernel(uint8_t* p, long n, uint8_t value) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = value;
}

__global__ void fill_col_kernel(int32_t* ids, int B, long ld, int col, int value) {
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x) ids[(long)b * ld + col] = value;
}

// Stop test of one chunk of a stop-aware decode (round 6): *flag = 1 when some id column in [col0, col1) holds the end
// token in every row (greedy: _greedy_search breaks after the first such step, models/vit_transformer_model.py:321-323)
// or, with fin, when every row has finished (sampling: scst_loss.py:246-249); flag is host-mapped memory the host reads
// after the chunk's event.  One block.
__global__ void stop_scan_kernel(const int32_t* ids, int B, long ld, int col0, int col1, int end, const uint8_t* fin,
                                 int* flag) {
  __shared__ int live[65];  // [c]: some row's token in column col0 + c is not end; [64]: some row has not finished
  const int nc = col1 - col0;
  for (int i = threadIdx.x; i < 65; i += blockDim.x) live[i] = 0;
  __syncthreads();
  for (long i = threadIdx.x; i < (long)B * nc; i += blockDim.x) {
    const int b = (int)(i / nc), c = (int)(i - (long)b * nc);
    if (ids[(long)b * ld + col0 + c] != end) live[c] = 1;
  }
  if (fin)
    for (int b = threadIdx.x; b < B; b += blockDim.x)
      if (!fin[b]) live[64] = 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    int stop = 0;
    if (fin) stop = !live[64];
    else
      for (int c = 0; c < nc; ++c) stop |= !live[c];
    __hip_atomic_store(flag, stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
  }
}

// The columns a stopped decode did not compute (steps >= t0): ids = end (the reference's generated sequence ends
// before them; the stop rules keep it), sampled log-probs = 0 (every row had finished: masked_fill semantics)
__global__ void stop_tail_kernel(int32_t* ids, int B, int L, int t0, int end, float* logp) {
  const int n = L - 1 - t0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (long)B * n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / n), t = t0 + (int)(i - (long)b * n);
    ids[(long)b * L + t + 1] = end;
    if (logp) logp[(long)b * (L - 1) + t] = 0.f;
  }
}

__global__ void split_f32_kernel(const float* src, long n, bf16_t* dst, long lo, int nsplit) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    store_planes(dst, i, lo, nsplit, src[i]);
}

// planes (hi at src, lo at src + lo when nsplit == 2) -> fp32 hi + lo
__global__ void planes_to_f32_kernel(const bf16_t* src, long lo, long n, int nsplit, float* dst) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dst[i] = nsplit == 2 ? bf2f(src[i]) + bf2f(src[i + lo]) : bf2f(src[i]);
}

// fp16 hi/lo planes (the ICAP_PREC_F16 trunk output; slo = 0: one fp16 plane) -> bf16 hi/lo planes of the same values
// (the bf16x2 Grid tail's input), and optionally their fp32 sum (the trunk features); 4 elements per thread
__global__ void f16planes_to_bf16_kernel(const bf16_t* src, long slo, long n4, bf16_t* dst, long dlo, float* f32) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const u32x2 h = *(const u32x2*)(src + 4 * i), l = slo ? *(const u32x2*)(src + 4 * i + slo) : (u32x2){0u, 0u};
    f32x4 v;
    bf16_t oh[4], ol[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sh = (r & 1) * 16;
      v[r] = h2f((bf16_t)((h[r >> 1] >> sh) & 0xffff)) + h2f((bf16_t)((l[r >> 1] >> sh) & 0xffff));
      split_bf(v[r], oh[r], ol[r]);
    }
    *(u32x2*)(dst + 4 * i) = (u32x2){(uint32_t)oh[0] | ((uint32_t)oh[1] << 16), (uint32_t)oh[2] | ((uint32_t)oh[3] << 16)};
    *(u32x2*)(dst + 4 * i + dlo) =
        (u32x2){(uint32_t)ol[0] | ((uint32_t)ol[1] << 16), (uint32_t)ol[2] | ((uint32_t)ol[3] << 16)};
    if (f32) *(f32x4*)(f32 + 4 * i) = v;
  }
}

__global__ void f32_to_bf16_kernel(const float* src, bf16_t* dst, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dst[i] = f2bf(src[i]);
}

// wk rows [h*hd + i][d] (i < hd, d < D)  ->  dst[h][d][i]   (W_h^T packing for the key absorption)
// lo_plane: write bf16(w - bf16(w)) instead (the low plane of hi/lo decoder weights)
__global__ void transpose_heads_kernel(const float* wk, int H, int hd, int D, bf16_t* dst, int lo_plane) {
  const long total = (long)H * hd * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ii = (int)(i % hd);
    const long r = i / hd;
    const int d = (int)(r % D), h = (int)(r / D);
    const float w = wk[((long)h * hd + ii) * D + d];
    bf16_t hi, lo;
    split_bf(w, hi, lo);
    dst[i] = lo_plane ? lo : hi;
  }
}

inline int grid_for(long n, int block = 256) {
  long g = (n + block - 1) / block;
  return (int)(g < 8192 ? (g < 1 ? 1 : g) : 8192);
}

}  // namespace

hipError_t launch_layernorm(const float* x, long ldx, int rows, int D, int in_group, long in_stride,
                            long in_off, const float* w, const float* b, float eps, float* out_f32,
                            long ld_f32, bf16_t* out_bf, long ld_bf, long bf_lo, int nsplit,
                            hipStream_t s, unsigned* range_flag) {
  dim3 grid((rows + 3) / 4);
  if (D == 512)
    hipLaunchKernelGGL(layernorm_kernel<8>, grid, dim3(256), 0, s, x, ldx, rows, in_group, in_stride, in_off,
                       w, b, eps, out_f32, ld_f32, out_bf, ld_bf, bf_lo, nsplit, range_flag);
  else if (D == 768)
    hipLaunchKernelGGL(layernorm_kernel<12>, grid, dim3(256), 0, s, x, ldx, rows, in_group, in_stride, in_off,
                       w, b, eps, out_f32, ld_f32, out_bf, ld_bf, bf_lo, nsplit, range_flag);
  else if (D == 256)
    hipLaunchKernelGGL(layernorm_kernel<4>, grid, dim3(256), 0, s, x, ldx, rows, in_group, in_stride, in_off,
                       w, b, eps, out_f32, ld_f32, out_bf, ld_bf, bf_lo, nsplit, range_flag);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_layernorm_i8(const float* x, long ldx, int rows, int D, int in_group, long in_stride, long in_off,
                               const float* w, const float* b, float eps, int8_t* out, float* scale, hipStream_t s) {
  dim3 grid((rows + 3) / 4);
  if (D == 512)
    hipLaunchKernelGGL(layernorm_i8_kernel<8>, grid, dim3(256), 0, s, x, ldx, rows, in_group, in_stride, in_off, w,
                       b, eps, out, scale);
  else if (D == 768)
    hipLaunchKernelGGL(layernorm_i8_kernel<12>, grid, dim3(256), 0, s, x, ldx, rows, in_group, in_stride, in_off, w,
                       b, eps, out, scale);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_pack_i8_rows(const float* w, int N, int K, int8_t* out, float* scale, hipStream_t s) {
  if (N <= 0 || K <= 0 || K % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_i8_rows_kernel, dim3((N + 3) / 4), dim3(256), 0, s, w, N, K, out, scale);
  return hipGetLastError();
}

hipError_t launch_residual_layernorm(float* x, int rows, int D, const float* parts, int nparts, long part_stride,
                                    const float* bias, const float* w, const float* b, float eps, bf16_t* out_bf,
                                    long bf_lo, int nsplit, hipStream_t s, DropCfg drop, int site,
                                    const float* x_in) {
  if (nparts < 0 || nparts > RLN_MAX_PARTS || rows <= 0) return hipErrorInvalidValue;
  dim3 grid(rows);
  const float* xi = x_in ? x_in : x;
  if (D == 512)
    hipLaunchKernelGGL(residual_layernorm_kernel<128>, grid, dim3(128), 0, s, xi, x, rows, parts, nparts, part_stride,
                       bias, w, b, eps, out_bf, bf_lo, nsplit, drop, site);
  else if (D == 768)
    hipLaunchKernelGGL(residual_layernorm_kernel<192>, grid, dim3(192), 0, s, xi, x, rows, parts, nparts, part_stride,
                       bias, w, b, eps, out_bf, bf_lo, nsplit, drop, site);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_im2col_patches(const float* img, int B, int C, int HW, int P, bf16_t* out, long lo,
                                 int nsplit, hipStream_t s) {
  if (HW % P || P % 8) return hipErrorInvalidValue;
  const long n = (long)B * (HW / P) * (HW / P) * (C * P * P / 8);
  hipLaunchKernelGGL(im2col_kernel, dim3(grid_for(n)), dim3(256), 0, s, img, B, C, HW, P, out, lo, nsplit);
  return hipGetLastError();
}

hipError_t launch_cls_rows(const float* cls, const float* pos, float* x, int B, int tokens, int D,
                           hipStream_t s) {
  hipLaunchKernelGGL(cls_rows_kernel, dim3(grid_for((long)B * D)), dim3(256), 0, s, cls, pos, x, B, tokens, D);
  return hipGetLastError();
}

hipError_t launch_nchw_to_rows(const float* feats, int B, int C, int S, bf16_t* out, long lo, int nsplit,
                               hipStream_t s) {
  hipLaunchKernelGGL(nchw_to_rows_kernel, dim3(grid_for((long)B * C * S)), dim3(256), 0, s, feats, B, C, S,
                     out, lo, nsplit);
  return hipGetLastError();
}

hipError_t launch_embed(const int32_t* tok, long tok_ld, int fixed_tok, int rows, int T, int t0, const float* emb,
                        const float* pe, int D, float scale, float* x, bf16_t* a, long lo, int nsplit, hipStream_t s,
                        DropCfg drop) {
  hipLaunchKernelGGL(embed_kernel, dim3(grid_for((long)rows * D)), dim3(256), 0, s, tok, tok_ld, fixed_tok, rows, T,
                     t0, emb, pe, D, scale, x, a, lo, nsplit, drop);
  return hipGetLastError();
}

hipError_t launch_fill_u8(uint8_t* p, long n, uint8_t value, hipStream_t s) {
  hipLaunchKernelGGL(fill_u8_kernel, dim3(grid_for(n)), dim3(256), 0, s, p, n, value);
  return hipGetLastError();
}

hipError_t launch_stop_scan(const int32_t* ids, int B, long ld, int col0, int col1, int end, const uint8_t* fin,
                            int* flag, hipStream_t s) {
  if (col1 <= col0 || col1 - col0 > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(stop_scan_kernel, dim3(1), dim3(256), 0, s, ids, B, ld, col0, col1, end, fin, flag);
  return hipGetLastError();
}

hipError_t launch_stop_tail(int32_t* ids, int B, int L, int t0, int end, float* logp, hipStream_t s) {
  if (t0 >= L - 1) return hipSuccess;
  hipLaunchKernelGGL(stop_tail_kernel, dim3(grid_for((long)B * (L - 1 - t0))), dim3(256), 0, s, ids, B, L, t0, end, logp);
  return hipGetLastError();
}

hipError_t launch_fill_col(int32_t* ids, int B, long ld, int col, int value, hipStream_t s) {
  hipLaunchKernelGGL(fill_col_kernel, dim3(grid_for(B)), dim3(256), 0, s, ids, B, ld, col, value);
  return hipGetLastError();
}

hipError_t launch_split_f32(const float* src, long n, bf16_t* dst, long lo, int nsplit, hipStream_t s) {
  hipLaunchKernelGGL(split_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, src, n, dst, lo, nsplit);
  return hipGetLastError();
}

hipError_t launch_f16planes_to_bf16(const bf16_t* src, long slo, long n, bf16_t* dst, long dlo, float* f32,
                                   hipStream_t s) {
  if (n % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(f16planes_to_bf16_kernel, dim3(grid_for(n / 4)), dim3(256), 0, s, src, slo, n / 4, dst, dlo, f32);
  return hipGetLastError();
}

hipError_t launch_planes_to_f32(const bf16_t* src, long lo, long n, int nsplit, float* dst, hipStream_t s) {
  hipLaunchKernelGGL(planes_to_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, src, lo, n, nsplit, dst);
  return hipGetLastError();
}

hipError_t launch_f32_to_f16(const float* src, bf16_t* dst, long n, hipStream_t s) {
  hipLaunchKernelGGL(split_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, src, n, dst, 0L, NS_F16);
  return hipGetLastError();
}

hipError_t launch_f32_to_bf16(const float* src, bf16_t* dst, long n, hipStream_t s) {
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, s, src, dst, n);
  return hipGetLastError();
}

hipError_t launch_transpose_heads_bf16(const float* wk, int H, int hd, int D, bf16_t* dst, hipStream_t s,
                                       int lo_plane) {
  hipLaunchKernelGGL(transpose_heads_kernel, dim3(grid_for((long)H * hd * D)), dim3(256), 0, s, wk, H, hd, D, dst,
                     lo_plane);
  return hipGetLastError();
}
