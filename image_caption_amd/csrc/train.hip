// Kernels of the decoder's training pass (SCST's teacher-forced log-prob recompute and its backward,
// utils/scst_loss.py:124-128 / the reference's autograd through scst_loss.py:210-254 and
// scripts/train_vit_transformer_scst_optimized.py:255-261): the forward saves what the backward needs,
// the backward produces the gradients of every TransformerDecoder parameter and of the memory.
//
// Every product is fp32 (v_mfma_f32_16x16x4_f32), as PyTorch's fp32 autograd computes them.
// One generic strided GEMM serves every forward, input-gradient, weight-gradient and per-(image, head)
// attention product: C[m][n] = alpha * sum_k A[m][k] B[n][k] (+ beta C) (+ bias[n]) (relu), with
// element strides on both index axes of A, B and C (transposes are strides) and two batch levels.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int TG_BM = 64, TG_BN = 64, TG_BK = 32, TG_LD = TG_BK + 1;  // fp32 LDS rows, padded

// One operand's 64 x 32 tile (rows r0.., k0..) into registers: 8 values per thread.  vec: 16-B loads of 4
// consecutive elements along the contiguous axis (k, or the rows of a transposed operand), else scalar
// loads walking the contiguous axis with consecutive threads.
struct TgTile {
  f32x4 v[2];
};
__device__ __forceinline__ void tg_load(const float* src, long s_row, long s_k, int rows, int K, int r0, int k0,
                                        int mode, TgTile& t) {
  const int tid = threadIdx.x;
  if (mode == 1) {  // k contiguous, 16-B aligned: thread -> row tid / 8 (+32), k = 4 (tid % 8)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (tid >> 3) + 32 * i, k = (tid & 7) * 4;
      t.v[i] = (r0 + r < rows && k0 + k < K) ? *(const f32x4*)(src + (long)(r0 + r) * s_row + k0 + k)
                                             : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  } else if (mode == 2) {  // rows contiguous (transposed), 16-B aligned: thread -> rows 4 (tid % 16), k = tid / 16 (+16)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (tid & 15) * 4, k = (tid >> 4) + 16 * i;
      t.v[i] = (r0 + r < rows && k0 + k < K) ? *(const f32x4*)(src + (long)(r0 + r) + (long)(k0 + k) * s_k)
                                             : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int r, k;
      if (s_k == 1) {
        k = tid & 31;
        r = (tid >> 5) + 8 * i;
      } else {
        r = tid & 63;
        k = (tid >> 6) + 4 * i;
      }
      t.v[i >> 2][i & 3] = (r0 + r < rows && k0 + k < K) ? src[(long)(r0 + r) * s_row + (long)(k0 + k) * s_k] : 0.f;
    }
  }
}
__device__ __forceinline__ void tg_store(const TgTile& t, int mode, bool k_unit, float (*dst)[TG_LD]) {
  const int tid = threadIdx.x;
  if (mode == 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[(tid >> 3) + 32 * i][(tid & 7) * 4 + e] = t.v[i][e];
  } else if (mode == 2) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[(tid & 15) * 4 + e][(tid >> 4) + 16 * i] = t.v[i][e];
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = k_unit ? (tid >> 5) + 8 * i : tid & 63, k = k_unit ? tid & 31 : (tid >> 6) + 4 * i;
      dst[r][k] = t.v[i >> 2][i & 3];
    }
  }
}

// 64 x 64 block tile, 4 waves of 32 x 32 (2 x 2 tiles of v_mfma_f32_16x16x4_f32: exact fp32 products,
// fp32 accumulation - the precision of PyTorch's fp32 GEMMs; a bf16 hi/lo split of both operands was
// measured at 1.9e-3 relative on weight gradients that sum 3712 rows, against 5e-4 for fp32 autograd).
// The next k-tile is loaded into registers while the current one is multiplied.  ksplit > 1: block z
// covers one K range and writes its raw sums to part[split][M][N] (tgemm_reduce_kernel finishes).
__global__ __launch_bounds__(256) void tgemm_kernel(TGemmArgs p, int amode, int bmode) {
  __shared__ float As[TG_BM][TG_LD];
  __shared__ float Bs[TG_BN][TG_LD];
  const int ks = p.ksplit, split = blockIdx.z % ks, z = blockIdx.z / ks;
  const int b1 = z / p.nb2, b2 = z - b1 * p.nb2;
  const float* A = p.A + b1 * p.sab1 + b2 * p.sab2;
  const float* B = p.B + b1 * p.sbb1 + b2 * p.sbb2;
  const int m0 = blockIdx.y * TG_BM, n0 = blockIdx.x * TG_BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int kc = ((p.K + ks - 1) / ks + TG_BK - 1) / TG_BK * TG_BK;
  const int kb = split * kc, ke = min(p.K, kb + kc);
  f32x4 acc[2][2] = {};
  TgTile ta, tb;
  if (kb < ke) {
    tg_load(A, p.sam, p.sak, p.M, ke, m0, kb, amode, ta);
    tg_load(B, p.sbn, p.sbk, p.N, ke, n0, kb, bmode, tb);
  }
  for (int k0 = kb; k0 < ke; k0 += TG_BK) {
    tg_store(ta, amode, p.sak == 1, As);
    tg_store(tb, bmode, p.sbk == 1, Bs);
    __syncthreads();
    if (k0 + TG_BK < ke) {
      tg_load(A, p.sam, p.sak, p.M, ke, m0, k0 + TG_BK, amode, ta);
      tg_load(B, p.sbn, p.sbk, p.N, ke, n0, k0 + TG_BK, bmode, tb);
    }
#pragma unroll
    for (int kk = 0; kk < TG_BK; kk += 4) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = As[wm + 16 * i + fr][kk + fq];
        b[i] = Bs[wn + 16 * i + fr][kk + fq];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  if (ks > 1) {  // raw partial sums
    float* P = p.part + (long)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn + 16 * j + fr;
        if (n >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm + 16 * i + 4 * fq + r;
          if (m < p.M) P[(long)m * p.N + n] = acc[i][j][r];
        }
      }
    return;
  }
  float* C = p.C + b1 * p.scb1 + b2 * p.scb2;
  // lane holds C[m = 4 fq + r][n = fr] of each 16 x 16 tile
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + 16 * j + fr;
      if (n >= p.N) continue;
      const float bias = p.bias ? p.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + 4 * fq + r;
        if (m >= p.M) continue;
        float* c = C + (long)m * p.scm + (long)n * p.scn;
        float v = p.alpha * acc[i][j][r] + bias;
        if (p.beta != 0.f) v += p.beta * *c;
        if (p.relu) v = fmaxf(v, 0.f);
        *c = v;
      }
    }
}

// C = alpha * sum over splits of part[s] (+ beta C) (+ bias) (relu), splits summed in order
__global__ void tgemm_reduce_kernel(TGemmArgs p) {
  const long n_el = (long)p.M * p.N;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n_el; i += (long)gridDim.x * blockDim.x) {
    const int m = (int)(i / p.N), n = (int)(i - (long)m * p.N);
    float v = 0.f;
    for (int s = 0; s < p.ksplit; ++s) v += p.part[(long)s * n_el + i];
    float* c = p.C + (long)m * p.scm + (long)n * p.scn;
    v = p.alpha * v + (p.bias ? p.bias[n] : 0.f);
    if (p.beta != 0.f) v += p.beta * *c;
    if (p.relu) v = fmaxf(v, 0.f);
    *c = v;
  }
}

// softmax over rows of length n in place (one wave per row); causal: row index within a group of T
// query rows is the query position t, keys j > t get probability 0 (torch's causal mask)
__global__ __launch_bounds__(256) void softmax_rows_kernel(float* x, long rows, int n, int T, int causal) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float* r = x + row * n;
  const int lim = causal ? (int)(row % T) + 1 : n;
  float m = -INFINITY;
  for (int j = lane; j < lim; j += 64) m = fmaxf(m, r[j]);
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < lim; j += 64) s += __expf(r[j] - m);
  s = wave_sum(s);
  const float inv = 1.f / s;
  for (int j = lane; j < n; j += 64) r[j] = j < lim ? __expf(r[j] - m) * inv : 0.f;
}

// dS = P * (dP - sum_j P dP), in place on dP (one wave per row)
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const float* P, float* dP, long rows, int n) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* p = P + row * n;
  float* d = dP + row * n;
  float s = 0.f;
  for (int j = lane; j < n; j += 64) s += p[j] * d[j];
  s = wave_sum(s);
  for (int j = lane; j < n; j += 64) d[j] = p[j] * (d[j] - s);
}

// y = LN(a + b) over D = 64 * PER columns (one wave per row); saves xhat and rstd for the backward
template <int PER>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* a, const float* b, const float* w,
                                                     const float* bias, float eps, int rows, float* y, float* xhat,
                                                     float* rstd) {
  constexpr int D = 64 * PER;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const long o = (long)row * D + lane + 64 * i;
    v[i] = a[o] + b[o];
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] -= mean;
    q += v[i] * v[i];
  }
  const float rs = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const long o = (long)row * D + c;
    const float xh = v[i] * rs;
    xhat[o] = xh;
    y[o] = xh * w[c] + bias[c];
  }
  if (lane == 0) rstd[row] = rs;
}

// LayerNorm backward in place: dy -> dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dy w;
// prod = dy * xhat (its column sums are the weight gradient)
template <int PER>
__global__ __launch_bounds__(256) void ln_bwd_kernel(float* dy, const float* xhat, const float* rstd, const float* w,
                                                     int rows, float* prod) {
  constexpr int D = 64 * PER;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  float g[PER], xh[PER];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const long o = (long)row * D + c;
    const float d = dy[o];
    xh[i] = xhat[o];
    prod[o] = d * xh[i];
    g[i] = d * w[c];
    s1 += g[i];
    s2 += g[i] * xh[i];
  }
  s1 = wave_sum(s1) / (float)D;
  s2 = wave_sum(s2) / (float)D;
  const float rs = rstd[row];
#pragma unroll
  for (int i = 0; i < PER; ++i) dy[(long)row * D + lane + 64 * i] = rs * (g[i] - s1 - xh[i] * s2);
}

// column sums of a (rows, n) matrix with row stride ld, two passes: partial[chunk][n] over row chunks,
// then the chunks in order (deterministic); dst (+)= the sums
constexpr int CS_CHUNKS = 64;
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* src, long ld, int rows, int n,
                                                             float* part) {
  const int c = blockIdx.x * 256 + threadIdx.x, chunk = blockIdx.y;
  if (c >= n) return;
  const int per = (rows + CS_CHUNKS - 1) / CS_CHUNKS, r0 = chunk * per, r1 = min(rows, r0 + per);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += src[(long)r * ld + c];
  part[(long)chunk * n + c] = s;
}
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* part, int n, float* dst, int accumulate) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n) return;
  float s = 0.f;
  for (int k = 0; k < CS_CHUNKS; ++k) s += part[(long)k * n + c];
  dst[c] = accumulate ? dst[c] + s : s;
}

__global__ void relu_bwd_kernel(float* dh, const float* h, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    if (!(h[i] > 0.f)) dh[i] = 0.f;
}

// x[m][c] = emb[tok[m]][c] * scale + pe[t][c], m = b * T + t, tok = ids[b][t] (row stride ld)
__global__ void embed_fwd_kernel(const int32_t* ids, long ld, int B, int T, const float* emb, const float* pe, int D,
                                 float scale, float* x) {
  const long n = (long)B * T * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long m = i / D;
    const int c = (int)(i - m * D), b = (int)(m / T), t = (int)(m - (long)b * T);
    x[i] = emb[(long)ids[(long)b * ld + t] * D + c] * scale + pe[(long)t * D + c];
  }
}

// dE[v][c] = scale * sum over rows m with tok[m] == v of dx[m][c], in row order (deterministic).  One workgroup
// per row m; the row that holds the FIRST occurrence of its token owns that token's dE row and sums the rows with
// the same token from m on; the others exit.  O(M^2) id compares + one read of dx, against O(V M D) for a
// workgroup per vocabulary row.  Rows of tokens that do not occur are zeroed by the launcher.
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int32_t* ids, long ld, int B, int T, const float* dx,
                                                        int D, int V, float scale, float* dE) {
  const int m = blockIdx.x, M = B * T;
  auto tok_of = [&](int r) { return ids[(long)(r / T) * ld + r % T]; };
  const int v = tok_of(m);
  if (v < 0 || v >= V) return;  // ids outside [0, V) break the call contract: never write outside dE
  int seen = 0;
  for (int r = threadIdx.x; r < m; r += 256) seen |= tok_of(r) == v;
  if (__syncthreads_or(seen)) return;
  for (int c = threadIdx.x; c < D; c += 256) {
    float s = 0.f;
    for (int r = m; r < M; ++r)
      if (tok_of(r) == v) s += dx[(long)r * D + c];
    dE[(long)v * D + c] = s * scale;
  }
}

// log p(ids[b][t+1] | prefix) from logits (B*T, V), zero after the row's first <end> among ids[b][1..t]
// (utils/scst_loss.py masked_token_logp, reference scst_loss.py:236-239); saves logsumexp
__global__ __launch_bounds__(256) void logp_fwd_kernel(const float* logits, int V, const int32_t* ids, long ld, int B,
                                                       int T, int end_token, float* logp, float* lse) {
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (m >= B * T) return;
  const int b = m / T, t = m - b * T;
  const float* r = logits + (long)m * V;
  float mx = -INFINITY;
  for (int j = lane; j < V; j += 64) mx = fmaxf(mx, r[j]);
  mx = wave_max(mx);
  float s = 0.f;
  for (int j = lane; j < V; j += 64) s += __expf(r[j] - mx);
  const float l = mx + logf(wave_sum(s));
  if (lane == 0) {
    bool fin = false;
    for (int k = 1; k <= t; ++k) fin |= ids[(long)b * ld + k] == end_token;
    const int tgt = ids[(long)b * ld + t + 1];
    logp[m] = fin ? 0.f : r[tgt] - l;
    lse[m] = l;
  }
}

__global__ __launch_bounds__(256) void logp_bwd_kernel(const float* logits, const float* lse, const float* dlogp,
                                                       int V, const int32_t* ids, long ld, int B, int T, int end_token,
                                                       float* dlogits) {
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (m >= B * T) return;
  const int b = m / T, t = m - b * T;
  bool fin = false;
  for (int k = 1; k <= t; ++k) fin |= ids[(long)b * ld + k] == end_token;
  const int tgt = ids[(long)b * ld + t + 1];
  const float g = fin ? 0.f : dlogp[m], l = lse[m];
  for (int j = lane; j < V; j += 64)
    dlogits[(long)m * V + j] = g * ((j == tgt ? 1.f : 0.f) - __expf(logits[(long)m * V + j] - l));
}

// dropout masks of the training pass (common.h): out = x * mask over a (B*T, n) matrix (row m = image
// m / T, position m % T, index = column) or over attention probabilities (B, H, T, Tk): image, head, query
// position, key -> index head * stride + key.  out may alias x.
__global__ void drop_rows_kernel(const float* x, float* out, int T, int n, long total, DropCfg d, int site) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long m = i / n;
    const int c = (int)(i - m * n);
    out[i] = x[i] * drop_mul(d, site, (int)(m / T), (int)(m % T), c);
  }
}
__global__ void drop_attn_kernel(const float* x, float* out, int H, int T, int Tk, int stride, long total, DropCfg d,
                                 int site) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long row = i / Tk;
    const int j = (int)(i - row * Tk), t = (int)(row % T), h = (int)((row / T) % H), b = (int)(row / ((long)T * H));
    out[i] = x[i] * drop_mul(d, site, b, t, h * stride + j);
  }
}

int ew_grid(long n) { return (int)std::min<long>((n + 255) / 256, 8192); }

}  // namespace

// operand load form: 1 = 16-B loads along k, 2 = 16-B loads along the rows (transposed), 0 = scalar
static int tg_mode(const float* base, long s_row, long s_k, long sb1, long sb2) {
  const bool al = ((uintptr_t)base & 15) == 0 && sb1 % 4 == 0 && sb2 % 4 == 0;
  if (al && s_k == 1 && s_row % 4 == 0) return 1;
  if (al && s_row == 1 && s_k % 4 == 0) return 2;
  return 0;
}

hipError_t launch_tgemm(const TGemmArgs& a0, int nbatch, hipStream_t s) {
  TGemmArgs a = a0;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0 || nbatch <= 0 || a.nb2 <= 0 || nbatch % a.nb2) return hipErrorInvalidValue;
  if (a.ksplit < 1) a.ksplit = 1;
  if (a.ksplit > 1 && (nbatch != 1 || !a.part)) return hipErrorInvalidValue;
  int amode = tg_mode(a.A, a.sam, a.sak, a.sab1, a.sab2), bmode = tg_mode(a.B, a.sbn, a.sbk, a.sbb1, a.sbb2);
  // the vector forms need whole 4-groups inside the tile's bounds checks
  if (amode == 1 && a.K % 4) amode = 0;
  if (amode == 2 && a.M % 4) amode = 0;
  if (bmode == 1 && a.K % 4) bmode = 0;
  if (bmode == 2 && a.N % 4) bmode = 0;
  hipLaunchKernelGGL(tgemm_kernel, dim3((a.N + TG_BN - 1) / TG_BN, (a.M + TG_BM - 1) / TG_BM, nbatch * a.ksplit),
                     dim3(256), 0, s, a, amode, bmode);
  if (a.ksplit > 1)
    hipLaunchKernelGGL(tgemm_reduce_kernel, dim3(ew_grid((long)a.M * a.N)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_softmax_rows(float* x, long rows, int n, int T, int causal, hipStream_t s) {
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, x, rows, n, T, causal);
  return hipGetLastError();
}

hipError_t launch_softmax_bwd(const float* P, float* dP, long rows, int n, hipStream_t s) {
  hipLaunchKernelGGL(softmax_bwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, P, dP, rows, n);
  return hipGetLastError();
}

hipError_t launch_ln_fwd(const float* a, const float* b, const float* w, const float* bias, float eps, int rows, int D,
                         float* y, float* xhat, float* rstd, hipStream_t s) {
  if (D != 512) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ln_fwd_kernel<8>, dim3((rows + 3) / 4), dim3(256), 0, s, a, b, w, bias, eps, rows, y, xhat, rstd);
  return hipGetLastError();
}

hipError_t launch_ln_bwd(float* dy, const float* xhat, const float* rstd, const float* w, int rows, int D, float* prod,
                         hipStream_t s) {
  if (D != 512) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ln_bwd_kernel<8>, dim3((rows + 3) / 4), dim3(256), 0, s, dy, xhat, rstd, w, rows, prod);
  return hipGetLastError();
}

size_t colsum_scratch_floats(int n) { return (size_t)CS_CHUNKS * n; }

hipError_t launch_colsum(const float* src, long ld, int rows, int n, float* part, float* dst, int accumulate,
                         hipStream_t s) {
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((n + 255) / 256, CS_CHUNKS), dim3(256), 0, s, src, ld, rows, n, part);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((n + 255) / 256), dim3(256), 0, s, part, n, dst, accumulate);
  return hipGetLastError();
}

hipError_t launch_relu_bwd(float* dh, const float* h, long n, hipStream_t s) {
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(ew_grid(n)), dim3(256), 0, s, dh, h, n);
  return hipGetLastError();
}

hipError_t launch_embed_fwd(const int32_t* ids, long ld, int B, int T, const float* emb, const float* pe, int D,
                            float scale, float* x, hipStream_t s) {
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(ew_grid((long)B * T * D)), dim3(256), 0, s, ids, ld, B, T, emb, pe, D,
                     scale, x);
  return hipGetLastError();
}

hipError_t launch_embed_bwd(const int32_t* ids, long ld, int B, int T, const float* dx, int D, int V, float scale,
                            float* dE, hipStream_t s) {
  hipError_t e = hipMemsetAsync(dE, 0, (size_t)V * D * sizeof(float), s);
  if (e != hipSuccess || B * T == 0) return e;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(B * T), dim3(256), 0, s, ids, ld, B, T, dx, D, V, scale, dE);
  return hipGetLastError();
}

hipError_t launch_logp_fwd(const float* logits, int V, const int32_t* ids, long ld, int B, int T, int end_token,
                           float* logp, float* lse, hipStream_t s) {
  hipLaunchKernelGGL(logp_fwd_kernel, dim3((B * T + 3) / 4), dim3(256), 0, s, logits, V, ids, ld, B, T, end_token,
                     logp, lse);
  return hipGetLastError();
}

hipError_t launch_logp_bwd(const float* logits, const float* lse, const float* dlogp, int V, const int32_t* ids,
                           long ld, int B, int T, int end_token, float* dlogits, hipStream_t s) {
  hipLaunchKernelGGL(logp_bwd_kernel, dim3((B * T + 3) / 4), dim3(256), 0, s, logits, lse, dlogp, V, ids, ld, B, T,
                     end_token, dlogits);
  return hipGetLastError();
}

hipError_t launch_drop_rows(const float* x, float* out, int B, int T, int n, DropCfg d, int site, hipStream_t s) {
  const long total = (long)B * T * n;
  hipLaunchKernelGGL(drop_rows_kernel, dim3(ew_grid(total)), dim3(256), 0, s, x, out, T, n, total, d, site);
  return hipGetLastError();
}

hipError_t launch_drop_attn(const float* x, float* out, int B, int H, int T, int Tk, int stride, DropCfg d, int site,
                            hipStream_t s) {
  const long total = (long)B * H * T * Tk;
  hipLaunchKernelGGL(drop_attn_kernel, dim3(ew_grid(total)), dim3(256), 0, s, x, out, H, T, Tk, stride, total, d,
                     site);
  return hipGetLastError();
}
