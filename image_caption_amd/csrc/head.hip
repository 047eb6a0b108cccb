// Output head of a decode step: fc_out (512 -> V=109) in exact fp32,
// then either argmax (greedy, first index on ties like torch CPU argmax; vit:315-316) or an
// inverse-CDF categorical sample on an injected uniform with its log-probability
// (`_sample_with_log_probs`, scst_loss:229-239), and the next step's embedding
// emb[tok] * sqrt(d) + pe[t+1] (vit:166-169) so the following layer GEMM can start at once.
// One 128-thread workgroup per image row.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int HEAD_LN_PARTS = 16;

// Row r of the head's input into xs: x itself, or (a.ln.parts set) the last decoder layer's residual LN3
// x = LN(x + sum of the FFN's split-K slabs + bias) computed here instead of by its own launch - threads
// 0..127 own 4 consecutive columns each, the layout and summation order of residual_layernorm_kernel<128>,
// so xs is bitwise what that kernel would have stored.  Called by every thread of the block (barriers).
__device__ __forceinline__ void head_row_in(const HeadArgs& a, int r, float* xs, float* red) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* x = a.x + (long)r * a.Dm;
  if (!a.ln.parts) {
    for (int d = tid; d < a.Dm; d += blockDim.x) xs[d] = x[d];
    __syncthreads();
    return;
  }
  const RlnArgs& ln = a.ln;
  const int col = 4 * tid;
  f32x4 v = {0.f, 0.f, 0.f, 0.f}, dv = v, wv = v, bv = v;
  if (tid < 128) {
    wv = *(const f32x4*)(ln.w + col), bv = *(const f32x4*)(ln.b + col);  // with the slabs: no load after the sums
    f32x4 pp[HEAD_LN_PARTS];
#pragma unroll
    for (int s = 0; s < HEAD_LN_PARTS; ++s)
      pp[s] = s < ln.nparts ? *(const f32x4*)(ln.parts + s * ln.part_stride + (long)r * 512 + col)
                            : (f32x4){0.f, 0.f, 0.f, 0.f};
    v = *(const f32x4*)(x + col);
    const f32x4 bb = ln.bias ? *(const f32x4*)(ln.bias + col) : (f32x4){0.f, 0.f, 0.f, 0.f};
    if (ln.drop.thr == 0) {
      v += bb;
#pragma unroll
      for (int s = 0; s < HEAD_LN_PARTS; ++s) v += pp[s];
    } else {
      f32x4 o = bb;
#pragma unroll
      for (int s = 0; s < HEAD_LN_PARTS; ++s) o += pp[s];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] += o[k] * drop_mul(ln.drop, ln.site, r, ln.drop.pos, col + k);
    }
    const float sm = wave_sum(v[0] + v[1] + v[2] + v[3]);
    if (lane == 0) red[w] = sm;
  }
  __syncthreads();
  const float mean = (red[0] + red[1]) / 512.f;
  if (tid < 128) {
    dv = v - mean;
    const float q = wave_sum(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2] + dv[3] * dv[3]);
    if (lane == 0) red[2 + w] = q;
  }
  __syncthreads();
  if (tid < 128) {
    const float rstd = 1.0f / sqrtf((red[2] + red[3]) / 512.f + ln.eps);
    f32x4 y;
#pragma unroll
    for (int k = 0; k < 4; ++k) y[k] = dv[k] * rstd * wv[k] + bv[k];
    *(f32x4*)(xs + col) = y;
  }
  __syncthreads();
}

__global__ __launch_bounds__(128) void head_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float hs[];
  float* xs = hs;             // [Dm]
  float* lg = hs + a.Dm;      // [128]
  __shared__ int s_tok;
  __shared__ float s_red[4];
  __shared__ int s_idx[2];
  __shared__ float s_ln[4];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  head_row_in(a, r, xs, s_ln);
  float logit = -INFINITY;
  if (tid < a.V) {
    // W4 (when set): fc_out as [Dm / 4][V][4], so the 4 weights a lane needs per step are 16 B and the wave's
    // loads one contiguous run (the [V][Dm] rows put every lane on its own line); same products, same order
    const float* wr = a.W4 ? a.W4 + (long)tid * 4 : a.W + (long)tid * a.Dm;
    const long wstep = a.W4 ? (long)a.V * 4 : 4;
    float acc = 0.f;
    // unrolled so the weight loads of 16 steps are in flight together (the FMA chain keeps its order): a rolled loop
    // waited one L2 round trip per 4 columns
#pragma unroll 16
    for (int d = 0; d < a.Dm; d += 4, wr += wstep) {
      const f32x4 wv = *(const f32x4*)wr;
      const f32x4 xv = *(const f32x4*)(xs + d);
      acc = fmaf(xv[0], wv[0], acc);
      acc = fmaf(xv[1], wv[1], acc);
      acc = fmaf(xv[2], wv[2], acc);
      acc = fmaf(xv[3], wv[3], acc);
    }
    logit = acc + a.bias[tid];
    if (a.logits) a.logits[(long)r * a.ld_logits + tid] = logit;
  }
  lg[tid] = logit;
  // argmax (value, lowest index on ties) within each wave, then across the two waves
  float bv = logit;
  int bi = tid < a.V ? tid : 0x7fffffff;
  wave_argmax(bv, bi);
  if (lane == 0) { s_red[w] = bv; s_idx[w] = bi; }
  __syncthreads();
  const float mx = fmaxf(s_red[0], s_red[1]);
  if (a.uniforms == nullptr) {
    if (tid == 0) {
      int tok = s_idx[0];
      if (s_red[1] > s_red[0] || (s_red[1] == s_red[0] && s_idx[1] < s_idx[0])) tok = s_idx[1];
      s_tok = tok;
    }
  } else {
    // softmax + inverse CDF: idx = #{v : cdf[v] <= u * cdf[V-1]}, sequential prefix like torch.cumsum
    const float e = tid < a.V ? __expf(logit - mx) : 0.f;
    lg[tid] = e;
    __syncthreads();
    if (tid == 0) {
      float c = 0.f;
      for (int v = 0; v < a.V; ++v) { c += lg[v]; lg[v] = c; }
      const float total = c;
      const float thr = a.uniforms[r] * total;
      int idx = 0;
      for (int v = 0; v < a.V; ++v) idx += (lg[v] <= thr) ? 1 : 0;
      idx = min(idx, a.V - 1);
      s_tok = idx;
      s_red[2] = logf(total);  // log-sum-exp offset for log_softmax of the chosen token
    }
    __syncthreads();
    if (tid == s_tok) {
      float lp = (logit - mx) - s_red[2];
      const bool fin = a.finished[r] != 0;
      a.logp[(long)r * a.ld_logp] = fin ? 0.f : lp;
    }
  }
  __syncthreads();
  const int tok = s_tok;
  if (tid == 0) {
    a.ids[(long)r * a.ld_ids + a.id_col] = tok;
    if (a.finished) a.finished[r] = (uint8_t)(a.finished[r] | (tok == a.end_token));
  }
  if (a.emb) {
    const long base = (long)r * a.Dm;
    for (int d = tid; d < a.Dm; d += 128) {
      float v = a.emb[(long)tok * a.Dm + d] * a.emb_scale + a.pe[(long)a.pe_pos * a.Dm + d];
      if (a.drop.thr) v *= drop_mul(a.drop, 0, r, a.pe_pos, d);  // PositionalEncoding's dropout
      a.x_next[base + d] = v;
      bf16_t hi, lo;
      split_bf(v, hi, lo);
      a.a_next[base + d] = hi;
      if (a.nsplit == 2) a.a_next[base + d + a.lo] = lo;
    }
  }
}

// Vocabularies above 128 (the reference builds its vocabulary from the captions with a min-count rule,
// utils/deepfashion_dataset.py:76-81, so V is a property of the dataset): the same head with 256 threads,
// each owning the logits v = tid, tid + 256, ... (exact fp32 dot products in the same order), the logits
// kept in LDS for the sampler's sequential prefix sum.
__global__ __launch_bounds__(256) void head_wide_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float hs[];
  float* xs = hs;             // [Dm]
  float* lg = hs + a.Dm;      // [V]
  __shared__ int s_tok;
  __shared__ float s_red[4], s_lse;
  __shared__ int s_idx[4];
  __shared__ float s_ln[4];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  head_row_in(a, r, xs, s_ln);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int v = tid; v < a.V; v += 256) {
    const float* wr = a.W + (long)v * a.Dm;
    float acc = 0.f;
    for (int d = 0; d < a.Dm; d += 4) {
      const f32x4 wv = *(const f32x4*)(wr + d);
      const f32x4 xv = *(const f32x4*)(xs + d);
      acc = fmaf(xv[0], wv[0], acc);
      acc = fmaf(xv[1], wv[1], acc);
      acc = fmaf(xv[2], wv[2], acc);
      acc = fmaf(xv[3], wv[3], acc);
    }
    const float logit = acc + a.bias[v];
    if (a.logits) a.logits[(long)r * a.ld_logits + v] = logit;
    lg[v] = logit;
    if (logit > bv) { bv = logit; bi = v; }  // v increases: the first maximum of this thread's subset
  }
  wave_argmax(bv, bi);
  if (lane == 0) { s_red[w] = bv; s_idx[w] = bi; }
  __syncthreads();
  if (tid == 0) {
    float m = s_red[0];
    int t = s_idx[0];
    for (int k = 1; k < 4; ++k)
      if (s_red[k] > m || (s_red[k] == m && s_idx[k] < t)) { m = s_red[k]; t = s_idx[k]; }
    s_red[0] = m;
    s_tok = t;
  }
  __syncthreads();
  const float mx = s_red[0];
  if (a.uniforms) {
    for (int v = tid; v < a.V; v += 256) lg[v] = __expf(lg[v] - mx);
    __syncthreads();
    if (tid == 0) {  // sequential prefix, as the 128-wide head (torch.cumsum order)
      float c = 0.f;
      for (int v = 0; v < a.V; ++v) { c += lg[v]; lg[v] = c; }
      const float thr = a.uniforms[r] * c;
      int idx = 0;
      for (int v = 0; v < a.V; ++v) idx += (lg[v] <= thr) ? 1 : 0;
      s_tok = min(idx, a.V - 1);
      s_lse = logf(c);
    }
    __syncthreads();
    if (tid == 0) {
      const float* wr = a.W + (long)s_tok * a.Dm;  // the chosen token's logit, recomputed in the same order
      float acc = 0.f;
      for (int d = 0; d < a.Dm; d += 4) {
        const f32x4 wv = *(const f32x4*)(wr + d);
        const f32x4 xv = *(const f32x4*)(xs + d);
        acc = fmaf(xv[0], wv[0], acc);
        acc = fmaf(xv[1], wv[1], acc);
        acc = fmaf(xv[2], wv[2], acc);
        acc = fmaf(xv[3], wv[3], acc);
      }
      const float lp = (acc + a.bias[s_tok] - mx) - s_lse;
      a.logp[(long)r * a.ld_logp] = a.finished[r] != 0 ? 0.f : lp;
    }
  }
  __syncthreads();
  const int tok = s_tok;
  if (tid == 0) {
    a.ids[(long)r * a.ld_ids + a.id_col] = tok;
    if (a.finished) a.finished[r] = (uint8_t)(a.finished[r] | (tok == a.end_token));
  }
  if (a.emb) {
    const long base = (long)r * a.Dm;
    for (int d = tid; d < a.Dm; d += 256) {
      float v = a.emb[(long)tok * a.Dm + d] * a.emb_scale + a.pe[(long)a.pe_pos * a.Dm + d];
      if (a.drop.thr) v *= drop_mul(a.drop, 0, r, a.pe_pos, d);
      a.x_next[base + d] = v;
      bf16_t hi, lo;
      split_bf(v, hi, lo);
      a.a_next[base + d] = hi;
      if (a.nsplit == 2) a.a_next[base + d + a.lo] = lo;
    }
  }
}

__global__ void head_w4_kernel(const float* __restrict__ w, int V, int Dm, float* __restrict__ w4) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one 4-weight group
  if (i >= (long)V * (Dm / 4)) return;
  const int v = (int)(i % V), d4 = (int)(i / V);
  *(f32x4*)(w4 + i * 4) = *(const f32x4*)(w + (long)v * Dm + d4 * 4);
}

}  // namespace

hipError_t launch_head_w4(const float* w, int V, int Dm, float* w4, hipStream_t s) {
  if (V < 1 || Dm % 4) return hipErrorInvalidValue;
  const long n = (long)V * (Dm / 4);
  hipLaunchKernelGGL(head_w4_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, V, Dm, w4);
  return hipGetLastError();
}

hipError_t launch_head(const HeadArgs& h, hipStream_t s) {
  if (h.V < 1 || h.V > HEAD_MAX_VOCAB || h.Dm % 4) return hipErrorInvalidValue;
  if (h.ln.parts && (h.Dm != 512 || h.ln.nparts < 1 || h.ln.nparts > HEAD_LN_PARTS)) return hipErrorInvalidValue;
  if (h.V <= 128) {
    hipLaunchKernelGGL(head_kernel, dim3(h.rows), dim3(128), (h.Dm + 128) * 4, s, h);
  } else {
    static bool attr = false;
    if (!attr) {
      const hipError_t e = hipFuncSetAttribute((const void*)head_wide_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (1024 + HEAD_MAX_VOCAB) * 4);
      if (e != hipSuccess) return e;
      attr = true;
    }
    hipLaunchKernelGGL(head_wide_kernel, dim3(h.rows), dim3(256), (h.Dm + h.V) * 4, s, h);
  }
  return hipGetLastError();
}
