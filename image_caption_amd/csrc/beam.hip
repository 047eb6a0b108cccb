// Batched beam search state machine (icap_decode_beam): B images x K beam slots decoded together
// as B*K rows of the KV-cached decoder; this file holds the per-step selection and bookkeeping.
//
// Reference semantics (models/vit_transformer_model.py:327-420, grid_transformer_model.py:253-322),
// restated per image i with k = live beam count (starts at K, shrinks as beams finish):
//   step 0:  top-k of log_softmax(logits of beam 0)                      (all beams are identical)
//   step t:  top-k over the k*V candidates scores[j] + log_softmax(logits[j])[v], flattened j*V + v
//   new beam b: sequence = sequence[parent] + word, score = candidate value
//   beams ending in <end> are appended to the completed list in beam order; then
//     ViT:  all ended -> stop;                    Grid: completed >= k -> stop
//     the survivors keep their order and become beams 0..k'-1 (k' = new beam count);
//     Grid also stops when k' == 0
//   result: completed sequence with the highest score (first maximum) if any, else the live beam
//   with the highest score (first maximum).
// Ties in top-k are broken towards the lower flattened index.
//
// Rows: physical row r = i*K + slot.  K/V of position q of a beam live in the row that held its
// ancestor at step q: anc[r][q] (the decoder's self-attention reads keys through it), so reordering
// beams copies Lmax ints per beam instead of KV caches.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace {

constexpr int BEAM_MAX = 16;
constexpr int VMAX = 512;

// Every slot of both double buffers starts valid (token <start>, ancestry = its own row): slots that
// go idle keep being decoded, so their token and ancestry entries must stay in range.
__global__ void beam_init_kernel(int B, int K, int start, int Lmax, int32_t* seq_a, int32_t* seq_b, int32_t* anc_a,
                                 int32_t* anc_b, float* scores, int* kcur, int* done, int* ncomp, float* best_score,
                                 int* best_len) {
  const long n = (long)B * K * Lmax;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    seq_a[e] = start;
    seq_b[e] = start;
    anc_a[e] = (int32_t)(e / Lmax);
    anc_b[e] = (int32_t)(e / Lmax);
  }
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * K) scores[i] = 0.f;
  if (i < B) {
    kcur[i] = K;
    done[i] = 0;
    ncomp[i] = 0;
    best_score[i] = -INFINITY;
    best_len[i] = 0;
  }
}

// (value desc, index asc) maximum over a wave / a 256-thread block; the result is in every lane / thread
__device__ __forceinline__ void wave_best(float& bv, int& bi) {
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
}
__device__ __forceinline__ void block_best(float& bv, int& bi, float* rv, int* ri, int lane, int wave) {
  wave_best(bv, bi);
  if (lane == 0) {
    rv[wave] = bv;
    ri[wave] = bi;
  }
  __syncthreads();
  bv = rv[0];
  bi = ri[0];
  for (int w = 1; w < 4; ++w)
    if (rv[w] > bv || (rv[w] == bv && ri[w] < bi)) {
      bv = rv[w];
      bi = ri[w];
    }
  __syncthreads();  // rv / ri are reused by the next call
}

// One 256-thread block per image.
__global__ __launch_bounds__(256) void beam_select_kernel(const float* __restrict__ logits, int V, int K, int t,
                                                          int Lmax, int grid_variant, int end_tok,
                                                          const int32_t* seq_c, int32_t* seq_n, const int32_t* anc_c,
                                                          int32_t* anc_n, const float* sc_c, float* sc_n, int* kcur,
                                                          int* done, int* ncomp, float* best_score, int32_t* best_seq,
                                                          int* best_len) {
  __shared__ float lp[BEAM_MAX * VMAX];  // log-probs of the live beams
  __shared__ float rv[8];
  __shared__ int ri[8];
  __shared__ int sel_idx[BEAM_MAX];
  __shared__ float sel_val[BEAM_MAX];
  __shared__ int slot_of[BEAM_MAX];
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = img * K;
  const int k = kcur[img];
  if (done[img]) {  // frozen: carry the state over to the next buffers
    for (int e = tid; e < K * Lmax; e += 256) {
      seq_n[(long)r0 * Lmax + e] = seq_c[(long)r0 * Lmax + e];
      anc_n[(long)r0 * Lmax + e] = anc_c[(long)r0 * Lmax + e];
    }
    if (tid < K) sc_n[r0 + tid] = sc_c[r0 + tid];
    return;
  }
  const int nrows = t == 0 ? 1 : k;
  if (V <= VMAX) {
    // log_softmax per live row (one wave per row)
    for (int j = wave; j < nrows; j += 4) {
      const float* lg = logits + (long)(r0 + j) * V;
      float m = -INFINITY;
      for (int v = lane; v < V; v += 64) m = fmaxf(m, lg[v]);
      m = wave_max(m);
      float s = 0.f;
      for (int v = lane; v < V; v += 64) s += __expf(lg[v] - m);
      const float lse = m + __logf(wave_sum(s));
      const float base = t == 0 ? 0.f : sc_c[r0 + j];
      for (int v = lane; v < V; v += 64) lp[j * V + v] = base + (lg[v] - lse);
    }
    __syncthreads();
    // top-k over nrows*V candidates: k rounds of a block argmax (value desc, index asc)
    const int ncand = nrows * V;
    for (int b = 0; b < k; ++b) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int c = tid; c < ncand; c += 256) {
        const float v = lp[c];
        if (v > bv || (v == bv && c < bi)) {
          bv = v;
          bi = c;
        }
      }
      block_best(bv, bi, rv, ri, lane, wave);
      if (tid == 0) {
        sel_idx[b] = bi;
        sel_val[b] = bv;
        lp[bi] = -INFINITY;  // exclude (the candidate array is private to this step)
      }
      __syncthreads();
    }
  } else {
    // Vocabularies above VMAX: the k*V log-probs do not fit LDS.  The global top-k (value desc, flattened
    // index asc) is contained in the union of the rows' own top-k (a candidate beaten by fewer than k
    // candidates overall is beaten by fewer than k of its own row), so each row's top-k is found by k
    // passes over its logits (pass r: the best candidate ordered after pass r-1's pick), then the
    // global top-k over those nrows*k candidates.  Log-probs are the same expression as above.
    __shared__ float cv[BEAM_MAX * BEAM_MAX];
    __shared__ int ci[BEAM_MAX * BEAM_MAX];
    for (int j = wave; j < nrows; j += 4) {
      const float* lg = logits + (long)(r0 + j) * V;
      float m = -INFINITY;
      for (int v = lane; v < V; v += 64) m = fmaxf(m, lg[v]);
      m = wave_max(m);
      float s = 0.f;
      for (int v = lane; v < V; v += 64) s += __expf(lg[v] - m);
      const float lse = m + __logf(wave_sum(s));
      const float base = t == 0 ? 0.f : sc_c[r0 + j];
      float pv = INFINITY;
      int pi = -1;
      for (int r = 0; r < k; ++r) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
        for (int v = lane; v < V; v += 64) {
          const float x = base + (lg[v] - lse);
          const bool after = x < pv || (x == pv && v > pi);
          if (after && (x > bv || (x == bv && v < bi))) {
            bv = x;
            bi = v;
          }
        }
        wave_best(bv, bi);
        if (lane == 0) {
          cv[j * k + r] = bv;
          ci[j * k + r] = bi == 0x7fffffff ? 0x7fffffff : j * V + bi;
        }
        pv = bv;
        pi = bi;
      }
    }
    __syncthreads();
    const int ncand = nrows * k;
    for (int b = 0; b < k; ++b) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int c = tid; c < ncand; c += 256) {
        const float v = cv[c];
        const int ix = ci[c];
        if (ix != -1 && (v > bv || (v == bv && ix < bi))) {
          bv = v;
          bi = ix;
        }
      }
      block_best(bv, bi, rv, ri, lane, wave);
      if (tid < ncand && ci[tid] == bi) ci[tid] = -1;  // exclude (flattened indices are unique)
      if (tid == 0) {
        sel_idx[b] = bi;
        sel_val[b] = bv;
      }
      __syncthreads();
    }
  }
  // bookkeeping (thread 0: at most BEAM_MAX beams)
  __shared__ int s_kn, s_stop;
  if (tid == 0) {
    int nend = 0;
    for (int b = 0; b < k; ++b) nend += (sel_idx[b] % V) == end_tok;
    int nc = ncomp[img];
    float best = best_score[img];
    int best_b = -1;
    for (int b = 0; b < k; ++b)
      if ((sel_idx[b] % V) == end_tok) {
        ++nc;
        if (sel_val[b] > best) {
          best = sel_val[b];
          best_b = b;
        }
      }
    int stop = 0;
    if (nend > 0) stop = grid_variant ? (nc >= k) : (nend == k);
    int kn = k;
    if (nend > 0 && !stop) {
      kn = 0;
      for (int b = 0; b < k; ++b) slot_of[b] = (sel_idx[b] % V) == end_tok ? -1 : kn++;
      if (grid_variant && kn == 0) stop = 1;
    } else {
      for (int b = 0; b < k; ++b) slot_of[b] = b;
    }
    ncomp[img] = nc;
    if (best_b >= 0) {
      best_score[img] = best;
      best_len[img] = t + 2;
      slot_of[BEAM_MAX - 1] = best_b;  // stash (k <= BEAM_MAX - 1 is enforced by the launcher)
    } else {
      slot_of[BEAM_MAX - 1] = -1;
    }
    if (stop) done[img] = 1;
    if (!stop) kcur[img] = kn;
    s_kn = kn;
    s_stop = stop;
  }
  __syncthreads();
  // write the new beams (and the new best completed sequence) into the next buffers
  const int best_b = slot_of[BEAM_MAX - 1];
  for (int e = tid; e < k * (t + 2); e += 256) {
    const int b = e / (t + 2), q = e - b * (t + 2);
    const int parent = t == 0 ? 0 : sel_idx[b] / V;
    const int word = sel_idx[b] % V;
    const int tok = q <= t ? seq_c[(long)(r0 + parent) * Lmax + q] : word;
    if (b == best_b) best_seq[(long)img * Lmax + q] = tok;
    int slot = slot_of[b];
    if (s_stop) slot = b;  // stopped: keep the state as it is (only the best matters)
    if (slot < 0) continue;
    seq_n[(long)(r0 + slot) * Lmax + q] = tok;
    if (q <= t) anc_n[(long)(r0 + slot) * Lmax + q] = q < t ? anc_c[(long)(r0 + parent) * Lmax + q] : r0 + parent;
  }
  if (tid < k) {
    const int slot = s_stop ? tid : slot_of[tid];
    if (slot >= 0) sc_n[r0 + slot] = sel_val[tid];
  }
  (void)s_kn;
}

__global__ void beam_finalize_kernel(int K, int Lmax, const int32_t* seq, const float* scores, const int* kcur,
                                     const int* ncomp, const int32_t* best_seq, const int* best_len, int32_t* ids,
                                     int32_t* lens) {
  const int img = blockIdx.x, tid = threadIdx.x;
  __shared__ int pick, len;
  if (tid == 0) {
    if (ncomp[img] > 0) {
      pick = -1;
      len = best_len[img];
    } else {
      const int k = kcur[img];
      int b = 0;
      for (int j = 1; j < k; ++j)
        if (scores[img * K + j] > scores[img * K + b]) b = j;
      pick = b;
      len = Lmax;
    }
    lens[img] = len;
  }
  __syncthreads();
  for (int q = tid; q < Lmax; q += blockDim.x) {
    int v = 0;
    if (q < len) v = pick < 0 ? best_seq[(long)img * Lmax + q] : seq[((long)img * K + pick) * Lmax + q];
    ids[(long)img * Lmax + q] = v;
  }
}

}  // namespace

hipError_t launch_beam_init(int B, int K, int start, int Lmax, int32_t* seq_a, int32_t* seq_b, int32_t* anc_a,
                            int32_t* anc_b, float* scores, int* kcur, int* done, int* ncomp, float* best_score,
                            int* best_len, hipStream_t s) {
  if (K < 1 || K >= BEAM_MAX) return hipErrorInvalidValue;
  const int blocks = std::max(1, std::min(1024, (int)(((long)B * K * Lmax + 255) / 256)));
  const int need = (std::max(B * K, B) + 255) / 256;
  hipLaunchKernelGGL(beam_init_kernel, dim3(std::max(blocks, need)), dim3(256), 0, s, B, K, start, Lmax, seq_a, seq_b,
                     anc_a, anc_b, scores, kcur, done, ncomp, best_score, best_len);
  return hipGetLastError();
}

hipError_t launch_beam_select(const float* logits, int V, int B, int K, int t, int Lmax, int grid_variant, int end_tok,
                              const int32_t* seq_c, int32_t* seq_n, const int32_t* anc_c, int32_t* anc_n,
                              const float* sc_c, float* sc_n, int* kcur, int* done, int* ncomp, float* best_score,
                              int32_t* best_seq, int* best_len, hipStream_t s) {
  if (K < 1 || K >= BEAM_MAX || V < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(beam_select_kernel, dim3(B), dim3(256), 0, s, logits, V, K, t, Lmax, grid_variant, end_tok, seq_c,
                     seq_n, anc_c, anc_n, sc_c, sc_n, kcur, done, ncomp, best_score, best_seq, best_len);
  return hipGetLastError();
}

hipError_t launch_beam_finalize(int B, int K, int Lmax, const int32_t* seq, const float* scores, const int* kcur,
                                const int* ncomp, const int32_t* best_seq, const int* best_len, int32_t* ids,
                                int32_t* lens, hipStream_t s) {
  hipLaunchKernelGGL(beam_finalize_kernel, dim3(B), dim3(64), 0, s, K, Lmax, seq, scores, kcur, ncomp, best_seq,
                     best_len, ids, lens);
  return hipGetLastError();
}
