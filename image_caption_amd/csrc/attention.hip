// Attention kernels of the captioning hot path.
//
// enc_attention: encoder self-attention (ViT N=197 x 12 heads, Grid N=49 x 8 heads; hd = 64,
//   non-causal).  One workgroup per (image, head), 4 waves.  K and V of the head are staged in
//   LDS once; each wave takes 16-query tiles.  Scores are computed transposed, S^T = K·Q^T,
//   with v_mfma_f32_16x16x32_bf16 so a query sits on the lane and its keys in the accumulator
//   registers: the softmax row-reduce is per-lane + two xor-shuffles, and the S^T accumulators
//   are used directly as the B operand of O^T = V^T·P^T (k order permuted consistently), with
//   V^T fragments delivered by ds_read_b64_tr_b16 transposed LDS reads.  In split mode every
//   product carries the three terms hi·hi + lo·hi + hi·lo (activations are hi/lo bf16 planes).
//
// dec_self_attn: one decode step's causal self-attention over an fp32 KV cache (t <= max_len
//   keys, one wave per (image, head), exact fp32 VALU math).
//
// cross_attn_mfma: decoder cross-attention with the key projection absorbed into the query,
//   score_h(s) = (q_h · Wk_h) · mem_s / sqrt(hd) (the q·bk term is constant over s and cancels
//   in the softmax), context c_h = sum_s p_h(s) mem_s; the caller applies Wv_h and bv (sum p = 1).
//   The memory is read once per layer-step (as bf16 hi/lo planes) instead of 6 per-layer K/V
//   projections.
#include "common.h"
#include "kernels.h"

namespace {

__device__ __forceinline__ void st_planes(bf16_t* base, long idx, long lo, int nsplit, float v) {
  bf16_t hi, l;
  split_bf(v, hi, l);
  base[idx] = hi;
  if (nsplit == 2) base[idx + lo] = l;
}

// Two ds_read_b64_tr_b16 (4 keys x 16 d each) concatenated into one 8-element MFMA operand.
// Built with whole-vector shuffles/bit-casts: per-element short->__bf16 bit-casts miscompile
// (hipcc ROCm 7.2 duplicated dwords via v_perm; found by tools/attn_debug.hip).
__device__ __forceinline__ bf16x8 tr_pair(const char* p0, const char* p1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)p0);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)p1);
  const s16x8 c = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}

// LDS chunk swizzles of the [keys][64] K / V matrices (16-B chunk c of row r stored at c ^ swz(r)),
// chosen for the 64-bank LDS: a ds_read_b128 pass covers 16 consecutive K rows at one logical chunk
// (bank = 32 (r & 1) + 4 chunk: (r >> 1) & 7 spreads the 8 rows of each parity over 8 chunks; the
// former r & 7 put rows r and r + 8 on the same banks, 2-way), and a ds_read_b64_tr_b16 pass covers
// 8 consecutive V rows x 2 chunks x 2 halves (the 4 rows of one parity need disjoint chunk pairs:
// 2 ((r >> 1) & 3); unswizzled V rows were 4-way conflicts).  PMC before: 26.8 M bank-conflict
// cycles against 8.1 M LDS-active cycles per launch.
__device__ __forceinline__ int kswz(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int vswz(int r) { return ((r >> 1) & 3) << 1; }

template <int NKT, bool SPLIT, int NW>
__global__ __launch_bounds__(NW * 64) void enc_attention_kernel(const bf16_t* __restrict__ qkv, long ld, long lo,
                                                            int N, int H, float scale, bf16_t* out,
                                                            long out_ld, long out_lo) {
  constexpr int NP = NKT * 16;           // padded keys (multiple of 32)
  constexpr int MAT = NP * 128;           // bytes of one [NP][64] bf16 matrix
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kh = smem;
  char* Vh = smem + MAT;
  char* Kl = smem + 2 * MAT;
  char* Vl = smem + 3 * MAT;
  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = H * 64;
  const bf16_t* base = qkv + (long)b * N * ld;

  // stage K and V by LDS-DMA, one instruction = 8 rows x 128 B (full lines), lane-linear image:
  // chunk c of row r stored at c ^ kswz(r) (K) / c ^ vswz(r) (V), pre-swizzled on the source
  // (conflict-free fragment and transposed reads; PMC before: 1.57 M conflict cycles against 0.46 M
  // LDS-active per Grid launch).  Rows >= N repeat row N - 1: their scores are masked to
  // -inf and their V rows meet p = 0.  All waves issue (LDS-DMA ingest scales with issuing waves).
  const int fr = lane & 15, g = lane >> 4;
  const int nqt = (N + 15) / 16;
  bf16x8 qh[2], ql[2];
  auto load_q = [&](int qt) {
    const int q = min(qt * 16 + fr, N - 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16_t* src = base + (long)q * ld + h * 64 + ks * 32 + g * 8;
      qh[ks] = *(const bf16x8*)src;
      if (SPLIT) ql[ks] = *(const bf16x8*)(src + lo);
    }
  };
  if (wave < nqt) load_q(wave);
  {
    constexpr int PER_MAT = NP / 8, NMAT = SPLIT ? 4 : 2;
    const int lrow = lane >> 3, lch = lane & 7;
    for (int ins = wave; ins < NMAT * PER_MAT; ins += NW) {
      const int mat = ins / PER_MAT, row = (ins - mat * PER_MAT) * 8 + lrow;  // mat: Kh, Vh, Kl, Vl
      const bool isK = !(mat & 1);
      const int ch = lch ^ (isK ? kswz(row) : vswz(row));
      const bf16_t* src = base + (mat >= 2 ? lo : 0) + (long)min(row, N - 1) * ld + (isK ? D : 2 * D) + h * 64 + ch * 8;
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src,
                                       (LDS_AS void*)(smem + mat * MAT + (ins - mat * PER_MAT) * 1024), 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int qt = wave; qt < nqt; qt += NW) {
    if (qt != wave) load_q(qt);
    // keys in chunks of CH tiles (an even count: the P.V MFMA takes 32 keys = 2 tiles) with an
    // online softmax, so only CH score tiles are live (16 waves per block fit in 128 VGPRs)
    constexpr int CH = 4;
    float m = -INFINITY, l = 0.f;  // running max / per-lane partial sum for query (lane & 15)
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int q4 = fr >> 2, p4 = fr & 3;
#pragma unroll 1
    for (int c0 = 0; c0 < NKT; c0 += CH) {  // rolled: unrolled chunks get interleaved and spill
      constexpr int CMAX = CH;
      const int nt = NKT - c0 < CH ? NKT - c0 : CH;
      f32x4 s[CMAX];
#pragma unroll
      for (int u = 0; u < CMAX; ++u) {
        if (u >= nt) break;
        const int kt = c0 + u;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const int row = kt * 16 + fr;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int off = row * 128 + (((ks * 4 + g) ^ kswz(row)) << 4);
          const bf16x8 kh = *(const bf16x8*)(Kh + off);
          acc = mfma16(kh, qh[ks], acc);
          if (SPLIT) {
            const bf16x8 kl = *(const bf16x8*)(Kl + off);
            acc = mfma16(kl, qh[ks], acc);
            acc = mfma16(kh, ql[ks], acc);
          }
        }
        s[u] = acc;
      }
      // key of s[u][r] = 16 (c0 + u) + 4 g + r
      float cm = -INFINITY;
#pragma unroll
      for (int u = 0; u < CMAX; ++u) {
        if (u >= nt) break;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = (c0 + u) * 16 + g * 4 + r;
          const float v = key < N ? s[u][r] * scale : -INFINITY;
          s[u][r] = v;
          cm = fmaxf(cm, v);
        }
      }
      cm = rows4_max(cm);
      const float m_new = fmaxf(m, cm);
      if (m_new == -INFINITY) continue;  // every key of this chunk is padding (uniform per query)
      const float alpha = __expf(m - m_new);
      m = m_new;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
#pragma unroll
      for (int u = 0; u < CMAX; ++u) {
        if (u >= nt) break;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __expf(s[u][r] - m_new);
          s[u][r] = e;
          l += e;
        }
      }
      // O^T[d][q] += sum_k V^T[d][k] P^T[k][q], 32 keys (2 tiles) per MFMA
#pragma unroll
      for (int u = 0; u < CMAX; u += 2) {
        if (u >= nt) break;
        bf16x8 ph, pl;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ph[j] = (__bf16)s[u][j];
          ph[4 + j] = (__bf16)s[u + 1][j];
          if (SPLIT) {
            pl[j] = (__bf16)(s[u][j] - (float)ph[j]);
            pl[4 + j] = (__bf16)(s[u + 1][j] - (float)ph[4 + j]);
          }
        }
        const int key0 = 16 * (c0 + u) + 4 * g + q4;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int off0 = key0 * 128 + (((dt * 2 + (p4 >> 1)) ^ vswz(key0)) << 4) + (p4 & 1) * 8;
          const int off1 = off0 + 16 * 128;
          const bf16x8 vh = tr_pair(Vh + off0, Vh + off1);
          o[dt] = mfma16(vh, ph, o[dt]);
          if (SPLIT) {
            const bf16x8 vl = tr_pair(Vl + off0, Vl + off1);
            o[dt] = mfma16(vl, ph, o[dt]);
            o[dt] = mfma16(vh, pl, o[dt]);
          }
        }
      }
    }
    l = rows4_sum(l);
    const float inv = 1.f / l;
    const int qq = qt * 16 + fr;
    if (qq < N) {
      bf16_t* dst = out + ((long)b * N + qq) * out_ld + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16_t hv[4], lv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) split_bf(o[dt][r] * inv, hv[r], lv[r]);
        const int d = dt * 16 + 4 * g;
        *(u32x2*)(dst + d) = (u32x2){(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16)};
        if (SPLIT)
          *(u32x2*)(dst + out_lo + d) =
              (u32x2){(uint32_t)lv[0] | ((uint32_t)lv[1] << 16), (uint32_t)lv[2] | ((uint32_t)lv[3] << 16)};
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// qkv rows: (b * n_new + i) with [q | k | v] of width 3D.  Cache kc/vc: [B][H][Lmax][64] fp32.
// anc (optional, beam search): anc[b * Lmax + j] = the cache row holding this row's key/value of
// position j < t0 (its ancestor at step j); without it the row's own cache is read.
// klen (optional, tgt_key_padding_mask): keys j >= klen[b] are masked for every query of row b
// (a query with no key left gets a zero context, as torch's scaled_dot_product_attention path of
// nn.MultiheadAttention(need_weights=False) returns for a fully masked row).
__global__ __launch_bounds__(64) void dec_self_attn_kernel(const float* __restrict__ qkv, int n_new, int t0,
                                                           int H, float* kc, float* vc, int Lmax, int causal,
                                                           float scale, bf16_t* out, long lo, int nsplit,
                                                           const int32_t* __restrict__ anc,
                                                           const int32_t* __restrict__ klen) {
  __shared__ float sq[64];
  __shared__ float sp[512];
  const int h = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
  const int D = H * 64;
  const long ld = 3L * D;
  float* kcb = kc + ((long)b * H + h) * Lmax * 64;
  float* vcb = vc + ((long)b * H + h) * Lmax * 64;
  const float* rows = qkv + (long)b * n_new * ld;
  for (int i = 0; i < n_new; ++i) {
    kcb[(long)(t0 + i) * 64 + lane] = rows[i * ld + D + h * 64 + lane];
    vcb[(long)(t0 + i) * 64 + lane] = rows[i * ld + 2 * D + h * 64 + lane];
  }
  for (int i = 0; i < n_new; ++i) {
    const int pos = t0 + i;
    int nkeys = causal ? pos + 1 : t0 + n_new;
    if (klen) nkeys = min(nkeys, max(klen[b], 0));
    __syncthreads();
    sq[lane] = rows[i * ld + h * 64 + lane];
    __syncthreads();
    float m = -INFINITY;
    for (int k0 = 0; k0 < nkeys; k0 += 64) {
      const int key = k0 + lane;
      float sc = -INFINITY;
      if (key < nkeys) {
        const float* kv;
        if (key >= t0) kv = rows + (key - t0) * ld + D + h * 64;
        else if (anc) kv = kc + ((long)anc[(long)b * Lmax + key] * H + h) * Lmax * 64 + (long)key * 64;
        else kv = kcb + (long)key * 64;
        float acc = 0.f;
#pragma unroll 16
        for (int d = 0; d < 64; ++d) acc = fmaf(sq[d], kv[d], acc);
        sc = acc * scale;
        sp[key] = sc;
      }
      m = fmaxf(m, sc);
    }
    m = wave_max(m);
    float l = 0.f;
    for (int k0 = 0; k0 < nkeys; k0 += 64) {
      const int key = k0 + lane;
      if (key < nkeys) {
        const float e = __expf(sp[key] - m);
        sp[key] = e;
        l += e;
      }
    }
    l = wave_sum(l);
    __syncthreads();
    float acc = 0.f;
    for (int key = 0; key < nkeys; ++key) {
      const float* vv;
      if (key >= t0) vv = rows + (key - t0) * ld + 2 * D + h * 64;
      else if (anc) vv = vc + ((long)anc[(long)b * Lmax + key] * H + h) * Lmax * 64 + (long)key * 64;
      else vv = vcb + (long)key * 64;
      acc = fmaf(sp[key], vv[lane], acc);
    }
    st_planes(out, ((long)b * n_new + i) * D + h * 64 + lane, lo, nsplit, nkeys > 0 ? acc / l : 0.f);
  }
}

// Pipelined form for longer sequences (ViT, N = 197): K and V stream through a 4-deep LDS ring of
// 32-key chunks (Kh, Vh, Kl, Vl: 16 KiB per chunk, one LDS-DMA instruction per wave) while the waves
// compute - each wave keeps its query tile's online-softmax state (running max, sum, 16 x 64 context)
// across chunks, so loads of chunks c+1..c+3 are in flight during chunk c instead of one 112 KiB
// stage-then-compute.  Counted vmcnt + raw s_barrier as in the GEMMs.
// HM: qkv in the head-major layout of GemmArgs::hm_n ([image][q|k|v x head][token][64]), so one
// (image, head)'s K and V rows are contiguous 128-byte rows; else row-major [token][3 D].
// QPW query tiles per wave: 16 / QPW waves per block (QPW = 2: 8 waves, two blocks per CU).

template <bool SPLIT, bool HM, int QPW, bool F16 = false>
__global__ __launch_bounds__(1024 / QPW, QPW == 2 ? 4 : 1) void enc_attention_pipe_kernel(
    const bf16_t* __restrict__ qkv, long ld, long lo, int N, int H, float scale, bf16_t* out, long out_ld,
    long out_lo) {
  constexpr int NW = 16 / QPW, CK = 32, NBUF = 4;
  constexpr int MAT = CK * 128;                // one [32][64] bf16 matrix
  constexpr int NMAT = SPLIT ? 4 : 2;          // Kh, Vh (, Kl, Vl)
  constexpr int CHUNK = NMAT * MAT;
  constexpr int INS = NMAT * CK / 8;           // 1 KiB DMA instructions per chunk (16 / 8)
  constexpr int IPW = INS / NW > 0 ? INS / NW : 1;  // per wave (waves >= INS / IPW issue)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = H * 64;
  const long rs = HM ? 64 : ld;  // row stride of Q / K / V
  const bf16_t* qb = HM ? qkv + ((long)b * 3 * H + h) * N * 64 : qkv + (long)b * N * ld + h * 64;
  const bf16_t* kb = HM ? qb + (long)H * N * 64 : qb + D;
  const bf16_t* vb = HM ? qb + 2L * H * N * 64 : qb + 2 * D;
  const int fr = lane & 15, g = lane >> 4;
  const int nqt = (N + 15) / 16, nch = (N + CK - 1) / CK;
  const int lrow = lane >> 3, lch = lane & 7;
  const bool uniform_issue = INS % NW == 0;  // every wave issues IPW instructions per chunk

  auto stage = [&](int c, int buf) {
#pragma unroll
    for (int k = 0; k < IPW; ++k) {
      const int ins = wave * IPW + k;
      if (ins < INS) {
        const int mat = ins / (CK / 8), part = ins % (CK / 8);
        const int row = part * 8 + lrow, key = c * CK + row;
        const bool isK = !(mat & 1);
        const int ch = lch ^ (isK ? kswz(row) : vswz(row));
        const bf16_t* src = (isK ? kb : vb) + (mat >= 2 ? lo : 0) + (long)min(key, N - 1) * rs + ch * 8;
        lds_dma16(src, (LDS_AS void*)(smem + buf * CHUNK + mat * MAT + part * 1024));
      }
    }
  };

  bf16x8 qh[QPW][2], ql[QPW][2];
#pragma unroll
  for (int t = 0; t < QPW; ++t) {
    const int q = min((wave + t * NW) * 16 + fr, N - 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16_t* src = qb + (long)q * rs + ks * 32 + g * 8;
      qh[t][ks] = *(const bf16x8*)src;
      if (SPLIT) ql[t][ks] = *(const bf16x8*)(src + lo);
    }
  }
#pragma unroll
  for (int c = 0; c < NBUF - 1; ++c)
    if (c < nch) stage(c, c);

  float m[QPW], l[QPW];
  f32x4 o[QPW][4];
#pragma unroll
  for (int t = 0; t < QPW; ++t) {
    m[t] = -INFINITY;
    l[t] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[t][dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  const int q4 = fr >> 2, p4 = fr & 3;
#pragma unroll 1
  for (int c = 0; c < nch; ++c) {
    const int younger = min(NBUF - 2, nch - 1 - c);
    // lgkmcnt(0): this wave's LDS reads of the slot read last iteration must be done before the
    // barrier after which another wave refills that slot
    if (!uniform_issue) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * IPW) : "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(IPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (c + NBUF - 1 < nch) stage(c + NBUF - 1, (c + NBUF - 1) % NBUF);
    const char* Kh = smem + (c % NBUF) * CHUNK;
    const char* Vh = Kh + MAT;
    const char* Kl = Kh + 2 * MAT;
    const char* Vl = Kh + 3 * MAT;
#pragma unroll
    for (int t = 0; t < QPW; ++t) {
      if ((wave + t * NW) >= nqt) break;  // wave-uniform
      f32x4 s[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const int row = u * 16 + fr;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int off = row * 128 + (((ks * 4 + g) ^ kswz(row)) << 4);
          const bf16x8 kh = *(const bf16x8*)(Kh + off);
          acc = mma<F16>(kh, qh[t][ks], acc);
          if (SPLIT) {
            const bf16x8 kl = *(const bf16x8*)(Kl + off);
            acc = mfma16(kl, qh[t][ks], acc);
            acc = mfma16(kh, ql[t][ks], acc);
          }
        }
        s[u] = acc;
      }
      if constexpr (F16) {
        // the f16 encoder's softmax in the exp2 domain with packed fp32 math: scores scaled by scale * log2(e) once
        // (v_pk_mul), the key mask only in a ragged last chunk, max through 3-input maxima, exponents
        // v_exp_f32(s - m) with the running max and sum in log2 units (the same softmax, ~half the VALU
        // instructions per score of the exp / compare / mask per element form)
        const float sc2 = scale * 1.44269504088896341f;
        s[0] *= sc2;
        s[1] *= sc2;
        if (c * CK + CK > N) {  // (wave-uniform) ragged last chunk
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (c * CK + u * 16 + g * 4 + r >= N) s[u][r] = -INFINITY;
        }
        float cm = fmaxf(fmaxf(s[0][0], s[0][1]), s[0][2]);
        cm = fmaxf(fmaxf(cm, s[0][3]), s[1][0]);
        cm = fmaxf(fmaxf(cm, s[1][1]), s[1][2]);
        cm = rows4_max(fmaxf(cm, s[1][3]));
        const float m_new = fmaxf(m[t], cm);  // finite: every chunk holds at least one real key
        const float alpha = __builtin_amdgcn_exp2f(m[t] - m_new);
        m[t] = m_new;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[t][dt] *= alpha;
        s[0] -= m_new;
        s[1] -= m_new;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[u][r] = __builtin_amdgcn_exp2f(s[u][r]);
        const f32x4 e4 = s[0] + s[1];
        l[t] = l[t] * alpha + ((e4[0] + e4[1]) + (e4[2] + e4[3]));
      } else {
        float cm = -INFINITY;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = c * CK + u * 16 + g * 4 + r;
            const float v = key < N ? s[u][r] * scale : -INFINITY;
            s[u][r] = v;
            cm = fmaxf(cm, v);
          }
        cm = rows4_max(cm);
        const float m_new = fmaxf(m[t], cm);  // finite: every chunk holds at least one real key
        const float alpha = __expf(m[t] - m_new);
        m[t] = m_new;
        l[t] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[t][dt] *= alpha;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = __expf(s[u][r] - m_new);
            s[u][r] = e;
            l[t] += e;
          }
      }
      bf16x8 ph, pl;
      if constexpr (F16) {  // probabilities as one fp16 plane
        const u32x2 p0 = pack16x4<true>(s[0]), p1 = pack16x4<true>(s[1]);
        ph = __builtin_bit_cast(bf16x8, (u32x4){p0[0], p0[1], p1[0], p1[1]});
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ph[j] = (__bf16)s[0][j];
          ph[4 + j] = (__bf16)s[1][j];
          if (SPLIT) {
            pl[j] = (__bf16)(s[0][j] - (float)ph[j]);
            pl[4 + j] = (__bf16)(s[1][j] - (float)ph[4 + j]);
          }
        }
      }
      const int key0 = 4 * g + q4;  // and key0 + 16: the same swizzle (vswz has period 8)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int off0 = key0 * 128 + (((dt * 2 + (p4 >> 1)) ^ vswz(key0)) << 4) + (p4 & 1) * 8;
        const int off1 = off0 + 16 * 128;
        const bf16x8 vh = tr_pair(Vh + off0, Vh + off1);
        o[t][dt] = mma<F16>(vh, ph, o[t][dt]);
        if (SPLIT) {
          const bf16x8 vl = tr_pair(Vl + off0, Vl + off1);
          o[t][dt] = mfma16(vl, ph, o[t][dt]);
          o[t][dt] = mfma16(vh, pl, o[t][dt]);
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < QPW; ++t) {
    const int qt = wave + t * NW;
    if (qt >= nqt) break;
    float lt = l[t];
    if constexpr (F16) {
      lt = rows4_sum(lt);
    } else {
      lt = rows4_sum(lt);
    }
    const float inv = 1.f / lt;
    const int qq = qt * 16 + fr;
    if constexpr (F16) {
      // 16-byte stores: lanes g (even) and g + 1 (16 lanes apart, same query) hold d = 16 dt + 4 g .. + 7 of
      // d-tiles dt and dt + 1; the even lane stores d-tile dt's 8 values, the odd lane d-tile dt + 1's
      const bool odd = g & 1;
      bf16_t* dst = out + ((long)b * N + qq) * out_ld + h * 64 + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; dt += 2) {
        const u32x2 p0 = pack16x4<true>(o[t][dt] * inv), p1 = pack16x4<true>(o[t][dt + 1] * inv);
        const u32x2 snd = odd ? p0 : p1;
        const u32x2 rcv = {xor16_partner(snd[0]), xor16_partner(snd[1])};
        const u32x4 w = odd ? (u32x4){rcv[0], rcv[1], p1[0], p1[1]} : (u32x4){p0[0], p0[1], rcv[0], rcv[1]};
        if (qq < N) *(u32x4*)(dst + (odd ? (dt + 1) * 16 - 4 : dt * 16)) = w;
      }
      continue;
    }
    if (qq < N) {
      bf16_t* dst = out + ((long)b * N + qq) * out_ld + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int d = dt * 16 + 4 * g;
        bf16_t hv[4], lv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) split_bf(o[t][dt][r] * inv, hv[r], lv[r]);
        *(u32x2*)(dst + d) = (u32x2){(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16)};
        if (SPLIT)
          *(u32x2*)(dst + out_lo + d) =
              (u32x2){(uint32_t)lv[0] | ((uint32_t)lv[1] << 16), (uint32_t)lv[2] | ((uint32_t)lv[3] << 16)};
      }
    }
  }
}

// One 16-query tile of the whole-sequence encoder attention (enc_attention_full_kernel / enc_attention_pers_kernel):
// K and V of the (image, head) in LDS (kswz / vswz images), the tile's Q fragments qh[2] in registers.  Returns the
// row sum l of the exact softmax and the unnormalised O = P V (4 d-tiles: lane = query fr, d = 16 dt + 4 g + r).
template <int NKT>
__device__ __forceinline__ float eaf_tile(const char* Ks, const char* Vs, const bf16x8* qh, int N, float sc2, int fr,
                                          int g, f32x4 (&o)[4]) {
  const int q4 = fr >> 2, p4 = fr & 3;
  // raw scores: lane holds query fr, keys 16 kt + 4 g + r
  f32x4 s[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int row = kt * 16 + fr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 kh = *(const bf16x8*)(Ks + row * 128 + (((ks * 4 + g) ^ kswz(row)) << 4));
      acc = mma<true>(kh, qh[ks], acc);
    }
    s[kt] = acc;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)  // the last tile's keys >= N
    if ((NKT - 1) * 16 + g * 4 + r >= N) s[NKT - 1][r] = -INFINITY;
  // maximum over the raw scores with llvm.maximum (gfx950 v_maximum3_f32: no canonicalising v_max per MFMA result,
  // unlike fmaxf, and a compiler-visible VALU read of the XDL results - a v_max3 from inline asm was not spaced from
  // them by the hazard recognizer: 8-wave forms of this kernel read stale maxima, tools/attn_repeat.py); the 1/8
  // scale is folded into the exponent's FMA
  float mx = s[0][0];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int r = (kt == 0 ? 1 : 0); r < 4; ++r) mx = __builtin_elementwise_maximum(mx, s[kt][r]);
  const float mxs = rows4_max(mx) * sc2;
  f32x2 l2 = {0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      s[kt][r] = __builtin_amdgcn_exp2f(fmaf(s[kt][r], sc2, -mxs));
      s[kt][r + 1] = __builtin_amdgcn_exp2f(fmaf(s[kt][r + 1], sc2, -mxs));
      l2 += (f32x2){s[kt][r], s[kt][r + 1]};
    }
  }
  const float l = rows4_sum(l2[0] + l2[1]);
  // O = P V: key-tile pairs (2 c, 2 c + 1) as one 32-deep k-step; P (fp16) element j < 4 -> key 4 g + j of the
  // first tile, j >= 4 -> of the second (odd NKT: the last pair's second tile contributes zeros)
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < (NKT + 1) / 2; ++c) {
    constexpr f32x4 z = {0.f, 0.f, 0.f, 0.f};
    const f32x4 s1 = 2 * c + 1 < NKT ? s[2 * c + 1 < NKT ? 2 * c + 1 : 0] : z;
    const u32x2 p0 = pack16x4<true>(s[2 * c]), p1 = pack16x4<true>(s1);
    const bf16x8 ph = __builtin_bit_cast(bf16x8, (u32x4){p0[0], p0[1], p1[0], p1[1]});
    const int key0 = c * 32 + 4 * g + q4;  // and key0 + 16 (vswz has period 8)
    const int second = 2 * c + 1 < NKT ? 16 * 128 : 0;  // past the last tile: re-read tile 2 c (finite, P = 0)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int off0 = key0 * 128 + (((dt * 2 + (p4 >> 1)) ^ vswz(key0)) << 4) + (p4 & 1) * 8;
      const bf16x8 vh = tr_pair(Vs + off0, Vs + off0 + second);
      o[dt] = mma<true>(vh, ph, o[dt]);
    }
  }
  return l;
}

// Whole-sequence form of the f16 encoder attention (round 4; head-major fp16 qkv, N <= 256): one workgroup of 4 waves
// per (image, head) stages ALL of its K and V (N x 64 fp16 each: 50 KiB at N = 197) in one DMA burst, and each wave
// takes query tiles w, w + 4, ...: S^T = K Q^T over every key tile at once (13 tiles x 2 MFMA at N = 197, 52 score
// registers), one exact softmax (no running max / rescale), P as fp16, O = P V over key-tile pairs with transposed V
// reads.  Against enc_attention_pipe_kernel (7 chunks of 32 keys, a counted wait + barrier and an online-softmax
// rescale per chunk, 2 blocks per CU at 98.5 us per ViT layer): no chunk loop, one barrier, and 3 workgroups per CU
// (50 KiB each) keep 12 waves resident.  Swizzles as the pipelined form (kswz / vswz over the whole image).
// NKT = ceil(N / 16) is a template parameter: every score register, key tile and guard is compile-time, so the
// softmax is straight-line (a runtime key count made hipcc guard each of 16 possible tiles: 2.4x the VALU
// instructions per query tile, and VALU is what bounds this kernel - timing ablations, tools/r4_eaf.sh: 110 us per
// ViT launch, 33 us of it loads only, 74 us without any loads).  The 1/8 scale is folded into the exponent's FMA
// (the maximum is taken over the raw scores).
// abl (tools knob ICAP_EAF_ABL, timing ablations; 0 in a product build): 1 = loads only, 2 = no K / V / Q loads,
// 3 = no output stores
// NW waves per workgroup (round 5, compile-time form ICAP_EAF_NW; 0 = ceil(NKT / 2), every wave at most two query
// tiles): with 4 waves the 13 query tiles of N = 197 give wave 0 four tiles and the others three, so a workgroup
// lasts four tile times for 3.25 tiles of work per wave.
template <int NKT, int NW = 4>
__global__ __launch_bounds__(NW * 64, NW <= 4 ? 3 : 2) void enc_attention_full_kernel(const bf16_t* __restrict__ qkv,
                                                                                     int N, int H, float scale,
                                                                                     bf16_t* out, long out_ld, int abl) {
  constexpr int NQW = (NKT + NW - 1) / NW;  // query tiles per wave (tiles w, w + NW, ...)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int h = blockIdx.x, b = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const bf16_t* qb = qkv + ((long)b * 3 * H + h) * N * 64;  // [q|k|v x head][token][64]
  const bf16_t* kb = qb + (long)H * N * 64;
  const bf16_t* vb = qb + 2L * H * N * 64;
  char* const Ks = smem;                    // [NKT * 16 rows][128 B]
  char* const Vs = smem + NKT * 16 * 128;   // [NKT * 16 rows][128 B]
  // stage: instruction i = 8 rows x 128 B of K (i < NKT * 2) or V; rows >= N read row N - 1 (finite; masked / P = 0)
  {
    const int lrow = lane >> 3, lch = lane & 7;
    constexpr int ni = NKT * 2;
    for (int i = wave; i < (abl == 2 ? 0 : 2 * ni); i += NW) {
      const bool isK = i < ni;
      const int row = (isK ? i : i - ni) * 8 + lrow;
      const int ch = lch ^ (isK ? kswz(row) : vswz(row));
      const bf16_t* src = (isK ? kb : vb) + (long)min(row, N - 1) * 64 + ch * 8;
      lds_dma16(src, (LDS_AS void*)((isK ? Ks : Vs) + (isK ? i : i - ni) * 1024));
    }
  }
  // every query tile of this wave loaded into registers in the same burst as the K / V DMA, so no tile pays its own
  // global-load latency after the barrier
  bf16x8 qreg[NQW][2];
#pragma unroll
  for (int qi = 0; qi < NQW; ++qi) {
    const int q = min((wave + NW * qi) * 16 + fr, N - 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qreg[qi][ks] = abl == 2 ? (bf16x8){} : *(const bf16x8*)(qb + (long)q * 64 + ks * 32 + g * 8);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (abl == 1) {
    if (__builtin_bit_cast(u32x4, qreg[0][0])[0] == 0x12345678u) out[threadIdx.x] = 0;  // keep the loads
    return;
  }
  const float sc2 = scale * 1.44269504088896341f;  // exp2 domain
#pragma unroll
  for (int qi = 0; qi < NQW; ++qi) {
    const int qt = wave + NW * qi;
    if (qt >= NKT) continue;  // (uniform per wave)
    f32x4 o[4];
    const float l = eaf_tile<NKT>(Ks, Vs, qreg[qi], N, sc2, fr, g, o);
    // 16-byte stores: lanes g (even) and g + 1 hold d = 16 dt + 4 g .. + 7 of d-tiles dt and dt + 1
    const float inv = 1.f / l;
    const int qq = qt * 16 + fr;
    const bool odd = g & 1;
    bf16_t* dst = out + ((long)b * N + qq) * out_ld + h * 64 + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 4; dt += 2) {
      const u32x2 a0 = pack16x4<true>(o[dt] * inv), a1 = pack16x4<true>(o[dt + 1] * inv);
      const u32x2 snd = odd ? a0 : a1;
      const u32x2 rcv = {xor16_partner(snd[0]), xor16_partner(snd[1])};
      const u32x4 w = odd ? (u32x4){rcv[0], rcv[1], a1[0], a1[1]} : (u32x4){a0[0], a0[1], rcv[0], rcv[1]};
      if (qq < N && (abl != 3 || w[0] == 0x12345678u)) *(u32x4*)(dst + (odd ? (dt + 1) * 16 - 4 : dt * 16)) = w;
    }
  }
}

// Persistent whole-sequence form (round 5, the default for N <= 240; ICAP_EAF_PERS).  enc_attention_full_kernel's three
// workgroups per CU start together, DMA together and compute together, so a CU alternates between an HBM-bound phase
// (three 75 KiB bursts) and a latency-bound compute phase instead of overlapping them: ≈ 4 generations x (load +
// compute).  Here one 16-wave workgroup per CU walks the (image, head) items it, it + G, ...: K / V live in a 2-item LDS
// ring (2 x 52 KiB at N = 197) and the next item's K / V DMA and Q loads are issued at the top of each item, so they
// land behind this item's compute; one barrier per item (every wave's pieces of item k landed, and every wave done
// reading item k - 1's buffer, which the DMA then refills).  Wave w takes query tile w (and w + NW).
// Counted wait: at the top of item k this wave's outstanding VMEM is [item k's DMA + Q loads][item k - 1's stores] (in
// order), so vmcnt(2 NQW) leaves the stores in flight; every wave issues exactly 2 NQW buffer stores per item (a tile
// it does not own, or rows >= N, store out of the resource's range: dropped), so the count - and the compiler's own
// wait for the Q registers - holds on every path.
// Waves per workgroup (ICAP_EAF_PERS_NW): 16 = one query tile per wave, four waves per SIMD at 108 registers: 71.8 us
// per ViT launch against 75.9 for enc_attention_full_kernel and 91-107 with 8 waves of two tiles (the tile's
// S -> softmax -> P V chain is latency-bound: more waves per SIMD, not fewer larger ones; profiles/r05/attn_pers.txt).
// The SIMD holding waves {w : w = 0 mod 4} carries 4 of the 13 tiles against 3.25 on average (the per-item barrier).
template <int NKT, int NW = 8>
__global__ __launch_bounds__(NW * 64, 1) void enc_attention_pers_kernel(const bf16_t* __restrict__ qkv, int N, int H,
                                                                        int items, float scale, bf16_t* out,
                                                                        long out_ld) {
  constexpr int NQW = (NKT + NW - 1) / NW, MAT = NKT * 16 * 128, ni = NKT * 2;
  static_assert(NQW == 1 || NQW == 2, "the stores-per-item count below");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, g = lane >> 4, lrow = lane >> 3, lch = lane & 7;
  const int G = gridDim.x;
  bf16x8 qn[NQW][2];
  auto issue = [&](int it, int buf) {  // item it's K / V into ring slot buf, its Q fragments into qn
    const int b = it / H, h = it - b * H;
    const bf16_t* qb = qkv + ((long)b * 3 * H + h) * N * 64;  // [q|k|v x head][token][64]
    const bf16_t* kb = qb + (long)H * N * 64;
    const bf16_t* vb = qb + 2L * H * N * 64;
    char* const d = smem + buf * 2 * MAT;
    for (int i = wave; i < 2 * ni; i += NW) {  // rows >= N read row N - 1 (finite; masked / P = 0)
      const bool isK = i < ni;
      const int row = (isK ? i : i - ni) * 8 + lrow;
      const int ch = lch ^ (isK ? kswz(row) : vswz(row));
      lds_dma16((isK ? kb : vb) + (long)min(row, N - 1) * 64 + ch * 8,
                (LDS_AS void*)(d + (isK ? 0 : MAT) + (isK ? i : i - ni) * 1024));
    }
#pragma unroll
    for (int qi = 0; qi < NQW; ++qi) {
      const int q = min((wave + NW * qi) * 16 + fr, N - 1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) qn[qi][ks] = *(const bf16x8*)(qb + (long)q * 64 + ks * 32 + g * 8);
    }
  };
  const float sc2 = scale * 1.44269504088896341f;  // exp2 domain
  int it = blockIdx.x;
  if (it < items) issue(it, 0);
  for (int k = 0; it < items; ++k, it += G) {
    if (k == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * NQW) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16x8 qc[NQW][2];
#pragma unroll
    for (int qi = 0; qi < NQW; ++qi) qc[qi][0] = qn[qi][0], qc[qi][1] = qn[qi][1];
    if (it + G < items) issue(it + G, (k + 1) & 1);
    const char* Ks = smem + (k & 1) * 2 * MAT;
    const int b = it / H, h = it - b * H;
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(out + (long)b * N * out_ld, 0, (int)(N * out_ld * 2), 0x00020000);
#pragma unroll
    for (int qi = 0; qi < NQW; ++qi) {
      const int qt = wave + NW * qi;
      f32x4 o[4] = {};
      float l = 1.f;
      if (qt < NKT) l = eaf_tile<NKT>(Ks, Ks + MAT, qc[qi], N, sc2, fr, g, o);  // (uniform per wave)
      const float inv = 1.f / l;
      const int qq = qt * 16 + fr;
      const bool odd = g & 1;
      // 16-byte stores: lanes g (even) and g + 1 hold d = 16 dt + 4 g .. + 7 of d-tiles dt and dt + 1
      const uint32_t ob = (uint32_t)((qq * out_ld + h * 64 + 4 * g) * 2);
#pragma unroll
      for (int dt = 0; dt < 4; dt += 2) {
        const u32x2 a0 = pack16x4<true>(o[dt] * inv), a1 = pack16x4<true>(o[dt + 1] * inv);
        const u32x2 snd = odd ? a0 : a1;
        const u32x2 rcv = {xor16_partner(snd[0]), xor16_partner(snd[1])};
        const u32x4 w = odd ? (u32x4){rcv[0], rcv[1], a1[0], a1[1]} : (u32x4){a0[0], a0[1], rcv[0], rcv[1]};
        const uint32_t off = ob + (uint32_t)((odd ? (dt + 1) * 16 - 4 : dt * 16) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(w, ro, qq < N ? off : 0x80000000u, 0, 0);
      }
    }
  }
}

#ifndef ICAP_EAF_P32
#define ICAP_EAF_P32 0
#endif
#if ICAP_EAF_P32  // (measured 4 % slower than the 16-wave persistent form: compiled only on request)
// 32-query tiles on v_mfma_f32_32x32x16_f16 (round 5, ICAP_EAF_P32): the persistent form with one 32-query tile per
// wave (8 waves, NB = ceil(N / 32) tiles per item, 2 waves per SIMD).  Against the 16-query tiles the MFMA issue per
// query halves (an MFMA holds the SIMD's issue for 8 of its 32 cycles instead of 8 of 16) and every K / V fragment read
// from LDS serves 32 queries.  S^T = K Q^T per 32-key block (lane: query l & 31, keys (r & 3) + 8 (r >> 2) + 4 (l >> 5)
// of the block in its 16 registers; cdna_hip_programming.md §3 maps); row max / sum over the lane's 16 NB values and
// its partner l ^ 32; P = S^T registers 8 s .. 8 s + 7 as the B operand of k-step s (the same permuted key order in
// the transposed V^T reads); O^T per 32-dim block.  K / V images, swizzles and the ring as enc_attention_pers_kernel
// (rows padded to 32 NB, rows >= N read row N - 1 and are masked / P = 0).  Counted wait: every wave issues exactly 4
// buffer stores per item (2 dim blocks x 2 16-byte stores; a wave without a tile stores out of range).
// Measured (parity exact, tests/test_gpu_6_ops.py): 75.6 against 72.6 us for the 16-wave form - 212 registers leave
// two waves per SIMD, and the tile's S -> softmax -> P V chain stays latency-bound (profiles/r05/attn_pers.txt).
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mma32h(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                0);
}
__device__ __forceinline__ uint32_t xor32_partner(uint32_t v) {
  const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (threadIdx.x & 32) ? p[0] : p[1];
}
template <int NB>
__global__ __launch_bounds__(512, 1) void enc_attention_p32_kernel(const bf16_t* __restrict__ qkv, int N, int H,
                                                                   int items, float scale, bf16_t* out, long out_ld) {
  constexpr int NW = 8, MAT = NB * 32 * 128, ni = NB * 4;  // ni: 8-row DMA pieces per matrix
  static_assert(NB <= NW, "one 32-query tile per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c32 = lane & 31, hh = lane >> 5, lrow = lane >> 3, lch = lane & 7;
  const int G = gridDim.x;
  bf16x8 qn[4];
  auto issue = [&](int it, int buf) {  // item it's K / V into ring slot buf, this wave's Q fragments into qn
    const int b = it / H, h = it - b * H;
    const bf16_t* qb = qkv + ((long)b * 3 * H + h) * N * 64;  // [q|k|v x head][token][64]
    const bf16_t* kb = qb + (long)H * N * 64;
    const bf16_t* vb = qb + 2L * H * N * 64;
    char* const d = smem + buf * 2 * MAT;
    for (int i = wave; i < 2 * ni; i += NW) {
      const bool isK = i < ni;
      const int row = (isK ? i : i - ni) * 8 + lrow;
      const int ch = lch ^ (isK ? kswz(row) : vswz(row));
      lds_dma16((isK ? kb : vb) + (long)min(row, N - 1) * 64 + ch * 8,
                (LDS_AS void*)(d + (isK ? 0 : MAT) + (isK ? i : i - ni) * 1024));
    }
    const int q = min(wave * 32 + c32, N - 1);  // B operand of k-step ks: dims 16 ks + 8 hh .. + 7 of query q
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qn[ks] = *(const bf16x8*)(qb + (long)q * 64 + ks * 16 + hh * 8);
  };
  const float sc2 = scale * 1.44269504088896341f;  // exp2 domain
  // transposed V^T reads: lane 4 qq + pp of its 16-lane group supplies row (key) qq, dims 4 pp .. 4 pp + 3 of the group's
  // 16 dims (dims 16 ((lane >> 4) & 1) of the 32-dim block)
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3, dsub = 16 * ((lane >> 4) & 1);
  int it = blockIdx.x;
  if (it < items) issue(it, 0);
  for (int k = 0; it < items; ++k, it += G) {
    if (k == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16x8 qc[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qc[ks] = qn[ks];
    if (it + G < items) issue(it + G, (k + 1) & 1);
    const char* Ks = smem + (k & 1) * 2 * MAT;
    const char* Vs = Ks + MAT;
    const int b = it / H, h = it - b * H;
    f32x16 o[2] = {};
    float l = 1.f;
    if (wave < NB) {  // (uniform per wave)
      f32x16 sacc[NB];
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) {
        f32x16 a = {};
        const int row = kb * 32 + c32;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const bf16x8 kf = *(const bf16x8*)(Ks + row * 128 + (((2 * ks + hh) ^ kswz(row)) << 4));
          a = mma32h(kf, qc[ks], a);
        }
        sacc[kb] = a;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r)  // the last block's keys >= N
        if ((NB - 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh >= N) sacc[NB - 1][r] = -INFINITY;
      // maximum and sum as four independent chains (two waves per SIMD cannot hide one 112-long dependent chain)
      float m4[4] = {sacc[0][0], sacc[0][1], sacc[0][2], sacc[0][3]};
#pragma unroll
      for (int kb = 0; kb < NB; ++kb)
#pragma unroll
        for (int r = (kb == 0 ? 4 : 0); r < 16; ++r) m4[r & 3] = __builtin_elementwise_maximum(m4[r & 3], sacc[kb][r]);
      float mx = __builtin_elementwise_maximum(__builtin_elementwise_maximum(m4[0], m4[1]),
                                               __builtin_elementwise_maximum(m4[2], m4[3]));
      mx = fmaxf(mx, __uint_as_float(xor32_partner(__float_as_uint(mx))));
      const float mxs = mx * sc2;
      f32x2 l4[4] = {};
#pragma unroll
      for (int kb = 0; kb < NB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          sacc[kb][r] = __builtin_amdgcn_exp2f(fmaf(sacc[kb][r], sc2, -mxs));
          sacc[kb][r + 1] = __builtin_amdgcn_exp2f(fmaf(sacc[kb][r + 1], sc2, -mxs));
          l4[(r >> 1) & 3] += (f32x2){sacc[kb][r], sacc[kb][r + 1]};
        }
      const f32x2 ls = (l4[0] + l4[1]) + (l4[2] + l4[3]);
      l = ls[0] + ls[1];
      l += __uint_as_float(xor32_partner(__float_as_uint(l)));
#pragma unroll
      for (int kb = 0; kb < NB; ++kb)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const f32x16& x = sacc[kb];
          const u32x2 p0 = pack16x4<true>((f32x4){x[8 * st], x[8 * st + 1], x[8 * st + 2], x[8 * st + 3]});
          const u32x2 p1 = pack16x4<true>((f32x4){x[8 * st + 4], x[8 * st + 5], x[8 * st + 6], x[8 * st + 7]});
          const bf16x8 ph = __builtin_bit_cast(bf16x8, (u32x4){p0[0], p0[1], p1[0], p1[1]});
          const int key0 = kb * 32 + 16 * st + 4 * hh + tq;  // and key0 + 8 (vswz has period 8)
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            const int off0 = key0 * 128 + (((4 * db + (dsub >> 3) + (tp >> 1)) ^ vswz(key0)) << 4) + (tp & 1) * 8;
            const bf16x8 vh = tr_pair(Vs + off0, Vs + off0 + 8 * 128);
            o[db] = mma32h(vh, ph, o[db]);
          }
        }
    }
    // O^T block db: lane (query c32, half hh) holds dims 32 db + (r & 3) + 8 (r >> 2) + 4 hh; 16-byte stores of dims
    // 8 m .. 8 m + 7 joined across the partner lane l ^ 32 (hh = 0 keeps m even, hh = 1 m odd)
    const float inv = 1.f / l;
    const int qq = wave * 32 + c32;
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(out + (long)b * N * out_ld, 0, (int)(N * out_ld * 2), 0x00020000);
    const uint32_t ob = (uint32_t)((qq * out_ld + h * 64) * 2);
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int mp = 0; mp < 2; ++mp) {
        const f32x16& x = o[db];
        const u32x2 g0 = pack16x4<true>((f32x4){x[8 * mp], x[8 * mp + 1], x[8 * mp + 2], x[8 * mp + 3]} * inv);
        const u32x2 g1 = pack16x4<true>((f32x4){x[8 * mp + 4], x[8 * mp + 5], x[8 * mp + 6], x[8 * mp + 7]} * inv);
        const u32x2 snd = hh ? g0 : g1;
        const u32x2 rcv = {xor32_partner(snd[0]), xor32_partner(snd[1])};
        const u32x4 w = hh ? (u32x4){rcv[0], rcv[1], g1[0], g1[1]} : (u32x4){g0[0], g0[1], rcv[0], rcv[1]};
        const int dim0 = 32 * db + 8 * (2 * mp + hh);
        __builtin_amdgcn_raw_buffer_store_b128(w, ro, qq < N ? ob + (uint32_t)dim0 * 2 : 0x80000000u, 0, 0);
      }
  }
}

#endif  // ICAP_EAF_P32

#ifndef ICAP_EAF_NW
#define ICAP_EAF_NW 4
#endif
template <int NKT>
hipError_t run_enc_full(const bf16_t* qkv, int B, int N, int H, float scale, bf16_t* out, long out_ld, int abl,
                        hipStream_t s, int max_grid) {
  constexpr int lds = 2 * NKT * 16 * 128;
  constexpr int NW = ICAP_EAF_NW ? ICAP_EAF_NW : (NKT + 1) / 2;
#ifndef ICAP_EAF_PERS_DEFAULT
#define ICAP_EAF_PERS_DEFAULT 1
#endif
  static const int pers = icap_knob("ICAP_EAF_PERS", ICAP_EAF_PERS_DEFAULT);
#ifndef ICAP_EAF_PERS_NW
#define ICAP_EAF_PERS_NW 16
#endif
  constexpr int PNW = ICAP_EAF_PERS_NW;
  // (NKT = 16 spills at 128 registers: the whole-sequence form; the dropped stores' offset is past every row)
#if ICAP_EAF_P32
  if (abl == 0 && (long)N * out_ld * 2 < (1L << 31)) {  // 32-query tiles (enc_attention_p32_kernel)
    constexpr int NB = (NKT + 1) / 2;
    static int cus32 = 0;
    if (!cus32) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus32, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus32 <= 0)
        return hipErrorInvalidValue;
      const hipError_t e = hipFuncSetAttribute((const void*)enc_attention_p32_kernel<NB>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 4 * NB * 32 * 128);
      if (e != hipSuccess) {
        cus32 = 0;
        return e;
      }
    }
    const int items = B * H;
    hipLaunchKernelGGL((enc_attention_p32_kernel<NB>), dim3(std::min(items, cus32)), dim3(512), 4 * NB * 32 * 128, s,
                       qkv, N, H, items, scale, out, out_ld);
    return hipGetLastError();
  }
#endif
  if constexpr (PNW < 16 || NKT < 16) {  // (not instantiated where it would spill)
  if (pers && abl == 0 && (long)N * out_ld * 2 < (1L << 31)) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return hipErrorInvalidValue;
      const hipError_t e = hipFuncSetAttribute((const void*)enc_attention_pers_kernel<NKT, PNW>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 2 * lds);
      if (e != hipSuccess) {
        cus = 0;
        return e;
      }
    }
    // one 16-wave workgroup per CU: under an encoder CU budget (a CU-masked stream, icap_set_encoder_cus) only that
    // many fit at once - a larger grid would run its surplus workgroups as a second round
    const int items = B * H, blocks = max_grid > 0 ? std::min(max_grid, cus) : cus;
    hipLaunchKernelGGL((enc_attention_pers_kernel<NKT, PNW>), dim3(std::min(items, blocks)), dim3(PNW * 64), 2 * lds, s,
                       qkv, N, H, items, scale, out, out_ld);
    return hipGetLastError();
  }
  }
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)enc_attention_full_kernel<NKT, NW>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((enc_attention_full_kernel<NKT, NW>), dim3(H, B), dim3(NW * 64), lds, s, qkv, N, H, scale, out,
                     out_ld, abl);
  return hipGetLastError();
}

template <int NKT, bool SPLIT>
hipError_t run_enc(const bf16_t* qkv, long ld, long lo, int B, int N, int H, float scale, bf16_t* out,
                   long out_ld, long out_lo, hipStream_t s) {
  // one wave per 16-query tile (ViT: 13 of 16 busy; grid: 4); the chunked softmax keeps the
  // score tiles to 4, which fits 128 VGPRs
  constexpr int NW = NKT > 4 ? 16 : 4;
  const int lds = NKT * 16 * 128 * (SPLIT ? 4 : 2);
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)enc_attention_kernel<NKT, SPLIT, NW>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((enc_attention_kernel<NKT, SPLIT, NW>), dim3(H, B), dim3(NW * 64), lds, s, qkv, ld, lo, N, H,
                     scale, out, out_ld, out_lo);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_enc_attention(const bf16_t* qkv, long ld, long lo, int B, int N, int H, float scale,
                                bf16_t* out, long out_ld, long out_lo, int nsplit, hipStream_t s, int head_major,
                                int max_grid) {
  if (N <= 0 || B <= 0) return hipErrorInvalidValue;
  if (head_major && (N <= 64 || N > 256)) return hipErrorInvalidValue;  // only the pipelined form reads it
  if (N <= 64) {
    return nsplit == 2 ? run_enc<4, true>(qkv, ld, lo, B, N, H, scale, out, out_ld, out_lo, s)
                       : run_enc<4, false>(qkv, ld, lo, B, N, H, scale, out, out_ld, out_lo, s);
  }
  if (nsplit == NS_F16) {  // one fp16 plane (ICAP_PREC_F16 encoder): the pipelined form
    if (N > 256) return hipErrorInvalidValue;
    const int lds = 4 * 2 * 32 * 128;
    // two query tiles per wave (8 waves, 119 VGPRs, two blocks per CU): every K/V fragment read from LDS serves
    // 32 queries - 1.57 -> 1.28 ms/step at B = 256 (tools/knob_ab.sh); ICAP_ENC_ATTN16_QPW=1 (tools): 16 waves
    static const int qpw16 = icap_knob("ICAP_ENC_ATTN16_QPW", 2);
    // round 4: the whole-sequence form (enc_attention_full_kernel; tools knob ICAP_ENC_ATTN16_FULL=0: the pipelined
    // form)
    static const int full = icap_knob("ICAP_ENC_ATTN16_FULL", 1);
    if (head_major && full) {
      static const int abl = icap_knob("ICAP_EAF_ABL", 0);
      switch ((N + 15) / 16) {  // N in (64, 256]
        case 5: return run_enc_full<5>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        case 6: return run_enc_full<6>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        case 7: return run_enc_full<7>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        case 8: return run_enc_full<8>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        case 9: return run_enc_full<9>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        case 10: return run_enc_full<10>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        case 11: return run_enc_full<11>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        case 12: return run_enc_full<12>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        case 13: return run_enc_full<13>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        case 14: return run_enc_full<14>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        case 15: return run_enc_full<15>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
        default: return run_enc_full<16>(qkv, B, N, H, scale, out, out_ld, abl, s, max_grid);
      }
    }
    if (head_major && qpw16 == 2)
      hipLaunchKernelGGL((enc_attention_pipe_kernel<false, true, 2, true>), dim3(H, B), dim3(512), lds, s, qkv, ld, lo,
                         N, H, scale, out, out_ld, out_lo);
    else if (head_major)
      hipLaunchKernelGGL((enc_attention_pipe_kernel<false, true, 1, true>), dim3(H, B), dim3(1024), lds, s, qkv, ld, lo,
                         N, H, scale, out, out_ld, out_lo);
    else
      hipLaunchKernelGGL((enc_attention_pipe_kernel<false, false, 1, true>), dim3(H, B), dim3(1024), lds, s, qkv, ld,
                         lo, N, H, scale, out, out_ld, out_lo);
    return hipGetLastError();
  }
  static const int pipe = icap_knob("ICAP_ENC_ATTN_PIPE", 1);  // 0: the stage-everything form for N > 64
  // ICAP_ENC_ATTN_QPW: query tiles per wave (1: 16 waves, 2: 8 waves, 2 blocks/CU)
  static const int qpw = icap_knob("ICAP_ENC_ATTN_QPW", 1) == 2 ? 2 : 1;
  if ((pipe || head_major) && N <= 256) {  // 16 query tiles
    const int lds = 4 * (nsplit == 2 ? 4 : 2) * 32 * 128;
    const dim3 gr(H, B), bl(1024 / qpw);
#define ICAP_ENC_PIPE(SP, HMJ, Q) \
  hipLaunchKernelGGL((enc_attention_pipe_kernel<SP, HMJ, Q>), gr, bl, lds, s, qkv, ld, lo, N, H, scale, out, out_ld, out_lo)
    if (qpw == 2) {
      if (nsplit == 2) { if (head_major) ICAP_ENC_PIPE(true, true, 2); else ICAP_ENC_PIPE(true, false, 2); }
      else { if (head_major) ICAP_ENC_PIPE(false, true, 2); else ICAP_ENC_PIPE(false, false, 2); }
    } else {
      if (nsplit == 2) { if (head_major) ICAP_ENC_PIPE(true, true, 1); else ICAP_ENC_PIPE(true, false, 1); }
      else { if (head_major) ICAP_ENC_PIPE(false, true, 1); else ICAP_ENC_PIPE(false, false, 1); }
    }
#undef ICAP_ENC_PIPE
    return hipGetLastError();
  }
  if (N <= 224) {
    return nsplit == 2 ? run_enc<14, true>(qkv, ld, lo, B, N, H, scale, out, out_ld, out_lo, s)
                       : run_enc<14, false>(qkv, ld, lo, B, N, H, scale, out, out_ld, out_lo, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_dec_self_attn(const float* qkv, int B, int n_new, int t0, int H, float* kc, float* vc, int Lmax,
                                int causal, float scale, bf16_t* out, long lo, int nsplit, hipStream_t s,
                                const int32_t* anc, const int32_t* klen) {
  if (t0 + n_new > Lmax || t0 + n_new > 512 || (anc && n_new != 1)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dec_self_attn_kernel, dim3(H, B), dim3(64), 0, s, qkv, n_new, t0, H, kc, vc, Lmax, causal,
                     scale, out, lo, nsplit, anc, klen);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------------------------
// Cross-attention, key-absorbed form on MFMA (flash-style over 32-key chunks).
// One 16-wave block per query row (LDS-DMA ingest scales with issuing waves, ~6 GB/s each).
//   scores  S^T[s][h] = sum_d mem[s][d] * qt[h][d]       (A = memory rows, B = q~^T, 8 heads in 16)
//           wave w: key tile w & 1, d range [64 (w >> 1), +64); the 8 d-partials are summed in two
//           levels through LDS; x 1/8; online softmax per head (head = lane & 15, lane-local stats)
//   context C^T[d][h] += sum_s mem^T[d][s] * P^T[s][h]    (A = mem^T via ds_read_b64_tr_b16,
//           B = the score accumulators themselves; wave w owns d in [32w, 32w + 32))
// memory and q~ arrive as bf16 planes (hi, lo); every product uses hi.hi + lo.hi + hi.lo.
// LDS: two 32-key chunk buffers x planes x 32 KiB, both in flight from the start (chunk c + 2 is
// issued once chunk c has been consumed); 16-byte chunk c of key row k stored at c ^ (k & 15), so the
// 16 key rows of a ds_read_b128 group hit 16 different banks.
// KS = 2: the chunks of a row pair split over two blocks (a block walks 4 chunks instead of 7 at S = 196
// and the launch fills twice the CUs).  Each block leaves its unnormalised context and softmax
// statistics in xpart with agent-scope stores, waits for them to complete, and takes a ticket on the
// pair's counter; the second block merges the two states (always in part order, so the result does
// not depend on which block finished last), writes the output and resets the counter for the next launch.
namespace {

constexpr int XA_PART_FLOATS = 8 * 1024 + 32;  // per block: context [8][1024 threads] + m, l [16 columns]

template <int NS, int KS>
__global__ __launch_bounds__(1024) void cross_attn_mfma_kernel(const bf16_t* __restrict__ qt, long qt_lo,
                                                               const bf16_t* __restrict__ mem, long mem_lo,
                                                               int rows_per_image, int S, float scale,
                                                               bf16_t* out, long out_lo, float* xpart,
                                                               int* xcnt) {
  constexpr int DM = 512, H = 8, CK = 32;        // model width, heads, keys per chunk
  constexpr int PLANE = CK * DM * 2;             // 32 KiB per plane per chunk
  constexpr int BUF = NS * PLANE;
  constexpr int PER_CHUNK = 2 * NS;              // LDS-DMA instructions per wave per chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = (float*)(smem + 2 * BUF);         // [8 d-groups][2 tiles][4 regs][64 lanes]
  float* tot = red + 8 * 512;                    // [2 tiles][4 regs][64 lanes]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int skt = wave & 1, sdg = wave >> 1;     // score role: key tile, d-group
  // Two query rows of the same image per block: MFMA column fr = (row fr >> 3, head fr & 7), so the
  // second row rides in the columns a single row leaves empty and the image's memory is streamed
  // once for both (beam slots, teacher-forced positions); with one row per image the odd columns
  // stay empty as before.
  const int bpi = (rows_per_image + 1) / 2;      // row pairs per image
  const int pb = blockIdx.x / KS, part = blockIdx.x - pb * KS;
  const int img = pb / bpi, pair = pb - img * bpi;
  const int slot = 2 * pair + (fr >> 3);         // this column's row within the image
  const bool valid = slot < rows_per_image;
  const long r = (long)img * rows_per_image + slot;
  const int hd = fr & 7;
  const bf16_t* mb = mem + (long)img * S * DM;
  const int nchunks = (S + CK - 1) / CK;
  const int cper = (nchunks + KS - 1) / KS, c0 = part * cper, c1 = min(nchunks, c0 + cper);

  // q~ fragments (B operand of the scores): column (row, head), d = 64 sdg + 32 ks + 8 fq + j
  bf16x8 qh[2], ql[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const long off = r * H * DM + hd * DM + sdg * 64 + ks * 32 + fq * 8;
    if (valid) {
      qh[ks] = *(const bf16x8*)(qt + off);
      if (NS == 2) ql[ks] = *(const bf16x8*)(qt + qt_lo + off);
    } else {
      qh[ks] = (bf16x8){};
      ql[ks] = (bf16x8){};
    }
  }

  // chunk staging: wave w loads key rows 2w, 2w + 1 of every plane (1 KiB per instruction);
  // lane-linear LDS destination, source 16-B chunk pre-swizzled.
  auto stage = [&](int c, int buf) {
#pragma unroll
    for (int pl = 0; pl < NS; ++pl) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int key = wave * 2 + i;
        const int g = min(c * CK + key, S - 1);
        const int cs = lane ^ (key & 15);
        const bf16_t* src = mb + (pl ? mem_lo : 0) + (long)g * DM + cs * 8;
        lds_dma16(src, (LDS_AS void*)(smem + buf * BUF + pl * PLANE + key * 1024));
      }
    }
  };

  f32x4 acc[2];
  acc[0] = (f32x4){0.f, 0.f, 0.f, 0.f};
  acc[1] = acc[0];
  float m_run = -INFINITY, l_run = 0.f;
  const int q4 = fr >> 2, p4 = fr & 3;

  stage(c0, 0);
  if (c0 + 1 < c1) stage(c0 + 1, 1);
  for (int c = c0; c < c1; ++c) {
    if (c + 1 < c1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_CHUNK) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const char* cb = smem + ((c - c0) & 1) * BUF;
    {  // partial scores: key tile skt, d-group sdg
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
      const int key = skt * 16 + fr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ch = (sdg * 64 + ks * 32 + fq * 8) >> 3;
        const int off = key * 1024 + ((ch ^ (key & 15)) << 4);
        const bf16x8 mh = *(const bf16x8*)(cb + off);
        a = mfma16(mh, qh[ks], a);
        if (NS == 2) {
          const bf16x8 ml = *(const bf16x8*)(cb + PLANE + off);
          a = mfma16(ml, qh[ks], a);
          a = mfma16(mh, ql[ks], a);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) red[((sdg * 2 + skt) * 4 + j) * 64 + lane] = a[j];
    }
    __syncthreads();
    if (threadIdx.x < 512) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) v += red[g * 512 + threadIdx.x];
      tot[threadIdx.x] = v;
    }
    __syncthreads();
    // total scores (every wave), scale, mask, online softmax per head (= lane & 15)
    f32x4 s[2];
    float cmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = c * CK + kt * 16 + fq * 4 + j;
        const float v = key < S ? tot[(kt * 4 + j) * 64 + lane] * scale : -INFINITY;
        s[kt][j] = v;
        cmax = fmaxf(cmax, v);
      }
    cmax = rows4_max(cmax);
    const float m_new = fmaxf(m_run, cmax);
    const float alpha = __expf(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float e = __expf(s[kt][j] - m_new);
        s[kt][j] = e;
        psum += e;
      }
    psum = rows4_sum(psum);
    l_run = l_run * alpha + psum;
    m_run = m_new;
    // P^T as the B operand (k = key, permuted): element j < 4 -> key 4fq + j, j >= 4 -> 16 + 4fq + j - 4
    bf16x8 ph, pl;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ph[j] = (__bf16)s[0][j];
      ph[4 + j] = (__bf16)s[1][j];
      if (NS == 2) {
        pl[j] = (__bf16)(s[0][j] - (float)ph[j]);
        pl[4 + j] = (__bf16)(s[1][j] - (float)ph[4 + j]);
      }
    }
    // context: C^T[d][h] for this wave's 2 d-tiles; A = mem^T via transposed LDS reads
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      acc[dt] *= alpha;
      const int d = wave * 32 + dt * 16 + 4 * p4;        // this lane's 4 d values in the tr block
      const int k0 = 4 * fq + q4, k1 = k0 + 16;
      const int o0 = k0 * 1024 + ((((d >> 3) ^ (k0 & 15))) << 4) + (d & 7) * 2;
      const int o1 = k1 * 1024 + ((((d >> 3) ^ (k1 & 15))) << 4) + (d & 7) * 2;
      const bf16x8 vh = tr_pair(cb + o0, cb + o1);
      acc[dt] = mfma16(vh, ph, acc[dt]);
      if (NS == 2) {
        const bf16x8 vl = tr_pair(cb + PLANE + o0, cb + PLANE + o1);
        acc[dt] = mfma16(vl, ph, acc[dt]);
        acc[dt] = mfma16(vh, pl, acc[dt]);
      }
    }
    if (c + 2 < c1) {
      __syncthreads();  // every wave is done with buffer (c - c0) & 1
      stage(c + 2, (c - c0) & 1);
    }
  }
  if (KS == 2) {
    float* mine = xpart + ((long)pb * 2 + part) * XA_PART_FLOATS;
    const float* other = xpart + ((long)pb * 2 + (part ^ 1)) * XA_PART_FLOATS;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        __hip_atomic_store(mine + (dt * 4 + rr) * 1024 + threadIdx.x, acc[dt][rr], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 16) {
      __hip_atomic_store(mine + 8 * 1024 + threadIdx.x, m_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(mine + 8 * 1024 + 16 + threadIdx.x, l_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's partial stores are complete
    __syncthreads();                                   // ... and every thread's
    int* flag = (int*)(smem + 2 * BUF + (8 * 512 + 512) * 4);  // after the score totals
    if (threadIdx.x == 0)
      *flag = __hip_atomic_fetch_add(xcnt + pb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*flag == 0) return;  // the partner block merges
    if (threadIdx.x == 0) __hip_atomic_store(xcnt + pb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float om = __hip_atomic_load(other + 8 * 1024 + fr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float ol = __hip_atomic_load(other + 8 * 1024 + 16 + fr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float oa[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      oa[k] = __hip_atomic_load(other + k * 1024 + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // part 0's state first whatever the arrival order
    const float m0 = part ? om : m_run, m1 = part ? m_run : om;
    const float l0 = part ? ol : l_run, l1 = part ? l_run : ol;
    const float mn = fmaxf(m0, m1), f0 = __expf(m0 - mn), f1 = __expf(m1 - mn);
    l_run = __fadd_rn(__fmul_rn(l0, f0), __fmul_rn(l1, f1));
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float x0 = part ? oa[dt * 4 + rr] : acc[dt][rr], x1 = part ? acc[dt][rr] : oa[dt * 4 + rr];
        acc[dt][rr] = __fadd_rn(__fmul_rn(x0, f0), __fmul_rn(x1, f1));
      }
  }
  // C^T layout: lane holds column (row, head), d = 16dt + 4fq + r (4 consecutive d) -> 8-byte stores
  if (valid) {
    const float inv = 1.f / l_run;
    bf16_t* dst = out + r * H * DM + hd * DM + wave * 32;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      bf16_t hv[4], lv[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) split_bf(acc[dt][rr] * inv, hv[rr], lv[rr]);
      const int d = dt * 16 + 4 * fq;
      *(u32x2*)(dst + d) = (u32x2){(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16)};
      if (NS == 2)
        *(u32x2*)(dst + out_lo + d) =
            (u32x2){(uint32_t)lv[0] | ((uint32_t)lv[1] << 16), (uint32_t)lv[2] | ((uint32_t)lv[3] << 16)};
    }
  }
}

constexpr int XA_RED_BYTES = (8 * 512 + 512) * 4 + 16;  // + the KS = 2 ticket

// Cross-attention over a single fp16 memory plane (the parity precisions' decoder: the memory rounded
// once to fp16 adds <= 2^-12 relative to the encoder's own error; CPU emulation, DESIGN.md §3: logit error
// 1.29e-4 -> 1.32e-4 at B = 16, no token changes).  Half the bytes of the bf16 hi/lo planes, so one
// 64-key chunk is 64 KiB: 4 chunks instead of 7 at S = 196, i.e. half the chunk steps (each costs three
// block barriers).  q~ arrives as bf16 hi/lo planes (the chain kernel's output) and is re-split into fp16
// hi/lo fragments once per block; the probabilities are fp16 hi/lo too; every product is
// mem.hi + mem.lo (2 MFMAs instead of 3).  Roles per 64-key chunk:
//   scores  wave w: key tile w & 3, d-group w >> 2 (128 = 4 k-steps); the 4 d-partials summed through LDS
//   context wave w: d in [32w, 32w + 32), keys as 2 k-steps of 32 (key tiles 2s, 2s + 1)
// drop (thr != 0, one row per image): train-mode dropout on the probabilities used for the context (the
// softmax normaliser stays undropped), mask of (row, drop.pos, head * 256 + memory token).
// KS = 2 (no dropout, >= 2 chunks): the chunks of a row pair split over two blocks (chunks [0, c/2) and
// [c/2, c)); each leaves its unnormalised context and softmax statistics (agent-scope stores), and the second
// to take the pair's ticket merges them in part order (deterministic) and resets the ticket (xpart / xcnt as
// cross_attn_mfma_kernel<KS = 2>).
// NB: chunk buffers in the LDS ring.  2: chunk c + 2 is issued after chunk c's context (one barrier more);
// >= 3: chunk c + NB - 1 goes into chunk c - 1's buffer right after chunk c's opening barrier, NB - 1 chunks
// in flight (tools knob ICAP_XATTN16_NB).
template <int KS, int CK, int NB = 2>
__global__ __launch_bounds__(CK * 16) void cross_attn_f16_kernel(const bf16_t* __restrict__ qt, long qt_lo,
                                                              const bf16_t* __restrict__ mem, int rows_per_image,
                                                              int S, float scale, bf16_t* out, long out_lo,
                                                              DropCfg drop, float* gsum, float* xpart, int* xcnt) {
  constexpr int DM = 512, H = 8;
  constexpr int NW = CK / 4, NT = NW * 64;      // waves (4 keys each per chunk), threads
  constexpr int NKT = CK / 16, NDT = DM / NW / 16, NS2 = CK / 32;  // key tiles, d tiles per wave, key k-steps
  constexpr int BUF = CK * DM * 2;              // 64 / 32 KiB per chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = (float*)(smem + NB * BUF);       // [4 d-groups][NKT tiles][4 regs][64 lanes]
  float* tot = red + NKT * 1024;                // [NKT tiles][4 regs][64 lanes]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int skt = wave % NKT, sdg = wave / NKT;
  const int bpi = (rows_per_image + 1) / 2;
  const int pb = blockIdx.x / KS, part = blockIdx.x - pb * KS;
  const int img = pb / bpi, pair = pb - img * bpi;
  const int slot = 2 * pair + (fr >> 3);
  const bool valid = slot < rows_per_image;
  const long r = (long)img * rows_per_image + slot;
  const int hd = fr & 7;
  const bf16_t* mb = mem + (long)img * S * DM;
  const int nchunks = (S + CK - 1) / CK;
  const int cper = (nchunks + KS - 1) / KS, c0 = part * cper, c1 = min(nchunks, c0 + cper);

  // q~ as fp16 hi/lo fragments: column (row, head), d = 128 sdg + 32 ks + 8 fq + j.  (Issuing these loads
  // behind the first chunks' DMA does not pay: the compiler then waits vmcnt(0) for the DMA as well,
  // 7.7 -> 9.6 us at S = 1, tools/xattn_time.py.)
  f16x8 qh[4], ql[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const long off = r * H * DM + hd * DM + sdg * 128 + ks * 32 + fq * 8;
    bf16x8 a = {}, b = {};
    if (valid) {
      a = *(const bf16x8*)(qt + off);
      b = *(const bf16x8*)(qt + qt_lo + off);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = (float)a[j] + (float)b[j];
      const _Float16 h = (_Float16)v;
      qh[ks][j] = h;
      ql[ks][j] = (_Float16)(v - (float)h);
    }
  }

  // chunk staging: wave w loads key rows 4w .. 4w + 3 (1 KiB per instruction), lane-linear LDS
  // destination, source 16-B chunk pre-swizzled c ^ (key & 15)
  auto stage = [&](int c, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int key = wave * 4 + i;
      const int g = min(c * CK + key, S - 1);
      const bf16_t* src = mb + (long)g * DM + (lane ^ (key & 15)) * 8;
      lds_dma16(src, (LDS_AS void*)(smem + buf * BUF + key * 1024));
    }
  };
  auto mma16h = [](f16x8 a, f16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); };

  f32x4 acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) acc[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f, d_run = 0.f;  // d_run: the dropped-probability mass (train mode)
  const int q4 = fr >> 2, p4 = fr & 3;

  if constexpr (NB == 2) {
    if (c0 < c1) stage(c0, 0);
    if (c0 + 1 < c1) stage(c0 + 1, 1);
  } else {
#pragma unroll
    for (int i = 0; i < NB - 1; ++i)
      if (c0 + i < c1) stage(c0 + i, i);
  }
  for (int c = c0; c < c1; ++c) {
    // chunks issued after c (4 DMA instructions each): NB = 2 issued c + 1 after chunk c - 1, NB >= 3 issued
    // c + NB - 2 at chunk c - 1's opening barrier
    const int younger = min(NB == 2 ? 1 : NB - 2, c1 - 1 - c);
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // every wave is past chunk c - 1: its buffer takes chunk c + NB - 1
    if (NB > 2 && c + NB - 1 < c1) stage(c + NB - 1, (c - c0 + NB - 1) % NB);
    const char* cb = smem + ((c - c0) % NB) * BUF;
    {  // partial scores: key tile skt, d-group sdg (the four memory fragments read before the MFMAs: one LDS wait,
       // not one per fragment)
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
      const int key = skt * 16 + fr;
      f16x8 mh[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int ch = (sdg * 128 + ks * 32 + fq * 8) >> 3;
        mh[ks] = *(const f16x8*)(cb + key * 1024 + ((ch ^ (key & 15)) << 4));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        a = mma16h(mh[ks], qh[ks], a);
        a = mma16h(mh[ks], ql[ks], a);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) red[((sdg * NKT + skt) * 4 + j) * 64 + lane] = a[j];
    }
    __syncthreads();
    {  // NT = NKT * 256 threads: one total each
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) v += red[g * NT + threadIdx.x];
      tot[threadIdx.x] = v;
    }
    __syncthreads();
    // total scores (every wave), scale, mask, online softmax per head (= lane & 15)
    f32x4 sc[NKT];
    float cmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = c * CK + kt * 16 + fq * 4 + j;
        const float v = key < S ? tot[(kt * 4 + j) * 64 + lane] * scale : -INFINITY;
        sc[kt][j] = v;
        cmax = fmaxf(cmax, v);
      }
    cmax = rows4_max(cmax);
    const float m_new = fmaxf(m_run, cmax);
    const float alpha = __expf(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float e = __expf(sc[kt][j] - m_new);
        sc[kt][j] = e;
        psum += e;
      }
    psum = rows4_sum(psum);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) acc[dt] *= alpha;
    if (drop.thr) {
      float dsum = 0.f;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = c * CK + kt * 16 + fq * 4 + j;
          if (valid && key < S) sc[kt][j] *= drop_mul(drop, 3, (int)r, drop.pos, hd * 256 + key);
          dsum += sc[kt][j];
        }
      dsum = rows4_sum(dsum);
      d_run = d_run * alpha + dsum;
    }
#pragma unroll
    for (int s2 = 0; s2 < NS2; ++s2) {
      // P^T as the B operand of key tiles 2 s2, 2 s2 + 1 (element j < 4 -> key 4fq + j of the first tile,
      // j >= 4 -> key 4fq + j - 4 of the second), fp16 hi/lo
      f16x8 ph, pl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const _Float16 h0 = (_Float16)sc[2 * s2][j], h1 = (_Float16)sc[2 * s2 + 1][j];
        ph[j] = h0;
        ph[4 + j] = h1;
        pl[j] = (_Float16)(sc[2 * s2][j] - (float)h0);
        pl[4 + j] = (_Float16)(sc[2 * s2 + 1][j] - (float)h1);
      }
      f16x8 vh[NDT];  // every d-tile's transposed memory fragment read before the MFMAs
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int d = wave * (16 * NDT) + dt * 16 + 4 * p4;
        const int k0 = 32 * s2 + 4 * fq + q4, k1 = k0 + 16;
        const int o0 = k0 * 1024 + ((((d >> 3) ^ (k0 & 15))) << 4) + (d & 7) * 2;
        const int o1 = k1 * 1024 + ((((d >> 3) ^ (k1 & 15))) << 4) + (d & 7) * 2;
        vh[dt] = __builtin_bit_cast(f16x8, tr_pair(cb + o0, cb + o1));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        acc[dt] = mma16h(vh[dt], ph, acc[dt]);
        acc[dt] = mma16h(vh[dt], pl, acc[dt]);
      }
    }
    if (NB == 2 && c + 2 < c1) {
      __syncthreads();  // every wave is done with buffer (c - c0) & 1
      stage(c + 2, (c - c0) & 1);
    }
  }
  if (KS == 2) {
    float* mine = xpart + ((long)pb * 2 + part) * XA_PART_FLOATS;
    const float* other = xpart + ((long)pb * 2 + (part ^ 1)) * XA_PART_FLOATS;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        __hip_atomic_store(mine + (dt * 4 + rr) * NT + threadIdx.x, acc[dt][rr], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 16) {
      __hip_atomic_store(mine + 8 * 1024 + threadIdx.x, m_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(mine + 8 * 1024 + 16 + threadIdx.x, l_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's partial stores are complete
    __syncthreads();                                   // ... and every thread's
    int* flag = (int*)(tot + NKT * 256);               // after the score totals
    if (threadIdx.x == 0)
      *flag = __hip_atomic_fetch_add(xcnt + pb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*flag == 0) return;  // the partner block merges
    if (threadIdx.x == 0) __hip_atomic_store(xcnt + pb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float om = __hip_atomic_load(other + 8 * 1024 + fr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float ol = __hip_atomic_load(other + 8 * 1024 + 16 + fr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float oa[NDT * 4];
#pragma unroll
    for (int k = 0; k < NDT * 4; ++k)
      oa[k] = __hip_atomic_load(other + k * NT + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // part 0's state first whatever the arrival order
    const float m0 = part ? om : m_run, m1 = part ? m_run : om;
    const float l0 = part ? ol : l_run, l1 = part ? l_run : ol;
    const float mn = fmaxf(m0, m1), f0 = __expf(m0 - mn), f1 = __expf(m1 - mn);
    l_run = __fadd_rn(__fmul_rn(l0, f0), __fmul_rn(l1, f1));
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float x0 = part ? oa[dt * 4 + rr] : acc[dt][rr], x1 = part ? acc[dt][rr] : oa[dt * 4 + rr];
        acc[dt][rr] = __fadd_rn(__fmul_rn(x0, f0), __fmul_rn(x1, f1));
      }
  }
  if (valid && drop.thr && gsum && wave == 0 && fq == 0) gsum[r * H + hd] = d_run / l_run;
  if (valid) {
    const float inv = 1.f / l_run;
    bf16_t* dst = out + r * H * DM + hd * DM + wave * (16 * NDT);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      bf16_t hv[4], lv[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) split_bf(acc[dt][rr] * inv, hv[rr], lv[rr]);
      const int d = dt * 16 + 4 * fq;
      *(u32x2*)(dst + d) = (u32x2){(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16)};
      *(u32x2*)(dst + out_lo + d) =
          (u32x2){(uint32_t)lv[0] | ((uint32_t)lv[1] << 16), (uint32_t)lv[2] | ((uint32_t)lv[3] << 16)};
    }
  }
}
// LDS of cross_attn_f16_kernel<KS, CK, NB>: NB chunk buffers + partial and total scores + the KS = 2 ticket flag
constexpr int xa16_lds(int ck, int nb = 2) { return nb * ck * 512 * 2 + (ck / 16) * (1024 + 256) * 4 + 16; }
constexpr int XA16_LDS = xa16_lds(64);

// ------------------------------------------------------------------------------------------------
// Cross-attention over the fp16 memory plane, key-split single-burst form (round 4; one decoder row per memory
// image and no dropout: the greedy / sampled decode).  cross_attn_f16_kernel spends its 15.5 us per launch at B = 256
// in its 7-chunk loop (a DMA round trip and three barriers per 32-key chunk, ~2.2 us each) - a row's 196 KiB of
// memory arrive at ~13 GB/s per workgroup.  Here the keys of a row split over two workgroups (part 0: keys [0, SH),
// part 1: [SH, S), SH = ceil(S / 2) rounded up to 16) and each stages its <= 128 keys in ONE DMA burst, then
//   scores   wave w < KT: key tile w (16 keys) x all 512 dims, 16 MFMA 16x16x32 f16 with q~ as the B operand's 16
//            columns = 8 heads x {fp16 hi, fp16 lo} of q~ (one MFMA per k-step covers both planes; column n + 8 is added
//            to column n by a DPP row rotate)
//   softmax  per head over the part's keys: wave maxima / sums through LDS (two barriers), P (fp32) -> LDS
//   context  wave w: dims [64 w, 64 w + 64) = 4 d-tiles x KT / 2 key steps, A = memory^T by transposed LDS reads,
//            B = P as {fp16 hi, fp16 lo} columns (summed as the scores)
// and leaves (unnormalised context, max, sum) with agent-scope stores; the second of the pair to take the row's ticket
// merges part 0 then part 1 (the same operations whatever the arrival order), normalises and writes c as bf16 hi / lo
// planes - the layout cross_attn_f16_kernel writes.  The pair shares an XCD under round-robin dispatch (blocks b and
// b + 8; speed only).  LDS: KTE x 16 keys x 1 KiB (KTE = KT rounded up to even; keys past S read row S - 1, P = 0)
// + 9 KiB.
#ifdef ICAP_TOOLS
#include "attention_tools.h"  // the measured-and-rejected cross-attention forms (tools build only)
#endif

}  // namespace

int cross_attn_splits(int S) {
  // opt-in (ICAP_XATTN_KS=2): 20.7 -> 18.5 us per launch, but the launch then holds every CU and the other
  // decode chain's kernels slow down: bench 6544 -> 6404 captions/s, beam 2973 -> 2791
#ifdef ICAP_TOOLS
  static const int ks = icap_knob("ICAP_XATTN_KS", 1);
  return ks == 2 && (S + 31) / 32 >= 4 ? 2 : 1;
#else
  (void)S;
  return 1;
#endif
}

size_t cross_attn_part_floats(int rows) { return (size_t)rows * 2 * XA_PART_FLOATS; }

// Both key-split forms of the fp16 cross-attention were measured slower and compile into the tools build only
// (a product build has neither kernel and launches the chunk loop):
int cross_attn_f16_splits() {
  // key split of the chunk loop (tools knob ICAP_XATTN16_KS=2; decode 12.8 -> 13.4 ms/step)
#ifdef ICAP_TOOLS
  static const int ks = icap_knob("ICAP_XATTN16_KS", 1);
  return ks == 2 ? 2 : 1;
#else
  return 1;
#endif
}

bool cross_attn_f16s_on() {
  // the key-split single-burst form (cross_attn_f16s_kernel) for one row per image without dropout: tools knob
  // ICAP_XATTN16_S=1.  Inside the three-chain decode graph it measured 18.2 us per launch against 15.5 for the
  // chunk-loop form (decode 14.5 vs 12.2 ms/step, same box, profiles/r04/xattn_split_ab.txt)
#ifdef ICAP_TOOLS
  static const int on = icap_knob("ICAP_XATTN16_S", 0);
  return on != 0;
#else
  return false;
#endif
}

hipError_t launch_cross_attn_f16(const bf16_t* qt, long qt_lo, const bf16_t* mem16, int rows, int rows_per_image,
                                 int S, float scale, bf16_t* out, long out_lo, hipStream_t s, DropCfg drop,
                                 float* gsum, float* xpart, int* xcnt) {
  if (S <= 0 || rows <= 0 || rows_per_image <= 0 || rows % rows_per_image) return hipErrorInvalidValue;
  if (drop.thr && (rows_per_image != 1 || S > 256 || !gsum)) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    {
      const hipError_t e = hipFuncSetAttribute((const void*)cross_attn_f16_kernel<1, 32>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, xa16_lds(32));
      if (e != hipSuccess) return e;
    }
#ifdef ICAP_TOOLS
    for (const void* f : {(const void*)cross_attn_f16_kernel<1, 64>, (const void*)cross_attn_f16_kernel<2, 64>}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, XA16_LDS);
      if (e != hipSuccess) return e;
    }
    {
      const hipError_t e = hipFuncSetAttribute((const void*)cross_attn_f16_kernel<2, 32>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, xa16_lds(32));
      if (e != hipSuccess) return e;
    }
    {
      hipError_t e = hipFuncSetAttribute((const void*)cross_attn_f16_kernel<1, 32, 3>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, xa16_lds(32, 3));
      if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)cross_attn_f16_kernel<1, 32, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                xa16_lds(32, 4));
      if (e != hipSuccess) return e;
    }
#endif
    attr = true;
  }
  // 32-key chunks, 8 waves, 74 KiB of LDS: two blocks (rows) share a CU, so the three decode chains' cross-
  // attentions hold half the CUs (decode 12.70 -> 12.47 ms/step, tools/knob_ab.sh); ICAP_XATTN16_CK=64 (tools):
  // 64-key chunks, 16 waves, 148 KiB (one block per CU)
#ifdef ICAP_TOOLS
  // round 4, measured slower and tools-only: the wave-owned key-tile form for one row per image without dropout
  // (knob ICAP_XATTN16_WK=1; 19.9 against 16.2 us at 256 rows x 196 keys, 10.2 against 7.1 at one key:
  // profiles/r04/xattn_wk.txt)
  static const int wk = icap_knob("ICAP_XATTN16_WK", 0);
  if (rows_per_image == 1 && !drop.thr && S <= 256 && wk && !cross_attn_f16s_on()) {
    static bool wattr = false;
    if (!wattr) {
      const hipError_t e = hipFuncSetAttribute((const void*)cross_attn_wk_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, XWK_LDS);
      if (e != hipSuccess) return e;
      wattr = true;
    }
    hipLaunchKernelGGL(cross_attn_wk_kernel, dim3(rows), dim3(512), XWK_LDS, s, qt, qt_lo, mem16, S, scale, out,
                       out_lo);
    return hipGetLastError();
  }
#endif
#ifdef ICAP_TOOLS
  if (rows_per_image == 1 && !drop.thr && xpart && xcnt && S <= 256 && cross_attn_f16s_on()) {
    static bool sattr = false;
    if (!sattr) {
      const hipError_t e = hipFuncSetAttribute((const void*)cross_attn_f16s_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, xas_lds(256));
      if (e != hipSuccess) return e;
      sattr = true;
    }
    hipLaunchKernelGGL(cross_attn_f16s_kernel, dim3((rows + 7) / 8 * 16), dim3(XAS_THREADS), xas_lds(S), s, qt, qt_lo,
                       mem16, rows, S, scale, out, out_lo, xpart, xcnt);
    return hipGetLastError();
  }
#endif
  static const int ck = icap_knob("ICAP_XATTN16_CK", 32) == 64 ? 64 : 32;
  const int pairs = rows / rows_per_image * ((rows_per_image + 1) / 2);
  const bool ks2 = xpart && xcnt && !drop.thr && S > ck && cross_attn_f16_splits() == 2;
#define XA16(KS_, CK_)                                                                                          \
  hipLaunchKernelGGL((cross_attn_f16_kernel<KS_, CK_>), dim3(KS_ * pairs), dim3(CK_ * 16), xa16_lds(CK_), s, qt, \
                     qt_lo, mem16, rows_per_image, S, scale, out, out_lo, drop, gsum, xpart, xcnt)
#ifdef ICAP_TOOLS
  // ICAP_XATTN16_NB (tools): 3 / 4 chunk buffers (32-key chunks, no key split)
  static const int nb = icap_knob("ICAP_XATTN16_NB", 2);
  if (ck == 32 && !ks2 && (nb == 3 || nb == 4)) {
    if (nb == 3)
      hipLaunchKernelGGL((cross_attn_f16_kernel<1, 32, 3>), dim3(pairs), dim3(512), xa16_lds(32, 3), s, qt, qt_lo, mem16,
                         rows_per_image, S, scale, out, out_lo, drop, gsum, xpart, xcnt);
    else
      hipLaunchKernelGGL((cross_attn_f16_kernel<1, 32, 4>), dim3(pairs), dim3(512), xa16_lds(32, 4), s, qt, qt_lo, mem16,
                         rows_per_image, S, scale, out, out_lo, drop, gsum, xpart, xcnt);
    return hipGetLastError();
  }
#endif
#ifdef ICAP_TOOLS
  if (ck == 32) {
    if (ks2) XA16(2, 32); else XA16(1, 32);
  } else {
    if (ks2) XA16(2, 64); else XA16(1, 64);
  }
#else
  (void)ck, (void)ks2;
  XA16(1, 32);
#endif
#undef XA16
  return hipGetLastError();
}

hipError_t launch_cross_attn_mfma(const bf16_t* qt, long qt_lo, const bf16_t* mem, long mem_lo, int rows,
                                  int rows_per_image, int S, float scale, bf16_t* out, long out_lo, int nsplit,
                                  hipStream_t s, float* xpart, int* xcnt) {
  if (S <= 0 || rows <= 0 || (nsplit != 1 && nsplit != 2)) return hipErrorInvalidValue;
  const int ks = xpart && xcnt ? cross_attn_splits(S) : 1;
  const int lds = 2 * nsplit * 32 * 512 * 2 + XA_RED_BYTES;
  static bool attr = false;
  if (!attr) {
    for (const void* f : {(const void*)cross_attn_mfma_kernel<2, 1>
#ifdef ICAP_TOOLS
                          , (const void*)cross_attn_mfma_kernel<2, 2>
#endif
         }) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               2 * 2 * 32 * 512 * 2 + XA_RED_BYTES);
      if (e != hipSuccess) return e;
    }
    for (const void* f : {(const void*)cross_attn_mfma_kernel<1, 1>
#ifdef ICAP_TOOLS
                          , (const void*)cross_attn_mfma_kernel<1, 2>
#endif
         }) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               2 * 32 * 512 * 2 + XA_RED_BYTES);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  if (rows_per_image <= 0 || rows % rows_per_image) return hipErrorInvalidValue;
  const int pairs = rows / rows_per_image * ((rows_per_image + 1) / 2);  // two rows of an image per block
  // KS = 2: xpart [pairs][2][XA_PART_FLOATS] partial states, xcnt [pairs] tickets (zero between launches)
  float* xp = xpart;
  int* xc = xcnt;
#define ICAP_XA(NSV, KSV)                                                                                      \
  hipLaunchKernelGGL((cross_attn_mfma_kernel<NSV, KSV>), dim3(pairs * KSV), dim3(1024), lds, s, qt, qt_lo, mem, \
                     mem_lo, rows_per_image, S, scale, out, out_lo, xp, xc)
#ifdef ICAP_TOOLS
  if (ks == 2) {
    if (nsplit == 2) ICAP_XA(2, 2); else ICAP_XA(1, 2);
    return hipGetLastError();
  }
#endif
  (void)ks;
  if (nsplit == 2) ICAP_XA(2, 1); else ICAP_XA(1, 1);
#undef ICAP_XA
  return hipGetLastError();
}
