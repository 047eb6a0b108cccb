// Tools-build-only kernel forms of attention.hip (measured and rejected): the wave-owned-key-tile
// and key-split cross-attention kernels.  Included by attention.hip inside its anonymous namespace under
// #ifdef ICAP_TOOLS only - a product build compiles none of this text.
#pragma once

// ------------------------------------------------------------------------------------------------
// Cross-attention, wave-owned key tiles (round 4; one decoder row per memory image, no dropout, S <= 256: the greedy /
// sampled decode).  One 8-wave workgroup per row; wave w owns key tiles w, w + 8 (16 keys each) and runs its own
// online softmax over them - no block barrier until the final merge:
//   stage    the tile's 16 key rows (16 KiB) by LDS-DMA into the wave's own region, one counted wait
//   scores   16 MFMA 16x16x32 f16, A = the key rows, B = q~ as 16 columns = 8 heads x {fp16 hi, fp16 lo} (column
//            n + 8 added to n by a DPP row rotate, both then hold the head's score)
//   context  32 MFMA 16x16x16 f16 (one per 16-dim tile), A = memory^T by ds_read_b64_tr_b16, B = the probabilities
//            straight from the score registers (the MFMA output layout IS the 16x16x16 B layout), columns fp16 hi /
//            fp16 lo of P (summed at the end)
//   merge    every wave's (max, sum, context) through LDS, combined in wave order (deterministic), normalised, bf16 hi /
//            lo planes out - the layout cross_attn_f16_kernel writes.
// Against cross_attn_f16_kernel (7 chunks of 32 keys, three block barriers and an LDS score reduction per chunk: 17 us
// per launch at 256 rows) the per-row critical path is two tile rounds of one wave.  LDS: 128 KiB of key rows (then
// the merge buffer) + 16 KiB of q~ fragments + 512 B.
constexpr int XWK_LDS = 8 * 16 * 1024 + 16 * 1024 + 2 * 64 * 4;
__global__ __launch_bounds__(512) void cross_attn_wk_kernel(const bf16_t* __restrict__ qt, long qt_lo,
                                                            const bf16_t* __restrict__ mem, int S, float scale,
                                                            bf16_t* out, long out_lo) {
  constexpr int DM = 512, H = 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4, q4 = fr >> 2, p4 = fr & 3;
  const int r = blockIdx.x;
  const int KT = (S + 15) >> 4;
  char* const cb = smem + wave * 16 * 1024;  // this wave's key rows [16][1024 B], chunk c at c ^ key
  const bf16_t* mb = mem + (long)r * S * DM;
  auto stage = [&](int t) {
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const int g = min(t * 16 + kk, S - 1);
      lds_dma16(mb + (long)g * DM + (lane ^ kk) * 8, (LDS_AS void*)(cb + kk * 1024));
    }
  };
  if (wave < KT) stage(wave);
  // q~ as the B operand, fragment s (k-step) of lane l at qfrag[s][l]: column n = l & 15 -> head n & 7, plane n >> 3
  // of the fp16 hi / lo split of (bf16 hi + bf16 lo); each thread converts fragments (s, l) = its own two
  f16x8* const qfrag = (f16x8*)(smem + 8 * 16 * 1024);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int s = wave * 2 + u, n = fr, hd = n & 7;
    const long off = (long)r * H * DM + hd * DM + s * 32 + fq * 8;
    const bf16x8 a = *(const bf16x8*)(qt + off), b = *(const bf16x8*)(qt + qt_lo + off);
    f16x8 q;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = (float)a[j] + (float)b[j];
      const _Float16 h = (_Float16)v;
      q[j] = n < 8 ? h : (_Float16)(v - (float)h);
    }
    qfrag[s * 64 + lane] = q;
  }
  __syncthreads();  // q~ fragments written (the key DMA stays in flight: counted per wave below)
  auto ror8 = [](float v) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, true)); };
  f32x4 acc[32];
#pragma unroll
  for (int dt = 0; dt < 32; ++dt) acc[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  for (int t = wave; t < KT; t += 8) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this tile's rows (and the q~ loads) landed
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const f16x8 mh = *(const f16x8*)(cb + fr * 1024 + (((s * 4 + fq) ^ fr) << 4));
      a = __builtin_amdgcn_mfma_f32_16x16x32_f16(mh, qfrag[s * 64 + lane], a, 0, 0, 0);
      if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // four k-steps of reads in flight at a time
    }
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = (a[i] + ror8(a[i])) * scale;  // hi + lo columns (fr < 8 and fr >= 8 both hold the sum)
      v[i] = t * 16 + fq * 4 + i < S ? x : -INFINITY;
    }
    const float mt = rows4_max(fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = __expf(m_run - m_new);
    float ps = 0.f;
    f16x4 pb;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float e = __expf(v[i] - m_new);
      ps += e;
      const _Float16 h = (_Float16)e;
      pb[i] = fr < 8 ? h : (_Float16)(e - (float)h);
    }
    l_run = l_run * alpha + rows4_sum(ps);
    m_run = m_new;
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // 8 d-tiles per group: the transposed reads of one group in flight at a time
      s16x4 ta[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int d = (g * 8 + u) * 16 + 4 * p4, k0 = 4 * fq + q4;
        ta[u] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (LDS_AS s16x4*)(cb + k0 * 1024 + (((d >> 3) ^ k0) << 4) + (d & 7) * 2));
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        f32x4& c = acc[g * 8 + u];
        c *= alpha;
        c = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4, ta[u]), pb, c, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t + 8 < KT) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the region are done
      stage(t + 8);
    }
  }
  // ---- merge: context [wave][head][512] (hi + lo columns summed), then (max, sum) per (wave, head)
  __syncthreads();  // every wave is done with its key region
  float* const mbuf = (float*)smem;
  float* const mst = (float*)(smem + 8 * 16 * 1024 + 16 * 1024);  // [wave][8] maxima, then [wave][8] sums
#pragma unroll
  for (int dt = 0; dt < 32; ++dt) {
    f32x4 c;
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = acc[dt][i] + ror8(acc[dt][i]);
    if (fr < 8) *(f32x4*)(mbuf + (wave * H + fr) * DM + dt * 16 + 4 * fq) = c;
  }
  if (lane < 8) {
    mst[wave * 8 + lane] = m_run;
    mst[64 + wave * 8 + lane] = l_run;
  }
  __syncthreads();
  {
    const int h = threadIdx.x >> 6, d0 = (threadIdx.x & 63) * 8;
    float M = mst[h];
#pragma unroll
    for (int w = 1; w < 8; ++w) M = fmaxf(M, mst[w * 8 + h]);
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, L = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const float mw = mst[w * 8 + h];
      const float f = mw == -INFINITY ? 0.f : __expf(mw - M);
      L += f * mst[64 + w * 8 + h];
      const f32x4 c0 = *(const f32x4*)(mbuf + (w * H + h) * DM + d0), c1 = *(const f32x4*)(mbuf + (w * H + h) * DM + d0 + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] += f * c0[i], o[4 + i] += f * c1[i];
    }
    const float inv = 1.f / L;
    bf16_t hv[8], lv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) split_bf(o[i] * inv, hv[i], lv[i]);
    u32x4 hw, lw;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hw[k] = (uint32_t)hv[2 * k] | ((uint32_t)hv[2 * k + 1] << 16);
      lw[k] = (uint32_t)lv[2 * k] | ((uint32_t)lv[2 * k + 1] << 16);
    }
    bf16_t* dst = out + (long)r * H * DM + h * DM + d0;
    *(u32x4*)dst = hw;
    *(u32x4*)(dst + out_lo) = lw;
  }
}

constexpr int XAS_THREADS = 512;
constexpr int xas_lds(int S) {
  const int sh = ((S + 1) / 2 + 15) & ~15, kte = ((sh / 16) + 1) & ~1;
  return kte * 16 * 1024 + 8 * 64 * 4 * 4 + 2 * 8 * 16 * 4 + 16;
}

__global__ __launch_bounds__(XAS_THREADS) void cross_attn_f16s_kernel(const bf16_t* __restrict__ qt, long qt_lo,
                                                                     const bf16_t* __restrict__ mem, int rows, int S,
                                                                     float scale, bf16_t* out, long out_lo, float* xpart,
                                                                     int* xcnt) {
  constexpr int DM = 512, H = 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int gq = blockIdx.x >> 3, part = gq & 1, r = (gq >> 1) * 8 + (blockIdx.x & 7);
  if (r >= rows) return;  // (the whole workgroup: grid padded to 8 rows)
  const int SH = ((S + 1) / 2 + 15) & ~15;
  const int k0 = part * SH, nk = min(S - k0, SH);              // this part's keys [k0, k0 + nk); nk <= 0: none
  const int KT = nk > 0 ? (nk + 15) >> 4 : 0, KTE = (KT + 1) & ~1;
  char* const cb = smem;                                        // keys [KTE * 16][1024 B], chunk c at c ^ (key & 15)
  float* const pimg = (float*)(smem + KTE * 16 * 1024);         // P [tile][lane][4]
  float* const wmax = pimg + 8 * 64 * 4;                        // [wave][16 columns]
  float* const wsum = wmax + 8 * 16;
  int* const flag = (int*)(wsum + 8 * 16);
  const bf16_t* mb = mem + (long)r * S * DM;

  // stage every key row of the part at once: wave w loads rows w, w + 8, ... (1 KiB per instruction)
  for (int key = wave; key < KTE * 16; key += 8) {
    const int g = min(k0 + key, S - 1);
    lds_dma16(mb + (long)g * DM + (lane ^ (key & 15)) * 8, (LDS_AS void*)(cb + key * 1024));
  }
  // q~ as the B operand: column n = fr -> head n & 7, plane n >> 3 of the fp16 hi / lo split of (bf16 hi + bf16 lo)
  const int hd = fr & 7;
  f16x8 qb[16];
  if (wave < KT) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const long off = (long)r * H * DM + hd * DM + s * 32 + fq * 8;
      const bf16x8 a = *(const bf16x8*)(qt + off), b = *(const bf16x8*)(qt + qt_lo + off);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = (float)a[j] + (float)b[j];
        const _Float16 h = (_Float16)v;
        qb[s][j] = fr < 8 ? h : (_Float16)(v - (float)h);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto mma16h = [](f16x8 a, f16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); };
  auto ror8 = [](float v) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, true)); };
  // ---- scores of key tile `wave`: lane holds column fr (head hd), keys 16 wave + 4 fq + i
  f32x4 sc = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  if (wave < KT) {
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
    const int key = wave * 16 + fr;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const f16x8 mh = *(const f16x8*)(cb + key * 1024 + (((s * 4 + fq) ^ (key & 15)) << 4));
      a = mma16h(mh, qb[s], a);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = (a[i] + ror8(a[i])) * scale;  // hi + lo columns (fr < 8 and fr >= 8 both hold the sum)
      sc[i] = wave * 16 + fq * 4 + i < nk ? v : -INFINITY;
    }
  }
  float mx = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
  mx = rows4_max(mx);
  if (lane < 16) wmax[wave * 16 + lane] = mx;
  __syncthreads();
  float m = wmax[fr];
#pragma unroll
  for (int w = 1; w < 8; ++w) m = fmaxf(m, wmax[w * 16 + fr]);
  f32x4 e = {0.f, 0.f, 0.f, 0.f};
  float es = 0.f;
  if (wave < KT) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      e[i] = sc[i] == -INFINITY ? 0.f : __expf(sc[i] - m);
      es += e[i];
    }
  }
  es = rows4_sum(es);
  if (lane < 16) wsum[wave * 16 + lane] = es;
  if (wave < KTE) *(f32x4*)(pimg + (wave * 64 + lane) * 4) = e;  // (tile KT of an odd KT: zeros)
  __syncthreads();
  float l = 0.f;
#pragma unroll
  for (int w = 0; w < 8; ++w) l += wsum[w * 16 + fr];

  // ---- context: wave w, d-tiles 4 w .. 4 w + 3 (dims 64 w + 16 dt + 4 (fr & 3) + ...), keys in pairs of tiles
  const int q4 = fr >> 2, p4 = fr & 3;
  f32x4 acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int s2 = 0; s2 < KTE / 2; ++s2) {
    // B = P^T: element j < 4 -> key 4 fq + j of tile 2 s2, j >= 4 -> key 4 fq + j - 4 of tile 2 s2 + 1; column fr:
    // fp16 hi of P (fr < 8) or the fp16 lo remainder (fr >= 8)
    const f32x4 p0 = *(const f32x4*)(pimg + ((2 * s2) * 64 + lane) * 4);
    const f32x4 p1 = *(const f32x4*)(pimg + ((2 * s2 + 1) * 64 + lane) * 4);
    f16x8 pb;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const _Float16 h0 = (_Float16)p0[j], h1 = (_Float16)p1[j];
      pb[j] = fr < 8 ? h0 : (_Float16)(p0[j] - (float)h0);
      pb[4 + j] = fr < 8 ? h1 : (_Float16)(p1[j] - (float)h1);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int d = wave * 64 + dt * 16 + 4 * p4;
      const int kk0 = 32 * s2 + 4 * fq + q4, kk1 = kk0 + 16;
      const int o0 = kk0 * 1024 + ((((d >> 3) ^ (kk0 & 15))) << 4) + (d & 7) * 2;
      const int o1 = kk1 * 1024 + ((((d >> 3) ^ (kk1 & 15))) << 4) + (d & 7) * 2;
      const f16x8 vh = __builtin_bit_cast(f16x8, tr_pair(cb + o0, cb + o1));
      acc[dt] = mma16h(vh, pb, acc[dt]);
    }
  }
  // lane (fr < 8): head fr's unnormalised context at dims 64 wave + 16 dt + 4 fq + i
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[dt][i] += ror8(acc[dt][i]);

  // ---- the pair's merge: both parts publish (context, max, sum); the second to take the ticket merges
  constexpr int CF = H * DM;  // context floats per part
  float* mine = xpart + ((long)r * 2 + part) * XA_PART_FLOATS;
  const float* other = xpart + ((long)r * 2 + (part ^ 1)) * XA_PART_FLOATS;
  if (fr < 8) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __hip_atomic_store(mine + hd * DM + wave * 64 + dt * 16 + fq * 4 + i, acc[dt][i], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x < 8) {
    __hip_atomic_store(mine + CF + threadIdx.x, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mine + CF + 8 + threadIdx.x, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's partial stores are complete
  __syncthreads();                                   // ... and every thread's
  if (threadIdx.x == 0) *flag = __hip_atomic_fetch_add(xcnt + r, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (*flag == 0) return;  // the partner merges
  if (threadIdx.x == 0) __hip_atomic_store(xcnt + r, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (fr >= 8) return;
  const float om = __hip_atomic_load(other + CF + hd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float ol = __hip_atomic_load(other + CF + 8 + hd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float m0 = part ? om : m, m1 = part ? m : om, l0 = part ? ol : l, l1 = part ? l : ol;
  const float mn = fmaxf(m0, m1);
  const float f0 = m0 == -INFINITY ? 0.f : __expf(m0 - mn), f1 = m1 == -INFINITY ? 0.f : __expf(m1 - mn);
  const float inv = 1.f / __fadd_rn(__fmul_rn(l0, f0), __fmul_rn(l1, f1));
  bf16_t* dst = out + (long)r * H * DM + hd * DM + wave * 64;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    bf16_t hv[4], lv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float o = __hip_atomic_load(other + hd * DM + wave * 64 + dt * 16 + fq * 4 + i, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
      const float x0 = part ? o : acc[dt][i], x1 = part ? acc[dt][i] : o;
      split_bf(__fadd_rn(__fmul_rn(x0, f0), __fmul_rn(x1, f1)) * inv, hv[i], lv[i]);
    }
    const int d = dt * 16 + 4 * fq;
    *(u32x2*)(dst + d) = (u32x2){(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16)};
    *(u32x2*)(dst + out_lo + d) =
        (u32x2){(uint32_t)lv[0] | ((uint32_t)lv[1] << 16), (uint32_t)lv[2] | ((uint32_t)lv[3] << 16)};
  }
}

