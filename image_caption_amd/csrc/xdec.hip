// Group-persistent decode step: all decoder layers of one KV-cached decode step (one new token per row) in ONE
// launch, with the batch split into 8 row groups of 32 workgroups each.
//
// Why.  The launch-per-block decode spends ~67 us per layer-step in eight dependent
// launches whose duration does not depend on the rows they carry: every block of a fused kernel ingests a whole
// head's / hidden slice's weights (128-256 KiB) for just 16 rows, at the ~25-90 GB/s one CU takes in, behind a
// launch boundary.  The first persistent form (decstep.hip) kept those bodies and measured slower.  Here the
// decomposition changes instead: group g (rows [g R, g R + R), R = ceil(B / 8) <= 32) is served by 32 workgroups
// (blocks b with b % 8 == g: one XCD under the observed round-robin placement - speed only, never correctness),
// and every product of the layer is split over the 32 workgroups BY OUTPUT COLUMNS, so a workgroup ingests 1/32 of
// each weight matrix (16-64 KiB, DMA'd into LDS one phase ahead, before the wait for the phase's inputs) plus the
// group's activation rows (<= 64 KiB).  Row-local work (self-attention per (row, head), LayerNorms, the
// cross-attention) takes one row per workgroup.  Phases of a layer (torch TransformerDecoderLayer, post-LN,
// transformer.py:1144-1153; the key-absorbed cross-attention of DESIGN.md §4):
//   P1  q|k|v = a Wqkv^T + b            48 columns per workgroup (k, v also appended to the KV cache at t0)
//   P2  causal attention                 row s, wave = head (the dec_sa_kernel body)
//   P3  y = ctx Wo^T + bo + x            16 columns
//   P4  x = LN1(y)                       row s
//   P5  q = a Wq^T + bq                  16 columns
//   P6  q~_h = q_h Wk_h                  head s / 4, 128 of its 512 columns
//   P7  c_h = softmax(q~_h mem^T) mem    row s (the cross_attn_f16_kernel<1, 32> body)
//   P8  o_h = c_h Wv_h^T + bv            head s / 4, 16 of its 64 columns
//   P9  y = o Wco^T + bco + x            16 columns
//   P10 x = LN2(y)                       row s
//   P11 slab_s = relu(a W1_s^T + b1_s) W2[:, s]^T   hidden slice s of 64 (fp32 slab per workgroup)
//   P12 x = LN3(x + b2 + sum_s slab_s)   row s (slabs summed in slice order: deterministic)
// Between phases the group meets at a barrier: every handed-off byte is stored write-through (sc1: 16-B buffer
// stores, 8-B agent-scope atomic stores), each storing wave drains vmcnt(0), the workgroup meets, one lane adds 1 to
// the group's counter (agent scope); the consumer's lane 0 polls the counter (relaxed, bounded) and the workgroup
// meets again; every load of handed-off bytes is an sc1 buffer load to registers (MI355X_MICROARCH.md, visibility,
// Valid forms table row 1 - no acquire fence).  The KV cache of earlier positions and the memory plane were written
// by earlier launches.  All 256 workgroups must be co-resident (one per CU: 160 KiB of LDS each); a group whose
// members are not resident gives up after ~1 s through the handle's status word instead of hanging.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace {

constexpr int D = 512, H = 8, HD = 64, FF = 2048, P = 32, NTH = 512;
constexpr int XR = 32;                      // rows of the activation image (R <= 32, padded)
constexpr int XIMG = 64 * 1024;             // activation image [K/64][2 planes][32 rows][128 B] (K = 512)
constexpr int WOFF = 64 * 1024;             // weight region: 96 KiB
constexpr int XDEC_LDS = 160 * 1024;

// The thread index through an opaque copy: inside the layer loop the phases' lane-dependent address arithmetic would
// otherwise be hoisted out of the loop as invariant and held in registers across all layers (spills).
__device__ __forceinline__ int tidx() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// ------------------------------------------------------------------ write-through stores / sc1 loads
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st16(const void* base, long byte_off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc(base), (int)byte_off, 0, 16);
}
__device__ __forceinline__ void st8(void* p, u32x2 v) {
  __hip_atomic_store((unsigned long long*)p, (unsigned long long)v[0] | ((unsigned long long)v[1] << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32x4 ld16(const void* base, long byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), (int)byte_off, 0, 16);
}
__device__ __forceinline__ f32x4 ld16f(const void* base, long byte_off) {
  return __builtin_bit_cast(f32x4, ld16(base, byte_off));
}
// planes of 4 values (lane's 4 consecutive columns) as bf16 hi / lo, write-through
__device__ __forceinline__ void st_planes4(bf16_t* base, long idx, long lo, f32x4 v) {
  uint32_t h0, l0, h1, l1;
  split_bf2((f32x2){v[0], v[1]}, h0, l0);
  split_bf2((f32x2){v[2], v[3]}, h1, l1);
  st8(base + idx, (u32x2){h0, h1});
  st8(base + idx + lo, (u32x2){l0, l1});
}

// ------------------------------------------------------------------ group barrier
struct Bar {
  int* ctr;
  unsigned* err;
  int n;  // barriers passed in this launch
  unsigned long long* trace;  // tools build: this workgroup's stamps [barrier][2], or null
};
__device__ __forceinline__ void stamp(const Bar& b, int k, int which) {
#ifdef ICAP_TOOLS
  if (b.trace && tidx() == 0 && k < XDEC_TRACE_BARRIERS) b.trace[k * 2 + which] = __builtin_amdgcn_s_memrealtime();
#endif
}
// every wave that stored in this phase drains its (write-through) stores, the workgroup meets, one lane arrives.
// Waves that did not store skip the drain, so weight DMA they issued for a later phase stays in flight.
__device__ __forceinline__ void arrive(Bar& b, bool stored = true) {
  if (stored) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(b, b.n, 0);
  if (tidx() == 0) __hip_atomic_fetch_add(b.ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ++b.n;
}
// lane 0 polls until the whole group arrived n times (bounded: a group that cannot complete - members not
// resident, or a bug - gives up through the status word, and every later wait returns at once); then the
// workgroup meets.  The loads that follow are sc1 loads, so no acquire fence is needed (see the file comment).
__device__ __forceinline__ void await(const Bar& b) {
  if (tidx() == 0) {
    const int target = P * b.n;
    unsigned spins = 0;
    while (__hip_atomic_load(b.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if ((++spins & 63) == 0 &&
          (__hip_atomic_load(b.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & DEC_STEP_GAVE_UP))
        break;
      if (spins > (1u << 20)) {
        __hip_atomic_fetch_or(b.err, DEC_STEP_GAVE_UP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  stamp(b, b.n - 1, 1);
}

// ------------------------------------------------------------------ operand images
// 128-B rows, 16-byte chunk c of row r stored at c ^ ((r >> 1) & 7) (conflict-free for the fragment reads)
__device__ __forceinline__ int swz(int r, int c) { return (c ^ ((r >> 1) & 7)) << 4; }
__device__ __forceinline__ bf16x8 frag(const char* img, int r0, int hf) {
  const int lane = tidx() & 63, r = r0 + (lane & 15), c = hf * 4 + (lane >> 4);
  return *(const bf16x8*)(img + r * 128 + swz(r, c));
}
// Weight rows [0, nrows) x 64 k of one k64 step (row stride ld bytes) -> image [nrows][128 B]: one LDS-DMA
// instruction per 8 rows, spread over waves 2..7 (waves 0 and 1 do the small tiles' compute and stores, and wave 0
// polls the barrier counters: they keep no DMA in flight); n counts this wave's instructions
constexpr int DMA_W0 = 2, DMA_NW = 6;
__device__ __forceinline__ void dma_w(const char* src, long ld, int nrows, char* dst, int& rr, int& n) {
  const int lane = tidx() & 63, wave = tidx() >> 6;
  for (int i = 0; i < nrows / 8; ++i) {
    if (wave != DMA_W0 + (rr++ % DMA_NW)) continue;
    const int r = i * 8 + (lane >> 3), pos = lane & 7;
    const char* s = src + (long)r * ld + ((pos ^ ((r >> 1) & 7)) << 4);
    __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)s, (LDS_AS void*)(dst + i * 1024), 16, 0, 0);
    ++n;
  }
}
// rows [n0, n0 + nrows) of W [.][K] (bf16), k in [k0, k0 + 64 K64) -> image [K64][nrows][128 B] at dst
__device__ __forceinline__ void dma_wslice(const bf16_t* W, int K, int n0, int nrows, int k0, int K64, char* dst, int& n) {
  int rr = 0;
  for (int k = 0; k < K64; ++k)
    dma_w((const char*)(W + (long)n0 * K + k0 + k * 64), (long)K * 2, nrows, dst + k * nrows * 128, rr, n);
}
// s_waitcnt vmcnt(n): everything but this wave's n youngest vector-memory operations is complete (n clamped to 24:
// beyond it the wait is merely longer than needed)
__device__ __forceinline__ void vm_wait(int n) {
#define VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n < 0 ? 0 : (n > 24 ? 24 : n)) {
    VMW(0) VMW(1) VMW(2) VMW(3) VMW(4) VMW(5) VMW(6) VMW(7) VMW(8) VMW(9) VMW(10) VMW(11) VMW(12)
    VMW(13) VMW(14) VMW(15) VMW(16) VMW(17) VMW(18) VMW(19) VMW(20) VMW(21) VMW(22) VMW(23) VMW(24)
  }
#undef VMW
}
// The group's activation rows (2 bf16 planes at plane stride lo, row stride ld elements, K columns from col0; rows
// >= R read row R - 1) -> image [K/64][2][32][128 B], through sc1 loads (handed-off bytes) and LDS stores.  Split in
// a load half and a store half so a wave can issue weight DMA for a later phase in between (vm_wait(dma count)).
template <int K>
struct XStage {
  static constexpr int KC = K / 8, PER = XR * KC * 2 / NTH;
  static_assert(PER >= 1 && XR * KC * 2 % NTH == 0, "image shape");
  u32x4 v[PER];
  __device__ __forceinline__ void load(const bf16_t* X, long ld, long lo, int col0, int R) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = tidx() + NTH * i, kc = q % KC, r = (q / KC) % XR, pl = q / (KC * XR);
      v[i] = ld16(X, ((long)pl * lo + (long)min(r, R - 1) * ld + col0 + kc * 8) * 2);
    }
  }
  __device__ __forceinline__ void store(char* img) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = tidx() + NTH * i, kc = q % KC, r = (q / KC) % XR, pl = q / (KC * XR);
      *(u32x4*)(img + (((kc >> 3) * 2 + pl) * XR + r) * 128 + swz(r, kc & 7)) = v[i];
    }
  }
};
// The group's pre-LN rows y (fp32 [rows][512], handed off) -> LN (w, b, eps 1e-5) of every row, as the bf16 planes
// image [8][2][32][128 B]; the workgroup that owns row `own` (own < R) also stores that row's LN output (fp32) to x.
// Thread t holds columns 4 (t & 127) .. + 3 of rows (t >> 7) + 4 i, i < 8: a row's 128 threads are waves 2 w', 2 w' + 1.
struct YStage {
  f32x4 v[8];
  __device__ __forceinline__ void load(const float* y, int R) {
    const int t = tidx(), c4 = t & 127, rb = t >> 7;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = ld16f(y, ((long)min(rb + 4 * i, R - 1) * D + 4 * c4) * 4);
  }
  // red: 2 x 32 x 2 floats of LDS (may lie inside the image: every read of it precedes a barrier before the writes)
  __device__ __forceinline__ void ln_store(char* img, const float* w, const float* b, float* red, float* x, int own) {
    const int t = tidx(), c4 = t & 127, rb = t >> 7, lane = t & 63, half = (t >> 6) & 1;
    float sm[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) sm[i] = wave_sum(v[i][0] + v[i][1] + v[i][2] + v[i][3]);
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < 8; ++i) red[(rb + 4 * i) * 2 + half] = sm[i];
    __syncthreads();
    f32x4 dv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = rb + 4 * i;
      const float mean = (red[r * 2] + red[r * 2 + 1]) / (float)D;
      dv[i] = v[i] - mean;
      sm[i] = wave_sum(dv[i][0] * dv[i][0] + dv[i][1] * dv[i][1] + dv[i][2] * dv[i][2] + dv[i][3] * dv[i][3]);
    }
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < 8; ++i) red[64 + (rb + 4 * i) * 2 + half] = sm[i];
    __syncthreads();
    const f32x4 wv = *(const f32x4*)(w + 4 * c4), bv = *(const f32x4*)(b + 4 * c4);
    const int col = 4 * c4, kc = col >> 3;
    float rs[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = rb + 4 * i;
      rs[i] = 1.0f / sqrtf((red[64 + r * 2] + red[64 + r * 2 + 1]) / (float)D + 1e-5f);
    }
    __syncthreads();  // red is read: the image may overwrite it
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = rb + 4 * i;
      const float rstd = rs[i];
      f32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = dv[i][k] * rstd * wv[k] + bv[k];
      uint32_t h0, l0, h1, l1;
      split_bf2((f32x2){o[0], o[1]}, h0, l0);
      split_bf2((f32x2){o[2], o[3]}, h1, l1);
      char* dst = img + ((kc >> 3) * 2 * XR + r) * 128 + swz(r, kc & 7) + (col & 7) * 2;
      *(u32x2*)dst = (u32x2){h0, h1};
      *(u32x2*)(dst + XR * 128) = (u32x2){l0, l1};
      if (r == own) st16(x, (long)col * 4, o);  // x = the owner row's base
    }
  }
};
// acc += W-image tile (rows w0.., k64 steps [k0, k1)) x X-image rows x0.. (both planes)
__device__ __forceinline__ f32x4 mma_tile(f32x4 acc, const char* wimg, int wrows, int w0, const char* ximg, int x0,
                                          int k0, int k1) {
  for (int k = k0; k < k1; ++k) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const bf16x8 b = frag(wimg + k * wrows * 128, w0, hf);
      acc = mfma16(b, frag(ximg + (k * 2) * XR * 128, x0, hf), acc);
      acc = mfma16(b, frag(ximg + (k * 2 + 1) * XR * 128, x0, hf), acc);
    }
  }
  return acc;
}

// ------------------------------------------------------------------ row LayerNorm (two waves, 4 columns per lane)
// x = LN(v) -> x row (fp32) and the a planes, write-through; v = the lanes' 4 columns (thread t < 128: 4t..4t+3)
__device__ __forceinline__ void ln_row(const XdecArgs& p, int row, f32x4 v, const float* w, const float* b, float* red) {
  const int t = tidx(), lane = t & 63, wave = t >> 6, col = 4 * t;
  float sm = wave_sum(v[0] + v[1] + v[2] + v[3]);
  if (lane == 0 && wave < 2) red[wave] = sm;
  __syncthreads();
  const float mean = (red[0] + red[1]) / (float)D;
  const f32x4 dv = v - mean;
  float q = wave_sum(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2] + dv[3] * dv[3]);
  if (lane == 0 && wave < 2) red[2 + wave] = q;
  __syncthreads();
  if (t >= 128) return;
  const float rstd = 1.0f / sqrtf((red[2] + red[3]) / (float)D + 1e-5f);
  const f32x4 wv = *(const f32x4*)(w + col), bv = *(const f32x4*)(b + col);
  f32x4 y;
#pragma unroll
  for (int k = 0; k < 4; ++k) y[k] = dv[k] * rstd * wv[k] + bv[k];
  st16(p.x, ((long)row * D + col) * 4, y);
  st_planes4(p.a, (long)row * D + col, p.aL, y);
}

// ------------------------------------------------------------------ P2: causal self-attention of (row, head = wave)
// (the attention of dec_sa_kernel: lane l holds key / value j = 4 i + (l >> 4), dims 4 (l & 15) ..).  The cached keys /
// values of positions < t0 were written by earlier launches: the first PRE x 4 are loaded before the phase's barrier.
constexpr int SA_PRE = 8;
struct SaPre {
  f32x4 k[SA_PRE], v[SA_PRE];
};
__device__ __forceinline__ void self_attn_prefetch(const XdecArgs& p, int l, int row, SaPre& pre) {
  const int lane = tidx() & 63, h = tidx() >> 6;
  const int dq = (lane & 15) * 4, jg = lane >> 4, t0 = p.t0;
  const long own = ((long)row * H + h) * p.Lmax * HD;
  const float* kc = p.kc + l * p.kvl;
  const float* vc = p.vc + l * p.kvl;
#pragma unroll
  for (int i = 0; i < SA_PRE; ++i) {
    const int j = 4 * i + jg;
    pre.k[i] = j < t0 ? *(const f32x4*)(kc + own + (long)j * HD + dq) : (f32x4){0.f, 0.f, 0.f, 0.f};
    pre.v[i] = j < t0 ? *(const f32x4*)(vc + own + (long)j * HD + dq) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
}
__device__ __forceinline__ void self_attn(const XdecArgs& p, int l, int row, const SaPre& pre) {
  const int lane = tidx() & 63, h = tidx() >> 6;
  const int dq = (lane & 15) * 4, jg = lane >> 4, t0 = p.t0, nkeys = t0 + 1;
  const long own = ((long)row * H + h) * p.Lmax * HD;
  const float* kc = p.kc + l * p.kvl;
  const float* vc = p.vc + l * p.kvl;
  const long qb = ((long)row * 3 * D + h * HD + dq) * 4;
  const f32x4 q4 = ld16f(p.qv, qb), kcur = ld16f(p.qv, qb + D * 4), vcur = ld16f(p.qv, qb + 2 * D * 4);
  auto hist = [&](const float* cache, int j) -> f32x4 { return *(const f32x4*)(cache + own + (long)j * HD + dq); };
  auto pick = [&](int j, f32x4 pre4) -> f32x4 { return j == t0 ? kcur : (j > t0 ? (f32x4){0.f, 0.f, 0.f, 0.f} : pre4); };
  float s_mine = -INFINITY;
  auto score = [&](int i, f32x4 k4) {
    float part = q4[0] * k4[0];
    part = fmaf(q4[1], k4[1], part);
    part = fmaf(q4[2], k4[2], part);
    part = fmaf(q4[3], k4[3], part);
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    const float sc = __shfl(part, ((lane - 4 * i) & 3) * 16, 64);
    if (lane >= 4 * i && lane < 4 * i + 4) s_mine = lane < nkeys ? sc * 0.125f : -INFINITY;
  };
#pragma unroll
  for (int i = 0; i < SA_PRE; ++i)
    if (4 * i < nkeys) score(i, pick(4 * i + jg, pre.k[i]));
  for (int i = SA_PRE; 4 * i < nkeys; ++i) {
    const int j = 4 * i + jg;
    score(i, pick(j, j < t0 ? hist(kc, j) : kcur));
  }
  const float m = wave_max(s_mine);
  const float e = lane < nkeys ? __expf(s_mine - m) : 0.f;
  const float lsum = wave_sum(e);
  f32x4 ctx = {0.f, 0.f, 0.f, 0.f};
  auto vpick = [&](int j, f32x4 pre4) -> f32x4 { return j == t0 ? vcur : (j > t0 ? (f32x4){0.f, 0.f, 0.f, 0.f} : pre4); };
#pragma unroll
  for (int i = 0; i < SA_PRE; ++i)
    if (4 * i < nkeys) {
      const int j = 4 * i + jg;
      ctx += __shfl(e, min(j, 63), 64) * vpick(j, pre.v[i]);
    }
  for (int i = SA_PRE; 4 * i < nkeys; ++i) {
    const int j = 4 * i + jg;
    ctx += __shfl(e, min(j, 63), 64) * vpick(j, j < t0 ? hist(vc, j) : vcur);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    ctx[k] += __shfl_xor(ctx[k], 16, 64);
    ctx[k] += __shfl_xor(ctx[k], 32, 64);
  }
  ctx /= lsum;
  if (lane < 16) st_planes4(p.ctx, (long)row * D + h * HD + dq, p.ctxL, ctx);
}

// ------------------------------------------------------------------ P7: cross-attention of one row
// The body of cross_attn_f16_kernel<1, 32, 2> (attention.hip) for one row over its image's fp16 memory plane,
// with the handed-off q~ read by sc1 loads and the context stored write-through.  LDS: two 32-key chunk buffers at
// cbuf (64 KiB), score partials / totals at red (10 KiB).
__device__ __forceinline__ bf16x8 tr_pair(const char* p0, const char* p1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)p0);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)p1);
  const s16x8 c = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}
// The first two 32-key chunks of row r's memory (written by an earlier launch) into the chunk buffers: issued before
// the phase's barrier (cross_attn_row then skips its own first staging)
__device__ __forceinline__ void cross_attn_prefetch(const XdecArgs& p, long r, char* cbuf) {
  const int lane = tidx() & 63, wave = tidx() >> 6;
  const bf16_t* mb = p.mem16 + r * (long)p.S * D;
  for (int i = 0; i < 64; ++i) {  // (chunk, key) = (i >> 5, i & 31): one 1-KiB key row per instruction
    if (wave != DMA_W0 + i % DMA_NW || (i >> 5) * 32 >= p.S) continue;
    const int key = i & 31, g = min(i, p.S - 1);
    __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(mb + (long)g * D + (lane ^ (key & 15)) * 8),
                                     (LDS_AS void*)(cbuf + (i >> 5) * 32 * D * 2 + key * 1024), 16, 0, 0);
  }
}
__device__ __forceinline__ void cross_attn_row(const XdecArgs& p, long r, char* cbuf, float* red) {
  constexpr int CK = 32, NW = CK / 4, NT = NW * 64, NKT = CK / 16, NDT = D / NW / 16, NS2 = CK / 32;
  constexpr int BUF = CK * D * 2;
  float* tot = red + NKT * 1024;
  const int lane = tidx() & 63, wave = tidx() >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int skt = wave % NKT, sdg = wave / NKT;
  const int hd = fr & 7;
  const bool valid = (fr >> 3) == 0;  // one row per block: MFMA columns 0..7 (heads), 8..15 unused
  const int S = p.S;
  const bf16_t* mb = p.mem16 + r * (long)S * D;
  const int nchunks = (S + CK - 1) / CK;
  f16x8 qh[4], ql[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const long off = r * H * D + hd * D + sdg * 128 + ks * 32 + fq * 8;
    bf16x8 a = {}, b = {};
    if (valid) {
      a = __builtin_bit_cast(bf16x8, ld16(p.qt, off * 2));
      b = __builtin_bit_cast(bf16x8, ld16(p.qt, (off + p.cL) * 2));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = (float)a[j] + (float)b[j];
      const _Float16 h = (_Float16)v;
      qh[ks][j] = h;
      ql[ks][j] = (_Float16)(v - (float)h);
    }
  }
  auto stage = [&](int c, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int key = wave * 4 + i;
      const int g = min(c * CK + key, S - 1);
      const bf16_t* src = mb + (long)g * D + (lane ^ (key & 15)) * 8;
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src, (LDS_AS void*)(cbuf + buf * BUF + key * 1024), 16,
                                       0, 0);
    }
  };
  auto mma16h = [](f16x8 a, f16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); };
  f32x4 acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) acc[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  const int q4 = fr >> 2, p4 = fr & 3;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the q~ loads and the prefetched chunks 0, 1
  for (int c = 0; c < nchunks; ++c) {
    if (c + 1 < nchunks) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const char* cb = cbuf + (c & 1) * BUF;
    {
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
      const int key = skt * 16 + fr;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int ch = (sdg * 128 + ks * 32 + fq * 8) >> 3;
        const f16x8 mh = *(const f16x8*)(cb + key * 1024 + ((ch ^ (key & 15)) << 4));
        a = mma16h(mh, qh[ks], a);
        a = mma16h(mh, ql[ks], a);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) red[((sdg * NKT + skt) * 4 + j) * 64 + lane] = a[j];
    }
    __syncthreads();
    {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) v += red[g * NT + tidx()];
      tot[tidx()] = v;
    }
    __syncthreads();
    f32x4 sc[NKT];
    float cmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = c * CK + kt * 16 + fq * 4 + j;
        const float v = key < S ? tot[(kt * 4 + j) * 64 + lane] * 0.125f : -INFINITY;
        sc[kt][j] = v;
        cmax = fmaxf(cmax, v);
      }
    cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
    cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
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
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) acc[dt] *= alpha;
#pragma unroll
    for (int s2 = 0; s2 < NS2; ++s2) {
      f16x8 ph, pl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const _Float16 h0 = (_Float16)sc[2 * s2][j], h1 = (_Float16)sc[2 * s2 + 1][j];
        ph[j] = h0;
        ph[4 + j] = h1;
        pl[j] = (_Float16)(sc[2 * s2][j] - (float)h0);
        pl[4 + j] = (_Float16)(sc[2 * s2 + 1][j] - (float)h1);
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int d = wave * (16 * NDT) + dt * 16 + 4 * p4;
        const int k0 = 32 * s2 + 4 * fq + q4, k1 = k0 + 16;
        const int o0 = k0 * 1024 + ((((d >> 3) ^ (k0 & 15))) << 4) + (d & 7) * 2;
        const int o1 = k1 * 1024 + ((((d >> 3) ^ (k1 & 15))) << 4) + (d & 7) * 2;
        const f16x8 vh = __builtin_bit_cast(f16x8, tr_pair(cb + o0, cb + o1));
        acc[dt] = mma16h(vh, ph, acc[dt]);
        acc[dt] = mma16h(vh, pl, acc[dt]);
      }
    }
    if (c + 2 < nchunks) {
      __syncthreads();
      stage(c + 2, c & 1);
    }
  }
  if (valid) {
    const float inv = 1.f / l_run;
    bf16_t* dst = p.c + r * H * D + hd * D + wave * (16 * NDT);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int d = dt * 16 + 4 * fq;
      st_planes4(dst, d, p.cL, acc[dt] * inv);
    }
  }
}

// ------------------------------------------------------------------ the kernel
// LDS: xi [0, 64 K) activation image / cross-attention chunks / LN partials; wr = weights, 96 KiB, in the slots
//   layer start   Wo [0, 16 K)  Wqkv [16, 64 K)                 (DMA'd in the previous layer's P12 or the prologue)
//   P3 ..         Wq_h [16, 80 K)  WkT_h slice [80, 96 K)          (issued at P3 by the non-storing waves)
//   P7 ..         Wv slice [0, 16 K)  Wco slice [16, 32 K)  cross-attention partials [86, 96 K)
//   P8 ..         W1 slice [32, 96 K)                            (issued at P8 by the non-storing waves)
//   P9 ..         W2 slice rows 0..127 [0, 16 K); rows 128..511 [16, 64 K) after FFN-1 (P11)
// Phases of a layer (the file comment's P4 / P6 / P10 merged into their consumers):
//   P1 qkv   P2 attention   P3 out   P456 LN1 + q_h + q~_h   P7 cross-attention   P8 v   P9 cout
//   P11 LN2 + FFN   P12 LN3
__global__ __launch_bounds__(512, 1) void xdec_kernel(XdecArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* xi = smem;
  char* wr = smem + WOFF;
  float* lnred = (float*)smem;  // row LayerNorm partials (the activation image is not live in P12)
  const int g = blockIdx.x & 7, s = blockIdx.x >> 3;
  const int RG = (p.rows + 7) / 8, r0 = g * RG, R = min(RG, p.rows - r0);
  if (R <= 0) return;  // (rows < 8: empty groups)
  const int lane = tidx() & 63, wave = tidx() >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int NRT = (R + 15) / 16;
  Bar bar{p.ctr + g * 16, p.err, 0, p.trace ? p.trace + (long)blockIdx.x * XDEC_TRACE_BARRIERS * 2 : nullptr};
  const bool myrow = s < R;
  const int row = r0 + s;          // P2 / P7 / P12, the LN outputs this workgroup stores
  const int hh = s >> 2, hq = s & 3;  // head and quarter of P456 / P8
  const bool small_st = wave < 2;  // the waves that compute and store the 16-column phases (NRT <= 2)
  int ndma = 0;

  auto prefetch_start = [&](const DecStepLayer& L) {  // Wo, Wqkv of layer L
    dma_wslice(L.Wo, D, 16 * s, 16, 0, 8, wr, ndma);
    dma_wslice(L.Wqkv, D, 48 * s, 48, 0, 8, wr + 16 * 1024, ndma);
  };
  prefetch_start(p.layers[0]);

  for (int l = 0; l < p.n_layers; ++l) {
    const DecStepLayer& L = p.layers[l];
    // ---------------- P1: q|k|v columns [48 s, 48 s + 48) (+ the self-attention's cached keys / values, prefetched)
    SaPre pre;
    if (myrow) self_attn_prefetch(p, l, row, pre);
    {
      XStage<D> xs;
      xs.load(p.a + (long)r0 * D, D, p.aL, 0, R);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      xs.store(xi);
    }
    __syncthreads();
    if (wave < NRT * 3) {
      const int rt = wave / 3, nt = wave % 3;
      f32x4 acc = mma_tile((f32x4){0.f, 0.f, 0.f, 0.f}, wr + 16 * 1024, 48, nt * 16, xi, rt * 16, 0, 8);
      const int m = rt * 16 + fr, c = 48 * s + nt * 16 + 4 * fq;
      acc += *(const f32x4*)(L.bqkv + c);
      if (m < R) {
        const int rw = r0 + m;
        st16(p.qv, ((long)rw * 3 * D + c) * 4, acc);
        if (c >= D) {  // k / v of position t0 into the cache (read by later launches)
          float* cache = (c < 2 * D ? p.kc : p.vc) + l * p.kvl;
          const int cc = c & (D - 1);
          *(f32x4*)(cache + (((long)rw * H + (cc >> 6)) * p.Lmax + p.t0) * HD + (cc & 63)) = acc;
        }
      }
    }
    arrive(bar, wave < NRT * 3);
    await(bar);
    // ---------------- P2: self-attention, row s, wave = head
    if (myrow) self_attn(p, l, row, pre);
    arrive(bar, myrow);
    await(bar);
    // ---------------- P3: y = ctx Wo^T + bo + x, columns [16 s, 16 s + 16); the P456 weights DMA'd meanwhile
    {
      XStage<D> xs;
      xs.load(p.ctx + (long)r0 * D, D, p.ctxL, 0, R);
      ndma = 0;
      dma_wslice(L.Wq, D, hh * HD, HD, 0, 8, wr + 16 * 1024, ndma);  // (the Wqkv slot: consumed in P1)
      int rr = 0;
      dma_w((const char*)(L.WkT + ((long)hh * D + hq * 128) * HD), HD * 2, 128, wr + 80 * 1024, rr, ndma);
      vm_wait(ndma);
      xs.store(xi);
    }
    __syncthreads();
    if (wave < NRT) {
      f32x4 acc = mma_tile((f32x4){0.f, 0.f, 0.f, 0.f}, wr, 16, 0, xi, wave * 16, 0, 8);
      const int m = wave * 16 + fr, c = 16 * s + 4 * fq;
      if (m < R) {
        const long o = ((long)(r0 + m) * D + c) * 4;
        acc += *(const f32x4*)(L.bo + c) + ld16f(p.x, o);
        st16(p.y, o, acc);
      }
    }
    arrive(bar, small_st);
    await(bar);
    // ---------------- P456: x1 = LN1(y) (every workgroup normalises the group's rows; the row owner stores x1),
    // q_h = x1 Wq_h^T + bq_h (all 64 columns of head s / 4), q~_h = q_h Wk_h (128 of its 512 columns)
    {
      YStage ys;
      ys.load(p.y + (long)r0 * D, R);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (also the P456 weights, DMA'd at P2)
      ys.ln_store(xi, L.n1w, L.n1b, (float*)xi, p.x + (long)row * D, myrow ? s : -1);
    }
    __syncthreads();
    {
      const int rt = wave >> 2, nt = wave & 3;
      f32x4 q = {0.f, 0.f, 0.f, 0.f};
      if (rt < NRT) {
        q = mma_tile(q, wr + 16 * 1024, 64, nt * 16, xi, rt * 16, 0, 8);
        q += *(const f32x4*)(L.bq + hh * HD + nt * 16 + 4 * fq);
      }
      __syncthreads();  // the LN image is no longer read: q_h planes -> image [1][2][32][128 B]
      if (rt < NRT) {
        const int m = rt * 16 + fr, n0 = nt * 16 + 4 * fq;
        uint32_t h0, l0, h1, l1;
        split_bf2((f32x2){q[0], q[1]}, h0, l0);
        split_bf2((f32x2){q[2], q[3]}, h1, l1);
        char* dst = xi + m * 128 + swz(m, n0 >> 3) + (n0 & 7) * 2;
        *(u32x2*)dst = (u32x2){h0, h1};
        *(u32x2*)(dst + XR * 128) = (u32x2){l0, l1};
      }
      __syncthreads();
      for (int rt2 = 0; rt2 < NRT; ++rt2) {  // wave = 16-column tile of the 128
        f32x4 acc = mma_tile((f32x4){0.f, 0.f, 0.f, 0.f}, wr + 80 * 1024, 128, wave * 16, xi, rt2 * 16, 0, 1);
        const int m = rt2 * 16 + fr, c = hq * 128 + wave * 16 + 4 * fq;
        if (m < R) st_planes4(p.qt, ((long)(r0 + m) * H + hh) * D + c, p.cL, acc);
      }
    }
    arrive(bar);
    if (myrow) cross_attn_prefetch(p, row, xi);  // (waves 2..7: chunks 0, 1 of this row's memory)
    await(bar);
    // ---------------- P7: cross-attention, row s; the value / output projection slices DMA'd first
    ndma = 0;
    dma_wslice(L.Wv, D, hh * HD + hq * 16, 16, 0, 8, wr, ndma);
    dma_wslice(L.Wco, D, 16 * s, 16, 0, 8, wr + 16 * 1024, ndma);
    if (myrow) cross_attn_row(p, row, xi, (float*)(wr + 86 * 1024));
    arrive(bar);
    await(bar);
    // ---------------- P8: o_h = c_h Wv_h^T + bv, head s / 4, columns 16 (s & 3) of its 64 (bf16 planes in ctx)
    {
      XStage<D> xs;
      xs.load(p.c + (long)r0 * H * D, (long)H * D, p.cL, hh * D, R);
      ndma = 0;
      dma_wslice(L.W1, D, 64 * s, 64, 0, 8, wr + 32 * 1024, ndma);  // FFN-1 slice (the waves that do not store)
      vm_wait(ndma);
      xs.store(xi);
    }
    __syncthreads();
    if (wave < NRT) {
      f32x4 acc = mma_tile((f32x4){0.f, 0.f, 0.f, 0.f}, wr, 16, 0, xi, wave * 16, 0, 8);
      const int m = wave * 16 + fr, c = hh * HD + hq * 16 + 4 * fq;
      acc += *(const f32x4*)(L.bv + c);
      if (m < R) st_planes4(p.ctx, (long)(r0 + m) * D + c, p.ctxL, acc);
    }
    arrive(bar, small_st);
    await(bar);
    // ---------------- P9: y = o Wco^T + bco + x1, columns [16 s, +16)
    {
      XStage<D> xs;
      xs.load(p.ctx + (long)r0 * D, D, p.ctxL, 0, R);
      ndma = 0;
      int rr = 0;
      dma_w((const char*)(L.W2 + 64 * s), (long)FF * 2, 128, wr, rr, ndma);  // W2 rows 0..127 (the Wv slot)
      vm_wait(ndma);
      xs.store(xi);
    }
    __syncthreads();
    if (wave < NRT) {
      f32x4 acc = mma_tile((f32x4){0.f, 0.f, 0.f, 0.f}, wr + 16 * 1024, 16, 0, xi, wave * 16, 0, 8);
      const int m = wave * 16 + fr, c = 16 * s + 4 * fq;
      if (m < R) {
        const long o = ((long)(r0 + m) * D + c) * 4;
        acc += *(const f32x4*)(L.bco + c) + ld16f(p.x, o);
        st16(p.y, o, acc);
      }
    }
    arrive(bar, small_st);
    await(bar);
    // ---------------- P11: x2 = LN2(y) (the row owner stores it), slab s = relu(x2 W1_s^T + b1_s) W2[:, s]^T
    {
      YStage ys;
      ys.load(p.y + (long)r0 * D, R);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (also W1 and W2 rows 0..255)
      ys.ln_store(xi, L.n2w, L.n2b, (float*)xi, p.x + (long)row * D, myrow ? s : -1);
    }
    __syncthreads();
    {
      f32x4 hacc = {0.f, 0.f, 0.f, 0.f};
      const int rt = wave >> 2, nt = wave & 3;
      if (rt < NRT) {
        hacc = mma_tile(hacc, wr + 32 * 1024, 64, nt * 16, xi, rt * 16, 0, 8);
        hacc += *(const f32x4*)(L.b1 + 64 * s + nt * 16 + 4 * fq);
#pragma unroll
        for (int k = 0; k < 4; ++k) hacc[k] = fmaxf(hacc[k], 0.f);
      }
      __syncthreads();  // the LN image and W1 are no longer read
      {  // W2 rows 128..511 -> [16, 64 K) (rows 0..127 arrived during P9; these land under the first tiles)
        int rr = 0, n2 = 0;
        dma_w((const char*)(L.W2 + 128L * FF + 64 * s), (long)FF * 2, 384, wr + 16 * 1024, rr, n2);
      }
      if (rt < NRT) {  // h planes -> image [1 k64][2][32][128 B]
        const int m = rt * 16 + fr, n0 = nt * 16 + 4 * fq;
        uint32_t h0, l0, h1, l1;
        split_bf2((f32x2){hacc[0], hacc[1]}, h0, l0);
        split_bf2((f32x2){hacc[2], hacc[3]}, h1, l1);
        char* dst = xi + m * 128 + swz(m, n0 >> 3) + (n0 & 7) * 2;
        *(u32x2*)dst = (u32x2){h0, h1};
        *(u32x2*)(dst + XR * 128) = (u32x2){l0, l1};
      }
      __syncthreads();  // the h image is complete
      auto ffn2 = [&](int nt2, const char* wimg, int w0) {  // output columns 16 nt2 .. (W2 rows), K = 64
        for (int rt2 = 0; rt2 < NRT; ++rt2) {
          f32x4 o = mma_tile((f32x4){0.f, 0.f, 0.f, 0.f}, wimg, 128, w0, xi, rt2 * 16, 0, 1);
          const int m = rt2 * 16 + fr, c = nt2 * 16 + 4 * fq;
          if (m < R) st16(p.slab, (((long)s * p.rows + r0 + m) * D + c) * 4, o);
        }
      };
      ffn2(wave, wr, wave * 16);  // column tiles 0..7 from rows 0..127 while the rest lands
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int j = 0; j < 3; ++j) {
        const int nt2 = 8 + wave * 3 + j;  // 8..31: quarter 1 + (nt2 - 8) / 8 at [16 K + 16 K ((nt2 - 8) >> 3))
        ffn2(nt2, wr + 16 * 1024 + ((nt2 - 8) >> 3) * 16 * 1024, ((nt2 - 8) & 7) * 16);
      }
    }
    arrive(bar);
    await(bar);
    // ---------------- P12: x = LN3(x2 + b2 + sum of the 32 slabs in slice order), row s; next layer's Wo / Wqkv
    ndma = 0;
    if (l + 1 < p.n_layers) prefetch_start(p.layers[l + 1]);
    if (myrow) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (tidx() < 128) {
        const long o = ((long)row * D + 4 * tidx()) * 4;
        v = ld16f(p.x, o) + *(const f32x4*)(L.b2 + 4 * tidx());
        f32x4 sl[8];
        for (int j0 = 0; j0 < P; j0 += 8) {
#pragma unroll
          for (int j = 0; j < 8; ++j) sl[j] = ld16f(p.slab, o + (long)(j0 + j) * p.rows * D * 4);
#pragma unroll
          for (int j = 0; j < 8; ++j) v += sl[j];
        }
      }
      ln_row(p, row, v, L.n3w, L.n3b, lnred);
    }
    if (l + 1 < p.n_layers) {
      arrive(bar, small_st);
      await(bar);
    }
  }
}

}  // namespace

size_t xdec_state_ints() { return 8 * 16; }

hipError_t launch_xdec(const XdecArgs& a, hipStream_t s) {
  if (a.rows <= 0 || a.rows > 8 * XR || a.n_layers <= 0 || a.n_layers > DEC_STEP_MAX_LAYERS || a.t0 < 0 ||
      a.t0 >= a.Lmax || a.t0 >= 64 || a.S <= 0 || a.S > 256 || !a.ctr || !a.err || !a.layers)
    return hipErrorInvalidValue;
  static int cus = 0;
  if (!cus) {
    const hipError_t e = hipFuncSetAttribute((const void*)xdec_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             XDEC_LDS);
    if (e != hipSuccess) return e;
    int dev = 0;
    hipError_t r = hipGetDevice(&dev);
    if (r == hipSuccess) r = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (r != hipSuccess) return r;
  }
  if (cus < 8 * P) return hipErrorNotSupported;  // every workgroup needs a CU of its own
  hipLaunchKernelGGL(xdec_kernel, dim3(8 * P), dim3(NTH), XDEC_LDS, s, a);
  return hipGetLastError();
}

int xdec_supported() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess)
    return 0;
  return cus >= 8 * P;
}
