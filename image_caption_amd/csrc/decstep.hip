// Persistent decode step: every decoder layer of one KV-cached decode step (one new token per row) in ONE launch.
//
// Why: the launch-per-kernel decode loop spends ~70 us per layer-step in 8 dependent kernels
// (dec_sa 14, LN 5, chain 7, cross-attention 16, chain 7, LN 5, FFN 10, LN 5 us at B = 256) whose duration does not
// depend on how many rows they carry (one chain of 256 rows takes as long as three chains of 85): each is a latency
// chain - launch, weight DMA, input DMA, compute, store drain - not a bandwidth problem.  Here the same bodies run
// as TASKS of one persistent grid (one 1024-thread workgroup per CU), so a task's weight DMA (the largest load,
// independent of the step's data) is issued BEFORE it waits for its inputs, and no launch boundary separates the
// phases of a 16-row tile.
//
// Tasks, per layer l and 16-row tile r (decoder layer = torch TransformerDecoderLayer, post-LN,
// transformer.py:1144-1153):
//   SA(h)  x8   q|k|v of head h, KV-cache append at t0, causal attention, out-projection slab h   (dec_sa_kernel)
//   LN1    x1   x = LN1(x + sum of 8 slabs + bias)                                              (residual LN)
//   C1(h)  x8   q_h = a Wq_h^T + bq_h, q~_h = q_h Wk_h (key-absorbed cross-attention)           (dec_chain_kernel)
//   XA(i)  x16  cross-attention of row i over the fp16 memory plane, 64-key chunks            (cross_attn_f16_kernel)
//   C2(h)  x8   o_h = c_h Wv_h^T + bv_h, out-projection slab h                                  (dec_chain_kernel)
//   LN2    x1
//   FF(j)  x16  relu(a W1_j^T + b1_j) W2[:, j]^T slab j                                         (dec_ffn_kernel)
//   LN3    x1   (not in the last layer: the head kernel folds it, HeadArgs::ln)
// Queue order is phase-major ((layer, phase) outer, tile, index inner): every task's inputs come from tasks earlier
// in the order.  A workgroup takes the next task index from a device counter only after finishing its previous
// task, so the lowest unfinished task always belongs to a running workgroup whose inputs are complete: the grid
// cannot deadlock, whatever the residency or dispatch order (no co-residency assumption).
//
// Hand-offs (MI355X_MICROARCH.md, visibility; cdna_hip_programming.md Guideline 16): every byte another task reads in
// this launch (slabs, residual rows, activation planes, q~, contexts) is stored write-through (sc1: 16-B buffer
// stores, 8-B / 4-B agent-scope atomic stores); each storing wave drains vmcnt(0), the workgroup meets at a barrier,
// and one lane adds 1 to the (layer, phase, tile) counter.  A consumer's wave 0 polls the counter relaxed (bounded,
// giving up through an error word), acquires once (buffer_inv sc1 + vmcnt(0)), and the workgroup meets at a RAW
// s_barrier - the weight DMA the other 15 waves issued before the wait stays in flight across it.  The KV cache of
// earlier positions and the memory plane were written by earlier launches: no hand-off.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace {

constexpr int D = 512, H = 8, HD = 64, FF = 2048, RT = 16, K64 = D / 64;
constexpr int STEP_LDS = 160 * 1024;
enum { P_SA, P_LN1, P_C1, P_XA, P_C2, P_LN2, P_FF, P_LN3, NPH };
constexpr int TASKS_PER_TILE = 59;  // 8 + 1 + 8 + 16 + 8 + 1 + 16 + 1

__device__ __forceinline__ int ph_n(int ph) {
  switch (ph) {
    case P_SA: case P_C1: case P_C2: return 8;
    case P_XA: case P_FF: return 16;
    default: return 1;
  }
}
__device__ __forceinline__ int ph_off(int ph) {  // tasks of the phases before `ph`, per tile
  constexpr int off[NPH + 1] = {0, 8, 9, 17, 33, 41, 42, 58, 59};
  int v = 0;
#pragma unroll
  for (int i = 0; i <= NPH; ++i) v = i == ph ? off[i] : v;
  return v;
}

// The thread index through an opaque (volatile asm) copy: inside the persistent task loop the bodies' lane-dependent
// address arithmetic would otherwise be hoisted out of the loop as invariant and held in registers across every task
// (measured: 128 VGPRs + 225 spilled; a non-inlined task call instead saves ~47 callee-saved VGPRs per call).
__device__ __forceinline__ int tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// ---------------------------------------------------------------- write-through (sc1) stores of handed-off bytes
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, long byte_off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)byte_off, 0, 16);
}
__device__ __forceinline__ void st8(void* p, u32x2 v) {
  __hip_atomic_store((unsigned long long*)p, (unsigned long long)v[0] | ((unsigned long long)v[1] << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st4(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32x2 pack_bf4(const bf16_t* v) {
  return (u32x2){(uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16)};
}

// ---------------------------------------------------------------- hand-off protocol
// Wave 0 waits for *c >= need (relaxed polls with s_sleep, bounded; an error anywhere ends every wait), then
// acquires; the workgroup then meets at a raw barrier (no vmcnt drain: prefetched weights stay in flight).
// Wave 0 must have no VMEM operation of its own in flight here (its vmcnt(0) would wait for it).
// tools build: per-task time stamps (s_memrealtime, 100 MHz) - dequeued, inputs ready, body done - into p.trace
__device__ __forceinline__ void stamp(const DecStepArgs& p, int slot) {
#ifdef ICAP_TOOLS
  if (p.trace && tid() == 0) {
    const int t = p.trace_cur[blockIdx.x];  // written by this same thread at the dequeue
    p.trace[(long)t * 4 + slot] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}
__device__ __forceinline__ void wait_inputs(const DecStepArgs& p, const int* c, int need) {
  if (c && tid() == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
      if (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & DEC_STEP_GAVE_UP) break;
      if (++spins > (1u << 21)) {  // ~1-2 s: a lost producer (a bug) - give up rather than hang the GPU
        __hip_atomic_fetch_or(p.err, DEC_STEP_GAVE_UP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  stamp(p, 1);
}
// Every wave drains its stores, the workgroup meets, one lane publishes.
__device__ __forceinline__ void publish(int* c) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (tid() == 0) __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- LDS-DMA staging (as decode.hip)
// One DMA instruction: rows 8i .. 8i + 7 x 128 B of src (row stride ld bytes) into the LDS image dst[rows][128 B]
// (chunk swizzle c ^ ((r >> 1) & 7)).
__device__ __forceinline__ void dma_8rows(const char* src, long ld, int i, char* dst) {
  const int lane = tid() & 63;
  const int r = i * 8 + (lane >> 3), pos = lane & 7;
  const char* s = src + (long)r * ld + ((pos ^ ((r >> 1) & 7)) << 4);
  __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)s, (LDS_AS void*)(dst + i * 1024), 16, 0, 0);
}
// all 16 waves (inputs, after the acquire)
__device__ __forceinline__ void dma_rows(const char* src, long ld, int nrows, char* dst, int first = 0) {
  const int wave = tid() >> 6;
  for (int i = (wave - first) & 15; i < nrows / 8; i += 16) dma_8rows(src, ld, i, dst);
}
// waves 1..15 only (weights prefetched before wait_inputs: wave 0 keeps its VM counter free for the acquire)
__device__ __forceinline__ void dma_rows_w(const char* src, long ld, int nrows, char* dst, int first = 0) {
  const int wave = tid() >> 6;
  if (wave == 0) return;
  for (int i = ((wave - 1 - first) % 15 + 15) % 15; i < nrows / 8; i += 15) dma_8rows(src, ld, i, dst);
}
__device__ __forceinline__ bf16x8 frag(const char* img, int r0, int hf) {
  const int lane = tid() & 63, r = r0 + (lane & 15), c = hf * 4 + (lane >> 4);
  return *(const bf16x8*)(img + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
}
// the 16 rows x 512 of A (2 planes at plane stride aL, row stride ld elements) -> X image [8 k64][2][16][128 B]
__device__ __forceinline__ void dma_x(const bf16_t* A, long aL, int row0, int rows, char* sx, long ld = D) {
  const int lane = tid() & 63, wave = tid() >> 6;
  const int lr = lane >> 3, pos = lane & 7;
  for (int i = wave; i < K64 * 2 * 2; i += 16) {  // 2 instructions (16 rows) per (k64, plane)
    const int kp = i >> 1, half = i & 1, k64 = kp >> 1, pl = kp & 1;
    const int r = half * 8 + lr, gr = min(row0 + r, rows - 1);
    const char* s = (const char*)(A + pl * aL + (long)gr * ld + k64 * 64) + ((pos ^ ((r >> 1) & 7)) << 4);
    __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)s, (LDS_AS void*)(sx + kp * 2048 + half * 1024), 16, 0, 0);
  }
}
__device__ __forceinline__ void put_planes(char* img, int m, int n0, f32x4 v) {
  bf16_t h[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) split_bf(v[r], h[r], l[r]);
  const int k64 = n0 >> 6, c = (n0 & 63) >> 3;
  char* dst = img + k64 * 2 * 2048 + m * 128 + ((c ^ ((m >> 1) & 7)) << 4) + (n0 & 7) * 2;
  *(u32x2*)dst = pack_bf4(h);
  *(u32x2*)(dst + 2048) = pack_bf4(l);
}
__device__ __forceinline__ f32x4 mma_rows(f32x4 acc, const char* wimg, int wrows, int w0, const char* ximg, int k0,
                                          int k1) {
#pragma unroll 2
  for (int k = k0; k < k1; ++k) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const bf16x8 b = frag(wimg + k * wrows * 128, w0, hf);
      acc = mfma16(b, frag(ximg + k * 2 * 2048, 0, hf), acc);
      acc = mfma16(b, frag(ximg + k * 2 * 2048 + 2048, 0, hf), acc);
    }
  }
  return acc;
}

// ---------------------------------------------------------------- SA(h): dec_sa_kernel as a task
__device__ __forceinline__ void task_sa(const DecStepArgs& p, const DecStepLayer& L, int l, int rt, int h, char* smem, const int* dep) {
  char* ra = smem;                 // 128 KiB weight region
  char* sx = smem + 128 * 1024;    // 32 KiB row region
  float* qkv = (float*)sx;         // after the v projection: [16][192]
  char* sc = sx + 16 * 192 * 4;    // ctx image [1 k64][2][16][128 B]
  const int lane = tid() & 63, wave = tid() >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int row0 = rt * RT;
  const char* wq = (const char*)(L.Wqkv + (long)(h * HD) * D);
  const char* wk = (const char*)(L.Wqkv + (long)(D + h * HD) * D);
  const char* wv = (const char*)(L.Wqkv + (long)(2 * D + h * HD) * D);
  for (int k = 0; k < K64; ++k) {  // Wq_h, Wk_h: image [k64][128 rows] (q rows 0..63, k rows 64..127)
    dma_rows_w(wq + k * 128, D * 2, 64, ra + k * 128 * 128, 8 * (2 * k));
    dma_rows_w(wk + k * 128, D * 2, 64, ra + k * 128 * 128 + 64 * 128, 8 * (2 * k + 1));
  }
  wait_inputs(p, dep, 1);
  dma_x(p.a, p.aL, row0, p.rows, sx);
  constexpr int PRE = 4;  // keys 0..15 prefetched (dec_sa_kernel: 8; registers of the persistent kernel)
  const int dq = (lane & 15) * 4, jg = lane >> 4;
  const int brow = row0 + wave, t0 = p.t0;
  const long own = ((long)brow * H + h) * p.Lmax * HD;
  float* kc = p.kc + l * p.kvl;
  float* vc = p.vc + l * p.kvl;
  auto hist = [&](const float* cache, int j) -> f32x4 { return *(const f32x4*)(cache + own + (long)j * HD + dq); };
  f32x4 kpre[PRE], vpre[PRE];
#pragma unroll
  for (int i = 0; i < PRE; ++i) {
    const int j = 4 * i + jg;
    kpre[i] = brow < p.rows && j < t0 ? hist(kc, j) : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (wave < 8) acc = mma_rows(acc, ra, 128, wave * 16, sx, 0, K64);  // q tiles 0..3, k tiles 4..7
  __syncthreads();  // Wq / Wk no longer read
  for (int k = 0; k < K64; ++k) dma_rows(wv + k * 128, D * 2, 64, ra + k * 64 * 128, 8 * k);
  dma_rows((const char*)(L.Wo + h * HD), D * 2, D, ra + K64 * 64 * 128);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (wave >= 8 && wave < 12) acc = mma_rows(acc, ra, 64, (wave - 8) * 16, sx, 0, K64);  // v tiles
  __syncthreads();  // X image no longer read: it becomes the q|k|v rows
  if (wave < 12) {
    const int c = wave * 16 + 4 * fq;  // column in [q | k | v] of this head
    acc += *(const f32x4*)(L.bqkv + (c >> 6) * D + h * HD + (c & 63));
    *(f32x4*)(qkv + fr * 192 + c) = acc;
  }
  __syncthreads();
  DropCfg dr = p.drop;
  dr.layer = l;
  dr.pos = t0;
  {  // attention, one wave per row over positions 0..t0 (the cache of positions < t0: earlier launches)
    const int r = wave, b = brow, nkeys = t0 + 1;
    const float* qr = qkv + r * 192;
    f32x4 ctx = {0.f, 0.f, 0.f, 0.f};
    float lsum = 1.f;
    if (b < p.rows) {
      if (lane < 16) {  // this step's key / value into the cache (read by later steps only)
        *(f32x4*)(kc + own + (long)t0 * HD + dq) = *(const f32x4*)(qr + 64 + dq);
        *(f32x4*)(vc + own + (long)t0 * HD + dq) = *(const f32x4*)(qr + 128 + dq);
      }
#pragma unroll
      for (int i = 0; i < PRE; ++i) {
        const int j = 4 * i + jg;
        vpre[i] = j < t0 ? hist(vc, j) : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      const f32x4 q4 = *(const f32x4*)(qr + dq);
      const f32x4 kcur = *(const f32x4*)(qr + 64 + dq), vcur = *(const f32x4*)(qr + 128 + dq);
      float s_mine = -INFINITY;
      auto score = [&](int i, f32x4 k4) {
        float part = q4[0] * k4[0];
        part = fmaf(q4[1], k4[1], part);
        part = fmaf(q4[2], k4[2], part);
        part = fmaf(q4[3], k4[3], part);
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
        const float scv = __shfl(part, ((lane - 4 * i) & 3) * 16, 64);
        if (lane >= 4 * i && lane < 4 * i + 4) s_mine = lane < nkeys ? scv * 0.125f : -INFINITY;
      };
      auto pick = [&](int j, f32x4 cur, f32x4 pre) -> f32x4 {
        return j == t0 ? cur : (j > t0 ? (f32x4){0.f, 0.f, 0.f, 0.f} : pre);
      };
#pragma unroll
      for (int i = 0; i < PRE; ++i)
        if (4 * i < nkeys) score(i, pick(4 * i + jg, kcur, kpre[i]));
      for (int i = PRE; 4 * i < nkeys; ++i) {
        const int j = 4 * i + jg;
        const f32x4 k4 = j < t0 ? hist(kc, j) : kcur;
        score(i, pick(j, kcur, k4));
      }
      const float m = wave_max(s_mine);
      const float e = lane < nkeys ? __expf(s_mine - m) : 0.f;
      lsum = wave_sum(e);
      const float ed = dr.thr && lane < nkeys ? e * drop_mul(dr, 1, b, t0, h * 128 + lane) : e;
#pragma unroll
      for (int i = 0; i < PRE; ++i)
        if (4 * i < nkeys) {
          const int j = 4 * i + jg;
          ctx += __shfl(ed, min(j, 63), 64) * pick(j, vcur, vpre[i]);
        }
      for (int i = PRE; 4 * i < nkeys; ++i) {
        const int j = 4 * i + jg;
        const f32x4 v4 = j < t0 ? hist(vc, j) : vcur;
        ctx += __shfl(ed, min(j, 63), 64) * pick(j, vcur, v4);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        ctx[k] += __shfl_xor(ctx[k], 16, 64);
        ctx[k] += __shfl_xor(ctx[k], 32, 64);
      }
      ctx /= lsum;
    }
    if (lane < 16) put_planes(sc, r, dq, ctx);
  }
  __syncthreads();
  // out-projection slab of head h: 16 rows x 512 columns, K = 64 (one k64 step)
  const char* wo = ra + K64 * 64 * 128;
  const __amdgpu_buffer_rsrc_t pr = rsrc_of(p.part);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
    o = mma_rows(o, wo, D, wave * 32 + i * 16, sc, 0, 1);
    const int row = row0 + fr;
    if (row < p.rows) st16(pr, ((long)h * p.PS + (long)row * D + wave * 32 + i * 16 + 4 * fq) * 4, o);
  }
}

// ---------------------------------------------------------------- residual LayerNorm of a 16-row tile
// x = LN(x + (bias + sum of nparts slabs, dropout site `site`)) in place, plus the bf16 hi/lo planes; wave = row,
// lane owns columns 4 lane + 256 c (c = 0, 1).
__device__ __forceinline__ void task_ln(const DecStepArgs& p, int l, int rt, int nparts, const float* bias, const float* w,
                        const float* b, int site, const int* dep, int need) {
  wait_inputs(p, dep, need);
  const int lane = tid() & 63, wave = tid() >> 6;
  const int row = rt * RT + wave;
  if (row >= p.rows) return;
  DropCfg dr = p.drop;
  dr.layer = l;
  dr.pos = p.t0;
  float* xr = p.x + (long)row * D;
  f32x4 v[2], o[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int col = c * 256 + lane * 4;
    v[c] = *(const f32x4*)(xr + col);
    o[c] = *(const f32x4*)(bias + col);
  }
  // slab loads issued 8 at a time before their adds (a runtime-bounded loop waited one round trip per slab)
  for (int s0 = 0; s0 < nparts; s0 += 8) {
    f32x4 pp[8][2];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        pp[s][c] = s0 + s < nparts ? *(const f32x4*)(p.part + (s0 + s) * p.PS + (long)row * D + c * 256 + lane * 4)
                                   : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int c = 0; c < 2; ++c) o[c] += pp[s][c];
  }
  float sm = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (dr.thr == 0) {
      v[c] += o[c];
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[c][k] += o[c][k] * drop_mul(dr, site, row, dr.pos, c * 256 + lane * 4 + k);
    }
    sm += v[c][0] + v[c][1] + v[c][2] + v[c][3];
  }
  const float mean = wave_sum(sm) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    v[c] -= mean;
    q += v[c][0] * v[c][0] + v[c][1] * v[c][1] + v[c][2] * v[c][2] + v[c][3] * v[c][3];
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + 1e-5f);
  const __amdgpu_buffer_rsrc_t xs = rsrc_of(p.x);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int col = c * 256 + lane * 4;
    const f32x4 wv = *(const f32x4*)(w + col), bv = *(const f32x4*)(b + col);
    f32x4 y;
    bf16_t hh[4], ll[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      y[k] = v[c][k] * rstd * wv[k] + bv[k];
      split_bf(y[k], hh[k], ll[k]);
    }
    st16(xs, ((long)row * D + col) * 4, y);
    bf16_t* ob = p.a + (long)row * D + col;
    st8(ob, pack_bf4(hh));
    st8(ob + p.aL, pack_bf4(ll));
  }
}

// ---------------------------------------------------------------- C1 / C2: dec_chain_kernel as a task
//   Y_h = X_h W1_h^T + b1_h (16 x 64, K = 512), O_h = Y_h W2_h^T (16 x 512, K = 64)
// split = true: O_h -> bf16 hi/lo planes at C + row ldc + h c_hstride (q~); else slab h of p.part
__device__ __forceinline__ void task_chain(const DecStepArgs& p, int rt, int h, char* smem, const bf16_t* X, long ldx, long x_lo,
                           long x_hstride, const bf16_t* W1, const float* b1, const bf16_t* W2, long ldw2,
                           long w2_hstride, bool split, bf16_t* C, long ldc, long c_lo, long c_hstride,
                           const float* b1_scale, const int* dep, int need) {
  char* w1i = smem;              // 64 KiB
  char* w2i = smem + 64 * 1024;  // 64 KiB
  char* sx = smem + 128 * 1024;  // 32 KiB: X image, then the k-quarter reduction + Y image
  f32x4* red = (f32x4*)sx;       // [3 quarters][4 tiles][64 lanes]
  char* sy = sx + 12 * 64 * 16;  // Y image [1 k64][2][16][128 B]
  const int lane = tid() & 63, wave = tid() >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int row0 = rt * RT;
  const char* w1 = (const char*)(W1 + (long)h * 64 * D);
  for (int k = 0; k < K64; ++k) dma_rows_w(w1 + k * 128, D * 2, 64, w1i + k * 64 * 128, 8 * k);
  dma_rows_w((const char*)(W2 + (long)h * w2_hstride), ldw2 * 2, D, w2i, 4);
  wait_inputs(p, dep, need);
  dma_x(X + (long)h * x_hstride, x_lo, row0, p.rows, sx, ldx);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = wave & 3, kq = wave >> 2;  // Y tile, k quarter (2 of the 8 k64 steps)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = mma_rows(acc, w1i, 64, t * 16, sx, kq * 2, kq * 2 + 2);
  __syncthreads();  // X no longer read
  if (kq) red[((kq - 1) * 4 + t) * 64 + lane] = acc;
  __syncthreads();
  if (!kq) {
#pragma unroll
    for (int q = 0; q < 3; ++q) acc += red[(q * 4 + t) * 64 + lane];
    const int n = t * 16 + 4 * fq;
    const f32x4 bv = *(const f32x4*)(b1 + h * 64 + n);
    if (b1_scale) acc += bv * b1_scale[(long)min(row0 + fr, p.rows - 1) * H + h];
    else acc += bv;
    put_planes(sy, fr, n, acc);
  }
  __syncthreads();
  const int row = row0 + fr;
  const __amdgpu_buffer_rsrc_t pr = rsrc_of(p.part);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
    o = mma_rows(o, w2i, D, wave * 32 + i * 16, sy, 0, 1);
    const int col = wave * 32 + i * 16 + 4 * fq;
    if (row >= p.rows) continue;
    if (!split) {
      st16(pr, ((long)h * p.PS + (long)row * D + col) * 4, o);
    } else {
      bf16_t hv[4], lv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) split_bf(o[r], hv[r], lv[r]);
      bf16_t* dst = C + (long)row * ldc + (long)h * c_hstride + col;
      st8(dst, pack_bf4(hv));
      st8(dst + c_lo, pack_bf4(lv));
    }
  }
}

// ---------------------------------------------------------------- XA(i): cross_attn_f16_kernel<1, 64> as a task
// One row (greedy / sampled decoding: one row per image), 16 waves, 64-key chunks of the fp16 memory plane in a
// 2-buffer ring; the first two chunks (the memory is an input of the whole decode) are DMA'd before the wait.
__device__ __forceinline__ void task_xa(const DecStepArgs& p, int l, int r, char* smem, const int* dep, int need) {
  constexpr int DM = 512, CK = 64, NW = 16, NT = NW * 64, NKT = CK / 16, NDT = DM / NW / 16, NS2 = CK / 32;
  constexpr int BUF = CK * DM * 2;
  float* red = (float*)(smem + 2 * BUF);  // [4 d-groups][NKT tiles][4 regs][64 lanes]
  float* tot = red + NKT * 1024;          // [NKT tiles][4 regs][64 lanes]
  const int lane = tid() & 63, wave = tid() >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int skt = wave % NKT, sdg = wave / NKT;
  const int S = p.S;
  const bool valid = (fr >> 3) == 0;  // MFMA columns 0..7 = (this row, head); 8..15 unused
  const int hd = fr & 7;
  const bf16_t* mb = p.mem16 + (long)r * S * DM;
  const int nchunks = (S + CK - 1) / CK;
  auto stage = [&](int c, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int key = wave * 4 + i;
      const int g = min(c * CK + key, S - 1);
      const bf16_t* src = mb + (long)g * DM + (lane ^ (key & 15)) * 8;
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src, (LDS_AS void*)(smem + buf * BUF + key * 1024), 16,
                                       0, 0);
    }
  };
  // chunks 0 and 1 before the wait by waves 1..15; wave 0 issues its rows of them after the acquire
  if (wave != 0) {
    stage(0, 0);
    if (nchunks > 1) stage(1, 1);
  }
  wait_inputs(p, dep, need);
  if (wave == 0) {
    stage(0, 0);
    if (nchunks > 1) stage(1, 1);
  }
  DropCfg dr = p.drop;
  dr.layer = l;
  dr.pos = p.t0;
  f16x8 qh[4], ql[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const long off = (long)r * H * DM + hd * DM + sdg * 128 + ks * 32 + fq * 8;
    bf16x8 a = {}, b = {};
    if (valid) {
      a = *(const bf16x8*)(p.qt + off);
      b = *(const bf16x8*)(p.qt + p.cL + off);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = (float)a[j] + (float)b[j];
      const _Float16 hv = (_Float16)v;
      qh[ks][j] = hv;
      ql[ks][j] = (_Float16)(v - (float)hv);
    }
  }
  auto mma16h = [](f16x8 a, f16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); };
  f32x4 acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) acc[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f, d_run = 0.f;
  const int q4 = fr >> 2, p4 = fr & 3;
  for (int c = 0; c < nchunks; ++c) {
    // every wave's DMA of chunk c is complete (the q~ loads above are older than nothing in the ring: wait all)
    if (c + 1 < nchunks) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const char* cb = smem + (c & 1) * BUF;
    {  // partial scores: key tile skt, d-group sdg
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
      for (int g = 0; g < 4; ++g) v += red[g * NT + tid()];
      tot[tid()] = v;
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
    if (dr.thr) {
      float dsum = 0.f;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = c * CK + kt * 16 + fq * 4 + j;
          if (valid && key < S) sc[kt][j] *= drop_mul(dr, 3, r, dr.pos, hd * 256 + key);
          dsum += sc[kt][j];
        }
      dsum += __shfl_xor(dsum, 16, 64);
      dsum += __shfl_xor(dsum, 32, 64);
      d_run = d_run * alpha + dsum;
    }
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
        const s16x4 ta = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(cb + o0));
        const s16x4 tb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(cb + o1));
        const f16x8 vh = __builtin_bit_cast(f16x8, __builtin_shufflevector(ta, tb, 0, 1, 2, 3, 4, 5, 6, 7));
        acc[dt] = mma16h(vh, ph, acc[dt]);
        acc[dt] = mma16h(vh, pl, acc[dt]);
      }
    }
    if (c + 2 < nchunks) {
      __syncthreads();  // every wave is done with buffer c & 1
      stage(c + 2, c & 1);
    }
  }
  if (valid && dr.thr && p.gs && wave == 0 && fq == 0) st4(p.gs + (long)r * H + hd, d_run / l_run);
  if (valid) {
    const float inv = 1.f / l_run;
    bf16_t* dst = p.c + (long)r * H * DM + hd * DM + wave * (16 * NDT);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      bf16_t hv[4], lv[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) split_bf(acc[dt][rr] * inv, hv[rr], lv[rr]);
      const int d = dt * 16 + 4 * fq;
      st8(dst + d, pack_bf4(hv));
      st8(dst + p.cL + d, pack_bf4(lv));
    }
  }
}

// ---------------------------------------------------------------- FF(j): dec_ffn_kernel as a task
__device__ __forceinline__ void task_ff(const DecStepArgs& p, const DecStepLayer& L, int l, int rt, int j, char* smem, const int* dep) {
  char* ra = smem;
  char* sx = smem + 128 * 1024;
  f32x4* red = (f32x4*)sx;        // after FFN-1: [8 tiles][64 lanes]
  char* sh = sx + 8 * 64 * 16;    // h image [2 k64][2][16][128 B]
  const int lane = tid() & 63, wave = tid() >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int row0 = rt * RT;
  const char* w1 = (const char*)(L.W1 + (long)j * 128 * D);
  for (int k = 0; k < K64; ++k) dma_rows_w(w1 + k * 128, D * 2, 128, ra + k * 128 * 128, 16 * k);
  wait_inputs(p, dep, 1);
  dma_x(p.a, p.aL, row0, p.rows, sx);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = wave & 7, kh = wave >> 3;  // FFN-1 tile, k half (4 of the 8 k64 steps)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = mma_rows(acc, ra, 128, t * 16, sx, kh * 4, kh * 4 + 4);
  __syncthreads();  // W1 and X no longer read
  const char* w2 = (const char*)(L.W2 + (long)j * 128);
  for (int k = 0; k < 2; ++k) dma_rows(w2 + k * 128, FF * 2, D, ra + k * D * 128);
  if (kh) red[t * 64 + lane] = acc;
  __syncthreads();
  if (!kh) {
    acc += red[t * 64 + lane];
    const int n = t * 16 + 4 * fq;
    acc += *(const f32x4*)(L.b1 + j * 128 + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = fmaxf(acc[r], 0.f);
    if (p.drop.thr) {
      DropCfg dr = p.drop;
      dr.layer = l;
      dr.pos = p.t0;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] *= drop_mul(dr, 5, row0 + fr, dr.pos, j * 128 + n + r);
    }
    put_planes(sh, fr, n, acc);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const __amdgpu_buffer_rsrc_t pr = rsrc_of(p.part);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
    o = mma_rows(o, ra, D, wave * 32 + i * 16, sh, 0, 2);
    const int row = row0 + fr;
    if (row < p.rows) st16(pr, ((long)j * p.PS + (long)row * D + wave * 32 + i * 16 + 4 * fq) * 4, o);
  }
}

// One task (inlined into the task loop; tid() keeps its address arithmetic inside the task).
__device__ __forceinline__ void run_task(const DecStepArgs& p, int task, char* smem) {
  const int NT = (p.rows + RT - 1) / RT, per_layer = TASKS_PER_TILE * NT;
  const int l = task / per_layer, rr = task - l * per_layer;
  int ph = 0;
  while (rr >= ph_off(ph + 1) * NT) ++ph;
  const int k = rr - ph_off(ph) * NT, n = ph_n(ph), rt = k / n, i = k - rt * n;
  const DecStepLayer& L = p.layers[l];
  auto ctr = [&](int ll, int pp) { return p.ctr + ((ll * NPH + pp) * NT + rt); };
  switch (ph) {
    case P_SA:
      task_sa(p, L, l, rt, i, smem, l ? ctr(l - 1, P_LN3) : nullptr);
      break;
    case P_LN1:
      task_ln(p, l, rt, H, L.bo, L.n1w, L.n1b, 2, ctr(l, P_SA), 8);
      break;
    case P_C1:  // q_h = a Wq_h^T + bq_h, then q~ (bf16 planes [rows][8][512]) = q_h Wk_h
      task_chain(p, rt, i, smem, p.a, D, p.aL, 0, L.Wq, L.bq, L.WkT, 64, (long)D * 64, true, p.qt, (long)H * D, p.cL,
                 D, nullptr, ctr(l, P_LN1), 1);
      break;
    case P_XA: {
      const int row = rt * RT + i;
      if (row < p.rows) task_xa(p, l, row, smem, ctr(l, P_C1), 8);
      break;
    }
    case P_C2:  // o_h = c_h Wv_h^T + bv_h (train mode: bv_h weighted by the kept mass), slab h = o_h Wco_h^T
      task_chain(p, rt, i, smem, p.c, (long)H * D, p.cL, D, L.Wv, L.bv, L.Wco, D, 64, false, nullptr, 0, 0, 0,
                 p.drop.thr ? p.gs : nullptr, ctr(l, P_XA), RT);  // every XA task publishes (rows past B too)
      break;
    case P_LN2:
      task_ln(p, l, rt, H, L.bco, L.n2w, L.n2b, 4, ctr(l, P_C2), 8);
      break;
    case P_FF:
      task_ff(p, L, l, rt, i, smem, ctr(l, P_LN2));
      break;
    default:  // P_LN3
      task_ln(p, l, rt, FF / 128, L.b2, L.n3w, L.n3b, 6, ctr(l, P_FF), 16);
      break;
  }
  stamp(p, 2);
  publish(ctr(l, ph));
}

// The arguments live in device memory (one pointer kernel argument).
__global__ __launch_bounds__(1024, 1) void dec_step_kernel(const DecStepArgs* pargs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const DecStepArgs& p = *pargs;
  const int NT = (p.rows + RT - 1) / RT;
  const int total = p.n_layers * TASKS_PER_TILE * NT - NT;  // the last layer's LN3 belongs to the head kernel
  int* slot = (int*)smem;
  for (;;) {
    if (tid() == 0) slot[0] = __hip_atomic_fetch_add(p.qhead, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int task = __builtin_amdgcn_readfirstlane(slot[0]);  // uniform: the dispatch is a scalar branch
    __syncthreads();  // slot[0] is read by every wave before any DMA may overwrite it
    if (task >= total) break;
#ifdef ICAP_TOOLS
    if (p.trace && tid() == 0) {  // the task index for stamp(); slot 3: the workgroup
      p.trace_cur[blockIdx.x] = task;
      p.trace[(long)task * 4 + 3] = blockIdx.x;
    }
#endif
    stamp(p, 0);
    run_task(p, task, smem);
  }
}

}  // namespace

size_t dec_step_state_ints(int n_layers, int rows) {
  const int NT = (rows + RT - 1) / RT;
  return (((size_t)n_layers * NPH * NT + 1) + 3) / 4 * 4;  // counters, queue head; 16-B multiple
}

hipError_t launch_dec_step(const DecStepArgs& a, const DecStepArgs* dev_args, hipStream_t s) {
  if (a.rows <= 0 || a.n_layers <= 0 || a.n_layers > DEC_STEP_MAX_LAYERS || a.t0 < 0 || a.t0 >= a.Lmax ||
      a.t0 >= 64 || a.S <= 0 || !a.ctr || !a.qhead || !a.err || !a.layers || !dev_args)
    return hipErrorInvalidValue;
  static int cus = 0;
  if (!cus) {
    const hipError_t e = hipFuncSetAttribute((const void*)dec_step_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             STEP_LDS);
    if (e != hipSuccess) return e;
    int dev = 0;
    hipError_t r = hipGetDevice(&dev);
    if (r == hipSuccess) r = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (r != hipSuccess) return r;
  }
  const int NT = (a.rows + RT - 1) / RT;
  const int tasks = a.n_layers * TASKS_PER_TILE * NT - NT;
  hipLaunchKernelGGL(dec_step_kernel, dim3(std::min(cus, tasks)), dim3(1024), STEP_LDS, s, dev_args);
  return hipGetLastError();
}
