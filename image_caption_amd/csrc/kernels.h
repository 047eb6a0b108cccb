// Host-side launch wrappers for the captioning kernels (all asynchronous on `stream`).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;

// Measurement knobs (ICAP_* environment variables that select measured-and-rejected variants, tile
// classes, rasters, ...).  Only a tools build (-DICAP_TOOLS, `python -m image_caption_amd.build --tools`)
// reads them; the product build compiles every knob to its default and icap_create refuses to run
// while one is set (icap_knobs_set), so no environment can change what the library computes.
#ifdef ICAP_TOOLS
#include <stdlib.h>

inline int icap_knob(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}
#else
inline int icap_knob(const char*, int dflt) { return dflt; }
#endif
// Name of the first knob set in the environment ("" when none); checked by icap_create in a product build.
extern "C" const char* icap_knobs_set();

#include "common.h"

// Dropout of the train-mode decoder (common.h icap_drop_hash): thr = round(p 2^32) (0: off), scale = 1/(1-p),
// the seed read from device memory (so a captured decode graph replays with each call's seed); row_base
// is added to a kernel's local row index (the chains of a batch), site / layer name the mask.
struct DropCfg {
  const uint32_t* seed; uint32_t thr; float scale; int row_base; int layer; int pos;
};
__device__ __forceinline__ float drop_mul(const DropCfg& d, int site, int row, int pos, int idx) {
  return icap_drop_hash(*d.seed, site, d.layer, d.row_base + row, pos, idx) >= d.thr ? d.scale : 0.f;
}

// Plane format argument of the row kernels (layernorm, im2col, split): 1 = one bf16 plane, 2 = bf16 hi/lo
// planes, NS_F16 = one fp16 plane (ICAP_PREC_F16 encoder).
constexpr int NS_F16 = -1;

// Epilogue / output selectors shared by kernels and the host dispatcher.
enum { EPI_NONE = 0, EPI_GELU = 1, EPI_RELU = 2 };
// OUT_I8K (launch_gemm_i8, 128 x 128 tiles only): C as int8 two-slice row images [M][N/64][2][64] with one
// scale per (row, 128-column block) in c_kscale[M][N/128] - the operand form of a following gemm_i8 with
// a_kscale (the GELU output of the ViT MLP feeding MLP-2)
enum { OUT_F32 = 0, OUT_BF16 = 1, OUT_SPLIT = 2, OUT_F32_RESID = 3, OUT_PARTIAL = 4, OUT_I8K = 5 };

// C[b] (+)= epi(A[b] · W[b]^T + bias[b] + addend) with A given as `nsplit` bf16 planes
// (plane p of row r at A + p*a_lo + r*lda); W is [N][K] bf16 (nn.Linear layout).
struct GemmArgs {
  const bf16_t* A; long lda; long a_batch; long a_lo;
  const bf16_t* W; long ldw; long w_batch;
  const float* bias; long bias_batch;
  void* C; long ldc; long c_batch; long c_lo; int c_planes;  // OUT_SPLIT: 1 = hi only, 2 = hi + lo
  int M, N, K, nsplit, batch;
  int epi, out;
  int rm_group; long rm_stride; long rm_off;          // output row remap (0 = identity)
  const float* addend; long add_ld; int add_group; int add_off;
  // convolution epilogue (ResNet trunk): v = acc * scale[n] + bias[n] (+ res planes) before the
  // activation; res = bf16 hi plane at res[row * res_ld + n], lo plane at + res_lo
  const float* scale; const bf16_t* res; long res_ld; long res_lo;
  int res_planes;  // 2 (default): hi + lo; 1: the hi plane only (the fp16 trunk's one-plane residual stream)
  // implicit-GEMM convolution (A is not materialised; rows = output pixels (b, oh, ow)):
  //   cv = 1: 3x3 / pad 1 / stride cv_stride over NHWC planes A [B][cv_H][cv_W][C], C = 1 << cv_cshift
  //           (>= 64), k = (kh*3 + kw)*C + c; taps outside the image read cv_zero (>= 16 zero bytes)
  //   cv = 2: 7x7 / stride 2 stem over a zero-bordered NHWC4 image A [B][cv_H][cv_W][4] (border 3),
  //           k = (kh*8 + kw)*4 + c, i.e. one 32-deep k-step = one kernel row = 64 contiguous bytes
  int cv, cv_H, cv_W, cv_cshift, cv_OW, cv_OHW, cv_stride; const bf16_t* cv_zero;
  // head-major split output (hm_n = tokens per image, 0 = off): element (row, col) of the bf16 planes
  // goes to ((row / hm_n * (N / 64) + col / 64) * hm_n + row % hm_n) * 64 + col % 64, i.e. the QKV
  // projection as [image][q|k|v x head][token][64] - one head's rows contiguous for the attention
  int hm_n;
  int nt_store;      // split-plane outputs with nontemporal stores (gemm_i8 LDS epilogue)
  int raster_group;  // tile raster inside an XCD: groups of raster_group row bands, column tiles outer (0: row-band major)
  // int8 two-slice operands (launch_gemm_i8 only): A and W are int8 row images [rows][K/64][2][64]
  // (row stride 2K bytes; lda / ldw / a_lo unused), v = s (256 x1 + x2) with a per-row scale:
  // a_scale[M] for A, w_scale[N] for W
  const float* a_scale; const float* w_scale;
  // block-scaled A (launch_gemm_i8, 128 x 128 tiles only): one scale per (row, 128-deep k block),
  // a_kscale[M][K/128] instead of a_scale; c_kscale: the block scales written by out = OUT_I8K
  const float* a_kscale; float* c_kscale;
  // tail split (launch_gemm_256, 128 x 256 tiles, no convolution): per XCD, the tiles of the last partial
  // round of split_slots block slots run as two K halves merged by the second finisher; split_ws holds
  // 2 x 128 x 256 fp32 partials per split tile (8 x split_slots tiles), split_cnt its tickets (zero at rest)
  float* split_ws; int* split_cnt; int split_slots;
  // f16 = 1: A and W are single fp16 planes (nsplit 1), fp16 MFMA; OUT_SPLIT writes one fp16 plane
  // (launch_gemm_256 128 x 256 path only: the ICAP_PREC_F16 encoder GEMMs)
  int f16;
  // fp16 range guard (gemm_f16p_kernel store-only fp16 outputs): set to 1 when a stored value is not finite in
  // fp16 (|v| >= 65520 before rounding, or NaN); nullptr = unchecked
  unsigned* range_flag;
  // persistent GEMMs: at most this many workgroups (0 = one per CU of the device) - the CUs a CU-masked encoder
  // stream owns (batch pipelining, icap_set_encoder_cus)
  int max_grid;
  int no_pre;     // tools (ICAP_CONV_PRE=0): the 64-deep conv forms load the residual after the k-loop
};
// bytes of split_ws for split_slots block slots per XCD
inline size_t gemm_split_ws_bytes(int split_slots) { return (size_t)8 * split_slots * 2 * 128 * 256 * 4; }
inline GemmArgs gemm_args() { GemmArgs g{}; g.batch = 1; g.nsplit = 1; g.c_planes = 2; g.res_planes = 2; return g; }
hipError_t launch_gemm(const GemmArgs& g, hipStream_t s);
// Which kernel launch_gemm picks (PROF_GEMM_256 / PROF_GEMM_128 / PROF_GEMM_64).
int gemm_tile_class(const GemmArgs& g);
// The profile class icap_profile_* records a GEMM launch under (the kernel family that runs it).
int gemm_prof_class(const GemmArgs& g);
// 256 x 256-tile, 8-wave encoder GEMM (batch 1, N % 256 == 0).
hipError_t launch_gemm_256(const GemmArgs& g, hipStream_t s);
// conv_rmw.hip: W-stationary persistent form of the fp16 trunk's residual 1x1 convolutions (K 64 / 128 / 256)
bool conv_rmw_ok(const GemmArgs& g);
hipError_t launch_conv_rmw(const GemmArgs& g, hipStream_t s, int cus);
#ifdef ICAP_TOOLS
// gemm_tools.hip (tools build only): takes the launch when a measurement knob selects a rejected form
bool launch_gemm_256_tools(const GemmArgs& g, hipStream_t s, int cus, hipError_t* err);
#endif
// int8 two-slice GEMM (batch 1, N % 256 == 0, K % 64 == 0): acc = 65536 A1.W1 + 256 (A1.W2 + A2.W1)
// in int32, then * a_scale[m] * w_scale[n] and the gemm_256 epilogue (bias, GELU, head-major, ...)
hipError_t launch_gemm_i8(const GemmArgs& g, hipStream_t s);
// LayerNorm rows -> int8 two-slice row images: y = LN(x); s = max|y| / 32639; q = rint(y / s);
// x1 = (q + 128) >> 8, x2 = q - 256 x1, element k of row r at out[r*2D + (k/64)*128 + slice*64 + k%64];
// scale[row] = s
hipError_t launch_layernorm_i8(const float* x, long ldx, int rows, int D, int in_group, long in_stride, long in_off,
                               const float* w, const float* b, float eps, int8_t* out, float* scale, hipStream_t s);
// fp32 [N][K] rows -> int8 two-slice row images (same layout, K % 64 == 0) + per-row scale
hipError_t launch_pack_i8_rows(const float* w, int N, int K, int8_t* out, float* scale, hipStream_t s);
enum { PROF_GEMM_128 = 0, PROF_GEMM_64 = 1, PROF_ENC_ATTN = 2, PROF_CROSS_ATTN = 3, PROF_GEMM_WAVE = 4, PROF_GEMM_256 = 5,
       PROF_GEMM_I8 = 6, PROF_DEC_FUSED = 7, PROF_GEMM_F16P = 8 };
// launch_gemm_256 runs g as the persistent fp16 kernel (gemm_f16p_kernel, store-only epilogue, whole row bands)
bool gemm_f16_persistent(const GemmArgs& g);

// Decode-step GEMM: each wave streams a (16 TM) x (16 TN) tile's operands into registers (no LDS);
// block = 4 waves along N.  ksplit > 1 with out = OUT_PARTIAL writes fp32 partial slabs
// C[split * part_stride + row * ldc + col] (bias is then the consumer's job).
enum { WAVE_2x2 = 0, WAVE_1x2 = 1, WAVE_1x1 = 2, WAVE_2x1 = 3 };
struct WaveGemmArgs {
  const bf16_t* A; long lda; long a_batch; long a_lo;
  const bf16_t* W; long ldw; long w_batch;
  const float* bias; long bias_batch;
  void* C; long ldc; long c_batch; long c_lo; int c_planes;
  int M, N, K, nsplit, batch, ksplit;
  long part_stride;
  int epi, out, tile;
  // hi/lo weights (launch_gemm_dec only): W_lo = bf16(W - W_hi), same layout and batch stride as W; the
  // product then adds W_lo . X_hi, so the weight enters with 16 significand bits (fp32 checkpoints)
  const bf16_t* W_lo;
};
inline WaveGemmArgs wave_args() {
  WaveGemmArgs g{};
  g.batch = 1; g.nsplit = 1; g.c_planes = 2; g.ksplit = 1; g.tile = WAVE_2x2;
  return g;
}
hipError_t launch_gemm_wave(const WaveGemmArgs& g, hipStream_t s);
// Same contract, 32 x 32 block tiles with the whole K' range (<= 1024 per split) DMA'd to LDS first.
hipError_t launch_gemm_dec(const WaveGemmArgs& g, hipStream_t s);

// A residual LayerNorm folded into the kernel that consumes it: y = LN(x + sum_{s<nparts} parts[s] + bias)
// (dropout `site` on the sublayer output, as launch_residual_layernorm), computed by the consumer for its own
// rows.  Used by the decode head for the last layer's LN3 (x_out unused) and, round 5, by the register-fragment
// decode blocks (DecSaArgs / ChainArgs / DecFfnArgs::fold, decode.hip): the block builds its X image from the fold
// instead of the DMA of the a planes, and the tile's writer block stores the normalised rows to x_out (!= x: the
// tile's other blocks still read x).  parts == nullptr: off.
struct RlnArgs {
  const float* x; float* x_out; const float* parts; int nparts; long part_stride;
  const float* bias; const float* w; const float* b; float eps;
  DropCfg drop; int site;
};

// Residual-LayerNorm merge in the producing decode block (round 4): the slabs go out as agent-scope (write-through)
// stores, and the LAST of the tile's nparts blocks to take the 16-row tile's ticket tick[row0 / 16] computes
// x = LN(x + bias + sum_p slab_p) for those rows (residual_layernorm_kernel's arithmetic, the dropout site `site`
// of `drop`) and writes x and the activation planes a (ns planes, plane stride aL), then resets the
// ticket.  tick == nullptr: no merge (the caller launches residual_layernorm_kernel).
struct SlabMerge {
  int* tick; float* x; const float* bias; const float* w; const float* b; float eps; bf16_t* a; long aL; int site;
  DropCfg drop;
};

// Two chained per-head GEMMs in one launch (decoder cross-attention block), for each head h:
//   Y_h = X_h W1_h^T + b1_h      X_h: rows x 512 (bf16 planes), W1_h: rows [64h, 64h + 64) of W1 [.][512]
//   O_h = Y_h W2_h^T             W2_h: N2 x 64 at W2 + h * w2_hstride, row stride ldw2
// out = OUT_SPLIT: planes of O_h at C + row * ldc + h * c_hstride (+ c_lo for the lo plane);
// out = OUT_PARTIAL: fp32 O_h into slab h at C + h * part_stride + row * ldc.
struct ChainArgs {
  const bf16_t* X; long ldx; long x_lo; long x_hstride;
  const bf16_t* W1; const float* b1;
  const bf16_t* W2; long ldw2; long w2_hstride;
  void* C; long ldc; long c_lo; long c_hstride; long part_stride;
  int M, N2, H, nsplit, out;
  // dec_chain only: b1 scaled per (row, head) by b1_scale[row * H + h] - the value projection of the
  // key-absorbed cross-attention under probability dropout, whose bias enters as sum_s P_s m_s (not 1)
  const float* b1_scale;
  // dec_chain only (frag_pack images, both or neither): W1 of head h as tiles h * 4 + t x 16 k32-steps, W2 as tiles
  // h * 32 + n x 2 k32-steps - each wave loads its own fragments straight into registers (no LDS weight staging)
  const bf16_t* W1f; const bf16_t* W2f;
  // dec_chain, hi/lo decoder weights (round 5): the lo planes' fragment images (both or neither; FR, two planes)
  const bf16_t* W1fl; const bf16_t* W2fl;
  SlabMerge mg;  // dec_chain, OUT_PARTIAL only
  RlnArgs fold;  // dec_chain FR with two planes, x_hstride 0: X = the residual LN of the producer's slabs (nparts 8)
  int xcd_tiles;  // dec_chain: the 8 head blocks of a row tile on one XCD (when the tile count is a multiple of 8)
};
hipError_t launch_chain_dec(const ChainArgs& a, hipStream_t s);

// Fused decode-step blocks (decode.hip), d_model 512, 8 heads of 64, dim_ff 2048, one new token per row.
// dec_sa: q|k|v of head h for 16 rows (Wqkv [1536][512] bf16, bqkv fp32), the new key/value appended to
// the fp32 cache kc/vc [rows][8][Lmax][64] at t0 (anc: beam ancestry as dec_self_attn), causal attention
// over positions 0..t0 (t0 < 64), and slab h of the out-projection part[h][rows][512] (Wo [512][512]).
struct DecSaArgs {
  const bf16_t* A; long aL; int nsplit, rows;
  const bf16_t* Wqkv; const float* bqkv; const bf16_t* Wo;
  float *kc, *vc; int Lmax, t0; float scale; const int32_t* anc;
  float* part; long part_stride;
  DropCfg drop;  // thr 0: no dropout (site 1: the attention probabilities)
  // frag_pack images (both or neither): Wqkv as tiles h * 12 + i (q 0-3, k 4-7, v 8-11) x 16 k32-steps (mode 1), Wo
  // as tiles h * 32 + n x 2 k32-steps (mode 2, ksl 64)
  const bf16_t* Wqkv_f; const bf16_t* Wo_f;
  const bf16_t* Wqkv_fl; const bf16_t* Wo_fl;  // hi/lo decoder weights: the lo planes' images (FR, two planes)
  SlabMerge mg;
  RlnArgs fold;  // FR with two planes: A = the residual LN of the producer's slabs (nparts 16)
  int xcd_tiles;  // the 8 head blocks of a row tile on one XCD (when the tile count is a multiple of 8)
};
hipError_t launch_dec_sa(const DecSaArgs& a, hipStream_t s);
// dec_ffn: slab j of 16 = relu(a W1[128j:128j+128]^T + b1) W2[:, 128j:128j+128]^T -> part[j][rows][512]
struct DecFfnArgs {
  const bf16_t* A; long aL; int nsplit, rows;
  const bf16_t* W1; const float* b1; const bf16_t* W2;
  float* part; long part_stride;
  DropCfg drop;  // site 5: the hidden activations (pos = the decode position)
  // frag_pack images (both or neither): W1 as tiles 0..127 x 16 k32-steps, W2 as tiles j * 32 + n x 4 k32-steps
  const bf16_t* W1f; const bf16_t* W2f;
  const bf16_t* W1fl; const bf16_t* W2fl;  // hi/lo decoder weights: the lo planes' images (FR, two planes)
  SlabMerge mg;
  RlnArgs fold;  // FR with two planes: A = the residual LN of the producer's slabs (nparts 8)
  int xcd_tiles;  // with fold: the 16 slice blocks of a row tile on one XCD (when the tile count is a multiple of 8)
};
hipError_t launch_dec_ffn(const DecFfnArgs& a, hipStream_t s);
// The chained per-head cross-attention products (ChainArgs as launch_chain_dec, N2 = 512) with 16-row
// blocks and one full-line DMA round (decode.hip); used by the decode loops.
hipError_t launch_dec_chain(const ChainArgs& a, hipStream_t s);
// MFMA fragment image of a bf16 matrix W [rows][ldw] for the decode blocks' register-direct weight loads: tile t,
// 32-deep k-step s -> 64 lanes x 16 B at out + (t * nk + s) * 512 elements, lane l = W[row0(t) + (l & 15)][k0(t) + 32 s
// + 8 (l >> 4) ..+7] (the A-operand fragment of v_mfma_f32_16x16x32 as frag() reads it from an LDS row image).
// mode 0: row0 = 16 t, k0 = 0; mode 1 (self-attention in_proj, d 512, 8 heads): t = 12 h + i, row0 = 512 (i >> 2) +
// 64 h + 16 (i & 3); mode 2 (column slices): t = tps j + n, row0 = 16 n, k0 = ksl j.
hipError_t launch_frag_pack(const bf16_t* W, long ldw, int ntiles, int nk, int mode, int tps, int ksl, bf16_t* out,
                            hipStream_t s);

// Persistent decode step (decstep.hip): all decoder layers of one decode step (one new token per row) in ONE
// launch of one 1024-thread workgroup per CU.  Work items are tasks of 16-row tiles - self-attention per head,
// residual LayerNorm, the two chained cross-attention products per head, cross-attention per row, feed-forward
// per hidden slice - pulled from a device queue in a dependency-respecting order; a task issues its weight DMA,
// then waits for the per-(layer, phase, tile) counter of its inputs, then loads them.  Handed-off outputs are
// write-through (sc1) stores published by a counter add; consumers acquire once per task.  The last layer's
// LN3 is left to the head kernel (HeadArgs::ln), as in the launch-per-kernel loop.
struct DecStepLayer {
  const bf16_t* Wqkv; const float* bqkv; const bf16_t* Wo; const float* bo;   // self-attention
  const float *n1w, *n1b;
  const bf16_t* Wq; const float* bq; const bf16_t* WkT;                       // q, then q~ = q Wk (per head)
  const bf16_t* Wv; const float* bv; const bf16_t* Wco; const float* bco;     // value, cross out-projection
  const float *n2w, *n2b;
  const bf16_t* W1; const float* b1; const bf16_t* W2; const float* b2;       // feed-forward
  const float *n3w, *n3b;
};
constexpr int DEC_STEP_MAX_LAYERS = 8;
struct DecStepArgs {
  const DecStepLayer* layers;             // device array [n_layers]
  int n_layers, rows, t0, Lmax, S;
  float* x; bf16_t* a; long aL;           // residual stream [rows][512] fp32 and its bf16 hi/lo planes
  float* kc; float* vc; long kvl;         // KV cache [layer][rows][8][Lmax][64] fp32 (kvl = layer stride)
  float* part; long PS;                   // split-K slabs [16][rows][512]
  bf16_t* qt; long cL;                    // q~ planes [rows][8][512]
  bf16_t* c;                              // cross-attention context planes [rows][8][512] (lo at + cL)
  const bf16_t* mem16;                    // the memory as one fp16 plane [rows][S][512]
  float* gs;                              // train mode: value-bias weights [rows][8]
  DropCfg drop;                           // thr 0: no dropout (layer / pos set per task)
  int* ctr;                               // [n_layers][8 phases][tiles] completion counters, zeroed per launch
  int* qhead;                             // task queue head, zeroed per launch
  unsigned* err;                          // the handle's sticky status word: DEC_STEP_GAVE_UP set on a give-up
  // tools build: per-task stamps [task][4] (dequeued, inputs ready, body done: s_memrealtime; workgroup) or null
  unsigned long long* trace; int* trace_cur;
};
constexpr unsigned DEC_STEP_GAVE_UP = 2;  // (bit 0 of the same word: the f16 encoder's range guard)
// a: the host copy (validated here); dev_args: the same struct in device memory (what the kernel reads)
hipError_t launch_dec_step(const DecStepArgs& a, const DecStepArgs* dev_args, hipStream_t s);
// ints of the per-launch state block (counters + queue head), zeroed before every launch
size_t dec_step_state_ints(int n_layers, int rows);

// Group-persistent decode step (xdec.hip): every decoder layer of one decode step in one launch of 8 row groups x 32
// workgroups (one per CU); products split over a group's workgroups by output columns, row-local work one row per
// workgroup, group barriers on write-through hand-offs.  rows <= 256, d 512 / 8 heads / dim_ff 2048, bf16 weights,
// two activation planes, eval mode (no dropout), one row per memory image.
struct XdecArgs {
  const DecStepLayer* layers;             // device array [n_layers]
  int n_layers, rows, t0, Lmax, S;
  float* x; bf16_t* a; long aL;           // residual stream [rows][512] fp32 and its bf16 hi/lo planes
  float* kc; float* vc; long kvl;         // KV cache [layer][rows][8][Lmax][64] fp32
  float* qv;                              // [rows][1536] fp32: this step's q | k | v
  bf16_t* ctx; long ctxL;                 // [rows][512] planes: self-attention context, then the value projection
  float* y;                               // [rows][512] fp32: the sums a LayerNorm normalises
  bf16_t* q2; long q2L;                   // [rows][512] planes: the cross-attention query
  bf16_t* qt; long cL;                    // [rows][8][512] planes: q~
  bf16_t* c;                              // [rows][8][512] planes (lo at + cL): cross-attention context
  float* slab;                            // [32][rows][512] fp32: feed-forward partials, one per hidden slice
  const bf16_t* mem16;                    // the memory as one fp16 plane [rows][S][512]
  int* ctr;                               // 8 group counters, 16 ints apart, zeroed before the launch
  unsigned* err;                          // the handle's status word (DEC_STEP_GAVE_UP on a give-up)
  // tools build: per-workgroup stamps [256][XDEC_TRACE_BARRIERS][2] (s_memrealtime at each arrival, and when the
  // barrier released the workgroup), or null
  unsigned long long* trace;
};
constexpr int XDEC_TRACE_BARRIERS = 12 * DEC_STEP_MAX_LAYERS;
size_t xdec_state_ints();
int xdec_supported();  // the device has the 256 CUs the launch needs
hipError_t launch_xdec(const XdecArgs& a, hipStream_t s);

// LayerNorm over rows of D fp32 values; optional fp32 output (may alias input) and
// bf16 hi(/lo) planes.  Input row r is read from (r / in_group) * in_stride + in_off + r % in_group.
hipError_t launch_layernorm(const float* x, long ldx, int rows, int D, int in_group, long in_stride,
                            long in_off, const float* w, const float* b, float eps, float* out_f32,
                            long ld_f32, bf16_t* out_bf, long ld_bf, long bf_lo, int nsplit,
                            hipStream_t s, unsigned* range_flag = nullptr);

// x = LN(x + sum_{s<nparts} parts[s*part_stride + row*D + col] + bias) in place (fp32), plus planes.
hipError_t launch_residual_layernorm(float* x, int rows, int D, const float* parts, int nparts, long part_stride,
                                    const float* bias, const float* w, const float* b, float eps, bf16_t* out_bf,
                                    long bf_lo, int nsplit, hipStream_t s, DropCfg drop = DropCfg{}, int site = 0,
                                    const float* x_in = nullptr);  // x_in: the residual input (default x, in place)
hipError_t launch_im2col_patches(const float* img, int B, int C, int HW, int P, bf16_t* out, long lo,
                                 int nsplit, hipStream_t s);
hipError_t launch_cls_rows(const float* cls, const float* pos, float* x, int B, int tokens, int D,
                           hipStream_t s);
hipError_t launch_nchw_to_rows(const float* feats, int B, int C, int S, bf16_t* out, long lo, int nsplit,
                               hipStream_t s);
// x[r] = emb[tok] * scale + pe[t0 + r % T], tok = tok_ptr[(r / T) * tok_ld + r % T] (or fixed_tok if null)
// ResNet trunk (trunk.hip): gathers into GEMM A operands (NHWC bf16 planes), max-pool, packing
hipError_t launch_subsample2(const bf16_t* x, long xlo, int B, int H, int W, int C, bf16_t* out, long lo, int nsplit,
                             hipStream_t s);
// (f16: fp16 planes, the ICAP_PREC_F16 trunk; subsample2 copies bits and serves both)
hipError_t launch_maxpool3s2(const bf16_t* x, long xlo, int B, int H, int W, int C, int OH, int OW, bf16_t* out,
                             long lo, int nsplit, hipStream_t s, bool f16 = false);
// [Cout][Kp] bf16 with k = (kh*kwp + kw)*cp + c (cp >= cin, kwp >= k; padding taps/channels are 0)
// CIDEr-D on token-id rows (cider.hip): hypothesis k belongs to image k % B; image i's references
// are rows ref_off[i] .. ref_off[i+1]; rows are raw ids (<start>/<pad> dropped, cut at <end>)
constexpr int CIDER_MAX_TOKENS = 192;
size_t cider_workspace_bytes(long ref_rows, int Lr);
hipError_t launch_cider(const int32_t* hyp, int n_hyp, int Lh, int B, const int32_t* refs, int n_ref, int Lr,
                        const int32_t* ref_off, int start, int end, int pad, double* scores, void* ws,
                        size_t ws_bytes, int* overflow, hipStream_t s);
// On-GPU eval preprocessing (preprocess.hip): uint8 RGB images -> normalised (B,3,S,S) fp32
hipError_t launch_preprocess(const uint8_t* px, const int64_t* offs, const int32_t* geom, int B, int S, int max_rows,
                             uint8_t* tmp, float* out, hipStream_t s);
hipError_t launch_pack_conv(const float* w, int cout, int cin, int k, int cp, int kwp, int Kp, bf16_t* out,
                            hipStream_t s, bool f16 = false);
// (B,3,HW,HW) fp32 -> zero-bordered NHWC4 planes [B][HW+2*border][HW+2*border][4] (channel 3 = 0)
hipError_t launch_image_nhwc4(const float* img, int B, int IH, int IW, int border, bf16_t* out, long lo, int nsplit,
                              hipStream_t s, bool f16 = false);
// Train-mode BatchNorm over the raw convolution output planes y [M][C] (in place): batch statistics
// (double sums over all M rows, deterministic), running statistics updated with momentum (unbiased variance),
// then y = relu?(y * scale + shift (+ res planes)).  part: bn_part_bytes(); scale / shift: C floats each.
inline size_t bn_part_bytes() { return (size_t)1024 * 64 * 2 * sizeof(double); }
hipError_t launch_bn_train(bf16_t* y, long lo, long M, int C, const float* gamma, const float* beta, float* run_mean,
                           float* run_var, float momentum, float eps, const bf16_t* res, long res_lo, int relu,
                           double* part, float* scale, float* shift, hipStream_t s);
hipError_t launch_bn_fold(const float* g, const float* b, const float* mean, const float* var, int C, float eps,
                          float* scale, float* shift, hipStream_t s);
hipError_t launch_embed(const int32_t* tok, long tok_ld, int fixed_tok, int rows, int T, int t0, const float* emb,
                        const float* pe, int D, float scale, float* x, bf16_t* a, long lo, int nsplit, hipStream_t s,
                        DropCfg drop = DropCfg{});
// byte fill as a kernel (captured into decode graphs: a captured small hipMemsetAsync was not
// re-applied on the second replay of the sampled-decode graph, ROCm 7.2)
hipError_t launch_fill_u8(uint8_t* p, long n, uint8_t value, hipStream_t s);
hipError_t launch_fill_col(int32_t* ids, int B, long ld, int col, int value, hipStream_t s);
// stop-aware decode (round 6): flag (host-mapped) = 1 when a column in [col0, col1) is all end (greedy) or every fin row
// is set (fin != nullptr); the tail fill of a stopped decode (ids columns > t0 = end, logp steps >= t0 = 0)
hipError_t launch_stop_scan(const int32_t* ids, int B, long ld, int col0, int col1, int end, const uint8_t* fin,
                            int* flag, hipStream_t s);
hipError_t launch_stop_tail(int32_t* ids, int B, int L, int t0, int end, float* logp, hipStream_t s);
hipError_t launch_split_f32(const float* src, long n, bf16_t* dst, long lo, int nsplit, hipStream_t s);
// bf16 planes -> fp32 (hi + lo)
hipError_t launch_planes_to_f32(const bf16_t* src, long lo, long n, int nsplit, float* dst, hipStream_t s);
// fp16 hi/lo planes -> bf16 hi/lo planes of the same values (+ their fp32 sum when f32 != nullptr); n % 4 == 0
hipError_t launch_f16planes_to_bf16(const bf16_t* src, long slo, long n, bf16_t* dst, long dlo, float* f32,
                                   hipStream_t s);
hipError_t launch_f32_to_bf16(const float* src, bf16_t* dst, long n, hipStream_t s);
hipError_t launch_f32_to_f16(const float* src, bf16_t* dst, long n, hipStream_t s);
hipError_t launch_transpose_heads_bf16(const float* wk, int H, int hd, int D, bf16_t* dst, hipStream_t s,
                                       int lo_plane = 0);

// Encoder self-attention (non-causal) over N tokens, heads of 64, MFMA bf16 (nsplit 1 or 2).
// head_major: qkv written with GemmArgs::hm_n = N (N in (64, 256])
hipError_t launch_enc_attention(const bf16_t* qkv, long ld, long lo, int B, int N, int H, float scale,
                                bf16_t* out, long out_ld, long out_lo, int nsplit, hipStream_t s, int head_major = 0,
                                int max_grid = 0);  // max_grid: the encoder CU budget of the persistent form (0 = all)
// Decoder self-attention with fp32 KV cache; n_new query rows per image starting at t0.
hipError_t launch_dec_self_attn(const float* qkv, int B, int n_new, int t0, int H, float* kc, float* vc,
                                int Lmax, int causal, float scale, bf16_t* out, long lo, int nsplit,
                                hipStream_t s, const int32_t* anc = nullptr, const int32_t* klen = nullptr);
// Cross-attention in the key-absorbed form on MFMA: rows hold q~_h = q_h·Wk_h (8 heads x 512) as bf16
// planes (plane stride qt_lo); memory (images, S, 512) as bf16 planes (mem_lo); context planes out.
// With xpart (cross_attn_part_floats(rows) floats) and xcnt (rows ints, zero at rest) the keys of
// a row pair split over cross_attn_splits(S) blocks (opt-in: ICAP_XATTN_KS=2).
hipError_t launch_cross_attn_mfma(const bf16_t* qt, long qt_lo, const bf16_t* mem, long mem_lo, int rows,
                                  int rows_per_image, int S, float scale, bf16_t* out, long out_lo, int nsplit,
                                  hipStream_t s, float* xpart = nullptr, int* xcnt = nullptr);
// The same over a single fp16 memory plane mem16 [B][S][512] (q~ bf16 hi/lo planes in, context bf16 hi/lo
// planes out): the decoder's cross-attention in the parity precisions (attention.hip).
// drop (train mode): gsum [rows][8] receives sum_s P_s m_s / sum_s P_s per (row, head) (the value bias's weight)
hipError_t launch_cross_attn_f16(const bf16_t* qt, long qt_lo, const bf16_t* mem16, int rows, int rows_per_image,
                                 int S, float scale, bf16_t* out, long out_lo, hipStream_t s,
                                 DropCfg drop = DropCfg{}, float* gsum = nullptr, float* xpart = nullptr,
                                 int* xcnt = nullptr);
int cross_attn_splits(int S);
// blocks per row pair of launch_cross_attn_f16 (2: key split, needs xpart / xcnt as launch_cross_attn_mfma)
int cross_attn_f16_splits();
// the key-split single-burst fp16 cross-attention (cross_attn_f16s_kernel: one row per image, no dropout, S <= 256;
// needs xpart / xcnt) is on
bool cross_attn_f16s_on();
size_t cross_attn_part_floats(int rows);
// Batched beam search (beam.hip): state init, per-step selection, final pick.
hipError_t launch_beam_init(int B, int K, int start, int Lmax, int32_t* seq_a, int32_t* seq_b, int32_t* anc_a,
                            int32_t* anc_b, float* scores, int* kcur, int* done, int* ncomp, float* best_score,
                            int* best_len, hipStream_t s);
hipError_t launch_beam_select(const float* logits, int V, int B, int K, int t, int Lmax, int grid_variant, int end_tok,
                              const int32_t* seq_c, int32_t* seq_n, const int32_t* anc_c, int32_t* anc_n,
                              const float* sc_c, float* sc_n, int* kcur, int* done, int* ncomp, float* best_score,
                              int32_t* best_seq, int* best_len, hipStream_t s);
hipError_t launch_beam_finalize(int B, int K, int Lmax, const int32_t* seq, const float* scores, const int* kcur,
                                const int* ncomp, const int32_t* best_seq, const int* best_len, int32_t* ids,
                                int32_t* lens, hipStream_t s);
// fc_out + argmax (greedy) or inverse-CDF sample; writes ids[r*ld_ids + col], optional logits, and
// (if emb != null) the next step's embedded token into x/a.
struct HeadArgs {
  const float* x; int rows; int Dm; const float* W; const float* bias; int V;
  float* logits; long ld_logits;
  int32_t* ids; long ld_ids; int id_col;
  const float* uniforms;  // null => argmax
  float* logp; long ld_logp; uint8_t* finished; int end_token;
  const float* emb; const float* pe; int pe_pos; float emb_scale; float* x_next; bf16_t* a_next; long lo; int nsplit;
  DropCfg drop;  // site 0 on the next step's embedding (positional-encoding dropout)
  RlnArgs ln;    // the last decoder layer's residual LN3 on x first (nparts <= 16; x_out unused), or off
  const float* W4 = nullptr;  // optional fc_out image [Dm / 4][V][4] (launch_head_w4) for V <= 128
};
hipError_t launch_head_w4(const float* w, int V, int Dm, float* w4, hipStream_t s);
constexpr int HEAD_MAX_VOCAB = 32768;  // logits of one row in LDS (128 KiB) for the sampler's prefix sum
hipError_t launch_head(const HeadArgs& h, hipStream_t s);

// ---- decoder training pass (train.hip): fp32-accurate strided GEMM and the row kernels around it ----
// C[b][m][n] = alpha * sum_k A[b][m][k] B[b][n][k] (+ beta * C) (+ bias[n]) (relu), element strides
// (sam, sak) / (sbn, sbk) / (scm, scn); batch index z in [0, nbatch): b1 = z / nb2, b2 = z % nb2 with
// strides sab1 / sab2 etc.  fp32 operands and products (v_mfma_f32_16x16x4_f32).
struct TGemmArgs {
  const float* A; long sam, sak, sab1, sab2;
  const float* B; long sbn, sbk, sbb1, sbb2;
  float* C; long scm, scn, scb1, scb2;
  const float* bias;
  int M, N, K, nb2;
  float alpha, beta;
  int relu;
  int ksplit; float* part;  // ksplit > 1 (unbatched only): K split over blocks, raw sums in part [ksplit][M][N]
};
hipError_t launch_tgemm(const TGemmArgs& a, int nbatch, hipStream_t s);
hipError_t launch_softmax_rows(float* x, long rows, int n, int T, int causal, hipStream_t s);
hipError_t launch_softmax_bwd(const float* P, float* dP, long rows, int n, hipStream_t s);
hipError_t launch_ln_fwd(const float* a, const float* b, const float* w, const float* bias, float eps, int rows, int D,
                         float* y, float* xhat, float* rstd, hipStream_t s);
hipError_t launch_ln_bwd(float* dy, const float* xhat, const float* rstd, const float* w, int rows, int D, float* prod,
                         hipStream_t s);
size_t colsum_scratch_floats(int n);
hipError_t launch_colsum(const float* src, long ld, int rows, int n, float* part, float* dst, int accumulate,
                         hipStream_t s);
hipError_t launch_relu_bwd(float* dh, const float* h, long n, hipStream_t s);
hipError_t launch_embed_fwd(const int32_t* ids, long ld, int B, int T, const float* emb, const float* pe, int D,
                            float scale, float* x, hipStream_t s);
hipError_t launch_embed_bwd(const int32_t* ids, long ld, int B, int T, const float* dx, int D, int V, float scale,
                            float* dE, hipStream_t s);
hipError_t launch_logp_fwd(const float* logits, int V, const int32_t* ids, long ld, int B, int T, int end_token,
                           float* logp, float* lse, hipStream_t s);
hipError_t launch_logp_bwd(const float* logits, const float* lse, const float* dlogp, int V, const int32_t* ids,
                           long ld, int B, int T, int end_token, float* dlogits, hipStream_t s);
hipError_t launch_drop_rows(const float* x, float* out, int B, int T, int n, DropCfg d, int site, hipStream_t s);
hipError_t launch_drop_attn(const float* x, float* out, int B, int H, int T, int Tk, int stride, DropCfg d, int site,
                            hipStream_t s);
