// libicap runtime: weight packing, workspace, and the launch schedules of the captioning hot
// path (ViT / Grid encoders, KV-cached greedy and sampled decode, full-prefix decoder forward).
// The C ABI is declared in include/icap.h; the reference functions each entry replaces are
// cited there.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>


#include "../../include/icap.h"
#include "kernels.h"

namespace {

thread_local std::string g_err;

struct Fail : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIPCHK(x)                                                                                    \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) throw Fail(std::string(#x) + ": " + hipGetErrorString(e_));                \
  } while (0)
#define REQUIRE(c, msg)                       \
  do {                                        \
    if (!(c)) throw Fail(std::string(msg)); \
  } while (0)

template <class F>
int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
  } catch (...) {
    g_err = "unknown error";
  }
  return 1;
}

int g_ws_generation = 0;  // bumped on every workspace (re)allocation: invalidates captured graphs

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  void ensure(size_t bytes) {
    if (bytes <= n) return;
    ++g_ws_generation;
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    n = 0;
    HIPCHK(hipMalloc(&p, bytes));
    n = bytes;
    static const bool poison = icap_knob("ICAP_POISON", 0) != 0;
    if (poison) HIPCHK(hipMemset(p, 0xFF, bytes));  // debug: NaN in fp32 and bf16 - exposes reads of unwritten workspace
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  template <class T>
  T* as() const { return (T*)p; }
};

struct Lin {  // packed nn.Linear: bf16 W [N][K] + fp32 bias (+ the lo plane bf16(W - W_hi) of hi/lo weights)
  bf16_t* w = nullptr;
  bf16_t* wl = nullptr;
  float* b = nullptr;
  int N = 0, K = 0;
};
struct Lin8 {  // nn.Linear as int8 two-slice row images [N][K/64][2][64] + per-row scale (ICAP_PREC_I8X2)
  int8_t* w = nullptr;
  float *sw = nullptr, *b = nullptr;
  int N = 0, K = 0;
};
struct LN {
  float *w = nullptr, *b = nullptr;
};
struct VitLayer {
  LN ln1, ln2;
  Lin qkv, out, mlp0, mlp3;
  Lin8 qkv8, mlp08, mlp38;
};
struct EncLayer {
  Lin qkv, out, lin1, lin2;
  LN n1, n2;
};
struct Conv {  // packed Conv2d + eval BatchNorm: bf16 W [cout][Kp] in (kh, kw, c) order, fp32 scale/shift
  bf16_t* w = nullptr;
  bf16_t* w16 = nullptr;  // the same in fp16 (ICAP_PREC_F16 Grid: the eval trunk on fp16 planes)
  float *scale = nullptr, *shift = nullptr;
  int cout = 0, cin = 0, k = 1, stride = 1, Kp = 0;
};
struct DecLayer {
  Lin sa_qkv, sa_out, ca_q, ca_out, lin1, lin2;
  bf16_t* ca_kT = nullptr;  // [H][d_model][64]: W_k,h^T for the key absorption
  bf16_t* ca_v = nullptr;   // [d_model][d_model] = rows [2d, 3d) of in_proj (per-head slices of 64 rows)
  float* ca_vb = nullptr;   // bias rows [2d, 3d)
  LN n1, n2, n3;
  // MFMA fragment images of the fused decode blocks' weights (launch_frag_pack; d 512 / 8 heads / dim_ff 2048 only):
  // the blocks load them straight into registers instead of staging weight slices through LDS
  bf16_t *f_qkv = nullptr, *f_sao = nullptr, *f_caq = nullptr, *f_kT = nullptr, *f_cav = nullptr, *f_cao = nullptr,
         *f_l1 = nullptr, *f_l2 = nullptr;
  // hi/lo decoder weights (round 5): the same images of the lo planes, so the fused blocks add W_lo . X_hi
  bf16_t *fl_qkv = nullptr, *fl_sao = nullptr, *fl_caq = nullptr, *fl_kT = nullptr, *fl_cav = nullptr,
         *fl_cao = nullptr, *fl_l1 = nullptr, *fl_l2 = nullptr;
};

}  // namespace

// Captured decode loop (hipGraph): all max_len-1 steps x ~80 kernels replayed with one launch.
struct DecodeGraph {
  int B = 0, S = 0, L = 0, mode = -1, start = -1, end = -1, gen = -1;
  uint32_t drop_thr = 0;
  bool logits = false;
  int calls = 0;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  // stop-aware form (chunk > 0): one graph per chunk of `chunk` steps, each ending in the chunk's stop test, and an
  // event per chunk (decode_loop)
  int chunk = 0;
  std::vector<hipGraph_t> cgraph;
  std::vector<hipGraphExec_t> cexec;
  std::vector<hipEvent_t> cev;
  DevBuf ids, lg, uni, lp;
  void reset() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    for (hipGraphExec_t e : cexec) (void)hipGraphExecDestroy(e);
    for (hipGraph_t e : cgraph) (void)hipGraphDestroy(e);
    cexec.clear();
    cgraph.clear();
    exec = nullptr;
    graph = nullptr;
    calls = 0;
  }
  ~DecodeGraph() {
    for (hipEvent_t e : cev) (void)hipEventDestroy(e);
  }
};

struct icap_handle {
  icap_model_desc d{};
  bool use_graphs = true;
  hipStream_t cap_stream = nullptr;
  // ICAP_DEC_BRANCHES: independent decode chains per batch.  One since round 4: with the register-fragment decode
  // blocks three chains of 85 rows are bound by the dispatch of their 3 x 8 graph nodes per layer-step (≈2.9 us each,
  // 4201 per decode), one chain of 256 rows by its own kernels: decode 12.12 -> 11.47 ms/step at B = 256
  // (profiles/r04/chains_sweep.txt)
  int dec_branches = 1;
  DevBuf drop_seed;                     // the sampler's dropout seed (device word read by the kernels)
  static constexpr int MAX_BRANCHES = 4;
  hipStream_t aux_stream[MAX_BRANCHES] = {};  // streams of chains 1.. (chain 0 runs on the caller's)
  hipEvent_t ev_fork = nullptr, ev_join[MAX_BRANCHES] = {};
  DecodeGraph dg[4];  // one captured loop per mode (0 greedy, 1 sample: SCST alternates them), + 2: stop-aware (chunked)
  // stop-aware decodes: one host-mapped stop flag per chunk and mode (written by stop_scan_kernel), and the decode
  // steps the last stop-aware decode executed
  static constexpr int MAX_CHUNKS = 256;
  int* stop_host = nullptr;
  int* stop_dev = nullptr;
  int last_steps = 0;
  int* stop_flags(int mode) {
    if (!stop_host) {
      HIPCHK(hipHostMalloc((void**)&stop_host, 2 * MAX_CHUNKS * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
      HIPCHK(hipHostGetDevicePointer((void**)&stop_dev, stop_host, 0));
    }
    return stop_dev + mode * MAX_CHUNKS;
  }
  int ns = 2;  // activation planes (1 = bf16, 2 = hi/lo)
  bool i8 = false;  // ICAP_PREC_I8X2: LayerNorm-fed ViT GEMMs on int8 two-slice operands
  bool i8k = false;  // ... and MLP-2 on the block-scaled int8 GELU output (ICAP_I8_MLP2=1, opt-in)
  bool f16 = false;  // ICAP_PREC_F16: the ViT encoder on single fp16 planes (fp16 MFMA); the decoder stays bf16x2
  // ICAP_PREC_F16 on a Grid model: the eval ResNet trunk on fp16 planes - the residual stream as one fp16 plane in
  // layer1-2 and as fp16 hi/lo planes (~22 bits) in layer3-4, the bottleneck branch (conv1 / conv2 outputs) as one
  // fp16 plane, fp16 weights and MFMA (encode_grid); the tail and the decoder stay bf16x2, train-mode
  // BatchNorm stays on the bf16x2 trunk
  bool t16 = false;
  int enc_cus = 0;  // icap_set_encoder_cus: persistent encoder GEMM grids sized for a CU-masked stream (0 = all CUs)
  int enc_attn_cus = 0;  // icap_set_encoder_attention_cus: the persistent encoder attention's own budget (0 = enc_cus)
  // hi/lo decoder weights (icap_model_desc.dec_weight_planes = 2: fp32 checkpoints that are not bf16-exact): every
  // decoder GEMM weight is packed as hi = bf16(W) and lo = bf16(W - hi) and the decode runs the unfused launches,
  // whose GEMMs add W_lo . X_hi; the train-mode dropout sampler keeps the fused blocks (W_hi only)
  bool wlo = false;
  std::vector<void*> owned;
  std::vector<size_t> owned_n;  // bytes of each owned buffer
  // icap_update_weights re-packs into the buffers icap_create allocated, in the same order: alloc()
  // then hands them out again (cursor) instead of allocating, so captured decode graphs stay valid
  bool repack = false;
  size_t cursor = 0, dec_allocs = 0;  // dec_allocs: buffers of the decoder part (allocated first)
  // decoder
  float *emb = nullptr, *pe = nullptr, *fc_w = nullptr, *fc_b = nullptr;
  float* fc_w4 = nullptr;  // fc_out as [D / 4][V][4] for the head's coalesced loads (launch_head_w4)
  std::vector<DecLayer> dec;
  // vit
  float *cls = nullptr, *pos = nullptr, *vit_ln_w = nullptr, *vit_ln_b = nullptr;
  Lin conv, proj;
  Lin8 proj8;
  std::vector<VitLayer> vit;
  // grid
  float* enc_pe = nullptr;
  int enc_pe_rows = 0;  // rows of the packed encoder PE table: the most grid tokens an image may have
  std::vector<EncLayer> enc;
  std::vector<Conv> trunk;  // stem, then per bottleneck block [downsample] conv1 conv2 conv3
  bf16_t* zero = nullptr;   // 256 zero bytes: the implicit-GEMM source of out-of-image taps
  // live kernel timing (icap_profile_*): HIP events bracket each launch of the hot kernels
  struct ProfRec {
    int cls;
    double flops, bytes;
    hipEvent_t a, b;
  };
  bool prof_on = false;
  int prof_every = 1;     // icap_profile_enable(h, N >= 2): only ViT encoder layers li % N == 0 are bracketed
  bool prof_gate = true;  // the current ViT layer is bracketed (set by the layer loops)
  void prof_layer(size_t li) { prof_gate = li % (size_t)prof_every == 0; }
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<ProfRec> prof;
  hipEvent_t ev() {
    if (ev_used == ev_pool.size()) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      ev_pool.push_back(e);
    }
    return ev_pool[ev_used++];
  }
  template <class F>
  void timed(int cls, double flops, double bytes, hipStream_t s, F&& launch) {
    if (!prof_on || !prof_gate) {
      launch();
      return;
    }
    ProfRec r{cls, flops, bytes, ev(), ev()};
    HIPCHK(hipEventRecord(r.a, s));
    launch();
    HIPCHK(hipEventRecord(r.b, s));
    prof.push_back(r);
  }
  void run_gemm(const GemmArgs& g, hipStream_t s) {
    const double flops = 2.0 * g.M * g.N * g.K * g.batch;  // algorithmic (one plane)
    const double bytes = 2.0 * g.batch * ((double)g.M * g.K * g.nsplit + (double)g.N * g.K);
    timed(gemm_prof_class(g), flops, bytes, s, [&] { HIPCHK(launch_gemm(g, s)); });
  }

  // workspaces
  DevBuf e_split, e_scnt;  // GEMM tail split: partial tiles + tickets (zero at rest)
  int split_slots = -1;     // block slots per XCD of the 128 x 256 GEMM (2 per CU); 0 = tail split off
  DevBuf e_x, e_a, e_qkv, e_h, e_patch, e_sa, e_hs;  // encoder (e_sa: int8 row scales, e_hs: MLP block scales)
  // the f16 ViT encoder's second half batch (encode_vit: two halves on two streams) - its own residual stream, planes
  DevBuf e2_x, e2_a, e2_qkv, e2_h, e2_patch;
  hipStream_t enc_aux = nullptr;
  hipEvent_t enc_fork = nullptr, enc_join = nullptr;
  DevBuf t_x, t_y, t_1, t_2, t_r, t_col;  // ResNet trunk (NHWC planes)
  DevBuf t_bn;                            // train-mode BatchNorm: partial sums + scale / shift
  // decoder workspaces, one set per decode mode (0: greedy / beam / teacher-forced, 1: sampled), so
  // the greedy and sampled graphs of an SCST step can replay concurrently on two streams
  struct DecWS {
    DevBuf x, a, qkv, q, qt, c, o, h, kv, fin, part, memp, xpart, xcnt;  // xpart / xcnt: split cross-attention
    DevBuf tick;  // SlabMerge tickets of the decode blocks (one int per row; zero at rest)
    DevBuf gs;  // train-mode cross-attention value-bias weights
  } dws[2];
  DevBuf d_beam;
  // ICAP_PREC_F16 range guard: one sticky device word, set by the fp16 encoder's LayerNorm and store-only GEMM
  // kernels when a value they write is not finite in fp16; read and cleared by icap_range_check
  DevBuf rflag;
  // persistent decode step (decstep.hip): per-layer weight pointers and per-step arguments in device memory, the
  // per-step counter blocks (zeroed by one memset per decode), and the key the argument array was built for
  bool use_step = false;  // icap_set_decode_step(1) / ICAP_DEC_STEP=1 (tools): the persistent task step (opt-in)
  bool use_xdec = false;  // icap_set_decode_step(2) / ICAP_DEC_STEP=2 (tools): the group-persistent step (xdec.hip)
  DevBuf step_layers, step_args[2], step_state[2];
  DevBuf step_trace;  // tools build (ICAP_DEC_STEP_TRACE=1): per-task stamps of every step, + per-workgroup slots
  long step_key[2][8] = {};
  unsigned* range_word() {
    if (!rflag.p) {
      rflag.ensure(16);
      HIPCHK(hipMemset(rflag.p, 0, 16));
    }
    return rflag.as<unsigned>();
  }

  ~icap_handle() {
    if (stop_host) (void)hipHostFree(stop_host);
    for (DecodeGraph& g : dg) {
      g.reset();
      for (DevBuf* b : {&g.ids, &g.lg, &g.uni, &g.lp}) b->release();
    }
    if (cap_stream) (void)hipStreamDestroy(cap_stream);
    for (hipStream_t a : aux_stream)
      if (a) (void)hipStreamDestroy(a);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    for (hipEvent_t e : ev_join)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
    for (void* p : owned) (void)hipFree(p);
    for (DevBuf* b : {&t_x, &t_y, &t_1, &t_2, &t_r, &t_col, &t_bn}) b->release();
    for (DevBuf* b : {&e_x, &e_a, &e_qkv, &e_h, &e_patch, &e_sa, &e_hs, &d_beam, &e_split, &e_scnt, &rflag,
                      &step_layers, &e2_x, &e2_a, &e2_qkv, &e2_h, &e2_patch})
      b->release();
    if (enc_aux) (void)hipStreamDestroy(enc_aux);
    if (enc_fork) (void)hipEventDestroy(enc_fork);
    if (enc_join) (void)hipEventDestroy(enc_join);
    for (int i = 0; i < 2; ++i) {
      step_args[i].release();
      step_state[i].release();
    }
    for (DecWS& w : dws)
      for (DevBuf* b : {&w.x, &w.a, &w.qkv, &w.q, &w.qt, &w.c, &w.o, &w.h, &w.kv, &w.fin, &w.part, &w.memp, &w.xpart,
                         &w.xcnt, &w.gs})
        b->release();
  }

  void* alloc(size_t bytes) {
    if (repack) {
      REQUIRE(cursor < owned.size() && owned_n[cursor] == bytes, "weight update does not match the packed layout");
      return owned[cursor++];
    }
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, bytes));
    owned.push_back(p);
    owned_n.push_back(bytes);
    return p;
  }
  float* own_f32(const float* src, size_t n, hipStream_t s) {
    REQUIRE(src != nullptr, "missing parameter pointer");
    float* p = (float*)alloc(n * 4);
    HIPCHK(hipMemcpyAsync(p, src, n * 4, hipMemcpyDeviceToDevice, s));
    return p;
  }
  bf16_t* own_bf16(const float* src, size_t n, hipStream_t s) {
    REQUIRE(src != nullptr, "missing parameter pointer");
    bf16_t* p = (bf16_t*)alloc(n * 2);
    HIPCHK(launch_f32_to_bf16(src, p, (long)n, s));
    return p;
  }
  bf16_t* own_f16(const float* src, size_t n, hipStream_t s) {
    REQUIRE(src != nullptr, "missing parameter pointer");
    bf16_t* p = (bf16_t*)alloc(n * 2);
    HIPCHK(launch_f32_to_f16(src, p, (long)n, s));
    return p;
  }
  // nn.Linear packing: bf16 weights, or fp16 (half = true: the ICAP_PREC_F16 encoder)
  Lin lin(const float* w, const float* b, int N, int K, hipStream_t s, bool half = false) {
    Lin l;
    l.w = half ? own_f16(w, (size_t)N * K, s) : own_bf16(w, (size_t)N * K, s);
    l.b = b ? own_f32(b, N, s) : nullptr;
    l.N = N;
    l.K = K;
    return l;
  }
  // decoder nn.Linear, hi/lo weights when the handle has them: W_hi at w, W_lo at wl = w + N K
  Lin dlin(const float* w, const float* b, int N, int K, hipStream_t s) {
    if (!wlo) return lin(w, b, N, K, s);
    Lin l;
    l.w = own_bf16_hl(w, (size_t)N * K, s);
    l.wl = l.w + (size_t)N * K;
    l.b = b ? own_f32(b, N, s) : nullptr;
    l.N = N;
    l.K = K;
    return l;
  }
  bf16_t* own_bf16_hl(const float* src, size_t n, hipStream_t s) {  // [hi n][lo n]
    REQUIRE(src != nullptr, "missing parameter pointer");
    bf16_t* p = (bf16_t*)alloc(n * 4);
    HIPCHK(launch_split_f32(src, (long)n, p, (long)n, 2, s));
    return p;
  }
  Lin8 lin8(const float* w, const float* b, int N, int K, hipStream_t s) {
    REQUIRE(w != nullptr, "missing parameter pointer");
    Lin8 l;
    l.w = (int8_t*)alloc((size_t)2 * N * K);
    l.sw = (float*)alloc((size_t)N * 4);
    HIPCHK(launch_pack_i8_rows(w, N, K, l.w, l.sw, s));
    l.b = b ? own_f32(b, N, s) : nullptr;
    l.N = N;
    l.K = K;
    return l;
  }
  LN ln(const icap_ln_w& p, int D, hipStream_t s) { return LN{own_f32(p.w, D, s), own_f32(p.b, D, s)}; }
  // nn.Linear fed by LayerNorm ln, folded (f16 encoder): fp16 W' = W diag(gamma), bias c = W beta + b, *sum = row sums of W'
  Conv pack_conv(const icap_conv_bn_w& c, hipStream_t s) {
    REQUIRE(c.w && c.bn_w && c.bn_b && c.bn_mean && c.bn_var, "missing trunk parameter pointer");
    REQUIRE(c.cout % 64 == 0 && c.k % 2 == 1 && (c.stride == 1 || c.stride == 2), "unsupported trunk conv");
    Conv o;
    o.cout = c.cout; o.cin = c.cin; o.k = c.k; o.stride = c.stride;
    // k order = the implicit-GEMM gather order: (kh, kw, c); the 7x7 stem as 7 rows of 8 taps x 4
    // channels (one 64-B NHWC4 row segment per 32-deep k-step), padded to 8 rows for BK = 64
    const bool stem = c.k == 7;
    REQUIRE(stem ? c.cin <= 4 : (c.k == 1 || (c.k == 3 && (c.cin & (c.cin - 1)) == 0 && c.cin >= 64)),
            "unsupported trunk conv shape");
    const int cp = stem ? 4 : c.cin, kwp = stem ? 8 : c.k;
    o.Kp = stem ? 8 * 8 * 4 : (c.cin * c.k * c.k + 63) / 64 * 64;
    o.w = (bf16_t*)alloc((size_t)o.cout * o.Kp * 2);
    HIPCHK(launch_pack_conv(c.w, c.cout, c.cin, c.k, cp, kwp, o.Kp, o.w, s));
    if (t16) {
      o.w16 = (bf16_t*)alloc((size_t)o.cout * o.Kp * 2);
      HIPCHK(launch_pack_conv(c.w, c.cout, c.cin, c.k, cp, kwp, o.Kp, o.w16, s, true));
    }
    o.scale = (float*)alloc((size_t)c.cout * 4);
    o.shift = (float*)alloc((size_t)c.cout * 4);
    HIPCHK(launch_bn_fold(c.bn_w, c.bn_b, c.bn_mean, c.bn_var, c.cout, 1e-5f, o.scale, o.shift, s));
    return o;
  }

  // ---------------------------------------------------------------- GEMM helper
  void gemm(const bf16_t* A, long lda, long a_lo, const Lin& W, int M, void* C, long ldc, long c_lo, int epi,
            int out, hipStream_t s, int hm_n = 0) {
    GemmArgs g = gemm_args();
    g.hm_n = hm_n;
    g.A = A; g.lda = lda; g.a_lo = a_lo;
    g.W = W.w; g.ldw = W.K;
    g.bias = W.b;
    g.C = C; g.ldc = ldc; g.c_lo = c_lo;
    g.M = M; g.N = W.N; g.K = W.K; g.nsplit = ns; g.c_planes = ns;
    g.epi = epi; g.out = out;
#ifdef ICAP_TOOLS
    if (out == OUT_F32_RESID) tail_split(g);
#endif
    run_gemm(g, s);
  }
  // fp16 single-plane GEMM (ICAP_PREC_F16 encoder): A one fp16 plane, W packed by lin(..., half = true);
  // OUT_SPLIT writes one fp16 plane
  void gemm16(const bf16_t* A, long lda, const Lin& W, int M, void* C, long ldc, int epi, int out, hipStream_t s,
              int hm_n = 0) {
    GemmArgs g = gemm_args();
    g.hm_n = hm_n;
    g.A = A; g.lda = lda;
    g.W = W.w; g.ldw = W.K;
    g.bias = W.b;
    g.C = C; g.ldc = ldc;
    g.M = M; g.N = W.N; g.K = W.K; g.nsplit = 1; g.c_planes = 1; g.f16 = 1;
    g.epi = epi; g.out = out;
    g.range_flag = range_word();
    g.max_grid = enc_cus;
#ifdef ICAP_TOOLS
    // (round 6, tools: per-GEMM-class overrides of a pipelined encode's CU budget)
    if (enc_cus > 0) {
      const int o = out == OUT_F32_RESID ? icap_knob("ICAP_PIPE_RESID_CUS", 0) : icap_knob("ICAP_PIPE_SO_CUS", 0);
      if (o > 0) g.max_grid = o;
    }
#endif
    run_gemm(g, s);
  }
  // residual-output GEMMs (N = 768 / 512: a partial last round of tiles) split their tail tiles in K when
  // ICAP_GEMM_TAIL=1 (opt-in: measured 344 -> 363 us per launch, bench 6564 -> 6495 captions/s, DESIGN.md
  // §5); the workspace is allocated on first use, outside any capture
  void tail_split(GemmArgs& g) {
    if (split_slots < 0) {
      int cus = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) cus = 0;
      split_slots = icap_knob("ICAP_GEMM_TAIL", 0) != 1 || cus < 8 ? 0 : 2 * cus / 8;
      if (split_slots) {
        e_split.ensure(gemm_split_ws_bytes(split_slots));
        e_scnt.ensure((size_t)8 * split_slots * 4);
        HIPCHK(hipMemset(e_scnt.p, 0, e_scnt.n));
      }
    }
    if (!split_slots) return;
    g.split_ws = e_split.as<float>();
    g.split_cnt = e_scnt.as<int>();
    g.split_slots = split_slots;
  }
  // int8 two-slice GEMM: A = int8 row images [M][K/64][2][64] with row scales sa
  // (a_kscale: A block-scaled per (row, 128-deep k block) instead of sa; out = OUT_I8K writes C as block-scaled
  // int8 row images with their scales in c_kscale)
  void gemm8(const int8_t* A, const float* sa, const Lin8& W, int M, void* C, long ldc, long c_lo, int epi, int out,
             hipStream_t s, int hm_n = 0, const float* a_kscale = nullptr, float* c_kscale = nullptr) {
    GemmArgs g = gemm_args();
    g.hm_n = hm_n;
    g.A = (const bf16_t*)A; g.a_scale = sa; g.a_kscale = a_kscale; g.c_kscale = c_kscale;
    g.W = (const bf16_t*)W.w; g.w_scale = W.sw;
    g.bias = W.b;
    g.C = C; g.ldc = ldc; g.c_lo = c_lo;
    g.M = M; g.N = W.N; g.K = W.K; g.nsplit = 2; g.c_planes = ns;
    g.epi = epi; g.out = out;
    const double flops = 2.0 * M * W.N * W.K;
    const double bytes = 2.0 * ((double)M * W.K + (double)W.N * W.K);
    timed(PROF_GEMM_I8, flops, bytes, s, [&] { HIPCHK(launch_gemm_i8(g, s)); });
  }
  // decode-step GEMM (wave tiles, optional split-K into fp32 partial slabs)
  void wgemm(const bf16_t* A, long lda, long a_lo, const bf16_t* W, long ldw, const float* bias, int M, int N, int K,
             void* C, long ldc, long c_lo, int epi, int out, int tile, int ksplit, long part_stride, hipStream_t s,
             int batch = 1, long a_batch = 0, long w_batch = 0, long bias_batch = 0, long c_batch = 0,
             const bf16_t* W_lo = nullptr) {
    WaveGemmArgs g = wave_args();
    g.A = A; g.lda = lda; g.a_lo = a_lo; g.a_batch = a_batch;
    g.W = W; g.ldw = ldw; g.w_batch = w_batch; g.W_lo = W_lo;
    g.bias = bias; g.bias_batch = bias_batch;
    g.C = C; g.ldc = ldc; g.c_lo = c_lo; g.c_batch = c_batch; g.c_planes = ns;
    g.M = M; g.N = N; g.K = K; g.nsplit = ns; g.batch = batch; g.ksplit = ksplit; g.part_stride = part_stride;
    g.epi = epi; g.out = out; g.tile = tile;
    const double flops = 2.0 * M * N * K * batch;
    const double bytes = 2.0 * batch * ((double)M * K * ns + (double)N * K);
    timed(PROF_GEMM_WAVE, flops, bytes, s, [&] { HIPCHK(launch_gemm_dec(g, s)); });
  }
  void chain(const ChainArgs& a, hipStream_t s, bool fused = false) {
    const double flops = 2.0 * a.M * a.H * (64.0 * 512 + (double)a.N2 * 64);
    const double bytes = 2.0 * a.H * ((double)a.M * 512 * ns + 64.0 * 512 + (double)a.N2 * 64);
    if (fused) timed(PROF_DEC_FUSED, flops, bytes, s, [&] { HIPCHK(launch_dec_chain(a, s)); });
    else timed(PROF_GEMM_WAVE, flops, bytes, s, [&] { HIPCHK(launch_chain_dec(a, s)); });
  }
  void attention(const bf16_t* qkv, long ld, long lo, int B, int N, int H, bf16_t* out, long out_ld, long out_lo,
                 hipStream_t s, int head_major = 0) {
    const double flops = 4.0 * B * H * (double)N * N * 64;
    const double bytes = 2.0 * ns * B * (double)N * H * 64 * 4;
    timed(PROF_ENC_ATTN, flops, bytes, s,
          [&] { HIPCHK(launch_enc_attention(qkv, ld, lo, B, N, H, 0.125f, out, out_ld, out_lo, ns, s, head_major)); });
  }
};

namespace {

// the head's fc_out image ([D / 4][V][4], coalesced loads; tools knob ICAP_HEAD_W4=0: the [V][D] rows)
const float* head_w4(const icap_handle* h) {
  static const int on = icap_knob("ICAP_HEAD_W4", 1);
  return on ? h->fc_w4 : nullptr;
}

// parts: ICAP_PART_DECODER | ICAP_PART_ENCODER.  On create both, allocating; on an update (h->repack)
// the selected parts are re-packed into the same buffers.
void pack(icap_handle* h, hipStream_t s, int parts = ICAP_PART_DECODER | ICAP_PART_ENCODER) {
  const icap_model_desc& d = h->d;
  const int D = d.d_model, F = d.dim_ff;
  REQUIRE(d.nhead * 64 == D && d.nhead == 8, "decoder must have 8 heads of 64");
  REQUIRE(d.vocab >= 1 && d.vocab <= HEAD_MAX_VOCAB, "vocab must be in [1, 32768]");
  if (parts & ICAP_PART_DECODER) {
  h->cursor = 0;
  h->dec.clear();
  h->emb = h->own_f32(d.emb, (size_t)d.vocab * D, s);
  h->pe = h->own_f32(d.pe, (size_t)d.pe_len * D, s);
  h->fc_w = h->own_f32(d.fc_w, (size_t)d.vocab * D, s);
  h->fc_b = h->own_f32(d.fc_b, d.vocab, s);
  h->fc_w4 = (float*)h->alloc((size_t)d.vocab * D * 4);
  HIPCHK(launch_head_w4(h->fc_w, d.vocab, D, h->fc_w4, s));
  for (int i = 0; i < d.n_dec_layers; ++i) {
    const icap_dec_layer_w& L = d.dec_layers[i];
    DecLayer o;
    o.sa_qkv = h->dlin(L.self_attn.in_w, L.self_attn.in_b, 3 * D, D, s);
    o.sa_out = h->dlin(L.self_attn.out_w, L.self_attn.out_b, D, D, s);
    o.ca_q = h->dlin(L.cross_attn.in_w, L.cross_attn.in_b, D, D, s);
    // hi/lo: the lo plane of each of W_k^T / W_v follows its hi plane (+ D * D)
    o.ca_kT = (bf16_t*)h->alloc((size_t)D * D * 2 * (h->wlo ? 2 : 1));
    HIPCHK(launch_transpose_heads_bf16(L.cross_attn.in_w + (size_t)D * D, d.nhead, 64, D, o.ca_kT, s));
    if (h->wlo)
      HIPCHK(launch_transpose_heads_bf16(L.cross_attn.in_w + (size_t)D * D, d.nhead, 64, D, o.ca_kT + (size_t)D * D, s,
                                         1));
    o.ca_v = h->wlo ? h->own_bf16_hl(L.cross_attn.in_w + (size_t)2 * D * D, (size_t)D * D, s)
                    : h->own_bf16(L.cross_attn.in_w + (size_t)2 * D * D, (size_t)D * D, s);
    o.ca_vb = h->own_f32(L.cross_attn.in_b + 2 * D, D, s);
    o.ca_out = h->dlin(L.cross_attn.out_w, L.cross_attn.out_b, D, D, s);
    o.lin1 = h->dlin(L.lin1_w, L.lin1_b, F, D, s);
    o.lin2 = h->dlin(L.lin2_w, L.lin2_b, D, F, s);
    o.n1 = h->ln(L.norm1, D, s);
    o.n2 = h->ln(L.norm2, D, s);
    o.n3 = h->ln(L.norm3, D, s);
    // round 4: register-direct weight fragments for the fused decode blocks (tools knob ICAP_DEC_FRAG=0: the LDS-staged
    // forms, for A/B)
    static const int frag_on = icap_knob("ICAP_DEC_FRAG", 1);
    if (frag_on && D == 512 && d.nhead == 8 && F == 2048) {
      auto fp = [&](const bf16_t* w, long ldw, int ntiles, int nk, int mode, int tps, int ksl) {
        bf16_t* out = (bf16_t*)h->alloc((size_t)ntiles * nk * 512 * 2);
        HIPCHK(launch_frag_pack(w, ldw, ntiles, nk, mode, tps, ksl, out, s));
        return out;
      };
      o.f_qkv = fp(o.sa_qkv.w, D, 96, 16, 1, 0, 0);
      o.f_sao = fp(o.sa_out.w, D, 256, 2, 2, 32, 64);
      o.f_caq = fp(o.ca_q.w, D, 32, 16, 0, 0, 0);
      o.f_kT = fp(o.ca_kT, 64, 256, 2, 0, 0, 0);
      o.f_cav = fp(o.ca_v, D, 32, 16, 0, 0, 0);
      o.f_cao = fp(o.ca_out.w, D, 256, 2, 2, 32, 64);
      o.f_l1 = fp(o.lin1.w, D, 128, 16, 0, 0, 0);
      o.f_l2 = fp(o.lin2.w, F, 512, 4, 2, 32, 128);
      if (h->wlo) {  // the lo planes (Lin::wl; W_k^T and W_v keep theirs at + D * D)
        o.fl_qkv = fp(o.sa_qkv.wl, D, 96, 16, 1, 0, 0);
        o.fl_sao = fp(o.sa_out.wl, D, 256, 2, 2, 32, 64);
        o.fl_caq = fp(o.ca_q.wl, D, 32, 16, 0, 0, 0);
        o.fl_kT = fp(o.ca_kT + (size_t)D * D, 64, 256, 2, 0, 0, 0);
        o.fl_cav = fp(o.ca_v + (size_t)D * D, D, 32, 16, 0, 0, 0);
        o.fl_cao = fp(o.ca_out.wl, D, 256, 2, 2, 32, 64);
        o.fl_l1 = fp(o.lin1.wl, D, 128, 16, 0, 0, 0);
        o.fl_l2 = fp(o.lin2.wl, F, 512, 4, 2, 32, 128);
      }
    }
    h->dec.push_back(o);
  }
  if (!h->repack) h->dec_allocs = h->owned.size();
  }
  if (!(parts & ICAP_PART_ENCODER)) return;
  h->cursor = h->dec_allocs;
  h->vit.clear();
  h->enc.clear();
  h->trunk.clear();
  if (d.kind == ICAP_KIND_VIT) {
    const int V = d.vit_dim, np = (d.image / d.patch) * (d.image / d.patch);
    REQUIRE(d.vit_heads * 64 == V, "ViT heads must be 64 wide");
    h->cls = h->own_f32(d.cls, V, s);
    h->pos = h->own_f32(d.pos, (size_t)(np + 1) * V, s);
    const bool hf = h->f16;
    h->conv = h->lin(d.conv_w, d.conv_b, V, 3 * d.patch * d.patch, s, hf);
    for (int i = 0; i < d.vit_layers; ++i) {
      const icap_vit_layer_w& L = d.vit_layers_w[i];
      VitLayer o;
      o.ln1 = h->ln(L.ln_1, V, s);
      o.qkv = h->lin(L.attn.in_w, L.attn.in_b, 3 * V, V, s, hf);
      o.out = h->lin(L.attn.out_w, L.attn.out_b, V, V, s, hf);
      o.ln2 = h->ln(L.ln_2, V, s);
      o.mlp0 = h->lin(L.mlp0_w, L.mlp0_b, d.vit_mlp, V, s, hf);
      o.mlp3 = h->lin(L.mlp3_w, L.mlp3_b, V, d.vit_mlp, s, hf);
      if (h->i8) {
        o.qkv8 = h->lin8(L.attn.in_w, L.attn.in_b, 3 * V, V, s);
        o.mlp08 = h->lin8(L.mlp0_w, L.mlp0_b, d.vit_mlp, V, s);
        if (h->i8k) o.mlp38 = h->lin8(L.mlp3_w, L.mlp3_b, V, d.vit_mlp, s);
      }
      h->vit.push_back(o);
    }
    h->vit_ln_w = h->own_f32(d.vit_ln_w, V, s);
    h->vit_ln_b = h->own_f32(d.vit_ln_b, V, s);
    h->proj = h->lin(d.proj_w, d.proj_b, D, V, s, hf);
    if (h->i8) h->proj8 = h->lin8(d.proj_w, d.proj_b, D, V, s);
  } else if (d.kind == ICAP_KIND_GRID) {
    h->proj = h->lin(d.proj_w, d.proj_b, D, d.cnn_dim, s);
    if (d.n_trunk) {
      int n = 1;
      for (int st = 0; st < 4; ++st) n += 3 * d.trunk_blocks[st] + (d.trunk_blocks[st] > 0);
      REQUIRE(d.trunk && d.n_trunk == n, "trunk conv count does not match trunk_blocks");
      REQUIRE(d.trunk[0].k == 7 && d.trunk[0].stride == 2 && d.trunk[0].cin == 3, "trunk stem must be 7x7/2 on RGB");
      for (int i = 0; i < n; ++i) h->trunk.push_back(h->pack_conv(d.trunk[i], s));
      h->zero = (bf16_t*)h->alloc(256);
      HIPCHK(hipMemsetAsync(h->zero, 0, 256, s));
      REQUIRE(h->trunk.back().cout == d.cnn_dim, "trunk output channels != projection input");
    }
    h->enc_pe_rows = std::max(d.grid_tokens, d.enc_pe_len);
    h->enc_pe = h->own_f32(d.enc_pe, (size_t)h->enc_pe_rows * D, s);
    for (int i = 0; i < d.n_enc_layers; ++i) {
      const icap_enc_layer_w& L = d.enc_layers[i];
      EncLayer o;
      o.qkv = h->lin(L.attn.in_w, L.attn.in_b, 3 * D, D, s);
      o.out = h->lin(L.attn.out_w, L.attn.out_b, D, D, s);
      o.lin1 = h->lin(L.lin1_w, L.lin1_b, F, D, s);
      o.lin2 = h->lin(L.lin2_w, L.lin2_b, D, F, s);
      o.n1 = h->ln(L.norm1, D, s);
      o.n2 = h->ln(L.norm2, D, s);
      h->enc.push_back(o);
    }
  } else {
    throw Fail("unknown model kind");
  }
}

// Post-LN transformer encoder layer (nn.TransformerEncoderLayer, eval) over M rows of D.
void enc_layer_postln(icap_handle* h, const EncLayer& L, int B, int N, float* x, bf16_t* a, bf16_t* qkv, bf16_t* hb,
                      hipStream_t s) {
  const int D = h->d.d_model, F = h->d.dim_ff, M = B * N;
  const long aL = (long)M * D, qL = (long)M * 3 * D, hL = (long)M * F;
  h->gemm(a, D, aL, L.qkv, M, qkv, 3 * D, qL, EPI_NONE, OUT_SPLIT, s);
  h->attention(qkv, 3 * D, qL, B, N, D / 64, a, D, aL, s);
  h->gemm(a, D, aL, L.out, M, x, D, 0, EPI_NONE, OUT_F32_RESID, s);
  HIPCHK(launch_layernorm(x, D, M, D, 0, 0, 0, L.n1.w, L.n1.b, 1e-5f, x, D, a, D, aL, h->ns, s));
  h->gemm(a, D, aL, L.lin1, M, hb, F, hL, EPI_RELU, OUT_SPLIT, s);
  h->gemm(hb, F, hL, L.lin2, M, x, D, 0, EPI_NONE, OUT_F32_RESID, s);
  HIPCHK(launch_layernorm(x, D, M, D, 0, 0, 0, L.n2.w, L.n2.b, 1e-5f, x, D, a, D, aL, h->ns, s));
}

// ICAP_PREC_F16 form of encode_vit: every GEMM and the attention on single fp16 planes (fp16 MFMA, fp32
// accumulate); the residual stream, LayerNorm statistics, softmax and GELU stay fp32.
// One f16 ViT encode of B images on stream s (ws = 0: the handle's encoder workspaces, 1: the second half batch's, see
// encode_vit), in three parts - the prologue (patch embedding, class rows), layer li, the epilogue (final LayerNorm,
// projection) - so that encode_vit can enqueue two half batches layer by layer.
struct VitF16Run {
  icap_handle* h;
  hipStream_t s;
  int B, V, np, T, M, Dm, Kp, F, hm;
  const float* img;
  float* memory;
  float* feats;
  bf16_t *patch, *a, *qkv, *hb;
  float* x;
  unsigned* rf;
  VitF16Run(icap_handle* h_, const float* img_, int B_, float* memory_, hipStream_t s_, float* feats_, int ws)
      : h(h_), s(s_), B(B_), img(img_), memory(memory_), feats(feats_) {
    const icap_model_desc& d = h->d;
    V = d.vit_dim;
    const int g = d.image / d.patch;
    np = g * g, T = np + 1, M = B * T, Dm = d.d_model, Kp = 3 * d.patch * d.patch, F = d.vit_mlp;
    hm = T > 64 && T <= 256 ? T : 0;
    REQUIRE(hm, "ICAP_PREC_F16 encoder needs 64 < tokens <= 256");
    DevBuf &wpatch = ws ? h->e2_patch : h->e_patch, &wx = ws ? h->e2_x : h->e_x, &wa = ws ? h->e2_a : h->e_a,
           &wqkv = ws ? h->e2_qkv : h->e_qkv, &wh = ws ? h->e2_h : h->e_h;
    wpatch.ensure((size_t)B * np * Kp * 2);
    wx.ensure((size_t)M * V * 4);
    wa.ensure((size_t)M * V * 2);
    wqkv.ensure((size_t)M * 3 * V * 2);
    wh.ensure((size_t)M * F * 2);
    patch = wpatch.as<bf16_t>(), a = wa.as<bf16_t>(), qkv = wqkv.as<bf16_t>(), hb = wh.as<bf16_t>();
    x = wx.as<float>();
    // range guard (DESIGN.md §3, f16 range contract): every LayerNorm and store-only GEMM output is fp16; a value
    // that overflows (or a non-finite residual row, which any earlier overflow becomes) sets the sticky word
    rf = h->range_word();
  }
  void prologue() {
    const icap_model_desc& d = h->d;
    HIPCHK(launch_im2col_patches(img, B, 3, d.image, d.patch, patch, 0, NS_F16, s));
    {  // patch-embed GEMM: rows (b, p) -> x[b*T + 1 + p] with conv bias + pos[1 + p]
      GemmArgs ga = gemm_args();
      ga.A = patch; ga.lda = Kp;
      ga.W = h->conv.w; ga.ldw = Kp; ga.bias = h->conv.b;
      ga.C = x; ga.ldc = V;
      ga.M = B * np; ga.N = V; ga.K = Kp; ga.nsplit = 1; ga.c_planes = 1; ga.f16 = 1;
      ga.epi = EPI_NONE; ga.out = OUT_F32;
      ga.rm_group = np; ga.rm_stride = T; ga.rm_off = 1;
      ga.addend = h->pos; ga.add_ld = V; ga.add_group = np; ga.add_off = 1;
      h->run_gemm(ga, s);
    }
    HIPCHK(launch_cls_rows(h->cls, h->pos, x, B, T, V, s));
  }
  void layer(size_t li) {
    const icap_model_desc& d = h->d;
    const VitLayer& L = h->vit[li];
    h->prof_layer(li);
    HIPCHK(launch_layernorm(x, V, M, V, 0, 0, 0, L.ln1.w, L.ln1.b, 1e-6f, nullptr, 0, a, V, 0, NS_F16, s, rf));
    h->gemm16(a, V, L.qkv, M, qkv, 3 * V, EPI_NONE, OUT_SPLIT, s, hm);  // head-major [image][q|k|v x head][token][64]
    {
      const double flops = 4.0 * B * d.vit_heads * (double)T * T * 64;
      const double bytes = 2.0 * B * (double)T * V * 4;
      h->timed(PROF_ENC_ATTN, flops, bytes, s, [&] {
        int acus = h->enc_attn_cus > 0 ? h->enc_attn_cus : h->enc_cus;
#ifdef ICAP_TOOLS
        if (h->enc_cus > 0 && icap_knob("ICAP_PIPE_ATTN_CUS", -1) >= 0) acus = icap_knob("ICAP_PIPE_ATTN_CUS", 0);
#endif
        HIPCHK(launch_enc_attention(qkv, 3 * V, 0, B, T, d.vit_heads, 0.125f, a, V, 0, NS_F16, s, 1, acus));
      });
    }
    h->gemm16(a, V, L.out, M, x, V, EPI_NONE, OUT_F32_RESID, s);
    HIPCHK(launch_layernorm(x, V, M, V, 0, 0, 0, L.ln2.w, L.ln2.b, 1e-6f, nullptr, 0, a, V, 0, NS_F16, s, rf));
    h->gemm16(a, V, L.mlp0, M, hb, F, EPI_GELU, OUT_SPLIT, s);
    h->gemm16(hb, F, L.mlp3, M, x, V, EPI_NONE, OUT_F32_RESID, s);
    h->prof_gate = true;
  }
  void epilogue() {  // final LN on patch rows only (drop CLS), then projection 768 -> d_model
    HIPCHK(launch_layernorm(x, V, B * np, V, np, T, 1, h->vit_ln_w, h->vit_ln_b, 1e-6f, feats, V, a, V, 0, NS_F16, s,
                            rf));
    h->gemm16(a, V, h->proj, B * np, memory, Dm, EPI_NONE, OUT_F32, s);
  }
};
void encode_vit_f16(icap_handle* h, const float* img, int B, float* memory, hipStream_t s, float* feats = nullptr) {
  VitF16Run r(h, img, B, memory, s, feats, 0);
  r.prologue();
  for (size_t li = 0; li < h->vit.size(); ++li) r.layer(li);
  r.epilogue();
}

// feats (optional): the final-LayerNorm output of the patch tokens, (B, 196, 768) fp32 - the projection's input
// ICAP_ENC_SPLIT (round 6, variant builds): the f16 encoder runs a batch of B >= ENC_SPLIT_MIN images as two half
// batches on two streams (the caller's and the handle's enc_aux, forked / joined by events, enqueued layer by layer):
// one half's kernels fill the other's kernel tails and launch gaps.  Encodes back to back: 12.68-12.74 -> 11.89-11.92
// ms at B = 256, the memory bit-identical (every output row depends on its own image only); but an encode that follows
// a decode and a host sync, as every bench / serving step does, gains 0.05-0.25 ms only (tools/r6_enc_time.py), and
// per-launch timing of overlapping half-batch kernels no longer measures one kernel - off.  Not
// under an encoder CU budget (icap_set_encoder_cus: the aux stream is not masked).
#ifndef ICAP_ENC_SPLIT
#define ICAP_ENC_SPLIT 0
#endif
constexpr int ENC_SPLIT_MIN = 64;
void encode_vit(icap_handle* h, const float* img, int B, float* memory, hipStream_t s, float* feats = nullptr) {
  if (h->f16) {
    if (!ICAP_ENC_SPLIT || B < ENC_SPLIT_MIN || h->enc_cus > 0) {
      encode_vit_f16(h, img, B, memory, s, feats);
      return;
    }
    const icap_model_desc& d = h->d;
    const int np = (d.image / d.patch) * (d.image / d.patch), B1 = (B + 1) / 2, B2 = B - B1;
    if (!h->enc_aux) HIPCHK(hipStreamCreateWithFlags(&h->enc_aux, hipStreamNonBlocking));
    if (!h->enc_fork) HIPCHK(hipEventCreateWithFlags(&h->enc_fork, hipEventDisableTiming));
    if (!h->enc_join) HIPCHK(hipEventCreateWithFlags(&h->enc_join, hipEventDisableTiming));
    HIPCHK(hipEventRecord(h->enc_fork, s));
    HIPCHK(hipStreamWaitEvent(h->enc_aux, h->enc_fork, 0));
    // enqueued layer by layer, alternating halves (one half enqueued whole before the other started the second half
    // only after the first half's ~60 launches: no gain at all in a bench step)
    VitF16Run r1(h, img, B1, memory, s, feats, 0);
    VitF16Run r2(h, img + (long)B1 * 3 * d.image * d.image, B2, memory + (long)B1 * np * d.d_model, h->enc_aux,
                 feats ? feats + (long)B1 * np * d.vit_dim : nullptr, 1);
    r1.prologue();
    r2.prologue();
    for (size_t li = 0; li < h->vit.size(); ++li) {
      r1.layer(li);
      r2.layer(li);
    }
    r1.epilogue();
    r2.epilogue();
    HIPCHK(hipEventRecord(h->enc_join, h->enc_aux));
    HIPCHK(hipStreamWaitEvent(s, h->enc_join, 0));
    return;
  }
  const icap_model_desc& d = h->d;
  const int V = d.vit_dim, g = d.image / d.patch, np = g * g, T = np + 1, M = B * T, Dm = d.d_model;
  const int Kp = 3 * d.patch * d.patch, ns = h->ns;
  static const int hm_env = icap_knob("ICAP_QKV_HEAD_MAJOR", 1);  // 0 = row-major QKV
  const int hm = hm_env && T > 64 && T <= 256 ? T : 0;
  h->e_patch.ensure((size_t)B * np * Kp * 2 * ns);
  h->e_x.ensure((size_t)M * V * 4);
  h->e_a.ensure((size_t)M * V * 2 * ns);
  h->e_qkv.ensure((size_t)M * 3 * V * 2 * ns);
  h->e_h.ensure((size_t)M * d.vit_mlp * 2 * ns);
  bf16_t* patch = h->e_patch.as<bf16_t>();
  float* x = h->e_x.as<float>();
  bf16_t* a = h->e_a.as<bf16_t>();
  bf16_t* qkv = h->e_qkv.as<bf16_t>();
  bf16_t* hb = h->e_h.as<bf16_t>();
  const long pL = (long)B * np * Kp, aL = (long)M * V, qL = (long)M * 3 * V, hL = (long)M * d.vit_mlp;
  // ICAP_PREC_I8X2: the LayerNorm outputs as int8 two-slice row images [M][V/64][2][64] (in e_a,
  // which the bf16x2 planes of the attention output reuse afterwards) + row scales
  int8_t* a8 = (int8_t*)a;
  float* sa = nullptr;
  if (h->i8) {
    h->e_sa.ensure((size_t)M * 4);
    sa = h->e_sa.as<float>();
  }
  // ICAP_I8_MLP2: the GELU output as block-scaled int8 row images [M][3072/64][2][64] (in e_h) + one scale
  // per (row, 128-column block), the A operand of MLP-2
  float* hs = nullptr;
  if (h->i8k) {
    h->e_hs.ensure((size_t)M * (d.vit_mlp / 128) * 4);
    hs = h->e_hs.as<float>();
  }

  HIPCHK(launch_im2col_patches(img, B, 3, d.image, d.patch, patch, pL, ns, s));
  {  // patch-embed GEMM: rows (b, p) -> x[b*T + 1 + p] with conv bias + pos[1 + p]
    GemmArgs ga = gemm_args();
    ga.A = patch; ga.lda = Kp; ga.a_lo = pL;
    ga.W = h->conv.w; ga.ldw = Kp; ga.bias = h->conv.b;
    ga.C = x; ga.ldc = V;
    ga.M = B * np; ga.N = V; ga.K = Kp; ga.nsplit = ns;
    ga.epi = EPI_NONE; ga.out = OUT_F32;
    ga.rm_group = np; ga.rm_stride = T; ga.rm_off = 1;
    ga.addend = h->pos; ga.add_ld = V; ga.add_group = np; ga.add_off = 1;
    h->run_gemm(ga, s);
  }
  HIPCHK(launch_cls_rows(h->cls, h->pos, x, B, T, V, s));
  for (size_t li = 0; li < h->vit.size(); ++li) {
    const VitLayer& L = h->vit[li];
    h->prof_layer(li);
    // QKV written head-major ([image][q|k|v x head][token][64]) for the attention's contiguous rows
    if (h->i8) {
      HIPCHK(launch_layernorm_i8(x, V, M, V, 0, 0, 0, L.ln1.w, L.ln1.b, 1e-6f, a8, sa, s));
      h->gemm8(a8, sa, L.qkv8, M, qkv, 3 * V, qL, EPI_NONE, OUT_SPLIT, s, hm);
    } else {
      HIPCHK(launch_layernorm(x, V, M, V, 0, 0, 0, L.ln1.w, L.ln1.b, 1e-6f, nullptr, 0, a, V, aL, ns, s));
      h->gemm(a, V, aL, L.qkv, M, qkv, 3 * V, qL, EPI_NONE, OUT_SPLIT, s, hm);
    }
    h->attention(qkv, 3 * V, qL, B, T, d.vit_heads, a, V, aL, s, hm ? 1 : 0);
    h->gemm(a, V, aL, L.out, M, x, V, 0, EPI_NONE, OUT_F32_RESID, s);
    if (h->i8) {
      HIPCHK(launch_layernorm_i8(x, V, M, V, 0, 0, 0, L.ln2.w, L.ln2.b, 1e-6f, a8, sa, s));
      if (h->i8k) {
        h->gemm8(a8, sa, L.mlp08, M, hb, 0, 0, EPI_GELU, OUT_I8K, s, 0, nullptr, hs);
        h->gemm8((const int8_t*)hb, nullptr, L.mlp38, M, x, V, 0, EPI_NONE, OUT_F32_RESID, s, 0, hs);
        continue;
      }
      h->gemm8(a8, sa, L.mlp08, M, hb, d.vit_mlp, hL, EPI_GELU, OUT_SPLIT, s);
    } else {
      HIPCHK(launch_layernorm(x, V, M, V, 0, 0, 0, L.ln2.w, L.ln2.b, 1e-6f, nullptr, 0, a, V, aL, ns, s));
      h->gemm(a, V, aL, L.mlp0, M, hb, d.vit_mlp, hL, EPI_GELU, OUT_SPLIT, s);
    }
    h->gemm(hb, d.vit_mlp, hL, L.mlp3, M, x, V, 0, EPI_NONE, OUT_F32_RESID, s);
  }
  h->prof_gate = true;
  // final LN on patch rows only (drop CLS), then projection 768 -> d_model
  const long a2L = (long)B * np * V;
  if (feats)
    HIPCHK(launch_layernorm(x, V, B * np, V, np, T, 1, h->vit_ln_w, h->vit_ln_b, 1e-6f, feats, V, nullptr, 0, 0, 1, s));
  if (h->i8) {
    HIPCHK(launch_layernorm_i8(x, V, B * np, V, np, T, 1, h->vit_ln_w, h->vit_ln_b, 1e-6f, a8, sa, s));
    h->gemm8(a8, sa, h->proj8, B * np, memory, Dm, 0, EPI_NONE, OUT_F32, s);
    return;
  }
  HIPCHK(launch_layernorm(x, V, B * np, V, np, T, 1, h->vit_ln_w, h->vit_ln_b, 1e-6f, nullptr, 0, a, V, a2L, ns, s));
  h->gemm(a, V, a2L, h->proj, B * np, memory, Dm, 0, EPI_NONE, OUT_F32, s);
}

// Grid tail over trunk features given as row planes [B*49][C] (row = b*49 + h*7 + w, i.e. the
// flatten(2).permute(0, 2, 1) order of grid:100-101): 1x1 projection + PE, 6 post-LN layers.
// N: tokens per image (the trunk's output grid h x w; 49 at 224 x 224), at most the packed PE table's rows
void encode_grid_rows(icap_handle* h, const bf16_t* rows, long rL, int B, int N, float* memory, hipStream_t s) {
  const icap_model_desc& d = h->d;
  REQUIRE(N >= 1 && N <= h->enc_pe_rows, "grid tokens exceed the encoder's positional-encoding table (max_len)");
  const int D = d.d_model, M = B * N, C = d.cnn_dim, ns = h->ns;
  h->e_a.ensure((size_t)M * D * 2 * ns);
  h->e_qkv.ensure((size_t)M * 3 * D * 2 * ns);
  h->e_h.ensure((size_t)M * d.dim_ff * 2 * ns);
  bf16_t* a = h->e_a.as<bf16_t>();
  {  // 1x1 conv projection + positional encoding
    GemmArgs ga = gemm_args();
    ga.A = rows; ga.lda = C; ga.a_lo = rL;
    ga.W = h->proj.w; ga.ldw = C; ga.bias = h->proj.b;
    ga.C = memory; ga.ldc = D;
    ga.M = M; ga.N = D; ga.K = C; ga.nsplit = ns;
    ga.epi = EPI_NONE; ga.out = OUT_F32;
    ga.addend = h->enc_pe; ga.add_ld = D; ga.add_group = N; ga.add_off = 0;
    h->run_gemm(ga, s);
  }
  // activation planes of x for the first encoder layer's QKV GEMM
  HIPCHK(launch_split_f32(memory, (long)M * D, a, (long)M * D, ns, s));
  for (const EncLayer& L : h->enc)
    enc_layer_postln(h, L, B, N, memory, a, h->e_qkv.as<bf16_t>(), h->e_h.as<bf16_t>(), s);
}

void encode_grid_tail(icap_handle* h, const float* feats, int B, int N, float* memory, hipStream_t s) {
  const icap_model_desc& d = h->d;
  const int M = B * N, C = d.cnn_dim, ns = h->ns;
  h->e_patch.ensure((size_t)M * C * 2 * ns);
  bf16_t* rows = h->e_patch.as<bf16_t>();
  const long rL = (long)M * C;
  HIPCHK(launch_nchw_to_rows(feats, B, C, N, rows, rL, ns, s));
  encode_grid_rows(h, rows, rL, B, N, memory, s);
}

// One trunk convolution as a GEMM: rows = output pixels (NHWC), out = 2 bf16 planes of
// epi(acc * bn_scale + bn_shift (+ residual planes)).  A is `ns` planes with row stride a_ld.
struct ConvGeom {  // implicit-GEMM input geometry (GemmArgs::cv); cv = 0: A is a plain [M][K] matrix
  int cv = 0, H = 0, W = 0, C = 0, OW = 0, OH = 0;
};

// bn (train mode): the GEMM writes the raw convolution, then launch_bn_train normalises it with the batch
// statistics (updating bn's running statistics) and applies the residual / ReLU.
struct BnTrain {
  const icap_conv_bn_w* bn = nullptr;  // n_trunk entries, desc order; null: eval (folded) BatchNorm
  float momentum = 0.1f;
};

// f16 (ICAP_PREC_F16 eval trunk): A is a_planes fp16 planes, the output out_planes fp16 planes (the residual planes,
// when given, fp16 hi/lo), fp16 weights (Conv::w16); stored values that overflow fp16 set the range guard word
struct Trunk16 {
  bool on = false;
  int a_planes = 1, out_planes = 1, res_planes = 2;
};

void trunk_conv(icap_handle* h, const Conv& c, const bf16_t* A, long a_ld, long a_lo, int M, bf16_t* out, long out_lo,
                bool relu, const bf16_t* res, long res_lo, hipStream_t s, const ConvGeom& cg = ConvGeom(),
                const icap_conv_bn_w* bn = nullptr, float momentum = 0.f, const Trunk16& t16 = Trunk16()) {
  GemmArgs g = gemm_args();
  if (cg.cv) {
    g.cv = cg.cv; g.cv_H = cg.H; g.cv_W = cg.W; g.cv_OW = cg.OW; g.cv_OHW = cg.OH * cg.OW;
    g.cv_stride = cg.cv == 2 ? 2 : c.stride; g.cv_zero = h->zero;
    g.cv_cshift = 0;
    while ((1 << g.cv_cshift) < cg.C) ++g.cv_cshift;
  }
  g.A = A; g.lda = a_ld; g.a_lo = a_lo;
  g.W = c.w; g.ldw = c.Kp;
  g.C = out; g.ldc = c.cout; g.c_lo = out_lo; g.c_planes = 2;
  g.M = M; g.N = c.cout; g.K = c.Kp; g.nsplit = h->ns;
  g.out = OUT_SPLIT;
  if (t16.on) {
    REQUIRE(c.w16 && !bn, "fp16 trunk: eval BatchNorm on a handle packed with fp16 weights");
    g.f16 = 1; g.W = c.w16; g.nsplit = t16.a_planes; g.c_planes = t16.out_planes; g.res_planes = t16.res_planes;
    g.range_flag = h->range_word();
  }
  if (!bn) {
    g.bias = c.shift; g.scale = c.scale;
    g.epi = relu ? EPI_RELU : EPI_NONE;
    g.res = res; g.res_ld = c.cout; g.res_lo = res_lo;
  }
  h->run_gemm(g, s);
  if (bn) {
    h->t_bn.ensure(bn_part_bytes() + (size_t)2 * 2048 * 4);
    REQUIRE(c.cout <= 2048, "train-mode BatchNorm workspace holds 2048 channels");
    double* part = h->t_bn.as<double>();
    float* sc = (float*)((char*)h->t_bn.p + bn_part_bytes());
    HIPCHK(launch_bn_train(out, out_lo, M, c.cout, bn->bn_w, bn->bn_b, const_cast<float*>(bn->bn_mean),
                           const_cast<float*>(bn->bn_var), momentum, 1e-5f, res, res_lo, relu ? 1 : 0, part, sc,
                           sc + 2048, s));
    // keep the handle's eval-mode fold equal to the module's updated running statistics
    HIPCHK(launch_bn_fold(bn->bn_w, bn->bn_b, bn->bn_mean, bn->bn_var, c.cout, 1e-5f, c.scale, c.shift, s));
  }
}

// ResNet-101 trunk (torchvision Bottleneck, stride on the 3x3) on NHWC bf16 planes, then the tail.
// Images go through in chunks of TRUNK_CHUNK so the stem GEMM grid and the workspaces stay bounded.
constexpr int TRUNK_CHUNK = 256;

// Trunk output grid of an IH x IW image (torchvision ResNet: 7x7/2 stem pad 3, 3x3/2 max-pool pad 1, one stride-2
// 3x3 per later stage): each halving is (x - 1) / 2 + 1.
inline void trunk_grid(const icap_handle* h, int IH, int IW, int& OH, int& OW) {
  auto half = [](int x) { return (x - 1) / 2 + 1; };
  OH = half(half(IH));
  OW = half(half(IW));
  size_t ci = 1;
  for (int st = 0; st < 4; ++st)
    for (int j = 0; j < h->d.trunk_blocks[st]; ++j) {
      if (j == 0) ++ci;
      if (h->trunk[ci + 1].stride == 2) {
        OH = half(OH);
        OW = half(OW);
      }
      ci += 3;
    }
}

// images (B,3,IH,IW) -> memory (B, OH*OW, d_model).  feats (optional): the trunk output as fp32 rows (B, OH*OW,
// cnn_dim) - self.cnn(images).flatten(2).permute(0, 2, 1).  Any image size (grid:86-110 takes whatever the
// trunk returns), up to the encoder PE table's rows of tokens.
// bt.bn (train mode): batch-statistics BatchNorm over the whole batch, so B <= the chunk (one chunk)
void encode_grid(icap_handle* h, const float* img, int B, int IH, int IW, float* memory, hipStream_t s,
                 float* feats = nullptr, const BnTrain& bt = BnTrain()) {
  const icap_model_desc& d = h->d;
  REQUIRE(!h->trunk.empty(), "handle was created without the ResNet trunk (n_trunk = 0)");
  REQUIRE(IH >= 1 && IW >= 1 && IH <= 4096 && IW <= 4096, "image size must be in [1, 4096]");
  auto bnp = [&](size_t i) { return bt.bn ? bt.bn + i : nullptr; };
  int GH, GW;
  trunk_grid(h, IH, IW, GH, GW);
  const int N = GH * GW;
  REQUIRE(N <= h->enc_pe_rows, "the trunk's output grid exceeds the encoder's positional-encoding table (max_len)");
  const int ns = h->ns;
  auto half = [](int x) { return (x - 1) / 2 + 1; };
  const int H1 = half(IH), W1 = half(IW), H2 = half(H1), W2 = half(W1);  // stem, max-pool
  const long act_per_img = [&] {  // largest NHWC activation of one image (elements of one plane)
    long m = (long)H1 * W1 * h->trunk[0].cout;
    int hh = H2, ww = W2;
    size_t ci = 1;
    for (int st = 0; st < 4; ++st)
      for (int j = 0; j < d.trunk_blocks[st]; ++j) {
        if (j == 0) ++ci;
        const Conv& c1 = h->trunk[ci];
        m = std::max(m, (long)hh * ww * std::max(c1.cin, c1.cout));
        if (h->trunk[ci + 1].stride == 2) {
          hh = half(hh);
          ww = half(ww);
        }
        m = std::max(m, (long)hh * ww * h->trunk[ci + 2].cout);
        ci += 3;
      }
    return m;
  }();
  constexpr int BORDER = 3;
  const int HP = IH + 2 * BORDER, WP = IW + 2 * BORDER;  // the stem's bordered NHWC4 image
  const long col_per_img = [&] {  // stem image / stride-2 subsample of a downsample's input
    long m = (long)HP * WP * 4;
    int hh = H2, ww = W2;
    size_t ci = 1;
    for (int st = 0; st < 4; ++st)
      for (int j = 0; j < d.trunk_blocks[st]; ++j) {
        const bool ds = j == 0;
        if (ds) ++ci;
        const Conv& c2 = h->trunk[ci + 1];
        const int oh = c2.stride == 2 ? half(hh) : hh, ow = c2.stride == 2 ? half(ww) : ww;
        if (ds) m = std::max(m, (long)oh * ow * h->trunk[ci - 1].cin);
        hh = oh;
        ww = ow;
        ci += 3;
      }
    return m;
  }();
  // images per chunk: 256 at 224 x 224, fewer for larger images (the workspaces stay at the 224 size)
  const long per224 = 112L * 112 * h->trunk[0].cout;
  const int chunk = (int)std::max<long>(1, std::min<long>(TRUNK_CHUNK, TRUNK_CHUNK * per224 / act_per_img));
  REQUIRE(!bt.bn || B <= chunk, "train-mode BatchNorm needs the whole batch in one trunk chunk (B <= 256 at 224)");
  const int bc_max = std::min(B, chunk);
  const long aL = act_per_img * bc_max, cL = col_per_img * bc_max;
  for (DevBuf* b : {&h->t_x, &h->t_y, &h->t_1, &h->t_2, &h->t_r}) b->ensure((size_t)aL * 2 * 2);
  h->t_col.ensure((size_t)cL * 2 * ns);
  bf16_t *X = h->t_x.as<bf16_t>(), *Y = h->t_y.as<bf16_t>(), *T1 = h->t_1.as<bf16_t>(), *T2 = h->t_2.as<bf16_t>(),
         *R = h->t_r.as<bf16_t>(), *col = h->t_col.as<bf16_t>();
  // fp16 eval trunk (ICAP_PREC_F16): the image and the bottleneck branch as one fp16 plane; the residual stream (stem /
  // max-pool output, block and downsample outputs) as one fp16 plane in layer1-2, where it is largest (the HBM-bound
  // stage: 802k / 401k elements per image), and as fp16 hi/lo planes in layer3-4, which hold 26 of the 33 roundings
  // (CPU emulation, DESIGN.md §3: trunk features 3.2e-4 relative, memory 1.1e-3, logits 1.1e-4)
  const bool f16 = h->t16 && !bt.bn;
#ifndef ICAP_TRUNK_SINGLE
#define ICAP_TRUNK_SINGLE 0
#endif
  // ICAP_TRUNK_SINGLE (compile-time form, round 5): one fp16 residual plane in layer3-4 as well
  auto xpl = [&](int st) { return f16 ? (st < 2 || ICAP_TRUNK_SINGLE ? 1 : 2) : ns; };  // residual-stream planes
  auto t16 = [&](int a_planes, int out_planes, int res_planes = 2) {
    Trunk16 t;
    t.on = f16; t.a_planes = a_planes; t.out_planes = out_planes; t.res_planes = res_planes;
    return t;
  };
  for (int b0 = 0; b0 < B; b0 += bc_max) {
    const int bc = std::min(bc_max, B - b0);
    const Conv& stem = h->trunk[0];
    HIPCHK(launch_image_nhwc4(img + (size_t)b0 * 3 * IH * IW, bc, IH, IW, BORDER, col, cL, f16 ? 1 : ns, s, f16));
    ConvGeom sg;
    sg.cv = 2; sg.H = HP; sg.W = WP; sg.C = 4; sg.OH = H1; sg.OW = W1;
    trunk_conv(h, stem, col, 0, cL, bc * H1 * W1, T1, aL, true, nullptr, 0, s, sg, bnp(0), bt.momentum,
               t16(1, xpl(0)));
    HIPCHK(launch_maxpool3s2(T1, aL, bc, H1, W1, stem.cout, H2, W2, X, aL, xpl(0), s, f16));
    int hh = H2, ww = W2;
    size_t ci = 1;
    for (int st = 0; st < 4; ++st)
      for (int j = 0; j < d.trunk_blocks[st]; ++j) {
        const size_t ids = ci;
        const Conv* ds = j == 0 ? &h->trunk[ci++] : nullptr;
        const size_t i1 = ci;
        const Conv &c1 = h->trunk[ci], &c2 = h->trunk[ci + 1], &c3 = h->trunk[ci + 2];
        ci += 3;
        const int oh = c2.stride == 2 ? half(hh) : hh, ow = c2.stride == 2 ? half(ww) : ww;
        const int Min = bc * hh * ww, Mout = bc * oh * ow;
        const int pin = xpl(j == 0 && st > 0 ? st - 1 : st), pout = xpl(st);  // planes of X and of the output
        const bf16_t* res = X;
        int rpl = pin;
        if (ds) {  // identity branch: 1x1 conv (stride = the block's) + BN, no ReLU
          const bf16_t* dsA = X;
          long dsL = aL;
          if (ds->stride == 2) {
            HIPCHK(launch_subsample2(X, aL, bc, hh, ww, ds->cin, col, cL, pin, s));
            dsA = col;
            dsL = cL;
          }
          trunk_conv(h, *ds, dsA, ds->cin, dsL, Mout, R, aL, false, nullptr, 0, s, ConvGeom(), bnp(ids), bt.momentum,
                     t16(pin, pout));
          res = R;
          rpl = pout;
        }
        // f16: conv1 reads only the hi plane of a hi/lo residual stream - the branch it starts is one fp16 plane anyway
        // (CPU emulation, tools/numerics_trunk16_c1.py: features 3.2e-4 -> 3.7e-4 relative, memory 1.14e-3 -> 1.38e-3,
        // logits 1.07e-4 -> 1.22e-4, ids equal), and layer3-4's conv1 GEMMs then run half the MFMA work
        trunk_conv(h, c1, X, c1.cin, aL, Min, T1, aL, true, nullptr, 0, s, ConvGeom(), bnp(i1), bt.momentum,
                   t16(f16 ? 1 : pin, 1));
        ConvGeom g3;  // 3x3 conv2 read straight from T1 (implicit GEMM)
        g3.cv = 1; g3.H = hh; g3.W = ww; g3.C = c1.cout; g3.OH = oh; g3.OW = ow;
        trunk_conv(h, c2, T1, 0, aL, Mout, T2, aL, true, nullptr, 0, s, g3, bnp(i1 + 1), bt.momentum, t16(1, 1));
        trunk_conv(h, c3, T2, c3.cin, aL, Mout, Y, aL, true, res, aL, s, ConvGeom(), bnp(i1 + 2), bt.momentum,
                   t16(1, pout, rpl));
        std::swap(X, Y);
        hh = oh;
        ww = ow;
      }
    REQUIRE(hh == GH && ww == GW, "trunk output grid mismatch");
    float* fb = feats ? feats + (size_t)b0 * N * d.cnn_dim : nullptr;
    if (f16) {  // the tail reads bf16 hi/lo planes: re-split the fp16 pair (and write the fp32 features)
      HIPCHK(launch_f16planes_to_bf16(X, xpl(3) == 2 ? aL : 0, (long)bc * N * d.cnn_dim, Y, aL, fb, s));
      std::swap(X, Y);
    } else if (fb) {  // trunk features (both planes: the values the tail consumes)
      HIPCHK(launch_planes_to_f32(X, aL, (long)bc * N * d.cnn_dim, 2, fb, s));
    }
    encode_grid_rows(h, X, aL, bc, N, memory + (size_t)b0 * N * d.d_model, s);
  }
}

constexpr int MAX_KSPLIT = 16;  // partial slabs: split-K GEMMs, 8 heads (dec_sa), 16 hidden slices (dec_ffn)
constexpr int XDEC_SLABS = 33;  // the group-persistent step: 32 feed-forward slabs + the pre-LN sums

struct DecodeBufs {
  float *x, *x2, *qkv, *kc, *vc, *part;  // x2: the second residual-stream buffer of the folded LayerNorms
  bf16_t *a, *q, *qt, *c, *o, *hb, *memp;
  long aL, qL, cL, hL, memL;
  size_t kvl;  // KV-cache stride between layers (of the whole buffer)
  long PS;     // split-K slab stride (of the whole buffer)
  float* xpart;  // split cross-attention partial states / tickets
  int* xcnt;
  float* gs;     // train-mode cross-attention: per (row, head) weight of the value bias [rows][8]
  int* tick;     // SlabMerge tickets (16-row tile t of a chain starting at row r0: tick[r0 + t])
};

// Rows [r0, r0 + n) of a decode buffer set (every plane / slab / layer stride stays the whole
// buffer's), for decoding a batch as independent sub-batches; mem_rows = memory images per row.
DecodeBufs sub_bufs(const DecodeBufs& b, const icap_model_desc& d, int r0, int Lmax, int S) {
  const int D = d.d_model, H = d.nhead;
  DecodeBufs v = b;
  v.x += (size_t)r0 * D; v.x2 += (size_t)r0 * D; v.a += (size_t)r0 * D; v.qkv += (size_t)r0 * 3 * D; v.q += (size_t)r0 * D;
  v.qt += (size_t)r0 * H * D; v.c += (size_t)r0 * H * D; v.o += (size_t)r0 * D; v.hb += (size_t)r0 * d.dim_ff;
  v.kc += (size_t)r0 * H * Lmax * 64; v.vc += (size_t)r0 * H * Lmax * 64;
  v.part += (size_t)r0 * D; v.memp += (size_t)r0 * S * D;
  v.gs += (size_t)r0 * H;
  v.tick += r0;
  if (v.xpart) {
    v.xpart += cross_attn_part_floats(r0);
    v.xcnt += r0;
  }
  return v;
}

// rows: decoder rows per pass; B: memory images; kv_rows: KV-cache rows (default B; B*K for beams)
DecodeBufs dec_bufs(icap_handle* h, int rows, int B, int Lmax, int S, int kv_rows = 0, int wsi = 0) {
  if (kv_rows <= 0) kv_rows = B;
  const icap_model_desc& d = h->d;
  const int D = d.d_model, ns = h->ns, H = d.nhead;
  icap_handle::DecWS& w = h->dws[wsi];
  w.x.ensure((size_t)2 * rows * D * 4);  // x and x2
  w.a.ensure((size_t)rows * D * 2 * ns);
  w.qkv.ensure((size_t)rows * 3 * D * 4);
  w.q.ensure((size_t)rows * D * 2 * ns);
  w.qt.ensure((size_t)rows * H * D * 2 * ns);
  w.memp.ensure((size_t)B * S * D * 2 * ns);
  w.c.ensure((size_t)rows * H * D * 2 * ns);
  w.o.ensure((size_t)rows * D * 2 * ns);
  w.h.ensure((size_t)rows * d.dim_ff * 2 * ns);
  w.kv.ensure((size_t)2 * d.n_dec_layers * kv_rows * H * Lmax * 64 * 4);
  w.part.ensure((size_t)XDEC_SLABS * rows * D * 4);  // (the split-K slabs use MAX_KSPLIT of them)
  w.gs.ensure((size_t)rows * H * 4);
  const bool xsplit = cross_attn_splits(S) > 1 || (ns == 2 && (cross_attn_f16_splits() > 1 || cross_attn_f16s_on()));
  if (xsplit) w.xpart.ensure(cross_attn_part_floats(rows) * 4);
  if (xsplit && w.xcnt.n < (size_t)rows * 4) {  // tickets: zero at rest (each launch resets its own)
    w.xcnt.ensure((size_t)rows * 4);
    HIPCHK(hipMemset(w.xcnt.p, 0, w.xcnt.n));
  }
  if (w.tick.n < (size_t)(rows + 16) * 4) {  // zero at rest: every merging block resets its tile's ticket
    w.tick.ensure((size_t)(rows + 16) * 4);
    HIPCHK(hipMemset(w.tick.p, 0, w.tick.n));
  }
  DecodeBufs b;
  b.tick = w.tick.as<int>();
  b.x = w.x.as<float>(); b.x2 = b.x + (size_t)rows * D; b.a = w.a.as<bf16_t>(); b.qkv = w.qkv.as<float>();
  b.q = w.q.as<bf16_t>(); b.qt = w.qt.as<bf16_t>(); b.c = w.c.as<bf16_t>();
  b.o = w.o.as<bf16_t>(); b.hb = w.h.as<bf16_t>();
  b.kc = w.kv.as<float>();
  b.xpart = w.xpart.as<float>(); b.xcnt = w.xcnt.as<int>();
  b.part = w.part.as<float>();
  b.gs = w.gs.as<float>();
  b.vc = b.kc + (size_t)d.n_dec_layers * kv_rows * H * Lmax * 64;
  b.memp = w.memp.as<bf16_t>(); b.memL = (long)B * S * D;
  b.aL = (long)rows * D; b.qL = (long)rows * D; b.cL = (long)rows * H * D; b.hL = (long)rows * d.dim_ff;
  b.kvl = (size_t)kv_rows * H * Lmax * 64;
  b.PS = (long)rows * D;
  return b;
}

// The decoder's copy of the memory for the cross-attention: one fp16 plane in the parity precisions (ns = 2,
// launch_cross_attn_f16), one bf16 plane in the bf16 mode.
void mem_planes(icap_handle* h, const float* mem, const DecodeBufs& b, hipStream_t s) {
  if (h->ns == 2) HIPCHK(launch_f32_to_f16(mem, b.memp, b.memL, s));
  else HIPCHK(launch_split_f32(mem, b.memL, b.memp, b.memL, h->ns, s));
}

// One pass of all decoder layers over `rows` query rows (n_new per image, positions t0..t0+n_new).
// Post-LN layer (torch TransformerDecoderLayer.forward, transformer.py:1144-1153):
//   x = LN1(x + SA(x)); x = LN2(x + CA(x, mem)); x = LN3(x + W2 relu(W1 x)).
// GEMMs are wave-tile decode GEMMs; the three N=512 residual GEMMs split K into fp32 partial
// slabs that the residual-LayerNorm kernel reduces together with bias + residual.
// B here counts KV rows (sequences); mem_rpi = decoder rows per memory image (default n_new; the
// beam slots of an image for beam search); anc = beam ancestry table for the self-attention.
// drop (one-token decode only): train-mode dropout masks (DropCfg; row_base = the chain's first row)
// tail_ln (one-token decode only): the caller's head folds the last layer's residual LN3 in (HeadArgs::ln);
// the layers then leave x = the LN2 output and the FFN slabs for it instead of launching that LN.
void decoder_layers(icap_handle* h, DecodeBufs& b, int B, int n_new, int t0, int Lmax, int causal,
                    int S, hipStream_t s, const int32_t* anc = nullptr, int mem_rpi = 0,
                    const int32_t* klen = nullptr, const DropCfg* drop = nullptr, RlnArgs* tail_ln = nullptr) {
  const icap_model_desc& d = h->d;
  const int D = d.d_model, H = d.nhead, F = d.dim_ff, rows = B * n_new, ns = h->ns;
  if (mem_rpi <= 0) mem_rpi = n_new;
  const size_t kv_layer = b.kvl;
  const long PS = b.PS;  // partial slab stride
  const int KS_D = 4, KS_F = 8;    // split-K of the K=512 and K=dim_ff residual GEMMs
  // one new token per sequence (the decode loops): the fused self-attention and feed-forward blocks
  // (decode.hip); the teacher-forced / padded forms keep the separate GEMM + attention launches
  // hi/lo decoder weights (a real fp32 checkpoint): the fused blocks' hi/lo forms (round 5: the lo planes' fragment
  // images, two activation planes) - the unfused launches (whose GEMMs take W_lo) only in the bf16 mode; the train-mode
  // dropout sampler keeps the fused blocks on W_hi (the differentiated log-probs use the fp32 weights themselves)
  const bool lo_frags = h->wlo && ns == 2 && !h->dec.empty() && h->dec[0].fl_qkv;
  const bool fused = n_new == 1 && !klen && causal && D == 512 && H == 8 && F == 2048 && t0 < 64 && t0 < Lmax &&
                     (!h->wlo || drop || lo_frags);
  const bool flo = fused && h->wlo && !drop;  // the fused blocks add W_lo . X_hi
  const bool wl = h->wlo && !fused;  // GEMMs add W_lo . X_hi
  REQUIRE(!drop || (fused && ns == 2 && !anc), "dropout needs the one-token decode blocks in a parity precision");
  // round 4, measured slower and tools-only: the residual LayerNorms merged into the producing decode blocks
  // (SlabMerge; knob ICAP_DEC_MERGE, a mask: 1 = LN1 in dec_sa, 2 = LN2 in dec_chain, 4 = LN3 in dec_ffn) - the
  // merging block's tail cost 8-15 us per producer against 5 us per residual_layernorm launch
  // (profiles/r04/merge_ab.txt); a product build compiles no merge and launches the LayerNorms
#ifdef ICAP_TOOLS
  static const int merge_knob = icap_knob("ICAP_DEC_MERGE", 0);
#else
  constexpr int merge_knob = 0;
#endif
  // round 5, measured slower and tools-only: the residual LN1 / LN2 folded into the register-fragment blocks that
  // consume them (the q~ chain, dec_ffn; decode.hip fold_issue / fold_finish; knob ICAP_DEC_FOLD, a mask: 1 = LN1,
  // 2 = LN2): each block's 288 KB of slab reads cost about the 5 us launch they remove - decode 11.18-11.23 against
  // 11.02-11.05 ms, 11.37-11.44 against 11.28-11.32 on a second box (profiles/r05/fold_ab.txt).  A fold reads the
  // residual from xc and writes the normalised rows to the other x buffer (the tile's other blocks still read xc), so
  // the two buffers alternate; dec_ffn's 16 slabs then go to the second slab set.  ICAP_DEC_XCD (tools), a mask: 1 = a
  // fold's row-tile blocks on one XCD (without it the folds cost 1 ms more), 2 = dec_sa / the output chain too (their
  // weights then leave the per-XCD L2: decode 11.36-11.41 against 11.28-11.32 ms).
#ifdef ICAP_TOOLS
  static const int fold_knob = icap_knob("ICAP_DEC_FOLD", 0);
  static const int xcd_knob = icap_knob("ICAP_DEC_XCD", 1);
#else
  constexpr int fold_knob = 0, xcd_knob = 0;
#endif
  const int fold = fused && ns == 2 && !merge_knob && !flo ? fold_knob : 0;
  const int merge = fused && !flo ? merge_knob : 0;
  float* xc = b.x;                                             // the residual stream's current buffer
  auto x_other = [&] { return xc == b.x ? b.x2 : b.x; };
  float* const PF = (fold & 2) ? b.part + (size_t)MAX_KSPLIT * PS : b.part;  // dec_ffn's slabs
  for (int l = 0; l < d.n_dec_layers; ++l) {
    const DecLayer& L = h->dec[l];
    bool merged2 = false;
    DropCfg dl{};
    if (drop) {
      dl = *drop;
      dl.layer = l;
      dl.pos = t0;
    }
    // self-attention block
    if (fused) {
      DecSaArgs sa{};
      sa.A = b.a; sa.aL = b.aL; sa.nsplit = ns; sa.rows = rows;
      sa.Wqkv = L.sa_qkv.w; sa.bqkv = L.sa_qkv.b; sa.Wo = L.sa_out.w;
      sa.Wqkv_f = L.f_qkv; sa.Wo_f = L.f_sao;
      if (flo) sa.Wqkv_fl = L.fl_qkv, sa.Wo_fl = L.fl_sao;
      if (merge & 1) sa.mg = SlabMerge{b.tick, b.x, L.sa_out.b, L.n1.w, L.n1.b, 1e-5f, b.a, b.aL, 2, dl};
      sa.kc = b.kc + l * kv_layer; sa.vc = b.vc + l * kv_layer; sa.Lmax = Lmax; sa.t0 = t0; sa.scale = 0.125f;
      sa.anc = anc;
      sa.part = b.part; sa.part_stride = PS;
      sa.drop = dl;
      sa.xcd_tiles = (xcd_knob & 2) != 0;
      h->timed(PROF_DEC_FUSED, 2.0 * rows * (3.0 * D * D + (double)D * D), 2.0 * (4.0 * D * D + (double)rows * D * ns),
               s, [&] { HIPCHK(launch_dec_sa(sa, s)); });
      if (!sa.mg.tick && !(fold & 1))
        HIPCHK(launch_residual_layernorm(xc, rows, D, b.part, H, PS, L.sa_out.b, L.n1.w, L.n1.b, 1e-5f, b.a, b.aL,
                                         ns, s, dl, 2));
    } else {
      h->wgemm(b.a, D, b.aL, L.sa_qkv.w, D, L.sa_qkv.b, rows, 3 * D, D, b.qkv, 3 * D, 0, EPI_NONE, OUT_F32, WAVE_2x2,
               1, 0, s, 1, 0, 0, 0, 0, wl ? L.sa_qkv.wl : nullptr);
      HIPCHK(launch_dec_self_attn(b.qkv, B, n_new, t0, H, b.kc + l * kv_layer, b.vc + l * kv_layer, Lmax, causal,
                                  0.125f, b.o, b.aL, ns, s, anc, klen));
      h->wgemm(b.o, D, b.aL, L.sa_out.w, D, nullptr, rows, D, D, b.part, D, 0, EPI_NONE, OUT_PARTIAL, WAVE_2x2, KS_D,
               PS, s, 1, 0, 0, 0, 0, wl ? L.sa_out.wl : nullptr);
      HIPCHK(launch_residual_layernorm(b.x, rows, D, b.part, KS_D, PS, L.sa_out.b, L.n1.w, L.n1.b, 1e-5f, b.a, b.aL,
                                       ns, s));
    }
    // cross-attention block (key-absorbed)
    // per head, one launch: q_h = a Wq_h^T + bq_h, then qt[:, h*D:(h+1)*D] = q_h Wk_h (bf16 planes)
    if (wl) {  // hi/lo weights: the same two products as two decode-GEMM launches (the second batched over heads)
      h->wgemm(b.a, D, b.aL, L.ca_q.w, D, L.ca_q.b, rows, D, D, b.q, D, b.qL, EPI_NONE, OUT_SPLIT, WAVE_2x2, 1, 0, s,
               1, 0, 0, 0, 0, L.ca_q.wl);
      h->wgemm(b.q, D, b.qL, L.ca_kT, 64, nullptr, rows, D, 64, b.qt, (long)H * D, b.cL, EPI_NONE, OUT_SPLIT,
               WAVE_2x2, 1, 0, s, H, 64, (long)D * 64, 0, D, L.ca_kT + (size_t)D * D);
    } else {
      ChainArgs c{};
      c.X = b.a; c.ldx = D; c.x_lo = b.aL; c.x_hstride = 0;
      c.W1 = L.ca_q.w; c.b1 = L.ca_q.b;
      c.W2 = L.ca_kT; c.ldw2 = 64; c.w2_hstride = (long)D * 64;
      c.C = b.qt; c.ldc = (long)H * D; c.c_lo = b.cL; c.c_hstride = D;
      c.M = rows; c.N2 = D; c.H = H; c.nsplit = ns; c.out = OUT_SPLIT;
      if (fused) c.W1f = L.f_caq, c.W2f = L.f_kT;
      if (flo) c.W1fl = L.fl_caq, c.W2fl = L.fl_kT;
      if (fold & 1) {  // X = LN1(x + SA): dec_sa's 8 slabs
        c.fold = RlnArgs{xc, x_other(), b.part, H, PS, L.sa_out.b, L.n1.w, L.n1.b, 1e-5f, dl, 2};
        c.xcd_tiles = xcd_knob & 1;
        xc = x_other();
      }
      h->chain(c, s, fused);
    }
    h->timed(PROF_CROSS_ATTN, 4.0 * rows * H * (double)S * D, 2.0 * (double)(rows / mem_rpi) * S * D, s, [&] {
      if (ns == 2)
        HIPCHK(launch_cross_attn_f16(b.qt, b.cL, b.memp, rows, mem_rpi, S, 0.125f, b.c, b.cL, s, dl,
                                     drop ? b.gs : nullptr, b.xpart, b.xcnt));
      else
        HIPCHK(launch_cross_attn_mfma(b.qt, b.cL, b.memp, b.memL, rows, mem_rpi, S, 0.125f, b.c, b.cL, ns, s,
                                      b.xpart, b.xcnt));
    });
    // per head, one launch: o_h = c_h Wv_h^T + bv_h, then slab h = o_h Wo[:, h*64:(h+1)*64]^T; the
    // residual LN sums the H slabs (the output projection as a split-K over heads)
    if (wl) {  // hi/lo weights: the value projection batched over heads into o, then a split-K out-projection
      h->wgemm(b.c, (long)H * D, b.cL, L.ca_v, D, L.ca_vb, rows, 64, D, b.o, D, b.aL, EPI_NONE, OUT_SPLIT, WAVE_2x2,
               1, 0, s, H, D, 64L * D, 64, 64, L.ca_v + (size_t)D * D);
      h->wgemm(b.o, D, b.aL, L.ca_out.w, D, nullptr, rows, D, D, b.part, D, 0, EPI_NONE, OUT_PARTIAL, WAVE_2x2, KS_D,
               PS, s, 1, 0, 0, 0, 0, L.ca_out.wl);
    } else {
      ChainArgs c{};
      c.X = b.c; c.ldx = (long)H * D; c.x_lo = b.cL; c.x_hstride = D;
      c.W1 = L.ca_v; c.b1 = L.ca_vb;
      c.W2 = L.ca_out.w; c.ldw2 = D; c.w2_hstride = 64;
      c.C = b.part; c.ldc = D; c.part_stride = PS;
      c.M = rows; c.N2 = D; c.H = H; c.nsplit = ns; c.out = OUT_PARTIAL;
      if (drop) c.b1_scale = b.gs;  // the value bias weighs sum_s P_s m_s under probability dropout
      if (fused) c.W1f = L.f_cav, c.W2f = L.f_cao;
      if (flo) c.W1fl = L.fl_cav, c.W2fl = L.fl_cao;
      c.xcd_tiles = fused && (xcd_knob & 2);
      if (fused && (merge & 2)) c.mg = SlabMerge{b.tick, b.x, L.ca_out.b, L.n2.w, L.n2.b, 1e-5f, b.a, b.aL, 4, dl};
      h->chain(c, s, fused);
      merged2 = c.mg.tick != nullptr;
    }
    if (!merged2 && !(fold & 2))
      HIPCHK(launch_residual_layernorm(xc, rows, D, b.part, wl ? KS_D : H, PS, L.ca_out.b, L.n2.w, L.n2.b, 1e-5f, b.a,
                                       b.aL, ns, s, dl, 4));
    // feed-forward block
    if (fused) {
      DecFfnArgs ff{};
      ff.A = b.a; ff.aL = b.aL; ff.nsplit = ns; ff.rows = rows;
      ff.W1 = L.lin1.w; ff.b1 = L.lin1.b; ff.W2 = L.lin2.w;
      ff.W1f = L.f_l1; ff.W2f = L.f_l2;
      if (flo) ff.W1fl = L.fl_l1, ff.W2fl = L.fl_l2;
      const bool head_folds = tail_ln && l + 1 == d.n_dec_layers;  // the caller's head normalises instead
      if ((merge & 4) && !head_folds)
        ff.mg = SlabMerge{b.tick, b.x, L.lin2.b, L.n3.w, L.n3.b, 1e-5f, b.a, b.aL, 6, dl};
      ff.part = PF; ff.part_stride = PS;
      ff.drop = dl;
      if (fold & 2) {  // X = LN2(x + CA): the chain's 8 slabs
        ff.fold = RlnArgs{xc, x_other(), b.part, H, PS, L.ca_out.b, L.n2.w, L.n2.b, 1e-5f, dl, 4};
        ff.xcd_tiles = xcd_knob & 1;
        xc = x_other();
      }
      h->timed(PROF_DEC_FUSED, 4.0 * rows * (double)D * F, 2.0 * (2.0 * D * F + (double)rows * D * ns), s,
               [&] { HIPCHK(launch_dec_ffn(ff, s)); });
      const RlnArgs ln3{xc, nullptr, PF, F / 128, PS, L.lin2.b, L.n3.w, L.n3.b, 1e-5f, dl, 6};
      if (tail_ln && l + 1 == d.n_dec_layers) {
        *tail_ln = ln3;  // the caller's head normalises (reading x from ln3.x)
      } else if (!ff.mg.tick) {  // back into b.x (the buffer the next layer's folds and the callers start from)
        HIPCHK(launch_residual_layernorm(b.x, rows, D, ln3.parts, ln3.nparts, PS, ln3.bias, ln3.w, ln3.b, ln3.eps, b.a,
                                         b.aL, ns, s, dl, 6, xc));
        xc = b.x;
      }
    } else {
      h->wgemm(b.a, D, b.aL, L.lin1.w, D, L.lin1.b, rows, F, D, b.hb, F, b.hL, EPI_RELU, OUT_SPLIT, WAVE_2x2, 1, 0, s,
               1, 0, 0, 0, 0, wl ? L.lin1.wl : nullptr);
      h->wgemm(b.hb, F, b.hL, L.lin2.w, F, nullptr, rows, D, F, b.part, D, 0, EPI_NONE, OUT_PARTIAL, WAVE_2x2, KS_F,
               PS, s, 1, 0, 0, 0, 0, wl ? L.lin2.wl : nullptr);
      HIPCHK(launch_residual_layernorm(b.x, rows, D, b.part, KS_F, PS, L.lin2.b, L.n3.w, L.n3.b, 1e-5f, b.a, b.aL,
                                       ns, s));
    }
  }
}

// ---- persistent decode steps (decstep.hip, xdec.hip): measured slower than the launch loop, compiled
// into the tools build only; a product build has neither kernel and icap_set_decode_step refuses modes 1 / 2.
#ifdef ICAP_TOOLS
#include "icap_tools_steps.inc"
#else
bool step_path(const icap_handle*, int, const DropCfg*) { return false; }
bool xdec_path(const icap_handle*, int, int, int, const DropCfg*) { return false; }
#endif

// Steps [t_begin, t_end) of the loop (t_end < 0: to the end); the prologue (start column, step-0 embedding, finished
// flags) only with t_begin = 0 - a stop-aware decode runs the loop as consecutive ranges (decode_loop)
void decode_loop_eager(icap_handle* h, const float* mem, int B, int S, int max_len, int start, int end, int32_t* ids,
                       float* step_logits, const float* uniforms, float* logp, hipStream_t s,
                       const DropCfg* drop = nullptr, int t_begin = 0, int t_end = -1) {
  const icap_model_desc& d = h->d;
  REQUIRE(B > 0 && max_len >= 1, "bad batch / max_len");
  REQUIRE(max_len <= d.pe_len, "max_len exceeds the positional-encoding table (PositionalEncoding max_len)");
  REQUIRE(S > 0 && S <= 256, "memory length must be in [1, 256]");
  if (t_end < 0) t_end = max_len - 1;
  const int D = d.d_model, wsi = uniforms ? 1 : 0;
  DecodeBufs b = dec_bufs(h, B, B, max_len, S, 0, wsi);
  const float scale = (float)std::sqrt((double)D);
  if (mem) mem_planes(h, mem, b, s);
  uint8_t* fin = nullptr;
  if (uniforms) {
    h->dws[wsi].fin.ensure((size_t)B);
    fin = h->dws[wsi].fin.as<uint8_t>();
  }
  if (t_begin == 0) {
    HIPCHK(launch_fill_col(ids, B, max_len, 0, start, s));
    HIPCHK(launch_embed(nullptr, 0, start, B, 1, 0, h->emb, h->pe, D, scale, b.x, b.a, b.aL, h->ns, s,
                        drop ? *drop : DropCfg{}));
    if (fin) HIPCHK(launch_fill_u8(fin, B, 0, s));  // a kernel node: reset on every graph replay
  }
  // The images are independent: with dec_branches = n the batch decodes as n independent chains of
  // consecutive rows on n streams (n parallel branches of the captured graph), so their latency-bound
  // launches overlap.
  // (two chains pay from 128 rows each: B = 256 +3.4 %, B = 128 -6 %, tools/ab_env.sh)
  // ICAP_DEC_MIN_ROWS: smallest chain (64-row chains measured slower)
  // Round 2 (fused decode blocks, tools/chains_r2.sh, B = 256): 2 chains 13.25 ms/step of decode, 3 chains of
  // 85 rows 12.73, 4 chains of 64 rows 13.37 - so 3 chains from 80 rows each (B = 128 keeps one chain).  Round 4:
  // one chain (icap_handle::dec_branches); icap_set_decode_chains still splits
  static const int min_rows = std::max(16, icap_knob("ICAP_DEC_MIN_ROWS", 80));
#ifdef ICAP_TOOLS
  if (xdec_path(h, B, S, max_len, drop)) {  // one group-persistent launch per step (all layers) + the head
    const size_t st = xdec_state_ints();
    h->step_state[wsi].ensure(st * 4 * (size_t)(max_len - 1));
    HIPCHK(hipMemsetAsync(h->step_state[wsi].p, 0, st * 4 * (size_t)(max_len - 1), s));
    const DecStepLayer* layers = step_layers(h);
    for (int t = 0; t + 1 < max_len; ++t) {
      XdecArgs a{};
      a.layers = layers; a.n_layers = d.n_dec_layers; a.rows = B; a.t0 = t; a.Lmax = max_len; a.S = S;
      a.x = b.x; a.a = b.a; a.aL = b.aL;
      a.kc = b.kc; a.vc = b.vc; a.kvl = (long)b.kvl;
      a.qv = b.qkv; a.ctx = b.o; a.ctxL = b.aL;
      a.slab = b.part; a.y = b.part + (size_t)32 * b.PS;
      a.q2 = b.q; a.q2L = b.qL; a.qt = b.qt; a.cL = b.cL; a.c = b.c;
      a.mem16 = b.memp;
      a.ctr = h->step_state[wsi].as<int>() + (size_t)t * st;
      a.err = h->range_word();
#ifdef ICAP_TOOLS
      static const int xtrace = icap_knob("ICAP_XDEC_TRACE", 0);
      if (xtrace) {  // per-workgroup barrier stamps of every step (tools/xdec_trace.py)
        const size_t per = (size_t)256 * XDEC_TRACE_BARRIERS * 2;
        h->step_trace.ensure(per * 8 * (size_t)(max_len - 1));
        a.trace = h->step_trace.as<unsigned long long>() + per * t;
      }
#endif
      const double fl = 2.0 * B * d.n_dec_layers * (4.0 * D * D * 2 + 2.0 * D * d.dim_ff + 4.0 * d.nhead * S * D);
      h->timed(PROF_DEC_FUSED, fl, 0.0, s, [&] { HIPCHK(launch_xdec(a, s)); });
      HeadArgs ha{};  // the kernel leaves x = the last layer's LN3 output: no fold
      ha.x = b.x; ha.rows = B; ha.Dm = D; ha.W = h->fc_w; ha.W4 = head_w4(h); ha.bias = h->fc_b; ha.V = d.vocab;
      ha.logits = step_logits ? step_logits + (size_t)t * B * d.vocab : nullptr;
      ha.ld_logits = d.vocab;
      ha.ids = ids; ha.ld_ids = max_len; ha.id_col = t + 1;
      ha.uniforms = uniforms ? uniforms + (size_t)t * B : nullptr;
      ha.logp = logp ? logp + t : nullptr; ha.ld_logp = max_len - 1;
      ha.finished = fin; ha.end_token = end;
      if (t + 2 < max_len) {
        ha.emb = h->emb; ha.pe = h->pe; ha.pe_pos = t + 1; ha.emb_scale = scale;
        ha.x_next = b.x; ha.a_next = b.a; ha.lo = b.aL; ha.nsplit = h->ns;
      }
      HIPCHK(launch_head(ha, s));
    }
    return;
  }
  if (step_path(h, max_len, drop)) {  // one persistent launch per step (all layers) + the head
    const DecStepArgs* dargs = step_args(h, b, B, S, max_len, wsi, drop, s);
    const size_t st_ints = dec_step_state_ints(d.n_dec_layers, B);
    HIPCHK(hipMemsetAsync(h->step_state[wsi].p, 0, st_ints * 4 * (size_t)(max_len - 1), s));
    for (int t = 0; t + 1 < max_len; ++t) {
      DecStepArgs a{};  // the host copy the launcher validates (the kernel reads dargs[t])
      a.layers = h->step_layers.as<DecStepLayer>();
      a.n_layers = d.n_dec_layers; a.rows = B; a.t0 = t; a.Lmax = max_len; a.S = S;
      a.ctr = h->step_state[wsi].as<int>(); a.qhead = a.ctr; a.err = h->range_word();
      const double fl = 2.0 * B * d.n_dec_layers * (4.0 * D * D * 2 + 2.0 * D * d.dim_ff + 4.0 * d.nhead * S * D);
      h->timed(PROF_DEC_FUSED, fl, 0.0, s, [&] { HIPCHK(launch_dec_step(a, dargs + t, s)); });
      const DecLayer& Ll = h->dec[d.n_dec_layers - 1];
      DropCfg dl{};
      if (drop) {
        dl = *drop;
        dl.row_base = 0;
        dl.layer = d.n_dec_layers - 1;
        dl.pos = t;
      }
      HeadArgs ha{};
      ha.ln = RlnArgs{b.x, nullptr, b.part, d.dim_ff / 128, b.PS, Ll.lin2.b, Ll.n3.w, Ll.n3.b, 1e-5f, dl, 6};
      ha.x = b.x; ha.rows = B; ha.Dm = D; ha.W = h->fc_w; ha.W4 = head_w4(h); ha.bias = h->fc_b; ha.V = d.vocab;
      ha.logits = step_logits ? step_logits + (size_t)t * B * d.vocab : nullptr;
      ha.ld_logits = d.vocab;
      ha.ids = ids; ha.ld_ids = max_len; ha.id_col = t + 1;
      ha.uniforms = uniforms ? uniforms + (size_t)t * B : nullptr;
      ha.logp = logp ? logp + t : nullptr; ha.ld_logp = max_len - 1;
      ha.finished = fin; ha.end_token = end;
      if (t + 2 < max_len) {
        ha.emb = h->emb; ha.pe = h->pe; ha.pe_pos = t + 1; ha.emb_scale = scale;
        ha.x_next = b.x; ha.a_next = b.a; ha.lo = b.aL; ha.nsplit = h->ns;
        if (drop) {
          ha.drop = *drop;
          ha.drop.row_base = 0;
        }
      }
      HIPCHK(launch_head(ha, s));
    }
    return;
  }
#endif
  const bool persist = step_path(h, max_len, drop);
  const int nb = persist ? 1 : std::max(1, std::min(h->dec_branches, B / min_rows));
  if (nb > 1) {
    if (!h->ev_fork) HIPCHK(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
    HIPCHK(hipEventRecord(h->ev_fork, s));
    for (int i = 1; i < nb; ++i) {
      if (!h->aux_stream[i]) HIPCHK(hipStreamCreateWithFlags(&h->aux_stream[i], hipStreamNonBlocking));
      if (!h->ev_join[i]) HIPCHK(hipEventCreateWithFlags(&h->ev_join[i], hipEventDisableTiming));
      HIPCHK(hipStreamWaitEvent(h->aux_stream[i], h->ev_fork, 0));
    }
  }
  // step-major issue order: launched eagerly, the chains' kernels reach their streams interleaved
  // (a captured graph has the same dependencies either way)
  for (int t = t_begin; t < t_end; ++t) {
    for (int part = 0; part < nb; ++part) {
      const int r0 = (int)((long)B * part / nb), n = (int)((long)B * (part + 1) / nb) - r0;
      hipStream_t st = part ? h->aux_stream[part] : s;
      DecodeBufs v = sub_bufs(b, d, r0, max_len, S);
      DropCfg dc{};
      if (drop) {
        dc = *drop;
        dc.row_base = r0;
      }
      HeadArgs ha{};
      decoder_layers(h, v, n, 1, t, max_len, 1, S, st, nullptr, 0, nullptr, drop ? &dc : nullptr, &ha.ln);
      ha.x = ha.ln.parts ? ha.ln.x : v.x; ha.rows = n; ha.Dm = D; ha.W = h->fc_w; ha.W4 = head_w4(h); ha.bias = h->fc_b; ha.V = d.vocab;
      ha.logits = step_logits ? step_logits + ((size_t)t * B + r0) * d.vocab : nullptr;
      ha.ld_logits = d.vocab;
      ha.ids = ids + (size_t)r0 * max_len; ha.ld_ids = max_len; ha.id_col = t + 1;
      ha.uniforms = uniforms ? uniforms + (size_t)t * B + r0 : nullptr;
      ha.logp = logp ? logp + (size_t)r0 * (max_len - 1) + t : nullptr; ha.ld_logp = max_len - 1;
      ha.finished = fin ? fin + r0 : nullptr; ha.end_token = end;
      if (t + 2 < max_len) {
        ha.emb = h->emb; ha.pe = h->pe; ha.pe_pos = t + 1; ha.emb_scale = scale;
        ha.x_next = v.x; ha.a_next = v.a; ha.lo = v.aL; ha.nsplit = h->ns;
        if (drop) ha.drop = dc;
      }
      HIPCHK(launch_head(ha, st));
    }
  }
  for (int i = 1; i < nb; ++i) {
    HIPCHK(hipEventRecord(h->ev_join[i], h->aux_stream[i]));
    HIPCHK(hipStreamWaitEvent(s, h->ev_join[i], 0));
  }
}

// Graph path: the first call with a new (B, S, max_len, mode) runs eagerly (allocates the
// workspace, sets kernel attributes); the second captures the whole loop on a private stream into
// a hipGraph over handle-owned in/out buffers; later calls copy memory in, replay, copy ids out.
// drop_p > 0 (sampling only): train-mode dropout masks under drop_seed (DropCfg, common.h)
// chunk > 0 (stop-aware, round 6): the loop as consecutive graphs of `chunk` steps, each ending in a stop test of its
// columns (stop_scan_kernel -> a host-mapped flag per chunk).  Before launching chunk c the host waits for chunk c - 2's
// event and reads its flag: once a chunk reports the reference's stop (greedy: a step whose every latest token is end,
// vit:321-323; sampling: every row finished, scst_loss:246-249) no further chunk is launched - the GPU always holds
// one more chunk than the host has checked, so the checks add no gap, and at most one chunk past the stop runs.  The
// columns not computed are filled (ids = end, log-probs = 0), so the callers' stop rules return the reference's
// sequence.  *steps = decode steps executed.  The host blocks until chunk (last - 1) has run.
void decode_loop(icap_handle* h, const float* mem, int B, int S, int max_len, int start, int end, int32_t* ids,
                 float* step_logits, const float* uniforms, float* logp, hipStream_t s, float drop_p = 0.f,
                 uint32_t drop_seed = 0, int chunk = 0, int* steps = nullptr) {
  const int mode = uniforms ? 1 : 0;
  const bool wl = step_logits != nullptr;
  const int nsteps = max_len - 1;
  if (chunk >= nsteps) chunk = 0;  // one chunk: the fixed-length graph
  REQUIRE(chunk >= 0 && (chunk == 0 || (nsteps + chunk - 1) / chunk <= icap_handle::MAX_CHUNKS) && chunk <= 64,
          "decode chunk: 0 (fixed length) or 1..64 steps, at most 256 chunks");
#ifdef ICAP_TOOLS
  if (chunk && (step_path(h, max_len, nullptr) || xdec_path(h, B, S, max_len, nullptr))) chunk = 0;
#endif
  if (steps) *steps = nsteps;
  DecodeGraph& g = h->dg[mode + (chunk ? 2 : 0)];
  DropCfg drop{};
  if (drop_p > 0.f) {
    REQUIRE(mode == 1 && drop_p < 1.f, "dropout applies to sampling, with p in [0, 1)");
    h->drop_seed.ensure(4 * 2);
    uint32_t* sp = h->drop_seed.as<uint32_t>() + mode;
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)sp, (int)drop_seed, 1, s));  // outside any captured graph
    drop.seed = sp;
    drop.thr = (uint32_t)std::min(4294967295.0, std::floor((double)drop_p * 4294967296.0 + 0.5));
    drop.scale = 1.0f / (1.0f - drop_p);
  }
  const DropCfg* dp = drop.thr ? &drop : nullptr;
  if (!h->use_graphs) {
    decode_loop_eager(h, mem, B, S, max_len, start, end, ids, step_logits, uniforms, logp, s, dp);
    return;
  }
  if (g.B != B || g.S != S || g.L != max_len || g.mode != mode || g.logits != wl || g.start != start ||
      g.end != end || g.drop_thr != drop.thr || g.chunk != chunk || ((g.exec || !g.cexec.empty()) && g.gen != g_ws_generation)) {
    g.reset();
    g.B = B; g.S = S; g.L = max_len; g.mode = mode; g.logits = wl; g.start = start; g.end = end;
    g.drop_thr = drop.thr; g.chunk = chunk;
  }
  const int nch = chunk ? (nsteps + chunk - 1) / chunk : 1;
  int* flags = chunk ? h->stop_flags(mode) : nullptr;
  // the chunk sequence with the host's stop checks (launch(c) enqueues chunk c and its stop test), then the tail fill
  auto run_chunks = [&](auto&& launch, int32_t* ids_buf, float* lp_buf) {
    while ((int)g.cev.size() < nch) {
      hipEvent_t e = nullptr;
      HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      g.cev.push_back(e);
    }
    int launched = 0;
    for (int c = 0; c < nch; ++c) {
      if (c >= 2) {
        HIPCHK(hipEventSynchronize(g.cev[c - 2]));
        if (__atomic_load_n(h->stop_host + mode * icap_handle::MAX_CHUNKS + c - 2, __ATOMIC_ACQUIRE)) break;
      }
      launch(c);
      HIPCHK(hipEventRecord(g.cev[c], s));
      launched = c + 1;
    }
    const int done = std::min(nsteps, launched * chunk);
    if (steps) *steps = done;
    h->last_steps = done;
    if (done < nsteps) HIPCHK(launch_stop_tail(ids_buf, B, max_len, done, end, mode ? lp_buf : nullptr, s));
  };
  if (!g.exec && g.cexec.empty() && g.calls++ == 0) {
    if (!chunk) {
      decode_loop_eager(h, mem, B, S, max_len, start, end, ids, step_logits, uniforms, logp, s, dp);
    } else {
      run_chunks([&](int c) {
        const int t0 = c * chunk, t1 = std::min(nsteps, t0 + chunk);
        decode_loop_eager(h, c ? nullptr : mem, B, S, max_len, start, end, ids, step_logits, uniforms, logp, s, dp, t0, t1);
        HIPCHK(launch_stop_scan(ids, B, max_len, t0 + 1, t1 + 1, end, mode ? h->dws[mode].fin.as<uint8_t>() : nullptr,
                                flags + c, s));
      }, ids, logp);
    }
    return;
  }
  const size_t lg_bytes = (size_t)(max_len - 1) * B * h->d.vocab * 4;
  if (!g.exec && g.cexec.empty()) {
    g.ids.ensure((size_t)B * max_len * 4);
    if (wl) g.lg.ensure(lg_bytes);
    if (mode) {
      g.uni.ensure((size_t)(max_len - 1) * B * 4);
      g.lp.ensure((size_t)B * (max_len - 1) * 4);
    }
    DecodeBufs pb = dec_bufs(h, B, B, max_len, S, 0, mode);  // make sure nothing allocates during capture
    if (mode) h->dws[mode].fin.ensure((size_t)B);
#ifdef ICAP_TOOLS
    if (step_path(h, max_len, dp)) step_args(h, pb, B, S, max_len, mode, dp, s);  // ... nor uploads
    if (xdec_path(h, B, S, max_len, dp)) {
      h->step_state[mode].ensure(xdec_state_ints() * 4 * (size_t)(max_len - 1));
      step_layers(h);
    }
#else
    (void)pb;
#endif
    if (!h->cap_stream) HIPCHK(hipStreamCreateWithFlags(&h->cap_stream, hipStreamNonBlocking));
    HIPCHK(hipStreamSynchronize(s));
    const bool prof = h->prof_on;
    h->prof_on = false;
    for (int c = 0; c < nch; ++c) {
      HIPCHK(hipStreamBeginCapture(h->cap_stream, hipStreamCaptureModeThreadLocal));
      try {
        const int t0 = chunk ? c * chunk : 0, t1 = chunk ? std::min(nsteps, t0 + chunk) : nsteps;
        decode_loop_eager(h, nullptr, B, S, max_len, start, end, g.ids.as<int32_t>(),
                          wl ? g.lg.as<float>() : nullptr, mode ? g.uni.as<float>() : nullptr,
                          mode ? g.lp.as<float>() : nullptr, h->cap_stream, dp, t0, t1);
        if (chunk)
          HIPCHK(launch_stop_scan(g.ids.as<int32_t>(), B, max_len, t0 + 1, t1 + 1, end,
                                  mode ? h->dws[mode].fin.as<uint8_t>() : nullptr, flags + c, h->cap_stream));
      } catch (...) {
        hipGraph_t dead = nullptr;
        (void)hipStreamEndCapture(h->cap_stream, &dead);
        if (dead) (void)hipGraphDestroy(dead);
        h->prof_on = prof;
        throw;
      }
      hipGraph_t gr = nullptr;
      hipGraphExec_t ex = nullptr;
      HIPCHK(hipStreamEndCapture(h->cap_stream, &gr));
      const hipError_t ie = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
      if (ie != hipSuccess) {
        (void)hipGraphDestroy(gr);
        h->prof_on = prof;
        HIPCHK(ie);
      }
      if (chunk) {
        g.cgraph.push_back(gr);
        g.cexec.push_back(ex);
      } else {
        g.graph = gr;
        g.exec = ex;
      }
    }
    h->prof_on = prof;
    g.gen = g_ws_generation;
  }
  DecodeBufs b = dec_bufs(h, B, B, max_len, S, 0, mode);  // no allocation: sized at capture
  mem_planes(h, mem, b, s);
  if (mode) HIPCHK(hipMemcpyAsync(g.uni.p, uniforms, (size_t)(max_len - 1) * B * 4, hipMemcpyDeviceToDevice, s));
  if (!chunk) {
    HIPCHK(hipGraphLaunch(g.exec, s));
  } else {
    run_chunks([&](int c) { HIPCHK(hipGraphLaunch(g.cexec[c], s)); }, g.ids.as<int32_t>(), mode ? g.lp.as<float>() : nullptr);
  }
  HIPCHK(hipMemcpyAsync(ids, g.ids.p, (size_t)B * max_len * 4, hipMemcpyDeviceToDevice, s));
  if (wl) HIPCHK(hipMemcpyAsync(step_logits, g.lg.p, lg_bytes, hipMemcpyDeviceToDevice, s));
  if (mode) HIPCHK(hipMemcpyAsync(logp, g.lp.p, (size_t)B * (max_len - 1) * 4, hipMemcpyDeviceToDevice, s));
}

// Batched beam search (models/vit_transformer_model.py:327-420, grid:253-322): B images x K beam
// slots as B*K decoder rows; per step the rows' logits go to beam_select (beam.hip), which keeps
// the per-image state (live beam count, scores, token histories, ancestry of the KV rows, the best
// completed sequence).  Images that stopped keep being decoded (their rows are ignored) so every
// launch has a fixed shape.
void decode_beam(icap_handle* h, const float* mem, int B, int S, int max_len, int K, int grid_variant, int start,
                 int end, int32_t* ids, int32_t* lens, hipStream_t s) {
  const icap_model_desc& d = h->d;
  REQUIRE(B > 0 && max_len >= 2 && K >= 1 && K <= 15, "bad batch / max_len / beam size (1..15)");
  REQUIRE(max_len <= d.pe_len, "max_len exceeds the positional-encoding table (PositionalEncoding max_len)");
  REQUIRE(S > 0 && S <= 256, "memory length must be in [1, 256]");
  const int D = d.d_model, rows = B * K, V = d.vocab;
  DecodeBufs b = dec_bufs(h, rows, B, max_len, S, rows);
  // beam state, carved from one buffer: seq[2] + anc[2] (rows x L ints), best_seq (B x L),
  // scores[2] (rows), kcur / done / ncomp / best_len (B ints), best_score (B), logits (rows x V)
  const size_t RL = (size_t)rows * max_len, BL = (size_t)B * max_len;
  const size_t n_i = 4 * RL + BL + 4 * (size_t)B, n_f = 2 * (size_t)rows + B + (size_t)rows * V;
  h->d_beam.ensure((n_i + n_f) * 4 + 64);
  int32_t* base = h->d_beam.as<int32_t>();
  int32_t* seq[2] = {base, base + RL};
  int32_t* anc[2] = {base + 2 * RL, base + 3 * RL};
  int32_t* best_seq = base + 4 * RL;
  int* kcur = base + 4 * RL + BL;
  int* done = kcur + B;
  int* ncomp = done + B;
  int* best_len = ncomp + B;
  float* fb = (float*)(best_len + B);
  float* sc[2] = {fb, fb + rows};
  float* best_score = fb + 2 * rows;
  float* logits = best_score + B;
  mem_planes(h, mem, b, s);
  HIPCHK(launch_beam_init(B, K, start, max_len, seq[0], seq[1], anc[0], anc[1], sc[0], kcur, done, ncomp, best_score,
                          best_len, s));
  const float scale = (float)std::sqrt((double)D);
  int cur = 0;
  for (int t = 0; t + 1 < max_len; ++t) {
    HIPCHK(launch_embed(seq[cur] + t, max_len, 0, rows, 1, t, h->emb, h->pe, D, scale, b.x, b.a, b.aL, h->ns, s));
    decoder_layers(h, b, rows, 1, t, max_len, 1, S, s, t > 0 ? anc[cur] : nullptr, K);
    HeadArgs ha{};
    ha.x = b.x; ha.rows = rows; ha.Dm = D; ha.W = h->fc_w; ha.W4 = head_w4(h); ha.bias = h->fc_b; ha.V = V;
    ha.logits = logits; ha.ld_logits = V;
    h->dws[0].fin.ensure((size_t)rows * 4);  // scratch argmax ids
    ha.ids = h->dws[0].fin.as<int32_t>(); ha.ld_ids = 1; ha.id_col = 0;
    HIPCHK(launch_head(ha, s));
    HIPCHK(launch_beam_select(logits, V, B, K, t, max_len, grid_variant, end, seq[cur], seq[cur ^ 1], anc[cur],
                              anc[cur ^ 1], sc[cur], sc[cur ^ 1], kcur, done, ncomp, best_score, best_seq, best_len,
                              s));
    cur ^= 1;
  }
  HIPCHK(launch_beam_finalize(B, K, max_len, seq[cur], sc[cur], kcur, ncomp, best_seq, best_len, ids, lens, s));
}

// ------------------------------------------------------------------------------------------------
// Decoder training pass (SCST's teacher-forced recompute with autograd, utils/scst_loss.py:124-128;
// reference: the autograd graph of SCSTLoss._sample_with_log_probs, scst_loss.py:210-254, and its
// loss.backward(), scripts/train_vit_transformer_scst_optimized.py:261).  fp32 parameters straight from
// the caller's tensors (no packing: they change every optimizer step), fp32-accurate products
// (train.hip).  The forward keeps every activation the backward reads in the caller's workspace.
struct TrainWS {
  int B, T, S, D, H, F, V, L, M, MS;
  struct Layer {
    float *x, *qkv, *p, *c, *xh1, *rs1, *x1, *q2, *k2, *v2, *p2, *c2, *xh2, *rs2, *x2, *hh, *xh3, *rs3;
    float *pd, *pd2, *hd;  // dropped attention probabilities / hidden (alias p, p2, hh without dropout)
  };
  DropCfg drop{};          // thr 0: eval-mode pass
  std::vector<Layer> lay;
  float *xL, *logits, *lse;
  float *dx, *dc, *tmp, *dq, *dqkv, *dp, *dh, *dk, *dv, *dlog, *part, *skpart, *dm;
  uint32_t* seed;
  static constexpr size_t SK_FLOATS = (size_t)8 << 20;  // split-K partial sums of the weight gradients
  size_t floats = 0;
  TrainWS(const icap_model_desc& d, int B_, int T_, int S_, float* base, float drop_p = 0.f) {
    B = B_; T = T_; S = S_; D = d.d_model; H = d.nhead; F = d.dim_ff; V = d.vocab; L = d.n_dec_layers;
    const bool dr = drop_p > 0.f;
    M = B * T; MS = B * S;
    size_t off = 0;
    auto take = [&](size_t n) {
      float* p = base ? base + off : nullptr;
      off += (n + 63) / 64 * 64;  // 256-B aligned carve-outs
      return p;
    };
    const size_t MD = (size_t)M * D, MSD = (size_t)MS * D;
    lay.resize(L);
    for (Layer& y : lay) {
      y.x = take(MD); y.qkv = take(3 * MD); y.p = take((size_t)B * H * T * T); y.c = take(MD);
      y.xh1 = take(MD); y.rs1 = take(M); y.x1 = take(MD); y.q2 = take(MD); y.k2 = take(MSD); y.v2 = take(MSD);
      y.p2 = take((size_t)B * H * T * S); y.c2 = take(MD); y.xh2 = take(MD); y.rs2 = take(M); y.x2 = take(MD);
      y.hh = take((size_t)M * F); y.xh3 = take(MD); y.rs3 = take(M);
      y.pd = dr ? take((size_t)B * H * T * T) : y.p;
      y.pd2 = dr ? take((size_t)B * H * T * S) : y.p2;
      y.hd = dr ? take((size_t)M * F) : y.hh;
    }
    xL = take(MD); logits = take((size_t)M * V); lse = take(M);
    dx = take(MD); dc = take(MD); tmp = take(MD); dq = take(MD); dqkv = take(3 * MD);
    dp = take((size_t)B * H * T * std::max(T, S)); dh = take((size_t)M * F); dk = take(MSD); dv = take(MSD);
    dlog = take((size_t)M * V);
    part = take(colsum_scratch_floats(std::max(std::max(3 * D, F), std::max(V, D))));
    skpart = take(SK_FLOATS);
    dm = dr ? take(MD) : nullptr;
    seed = (uint32_t*)take(64);
    if (dr) {
      drop.seed = seed;
      drop.thr = (uint32_t)std::min(4294967295.0, std::floor((double)drop_p * 4294967296.0 + 0.5));
      drop.scale = 1.0f / (1.0f - drop_p);
    }
    floats = off;
  }
};

void train_check(const icap_model_desc* d, int B, int T, int S) {
  REQUIRE(d && d->dec_layers && d->emb && d->pe && d->fc_w && d->fc_b, "null decoder parameters");
  REQUIRE(d->d_model == 512 && d->nhead == 8, "the training pass needs d_model 512, 8 heads");
  REQUIRE(B > 0 && T > 0 && S > 0 && T <= d->pe_len, "bad batch / length / memory length");
}

struct TG {  // strided GEMM call builder (train.hip TGemmArgs)
  TGemmArgs a{};
  int nb = 1;
  TG(const float* A, long sam, long sak, const float* B, long sbn, long sbk, float* C, long scm, long scn, int M, int N,
     int K) {
    a.A = A; a.sam = sam; a.sak = sak; a.B = B; a.sbn = sbn; a.sbk = sbk; a.C = C; a.scm = scm; a.scn = scn;
    a.M = M; a.N = N; a.K = K; a.nb2 = 1; a.alpha = 1.f; a.beta = 0.f;
  }
  TG& batch(int nb1, int nb2, long sab1, long sab2, long sbb1, long sbb2, long scb1, long scb2) {
    nb = nb1 * nb2; a.nb2 = nb2;
    a.sab1 = sab1; a.sab2 = sab2; a.sbb1 = sbb1; a.sbb2 = sbb2; a.scb1 = scb1; a.scb2 = scb2;
    return *this;
  }
  TG& alpha(float v) { a.alpha = v; return *this; }
  TG& beta(float v) { a.beta = v; return *this; }
  TG& bias(const float* b) { a.bias = b; return *this; }
  TG& relu() { a.relu = 1; return *this; }
  void run(hipStream_t s) { HIPCHK(launch_tgemm(a, nb, s)); }
};
// Y (M x N) = X (M x K) W^T (+ b): nn.Linear
void t_lin(const float* X, const float* W, const float* b, float* Y, int M, int N, int K, hipStream_t s,
           bool relu = false) {
  TG g(X, K, 1, W, K, 1, Y, N, 1, M, N, K);
  g.bias(b);
  if (relu) g.relu();
  g.run(s);
}
// dX (M x K) (+)= dY (M x N) W (N x K)
void t_dx(const float* dY, const float* W, float* dX, int M, int N, int K, hipStream_t s, float beta = 0.f) {
  TG(dY, N, 1, W, 1, K, dX, K, 1, M, K, N).beta(beta).run(s);
}
// dW (N x K) = dY^T (N x M) X (M x K): few output tiles and a long sum over the rows, so the sum is
// split over blocks (partials in skpart, reduced in split order) until the launch has ~512 blocks
void t_dw(const float* dY, const float* X, float* dW, int M, int N, int K, hipStream_t s, float* skpart) {
  TG g(dY, 1, N, X, 1, K, dW, K, 1, N, K, M);
  const long tiles = (long)((N + 63) / 64) * ((K + 63) / 64);
  int ks = (int)std::min<long>(16, (512 + tiles - 1) / tiles);
  while (ks > 1 && ((long)ks * N * K > (long)TrainWS::SK_FLOATS || M / ks < 128)) --ks;
  if (ks > 1) {
    g.a.ksplit = ks;
    g.a.part = skpart;
  }
  g.run(s);
}

void train_forward(const icap_model_desc& d, TrainWS& w, const int32_t* ids, const float* mem, int end,
                   float* logp, hipStream_t s) {
  const int B = w.B, T = w.T, S = w.S, D = w.D, H = w.H, F = w.F, V = w.V, M = w.M, MS = w.MS;
  const long ld = T + 1;
  const bool dr = w.drop.thr != 0;
  auto drop_at = [&](int layer) {
    DropCfg c = w.drop;
    c.layer = layer;
    return c;
  };
  HIPCHK(launch_embed_fwd(ids, ld, B, T, d.emb, d.pe, D, (float)std::sqrt((double)D), w.lay[0].x, s));
  if (dr) HIPCHK(launch_drop_rows(w.lay[0].x, w.lay[0].x, B, T, D, drop_at(0), 0, s));
  for (int l = 0; l < w.L; ++l) {
    const icap_dec_layer_w& P = d.dec_layers[l];
    TrainWS::Layer& y = w.lay[l];
    float* xnext = l + 1 < w.L ? w.lay[l + 1].x : w.xL;
    const DropCfg dl = drop_at(l);
    // self-attention (causal): per (image, head) S = q k^T / 8 -> softmax -> P v
    t_lin(y.x, P.self_attn.in_w, P.self_attn.in_b, y.qkv, M, 3 * D, D, s);
    TG(y.qkv, 3 * D, 1, y.qkv + D, 3 * D, 1, y.p, T, 1, T, T, 64)
        .batch(B, H, (long)T * 3 * D, 64, (long)T * 3 * D, 64, (long)H * T * T, (long)T * T).alpha(0.125f).run(s);
    HIPCHK(launch_softmax_rows(y.p, (long)B * H * T, T, T, 1, s));
    if (dr) HIPCHK(launch_drop_attn(y.p, y.pd, B, H, T, T, 128, dl, 1, s));
    TG(y.pd, T, 1, y.qkv + 2 * D, 1, 3 * D, y.c, D, 1, T, 64, T)
        .batch(B, H, (long)H * T * T, (long)T * T, (long)T * 3 * D, 64, (long)T * D, 64).run(s);
    t_lin(y.c, P.self_attn.out_w, P.self_attn.out_b, w.tmp, M, D, D, s);
    if (dr) HIPCHK(launch_drop_rows(w.tmp, w.tmp, B, T, D, dl, 2, s));
    HIPCHK(launch_ln_fwd(y.x, w.tmp, P.norm1.w, P.norm1.b, 1e-5f, M, D, y.x1, y.xh1, y.rs1, s));
    // cross-attention over the memory
    t_lin(y.x1, P.cross_attn.in_w, P.cross_attn.in_b, y.q2, M, D, D, s);
    t_lin(mem, P.cross_attn.in_w + (size_t)D * D, P.cross_attn.in_b + D, y.k2, MS, D, D, s);
    t_lin(mem, P.cross_attn.in_w + (size_t)2 * D * D, P.cross_attn.in_b + 2 * D, y.v2, MS, D, D, s);
    TG(y.q2, D, 1, y.k2, D, 1, y.p2, S, 1, T, S, 64)
        .batch(B, H, (long)T * D, 64, (long)S * D, 64, (long)H * T * S, (long)T * S).alpha(0.125f).run(s);
    HIPCHK(launch_softmax_rows(y.p2, (long)B * H * T, S, T, 0, s));
    if (dr) HIPCHK(launch_drop_attn(y.p2, y.pd2, B, H, T, S, 256, dl, 3, s));
    TG(y.pd2, S, 1, y.v2, 1, D, y.c2, D, 1, T, 64, S)
        .batch(B, H, (long)H * T * S, (long)T * S, (long)S * D, 64, (long)T * D, 64).run(s);
    t_lin(y.c2, P.cross_attn.out_w, P.cross_attn.out_b, w.tmp, M, D, D, s);
    if (dr) HIPCHK(launch_drop_rows(w.tmp, w.tmp, B, T, D, dl, 4, s));
    HIPCHK(launch_ln_fwd(y.x1, w.tmp, P.norm2.w, P.norm2.b, 1e-5f, M, D, y.x2, y.xh2, y.rs2, s));
    // feed-forward
    t_lin(y.x2, P.lin1_w, P.lin1_b, y.hh, M, F, D, s, true);
    if (dr) HIPCHK(launch_drop_rows(y.hh, y.hd, B, T, F, dl, 5, s));
    t_lin(y.hd, P.lin2_w, P.lin2_b, w.tmp, M, D, F, s);
    if (dr) HIPCHK(launch_drop_rows(w.tmp, w.tmp, B, T, D, dl, 6, s));
    HIPCHK(launch_ln_fwd(y.x2, w.tmp, P.norm3.w, P.norm3.b, 1e-5f, M, D, xnext, y.xh3, y.rs3, s));
  }
  t_lin(w.xL, d.fc_w, d.fc_b, w.logits, M, V, D, s);
  HIPCHK(launch_logp_fwd(w.logits, V, ids, ld, B, T, end, logp, w.lse, s));
}

void train_backward(const icap_model_desc& d, const icap_model_desc& g, TrainWS& w, const int32_t* ids,
                    const float* mem, int end, const float* dlogp, float* dmem, hipStream_t s) {
  const int B = w.B, T = w.T, S = w.S, D = w.D, H = w.H, F = w.F, V = w.V, M = w.M, MS = w.MS;
  const long ld = T + 1;
  auto G = [](const float* p) { return const_cast<float*>(p); };
  auto colsum = [&](const float* src, int rows, int n, const float* dst) {
    HIPCHK(launch_colsum(src, n, rows, n, w.part, G(dst), 0, s));
  };
  auto ln_back = [&](const float* xh, const float* rs, const icap_ln_w& P, const icap_ln_w& Pg) {
    colsum(w.dx, M, D, Pg.b);
    HIPCHK(launch_ln_bwd(w.dx, xh, rs, P.w, M, D, w.tmp, s));
    colsum(w.tmp, M, D, Pg.w);
  };
  const bool dr = w.drop.thr != 0;
  // do = dropout mask * ds (the sub-layer output's gradient; ds itself stays in dx for the residual)
  auto masked = [&](int layer, int site) -> const float* {
    if (!dr) return w.dx;
    DropCfg c = w.drop;
    c.layer = layer;
    HIPCHK(launch_drop_rows(w.dx, w.dm, B, T, D, c, site, s));
    return w.dm;
  };
  HIPCHK(launch_logp_bwd(w.logits, w.lse, dlogp, V, ids, ld, B, T, end, w.dlog, s));
  t_dw(w.dlog, w.xL, G(g.fc_w), M, V, D, s, w.skpart);
  colsum(w.dlog, M, V, g.fc_b);
  t_dx(w.dlog, d.fc_w, w.dx, M, V, D, s);
  for (int l = w.L - 1; l >= 0; --l) {
    const icap_dec_layer_w& P = d.dec_layers[l];
    const icap_dec_layer_w& Pg = g.dec_layers[l];
    TrainWS::Layer& y = w.lay[l];
    DropCfg dl = w.drop;
    dl.layer = l;
    // x3 = LN3(x2 + drop(W2 drop(relu(W1 x2 + b1)) + b2))
    ln_back(y.xh3, y.rs3, P.norm3, Pg.norm3);
    const float* df = masked(l, 6);
    t_dw(df, y.hd, G(Pg.lin2_w), M, D, F, s, w.skpart);
    colsum(df, M, D, Pg.lin2_b);
    t_dx(df, P.lin2_w, w.dh, M, D, F, s);
    if (dr) HIPCHK(launch_drop_rows(w.dh, w.dh, B, T, F, dl, 5, s));
    HIPCHK(launch_relu_bwd(w.dh, y.hh, (long)M * F, s));
    t_dw(w.dh, y.x2, G(Pg.lin1_w), M, F, D, s, w.skpart);
    colsum(w.dh, M, F, Pg.lin1_b);
    t_dx(w.dh, P.lin1_w, w.dx, M, F, D, s, 1.f);
    // x2 = LN2(x1 + CA(x1, mem))
    ln_back(y.xh2, y.rs2, P.norm2, Pg.norm2);
    const float* do2 = masked(l, 4);
    t_dw(do2, y.c2, G(Pg.cross_attn.out_w), M, D, D, s, w.skpart);
    colsum(do2, M, D, Pg.cross_attn.out_b);
    t_dx(do2, P.cross_attn.out_w, w.dc, M, D, D, s);
    TG(w.dc, D, 1, y.v2, D, 1, w.dp, S, 1, T, S, 64)  // d(dropped P2) = dc2 V2^T
        .batch(B, H, (long)T * D, 64, (long)S * D, 64, (long)H * T * S, (long)T * S).run(s);
    TG(y.pd2, 1, S, w.dc, 1, D, w.dv, D, 1, S, 64, T)  // dV2 = (dropped P2)^T dc2
        .batch(B, H, (long)H * T * S, (long)T * S, (long)T * D, 64, (long)S * D, 64).run(s);
    if (dr) HIPCHK(launch_drop_attn(w.dp, w.dp, B, H, T, S, 256, dl, 3, s));
    HIPCHK(launch_softmax_bwd(y.p2, w.dp, (long)B * H * T, S, s));
    TG(w.dp, S, 1, y.k2, 1, D, w.dq, D, 1, T, 64, S)  // dq2 = dS2 K2 / 8
        .batch(B, H, (long)H * T * S, (long)T * S, (long)S * D, 64, (long)T * D, 64).alpha(0.125f).run(s);
    TG(w.dp, 1, S, y.q2, 1, D, w.dk, D, 1, S, 64, T)  // dK2 = dS2^T q2 / 8
        .batch(B, H, (long)H * T * S, (long)T * S, (long)T * D, 64, (long)S * D, 64).alpha(0.125f).run(s);
    t_dw(w.dq, y.x1, G(Pg.cross_attn.in_w), M, D, D, s, w.skpart);
    colsum(w.dq, M, D, Pg.cross_attn.in_b);
    t_dx(w.dq, P.cross_attn.in_w, w.dx, M, D, D, s, 1.f);
    t_dw(w.dk, mem, G(Pg.cross_attn.in_w) + (size_t)D * D, MS, D, D, s, w.skpart);
    colsum(w.dk, MS, D, Pg.cross_attn.in_b + D);
    t_dw(w.dv, mem, G(Pg.cross_attn.in_w) + (size_t)2 * D * D, MS, D, D, s, w.skpart);
    colsum(w.dv, MS, D, Pg.cross_attn.in_b + 2 * D);
    if (dmem) {
      t_dx(w.dk, P.cross_attn.in_w + (size_t)D * D, dmem, MS, D, D, s, l == w.L - 1 ? 0.f : 1.f);
      t_dx(w.dv, P.cross_attn.in_w + (size_t)2 * D * D, dmem, MS, D, D, s, 1.f);
    }
    // x1 = LN1(x + SA(x))
    ln_back(y.xh1, y.rs1, P.norm1, Pg.norm1);
    const float* do1 = masked(l, 2);
    t_dw(do1, y.c, G(Pg.self_attn.out_w), M, D, D, s, w.skpart);
    colsum(do1, M, D, Pg.self_attn.out_b);
    t_dx(do1, P.self_attn.out_w, w.dc, M, D, D, s);
    TG(w.dc, D, 1, y.qkv + 2 * D, 3 * D, 1, w.dp, T, 1, T, T, 64)  // d(dropped P) = dc v^T
        .batch(B, H, (long)T * D, 64, (long)T * 3 * D, 64, (long)H * T * T, (long)T * T).run(s);
    TG(y.pd, 1, T, w.dc, 1, D, w.dqkv + 2 * D, 3 * D, 1, T, 64, T)  // dv = (dropped P)^T dc
        .batch(B, H, (long)H * T * T, (long)T * T, (long)T * D, 64, (long)T * 3 * D, 64).run(s);
    if (dr) HIPCHK(launch_drop_attn(w.dp, w.dp, B, H, T, T, 128, dl, 1, s));
    HIPCHK(launch_softmax_bwd(y.p, w.dp, (long)B * H * T, T, s));
    TG(w.dp, T, 1, y.qkv + D, 1, 3 * D, w.dqkv, 3 * D, 1, T, 64, T)  // dq = dS k / 8
        .batch(B, H, (long)H * T * T, (long)T * T, (long)T * 3 * D, 64, (long)T * 3 * D, 64).alpha(0.125f).run(s);
    TG(w.dp, 1, T, y.qkv, 1, 3 * D, w.dqkv + D, 3 * D, 1, T, 64, T)  // dk = dS^T q / 8
        .batch(B, H, (long)H * T * T, (long)T * T, (long)T * 3 * D, 64, (long)T * 3 * D, 64).alpha(0.125f).run(s);
    t_dw(w.dqkv, y.x, G(Pg.self_attn.in_w), M, 3 * D, D, s, w.skpart);
    colsum(w.dqkv, M, 3 * D, Pg.self_attn.in_b);
    t_dx(w.dqkv, P.self_attn.in_w, w.dx, M, 3 * D, D, s, 1.f);
  }
  if (dr) {
    DropCfg c = w.drop;
    c.layer = 0;
    HIPCHK(launch_drop_rows(w.dx, w.dx, B, T, D, c, 0, s));
  }
  HIPCHK(launch_embed_bwd(ids, ld, B, T, w.dx, D, V, (float)std::sqrt((double)D), G(g.emb), s));
}

}  // namespace

// ================================================================================== C ABI
extern "C" {

int icap_abi_version(void) { return ICAP_ABI_VERSION; }
const char* icap_last_error(void) { return g_err.c_str(); }

const char* icap_knobs_set() {
  static const char* const names[] = {
      "ICAP_CONV_CLASS", "ICAP_GEMM_GROUP", "ICAP_GEMM256_WAVES", "ICAP_GEMM_TALL_MIN_K", "ICAP_GEMM_TALL_BM",
      "ICAP_GEMM_TALL_KS", "ICAP_I8_NOMFMA", "ICAP_I8_GROUP", "ICAP_I8_NT_STORE", "ICAP_I8_TILE",
      "ICAP_ENC_ATTN_PIPE", "ICAP_ENC_ATTN_QPW", "ICAP_XATTN_KS", "ICAP_POISON", "ICAP_GEMM_TAIL",
      "ICAP_QKV_HEAD_MAJOR", "ICAP_DEC_MIN_ROWS", "ICAP_I8_MLP2", "ICAP_DEC_BRANCHES", "ICAP_F16_GEMM",
      "ICAP_F16_PRES", "ICAP_XATTN16_KS", "ICAP_XATTN16_CK", "ICAP_ENC_ATTN16_QPW", "ICAP_F16_PP", "ICAP_DEC_FRAG",
      "ICAP_ENC_ATTN16_FULL", "ICAP_XATTN16_S", "ICAP_EAF_ABL", "ICAP_DEC_MERGE", "ICAP_XATTN16_WK",
      "ICAP_F16P_ABL", "ICAP_F16_RES_BM", "ICAP_XATTN16_NB",
      "ICAP_HEAD_W4", "ICAP_DEC_STEP", "ICAP_DEC_STEP_TRACE", "ICAP_XDEC_TRACE", "ICAP_GEMM_NARROW",
      "ICAP_GEMM_C3", "ICAP_CONV_PRE", "ICAP_CONV_RMW", "ICAP_DEC_FOLD", "ICAP_DEC_XCD", "ICAP_EAF_PERS",
      "ICAP_PIPE_RESID_CUS", "ICAP_PIPE_SO_CUS", "ICAP_PIPE_ATTN_CUS"};
  for (const char* n : names)
    if (getenv(n)) return n;
  return "";
}

int icap_tools_build(void) {
#ifdef ICAP_TOOLS
  return 1;
#else
  return 0;
#endif
}

int icap_create(const icap_model_desc* desc, void* stream, icap_handle** out) {
  return guarded([&] {
    REQUIRE(desc && out, "null argument");
#ifndef ICAP_TOOLS
    if (*icap_knobs_set())
      throw Fail(std::string(icap_knobs_set()) +
                 " is set: it is a measurement knob that only a tools build (-DICAP_TOOLS) reads; "
                 "unset it or build with `python -m image_caption_amd.build --tools`");
#endif
    REQUIRE(desc->precision == ICAP_PREC_BF16 || desc->precision == ICAP_PREC_BF16X2 ||
                desc->precision == ICAP_PREC_I8X2 || desc->precision == ICAP_PREC_F16,
            "bad precision");
    icap_handle* h = new icap_handle();
    try {
      h->d = *desc;
      h->ns = desc->precision == ICAP_PREC_BF16 ? 1 : 2;
      h->i8 = desc->precision == ICAP_PREC_I8X2 && desc->kind == ICAP_KIND_VIT;
      h->f16 = desc->precision == ICAP_PREC_F16 && desc->kind == ICAP_KIND_VIT;
      h->t16 = desc->precision == ICAP_PREC_F16 && desc->kind == ICAP_KIND_GRID;
      REQUIRE(desc->dec_weight_planes >= 0 && desc->dec_weight_planes <= 2, "dec_weight_planes must be 0, 1 or 2");
      h->wlo = desc->dec_weight_planes == 2;
#ifdef ICAP_TOOLS
      {
        const int mode = icap_knob("ICAP_DEC_STEP", 0);
        h->use_step = mode == 1;
        h->use_xdec = mode == 2;
      }
#endif
      // measured and rejected as the default: MLP-2 fed by the block-scaled GELU output takes
      // 1211 us (two-step fold: 256 VGPRs, 30 spilled) / 646 us (per-step fold, 64-column blocks) against
      // 467 us for the bf16x2 form
      h->i8k = h->i8 && icap_tools_build() && icap_knob("ICAP_I8_MLP2", 0) == 1;
      h->dec_branches = std::max(1, std::min(icap_handle::MAX_BRANCHES, icap_knob("ICAP_DEC_BRANCHES", h->dec_branches)));
      pack(h, (hipStream_t)stream);
      HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    } catch (...) {
      delete h;
      throw;
    }
    // layer pointers in the desc belong to the caller; drop them
    h->d.dec_layers = nullptr;
    h->d.vit_layers_w = nullptr;
    h->d.enc_layers = nullptr;
    h->d.trunk = nullptr;
    *out = h;
  });
}

// Streams restricted to a subset of the CUs (hipExtStreamCreateWithCUMask), for running the
// encoder of one batch beside the decode of the previous one without the two fighting over CUs.
// The n selected CUs are taken 8 per 32-CU block (bits i with i % 32 < n / 8), which spreads them
// evenly over the 8 XCDs whether mask bits enumerate CUs XCD-major or XCD-interleaved.
int icap_stream_create_cu_mask(int n_cus, int complement, int priority, void** out) {
  return guarded([&] {
    REQUIRE(out, "null argument");
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, dev));
    const int total = prop.multiProcessorCount;
    REQUIRE(total % 32 == 0 && n_cus > 0 && n_cus < total && n_cus % (total / 32) == 0,
            "n_cus must be a positive multiple of (CUs / 32) below the CU count");
    const int per_block = n_cus / (total / 32);
    std::vector<uint32_t> mask((total + 31) / 32, 0u);
    for (int i = 0; i < total; ++i) {
      const bool sel = (i % 32) < per_block;
      if (sel != (complement != 0)) mask[i / 32] |= 1u << (i % 32);
    }
    hipStream_t st = nullptr;
    HIPCHK(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    (void)priority;
    *out = st;
  });
}

int icap_stream_destroy(void* stream) {
  return guarded([&] { HIPCHK(hipStreamDestroy((hipStream_t)stream)); });
}

int icap_update_weights(icap_handle* h, const icap_model_desc* desc, int parts, void* stream) {
  return guarded([&] {
    REQUIRE(h && desc, "null argument");
    REQUIRE(parts > 0 && (parts & ~(ICAP_PART_DECODER | ICAP_PART_ENCODER)) == 0, "bad parts");
    const icap_model_desc& o = h->d;
    REQUIRE(desc->kind == o.kind && desc->precision == o.precision && desc->d_model == o.d_model &&
                desc->nhead == o.nhead && desc->dim_ff == o.dim_ff && desc->n_dec_layers == o.n_dec_layers &&
                desc->vocab == o.vocab && desc->pe_len == o.pe_len && desc->vit_dim == o.vit_dim &&
                desc->vit_layers == o.vit_layers && desc->vit_mlp == o.vit_mlp && desc->patch == o.patch &&
                desc->cnn_dim == o.cnn_dim && desc->n_enc_layers == o.n_enc_layers && desc->n_trunk == o.n_trunk,
            "weight update must keep the model's shapes");
    REQUIRE(!(parts & ICAP_PART_DECODER) || desc->dec_layers, "decoder layer pointers missing");
    const hipStream_t s = (hipStream_t)stream;
    h->d = *desc;
    h->repack = true;
    try {
      pack(h, s, parts);
    } catch (...) {
      h->repack = false;
      h->d.dec_layers = nullptr; h->d.vit_layers_w = nullptr; h->d.enc_layers = nullptr; h->d.trunk = nullptr;
      throw;
    }
    h->repack = false;
    h->d.dec_layers = nullptr; h->d.vit_layers_w = nullptr; h->d.enc_layers = nullptr; h->d.trunk = nullptr;
  });
}

int icap_destroy(icap_handle* h) {
  return guarded([&] {
    if (h) {
      (void)hipDeviceSynchronize();
      delete h;
    }
  });
}

int icap_encode_vit(icap_handle* h, const float* images, int B, float* memory, void* stream) {
  return guarded([&] {
    REQUIRE(h && images && memory && B > 0, "bad arguments");
    REQUIRE(h->d.kind == ICAP_KIND_VIT, "handle is not a ViT model");
    encode_vit(h, images, B, memory, (hipStream_t)stream);
  });
}

int icap_encode_vit_features(icap_handle* h, const float* images, int B, float* memory, float* feats, void* stream) {
  return guarded([&] {
    REQUIRE(h && images && memory && feats && B > 0, "bad arguments");
    REQUIRE(h->d.kind == ICAP_KIND_VIT, "handle is not a ViT model");
    encode_vit(h, images, B, memory, (hipStream_t)stream, feats);
  });
}

int icap_encode_grid_tail(icap_handle* h, const float* feats, int B, float* memory, void* stream) {
  return guarded([&] {
    REQUIRE(h && feats && memory && B > 0, "bad arguments");
    REQUIRE(h->d.kind == ICAP_KIND_GRID, "handle is not a Grid model");
    encode_grid_tail(h, feats, B, h->d.grid_tokens, memory, (hipStream_t)stream);
  });
}

int icap_encode_grid_tail_n(icap_handle* h, const float* feats, int B, int N, float* memory, void* stream) {
  return guarded([&] {
    REQUIRE(h && feats && memory && B > 0 && N > 0, "bad arguments");
    REQUIRE(h->d.kind == ICAP_KIND_GRID, "handle is not a Grid model");
    encode_grid_tail(h, feats, B, N, memory, (hipStream_t)stream);
  });
}

int icap_grid_tokens(icap_handle* h, int H, int W, int* tokens) {
  return guarded([&] {
    REQUIRE(h && tokens && H > 0 && W > 0, "bad arguments");
    REQUIRE(h->d.kind == ICAP_KIND_GRID && !h->trunk.empty(), "not a Grid model with its trunk");
    int gh, gw;
    trunk_grid(h, H, W, gh, gw);
    *tokens = gh * gw;
  });
}

int icap_encode_grid_hw(icap_handle* h, const float* images, int B, int H, int W, float* memory, float* feats,
                        void* stream) {
  return guarded([&] {
    REQUIRE(h && images && memory && B > 0, "bad arguments");
    REQUIRE(h->d.kind == ICAP_KIND_GRID, "not a Grid model");
    encode_grid(h, images, B, H, W, memory, (hipStream_t)stream, feats);
  });
}

int icap_encode_grid(icap_handle* h, const float* images, int B, float* memory, void* stream) {
  return guarded([&] {
    REQUIRE(h && images && memory && B > 0, "bad arguments");
    REQUIRE(h->d.kind == ICAP_KIND_GRID, "icap_encode_grid on a non-Grid model");
    encode_grid(h, images, B, 224, 224, memory, (hipStream_t)stream);
  });
}

int icap_encode_grid_features(icap_handle* h, const float* images, int B, float* memory, float* feats, void* stream) {
  return guarded([&] {
    REQUIRE(h && images && memory && feats && B > 0, "bad arguments");
    REQUIRE(h->d.kind == ICAP_KIND_GRID, "not a Grid model");
    encode_grid(h, images, B, 224, 224, memory, (hipStream_t)stream, feats);
  });
}

int icap_encode_grid_train(icap_handle* h, const float* images, int B, const icap_conv_bn_w* bn, float momentum,
                           float* memory, float* feats, void* stream) {
  return guarded([&] {
    REQUIRE(h && images && memory && feats && bn && B > 1, "bad arguments (B >= 2 for batch statistics)");
    REQUIRE(h->d.kind == ICAP_KIND_GRID, "not a Grid model");
    REQUIRE(momentum >= 0.f && momentum <= 1.f, "momentum must be in [0, 1]");
    for (size_t i = 0; i < h->trunk.size(); ++i)
      REQUIRE(bn[i].bn_w && bn[i].bn_b && bn[i].bn_mean && bn[i].bn_var && bn[i].cout == h->trunk[i].cout,
              "bn entries must match the handle's trunk");
    BnTrain bt;
    bt.bn = bn;
    bt.momentum = momentum;
    encode_grid(h, images, B, 224, 224, memory, (hipStream_t)stream, feats, bt);
  });
}

size_t icap_cider_workspace_bytes(long n_ref, int Lr) { return cider_workspace_bytes(n_ref, Lr); }

int icap_cider_d(const int32_t* hyp, int n_hyp, int Lh, int B, const int32_t* refs, int n_ref, int Lr,
                 const int32_t* ref_off, int start_token, int end_token, int pad_token, double* scores,
                 void* workspace, size_t workspace_bytes, int32_t* status, void* stream) {
  return guarded([&] {
    REQUIRE(hyp && refs && ref_off && scores && workspace && status, "bad arguments");
    REQUIRE(Lh <= CIDER_MAX_TOKENS && Lr <= CIDER_MAX_TOKENS, "caption rows longer than 192 tokens");
    HIPCHK(launch_cider(hyp, n_hyp, Lh, B, refs, n_ref, Lr, ref_off, start_token, end_token, pad_token, scores,
                        workspace, workspace_bytes, status, (hipStream_t)stream));
  });
}

int icap_preprocess(const uint8_t* pixels, const int64_t* offsets, const int32_t* geom, int B, int S, int max_rows,
                    uint8_t* tmp, float* out, void* stream) {
  return guarded([&] {
    REQUIRE(pixels && offsets && geom && tmp && out && B > 0 && S > 0 && max_rows > 0, "bad arguments");
    HIPCHK(launch_preprocess(pixels, offsets, geom, B, S, max_rows, tmp, out, (hipStream_t)stream));
  });
}

int icap_decode_greedy(icap_handle* h, const float* memory, int B, int S, int max_len, int start_token,
                       int end_token, int32_t* ids, float* step_logits, void* stream) {
  return guarded([&] {
    REQUIRE(h && memory && ids, "bad arguments");
    decode_loop(h, memory, B, S, max_len, start_token, end_token, ids, step_logits, nullptr, nullptr,
                (hipStream_t)stream);
  });
}

int icap_decode_sample(icap_handle* h, const float* memory, int B, int S, int max_len, int start_token,
                       int end_token, const float* uniforms, int32_t* ids, float* logp, void* stream) {
  return guarded([&] {
    REQUIRE(h && memory && ids && uniforms && logp, "bad arguments");
    decode_loop(h, memory, B, S, max_len, start_token, end_token, ids, nullptr, uniforms, logp,
                (hipStream_t)stream);
  });
}

int icap_decode_sample_dropout(icap_handle* h, const float* memory, int B, int S, int max_len, int start_token,
                               int end_token, const float* uniforms, float p, uint32_t seed, int32_t* ids, float* logp,
                               void* stream) {
  return guarded([&] {
    REQUIRE(h && memory && ids && uniforms && logp, "bad arguments");
    REQUIRE(p >= 0.f && p < 1.f, "dropout p must be in [0, 1)");
    decode_loop(h, memory, B, S, max_len, start_token, end_token, ids, nullptr, uniforms, logp, (hipStream_t)stream,
                p, seed);
  });
}

namespace {
int stop_chunk(int chunk_steps, int B) { return chunk_steps > 0 ? chunk_steps : (B <= 64 ? 4 : 8); }
}  // namespace

int icap_decode_greedy_stop(icap_handle* h, const float* memory, int B, int S, int max_len, int start_token,
                            int end_token, int chunk_steps, int32_t* ids, float* step_logits, int* steps_executed,
                            void* stream) {
  return guarded([&] {
    REQUIRE(h && memory && ids, "bad arguments");
    decode_loop(h, memory, B, S, max_len, start_token, end_token, ids, step_logits, nullptr, nullptr,
                (hipStream_t)stream, 0.f, 0, stop_chunk(chunk_steps, B), steps_executed);
  });
}

int icap_decode_sample_stop(icap_handle* h, const float* memory, int B, int S, int max_len, int start_token,
                            int end_token, const float* uniforms, float p, uint32_t seed, int chunk_steps, int32_t* ids,
                            float* logp, int* steps_executed, void* stream) {
  return guarded([&] {
    REQUIRE(h && memory && ids && uniforms && logp, "bad arguments");
    REQUIRE(p >= 0.f && p < 1.f, "dropout p must be in [0, 1)");
    decode_loop(h, memory, B, S, max_len, start_token, end_token, ids, nullptr, uniforms, logp, (hipStream_t)stream, p,
                seed, stop_chunk(chunk_steps, B), steps_executed);
  });
}

int icap_decode_beam(icap_handle* h, const float* memory, int B, int S, int max_len, int beam_size, int grid_variant,
                     int start_token, int end_token, int32_t* ids, int32_t* lengths, void* stream) {
  return guarded([&] {
    REQUIRE(h && memory && ids && lengths, "bad arguments");
    decode_beam(h, memory, B, S, max_len, beam_size, grid_variant != 0, start_token, end_token, ids, lengths,
                (hipStream_t)stream);
  });
}

int icap_decoder_forward(icap_handle* h, const int32_t* tgt, int B, int T, const float* memory, int S, int causal,
                         const int32_t* key_lengths, float* logits, void* stream) {
  return guarded([&] {
    REQUIRE(h && tgt && memory && logits && B > 0 && T > 0, "bad arguments");
    REQUIRE(T <= h->d.pe_len, "sequence longer than the positional-encoding table");
    REQUIRE(S > 0 && S <= 256, "memory length must be in [1, 256]");
    hipStream_t s = (hipStream_t)stream;
    const int D = h->d.d_model, rows = B * T;
    DecodeBufs b = dec_bufs(h, rows, B, T, S);
    mem_planes(h, memory, b, s);
    const float scale = (float)std::sqrt((double)D);
    HIPCHK(launch_embed(tgt, T, 0, rows, T, 0, h->emb, h->pe, D, scale, b.x, b.a, b.aL, h->ns, s));
    decoder_layers(h, b, B, T, 0, T, causal, S, s, nullptr, 0, key_lengths);
    HeadArgs ha{};
    ha.x = b.x; ha.rows = rows; ha.Dm = D; ha.W = h->fc_w; ha.W4 = head_w4(h); ha.bias = h->fc_b; ha.V = h->d.vocab;
    ha.logits = logits; ha.ld_logits = h->d.vocab;
    h->dws[0].fin.ensure((size_t)rows * 4);  // scratch ids
    ha.ids = h->dws[0].fin.as<int32_t>(); ha.ld_ids = 1; ha.id_col = 0;
    HIPCHK(launch_head(ha, s));
  });
}

int icap_range_check(icap_handle* h, void* stream, int* overflowed) {
  return guarded([&] {
    REQUIRE(h && overflowed, "null handle / output");
    hipStream_t s = (hipStream_t)stream;
    unsigned* w = h->range_word();
    unsigned v = 0;
    HIPCHK(hipMemcpyAsync(&v, w, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (v) HIPCHK(hipMemsetAsync(w, 0, 16, s));
    *overflowed = (v & 1u) ? 1 : 0;
    REQUIRE(!(v & DEC_STEP_GAVE_UP), "internal error: a persistent decode step gave up waiting for a dependency");
  });
}

int icap_set_encoder_cus(icap_handle* h, int cus) {
  return guarded([&] {
    REQUIRE(h && cus >= 0, "null handle / negative CU count");
    h->enc_cus = cus;
  });
}

int icap_set_encoder_attention_cus(icap_handle* h, int cus) {
  return guarded([&] {
    REQUIRE(h && cus >= 0, "null handle / negative CU count");
    h->enc_attn_cus = cus;
  });
}

int icap_set_decode_chains(icap_handle* h, int chains) {
  return guarded([&] {
    REQUIRE(h, "null handle");
    REQUIRE(chains >= 1 && chains <= icap_handle::MAX_BRANCHES, "decode chains must be in [1, 4]");
    h->dec_branches = chains;
    for (DecodeGraph& g : h->dg) g.reset();
  });
}

int icap_set_decode_step(icap_handle* h, int mode) {
  return guarded([&] {
    REQUIRE(h, "null handle");
    REQUIRE(mode >= 0 && mode <= 2, "decode step mode must be 0, 1 or 2");
#ifndef ICAP_TOOLS
    REQUIRE(mode == 0, "decode step modes 1 / 2 (the persistent steps, measured slower) exist in the tools build only");
#endif
    if (h->use_step != (mode == 1) || h->use_xdec != (mode == 2))
      for (DecodeGraph& g : h->dg) g.reset();  // the captured loops follow the mode
    h->use_step = mode == 1;
    h->use_xdec = mode == 2;
  });
}

#ifdef ICAP_TOOLS
// tools build: the persistent decode's per-task stamps (ICAP_DEC_STEP_TRACE=1) -> host (synchronous)
int icap_dec_step_trace_read(icap_handle* h, void* host, size_t bytes) {
  return guarded([&] {
    REQUIRE(h && h->step_trace.p && bytes <= h->step_trace.n, "no trace (ICAP_DEC_STEP_TRACE=1, tools build)");
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(host, h->step_trace.p, bytes, hipMemcpyDeviceToHost));
  });
}
#endif

int icap_set_graphs(icap_handle* h, int enable) {
  return guarded([&] {
    REQUIRE(h, "null handle");
    h->use_graphs = enable != 0;
    for (DecodeGraph& g : h->dg) g.reset();
  });
}

int icap_profile_enable(icap_handle* h, int enable) {
  return guarded([&] {
    REQUIRE(h, "null handle");
    h->prof_on = enable != 0;
    h->prof_every = enable > 1 ? enable : 1;
    h->prof_gate = true;
    h->prof.clear();
    h->ev_used = 0;
  });
}

int icap_profile_read(icap_handle* h, int kernel_class, double* total_ms, long* launches, double* flops,
                      double* bytes) {
  return guarded([&] {
    REQUIRE(h && total_ms && launches && flops && bytes, "bad arguments");
    double t = 0, f = 0, b = 0;
    long n = 0;
    for (const auto& r : h->prof) {
      if (r.cls != kernel_class) continue;
      HIPCHK(hipEventSynchronize(r.b));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, r.a, r.b));
      t += ms;
      f += r.flops;
      b += r.bytes;
      ++n;
    }
    *total_ms = t;
    *launches = n;
    *flops = f;
    *bytes = b;
  });
}

int icap_op_gemm(const uint16_t* A, long lda, long a_lo, int nsplit, const uint16_t* W, const float* bias, void* C,
                 long ldc, long c_lo, int M, int N, int K, int epi, int out, void* stream) {
  return guarded([&] {
    GemmArgs g = gemm_args();
    g.A = A; g.lda = lda; g.a_lo = a_lo; g.nsplit = nsplit;
    g.W = W; g.ldw = K; g.bias = bias;
    g.C = C; g.ldc = ldc; g.c_lo = c_lo;
    g.M = M; g.N = N; g.K = K; g.epi = epi; g.out = out;
    if (nsplit == NS_F16) {  // fp16 A and W, one fp16 output plane
      REQUIRE(N % 256 == 0 && K % 32 == 0 && K >= 128, "fp16 GEMM: N % 256 == 0, K % 32 == 0, K >= 128");
      g.nsplit = 1; g.c_planes = 1; g.f16 = 1;
    }
    HIPCHK(launch_gemm(g, (hipStream_t)stream));
  });
}

int icap_op_gemm_tail_split(const uint16_t* A, long lda, long a_lo, int nsplit, const uint16_t* W, const float* bias,
                            float* C, long ldc, int M, int N, int K, int split_slots, float* ws, int* cnt,
                            void* stream) {
  return guarded([&] {
    REQUIRE(icap_tools_build(), "measured-and-rejected variant: tools build only (-DICAP_TOOLS)");
    REQUIRE(split_slots > 0 && ws && cnt, "split_slots, ws and cnt are required");
    GemmArgs g = gemm_args();
    g.A = A; g.lda = lda; g.a_lo = a_lo; g.nsplit = nsplit;
    g.W = W; g.ldw = K; g.bias = bias;
    g.C = C; g.ldc = ldc;
    g.M = M; g.N = N; g.K = K; g.epi = EPI_NONE; g.out = OUT_F32_RESID;
    g.split_ws = ws; g.split_cnt = cnt; g.split_slots = split_slots;
    HIPCHK(launch_gemm(g, (hipStream_t)stream));
  });
}

int icap_op_layernorm(const float* x, int rows, int D, const float* w, const float* b, float eps, float* out_f32,
                      uint16_t* out_bf, long bf_lo, int nsplit, void* stream) {
  return guarded([&] {
    HIPCHK(launch_layernorm(x, D, rows, D, 0, 0, 0, w, b, eps, out_f32, D, out_bf, D, bf_lo, nsplit,
                            (hipStream_t)stream));
  });
}

int icap_op_pack_i8(const float* x, int rows, int K, int8_t* out, float* scale, void* stream) {
  return guarded([&] { HIPCHK(launch_pack_i8_rows(x, rows, K, out, scale, (hipStream_t)stream)); });
}

int icap_op_layernorm_i8(const float* x, int rows, int D, const float* w, const float* b, float eps, int8_t* out,
                         float* scale, void* stream) {
  return guarded([&] { HIPCHK(launch_layernorm_i8(x, D, rows, D, 0, 0, 0, w, b, eps, out, scale, (hipStream_t)stream)); });
}

int icap_op_gemm_i8(const int8_t* A, const float* a_scale, const int8_t* W, const float* w_scale, const float* bias,
                    void* C, int M, int N, int K, int epi, int out, int hm_n, void* stream) {
  return guarded([&] {
    REQUIRE(out == OUT_F32 || out == OUT_SPLIT, "out must be OUT_F32 or OUT_SPLIT");
    GemmArgs g = gemm_args();
    g.A = (const bf16_t*)A; g.a_scale = a_scale; g.nsplit = 2;
    g.W = (const bf16_t*)W; g.w_scale = w_scale; g.bias = bias;
    g.C = C; g.ldc = N; g.c_lo = (long)M * N; g.hm_n = hm_n;
    g.M = M; g.N = N; g.K = K; g.epi = epi; g.out = out;
    HIPCHK(launch_gemm_i8(g, (hipStream_t)stream));
  });
}

int icap_op_gemm_i8_blocks(const int8_t* A, const float* a_scale, const float* a_kscale, const int8_t* W,
                           const float* w_scale, const float* bias, void* C, float* c_kscale, int M, int N, int K,
                           int epi, int out, void* stream) {
  return guarded([&] {
    REQUIRE(icap_tools_build(), "measured-and-rejected variant: tools build only (-DICAP_TOOLS)");
    REQUIRE(out == OUT_F32 || out == OUT_F32_RESID || out == OUT_I8K, "out must be OUT_F32, OUT_F32_RESID or OUT_I8K");
    REQUIRE((a_scale != nullptr) != (a_kscale != nullptr), "exactly one of a_scale / a_kscale");
    REQUIRE(out != OUT_I8K || c_kscale != nullptr, "OUT_I8K needs c_kscale");
    GemmArgs g = gemm_args();
    g.A = (const bf16_t*)A; g.a_scale = a_scale; g.a_kscale = a_kscale; g.nsplit = 2;
    g.W = (const bf16_t*)W; g.w_scale = w_scale; g.bias = bias;
    g.C = C; g.ldc = N; g.c_kscale = c_kscale;
    g.M = M; g.N = N; g.K = K; g.epi = epi; g.out = out;
    HIPCHK(launch_gemm_i8(g, (hipStream_t)stream));
  });
}

int icap_op_enc_attention(const uint16_t* qkv, long lo, int B, int N, int H, uint16_t* out, long out_lo, int nsplit,
                          void* stream) {
  return guarded([&] {
    HIPCHK(launch_enc_attention(qkv, 3L * H * 64, lo, B, N, H, 0.125f, out, (long)H * 64, out_lo, nsplit,
                                (hipStream_t)stream));
  });
}

int icap_op_enc_attention_hm(const uint16_t* qkv, int B, int N, int H, uint16_t* out, void* stream) {
  return guarded([&] {
    HIPCHK(launch_enc_attention(qkv, 0, 0, B, N, H, 0.125f, out, (long)H * 64, 0, NS_F16, (hipStream_t)stream, 1));
  });
}

size_t icap_decoder_train_workspace(const icap_model_desc* d, int B, int T, int S, float drop_p) {
  if (!d) return 0;
  return TrainWS(*d, B, T, S, nullptr, drop_p).floats * sizeof(float);
}

// What each live training workspace holds: the forward records the call that filled `ws`; the backward must be
// the backward of that call (same decoder, shapes, ids, memory and dropout), else it would differentiate
// activations of another batch.  Host-side (no device read, no sync), keyed by the workspace pointer.
struct TrainRecord {
  const void* emb;  // the decoder's parameter storage (the descriptor struct itself is rebuilt per call)
  const void* fc_w;
  const void* ids;
  const void* memory;
  int B, T, S, end_token;
  float drop_p;
};
static std::mutex g_train_mu;
static std::map<const void*, TrainRecord> g_train_ws;

int icap_decoder_train_forward(const icap_model_desc* d, const int32_t* ids, int B, int T, const float* memory, int S,
                               int end_token, float drop_p, uint32_t drop_seed, float* logp, void* ws, size_t ws_bytes,
                               void* stream) {
  return guarded([&] {
    train_check(d, B, T, S);
    REQUIRE(ids && memory && logp && ws, "null argument");
    REQUIRE(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || (T <= 128 && S <= 256)), "bad dropout p / lengths");
    TrainWS w(*d, B, T, S, (float*)ws, drop_p);
    REQUIRE(ws_bytes >= w.floats * sizeof(float), "workspace too small (icap_decoder_train_workspace)");
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)w.seed, (int)drop_seed, 1, (hipStream_t)stream));
    train_forward(*d, w, ids, memory, end_token, logp, (hipStream_t)stream);
    std::lock_guard<std::mutex> lk(g_train_mu);
    g_train_ws[ws] = TrainRecord{d->emb, d->fc_w, ids, memory, B, T, S, end_token, drop_p};
  });
}

int icap_decoder_train_backward(const icap_model_desc* d, const icap_model_desc* grad, const int32_t* ids, int B, int T,
                                const float* memory, int S, int end_token, float drop_p, const float* dlogp,
                                float* dmemory, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    train_check(d, B, T, S);
    REQUIRE(grad && grad->dec_layers && grad->emb && grad->fc_w && grad->fc_b, "null gradient pointers");
    REQUIRE(ids && memory && dlogp && ws, "null argument");
    {
      std::lock_guard<std::mutex> lk(g_train_mu);
      auto it = g_train_ws.find(ws);
      REQUIRE(it != g_train_ws.end(), "workspace holds no forward (icap_decoder_train_forward first)");
      const TrainRecord& r = it->second;
      REQUIRE(r.B == B && r.T == T && r.S == S && r.end_token == end_token && r.drop_p == drop_p,
              "backward arguments differ from the forward that filled ws (B, T, S, end_token, drop_p)");
      REQUIRE(r.emb == d->emb && r.fc_w == d->fc_w && r.ids == ids && r.memory == memory,
              "backward decoder / ids / memory differ from the forward that filled ws");
    }
    TrainWS w(*d, B, T, S, (float*)ws, drop_p);  // the seed word the forward left in ws
    REQUIRE(ws_bytes >= w.floats * sizeof(float), "workspace too small (icap_decoder_train_workspace)");
    train_backward(*d, *grad, w, ids, memory, end_token, dlogp, dmemory, (hipStream_t)stream);
    std::lock_guard<std::mutex> lk(g_train_mu);
    g_train_ws.erase(ws);
  });
}

int icap_op_residual_layernorm(float* x, int rows, const float* parts, int nparts, long part_stride, const float* bias,
                               const float* w, const float* b, uint16_t* out, long out_lo, float drop_p,
                               const uint32_t* seed, int layer, int pos, int site, void* stream) {
  return guarded([&] {
    DropCfg d{};
    if (drop_p > 0.f) {
      d.seed = seed;
      d.thr = (uint32_t)std::min(4294967295.0, std::floor((double)drop_p * 4294967296.0 + 0.5));
      d.scale = 1.0f / (1.0f - drop_p);
      d.layer = layer;
      d.pos = pos;
    }
    HIPCHK(launch_residual_layernorm(x, rows, 512, parts, nparts, part_stride, bias, w, b, 1e-5f, out, out_lo, 2,
                                     (hipStream_t)stream, d, site));
  });
}

uint32_t icap_drop_hash_host(uint32_t seed, uint32_t site, uint32_t layer, uint32_t row, uint32_t pos, uint32_t idx) {
  return icap_drop_hash(seed, site, layer, row, pos, idx);
}

int icap_op_cross_attn(const uint16_t* qt, long qt_lo, const uint16_t* mem16, int rows, int rows_per_image, int S,
                       uint16_t* out, long out_lo, void* stream) {
  return guarded([&] {
    float* xp = nullptr;
    int* xc = nullptr;
#ifdef ICAP_TOOLS
    // the tools-only key-split forms' partial states and tickets: one workspace per device, allocated only when a
    // knob selects them, tickets zero at rest (the launch that takes a ticket resets it); callers on one device
    // are serialised by the lock for the allocation only - the key-split op entry is a single-caller measurement
    if (rows > 0 && (cross_attn_f16s_on() || cross_attn_f16_splits() == 2)) {
      static std::mutex mu;
      static std::map<int, std::pair<DevBuf, DevBuf>> per_dev;
      int dev = 0;
      HIPCHK(hipGetDevice(&dev));
      std::lock_guard<std::mutex> lk(mu);
      auto& w = per_dev[dev];
      if (w.second.n < (size_t)rows * 4) {
        w.first.ensure(cross_attn_part_floats(rows) * 4);
        w.second.ensure((size_t)rows * 4);
        HIPCHK(hipMemsetAsync(w.second.p, 0, w.second.n, (hipStream_t)stream));
      }
      xp = w.first.as<float>();
      xc = w.second.as<int>();
    }
#endif
    HIPCHK(launch_cross_attn_f16(qt, qt_lo, mem16, rows, rows_per_image, S, 0.125f, out, out_lo,
                                 (hipStream_t)stream, DropCfg{}, nullptr, xp, xc));
  });
}

}  // extern "C"
