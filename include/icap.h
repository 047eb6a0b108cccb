/*
 * icap.h — C ABI of the MI355X-native image-captioning hot path (libicap.so).
 *
 * The reference (wonder-dream/image_caption) is pure PyTorch; its "plugin API" for this path is
 * the nn.Module surface of models/{vit,grid}_transformer_model.py.  These entry points are what
 * that surface binds through ctypes (image_caption_amd/_lib.py); each one cites the reference
 * function it replaces.  Conventions:
 *   - plain pointers and sizes only; every tensor pointer is caller-owned DEVICE memory
 *     (row-major, contiguous); `stream` is a hipStream_t (may be NULL = legacy stream);
 *   - the library owns only packed weights and its workspace;
 *   - every call returns 0 on success, non-zero on error, with icap_last_error() describing it;
 *     no C++ exception crosses the ABI; calls are asynchronous on `stream`;
 *   - a handle is not thread-safe.
 */
#ifndef ICAP_H_
#define ICAP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ICAP_ABI_VERSION 3

#define ICAP_KIND_VIT 0   /* ViTTransformerCaptioning  (models/vit_transformer_model.py:185)  */
#define ICAP_KIND_GRID 1  /* GridTransformerCaptioning (models/grid_transformer_model.py:161) */

#define ICAP_PREC_BF16 1   /* bf16 operands, fp32 accumulate                                  */
#define ICAP_PREC_BF16X2 2 /* activations as hi+lo bf16 pairs (~16 mantissa bits), fp32 acc  */
#define ICAP_PREC_I8X2 3   /* bf16x2, except the LayerNorm-fed ViT GEMMs (QKV, MLP-1, projection):
                              both operands as two int8 slices (16-bit fixed point per row), int32 acc */
#define ICAP_PREC_F16 4    /* ViT encoder on single fp16 planes (11-bit significand, fp16 MFMA, fp32 acc);
                              decoder as bf16x2 */

typedef struct icap_handle icap_handle;

/* Parameter pointers are device fp32 tensors with the reference state_dict shapes. */
typedef struct { const float *w, *b; } icap_ln_w;                                 /* nn.LayerNorm */
typedef struct { const float *in_w, *in_b, *out_w, *out_b; } icap_mha_w;         /* nn.MultiheadAttention */

typedef struct { /* torchvision EncoderBlock: encoder.vit.encoder.layers.encoder_layer_{i} */
  icap_ln_w ln_1;
  icap_mha_w attn;
  icap_ln_w ln_2;
  const float *mlp0_w, *mlp0_b, *mlp3_w, *mlp3_b;
} icap_vit_layer_w;

typedef struct { /* nn.TransformerEncoderLayer (post-LN, ReLU): encoder.transformer_encoder.layers.{i} */
  icap_mha_w attn;
  const float *lin1_w, *lin1_b, *lin2_w, *lin2_b;
  icap_ln_w norm1, norm2;
} icap_enc_layer_w;

typedef struct { /* nn.TransformerDecoderLayer (post-LN, ReLU): decoder.transformer_decoder.layers.{i} */
  icap_mha_w self_attn, cross_attn;
  const float *lin1_w, *lin1_b, *lin2_w, *lin2_b;
  icap_ln_w norm1, norm2, norm3;
} icap_dec_layer_w;

typedef struct { /* Conv2d(bias=False) + eval BatchNorm2d of the torchvision ResNet-101 trunk */
  const float* w;                                  /* (cout, cin, k, k)                            */
  const float *bn_w, *bn_b, *bn_mean, *bn_var;     /* (cout) each; eps 1e-5                         */
  int cout, cin, k, stride;                        /* padding = k / 2                               */
} icap_conv_bn_w;

typedef struct {
  int kind, precision;
  /* decoder (TransformerDecoder, vit:103-182) */
  int d_model, nhead, dim_ff, n_dec_layers, vocab, pe_len;
  const float *emb, *pe, *fc_w, *fc_b;
  const icap_dec_layer_w* dec_layers;
  /* ViT-B/16 trunk + projection (VisionTransformerEncoder, vit:36-100) */
  int vit_dim, vit_heads, vit_mlp, vit_layers, patch, image;
  const float *cls, *conv_w, *conv_b, *pos, *vit_ln_w, *vit_ln_b;
  const icap_vit_layer_w* vit_layers_w;
  /* encoder.projection: Linear(768->d) for ViT, Conv2d(2048->d, 1x1) for Grid */
  const float *proj_w, *proj_b;
  /* Grid tail (GridFeatureEncoder after self.cnn, grid:97-108) */
  int cnn_dim, grid_tokens, n_enc_layers;
  const float* enc_pe;
  const icap_enc_layer_w* enc_layers;
  /* Grid ResNet-101 trunk (GridFeatureEncoder.cnn = resnet101 children[:-2], grid:51), optional
   * (n_trunk = 0: only icap_encode_grid_tail is available).  Order: stem conv1+bn1 (7x7/2), then
   * for each stage s and bottleneck block j: [downsample.0+.1 when j == 0], conv1+bn1 (1x1),
   * conv2+bn2 (3x3, the stage stride on j == 0), conv3+bn3 (1x1); trunk_blocks = blocks per stage. */
  int n_trunk, trunk_blocks[4];
  const icap_conv_bn_w* trunk;
  /* decoder GEMM weight planes: 0 or 1 = bf16 (exact for bf16-representable weights), 2 = bf16 hi/lo
   * (hi = bf16(W), lo = bf16(W - hi): 16 significand bits, for fp32 checkpoints whose weights are not
   * bf16-exact; every decoder product adds W_lo . X_hi - since round 5 inside the fused decode blocks too, whose
   * fragment images then carry the lo planes; the teacher-forced / padded forms and the bf16 mode keep the unfused
   * GEMMs - DESIGN.md §3) */
  int dec_weight_planes;
  /* rows of enc_pe (the Grid encoder's PositionalEncoding table, max_len 100 in grid:74); 0 = grid_tokens */
  int enc_pe_len;
} icap_model_desc;

int icap_abi_version(void);
/* 1 when the library was built with -DICAP_TOOLS (measurement knobs read from the environment and
 * the measured-and-rejected kernel variants compiled in), 0 for the product build. */
int icap_tools_build(void);
const char* icap_last_error(void);

/* Packs the model's weights (bf16 GEMM operands + fp32 small params) into handle-owned memory.
 * Replaces: build_model(...) + load_state_dict(...) + .to(device)
 * (models/vit_transformer_model.py:423-444, scripts/inference_vit_transformer.py:50-52). */
int icap_create(const icap_model_desc* desc, void* stream, icap_handle** out);
int icap_destroy(icap_handle* h);

/* Re-packs the weights of the selected parts from `desc` (same shapes as at icap_create) into the
 * handle's existing buffers, in stream order: training loops (SCST) refresh the packed model after an
 * optimizer step without re-packing frozen parts, re-allocating, or losing the captured decode graphs.
 * parts: ICAP_PART_DECODER (the TransformerDecoder) and/or ICAP_PART_ENCODER (everything else). */
#define ICAP_PART_DECODER 1
#define ICAP_PART_ENCODER 2
int icap_update_weights(icap_handle* h, const icap_model_desc* desc, int parts, void* stream);

/* images (B,3,224,224) fp32 normalised -> memory (B,196,d_model) fp32.
 * Replaces: VisionTransformerEncoder.forward, models/vit_transformer_model.py:71-100. */
int icap_encode_vit(icap_handle* h, const float* images, int B, float* memory, void* stream);
/* The same, also writing the frozen trunk's output feats (B,196,vit_dim) fp32 = the encoder.projection
 * input (vit:88-100: the final LayerNorm of the patch tokens): the SCST step applies the trainable
 * projection in PyTorch so its gradient flows (the ViT itself is frozen, vit:64). */
int icap_encode_vit_features(icap_handle* h, const float* images, int B, float* memory, float* feats, void* stream);

/* ResNet trunk features (B,cnn_dim,7,7) fp32 -> memory (B,49,d_model) fp32.
 * Replaces: GridFeatureEncoder.forward after self.cnn, models/grid_transformer_model.py:97-108. */
int icap_encode_grid_tail(icap_handle* h, const float* feats, int B, float* memory, void* stream);

/* images (B,3,224,224) fp32 normalised -> memory (B,49,d_model) fp32: the ResNet-101 trunk as
 * MFMA GEMMs over NHWC activation planes (BatchNorm folded into the epilogue), then the tail.
 * Replaces: GridFeatureEncoder.forward, models/grid_transformer_model.py:86-108 (self.cnn included). */
int icap_encode_grid(icap_handle* h, const float* images, int B, float* memory, void* stream);
/* As icap_encode_grid, and also the trunk output itself: feats (B, 49, cnn_dim) fp32 =
 * self.cnn(images).flatten(2).permute(0, 2, 1) (grid:94, :100-101), the values the tail consumes. */
int icap_encode_grid_features(icap_handle* h, const float* images, int B, float* memory, float* feats, void* stream);
/* As icap_encode_grid_features with the trunk in TRAINING mode, as the reference's SCST step runs it
 * (model.train() then model.encoder(images), utils/scst_loss.py:161, :213; GridFeatureEncoder.forward,
 * grid:86-95): every BatchNorm2d normalises with the batch statistics of these B images (biased variance)
 * and updates its running statistics in place, bn_mean = (1 - momentum) bn_mean + momentum mean,
 * bn_var likewise with the unbiased variance (torch.nn.BatchNorm2d.forward in training mode; the caller
 * increments num_batches_tracked).  bn: n_trunk entries in the desc's order (only bn_w, bn_b, bn_mean,
 * bn_var are read; bn_mean / bn_var are written); the convolution weights are the handle's.  B <= 256. */
/* Any image size (reference: GridFeatureEncoder.forward, grid:86-110, takes whatever grid the trunk returns):
 * images (B,3,H,W) -> memory (B, N, d_model), N = the trunk's output grid h x w (icap_grid_tokens), at most the
 * encoder positional-encoding table's rows (PositionalEncoding(max_len=100), grid:74).  feats: optional trunk
 * output (B, N, cnn_dim) fp32 or NULL. */
int icap_grid_tokens(icap_handle* h, int H, int W, int* tokens);
int icap_encode_grid_hw(icap_handle* h, const float* images, int B, int H, int W, float* memory, float* feats,
                        void* stream);
/* The tail over trunk features (B, cnn_dim, N) of any grid (N tokens, row-major h x w). */
int icap_encode_grid_tail_n(icap_handle* h, const float* feats, int B, int N, float* memory, void* stream);
int icap_encode_grid_train(icap_handle* h, const float* images, int B, const icap_conv_bn_w* bn, float momentum,
                           float* memory, float* feats, void* stream);

/* CIDEr-D rewards on the GPU over token-id rows (pycocoevalcap CiderScorer: n = 1..4, tf-idf with
 * the document frequency over THIS call's reference sets, clipped cosine, Gaussian length penalty,
 * sigma 6, x10).  hyp (n_hyp, Lh) int32: hypothesis k scores against image k % B (n_hyp = H * B lets
 * several hypothesis sets - SCST sample and greedy - share one df pass); refs (n_ref, Lr) int32, image
 * i's references are rows ref_off[i] .. ref_off[i+1] (ref_off: B+1 int32).  Rows are raw ids:
 * <start>/<pad> are dropped and a row ends at its first <end>.  Lh, Lr <= 192.  scores (n_hyp) fp64.
 * workspace >= icap_cider_workspace_bytes(n_ref, Lr) device bytes; status (1 int32, device) is set
 * non-zero when an image's reference set exceeds 4096 distinct n-grams (scores then invalid).
 * Replaces: CiderRewardCalculator.compute_reward -> Cider().compute_score, utils/scst_loss.py:20-54,
 * called twice per SCST step (:179-180). */
size_t icap_cider_workspace_bytes(long n_ref, int Lr);
int icap_cider_d(const int32_t* hyp, int n_hyp, int Lh, int B, const int32_t* refs, int n_ref, int Lr,
                 const int32_t* ref_off, int start_token, int end_token, int pad_token, double* scores,
                 void* workspace, size_t workspace_bytes, int32_t* status, void* stream);

/* Eval preprocessing on the GPU, bit-identical to the reference's torchvision-on-PIL transforms:
 * decoded RGB uint8 images (HWC, any size; image b at pixels + offsets[b]) -> out (B,3,S,S) fp32
 * normalised with the ImageNet mean/std.  geom (B x 8 int32: in_h, in_w, resized h, resized w,
 * crop top, crop left, first source row, source row count) selects Resize(256)+CenterCrop(S) or
 * Resize((S,S)); tmp holds B x max_rows x S x 4 bytes.  Model-independent (no handle).
 * Replaces: the transforms.Compose of scripts/inference_vit_transformer.py:75-80 /
 * scripts/inference_grid_transformer.py:43-47 (utils/deepfashion_dataset.py:223-228 for eval). */
int icap_preprocess(const uint8_t* pixels, const int64_t* offsets, const int32_t* geom, int B, int S, int max_rows,
                    uint8_t* tmp, float* out, void* stream);

/* Greedy decode of max_len-1 steps with a KV cache: ids (B,max_len) int32, column 0 = start.
 * step_logits (max_len-1,B,vocab) fp32 is optional (NULL to skip).  The reference's batch-global
 * stop rule (break when every latest token == end) is applied by the caller on the returned ids.
 * Replaces: _greedy_search loop, models/vit_transformer_model.py:306-325 (grid:237-249). */
int icap_decode_greedy(icap_handle* h, const float* memory, int B, int S, int max_len, int start_token,
                       int end_token, int32_t* ids, float* step_logits, void* stream);

/* Stop-aware greedy decode (round 6): the same decode, ending as the reference's loop does - after the first step at
 * which every latest token == end (models/vit_transformer_model.py:321-323, grid:248-249) - instead of running all
 * max_len-1 steps.  The steps run as captured graphs of chunk_steps steps (<= 0: 4 for B <= 64, else 8) that end in
 * a stop test; the host checks chunk c-2's test before launching chunk c, so at most one chunk past the stop runs
 * and the call returns once the second-to-last launched chunk has finished (a partially blocking call).  ids columns
 * after the executed steps are end (the stop rule's result is the reference's sequence); step_logits of steps not
 * executed are left untouched.  steps_executed (host int, optional) = decode steps run.
 * Replaces: _greedy_search's early break (vit:321-323) for the drop-in generate (scripts/inference_vit_transformer.py
 * :88,108-114 calls it per image with max_len 50). */
int icap_decode_greedy_stop(icap_handle* h, const float* memory, int B, int S, int max_len, int start_token,
                            int end_token, int chunk_steps, int32_t* ids, float* step_logits, int* steps_executed,
                            void* stream);
/* The sampled decode with the reference's stop (break once every row has emitted end, scst_loss.py:246-249), in the
 * chunked form above; p > 0: train-mode dropout (as icap_decode_sample_dropout); log-probs of steps not executed are 0.
 * Replaces: SCSTLoss._sample_with_log_probs's early break (utils/scst_loss.py:246-249). */
int icap_decode_sample_stop(icap_handle* h, const float* memory, int B, int S, int max_len, int start_token,
                            int end_token, const float* uniforms, float p, uint32_t seed, int chunk_steps, int32_t* ids,
                            float* logp, int* steps_executed, void* stream);

/* Batched beam search, beam_size K in [1, 15]: every image runs the reference's per-image beam
 * search (log-softmax scores, top-K over beam x vocab, finished beams collected and pruned so the
 * live beam count shrinks); grid_variant != 0 selects the Grid model's stop tests (completed >= live
 * beams, or no live beam) instead of the ViT's (every live beam ended).  ids (B,max_len) int32 =
 * the chosen sequence (start token first) zero-padded, lengths (B) int32 its token count.
 * Replaces: _beam_search, models/vit_transformer_model.py:327-420 (grid:253-322), run for all
 * images at once as B*K rows of the KV-cached decoder. */
int icap_decode_beam(icap_handle* h, const float* memory, int B, int S, int max_len, int beam_size, int grid_variant,
                     int start_token, int end_token, int32_t* ids, int32_t* lengths, void* stream);

/* Sampled decode with injected uniforms (max_len-1,B) in [0,1): ids (B,max_len) int32 and
 * log-probs (B,max_len-1) fp32, zeroed after a sample has emitted end (masked_fill semantics).
 * Replaces: SCSTLoss._sample_with_log_probs, utils/scst_loss.py:202-254 (torch.multinomial ->
 * inverse CDF on the injected uniforms). */
int icap_decode_sample(icap_handle* h, const float* memory, int B, int S, int max_len, int start_token,
                       int end_token, const float* uniforms, int32_t* ids, float* logp, void* stream);
/* The same in train mode: TransformerDecoder's dropout (p: nn.Dropout of the positional encoding and of
 * every TransformerDecoderLayer) active, as the reference samples after model.train() (scst_loss.py:161).
 * Masks are a counter-based hash of (seed, site, layer, image row, position, index) (common.h
 * icap_drop_hash; oracle/dropout.py restates it): the mask of a position does not depend on the step, so
 * icap_decoder_train_forward / _backward with the same (p, seed) differentiate exactly the distribution
 * sampled from.  Needs a parity precision and max_len <= 65. */
/* The decode loops' residual LayerNorm (d_model 512): x = LN(x + drop(sum of nparts slabs + bias)) in place,
 * bf16 hi/lo planes of x -> out; drop_p > 0: the train-mode mask of (seed[0] device word, site, layer, row,
 * pos, column). */
int icap_op_residual_layernorm(float* x, int rows, const float* parts, int nparts, long part_stride, const float* bias,
                               const float* w, const float* b, uint16_t* out, long out_lo, float drop_p,
                               const uint32_t* seed, int layer, int pos, int site, void* stream);
/* The dropout mask hash itself (host side, no device work): keep <=> hash >= round(p 2^32). */
uint32_t icap_drop_hash_host(uint32_t seed, uint32_t site, uint32_t layer, uint32_t row, uint32_t pos, uint32_t idx);
int icap_decode_sample_dropout(icap_handle* h, const float* memory, int B, int S, int max_len, int start_token,
                               int end_token, const float* uniforms, float p, uint32_t seed, int32_t* ids, float* logp,
                               void* stream);

/* Full-prefix decoder forward: tgt (B,T) int32 -> logits (B,T,vocab) fp32, causal or unmasked.
 * key_lengths (B int32, device, optional): tgt_key_padding_mask as lengths - keys j >= key_lengths[b]
 * are masked in the self-attention (NULL = no padding mask).
 * Replaces: TransformerDecoder.forward, models/vit_transformer_model.py:155-182 (causal=0 is the
 * scripts/inference.py:79 call without tgt_mask); with key_lengths, the teacher-forced forward
 * ViTTransformerCaptioning.forward vit:216-255 (lengths) / grid:185-207 (lengths - 1). */
int icap_decoder_forward(icap_handle* h, const int32_t* tgt, int B, int T, const float* memory, int S,
                         int causal, const int32_t* key_lengths, float* logits, void* stream);

/* Enable (1, default) / disable (0) hipGraph capture of the decode loop: the first decode call
 * with a new (B, S, max_len, mode) runs eagerly, the next captures ~80 kernels x (max_len-1)
 * steps into one graph that later calls replay (kernel timing via icap_profile_* is recorded on
 * the eager calls only). */
int icap_set_graphs(icap_handle* h, int enable);

/* fp16 range guard of ICAP_PREC_F16.  The reference encoder computes in fp32
 * (models/vit_transformer_model.py:71-100); the f16 precision stores LayerNorm outputs, Q/K/V and the GELU
 * output as fp16 (max 65504).  Those kernels set a sticky device word when a value they store is not finite
 * in fp16 (an overflow, or a non-finite residual row that an earlier overflow turned into); this call
 * synchronises `stream`, returns the word in *overflowed (0/1) and clears it.  On 1 the memory of the encodes
 * since the last check is not trustworthy: re-encode with a 16-bit-significand precision (bf16x2). */
int icap_range_check(icap_handle* h, void* stream, int* overflowed);

/* Decode loop form: 0 (default) = one launch per fused block; 1 = one persistent launch per decode
 * step running every decoder layer as dependency-ordered tasks (decstep.hip); 2 = one group-persistent launch per
 * step (xdec.hip: 8 row groups x 32 workgroups, products split by output columns, eval mode, <= 256 rows, a device
 * with >= 256 CUs).  1 and 2 apply where the shapes allow (d_model 512, 8 heads, dim_ff 2048, max_len <= 65, two
 * activation planes, bf16 decoder weights), else the loop falls back to 0.  Same results to rounding (sums in
 * another order). */
int icap_set_decode_step(icap_handle* h, int mode);

/* Encoder CU budget (batch pipelining, image_caption_amd/pipeline.py): the persistent encoder GEMMs (and attention)
 * launch at most `cus` workgroups - the CUs of the CU-masked stream the encoder runs on while the previous batch decodes
 * on the others, or (unmasked streams, the pipeline's default) the CUs the encoder may hold so that the decode's
 * launches find free ones (0 = one per CU of the device, the default).  Results are unchanged. */
int icap_set_encoder_cus(icap_handle* h, int cus);

/* The persistent encoder attention's own CU budget (0 = follow icap_set_encoder_cus, the default).  Round 6: an encode
 * overlapping a decode on unmasked streams runs its GEMMs on 160 and its attention on 96 of 256 CUs (the attention's
 * 16-wave workgroups at a 160-CU grid delay the decode more than they gain; profiles/r06/pipe_attn_ab.txt).  Results
 * are unchanged. */
int icap_set_encoder_attention_cus(icap_handle* h, int cus);

/* Number of independent decode chains a batch is split into (1..4, default 1 since round 4; used from 80 rows per
 * chain): the chains are parallel branches of the captured decode graph (DESIGN.md §4 "Decode, round 4"). */
int icap_set_decode_chains(icap_handle* h, int chains);

/* ---- live kernel timing (bench.py roofline) ----
 * Launch classes recorded by icap_profile_* (eager launches only: kernels inside a replayed decode
 * graph are not event-bracketed; bench.py times the decode phase as a whole instead). */
#define ICAP_PROF_GEMM_128 0   /* gemm_bf16_kernel<128,128,64,64>: trunk convolutions of that tile class  */
#define ICAP_PROF_GEMM_64 1    /* gemm_bf16_kernel<64,64,32,32>: small GEMMs (trunk layer1, N <= 128)    */
#define ICAP_PROF_ENC_ATTN 2   /* encoder self-attention: enc_attention_pers_kernel (f16, N <= 240) /
                                  enc_attention_full_kernel / enc_attention_pipe_kernel / enc_attention_kernel */
#define ICAP_PROF_CROSS_ATTN 3 /* decoder cross-attention: cross_attn_f16_kernel (f16 memory plane) /
                                  cross_attn_mfma_kernel (bf16 planes)                                     */
#define ICAP_PROF_GEMM_WAVE 4  /* gemm_dec_kernel / chain_dec_kernel (decode-step GEMMs)                   */
#define ICAP_PROF_GEMM_256 5   /* gemm_256_kernel: encoder GEMMs (128x256 or 256x256 tiles; fp16 residual ones) */
#define ICAP_PROF_GEMM_I8 6    /* gemm_i8_kernel: int8 two-slice encoder GEMMs (ICAP_PREC_I8X2)            */
#define ICAP_PROF_DEC_FUSED 7  /* dec_sa_kernel / dec_ffn_kernel (fused decode-step blocks, eager launches)   */
#define ICAP_PROF_GEMM_F16P 8  /* gemm_f16p_kernel: persistent fp16 encoder GEMMs (ViT QKV, MLP-1)          */
/* Enable (1) / disable (0) HIP-event bracketing of every hot-kernel launch; clears records.  enable = N >= 2: inside
 * the ViT encoder's layer loop only layers 0, N, 2N, ... are bracketed (every other launch as with 1): each timing
 * event pair costs the stream about 3 us of command-processor time, so bracketing all 60 encoder-layer launches of
 * a step adds ~0.4 ms to it (tools/r6_gap.py) - the layers share their shapes, so a sample measures the same kernels. */
int icap_profile_enable(icap_handle* h, int enable);
/* Sum over recorded launches of one class: device ms, launch count, algorithmic flops and bytes
 * (flops count one activation plane; bytes are the operand bytes the launches must read). */
int icap_profile_read(icap_handle* h, int kernel_class, double* total_ms, long* launches, double* flops,
                      double* bytes);

/* ---- op-level entry points (kernel parity tests) ---- */
/* C = epi(A·W^T + bias); A = nsplit bf16 planes (plane stride a_lo); W (N,K) bf16.
 * epi: 0 none, 1 GELU(erf), 2 ReLU.  out: 0 fp32, 1 bf16, 2 split bf16 planes, 3 fp32 +=.
 * nsplit = -1: A, W and the out = 2 plane are fp16 (ICAP_PREC_F16; N % 256 == 0, K >= 128).
 * icap_op_layernorm / icap_op_enc_attention take nsplit = -1 for one fp16 plane the same way. */
int icap_op_gemm(const uint16_t* A, long lda, long a_lo, int nsplit, const uint16_t* W, const float* bias,
                 void* C, long ldc, long c_lo, int M, int N, int K, int epi, int out, void* stream);
int icap_op_layernorm(const float* x, int rows, int D, const float* w, const float* b, float eps,
                      float* out_f32, uint16_t* out_bf, long bf_lo, int nsplit, void* stream);
/* A stream whose kernels run only on n_cus of the device's CUs (8 per 32-CU block, i.e. spread over
   the XCDs), or on the other CUs when complement != 0 (image_caption_amd/pipeline.py: encoder and
   decoder of consecutive batches side by side).  Destroy with icap_stream_destroy. */
int icap_stream_create_cu_mask(int n_cus, int complement, int priority, void** out);
int icap_stream_destroy(void* stream);
/* int8 two-slice operands (ICAP_PREC_I8X2): fp32 rows -> row images out[r*2K + (k/64)*128 + j*64 + k%64]
   (slice j = 0, 1) with v = scale[r] (256 x1 + x2), 16-bit fixed point relative to the row maximum
   (pack: the rows as given; layernorm_i8: their LayerNorm, then the same quantisation). K % 64 == 0. */
int icap_op_pack_i8(const float* x, int rows, int K, int8_t* out, float* scale, void* stream);
int icap_op_layernorm_i8(const float* x, int rows, int D, const float* w, const float* b, float eps, int8_t* out,
                         float* scale, void* stream);
/* C = epi(dequant(A) dequant(W)^T + bias) on the int8 two-slice GEMM (N % 256 == 0, K % 64 == 0):
   out 0 = fp32 (M,N); out 2 = bf16 hi/lo planes [2][M][N], head-major when hm_n > 0 (the encoder's
   QKV form, element (m, n) at ((m / hm_n * N/64 + n / 64) * hm_n + m % hm_n) * 64 + n % 64). */
int icap_op_gemm_i8(const int8_t* A, const float* a_scale, const int8_t* W, const float* w_scale, const float* bias,
                    void* C, int M, int N, int K, int epi, int out, int hm_n, void* stream);
/* The residual encoder GEMM (C += A.W^T + bias, fp32 C; the out-projection / MLP-2 products of the ViT
 * and Grid encoder layers) with its tail split: per XCD, the tiles of the last partial round of
 * split_slots block slots run as two K halves.  ws: 8 * split_slots * 2 * 128 * 256 floats, cnt:
 * 8 * split_slots ints, zero on entry and on return. */
int icap_op_gemm_tail_split(const uint16_t* A, long lda, long a_lo, int nsplit, const uint16_t* W, const float* bias,
                            float* C, long ldc, int M, int N, int K, int split_slots, float* ws, int* cnt,
                            void* stream);
/* Block-scaled int8 two-slice GEMM (the ViT MLP-2 pair in ICAP_PREC_I8X2; replaces the same
 * nn.Linear products as icap_op_gemm_i8).  A as [M][K/64][2][64] row images with EITHER a_scale[M]
 * (one scale per row) OR a_kscale[M][K/128] (one per row and 128-deep k block); out = 0 (fp32 C[M][N]),
 * 3 (fp32 C += result: residual) or 5 (C as block-scaled int8 row images [M][N/64][2][64], scales to
 * c_kscale[M][N/128]).  N % 128 == 0, K % 64 == 0 (K % 128 == 0 with a_kscale). */
int icap_op_gemm_i8_blocks(const int8_t* A, const float* a_scale, const float* a_kscale, const int8_t* W,
                           const float* w_scale, const float* bias, void* C, float* c_kscale, int M, int N, int K,
                           int epi, int out, void* stream);
/* ---- decoder training pass (SCST's teacher-forced log-prob recompute and its backward) ----
 * Replaces the autograd graph the reference builds while sampling (SCSTLoss._sample_with_log_probs,
 * utils/scst_loss.py:210-254: decoder forward + log_softmax + gather + masked_fill) and its backward
 * (loss.backward(), scripts/train_vit_transformer_scst_optimized.py:261), for the TransformerDecoder
 * (vit:103-182) as torch.autograd.Function (image_caption_amd/train.py).  drop_p > 0: train mode, the
 * dropout masks of icap_decode_sample_dropout under drop_seed (the forward stores the seed in ws; the
 * backward of the same call takes the same drop_p); drop_p = 0: eval mode.
 * `d` holds the decoder's CURRENT fp32 parameters (only the decoder fields are read); ids (B, T+1) int32:
 * inputs ids[:, :T], targets ids[:, 1:]; memory (B, S, d_model) fp32; logp (B, T) = log p(target) with
 * the steps after a row's first end_token zeroed.  The forward keeps its activations in ws (bytes from
 * icap_decoder_train_workspace), which the backward of the same call reads: dlogp (B, T) -> gradients of
 * every decoder parameter written (not accumulated) to the pointers of `grad` (same layout as `d`) and
 * dmemory (B, S, d_model) (may be NULL).  fp32 products (fp32 MFMA).  The forward records its call per
 * ws; a backward whose parameter (emb, fc_w) / ids / memory pointers, B, T, S, end_token or drop_p
 * differ from that record, or on a ws no forward filled, returns non-zero (icap_last_error says which). */
size_t icap_decoder_train_workspace(const icap_model_desc* d, int B, int T, int S, float drop_p);
int icap_decoder_train_forward(const icap_model_desc* d, const int32_t* ids, int B, int T, const float* memory, int S,
                               int end_token, float drop_p, uint32_t drop_seed, float* logp, void* ws, size_t ws_bytes,
                               void* stream);
int icap_decoder_train_backward(const icap_model_desc* d, const icap_model_desc* grad, const int32_t* ids, int B, int T,
                                const float* memory, int S, int end_token, float drop_p, const float* dlogp,
                                float* dmemory, void* ws, size_t ws_bytes, void* stream);

/* qkv planes (B*N, 3*H*64) -> out planes (B*N, H*64), non-causal softmax(QK^T/8)V. */
int icap_op_enc_attention(const uint16_t* qkv, long lo, int B, int N, int H, uint16_t* out, long out_lo,
                          int nsplit, void* stream);
/* The f16 ViT encoder's attention on the head-major fp16 qkv the QKV GEMM writes ([B][q|k|v][H][N][64], GemmArgs::hm_n)
 * -> out fp16 (B*N, H*64); N in (64, 256] (replaces the self-attention of torchvision's EncoderBlock,
 * models/vit_transformer_model.py:71-100 through VisionTransformer.encoder). */
int icap_op_enc_attention_hm(const uint16_t* qkv, int B, int N, int H, uint16_t* out, void* stream);
/* Decoder cross-attention, key-absorbed (the decode loops' form): q~ (rows, 8, 512) as bf16 hi/lo planes
 * (plane stride qt_lo), memory (rows / rows_per_image, S, 512) as one fp16 plane; row r attends to image
 * r / rows_per_image: out[r][h] = softmax_s(q~[r][h] . mem[s] / 8) . mem -> (rows, 8, 512) bf16 hi/lo
 * planes (plane stride out_lo).  The value projection is applied by the caller. */
int icap_op_cross_attn(const uint16_t* qt, long qt_lo, const uint16_t* mem16, int rows, int rows_per_image, int S,
                       uint16_t* out, long out_lo, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ICAP_H_ */
