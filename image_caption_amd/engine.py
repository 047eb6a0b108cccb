"""Host side of the HIP hot path: packs a captioning model's state_dict into a libicap handle
and runs the encoders / decode loops on the current torch stream.

This mirrors the reference's operator surface for the path (models/vit_transformer_model.py):
`encode` = VisionTransformerEncoder.forward (vit:71-100) / GridFeatureEncoder.forward tail
(grid:97-108); `greedy` = the `_greedy_search` loop (vit:306-325) including its batch-global
stop rule; `sample` = SCSTLoss._sample_with_log_probs (scst_loss:202-254) with injected
uniforms; `decoder_forward` = TransformerDecoder.forward (vit:155-182).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Tuple

import torch

from . import _lib
from ._lib import (ConvBnW, DecLayerW, EncLayerW, LnW, MhaW, ModelDesc, VitLayerW, check, stream_ptr)

DEFAULT_PRECISION = "f16"


def _ln(sd, p):
    return LnW(sd[p + ".weight"].data_ptr(), sd[p + ".bias"].data_ptr())


def _mha(sd, p):
    return MhaW(sd[p + ".in_proj_weight"].data_ptr(), sd[p + ".in_proj_bias"].data_ptr(),
                sd[p + ".out_proj.weight"].data_ptr(), sd[p + ".out_proj.bias"].data_ptr())


def _conv_bn(sd, conv, bn, stride):
    w = sd[conv + ".weight"]
    return ConvBnW(w.data_ptr(), sd[bn + ".weight"].data_ptr(), sd[bn + ".bias"].data_ptr(),
                   sd[bn + ".running_mean"].data_ptr(), sd[bn + ".running_var"].data_ptr(),
                   w.shape[0], w.shape[1], w.shape[2], stride)


def trunk_convs(sd, prefix="encoder.cnn."):
    """The ResNet trunk of a GridFeatureEncoder state_dict (cnn = resnet children[:-2]: 0 conv1,
    1 bn1, 4..7 layer1..4) in icap_model_desc order, with the blocks per stage.  None if absent."""
    if prefix + "0.weight" not in sd:
        return None
    convs = [_conv_bn(sd, prefix + "0", prefix + "1", 2)]
    blocks = []
    for st in range(4):
        n = 0
        while f"{prefix}{4 + st}.{n}.conv1.weight" in sd:
            p = f"{prefix}{4 + st}.{n}"
            stride = 2 if (st > 0 and n == 0) else 1
            if n == 0:
                convs.append(_conv_bn(sd, p + ".downsample.0", p + ".downsample.1", stride))
            convs.append(_conv_bn(sd, p + ".conv1", p + ".bn1", 1))
            convs.append(_conv_bn(sd, p + ".conv2", p + ".bn2", stride))
            convs.append(_conv_bn(sd, p + ".conv3", p + ".bn3", 1))
            n += 1
        blocks.append(n)
    return convs, blocks


def apply_stop_rule(ids: torch.Tensor, end_token: int) -> torch.Tensor:
    """Truncate fixed-length greedy output to the reference's length: `_greedy_search` breaks
    after the first step at which every sample's newest token is <end> (vit:321-323)."""
    all_end = (ids[:, 1:] == end_token).all(dim=0)
    if bool(all_end.any()):
        L = int(torch.nonzero(all_end)[0, 0]) + 2
        return ids[:, :L]
    return ids


class Engine:
    """One packed model on one device.  Not thread-safe (a handle per thread)."""

    def __init__(self, state_dict: Dict[str, torch.Tensor], kind: str, config: dict,
                 precision: str = DEFAULT_PRECISION, device: torch.device | str | None = None,
                 decoder_weight_planes: Optional[int] = None):
        self.lib = _lib.load()
        if precision not in _lib.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_lib.PRECISIONS)}")
        device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if device.type != "cuda":
            raise _lib.IcapError("the HIP engine needs a GPU device")
        self.device = device
        self.kind = kind
        self.has_trunk = False
        self.precision = precision
        self.d_model = int(config.get("d_model", 512))
        self.nhead = int(config.get("nhead", 8))
        # decoder GEMM weights as bf16 (1) or bf16 hi/lo (2); None = 2 exactly when some decoder
        # GEMM weight is not bf16-representable (an fp32 checkpoint), so the logits keep the 1e-3 bar.  Fixed at
        # creation: update_weights re-packs into the same layout.
        self.dec_weight_planes = decoder_weight_planes
        desc, keep = self._desc(state_dict)
        handle = ctypes.c_void_p()
        with torch.cuda.device(device):
            check(self.lib.icap_create(ctypes.byref(desc), stream_ptr(device), ctypes.byref(handle)), "icap_create")
        self.handle = handle
        del keep

    def dropout_sampling_ok(self, max_len: int) -> bool:
        """Whether `sample(..., dropout=...)` can run: the train-mode masks live in the fused one-token decode
        blocks (csrc/decode.hip), which serve d_model 512 / 8 heads / dim_feedforward 2048, a parity precision
        (two activation planes: not "bf16") and decode positions below 64 (max_len <= 65)."""
        return (self.precision != "bf16" and self.d_model == 512 and self.nhead == 8 and self.dim_ff == 2048
                and 2 <= max_len <= min(65, self.pe_len))

    def update_weights(self, state_dict: Dict[str, torch.Tensor], decoder: bool = True, encoder: bool = True) -> None:
        """Re-pack the decoder and/or encoder weights of `state_dict` (same shapes) into this handle's
        buffers on the current stream (icap_update_weights): no re-allocation, frozen parts untouched,
        captured decode graphs kept."""
        parts = (_lib.PART_DECODER if decoder else 0) | (_lib.PART_ENCODER if encoder else 0)
        if not parts:
            return
        desc, keep = self._desc(state_dict)
        check(self.lib.icap_update_weights(self.handle, ctypes.byref(desc), parts, stream_ptr(self.device)),
              "icap_update_weights")
        torch.cuda.current_stream(self.device).synchronize()  # the fp32 copies in `keep` must outlive the packing
        del keep

    def _desc(self, state_dict: Dict[str, torch.Tensor]):
        """icap_model_desc over fp32 device copies of `state_dict` (returned with the objects that must
        stay alive until the library has read them)."""
        device, kind = self.device, self.kind
        sd = {k: v.detach().to(device=device, dtype=torch.float32).contiguous()
              for k, v in state_dict.items() if torch.is_floating_point(v)}
        emb = sd["decoder.embedding.weight"]
        self.vocab = emb.shape[0]
        self.pe_len = sd["decoder.pos_encoder.pe"].shape[1]
        n_dec = 0
        while f"decoder.transformer_decoder.layers.{n_dec}.norm1.weight" in sd:
            n_dec += 1
        dec = (DecLayerW * n_dec)()
        for i in range(n_dec):
            p = f"decoder.transformer_decoder.layers.{i}"
            dec[i] = DecLayerW(_mha(sd, p + ".self_attn"), _mha(sd, p + ".multihead_attn"),
                               sd[p + ".linear1.weight"].data_ptr(), sd[p + ".linear1.bias"].data_ptr(),
                               sd[p + ".linear2.weight"].data_ptr(), sd[p + ".linear2.bias"].data_ptr(),
                               _ln(sd, p + ".norm1"), _ln(sd, p + ".norm2"), _ln(sd, p + ".norm3"))
        dim_ff = sd["decoder.transformer_decoder.layers.0.linear1.weight"].shape[0]
        if self.dec_weight_planes is None:
            gemm_w = [v for k, v in sd.items() if k.startswith("decoder.transformer_decoder.")
                      and k.endswith(("in_proj_weight", "out_proj.weight", "linear1.weight", "linear2.weight"))]
            exact = all(torch.equal(w, w.to(torch.bfloat16).float()) for w in gemm_w)
            self.dec_weight_planes = 1 if exact else 2
        if self.dec_weight_planes not in (1, 2):
            raise ValueError("decoder_weight_planes must be 1 (bf16) or 2 (bf16 hi/lo)")
        desc = ModelDesc()
        desc.dec_weight_planes = self.dec_weight_planes
        desc.precision = _lib.PRECISIONS[self.precision]
        desc.d_model, desc.nhead, desc.dim_ff = self.d_model, self.nhead, dim_ff
        self.dim_ff = dim_ff
        desc.n_dec_layers, desc.vocab, desc.pe_len = n_dec, self.vocab, self.pe_len
        desc.emb = emb.data_ptr()
        desc.pe = sd["decoder.pos_encoder.pe"].data_ptr()
        desc.fc_w = sd["decoder.fc_out.weight"].data_ptr()
        desc.fc_b = sd["decoder.fc_out.bias"].data_ptr()
        desc.dec_layers = ctypes.cast(dec, ctypes.POINTER(DecLayerW))
        keep = [dec, sd]
        if kind == "vit":
            P = "encoder.vit."
            conv = sd[P + "conv_proj.weight"]
            n_vit = 0
            while f"{P}encoder.layers.encoder_layer_{n_vit}.ln_1.weight" in sd:
                n_vit += 1
            vl = (VitLayerW * n_vit)()
            for i in range(n_vit):
                L = f"{P}encoder.layers.encoder_layer_{i}"
                vl[i] = VitLayerW(_ln(sd, L + ".ln_1"), _mha(sd, L + ".self_attention"), _ln(sd, L + ".ln_2"),
                                  sd[L + ".mlp.0.weight"].data_ptr(), sd[L + ".mlp.0.bias"].data_ptr(),
                                  sd[L + ".mlp.3.weight"].data_ptr(), sd[L + ".mlp.3.bias"].data_ptr())
            keep.append(vl)
            desc.kind = _lib.KIND_VIT
            desc.vit_dim = conv.shape[0]
            self.vit_dim = int(conv.shape[0])
            desc.vit_heads = conv.shape[0] // 64
            desc.vit_mlp = sd[f"{P}encoder.layers.encoder_layer_0.mlp.0.weight"].shape[0]
            desc.vit_layers = n_vit
            desc.patch = conv.shape[-1]
            desc.image = 224
            desc.cls = sd[P + "class_token"].data_ptr()
            desc.conv_w = conv.data_ptr()
            desc.conv_b = sd[P + "conv_proj.bias"].data_ptr()
            desc.pos = sd[P + "encoder.pos_embedding"].data_ptr()
            desc.vit_ln_w = sd[P + "encoder.ln.weight"].data_ptr()
            desc.vit_ln_b = sd[P + "encoder.ln.bias"].data_ptr()
            desc.vit_layers_w = ctypes.cast(vl, ctypes.POINTER(VitLayerW))
            desc.proj_w = sd["encoder.projection.weight"].data_ptr()
            desc.proj_b = sd["encoder.projection.bias"].data_ptr()
            self.mem_tokens = (224 // desc.patch) ** 2
        elif kind == "grid":
            n_enc = 0
            while f"encoder.transformer_encoder.layers.{n_enc}.norm1.weight" in sd:
                n_enc += 1
            el = (EncLayerW * n_enc)()
            for i in range(n_enc):
                L = f"encoder.transformer_encoder.layers.{i}"
                el[i] = EncLayerW(_mha(sd, L + ".self_attn"), sd[L + ".linear1.weight"].data_ptr(),
                                  sd[L + ".linear1.bias"].data_ptr(), sd[L + ".linear2.weight"].data_ptr(),
                                  sd[L + ".linear2.bias"].data_ptr(), _ln(sd, L + ".norm1"), _ln(sd, L + ".norm2"))
            keep.append(el)
            pw = sd["encoder.projection.weight"]
            desc.kind = _lib.KIND_GRID
            desc.proj_w = pw.data_ptr()
            desc.proj_b = sd["encoder.projection.bias"].data_ptr()
            desc.cnn_dim = pw.shape[1]
            self.cnn_dim = int(pw.shape[1])
            desc.grid_tokens = 49
            desc.n_enc_layers = n_enc
            desc.enc_pe = sd["encoder.pos_encoder.pe"].data_ptr()
            desc.enc_pe_len = int(sd["encoder.pos_encoder.pe"].shape[1])
            self.enc_pe_len = desc.enc_pe_len
            desc.enc_layers = ctypes.cast(el, ctypes.POINTER(EncLayerW))
            trunk = trunk_convs(sd)
            if trunk is not None:
                convs, blocks = trunk
                tw = (ConvBnW * len(convs))(*convs)
                keep.append(tw)
                desc.n_trunk = len(convs)
                desc.trunk_blocks[:] = blocks
                desc.trunk = ctypes.cast(tw, ctypes.POINTER(ConvBnW))
            self.has_trunk = trunk is not None
            self.mem_tokens = 49
        else:
            raise ValueError(f"unknown model kind {kind!r}")
        return desc, keep

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self.lib.icap_destroy(h)
            except Exception:
                pass
            self.handle = None

    def range_overflowed(self) -> bool:
        """fp16 range guard of the f16 encoders (icap_range_check): True when a ViT LayerNorm /
        Q,K,V / GELU output or a Grid trunk activation stored as fp16 since the last check was not finite
        (|v| >= 65520 or NaN), i.e. the
        memory of those encodes is not trustworthy and must be recomputed in bf16x2.  Synchronises the
        engine's current stream; always False for precisions without fp16 activations.  Also the health check of
        the persistent decode: raises IcapError if a decode step gave up waiting for a dependency.""" 
        out = ctypes.c_int(0)
        # raises if a persistent decode step gave up waiting for a dependency (an internal error, never silent)
        check(self.lib.icap_range_check(self.handle, stream_ptr(self.device), ctypes.byref(out)), "icap_range_check")
        return bool(out.value) and self.precision == "f16"

    # ------------------------------------------------------------------ encoders
    def encode(self, images: torch.Tensor) -> torch.Tensor:
        """ViT: images (B,3,224,224) -> memory (B,196,d).  Grid: images (B,3,224,224) through the HIP
        ResNet trunk, or trunk features (B,2048,7,7) through the tail only."""
        x = images.to(device=self.device, dtype=torch.float32).contiguous()
        B = x.shape[0]
        mem = torch.empty(B, self.mem_tokens, self.d_model, device=self.device, dtype=torch.float32)
        if self.kind == "vit":
            if tuple(x.shape[1:]) != (3, 224, 224):
                raise ValueError(f"expected (B,3,224,224) images, got {tuple(x.shape)}")
            check(self.lib.icap_encode_vit(self.handle, x.data_ptr(), B, mem.data_ptr(), stream_ptr(self.device)),
                  "icap_encode_vit")
        elif tuple(x.shape[1:]) == (3, 224, 224):
            if not self.has_trunk:
                raise _lib.IcapError("this Grid engine was built without the encoder.cnn weights")
            check(self.lib.icap_encode_grid(self.handle, x.data_ptr(), B, mem.data_ptr(), stream_ptr(self.device)),
                  "icap_encode_grid")
        elif x.dim() == 4 and x.shape[1] == 3 and self.has_trunk:
            # any other image size on the HIP trunk (grid:86-110): the memory has the trunk grid's h x w tokens
            n = self.grid_tokens(x.shape[2], x.shape[3])
            mem = torch.empty(B, n, self.d_model, device=self.device, dtype=torch.float32)
            check(self.lib.icap_encode_grid_hw(self.handle, x.data_ptr(), B, x.shape[2], x.shape[3], mem.data_ptr(),
                                               None, stream_ptr(self.device)), "icap_encode_grid_hw")
        else:
            if x.dim() != 4 or x.shape[1] != self.cnn_dim:
                raise ValueError(f"expected (B,3,H,W) images or (B,{self.cnn_dim},h,w) trunk features, "
                                 f"got {tuple(x.shape)}")
            n = x.shape[2] * x.shape[3]
            if n > self.enc_pe_len:
                raise ValueError(f"{n} grid tokens exceed the encoder's positional encoding ({self.enc_pe_len})")
            mem = torch.empty(B, n, self.d_model, device=self.device, dtype=torch.float32)
            check(self.lib.icap_encode_grid_tail_n(self.handle, x.data_ptr(), B, n, mem.data_ptr(),
                                                   stream_ptr(self.device)), "icap_encode_grid_tail_n")
        return mem

    def grid_tokens(self, height: int, width: int) -> int:
        """Tokens of the memory of an (height, width) image: the ResNet trunk's output grid h x w."""
        out = ctypes.c_int(0)
        check(self.lib.icap_grid_tokens(self.handle, int(height), int(width), ctypes.byref(out)), "icap_grid_tokens")
        return int(out.value)

    def encode_vit_features(self, images: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """ViT: images (B,3,224,224) -> (memory (B,196,d), trunk output (B,196,vit_dim) = the projection's
        input) in one pass (icap_encode_vit_features)."""
        x = images.to(device=self.device, dtype=torch.float32).contiguous()
        if self.kind != "vit" or tuple(x.shape[1:]) != (3, 224, 224):
            raise ValueError("encode_vit_features needs a ViT engine and (B,3,224,224) images")
        B = x.shape[0]
        mem = torch.empty(B, self.mem_tokens, self.d_model, device=self.device, dtype=torch.float32)
        feats = torch.empty(B, self.mem_tokens, self.vit_dim, device=self.device, dtype=torch.float32)
        check(self.lib.icap_encode_vit_features(self.handle, x.data_ptr(), B, mem.data_ptr(), feats.data_ptr(),
                                                stream_ptr(self.device)), "icap_encode_vit_features")
        return mem, feats

    def encode_grid_features(self, images: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Grid: images (B,3,224,224) -> (memory (B,49,d), trunk features (B,cnn_dim,7,7)) in one pass."""
        x = images.to(device=self.device, dtype=torch.float32).contiguous()
        if self.kind != "grid" or not self.has_trunk or tuple(x.shape[1:]) != (3, 224, 224):
            raise ValueError("encode_grid_features needs a Grid engine with its trunk and (B,3,224,224) images")
        B = x.shape[0]
        mem = torch.empty(B, self.mem_tokens, self.d_model, device=self.device, dtype=torch.float32)
        rows = torch.empty(B, self.mem_tokens, self.cnn_dim, device=self.device, dtype=torch.float32)
        check(self.lib.icap_encode_grid_features(self.handle, x.data_ptr(), B, mem.data_ptr(), rows.data_ptr(),
                                                 stream_ptr(self.device)), "icap_encode_grid_features")
        return mem, rows.permute(0, 2, 1).reshape(B, self.cnn_dim, 7, 7)

    def encode_grid_train(self, images: torch.Tensor, cnn: torch.nn.Module) -> Tuple[torch.Tensor, torch.Tensor]:
        """Grid: the trunk in TRAINING mode (icap_encode_grid_train): every BatchNorm of `cnn` (the
        GridFeatureEncoder.cnn whose weights this engine packed) normalises with the batch statistics and
        updates its running_mean / running_var in place (num_batches_tracked + 1 here), as cnn(images) under
        cnn.train() does.  -> (memory (B,49,d), trunk features (B,cnn_dim,7,7))."""
        x = images.to(device=self.device, dtype=torch.float32).contiguous()
        if self.kind != "grid" or not self.has_trunk or tuple(x.shape[1:]) != (3, 224, 224):
            raise ValueError("encode_grid_train needs a Grid engine with its trunk and (B,3,224,224) images")
        sd = {"cnn." + k: v for k, v in cnn.state_dict(keep_vars=True).items()}
        convs, _ = trunk_convs(sd, prefix="cnn.")
        for v in sd.values():
            if not (v.is_cuda and v.device == x.device and v.dtype in (torch.float32, torch.int64) and v.is_contiguous()):
                raise ValueError("the trunk's parameters and buffers must be contiguous fp32 on the engine's device")
        bns = [m for m in cnn.modules() if isinstance(m, torch.nn.BatchNorm2d)]
        moms = {m.momentum for m in bns}
        if len(moms) != 1 or None in moms or any(not m.track_running_stats or m.eps != 1e-5 for m in bns):
            raise ValueError("the HIP train-mode trunk needs one fixed BatchNorm momentum, eps 1e-5, running stats")
        momentum = moms.pop()
        bn = (ConvBnW * len(convs))(*convs)
        B = x.shape[0]
        mem = torch.empty(B, self.mem_tokens, self.d_model, device=self.device, dtype=torch.float32)
        rows = torch.empty(B, self.mem_tokens, self.cnn_dim, device=self.device, dtype=torch.float32)
        check(self.lib.icap_encode_grid_train(self.handle, x.data_ptr(), B, bn, float(momentum), mem.data_ptr(),
                                              rows.data_ptr(), stream_ptr(self.device)), "icap_encode_grid_train")
        for m in bns:
            m.num_batches_tracked.add_(1)
        return mem, rows.permute(0, 2, 1).reshape(B, self.cnn_dim, 7, 7)

    # ------------------------------------------------------------------ decoders
    def greedy_raw(self, memory: torch.Tensor, start: int, end: int, max_len: int,
                   want_logits: bool = False) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        mem = memory.to(device=self.device, dtype=torch.float32).contiguous()
        B, S = mem.shape[0], mem.shape[1]
        ids = torch.empty(B, max_len, device=self.device, dtype=torch.int32)
        logits = (torch.empty(max_len - 1, B, self.vocab, device=self.device, dtype=torch.float32)
                  if want_logits else None)
        check(self.lib.icap_decode_greedy(self.handle, mem.data_ptr(), B, S, max_len, int(start), int(end),
                                          ids.data_ptr(), _lib.ptr(logits), stream_ptr(self.device)),
              "icap_decode_greedy")
        return ids, logits

    def greedy(self, memory: torch.Tensor, start: int, end: int, max_len: int, stop_early: bool = True,
               chunk: int = 0) -> torch.Tensor:
        """Reference-identical greedy output (int64, stop rule applied).  With the f16 encoder, a direct Engine user
        checks range_overflowed() after encode (the drop-in models do; CaptionPipeline(check_range=True) does).
        stop_early (default): the decode itself ends as `_greedy_search` does (icap_decode_greedy_stop: chunks of
        `chunk` steps, 0 = auto), so a batch that ends after k steps costs about k steps, not max_len - 1;
        last_decode_steps then holds the steps executed.  The call returns after the decode's next-to-last chunk."""
        if not stop_early:
            ids, _ = self.greedy_raw(memory, start, end, max_len)
            return apply_stop_rule(ids.long(), end)
        ids, _ = self.greedy_stop_raw(memory, start, end, max_len, chunk=chunk)
        return apply_stop_rule(ids.long(), end)

    def greedy_stop_raw(self, memory: torch.Tensor, start: int, end: int, max_len: int, chunk: int = 0,
                        want_logits: bool = False) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """Stop-aware greedy decode (icap_decode_greedy_stop): ids (B,max_len) int32 whose columns after the executed
        steps are end, optional step logits (steps not executed: unwritten); last_decode_steps = steps executed."""
        mem = memory.to(device=self.device, dtype=torch.float32).contiguous()
        B, S = mem.shape[0], mem.shape[1]
        ids = torch.empty(B, max_len, device=self.device, dtype=torch.int32)
        logits = (torch.empty(max_len - 1, B, self.vocab, device=self.device, dtype=torch.float32)
                  if want_logits else None)
        steps = ctypes.c_int(0)
        check(self.lib.icap_decode_greedy_stop(self.handle, mem.data_ptr(), B, S, max_len, int(start), int(end),
                                               int(chunk), ids.data_ptr(), _lib.ptr(logits), ctypes.byref(steps),
                                               stream_ptr(self.device)), "icap_decode_greedy_stop")
        self.last_decode_steps = steps.value
        return ids, logits

    def sample(self, memory: torch.Tensor, uniforms: torch.Tensor, start: int, end: int,
               max_len: int, dropout: Optional[Tuple[float, int]] = None,
               stop_early: bool = False, chunk: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
        """Sampled ids (B,max_len) int32 and per-step log-probs (B,max_len-1).
        dropout = (p, seed): train-mode sampling (icap_decode_sample_dropout).  stop_early: the decode ends once every
        row has emitted end, as the reference's loop (icap_decode_sample_stop; columns not computed: ids = end,
        log-probs = 0; partially blocking - off by default, so a sampler and a greedy baseline on two streams
        still overlap)."""
        mem = memory.to(device=self.device, dtype=torch.float32).contiguous()
        B, S = mem.shape[0], mem.shape[1]
        u = uniforms.to(device=self.device, dtype=torch.float32).contiguous()
        if tuple(u.shape) != (max_len - 1, B):
            raise ValueError("uniforms must be (max_len-1, B)")
        ids = torch.empty(B, max_len, device=self.device, dtype=torch.int32)
        logp = torch.empty(B, max_len - 1, device=self.device, dtype=torch.float32)
        if stop_early:
            p, seed = dropout if dropout is not None else (0.0, 0)
            steps = ctypes.c_int(0)
            check(self.lib.icap_decode_sample_stop(self.handle, mem.data_ptr(), B, S, max_len, int(start), int(end),
                                                   u.data_ptr(), float(p), int(seed) & 0xFFFFFFFF, int(chunk),
                                                   ids.data_ptr(), logp.data_ptr(), ctypes.byref(steps),
                                                   stream_ptr(self.device)), "icap_decode_sample_stop")
            self.last_decode_steps = steps.value
            return ids, logp
        if dropout is not None and dropout[0] > 0:
            check(self.lib.icap_decode_sample_dropout(self.handle, mem.data_ptr(), B, S, max_len, int(start),
                                                      int(end), u.data_ptr(), float(dropout[0]),
                                                      int(dropout[1]) & 0xFFFFFFFF, ids.data_ptr(), logp.data_ptr(),
                                                      stream_ptr(self.device)), "icap_decode_sample_dropout")
            return ids, logp
        check(self.lib.icap_decode_sample(self.handle, mem.data_ptr(), B, S, max_len, int(start), int(end),
                                          u.data_ptr(), ids.data_ptr(), logp.data_ptr(), stream_ptr(self.device)),
              "icap_decode_sample")
        return ids, logp

    def beam(self, memory: torch.Tensor, start: int, end: int, max_len: int, beam_size: int,
             grid_variant: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
        """Beam search for every image at once: ids (B,max_len) int32 zero-padded, lengths (B) int32."""
        mem = memory.to(device=self.device, dtype=torch.float32).contiguous()
        B, S = mem.shape[0], mem.shape[1]
        ids = torch.empty(B, max_len, device=self.device, dtype=torch.int32)
        lens = torch.empty(B, device=self.device, dtype=torch.int32)
        check(self.lib.icap_decode_beam(self.handle, mem.data_ptr(), B, S, max_len, int(beam_size),
                                        int(bool(grid_variant)), int(start), int(end), ids.data_ptr(),
                                        lens.data_ptr(), stream_ptr(self.device)), "icap_decode_beam")
        return ids, lens

    def decoder_forward(self, tgt: torch.Tensor, memory: torch.Tensor, causal: bool,
                        key_lengths: torch.Tensor | None = None) -> torch.Tensor:
        """Full-prefix decoder: tgt (B,T) -> logits (B,T,V).  key_lengths (B,): tgt_key_padding_mask as
        lengths (keys j >= key_lengths[b] masked), None = no padding mask."""
        t = tgt.to(device=self.device, dtype=torch.int32).contiguous()
        mem = memory.to(device=self.device, dtype=torch.float32).contiguous()
        B, T = t.shape
        kl = None
        if key_lengths is not None:
            kl = key_lengths.to(device=self.device, dtype=torch.int32).contiguous()
            if kl.shape != (B,):
                raise ValueError(f"key_lengths must have shape ({B},), got {tuple(kl.shape)}")
        logits = torch.empty(B, T, self.vocab, device=self.device, dtype=torch.float32)
        check(self.lib.icap_decoder_forward(self.handle, t.data_ptr(), B, T, mem.data_ptr(), mem.shape[1],
                                            int(bool(causal)), None if kl is None else kl.data_ptr(),
                                            logits.data_ptr(), stream_ptr(self.device)),
              "icap_decoder_forward")
        return logits

    def set_decode_chains(self, chains: int) -> None:
        """Independent decode chains per batch (1..4, default 1 since round 4, used from 80 rows per chain)."""
        check(self.lib.icap_set_decode_chains(self.handle, int(chains)), "icap_set_decode_chains")

    def set_decode_step(self, mode) -> None:
        """Decode loop form (icap_set_decode_step): 0 / False = one launch per fused block, 1 / True = the persistent
        task step (decstep.hip), 2 = the group-persistent step (xdec.hip)."""
        check(self.lib.icap_set_decode_step(self.handle, int(mode)), "icap_set_decode_step")

    def set_encoder_cus(self, cus: int) -> None:
        """Persistent encoder GEMM grids for an encoder stream restricted to `cus` CUs (0 = every CU).  The value
        belongs to the handle: a user that changes it restores the previous one (encoder_cus) when done."""
        check(self.lib.icap_set_encoder_cus(self.handle, int(cus)), "icap_set_encoder_cus")
        self._encoder_cus = int(cus)

    @property
    def encoder_cus(self) -> int:
        return getattr(self, "_encoder_cus", 0)

    def set_encoder_attention_cus(self, cus: int) -> None:
        """The persistent encoder attention's own CU budget (0 = follow set_encoder_cus, the default)."""
        check(self.lib.icap_set_encoder_attention_cus(self.handle, int(cus)), "icap_set_encoder_attention_cus")
        self._encoder_attention_cus = int(cus)

    @property
    def encoder_attention_cus(self) -> int:
        return getattr(self, "_encoder_attention_cus", 0)

    def set_graphs(self, enable: bool) -> None:
        """hipGraph replay of the decode loop (default on)."""
        check(self.lib.icap_set_graphs(self.handle, int(bool(enable))), "icap_set_graphs")

    # ------------------------------------------------------------------ live kernel timing
    def profile(self, enable: bool, every: int = 1) -> None:
        """HIP-event timing of the hot-kernel launches (icap_profile_enable); every = N >= 2 brackets only ViT encoder
        layers 0, N, 2N, ... (each event pair costs the stream ~3 us; the layers share their shapes)."""
        check(self.lib.icap_profile_enable(self.handle, max(1, int(every)) if enable else 0), "icap_profile_enable")

    def profile_read(self, kernel_class: int) -> dict:
        """Device time of every recorded launch of one kernel class (HIP events on the launch
        stream), with the launches' algorithmic flops and operand bytes."""
        t, n = ctypes.c_double(), ctypes.c_long()
        f, b = ctypes.c_double(), ctypes.c_double()
        check(self.lib.icap_profile_read(self.handle, kernel_class, ctypes.byref(t), ctypes.byref(n),
                                         ctypes.byref(f), ctypes.byref(b)), "icap_profile_read")
        return {"kernel": _lib.PROF_NAMES[kernel_class], "ms": t.value, "launches": n.value,
                "flops": f.value, "bytes": b.value}
