"""ctypes binding of libicap.so (include/icap.h).  Fails loudly when the library is missing.

`import torch` happens first so that the HIP runtime torch ships (soname libamdhip64.so.7) is
the one libicap.so binds to: one runtime per process, shared device pointers and streams.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int, c_long, c_void_p
from pathlib import Path

import torch  # noqa: F401  (load torch's HIP runtime before libicap)

LIB_PATH = Path(__file__).resolve().parent / "libicap.so"
ABI_VERSION = 3

KIND_VIT, KIND_GRID = 0, 1
PREC_BF16, PREC_BF16X2, PREC_I8X2, PREC_F16 = 1, 2, 3, 4
PRECISIONS = {"bf16": PREC_BF16, "bf16x2": PREC_BF16X2, "i8x2": PREC_I8X2, "f16": PREC_F16}
PROF_GEMM_128, PROF_GEMM_64, PROF_ENC_ATTN, PROF_CROSS_ATTN, PROF_GEMM_WAVE, PROF_GEMM_256 = 0, 1, 2, 3, 4, 5
PROF_GEMM_I8 = 6
PROF_DEC_FUSED = 7
PROF_GEMM_F16P = 8
PART_DECODER, PART_ENCODER = 1, 2
PROF_NAMES = {PROF_GEMM_128: "gemm_bf16_kernel<128,128,64,64>", PROF_GEMM_64: "gemm_bf16_kernel<64,64,32,32>",
              PROF_ENC_ATTN: "enc_attention_kernel", PROF_CROSS_ATTN: "cross_attn_mfma_kernel",
              PROF_GEMM_WAVE: "gemm_dec_kernel", PROF_GEMM_256: "gemm_256_kernel", PROF_GEMM_I8: "gemm_i8_kernel",
              PROF_DEC_FUSED: "dec_sa_kernel/dec_ffn_kernel", PROF_GEMM_F16P: "gemm_f16p_kernel"}


class LnW(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("b", c_void_p)]


class MhaW(ctypes.Structure):
    _fields_ = [("in_w", c_void_p), ("in_b", c_void_p), ("out_w", c_void_p), ("out_b", c_void_p)]


class VitLayerW(ctypes.Structure):
    _fields_ = [("ln_1", LnW), ("attn", MhaW), ("ln_2", LnW), ("mlp0_w", c_void_p), ("mlp0_b", c_void_p),
                ("mlp3_w", c_void_p), ("mlp3_b", c_void_p)]


class EncLayerW(ctypes.Structure):
    _fields_ = [("attn", MhaW), ("lin1_w", c_void_p), ("lin1_b", c_void_p), ("lin2_w", c_void_p),
                ("lin2_b", c_void_p), ("norm1", LnW), ("norm2", LnW)]


class DecLayerW(ctypes.Structure):
    _fields_ = [("self_attn", MhaW), ("cross_attn", MhaW), ("lin1_w", c_void_p), ("lin1_b", c_void_p),
                ("lin2_w", c_void_p), ("lin2_b", c_void_p), ("norm1", LnW), ("norm2", LnW), ("norm3", LnW)]


class ConvBnW(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("bn_w", c_void_p), ("bn_b", c_void_p), ("bn_mean", c_void_p),
                ("bn_var", c_void_p), ("cout", c_int), ("cin", c_int), ("k", c_int), ("stride", c_int)]


class ModelDesc(ctypes.Structure):
    _fields_ = [
        ("kind", c_int), ("precision", c_int),
        ("d_model", c_int), ("nhead", c_int), ("dim_ff", c_int), ("n_dec_layers", c_int), ("vocab", c_int),
        ("pe_len", c_int),
        ("emb", c_void_p), ("pe", c_void_p), ("fc_w", c_void_p), ("fc_b", c_void_p),
        ("dec_layers", POINTER(DecLayerW)),
        ("vit_dim", c_int), ("vit_heads", c_int), ("vit_mlp", c_int), ("vit_layers", c_int), ("patch", c_int),
        ("image", c_int),
        ("cls", c_void_p), ("conv_w", c_void_p), ("conv_b", c_void_p), ("pos", c_void_p), ("vit_ln_w", c_void_p),
        ("vit_ln_b", c_void_p),
        ("vit_layers_w", POINTER(VitLayerW)),
        ("proj_w", c_void_p), ("proj_b", c_void_p),
        ("cnn_dim", c_int), ("grid_tokens", c_int), ("n_enc_layers", c_int),
        ("enc_pe", c_void_p),
        ("enc_layers", POINTER(EncLayerW)),
        ("n_trunk", c_int), ("trunk_blocks", c_int * 4),
        ("trunk", POINTER(ConvBnW)),
        ("dec_weight_planes", c_int),
        ("enc_pe_len", c_int),
    ]


# name -> (restype, argtypes); exactly the entry points include/icap.h declares
SIGNATURES = {
    "icap_abi_version": (c_int, []),
    "icap_tools_build": (c_int, []),
    "icap_last_error": (ctypes.c_char_p, []),
    "icap_create": (c_int, [POINTER(ModelDesc), c_void_p, POINTER(c_void_p)]),
    "icap_destroy": (c_int, [c_void_p]),
    "icap_update_weights": (c_int, [c_void_p, POINTER(ModelDesc), c_int, c_void_p]),
    "icap_encode_vit": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "icap_encode_vit_features": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "icap_encode_grid_tail": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "icap_encode_grid": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "icap_encode_grid_features": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "icap_encode_grid_train": (c_int, [c_void_p, c_void_p, c_int, POINTER(ConvBnW), ctypes.c_float, c_void_p,
                                       c_void_p, c_void_p]),
    "icap_cider_workspace_bytes": (ctypes.c_size_t, [c_long, c_int]),
    "icap_cider_d": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int,
                             c_void_p, c_void_p, ctypes.c_size_t, c_void_p, c_void_p]),
    "icap_preprocess": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "icap_decode_greedy": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                   c_void_p]),
    "icap_decode_sample": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
    "icap_op_residual_layernorm": (c_int, [c_void_p, c_int, c_void_p, c_int, c_long, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_long, c_float, c_void_p, c_int, c_int, c_int, c_void_p]),
    "icap_drop_hash_host": (ctypes.c_uint32, [ctypes.c_uint32] * 6),
    "icap_decode_sample_dropout": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_float,
                                           ctypes.c_uint32, c_void_p, c_void_p, c_void_p]),
    "icap_decode_greedy_stop": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                        c_void_p, POINTER(c_int), c_void_p]),
    "icap_decode_sample_stop": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_float,
                                        ctypes.c_uint32, c_int, c_void_p, c_void_p, POINTER(c_int), c_void_p]),
    "icap_decode_beam": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                 c_void_p, c_void_p]),
    "icap_decoder_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                     c_void_p, c_void_p]),
    "icap_set_graphs": (c_int, [c_void_p, c_int]),
    "icap_set_decode_chains": (c_int, [c_void_p, c_int]),
    "icap_set_decode_step": (c_int, [c_void_p, c_int]),
    "icap_set_encoder_cus": (c_int, [c_void_p, c_int]),
    "icap_set_encoder_attention_cus": (c_int, [c_void_p, c_int]),
    "icap_range_check": (c_int, [c_void_p, c_void_p, POINTER(c_int)]),
    "icap_grid_tokens": (c_int, [c_void_p, c_int, c_int, POINTER(c_int)]),
    "icap_encode_grid_hw": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "icap_encode_grid_tail_n": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "icap_profile_enable": (c_int, [c_void_p, c_int]),
    "icap_profile_read": (c_int, [c_void_p, c_int, POINTER(ctypes.c_double), POINTER(c_long),
                                  POINTER(ctypes.c_double), POINTER(ctypes.c_double)]),
    "icap_op_gemm": (c_int, [c_void_p, c_long, c_long, c_int, c_void_p, c_void_p, c_void_p, c_long, c_long, c_int,
                             c_int, c_int, c_int, c_int, c_void_p]),
    "icap_op_layernorm": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_long,
                                  c_int, c_void_p]),
    "icap_op_enc_attention": (c_int, [c_void_p, c_long, c_int, c_int, c_int, c_void_p, c_long, c_int, c_void_p]),
    "icap_op_enc_attention_hm": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "icap_op_cross_attn": (c_int, [c_void_p, c_long, c_void_p, c_int, c_int, c_int, c_void_p, c_long, c_void_p]),
    "icap_decoder_train_workspace": (ctypes.c_size_t, [c_void_p, c_int, c_int, c_int, c_float]),
    "icap_decoder_train_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_float,
                                           ctypes.c_uint32, c_void_p, c_void_p, ctypes.c_size_t, c_void_p]),
    "icap_decoder_train_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int,
                                            c_float, c_void_p, c_void_p, c_void_p, ctypes.c_size_t, c_void_p]),
    "icap_stream_create_cu_mask": (c_int, [c_int, c_int, c_int, POINTER(c_void_p)]),
    "icap_stream_destroy": (c_int, [c_void_p]),
    "icap_op_pack_i8": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "icap_op_layernorm_i8": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                     c_void_p]),
    "icap_op_gemm_i8": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                c_int, c_int, c_void_p]),
    "icap_op_gemm_tail_split": (c_int, [c_void_p, c_long, c_long, c_int, c_void_p, c_void_p, c_void_p, c_long, c_int,
                                        c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "icap_op_gemm_i8_blocks": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_int, c_int, c_int, c_int, c_int, c_void_p]),
}

_LIB = None


class IcapError(RuntimeError):
    pass


def load(path: os.PathLike | None = None) -> ctypes.CDLL:
    """Load libicap.so (once).  Raises if it is missing: there is no fallback."""
    global _LIB
    if _LIB is not None:
        return _LIB
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise IcapError(f"{p} is missing: build it with `python -m image_caption_amd.build` "
                        "(the HIP path has no CPU fallback)")
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.icap_abi_version() != ABI_VERSION:
        raise IcapError(f"libicap ABI {lib.icap_abi_version()} != expected {ABI_VERSION}")
    _LIB = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _LIB.icap_last_error().decode(errors="replace") if _LIB else "?"
        raise IcapError(f"{what} failed: {msg}")


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()
