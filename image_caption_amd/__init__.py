"""MI355X-native image-captioning hot path (ViT/Grid encoder + Transformer decoder + greedy /
sampled token loop) behind the reference's nn.Module surface.

Layout: csrc/ (HIP kernels + C-ABI runtime -> libicap.so), _lib.py (ctypes binding of
include/icap.h), engine.py (weight packing + launch API), weights.py (seeded synthetic weights),
parallel.py (data-parallel sharding + RCCL all-gather of token ids), cider.py (CIDEr-D on ids).
"""
__version__ = "0.1.0"
