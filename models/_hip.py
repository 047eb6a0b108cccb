"""Routing between the nn.Module surface and the HIP engine (image_caption_amd.engine).

Rule: a call takes the HIP path when its tensors are on a GPU, autograd is off,
the module is in eval mode and the call is expressible by the engine (generate/greedy; decoder
forward with no mask or the causal mask and no padding masks; encoder forward).  Training calls
(grad on, dropout on, padding masks) keep the module's own PyTorch semantics - those are not the
hot path.  On a GPU the HIP path has no silent fallback: if libicap.so cannot load, the call
raises.  `backend="torch"` in the model config forces the PyTorch modules, `backend="hip"`
forbids them.
"""
from __future__ import annotations

import copy
import weakref
from typing import Optional

import torch

BACKENDS = ("auto", "hip", "torch")


def attach_owner(child: torch.nn.Module, owner: torch.nn.Module) -> None:
    object.__setattr__(child, "_hip_owner", weakref.ref(owner))


def owner_of(child: torch.nn.Module) -> Optional[torch.nn.Module]:
    ref = getattr(child, "_hip_owner", None)
    return ref() if ref is not None else None


def is_causal_mask(mask: torch.Tensor, T: int) -> bool:
    """Same test as torch's _detect_is_causal_mask: equal to the standard causal float mask."""
    if mask is None or mask.dim() != 2 or mask.shape != (T, T):
        return False
    ref = torch.triu(torch.full((T, T), float("-inf"), device=mask.device, dtype=mask.dtype), diagonal=1)
    if mask.dtype == torch.bool:
        return bool(torch.equal(mask, ref.isinf()))
    return bool(torch.equal(mask, ref))


class HipRouted:
    """Mixin for the top-level captioning models (engine cache + routing decision)."""

    _hip_kind = "vit"

    def _hip_setup(self, backend: str = "auto", precision: str = "f16") -> None:
        if backend not in BACKENDS:
            raise ValueError(f"backend must be one of {BACKENDS}")
        object.__setattr__(self, "hip_backend", backend)
        object.__setattr__(self, "hip_precision", precision)
        object.__setattr__(self, "_hip_cache", None)
        object.__setattr__(self, "_hip_cache_fb", None)

    def use_hip(self, x: torch.Tensor, *, grad_ok: bool = False) -> bool:
        if self.hip_backend == "torch":
            return False
        on_gpu = x.is_cuda
        if self.hip_backend == "hip" and not on_gpu:
            raise RuntimeError("backend='hip' needs GPU tensors")
        if not on_gpu:
            return False
        if self.training or (torch.is_grad_enabled() and not grad_ok):
            if self.hip_backend == "hip":
                raise RuntimeError("backend='hip' serves eval-mode, no-grad calls only")
            return False
        return True

    def __deepcopy__(self, memo):
        """A copy never shares (or copies) the packed engine - its device handle belongs to this module - and
        its encoder / decoder route to the COPY's engine, built on first use from the copy's weights."""
        new = self.__class__.__new__(self.__class__)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            object.__setattr__(new, k, None if k in ("_hip_cache", "_hip_cache_fb") else copy.deepcopy(v, memo))
        for name in ("encoder", "decoder"):
            child = getattr(new, name, None)
            if isinstance(child, torch.nn.Module):
                attach_owner(child, new)
        return new

    def hip_engine(self, device: torch.device, precision: Optional[str] = None):
        """The packed engine of this module's current weights.  After an optimizer step only the parts
        whose tensors changed (decoder / encoder, by data_ptr and version) are re-packed in place
        (icap_update_weights): frozen encoder weights are not re-packed and the captured decode graphs
        survive, so an SCST training loop keeps replaying them.  `precision` other than the model's
        hip_precision: a second engine kept beside it (the f16 range guard's bf16x2 re-encode)."""
        if precision is None or precision == self.hip_precision:
            return self._engine_slot("_hip_cache", self.hip_precision, device)
        return self._engine_slot("_hip_cache_fb", precision, device)

    def checked_encode(self, images: torch.Tensor):
        """(engine, memory) of `images`; if the f16 encoder's range guard fired (an fp16 activation overflowed,
        DESIGN.md §3) the memory is recomputed by a bf16x2 engine of the same weights, which is returned
        instead.  Synchronises the stream once (f16 only)."""
        eng = self.hip_engine(images.device)
        mem = eng.encode(images)
        if eng.range_overflowed():
            eng = self.hip_engine(images.device, precision="bf16x2")
            mem = eng.encode(images)
        return eng, mem

    def _engine_slot(self, attr: str, precision: str, device: torch.device):
        from image_caption_amd.engine import Engine

        sd = self.state_dict()

        def key(prefix_dec: bool):
            # num_batches_tracked feeds no computation (fixed momentum); the HIP train-mode trunk bumps it
            # each SCST step while it updates the running statistics and the handle's BatchNorm fold itself
            return tuple((k, t.data_ptr(), t._version) for k, t in sd.items()
                         if torch.is_tensor(t) and k.startswith("decoder.") == prefix_dec
                         and not k.endswith("num_batches_tracked"))

        base = (str(device), precision)
        kd, ke = key(True), key(False)
        cache = getattr(self, attr, None)
        if cache is not None and cache[0] == base:
            eng = cache[3]
            dec, enc = cache[1] != kd, cache[2] != ke
            if dec or enc:
                eng.update_weights(sd, decoder=dec, encoder=enc)
                object.__setattr__(self, attr, (base, kd, ke, eng))
            return eng
        eng = Engine(sd, self._hip_kind, {"d_model": self.d_model}, precision=precision, device=device)
        object.__setattr__(self, attr, (base, kd, ke, eng))
        return eng
