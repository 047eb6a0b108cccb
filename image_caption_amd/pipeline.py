"""Batch-pipelined captioning: the encoder of batch i+1 runs while batch i decodes.

The greedy decode of a batch (`_greedy_search`'s loop, vit:296-325) is a chain of small, latency-bound
launches (29 steps x 6 layers x ~11 kernels, replayed from a hipGraph) that leaves most of the chip
idle, while the next batch's encoder is a handful of large MFMA GEMMs that fill it.  Running them on
two streams - the decode on a high-priority stream, so its workgroups take CUs as soon as encoder
blocks retire - overlaps the two phases of consecutive batches.  Every batch still goes through the
exact same kernels, so the captions are bit-identical to `Engine.greedy(Engine.encode(x))` per batch.

Buffer hand-off: each batch's memory tensor is allocated on the encoder stream and marked with
`record_stream(decode stream)`, so the caching allocator does not hand it to a later encode before
the decode that reads it has finished; the decode graph copies it into its own buffer on entry.
"""
from __future__ import annotations

from typing import Callable, Iterable, List, Optional

import torch

from . import _lib
from .engine import Engine


class CaptionPipeline:
    """decode_cus = None (the default): two ordinary streams, the decode one at high priority, and the encodes that
    overlap a decode hold their persistent grids to a CU budget (encoder_cus / attention_cus) so the decode's launches
    find free CUs.  decode_cus = n: the decode stream runs on n CUs and the encoder stream on the others
    (icap_stream_create_cu_mask), so neither phase waits for the other's workgroups to retire before it gets a CU
    (measured slower)."""

    # the encoder CU budget of an encode that overlaps a decode (unmasked streams): round 6, bench sweep of 96-256 CUs
    # (profiles/r06/pipe_tune.txt): 160-192 of 256 CUs leave the decode's small launches free CUs and give the
    # best steps (21.1-21.4 against 23.2 ms with the encoder on every CU; 128 and below starve the encoder)
    OVERLAP_CU_SHARE = 0.625
    # and the persistent encoder attention's: 96 or 128 CUs against the GEMMs' 160 (+1-2 %, 96 ahead in two of three
    # same-box sweeps, 48-64 starve it; profiles/r06/pipe_attn_ab.txt, pipe_attn_sweep.txt)
    OVERLAP_ATTN_CU_SHARE = 0.375

    def __init__(self, engine: Engine, start: int, end: int, max_len: int, decode_priority: int = -1,
                 decode_cus: Optional[int] = None, check_range: bool = False, encoder_cus: Optional[int] = None,
                 attention_cus: Optional[int] = None):
        """check_range: after each run(), raise if the f16 encoder's fp16 range guard fired for any batch
        (Engine.range_overflowed, DESIGN.md §3: those memories must be re-encoded in bf16x2, which the drop-in
        models do by themselves; a direct Engine / pipeline user opts in here).  Costs one stream sync per run.
        encoder_cus (unmasked streams only): the persistent encoder grids' CU budget for the encodes that overlap a
        decode (None = OVERLAP_CU_SHARE of the device's CUs, a multiple of 8 = whole CUs on each XCD, for an f16 ViT
        engine - the budget sizes its persistent encoder grids - and 0 otherwise; 0 = every CU).
        attention_cus: the same for the persistent encoder attention (None = OVERLAP_ATTN_CU_SHARE of the CUs when
        the GEMMs have a budget).  The first batch's encode, which has no decode beside it, runs at the engine's own
        budgets."""
        import ctypes

        self.eng = engine
        self.check_range = bool(check_range)
        self.start, self.end, self.max_len = int(start), int(end), int(max_len)
        dev = engine.device
        self._owned = []
        if decode_cus:
            lib = engine.lib
            ptrs = []
            for comp in (0, 1):
                p = ctypes.c_void_p()
                _lib.check(lib.icap_stream_create_cu_mask(int(decode_cus), comp, 0, ctypes.byref(p)),
                           "icap_stream_create_cu_mask")
                ptrs.append(p.value)
            self._owned = ptrs
            # the persistent encoder GEMMs size their grids to the encoder stream's CUs.  The engine keeps one budget;
            # its CU-masked pipelines form a stack on it (base budget first), so destroying them in any order leaves
            # the budget of the newest live one (or the base) in force
            budgets = engine.__dict__.setdefault("_cu_budgets", [("base", engine.encoder_cus)])
            if len(budgets) == 1:  # no live CU-masked pipeline: the caller may have changed the budget since
                budgets[0] = ("base", engine.encoder_cus)
            budgets.append((id(self), torch.cuda.get_device_properties(dev).multi_processor_count - int(decode_cus)))
            engine.set_encoder_cus(budgets[-1][1])
            self.dec_stream = torch.cuda.ExternalStream(ptrs[0], device=dev)
            self.enc_stream = torch.cuda.ExternalStream(ptrs[1], device=dev)
        else:
            lo, hi = torch.cuda.Stream.priority_range()
            prio = max(min(decode_priority, lo), hi)
            self.enc_stream = torch.cuda.Stream(device=dev, priority=0)
            self.dec_stream = torch.cuda.Stream(device=dev, priority=prio)
        self.post_stream = torch.cuda.Stream(device=dev)  # run()'s post steps, one batch behind the decode
        self.defer_post = True
        self.overlap_cus = self.overlap_attn_cus = 0
        if not decode_cus:
            if encoder_cus is None and not (engine.kind == "vit" and engine.precision == "f16"):
                encoder_cus = 0  # the budget sizes the f16 ViT encoder's persistent grids only
            cus = torch.cuda.get_device_properties(dev).multi_processor_count
            if encoder_cus is None:
                encoder_cus = max(8, int(cus * self.OVERLAP_CU_SHARE) // 8 * 8)
            self.overlap_cus = int(encoder_cus)
            if attention_cus is None:
                attention_cus = max(8, int(cus * self.OVERLAP_ATTN_CU_SHARE) // 8 * 8) if self.overlap_cus else 0
            self.overlap_attn_cus = int(attention_cus)

    def __del__(self):
        if getattr(self, "_owned", []):
            try:  # drop this pipeline's budget; the newest remaining one (or the base) applies again
                budgets = self.eng._cu_budgets
                budgets[:] = [b for b in budgets if b[0] != id(self)]
                self.eng.set_encoder_cus(budgets[-1][1])
            except Exception:
                pass
        for p in getattr(self, "_owned", []):
            try:
                torch.cuda.synchronize(self.eng.device)
                self.eng.lib.icap_stream_destroy(p)
            except Exception:
                pass
        self._owned = []

    def run(self, batches: Iterable[torch.Tensor],
            post: Optional[Callable[[torch.Tensor], object]] = None,
            timing: Optional[list] = None) -> List[object]:
        """Greedy-caption every batch; returns post(ids) per batch (default: the raw int32 ids
        (B, max_len) before the stop rule).  `post(ids)` of batch i runs on its own stream, ordered after batch i's
        decode, once decode i + 1 and encode i + 2 are queued, so a host sync inside it (the stop rule's length)
        waits for batch i's decode while both streams hold work.  timing: a list that
        receives per batch (encode start, encode end, decode start, decode end) timing events, recorded on the
        encoder / decode streams (the two phases of consecutive batches overlap)."""
        eng, E, D = self.eng, self.enc_stream, self.dec_stream
        cur = torch.cuda.current_stream(eng.device)
        it = iter(batches)
        outs: List[object] = []
        first = next(it, None)
        if first is None:
            return outs
        E.wait_stream(cur)  # inputs produced on the caller's stream
        D.wait_stream(cur)

        def mark(stream):
            if timing is None:
                return None
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            return e

        def encode(batch):
            with torch.cuda.stream(E):
                e0 = mark(E)
                m = eng.encode(batch)
                return m, (e0, mark(E))

        mem, enc_ev = encode(first)
        nxt = next(it, None)
        base = (eng.encoder_cus, eng.encoder_attention_cus)
        try:
            self._overlap(outs, mem, enc_ev, nxt, it, post, timing, encode, mark)
        finally:
            if (eng.encoder_cus, eng.encoder_attention_cus) != base:
                eng.set_encoder_cus(base[0])
                eng.set_encoder_attention_cus(base[1])
        cur.wait_stream(D)
        cur.wait_stream(E)
        cur.wait_stream(self.post_stream)
        if self.check_range and eng.range_overflowed():
            raise RuntimeError("fp16 range guard: an f16 encoder activation overflowed in this run; re-encode the "
                               "batches with a bf16x2 engine (Engine(..., precision='bf16x2'))")
        return outs

    def _overlap(self, outs, mem, enc_ev, nxt, it, post, timing, encode, mark):
        """The steady state of run(): decode batch i on D, then encode batch i + 1 on E under the overlap budget, then
        the post step of batch i - 1 on its own stream P.  Round 6: with the post step of batch i on D right after
        its encode was queued, the host sat in that step's sync until decode i ended and only then queued decode
        i + 1 and encode i + 2, so every other batch both streams idled ≈ 0.8 ms (tools/r6_pipe_gaps.py,
        profiles/r06/pipe_gaps.txt); one batch later, behind an event on decode i - 1 alone, the host waits while
        decode i and encode i + 1 are already queued."""
        eng, E, D, P = self.eng, self.enc_stream, self.dec_stream, self.post_stream
        pending = None

        def flush(item):
            ids, done = item
            P.wait_event(done)
            ids.record_stream(P)
            with torch.cuda.stream(P):
                outs.append(post(ids) if post is not None else ids)

        while mem is not None:
            ev = E.record_event()
            D.wait_event(ev)
            mem.record_stream(D)
            with torch.cuda.stream(D):
                d0 = mark(D)
                ids, _ = eng.greedy_raw(mem, self.start, self.end, self.max_len)
                d1 = mark(D)
            if timing is not None:
                timing.append((enc_ev[0], enc_ev[1], d0, d1))
            mem = None
            if nxt is not None:
                target = (self.overlap_cus, self.overlap_attn_cus)
                if any(target) and (eng.encoder_cus, eng.encoder_attention_cus) != target:
                    eng.set_encoder_cus(target[0])
                    eng.set_encoder_attention_cus(target[1])
                mem, enc_ev = encode(nxt)
                nxt = next(it, None)
            if pending is not None:
                flush(pending)
            pending = (ids, D.record_event())
            if not self.defer_post:  # (measurement: the round-6 form, the host waits for this batch's decode now)
                flush(pending)
                pending = None
        if pending is not None:
            flush(pending)
