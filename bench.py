"""Headline benchmark: captions/s of the ViT-B/16 + 6-layer decoder greedy path (224x224,
max_len=30) on N MI355X, data-parallel over images (BASELINE.json `metric`, configs[1] at N=1,
configs[3] shape at N=8 with 256 images per GPU).

A step = one pass of the hot path over one batch of synthetic images already resident in HBM:
ViT encoder -> 29 KV-cached greedy decode steps -> (N>1) one RCCL all-gather of the int32 ids ->
the reference's batch-global stop rule.  Launch as
  python bench.py [--gpus 1 --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
Rank 0 prints ONE JSON line.  `roofline` is the dominant kernel's algorithmic rate measured
with HIP events around each of its launches inside the timed region; its `traffic` is the HBM-side
bytes per launch of that kernel from the committed rocprofv3 PMC summary (tools/pmc_bench.sh:
FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction) when one exists for it; `cpu_baseline` times
the CPU oracle (fp32 restatement of the reference algorithm, full-prefix recompute) on the host.
`--model grid` measures config 3 (ResNet-101 trunk as HIP MFMA GEMMs over NHWC planes, then the
HIP encoder tail and decode loop; `--torch-trunk` runs the trunk through PyTorch/MIOpen fp32 instead); `--mode scst` measures config 5's reward step
(encode once, HIP sample on injected uniforms + HIP greedy baseline from the same memory, all-gather
of both id sets, CIDEr-D over the GLOBAL batch on rank 0); `--mode beam`
measures the batched beam search (§8(f)1: encode + icap_decode_beam, every image at once).  None of
these is the headline line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from image_caption_amd import _lib, parallel  # noqa: E402
from image_caption_amd import weights as W  # noqa: E402
from image_caption_amd.engine import Engine, apply_stop_rule  # noqa: E402

METRIC = "captions/sec (224×224, max_len=30, greedy) at 1/2/4/8 MI355X vs CPU ref"
PEAK_BF16_TFLOPS = 2500.0  # dense bf16 MFMA, MI355X_MICROARCH.md chip table
PEAK_I8_TOPS = 5000.0      # dense i8 MFMA (2x bf16 per clock: 16x16x64 i8 = cycles of 16x16x32 bf16), same table
PEAK_HBM_GBS = 8000.0
# HBM-side bytes per launch from rocprofv3 PMC passes over the default bench of each greedy workload
# (tools/pmc.sh; the ViT line since the pipelined default: MODELS=vit PMC_ARGS="--steps 10 --warmup 3", the budgeted
# persistent GEMMs fetch more per launch than on every CU; "vit_sequential" = the --sequential line's summary); the
# round-2 summary is the fallback for the ViT line
TRAFFIC_JSON = {"vit": [os.path.join(ROOT, "profiles", "r06", "pmc_traffic_vit.json"),
                        os.path.join(ROOT, "profiles", "r05", "pmc_traffic_vit.json"),
                        os.path.join(ROOT, "profiles", "r04", "pmc_traffic_vit.json"),
                        os.path.join(ROOT, "profiles", "r03", "pmc_traffic_vit.json"),
                        os.path.join(ROOT, "profiles", "r02", "pmc_traffic.json")],
                "vit_sequential": [os.path.join(ROOT, "profiles", "r06", "pmc_traffic_vit_sequential.json")],
                "grid": [os.path.join(ROOT, "profiles", "r06", "pmc_traffic_grid.json"),
                         os.path.join(ROOT, "profiles", "r05", "pmc_traffic_grid.json"),
                         os.path.join(ROOT, "profiles", "r04", "pmc_traffic_grid.json"),
                         os.path.join(ROOT, "profiles", "r03", "pmc_traffic_grid.json")]}


def traffic_source(workload):
    for path in TRAFFIC_JSON.get(workload, []):
        if os.path.exists(path):
            return os.path.relpath(path, ROOT)
    return None


def pmc_traffic(kernel: str, workload):
    """Per-launch HBM-side bytes of `kernel` from the committed PMC summary of `workload` ("vit" / "grid" greedy,
    collected on this bench's default command), or None when there is none (other modes)."""
    src = traffic_source(workload)
    if src is None:
        return None
    try:
        with open(os.path.join(ROOT, src)) as f:
            table = json.load(f)
    except (OSError, ValueError):
        return None
    # every template variant; the 256-family class also covers the W-stationary conv form it launches (conv_rmw.hip)
    fam = {kernel, "conv_rmw_kernel"} if kernel == "gemm_256_kernel" else {kernel}
    rows = [row for name, row in table.items() if name.split("<")[0] in fam]
    n = sum(r["launches"] for r in rows)
    return int(sum(r["traffic_bytes"] * r["launches"] for r in rows) / n) if n else None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Algorithmic work per caption: encoder FLOPs (MFMA phase) and decode bytes at B = 256
# (HBM phase: cross-attention memory reads, self-KV reads/writes, amortised weights; KV-cached decoder)
ENC_FLOP = {"vit": 35.28e9, "grid": 17.58e9}
DEC_BYTES = {"vit": 83.7e6, "grid": 29.5e6}
CPU_VALIDATION = os.path.join(ROOT, "profiles", "r02", "cpu_ref_timing.json")


def host_threads() -> int:
    """Threads the CPU baseline may use: the cores this process may run on, capped by OMP_NUM_THREADS
    when the launcher sets it (the GPU box grants 16 cores of a larger machine and sets it to 16)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds: float, batch: int, max_len: int) -> dict:
    """Oracle (port of the reference algorithm, fp32, full-prefix recompute) on host cores."""
    from oracle import captioner as O

    threads = host_threads()
    torch.set_num_threads(threads)
    sd = W.to_torch(W.vit_state_dict(0))
    imgs = torch.from_numpy(W.synthetic_images(batch, seed=99))
    O.greedy_search(sd, imgs, W.START_TOKEN, W.END_TOKEN, max_len)  # warm
    n, t0 = 0, time.perf_counter()
    while True:
        O.greedy_search(sd, imgs, W.START_TOKEN, W.END_TOKEN, max_len)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    out = {"value": round(n * batch / el, 3), "unit": "captions/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
           "sample": f"oracle/captioner.py greedy_search fp32, {n} call(s) x {batch} images, max_len={max_len}, "
                     f"{el:.1f} s on {threads} host threads (affinity {len(os.sched_getaffinity(0))} cores, "
                     f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')})"}
    try:  # the container-side check of the port against the reference's own generate (tools/cpu_ref_timing.py)
        with open(CPU_VALIDATION) as f:
            v = json.load(f)
        out["port_vs_reference"] = {"ratio": v["oracle_over_reference"], "threads": v["threads"],
                                    "cpu_model": v["cpu_model"], "source": "profiles/r02/cpu_ref_timing.json"}
    except (OSError, ValueError, KeyError):
        pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--max-len", type=int, default=30)
    ap.add_argument("--precision", default="f16", choices=sorted(_lib.PRECISIONS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-batch", type=int, default=16,
                    help="images per oracle call of the CPU baseline sample (a slice of the B = 256 workload)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graphs", action="store_true", help="launch the decode loop eagerly (no hipGraph)")
    ap.add_argument("--decode-chains", type=int, default=0,
                    help="independent decode chains per batch (icap_set_decode_chains; 0 = library default)")
    ap.add_argument("--decode-step", type=int, default=-1, choices=[-1, 0, 1, 2],
                    help="decode loop form (icap_set_decode_step: 0 launch per block, 1 task step, 2 group step; "
                         "-1 = library default)")
    ap.add_argument("--prof-every", type=int, default=0,
                    help="bracket ViT encoder layers 0, N, 2N, ... with timing events (0: 6 for the f16 ViT, else 1)")
    ap.add_argument("--model", default="vit", choices=["vit", "grid"])
    ap.add_argument("--torch-trunk", action="store_true", help="grid: ResNet trunk via PyTorch/MIOpen fp32")
    ap.add_argument("--mode", default="greedy", choices=["greedy", "scst", "beam"])
    ap.add_argument("--beam", type=int, default=5, help="beam width of --mode beam")
    ap.add_argument("--fp32-weights", action="store_true",
                    help="weights NOT rounded to bf16 (a real fp32 checkpoint): the engine packs the decoder's GEMM weights "
                         "as hi/lo bf16 pairs, which the fused decode blocks carry as lo fragment images "
                         "(config.dec_weight_planes = 2)")
    ap.add_argument("--sequential", action="store_true",
                    help="greedy: run each step's encode, decode and stop rule one after the other (the round-5 "
                         "line) instead of the default batch pipeline - the encode of batch i+1 on its own stream "
                         "beside the decode of batch i, on 160 of the 256 CUs (image_caption_amd/pipeline.py; round 6: "
                         "12,246-12,349 against 10,617 sequential, profiles/r06/pipe_cus_ab.txt, pipe_ab.txt)")
    ap.add_argument("--pipeline", action="store_true", help="(the default for greedy; kept for old command lines)")
    args = ap.parse_args()

    # BENCH_DIST_BACKEND / BENCH_ONE_DEVICE: rehearsal of the N > 1 flow on a one-GPU box (every rank on cuda:0,
    # gloo collectives; tools/r3_dist_rehearsal.sh) - never set for a measured line
    rank, ws, local = parallel.init(backend=os.environ.get("BENCH_DIST_BACKEND") or None)
    if ws != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={ws}; using WORLD_SIZE")
    dev = torch.device("cuda", 0 if os.environ.get("BENCH_ONE_DEVICE") == "1" else local)
    torch.cuda.set_device(dev)

    exact = not args.fp32_weights
    sd = W.to_torch(W.vit_state_dict(0, bf16_exact=exact) if args.model == "vit" else W.grid_state_dict(0, bf16_exact=exact))
    eng = Engine(sd, args.model, {}, precision=args.precision, device=dev)
    trunk = None
    if args.model == "grid" and args.torch_trunk:
        from models.grid_transformer_model import GridFeatureEncoder

        genc = GridFeatureEncoder(pretrained_cnn=False)
        genc.load_state_dict({k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")})
        trunk = genc.cnn.to(dev).eval()
    if args.no_graphs:
        eng.set_graphs(False)
    if args.decode_chains:
        eng.set_decode_chains(args.decode_chains)
    if args.decode_step >= 0:
        eng.set_decode_step(args.decode_step)
    B = args.batch
    total = B * ws
    imgs = torch.from_numpy(W.synthetic_images(B, seed=1 + rank)).to(dev)
    L = args.max_len

    def encode():
        if trunk is not None:
            with torch.no_grad():
                return eng.encode(trunk(imgs))
        return eng.encode(imgs)

    # phase events of the timed greedy steps (torch's current stream = the stream libicap launches on;
    # the decode graph's second chain forks from and joins back into it)
    phase_ev, recording = [], [False]

    def mark():
        if not recording[0]:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def step():
        e0 = mark()
        mem = encode()
        e1 = mark()
        ids, _ = eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, L)
        e2 = mark()
        if ws > 1:
            ids = parallel.gather_rows(ids, total)
        e3 = mark()
        if recording[0]:
            phase_ev.append((e0, e1, e2, e3))
        return apply_stop_rule(ids.long(), W.END_TOKEN)

    if args.mode == "beam":
        def step():  # noqa: F811
            mem = encode()
            ids, lens = eng.beam(mem, W.START_TOKEN, W.END_TOKEN, L, args.beam, grid_variant=args.model == "grid")
            if ws > 1:
                ids = parallel.gather_rows(ids, total)
            return ids

    if args.mode == "scst":
        from image_caption_amd import cider
        from image_caption_amd.scst import sample_and_greedy
        from utils.scst_loss import sample_stop_length

        gen = torch.Generator(device="cpu").manual_seed(5)
        # one synthetic reference caption (5-12 tokens) per image of the global batch
        refs = [[torch.randint(1, 100, (int(torch.randint(5, 13, (1,), generator=gen)),), generator=gen).tolist()]
                for _ in range(total)]
        uni = torch.rand(L - 1, B, generator=gen).to(dev)
        ref_rows, ref_off = cider.pack_references(refs, W.PAD_TOKEN, W.END_TOKEN, W.VOCAB_SIZE)
        ref_rows, ref_off = ref_rows.to(dev), ref_off.to(dev)

        def step():  # noqa: F811
            mem = encode()
            # sampled + greedy decodes of the same memory, concurrently on two streams
            sid, _, gid = sample_and_greedy(eng, mem, uni, W.START_TOKEN, W.END_TOKEN, L)
            if ws > 1:
                sid, gid = parallel.gather_rows(sid, total), parallel.gather_rows(gid, total)
            sid, gid = sid.long(), apply_stop_rule(gid.long(), W.END_TOKEN)
            sid = sid[:, : sample_stop_length(sid, W.END_TOKEN)]
            if rank == 0:  # CIDEr-D of both sets over the GLOBAL batch, one GPU pass (icap_cider_d)
                hyp = torch.full((2 * total, max(sid.shape[1], gid.shape[1])), W.PAD_TOKEN, dtype=torch.int32,
                                 device=dev)
                hyp[:total, : sid.shape[1]] = sid
                hyp[total:, : gid.shape[1]] = gid
                r = cider.cider_d_device(hyp, ref_rows, ref_off, W.START_TOKEN, W.END_TOKEN, W.PAD_TOKEN).float()
                return r[:total] - r[total:]
            return gid

    pipe = None
    pipe_ev = []  # pipelined steps: per batch (encode start, end, decode start, end) on the two streams
    if args.mode == "greedy" and trunk is None and not args.sequential:
        from image_caption_amd.pipeline import CaptionPipeline

        dcus = int(os.environ.get("ICAP_PIPE_DECODE_CUS", "0")) or None
        dprio = int(os.environ.get("ICAP_PIPE_DECODE_PRIORITY", "-1"))
        ecus = os.environ.get("ICAP_PIPE_ENC_CUS")  # measurement knob: the overlapped encodes' CU budget (0 = all CUs)
        acus = os.environ.get("ICAP_PIPE_ENC_ATTN_CUS")  # and their attention's (0 = the GEMMs' budget)
        pipe = CaptionPipeline(eng, W.START_TOKEN, W.END_TOKEN, L, decode_priority=dprio, decode_cus=dcus,
                               encoder_cus=int(ecus) if ecus else None, attention_cus=int(acus) if acus else None)
        pipe.defer_post = os.environ.get("ICAP_PIPE_DEFER_POST", "1") != "0"  # measurement knob (0: post not deferred)

        def post(ids):
            if ws > 1:
                ids = parallel.gather_rows(ids, total)
            return apply_stop_rule(ids.long(), W.END_TOKEN)

    def run_steps(n):
        if pipe is not None:  # n steps = n batches, encode(i+1) overlapping decode(i)
            return pipe.run([imgs] * n, post, timing=pipe_ev if recording[0] else None)[-1] if n else None
        o = None
        for _ in range(n):
            o = step()
        return o

    out = run_steps(args.warmup)
    torch.cuda.synchronize()

    # live launch timing over the timed steps: HIP event pairs cost the stream ~3 us each (tools/r6_gap.py: bracketing
    # all 60 encoder-layer launches of a ViT step added 0.4 ms), so the f16 ViT brackets layers 0 and 6 of every step
    # (8 of the 48 persistent-GEMM launches, 2 of the 12 attentions - the layers share their shapes)
    prof_every = args.prof_every or (6 if args.model == "vit" and args.precision == "f16" else 1)
    sampled = {"gemm_f16p_kernel", "enc_attention_kernel"} if prof_every > 1 else set()
    eng.profile(True, every=prof_every)
    recording[0] = True
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = run_steps(args.steps)
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    recording[0] = False
    prof = [eng.profile_read(c) for c in sorted(_lib.PROF_NAMES)]
    eng.profile(False)
    phases = None
    if phase_ev or pipe_ev:  # encoder = MFMA-bound phase, decode = HBM-bound phase (SURVEY.md §8(d) phase-wise roofline)
        if pipe_ev:  # pipelined: each phase on its own stream (batch i's decode overlaps batch i + 1's encode)
            n = len(pipe_ev)
            enc_ms = sum(a.elapsed_time(b) for a, b, _, _ in pipe_ev) / n
            dec_ms = sum(c.elapsed_time(d) for _, _, c, d in pipe_ev) / n
            gat_ms = 0.0  # (the all-gather runs inside the decode stream's post step, not timed apart)
        else:
            n = len(phase_ev)
            enc_ms = sum(a.elapsed_time(b) for a, b, _, _ in phase_ev) / n
            dec_ms = sum(b.elapsed_time(c) for _, b, c, _ in phase_ev) / n
            gat_ms = sum(c.elapsed_time(d) for _, _, c, d in phase_ev) / n
        if ws > 1:  # the slowest rank's phases
            t = torch.tensor([enc_ms, dec_ms, gat_ms], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            enc_ms, dec_ms, gat_ms = t.tolist()
        enc_tf = ENC_FLOP[args.model] * B / (enc_ms * 1e-3) / 1e12
        dec_gbs = DEC_BYTES[args.model] * B / (dec_ms * 1e-3) / 1e9
        phases = {
            "encoder": {"ms_per_step": round(enc_ms, 3), "bound": "mfma", "achieved": round(enc_tf, 1),
                        "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(enc_tf / PEAK_BF16_TFLOPS, 4),
                        "work": f"{ENC_FLOP[args.model] / 1e9:.2f} GFLOP/image algorithmic (SURVEY.md 8d) x {B}"},
            "decode": {"ms_per_step": round(dec_ms, 3), "bound": "hbm", "achieved": round(dec_gbs, 1),
                       "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(dec_gbs / PEAK_HBM_GBS, 4),
                       "work": f"{DEC_BYTES[args.model] / 1e6:.1f} MB/caption algorithmic (SURVEY.md 8d) x {B}, "
                               f"{L - 1} steps"},
            "allgather_ms_per_step": round(gat_ms, 3),
        }
        if pipe_ev:
            phases["overlapped"] = True  # encoder and decode ms of one batch; consecutive batches' phases overlap
    # multi-GPU self-check: the stop rule on the gathered ids equals the all-reduce form of SURVEY.md §8(e)
    # (each rank's per-column "every row ended" mask AND-reduced over ranks), so the line can be verified alone
    stop_check = None
    if args.mode == "greedy":
        mem = encode()
        ids, _ = eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, L)
        col = (ids[:, 1:] == W.END_TOKEN).all(dim=0).to(torch.int32)
        if ws > 1:
            dist.all_reduce(col, op=dist.ReduceOp.MIN)
            gathered = parallel.gather_rows(ids, total)
        else:
            gathered = ids
        hit = torch.nonzero(col)
        want = int(hit[0, 0]) + 2 if hit.numel() else L
        stop_check = {"ranks": ws, "per_rank_batch": B, "gathered_rows": int(gathered.shape[0]),
                      "output_len": int(apply_stop_rule(gathered.long(), W.END_TOKEN).shape[1]),
                      "allreduce_len": want}
        stop_check["ok"] = stop_check["output_len"] == want and stop_check["gathered_rows"] == total
    value = total * args.steps / el
    if rank == 0:
        step_ms = el / args.steps * 1e3
        for p in prof:  # sampled classes: the recorded launches stand for prof_every times as many
            p["scale"] = prof_every if p["kernel"] in sampled else 1
        dom = max(prof, key=lambda p: p["ms"] * p["scale"])
        workload = args.model if args.mode == "greedy" else None  # the PMC summaries' workloads
        if workload == "vit" and pipe is None:
            workload = "vit_sequential"
        avg_ms = dom["ms"] / max(dom["launches"], 1)
        for p in prof:
            if not p["launches"]:
                continue
            log(f"  {p['kernel']:34s} launches {p['launches']:6d}  {p['ms'] * p['scale'] / args.steps:9.3f} ms/step  "
                f"{p['flops'] / max(p['ms'], 1e-9) / 1e9:9.1f} TFLOP/s alg  "
                f"{p['bytes'] / max(p['ms'], 1e-9) / 1e6:9.1f} GB/s operand")
        if "attn" in dom["kernel"] and "cross" in dom["kernel"]:
            achieved = dom["bytes"] / dom["launches"] / (avg_ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": pmc_traffic(dom["kernel"], workload)}
        else:
            # achieved = algorithmic 2MNK per launch / launch time.  The MFMA work behind it: bf16x2 GEMMs
            # issue 2 bf16 products per algorithmic MAC (hi and lo activation planes), the i8x2 GEMM 3 i8
            # products (A1.W1, A1.W2, A2.W1) against the i8 peak - reported as mfma_issue_frac.
            i8 = "i8" in dom["kernel"]
            peak = PEAK_I8_TOPS if i8 else PEAK_BF16_TFLOPS
            work = 3 if i8 else (1 if args.precision in ("bf16", "f16") else 2)
            achieved = dom["flops"] / dom["launches"] / (avg_ms * 1e-3) / 1e12
            roof = {"bound": "mfma", "achieved": round(achieved, 1), "peak": peak,
                    "unit": "TFLOP/s", "peak_dtype": "i8" if i8 else ("f16" if args.precision == "f16" else "bf16"), "frac": round(achieved / peak, 4),
                    "traffic": pmc_traffic(dom["kernel"], workload),
                    "mfma_products_per_alg_mac": work, "mfma_issue_frac": round(achieved * work / peak, 4)}
        roof.update({"kernel": dom["kernel"], "launches_per_step": dom["launches"] * dom["scale"] // args.steps,
                     "launches_timed_per_step": dom["launches"] // args.steps,
                     "avg_launch_us": round(avg_ms * 1e3, 2),
                     "share_of_step": round(dom["ms"] * dom["scale"] / args.steps / step_ms, 3)})
        if pipe is not None and pipe.overlap_cus and dom["kernel"] in sampled:
            # pipelined: the overlapped encodes' persistent grids hold overlap_cus of the CUs (the first timed encode
            # all of them), the rest left to the decode stream - frac of the CUs the kernel was given beside frac
            cus = torch.cuda.get_device_properties(dev).multi_processor_count
            granted = (cus + (args.steps - 1) * pipe.overlap_cus) / args.steps
            roof["cus_granted_avg"] = round(granted, 1)
            roof["frac_of_granted_cus"] = round(roof["frac"] * cus / granted, 4)
        cpu = None
        if roof["traffic"] is not None:
            roof["traffic_unit"] = f"bytes/launch (HBM-side, rocprofv3 PMC, {traffic_source(workload)})"
        if ws == 1 and not args.no_cpu_baseline and args.model == "vit":
            cpu = cpu_baseline(args.cpu_seconds, args.cpu_batch, L)
        line = {
            "metric": {"greedy": METRIC, "scst": "images/sec, SCST reward step (sample + greedy + CIDEr-D)",
                       "beam": f"captions/sec, beam search (beam {args.beam}, max_len={L})"}[args.mode],
            "value": round(value, 2), "unit": "images/s" if args.mode == "scst" else "captions/s", "n_gpus": ws, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(step_ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"bf16": "bf16", "bf16x2": "bf16x2", "i8x2": "i8x2+bf16x2", "f16": "f16+bf16x2"}[args.precision], "data": "synthetic images N(0,1) + seeded random-init weights",
            "config": {"workload": ("vit_b16 encoder + 6-layer decoder, greedy, 224x224, max_len=30" if args.model == "vit"
                                    else f"grid resnet101 ({'torch/MIOpen fp32' if args.torch_trunk else 'HIP'}) "
                                         "+ 6-layer encoder + 6-layer decoder, greedy, 224x224, max_len=30")
                       + {"greedy": "", "scst": "; SCST reward step: sample + greedy + CIDEr-D (global batch)",
                          "beam": f"; beam search, beam {args.beam}"}[args.mode],
                       "per_gpu_batch": B, "global_batch": total, "max_len": L, "precision": args.precision,
                       "decode_steps": L - 1, "output_len": int(out.shape[1]) if args.mode == "greedy" else None,
                       "parallelism": f"dp{ws}",
                       "pipelined": pipe is not None,
                       "encoder_cus_overlapped": pipe.overlap_cus if pipe is not None else None,
                       "attention_cus_overlapped": pipe.overlap_attn_cus if pipe is not None else None,
                       # 1: bf16-exact decoder weights (the seeded synthetic weights); 2: hi/lo pairs (--fp32-weights, a
                       # real fp32 checkpoint) - both through the fused decode blocks (round 5)
                       "dec_weight_planes": eng.dec_weight_planes},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if phases is not None:
            line["roofline"]["phases"] = phases
        if stop_check is not None:
            line["config"]["multi_gpu_check"] = stop_check
        if os.environ.get("BENCH_DIST_BACKEND") or os.environ.get("BENCH_ONE_DEVICE") == "1":
            # a rehearsal of the N > 1 flow with every rank on one GPU: not a measurement of N GPUs
            line["rehearsal"] = True
            line["physical_devices"] = 1 if os.environ.get("BENCH_ONE_DEVICE") == "1" else None
            line["rehearsal_value"] = line["value"]
            line["value"] = None
            line["metric"] = "REHEARSAL (ranks share one GPU, not a measurement): " + line["metric"]
        print(json.dumps(line), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
