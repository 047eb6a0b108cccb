"""Container-side check of bench.py's CPU baseline: the oracle (oracle/captioner.py greedy_search, the
`cpu_baseline` leg, kind "port") against the reference's OWN ViTTransformerCaptioning.generate
(models/vit_transformer_model.py:276-325, imported by file path from /root/reference with the build's
torchvision restatement as its ViT trunk) at B = 4, greedy max_len 30, same weights, images, threads.
SURVEY.md §8(d) asks the port's CPU time to be within +-15 % of the reference's before it is trusted.

Usage: python tools/cpu_ref_timing.py [threads] [repeats]   (writes profiles/r02/cpu_ref_timing.json)
"""
import json
import os
import platform
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from image_caption_amd import weights as W  # noqa: E402
from oracle import captioner as O  # noqa: E402


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def timed(fn, repeats):
    fn()  # warm
    ts = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), sum(ts) / len(ts)


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else len(os.sched_getaffinity(0))
    repeats = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    torch.set_num_threads(threads)
    import make_golden as M

    sd = W.to_torch(W.vit_state_dict(0))
    ref = M.ref_vit_model(M.load_ref_vit_module(), sd)
    imgs = torch.from_numpy(W.synthetic_images(4, seed=99))
    with torch.no_grad():
        a = ref.generate(imgs, W.START_TOKEN, W.END_TOKEN, max_len=30)
    b = O.greedy_search(sd, imgs, W.START_TOKEN, W.END_TOKEN, 30)
    assert torch.equal(a, b), "oracle and reference disagree"

    def run_ref():
        with torch.no_grad():
            ref.generate(imgs, W.START_TOKEN, W.END_TOKEN, max_len=30)

    def run_oracle():
        O.greedy_search(sd, imgs, W.START_TOKEN, W.END_TOKEN, 30)

    r_min, r_avg = timed(run_ref, repeats)
    o_min, o_avg = timed(run_oracle, repeats)
    out = {"cpu_model": cpu_model(), "threads": threads, "batch": 4, "max_len": 30, "repeats": repeats,
           "reference_captions_per_s": round(4 / r_avg, 3), "oracle_captions_per_s": round(4 / o_avg, 3),
           "oracle_over_reference": round(r_avg / o_avg, 3),
           "reference_s": [round(r_min, 3), round(r_avg, 3)], "oracle_s": [round(o_min, 3), round(o_avg, 3)],
           "ids_equal": True}
    print(json.dumps(out))
    os.makedirs(os.path.join(ROOT, "profiles", "r02"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r02", "cpu_ref_timing.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
