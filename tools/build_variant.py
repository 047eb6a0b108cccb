"""Product-build variants for same-box A/B (tools/ab_libs.sh): icap.cpp recompiled with extra -D defines (the
compile-time defaults of the decode-loop choices, e.g. -DICAP_DEC_FOLD_DEFAULT=0) and linked with the product objects
of the current build.  usage: python tools/build_variant.py OUT.so [--src a.hip,b.cpp] -DNAME=VALUE ...
(--src: the sources recompiled with the defines, default icap.cpp)"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from image_caption_amd import build as B  # noqa: E402


def main():
    out, args = Path(sys.argv[1]), sys.argv[2:]
    srcs = ["icap.cpp"]
    if args and args[0] == "--src":
        srcs, args = args[1].split(","), args[2:]
    B.build()  # the product objects are current
    objs = [B.HERE / "build" / (s + ".o") for s in B.SOURCES if s not in srcs]
    new = []
    for src in srcs:
        obj = out.with_suffix("." + src + ".o")
        subprocess.run([B.HIPCC, *B.FLAGS, *args, "-x", "hip", "-c", str(B.CSRC / src), "-o", str(obj)], check=True)
        new.append(obj)
    subprocess.run([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(out), *map(str, objs + new)],
                   check=True)
    for obj in new:
        obj.unlink()
    print(out)


if __name__ == "__main__":
    main()
