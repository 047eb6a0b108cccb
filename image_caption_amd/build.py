"""Build libicap.so for gfx950 with hipcc (in-tree, so it travels to the GPU box)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
LIB = HERE / "libicap.so"
SOURCES = ["gemm.hip", "rows.hip", "attention.hip", "head.hip", "beam.hip", "decode.hip", "trunk.hip", "conv_rmw.hip", "preprocess.hip", "cider.hip", "train.hip", "icap.cpp"]
# measured-and-rejected kernel forms: compiled into the tools build only
TOOLS_SOURCES = ["gemm_tools.hip", "decstep.hip", "xdec.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-munsafe-fp-atomics"]


FLAVOR = HERE / "build" / "flavor"


def _stale(tools: bool = False) -> bool:
    if not LIB.exists():
        return True
    if not FLAVOR.exists() or FLAVOR.read_text().strip() != ("tools" if tools else "product"):
        return True
    t = LIB.stat().st_mtime
    deps = [CSRC / s for s in SOURCES + (TOOLS_SOURCES if tools else [])] + list(CSRC.glob("*.h")) + list(CSRC.glob("*.inc")) + [HERE.parent / "include" / "icap.h"]
    return any(p.stat().st_mtime > t for p in deps)


def build(force: bool = False, verbose: bool = True, tools: bool = False) -> Path:
    """Product build by default.  tools=True adds -DICAP_TOOLS: the ICAP_* measurement knobs are read
    from the environment and the measured-and-rejected kernel variants are compiled in (tools/*.sh)."""
    if not force and not _stale(tools):
        return LIB
    objs = []
    obj_dir = HERE / "build"
    obj_dir.mkdir(exist_ok=True)
    procs = []
    for src in SOURCES + (TOOLS_SOURCES if tools else []):
        obj = obj_dir / (src + ".o")
        objs.append(obj)
        cmd = [HIPCC, *FLAGS, *(["-DICAP_TOOLS"] if tools else []), "-x", "hip", "-c", str(CSRC / src), "-o", str(obj)]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out.decode())
            raise RuntimeError("hipcc failed: " + " ".join(cmd))
        if verbose and out.strip():
            sys.stderr.write(out.decode())
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    FLAVOR.write_text("tools" if tools else "product")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv or "--tools" in sys.argv, tools="--tools" in sys.argv))
