"""Build libzeroclone_amd.so in-tree with hipcc for gfx950 (no JIT cache, no pip install).

The library is the product: every search entry point of the package goes through it, and
the package refuses to run a search when it is missing (zeroclone_amd/_native.py).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libzeroclone_amd.so")
SOURCES = ["engine.hip", "c4_search.hip", "c4_ext.hip", "chess.hip"]
HEADERS = ["zc_internal.h", "c4_order_table.h", "c4_device.h", "chess_device.h", os.path.join("..", "..", "include", "zeroclone.h")]
ARCH = os.environ.get("ZC_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm 7.x required)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    tmp = LIB + ".tmp"
    # -ffp-contract=off: the UCT arithmetic must round exactly like the reference's
    # (explicit fma only where GCC emitted one for mcts.cpp:44).
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-fno-fast-math", "-Wall", "-o", tmp] + srcs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
