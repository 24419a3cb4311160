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
# ZC_LIB: load (and build) another copy of the library, e.g. a variant for an A/B timing run
LIB = os.environ.get("ZC_LIB") or os.path.join(HERE, "libzeroclone_amd.so")
SOURCES = ["engine.hip", "c4_search.hip", "c4_ext.hip", "chess.hip", "chess_search.hip", "chess_puct.hip", "net_conv.hip", "selfplay.hip", "c4_puct.hip", "gen_search.hip"]
HEADERS = ["zc_internal.h", "c4_order_table.h", "c4_device.h", "chess_device.h", "chess_tree.h", "counter_rng.h", "puct_common.h", os.path.join("..", "..", "include", "zeroclone.h")]
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


FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall"]
# per-source extras: the search kernels are one long dependent chain per wave; LLVM's iterative
# ILP machine scheduler orders them 1 % faster than the default (same-box A/B, outputs identical,
# profiles/r03_ab_sched.log; max-memory-clause and iterative-maxocc were 0.9 % slower).  Only
# there: ROCm 7.2's clang crashes in register allocation with it on chess_search.hip.  The
# network tower (net_conv.hip) too: 6x7 x 131072 18.85 -> 18.66 ms, 8x8 x 32768 equal, outputs
# identical (profiles/r05_ab_tower_sched.log; max-ilp: no gain).  chess_search.hip under
# max-ilp or iterative-maxocc: equal to the default (profiles/r05_ab_chess_sched.log).
SOURCE_FLAGS = {"c4_search.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
                "net_conv.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]}
# A/B builds only: ZC_C4_SCHED=<strategy> ("default": none) replaces c4_search.hip's strategy
if os.environ.get("ZC_C4_SCHED"):
    SOURCE_FLAGS["c4_search.hip"] = ([] if os.environ["ZC_C4_SCHED"] == "default" else
                                     ["-mllvm", "-amdgpu-sched-strategy=" + os.environ["ZC_C4_SCHED"]])


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every source to an object in parallel, then link the shared library."""
    if not force and not _stale():
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    objdir = os.path.join(HERE, "build_obj" if LIB.endswith("libzeroclone_amd.so") else "build_obj_" + os.path.basename(LIB))
    os.makedirs(objdir, exist_ok=True)
    # -ffp-contract=off: the UCT arithmetic must round exactly like the reference's
    # (explicit fma only where GCC emitted one for mcts.cpp:44).
    def compile_one(src):
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc(), f"--offload-arch={ARCH}", *FLAGS, *SOURCE_FLAGS.get(src, []),
               *os.environ.get("ZC_CFLAGS", "").split(), "-c",
               os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return obj
    jobs = min(len(SOURCES), int(os.environ.get("MAX_JOBS", "8")))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
