#!/usr/bin/env python3
"""GPU diagnostics for the Connect4 search kernel: timing vs game count, phase shares."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from zeroclone_amd import _native  # noqa: E402


def timed(eng, G, S, B, reps=7):
    roots = np.zeros(G, _native.C4_STATE_DTYPE)
    eng.seed(0, list(range(G)))
    eng.c4_search(roots, S, 1.4, B)  # warm
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        mv, na, st = eng.c4_search(roots, S, 1.4, B)
        ts.append(time.perf_counter() - t)
    ts.sort()
    return ts[len(ts) // 2], st


def main():
    S, B = 800, 32
    eng = _native.NativeEngine(max_games=16384, max_sims=S, max_batch=B)
    res = {}
    for G in [64, 512, 2048, 4096, 8192, 16384]:
        t, st = timed(eng, G, S, B)
        res[G] = {"ms": round(t * 1e3, 3), "Mexp_s": round(st["expansions"].sum() / t / 1e6, 2),
                  "plies_per_leaf": round(st["rollout_plies"].sum() / st["leaves"].sum(), 2),
                  "words_per_leaf": round(st["rng_words"].sum() / st["leaves"].sum(), 2),
                  "blocks_per_leaf": round(st["rollout_blocks"].sum() / st["leaves"].sum(), 3)}
        print(G, res[G], flush=True)
    eng.c4_rollout_mode("philox", 12345)
    for G in (4096, 16384):
        t, st = timed(eng, G, S, B)
        print("philox", G, {"ms": round(t * 1e3, 3), "Mexp_s": round(st["expansions"].sum() / t / 1e6, 2),
                            "plies_per_leaf": round(st["rollout_plies"].sum() / st["leaves"].sum(), 2)}, flush=True)
    eng.phase_cycles(True)
    roots = np.zeros(4096, _native.C4_STATE_DTYPE)
    eng.seed(0, list(range(4096)))
    eng.c4_search(roots, S, 1.4, B)
    ph = eng.phase_cycles(False)
    tot = sum(ph.values())
    print("philox phase shares (4096 games):", {k: round(v / tot, 4) for k, v in ph.items()},
          "cycles/game/sim:", round(tot / 4096 / S, 1), flush=True)
    eng.c4_rollout_mode("exact")
    for G in (4096, 256):
        eng.phase_cycles(True)
        roots = np.zeros(G, _native.C4_STATE_DTYPE)
        eng.seed(0, list(range(G)))
        eng.c4_search(roots, S, 1.4, B)
        ph = eng.phase_cycles(False)
        tot = sum(ph.values())
        print(f"phase shares ({G} games, stamped build):", {k: round(v / tot, 4) for k, v in ph.items()},
              "cycles/game/sim:", round(tot / G / S, 1),
              "per phase:", {k: round(v / G / S, 1) for k, v in ph.items()}, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
