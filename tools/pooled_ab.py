"""A/B on the GPU box: free-running self-play (C4SelfPlay.run, K moves per game) against the
pooled launch (C4SelfPlay.run_pooled, G*K moves shared by the games, at most CAP per game),
alternating on one steady-state pool.  Prints expansions/s and ms per G moves of each."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import burn_in  # noqa: E402
from zeroclone_amd.selfplay import C4SelfPlay  # noqa: E402


def timed(sp, fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = fn()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = sp.stats[:, [0, 2]].sum(0).tolist()
    per_game = (res != 4).sum(0).float()
    moves = int(per_game.sum().item())
    return {"dt": dt, "expansions": int(st[0]), "leaves": int(st[1]), "moves": moves,
            "per_game_moves": {"min": int(per_game.min()), "max": int(per_game.max()),
                               "p99": float(per_game.quantile(0.99)), "mean": float(per_game.mean())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--k", type=int, default=60)
    ap.add_argument("--cap", type=int, default=120)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    sp = C4SelfPlay(a.games, 800, c=1.4, batch_size=32, seed=0, record=True)
    sp.start()
    print("burn-in steps", burn_in(sp), flush=True)
    out = {"free": [], "pooled": []}
    for r in range(a.rounds):
        f = timed(sp, lambda: sp.run(a.k))
        p = timed(sp, lambda: sp.run_pooled(a.games * a.k, a.cap))
        sp.take()
        for name, x in (("free", f), ("pooled", p)):
            x["exp_per_s"] = x["expansions"] / x["dt"]
            x["ms_per_G_moves"] = x["dt"] * 1e3 / (x["moves"] / a.games)
            out[name].append(x)
        print(json.dumps({"round": r, "free": f, "pooled": p}), flush=True)
    for name in out:
        v = [x["exp_per_s"] for x in out[name]]
        print(name, "exp/s", [round(x / 1e9, 4) for x in v], flush=True)


if __name__ == "__main__":
    main()
