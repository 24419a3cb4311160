#!/usr/bin/env python3
"""A/B in one process: the chess value-network pool (BASELINE C4: 1024 games x 400 sims, the
bench's chess_modes value_net) with the short last flush run on its leaves only
(NetValue.rows) and with every slot evaluated; one graph per step, alternating rounds."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from zeroclone_amd import _native  # noqa: E402
from zeroclone_amd.nets import ValueNetwork, for_inference  # noqa: E402
from zeroclone_amd.selfplay import ChessSelfPlay  # noqa: E402


class FullNetValue:
    """NetValue without `rows`: the short last flush evaluates every slot."""

    def __init__(self, model):
        self.model = model

    def __call__(self, leaves, planes, counts):
        return self.model(planes).reshape(-1).to(torch.float64)


def main():
    dev = torch.device("cuda", 0)
    crude, burn = bench.chess_burned_pool(dev)
    torch.manual_seed(0)
    model = for_inference(ValueNetwork(128, 8).eval(), dev, torch.float16)
    res = {}
    pools = {}
    for name in ("trimmed", "full"):
        pool = ChessSelfPlay(1024, 400, batch_size=32, seed=4, device=0, net=model,
                             policy=_native.ZC_POLICY_RANDOM, freedom=0.0)
        pool.adopt(crude)
        if name == "full":
            pool.value_fn = FullNetValue(pool.value_fn.model)
        pools[name] = (pool, pool.capture_step())
        res[name] = []
    for rnd in range(3):
        for name, (pool, g) in pools.items():
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t) / 3 * 1e3)
    for name in res:
        print(f"{name}: {statistics.median(res[name]):.2f} ms per move  all {[round(x, 2) for x in res[name]]}")


if __name__ == "__main__":
    main()
