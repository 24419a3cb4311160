#!/usr/bin/env python3
"""Where the free-running (lockstep) launch's waves run (zc_debug_c4_launch_stamps' placement
word: HW_ID's SIMD / CU / SH / SE and the XCC) on the bench workload (4096 burned-in games x
800 sims x bs 32, K-move free launches): whether the game -> SIMD mapping repeats from launch
to launch, how the SIMD groups follow the game (slot) index, and how unequal the SIMDs'
measured work is (the sum of their games' wave times, each game's end - start)."""
import collections
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from zeroclone_amd import _native  # noqa: E402
from zeroclone_amd.selfplay import C4SelfPlay  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.cuda.set_device(0)
    G = 4096
    sp = C4SelfPlay(G, 800, c=1.4, batch_size=32, seed=0, device=0, record=True)
    bench.burn_in(sp)
    buf = torch.zeros((G, 4), dtype=torch.int64, device="cuda")
    _native.check(_native.lib().zc_debug_c4_launch_stamps(sp.eng._h, buf.data_ptr()))
    maps, parts, durs, stones = [], [], [], []
    for rep in range(4):
        roots = sp.roots.cpu().numpy().reshape(G, -1)
        st = np.array([bin(int(r[0]) & ((1 << 64) - 1)).count("1") + bin(int(r[1]) & ((1 << 64) - 1)).count("1")
                       for r in roots])
        stones.append(st)
        buf.zero_()
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        sp.run(K, kernel_done=ev[1])
        torch.cuda.synchronize()
        ts = buf.cpu().numpy()
        hw = (ts[:, 3] >> 32) & 0xFFFFFFFF
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 7
        xcc = (hw >> 16) & 15
        key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
        maps.append(key)
        dur = (ts[:, 2] - ts[:, 0]).astype(np.float64) / 1e5   # ms per game (wave lifetime)
        groups = collections.defaultdict(list)
        for g in range(G):
            groups[int(key[g])].append(g)
        sizes = collections.Counter(len(v) for v in groups.values())
        simd_work = np.array([dur[v].sum() for v in groups.values()])
        simd_max = np.array([dur[v].max() for v in groups.values()])
        ex = list(groups.values())[:4]
        part = sorted(tuple(sorted(v)) for v in groups.values())
        parts.append(part)
        durs.append(dur)
        corr = {}
        if rep:
            corr["prev_launch"] = round(float(np.corrcoef(dur, durs[-2])[0, 1]), 3)
        for name, f in (("empty_cells", 42 - st), ("empty_cells_sq", (42 - st) ** 2)):
            corr[name] = round(float(np.corrcoef(dur, f)[0, 1]), 3)
        rec = {"rep": rep, "same_partition_as_first": part == parts[0], "corr_game_ms_with": corr, "launch_ms": round(ev[0].elapsed_time(ev[1]), 3), "simds": len(groups),
               "games_per_simd": dict(sizes), "example_groups": ex,
               "same_as_first": bool(np.array_equal(key, maps[0])),
               "game_ms_mean_max": [round(float(dur.mean()), 3), round(float(dur.max()), 3)],
               "simd_sum_ms_mean_p99_max": [round(float(simd_work.mean()), 3),
                                            round(float(np.percentile(simd_work, 99)), 3),
                                            round(float(simd_work.max()), 3)],
               "simd_longest_game_ms_mean_max": [round(float(simd_max.mean()), 3), round(float(simd_max.max()), 3)],
               "lib_sha256": bench.lib_sha()[:12]}
        print(json.dumps(rec), flush=True)
    _native.check(_native.lib().zc_debug_c4_launch_stamps(sp.eng._h, None))
    sp.close()


if __name__ == "__main__":
    main()
