#!/usr/bin/env python3
"""Per-phase cycles of the chess crude search (diagnostic build: ZC_CHESS_STAMP=1), on the
tools/ab_chess.py workload (1024 games x 400 sims x bs 32, half opening / half mixed roots):

    ZC_LIB=$PWD/zeroclone_amd/libzc_cst.so python tools/chess_stamps.py

Prints, per simulation, the s_memtime cycles of each phase summed over a move (median over
games) and their shares of the whole search."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import oracle  # noqa: E402
from zeroclone_amd import _native  # noqa: E402

PHASES = ["walk", "policy+erase", "apply_move", "create_node", "values", "backup", "select_flush", "whole",
          "legal_moves_check", "material", "node_writes", "lmc.emission", "lmc.runs_masks", "lmc.legality", "lmc.bitview_check",
          "lmc.runs_emit", "pe.cached_path", "pe.node_fields+lazy_gen", "pe.untried_loads", "pe.pick+erase",
          "pe.cached_count", "helper_wait", "pe.cached_pick", "pe.cached_erase"]
NS = len(PHASES)


def main():
    G, S, B = 1024, 400, 32
    eng = _native.NativeEngine(max_games=G, max_sims=S, max_batch=B)
    rs = np.random.default_rng(5)
    roots = []
    for i in range(G):
        st = oracle.chess_init()
        for _ in range(int(rs.integers(0, 24)) if i % 2 else 0):
            ms = oracle.chess_moves(st)
            if not ms:
                break
            nxt = oracle.chess_play(st, ms[int(rs.integers(0, len(ms)))])
            if oracle.chess_win(nxt) or oracle.chess_draw(nxt) or not oracle.chess_moves(nxt):
                break
            st = nxt
        r = np.zeros(1, _native.CHESS_STATE_DTYPE)
        r["board"][0] = np.frombuffer(bytes(st.board), np.uint8)
        r["turn"], r["fifty"], r["castle"] = st.turn, st.fifty, st.castle
        roots.append(r)
    roots = torch.from_numpy(np.concatenate(roots).view(np.uint8).reshape(G, 72).copy()).cuda()
    mv = torch.zeros(G, dtype=torch.int16, device="cuda")
    na = torch.zeros((G, 256), dtype=torch.int32, device="cuda")
    st = torch.zeros((G, 8), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    eng.seed(0, list(range(G)))
    L = _native.lib()
    f = L.zc_debug_chess_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    buf = np.zeros(4096 * NS, np.uint64)
    run = lambda: eng.chess_search_async(0, G, roots.data_ptr(), S, 1.4, B, 1, 3.0, mv.data_ptr(),  # noqa: E731
                                         na.data_ptr(), st.data_ptr(), s)
    run()
    torch.cuda.synchronize()
    assert f(buf.ctypes.data, buf.size, 1) == 0
    reps = 3
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    assert f(buf.ctypes.data, buf.size, 1) == 0
    per = buf[: G * NS].reshape(G, NS).astype(np.float64) / reps / S   # cycles per simulation
    med = np.median(per, axis=0)
    out = {"workload": "1024 games x 400 sims x bs 32, crude, half opening / half mixed roots (tools/ab_chess.py)",
           "cycles_per_simulation_median_over_games": {k: round(float(v), 1) for k, v in zip(PHASES, med)},
           "share_of_whole": {k: round(float(v / med[7]), 4) for k, v in zip(PHASES, med) if k != "whole"},
           "expansions": int(st[:, 0].sum())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
