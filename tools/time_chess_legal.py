#!/usr/bin/env python3
"""Time of one chess_legal launch (1 wave per position) for n opening / midgame positions:
what one legal-move generation costs a search wave."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeroclone_amd import _native  # noqa: E402

eng = _native.NativeEngine(max_games=16, max_sims=8, max_batch=8)
fens = ["rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
        "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1"]
for fen in fens:
    for n in (1024, 65536):
        st = np.array([_native.chess_from_fen(fen)] * n, _native.CHESS_STATE_DTYPE)
        d = torch.from_numpy(st.view(np.uint8).reshape(n, -1).copy()).cuda()
        mv = torch.zeros((n, _native.CHESS_MAX_MOVES), dtype=torch.int16, device="cuda")
        cnt = torch.zeros(n, dtype=torch.int32, device="cuda")
        f = lambda: eng.chess_legal_moves_async(n, d.data_ptr(), mv.data_ptr(), cnt.data_ptr())  # noqa: E731
        f()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            f()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 20
        print(fen.split()[0][:20], n, "moves", int(cnt[0]), f"{ms * 1e3:.1f} us per launch", flush=True)
