"""Value('random_rollout') on chess at scale (zc_chess_rollouts_async, chess_search.hip's
rollout kernel) against the oracle's restatement (oracle.chess_rollout, itself pinned to the
reference's rollouts in tests/test_fallback_cpu.py): 192 positions reached by seeded random
play — openings, middle games, endgames, histories of up to ~150 moves per side, some ending
in repetition shuffles — rolled out in order on one stream; every value and the stream's
state afterwards must be identical (value_functions.py:35-45, chess_backend.cpp:148-180,
404-441)."""
import random

import numpy as np
import pytest
import torch

import oracle
from zeroclone_amd import _native

pytestmark = pytest.mark.gpu


def positions(k, rng):
    out = []
    while len(out) < k:
        s = oracle.chess_init()
        plies = rng.choice([0, 3, 10, 30, 60, 120, 200, 300])
        shuffle = rng.random() < 0.2
        for p in range(plies):
            if oracle.chess_win(s) or oracle.chess_draw(s):
                break
            ms = oracle.chess_moves(s)
            if shuffle and p >= plies - 6:   # knight-like back and forth: a repetition draw nearby
                m = ms[0] if p % 2 == 0 else ms[-1]
            else:
                m = ms[rng.randrange(len(ms))]
            s = oracle.chess_play(s, m)
        out.append(s)
    return out


def device_rows(states):
    n = len(states)
    rows = np.zeros(n, _native.CHESS_STATE_DTYPE)
    cap = max(1, max(max(s.nhw, s.nhb) for s in states))
    hist = np.zeros((n, 2, cap), np.uint16)
    hlen = np.zeros((n, 2), np.int32)
    for i, s in enumerate(states):
        rows[i]["board"] = list(s.board)
        rows[i]["turn"], rows[i]["fifty"], rows[i]["castle"] = s.turn, s.fifty, s.castle
        for side, (arr, k) in enumerate(((s.hw, s.nhw), (s.hb, s.nhb))):
            for j in range(k):   # oracle: most recent first; device: play order
                m = arr[k - 1 - j]
                hist[i, side, j] = _native.pack_chess_move(m.fr, m.fc, m.tr, m.tc, m.value)
            hlen[i, side] = k
    return rows, hist, hlen


def test_chess_rollouts_match_the_oracle_at_scale():
    rng = random.Random(11)
    states = positions(192, rng)
    rows, hist, hlen = device_rows(states)
    eng = _native.NativeEngine(max_games=1, max_sims=1, max_batch=1)
    eng.seed(0, [4242])
    dev = torch.device("cuda", 0)
    d_rows = torch.from_numpy(rows.view(np.uint8).reshape(len(states), 72).copy()).to(dev)
    d_hist, d_hlen = torch.from_numpy(hist).to(dev), torch.from_numpy(hlen).to(dev)
    vals = torch.zeros(len(states), dtype=torch.float64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    eng.chess_rollouts_async(0, len(states), d_rows.data_ptr(), d_hist.data_ptr(), d_hlen.data_ptr(), hist.shape[2],
                             vals.data_ptr(), status.data_ptr(), s.cuda_stream)
    s.synchronize()
    assert int(status.item()) == 0
    mt = oracle.MT(4242)
    exp, plies = [], 0
    for st in states:
        v, q = oracle.chess_rollout(st, mt)
        assert v != 2
        exp.append(float(v))
        plies += q
    assert vals.cpu().tolist() == exp
    m, idx = eng.get_rng_state(0)
    assert [int(x) for x in m] == list(mt.s.mt) and idx == mt.s.index
    assert plies > 20000 and {-1.0, 0.0, 1.0} <= set(exp)
    eng.close()


def test_chess_rollouts_refuse_a_history_longer_than_its_buffer():
    """A history length above hist_cap: the kernel reports ZC_STATUS_CAPACITY
    instead of rolling out on a truncated history (which would drop the most recent moves, the
    ones the repetition draw reads); a consistent length on the same buffers runs."""
    rng = random.Random(5)
    states = positions(2, rng)
    rows, hist, hlen = device_rows(states)
    eng = _native.NativeEngine(max_games=1, max_sims=1, max_batch=1)
    eng.seed(0, [7])
    dev = torch.device("cuda", 0)
    d_rows = torch.from_numpy(rows.view(np.uint8).reshape(len(states), 72).copy()).to(dev)
    d_hist = torch.from_numpy(hist).to(dev)
    s = torch.cuda.current_stream(dev)
    for over, want in ((True, _native.ZC_STATUS_CAPACITY), (False, 0)):
        bad = hlen.copy()
        if over:
            bad[1, 0] = hist.shape[2] + 1
        d_hlen = torch.from_numpy(bad).to(dev)
        vals = torch.zeros(len(states), dtype=torch.float64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        eng.chess_rollouts_async(0, len(states), d_rows.data_ptr(), d_hist.data_ptr(), d_hlen.data_ptr(),
                                 hist.shape[2], vals.data_ptr(), status.data_ptr(), s.cuda_stream)
        s.synchronize()
        assert int(status.item()) == want, over
    eng.close()
