"""CPU checks behind the §8(b) fallback's device code (no GPU needed).

* The chess rollout kernel keeps has_repeated_prefix(hist, 2, 3) (chess_backend.cpp:148-180)
  incrementally: per side, c_p = the number of trailing i with a[i] == a[i-p] (a = the
  history in play order), updated per push, and the answer "some p >= 2 with c_p >= 2p and
  c_1 < 3p - 1" (chess_search.hip, roll_side_push).  Checked here against the KMP test on
  random and periodic histories, push by push, in the kernel's own update order.
* chess_backend.pack_histories: the device history layout (play order, packed moves).
* oracle.selfplay_batch (bench.py's like-for-like CPU baseline) = the oracle's get_move +
  play + evaluate + refill, move by move.
"""
import random

import numpy as np

import oracle
from zeroclone_amd import _native
from zeroclone_amd.engine.games.chess import chess_backend as cb


class IncrementalRepetition:
    """roll_side_init / roll_side_push of chess_search.hip, restated."""

    def __init__(self, a):
        self.a = list(a)
        n = len(self.a)
        self.cnt = [0] * (n + 2)
        for p in range(1, n + 1):
            c, i = 0, n - 1
            while i >= p and self.a[i] == self.a[i - p]:
                c += 1
                i -= 1
            self.cnt[p] = c
        self.c1 = self.cnt[1] if n >= 1 else 0
        self.rep = any(self.cnt[p] >= 2 * p and self.c1 < 3 * p - 1 for p in range(2, n + 1))

    def push(self, x):
        n = len(self.a)
        self.c1 = self.c1 + 1 if n >= 1 and self.a[n - 1] == x else 0
        hit = False
        for p in range(1, n + 1):
            c = self.cnt[p] + 1 if self.a[n - p] == x else 0
            self.cnt[p] = c
            if p >= 2 and c >= 2 * p and self.c1 < 3 * p - 1:
                hit = True
        self.a.append(x)
        self.cnt.append(0)
        self.rep = hit


def test_incremental_repetition_equals_kmp():
    rng = random.Random(3)
    checked = 0
    for trial in range(400):
        alphabet = rng.choice([2, 3, 4, 6, 20])
        start = [rng.randrange(alphabet) for _ in range(rng.randrange(0, 12))]
        inc = IncrementalRepetition(start)
        assert inc.rep == cb.has_repeated_prefix(list(reversed(start)))
        seq = list(start)
        for _ in range(rng.randrange(1, 40)):
            if rng.random() < 0.5 and len(seq) >= 2:   # periodic continuations make repetitions likely
                x = seq[-rng.choice([1, 2, 3, 4]) if len(seq) >= 4 else -1]
            else:
                x = rng.randrange(alphabet)
            inc.push(x)
            seq.append(x)
            # the deque is most recent first
            assert inc.rep == cb.has_repeated_prefix(list(reversed(seq))), (trial, seq)
            checked += 1
    assert checked > 5000


def test_kmp_quirks_are_kept():
    # a constant run has smallest period 1: never a repetition, however long
    assert not cb.has_repeated_prefix([7] * 30)
    inc = IncrementalRepetition([])
    for _ in range(30):
        inc.push(7)
        assert not inc.rep
    # period 2 three times
    inc = IncrementalRepetition([])
    for x in [1, 2, 1, 2, 1]:
        inc.push(x)
        assert not inc.rep
    inc.push(2)
    assert inc.rep and cb.has_repeated_prefix([2, 1, 2, 1, 2, 1])


def test_pack_histories_play_order():
    s = cb.State([32] * 64, 0, 0, 0, 0, 0, 0, [((6, 4, 4, 4), 0.0), ((7, 6, 5, 5), 0.0)], [((1, 4, 3, 4), 1.0)])
    h, n = cb.pack_histories([s], cap=4)
    assert h.shape == (1, 2, 4) and list(n[0]) == [2, 1]
    assert _native.unpack_chess_move(int(h[0, 0, 0])) == ((7, 6, 5, 5), 0.0)   # oldest first
    assert _native.unpack_chess_move(int(h[0, 0, 1])) == ((6, 4, 4, 4), 0.0)
    assert _native.unpack_chess_move(int(h[0, 1, 0])) == ((1, 4, 3, 4), 1.0)


def test_oracle_selfplay_batch_is_get_move_play_refill():
    boards, turns = [], []
    b, t = "." * 42, 0
    for col in [3, 3, 2, 4, 5, 1, 0, 6, 3]:
        b, t = oracle.play(b, t, col)
    boards = ["." * 42, b, "X" * 0 + b]
    turns = [0, t, t]
    mts = [oracle.MT(11), oracle.MT(12), oracle.MT(13)]
    ref = [oracle.MT(11), oracle.MT(12), oracle.MT(13)]
    oracle.selfplay_batch(boards, turns, mts, 5, 120, 1.4, 16, threads=3)
    for g in range(3):
        bb, tt, m = boards[g], turns[g], ref[g]
        for _ in range(5):
            col, _, _ = oracle.get_move_mt(bb, tt, m, 120, 1.4, 16)
            bb, tt = oracle.play(bb, tt, col)
            if oracle.check_win(bb, tt) or oracle.check_draw(bb):
                bb, tt = "." * 42, 0
        assert m.state() == mts[g].state()


def test_oracle_chess_rollout_is_pinned_to_the_reference():
    """oracle.chess_rollout (chess_oracle.c: zcc_rollout) reproduces every rollout value and
    ply count of the reference's Value('random_rollout') on its chess backend
    (tests/golden/fallback_get_move.json, chess_rollouts) and the stream afterwards."""
    import json
    import os
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "fallback_get_move.json")))
    n = 0
    for case in fx["chess_rollouts"]:
        mt = oracle.MT(case["seed"])
        for e, v, q in zip(case["states"], case["values"], case["plies"]):
            assert oracle.chess_rollout(oracle.chess_from_json(e), mt) == (v, q)
            n += 1
        assert mt.u32() == case["next_word"]
    assert n >= 30
