"""GPU tests of the Connect4 search's Philox rollout mode (ZC_ROLLOUT_PHILOX; SURVEY §8(d)
C2(ii) "rollout fast mode"): exact against its specification (the oracle's search driven by
tests/c4_philox_ref.py values — expansions on the game's MT stream, playouts on per-leaf
Philox-seeded streams), and in distribution against the exact (reference-stream) mode."""
import numpy as np
import pytest

import oracle
from c4_philox_ref import value_batch

pytestmark = pytest.mark.gpu

SEED = 0x5EED_0C4F_2024


@pytest.fixture(scope="module")
def eng():
    from zeroclone_amd._native import NativeEngine
    e = NativeEngine(max_games=4096, max_sims=800, max_batch=64)
    yield e
    e.close()


def _roots(cases):
    from zeroclone_amd._native import C4_STATE_DTYPE, c4_from_rows
    out = np.zeros(len(cases), C4_STATE_DTYPE)
    for i, (b, t) in enumerate(cases):
        out[i] = c4_from_rows(b, t)
    return out


MID = ("......." "......." "...O..." "...X..." "..XO..." ".OXXO..")
NEAR_WIN = ("......." "......." "......." "X......" "XO....." "XO.O...")  # X to move wins at column 0


@pytest.mark.parametrize("sims,bs", [(200, 32), (97, 8), (64, 64)])
def test_philox_search_is_its_specification(eng, sims, bs):
    cases = [("." * 42, 0), (MID, 0), (NEAR_WIN, 0)] * 4
    seeds = [31 + 7 * i for i in range(len(cases))]
    eng.c4_rollout_mode("philox", SEED)
    try:
        eng.seed(0, seeds)
        mv, na, st = eng.c4_search(_roots(cases), sims, 1.4, bs)
        mv2, na2, st2 = eng.c4_search(_roots(cases), sims, 1.4, bs)  # next move: a new Philox tag
    finally:
        eng.c4_rollout_mode("exact")
    for i, (board, turn) in enumerate(cases):
        mt = oracle.MT(seeds[i])
        col, rna, order = oracle.get_move_valued(board, turn, mt, sims, 1.4, bs, value_batch(624, i, SEED))
        assert [int(na[i, c]) for c in order] == rna, i
        assert int(mv[i]) == col
        assert int(st["rng_words"][i]) == mt.drawn - 0  # expansion draws only
        tag = 624 + mt.drawn
        col2, rna2, order2 = oracle.get_move_valued(board, turn, mt, sims, 1.4, bs, value_batch(tag, i, SEED))
        assert [int(na2[i, c]) for c in order2] == rna2, i
        assert int(mv2[i]) == col2


def test_philox_mode_matches_exact_mode_in_distribution(eng):
    """4096 games x 800 sims from the empty board: the mean root visit distribution of the
    Philox mode against the exact mode, compared with the spread between two exact runs on
    disjoint seeds."""
    from zeroclone_amd._native import C4_STATE_DTYPE
    G, S = 4096, 800
    roots = np.zeros(G, C4_STATE_DTYPE)

    def mean_dist(mode, seed0):
        eng.c4_rollout_mode(mode, SEED + seed0)
        try:
            eng.seed(0, list(range(seed0, seed0 + G)))
            _, na, _ = eng.c4_search(roots, S, 1.4, 32)
        finally:
            eng.c4_rollout_mode("exact")
        d = na / na.sum(axis=1, keepdims=True)
        return d.mean(axis=0)

    ex_a = mean_dist("exact", 0)
    ex_b = mean_dist("exact", 10_000)
    ph = mean_dist("philox", 20_000)
    noise = np.abs(ex_a - ex_b).sum()
    l1 = np.abs(ph - (ex_a + ex_b) / 2).sum()
    print("L1 philox vs exact", l1, "exact vs exact", noise, ph, ex_a)
    assert l1 < max(4 * noise, 0.01)
