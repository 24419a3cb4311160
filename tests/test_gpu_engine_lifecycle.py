"""Engine lifecycle on the device: engines created and destroyed back to back (the arena is
one device allocation; streams and pinned staging blocks go back to per-process pools,
engine.hip take_stream / take_pinned) and engines alive at once, searched from concurrent
threads, give the searches a fresh engine gives — and the C port's moves."""
import threading

import numpy as np
import pytest

import oracle
from zeroclone_amd import _native

pytestmark = pytest.mark.gpu

SIMS, BS, N = 200, 32, 8


def _search(eng, games=range(N)):
    roots = np.zeros(len(games), _native.C4_STATE_DTYPE)  # the opening, X to move
    return eng.c4_search_games(list(games), roots, SIMS, 1.4, BS)


def _fresh(max_games=64):
    return _native.NativeEngine(max_games=max_games, max_sims=SIMS, max_batch=BS, device=0)


def test_engines_created_and_destroyed_back_to_back_search_alike():
    e = _fresh()
    ref = _search(e)
    e.close()
    assert (ref[1].sum(axis=1) == SIMS).all()
    # game g starts as random.seed(g): the C port from the same stream picks the same column
    for g in range(4):
        col, _, _ = oracle.get_move_mt("." * 42, 0, oracle.MT(g), SIMS, 1.4, BS)
        assert int(ref[0][g]) == col
    # capacities up and down: a smaller engine takes a larger pooled pinned block, a larger
    # one allocates its own; the games' streams depend on their index only
    for cap in [64, 8, 4096, 8, 64] * 4:
        e = _fresh(cap)
        got = _search(e)
        e.close()
        np.testing.assert_array_equal(got[0], ref[0])
        np.testing.assert_array_equal(got[1], ref[1])
        np.testing.assert_array_equal(got[2]["expansions"], ref[2]["expansions"])


def test_live_engines_searched_from_threads_match_serial_searches():
    engines = [_fresh() for _ in range(3)]
    serial = [_search(e) for e in engines]
    for e in engines:  # every engine's games back to their seeds (the searches moved them on)
        e.seed(0, list(range(64)))
    expect = [[_search(e) for _ in range(4)] for e in engines]
    for e in engines:
        e.seed(0, list(range(64)))
    got = [[] for _ in engines]
    errors = []

    def run(i):
        try:
            for _ in range(4):
                got[i].append(_search(engines[i]))
        except Exception as exc:  # noqa: BLE001  (re-raised below, on the test's thread)
            errors.append(exc)

    threads = [threading.Thread(target=run, args=(i,)) for i in range(len(engines))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    for i in range(len(engines)):
        np.testing.assert_array_equal(expect[i][0][0], serial[i][0])
        for k in range(4):
            np.testing.assert_array_equal(got[i][k][0], expect[i][k][0])
            np.testing.assert_array_equal(got[i][k][1], expect[i][k][1])
    for e in engines:
        e.close()
