"""GPU parity tests: the HIP search path (through the C-ABI) against the reference's golden
outputs and the oracle.  The bar is bit-exact: root visit counts, chosen move and the exact
number of MT19937 words consumed."""
import ctypes
import ctypes.util
import math
import random
from collections import defaultdict

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from zeroclone_amd._native import NativeEngine
    e = NativeEngine(max_games=4096, max_sims=1600, max_batch=128)
    yield e
    e.close()


def to_state(board, turn):
    from zeroclone_amd._native import c4_from_rows
    return c4_from_rows(board, turn)


def states(cases):
    from zeroclone_amd._native import C4_STATE_DTYPE
    out = np.zeros(len(cases), C4_STATE_DTYPE)
    for i, c in enumerate(cases):
        out[i] = to_state(c["board"], c["turn"])
    return out


def test_uct_is_bitwise_the_reference_arithmetic(eng):
    libm = ctypes.CDLL(ctypes.util.find_library("m"))
    libm.fma.restype = ctypes.c_double
    libm.fma.argtypes = [ctypes.c_double] * 3
    rng = np.random.default_rng(0)
    n = 200_000
    N = rng.integers(1, 70000, n)
    na = np.minimum(rng.integers(0, 70000, n), N)
    na[:1000] = 0
    w = rng.integers(-1, 2, n) * rng.integers(0, 70000, n)
    logn = np.log(N.astype(np.float64))
    q = np.where(na > 0, w / np.maximum(na, 1), 0.0)
    for c in (1.4, 0.0, 2.5, 1.25, 0.7071):
        got = eng.debug_uct(logn, na, q, c)
        for i in range(0, n, 97):
            exp = math.inf if na[i] == 0 else libm.fma(c, math.sqrt(logn[i] / float(na[i])), q[i])
            assert got[i] == exp or (math.isnan(got[i]) and math.isnan(exp)), (i, got[i], exp)
        # vectorised full comparison via numpy (its fma-free path is only a cross-check on c=0)
        if c == 0.0:
            assert np.array_equal(got[na > 0], q[na > 0])


def test_rollouts_match_reference(eng, golden):
    cases = golden("c4_rollout.json")["cases"]
    eng.seed(0, [c["seed"] for c in cases])
    v, words = eng.debug_c4_rollout(states(cases))
    assert [int(x) for x in v] == [c["value"] for c in cases]
    assert [int(x) for x in words] == [c["consumed"] for c in cases]


def test_sequential_rollouts_stress_block_logic(eng):
    """Thousands of rollouts back to back on ONE stream (value.batch order), from positions of
    every depth — many with full or nearly full columns, won and drawn boards included — so
    that blocks cross stream windows and absorb column fills (one or two per block, ply-30
    caps, board-full draws) in every combination.  Each value and the stream position after
    the whole sequence must equal the oracle's."""
    rng = random.Random(2024)
    boards = []
    while len(boards) < 3000:
        b, t = "." * 42, 0
        depth = rng.randint(0, 42)
        lean = rng.sample(range(7), rng.randint(1, 7))  # columns the game prefers: fills come early
        for _ in range(depth):
            legal = [col for col in range(7) if b[col] == "."]
            if not legal:
                break
            pref = [col for col in legal if col in lean]
            col = rng.choice(pref if pref and rng.random() < 0.8 else legal)
            b, t = oracle.play(b, t, col)
            if oracle.check_win(b, t) and rng.random() < 0.7:
                break
        boards.append((b, t))
    seed = 77
    mt = oracle.MT(seed)
    exp = []
    for b, t in boards:
        exp.append(oracle.lib().zco_rollout(b.encode(), t, ctypes.byref(mt.s)))
    eng.seed(3, [seed])
    got, words = eng.c4_rollouts(states([{"board": b, "turn": t} for b, t in boards]), game=3)
    assert [int(x) for x in got] == exp
    assert words == mt.drawn


def test_get_move_matches_reference(eng, golden):
    cases = golden("c4_get_move.json")["cases"]
    groups = defaultdict(list)
    for c in cases:
        groups[(c["sims"], c["bs"], c["c"])].append(c)
    for (sims, bs, cc), cs in groups.items():
        eng.seed(0, [c["seed"] for c in cs])
        mv, na, st = eng.c4_search(states(cs), sims, cc, bs)
        for i, c in enumerate(cs):
            assert [int(na[i][col]) for col in c["order"]] == c["root_na"], (c["seed"], sims, bs)
            assert int(mv[i]) == c["move"]
            assert int(st[i]["rng_words"]) == c["consumed"]
            assert int(st[i]["leaves"]) == sims


def test_rng_state_roundtrips_through_python(eng, golden):
    c = golden("c4_get_move.json")["cases"][40]
    eng.seed(5, [c["seed"]])
    eng.c4_search(states([c]), c["sims"], c["c"], c["bs"], first_game=5)
    mt, idx = eng.get_rng_state(5)
    r = random.Random(c["seed"])
    for _ in range(c["consumed"]):
        r.getrandbits(32)
    st = r.getstate()[1]
    assert list(mt) == list(st[:624]) and idx == st[624]
    # and back: setstate into another game continues the same stream
    eng.set_rng_state(6, mt, idx)
    a = eng.debug_c4_rollout(states([c]), first_game=6)
    eng.set_rng_state(7, mt, idx)
    b = eng.debug_c4_rollout(states([c]), first_game=7)
    assert a[0][0] == b[0][0] and a[1][0] == b[1][0]


def test_selfplay_games_match_reference(eng, golden):
    games = golden("c4_selfplay.json")["games"]
    from zeroclone_amd._native import C4_STATE_DTYPE
    eng.seed(0, [g["seed"] for g in games])
    boards = [("." * 42, 0) for _ in games]
    moves = [[] for _ in games]
    live = list(range(len(games)))
    words = [0] * len(games)
    while live:
        # search only live games: one call per game keeps game index == engine slot
        for gi in list(live):
            b, t = boards[gi]
            mv, na, st = eng.c4_search(states([{"board": b, "turn": t}]), 100, 1.4, 32, first_game=gi)
            words[gi] += int(st[0]["rng_words"])
            moves[gi].append(int(mv[0]))
            boards[gi] = oracle.play(b, t, int(mv[0]))
            nb, nt = boards[gi]
            if oracle.check_win(nb, nt) or oracle.check_draw(nb):
                live.remove(gi)
    for gi, g in enumerate(games):
        assert moves[gi] == g["moves"]
        assert words[gi] == g["consumed"]


def test_full_size_batch_matches_oracle(eng):
    """C2 shape: 4096 games x 800 sims, bs 32 — every game compared with the oracle."""
    n, sims = 4096, 800
    rng = random.Random(11)
    boards = []
    for g in range(n):
        b, t = "." * 42, 0
        for _ in range(rng.randint(0, 6)):
            legal = [col for col in range(7) if b[col] == "."]
            b, t = oracle.play(b, t, rng.choice(legal))
        boards.append((b, t))
    # drop positions that are already won (still legal for get_move, but keep the mix simple)
    seeds = [1_000_003 * g + 17 for g in range(n)]
    eng.seed(0, seeds)
    from zeroclone_amd._native import C4_STATE_DTYPE
    st = np.zeros(n, C4_STATE_DTYPE)
    for i, (b, t) in enumerate(boards):
        st[i] = to_state(b, t)
    mv, na, stats = eng.c4_search(st, sims, 1.4, 32)
    omv, ona, ocons = oracle.get_move_batch([b for b, _ in boards], [t for _, t in boards], seeds, sims, 1.4, 32,
                                            threads=16)
    assert np.array_equal(mv, omv)
    assert np.array_equal(na, ona)
    assert np.array_equal(stats["rng_words"], ocons.astype(np.int64))
    assert (stats["leaves"] == sims).all() and (stats["status"] == 0).all()


@pytest.mark.parametrize("bs", [1, 2, 7, 8, 13, 32, 63, 64, 100])
def test_planned_flush_deep_roots_match_oracle(eng, bs):
    """The planned flush (select_flush_plan, batch sizes < 64; select_flush at 64 and up) from
    deep roots: chains that reach a full board (a terminal chain node takes the rest of the
    flush's leaves), nodes with one to seven moves, fills on the chain, draws spanning views.
    Every game's move, root visits and stream words equal the oracle's."""
    n, sims = 768, 240
    rng = random.Random(500 + bs)
    boards = []
    while len(boards) < n:
        b, t = "." * 42, 0
        lean = rng.sample(range(7), rng.randint(1, 3))  # columns filled first: chains hit full columns
        ok = True
        for _ in range(rng.randint(18, 41)):
            legal = [col for col in range(7) if b[col] == "."]
            pref = [col for col in legal if col in lean]
            b, t = oracle.play(b, t, rng.choice(pref if pref and rng.random() < 0.7 else legal))
            if oracle.check_win(b, t):
                ok = rng.random() < 0.1  # a few already-won roots stay (get_move still searches them)
                break
        if ok and not oracle.check_draw(b):
            boards.append((b, t))
    seeds = [7919 * g + bs for g in range(n)]
    eng.seed(0, seeds)
    from zeroclone_amd._native import C4_STATE_DTYPE
    st = np.zeros(n, C4_STATE_DTYPE)
    for i, (b, t) in enumerate(boards):
        st[i] = to_state(b, t)
    mv, na, stats = eng.c4_search(st, sims, 1.4, bs)
    omv, ona, ocons = oracle.get_move_batch([b for b, _ in boards], [t for _, t in boards], seeds, sims, 1.4, bs,
                                            threads=16)
    assert np.array_equal(mv, omv)
    assert np.array_equal(na, ona)
    assert np.array_equal(stats["rng_words"], ocons.astype(np.int64))


def test_invalid_roots_raise(eng):
    full = "XOXOXOX" * 6
    with pytest.raises(ValueError):
        eng.c4_search(states([{"board": full, "turn": 0}]), 10)
    with pytest.raises(ValueError):
        eng.c4_search(states([{"board": "." * 42, "turn": 0}]), 0)
    with pytest.raises(ValueError):
        eng.c4_search(states([{"board": "." * 42, "turn": 0}]), 10, batch_size=0)
