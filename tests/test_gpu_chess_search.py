"""GPU parity of the chess tree search (chess_search.hip): crude_chess_score searches
against the reference's own get_move outputs (tests/golden/chess_get_move.json), and the
stepwise search with caller values against the oracle (hash values; fp16 network values
replayed flush by flush)."""
import random
from collections import defaultdict

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
MAXM = 256


@pytest.fixture(scope="module")
def eng():
    from zeroclone_amd._native import NativeEngine
    e = NativeEngine(max_games=64, max_sims=512, max_batch=64)
    yield e
    e.close()


def roots_of(fens):
    from zeroclone_amd._native import CHESS_STATE_DTYPE, chess_from_fen
    a = np.array([chess_from_fen(f) for f in fens], CHESS_STATE_DTYPE)
    return torch.from_numpy(a.view(np.uint8).reshape(len(fens), 72).copy()).cuda()


def decode(m):
    from zeroclone_amd._native import unpack_chess_move
    (fr, fc, tr, tc), v = unpack_chess_move(int(m) & 0xFFFF)
    return [fr, fc, tr, tc, v]


def test_crude_search_matches_reference(eng, golden):
    from zeroclone_amd._native import ZC_POLICY_IMMEDIATE_VALUE, ZC_POLICY_RANDOM
    groups = defaultdict(list)
    for c in golden("chess_get_move.json")["cases"]:
        groups[(c["sims"], c["bs"], c["c"], c["policy"], c["freedom"])].append(c)
    for (sims, bs, cc, pol, fr), grp in groups.items():
        n = len(grp)
        eng.seed(0, [c["seed"] for c in grp])
        roots = roots_of([c["fen"] for c in grp])
        mv = torch.zeros(n, dtype=torch.int16, device="cuda")
        na = torch.zeros((n, MAXM), dtype=torch.int32, device="cuda")
        st = torch.zeros((n, 8), dtype=torch.int64, device="cuda")
        eng.chess_search_async(0, n, roots.data_ptr(), sims, cc, bs,
                               ZC_POLICY_IMMEDIATE_VALUE if pol == "immediate_value" else ZC_POLICY_RANDOM, fr,
                               mv.data_ptr(), na.data_ptr(), st.data_ptr())
        torch.cuda.synchronize()
        mv, na, st = mv.cpu().numpy(), na.cpu().numpy(), st.cpu().numpy()
        for i, c in enumerate(grp):
            k = len(c["root_moves"])
            assert st[i, 5] == 0, (c["fen"], st[i])
            assert list(na[i, :k]) == c["root_na"], c["fen"]
            assert decode(mv[i]) == c["move"]
            assert st[i, 4] == c["consumed"]
            mt, idx = eng.get_rng_state(i)
            r = random.Random()
            r.setstate((3, tuple(int(x) for x in mt) + (idx,), None))
            assert r.getrandbits(32) == c["next_word"]


M64 = (1 << 64) - 1


def board_hash_value(board: bytes, turn: int) -> float:
    h = 0x84222325CBF29CE4
    for b in board:
        h = ((h ^ b) * 0x100000001B3) & M64
    h = (h ^ (turn * 0x9E3779B97F4A7C15)) & M64
    h ^= h >> 31
    return ((h % 400001) - 200000) / 200003.0


FENS = ["rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
        "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1",
        "8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1",
        "r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1"]


@pytest.mark.parametrize("policy", ["random", "immediate_value"])
def test_stepwise_search_with_hash_values_matches_oracle(eng, policy):
    from zeroclone_amd._native import ZC_POLICY_IMMEDIATE_VALUE, ZC_POLICY_RANDOM
    from zeroclone_amd.valued import ChessValuedSearch
    fens = FENS * 4
    n, sims, bs = len(fens), 200, 16
    seeds = [50 + i for i in range(n)]
    eng.seed(0, seeds)
    pol = ZC_POLICY_IMMEDIATE_VALUE if policy == "immediate_value" else ZC_POLICY_RANDOM

    def fn(leaves, planes, counts):
        rows = leaves.cpu().numpy()
        return torch.tensor([board_hash_value(bytes(r[:64]), int(r[64])) for r in rows], dtype=torch.float64).cuda()

    vs = ChessValuedSearch(eng, n, bs, policy=pol, freedom=3.0)
    mv, na, st = vs.run(roots_of(fens), sims, 1.4, fn)
    mv, na, st = mv.cpu().numpy(), na.cpu().numpy(), st.cpu().numpy()
    for i, fen in enumerate(fens):
        mt = oracle.MT(seeds[i])
        best, moves, rna = oracle.chess_get_move(oracle.chess_from_fen(fen), mt, sims, 1.4, bs, policy, 3.0,
                                                 value_batch=lambda ls: [board_hash_value(b, t) for b, t, _, _ in ls])
        assert st[i, 5] == 0
        assert list(na[i, :len(moves)]) == rna, fen
        assert decode(mv[i]) == list(moves[best])
        assert st[i, 4] == mt.drawn


def test_network_values_replay_into_oracle(eng):
    """chess_value.yaml path: fp16 ValueNetwork(17 planes) on the device planes, values
    replayed into the oracle search flush by flush — the searches must agree exactly."""
    from zeroclone_amd.nets import ValueNetwork, for_inference
    from zeroclone_amd.valued import ChessValuedSearch, NetValue
    torch.manual_seed(0)
    net = NetValue(for_inference(ValueNetwork(32, 2).eval(), "cuda", torch.float16))
    fens = FENS * 2
    n, sims, bs = len(fens), 128, 32
    seeds = [7 + i for i in range(n)]
    eng.seed(0, seeds)
    log = []

    def fn(leaves, planes, counts):
        v = net(leaves, planes, counts)
        log.append(v.cpu().numpy().copy())
        return v

    mv, na, st = ChessValuedSearch(eng, n, bs).run(roots_of(fens), sims, 1.4, fn)
    na = na.cpu().numpy()
    for i, fen in enumerate(fens):
        it = iter(range(len(log)))

        def replay(ls, i=i, it=it):
            f = next(it)
            return [float(x) for x in log[f][i * bs: i * bs + len(ls)]]

        best, moves, rna = oracle.chess_get_move(oracle.chess_from_fen(fen), oracle.MT(seeds[i]), sims, 1.4, bs,
                                                 "random", 0.0, value_batch=replay)
        assert list(na[i, :len(moves)]) == rna, fen


def test_planes_of_leaves(eng):
    from zeroclone_amd.engine.games.chess import chess_backend as cb
    from zeroclone_amd.valued import ChessValuedSearch
    n, bs = 4, 8
    eng.seed(0, list(range(n)))
    seen = []

    def fn(leaves, planes, counts):
        seen.append((leaves.cpu().numpy().copy(), planes.float().cpu().numpy().copy()))
        return torch.zeros(n * bs, dtype=torch.float64, device="cuda")

    ChessValuedSearch(eng, n, bs).run(roots_of(FENS), 16, 1.4, fn)
    from zeroclone_amd._native import CHESS_STATE_DTYPE
    for rows, pl in seen:
        for k in range(0, rows.shape[0], 3):
            st = cb.from_zc(rows[k].view(CHESS_STATE_DTYPE)[0])
            np.testing.assert_array_equal(pl[k], cb.state_to_tensor(st))


def test_rng_state_after_chess_search_is_pythons(eng):
    """zc_rng_get_state after searches that generate their stream only as far as they read
    (the HBM-ring searches: chess, the stepwise Connect4 search): the returned state is
    CPython's — the whole 624-word block of the last consumed word, twisted — for every game,
    across several consecutive searches (random.getstate after as many draws)."""
    fens = ["rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
            "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1"] * 8
    n = len(fens)
    seeds = [31 * g + 5 for g in range(n)]
    eng.seed(0, seeds)
    roots = roots_of(fens)
    mv = torch.zeros(n, dtype=torch.int16, device="cuda")
    na = torch.zeros((n, 256), dtype=torch.int32, device="cuda")
    st = torch.zeros((n, 8), dtype=torch.int64, device="cuda")
    used = [0] * n
    for sims in (37, 64, 101):
        eng.chess_search_async(0, n, roots.data_ptr(), sims, 1.4, 16, 0, 0.0, mv.data_ptr(), na.data_ptr(),
                               st.data_ptr())
        torch.cuda.synchronize()
        for g in range(n):
            used[g] += int(st[g, 4])
            r = random.Random(seeds[g])
            for _ in range(used[g]):
                r.getrandbits(32)
            want = r.getstate()[1]
            mt, idx = eng.get_rng_state(g)
            assert [int(x) for x in mt] == list(want[:624]) and idx == want[624], (sims, g)


CROWDED = ["qqqqkqqq/8/8/8/8/8/8/QQQQKQQQ w - - 0 1",   # ~100 moves a side: the slot pool runs out
           "qqqqkqqq/8/8/8/8/8/8/QQQQKQQQ b - - 0 1"]


def _crude_value(rows):
    """crude_chess_score (value_functions.py:48-55) of leaf rows on the host, as the fused
    kernel scores them: 1000 for the side to move checkmated, else the material for it."""
    vals = {"P": 1, "N": 3, "B": 3, "R": 5, "Q": 9}
    out = []
    for r in rows:
        st = oracle.chess_state(bytes(r[:64]).decode("latin-1"), int(r[64]), int(r[65]), int(r[66]))
        if oracle.chess_win(st):
            out.append(1000.0)
            continue
        mat = sum(vals.get(chr(b).upper(), 0) * (1 if chr(b).isupper() else -1) for b in r[:64] if chr(b) != " ")
        out.append(float(mat if st.turn == 0 else -mat))
    return out


@pytest.mark.parametrize("sims", [200, 500])
def test_paired_crude_search_equals_the_stepwise_one(eng, sims):
    """The fused crude search pairs consecutive expansions of one node across two waves
    (chess_search.hip Helper); the stepwise search (zc_chess_ext_*, one wave) does not.  With
    the crude score computed on the host for the stepwise one, both must build the same tree:
    root visits, move, counters and MT words.  Both create nodes lazily (a legal-move probe at
    creation, the list generated at a node's first expansion), so the crowded boards at 500
    simulations (~80-100 moves a node against 64 slots a node), which ran the eager searches
    out of slots (ZC_STATUS_CAPACITY) before round 6, now complete: slots go to expanded nodes
    only (~6 % of the nodes of a 400-simulation chess search)."""
    from zeroclone_amd._native import ZC_POLICY_IMMEDIATE_VALUE, ZC_STATUS_CAPACITY
    from zeroclone_amd.valued import ChessValuedSearch
    fens = FENS * 2 + CROWDED * 2
    n, bs = len(fens), 32
    seeds = [300 + i for i in range(n)]
    roots = roots_of(fens)
    eng.seed(0, seeds)
    mv = torch.zeros(n, dtype=torch.int16, device="cuda")
    na = torch.zeros((n, MAXM), dtype=torch.int32, device="cuda")
    st = torch.zeros((n, 8), dtype=torch.int64, device="cuda")
    eng.chess_search_async(0, n, roots.data_ptr(), sims, 1.4, bs, ZC_POLICY_IMMEDIATE_VALUE, 3.0, mv.data_ptr(),
                           na.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    fused = (mv.cpu().numpy(), na.cpu().numpy(), st.cpu().numpy())
    eng.seed(0, seeds)

    def fn(leaves, planes, counts):
        return torch.tensor(_crude_value(leaves.cpu().numpy()), dtype=torch.float64).cuda()

    vs = ChessValuedSearch(eng, n, bs, planes=False, policy=ZC_POLICY_IMMEDIATE_VALUE, freedom=3.0)
    smv, sna, sst = (x.cpu().numpy() for x in vs.run(roots, sims, 1.4, fn))
    fmv, fna, fst = fused
    assert int((sst[:, 5] == ZC_STATUS_CAPACITY).sum()) == 0, [list(r) for r in sst]
    assert int((fst[:, 5] != 0).sum()) == 0, [list(r) for r in fst]
    for i, fen in enumerate(fens):
        assert list(fst[i, [0, 1, 4, 5]]) == list(sst[i, [0, 1, 4, 5]]), (fen, fst[i], sst[i])
        assert list(fna[i]) == list(sna[i]), fen
        assert fmv[i] == smv[i], fen


def test_short_last_flush_runs_the_network_on_its_leaves_only(eng):
    """sims not a multiple of the batch: NetValue.rows evaluates the last flush's n*nb boards
    only (valued.ChessValuedSearch); the search must equal the one that evaluates all n*bs
    slots (the same network called through a plain function)."""
    from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork
    from zeroclone_amd.valued import ChessValuedSearch, NetValue
    torch.manual_seed(3)
    net = NetValue(MfmaValueNetwork(ValueNetwork(128, 2).eval(), "cuda"))
    fens = FENS * 3
    n, sims, bs = len(fens), 100, 32   # the last flush holds 4 leaves a game
    seeds = [40 + i for i in range(n)]
    calls = []

    def full(leaves, planes, counts):
        calls.append(planes.shape[0])
        return net(leaves, planes, counts)

    outs = []
    for fn in (net, full):
        eng.seed(0, seeds)
        vs = ChessValuedSearch(eng, n, bs)
        outs.append([x.cpu().numpy().copy() for x in vs.run(roots_of(fens), sims, 1.4, fn)])
    assert calls == [n * bs] * 4
    for a, b in zip(*outs):
        assert (a == b).all()
    assert (outs[0][2][:, 5] == 0).all() and (outs[0][2][:, 0] == sims).all()


@pytest.mark.parametrize("bs", [64, 128])
def test_crude_search_large_flushes_match_oracle(bs):
    """The fused crude search's backup (chess_search.hip crude_values_backup) aggregates a
    flush's edges in an LDS hash table, and keeps the leaf-by-leaf backup for flushes of more
    than 64 leaves or with more (leaf, level) pairs than half the table.  Flushes of 64 leaves
    (the table, or leaf by leaf past half of it on the endgames' deep trees) and of 128 (leaf
    by leaf), against the oracle's get_move: root visits, move and the words drawn."""
    from zeroclone_amd._native import ZC_POLICY_IMMEDIATE_VALUE, NativeEngine
    fens = FENS * 2 + ["8/8/3k4/8/8/3K4/3Q4/8 w - - 0 1", "6k1/5ppp/8/8/8/8/5PPP/3R2K1 w - - 0 1",
                       "8/8/8/4k3/8/8/8/R3K3 w - - 0 1", "7k/8/8/8/8/8/8/K6Q w - - 0 1"]
    n, sims = len(fens), 400
    e = NativeEngine(max_games=n, max_sims=sims, max_batch=bs)
    try:
        seeds = [90 + i for i in range(n)]
        e.seed(0, seeds)
        roots = roots_of(fens)
        mv = torch.zeros(n, dtype=torch.int16, device="cuda")
        na = torch.zeros((n, MAXM), dtype=torch.int32, device="cuda")
        st = torch.zeros((n, 8), dtype=torch.int64, device="cuda")
        e.chess_search_async(0, n, roots.data_ptr(), sims, 1.4, bs, ZC_POLICY_IMMEDIATE_VALUE, 3.0, mv.data_ptr(),
                             na.data_ptr(), st.data_ptr())
        torch.cuda.synchronize()
        mv, na, st = mv.cpu().numpy(), na.cpu().numpy(), st.cpu().numpy()
        for i, fen in enumerate(fens):
            mt = oracle.MT(seeds[i])
            best, moves, rna = oracle.chess_get_move(oracle.chess_from_fen(fen), mt, sims, 1.4, bs, "immediate_value",
                                                     3.0)
            assert st[i, 5] == 0, (fen, st[i])
            assert list(na[i, :len(moves)]) == rna, fen
            assert decode(mv[i]) == list(moves[best]), fen
            assert st[i, 4] == mt.drawn, fen
    finally:
        e.close()
