"""Full-shape parity of the network search modes (BASELINE configs C2(iii), C4, C5 per GPU),
with the hand-written MFMA tower in the loop.

The searches are exact given their leaf values (and, for PUCT, priors), so each test runs
the whole configuration on the device with a random-init fp16 network, logs what the
network returned, and replays it into the CPU specification for sampled games:
  * C2(iii) — Connect4, 4096 games x 800 sims, ValueNetwork(128, 8, in_planes=2): the
    oracle's valued get_move (oracle/c4_oracle.c, = mcts.cpp:102-160 with Value.batch as a
    callback) must reproduce every sampled game's root visit counts and move;
  * C4 — chess (configs/chess_value.yaml), 1024 games x 400 sims, ValueNetwork(128, 8): the
    oracle's chess get_move with the logged values, root Na exact;
  * C5 per GPU — chess PUCT, 1024 games x 1600 sims, policy + value network, Dirichlet root
    noise: tests/puct_ref.py with the logged values and the device's priors must reproduce
    the root visit counts; the priors are the softmax of the logged logits (fp32 tolerance),
    and the root noise has Dirichlet(0.3) statistics across the 1024 games.
Reference: engine/value_functions.py:61-99 (network values), models/chess_value/network.py:24-45.
"""
import numpy as np
import pytest
import torch

import oracle
from oracle import puct_ref

pytestmark = pytest.mark.gpu

START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"


def _sample(n, k):
    return sorted({int(round(x)) for x in np.linspace(0, n - 1, k)})


def _chess_roots(n, fen=START):
    from zeroclone_amd._native import CHESS_STATE_DTYPE, chess_from_fen
    a = np.array([chess_from_fen(fen)] * n, CHESS_STATE_DTYPE)
    return torch.from_numpy(a.view(np.uint8).reshape(n, 72).copy()).cuda()


def test_c2iii_connect4_value_net_full_shape():
    from zeroclone_amd._native import NativeEngine
    from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork, for_inference
    from zeroclone_amd.valued import C4ValuedSearch, NetValue
    G, sims, bs = 4096, 800, 32
    torch.manual_seed(11)
    model = for_inference(ValueNetwork(128, 8, in_planes=2).eval(), "cuda", torch.float16)
    assert isinstance(model, MfmaValueNetwork)   # the hand-written MFMA tower, not MIOpen
    eng = NativeEngine(max_games=G, max_sims=sims, max_batch=bs)
    seeds = [1000 + g for g in range(G)]
    eng.seed(0, seeds)
    net = NetValue(model)
    log = []

    def fn(leaves, planes, counts):
        v = net(leaves, planes, counts)
        log.append((v.cpu().numpy().copy(), counts.cpu().numpy().copy()))
        return v

    roots = torch.zeros((G, 3), dtype=torch.int64, device="cuda")
    mv, na, st = C4ValuedSearch(eng, G, bs).run(roots, sims, 1.4, fn)
    mv, na, st = mv.cpu().numpy(), na.cpu().numpy(), st.cpu().numpy()
    eng.close()
    assert (st[:, 5] == 0).all() and (na.sum(axis=1) == sims).all()
    assert len(log) == (sims + bs - 1) // bs
    assert np.unique(np.round(log[-1][0], 6)).size > 20   # not a constant network
    for i in _sample(G, 16):
        it = iter(range(len(log)))

        def replay(boards, turns, i=i, it=it):
            vals, cnt = log[next(it)]
            assert cnt[i] == len(boards)
            return [float(x) for x in vals[i * bs: i * bs + len(boards)]]

        col, rna, order = oracle.get_move_valued("." * 42, 0, oracle.MT(seeds[i]), sims, 1.4, bs, replay)
        assert [int(na[i, c]) for c in order] == rna, i
        assert int(mv[i]) == col


def test_c4_chess_value_net_full_shape():
    from zeroclone_amd._native import NativeEngine
    from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork, for_inference
    from zeroclone_amd.valued import ChessValuedSearch, NetValue
    G, sims, bs = 1024, 400, 32
    torch.manual_seed(12)
    model = for_inference(ValueNetwork(128, 8).eval(), "cuda", torch.float16)
    assert isinstance(model, MfmaValueNetwork)
    eng = NativeEngine(max_games=G, max_sims=sims, max_batch=bs)
    seeds = [2000 + g for g in range(G)]
    eng.seed(0, seeds)
    net = NetValue(model)
    log = []

    def fn(leaves, planes, counts):
        v = net(leaves, planes, counts)
        log.append(v.cpu().numpy().copy())
        return v

    mv, na, st = ChessValuedSearch(eng, G, bs).run(_chess_roots(G), sims, 1.4, fn)
    na, st = na.cpu().numpy(), st.cpu().numpy()
    eng.close()
    assert (st[:, 5] == 0).all() and (na.sum(axis=1) == sims).all()
    assert np.unique(np.round(log[-1], 6)).size > 20
    root = oracle.chess_from_fen(START)
    for i in _sample(G, 16):
        it = iter(range(len(log)))

        def replay(ls, i=i, it=it):
            return [float(x) for x in log[next(it)][i * bs: i * bs + len(ls)]]

        best, moves, rna = oracle.chess_get_move(root, oracle.MT(seeds[i]), sims, 1.4, bs, "random", 0.0,
                                                 value_batch=replay)
        assert list(na[i, :len(moves)]) == rna, i


def _key_zcc(s):
    return bytes(s.board), int(s.turn), int(s.fifty), int(s.castle)


def _key_row(r):
    r = bytes(r)
    return r[:64], r[64], r[65], r[66]


def test_c5_chess_puct_full_shape():
    from zeroclone_amd._native import NativeEngine
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork
    from zeroclone_amd.valued import ChessPuctSearch
    G, sims, bs, c, alpha, eps = 1024, 1600, 32, 1.5, 0.3, 0.25
    torch.manual_seed(13)
    net = MfmaPolicyValueNetwork(PolicyValueNetwork().eval())
    eng = NativeEngine(max_games=G, max_sims=sims, max_batch=bs)
    ps = ChessPuctSearch(eng, G, bs, c_puct=c, dirichlet_alpha=alpha, dirichlet_eps=eps, seed=21)
    sampled = _sample(G, 8)
    rows_idx = torch.tensor([g * bs + j for g in sampled for j in range(bs)], device="cuda")
    logs = {g: {} for g in sampled}   # position key -> (value, logits[4096])
    root_logits = []

    def fn(leaves, planes, counts):
        v, logits = net(planes)
        lv = leaves[rows_idx].cpu().numpy()
        vv = v.reshape(-1)[rows_idx].cpu().numpy()
        ll = logits[rows_idx].float().cpu().numpy()
        cnt = counts.cpu().numpy()
        for a, g in enumerate(sampled):
            for j in range(int(cnt[g])):
                k = a * bs + j
                logs[g].setdefault(_key_row(lv[k]), (float(vv[k]), ll[k]))
        if not root_logits:
            root_logits.append(ll[0])
        return v, logits

    mv, na, st = ps.run(_chess_roots(G), sims, fn)
    na, st, prior = na.cpu().numpy(), st.cpu().numpy(), ps.prior.cpu().numpy().astype(np.float64)
    assert (st[:, 5] == 0).all() and (na.sum(axis=1) == sims - 1).all()

    root = oracle.chess_from_fen(START)
    rmoves = oracle.chess_moves(root)
    idx = np.array([(m[0] * 8 + m[1]) * 64 + m[2] * 8 + m[3] for m in rmoves])
    lg = root_logits[0][idx].astype(np.float64)
    sm = np.exp(lg - lg.max())
    sm /= sm.sum()
    # Dirichlet root noise: prior = (1 - eps) softmax + eps noise, noise ~ Dir(alpha) per game
    noise = (prior[:, :len(rmoves)] - (1 - eps) * sm) / eps
    assert noise.min() > -1e-4
    np.testing.assert_allclose(noise.sum(axis=1), 1.0, atol=1e-4)
    k = len(rmoves)
    np.testing.assert_allclose(noise.mean(axis=0), 1.0 / k, atol=0.012)
    var = alpha * (k * alpha - alpha) / ((k * alpha) ** 2 * (k * alpha + 1))
    assert abs(noise.var(axis=0).mean() / var - 1.0) < 0.2
    assert len({tuple(np.round(r, 5)) for r in noise}) == G   # every game its own draw

    for g in sampled:
        tree = eng.debug_chess_tree(g)
        nodes, tp = tree["nodes"], tree["prior"]
        pri = {}
        checked = 0
        for i, nd in enumerate(nodes):
            if not nd["evaluated"] or i == 0:
                continue
            key = _key_row(nd["st"])
            p = tp[nd["base"]: nd["base"] + nd["nmoves"]].astype(np.float64)
            if key in pri:
                assert np.array_equal(pri[key], p)
            pri[key] = p
            if checked < 64:   # priors = softmax of the logged logits over the legal moves
                mvs = tree["mv"][nd["base"]: nd["base"] + nd["nmoves"]].astype(np.int64)
                lgn = logs[g][key][1][(mvs & 63) * 64 + ((mvs >> 6) & 63)].astype(np.float64)
                e = np.exp(lgn - lgn.max())
                np.testing.assert_allclose(p, e / e.sum(), rtol=2e-5, atol=1e-7)
                checked += 1
        assert checked > 10
        root_p = tp[nodes[0]["base"]: nodes[0]["base"] + nodes[0]["nmoves"]].astype(np.float64)
        calls = []

        def prior_fn(node, g=g):
            calls.append(1)
            return list(root_p) if len(calls) == 1 else list(pri[_key_zcc(node.s)])

        moves, N, best = puct_ref.search(root, sims, bs, c, lambda s, g=g: logs[g][_key_zcc(s)][0], prior_fn)
        assert N == [int(x) for x in na[g, :len(moves)]], g
    eng.close()
