"""GPU checks of the Connect4 PUCT search (c4_puct.hip; SURVEY §8 a21 on the target game, no
reference counterpart): exact agreement with its plain-Python specification
(tests/puct_ref.py, C4Rules over the oracle's Connect4 rules) on uniform priors and
deterministic values; Dirichlet root noise; the 7-logit policy + value network on the MFMA
tower against PyTorch fp32; the full C2 shape (4096 games x 800 sims) with that network,
replayed through the specification; graph capture = eager."""
import numpy as np
import pytest
import torch

import oracle
from oracle import puct_ref
from c4_values import bits_from_rows, hash_value

pytestmark = pytest.mark.gpu

EMPTY = "." * 42


def _board(cols):
    b, t = EMPTY, 0
    for col in cols:
        b, t = oracle.play(b, t, col)
    return b, t


POSITIONS = [_board([]), _board([3, 3, 2, 4]), _board([0, 0, 0, 0, 0, 0, 1, 2]),   # column 0 full
             _board([3, 2, 3, 2, 3]),                                              # X wins by playing 3
             _board([1, 1, 2, 2, 4, 4, 5, 6, 6, 5, 0])]


def _roots(positions):
    from zeroclone_amd._native import c4_from_rows
    rows = np.array([c4_from_rows(b, t) for b, t in positions])
    return torch.from_numpy(rows.view(np.int64).reshape(len(positions), 3).copy()).cuda()


def _hash_net(leaves, planes, counts):
    r = leaves.cpu().numpy().view(np.uint64)
    v = torch.tensor([hash_value(int(x[0]), int(x[1]), int(x[2]) & 1) for x in r], dtype=torch.float64).cuda()
    return v, torch.zeros((r.shape[0], 7), dtype=torch.float32, device="cuda")


def _hv(s):
    s0, s1 = bits_from_rows(s[0])
    return hash_value(s0, s1, s[1])


@pytest.fixture(scope="module")
def eng():
    from zeroclone_amd._native import NativeEngine
    e = NativeEngine(max_games=64, max_sims=400, max_batch=32)
    yield e
    e.close()


@pytest.mark.parametrize("sims,bs,c", [(65, 8, 1.5), (200, 32, 2.5), (40, 16, 0.7)])
def test_c4_puct_matches_its_specification(eng, sims, bs, c):
    from zeroclone_amd.valued import C4PuctSearch
    pos = POSITIONS * 2
    ps = C4PuctSearch(eng, len(pos), bs, c_puct=c, dirichlet_eps=0.0)
    mv, na, st = ps.run(_roots(pos), sims, _hash_net)
    mv, na, st = mv.cpu().numpy(), na.cpu().numpy(), st.cpu().numpy()
    for i, s in enumerate(pos):
        moves, N, best = puct_ref.search(s, sims, bs, c, _hv,
                                         lambda node: [float(np.float32(1.0) / np.float32(len(node.moves)))]
                                         * len(node.moves), rules=puct_ref.C4Rules)
        assert st[i, 5] == 0
        assert [int(na[i, col]) for col in moves] == N, (i, s)
        assert sum(N) == sims - 1 and int(na[i].sum()) == sims - 1
        assert int(mv[i]) == moves[best]


def test_c4_puct_terminal_root_and_capacity_errors(eng):
    from zeroclone_amd.valued import C4PuctSearch
    won = _board([3, 2, 3, 2, 3, 2, 3])   # X has four: a finished game
    ps = C4PuctSearch(eng, 1, 8, dirichlet_eps=0.0)
    mv, na, st = ps.run(_roots([won]), 9, _hash_net)
    assert int(st[0, 5].item()) == 1 and int(mv[0].item()) == -1   # ZC_STATUS_NO_MOVES


def test_c4_dirichlet_root_noise(eng):
    from zeroclone_amd.valued import C4PuctSearch
    n = 64
    pri = []
    for seed in (1, 1, 2):
        ps = C4PuctSearch(eng, n, 8, dirichlet_alpha=0.3, dirichlet_eps=0.25, seed=seed)
        ps.run(_roots([POSITIONS[0]] * n), 9, _hash_net)
        pri.append(ps.prior.cpu().numpy().astype(np.float64))
    assert np.array_equal(pri[0], pri[1]) and not np.array_equal(pri[0], pri[2])
    p = pri[0]
    np.testing.assert_allclose(p.sum(axis=1), 1.0, atol=1e-5)
    assert (p.min(axis=1) >= 0.75 / 7 - 1e-6).all()
    assert len({tuple(np.round(r, 6)) for r in p}) == n


def _c4_net(seed=0):
    from zeroclone_amd.nets import PolicyValueNetwork
    torch.manual_seed(seed)
    net = PolicyValueNetwork(in_planes=2, board=(6, 7), n_logits=7).eval()
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
    return net


def test_c4_policy_value_network_mfma_matches_torch():
    from zeroclone_amd.nets import MfmaPolicyValueNetwork
    net = _c4_net()
    x = (torch.rand(53, 2, 6, 7) < 0.3).float()
    with torch.no_grad():
        v_ref, l_ref = net(x)
    v, lg = MfmaPolicyValueNetwork(net)(x.cuda().half())
    np.testing.assert_allclose(v.cpu().numpy(), v_ref.reshape(-1).double().numpy(), atol=2e-2)
    np.testing.assert_allclose(lg.float().cpu().numpy(), l_ref.numpy(), atol=5e-2, rtol=2e-2)


def test_c4_puct_full_shape_network_replay():
    """C2 shape with the PUCT extension: 4096 games x 800 sims, the policy + value network on
    the MFMA tower, Dirichlet noise.  For 8 sampled games the logged values and the device's
    priors replay through puct_ref to the same root visits; the priors are the softmax of the
    logged logits; the root noise has Dirichlet(0.3) statistics over the 4096 games."""
    from zeroclone_amd._native import NativeEngine
    from zeroclone_amd.nets import MfmaPolicyValueNetwork
    from zeroclone_amd.valued import C4PuctSearch
    G, sims, bs, c, alpha, eps = 4096, 800, 32, 1.5, 0.3, 0.25
    net = MfmaPolicyValueNetwork(_c4_net(seed=3))
    e = NativeEngine(max_games=G, max_sims=sims, max_batch=bs)
    ps = C4PuctSearch(e, G, bs, c_puct=c, dirichlet_alpha=alpha, dirichlet_eps=eps, seed=5)
    sampled = sorted({int(round(x)) for x in np.linspace(0, G - 1, 8)})
    rows_idx = torch.tensor([g * bs + j for g in sampled for j in range(bs)], device="cuda")
    logs = {g: {} for g in sampled}   # (s0, s1, turn) -> (value, logits[7])
    root_logits = []

    def fn(leaves, planes, counts):
        v, logits = net(planes)
        lv = leaves[rows_idx].cpu().numpy().view(np.uint64)
        vv = v.reshape(-1)[rows_idx].cpu().numpy()
        ll = logits[rows_idx].float().cpu().numpy()
        cnt = counts.cpu().numpy()
        for a, g in enumerate(sampled):
            for j in range(int(cnt[g])):
                k = a * bs + j
                logs[g].setdefault((int(lv[k, 0]), int(lv[k, 1]), int(lv[k, 2]) & 1), (float(vv[k]), ll[k]))
        if not root_logits:
            root_logits.append(ll[0])
        return v, logits

    roots = torch.zeros((G, 3), dtype=torch.int64, device="cuda")
    mv, na, st = ps.run(roots, sims, fn)
    na, st, prior = na.cpu().numpy(), st.cpu().numpy(), ps.prior.cpu().numpy().astype(np.float64)
    assert (st[:, 5] == 0).all() and (na.sum(axis=1) == sims - 1).all()
    lg = root_logits[0].astype(np.float64)
    sm = np.exp(lg - lg.max())
    sm /= sm.sum()
    noise = (prior - (1 - eps) * sm) / eps
    assert noise.min() > -1e-4
    np.testing.assert_allclose(noise.sum(axis=1), 1.0, atol=1e-4)
    np.testing.assert_allclose(noise.mean(axis=0), 1.0 / 7, atol=0.01)
    var = alpha * (7 * alpha - alpha) / ((7 * alpha) ** 2 * (7 * alpha + 1))
    assert abs(noise.var(axis=0).mean() / var - 1.0) < 0.15
    for g in sampled:
        nodes = e.debug_c4_puct_tree(g)
        pri, checked = {}, 0
        for i, nd in enumerate(nodes):
            if not nd["evaluated"] or i == 0:
                continue
            key = (int(nd["s0"]), int(nd["s1"]), int(nd["turn"]))
            p = nd["pr"][: nd["nmoves"]].astype(np.float64)
            pri[key] = p
            if checked < 64:   # priors = softmax of the logged column logits over the move list
                cols = [(int(nd["order"]) >> (3 * k)) & 7 for k in range(nd["nmoves"])]
                lgn = logs[g][key][1][cols].astype(np.float64)
                ex = np.exp(lgn - lgn.max())
                np.testing.assert_allclose(p, ex / ex.sum(), rtol=2e-5, atol=1e-7)
                checked += 1
        assert checked > 10
        root_p = list(nodes[0]["pr"][: nodes[0]["nmoves"]].astype(np.float64))
        calls = []

        def key_of(s):
            s0, s1 = bits_from_rows(s[0])
            return s0, s1, s[1]

        def prior_fn(node):
            calls.append(1)
            return root_p if len(calls) == 1 else list(pri[key_of(node.s)])

        moves, N, best = puct_ref.search((EMPTY, 0), sims, bs, c, lambda s, g=g: logs[g][key_of(s)][0], prior_fn,
                                         rules=puct_ref.C4Rules)
        assert N == [int(na[g, col]) for col in moves], g
    e.close()


def test_c4_puct_graph_capture_replays_the_eager_move(eng):
    from zeroclone_amd.nets import MfmaPolicyValueNetwork
    from zeroclone_amd.valued import C4PuctSearch
    net = MfmaPolicyValueNetwork(_c4_net(seed=4))
    fn = lambda leaves, planes, counts: net(planes)  # noqa: E731
    pos = POSITIONS * 4
    ps = C4PuctSearch(eng, len(pos), 16, seed=3)
    r = _roots(pos)
    mv, na, _ = ps.run(r, 97, fn, temperature=1.0)
    mv, na = mv.clone(), na.clone()
    g = ps.capture(r, 97, fn, temperature=1.0)
    ps.na.zero_()
    ps.search_no.zero_()   # the eager search was search 0 of every game; replay it as search 0
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(ps.na, na) and torch.equal(ps.move, mv)


def test_c4_consecutive_searches_draw_fresh_noise(eng):
    """Each search of a game advances its search number (on the device, so graph replays do
    too): two consecutive searches of the same roots draw different root noise and sample at
    a different point of the visit CDF; resetting the numbers replays the first search."""
    from zeroclone_amd.valued import C4PuctSearch
    n = 64
    ps = C4PuctSearch(eng, n, 8, dirichlet_alpha=0.3, dirichlet_eps=0.25, seed=9)
    r = _roots([POSITIONS[0]] * n)
    out = []
    for _ in range(2):
        mv, na, _ = ps.run(r, 33, _hash_net, temperature=1.0)
        out.append((ps.prior.cpu().numpy().copy(), mv.cpu().numpy().copy()))
    assert ps.search_no.cpu().tolist() == [2] * n
    assert all(not np.array_equal(out[0][0][i], out[1][0][i]) for i in range(n))
    assert not np.array_equal(out[0][1], out[1][1])   # 64 temperature samples: some differ
    ps.search_no.zero_()
    mv, _, _ = ps.run(r, 33, _hash_net, temperature=1.0)
    assert np.array_equal(ps.prior.cpu().numpy(), out[0][0]) and np.array_equal(mv.cpu().numpy(), out[0][1])


@pytest.mark.parametrize("k", [2, 4])
def test_c4_split_stream_search_equals_the_single_stream_search(eng, k):
    """C4PuctSearch with k network callables (valued._split_flushes): the games in k parts on
    k streams; moves, root visits, priors and counters equal the one-stream search's."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork
    from zeroclone_amd.valued import C4PuctSearch
    net = MfmaPolicyValueNetwork(_c4_net(seed=6))
    pos = (POSITIONS * 8)[:37]
    r = _roots(pos)
    outs = []
    for split in (False, True):
        ps = C4PuctSearch(eng, len(pos), 16, seed=5)
        fn = [(lambda l, p, c, m=net.replica(): m(p)) for _ in range(k)] if split else (lambda l, p, c: net(p))
        mv, na, st = ps.run(r, 97, fn, temperature=1.0)
        outs.append((mv.cpu().clone(), na.cpu().clone(), ps.prior.cpu().clone(), st[:, :3].cpu().clone()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def test_value_searches_split_over_streams_equal_the_single_stream_ones(eng):
    """C4ValuedSearch and ChessValuedSearch with a list of network values (one per part and
    stream, valued._split_flushes; 99 simulations, so the short last flush's rows path runs
    in every part): the same moves, root visits and counters as one stream."""
    from zeroclone_amd._native import NativeEngine, chess_from_fen, CHESS_STATE_DTYPE
    from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork
    from zeroclone_amd.valued import C4ValuedSearch, ChessValuedSearch, NetValue
    torch.manual_seed(8)
    c4net = MfmaValueNetwork(ValueNetwork(128, 2, in_planes=2).eval(), "cuda")
    pos = (POSITIONS * 8)[:29]
    r = _roots(pos)
    for k in (2, 3):
        outs = []
        for split in (False, True):
            eng.seed(0, list(range(100, 100 + len(pos))))
            vs = C4ValuedSearch(eng, len(pos), 32)
            fn = [NetValue(c4net.replica()) for _ in range(k)] if split else NetValue(c4net)
            outs.append([x.cpu().clone() for x in vs.run(r, 99, 1.4, fn)])
        for x, y in zip(*outs):
            assert torch.equal(x, y)
    ce = NativeEngine(max_games=24, max_sims=128, max_batch=32)
    chnet = MfmaValueNetwork(ValueNetwork(128, 2).eval(), "cuda")
    fens = ["rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
            "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1"] * 10
    a = np.array([chess_from_fen(f) for f in fens], CHESS_STATE_DTYPE)
    croots = torch.from_numpy(a.view(np.uint8).reshape(len(fens), 72).copy()).cuda()
    outs = []
    for split in (False, True):
        ce.seed(0, list(range(200, 200 + len(fens))))
        vs = ChessValuedSearch(ce, len(fens), 32)
        fn = [NetValue(chnet.replica()) for _ in range(3)] if split else NetValue(chnet)
        outs.append([x.cpu().clone() for x in vs.run(croots, 99, 1.4, fn)])
    ce.close()
    for x, y in zip(*outs):
        assert torch.equal(x, y)


@pytest.mark.parametrize("k", [1, 4])
def test_c4_roots_flush_on_the_roots_alone_equals_the_full_flush(eng, k):
    """As the chess test: PolicyNet's roots-only flush 0 against the all-slot flush."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork
    from zeroclone_amd.valued import C4PuctSearch, PolicyNet
    net = MfmaPolicyValueNetwork(_c4_net(seed=9))
    pos = (POSITIONS * 8)[:37]
    r = _roots(pos)
    outs = []
    for trimmed in (False, True):
        ps = C4PuctSearch(eng, len(pos), 16, seed=2)
        if trimmed:
            fn = PolicyNet(net) if k == 1 else [PolicyNet(net.replica()) for _ in range(k)]
        else:
            fn = (lambda l, p, c: net(p)) if k == 1 else [(lambda l, p, c, m=net.replica(): m(p)) for _ in range(k)]
        mv, na, st = ps.run(r, 81, fn, temperature=1.0)
        outs.append((mv.cpu().clone(), na.cpu().clone(), ps.prior.cpu().clone(), st[:, :3].cpu().clone()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
