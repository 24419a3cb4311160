"""GPU checks of the PUCT search (chess_puct.hip; SURVEY §8 a21, no reference counterpart):
exact agreement with its plain-Python specification (tests/puct_ref.py) on uniform priors
and deterministic values, Dirichlet root noise properties, the policy+value network on the
MFMA kernels against PyTorch fp32, and a full search with that network."""
import numpy as np
import pytest
import torch

import oracle
from oracle import puct_ref

pytestmark = pytest.mark.gpu

FENS = ["rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
        "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1",
        "8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1",
        "r1bqkbnr/pppp1ppp/2n5/4p3/2B1P3/5Q2/PPPP1PPP/RNB1K1NR w KQkq - 2 3",
        "6k1/5ppp/8/8/8/8/5PPP/3R2K1 w - - 0 1"]
M64 = (1 << 64) - 1


def hv(board: bytes, turn: int) -> float:
    h = 0x84222325CBF29CE4
    for b in board:
        h = ((h ^ b) * 0x100000001B3) & M64
    h = (h ^ (turn * 0x9E3779B97F4A7C15)) & M64
    h ^= h >> 31
    return ((h % 400001) - 200000) / 200003.0


@pytest.fixture(scope="module")
def eng():
    from zeroclone_amd._native import NativeEngine
    e = NativeEngine(max_games=64, max_sims=300, max_batch=32)
    yield e
    e.close()


def roots_of(fens):
    from zeroclone_amd._native import CHESS_STATE_DTYPE, chess_from_fen
    a = np.array([chess_from_fen(f) for f in fens], CHESS_STATE_DTYPE)
    return torch.from_numpy(a.view(np.uint8).reshape(len(fens), 72).copy()).cuda()


def decode(m):
    from zeroclone_amd._native import unpack_chess_move
    (fr, fc, tr, tc), v = unpack_chess_move(int(m) & 0xFFFF)
    return (fr, fc, tr, tc, v)


def hash_net(leaves, planes, counts):
    rows = leaves.cpu().numpy()
    v = torch.tensor([hv(bytes(r[:64]), int(r[64])) for r in rows], dtype=torch.float64).cuda()
    return v, torch.zeros((rows.shape[0], 4096), dtype=torch.float32, device="cuda")


@pytest.mark.parametrize("sims,bs,c", [(65, 8, 1.5), (129, 16, 2.5), (40, 32, 1.0)])
def test_puct_matches_its_specification(eng, sims, bs, c):
    from zeroclone_amd.valued import ChessPuctSearch
    fens = FENS * 2
    ps = ChessPuctSearch(eng, len(fens), bs, c_puct=c, dirichlet_eps=0.0)
    mv, na, st = ps.run(roots_of(fens), sims, hash_net)
    mv, na, st = mv.cpu().numpy(), na.cpu().numpy(), st.cpu().numpy()
    for i, fen in enumerate(fens):
        moves, N, best = puct_ref.search(oracle.chess_from_fen(fen), sims, bs, c,
                                         lambda s: hv(bytes(s.board), s.turn),
                                         lambda node: [float(np.float32(1.0) / np.float32(len(node.moves)))] * len(node.moves))
        assert st[i, 5] == 0
        assert list(na[i, :len(moves)]) == N, fen
        assert sum(N) == sims - 1
        assert decode(mv[i]) == moves[best]


def test_dirichlet_root_noise(eng):
    from zeroclone_amd.valued import ChessPuctSearch
    n = 64
    fens = [FENS[0]] * n
    pri = []
    for seed in (1, 1, 2):
        ps = ChessPuctSearch(eng, n, 8, dirichlet_alpha=0.3, dirichlet_eps=0.25, seed=seed)
        ps.run(roots_of(fens), 9, hash_net)
        pri.append(ps.prior.cpu().numpy()[:, :20].astype(np.float64))
    assert np.array_equal(pri[0], pri[1])          # same seed: same noise
    assert not np.array_equal(pri[0], pri[2])      # another seed: another draw
    p = pri[0]
    np.testing.assert_allclose(p.sum(axis=1), 1.0, atol=1e-5)
    assert (p.min(axis=1) >= 0.75 / 20 - 1e-6).all()   # (1 - eps) * uniform + eps * noise
    assert len({tuple(np.round(r, 6)) for r in p}) == n   # every game its own draw
    np.testing.assert_allclose(p.mean(axis=0), 1 / 20, atol=0.02)   # E[noise] = uniform


def test_policy_value_network_mfma_matches_torch():
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork
    torch.manual_seed(0)
    net = PolicyValueNetwork().eval()
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
    x = (torch.rand(37, 17, 8, 8) < 0.2).float()
    with torch.no_grad():
        v_ref, l_ref = net(x)
    v, l = MfmaPolicyValueNetwork(net)(x.cuda().half())
    np.testing.assert_allclose(v.cpu().numpy(), v_ref.reshape(-1).double().numpy(), atol=2e-2)
    np.testing.assert_allclose(l.float().cpu().numpy(), l_ref.numpy(), atol=5e-2, rtol=2e-2)


def test_convolutional_policy_head_matches_fp32():
    """PolicyValueNetwork(head="conv") (round 5): the 1x1 conv 128 -> 64 epilogue writes the
    logits (pixel = from square, channel = to square) in the tower launch; against torch fp32
    of the same network on the same tower activation (fp16 output rounding: 1e-2 abs + 1e-2
    rel), values bit-identical to the value-only launch of the same tower, ragged tiles."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork, _fold
    torch.manual_seed(6)
    net = PolicyValueNetwork(head="conv").eval()
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
    mnet = MfmaPolicyValueNetwork(net)
    assert mnet.conv_head and mnet.fused
    n = 37
    x = ((torch.rand(n, 17, 8, 8) < 0.3).half()).cuda()
    v, logits = mnet(x)
    logits = logits.float().clone()
    a, vals = mnet.tower.tower(x, head=True)
    folded = _fold(net.policy[0], net.policy[1])
    wf = folded.weight.detach().float().reshape(64, -1).cuda()
    ref = (a.float() @ wf.t() + folded.bias.detach().float().cuda()).reshape(n, 4096)   # [n, from, to]
    torch.cuda.synchronize()
    assert logits.shape == (n, 4096)
    np.testing.assert_allclose(logits.cpu().numpy(), ref.cpu().numpy(), atol=1e-2, rtol=1e-2)
    assert torch.equal(v, vals)
    assert ref.abs().max().item() > 0.1 and (ref < 0).any()   # no ReLU on logits


@pytest.mark.parametrize("shape", [(37, 17, 8, 8, 4096), (53, 2, 6, 7, 7)])
def test_fused_policy_conv_matches_fp32(shape):
    """The policy 1x1 conv fused into the tower launch (zc_net_tower_policy_async) against a
    torch fp32 1x1 conv + bias + ReLU of the SAME tower activation (written by the unfused
    launch): within fp16 output rounding (tolerance 1e-2 abs + 1e-2 rel; the fp32 MFMA sums
    128 products in another order); values bit-identical to the unfused launch; logits of
    both paths within 2e-2.  Ragged last tiles (37 / 53 boards)."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork, _fold
    n, cin, h, w, nl = shape
    torch.manual_seed(5)
    net = PolicyValueNetwork(in_planes=cin, board=(h, w), n_logits=nl).eval()
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
    mnet = MfmaPolicyValueNetwork(net)
    assert mnet.fused
    x = ((torch.rand(n, cin, h, w) < 0.3).half()).cuda()
    v_f, l_f = mnet(x)
    p_f = mnet._pout[(n, h * w)].float().clone()
    v_u, l_u = mnet(x, fused=False)
    a, _ = mnet.tower.tower(x, head=False)
    folded = _fold(net.policy[0], net.policy[1])
    wf = folded.weight.detach().float().reshape(32, -1).cuda()
    p_ref = torch.relu(a.float() @ wf.t() + folded.bias.detach().float().cuda())
    torch.cuda.synchronize()
    np.testing.assert_allclose(p_f.cpu().numpy(), p_ref.cpu().numpy(), atol=1e-2, rtol=1e-2)
    assert torch.equal(v_f, v_u)
    np.testing.assert_allclose(l_f.float().cpu().numpy(), l_u.float().cpu().numpy(), atol=2e-2, rtol=1e-2)


def test_puct_with_the_network_end_to_end(eng):
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork
    from zeroclone_amd.valued import ChessPuctSearch
    torch.manual_seed(1)
    net = MfmaPolicyValueNetwork(PolicyValueNetwork().eval())
    fens = FENS * 4
    ps = ChessPuctSearch(eng, len(fens), 32, seed=7)
    mv, na, st = ps.run(roots_of(fens), 161, lambda leaves, planes, counts: net(planes), temperature=1.0)
    na, st = na.cpu().numpy(), st.cpu().numpy()
    assert (st[:, 5] == 0).all()
    assert (na.sum(axis=1) == 160).all()
    for i, fen in enumerate(fens):
        assert decode(mv.cpu().numpy()[i]) in oracle.chess_moves(oracle.chess_from_fen(fen))
    g = ps.capture(roots_of(fens), 161, lambda leaves, planes, counts: net(planes))
    g.replay()
    torch.cuda.synchronize()
    assert (ps.na.cpu().numpy().sum(axis=1) == 160).all()


def test_consecutive_searches_draw_fresh_noise(eng):
    """ChessPuctSearch: the per-game search number moves the root noise on every search."""
    from zeroclone_amd.valued import ChessPuctSearch
    n = 16
    ps = ChessPuctSearch(eng, n, 8, dirichlet_alpha=0.3, dirichlet_eps=0.25, seed=4)
    pri = []
    for _ in range(2):
        ps.run(roots_of([FENS[0]] * n), 9, hash_net)
        pri.append(ps.prior.cpu().numpy()[:, :20].copy())
    assert ps.search_no.cpu().tolist() == [2] * n
    assert all(not np.array_equal(pri[0][i], pri[1][i]) for i in range(n))


@pytest.mark.parametrize("k", [2, 3, 4])
def test_split_stream_search_equals_the_single_stream_search(eng, k):
    """ChessPuctSearch with k network callables: the games in k contiguous parts on k streams
    (one part's select / backup / policy GEMM beside another part's tower).  The parts share
    nothing, so moves, root visits, root priors (noise included: the per-game search numbers
    of a sub-range launch) and counters equal the one-stream search's — eagerly and replayed
    from a captured graph."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork
    from zeroclone_amd.valued import ChessPuctSearch
    torch.manual_seed(3)
    net = MfmaPolicyValueNetwork(PolicyValueNetwork().eval())
    fens = (FENS * 8)[:37]
    roots = roots_of(fens)
    outs = []
    for split in (False, True):
        ps = ChessPuctSearch(eng, len(fens), 32, seed=9)
        fn = [(lambda l, p, c, m=net.replica(): m(p)) for _ in range(k)] if split else (lambda l, p, c: net(p))
        mv, na, st = ps.run(roots, 97, fn, temperature=1.0)
        first = (mv.cpu().clone(), na.cpu().clone(), ps.prior.cpu().clone(), st[:, :3].cpu().clone())
        g = ps.capture(roots, 97, fn, temperature=1.0)
        g.replay()
        torch.cuda.synchronize()
        second = (ps.move.cpu().clone(), ps.na.cpu().clone(), ps.prior.cpu().clone())
        assert ps.search_no.cpu().tolist() == [2] * len(fens)
        outs.append((first, second))
    (a1, a2), (b1, b2) = outs
    for x, y in zip(a1 + a2, b1 + b2):
        assert torch.equal(x, y)
    assert (a1[1].sum(dim=1) == 96).all()


@pytest.mark.parametrize("k", [1, 2])
def test_roots_flush_on_the_roots_alone_equals_the_full_flush(eng, k):
    """valued.PolicyNet: flush 0 (one root a game) runs the network on the n roots alone and
    backs up with one row a game (zc_chess_puct_backup_ex rows = 1); the search must equal the
    one that evaluates all n * batch_size slots of flush 0 (a plain function)."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork
    from zeroclone_amd.valued import ChessPuctSearch, PolicyNet
    torch.manual_seed(5)
    net = MfmaPolicyValueNetwork(PolicyValueNetwork(head="conv").eval())
    fens = (FENS * 8)[:29]
    roots = roots_of(fens)
    outs = []
    for trimmed in (False, True):
        ps = ChessPuctSearch(eng, len(fens), 32, seed=4)
        if trimmed:
            fn = PolicyNet(net) if k == 1 else [PolicyNet(net.replica()) for _ in range(k)]
        else:
            fn = (lambda l, p, c: net(p)) if k == 1 else [(lambda l, p, c, m=net.replica(): m(p)) for _ in range(k)]
        mv, na, st = ps.run(roots, 65, fn, temperature=1.0)
        outs.append((mv.cpu().clone(), na.cpu().clone(), ps.prior.cpu().clone(), st[:, :3].cpu().clone()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def test_rows_per_game_only_for_the_roots_flush(eng):
    from zeroclone_amd._native import lib
    v = torch.zeros(64, dtype=torch.float64, device="cuda")
    lg = torch.zeros((64, 4096), dtype=torch.float16, device="cuda")
    rc = lib().zc_chess_puct_backup_ex(eng._h, 0, 1, 1, v.data_ptr(), lg.data_ptr(), 1, 1, None)
    assert rc != 0


@pytest.mark.parametrize("k", [1, 4])
def test_nhwc_planes_equal_the_state_to_tensor_planes(eng, k):
    """ChessPuctSearch(planes_nhwc=True): the select kernel writes the planes in the MFMA
    tower's input layout (ZC_F16_NHWC32, [n*bs, 64, 32], the 17 planes then zeros) and the
    network skips its conversion launch.  The planes are the converted state_to_tensor planes
    bit for bit, and the search (moves, root visits, priors, counters) equals the one on the
    [n*bs, 17, 8, 8] planes — one stream and split over 4, through PolicyNet (roots-only flush)."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork
    from zeroclone_amd.valued import ChessPuctSearch, PolicyNet
    torch.manual_seed(11)
    net = MfmaPolicyValueNetwork(PolicyValueNetwork(head="conv").eval())
    fens = (FENS * 8)[:23]
    roots = roots_of(fens)
    outs, planes = [], []
    for nhwc in (False, True):
        ps = ChessPuctSearch(eng, len(fens), 32, seed=6, planes_nhwc=nhwc)
        fn = PolicyNet(net) if k == 1 else [PolicyNet(net.replica()) for _ in range(k)]
        mv, na, st = ps.run(roots, 81, fn, temperature=1.0)
        outs.append((mv.cpu().clone(), na.cpu().clone(), ps.prior.cpu().clone(), st[:, :3].cpu().clone()))
        planes.append(ps.planes.clone())
    for x, y in zip(*outs):
        assert torch.equal(x, y)
    # the last flush's planes: NCHW [L, 17, 8, 8] -> NHWC [L, 64, 32] zero-padded
    a = planes[0].reshape(planes[0].shape[0], 17, 64).permute(0, 2, 1)
    want = torch.zeros_like(planes[1])
    want[:, :, :17] = a
    assert torch.equal(planes[1], want)
