"""Chess self-play on the device: the fused crude-score launches
(zc_chess_selfplay_async / _pooled_async: search, Engine.play_move + _evaluate with the
repetition histories in HBM, refill — K moves per game in ONE launch) must equal K lockstep
steps (zc_chess_search_async + zc_chess_play_step_async) exactly; the lockstep step itself is
pinned to the reference's Engine in test_gpu_selfplay.py.  The PUCT pool records its games,
and a captured step graph replays the eager steps."""
import pytest
import torch

from zeroclone_amd.selfplay import ChessSelfPlay

pytestmark = pytest.mark.gpu

MATE_IN_ONE = "r1bqkbnr/pppp1ppp/2n5/4p3/2B1P3/5Q2/PPPP1PPP/RNB1K1NR w KQkq - 2 3"
FIFTY_NEXT = "4k3/8/8/8/8/8/8/4K2R w K - 49 30"
KQK = "8/8/4k3/8/8/8/3QK3/8 w - - 0 1"   # short games: mates, stalemates, repetitions


def pool(sp):
    b = sp.take()
    return b.rows.cpu(), b.labels.cpu(), b.moves.cpu(), b.games.cpu()


@pytest.mark.parametrize("fen", [None, MATE_IN_ONE, FIFTY_NEXT, KQK])
def test_chess_run_equals_lockstep_steps(fen):
    G, S, B = 40, 48, 16
    a = ChessSelfPlay(G, S, batch_size=B, seed=13, init_fen=fen, hist_cap=256)
    b = ChessSelfPlay(G, S, batch_size=B, seed=13, init_fen=fen, hist_cap=256)
    steps = [a.step().clone() for _ in range(14)]
    res = torch.cat([b.run(5).clone(), b.run(9).clone()])
    assert torch.equal(torch.stack(steps), res)
    assert torch.equal(a.roots, b.roots) and torch.equal(a.hlen, b.hlen)
    assert torch.equal(a.hist, b.hist)
    pa, pb = pool(a), pool(b)
    if fen in (FIFTY_NEXT, KQK):   # games that end within the window
        assert pa[0].shape[0] > 0
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)
    for g in (0, 11, G - 1):
        ma, ia = a.eng.get_rng_state(g)
        mb, ib = b.eng.get_rng_state(g)
        assert ma.tolist() == mb.tolist() and ia == ib
    assert int(b.stats[:, 2].sum()) == 9 * G * S   # leaves of the last launch's 9 moves
    a.close()
    b.close()


def test_chess_pooled_run_is_a_prefix_of_the_free_run():
    G, S, B, cap = 48, 40, 8, 10
    budget = G * cap * 3 // 4
    a = ChessSelfPlay(G, S, batch_size=B, seed=21, init_fen=KQK, hist_cap=256)
    b = ChessSelfPlay(G, S, batch_size=B, seed=21, init_fen=KQK, hist_cap=256)
    ra = a.run(cap).clone()
    sa, ma = a._run_states.clone(), a._run_moves.clone()
    rb = b.run_pooled(budget, cap).clone()
    sb, mb = b._run_states.clone(), b._run_moves.clone()
    played = rb != 4
    m = played.sum(0)
    assert torch.equal(played, torch.arange(cap, device=rb.device)[:, None] < m[None, :])
    assert int(m.sum()) == budget
    assert torch.equal(rb[played], ra[played]) and torch.equal(mb[played], ma[played])
    assert torch.equal(sb[played], sa[played])
    assert bool((mb[~played] == -1).all())
    fin = int(((rb != 2) & (rb != 4)).sum())
    assert b.take().games.shape[0] == fin and fin > 0
    assert int(b._ticket[1]) == int(m.max())
    a.close()
    b.close()


def _chess_pv_net(seed=0):
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork
    torch.manual_seed(seed)
    return MfmaPolicyValueNetwork(PolicyValueNetwork().eval())


def test_chess_puct_selfplay_records_and_graph_replays_eager_steps():
    """ChessSelfPlay with the PUCT search (C5's per-GPU shape, reduced): games advance and
    finish into the pool; a captured step graph gives exactly the eager steps (the search
    numbers advance on the device, so every replay draws fresh root noise)."""
    net = _chess_pv_net(2)
    G, S, B = 16, 33, 16
    a = ChessSelfPlay(G, S, batch_size=B, seed=5, init_fen=FIFTY_NEXT, puct_net=net, hist_cap=128)
    b = ChessSelfPlay(G, S, batch_size=B, seed=5, init_fen=FIFTY_NEXT, puct_net=net, hist_cap=128)
    ra = [a.step().clone() for _ in range(3)]
    g = b.capture_step()
    rb = []
    for _ in range(3):
        g.replay()
        rb.append(b.results.clone())
    torch.cuda.synchronize()
    assert all(torch.equal(x, y) for x, y in zip(ra, rb))
    assert torch.equal(a.roots, b.roots)
    assert a.ps.search_no.cpu().tolist() == [3] * G == b.ps.search_no.cpu().tolist()
    pa, pb = pool(a), pool(b)
    assert pa[3].shape[0] > 0
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)
    a.close()
    b.close()


def test_c4_value_and_puct_selfplay_pools():
    """C4SelfPlay's network modes: value-network search (C2(iii)) and PUCT with a policy +
    value network: a captured step equals the eager step, and games finish into the pool
    with Engine.get_dataset labels."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork, ValueNetwork, for_inference
    from zeroclone_amd.selfplay import C4SelfPlay, dataset_labels
    import numpy as np
    torch.manual_seed(0)
    vnet = for_inference(ValueNetwork(32, 2, in_planes=2).eval(), torch.device("cuda"), torch.float16)
    pnet = MfmaPolicyValueNetwork(PolicyValueNetwork(in_planes=2, board=(6, 7), n_logits=7).eval())
    for kw in ({"net": vnet}, {"puct_net": pnet}):
        a = C4SelfPlay(32, 33, batch_size=16, seed=4, **kw)
        b = C4SelfPlay(32, 33, batch_size=16, seed=4, **kw)
        ra = [a.step().clone() for _ in range(30)]
        g = b.capture_step()
        rb = []
        for _ in range(30):
            g.replay()
            rb.append(b.results.clone())
        torch.cuda.synchronize()
        assert all(torch.equal(x, y) for x, y in zip(ra, rb)), kw.keys()
        bt = b.take()
        assert bt.games.shape[0] > 0
        lab = bt.labels.cpu().numpy()
        for gno, slot, r, off, n in bt.games.cpu().numpy().tolist():
            assert np.array_equal(lab[off:off + n].astype(np.float32), dataset_labels(n, r))
        a.close()
        b.close()


def test_chess_pooled_launch_refuses_more_games_than_resident():
    from zeroclone_amd import _native
    import ctypes
    n = ctypes.c_int32(0)
    _native.check(_native.lib().zc_chess_pooled_max_games(64, ctypes.byref(n)))
    cap = n.value
    assert cap >= 1024   # C4 / C5's 1024 games per GPU fit
    sp = ChessSelfPlay(cap + 64, 4, batch_size=4, hist_cap=64)
    with pytest.raises(ValueError):
        sp.run_pooled(2 * (cap + 64), 4)
    sp.close()


def test_simulate_games_grows_the_trajectory_pool_on_demand():
    """simulate_games with a quota on a chess pool whose trajectory pool starts small: the
    positions grow on demand before each step (the worst case of one step is known: every
    active slot's history + 1), nothing is dropped, every game is recorded whole, and the
    pool ends far below round 4's up-front quota x max_len reservation."""
    from zeroclone_amd.selfplay import ChessSelfPlay, simulate_games
    G, S, B, total = 8, 24, 8, 48
    sp = ChessSelfPlay(G, S, batch_size=B, seed=31, init_fen=KQK, hist_cap=256, games_cap=8)
    sp.traj._alloc_pool(8, 64)   # start tiny: 64 positions
    cap0 = sp.traj.pool_cap
    res = simulate_games(sp, total, max_steps=3000)
    assert len(res) == total
    b = sp.last_batch
    lens = b.games[:, 4].cpu().numpy()
    assert int(lens.sum()) == b.rows.shape[0] and (lens >= 2).all()
    assert sp.traj.pool_cap >= int(lens.sum())
    assert sp.traj.pool_cap < total * sp.traj.max_len
    assert int(lens.sum()) > cap0 and sp.traj.pool_cap > cap0   # it had to grow
    sp.close()
