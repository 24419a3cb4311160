"""The free-running self-play launch (zc_c4_selfplay_async / C4SelfPlay.run): K moves per game
in one launch, each game at its own pace, must equal K lockstep steps (search + play +
record per step) exactly — moves, results, positions, the trajectory pool and its labels,
and every game's RNG stream afterwards."""
import pytest
import torch

from zeroclone_amd.selfplay import C4SelfPlay

pytestmark = pytest.mark.gpu


def pool(sp):
    b = sp.take()
    return b.rows.cpu(), b.labels.cpu(), b.moves.cpu(), b.games.cpu()


@pytest.mark.parametrize("mode", ["exact", "philox"])
def test_run_equals_lockstep_steps(mode):
    G, S, B = 192, 160, 16
    a = C4SelfPlay(G, S, batch_size=B, seed=7)
    b = C4SelfPlay(G, S, batch_size=B, seed=7)
    for sp in (a, b):
        sp.eng.c4_rollout_mode(mode, 99)
    steps = [a.step().clone() for _ in range(23)]   # long enough for games to finish and restart
    res = torch.cat([b.run(9).clone(), b.run(14).clone()])
    assert torch.equal(torch.stack(steps), res)
    assert torch.equal(a.roots, b.roots)
    pa, pb = pool(a), pool(b)
    assert pa[0].shape[0] > 0
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)
    for g in (0, 17, G - 1):
        assert a.eng.get_rng_state(g)[0].tolist() == b.eng.get_rng_state(g)[0].tolist()
        assert a.eng.get_rng_state(g)[1] == b.eng.get_rng_state(g)[1]
    a.close()
    b.close()


def test_run_counts_expansions_and_finishes():
    G, S, B = 128, 96, 32
    a = C4SelfPlay(G, S, batch_size=B, seed=3)
    b = C4SelfPlay(G, S, batch_size=B, seed=3)
    exp = fin = 0
    for _ in range(10):
        r = a.step()
        exp += int(a.stats[:, 0].sum().item())
        fin += int(((r != 2) & (r != 3)).sum().item())
    b.run(10)
    assert int(b.stats[:, 0].sum().item()) == exp
    assert int(b.stats[:, 7].sum().item()) == fin
    assert int(b.stats[:, 2].sum().item()) == 10 * G * S
    a.close()
    b.close()


def test_run_refuses_a_quota():
    sp = C4SelfPlay(64, 32, batch_size=8, seed=1)
    sp.start(quota=70)
    with pytest.raises(ValueError):
        sp.run(3)
    sp.close()


@pytest.mark.parametrize("mode", ["exact", "philox"])
def test_pooled_run_is_a_prefix_of_the_free_run(mode):
    """zc_c4_selfplay_pooled_async: the games share a move budget; each game's moves are the
    first m_g moves of run() (states, moves, results), the budget is spent exactly, skipped
    steps leave the trajectory slots alone, and a game's pool rows match its recorded moves."""
    G, S, B, cap = 160, 128, 16, 12
    budget = G * cap * 3 // 4
    a = C4SelfPlay(G, S, batch_size=B, seed=11)
    b = C4SelfPlay(G, S, batch_size=B, seed=11)
    for sp in (a, b):
        sp.eng.c4_rollout_mode(mode, 5)
    ra = a.run(cap).clone()
    sa, ma = a._run_states.clone(), a._run_moves.clone()
    rb = b.run_pooled(budget, cap).clone()
    sb, mb = b._run_states.clone(), b._run_moves.clone()
    played = rb != 4
    m = played.sum(0)
    # every game's played steps are a prefix, the budget is spent exactly
    assert torch.equal(played, torch.arange(cap, device=rb.device)[:, None] < m[None, :])
    assert int(m.sum()) == budget
    assert int(b.stats[:, 2].sum()) == budget * S
    assert torch.equal(rb[played], ra[played])
    assert torch.equal(mb[played], ma[played])
    assert torch.equal(sb[played], sa[played])
    assert bool((mb[~played] == -1).all())
    # the roots: the position after the game's last move (refilled when it ended the game)
    for g in range(G):
        k = int(m[g])
        if k == 0:
            continue
        exp = sa[k - 1, g] if int(ra[k - 1, g]) == 2 else torch.zeros(3, dtype=torch.int64, device=sa.device)
        assert torch.equal(b.roots[g], exp), g
    # games finished in the pooled run == games in its trajectory pool; each pooled game's
    # last move is its finishing move
    fin = int(((rb != 2) & (rb != 4)).sum())
    pb = b.take()
    assert pb.games.shape[0] == fin and fin > 0
    # the device's count of the most moves any game played (the record's early exit)
    assert int(b._ticket[1]) == int(m.max())
    # each game's RNG stream: where it played every step, the free run's stream exactly
    full = [g for g in range(G) if int(m[g]) == cap][:4]
    for g in full:
        assert a.eng.get_rng_state(g)[0].tolist() == b.eng.get_rng_state(g)[0].tolist()
        assert a.eng.get_rng_state(g)[1] == b.eng.get_rng_state(g)[1]
    a.close()
    b.close()


@pytest.mark.parametrize("mode", ["exact", "philox"])
def test_carried_moves_resume_to_the_free_run(mode):
    """zc_c4_selfplay_carry_async: once a launch's budget is spent its in-flight moves stop at a
    flush boundary and resume in the next launch.  Every ticketed move finishes exactly once
    (the launches' finished moves, drain included, sum to their budgets), and each game's
    finished moves, launch after launch, are its free-run moves (states, moves, results) —
    the carried searches resume with the same tree and stream."""
    G, S, B, cap = 160, 128, 16, 8
    budgets = [G * cap // 2, G * cap // 3, G * cap // 2]
    a = C4SelfPlay(G, S, batch_size=B, seed=13)
    b = C4SelfPlay(G, S, batch_size=B, seed=13)
    for sp in (a, b):
        sp.eng.c4_rollout_mode(mode, 5)
    total = len(budgets) * cap + 1
    ra = a.run(total).clone()
    sa, ma = a._run_states.clone(), a._run_moves.clone()
    seq = [[] for _ in range(G)]
    finished, leaves, carried = 0, 0, 0
    for i, bud in enumerate(budgets + [0]):
        rb = (b.run_pooled(bud, cap, carry=True) if i < len(budgets) else b.drain()).clone()
        sb, mb = b._run_states.clone(), b._run_moves.clone()
        played = rb != 4
        m = played.sum(0)
        k = rb.shape[0]
        assert torch.equal(played, torch.arange(k, device=rb.device)[:, None] < m[None, :])
        finished += int(m.sum())
        leaves += int(b.stats[:, 2].sum())
        if i < len(budgets):
            carried = max(carried, int(sum(budgets[: i + 1])) - finished)   # in flight now
            assert b.carry_pending
            with pytest.raises(RuntimeError):
                b.step()
            with pytest.raises(ValueError):   # ZC_EINVAL: the engine refuses as well
                b.eng.seed(0, list(range(G)))
        for g in range(G):
            for j in range(int(m[g])):
                seq[g].append((int(rb[j, g]), int(mb[j, g]), sb[j, g].tolist()))
    assert carried > 0                      # moves did carry over
    assert finished == sum(budgets)         # ... and each finished exactly once
    assert leaves == sum(budgets) * S       # simulations counted where they ran
    assert not b.carry_pending
    for g in range(G):
        n = len(seq[g])
        assert n <= total
        exp = [(int(ra[j, g]), int(ma[j, g]), sa[j, g].tolist()) for j in range(n)]
        assert seq[g] == exp, g
    # the drained pool searches again; a restart drops carried moves
    b.run_pooled(G, 2, carry=True)
    b.start()
    assert not b.carry_pending
    b.step()
    a.close()
    b.close()
