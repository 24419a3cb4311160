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
