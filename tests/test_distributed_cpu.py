"""Multi-rank pieces on CPU: the trajectory all-gather over gloo (world_size 2), dataset
labels, replay buffer, compact-position planes."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from zeroclone_amd.selfplay import ReplayBuffer, dataset_labels, gather_positions, planes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_rows(rank):
    n = 3 + 4 * rank   # ragged per rank
    rows = np.zeros((n, 3), np.int64)
    rows[:, 0] = np.arange(n) + 100 * rank
    rows[:, 1] = rank
    rows[:, 2] = (rank & 1) | (np.int64(-1) << 32)
    return rows


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    local = torch.from_numpy(_rank_rows(rank))
    got = gather_positions(local)
    empty = gather_positions(torch.zeros((0, 3), dtype=torch.int64))
    out[rank] = (got.numpy().tolist(), empty.shape[0])
    dist.barrier()
    dist.destroy_process_group()


def test_gather_positions_gloo_world2():
    world, port = 2, _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    expect = np.concatenate([_rank_rows(r) for r in range(world)]).tolist()
    for r in range(world):
        rows, n_empty = out[r]
        assert rows == expect
        assert n_empty == 0


def test_dataset_labels_match_engine_get_dataset():
    from zeroclone_amd.engine import Engine
    e = Engine({"game": "connect4", "backend": "c4_backend", "value_function": "random_rollout", "threads": 1})
    for col in [0, 1, 0, 1, 0, 1, 0]:
        res = e.play_move((col, 0), 0)
    X, y = e.get_dataset()
    assert np.array_equal(y, dataset_labels(len(X), res))
    assert np.array_equal(dataset_labels(4, 0), np.zeros(4, np.float32))


def test_planes_match_state_to_tensor():
    from zeroclone_amd.engine.games.connect4 import c4_backend as c4
    rng = np.random.default_rng(0)
    rows, tens = [], []
    for _ in range(50):
        st = c4.create_init_state()
        for _ in range(rng.integers(0, 20)):
            legal = sorted(c4.get_legal_moves(st))
            st = c4.play_move(st, legal[rng.integers(len(legal))])
        s0, s1, t = c4.to_zc(st)
        rows.append([np.int64(np.uint64(s0)), np.int64(np.uint64(s1)), t])
        tens.append(c4.state_to_tensor(st))
    assert np.array_equal(planes(np.array(rows, dtype=np.int64)), np.stack(tens))


def _reference_update_replay(store, states_new, values_new, frac_old=0.30):
    """scripts/train.py:_update_replay (:27-50), restated (the module-level lists are `store`)."""
    if not store[0]:
        store[0].append(states_new)
        store[1].append(values_new)
        return states_new, values_new
    old_states, old_values = np.concatenate(store[0], axis=0), np.concatenate(store[1], axis=0)
    k = int(frac_old * len(old_states))
    if k > 0:
        idx = np.random.choice(len(old_states), k, replace=False)
        ss, sv = old_states[idx], old_values[idx]
    else:
        ss, sv = old_states[:0], old_values[:0]
    store[0].append(states_new)
    store[1].append(values_new)
    return np.concatenate([ss, states_new], axis=0), np.concatenate([sv, values_new], axis=0)


def test_replay_buffer_global_numpy_stream_matches_train_py():
    """Default ReplayBuffer draws with numpy's global generator, as train.py does: after the
    same np.random.seed, the same training sets — for numpy arrays and torch tensors."""
    rng = np.random.default_rng(1)
    batches = [(rng.integers(0, 1 << 40, (n, 3)), rng.integers(-1, 2, n).astype(np.float32)) for n in (40, 17, 33, 8)]
    store = ([], [])
    np.random.seed(123)
    want = [_reference_update_replay(store, s, v) for s, v in batches]
    for conv in (lambda x: x, torch.from_numpy):
        rb = ReplayBuffer()
        np.random.seed(123)
        for (s, v), (ws, wv) in zip(batches, want):
            gs, gv = rb.update(conv(s), conv(v))
            gs, gv = (gs.numpy(), gv.numpy()) if torch.is_tensor(gs) else (gs, gv)
            assert np.array_equal(gs, ws) and np.array_equal(gv, wv)


def test_replay_buffer_semantics():
    rb = ReplayBuffer(seed=0)
    s1, v1 = np.arange(10)[:, None], np.arange(10)
    a, b = rb.update(s1, v1)
    assert np.array_equal(a, s1)
    s2, v2 = np.arange(10, 15)[:, None], np.arange(10, 15)
    a, b = rb.update(s2, v2)
    assert len(a) == 3 + 5 and np.array_equal(a[-5:], s2)
    assert len(set(a[:3, 0].tolist())) == 3 and all(x < 10 for x in a[:3, 0])


def _bench_worker(rank, world, port, out):
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank r ran (10 + r) expansions ... in (1 + r) s; kernels 2r ms
    counts, dt, kms = bench.reduce_over_ranks([10 + rank, 20 + rank, rank, 5], 1.0 + rank, 2.0 * rank, "cpu")
    out[rank] = (counts, dt, kms)
    dist.barrier()
    dist.destroy_process_group()


def test_bench_aggregation_gloo_world2():
    """bench.py's whole-job reduction: counters summed over ranks, wall and kernel time the
    max over ranks — the value the driver's N-GPU line reports."""
    world, port = 2, _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bench_worker, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        assert out[r] == ([21, 41, 1, 10], 2.0, 2.0)


def test_bench_rank_ranges_and_launcher_errors():
    import subprocess
    import sys

    import bench
    assert bench.rank_ranges(2, 4096) == [[0, 4095], [4096, 8191]]
    assert bench.rank_ranges(8, 4096)[7] == [7 * 4096, 8 * 4096 - 1]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    # more GPUs than visible: a clear error before any GPU work (no GPU in this container)
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=repo, env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode != 0 and ("GPU(s) visible" in p.stderr or "cannot count GPUs" in p.stderr)
    # under torchrun the world size must match --gpus
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "4"], cwd=repo, env={**env, "WORLD_SIZE": "2"},
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in p.stderr


def test_visible_gpus_reads_the_kfd_topology(tmp_path, monkeypatch):
    """bench.visible_gpus counts GPU nodes of the KFD topology (simd_count > 0) with no HIP
    call, honours *_VISIBLE_DEVICES, and fails loudly when the topology is missing."""
    import bench
    for i, simds in enumerate([0, 1024, 1024, 0, 1024]):   # two CPU nodes, three GPUs
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count {0 if simds else 64}\nsimd_count {simds}\n")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert bench.visible_gpus(str(tmp_path)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert bench.visible_gpus(str(tmp_path)) == 2
    with pytest.raises(RuntimeError):
        bench.visible_gpus(str(tmp_path / "absent"))


def _games_of_rank(rank):
    """A TrajBatch of finished Connect4 games as the device pool returns them (rows, labels
    by Engine.get_dataset, moves, game records), built on the host from real games."""
    from zeroclone_amd.engine.games.connect4 import c4_backend as c4
    from zeroclone_amd.selfplay import TrajBatch
    rng = np.random.default_rng(10 + rank)
    rows, labels, moves, games = [], [], [], []
    for gno in range(2 + 3 * rank):
        st, hist, mv = c4.create_init_state(), [], []
        res = None
        while res is None:
            hist.append(c4.to_zc(st))
            legal = sorted(c4.get_legal_moves(st))
            m = legal[rng.integers(len(legal))]
            mv.append(m[0])
            st = c4.play_move(st, m)
            res = (st.turn * 2 - 1) if c4.check_win(st) else (0 if c4.check_draw(st) else None)
        hist.append(c4.to_zc(st))
        mv.append(-1)
        games.append([gno, rank, res, len(rows), len(hist)])
        rows += [[np.int64(np.uint64(s0)), np.int64(np.uint64(s1)), t] for s0, s1, t in hist]
        labels += dataset_labels(len(hist), res).astype(np.int32).tolist()
        moves += mv
    t = lambda a, dt: torch.tensor(np.asarray(a), dtype=dt)  # noqa: E731
    return TrajBatch(t(rows, torch.int64), t(labels, torch.int32), t(moves, torch.int16), t(games, torch.int64))


def _traj_worker(rank, world, port, out):
    import bench
    from zeroclone_amd.selfplay import positions_of
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rep, rows = bench.exchange_positions(positions_of(_games_of_rank(rank)), world)
    out[rank] = (rep, rows.numpy().tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_trajectory_exchange_gloo_world2():
    """bench.py's C3 exchange on TrajBatch-shaped rows from real games: every rank receives
    every rank's positions in rank order, labels packed as Engine.get_dataset's."""
    from zeroclone_amd.selfplay import positions_of
    world, port = 2, _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_traj_worker, args=(world, port, out), nprocs=world, join=True)
    want = np.concatenate([positions_of(_games_of_rank(r)).numpy() for r in range(world)])
    for r in range(world):
        rep, rows = out[r]
        rows = np.asarray(rows, np.int64)
        assert np.array_equal(rows, want)
        assert rep["rows"] == len(want) and rep["bytes"] == want.size * 8 and rep["ms"] >= 0
    lab = (want[:, 2] >> 32).astype(np.int64)
    b0 = _games_of_rank(0)
    assert np.array_equal(lab[: b0.labels.shape[0]], b0.labels.numpy())
