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


def test_replay_buffer_semantics():
    rb = ReplayBuffer(seed=0)
    s1, v1 = np.arange(10)[:, None], np.arange(10)
    a, b = rb.update(s1, v1)
    assert np.array_equal(a, s1)
    s2, v2 = np.arange(10, 15)[:, None], np.arange(10, 15)
    a, b = rb.update(s2, v2)
    assert len(a) == 3 + 5 and np.array_equal(a[-5:], s2)
    assert len(set(a[:3, 0].tolist())) == 3 and all(x < 10 for x in a[:3, 0])
