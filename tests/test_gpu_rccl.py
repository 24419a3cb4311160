"""The scale-out exchange on the GPU: RCCL (torch.distributed "nccl" on ROCm) all-gathers of
real self-play trajectory rows (C4SelfPlay.take_positions, device tensors), in a world of one
rank on this box's one GPU — the communicator set-up, the count all-gather and the padded
payload all-gather of selfplay.gather_positions and bench.exchange_positions run through
RCCL exactly as on the 8-GPU node; the world-2 semantics are covered by the
gloo tests in test_distributed_cpu.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_trajectory_exchange_one_rank():
    import bench
    from zeroclone_amd.selfplay import C4SelfPlay, gather_positions
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port())})
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        sp = C4SelfPlay(128, 24, batch_size=8, seed=2)
        sp.run(40)
        rows = sp.take_positions()
        assert rows.is_cuda and rows.shape[0] > 0
        got = gather_positions(rows)
        assert torch.equal(got, rows)
        empty = gather_positions(rows[:0])
        assert empty.shape == (0, 3)
        rep, _ = bench.exchange_positions(rows, 1)
        assert rep["local_rows"] == rows.shape[0]
        sp.close()
    finally:
        dist.destroy_process_group()
