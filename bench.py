#!/usr/bin/env python3
"""bench.py — MCTS node-expansions/sec, Connect4 self-play at 800 sims/move (BASELINE.json).

Workload (BASELINE.json configs[1] = SURVEY.md §8(d) C2; with --gpus N it is C3's sharding):
4096 concurrent Connect4 self-play games per GPU, 800 simulations per move, leaf batch 32,
c = 1.4, the reference's random_rollout value and random expansion policy, exact-RNG mode
(every game's CPython MT19937 stream consumed in the reference's order).  One STEP = one
move for every game: the whole search (select/expand/rollout/backup x 800) on the GPU,
then Engine.play_move + _evaluate on the device, finished games restarting from the
opening (scripts/train.py:151-170 refill).  Games are sharded across ranks by global game
id (seed = base + id) — no collective on the data path, so "scaling" is "weak".

value = expansions created on all ranks in the K timed steps / max over ranks of the
wall time of those K steps (barrier + device sync on both sides).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch  # noqa: E402  (first: our library then shares torch's HIP runtime)
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from zeroclone_amd import _native  # noqa: E402

METRIC = "MCTS node-expansions/sec (whole node), Connect4 800 sims/move at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def bytes_per_expansion_model(expansions: int, depth_sum: int) -> int:
    """bytes(d) = 152*d + 96 algorithmic tree-walk bytes per expansion."""
    return 152 * depth_sum + 96 * expansions


def cpu_baseline(sims: int, bs: int, c: float, budget_s: float = 15.0):
    """The oracle port (oracle/c4_oracle.c, bit-exact to the reference), timed on host cores."""
    import oracle
    threads = max(1, min(16, os.cpu_count() or 1))
    # calibrate on a small sample, then size the timed sample to ~budget_s
    n0 = threads
    t = time.perf_counter()
    oracle.get_move_batch(["." * 42] * n0, [0] * n0, list(range(n0)), sims, c, bs, threads=threads)
    rate0 = n0 * sims / max(time.perf_counter() - t, 1e-6)
    n = int(max(threads, min(65536, rate0 * budget_s / sims)))
    n = max(threads, (n // threads) * threads)
    t = time.perf_counter()
    _, _, _ = oracle.get_move_batch(["." * 42] * n, [0] * n, list(range(1000, 1000 + n)), sims, c, bs, threads=threads)
    dt = time.perf_counter() - t
    return {"value": round(n * sims / dt, 1), "unit": "expansions/s", "cores": threads, "kind": "port",
            "sample": f"{n} games x 1 move x {sims} sims from the opening (expansions = sims there), "
                      f"batch {bs}, {threads} pthreads, oracle/c4_oracle.c, {dt:.1f}s"}


MFMA_F16_PEAK_TFLOPS = 2500.0  # MI355X dense fp16 MFMA peak, ~2.5 PF (MI355X_MICROARCH.md; no sparsity)


def net_mode(games: int, sims: int, bs: int, c: float, steps: int, dev) -> dict:
    """C2(iii): the same search with a random-init value network instead of rollouts
    (stepwise search zc_c4_ext_*, fp16 ValueNetwork(128, 8, in_planes=2) between the select
    and backup kernels of every flush), one move per step captured in a HIP graph."""
    from zeroclone_amd.nets import ValueNetwork, flops_per_position, for_inference
    from zeroclone_amd.valued import C4ValuedSearch, NetValue
    torch.manual_seed(0)
    model = for_inference(ValueNetwork(128, 8, in_planes=2).eval(), dev, torch.float16)
    eng = _native.NativeEngine(max_games=games, max_sims=sims, max_batch=bs, device=dev.index)
    eng.seed(0, list(range(games)))
    vs = C4ValuedSearch(eng, games, bs, leaves=False)
    roots = torch.zeros((games, 3), dtype=torch.int64, device=dev)
    g = vs.capture(roots, sims, c, NetValue(model))
    g.replay()   # warm-up move
    torch.cuda.synchronize(dev)
    exp = 0
    t = time.perf_counter()
    for _ in range(steps):
        g.replay()
        exp += int(vs.stats[:, 0].sum().item())
    dt = time.perf_counter() - t
    flushes = (sims + bs - 1) // bs
    fl = flops_per_position(128, 8, 2, 6, 7) * games * bs * flushes * steps
    eng.close()
    return {"value": round(exp / dt, 1), "unit": "expansions/s", "ms_per_move": round(dt / steps * 1e3, 1),
            "net": "ValueNetwork(128, 8, in_planes=2) random init, fp16, BN folded, this package's MFMA conv kernels",
            "net_tflops_lower": round(fl / dt / 1e12, 1),
            "mfma_frac_lower": round(fl / dt / 1e12 / MFMA_F16_PEAK_TFLOPS, 4),
            "note": "TFLOP/s = network FLOPs / whole move time (search kernels included), so a lower bound "
                    "on the network's own rate; stepwise search, per-flush leaf planes built on the device"}


def chess_modes(steps: int, dev) -> dict:
    """BASELINE configs[3] (C4): chess, 1024 games, 400 sims/move — the crude-score search
    (configs/crude_chess.yaml, value in the kernel) and the value-network search
    (configs/chess_value.yaml: ValueNetwork(128, 8) random init, fp16, one move per HIP graph)."""
    import numpy as np
    from zeroclone_amd.nets import ValueNetwork, flops_per_position, for_inference
    from zeroclone_amd.valued import ChessValuedSearch, NetValue
    G, S, B = 1024, 400, 32
    eng = _native.NativeEngine(max_games=G, max_sims=S, max_batch=B, device=dev.index)
    eng.seed(0, list(range(G)))
    rows = np.array([_native.chess_init()] * G, _native.CHESS_STATE_DTYPE).view(np.uint8).reshape(G, 72)
    roots = torch.from_numpy(rows.copy()).to(dev)
    mv = torch.zeros(G, dtype=torch.int16, device=dev)
    na = torch.zeros((G, _native.CHESS_MAX_MOVES), dtype=torch.int32, device=dev)
    st = torch.zeros((G, _native.STATS_FIELDS), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    crude = lambda: eng.chess_search_async(0, G, roots.data_ptr(), S, 1.4, B, _native.ZC_POLICY_IMMEDIATE_VALUE,  # noqa
                                           3.0, mv.data_ptr(), na.data_ptr(), st.data_ptr(), s)
    crude()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    exp = 0
    for _ in range(steps):
        crude()
        exp += int(st[:, 0].sum().item())
    dt = time.perf_counter() - t
    out = {"crude": {"value": round(exp / dt, 1), "unit": "expansions/s", "ms_per_move": round(dt / steps * 1e3, 2),
                     "config": "1024 games x 400 sims, crude_chess_score, immediate_value(3), from the opening"}}
    torch.manual_seed(0)
    model = for_inference(ValueNetwork(128, 8).eval(), dev, torch.float16)
    vs = ChessValuedSearch(eng, G, B, leaves=False)
    g = vs.capture(roots, S, 1.4, NetValue(model))
    g.replay()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    exp = 0
    for _ in range(steps):
        g.replay()
        exp += int(vs.stats[:, 0].sum().item())
    dt = time.perf_counter() - t
    fl = flops_per_position(128, 8, 17, 8, 8) * G * B * ((S + B - 1) // B) * steps
    out["value_net"] = {"value": round(exp / dt, 1), "unit": "expansions/s", "ms_per_move": round(dt / steps * 1e3, 1),
                        "config": "1024 games x 400 sims, ValueNetwork(128, 8) random init fp16 (MFMA kernels), random policy",
                        "net_tflops_lower": round(fl / dt / 1e12, 1),
                        "mfma_frac_lower": round(fl / dt / 1e12 / MFMA_F16_PEAK_TFLOPS, 4)}
    eng.close()
    return out


def puct_mode(steps: int, dev) -> dict:
    """BASELINE configs[4] (C5) per GPU: chess PUCT self-play search, 1024 games x 1600 sims,
    policy + value ResNet (128 x 8, random init, fp16; tower on the MFMA kernels), Dirichlet
    root noise, one move per HIP graph."""
    import numpy as np
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork, flops_per_position
    from zeroclone_amd.valued import ChessPuctSearch
    G, S, B = 1024, 1600, 32
    eng = _native.NativeEngine(max_games=G, max_sims=S, max_batch=B, device=dev.index)
    rows = np.array([_native.chess_init()] * G, _native.CHESS_STATE_DTYPE).view(np.uint8).reshape(G, 72)
    roots = torch.from_numpy(rows.copy()).to(dev)
    torch.manual_seed(0)
    net = MfmaPolicyValueNetwork(PolicyValueNetwork().eval(), dev)
    ps = ChessPuctSearch(eng, G, B, seed=1, leaves=False)
    fn = lambda leaves, planes, counts: net(planes)  # noqa: E731
    g = ps.capture(roots, S, fn, temperature=1.0)
    g.replay()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    exp = 0
    for _ in range(steps):
        g.replay()
        exp += int(ps.stats[:, 0].sum().item())
    dt = time.perf_counter() - t
    nfl = _native.check(_native.lib().zc_chess_puct_flushes(S, B))
    fl = flops_per_position(128, 8, 17, 8, 8) * G * B * nfl * steps
    eng.close()
    return {"value": round(exp / dt, 1), "unit": "expansions/s", "ms_per_move": round(dt / steps * 1e3, 1),
            "config": "C5 per GPU: 1024 games x 1600 sims, PUCT c 1.5, Dirichlet(0.3, 0.25), policy+value ResNet "
                      "128x8 random init fp16 (MFMA tower), temperature 1",
            "net_tflops_lower": round(fl / dt / 1e12, 1), "mfma_frac_lower": round(fl / dt / 1e12 / MFMA_F16_PEAK_TFLOPS, 4)}


def philox_mode(eng, step, evs, acc, args, G: int, dev) -> dict:
    """C2(ii): the same self-play steps with ZC_ROLLOUT_PHILOX (leaf-parallel rollouts on
    per-leaf Philox-seeded streams; statistical parity, tests/test_gpu_philox.py)."""
    eng.c4_rollout_mode("philox", args.seed + 0xC2)
    try:
        step()
        torch.cuda.synchronize(dev)
        acc.zero_()
        t0 = time.perf_counter()
        for k in range(args.steps):
            step(evs[k])
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
    finally:
        eng.c4_rollout_mode("exact")
    kernel_ms = [a.elapsed_time(b) for a, b in evs]
    expansions = int(acc[0].item())
    return {"value": round(expansions / dt, 1), "unit": "expansions/s", "ms_per_step": round(dt / args.steps * 1e3, 3),
            "search_ms_per_step": [round(x, 3) for x in kernel_ms], "expansions": expansions,
            "config": f"C2(ii) {G} games x {args.sims} sims, batch {args.batch}: Philox rollout mode"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--games", type=int, default=4096, help="games per GPU")
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--c", type=float, default=1.4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--net-steps", type=int, default=1,
                    help="moves of the C2(iii) value-network mode reported under extra (0 = skip; N=1 only)")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="per-launch HBM bytes of the search kernel from a separate rocprofv3 --pmc pass")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    G, S, B = args.games, args.sims, args.batch
    eng = _native.NativeEngine(max_games=G, max_sims=S, max_batch=B, device=local)
    first_id = rank * G
    eng.seed(0, [args.seed + first_id + g for g in range(G)])

    roots = torch.zeros((G, 3), dtype=torch.int64, device=dev)   # zc_c4_state: stones[2], turn|reserved
    moves = torch.zeros(G, dtype=torch.int32, device=dev)
    na = torch.zeros((G, 7), dtype=torch.int32, device=dev)
    stats = torch.zeros((G, _native.STATS_FIELDS), dtype=torch.int64, device=dev)   # zc_game_stats
    results = torch.zeros(G, dtype=torch.int32, device=dev)
    acc = torch.zeros(4, dtype=torch.int64, device=dev)          # expansions, depth_sum, finished, leaves

    torch_stream = torch.cuda.Stream(dev)   # every launch of the step, and the timing events, on it
    torch.cuda.set_stream(torch_stream)

    def step(ev=None):
        stream = torch_stream.cuda_stream
        if ev is not None:
            ev[0].record()
        eng.c4_search_async(roots.data_ptr(), G, S, args.c, B, moves.data_ptr(), na.data_ptr(),
                            stats.data_ptr(), stream=stream)
        if ev is not None:
            ev[1].record()
        eng.c4_play_async(roots.data_ptr(), G, moves.data_ptr(), results.data_ptr(), reset=True, stream=stream)
        acc[0] += stats[:, 0].sum()
        acc[1] += stats[:, 1].sum()
        acc[2] += (results != _native.ZC_C4_ONGOING).sum()
        acc[3] += stats[:, 2].sum()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    acc.zero_()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0

    bad = int((stats[:, 5] != 0).sum().item())
    if bad:
        raise RuntimeError(f"{bad} games reported a nonzero search status")
    kernel_ms = [a.elapsed_time(b) for a, b in evs]
    tot = acc.clone()
    dtt = torch.tensor([dt], dtype=torch.float64, device=dev)
    kms = torch.tensor([sum(kernel_ms)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(dtt, op=dist.ReduceOp.MAX)
        dist.all_reduce(kms, op=dist.ReduceOp.MAX)
    expansions, depth_sum, finished, leaves = (int(x) for x in tot.tolist())
    dt_max = float(dtt.item())

    traffic, traffic_src = args.traffic_bytes, "--traffic-bytes" if args.traffic_bytes else None
    if traffic is None:  # the committed PMC summary of this kernel (tools/summarize_profile.py)
        import glob
        prof = sorted(glob.glob(os.path.join(HERE, "profiles", "r*_c4_search_summary.json")))
        if prof:
            with open(prof[-1]) as fh:
                hbm = json.load(fh).get("hbm")
            if hbm:
                traffic = hbm["bytes_per_launch"]
                traffic_src = os.path.relpath(prof[-1], HERE)

    # C3's one exchange: the all-gather of finished trajectories into the
    # replay buffer — here a payload of the right shape, this rank's K steps x G positions
    # (24-B zc_c4_state rows), through selfplay.gather_positions (RCCL over xGMI).  Off the
    # expansions/s clock, reported beside it.
    gather = None
    if world > 1:
        from zeroclone_amd.selfplay import gather_positions
        local = roots.repeat(args.steps, 1)
        gather_positions(local)  # warm the communicator
        dist.barrier()
        torch.cuda.synchronize(dev)
        tg = time.perf_counter()
        allpos = gather_positions(local)
        torch.cuda.synchronize(dev)
        gms = torch.tensor([(time.perf_counter() - tg) * 1e3], dtype=torch.float64, device=dev)
        dist.all_reduce(gms, op=dist.ReduceOp.MAX)
        gather = {"rows": int(allpos.shape[0]), "bytes": int(allpos.numel() * allpos.element_size()),
                  "ms": round(float(gms.item()), 3), "collective": "all_gather (counts, padded payload), backend nccl=RCCL"}

    if rank == 0:
        launches = args.steps * world
        bytes_launch = bytes_per_expansion_model(expansions, depth_sum) / launches
        avg_kernel_s = float(kms.item()) / 1e3 / args.steps
        achieved = bytes_launch / avg_kernel_s / 1e9
        out = {
            "metric": METRIC,
            "value": round(expansions / dt_max, 1),
            "unit": "expansions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: self-play from the empty board, per-game CPython MT19937 seeds base+game_id",
            "config": {"workload": f"C2/C3 Connect4 self-play, {G} games/GPU, {S} sims/move, batch {B}, "
                                   f"c {args.c}, random_rollout exact-RNG mode",
                       "games_per_gpu": G, "global_games": G * world, "sims": S, "batch_size": B,
                       "parallelism": f"games sharded over {world} GPU(s), 1 process/GPU"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "c4_search_kernel", "avg_launch_ms": round(avg_kernel_s * 1e3, 3),
                         "bytes_per_launch_model": round(bytes_launch),
                         "model": "SURVEY §8(d): 152*d+96 B per expansion, d counted in-kernel"},
            "extra": {"expansions": expansions, "leaves": leaves, "mean_depth": round(depth_sum / max(expansions, 1), 3),
                      "games_finished": finished, "search_ms_per_step": [round(x, 3) for x in kernel_ms]},
        }
        if gather is not None:
            out["extra"]["trajectory_allgather"] = gather
        # per-phase times (s_memtime stamps, one extra search with the stamped
        # kernel; shares applied to the unstamped launch time) and the tree-walk-only roofline
        # (select + expand-write + backup + publish; rollouts are integer VALU, not HBM).
        if world == 1:
            eng.phase_cycles(True)
            eng.c4_search_async(roots.data_ptr(), G, S, args.c, B, moves.data_ptr(), na.data_ptr(), stats.data_ptr(),
                                stream=torch_stream.cuda_stream)
            torch.cuda.synchronize(dev)
            ph = eng.phase_cycles(False)
            tot_c = max(sum(ph.values()), 1)
            share = {k: v / tot_c for k, v in ph.items() if k != "sub"}
            walk = sum(share[k] for k in ("rng", "walk_first", "walk_resumed", "expand", "backup", "publish"))
            out["extra"]["phases"] = {
                "share": {k: round(v, 4) for k, v in share.items()},
                "ms_per_launch": {k: round(v * avg_kernel_s * 1e3, 3) for k, v in share.items()},
                "walk_roofline": {"t_walk_ms": round(walk * avg_kernel_s * 1e3, 3),
                                  "achieved": round(bytes_launch / (walk * avg_kernel_s) / 1e9, 2),
                                  "frac": round(bytes_launch / (walk * avg_kernel_s) / 1e9 / HBM_PEAK_GBS, 5),
                                  "note": "SURVEY §8(d) roofline definition: model bytes / tree-walk time only"}}
        if world == 1 and args.net_steps > 0:
            out["extra"]["c2_philox"] = philox_mode(eng, step, evs, acc, args, G, dev)
            out["extra"]["c2_value_net"] = net_mode(G, S, B, args.c, args.net_steps, dev)
            out["extra"]["c4_chess"] = chess_modes(args.net_steps, dev)
            out["extra"]["c5_chess_puct"] = puct_mode(args.net_steps, dev)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(S, B, args.c)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
