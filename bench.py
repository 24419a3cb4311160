#!/usr/bin/env python3
"""bench.py — MCTS node-expansions/sec, Connect4 self-play at 800 sims/move (BASELINE.json).

Workload (BASELINE.json configs[1] = SURVEY.md §8(d) C2; with --gpus N it is C3's sharding):
4096 concurrent Connect4 self-play games per GPU, 800 simulations per move, leaf batch 32,
c = 1.4, the reference's random_rollout value and random expansion policy, exact-RNG mode
(every game's CPython MT19937 stream consumed in the reference's order).  One STEP = one
move for every game: the whole search (select/expand/rollout/backup x 800) on the GPU, then
Engine.play_move + _evaluate, trajectory recording (positions appended, finished games
labelled as Engine.get_dataset and pooled) and the refill of finished games
(scripts/train.py:151-170), all on the device (selfplay.C4SelfPlay).  Before the warm-up
the pool is run until every game slot has finished a game and started another, so the
timed steps see games of mixed ages (steady-state self-play), not the lockstep opening.
The K timed steps run as one free-running launch (C4SelfPlay.run, zc_c4_selfplay_async):
every game plays its K moves at its own pace — the same moves, trajectories and RNG streams
as K lockstep steps (tests/test_gpu_selfplay_run.py) — so young games (long rollouts) do not
stall the whole pool once per move.

Games are sharded across ranks by global game id (seed = base + id) — no collective on the
data path ("scaling": "weak").  `--gpus N` without torchrun spawns N fresh processes (one
per GPU; the parent never touches the GPU); under torchrun WORLD_SIZE must equal --gpus.
After the timed steps the positions of the games finished on every rank are all-gathered
into the replay buffer (RCCL over xGMI) — C3's one exchange, timed beside the metric.

value = expansions created on all ranks in the K timed steps / max over ranks of the wall
time of those K steps (barrier + device sync on both sides).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
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


def host_cpus() -> dict:
    """What the CPU baseline ran on: the threads used (the process's CPU share: the
    scheduler affinity, capped by OMP_NUM_THREADS where the box sets it), nproc, the model,
    and why (the affinity mask the process was given)."""
    aff_set = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    aff = len(aff_set)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    threads = max(1, min(aff, omp) if omp else aff)
    why = (f"the process's CPU share: sched_getaffinity allows {aff} of nproc {os.cpu_count()} CPUs "
           f"({_ranges(aff_set)})" + (f", OMP_NUM_THREADS={omp}" if omp else "")
           + f" -> {threads} threads")
    return {"threads": threads, "nproc": os.cpu_count(), "affinity": aff, "affinity_mask": _ranges(aff_set),
            "cpu_model": model, "why": why}


def _ranges(xs) -> str:
    out, i = [], 0
    while i < len(xs):
        j = i
        while j + 1 < len(xs) and xs[j + 1] == xs[j] + 1:
            j += 1
        out.append(str(xs[i]) if i == j else f"{xs[i]}-{xs[j]}")
        i = j + 1
    return ",".join(out)


def c4_row_board(row) -> tuple[str, int]:
    """[stones X, stones O, turn] -> (42-char board, row 0 at the top, '.' empty; turn)."""
    s0, s1, t = (int(x) for x in row)
    cells = []
    for r in range(6):
        for col in range(7):
            bit = 1 << (7 * col + (5 - r))
            cells.append("X" if s0 & bit else ("O" if s1 & bit else "."))
    return "".join(cells), t & 1


def pool_snapshot(sp, n: int = 1 << 30) -> dict:
    """The burned-in pool's state at the timed window's start, for the like-for-like CPU
    baseline: up to n games spread over the pool (every G/n-th slot; default all), their
    positions and their MT19937 states."""
    import oracle
    step = max(1, sp.G // n)
    idx = list(range(0, sp.G, step))[:n]
    rows = sp.roots.cpu().numpy()
    boards, turns, mts = [], [], []
    for g in idx:
        b, t = c4_row_board(rows[g])
        boards.append(b)
        turns.append(t)
        mt, k = sp.eng.get_rng_state(g)
        o = oracle.MT(0)
        o.s.mt[:] = [int(x) for x in mt]
        o.s.index = k
        mts.append(o)
    return {"boards": boards, "turns": turns, "mts": mts, "slots": idx}


def cpu_baseline(sims: int, bs: int, c: float, snap: dict, moves: int, budget_s: float = 20.0):
    """The oracle port (oracle/c4_oracle.c, bit-exact to the reference's get_move on the
    committed fixtures) on the SAME workload as the GPU window: the burned-in pool's games
    from the snapshot taken before the timed steps (mixed ages, their own MT19937 states),
    each playing the window's `moves` consecutive self-play moves (search, play, evaluate,
    refill) — the lockstep schedule of the same window, one game per pthread task across the
    host's CPU share.  A calibration round sizes the sample to about `budget_s` of CPU work:
    every game while that fits, else an evenly spread subset.  Expansions are counted as the
    GPU counts them (nodes created)."""
    import copy
    import oracle
    hc = host_cpus()
    threads = hc["threads"]
    boards, turns, mts = snap["boards"], snap["turns"], snap["mts"]
    G = len(boards)
    window = moves
    probe = list(range(0, G, max(1, G // (4 * threads))))[: 4 * threads]
    t = time.perf_counter()
    e0 = oracle.selfplay_batch([boards[i] for i in probe], [turns[i] for i in probe],
                               [copy.deepcopy(mts[i]) for i in probe], 1, sims, c, bs, threads=threads)
    per_game_move_s = (time.perf_counter() - t) / len(probe) * threads
    n = int(min(G, max(threads, budget_s * threads / (per_game_move_s * moves))))
    idx = list(range(G)) if n >= G else [int(i * G / n) for i in range(n)]
    if n >= G:   # the whole window fits the budget: play on past it (more of the same steady state)
        moves = int(min(4 * moves, max(moves, budget_s * threads / (per_game_move_s * G))))
    t = time.perf_counter()
    exp = oracle.selfplay_batch([boards[i] for i in idx], [turns[i] for i in idx], [copy.deepcopy(mts[i]) for i in idx],
                                moves, sims, c, bs, threads=threads)
    dt = time.perf_counter() - t
    ages = [sum(ch != "." for ch in boards[i]) for i in idx]
    value = float(exp.sum()) / dt
    # one thread on an evenly spread subset (~budget/6 s): the per-core rate, the scaling over
    # the CPU share, and what the whole affinity mask would give at that efficiency
    n1 = max(1, min(G, int(budget_s / 6 / (per_game_move_s / threads * moves))))
    i1 = [int(i * G / n1) for i in range(n1)]
    t = time.perf_counter()
    e1 = oracle.selfplay_batch([boards[i] for i in i1], [turns[i] for i in i1], [copy.deepcopy(mts[i]) for i in i1],
                               moves, sims, c, bs, threads=1)
    r1 = float(e1.sum()) / (time.perf_counter() - t)
    eff = value / (r1 * threads)
    scaling = {"one_thread": round(r1, 1), "one_thread_sample": f"{n1} games x {moves} moves",
               "efficiency_at_threads": round(eff, 3)}
    # The whole affinity mask is NOT run: on the GPU boxes sched_getaffinity shows the whole
    # machine's CPUs, but the harness gives each GPU's job a share of them (OMP_NUM_THREADS, 16 for
    # one GPU) and requires worker pools to be sized to that share — the other CPUs run the other
    # GPUs' jobs.  So the measured baseline is the share, and nothing is extrapolated beyond it.
    full_mask = {"value": None, "measured": False, "affinity": hc["affinity"],
                 "why": f"the harness allots this GPU's job {threads} of the {hc['affinity']} CPUs in the affinity "
                        f"mask (OMP_NUM_THREADS) and requires worker pools sized to that share; the port is timed "
                        f"on the share only, one thread and {threads} threads, and not extrapolated"}
    return {"value": round(value, 1), "unit": "expansions/s", "cores": threads, "kind": "port",
            "nproc": hc["nproc"], "cpu_model": hc["cpu_model"], "threads_why": hc["why"], "thread_scaling": scaling,
            "full_mask": full_mask,
            "port": "oracle/c4_oracle.c: C restatement pinned bit-exact to the reference's own get_move outputs "
                    "(tests/golden/c4_get_move.json, 150 cases incl. 800 sims) and rollouts",
            "sample": f"{len(idx)} of the {G} games of the burned-in GPU pool's snapshot before the timed window "
                      f"(mixed ages: {min(ages)}-{max(ages)} stones, their own MT19937 states) x {moves} consecutive "
                      f"self-play moves each (the window's {window} and on; search, play, evaluate, refill: the lockstep "
                      f"schedule), "
                      f"{sims} sims, batch {bs}; {int(exp.sum())} expansions counted as nodes created; {threads} "
                      f"pthreads, {dt:.1f}s (calibration: {len(probe)} games x 1 move, {e0.sum()} expansions)"}


def chess_pool_snapshot(pool) -> dict:
    """The burned-in crude chess pool's games at the timed window's start: positions
    (zc_chess_state rows) and MT19937 states, for the like-for-like chess CPU baseline."""
    import oracle
    rows = pool.roots.cpu().numpy().copy()
    mts = []
    for g in range(pool.G):
        mt, k = pool.eng.get_rng_state(g)
        o = oracle.MT(0)
        o.s.mt[:] = [int(x) for x in mt]
        o.s.index = k
        mts.append(o)
    return {"rows": rows, "mts": mts}


def cpu_baseline_chess(snap: dict, moves: int, sims: int = 400, bs: int = 32, c: float = 1.4, budget_s: float = 10.0):
    """Same-run CPU baseline of the chess crude mode (configs/crude_chess.yaml, C4 shape) on
    the SAME workload as the GPU window: the burned-in pool's games from the snapshot taken
    before the timed launch (mixed ages, their own MT19937 states), each playing consecutive
    crude-score self-play moves (search, play, judge, refill: oracle/chess_oracle.c
    zcc_selfplay_batch, whose search is bit-exact to the reference's get_move on the 26
    committed goldens) on the host's CPU share, sized by a calibration round to ~budget_s.
    Expansions are counted as nodes created, as the GPU counts them.  The positions carry no
    move histories (the pool's are on the device): a repetition draw can only come from moves
    played after the snapshot."""
    import copy
    import oracle
    hc = host_cpus()
    threads = hc["threads"]
    rows, mts = snap["rows"], snap["mts"]
    G = len(mts)
    probe = list(range(0, G, max(1, G // (2 * threads))))[: 2 * threads]
    t = time.perf_counter()
    oracle.chess_selfplay_batch(rows[probe], [copy.deepcopy(mts[i]) for i in probe], 1, sims, c, bs, threads=threads)
    per_game_move_s = (time.perf_counter() - t) / len(probe) * threads
    n = int(min(G, max(threads, budget_s * threads / (per_game_move_s * moves))))
    idx = list(range(G)) if n >= G else [int(i * G / n) for i in range(n)]
    if n >= G:
        moves = int(min(4 * moves, max(moves, budget_s * threads / (per_game_move_s * G))))
    t = time.perf_counter()
    exp = oracle.chess_selfplay_batch(rows[idx], [copy.deepcopy(mts[i]) for i in idx], moves, sims, c, bs,
                                      threads=threads)
    dt = time.perf_counter() - t
    return {"value": round(float(exp.sum()) / dt, 1), "unit": "expansions/s", "cores": threads, "kind": "port",
            "sample": f"{len(idx)} of the {G} games of the burned-in GPU pool's snapshot before the timed launch "
                      f"(mixed ages, their own MT19937 states) x {moves} consecutive crude-score self-play moves each "
                      f"(search, play, judge, refill; lockstep), {sims} sims, batch {bs}, immediate_value(3); "
                      f"{int(exp.sum())} expansions counted as nodes created; {threads} pthreads, {dt:.1f}s"}


def _cpu_net(planes: int, policy: bool = False, head: str = "conv"):
    """The network the reference evaluates on a host without a GPU (value_functions.py:61-99:
    DEVICE "cpu", DTYPE float32; models/chess_value/network.py:24-45), random init, with the
    process's CPU share as torch's intra-op threads."""
    from zeroclone_amd.nets import PolicyValueNetwork, ValueNetwork
    threads = host_cpus()["threads"]
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    if policy:
        return PolicyValueNetwork(head=head).eval(), threads
    return ValueNetwork(128, 8, in_planes=planes).eval(), threads


def _timed_moves(one, budget_s: float):
    """Calls one(k) for k = 0, 1, ... until budget_s has passed (at least twice); returns
    (moves, seconds)."""
    t = time.perf_counter()
    n = 0
    while n < 2 or time.perf_counter() - t < budget_s:
        one(n)
        n += 1
    return n, time.perf_counter() - t


def cpu_baseline_c4_net(sims: int, bs: int, c: float, budget_s: float = 10.0):
    """C2(iii) CPU baseline: the oracle's valued Connect4 get_move (oracle/c4_oracle.c,
    pinned to the reference's get_move on 40 valued goldens) with the fp32 ValueNetwork(128,
    8, in_planes=2) on the host, one batched forward per flush — the reference's network
    mode on a CPU box."""
    import numpy as np
    import oracle
    net, threads = _cpu_net(2)

    def vb(boards, turns):
        x = np.zeros((len(boards), 2, 6, 7), np.float32)
        for j, (b, t) in enumerate(zip(boards, turns)):
            a = np.frombuffer(b.encode(), np.uint8).reshape(6, 7)
            me, op = (ord("X"), ord("O")) if t == 0 else (ord("O"), ord("X"))
            x[j, 0], x[j, 1] = a == me, a == op
        with torch.no_grad():
            return net(torch.from_numpy(x)).reshape(-1).double().tolist()

    n, dt = _timed_moves(lambda k: oracle.get_move_valued("." * 42, 0, oracle.MT(1000 + k), sims, c, bs, vb), budget_s)
    return {"value": round(n * sims / dt, 1), "unit": "expansions/s", "cores": threads, "kind": "port",
            "sample": f"{n} Connect4 openings x {sims} sims (expansions ~= sims), batch {bs}, oracle valued get_move + "
                      f"fp32 ValueNetwork(128, 8, in_planes=2) on {threads} torch threads, {dt:.1f}s"}


def cpu_baseline_chess_net(sims: int = 400, bs: int = 32, c: float = 1.4, budget_s: float = 10.0):
    """C4 (chess value network) CPU baseline: the oracle's chess get_move (random policy,
    pinned to the reference's on 26 goldens) with the fp32 ValueNetwork(128, 8) over
    state_to_tensor planes, one batched forward per flush."""
    import numpy as np
    import oracle
    net, threads = _cpu_net(17)
    root = oracle.chess_init()

    def vb(leaves):
        x = np.stack([oracle.chess_tensor(oracle.chess_state(b.decode("latin-1"), t, f, cs)) for b, t, f, cs in leaves])
        with torch.no_grad():
            return net(torch.from_numpy(x)).reshape(-1).double().tolist()

    n, dt = _timed_moves(lambda k: oracle.chess_get_move(root, oracle.MT(2000 + k), sims, c, bs, value_batch=vb),
                         budget_s)
    return {"value": round(n * sims / dt, 1), "unit": "expansions/s", "cores": threads, "kind": "port",
            "sample": f"{n} chess openings x {sims} sims (expansions ~= sims), batch {bs}, oracle chess get_move + "
                      f"fp32 ValueNetwork(128, 8) on {threads} torch threads, {dt:.1f}s"}


def cpu_baseline_chess_puct(sims: int = 1600, bs: int = 32, c: float = 1.5, budget_s: float = 10.0):
    """C5 CPU baseline (PUCT has no reference counterpart): oracle/puct_ref.py, the search's
    executable specification, with the fp32 policy + value network on the host evaluating
    each flush's leaves in one batch (root noise off: it does not change the work)."""
    import numpy as np
    import oracle
    from oracle import puct_ref
    net, threads = _cpu_net(17, policy=True)
    root = oracle.chess_init()

    def one(k):
        cache = {}

        def key(s):
            return bytes(s.board) + bytes([s.turn, s.fifty, s.castle])

        def flush(states):
            if not states:
                return
            x = np.stack([oracle.chess_tensor(s) for s in states])
            with torch.no_grad():
                v, lg = net(torch.from_numpy(x))
            for s, vv, ll in zip(states, v.reshape(-1).tolist(), lg.numpy()):
                cache[key(s)] = (vv, ll)

        def prior(node):
            ll = cache[key(node.s)][1]
            idx = [(fr * 8 + fc) * 64 + tr * 8 + tc for fr, fc, tr, tc, _ in node.moves]
            e = np.exp(ll[idx] - ll[idx].max())
            return list(e / e.sum())

        puct_ref.search(root, sims, bs, c, lambda s: cache[key(s)][0], prior, flush_fn=flush)

    n, dt = _timed_moves(one, budget_s)
    return {"value": round(n * (sims - 1) / dt, 1), "unit": "expansions/s", "cores": threads, "kind": "port",
            "sample": f"{n} chess openings x {sims} sims, batch {bs}, PUCT specification oracle/puct_ref.py + fp32 conv-head "
                      f"PolicyValueNetwork (128 x 8) on {threads} torch threads, {dt:.1f}s"}


MFMA_F16_PEAK_TFLOPS = 2500.0  # MI355X dense fp16 MFMA peak, ~2.5 PF (MI355X_MICROARCH.md; no sparsity)


def _timed_pool_steps(pool, steps: int, warm: int = 1):
    """Steady-state network-mode self-play: the pool's whole step (search with its network
    between the select and backup kernels, play, record) captured as one HIP graph, `warm`
    untimed replays, then `steps` timed replays.  Returns (expansions, seconds) — the
    expansions from the pool's device totals (no per-step host read)."""
    g = pool.capture_step()
    for _ in range(warm):
        g.replay()
    torch.cuda.synchronize(pool.dev)
    pool.totals.zero_()
    t = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize(pool.dev)
    dt = time.perf_counter() - t
    exp = int(pool.totals[0].item())
    return exp, dt


MIXED = "steady-state self-play: the pool adopts a burned-in pool's games in progress (mixed ages), "


def net_rates(fl_pos: int, games: int, sims: int, bs: int, nfl: int, steps: int, dt: float,
              slots: int | None = None) -> dict:
    """Network FLOP rates of a network-mode step.  Useful FLOPs count the leaves the search
    evaluates (`sims` per move: every simulation's leaf, the PUCT root included); executed
    FLOPs count every slot the tower computes (`slots` per move; by default `nfl` flushes x
    `bs`: a short last flush's or the PUCT root flush's unused slots are padding).  Both over
    the whole step time (search, play and record included), so each is a lower bound on the
    tower's own rate at that work."""
    slots = bs * nfl if slots is None else slots
    useful = fl_pos * games * sims * steps
    executed = fl_pos * games * slots * steps
    return {"net_tflops_lower": round(useful / dt / 1e12, 1),
            "mfma_frac_lower": round(useful / dt / 1e12 / MFMA_F16_PEAK_TFLOPS, 4),
            "net_tflops_executed": round(executed / dt / 1e12, 1),
            "net_slots_per_move": slots, "net_leaves_per_move": sims}


def net_mode(src, games: int, sims: int, bs: int, c: float, steps: int, dev) -> dict:
    """C2(iii): Connect4 self-play whose search takes its leaf values from a random-init
    value network (stepwise search zc_c4_ext_*, fp16 ValueNetwork(128, 8, in_planes=2) on
    this package's MFMA tower between the select and backup kernels of every flush), from the
    burned-in rollout pool's positions; `steps` timed moves."""
    from zeroclone_amd.nets import ValueNetwork, flops_per_position, for_inference
    from zeroclone_amd.selfplay import C4SelfPlay
    torch.manual_seed(0)
    model = for_inference(ValueNetwork(128, 8, in_planes=2).eval(), dev, torch.float16)
    streams = 1   # split streams measured no faster here (profiles/r05_ab_split_streams.log)
    pool = C4SelfPlay(games, sims, c=c, batch_size=bs, seed=7, device=dev.index, net=model, streams=streams)
    pool.adopt(src)
    exp, dt = _timed_pool_steps(pool, steps)
    pool.close()
    rates = net_rates(flops_per_position(128, 8, 2, 6, 7), games, sims, bs, (sims + bs - 1) // bs, steps, dt)
    return {"value": round(exp / dt, 1), "unit": "expansions/s", "ms_per_move": round(dt / steps * 1e3, 1),
            "steps": steps, "config": MIXED + f"{games} games x {sims} sims, batch {bs}", "search_streams": streams,
            "net": "ValueNetwork(128, 8, in_planes=2) random init, fp16, BN folded, this package's MFMA conv kernels",
            **rates,
            "note": "net_tflops_lower = network FLOPs of the evaluated leaves / whole step time (search, play and "
                    "record included), a lower bound on the network's own rate; net_tflops_executed counts the "
                    "padded flush slots the tower also computes; one HIP graph per step"}


def c4_puct_mode(src, games: int, sims: int, bs: int, steps: int, dev) -> dict:
    """C2 with the PUCT extension (SURVEY §8 a21 on the target game): Connect4 self-play,
    4096 games x 800 sims, policy (7 column logits) + value ResNet 128x8 random init fp16 on
    the MFMA tower, Dirichlet root noise (fresh per move: per-game search numbers),
    temperature 1, from the burned-in rollout pool's positions."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork, flops_per_position
    from zeroclone_amd.selfplay import C4SelfPlay
    torch.manual_seed(0)
    net = MfmaPolicyValueNetwork(PolicyValueNetwork(in_planes=2, board=(6, 7), n_logits=7).eval(), dev)
    streams = 4   # the games in four parts on four streams (valued._split_flushes)
    pool = C4SelfPlay(games, sims, batch_size=bs, seed=7, device=dev.index, puct_net=net, temperature=1.0,
                      streams=streams)
    pool.adopt(src)
    exp, dt = _timed_pool_steps(pool, steps)
    pool.close()
    nfl = _native.check(_native.lib().zc_chess_puct_flushes(sims, bs))
    return {"value": round(exp / dt, 1), "unit": "expansions/s", "ms_per_move": round(dt / steps * 1e3, 1),
            "steps": steps, "search_streams": streams,
            "config": MIXED + f"C2 + PUCT: {games} games x {sims} sims, c_puct 1.5, Dirichlet(0.3, 0.25), policy "
                              "(7 logits) + value ResNet 128x8 random init fp16 (MFMA tower), temperature 1",
            # flush 0 runs the network on the roots alone (valued.PolicyNet): 1 + (nfl - 1) x bs boards
            **net_rates(flops_per_position(128, 8, 2, 6, 7), games, sims, bs, nfl, steps, dt,
                        slots=1 + (nfl - 1) * bs)}


def chess_burned_pool(dev, games: int = 1024, sims: int = 400, bs: int = 32, max_moves: int = 600):
    """The crude-score chess pool (configs/crude_chess.yaml: immediate_value(3)) run with the
    fused self-play launch until every slot has finished a game and started another (or
    max_moves): the mixed-age roots of the chess modes."""
    from zeroclone_amd.selfplay import ChessSelfPlay
    pool = ChessSelfPlay(games, sims, batch_size=bs, seed=3, device=dev.index)
    moves = 0
    while moves < max_moves:
        pool.run(25)
        moves += 25
        if int(pool.traj.slot[:, 1].min().item()) >= games:
            break
    pool.take()
    return pool, moves


def chess_modes(steps: int, dev) -> dict:
    """BASELINE configs[3] (C4): chess self-play, 1024 games, 400 sims/move — the crude-score
    search (configs/crude_chess.yaml, value in the kernel; the fused pooled launch) and the
    value-network search (configs/chess_value.yaml: ValueNetwork(128, 8) random init, fp16;
    one HIP graph per step), both from a burned-in pool (mixed game ages)."""
    from zeroclone_amd.nets import ValueNetwork, flops_per_position, for_inference
    from zeroclone_amd.selfplay import ChessSelfPlay
    G, S, B = 1024, 400, 32
    crude, burn = chess_burned_pool(dev, G, S, B)
    snap = chess_pool_snapshot(crude)
    K = max(steps, 20)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    ev[0].record()
    res = crude.run_pooled(K * G, 2 * K, kernel_done=ev[1])
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t
    exp = int(crude.stats[:, 0].sum().item())
    moves = int(((res != _native.ZC_SLOT_SKIP)).sum().item())
    out = {"crude": {"value": round(exp / dt, 1), "unit": "expansions/s", "ms_per_step": round(dt / K * 1e3, 3),
                     "steps": K, "moves": moves, "launch_ms": round(ev[0].elapsed_time(ev[1]), 2),
                     "burn_in_moves": burn,
                     "config": f"steady-state self-play (burned-in pool), {G} games x {S} sims, crude_chess_score, "
                               f"immediate_value(3); one pooled launch of {K} x {G} moves + its recording"}}
    torch.manual_seed(0)
    model = for_inference(ValueNetwork(128, 8).eval(), dev, torch.float16)
    pool = ChessSelfPlay(G, S, batch_size=B, seed=4, device=dev.index, net=model,
                         policy=_native.ZC_POLICY_RANDOM, freedom=0.0, streams=4)
    pool.adopt(crude)
    exp, dt = _timed_pool_steps(pool, steps)
    pool.close()
    out["value_net"] = {"value": round(exp / dt, 1), "unit": "expansions/s", "ms_per_move": round(dt / steps * 1e3, 1),
                        "steps": steps, "search_streams": 4,
                        "config": MIXED + f"{G} games x {S} sims, ValueNetwork(128, 8) random init fp16 (MFMA "
                                          "kernels), random policy",
                        # the short last flush runs the network on its leaves only (NetValue.rows)
                        **net_rates(flops_per_position(128, 8, 17, 8, 8), G, S, B, (S + B - 1) // B, steps, dt,
                                    slots=S)}
    out["_pool"] = crude
    out["_snap"] = snap
    return out


def puct_mode(src, steps: int, dev, head: str = "conv", streams: int = 4) -> dict:
    """BASELINE configs[4] (C5) per GPU: chess PUCT self-play, 1024 games x 1600 sims, policy
    + value ResNet (128 x 8, random init, fp16; tower on the MFMA kernels), Dirichlet root
    noise, temperature 1, from the burned-in crude pool's positions; one graph per step."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork, flops_per_position
    from zeroclone_amd.selfplay import ChessSelfPlay
    G, S, B = 1024, 1600, 32
    torch.manual_seed(0)
    net = MfmaPolicyValueNetwork(PolicyValueNetwork(head=head).eval(), dev)
    pool = ChessSelfPlay(G, S, batch_size=B, seed=6, device=dev.index, puct_net=net, temperature=1.0,
                         puct_streams=streams)
    pool.adopt(src)
    exp, dt = _timed_pool_steps(pool, steps)
    pool.close()
    nfl = _native.check(_native.lib().zc_chess_puct_flushes(S, B))
    return {"value": round(exp / dt, 1), "unit": "expansions/s", "ms_per_move": round(dt / steps * 1e3, 1),
            "steps": steps,
            "config": MIXED + "C5 per GPU: 1024 games x 1600 sims, PUCT c 1.5, Dirichlet(0.3, 0.25), policy+value "
                              "ResNet 128x8 random init fp16 (MFMA tower), temperature 1",
            "policy_head": ("convolutional (AlphaZero: 1x1 conv 128 -> 64, logit(from, to) = channel to at pixel "
                            "from; an epilogue of the tower launch, no GEMM)" if head == "conv" else
                            "linear (1x1 conv 128 -> 32 in the tower launch + Linear 2048 -> 4096 as a GEMM)"),
            "search_streams": streams,
            **net_rates(flops_per_position(128, 8, 17, 8, 8), G, S, B, nfl, steps, dt, slots=1 + (nfl - 1) * B)}


def c1_mode(dev, sims: int = 100, games: int = 4) -> dict:
    """BASELINE configs[0] (C1, plumbing): configs/connect4.yaml through the reference's own
    API — Engine(config).play_mcts(0, 100 sims) move after move until the game ends, 1 game —
    on the GPU (the package runs no search on the CPU), beside the C port playing the same
    games on one host thread.  Expansions per move = the sims (every simulation from a
    non-terminal position expands until the tree holds the whole game)."""
    import oracle
    from zeroclone_amd.engine import Engine
    cfg = os.path.join(HERE, "configs", "connect4.yaml")
    moves = 0
    t = time.perf_counter()
    for g in range(games):
        e = Engine(cfg)
        e.seed = 1000 + g
        while e.play_mcts(0, sims) is None:
            moves += 1
        moves += 1
    dt = time.perf_counter() - t
    tc = time.perf_counter()
    cmoves = 0
    for g in range(games):
        b, turn, mt = "." * 42, 0, oracle.MT(1000 + g)
        while True:
            col, _, _ = oracle.get_move_mt(b, turn, mt, sims, 1.4, 32)
            b, turn = oracle.play(b, turn, col)
            cmoves += 1
            if oracle.check_win(b, turn) or oracle.check_draw(b):
                break
    dtc = time.perf_counter() - tc
    return {"value": round(moves * sims / dt, 1), "unit": "simulations/s", "moves": moves, "games": games,
            "ms_per_move": round(dt / moves * 1e3, 2),
            "config": f"configs/connect4.yaml via Engine.play_mcts, 1 game at a time, {sims} sims/move, random_rollout, "
                      "whole games (host round trip per move: the reference's API, not a batched launch)",
            "cpu_baseline": {"value": round(cmoves * sims / dtc, 1), "unit": "simulations/s", "cores": 1, "kind": "port",
                             "sample": f"the same {games} games' moves on oracle/c4_oracle.c, one thread, {dtc:.2f}s"}}


def philox_mode(sp, args) -> dict:
    """C2(ii): the same self-play steps with ZC_ROLLOUT_PHILOX (leaf-parallel rollouts on
    per-leaf Philox-seeded streams; statistical parity, tests/test_gpu_philox.py)."""
    sp.eng.c4_rollout_mode("philox", args.seed + 0xC2)
    try:
        r = run_steps(sp, args.steps, warmup=1)
    finally:
        sp.eng.c4_rollout_mode("exact")
    return {"value": round(r["expansions"] / r["dt"], 1), "unit": "expansions/s",
            "ms_per_step": round(r["dt"] / args.steps * 1e3, 3),
            "selfplay_launch_ms": round(r["launch_ms"], 3), "expansions": r["expansions"],
            "config": f"C2(ii) {sp.G} games x {args.sims} sims, batch {args.batch}: Philox rollout mode"}


# ---------------------------------------------------------------------------------------------
def burn_in(sp, max_steps: int = 200, check_every: int = 8) -> int:
    """Step the pool until every slot has finished a game and started another (game numbers
    >= G everywhere): the timed window then sees games of mixed ages.  Returns the steps."""
    steps = 0
    while steps < max_steps:
        sp.run(check_every)
        steps += check_every
        if int(sp.traj.slot[:, 1].min().item()) >= sp.G:
            break
    sp.take()   # the burn-in's games are not the timed window's
    return steps


def run_steps(sp, steps: int, warmup: int, world: int = 1, launch: str = "pooled", carry: bool = True,
              drain: bool = True) -> dict:
    """W untimed moves, then K timed steps (K x G moves) bracketed by barrier + device sync,
    as ONE self-play launch followed by its trajectory recording; HIP events around it on its
    stream.  launch "pooled" (the default, C4SelfPlay.run_pooled): the G games share a budget
    of K x G moves drawn from a device counter, at most 2K per game, every move a full search
    — a throughput schedule (train.py:151-170 itself is lockstep: one move per unfinished
    game per call; each game's moves are exactly its free-run moves); "free"
    (C4SelfPlay.run): exactly K moves per game, so the launch waits for its slowest game.
    carry (pooled only, zc_c4_selfplay_carry_async): the warmup is a pooled launch too, and
    each launch's in-flight moves stop at their next flush once its budget is spent and
    resume in the next launch — the steady state of back-to-back launches: the timed launch
    finishes the moves the warmup left in flight and leaves its own for the (untimed) drain.
    Expansions are counted as they are made, so the window's work is what ran inside it."""
    dev = sp.dev
    stream = torch.cuda.current_stream(dev)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
          torch.cuda.Event(enable_timing=True))
    carry = carry and launch == "pooled"
    if warmup:
        if carry:
            sp.run_pooled(warmup * sp.G, 2 * warmup, carry=True)
        else:
            sp.run(warmup)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev[0].record(stream)
    if launch == "pooled":
        res = sp.run_pooled(steps * sp.G, 2 * steps, kernel_done=ev[2], carry=carry)
    else:
        res = sp.run(steps, kernel_done=ev[2])
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    st = sp.stats
    if int((st[:, 5] != 0).sum().item()):
        raise RuntimeError("a game reported a nonzero search status")
    fin = int(((res != _native.ZC_C4_ONGOING) & (res != _native.ZC_SLOT_IDLE)
               & (res != _native.ZC_SLOT_SKIP)).sum().item())
    moves = int(((res != _native.ZC_SLOT_IDLE) & (res != _native.ZC_SLOT_SKIP)).sum().item())
    tot = [int(x) for x in st[:, [0, 1, 2]].sum(0).tolist()]
    if carry and drain:   # untimed: finish the moves left in flight (the pool's later users search it)
        sp.drain()
        torch.cuda.synchronize(dev)
    return {"dt": dt, "launch_ms": ev[0].elapsed_time(ev[2]), "launch_record_ms": ev[0].elapsed_time(ev[1]), "expansions": tot[0], "depth_sum": tot[1],
            "finished": fin, "leaves": tot[2], "moves": moves}


def reduce_over_ranks(counts, dt: float, kernel_ms_sum: float, device) -> tuple[list[int], float, float]:
    """Whole-job aggregation: counters summed over ranks, wall time and kernel time the max
    over ranks (a no-op at world size 1)."""
    tot = torch.tensor(list(counts), dtype=torch.int64, device=device)
    t = torch.tensor([dt, kernel_ms_sum], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [int(x) for x in tot.tolist()], float(t[0].item()), float(t[1].item())


def rank_ranges(world: int, games: int) -> list[list[int]]:
    """Global game ids [first, last] of each rank (rank r owns r*G .. r*G+G-1)."""
    return [[r * games, r * games + games - 1] for r in range(world)]


def gather_trajectories(sp, world: int) -> dict:
    """C3's one collective: this rank's finished games' positions (the device
    pool, labels packed with the rows) all-gathered over ranks into the replay buffer."""
    out, _ = exchange_positions(sp.take_positions(), world, lambda: torch.cuda.synchronize(sp.dev))
    return out


def exchange_positions(local, world: int, sync=lambda: None):
    """The timed all-gather of `local` position rows (selfplay.positions_of) over the ranks:
    a warm-up exchange, barrier + sync, the timed one, its time max-reduced over ranks.
    Returns (report, gathered rows; None at world size 1)."""
    from zeroclone_amd.selfplay import gather_positions
    out = {"local_rows": int(local.shape[0])}
    if world == 1:
        return out, None
    gather_positions(local)  # warm the communicator
    dist.barrier()
    sync()
    tg = time.perf_counter()
    allpos = gather_positions(local)
    sync()
    gms = torch.tensor([(time.perf_counter() - tg) * 1e3], dtype=torch.float64, device=local.device)
    dist.all_reduce(gms, op=dist.ReduceOp.MAX)
    out.update({"rows": int(allpos.shape[0]), "bytes": int(allpos.numel() * allpos.element_size()),
                "ms": round(float(gms.item()), 3),
                "collective": "all_gather (counts, padded payload) of finished games' 24-B positions, "
                              + ("nccl=RCCL" if dist.get_backend() == "nccl" else dist.get_backend())})
    return out, allpos


# the committed rocprofv3 summaries (tools/summarize_profile.py, stamped with the sha256 of the
# library they profiled): the self-play kernel (HBM bytes per launch from separate FETCH_SIZE /
# WRITE_SIZE passes, SQ issue counters) and the walk-only replay kernel (tools/prof_walk.py)
SEARCH_PROFILE = os.path.join("profiles", "r06_c4_search_summary.json")
WALK_PROFILE = os.path.join("profiles", "r06_walk_summary.json")


def lib_sha() -> str:
    import hashlib
    with open(_native.LIB, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def load_profile(rel: str):
    """(summary, source) of a committed profile; the source says STALE when the summary's
    library stamp differs from the library this process loaded (its counters then describe
    other code)."""
    path = os.path.join(HERE, rel)
    if not os.path.exists(path):
        return {}, None
    with open(path) as fh:
        prof = json.load(fh)
    stamp = prof.get("lib_sha256")
    if stamp != lib_sha():
        return prof, f"{rel} (STALE: profiled library {str(stamp)[:12]}, loaded {lib_sha()[:12]})"
    return prof, rel


def search_profile():
    return load_profile(SEARCH_PROFILE)


def run_rank(args, rank: int, world: int, local: int):
    if args.share_device:   # rehearsal: every rank on GPU 0 (RCCL needs one GPU per rank)
        local = 0
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from zeroclone_amd.selfplay import C4SelfPlay
    G, S, B = args.games, args.sims, args.batch
    torch.cuda.set_stream(torch.cuda.Stream(dev))   # every launch and the timing events on one stream
    sp = C4SelfPlay(G, S, c=args.c, batch_size=B, seed=args.seed, rank=rank, device=local, record=True)
    burn = burn_in(sp) if args.burn_in else 0
    snap = pool_snapshot(sp) if (world == 1 and not args.no_cpu_baseline) else None
    r = run_steps(sp, args.steps, args.warmup, world, launch=args.launch, carry=not args.no_carry)
    gather = gather_trajectories(sp, world)
    counts, dt_max, kms = reduce_over_ranks([r["expansions"], r["depth_sum"], r["finished"], r["leaves"]], r["dt"],
                                            r["launch_ms"], dev)
    expansions, depth_sum, finished, leaves = counts
    if rank == 0:
        prof, prof_src = search_profile()
        traffic = args.traffic_bytes or (prof.get("hbm") or {}).get("bytes_per_launch")
        traffic_src = "--traffic-bytes" if args.traffic_bytes else prof_src
        traffic_stale = bool(traffic_src and "STALE" in traffic_src)
        launches = args.steps * world
        bytes_launch = bytes_per_expansion_model(expansions, depth_sum) / launches
        avg_kernel_s = kms / 1e3 / args.steps   # per move
        achieved = bytes_launch / avg_kernel_s / 1e9
        out = {
            "metric": METRIC if not args.share_device else "REHEARSAL (ranks share one GPU; not the metric): " + METRIC,
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
                                   f"c {args.c}, random_rollout exact-RNG mode, steady state (mixed game ages)",
                       "launch": (f"pooled: each step = {G} moves drawn by the games from one shared budget "
                                  f"(K x {G} per launch, <= 2K per game; every move a full {S}-sim search)"
                                  + ("; carry: once the budget is spent, in-flight moves stop at their next "
                                     "flush and resume in the next launch (warmup launch -> timed launch -> "
                                     "untimed drain), expansions counted as made" if not args.no_carry else "")
                                  if args.launch == "pooled" else f"free: K moves per game per launch"),
                       "games_per_gpu": G, "global_games": G * world, "sims": S, "batch_size": B,
                       "world_size": world, "rank_games": rank_ranges(world, G), "burn_in_steps": burn,
                       "parallelism": (f"games sharded over {world} GPU(s), 1 process/GPU" if not args.share_device
                                       else f"rehearsal: {world} ranks sharing GPU 0 over {args.dist_backend}")},
            # The search kernel is a per-game serial chain: SQ counters show neither HBM nor
            # an issue port saturated (profiles/r06_c4_search_summary.json: ~0.03 of HBM
            # bandwidth, SALU ~0.55 / VALU ~0.42 issue) — latency and issue arbitration bound it.  achieved / peak / frac
            # keep SURVEY §8(d)'s algorithmic HBM roofline; `issue` is the counter roofline.
            "roofline": {"bound": "issue", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "traffic_source": traffic_src, "traffic_stale": traffic_stale,
                         "kernel": "c4_selfplay_kernel (K x G moves per launch; per-step figures = launch / K)",
                         "avg_launch_ms": round(avg_kernel_s * 1e3, 3),
                         "bytes_per_launch_model": round(bytes_launch),
                         "model": "SURVEY §8(d): 152*d+96 B per expansion, d counted in-kernel",
                         "issue": dict(prof.get("issue") or {}, source=prof_src) if prof.get("issue") else None,
                         "limiter": "the per-game serial dependency chain (latency + issue arbitration), not HBM: "
                                    "roofline.issue (SQ counters) and DESIGN §4"},
            "extra": {"expansions": expansions, "leaves": leaves, "mean_depth": round(depth_sum / max(expansions, 1), 3),
                      "games_finished": finished, "moves": r["moves"],
                      "selfplay_launch_ms": round(r["launch_ms"], 3),
                      "trajectory_allgather": gather},
        }
        if world == 1:
            out["extra"]["phases"] = phases(sp, args, bytes_launch, avg_kernel_s)
            other = "free" if args.launch == "pooled" else "pooled"
            # the other schedule's own steady state: its warmup first (a pooled window leaves
            # more young, slow games in the pool than the lockstep schedule does)
            ro = run_steps(sp, args.steps, args.warmup, launch=other)
            out["extra"][f"launch_{other}"] = {"value": round(ro["expansions"] / ro["dt"], 1), "unit": "expansions/s",
                                               "ms_per_step": round(ro["dt"] / args.steps * 1e3, 3),
                                               "moves": ro["moves"], "expansions": ro["expansions"]}
            if args.launch == "pooled" and not args.no_carry:   # the same launch without carry-over
                rn = run_steps(sp, args.steps, 0, launch="pooled", carry=False)
                out["extra"]["launch_pooled_no_carry"] = {
                    "value": round(rn["expansions"] / rn["dt"], 1), "unit": "expansions/s",
                    "ms_per_step": round(rn["dt"] / args.steps * 1e3, 3),
                    "selfplay_launch_ms": round(rn["launch_ms"], 3), "moves": rn["moves"],
                    "note": "every in-flight move finished inside the launch: its tail (games finishing the "
                            "moves started just before the budget ran out, on an emptying device) is timed"}
            lock = out["value"] if args.launch == "free" else out["extra"]["launch_free"]["value"]
            out["extra"]["reference_schedule"] = {
                "value": lock, "unit": "expansions/s",
                "note": "scripts/train.py:151-170's lockstep schedule (every game exactly K moves per launch, the "
                        "launch ends with its slowest game) on the same pool and kernel, after W warmup moves of its "
                        "own; games behind the launch's average pace run at raised wave priority (pace balancing, "
                        "DESIGN round 6); the headline `value` is the pooled schedule (the games share K x G moves; "
                        "each game's moves are its lockstep moves)"}
        if world == 1 and args.net_steps > 0:
            out["extra"]["c2_philox"] = philox_mode(sp, args)
            out["extra"]["c2_value_net"] = net_mode(sp, G, S, B, args.c, args.net_steps, dev)
            out["extra"]["c2_puct"] = c4_puct_mode(sp, G, S, B, args.net_steps, dev)
            out["extra"]["record_overhead"] = record_overhead(sp, args)
            sp.close()
            sp = None
            chess = chess_modes(args.net_steps, dev)
            crude_pool = chess.pop("_pool")
            chess_snap = chess.pop("_snap")
            out["extra"]["c4_chess"] = chess
            out["extra"]["c5_chess_puct"] = puct_mode(crude_pool, args.net_steps, dev)
            # round 4's C5 network and schedule (linear policy head, one stream), for continuity
            out["extra"]["c5_chess_puct_linear_head"] = puct_mode(crude_pool, args.net_steps, dev, head="linear",
                                                                 streams=1)
            crude_pool.close()
            out["extra"]["net_tower"] = tower_mode(dev)
            out["extra"]["c1_engine"] = c1_mode(dev)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(S, B, args.c, snap, args.steps)
            if args.net_steps > 0:
                out["extra"]["c4_chess"]["crude"]["cpu_baseline"] = cpu_baseline_chess(
                    chess_snap, out["extra"]["c4_chess"]["crude"]["steps"])
                out["extra"]["c2_value_net"]["cpu_baseline"] = cpu_baseline_c4_net(S, B, args.c)
                out["extra"]["c4_chess"]["value_net"]["cpu_baseline"] = cpu_baseline_chess_net()
                out["extra"]["c5_chess_puct"]["cpu_baseline"] = cpu_baseline_chess_puct()
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if sp is not None:
        sp.close()
    if world > 1:
        dist.destroy_process_group()


def phases(sp, args, bytes_launch: float, avg_kernel_s: float) -> dict:
    """SURVEY §8(d) per-phase times (s_memtime stamps from one extra search with the stamped
    kernel build, shares applied to the unstamped launch time) and the tree walk MEASURED on
    its own: the walk-only replay kernel (walk_measure: the same search from a snapshot with
    the recorded rollout values in place of the rollouts, identical tree) timed with HIP
    events here, its HBM bytes per expansion from the committed rocprofv3 passes over the same
    workload (WALK_PROFILE: FETCH_SIZE x2 + WRITE_SIZE, tools/prof_walk.py)."""
    sp.eng.phase_cycles(True)
    sp.step()
    torch.cuda.synchronize(sp.dev)
    ph = sp.eng.phase_cycles(False)
    tot_c = max(sum(ph.values()), 1)
    share = {k: v / tot_c for k, v in ph.items() if k != "sub"}
    w = walk_measure(sp, reps=3)
    wprof, wsrc = load_profile(WALK_PROFILE)
    hbm = wprof.get("hbm") or {}
    run = wprof.get("run") or {}
    walk = {"kernel": "c4_walk_kernel<2> (replay) vs c4_search_kernel<false, false> (the full lockstep search)",
            "walk_ms": w["walk_ms"], "search_ms": w["search_ms"], "walk_share_of_search": w["walk_share_of_search"],
            "expansions": w["expansions"], "model_bytes": w["model_bytes"],
            "model_gbs": round(w["model_bytes"] / (w["walk_ms"] * 1e-3) / 1e9, 2),
            "profile": wsrc}
    if hbm.get("bytes_per_launch") and run.get("expansions"):
        per_exp = hbm["bytes_per_launch"] / run["expansions"]
        measured = per_exp * w["expansions"]
        gbs = measured / (w["walk_ms"] * 1e-3) / 1e9
        walk.update({"measured_bytes": round(measured), "measured_bytes_per_expansion": round(per_exp, 2),
                     "measured_gbs": round(gbs, 2), "measured_frac": round(gbs / HBM_PEAK_GBS, 5),
                     "profile_walk_ns": (wprof.get("trace_last_avg_ns") or None),
                     "stale": bool(wsrc and "STALE" in wsrc)})
    walk["note"] = ("measured_frac = the walk-only kernel's PMC HBM bytes (per expansion, from the profile, times "
                    "this run's expansions) over its own event time; model_gbs = SURVEY §8(d)'s 152 d + 96 model "
                    "bytes over the same time (the model charges a root-to-leaf re-read per simulation that the "
                    "kernel serves from LDS / L2, so it is not a rate and carries no frac)")
    return {"share": {k: round(v, 4) for k, v in share.items()},
            "ms_per_launch": {k: round(v * avg_kernel_s * 1e3, 3) for k, v in share.items()},
            "walk_roofline": walk}


def walk_measure(sp, reps: int = 5, check: bool = True) -> dict:
    """Record / search / replay from one snapshot of pool `sp` (see the module docstring);
    returns times (ms per launch, HIP events on the launch stream) and counts per launch."""
    G, S, B = sp.G, sp.sims, sp.bs
    dev = sp.dev
    st = torch.cuda.current_stream(dev)
    s = st.cuda_stream
    nfl = (S + B - 1) // B
    vals = torch.zeros((G, S), dtype=torch.int8, device=dev)
    words = torch.zeros((G, nfl), dtype=torch.int32, device=dev)
    rngbuf = torch.zeros(G * (4096 * 4 + 16), dtype=torch.uint8, device=dev)
    roots = sp.roots.clone()

    def outs():
        return (torch.zeros(G, dtype=torch.int32, device=dev), torch.zeros((G, 7), dtype=torch.int32, device=dev),
                torch.zeros((G, _native.STATS_FIELDS), dtype=torch.int64, device=dev))

    sp.eng.rng_copy(0, G, rngbuf.data_ptr(), False, s)
    rec = outs()
    sp.eng.c4_walk_async(0, G, roots.data_ptr(), S, sp.c, B, 1, vals.data_ptr(), words.data_ptr(),
                         rec[0].data_ptr(), rec[1].data_ptr(), rec[2].data_ptr(), s)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    sp.eng.rng_copy(0, G, rngbuf.data_ptr(), True, s)
    ful = outs()
    ev[0].record(st)
    sp.eng.c4_search_async(roots.data_ptr(), G, S, sp.c, B, ful[0].data_ptr(), ful[1].data_ptr(), ful[2].data_ptr(),
                           stream=s)
    ev[1].record(st)
    torch.cuda.synchronize(dev)
    search_ms = ev[0].elapsed_time(ev[1])
    walk = []
    for _ in range(reps):
        sp.eng.rng_copy(0, G, rngbuf.data_ptr(), True, s)
        rep = outs()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        sp.eng.c4_walk_async(0, G, roots.data_ptr(), S, sp.c, B, 2, vals.data_ptr(), words.data_ptr(),
                             rep[0].data_ptr(), rep[1].data_ptr(), rep[2].data_ptr(), s)
        e1.record(st)
        torch.cuda.synchronize(dev)
        walk.append(e0.elapsed_time(e1))
        if check:
            for a, b in ((rec, ful), (rec, rep)):
                assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), "moves / root visits differ"
                for k in (0, 1, 2, 4, 5):   # expansions, depth sum, leaves, words consumed, status
                    assert torch.equal(a[2][:, k], b[2][:, k]), f"stats field {k} differs"
    sp.eng.rng_copy(0, G, rngbuf.data_ptr(), True, s)   # leave the pool's streams as they were
    tot = rec[2][:, :2].sum(0).tolist()
    exp, dsum = int(tot[0]), int(tot[1])
    walk_ms = sorted(walk)[len(walk) // 2]
    return {"games": G, "sims": S, "batch": B, "expansions": exp, "depth_sum": dsum,
            "model_bytes": bytes_per_expansion_model(exp, dsum), "search_ms": round(search_ms, 4),
            "walk_ms": round(walk_ms, 4), "walk_ms_all": [round(x, 4) for x in walk],
            "walk_share_of_search": round(walk_ms / search_ms, 4)}


def tower_mode(dev, reps: int = 20, warm_s: float = 1.0) -> dict:
    """The value tower alone (ValueNetwork(128, 8) random init, chess 8x8 x 32768 boards = one
    C4 flush of 1024 games x 32 leaves): the fused launch (zc_net_tower_async, what every
    network mode runs) and the layer-by-layer packed launches, timed with HIP events; TFLOP/s
    over the MFMA work (stem on its 32 padded planes + 16 layers).  Timed the way the network
    modes run it, so that it is their ceiling: after ~warm_s of back-to-back launches (the clock
    settled under the MFMA load, as in a search's steps), once on one stream and once split over
    4 streams (quarter batches side by side, as the split-stream searches launch their parts);
    `ceiling` is the better of the two.  frac_of_2p5PF is the fraction of the nominal dense fp16
    peak, not of anything this chip sustains under its power cap."""
    from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork, flops_per_position
    from zeroclone_amd import _native
    torch.manual_seed(0)
    net = MfmaValueNetwork(ValueNetwork(128, 8, in_planes=17), dev)
    nets4 = [net.replica() if hasattr(net, "replica") else net for _ in range(4)]
    n = 32768
    x = (torch.rand(n, 17, 8, 8, device=dev) < 0.3).half()
    xs = list(x.chunk(4))
    flop = flops_per_position(128, 8, 32, 8, 8) * n
    out = {"boards": n, "board": "8x8", "net": "ValueNetwork(128, 8), fp16, BN folded",
           "form": "fused: 16x16x32 MFMA form (the default); fused_32x32x16: the round-3 form (tower_mf 32)",
           "timing": f"HIP events over {reps} launches after ~{warm_s:.1f} s of warm-up launches; streams4: the "
                     "batch as 4 quarter launches on 4 streams per rep (the split-stream searches' pattern)"}
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    saved = _native.net_switch("tower_mf", 0)

    def timed(fn, nreps):
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        torch.cuda.synchronize(dev)
        ev[0].record()
        for _ in range(nreps):
            fn()
        ev[1].record()
        torch.cuda.synchronize(dev)
        return ev[0].elapsed_time(ev[1]) / nreps

    def split4():
        cur = torch.cuda.current_stream(dev)
        for st, nt, xq in zip(streams, nets4, xs):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                nt.tower(xq)
        for st in streams:
            cur.wait_stream(st)

    for key, fused, mf in (("fused", True, 0), ("fused_32x32x16", True, 32), ("layered", False, 0)):
        _native.net_switch("tower_mf", mf)
        one = timed(lambda: net.tower(x, fused=fused), 1)
        timed(lambda: net.tower(x, fused=fused), max(1, int(warm_s * 1e3 / max(one, 0.1))))   # warm the clock
        ms = timed(lambda: net.tower(x, fused=fused), reps)
        out[key] = {"ms": round(ms, 3), "tflops": round(flop / ms / 1e9, 1),
                    "frac_of_2p5PF": round(flop / ms / 1e9 / MFMA_F16_PEAK_TFLOPS, 4)}
    _native.net_switch("tower_mf", 0)
    timed(split4, max(1, int(warm_s * 1e3 / max(out["fused"]["ms"], 0.1))))
    ms4 = timed(split4, reps)
    out["fused_streams4"] = {"ms": round(ms4, 3), "tflops": round(flop / ms4 / 1e9, 1),
                             "frac_of_2p5PF": round(flop / ms4 / 1e9 / MFMA_F16_PEAK_TFLOPS, 4)}
    _native.net_switch("tower_mf", saved)
    best = max(out["fused"]["tflops"], out["fused_streams4"]["tflops"])
    out["ceiling_tflops"] = best
    out["ceiling_note"] = ("the better of the warm one-stream and the 4-stream fused tower: the rate the network "
                           "modes' towers cannot exceed on this shape (their net_tflops_lower counts the whole step)")
    out["pmc"] = "profiles/r06_tower_pmc.json (MFMA busy, held clock, LDS bank conflicts)"
    return out


def record_overhead(sp, args) -> dict:
    """Trajectory recording's cost: the same steady-state steps with and without the
    recording (zc_traj_record_steps_async).  The unrecorded run leaves the pool's slot
    histories behind its games, so it runs last, just before the pool is closed."""
    on = run_steps(sp, args.steps, warmup=1)
    sp.record = False
    try:
        off = run_steps(sp, args.steps, warmup=1)
    finally:
        sp.record = True
    return {"ms_per_step_recorded": round(on["dt"] / args.steps * 1e3, 3),
            "ms_per_step_unrecorded": round(off["dt"] / args.steps * 1e3, 3),
            "ratio": round(on["dt"] / max(off["dt"], 1e-9), 4)}


def visible_gpus(kfd_root: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs this process may use, counted WITHOUT initialising HIP (the parent must not touch
    the GPU before it spawns the ranks): the KFD topology's GPU nodes (simd_count > 0),
    narrowed by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES.  Raises
    when the topology is unreadable: no fallback to hipGetDeviceCount."""
    try:
        nodes = [os.path.join(kfd_root, d) for d in os.listdir(kfd_root)]
    except OSError as e:
        raise RuntimeError(f"cannot count GPUs without HIP: {kfd_root} unreadable ({e})") from None
    n = 0
    for d in nodes:
        try:
            with open(os.path.join(d, "properties")) as fh:
                props = dict(line.split()[:2] for line in fh if len(line.split()) >= 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawned(rank: int, args, world: int, port: int):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world)})
    run_rank(args, rank, world, rank)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60,
                    help="timed moves (one free-running launch; about a game length, so every slot's "
                         "games of all ages share the window)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--launch", choices=["pooled", "free"], default="pooled",
                    help="pooled: the games share K x G moves per launch; free: K moves per game")
    ap.add_argument("--no-carry", action="store_true",
                    help="pooled launches finish their in-flight moves (no carry-over into the next launch)")
    ap.add_argument("--games", type=int, default=4096, help="games per GPU")
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--c", type=float, default=1.4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-burn-in", dest="burn_in", action="store_false",
                    help="time from the lockstep opening instead of steady-state self-play")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--net-steps", type=int, default=5,
                    help="timed steady-state moves of the network / chess modes reported under extra "
                         "(0 = skip; N=1 only)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend of the N-rank run (nccl = RCCL over xGMI)")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal of the N-rank path on a one-GPU box: every rank on GPU 0 (use gloo); "
                         "the line is marked as a rehearsal, never the metric")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="per-launch HBM bytes of the search kernel from a separate rocprofv3 --pmc pass")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if "WORLD_SIZE" in os.environ:   # launched by torchrun: one rank per process already
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
        run_rank(args, int(os.environ.get("RANK", "0")), world, int(os.environ.get("LOCAL_RANK", "0")))
        return
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus == 1:
        run_rank(args, 0, 1, 0)
        return
    try:
        visible = visible_gpus()   # the KFD topology: no HIP call in this (parent) process
    except RuntimeError as e:
        raise SystemExit(f"bench.py: {e}")
    if args.gpus > visible and not (args.share_device and visible >= 1):
        raise SystemExit(f"bench.py: --gpus {args.gpus} but only {visible} GPU(s) visible")
    if args.share_device and args.dist_backend == "nccl":
        raise SystemExit("bench.py: --share-device needs --dist-backend gloo (RCCL wants one GPU per rank)")
    import torch.multiprocessing as mp
    mp.spawn(_spawned, args=(args, args.gpus, _free_port()), nprocs=args.gpus, join=True)


if __name__ == "__main__":
    main()
