"""The self-play pools bench.py times, replayed through the oracle at their own shapes
(BASELINE configs C2(iii), C4 and C5 per GPU), from burned-in pools of mixed game ages —
what scripts/train.py:151-170 drives over engine/engine.py:119-153: per game, per move, the
search (mcts.get_move, engine/mcts/src/mcts.cpp:102-160), play_move and _evaluate
(chess_backend.cpp:364-441: checkmate, stalemate, the fifty-move rule, both sides'
repetition histories), and the refill of a finished game.

* chess crude pool (configs/crude_chess.yaml, 1024 games x 400 sims, batch 32): the pooled
  launch (chess_selfplay_kernel, 2 x 1024 moves, <= 4 per game) — every move of 64 sampled
  games through oracle.chess_get_move (immediate_value(3), crude_chess_score) from the
  snapshotted root, both sides' histories and MT19937 state; move, post-move row, result,
  refill and the MT state after the launch;
* chess value-network pool (configs/chess_value.yaml: ValueNetwork(128, 8) fp16 on the
  MFMA tower, random policy) adopting that pool: 2 steps (search, chess_play_step_kernel,
  record), the network's values logged per flush and replayed into oracle.chess_get_move;
* chess PUCT pool (C5 per GPU: 1024 games x 1600 sims, policy + value net, Dirichlet noise,
  temperature 1) adopting it: 1 step, root visit counts of sampled games through
  oracle/puct_ref.py with the logged values and the device's priors, the move played and
  judged against the oracle;
* Connect4 value-network pool (C2(iii): 4096 games x 800 sims, ValueNetwork(128, 8,
  in_planes=2)) adopting a burned-in rollout pool: 2 steps, values replayed into
  oracle.get_move_valued.
"""
import numpy as np
import pytest
import torch

import oracle
from oracle import puct_ref
from zeroclone_amd import _native

pytestmark = pytest.mark.gpu

ONGOING, SKIP = _native.ZC_C4_ONGOING, _native.ZC_SLOT_SKIP
CG, CS, CB = 1024, 400, 32


def oracle_mt(eng, g):
    mt, idx = eng.get_rng_state(g)
    o = oracle.MT(0)
    o.s.mt[:] = [int(x) for x in mt]
    o.s.index = idx
    return o


def same_mt(eng, g, mt):
    m, idx = eng.get_rng_state(g)
    return [int(x) for x in m] == list(mt.s.mt) and idx == mt.s.index


def pack(m):
    fr, fc, tr, tc, v = m
    return (fr * 8 + fc) | ((tr * 8 + tc) << 6) | (int(v) << 12)


def ostate(row, hist, hlen):
    """Device row (zc_chess_state) + histories (play order) -> oracle state (most recent first)."""
    r = np.asarray(row, np.uint8).view(_native.CHESS_STATE_DTYPE)[0]
    s = oracle.ZccState()
    s.board[:] = [int(x) for x in r["board"]]
    s.turn, s.fifty, s.castle = int(r["turn"]), int(r["fifty"]), int(r["castle"])
    for side, name in ((0, "hw"), (1, "hb")):
        n = int(hlen[side])
        if n > oracle.ZCC_HIST - 16:   # longer than the oracle's history holds: not sampled
            return None
        arr = getattr(s, name)
        for i in range(n):
            m = int(hist[side, n - 1 - i]) & 0xFFFF
            (fr, fc, tr, tc), v = _native.unpack_chess_move(m)
            arr[i] = oracle.ZccMove(fr, fc, tr, tc, v)
        setattr(s, "n" + name, n)
    return s


def same_row(s, row):
    r = np.asarray(row, np.uint8).view(_native.CHESS_STATE_DTYPE)[0]
    return (list(r["board"]) == list(s.board) and int(r["turn"]) == s.turn and int(r["fifty"]) == s.fifty
            and int(r["castle"]) == s.castle)


def judge(s):
    """Engine._evaluate (engine.py:148-153) of the oracle state."""
    if oracle.chess_win(s):
        return s.turn * 2 - 1
    return 0 if oracle.chess_draw(s) else ONGOING


def snapshot(pool, sample):
    roots = pool.roots.cpu().numpy().copy()
    hist = pool.hist.cpu().numpy().copy()
    hlen = pool.hlen.cpu().numpy().copy()
    snap = {g: (ostate(roots[g], hist[g], hlen[g]), oracle_mt(pool.eng, g)) for g in sample}
    snap = {g: v for g, v in snap.items() if v[0] is not None}
    assert len(snap) >= len(sample) - max(2, len(sample) // 50)
    return snap, roots


FIFTY_NEXT = "4k3/8/8/8/8/8/8/4K2R w K - 49 30"   # every legal move is quiet: a fifty-move draw


def inject_fifty(pool, slots):
    """Put a position one quiet move from the fifty-move draw (no history) into `slots`: each
    of these games ends at its next move and its slot refills — so every pool test below sees
    at least one game end and refill at the timed shape (VERDICT r4 Weak 8)."""
    from zeroclone_amd.engine.games.chess import chess_backend as cb
    row = torch.from_numpy(cb.to_zc(cb.state_from_fen(FIFTY_NEXT)).reshape(1).view(np.uint8).copy()).to(pool.dev)
    for g in slots:
        pool.roots[g] = row
        pool.hlen[g] = 0


def ended_slots(res, limit):
    """Slots (sorted) whose game ended during the replayed steps, at most `limit`."""
    r = np.asarray(res).reshape(-1, np.asarray(res).shape[-1])
    hit = ((r != ONGOING) & (r != SKIP)).any(axis=0)
    return sorted(np.nonzero(hit)[0].tolist())[:limit]


@pytest.fixture(scope="module")
def chess_pool():
    from zeroclone_amd.selfplay import ChessSelfPlay
    pool = ChessSelfPlay(CG, CS, batch_size=CB, seed=3)   # configs/crude_chess.yaml: immediate_value(3)
    moves = 0
    while moves < 600:   # bench.py chess_burned_pool: every slot has finished a game and started another
        pool.run(25)
        moves += 25
        if int(pool.traj.slot[:, 1].min().item()) >= CG:
            break
    pool.take()
    yield pool
    pool.close()


def test_chess_crude_pooled_launch_matches_oracle(chess_pool):
    """64 evenly spread games plus up to 16 whose game ended in the launch (two of them put one
    move from the fifty-move draw first), every move replayed through the oracle: at least one
    game end and refill is checked at the timed shape."""
    pool = chess_pool
    inject_fifty(pool, [7, 519])
    snap_all, roots = snapshot(pool, list(range(CG)))
    assert len({bytes(r[:64]) for r in roots}) > CG // 2, "mixed positions, not the lockstep opening"
    res = pool.run_pooled(2 * CG, 4).cpu().numpy()
    states, moves = pool._run_states.cpu().numpy(), pool._run_moves.cpu().numpy()
    assert int((res != SKIP).sum()) == 2 * CG
    pool.check()
    sample = sorted(set(range(0, CG, 16)) | set(ended_slots(res, 16)))
    snap = {g: snap_all[g] for g in sample if g in snap_all}
    checked = ended = 0
    for g, (s, mt) in snap.items():
        for k in range(res.shape[0]):
            r = int(res[k, g])
            if r == SKIP:
                assert (res[k:, g] == SKIP).all(), g
                break
            best, ms, _ = oracle.chess_get_move(s, mt, CS, 1.4, CB, "immediate_value", 3.0)
            assert int(moves[k, g]) & 0xFFFF == pack(ms[best]), (g, k)
            s = oracle.chess_play(s, ms[best])
            assert same_row(s, states[k, g]), (g, k)
            exp = judge(s)
            assert r == exp, (g, k, r, exp)
            if exp != ONGOING:
                s = oracle.chess_init()
                ended += 1
            checked += 1
        assert same_mt(pool.eng, g, mt), g
    assert checked >= len(sample)
    assert ended >= 2, ended   # the refill path ran (at least the two fifty-move slots)


def test_chess_value_net_pool_matches_oracle(chess_pool):
    from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork, for_inference
    from zeroclone_amd.selfplay import ChessSelfPlay
    torch.manual_seed(0)
    model = for_inference(ValueNetwork(128, 8).eval(), "cuda", torch.float16)
    assert isinstance(model, MfmaValueNetwork)
    pool = ChessSelfPlay(CG, CS, batch_size=CB, seed=4, net=model, policy=_native.ZC_POLICY_RANDOM, freedom=0.0)
    pool.adopt(chess_pool)
    inject_fifty(pool, [37, 901])
    snap_all, _ = snapshot(pool, list(range(CG)))
    log = []
    inner = pool.value_fn

    def logged(leaves, planes, counts):
        v = inner(leaves, planes, counts)
        log.append(v.reshape(-1).cpu().numpy().copy())
        return v

    pool.value_fn = logged
    steps = []
    for _ in range(2):
        res = pool.step().cpu().numpy().copy()
        steps.append((pool.moves.cpu().numpy().copy(), pool.post.cpu().numpy().copy(), res,
                      pool.roots.cpu().numpy().copy()))
    pool.check()
    nfl = (CS + CB - 1) // CB
    assert len(log) == 2 * nfl
    assert np.unique(np.round(log[-1], 5)).size > 20   # not a constant network
    sample = sorted(set(range(5, CG, 32)) | set(ended_slots([st[2] for st in steps], 16)))
    snap = {g: snap_all[g] for g in sample if g in snap_all}
    ended = 0
    for g, (s, mt) in snap.items():
        for k, (mv, post, res, roots_after) in enumerate(steps):
            it = iter(log[k * nfl:(k + 1) * nfl])

            def replay(ls, g=g, it=it):
                v = next(it)
                return [float(x) for x in v[g * CB: g * CB + len(ls)]]

            best, ms, _ = oracle.chess_get_move(s, mt, CS, 1.4, CB, "random", 0.0, value_batch=replay)
            assert int(mv[g]) & 0xFFFF == pack(ms[best]), (g, k)
            s = oracle.chess_play(s, ms[best])
            exp = judge(s)
            assert int(res[g]) == exp, (g, k)
            if exp != ONGOING:   # the refill: the opening, empty histories
                s = oracle.chess_init()
                ended += 1
            # the step's post-move row; the recording refills a finished game's row in place
            assert same_row(s, post[g]), (g, k)
            assert same_row(s, roots_after[g]), (g, k)
        assert same_mt(pool.eng, g, mt), g
    assert ended >= 2, ended
    pool.close()


def _key_row(r):
    r = bytes(r)
    return r[:64], r[64], r[65], r[66]


def _key_zcc(s):
    return bytes(s.board), int(s.turn), int(s.fifty), int(s.castle)


def test_c5_chess_puct_pool_matches_puct_ref(chess_pool):
    from zeroclone_amd.nets import MfmaPolicyValueNetwork, PolicyValueNetwork
    from zeroclone_amd.selfplay import ChessSelfPlay
    S = 1600
    torch.manual_seed(13)
    net = MfmaPolicyValueNetwork(PolicyValueNetwork(head="conv").eval())   # the head bench.py times
    # the schedule bench.py times: the games in two halves on two streams (ChessPuctSearch._enqueue_split)
    pool = ChessSelfPlay(CG, S, batch_size=CB, seed=6, puct_net=net, temperature=1.0, puct_streams=2)
    pool.adopt(chess_pool)
    pool.ps.leaves = torch.zeros((CG * CB, 72), dtype=torch.uint8, device=pool.dev)   # export leaves (test hook)
    sampled = list(range(3, CG, 32)) + [68, 644]   # 32 spread games + two one move from the fifty-move draw
    inject_fifty(pool, [68, 644])
    snap, _ = snapshot(pool, sampled)
    assert len(snap) >= 32
    logs = {g: {} for g in sampled}

    def part_fn(lo, hi):   # the logging network of the part holding games [lo, hi)
        mine = [g for g in sampled if lo <= g < hi]
        rows_idx = torch.tensor([(g - lo) * CB + j for g in mine for j in range(CB)], device=pool.dev,
                                dtype=torch.long)
        m = net.replica()

        def fn(leaves, planes, counts):
            v, logits = m(planes)
            if mine:
                lv = leaves[rows_idx].cpu().numpy()
                vv = v.reshape(-1)[rows_idx].cpu().numpy()
                ll = logits[rows_idx].float().cpu().numpy()
                cnt = counts.cpu().numpy()
                for a, g in enumerate(mine):
                    for j in range(int(cnt[g - lo])):
                        logs[g].setdefault(_key_row(lv[a * CB + j]), (float(vv[a * CB + j]), ll[a * CB + j]))
            return v, logits
        return fn

    pool.net_fn = [part_fn(0, CG // 2), part_fn(CG // 2, CG)]
    res = pool.step().cpu().numpy()
    mv, post = pool.moves.cpu().numpy(), pool.post.cpu().numpy()
    roots_after = pool.roots.cpu().numpy()
    na = pool.ps.na.cpu().numpy()
    pool.check()
    ended = 0
    for g, (root, _) in snap.items():
        tree = pool.eng.debug_chess_tree(g)
        nodes, tp = tree["nodes"], tree["prior"]
        pri = {}
        for i, nd in enumerate(nodes):
            if nd["evaluated"] and i:
                pri[_key_row(nd["st"])] = tp[nd["base"]: nd["base"] + nd["nmoves"]].astype(np.float64)
        root_p = tp[nodes[0]["base"]: nodes[0]["base"] + nodes[0]["nmoves"]].astype(np.float64)
        calls = []

        def prior_fn(node, g=g, pri=pri, root_p=root_p, calls=calls):
            calls.append(1)
            return list(root_p) if len(calls) == 1 else list(pri[_key_zcc(node.s)])

        moves, N, _ = puct_ref.search(root, S, CB, 1.5, lambda s, g=g: logs[g][_key_zcc(s)][0], prior_fn)
        assert N == [int(x) for x in na[g, :len(moves)]], g
        # the move played: a visited root move (temperature 1 samples by N), then play + judge
        played = [m for m in moves if pack(m) == int(mv[g]) & 0xFFFF]
        assert len(played) == 1 and N[moves.index(played[0])] > 0, g
        s = oracle.chess_play(root, played[0])
        assert int(res[g]) == judge(s), g
        if int(res[g]) != ONGOING:   # the refill: the next root (and the recorded row) is the opening
            ended += 1
            s = oracle.chess_init()
        assert same_row(s, post[g]), g
        assert same_row(s, roots_after[g]), g
    assert ended >= 2, ended
    pool.close()


@pytest.fixture(scope="module")
def c4_pool():
    from zeroclone_amd.selfplay import C4SelfPlay
    sp = C4SelfPlay(4096, 800, batch_size=32, seed=2024, record=True)
    burn = 0
    while burn < 200:   # bench.py burn_in
        sp.run(8)
        burn += 8
        if int(sp.traj.slot[:, 1].min().item()) >= sp.G:
            break
    sp.take()
    yield sp
    sp.close()


def _board(row):
    s0, s1, t = (int(x) for x in row)
    cells = []
    for r in range(6):
        for c in range(7):
            bit = 1 << (7 * c + (5 - r))
            cells.append("X" if s0 & bit else ("O" if s1 & bit else "."))
    return "".join(cells), t & 1


def test_c2iii_connect4_value_net_pool_matches_oracle(c4_pool):
    from zeroclone_amd.nets import MfmaValueNetwork, ValueNetwork, for_inference
    from zeroclone_amd.selfplay import C4SelfPlay
    G, S, B = 4096, 800, 32
    torch.manual_seed(0)
    model = for_inference(ValueNetwork(128, 8, in_planes=2).eval(), "cuda", torch.float16)
    assert isinstance(model, MfmaValueNetwork)
    pool = C4SelfPlay(G, S, batch_size=B, seed=7, net=model)
    pool.adopt(c4_pool)
    roots = pool.roots.cpu().numpy().copy()
    ages = [sum(ch != "." for ch in _board(roots[g])[0]) for g in range(1, G, 64)]
    assert max(ages) - min(ages) >= 10   # mixed game ages
    mts = {g: oracle_mt(pool.eng, g) for g in range(G)}
    log = []
    inner = pool.value_fn

    def logged(leaves, planes, counts):
        v = inner(leaves, planes, counts)
        log.append((v.reshape(-1).cpu().numpy().copy(), counts.cpu().numpy().copy()))
        return v

    pool.value_fn = logged
    steps = []
    for _ in range(2):
        res = pool.step().cpu().numpy().copy()
        steps.append((pool.moves.cpu().numpy().copy(), res, pool.roots.cpu().numpy().copy()))
    assert int(pool.stats[:, 5].abs().sum()) == 0
    nfl = (S + B - 1) // B
    assert len(log) == 2 * nfl
    # 64 spread games plus up to 32 whose game ended in one of the two steps
    sample = sorted(set(range(1, G, 64)) | set(ended_slots([st[1] for st in steps], 32)))
    ended = 0
    for g in sample:
        b, t = _board(roots[g])
        mt = mts[g]
        for k, (mv, res, roots_after) in enumerate(steps):
            it = iter(log[k * nfl:(k + 1) * nfl])

            def replay(boards, turns, g=g, it=it):
                vals, cnt = next(it)
                assert cnt[g] == len(boards)
                return [float(x) for x in vals[g * B: g * B + len(boards)]]

            col, _, _ = oracle.get_move_valued(b, t, mt, S, 1.4, B, replay)
            assert int(mv[g]) == col, (g, k)
            b, t = oracle.play(b, t, col)
            exp = t * 2 - 1 if oracle.check_win(b, t) else (0 if oracle.check_draw(b) else ONGOING)
            assert int(res[g]) == exp, (g, k)
            if exp != ONGOING:
                b, t = "." * 42, 0
                ended += 1
            assert _board(roots_after[g]) == (b, t), (g, k)
        assert same_mt(pool.eng, g, mt), g
    assert ended >= 8, ended   # Connect4 games end every ~20-40 moves: dozens of the 4096 do here
    pool.close()


def test_captured_step_graph_pins_the_trajectory_pool():
    """A step graph has the trajectory pool's buffers baked into its record kernel: once one
    is captured, a start(quota) that would need a larger pool is refused, and a
    quota that fits keeps the graph valid."""
    from zeroclone_amd.selfplay import C4SelfPlay
    sp = C4SelfPlay(64, 16, batch_size=8, seed=1, games_cap=256)
    g = sp.capture_step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError):
        sp.start(100_000)
    sp.start(128)   # fits the pool sized at construction
    for _ in range(60):
        g.replay()
    torch.cuda.synchronize()
    assert sp.traj.finished() > 0
    sp.close()
