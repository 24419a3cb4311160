"""Dispatch of a batched search to the right device path, by game and plugin kind.

    game      value object                         device path
    connect4  Value('random_rollout')              zc_c4_search_games (fused rollouts)
    connect4  network Value / any .batch object    zc_c4_ext_* + NetValue / HostValue
    chess     Value('crude_chess_score')           zc_chess_search_async (value in-kernel)
    chess     network Value / any .batch object    zc_chess_ext_* + NetValue / HostValue

Policy('random') and Policy('immediate_value', policy_freedom=f) run on the device for
chess; Connect4 moves carry no capture value, so for Connect4 immediate_value picks among
all untried moves exactly like random (policy_functions.py:14-17 with all values 0) and both
map to the same device policy.

Any other policy callable (SURVEY §8(b)'s fallback) runs the search in host-policy mode: the
tree stays on the device and every expansion calls policy(untried_moves) on the host, where
mcts.cpp:65-78 calls it (zc_c4_hp_* / zc_chess_hp_*: `c4_host_policy_moves`,
`chess_host_policy_moves`).

Any other game backend (a module with the six functions of engine/README.md:17-24) runs
`generic_moves`: the tree on the device (zc_gen_*), the backend, policy and value -- Python
objects the device cannot run -- called on the host exactly where mcts.cpp calls them.
"""
from __future__ import annotations

import numpy as np

from .. import _native


def game_of(backend, state) -> str:
    g = getattr(backend, "ZC_GAME", None)
    if g:
        return g
    name = getattr(backend, "__name__", "") or type(backend).__name__
    if name.endswith("c4_backend"):
        return "connect4"
    if name.endswith("chess_backend"):
        return "chess"
    if hasattr(state, "fifty_move_rule_counter"):
        return "chess"
    from .games.connect4 import c4_backend as c4
    if c4.is_state(state):
        return "connect4"
    for fn in ("get_legal_moves", "play_move"):
        if not callable(getattr(backend, fn, None)):
            raise TypeError(f"backend {name!r} has no {fn}() (the plugin contract, engine/README.md:17-24)")
    return "generic"


HOST_POLICY = -1   # any other callable: called on the host at each expansion


def policy_of(policy):
    from .policy_functions import Policy
    name = getattr(policy, "name", None) or "random"
    ours = isinstance(policy, Policy) and type(policy).random is Policy.random and \
        type(policy).immediate_value is Policy.immediate_value
    # the reference's own Policy objects (engine/policy_functions.py) are accepted as well
    theirs = type(policy).__name__ == "Policy" and type(policy).__module__.endswith("policy_functions") and \
        not isinstance(policy, Policy)
    builtin = ours or theirs
    if builtin and name == "random":
        return _native.ZC_POLICY_RANDOM, 0.0
    if builtin and name == "immediate_value":
        return _native.ZC_POLICY_IMMEDIATE_VALUE, float(getattr(policy, "args", {}).get("policy_freedom", 0))
    if isinstance(policy, Policy) and not callable(getattr(policy, name, None)):
        # the reference fails at the first expansion (policy_functions.py:7 getattr)
        raise AttributeError(f"'{type(policy).__name__}' object has no attribute {name!r}")
    if callable(policy):
        return HOST_POLICY, 0.0
    raise TypeError("a policy must be callable as policy(untried_moves) (policy_functions.py:6-8)")


def value_kind(value) -> str:
    name = getattr(value, "name", None)
    if name == "random_rollout" and not hasattr(value, "_req_q"):
        return "rollout"
    if name == "crude_chess_score":
        return "crude"
    if getattr(value, "zc_model", None) is not None:
        return "net"
    if callable(getattr(value, "batch", None)):
        return "host"
    raise NotImplementedError("value objects must provide .batch(states, backend=) (value_functions.py:20)")


def chess_roots(states) -> np.ndarray:
    from .games.chess import chess_backend as cb
    return np.stack([cb.to_zc(s) for s in states]).astype(_native.CHESS_STATE_DTYPE)


def chess_moves(eng, ids, states, sims, c, bs, value, policy, backend):
    """Search chess games `ids` (engine game indices) from `states`; returns list of moves
    ((fr, fc, tr, tc), capture_value), None for a game with no legal move."""
    import torch
    pol, freedom = policy_of(policy)
    if pol == HOST_POLICY:
        return chess_host_policy_moves(eng, ids, states, sims, c, bs, value, policy, backend)
    kind = value_kind(value)
    n = len(ids)
    dev = torch.device("cuda", eng.device)
    first = int(ids[0])
    if list(ids) != list(range(first, first + n)):
        raise ValueError("chess searches take a contiguous range of engine games")
    roots = torch.from_numpy(chess_roots(states).view(np.uint8).reshape(n, 72).copy()).to(dev)
    if kind == "crude":
        mv = torch.zeros(n, dtype=torch.int16, device=dev)
        na = torch.zeros((n, _native.CHESS_MAX_MOVES), dtype=torch.int32, device=dev)
        st = torch.zeros((n, _native.STATS_FIELDS), dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        eng.chess_search_async(first, n, roots.data_ptr(), sims, c, bs, pol, freedom,
                               mv.data_ptr(), na.data_ptr(), st.data_ptr(), s)
        torch.cuda.current_stream(dev).synchronize()
    else:
        from ..valued import ChessValuedSearch, NetValue
        vs = ChessValuedSearch(eng, n, bs, policy=pol, freedom=freedom, planes=(kind == "net"),
                               leaves=(kind == "host"))
        if kind == "net":
            fn = NetValue(value.zc_model)
        elif kind == "rollout":
            fn = _ChessRolloutValue(eng, states, bs, dev)
        else:
            fn = _ChessHostValue(value, backend, eng, vs, states)
        mv, na, st = vs.run(roots, sims, c, fn, first_game=first)
        if kind == "rollout":
            fn.check()
    st = st.cpu().numpy()
    bad = st[:, 5]
    if (bad == _native.ZC_STATUS_CAPACITY).any():
        raise RuntimeError("chess search exceeded the tree's child-slot pool or depth limit")
    mv = mv.cpu().numpy().view(np.uint16)
    return [None if m == 0xFFFF else _native.unpack_chess_move(m) for m in mv]


class _ChessRolloutValue:
    """Value('random_rollout') on chess inside the stepwise search (value_functions.py:35-45
    at mcts.cpp:116): every flush's pending leaves are rolled out on the device in pending
    order on their game's stream (zc_chess_ext_rollouts), right after the flush's expansion
    draws; a leaf's move histories are its root's plus the path's moves."""

    def __init__(self, eng, states, bs, dev):
        import torch
        from .games.chess import chess_backend as cb
        hist, hlen = cb.pack_histories(states)
        self.eng = eng
        self.h, self.hl = torch.from_numpy(hist).to(dev), torch.from_numpy(hlen).to(dev)
        self.values = torch.zeros(len(states) * bs, dtype=torch.float64, device=dev)
        self.status = torch.zeros(len(states), dtype=torch.int32, device=dev)

    def flush_values(self, first, n, f, stream):
        self.eng.chess_ext_rollouts(first, n, f, self.h.data_ptr(), self.hl.data_ptr(), self.h.shape[2],
                                    self.values.data_ptr(), self.status.data_ptr(), stream)
        return self.values

    def check(self):
        if int(self.status.max().item()):
            raise RuntimeError(f"chess rollout exceeded {_native.CHESS_ROLL_CAP} moves per side in its history")


def chess_leaf_states(eng, first, n, f, bs, rows, counts, roots):
    """The flush's pending leaves as chess_backend States with the move histories the
    reference's leaf State carries: the root's, plus the path's moves pushed at the front of
    the mover's history (play_move, chess_backend.cpp:374) — zc_chess_ext_leaf_moves.
    Returns one list of States per game."""
    import torch
    from .games.chess import chess_backend as cb
    dev = torch.device("cuda", eng.device)
    moves = torch.zeros((n * bs, 64), dtype=torch.int16, device=dev)
    depth = torch.zeros(n * bs, dtype=torch.int32, device=dev)
    eng.chess_ext_leaf_moves(first, n, f, moves.data_ptr(), depth.data_ptr(),
                             torch.cuda.current_stream(dev).cuda_stream)
    mv, dp = moves.cpu().numpy().view(np.uint16), depth.cpu().numpy()
    out = []
    for i, k in enumerate(counts):
        root = roots[i]
        t0 = int(root.turn)
        games = []
        for j in range(int(k)):
            o = i * bs + j
            hw, hb = list(root.hist_white), list(root.hist_black)
            for lv in range(int(dp[o])):
                m = _native.unpack_chess_move(int(mv[o, lv]))
                (hw if (t0 + lv) % 2 == 0 else hb).insert(0, m)
            games.append(cb.from_zc(rows[o].view(_native.CHESS_STATE_DTYPE)[0], hw, hb))
        out.append(games)
    return out


class _ChessHostValue:
    """Any other value object on chess: value.batch(leaf States, backend=) per game per
    flush on the host (mcts.cpp:116), the leaves carrying their move histories, Python's
    `random` being the game's device stream during the call (_device.game_stream)."""

    def __init__(self, value, backend, eng, vs, roots):
        self.value, self.backend, self.eng, self.vs, self.roots = value, backend, eng, vs, roots

    def flush_values(self, first, n, f, stream):
        import torch
        from ._device import game_stream
        vs = self.vs
        rows = vs.leaves.cpu().numpy()
        cnt = vs.counts.cpu().numpy()
        out = np.zeros(rows.shape[0], np.float64)
        for i, states in enumerate(chess_leaf_states(self.eng, first, n, f, vs.bs, rows, cnt, self.roots)):
            if states:
                with game_stream(self.eng, first + i):
                    v = self.value.batch(states, backend=self.backend)
                out[i * vs.bs: i * vs.bs + len(states)] = [float(x) for x in v]
        return torch.from_numpy(out).to(vs.dev)


def c4_moves(eng, ids, roots, sims, c, bs, value, backend):
    """Connect4: fused rollouts for Value('random_rollout'), stepwise otherwise."""
    kind = value_kind(value)
    if kind == "rollout":
        mv, _, st = eng.c4_search_games(ids, roots, sims, c, bs)
        return [(int(m), 0) for m in mv]
    import torch
    from ..valued import C4ValuedSearch, HostValue, NetValue
    n = len(ids)
    first = int(ids[0])
    if list(ids) != list(range(first, first + n)):
        raise ValueError("stepwise searches take a contiguous range of engine games")
    vs = C4ValuedSearch(eng, n, bs, planes=(kind == "net"))
    r = torch.from_numpy(roots.view(np.int64).reshape(n, 3).copy()).to(vs.dev)
    fn = NetValue(value.zc_model) if kind == "net" else HostValue(value, backend, eng, first)
    mv, _, st = vs.run(r, sims, c, fn, first_game=first)
    st = st.cpu().numpy()
    if st[:, 5].any():
        raise ValueError(f"invalid root for the search (status {int(st[:, 5].max())})")
    return [(int(m), 0) for m in mv.cpu().numpy()]


def c4_host_policy_moves(eng, ids, roots, sims, c, bs, value, policy, backend):
    """The §8(b) fallback: mcts.get_move with an arbitrary policy callable.  Per game, per
    simulation: zc_c4_hp_walk selects (mcts.cpp:47-63) on the device tree, the policy picks
    among the untried moves on the host exactly as mcts.cpp:67-70 calls it (the untried moves
    as a list in the node's order; the action's list.index), zc_c4_hp_expand expands; each
    flush's leaves go to value.batch (mcts.cpp:116) and zc_c4_ext_backup.  Python's `random`
    is used only by the policy and the value themselves, in the reference's order."""
    import torch
    from .games.connect4 import c4_backend as zb
    dev = torch.device("cuda", eng.device)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream
    node = torch.zeros(_native.C4_HP_NODE_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    leaf = torch.zeros(3, dtype=torch.int64, device=dev)
    vals = torch.zeros(bs, dtype=torch.float64, device=dev)
    mv = torch.zeros(1, dtype=torch.int32, device=dev)
    na = torch.zeros((1, 7), dtype=torch.int32, device=dev)
    st = torch.zeros((1, _native.STATS_FIELDS), dtype=torch.int64, device=dev)
    out = []
    for gi, root in zip(ids, roots):
        r = torch.from_numpy(np.asarray([root], _native.C4_STATE_DTYPE).view(np.int64).reshape(1, 3).copy()).to(dev)
        eng.c4_ext_begin(int(gi), 1, r.data_ptr(), sims, c, bs, s)
        for f in range((sims + bs - 1) // bs):
            nb = min(bs, sims - f * bs)
            states = []
            for j in range(nb):
                eng.c4_hp_walk(int(gi), f, j, node.data_ptr(), s)
                nd = node.cpu().numpy().view(_native.C4_HP_NODE_DTYPE)[0]
                if int(nd["node"]) < 0:
                    raise ValueError("invalid root for the search (bad state or no legal move)")
                k = -1
                n_un = int(nd["n_untried"])
                if n_un:
                    moves = [(int(col), 0) for col in nd["untried"][:n_un]]
                    k = moves.index(policy(moves))
                eng.c4_hp_expand(int(gi), f, j, k, leaf.data_ptr(), s)
                row = leaf.cpu().numpy().view(np.uint64)
                states.append(zb.from_zc(int(row[0]), int(row[1]), int(row[2]) & 1))
            v = [float(x) for x in value.batch(states, backend=backend)]
            vals[:nb].copy_(torch.tensor(v, dtype=torch.float64))
            eng.c4_ext_backup(int(gi), 1, f, vals.data_ptr(), s)
        eng.c4_ext_end(int(gi), 1, mv.data_ptr(), na.data_ptr(), st.data_ptr(), s)
        stream.synchronize()
        if int(st[0, 5].item()):
            raise RuntimeError(f"host-policy search failed (status {int(st[0, 5].item())})")
        out.append((int(mv[0].item()), 0))
    return out


def chess_host_policy_moves(eng, ids, states, sims, c, bs, value, policy, backend):
    """The §8(b) fallback for chess: as c4_host_policy_moves, on the chess tree
    (zc_chess_hp_walk / zc_chess_hp_expand inside a zc_chess_ext_* search).  The policy gets
    the untried moves as the reference's move objects ((fr, fc, tr, tc), capture value), in
    the node's untried order; a game with no legal move gives None."""
    import torch
    from .games.chess import chess_backend as cb
    dev = torch.device("cuda", eng.device)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream
    node = torch.zeros(_native.CHESS_HP_NODE_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    leaf = torch.zeros(72, dtype=torch.uint8, device=dev)
    vals = torch.zeros(bs, dtype=torch.float64, device=dev)
    mv = torch.zeros(1, dtype=torch.int16, device=dev)
    na = torch.zeros((1, _native.CHESS_MAX_MOVES), dtype=torch.int32, device=dev)
    st = torch.zeros((1, _native.STATS_FIELDS), dtype=torch.int64, device=dev)
    out = []
    for gi, state in zip(ids, states):
        root = torch.from_numpy(chess_roots([state]).view(np.uint8).reshape(1, 72).copy()).to(dev)
        eng.chess_ext_begin(int(gi), 1, root.data_ptr(), sims, c, bs, _native.ZC_POLICY_RANDOM, 0.0, s)
        live = True
        for f in range((sims + bs - 1) // bs):
            nb = min(bs, sims - f * bs)
            leaves = []
            for j in range(nb):
                eng.chess_hp_walk(int(gi), f, j, node.data_ptr(), s)
                nd = node.cpu().numpy().view(_native.CHESS_HP_NODE_DTYPE)[0]
                if int(nd["node"]) < 0:
                    live = False
                    break
                k = -1
                n_un = int(nd["n_untried"])
                if n_un:
                    moves = [_native.unpack_chess_move(m) for m in nd["untried"][:n_un]]
                    k = moves.index(policy(moves))
                eng.chess_hp_expand(int(gi), f, j, k, leaf.data_ptr(), s)
                leaves.append(leaf.cpu().numpy().copy())
            if not live:
                break
            leaves = chess_leaf_states(eng, int(gi), 1, f, bs, np.stack(leaves), [nb], [state])[0]
            v = [float(x) for x in value.batch(leaves, backend=backend)]
            vals[:nb].copy_(torch.tensor(v, dtype=torch.float64))
            eng.chess_ext_backup(int(gi), 1, f, vals.data_ptr(), s)
        eng.chess_ext_end(int(gi), 1, mv.data_ptr(), na.data_ptr(), st.data_ptr(), s)
        stream.synchronize()
        status = int(st[0, 5].item())
        if status == _native.ZC_STATUS_NO_MOVES:
            out.append(None)
            continue
        if status:
            raise RuntimeError(f"host-policy chess search failed (status {status})")
        m = int(mv[0].item()) & 0xFFFF
        out.append(None if m == 0xFFFF else _native.unpack_chess_move(m))
    return out


def generic_moves(eng, state, sims, c, bs, value, policy, backend):
    """mcts.get_move (mcts.cpp:102-160) for ANY backend: the tree lives on the
    device (zc_gen_*: UCT selection, the expansion bookkeeping, the fp64 pending-order
    backup); the states and moves are the backend's Python objects, kept here by node id.
    Per simulation, in the reference's order: the device walk (select, :47-63); if the node
    has untried moves, policy(untried moves in list order), list.index of its pick, the
    backend's play_move and get_legal_moves (expand, :65-78), then the device expansion;
    every batch_size leaves value.batch(states, backend=backend) (:112-127) and the device
    backup.  Returns root_moves[first child with the most visits] (:150-157)."""
    import torch
    dev = torch.device("cuda", eng.device)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream
    root_moves = list(backend.get_legal_moves(state))
    states, moves = [state], [root_moves]
    eng.gen_begin(sims, c, bs, len(root_moves), s)
    n_cap, s_cap = eng.gen_capacity()
    slots = len(root_moves)
    out = torch.zeros(5 + max(64, slots), dtype=torch.int32, device=dev)
    vals = torch.zeros(bs, dtype=torch.float64, device=dev)
    pending = []

    def flush():
        if not pending:
            return
        v = value.batch(list(pending), backend=backend)
        v = [float(v[i]) for i in range(len(pending))]
        vals[:len(v)].copy_(torch.tensor(v, dtype=torch.float64))
        eng.gen_backup(len(v), vals.data_ptr(), s)
        pending.clear()

    for _ in range(sims):
        eng.gen_walk(out.data_ptr(), out.numel(), s)
        o = out.cpu().numpy()
        if o[4]:
            raise RuntimeError(f"any-backend search failed on the device (status {int(o[4])})")
        node, nu = int(o[0]), int(o[1])
        if nu and 5 + nu > out.numel():   # a longer untried list than the buffer: walk again (no side effects)
            out = torch.zeros(5 + nu, dtype=torch.int32, device=dev)
            eng.gen_walk(out.data_ptr(), out.numel(), s)
            o = out.cpu().numpy()
        if nu:
            untried = [moves[node][int(k)] for k in o[5:5 + nu]]
            action = policy(untried)
            local = untried.index(action)
            new_state = backend.play_move(states[node], action)
            new_moves = list(backend.get_legal_moves(new_state))
            if slots + len(new_moves) > s_cap:
                eng.gen_reserve(n_cap, max(2 * s_cap, slots + len(new_moves), 1024))
                n_cap, s_cap = eng.gen_capacity()
            eng.gen_expand(local, len(new_moves), s)
            slots += len(new_moves)
            states.append(new_state)
            moves.append(new_moves)
            pending.append(new_state)
        else:
            eng.gen_expand(-1, 0, s)
            pending.append(states[node])
        if len(pending) >= bs:
            flush()
    flush()
    res = torch.zeros(5, dtype=torch.int32, device=dev)
    eng.gen_end(res.data_ptr(), 0, 0, s)
    r = res.cpu().numpy()
    if r[1]:
        raise RuntimeError(f"any-backend search failed on the device (status {int(r[1])})")
    if int(r[4]) != len(states):
        raise RuntimeError("any-backend search: device and host trees disagree")
    if r[0] < 0:
        raise ValueError("root has no legal move (the reference indexes moves[-1] here)")
    return root_moves[int(r[0])]
