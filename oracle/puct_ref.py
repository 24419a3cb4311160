"""A plain-Python restatement of the PUCT searches of zeroclone_amd/csrc/chess_puct.hip and
c4_puct.hip, for the parity tests and bench.py's C5 CPU baseline (TEST INFRASTRUCTURE ONLY;
the rules come from the oracle).  The search has no
reference counterpart, so this file is its specification in executable
form: same arithmetic order in fp64, same tie-breaking, same flush / virtual-loss protocol.
"""
import math

import oracle


class ChessRules:
    """chess_puct.hip: the reference's chess rules (oracle restatement of chess_backend.cpp)."""
    moves = staticmethod(oracle.chess_moves)
    play = staticmethod(oracle.chess_play)
    win = staticmethod(oracle.chess_win)


class C4Rules:
    """c4_puct.hip: Connect4 (c4_backend.py) on state = (42-char board, side to move): moves
    are the legal columns in CPython set order, none once the last mover has four or the
    board is full; win = the last mover has four."""

    @staticmethod
    def moves(s):
        b, t = s
        if oracle.check_win(b, t) or oracle.check_draw(b):
            return []
        return oracle.set_order(sum(1 << col for col in range(7) if b[col] == "."))

    @staticmethod
    def play(s, col):
        return oracle.play(s[0], s[1], col)

    @staticmethod
    def win(s):
        return oracle.check_win(s[0], s[1])


class Node:
    def __init__(self, state, rules=ChessRules):
        self.s = state
        self.moves = rules.moves(state)
        n = len(self.moves)
        self.N = [0] * n
        self.W = [0.0] * n
        self.P = [0.0] * n
        self.child = [None] * n
        self.evaluated = False


def search(state, sims, bs, c, value_fn, prior_fn, rules=ChessRules, flush_fn=None):
    """value_fn(state) -> value for the side to move; prior_fn(node) -> priors (list,
    float) for the node's moves.  flush_fn(states), if given, is called once per flush with
    the states of its non-terminal leaves before any value_fn / prior_fn call of that flush
    (a batched network fills the cache they read).  Returns (root moves, root visits,
    chosen index)."""
    root = Node(state, rules)
    flushes = 1 + (sims - 1 + bs - 1) // bs
    for f in range(flushes):
        nb = 1 if f == 0 else max(0, min(bs, sims - 1 - (f - 1) * bs))
        leaves = []
        for _ in range(nb):
            if f == 0:
                leaves.append((root, []))
                continue
            node, path = root, []
            while len(node.moves) and node.evaluated:
                sq = math.sqrt(float(sum(node.N)))
                best, bv = -1, -math.inf
                for j in range(len(node.moves)):
                    q = node.W[j] / node.N[j] if node.N[j] > 0 else 0.0
                    v = q + c * node.P[j] * sq / float(1 + node.N[j])
                    if v > bv:
                        bv, best = v, j
                node.N[best] += 1
                node.W[best] -= 1.0
                path.append((node, best))
                if node.child[best] is None:
                    node.child[best] = Node(rules.play(node.s, node.moves[best]), rules)
                    node = node.child[best]
                    break
                node = node.child[best]
            leaves.append((node, path))
        if flush_fn is not None:
            flush_fn([node.s for node, _ in leaves if len(node.moves)])
        for node, path in leaves:
            if len(node.moves) == 0:
                v = -1.0 if rules.win(node.s) else 0.0
            else:
                v = value_fn(node.s)
                if not node.evaluated:
                    node.P = prior_fn(node)
                    node.evaluated = True
            d = len(path)
            for l, (par, a) in enumerate(path, start=1):
                r = v if (d - l) % 2 == 0 else -v
                par.W[a] = par.W[a] + 1.0 - r
    best, bn = -1, -1
    for j, n in enumerate(root.N):
        if n > bn:
            bn, best = n, j
    return root.moves, root.N, best
