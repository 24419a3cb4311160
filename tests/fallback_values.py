"""Value objects for the §8(b) fallback tests: arbitrary `.batch(states, backend=)` objects
that the device cannot run and that DRAW FROM PYTHON'S GLOBAL `random` (and read what the
reference's states carry).  The reference calls them once per flush, after the flush's
expansion draws (mcts.cpp:112-127), so their numbers interleave with the search's own.
Shared by tests/golden/gen_golden_fallback.py (run against the reference's compiled get_move)
and tests/test_gpu_fallback.py (run against this package)."""
import random


class NoisyValue:
    """Connect4 or chess: a value in [-1, 1) from random.random() alone (one draw per leaf:
    53 bits = two 32-bit words)."""

    def batch(self, states, **kw):
        return [2.0 * random.random() - 1.0 for _ in states]


class ShuffleValue:
    """random.randrange / random.shuffle draws (getrandbits of several widths) mixed with a
    feature of the position: the number of stones / pieces."""

    def batch(self, states, **kw):
        out = []
        for s in states:
            pieces = _pieces(s)
            k = list(range(1 + pieces % 5))
            random.shuffle(k)
            out.append((random.randrange(1000) - 500) / 1000.0 + 0.01 * k[0])
        return out


class HistoryValue:
    """Chess: reads the leaf's move histories (what the reference's leaf State carries: the
    root's histories plus the path's moves, pushed at the front) and draws from `random`."""

    def batch(self, states, **kw):
        out = []
        for s in states:
            hw, hb = list(s.hist_white), list(s.hist_black)
            h = 17 * len(hw) + 5 * len(hb)
            for i, m in enumerate(hw[:4] + hb[:4]):
                (fr, fc, tr, tc), v = m
                h = (h * 31 + (i + 1) * (fr * 512 + fc * 64 + tr * 8 + tc) + int(v)) % 1000003
            out.append((h % 2001 - 1000) / 1000.0 + 0.001 * random.random())
        return out


def _pieces(s):
    b = s.board
    if isinstance(b, (list, tuple)) and b and isinstance(b[0], (list, tuple)):
        return sum(1 for row in b for ch in row if ch in ("X", "O"))
    return sum(1 for x in b if x not in (0, 32))


VALUES = {"noisy": NoisyValue, "shuffle": ShuffleValue, "history": HistoryValue}
