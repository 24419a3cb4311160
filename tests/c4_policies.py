"""Custom policy callables for the host-policy fallback tests: arbitrary Python
callables, as the reference's mcts.get_move accepts (mcts.cpp:65-70 calls policy(untried)
and takes list.index of the result).  Shared by tests/golden/gen_golden_hostpolicy.py (run
against the reference's compiled get_move) and tests/test_gpu_hostpolicy.py.  Connect4
moves are (column, 0); chess moves ((fr, fc, tr, tc), capture value)."""
import random


def last_move(moves):
    """Deterministic: the last untried move in list order (no random numbers)."""
    return moves[-1]


def shuffled_first(moves):
    """random.shuffle of a copy, then its first move: draws from the global stream in a
    pattern unlike random.choice."""
    ms = list(moves)
    random.shuffle(ms)
    return ms[0]


class CentreBias:
    """A stateful object policy: prefers central columns, noise from random.random()."""

    def __init__(self, weight=0.35):
        self.weight = weight
        self.calls = 0

    def __call__(self, moves):
        self.calls += 1
        return max(moves, key=lambda m: random.random() - self.weight * abs(m[0] - 3))


POLICIES = {"last_move": last_move, "shuffled_first": shuffled_first, "centre_bias": CentreBias}


def best_capture(moves):
    """Deterministic: the first move with the largest capture value."""
    return max(moves, key=lambda m: m[1])


class ValueNoise:
    """Capture value plus noise from random.random()."""

    def __call__(self, moves):
        return max(moves, key=lambda m: random.random() + 0.5 * m[1])


CHESS_POLICIES = {"last_move": last_move, "shuffled_first": shuffled_first, "best_capture": best_capture,
                  "value_noise": ValueNoise}


def make(name):
    p = POLICIES.get(name) or CHESS_POLICIES[name]
    return p() if isinstance(p, type) else p


def chess_code(m):
    (fr, fc, tr, tc), _ = m
    return int(fr) * 512 + int(fc) * 64 + int(tr) * 8 + int(tc)


class ChessRecording:
    """Wraps a chess policy; records each call as 'n:pick:checksum of the untried list'."""

    def __init__(self, inner):
        self.inner = inner
        self.calls = []

    def __call__(self, moves):
        a = self.inner(moves)
        ck = sum((i + 1) * chess_code(m) for i, m in enumerate(moves)) % 1000003
        self.calls.append(f"{len(moves)}:{moves.index(a)}:{ck}")
        return a


class Recording:
    """Wraps a policy and records each call's untried columns (as a digit string) and pick."""

    def __init__(self, inner):
        self.inner = inner
        self.calls = []

    def __call__(self, moves):
        a = self.inner(moves)
        self.calls.append("".join(str(m[0]) for m in moves) + ":" + str(a[0]))
        return a
