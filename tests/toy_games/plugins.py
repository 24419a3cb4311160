"""Policies and values for the any-backend tests: arbitrary Python callables / .batch
objects, as mcts.get_move accepts them (mcts.cpp:65-70, :116)."""
import random


def last_move(moves):
    return moves[-1]


def shuffled_first(moves):
    ms = list(moves)
    random.shuffle(ms)
    return ms[0]


POLICIES = {"last_move": last_move, "shuffled_first": shuffled_first}


class HashValue:
    """A deterministic fp64 value of the encoded state (no random numbers)."""

    def __init__(self, encode):
        self.encode = encode

    def batch(self, states, backend=None):
        out = []
        for s in states:
            h = 0
            for x in self.encode(s):
                h = (h * 1000003 + int(x) + 7) % 2147483647
            out.append(((h % 20001) - 10000) / 10007.0)
        return out


class Recording:
    """Records every call: the untried moves it was given and its pick."""

    def __init__(self, inner):
        self.inner = inner
        self.calls = []

    def __call__(self, moves):
        pick = self.inner(moves)
        self.calls.append([list(moves), pick])
        return pick


class RecordingValue:
    """Records the leaves of every flush (encoded), then delegates."""

    def __init__(self, inner, encode):
        self.inner, self.encode = inner, encode
        self.flushes = []

    def batch(self, states, **kw):
        self.flushes.append([self.encode(s) for s in states])
        return self.inner.batch(states, **kw)
