"""Expansion-order policies with the reference's interface (engine/policy_functions.py:1-16).

`Policy('random')` is what the GPU search implements (random.choice over the untried moves,
drawn from the game's CPython MT19937 stream); calling a Policy object directly runs the
same rule on the host, as the reference does.
"""
import random as _random


class Policy:
    def __init__(self, name=None, **kwargs):
        self.name = name if name is not None else "random"
        self.args = kwargs

    def __call__(self, moves, **kwargs):
        method_ref = getattr(self, self.name)
        return method_ref(moves, self.args | kwargs)

    def random(self, moves, args):
        return _random.choice(moves)

    def immediate_value(self, moves, args):
        best = max(m[1] for m in moves)
        return _random.choice([m for m in moves if m[1] >= best - args.get("policy_freedom", 0)])
