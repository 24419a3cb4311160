"""Subtraction game: a pile of stones, a move takes 1, 2 or 3; whoever takes the last stone
wins.  get_legal_moves returns a TUPLE of strings (the reference converts any sequence to a
list, mcts.cpp:74-75), check_draw is never true."""
from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class State:
    pile: int
    turn: int


def create_init_state() -> State:
    return State(21, 0)


def get_legal_moves(state: State):
    return tuple(f"take{k}" for k in (3, 1, 2) if k <= state.pile)


def play_move(state: State, move) -> State:
    return State(state.pile - int(move[4:]), state.turn ^ 1)


def check_win(state: State) -> bool:
    return state.pile == 0


def check_draw(state: State) -> bool:
    return False


def state_to_tensor(state: State) -> np.ndarray:
    return np.full((1, 1, 1), state.pile, np.float32)


def encode(state: State) -> list:
    return [state.pile, state.turn]
