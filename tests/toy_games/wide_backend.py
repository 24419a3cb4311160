"""A game with 300 moves per position, ten plies deep: its child-move slots outgrow the
any-backend tree's first pool (tests the zc_gen_reserve growth path)."""
from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class State:
    ply: int
    last: int
    turn: int


def create_init_state() -> State:
    return State(0, -1, 0)


def get_legal_moves(state: State):
    return [] if state.ply >= 10 else list(range(300))


def play_move(state: State, move) -> State:
    return State(state.ply + 1, move, state.turn ^ 1)


def check_win(state: State) -> bool:
    return state.ply >= 10 and state.last % 3 == 0


def check_draw(state: State) -> bool:
    return state.ply >= 10 and state.last % 3 != 0


def state_to_tensor(state: State) -> np.ndarray:
    return np.full((1, 1, 1), state.ply, np.float32)


def encode(state: State) -> list:
    return [state.ply, state.last, state.turn]
