"""Tic-tac-toe.  Like the reference's Connect4 backend, the legal moves are the empty cells
whether or not the game is over, check_win looks at the last mover, check_draw at a full
board.  Moves are cell indices 0..8."""
from dataclasses import dataclass

import numpy as np

LINES = [(0, 1, 2), (3, 4, 5), (6, 7, 8), (0, 3, 6), (1, 4, 7), (2, 5, 8), (0, 4, 8), (2, 4, 6)]


@dataclass(frozen=True)
class State:
    board: tuple   # 9 cells: 0 empty, 1 'X' (player 0), 2 'O' (player 1)
    turn: int      # side to move


def create_init_state() -> State:
    return State((0,) * 9, 0)


def get_legal_moves(state: State):
    return [i for i in range(9) if state.board[i] == 0]


def play_move(state: State, move) -> State:
    b = list(state.board)
    b[move] = state.turn + 1
    return State(tuple(b), state.turn ^ 1)


def check_win(state: State) -> bool:
    mark = (state.turn ^ 1) + 1
    return any(all(state.board[i] == mark for i in line) for line in LINES)


def check_draw(state: State) -> bool:
    return all(c != 0 for c in state.board)


def state_to_tensor(state: State) -> np.ndarray:
    b = np.asarray(state.board).reshape(3, 3)
    me, opp = state.turn + 1, (state.turn ^ 1) + 1
    return np.stack([(b == me), (b == opp)]).astype(np.float32)


def encode(state: State) -> list:
    return list(state.board) + [state.turn]
