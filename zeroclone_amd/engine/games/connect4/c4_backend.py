"""Connect4 backend with the reference's plugin API (engine/games/connect4/c4_backend.py).

Same State type and semantics as the reference module — a namedtuple (board, turn) with a
6x7 list board, row 0 at the TOP, 'X' for turn 0 and 'O' for turn 1 — so states, moves and
results are interchangeable with the reference.  These functions are the host-side game
API; the search itself never calls them: mcts.get_move / Engine hand the position to the
GPU as a bitboard (to_zc) and the HIP kernels play the rules there.
"""
from collections import namedtuple

import numpy as np

ZC_GAME = "connect4"   # marks this module as a GPU-native backend for zeroclone_amd

State = namedtuple("State", ["board", "turn"])

ROWS = 6
COLS = 7

tokens = ["X", "O"]


def create_init_state():
    return State([[" " for _ in range(COLS)] for _ in range(ROWS)], 0)


def play_move(state, move):
    """Drop tokens[turn] into column move[0]; a full column is left unchanged (reference
    c4_backend.py:14-23: the turn still flips)."""
    board = [row.copy() for row in state.board]
    col = move[0]
    for r in range(ROWS - 1, -1, -1):
        if board[r][col] == " ":
            board[r][col] = tokens[state.turn]
            break
    return state._replace(board=board, turn=1 - state.turn)


def _four(board, tok):
    """Four cells == tok in a row, column or diagonal (the reference's four scans), as one
    bitboard test: cell (r, c) -> bit 7 c + 5 - r, a zero sentinel bit on top of each column."""
    b = 0
    for r in range(ROWS):
        row = board[r]
        sh = 5 - r
        for c in range(COLS):
            if row[c] == tok:
                b |= 1 << (7 * c + sh)
    for d in (1, 7, 6, 8):  # vertical, horizontal, the two diagonals
        m = b & (b >> d)
        if m & (m >> (2 * d)):
            return True
    return False


def check_win(state):
    """Four in a row for the player who moved LAST (tokens[1 - turn]), as the reference."""
    return _four(state.board, tokens[1 - state.turn])


def check_draw(state):
    return all(cell != " " for row in state.board for cell in row)


def get_legal_moves(state):
    """A set of (column, 0) tuples — a set, like the reference, so iteration order is
    CPython's (the GPU search reproduces exactly that order)."""
    return {(i, 0) for i in range(COLS) if state.board[0][i] == " "}


def state_to_tensor(state):
    cur = tokens[state.turn]
    opp = tokens[1 - state.turn]
    arr = np.array(state.board)
    return np.stack([(arr == cur).astype(np.float32), (arr == opp).astype(np.float32)], axis=0)


# ---------------------------------------------------------------- bitboard conversion
def to_zc(state):
    """State -> (stones_X, stones_O, turn) in the zc_c4_state layout (include/zeroclone.h):
    bit 7*col + (5 - row) for the cell board[row][col]."""
    s0 = s1 = 0
    for r in range(ROWS):
        row = state.board[r]
        for c in range(COLS):
            ch = row[c]
            if ch == "X":
                s0 |= 1 << (7 * c + (5 - r))
            elif ch == "O":
                s1 |= 1 << (7 * c + (5 - r))
    return s0, s1, int(state.turn)


def from_zc(s0, s1, turn):
    board = [[" "] * COLS for _ in range(ROWS)]
    for r in range(ROWS):
        for c in range(COLS):
            bit = 1 << (7 * c + (5 - r))
            if s0 & bit:
                board[r][c] = "X"
            elif s1 & bit:
                board[r][c] = "O"
    return State(board, int(turn))


def is_state(state):
    b = getattr(state, "board", None)
    return (b is not None and hasattr(state, "turn") and len(b) == ROWS
            and all(len(row) == COLS for row in b))
