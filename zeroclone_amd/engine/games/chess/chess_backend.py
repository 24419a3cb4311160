"""Chess backend with the reference's plugin API (engine/games/chess: bindings_chess.cpp,
chess_backend.cpp, include/state.h).

Same surface as the reference's pybind11 module: `State(board, turn,
fifty_move_rule_counter, w_ck, w_cq, b_ck, b_cq, hist_white, hist_black)` with a 64-entry
board of piece bytes (index 0 = a8), moves as ((fr, fc, tr, tc), capture_value) tuples, and
get_legal_moves / play_move / check_win / check_draw / create_init_state / state_to_tensor /
state_from_fen.  The rules run on the GPU (chess.hip, through the C-ABI): every call here
is a batch-of-one launch of the same kernels the batched search uses.  Only the move
histories — host objects that only check_draw's repetition test reads
(chess_backend.cpp:148-180, :432-436) — are handled here on the host.
"""
from __future__ import annotations

import threading
from collections import deque

import numpy as np

from .... import _native

ZC_GAME = "chess"   # marks this module as a GPU-native backend for zeroclone_amd

_lock = threading.Lock()
_eng = None


def _engine():
    global _eng
    with _lock:
        if _eng is None:
            _eng = _native.NativeEngine(max_games=1, max_sims=1, max_batch=1)
        return _eng


class State:
    __slots__ = ("board", "turn", "fifty_move_rule_counter", "w_ck", "w_cq", "b_ck", "b_cq", "hist_white",
                 "hist_black")

    def __init__(self, board, turn, fifty_move_rule_counter, w_ck, w_cq, b_ck, b_cq, hist_white=(), hist_black=()):
        self.board = [int(x) for x in board]
        if len(self.board) != 64:
            raise ValueError("board must have 64 squares")
        self.turn = int(turn)
        self.fifty_move_rule_counter = int(fifty_move_rule_counter) & 0xFF
        self.w_ck, self.w_cq, self.b_ck, self.b_cq = bool(w_ck), bool(w_cq), bool(b_ck), bool(b_cq)
        self.hist_white = list(hist_white)
        self.hist_black = list(hist_black)

    def __repr__(self):
        return f"State(turn={self.turn}, board={bytes(self.board).decode('latin-1')!r})"


def to_zc(state) -> np.ndarray:
    """State -> zc_chess_state (include/zeroclone.h)."""
    a = np.zeros((), _native.CHESS_STATE_DTYPE)
    a["board"] = np.asarray(state.board, np.uint8)
    a["turn"] = state.turn
    a["fifty"] = state.fifty_move_rule_counter & 0xFF
    a["castle"] = int(state.w_ck) | int(state.w_cq) << 1 | int(state.b_ck) << 2 | int(state.b_cq) << 3
    return a


def from_zc(a, hist_white=(), hist_black=()) -> State:
    c = int(a["castle"])
    return State(list(a["board"]), int(a["turn"]), int(a["fifty"]), c & 1, c & 2, c & 4, c & 8,
                 hist_white, hist_black)


def _run(fn, states, out_shape, out_dtype, *extra):
    import torch
    e = _engine()
    arr = np.stack([to_zc(s) for s in states]) if not isinstance(states, np.ndarray) else states
    d = torch.from_numpy(arr.view(np.uint8).reshape(len(arr), 72).copy()).cuda(e.device)
    out = torch.zeros(out_shape, dtype=out_dtype, device=d.device)
    fn(e, len(arr), d, out, *extra)
    torch.cuda.synchronize(d.device)
    return out.cpu().numpy()


def get_legal_moves(state):
    """Legal moves in the reference's order: [((fr, fc, tr, tc), capture_value), ...]."""
    import torch

    def fn(e, n, d, out):
        counts = torch.zeros(n, dtype=torch.int32, device=d.device)
        e.chess_legal_moves_async(n, d.data_ptr(), out.data_ptr(), counts.data_ptr())
        out[:, -1] = counts.to(torch.int16)   # count rides in the last slot (never a move: < 256 used)

    res = _run(fn, [state], (1, _native.CHESS_MAX_MOVES + 1), torch.int16)[0].view(np.uint16)
    n = int(res[-1])
    if n > _native.CHESS_MAX_MOVES:
        raise RuntimeError("position has more legal moves than the device move list holds")
    return [_native.unpack_chess_move(m) for m in res[:n]]


def play_move(state, move):
    import torch
    (fr, fc, tr, tc), v = move
    m = _native.pack_chess_move(fr, fc, tr, tc, v)

    def fn(e, n, d, out):
        mv = torch.tensor([m], dtype=torch.int32, device=d.device).to(torch.int16)
        e.chess_play_async(n, d.data_ptr(), mv.data_ptr(), out.data_ptr())

    res = _run(fn, [state], (1, 72), torch.uint8)[0].view(_native.CHESS_STATE_DTYPE)[0]
    mv = ((int(fr), int(fc), int(tr), int(tc)), float(v))
    hw, hb = list(state.hist_white), list(state.hist_black)
    if state.turn == 0:
        hw.insert(0, mv)
    else:
        hb.insert(0, mv)
    return from_zc(res, hw, hb)


def _flags(state) -> int:
    import torch

    def fn(e, n, d, out):
        e.chess_terminal_async(n, d.data_ptr(), out.data_ptr())

    return int(_run(fn, [state], (1,), torch.int32)[0])


def check_win(state) -> bool:
    return bool(_flags(state) & _native.ZC_CHESS_WIN)


def has_repeated_prefix(moves, min_pattern_len: int = 2, min_repeats: int = 3) -> bool:
    """chess_backend.cpp:148-180: some prefix of the history (most recent move first) is a
    whole number >= min_repeats of copies of a block of >= min_pattern_len moves (KMP)."""
    n = len(moves)
    if n < min_pattern_len * min_repeats:
        return False
    pi = [0] * n
    j = 0
    for i in range(1, n):
        while j > 0 and moves[i] != moves[j]:
            j = pi[j - 1]
        if moves[i] == moves[j]:
            j += 1
        pi[i] = j
    for i in range(n):
        length = i + 1
        p = length - pi[i]
        if p >= min_pattern_len and length % p == 0 and length // p >= min_repeats:
            return True
    return False


def check_draw(state) -> bool:
    f = _flags(state)
    if f & (_native.ZC_CHESS_STALEMATE | _native.ZC_CHESS_FIFTY):
        return True
    return has_repeated_prefix(state.hist_white) and has_repeated_prefix(state.hist_black)


def create_init_state():
    return from_zc(_native.chess_init())


def state_from_fen(fen: str):
    return from_zc(_native.chess_from_fen(fen))


def state_to_tensor(state):
    import torch

    def fn(e, n, d, out):
        e.chess_planes_async(n, d.data_ptr(), out.data_ptr(), False)

    return _run(fn, [state], (1, 17, 8, 8), torch.float32)[0]


def pack_histories(states, cap: int | None = None):
    """Both sides' move histories of `states` as the device takes them: uint16 [n, 2, cap]
    packed moves in play order (the State's lists are most recent first, as the reference's
    deques) and their lengths int32 [n, 2]."""
    cap = cap or max([1] + [max(len(s.hist_white), len(s.hist_black)) for s in states])
    h = np.zeros((len(states), 2, cap), np.uint16)
    n = np.zeros((len(states), 2), np.int32)
    for i, s in enumerate(states):
        for side, lst in enumerate((s.hist_white, s.hist_black)):
            if len(lst) > cap:
                raise ValueError(f"a history of {len(lst)} moves exceeds {cap}")
            for k, ((fr, fc, tr, tc), v) in enumerate(reversed(list(lst))):
                h[i, side, k] = _native.pack_chess_move(fr, fc, tr, tc, v)
            n[i, side] = len(lst)
    return h, n


def moves_from_hist(h: str):
    """Decode a history string of the golden fixtures (5 digits per move, most recent first)."""
    return [((int(h[i]), int(h[i + 1]), int(h[i + 2]), int(h[i + 3])), float(h[i + 4])) for i in range(0, len(h), 5)]
