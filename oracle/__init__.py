"""oracle — TEST INFRASTRUCTURE ONLY.

ctypes view of ``oracle/lib/libzc_oracle.so`` (the C restatement in ``c4_oracle.c``).
Allowed importers: ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg — always as the checker or the baseline, never as the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libzc_oracle.so")


def build(quiet: bool = True) -> str:
    subprocess.run(["make", "-C", HERE, "lib"], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)
    return LIB_PATH


class _MT(ctypes.Structure):
    _fields_ = [("mt", ctypes.c_uint32 * 624), ("index", ctypes.c_int), ("drawn", ctypes.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        L.zco_mt_seed.argtypes = [P(_MT), ctypes.c_uint64]
        L.zco_mt_u32.argtypes = [P(_MT)]
        L.zco_mt_u32.restype = ctypes.c_uint32
        L.zco_randbelow.argtypes = [P(_MT), ctypes.c_uint32]
        L.zco_randbelow.restype = ctypes.c_uint32
        L.zco_set_order.argtypes = [ctypes.c_int, P(ctypes.c_int)]
        L.zco_check_win.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.zco_check_draw.argtypes = [ctypes.c_char_p]
        L.zco_rollout.argtypes = [ctypes.c_char_p, ctypes.c_int, P(_MT)]
        L.zco_get_move.argtypes = [ctypes.c_char_p, ctypes.c_int, P(_MT), ctypes.c_int, ctypes.c_double,
                                   ctypes.c_int, P(ctypes.c_int), P(ctypes.c_int), P(ctypes.c_int)]
        L.zco_get_move_batch.argtypes = [ctypes.c_int, ctypes.c_char_p, P(ctypes.c_int), P(ctypes.c_uint64),
                                         ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                         P(ctypes.c_int), P(ctypes.c_int), P(ctypes.c_uint64)]
        L.zco_selfplay_batch.argtypes = [ctypes.c_int, ctypes.c_char_p, P(ctypes.c_int), P(_MT), ctypes.c_int,
                                         ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                         P(ctypes.c_uint64)]
        L.zco_get_move_valued.argtypes = [ctypes.c_char_p, ctypes.c_int, P(_MT), ctypes.c_int, ctypes.c_double,
                                          ctypes.c_int, P(ctypes.c_int), P(ctypes.c_int), P(ctypes.c_int),
                                          VALUE_FN, ctypes.c_void_p]
        _lib = L
    return _lib


# void vfn(void *ctx, int n, const char *boards, const int *turns, double *out)
VALUE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char),
                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double))


class MT:
    """CPython-compatible MT19937 stream (oracle restatement)."""

    def __init__(self, seed: int):
        self.s = _MT()
        lib().zco_mt_seed(ctypes.byref(self.s), seed)

    def u32(self) -> int:
        return lib().zco_mt_u32(ctypes.byref(self.s))

    def randbelow(self, n: int) -> int:
        return lib().zco_randbelow(ctypes.byref(self.s), n)

    @property
    def drawn(self) -> int:
        return self.s.drawn

    def state(self):
        return list(self.s.mt), self.s.index


def set_order(mask: int) -> list[int]:
    out = (ctypes.c_int * 7)()
    n = lib().zco_set_order(mask, out)
    return list(out[:n])


def check_win(board: str, turn: int) -> bool:
    return bool(lib().zco_check_win(board.encode(), turn))


def check_draw(board: str) -> bool:
    return bool(lib().zco_check_draw(board.encode()))


def rollout(board: str, turn: int, seed: int):
    mt = MT(seed)
    v = lib().zco_rollout(board.encode(), turn, ctypes.byref(mt.s))
    return v, mt.drawn


def get_move(board: str, turn: int, seed: int, sims: int, c: float = 1.4, bs: int = 32):
    """Returns (column, root_na in move-list order, move-list order, words consumed)."""
    mt = MT(seed)
    na = (ctypes.c_int * 7)()
    order = (ctypes.c_int * 7)()
    n = ctypes.c_int(0)
    col = lib().zco_get_move(board.encode(), turn, ctypes.byref(mt.s), sims, c, bs, na, order, ctypes.byref(n))
    return col, list(na[:n.value]), list(order[:n.value]), mt.drawn


def get_move_mt(board: str, turn: int, mt: MT, sims: int, c: float = 1.4, bs: int = 32):
    """get_move continuing an existing stream (self-play: one random.seed per game)."""
    na = (ctypes.c_int * 7)()
    order = (ctypes.c_int * 7)()
    n = ctypes.c_int(0)
    col = lib().zco_get_move(board.encode(), turn, ctypes.byref(mt.s), sims, c, bs, na, order, ctypes.byref(n))
    return col, list(na[:n.value]), list(order[:n.value])


def get_move_valued(board: str, turn: int, mt: "MT", sims: int, c: float, bs: int, value_batch):
    """get_move with Value.batch = value_batch(boards: list[str], turns: list[int]) -> values
    (one call per flush, pending order).  Returns (column, root_na, order)."""
    def cb(_ctx, n, boards, turns, out):
        raw = ctypes.string_at(boards, 42 * n).decode()
        vals = value_batch([raw[42 * j: 42 * j + 42] for j in range(n)], [turns[j] for j in range(n)])
        for j in range(n):
            out[j] = float(vals[j])
    fn = VALUE_FN(cb)
    na = (ctypes.c_int * 7)()
    order = (ctypes.c_int * 7)()
    k = ctypes.c_int(0)
    col = lib().zco_get_move_valued(board.encode(), turn, ctypes.byref(mt.s), sims, c, bs, na, order,
                                    ctypes.byref(k), fn, None)
    return col, list(na[:k.value]), list(order[:k.value])


def play(board: str, turn: int, col: int):
    """c4_backend.play_move on the 42-char encoding (row 0 = top)."""
    b = list(board)
    for r in range(5, -1, -1):
        if b[r * 7 + col] == ".":
            b[r * 7 + col] = "XO"[turn]
            break
    return "".join(b), 1 - turn


def get_move_batch(boards: list[str], turns, seeds, sims: int, c: float = 1.4, bs: int = 32, threads: int = 1):
    """Baseline entry: returns (moves[n], root_na_by_column[n,7], consumed[n])."""
    n = len(boards)
    b = "".join(boards).encode()
    t = np.ascontiguousarray(turns, dtype=np.int32)
    s = np.ascontiguousarray(seeds, dtype=np.uint64)
    mv = np.zeros(n, np.int32)
    na = np.zeros((n, 7), np.int32)
    cons = np.zeros(n, np.uint64)
    P = ctypes.POINTER
    lib().zco_get_move_batch(n, b, t.ctypes.data_as(P(ctypes.c_int)), s.ctypes.data_as(P(ctypes.c_uint64)),
                             sims, c, bs, threads, mv.ctypes.data_as(P(ctypes.c_int)),
                             na.ctypes.data_as(P(ctypes.c_int)), cons.ctypes.data_as(P(ctypes.c_uint64)))
    return mv, na, cons


def selfplay_batch(boards: list[str], turns, mts: list["MT"], moves: int, sims: int, c: float = 1.4, bs: int = 32,
                   threads: int = 1):
    """zco_selfplay_batch: each game plays `moves` moves (search, play, evaluate, refill) from
    its board and MT state (the MT objects are advanced); returns expansions per game."""
    import numpy as np
    n = len(boards)
    b = "".join(boards).encode()
    t = np.asarray(turns, np.int32)
    arr = (_MT * max(n, 1))()
    for i, m in enumerate(mts):
        arr[i] = m.s
    exp = np.zeros(n, np.uint64)
    P = ctypes.POINTER
    lib().zco_selfplay_batch(n, b, t.ctypes.data_as(P(ctypes.c_int)), arr, moves, sims, c, bs, threads,
                             exp.ctypes.data_as(P(ctypes.c_uint64)))
    for i, m in enumerate(mts):
        m.s = arr[i]
    return exp


# ---------------------------------------------------------------- chess (chess_oracle.c)
class ZccMove(ctypes.Structure):
    _fields_ = [("fr", ctypes.c_uint8), ("fc", ctypes.c_uint8), ("tr", ctypes.c_uint8), ("tc", ctypes.c_uint8),
                ("value", ctypes.c_double)]


ZCC_HIST = 512
ZCC_MAX_MOVES = 256


class ZccState(ctypes.Structure):
    _fields_ = [("board", ctypes.c_uint8 * 64), ("turn", ctypes.c_uint8), ("fifty", ctypes.c_uint8),
                ("castle", ctypes.c_uint8), ("overflow", ctypes.c_uint8), ("nhw", ctypes.c_int), ("nhb", ctypes.c_int),
                ("hw", ZccMove * ZCC_HIST), ("hb", ZccMove * ZCC_HIST)]


def _chess_lib():
    L = lib()
    if not getattr(L, "_chess_ready", False):
        P = ctypes.POINTER
        L.zcc_init.argtypes = [P(ZccState)]
        L.zcc_from_fen.argtypes = [ctypes.c_char_p, P(ZccState)]
        L.zcc_legal_moves.argtypes = [P(ZccState), P(ZccMove)]
        L.zcc_play.argtypes = [P(ZccState), P(ZccMove), P(ZccState)]
        L.zcc_check_win.argtypes = [P(ZccState)]
        L.zcc_check_draw.argtypes = [P(ZccState)]
        L.zcc_state_to_tensor.argtypes = [P(ZccState), P(ctypes.c_float)]
        L.zcc_perft.argtypes = [P(ZccState), ctypes.c_int]
        L.zcc_perft.restype = ctypes.c_uint64
        L._chess_ready = True
    return L


def _hist_moves(h: str):
    return [(int(h[i]), int(h[i + 1]), int(h[i + 2]), int(h[i + 3]), float(h[i + 4])) for i in range(0, len(h), 5)]


def chess_state(board: str, turn: int = 0, fifty: int = 0, castle: int = 0, hw: str = "", hb: str = "") -> ZccState:
    """Fields as in tests/golden/chess_*.json (history strings: 5 digits per move)."""
    s = ZccState()
    s.board[:] = list(board.encode("latin-1"))
    s.turn, s.fifty, s.castle = turn, fifty, castle
    for name, h in (("hw", hw), ("hb", hb)):
        ms = _hist_moves(h)
        arr = getattr(s, name)
        for i, m in enumerate(ms):
            arr[i] = ZccMove(*m)
        setattr(s, "n" + name, len(ms))
    return s


def chess_from_json(e: dict) -> ZccState:
    return chess_state(e["board"], e["turn"], e["fifty"], e["castle"], e.get("hw", ""), e.get("hb", ""))


def chess_init() -> ZccState:
    s = ZccState()
    _chess_lib().zcc_init(ctypes.byref(s))
    return s


def chess_from_fen(fen: str) -> ZccState:
    s = ZccState()
    if _chess_lib().zcc_from_fen(fen.encode(), ctypes.byref(s)):
        raise ValueError(fen)
    return s


def chess_moves(s: ZccState):
    out = (ZccMove * ZCC_MAX_MOVES)()
    n = _chess_lib().zcc_legal_moves(ctypes.byref(s), out)
    return [(m.fr, m.fc, m.tr, m.tc, m.value) for m in out[:n]]


def chess_play(s: ZccState, move) -> ZccState:
    o = ZccState()
    _chess_lib().zcc_play(ctypes.byref(s), ctypes.byref(ZccMove(*move)), ctypes.byref(o))
    return o


def chess_win(s: ZccState) -> bool:
    return bool(_chess_lib().zcc_check_win(ctypes.byref(s)))


def chess_draw(s: ZccState) -> bool:
    return bool(_chess_lib().zcc_check_draw(ctypes.byref(s)))


def chess_rollout(s: ZccState, mt: "MT"):
    """Value('random_rollout') on the chess rules from s on the stream mt (advanced):
    (value, plies); value 2 = a history outgrew the restatement's ZCC_HIST."""
    L = _chess_lib()
    L.zcc_rollout.argtypes = [ctypes.POINTER(ZccState), ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    q = ctypes.c_int(0)
    v = L.zcc_rollout(ctypes.byref(s), ctypes.cast(ctypes.byref(mt.s), ctypes.c_void_p), ctypes.byref(q))
    return v, q.value


def chess_tensor(s: ZccState):
    import numpy as np
    out = np.zeros(17 * 64, np.float32)
    _chess_lib().zcc_state_to_tensor(ctypes.byref(s), out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return out.reshape(17, 8, 8)


def chess_perft(s: ZccState, depth: int) -> int:
    return int(_chess_lib().zcc_perft(ctypes.byref(s), depth))


class ZccLight(ctypes.Structure):
    _fields_ = [("board", ctypes.c_uint8 * 64), ("turn", ctypes.c_uint8), ("fifty", ctypes.c_uint8),
                ("castle", ctypes.c_uint8), ("pad", ctypes.c_uint8)]


CHESS_VALUE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ZccLight),
                                  ctypes.POINTER(ctypes.c_double))


def chess_light(s: ZccState) -> ZccLight:
    l = ZccLight()
    l.board[:] = list(s.board)
    l.turn, l.fifty, l.castle = s.turn, s.fifty, s.castle
    return l


def chess_get_move(s: ZccState, mt: MT, sims: int, c: float, bs: int, policy: str = "random", freedom: float = 0.0,
                   value_batch=None):
    """mcts.get_move for chess (crude_chess_score unless value_batch(list of (board bytes,
    turn, fifty, castle)) -> values is given).  Returns (best index, root moves, root visits)."""
    L = _chess_lib()
    L.zcc_get_move.argtypes = [ctypes.POINTER(ZccLight), ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                               ctypes.c_int, ctypes.c_double, CHESS_VALUE_FN, ctypes.c_void_p,
                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ZccMove), ctypes.POINTER(ctypes.c_int)]
    if value_batch is not None:
        def cb(_ctx, n, leaves, out):
            vals = value_batch([(bytes(leaves[j].board), leaves[j].turn, leaves[j].fifty, leaves[j].castle)
                                for j in range(n)])
            for j in range(n):
                out[j] = float(vals[j])
        fn = CHESS_VALUE_FN(cb)
    else:
        fn = ctypes.cast(None, CHESS_VALUE_FN)
    na = (ctypes.c_int * ZCC_MAX_MOVES)()
    mv = (ZccMove * ZCC_MAX_MOVES)()
    n = ctypes.c_int(0)
    best = L.zcc_get_move(ctypes.byref(chess_light(s)), ctypes.cast(ctypes.byref(mt.s), ctypes.c_void_p), sims, c, bs,
                          1 if policy == "immediate_value" else 0, float(freedom), fn, None, na,
                          mv, ctypes.byref(n))
    moves = [(m.fr, m.fc, m.tr, m.tc, m.value) for m in mv[:n.value]]
    return best, moves, list(na[:n.value])


def chess_selfplay_batch(rows, mts: list["MT"], moves: int, sims: int, c: float = 1.4, bs: int = 32,
                         policy: str = "immediate_value", freedom: float = 3.0, threads: int = 1):
    """zcc_selfplay_batch: crude-score self-play, each game `moves` moves (search, play, judge,
    refill) from its position — rows: [n, >= 67] uint8 zc_chess_state rows (board, turn, fifty,
    castle) — and MT state (advanced); returns expansions (nodes created) per game."""
    import numpy as np
    rows = np.ascontiguousarray(rows, np.uint8)
    n = rows.shape[0]
    light = (ZccLight * max(n, 1))()
    for i in range(n):
        light[i].board[:] = [int(x) for x in rows[i, :64]]
        light[i].turn, light[i].fifty, light[i].castle = int(rows[i, 64]), int(rows[i, 65]), int(rows[i, 66])
    arr = (_MT * max(n, 1))()
    for i, m in enumerate(mts):
        arr[i] = m.s
    exp = np.zeros(n, np.uint64)
    L = _chess_lib()
    L.zcc_selfplay_batch.argtypes = [ctypes.c_int, ctypes.POINTER(ZccLight), ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_uint64)]
    L.zcc_selfplay_batch(n, light, ctypes.cast(arr, ctypes.c_void_p), moves, sims, c, bs,
                         1 if policy == "immediate_value" else 0, float(freedom), threads,
                         exp.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    for i, m in enumerate(mts):
        m.s = arr[i]
    return exp
