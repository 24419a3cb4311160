"""ctypes binding of libzeroclone_amd.so (the C-ABI in include/zeroclone.h).

There is no CPU fallback: if the library or a GPU is missing, constructing an engine raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

from .build import LIB

P = ctypes.POINTER

ZC_OK = 0
ZC_EINVAL = -1
ZC_EHIP = -2
ZC_ENOMEM = -3
ZC_ECAPACITY = -4
ZC_EDEVICE = -5
ZC_C4_ONGOING = 2
ZC_STATUS_NO_MOVES = 1
ROLLOUT_EXACT = 0   # ZC_ROLLOUT_EXACT
ROLLOUT_PHILOX = 1  # ZC_ROLLOUT_PHILOX
ZC_STATUS_BAD_STATE = 2
ZC_F32 = 0
ZC_F16 = 1
ZC_F16_NHWC32 = 2   # planes only: fp16 NHWC [n][h*w][32], the MFMA tower's input layout


class C4State(ctypes.Structure):
    _fields_ = [("stones", ctypes.c_uint64 * 2), ("turn", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class GameStats(ctypes.Structure):
    _fields_ = [("expansions", ctypes.c_int64), ("depth_sum", ctypes.c_int64), ("leaves", ctypes.c_int64),
                ("rollout_plies", ctypes.c_int64), ("rng_words", ctypes.c_int64), ("status", ctypes.c_int64),
                ("rollout_blocks", ctypes.c_int64), ("reserved", ctypes.c_int64)]


class EngineConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("max_games", ctypes.c_int32), ("max_sims", ctypes.c_int32),
                ("max_batch", ctypes.c_int32)]


class ChessPlayBuffers(ctypes.Structure):
    """zc_chess_play_buffers (include/zeroclone.h): a chess self-play pool's device buffers."""
    _fields_ = [("d_roots", ctypes.c_void_p), ("d_init", ctypes.c_void_p), ("d_hist", ctypes.c_void_p),
                ("d_hist_len", ctypes.c_void_p), ("hist_cap", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("d_err", ctypes.c_void_p)]


class TrajBuffers(ctypes.Structure):
    """zc_traj_buffers (include/zeroclone.h): device pointers of a self-play trajectory pool."""
    _fields_ = [("row_bytes", ctypes.c_int32), ("max_len", ctypes.c_int32), ("pool_cap", ctypes.c_int64),
                ("games_cap", ctypes.c_int32), ("reserved", ctypes.c_int32), ("d_hist", ctypes.c_void_p),
                ("d_hmoves", ctypes.c_void_p), ("d_slot", ctypes.c_void_p), ("d_pool", ctypes.c_void_p),
                ("d_labels", ctypes.c_void_p), ("d_pool_moves", ctypes.c_void_p), ("d_games", ctypes.c_void_p),
                ("d_ctl", ctypes.c_void_p), ("d_init", ctypes.c_void_p)]


ZC_TRAJ_POSITIONS, ZC_TRAJ_GAMES, ZC_TRAJ_NEXT, ZC_TRAJ_QUOTA, ZC_TRAJ_FINISHED, ZC_TRAJ_OVERFLOW = range(6)
ZC_SLOT_IDLE = 3
ZC_SLOT_SKIP = 4

C4_STATE_DTYPE = np.dtype([("stones", "<u8", (2,)), ("turn", "<i4"), ("reserved", "<i4")])
# zc_c4_hp_node: the host-policy walk's end (include/zeroclone.h)
C4_HP_NODE_DTYPE = np.dtype([("state", C4_STATE_DTYPE), ("node", "<i4"), ("n_untried", "<i4"), ("depth", "<i4"),
                             ("untried", "<i4", (7,))])
STATS_DTYPE = np.dtype([("expansions", "<i8"), ("depth_sum", "<i8"), ("leaves", "<i8"),
                        ("rollout_plies", "<i8"), ("rng_words", "<i8"), ("status", "<i8"),
                        ("rollout_blocks", "<i8"), ("reserved", "<i8")])
CHESS_STATE_DTYPE = np.dtype([("board", "u1", (64,)), ("turn", "u1"), ("fifty", "u1"), ("castle", "u1"),
                              ("reserved", "u1", (5,))])
CHESS_MAX_MOVES = 256
CHESS_ROLL_CAP = 2048   # ZC_CHESS_ROLL_CAP: moves per side a chess rollout's history holds
# zc_chess_hp_node: the chess host-policy walk's end (include/zeroclone.h)
CHESS_HP_NODE_DTYPE = np.dtype([("state", CHESS_STATE_DTYPE), ("node", "<i4"), ("n_untried", "<i4"), ("depth", "<i4"),
                                ("reserved", "<i4"), ("untried", "<u2", (CHESS_MAX_MOVES,))])
# ChessNode (zc_internal.h): the device tree's node record, as zc_debug_chess_tree copies it
CHESS_NODE_DTYPE = np.dtype([("st", "u1", (72,)), ("base", "<u4"), ("nmoves", "<u2"), ("nu", "<u2"),
                             ("parent", "<u2"), ("pact", "<u2"), ("depth", "<u2"), ("material", "<i2"),
                             ("check", "u1"), ("evaluated", "u1"), ("pad", "u1", (6,))])
assert CHESS_NODE_DTYPE.itemsize == 96
# C4PNode (zc_internal.h): the Connect4 PUCT tree's node record
C4_PNODE_DTYPE = np.dtype([("s0", "<u8"), ("s1", "<u8"), ("order", "<u4"), ("turn", "u1"), ("nmoves", "u1"),
                           ("evaluated", "u1"), ("won", "u1"), ("parent", "<u2"), ("pact", "u1"), ("depth", "u1"),
                           ("pad0", "<u4"), ("child", "<u2", (8,)), ("na", "<i4", (8,)), ("pr", "<f4", (8,)),
                           ("w", "<f8", (8,)), ("pad1", "u1", (16,))])
assert C4_PNODE_DTYPE.itemsize == 192
ZC_CHESS_WIN, ZC_CHESS_STALEMATE, ZC_CHESS_FIFTY, ZC_CHESS_OVERFLOW = 1, 2, 4, 8
ZC_POLICY_RANDOM, ZC_POLICY_IMMEDIATE_VALUE = 0, 1
ZC_STATUS_CAPACITY = 4
assert CHESS_STATE_DTYPE.itemsize == 72
assert C4_STATE_DTYPE.itemsize == ctypes.sizeof(C4State) == 24
assert STATS_DTYPE.itemsize == ctypes.sizeof(GameStats) == 64
STATS_FIELDS = 8

# Every symbol include/zeroclone.h declares: (name, restype, argtypes)
SIGNATURES = [
    ("zc_version", ctypes.c_char_p, []),
    ("zc_last_error", ctypes.c_char_p, []),
    ("zc_device_count", ctypes.c_int, [P(ctypes.c_int32)]),
    ("zc_engine_create", ctypes.c_int, [P(EngineConfig), P(ctypes.c_void_p)]),
    ("zc_engine_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("zc_engine_footprint", ctypes.c_int, [ctypes.c_void_p, P(ctypes.c_int64)]),
    ("zc_rng_seed", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, P(ctypes.c_uint64)]),
    ("zc_rng_set_state", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_uint32), ctypes.c_int32]),
    ("zc_rng_get_state", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_uint32), P(ctypes.c_int32)]),
    ("zc_c4_search", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                    ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_c4_search_games", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_c4_set_rollout_mode", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64]),
    ("zc_c4_search_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_c4_play_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    ("zc_c4_ext_begin", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_void_p]),
    ("zc_c4_ext_select", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    ("zc_c4_ext_backup", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_c4_selfplay_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                            ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p]),
    ("zc_c4_selfplay_pooled_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                                   ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                                   ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_c4_selfplay_carry_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                                  ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                                  ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_c4_carry_discard", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]),
    ("zc_chess_play_step_async", ctypes.c_int, [ctypes.c_int32, P(ChessPlayBuffers), ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_selfplay_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, P(ChessPlayBuffers),
                                               ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_double, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_selfplay_pooled_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                                      P(ChessPlayBuffers), ctypes.c_int32, ctypes.c_double,
                                                      ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_int32,
                                                      ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_pooled_max_games", ctypes.c_int, [ctypes.c_int32, P(ctypes.c_int32)]),
    ("zc_c4_pooled_max_games", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_int32)]),
    ("zc_traj_steps_scratch_bytes", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, P(ctypes.c_int64)]),
    ("zc_traj_record_steps_async", ctypes.c_int, [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_int64, ctypes.c_void_p]),
    ("zc_c4_hp_walk", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                     ctypes.c_void_p]),
    ("zc_c4_hp_expand", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_c4_ext_end", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_c4_rollouts", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                      ctypes.c_void_p, P(ctypes.c_int64)]),
    ("zc_chess_legal_moves_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_children_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_play_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_repetition_async", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_terminal_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p]),
    ("zc_chess_planes_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_int32, ctypes.c_void_p]),
    ("zc_chess_reserve", ctypes.c_int, [ctypes.c_void_p]),
    ("zc_chess_search_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                             ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p]),
    ("zc_chess_ext_begin", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_double, ctypes.c_void_p]),
    ("zc_chess_ext_select", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    ("zc_chess_ext_backup", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_hp_walk", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_hp_expand", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_ext_end", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_rollouts_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_ext_rollouts", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_ext_leaf_moves", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_puct_flushes", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32]),
    ("zc_chess_puct_begin", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_puct_select", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                            ctypes.c_void_p]),
    ("zc_chess_puct_backup", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    ("zc_chess_puct_backup_ex", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_void_p]),
    ("zc_chess_puct_end", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    ("zc_c4_puct_begin", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_float,
                                        ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_c4_puct_select", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    ("zc_c4_puct_backup", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    ("zc_c4_puct_backup_ex", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_void_p]),
    ("zc_c4_puct_end", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    ("zc_debug_c4_puct_tree", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                             ctypes.c_void_p]),
    ("zc_net_conv3x3_async", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    ("zc_net_conv3x3_pack_async", ctypes.c_int, [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_net_conv3x3_packed_async", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    ("zc_net_tower_async", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    ("zc_net_tower_policy_async", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_net_tower_policy_ex_async", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                    ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                                    ctypes.c_void_p]),
    ("zc_net_planes_to_nhwc_async", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_net_value_head_async", ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_traj_record_async", ctypes.c_int, [ctypes.c_int32, P(TrajBuffers), ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_chess_from_fen", ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p]),
    ("zc_chess_init", ctypes.c_int, [ctypes.c_void_p]),
    ("zc_c4_from_rows", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32, P(C4State)]),
    ("zc_c4_to_rows", ctypes.c_int, [P(C4State), ctypes.c_char_p]),
    ("zc_c4_legal_order", ctypes.c_int, [ctypes.c_int32, P(ctypes.c_int32)]),
    ("zc_gen_reserve", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64]),
    ("zc_gen_capacity", ctypes.c_int, [ctypes.c_void_p, P(ctypes.c_int32), P(ctypes.c_int64)]),
    ("zc_gen_begin", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_void_p]),
    ("zc_gen_walk", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    ("zc_gen_expand", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]),
    ("zc_gen_backup", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_gen_end", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    ("zc_debug_uct", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p]),
    ("zc_debug_chess_probe_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p]),
    ("zc_debug_chess_tree", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_debug_c4_walk_async", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                              ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_debug_rng_copy", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                         ctypes.c_int32, ctypes.c_void_p]),
    ("zc_debug_phase_cycles", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_int64)]),
    ("zc_debug_phase_cycles_games", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_int64)]),
    ("zc_debug_net_switch", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32, P(ctypes.c_int32)]),
    ("zc_debug_c4_launch_stamps", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("zc_debug_c4_rollout", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]),
]

_lib = None
_lock = threading.Lock()


class ZeroCloneError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[zc {code}] {msg}")
        self.code = code


def lib(build_if_missing: bool = True):
    """Load libzeroclone_amd.so (building it with hipcc if absent and allowed)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB):
                if not build_if_missing:
                    raise ImportError(f"{LIB} not built (run python -m zeroclone_amd.build)")
                from .build import build
                build()
            L = ctypes.CDLL(LIB)
            for name, res, args in SIGNATURES:
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int):
    if rc < 0:
        msg = lib().zc_last_error().decode(errors="replace")
        if rc == ZC_EINVAL:
            raise ValueError(msg)
        raise ZeroCloneError(rc, msg)
    return rc


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def device_count() -> int:
    n = ctypes.c_int32(0)
    check(lib().zc_device_count(ctypes.byref(n)))
    return n.value


def c4_from_rows(rows42: str, turn: int) -> np.void:
    s = C4State()
    check(lib().zc_c4_from_rows(rows42.encode(), int(turn), ctypes.byref(s)))
    out = np.zeros((), C4_STATE_DTYPE)
    out["stones"] = (s.stones[0], s.stones[1])
    out["turn"] = s.turn
    return out


def c4_legal_order(mask: int) -> list[int]:
    cols = (ctypes.c_int32 * 7)()
    n = check(lib().zc_c4_legal_order(int(mask), cols))
    return list(cols[:n])


def chess_from_fen(fen: str) -> np.ndarray:
    out = np.zeros(1, CHESS_STATE_DTYPE)
    check(lib().zc_chess_from_fen(fen.encode(), _ptr(out)))
    return out[0]


def chess_init() -> np.ndarray:
    out = np.zeros(1, CHESS_STATE_DTYPE)
    check(lib().zc_chess_init(_ptr(out)))
    return out[0]


def unpack_chess_move(m: int):
    """uint16 move -> ((fr, fc, tr, tc), capture value)."""
    m = int(m)
    f, t = m & 63, (m >> 6) & 63
    return (f >> 3, f & 7, t >> 3, t & 7), float((m >> 12) & 15)


def pack_chess_move(fr: int, fc: int, tr: int, tc: int, value: float) -> int:
    return (fr * 8 + fc) | ((tr * 8 + tc) << 6) | (int(value) << 12)


class NativeEngine:
    """One HIP device's arena: `max_games` resident games, trees of max_sims+1 nodes."""

    def __init__(self, max_games: int, max_sims: int, max_batch: int = 32, device: int = 0):
        L = lib()
        cfg = EngineConfig(device, max_games, max_sims, max_batch)
        h = ctypes.c_void_p()
        check(L.zc_engine_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.max_games, self.max_sims, self.max_batch, self.device = max_games, max_sims, max_batch, device

    def close(self):
        if getattr(self, "_h", None):
            lib().zc_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def footprint(self) -> int:
        b = ctypes.c_int64(0)
        check(lib().zc_engine_footprint(self._h, ctypes.byref(b)))
        return b.value

    # ---- random streams
    def seed(self, first_game: int, seeds) -> None:
        s = np.ascontiguousarray(seeds, dtype=np.uint64)
        check(lib().zc_rng_seed(self._h, first_game, len(s), s.ctypes.data_as(P(ctypes.c_uint64))))

    def set_rng_state(self, game: int, mt624, index: int) -> None:
        mt = np.ascontiguousarray(mt624, dtype=np.uint32)
        assert mt.shape == (624,)
        check(lib().zc_rng_set_state(self._h, game, mt.ctypes.data_as(P(ctypes.c_uint32)), int(index)))

    def get_rng_state(self, game: int):
        mt = np.zeros(624, np.uint32)
        idx = ctypes.c_int32(0)
        check(lib().zc_rng_get_state(self._h, game, mt.ctypes.data_as(P(ctypes.c_uint32)), ctypes.byref(idx)))
        return mt, idx.value

    # ---- search
    def c4_search(self, roots: np.ndarray, sims: int, c: float = 1.4, batch_size: int = 32, first_game: int = 0):
        roots = np.ascontiguousarray(roots, dtype=C4_STATE_DTYPE)
        n = roots.shape[0]
        mv = np.zeros(n, np.int32)
        na = np.zeros((n, 7), np.int32)
        st = np.zeros(n, STATS_DTYPE)
        check(lib().zc_c4_search(self._h, first_game, n, _ptr(roots), int(sims), float(c), int(batch_size),
                                 _ptr(mv), _ptr(na), _ptr(st)))
        return mv, na, st

    def c4_search_games(self, games, roots: np.ndarray, sims: int, c: float = 1.4, batch_size: int = 32):
        ids = np.ascontiguousarray(games, dtype=np.int32)
        roots = np.ascontiguousarray(roots, dtype=C4_STATE_DTYPE)
        n = roots.shape[0]
        assert ids.shape == (n,)
        mv = np.zeros(n, np.int32)
        na = np.zeros((n, 7), np.int32)
        st = np.zeros(n, STATS_DTYPE)
        check(lib().zc_c4_search_games(self._h, n, _ptr(ids), _ptr(roots), int(sims), float(c), int(batch_size),
                                       _ptr(mv), _ptr(na), _ptr(st)))
        return mv, na, st

    def c4_rollout_mode(self, mode: str = "exact", seed: int = 0) -> None:
        """"exact" (the game's MT19937 stream, bit-identical to the reference) or "philox"
        (leaf-parallel rollouts on per-leaf counter-based streams; statistical parity only)."""
        m = {"exact": ROLLOUT_EXACT, "philox": ROLLOUT_PHILOX}[mode]
        check(lib().zc_c4_set_rollout_mode(self._h, m, int(seed) & (2**64 - 1)))

    def c4_search_async(self, d_roots: int, n: int, sims: int, c: float, batch_size: int, d_move: int, d_na: int,
                        d_stats: int, stream: int = 0, first_game: int = 0) -> None:
        """Device-pointer entry (ints from torch .data_ptr()); enqueued on `stream`."""
        check(lib().zc_c4_search_async(self._h, first_game, n, ctypes.c_void_p(d_roots), int(sims), float(c),
                                       int(batch_size), ctypes.c_void_p(d_move), ctypes.c_void_p(d_na),
                                       ctypes.c_void_p(d_stats), ctypes.c_void_p(stream or None)))

    def c4_selfplay_async(self, d_roots: int, n: int, sims: int, c: float, batch_size: int, moves: int,
                          d_states: int, d_moves16: int, d_results: int, d_stats: int, stream: int = 0,
                          first_game: int = 0) -> None:
        """`moves` self-play moves per game in one launch (zc_c4_selfplay_async)."""
        check(lib().zc_c4_selfplay_async(self._h, first_game, n, ctypes.c_void_p(d_roots), int(sims), float(c),
                                         int(batch_size), int(moves), ctypes.c_void_p(d_states),
                                         ctypes.c_void_p(d_moves16), ctypes.c_void_p(d_results),
                                         ctypes.c_void_p(d_stats), ctypes.c_void_p(stream or None)))

    def c4_selfplay_pooled_async(self, d_roots: int, n: int, sims: int, c: float, batch_size: int, moves_cap: int,
                                 budget: int, d_ticket: int, d_states: int, d_moves16: int, d_results: int,
                                 d_stats: int, stream: int = 0, first_game: int = 0, carry: bool = False) -> None:
        """`budget` self-play moves shared by the games in one launch, at most `moves_cap` per
        game (zc_c4_selfplay_pooled_async; carry: in-flight moves carry over into the next
        launch, zc_c4_selfplay_carry_async)."""
        fn = lib().zc_c4_selfplay_carry_async if carry else lib().zc_c4_selfplay_pooled_async
        check(fn(self._h, first_game, n, ctypes.c_void_p(d_roots), int(sims),
                                                float(c), int(batch_size), int(moves_cap), int(budget),
                                                ctypes.c_void_p(d_ticket), ctypes.c_void_p(d_states),
                                                ctypes.c_void_p(d_moves16), ctypes.c_void_p(d_results),
                                                ctypes.c_void_p(d_stats), ctypes.c_void_p(stream or None)))

    def c4_carry_discard(self, first_game: int, n: int, stream: int = 0) -> None:
        check(lib().zc_c4_carry_discard(self._h, int(first_game), int(n), ctypes.c_void_p(stream or None)))

    def c4_pooled_max_games(self, batch_size: int) -> int:
        n = ctypes.c_int32(0)
        check(lib().zc_c4_pooled_max_games(self._h, int(batch_size), ctypes.byref(n)))
        return n.value

    # ---- any game backend (zc_gen_*)
    def gen_reserve(self, nodes: int, slots: int) -> None:
        check(lib().zc_gen_reserve(self._h, int(nodes), int(slots)))

    def gen_capacity(self):
        n, s = ctypes.c_int32(0), ctypes.c_int64(0)
        check(lib().zc_gen_capacity(self._h, ctypes.byref(n), ctypes.byref(s)))
        return n.value, s.value

    def gen_begin(self, sims: int, c: float, batch_size: int, root_moves: int, stream: int = 0) -> None:
        check(lib().zc_gen_begin(self._h, int(sims), float(c), int(batch_size), int(root_moves),
                                 ctypes.c_void_p(stream or None)))

    def gen_walk(self, d_out: int, out_cap: int, stream: int = 0) -> None:
        check(lib().zc_gen_walk(self._h, ctypes.c_void_p(d_out), int(out_cap), ctypes.c_void_p(stream or None)))

    def gen_expand(self, untried_index: int, child_moves: int, stream: int = 0) -> None:
        check(lib().zc_gen_expand(self._h, int(untried_index), int(child_moves), ctypes.c_void_p(stream or None)))

    def gen_backup(self, n: int, d_values: int, stream: int = 0) -> None:
        check(lib().zc_gen_backup(self._h, int(n), ctypes.c_void_p(d_values), ctypes.c_void_p(stream or None)))

    def gen_end(self, d_out: int, d_root_na: int = 0, na_cap: int = 0, stream: int = 0) -> None:
        check(lib().zc_gen_end(self._h, ctypes.c_void_p(d_out), ctypes.c_void_p(d_root_na or None), int(na_cap),
                               ctypes.c_void_p(stream or None)))

    def c4_play_async(self, d_states: int, n: int, d_moves: int, d_results: int, reset: bool = True,
                      stream: int = 0) -> None:
        check(lib().zc_c4_play_async(self._h, n, ctypes.c_void_p(d_states), ctypes.c_void_p(d_moves),
                                     ctypes.c_void_p(d_results), int(bool(reset)), ctypes.c_void_p(stream or None)))

    # ---- stepwise search (caller-supplied values); device pointers as ints, 0 = NULL
    def c4_ext_begin(self, first_game: int, n: int, d_roots: int, sims: int, c: float, batch_size: int,
                     stream: int = 0) -> None:
        check(lib().zc_c4_ext_begin(self._h, first_game, n, ctypes.c_void_p(d_roots), int(sims), float(c),
                                    int(batch_size), ctypes.c_void_p(stream or None)))

    def c4_ext_select(self, first_game: int, n: int, flush: int, d_leaves: int = 0, d_planes: int = 0,
                      planes_f16: bool = True, d_counts: int = 0, stream: int = 0) -> None:
        check(lib().zc_c4_ext_select(self._h, first_game, n, int(flush), ctypes.c_void_p(d_leaves or None),
                                     ctypes.c_void_p(d_planes or None), ZC_F16 if planes_f16 else ZC_F32,
                                     ctypes.c_void_p(d_counts or None), ctypes.c_void_p(stream or None)))

    def c4_ext_backup(self, first_game: int, n: int, flush: int, d_values: int, stream: int = 0) -> None:
        check(lib().zc_c4_ext_backup(self._h, first_game, n, int(flush), ctypes.c_void_p(d_values),
                                     ctypes.c_void_p(stream or None)))

    def c4_hp_walk(self, game: int, flush: int, leaf: int, d_node: int, stream: int = 0) -> None:
        check(lib().zc_c4_hp_walk(self._h, game, int(flush), int(leaf), ctypes.c_void_p(d_node),
                                  ctypes.c_void_p(stream or None)))

    def c4_hp_expand(self, game: int, flush: int, leaf: int, index: int, d_leaf: int = 0, stream: int = 0) -> None:
        check(lib().zc_c4_hp_expand(self._h, game, int(flush), int(leaf), int(index), ctypes.c_void_p(d_leaf or None),
                                    ctypes.c_void_p(stream or None)))

    def c4_ext_end(self, first_game: int, n: int, d_move: int, d_na: int, d_stats: int, stream: int = 0) -> None:
        check(lib().zc_c4_ext_end(self._h, first_game, n, ctypes.c_void_p(d_move), ctypes.c_void_p(d_na),
                                  ctypes.c_void_p(d_stats), ctypes.c_void_p(stream or None)))

    # ---- chess rules (device pointers; stream 0 = null stream)
    def chess_legal_moves_async(self, n: int, d_states: int, d_moves: int, d_counts: int, stream: int = 0):
        check(lib().zc_chess_legal_moves_async(self._h, n, ctypes.c_void_p(d_states), ctypes.c_void_p(d_moves),
                                               ctypes.c_void_p(d_counts), ctypes.c_void_p(stream or None)))

    def chess_children_async(self, n: int, d_states: int, d_children: int, d_moves: int, d_counts: int,
                             stream: int = 0):
        check(lib().zc_chess_children_async(self._h, n, ctypes.c_void_p(d_states), ctypes.c_void_p(d_children),
                                            ctypes.c_void_p(d_moves or None), ctypes.c_void_p(d_counts),
                                            ctypes.c_void_p(stream or None)))

    def debug_chess_tree(self, game: int, max_nodes: int = 1 << 16, max_slots: int = 1 << 22) -> dict:
        """Game `game`'s chess tree after a search (test hook): node records and slot arrays."""
        nodes = np.zeros(max_nodes, CHESS_NODE_DTYPE)
        mv = np.zeros(max_slots, np.uint16)
        pr = np.zeros(max_slots, np.float32)
        na = np.zeros(max_slots, np.int32)
        w = np.zeros(max_slots, np.float64)
        ch = np.zeros(max_slots, np.uint16)
        cnt = np.zeros(2, np.int32)
        check(lib().zc_debug_chess_tree(self._h, int(game), max_nodes, max_slots, _ptr(nodes), _ptr(mv), _ptr(pr),
                                        _ptr(na), _ptr(w), _ptr(ch), _ptr(cnt)))
        n, s = int(cnt[0]), int(cnt[1])
        return {"nodes": nodes[:n], "mv": mv[:s], "prior": pr[:s], "na": na[:s], "w": w[:s], "child": ch[:s]}

    def chess_play_async(self, n: int, d_in: int, d_moves: int, d_out: int, stream: int = 0):
        check(lib().zc_chess_play_async(self._h, n, ctypes.c_void_p(d_in), ctypes.c_void_p(d_moves),
                                        ctypes.c_void_p(d_out), ctypes.c_void_p(stream or None)))

    def debug_chess_probe_async(self, n: int, d_states: int, d_out: int, stream: int = 0):
        """zc_debug_chess_probe_async: -2 (a legal move proven, no list) or the list length."""
        check(lib().zc_debug_chess_probe_async(self._h, n, ctypes.c_void_p(d_states), ctypes.c_void_p(d_out),
                                               ctypes.c_void_p(stream or None)))

    def chess_terminal_async(self, n: int, d_states: int, d_flags: int, stream: int = 0):
        check(lib().zc_chess_terminal_async(self._h, n, ctypes.c_void_p(d_states), ctypes.c_void_p(d_flags),
                                            ctypes.c_void_p(stream or None)))

    def chess_planes_async(self, n: int, d_states: int, d_planes: int, f16: bool = False, stream: int = 0):
        check(lib().zc_chess_planes_async(self._h, n, ctypes.c_void_p(d_states), ctypes.c_void_p(d_planes),
                                          ZC_F16 if f16 else ZC_F32, ctypes.c_void_p(stream or None)))

    # ---- chess tree search (device pointers)
    def chess_reserve(self):
        check(lib().zc_chess_reserve(self._h))

    def chess_search_async(self, first_game: int, n: int, d_roots: int, sims: int, c: float, batch_size: int,
                           policy: int, freedom: float, d_move: int, d_na: int, d_stats: int, stream: int = 0):
        check(lib().zc_chess_search_async(self._h, first_game, n, ctypes.c_void_p(d_roots), int(sims), float(c),
                                          int(batch_size), int(policy), float(freedom), ctypes.c_void_p(d_move),
                                          ctypes.c_void_p(d_na), ctypes.c_void_p(d_stats),
                                          ctypes.c_void_p(stream or None)))

    def chess_ext_begin(self, first_game: int, n: int, d_roots: int, sims: int, c: float, batch_size: int,
                        policy: int = 0, freedom: float = 0.0, stream: int = 0):
        check(lib().zc_chess_ext_begin(self._h, first_game, n, ctypes.c_void_p(d_roots), int(sims), float(c),
                                       int(batch_size), int(policy), float(freedom), ctypes.c_void_p(stream or None)))

    def chess_ext_select(self, first_game: int, n: int, flush: int, d_leaves: int = 0, d_planes: int = 0,
                         planes_f16: bool = True, d_counts: int = 0, stream: int = 0):
        check(lib().zc_chess_ext_select(self._h, first_game, n, int(flush), ctypes.c_void_p(d_leaves or None),
                                        ctypes.c_void_p(d_planes or None), ZC_F16 if planes_f16 else ZC_F32,
                                        ctypes.c_void_p(d_counts or None), ctypes.c_void_p(stream or None)))

    def chess_ext_backup(self, first_game: int, n: int, flush: int, d_values: int, stream: int = 0):
        check(lib().zc_chess_ext_backup(self._h, first_game, n, int(flush), ctypes.c_void_p(d_values),
                                        ctypes.c_void_p(stream or None)))

    def chess_hp_walk(self, game: int, flush: int, leaf: int, d_node: int, stream: int = 0) -> None:
        check(lib().zc_chess_hp_walk(self._h, game, int(flush), int(leaf), ctypes.c_void_p(d_node),
                                     ctypes.c_void_p(stream or None)))

    def chess_hp_expand(self, game: int, flush: int, leaf: int, index: int, d_leaf: int = 0, stream: int = 0) -> None:
        check(lib().zc_chess_hp_expand(self._h, game, int(flush), int(leaf), int(index),
                                       ctypes.c_void_p(d_leaf or None), ctypes.c_void_p(stream or None)))

    def chess_ext_end(self, first_game: int, n: int, d_move: int, d_na: int, d_stats: int, stream: int = 0):
        check(lib().zc_chess_ext_end(self._h, first_game, n, ctypes.c_void_p(d_move), ctypes.c_void_p(d_na),
                                     ctypes.c_void_p(d_stats), ctypes.c_void_p(stream or None)))

    # ---- the walk diagnostic (device pointers; tools/prof_walk.py)
    def c4_walk_async(self, first_game: int, n: int, d_roots: int, sims: int, c: float, batch_size: int, mode: int,
                      d_vals: int, d_words: int, d_move: int, d_na: int, d_stats: int, stream: int = 0):
        check(lib().zc_debug_c4_walk_async(self._h, first_game, n, ctypes.c_void_p(d_roots), int(sims), float(c),
                                           int(batch_size), int(mode), ctypes.c_void_p(d_vals),
                                           ctypes.c_void_p(d_words), ctypes.c_void_p(d_move), ctypes.c_void_p(d_na),
                                           ctypes.c_void_p(d_stats), ctypes.c_void_p(stream or None)))

    def rng_copy(self, first_game: int, n: int, d_buf: int, restore: bool, stream: int = 0):
        check(lib().zc_debug_rng_copy(self._h, first_game, n, ctypes.c_void_p(d_buf), 1 if restore else 0,
                                      ctypes.c_void_p(stream or None)))

    # ---- Value('random_rollout') on chess (device pointers)
    def chess_rollouts_async(self, game: int, n: int, d_states: int, d_hist: int, d_hist_len: int, hist_cap: int,
                             d_values: int, d_status: int = 0, stream: int = 0):
        check(lib().zc_chess_rollouts_async(self._h, int(game), int(n), ctypes.c_void_p(d_states),
                                            ctypes.c_void_p(d_hist), ctypes.c_void_p(d_hist_len), int(hist_cap),
                                            ctypes.c_void_p(d_values), ctypes.c_void_p(d_status or None),
                                            ctypes.c_void_p(stream or None)))

    def chess_ext_rollouts(self, first_game: int, n: int, flush: int, d_hist: int, d_hist_len: int, hist_cap: int,
                           d_values: int, d_status: int = 0, stream: int = 0):
        check(lib().zc_chess_ext_rollouts(self._h, first_game, n, int(flush), ctypes.c_void_p(d_hist),
                                          ctypes.c_void_p(d_hist_len), int(hist_cap), ctypes.c_void_p(d_values),
                                          ctypes.c_void_p(d_status or None), ctypes.c_void_p(stream or None)))

    def chess_ext_leaf_moves(self, first_game: int, n: int, flush: int, d_moves: int, d_depth: int, stream: int = 0):
        check(lib().zc_chess_ext_leaf_moves(self._h, first_game, n, int(flush), ctypes.c_void_p(d_moves),
                                            ctypes.c_void_p(d_depth), ctypes.c_void_p(stream or None)))

    # ---- chess PUCT search (device pointers)
    def chess_puct_begin(self, first_game, n, d_roots, sims, c_puct, batch_size, alpha, eps, seed, d_search_no=0,
                        stream=0):
        check(lib().zc_chess_puct_begin(self._h, first_game, n, ctypes.c_void_p(d_roots), int(sims), float(c_puct),
                                        int(batch_size), float(alpha), float(eps), int(seed) & (2**64 - 1),
                                        ctypes.c_void_p(d_search_no or None), ctypes.c_void_p(stream or None)))

    def chess_puct_select(self, first_game, n, flush, d_leaves=0, d_planes=0, planes_f16=True, d_counts=0, stream=0,
                          planes_nhwc=False):
        """planes_nhwc: fp16 planes in the tower's input layout [n*bs][64][32] (ZC_F16_NHWC32)."""
        code = ZC_F16_NHWC32 if planes_nhwc else ZC_F16 if planes_f16 else ZC_F32
        check(lib().zc_chess_puct_select(self._h, first_game, n, int(flush), ctypes.c_void_p(d_leaves or None),
                                         ctypes.c_void_p(d_planes or None), code,
                                         ctypes.c_void_p(d_counts or None), ctypes.c_void_p(stream or None)))

    def chess_puct_backup(self, first_game, n, flush, d_values, d_logits, logits_f16=False, stream=0, rows=0):
        """rows: values / logits rows per game (0: batch_size; flush 0 also takes 1 — the roots alone)."""
        check(lib().zc_chess_puct_backup_ex(self._h, first_game, n, int(flush), ctypes.c_void_p(d_values),
                                            ctypes.c_void_p(d_logits), ZC_F16 if logits_f16 else ZC_F32, int(rows),
                                            ctypes.c_void_p(stream or None)))

    def chess_puct_end(self, first_game, n, temperature, d_move, d_na, d_prior, d_stats, stream=0):
        check(lib().zc_chess_puct_end(self._h, first_game, n, float(temperature), ctypes.c_void_p(d_move),
                                      ctypes.c_void_p(d_na), ctypes.c_void_p(d_prior or None),
                                      ctypes.c_void_p(d_stats), ctypes.c_void_p(stream or None)))

    # ---- Connect4 PUCT search (device pointers as ints)
    def c4_puct_begin(self, first_game, n, d_roots, sims, c_puct, batch_size, alpha, eps, seed, d_search_no=0,
                        stream=0):
        check(lib().zc_c4_puct_begin(self._h, first_game, n, ctypes.c_void_p(d_roots), int(sims), float(c_puct),
                                     int(batch_size), float(alpha), float(eps), int(seed) & (2**64 - 1),
                                     ctypes.c_void_p(d_search_no or None), ctypes.c_void_p(stream or None)))

    def c4_puct_select(self, first_game, n, flush, d_leaves=0, d_planes=0, planes_f16=True, d_counts=0, stream=0):
        check(lib().zc_c4_puct_select(self._h, first_game, n, int(flush), ctypes.c_void_p(d_leaves or None),
                                      ctypes.c_void_p(d_planes or None), ZC_F16 if planes_f16 else ZC_F32,
                                      ctypes.c_void_p(d_counts or None), ctypes.c_void_p(stream or None)))

    def c4_puct_backup(self, first_game, n, flush, d_values, d_logits, logits_f16=False, stream=0, rows=0):
        """rows: as chess_puct_backup."""
        check(lib().zc_c4_puct_backup_ex(self._h, first_game, n, int(flush), ctypes.c_void_p(d_values),
                                         ctypes.c_void_p(d_logits), ZC_F16 if logits_f16 else ZC_F32, int(rows),
                                         ctypes.c_void_p(stream or None)))

    def c4_puct_end(self, first_game, n, temperature, d_move, d_na, d_prior, d_stats, stream=0):
        check(lib().zc_c4_puct_end(self._h, first_game, n, float(temperature), ctypes.c_void_p(d_move),
                                   ctypes.c_void_p(d_na), ctypes.c_void_p(d_prior or None),
                                   ctypes.c_void_p(d_stats), ctypes.c_void_p(stream or None)))

    def debug_c4_puct_tree(self, game: int, max_nodes: int = 1 << 16) -> np.ndarray:
        """Game `game`'s Connect4 PUCT tree (test hook): node records (C4_PNODE_DTYPE)."""
        out = np.zeros(max_nodes, C4_PNODE_DTYPE)
        cnt = np.zeros(1, np.int32)
        check(lib().zc_debug_c4_puct_tree(self._h, int(game), max_nodes, _ptr(out), _ptr(cnt)))
        return out[:int(cnt[0])]

    def c4_rollouts(self, states: np.ndarray, game: int = 0):
        """Sequential rollouts of `states` on one game's stream: (values[n], words consumed)."""
        states = np.ascontiguousarray(states, dtype=C4_STATE_DTYPE)
        v = np.zeros(states.shape[0], np.int32)
        w = ctypes.c_int64(0)
        check(lib().zc_c4_rollouts(self._h, game, states.shape[0], _ptr(states), _ptr(v), ctypes.byref(w)))
        return v, w.value

    # ---- self-test hooks
    def debug_uct(self, logn, na, q, c: float):
        logn = np.ascontiguousarray(logn, np.float64)
        na = np.ascontiguousarray(na, np.int32)
        q = np.ascontiguousarray(q, np.float64)
        out = np.zeros(len(logn), np.float64)
        check(lib().zc_debug_uct(self._h, len(logn), _ptr(logn), _ptr(na), _ptr(q), float(c), _ptr(out)))
        return out

    def phase_cycles_games(self, n: int) -> np.ndarray:
        """Per-game stamp cycles [n, 8] accumulated since the last phase_cycles() reset."""
        out = np.zeros((n, 8), np.int64)
        check(lib().zc_debug_phase_cycles_games(self._h, int(n), out.ctypes.data_as(P(ctypes.c_int64))))
        return out

    def phase_cycles(self, enable: bool):
        out = (ctypes.c_int64 * 8)()
        check(lib().zc_debug_phase_cycles(self._h, int(bool(enable)), out))
        return dict(zip(["rng", "walk_first", "walk_resumed", "expand", "rollout", "backup", "publish", "sub"],
                        list(out)))

    def debug_c4_rollout(self, states: np.ndarray, first_game: int = 0):
        states = np.ascontiguousarray(states, dtype=C4_STATE_DTYPE)
        n = states.shape[0]
        v = np.zeros(n, np.int32)
        w = np.zeros(n, np.int64)
        check(lib().zc_debug_c4_rollout(self._h, first_game, n, _ptr(states), _ptr(v), _ptr(w)))
        return v, w


def net_switch(name: str, value: int) -> int:
    """Set one of the network launches' A/B / test switches (zc_debug_net_switch: "tower_mf",
    "tower_epi", "head_raw"); returns the previous value."""
    old = ctypes.c_int32(0)
    check(lib().zc_debug_net_switch(name.encode(), int(value), ctypes.byref(old)))
    return old.value
