"""Deterministic test value functions for the stepwise (caller-valued) search.

`hash_value(s0, s1, turn)` is a fixed pseudo-random function of the position (zc_c4_state
bitboards: bit 7*col + row-from-bottom) with full fp64 mantissas, so backups exercise the
order of the fp64 Wa subtractions (mcts.cpp:90).  Used by tests/golden/gen_golden_valued.py
(to drive the reference) and by the tests (to drive the oracle and the GPU path)."""
M64 = (1 << 64) - 1


def hash_value(s0: int, s1: int, turn: int) -> float:
    h = (s0 * 0x9E3779B97F4A7C15 + s1 * 0xC2B2AE3D27D4EB4F + turn * 0x165667B19E3779F9) & M64
    h ^= h >> 29
    h = (h * 0xBF58476D1CE4E5B9) & M64
    h ^= h >> 32
    return ((h % 200001) - 100000) / 100003.0


def bits_from_rows(rows):
    """6x7 board (row 0 = top; 'X' / 'O' / other) or a 42-char string -> (s0, s1)."""
    if isinstance(rows, str):
        cells = rows
    else:
        cells = "".join("".join(r) for r in rows)
    s0 = s1 = 0
    for r in range(6):
        for c in range(7):
            ch = cells[r * 7 + c]
            bit = 1 << (7 * c + (5 - r))
            if ch == "X":
                s0 |= bit
            elif ch == "O":
                s1 |= bit
    return s0, s1
