"""CPU checks of the Philox rollout mode's specification (tests/c4_philox_ref.py): its two
generators against their published known-answer vectors, and its playouts against the
oracle's MT19937 rollouts (the reference's Value.random_rollout) in distribution."""
import math

import oracle
from c4_philox_ref import Xoshiro128, bits_from_board, philox4x32_10, rollout


def test_philox4x32_10_known_answers():
    # Random123 kat_vectors, philox4x32_10
    assert philox4x32_10((0, 0, 0, 0), (0, 0)) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    assert philox4x32_10((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2) == (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)
    assert philox4x32_10((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0)) == \
        (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)


def test_xoshiro128ss_known_answers():
    x = Xoshiro128((1, 2, 3, 4))
    assert [x.next() for _ in range(5)] == [11520, 0, 5927040, 70819200, 2031721883]


def _freq(vals):
    n = len(vals)
    return {v: vals.count(v) / n for v in (-1, 0, 1)}


def test_playouts_match_the_reference_rollout_in_distribution():
    """Outcome frequencies of Philox playouts vs the oracle's CPython-MT playouts from the
    empty board and from a mid-game position: equal within 5 binomial standard errors."""
    n = 4000
    mid = ("......." "......." "...O..." "...X..." "..XO..." ".OXXO..")
    for board, turn in (("." * 42, 0), (mid, 0)):
        x, o = bits_from_board(board)
        ph = [rollout(x, o, turn, i, 624, 7, 12345) for i in range(n)]
        mt = [oracle.rollout(board, turn, 1000 + i)[0] for i in range(n)]
        fp, fm = _freq(ph), _freq(mt)
        for v in (-1, 0, 1):
            p = (fp[v] + fm[v]) / 2
            se = math.sqrt(max(p * (1 - p), 1e-4) * 2 / n)
            assert abs(fp[v] - fm[v]) < 5 * se, (board, v, fp, fm)
