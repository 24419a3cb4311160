"""Plain-Python specification of the Connect4 search's Philox rollout mode
(ZC_ROLLOUT_PHILOX, include/zeroclone.h; SURVEY §8(d) C2(ii) "rollout fast mode").

The playout is the reference's Value.random_rollout (engine/value_functions.py:35-45):
uniform random legal moves until the last mover has four (check_win) or the board is full
(check_draw); a win is worth +1 to the leaf's side to move if that side made the last move,
-1 otherwise; a leaf whose last mover already won is -1.  Only the random numbers differ from
the reference: leaf j of the flush starting at simulation `leaf0` seeds xoshiro128** with
Philox4x32-10(counter = (leaf0 + j, tag, game, 0x0C4F0A57), key = (seed_lo, seed_hi)); each ply
takes one 32-bit draw u and plays the k-th legal column in ascending order, k = (u * n) >> 32.

`value_batch(tag, game, seed)` returns a Value.batch stand-in for oracle.get_move_valued
(one call per flush, pending order), so the oracle's search with these values is the exact
specification of the device's Philox-mode search.  Test infrastructure only.
"""
M32 = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """Random123 philox4x32-10; ctr = 4 words, key = 2 words."""
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c3 ^ k1) & M32, p0 & M32
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c0, c1, c2, c3


def _rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & M32


class Xoshiro128:
    """xoshiro128** (Blackman & Vigna)."""

    def __init__(self, s):
        self.s = list(s)

    def next(self):
        s = self.s
        r = (_rotl((s[1] * 5) & M32, 7) * 9) & M32
        t = (s[1] << 9) & M32
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = _rotl(s[3], 11)
        return r


TOP = sum(1 << (7 * c + 5) for c in range(7))


def has_four(b):
    for d in (1, 7, 6, 8):
        m = b & (b >> d)
        if m & (m >> (2 * d)):
            return True
    return False


def bits_from_board(board42: str):
    """42-char rows (row 0 = top, 'X' / 'O' / '.') -> (X stones, O stones), bit 7*col + row
    counted from the bottom."""
    x = o = 0
    for r in range(6):
        for c in range(7):
            ch = board42[r * 7 + c]
            bit = 1 << (7 * c + (5 - r))
            if ch == "X":
                x |= bit
            elif ch == "O":
                o |= bit
    return x, o


def rollout(x, o, turn, leaf_index, tag, game, seed):
    """Value of one leaf for its side to move (turn 0 = X)."""
    me, op = (o, x) if turn else (x, o)
    stones = bin(me | op).count("1")
    if has_four(op):
        return -1
    if stones >= 42:
        return 0
    legal = sum(1 << c for c in range(7) if not ((me | op) >> (7 * c + 5)) & 1)
    s = philox4x32_10((leaf_index & M32, tag & M32, game & M32, 0x0C4F0A57), (seed & M32, (seed >> 32) & M32))
    if not any(s):
        s = (1, 0, 0, 0)
    rng = Xoshiro128(s)
    q = 0
    while True:
        cols = [c for c in range(7) if (legal >> c) & 1]
        k = (rng.next() * len(cols)) >> 32
        col = cols[k]
        h = bin(((me | op) >> (7 * col)) & 0x3F).count("1")
        me |= 1 << (7 * col + h)
        q += 1
        stones += 1
        if h == 5:
            legal &= ~(1 << col)
        if has_four(me):
            return 1 if q & 1 else -1
        if stones == 42:
            return 0
        me, op = op, me


def value_batch(tag, game, seed):
    """Value.batch for oracle.get_move_valued: leaves are numbered by simulation in the
    order the flushes hand them over."""
    done = [0]

    def fn(boards, turns):
        out = []
        for j, (b, t) in enumerate(zip(boards, turns)):
            x, o = bits_from_board(b)
            out.append(rollout(x, o, t, done[0] + j, tag, game, seed))
        done[0] += len(boards)
        return out

    return fn
