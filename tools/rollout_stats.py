"""Per-leaf rollout statistics of a library build (ZC_LIB) on 4096 mixed-depth roots x 800 sims:
blocks, plies and MT words per leaf (a ZC_DIAG_* build repurposes the blocks / plies counters)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from zeroclone_amd import _native  # noqa: E402


def has4(b):
    for sh in (1, 7, 6, 8):
        m = b & (b >> sh)
        if m & (m >> (2 * sh)):
            return True
    return False


def mixed_roots(G: int = 4096, seed: int = 7, max_depth: int = 28) -> np.ndarray:
    """G random-play positions of depth 0 .. max_depth-1 without a four."""
    rs = np.random.default_rng(seed)
    roots = np.zeros(G, _native.C4_STATE_DTYPE)
    for i in range(G):
        while True:
            st, turn, ok = [0, 0], 0, True
            for _ in range(int(rs.integers(0, max_depth))):
                occ = st[0] | st[1]
                cols = [c for c in range(7) if not (occ >> (7 * c + 5)) & 1]
                c = int(rs.choice(cols))
                st[turn] |= (occ + (1 << (7 * c))) & (0x3F << (7 * c))
                if has4(st[turn]):
                    ok = False
                    break
                turn ^= 1
            if ok:
                break
        roots[i]["stones"] = st
        roots[i]["turn"] = turn
    return roots


if __name__ == "__main__":
    G = 4096
    roots = mixed_roots(G)
    eng = _native.NativeEngine(max_games=G, max_sims=800, max_batch=32)
    eng.seed(0, list(range(G)))
    mv, na, st = eng.c4_search(roots, 800, 1.4, 32)
    lv = st["leaves"].sum()
    print("blocks/leaf", st["rollout_blocks"].sum() / lv, "plies/leaf", st["rollout_plies"].sum() / lv,
          "words/leaf", st["rng_words"].sum() / lv, "expansions/leaf", st["expansions"].sum() / lv)
