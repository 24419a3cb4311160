"""Diagnostic: where do the lockstep and fused chess self-play RNG streams part?"""
import random
import sys
import torch
sys.path.insert(0, ".")
from zeroclone_amd.selfplay import ChessSelfPlay

FEN = "r1bqkbnr/pppp1ppp/2n5/4p3/2B1P3/5Q2/PPPP1PPP/RNB1K1NR w KQkq - 2 3"
G, S, B = 40, 48, 16
a = ChessSelfPlay(G, S, batch_size=B, seed=13, init_fen=FEN, hist_cap=256)
b = ChessSelfPlay(G, S, batch_size=B, seed=13, init_fen=FEN, hist_cap=256)
used = [0] * G
for k in range(14):
    ra = a.step().clone()
    rb = b.run(1).clone()[0]
    torch.cuda.synchronize()
    bad = []
    for g in range(G):
        used[g] += int(a.stats[g, 4])
        ma, ia = a.eng.get_rng_state(g)
        mb, ib = b.eng.get_rng_state(g)
        r = random.Random(13 + g)
        for _ in range(used[g]):
            r.getrandbits(32)
        st = r.getstate()[1]
        pa = ma.tolist() == list(st[:624]) and ia == st[624]
        pb = mb.tolist() == list(st[:624]) and ib == st[624]
        if ma.tolist() != mb.tolist() or ia != ib:
            nd = [i for i in range(624) if ma[i] != mb[i]]
            bad.append((g, used[g], ia, ib, st[624], pa, pb, int(b.stats[g, 4]), nd[:5], len(nd)))
    print(k, "py-match a", sum(1 for g in range(G) if True), "results equal", torch.equal(ra, rb), "roots equal", torch.equal(a.roots, b.roots), "bad", bad[:4],
          flush=True)
    if bad:
        break
