"""Where C1's time goes (configs/connect4.yaml through Engine.play_mcts, 1 game, 100 sims per
move): the Engine's construction, the whole play_mcts call, the native zc_c4_search_games call
alone, and the Python around it.  GPU box only."""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from zeroclone_amd.engine import Engine  # noqa: E402
from zeroclone_amd.engine import _device  # noqa: E402

cfg = os.path.join(HERE, "configs", "connect4.yaml")
sims = 100
Engine(cfg).play_mcts(0, sims)  # load the library, first launch
for rep in range(2):
    t0 = time.perf_counter()
    e = Engine(cfg)
    e.seed = 1000 + rep
    t1 = time.perf_counter()
    moves = 0
    while e.play_mcts(0, sims) is None:
        moves += 1
    moves += 1
    t2 = time.perf_counter()
    print(f"rep {rep}: Engine() {1e3 * (t1 - t0):.2f} ms, {moves} moves, play_mcts {1e6 * (t2 - t1) / moves:.1f} us/move",
          flush=True)

eng = e._dev.eng
roots = _device.c4_roots([e.backend.create_init_state()], e.backend)
ids = [0]
for rep in range(3):
    n = 200
    t = time.perf_counter()
    for _ in range(n):
        eng.c4_search_games(ids, roots, sims, 1.4, 32)
    dt = (time.perf_counter() - t) / n
    print(f"c4_search_games (opening, {sims} sims): {1e6 * dt:.1f} us/call", flush=True)
for s in (1, 32):
    n = 200
    t = time.perf_counter()
    for _ in range(n):
        eng.c4_search_games(ids, roots, s, 1.4, 32)
    dt = (time.perf_counter() - t) / n
    print(f"c4_search_games ({s} sims): {1e6 * dt:.1f} us/call", flush=True)
from zeroclone_amd import _native  # noqa: E402
for rep in range(3):
    t = time.perf_counter()
    ne = _native.NativeEngine(max_games=64, max_sims=sims, max_batch=32, device=0)
    t1 = time.perf_counter()
    ne.close()
    print(f"NativeEngine(64 games) {1e3 * (t1 - t):.2f} ms, close {1e3 * (time.perf_counter() - t1):.2f} ms", flush=True)
st = e.backend.create_init_state()
n = 2000
t = time.perf_counter()
for _ in range(n):
    e._evaluate(st)
    _device.c4_roots([st], e.backend)
print(f"_evaluate + c4_roots: {1e6 * (time.perf_counter() - t) / n:.1f} us", flush=True)

import cProfile, pstats
e = Engine(cfg)
e.seed = 7
pr = cProfile.Profile()
pr.enable()
for g in range(3):
    e.reset_all_games()
    while e.play_mcts(0, sims) is None:
        pass
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
