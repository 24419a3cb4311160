"""Per-simulation cycles of each rollout region (libraries from tools/rstamp_libs.sh), stamped
build on 4096 mixed-depth roots x 800 sims (the roots of tools/rollout_stats.py)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CHILD = r'''
import sys
sys.path.insert(0, %r)
import numpy as np, torch
sys.path.insert(0, %r)
from rollout_stats import mixed_roots, _native
G = 4096
roots = mixed_roots(G)
eng = _native.NativeEngine(max_games=G, max_sims=800, max_batch=32)
eng.seed(0, list(range(G)))
eng.c4_search(roots, 800, 1.4, 32)
eng.phase_cycles(True)
eng.seed(0, list(range(G)))
eng.c4_search(roots, 800, 1.4, 32)
ph = eng.phase_cycles(False)
print({k: round(v / G / 800, 1) for k, v in ph.items()})
'''
names = {1: "leaf setup", 2: "view", 3: "first segment", 4: "absorbed fill", 5: "win test", 6: "block tail"}
for k in range(1, 7):
    env = dict(os.environ, ZC_LIB=os.path.join(ROOT, "zeroclone_amd", f"lib_rs{k}.so"))
    out = subprocess.run([sys.executable, "-c", CHILD % (ROOT, HERE)], env=env,
                         check=True, capture_output=True, text=True, timeout=300).stdout.strip().splitlines()[-1]
    print(k, names[k], out, flush=True)
