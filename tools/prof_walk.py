#!/usr/bin/env python3
"""The tree walk measured on its own (select + expand-write + backup, the
roofline object), not modelled: the bench's workload — C4SelfPlay at 4096 games x 800 sims x
bs 32 burned in to steady state (bench.burn_in) — then, from one snapshot of the roots and the
games' MT19937 streams:

  1. the lockstep search with its rollouts RECORDED (c4_walk_kernel<1>: every leaf's value,
     every flush's rollout words) — the full search kernel's work;
  2. the product search kernel (c4_search_kernel<false, false>) from the same snapshot: its
     moves, root visits and counters must equal 1.'s (recording changes nothing);
  3. --reps launches of the walk REPLAY (c4_walk_kernel<2>): the recorded values instead of
     the rollouts, the stream moved past the recorded words — the identical tree (moves, root
     visits, expansions, depth sum and words consumed are checked equal), with no rollout.

HIP events on the launch stream time 2. and 3.; rocprofv3 passes over this script (kernel
trace, --pmc FETCH_SIZE, --pmc WRITE_SIZE: tools/gpu_check.sh stages wprof / whbm / wpmc) give the replay kernel's
duration and HBM bytes.  Prints one JSON line: per launch the expansions, the SURVEY §8(d)
model bytes (152 d + 96 per expansion) and the event times."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from zeroclone_amd.selfplay import C4SelfPlay  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream(torch.device("cuda", 0)))
    sp = C4SelfPlay(a.games, a.sims, c=1.4, batch_size=a.batch, seed=0, device=0, record=True)
    burn = bench.burn_in(sp)
    out = bench.walk_measure(sp, a.reps)
    out["burn_in_steps"] = burn
    out["lib_sha256"] = bench.lib_sha()   # the library this run loaded (stamps the profile summary)
    print(json.dumps(out), flush=True)
    sp.close()


if __name__ == "__main__":
    main()
