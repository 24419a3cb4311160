#!/usr/bin/env python3
"""Golden vectors for the value network (SURVEY.md §8c fixture 10).

Runs ONLY in the build container: imports the reference's models/chess_value/network.py by
file path (unmodified), builds `ValueNetwork()` after torch.manual_seed(SEED) on the CPU in
eval mode, and records its fp32 outputs on 64 fixed random 0/1 plane stacks, plus the
state_dict names and shapes.  The inputs are stored as packed bits; no weights are stored
(the seeded init regenerates them).

Usage: python tests/golden/gen_golden_nn.py
"""
import importlib.util
import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("ZC_REFERENCE", "/root/reference")
SEED = 1234
N = 64


def main():
    spec = importlib.util.spec_from_file_location("ref_network", os.path.join(REF, "models/chess_value/network.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(SEED)
    net = mod.ValueNetwork().eval()
    rng = np.random.default_rng(7)
    x = (rng.random((N, 17, 8, 8)) < 0.2).astype(np.float32)
    with torch.no_grad():
        y = net(torch.from_numpy(x)).reshape(-1).numpy().astype(np.float64)
    out = {
        "seed": SEED,
        "shape": [N, 17, 8, 8],
        "inputs_packed_hex": np.packbits(x.astype(np.uint8).reshape(-1)).tobytes().hex(),
        "outputs": [float(v) for v in y],
        "state_dict": [[k, list(v.shape)] for k, v in net.state_dict().items()],
        "torch": torch.__version__,
    }
    with open(os.path.join(HERE, "value_network.json"), "w") as f:
        json.dump(out, f)
    print("wrote value_network.json", y[:4])


if __name__ == "__main__":
    main()
