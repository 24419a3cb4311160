#!/usr/bin/env python3
"""Golden vectors for the value network (SURVEY.md §8c fixture 10).

Runs ONLY in the build container: imports the reference's models/chess_value/network.py by
file path (unmodified), builds `ValueNetwork()` after torch.manual_seed(SEED) on the CPU in
eval mode, and records its fp32 outputs on 64 fixed random 0/1 plane stacks, plus the
state_dict names and shapes.  The inputs are stored as packed bits; the tower's weights are
not stored (the seeded init regenerates them).

Two heads over the same tower (network.py:37-45: avg-pool -> Linear(128, 1) -> tanh):
  * "outputs": the seeded head as initialised.  Its outputs span only -0.08 .. -0.04 (std
    0.0098): a random-init tower's pooled features vary little between inputs.
  * "outputs_wide": the head's Linear replaced by the top principal direction of the 64
    inputs' pooled features (the direction along which the inputs differ most), scaled so
    the pre-tanh sum has std 1.2 and mean 0 — outputs spanning most of tanh's range, so a
    tolerance of a few 1e-3 is a small fraction of the signal.  The 128 + 1 head parameters
    are committed ("head_weight_wide", "head_bias_wide"); a test loads them into the seeded
    network.

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
WIDE_STD = 1.2


def main():
    spec = importlib.util.spec_from_file_location("ref_network", os.path.join(REF, "models/chess_value/network.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(SEED)
    net = mod.ValueNetwork().eval()
    rng = np.random.default_rng(7)
    x = (rng.random((N, 17, 8, 8)) < 0.2).astype(np.float32)
    xt = torch.from_numpy(x)
    with torch.no_grad():
        y = net(xt).reshape(-1).numpy().astype(np.float64)
        # the pooled features the head sees (network.py's head[0:2]: avg-pool, flatten)
        feat = net.head[1](net.head[0](net.res(net.stem(xt)))).double()
    state = {k: [list(v.shape)] for k, v in net.state_dict().items()}
    centred = feat - feat.mean(0)
    _, _, vt = torch.linalg.svd(centred, full_matrices=False)
    d = vt[0]
    proj = centred @ d
    scale = WIDE_STD / proj.std().item()
    w_wide = (d * scale).float()
    b_wide = float(-(feat.mean(0) @ (d * scale)).item())
    lin = net.head[2]
    with torch.no_grad():
        lin.weight.copy_(w_wide.reshape(1, -1))
        lin.bias.fill_(b_wide)
        y_wide = net(xt).reshape(-1).numpy().astype(np.float64)
    out = {
        "seed": SEED,
        "shape": [N, 17, 8, 8],
        "inputs_packed_hex": np.packbits(x.astype(np.uint8).reshape(-1)).tobytes().hex(),
        "outputs": [float(v) for v in y],
        "head_weight_wide": [float(v) for v in lin.weight.detach().reshape(-1)],
        "head_bias_wide": float(lin.bias.detach().item()),
        "outputs_wide": [float(v) for v in y_wide],
        "state_dict": [[k, v[0]] for k, v in state.items()],
        "torch": torch.__version__,
    }
    with open(os.path.join(HERE, "value_network.json"), "w") as f:
        json.dump(out, f)
    print("wrote value_network.json", y[:4], "std", y.std(), "| wide", y_wide.min(), y_wide.max(), "std", y_wide.std())


if __name__ == "__main__":
    main()
