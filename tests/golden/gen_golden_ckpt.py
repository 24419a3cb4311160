#!/usr/bin/env python3
"""A checkpoint in the reference's own on-disk format, for the loader test.

Runs ONLY in the build container: imports the reference's models/chess_value/network.py
under its own qualified name (`models.chess_value.network`, sys.path = the reference root,
unmodified), builds a small `ValueNetwork(channels=8, blocks=1)` after torch.manual_seed(SEED),
gives every BatchNorm seeded running statistics (so a loader that drops them is caught), and
saves the WHOLE module with `torch.save(model, path)` exactly as scripts/train.py:143 does.
Records the module's fp32 CPU outputs on 16 fixed 0/1 plane stacks.

Usage: python tests/golden/gen_golden_ckpt.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("ZC_REFERENCE", "/root/reference")
SEED = 99
N = 16


def main():
    sys.path.insert(0, REF)
    import models.chess_value.network as refnet  # the qualified name train.py pickles

    torch.manual_seed(SEED)
    net = refnet.ValueNetwork(channels=8, blocks=1)
    g = torch.Generator().manual_seed(SEED + 1)
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.weight.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.bias.copy_(torch.randn(m.num_features, generator=g) * 0.1)
    net.eval()
    path = os.path.join(HERE, "ref_value_net_c8b1.pth")
    torch.save(net, path)
    rng = np.random.default_rng(11)
    x = (rng.random((N, 17, 8, 8)) < 0.2).astype(np.float32)
    with torch.no_grad():
        y = net(torch.from_numpy(x)).reshape(-1).numpy().astype(np.float64)
    out = {"seed": SEED, "file": os.path.basename(path), "channels": 8, "blocks": 1, "shape": [N, 17, 8, 8],
           "inputs_packed_hex": np.packbits(x.astype(np.uint8).reshape(-1)).tobytes().hex(),
           "outputs": [float(v) for v in y], "torch": torch.__version__}
    with open(os.path.join(HERE, "ref_value_net_c8b1.json"), "w") as f:
        json.dump(out, f)
    print("wrote", path, os.path.getsize(path), "bytes", y[:4])


if __name__ == "__main__":
    main()
