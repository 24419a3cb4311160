#!/usr/bin/env python3
"""One C5 move (bench.puct_mode) for rocprofv3 --kernel-trace --stats: the kernel split of
the PUCT search with the policy+value network."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

print(bench.puct_mode(1, torch.device("cuda", 0)), flush=True)
