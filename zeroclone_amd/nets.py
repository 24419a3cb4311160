"""Value networks for the stepwise search (C2(iii), C4, C5).

`ValueNetwork` is the reference's residual value net (models/chess_value/network.py:24-45:
conv3x3-BN-ReLU stem, `blocks` residual blocks of two conv3x3-BN, global average pool,
linear, tanh) with the input-plane count as a parameter: 17 for chess
(chess_backend.cpp:461-521 state_to_tensor), 2 for Connect4 (c4_backend.py:52-61).  Module
names and construction order match the reference, so `torch.manual_seed(s); ValueNetwork()`
draws the same initial weights and a reference checkpoint's state_dict loads as is.

`for_inference` turns a trained/random-init model into the form the search evaluates on the
GPU: BatchNorm folded into the preceding convolution (eval-mode statistics, exact algebra),
fp16 weights, channels-last activations so MIOpen picks its NHWC MFMA kernels.  The reference
runs the same model in fp16 on its GPU (value_functions.py:4-5, 64-66).
"""
from __future__ import annotations

import copy

import torch
import torch.nn as nn


class ResidualBlock(nn.Module):
    def __init__(self, c: int):
        super().__init__()
        self.seq = nn.Sequential(
            nn.Conv2d(c, c, 3, padding=1, bias=False),
            nn.BatchNorm2d(c),
            nn.ReLU(inplace=True),
            nn.Conv2d(c, c, 3, padding=1, bias=False),
            nn.BatchNorm2d(c),
        )
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.relu(x + self.seq(x))


class ValueNetwork(nn.Module):
    def __init__(self, channels: int = 128, blocks: int = 8, in_planes: int = 17):
        super().__init__()
        self.stem = nn.Sequential(
            nn.Conv2d(in_planes, channels, 3, padding=1, bias=False),
            nn.BatchNorm2d(channels),
            nn.ReLU(inplace=True),
        )
        self.res = nn.Sequential(*(ResidualBlock(channels) for _ in range(blocks)))
        self.head = nn.Sequential(
            nn.AdaptiveAvgPool2d(1),
            nn.Flatten(),
            nn.Linear(channels, 1),
            nn.Tanh(),
        )

    def forward(self, x):
        return self.head(self.res(self.stem(x)))


def flops_per_position(channels: int, blocks: int, in_planes: int, h: int, w: int) -> int:
    """Multiply-adds x 2 of one forward (convolutions dominate; pool/linear included)."""
    conv = 2 * 9 * h * w * channels * (in_planes + 2 * blocks * channels)
    return conv + 2 * channels + h * w * channels


def _fold(conv: nn.Conv2d, bn: nn.BatchNorm2d) -> nn.Conv2d:
    scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    out = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, padding=conv.padding, bias=True)
    with torch.no_grad():
        out.weight.copy_(conv.weight * scale.reshape(-1, 1, 1, 1))
        b = conv.bias if conv.bias is not None else torch.zeros_like(bn.running_mean)
        out.bias.copy_((b - bn.running_mean) * scale + bn.bias)
    return out


class _FoldedBlock(nn.Module):
    def __init__(self, blk: ResidualBlock):
        super().__init__()
        s = blk.seq
        self.c1 = _fold(s[0], s[1])
        self.c2 = _fold(s[3], s[4])

    def forward(self, x):
        return torch.relu(x + self.c2(torch.relu(self.c1(x))))


class FoldedValueNetwork(nn.Module):
    """Inference form of ValueNetwork (eval-mode BN folded into the convolutions)."""

    def __init__(self, net: ValueNetwork):
        super().__init__()
        net = copy.deepcopy(net).eval()
        self.stem = _fold(net.stem[0], net.stem[1])
        self.res = nn.Sequential(*(_FoldedBlock(b) for b in net.res))
        self.fc = net.head[2]

    def forward(self, x):
        x = x.contiguous(memory_format=torch.channels_last)
        x = torch.relu(self.stem(x))
        x = self.res(x)
        x = x.mean(dim=(2, 3))
        return torch.tanh(self.fc(x))


def for_inference(net: ValueNetwork, device, dtype=torch.float16) -> nn.Module:
    m = FoldedValueNetwork(net).to(device=device, dtype=dtype)
    return m.to(memory_format=torch.channels_last).eval()
