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


def mfma_supported(net: ValueNetwork) -> bool:
    """Shapes the hand-written MFMA tower covers: 128 channels, <= 32 input planes."""
    conv = net.stem[0]
    return conv.out_channels == 128 and conv.in_channels <= 32


def for_inference(net: ValueNetwork, device, dtype=torch.float16, backend: str = "auto"):
    """The network as the search evaluates it.  backend "mfma" (default when the shape is
    covered and the device is a GPU): this package's MFMA kernels (MfmaValueNetwork);
    "torch": the folded module in fp16, channels-last, on PyTorch-ROCm (MIOpen)."""
    use_mfma = backend == "mfma" or (backend == "auto" and dtype == torch.float16 and mfma_supported(net)
                                     and torch.device(device).type == "cuda")
    if use_mfma:
        return MfmaValueNetwork(net, device)
    m = FoldedValueNetwork(net).to(device=device, dtype=dtype)
    return m.to(memory_format=torch.channels_last).eval()


class MfmaValueNetwork:
    """The folded ValueNetwork on this package's own MFMA kernels (csrc/net_conv.hip):
    NHWC fp16 activations, implicit-GEMM conv3x3 on v_mfma_f32_32x32x16_f16 (the packed,
    streamed-weight form: zc_net_conv3x3_packed_async) with the
    bias / residual / ReLU epilogue fused, and the pooled tanh head writing fp64 values.
    Call with state_to_tensor planes [n, in_planes, H, W] fp16 (as the stepwise search
    exports them); returns fp64 values [n].  Buffers are cached per batch size, so a call
    can be captured in a HIP graph."""

    def __init__(self, net: ValueNetwork, device="cuda"):
        import torch
        f = FoldedValueNetwork(net)
        self.dev = torch.device(device)
        self.in_planes = f.stem.in_channels
        self.cpad = 32
        if self.in_planes > self.cpad or f.stem.out_channels != 128:
            raise ValueError("MFMA path: in_planes <= 32 and 128 channels")
        convs = [(f.stem, self.cpad)] + [(c, 128) for b in f.res for c in (b.c1, b.c2)]
        self.w, self.b = [], []
        for conv, cin in convs:
            wt = conv.weight.detach().float()                      # [128][ci][3][3]
            wp = torch.zeros(128, cin, 3, 3)
            wp[:, : wt.shape[1]] = wt
            self.w.append(wp.permute(2, 3, 0, 1).reshape(9, 128, cin).contiguous().to(self.dev, torch.float16))
            self.b.append(conv.bias.detach().float().contiguous().to(self.dev))
        # the streamed-weight kernel's operand order (zc_net_conv3x3_pack_async), packed once
        from . import _native
        self.wp = []
        for wt in self.w:
            wp = torch.empty_like(wt)
            _native.check(_native.lib().zc_net_conv3x3_pack_async(wt.shape[2], wt.data_ptr(), wp.data_ptr(),
                                                                  ctypes_stream(self.dev)))
            self.wp.append(wp)
        # the same packed weights back to back and the biases [nconv][128], for the fused tower
        self.wall = torch.cat([w.reshape(-1) for w in self.wp]).contiguous()
        self.ball = torch.stack(self.b).contiguous()
        torch.cuda.current_stream(self.dev).synchronize()
        self.fcw = f.fc.weight.detach().float().reshape(-1).contiguous().to(self.dev)
        self.fcb = float(f.fc.bias.detach().float().item())
        self._bufs = {}

    def replica(self) -> "MfmaValueNetwork":
        """The same network (weights shared) with buffers of its own: a second stream can
        evaluate it concurrently (valued.ChessPuctSearch's split search)."""
        r = copy.copy(self)
        r._bufs = {}
        return r

    def _buffers(self, n, hw):
        import torch
        key = (n, hw)
        if key not in self._bufs:
            mk = lambda c: torch.empty((n, hw, c), dtype=torch.float16, device=self.dev)  # noqa: E731
            self._bufs[key] = (mk(self.cpad), mk(128), mk(128), mk(128),
                               torch.empty(n, dtype=torch.float64, device=self.dev))
        return self._bufs[key]

    def tower(self, planes, fused: bool = True, head: bool = False, activation: bool = True):
        """Stem + residual blocks: the final activation, NHWC fp16 [n, h*w, 128].  fused: one
        launch for the whole tower (zc_net_tower_async); otherwise one launch per layer
        (zc_net_conv3x3_packed_async) — bit-identical.  head (fused only): the value head runs
        in the same launch into the returned fp64 values; activation=False skips writing the
        activation (a value-only network needs none)."""
        import torch
        from . import _native
        L = _native.lib()
        n, c, h, w = planes.shape
        if c != self.in_planes or planes.dtype != torch.float16:
            raise ValueError("planes must be fp16 [n, in_planes, h, w]")
        planes = planes.contiguous()
        hw = h * w
        x0, a, t, b, vals = self._buffers(n, hw)
        s = ctypes_stream(self.dev)
        _native.check(L.zc_net_planes_to_nhwc_async(n, c, hw, self.cpad, planes.data_ptr(), x0.data_ptr(), s))
        if fused:
            _native.check(L.zc_net_tower_async(n, h, w, self.cpad, len(self.wp), x0.data_ptr(), self.wall.data_ptr(),
                                               self.ball.data_ptr(), a.data_ptr() if activation or not head else None,
                                               self.fcw.data_ptr() if head else None, self.fcb,
                                               vals.data_ptr() if head else None, s))
            return a, vals
        if head:
            raise ValueError("head=True needs the fused tower")

        def conv(i, src, dst, res):
            _native.check(L.zc_net_conv3x3_packed_async(n, h, w, src.shape[2], src.data_ptr(), self.wp[i].data_ptr(),
                                                        self.b[i].data_ptr(), res.data_ptr() if res is not None else None,
                                                        dst.data_ptr(), 1, s))
        conv(0, x0, a, None)
        for k in range((len(self.w) - 1) // 2):
            conv(1 + 2 * k, a, t, None)
            conv(2 + 2 * k, t, b, a)
            a, b = b, a
        return a, vals

    def tower_policy(self, planes, pw, pb, pout, relu: bool = True):
        """The tower, the value head and a policy 1x1 conv 128 -> P (P = 32 or 64; pw:
        pack_policy_1x1's fragments, pb fp32 [P]) in ONE launch (zc_net_tower_policy_ex_async):
        fp64 values [n]; pout [n, h*w, P] fp16 receives conv1x1 + pb, ReLU'd when `relu`.  No
        tower activation is written."""
        import torch
        from . import _native
        if planes.dim() == 3:   # already the tower's input layout, [n, h*w, cpad] fp16 (8x8 boards)
            n, hw, cp = planes.shape
            h = w = 8
            if hw != 64 or cp != self.cpad or planes.dtype != torch.float16 or not planes.is_contiguous():
                raise ValueError(f"NHWC planes must be contiguous fp16 [n, 64, {self.cpad}]")
        else:
            n, c, h, w = planes.shape
            if c != self.in_planes or planes.dtype != torch.float16:
                raise ValueError("planes must be fp16 [n, in_planes, h, w]")
        P = pout.shape[-1] if pout.dim() == 3 else 0
        if P not in (32, 64) or pout.shape != (n, h * w, P) or pout.dtype != torch.float16 or not pout.is_contiguous():
            raise ValueError("pout must be contiguous fp16 [n, h*w, 32 or 64]")
        x0, _, _, _, vals = self._buffers(n, h * w)
        s = ctypes_stream(self.dev)
        L = _native.lib()
        if planes.dim() == 3:
            x0 = planes
        else:
            planes = planes.contiguous()
            _native.check(L.zc_net_planes_to_nhwc_async(n, c, h * w, self.cpad, planes.data_ptr(), x0.data_ptr(), s))
        _native.check(L.zc_net_tower_policy_ex_async(n, h, w, self.cpad, len(self.wp), x0.data_ptr(),
                                                     self.wall.data_ptr(), self.ball.data_ptr(), self.fcw.data_ptr(),
                                                     self.fcb, vals.data_ptr(), pw.data_ptr(), pb.data_ptr(), P,
                                                     1 if relu else 0, pout.data_ptr(), s))
        return vals

    def __call__(self, planes, fused: bool = True):
        """fp64 values [n]: the tower and the value head in one launch (fused), or the layered
        tower + zc_net_value_head_async — bit-identical."""
        from . import _native
        if fused:
            return self.tower(planes, head=True, activation=False)[1]
        a, vals = self.tower(planes, fused=False)
        n, hw = a.shape[0], a.shape[1]
        _native.check(_native.lib().zc_net_value_head_async(n, hw, a.data_ptr(), self.fcw.data_ptr(), self.fcb,
                                                            vals.data_ptr(), ctypes_stream(self.dev)))
        return vals


def ctypes_stream(dev):
    import ctypes
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream or None)


def pack_policy_1x1(weight):
    """A [P, 128] (out, in) 1x1 conv weight, P = 32 or 64, as the tower kernel's
    v_mfma_f32_32x32x16_f16 A fragments, fp16 [P / 32 blocks][8 k-steps][64 lanes][8]: lane l of
    k-step kc of block mb holds weight[32 mb + l % 32, 16 kc + 8 (l // 32) + e]
    (csrc/net_conv.hip TowerPolicy)."""
    co, ci = weight.shape
    if co not in (32, 64) or ci != 128:
        raise ValueError("the fused policy conv is 128 -> 32 or 64 channels")
    mb = co // 32
    return weight.reshape(mb, 32, 8, 2, 8).permute(0, 2, 3, 1, 4).reshape(mb, 8, 64, 8).contiguous()


class PolicyValueNetwork(nn.Module):
    """The PUCT search's network (no reference counterpart): the
    ValueNetwork tower and value head plus a policy head — conv1x1 to `policy_planes`, BN,
    ReLU, Linear to one logit per (from, to) square pair (index from*64 + to; the reference's
    rules promote to a queen only, so from/to identifies a move)."""

    def __init__(self, channels: int = 128, blocks: int = 8, in_planes: int = 17, board=(8, 8),
                 policy_planes: int = 32, n_logits: int = 4096, head: str = "linear"):
        super().__init__()
        base = ValueNetwork(channels, blocks, in_planes)
        self.stem, self.res, self.head = base.stem, base.res, base.head
        h, w = board
        self.head_kind = head
        if head == "conv":
            # AlphaZero's convolutional policy head: logit(from, to) = channel `to` of a 1x1 conv
            # at pixel `from` — one logit per (from, to) square pair, index from*64 + to, with no
            # fully connected layer (on the GPU it is an MFMA epilogue of the tower: no GEMM)
            if h * w * h * w != n_logits:
                raise ValueError("the convolutional head needs n_logits = (h*w)**2 (one per square pair)")
            self.policy = nn.Sequential(nn.Conv2d(channels, h * w, 1, bias=False), nn.BatchNorm2d(h * w))
        elif head == "linear":
            self.policy = nn.Sequential(
                nn.Conv2d(channels, policy_planes, 1, bias=False),
                nn.BatchNorm2d(policy_planes),
                nn.ReLU(inplace=True),
                nn.Flatten(),
                nn.Linear(policy_planes * h * w, n_logits),
            )
        else:
            raise ValueError("head must be 'linear' or 'conv'")

    def value_network(self) -> ValueNetwork:
        v = ValueNetwork(self.stem[0].out_channels, len(self.res), self.stem[0].in_channels)
        v.stem, v.res, v.head = self.stem, self.res, self.head
        return v

    def policy_logits(self, t):
        if self.head_kind == "conv":   # [n, to, h, w] -> [n, from, to] -> [n, from*64 + to]
            return self.policy(t).flatten(2).transpose(1, 2).reshape(t.shape[0], -1)
        return self.policy(t)

    def forward(self, x):
        t = self.res(self.stem(x))
        return self.head(t), self.policy_logits(t)


class MfmaPolicyValueNetwork:
    """PolicyValueNetwork for inference, ONE kernel launch up to the policy logits' GEMM: the
    tower, the value head and the policy head's 1x1 conv (BN folded, ReLU) run in the fused
    tower kernel (zc_net_tower_policy_async; the conv as an MFMA epilogue on the on-chip
    activation, so the 128-channel activation never reaches HBM); the flatten + Linear to
    the 4096 logits is one fp16 GEMM on PyTorch-ROCm over its [n, h*w*32] output.  Returns
    (fp64 values [n], fp16 logits [n, 4096]).  fused=False: the tower's activation written
    out and the 1x1 conv as a GEMM (the pre-round-4 path, kept for the A/B).

    With the convolutional head (PolicyValueNetwork(head="conv"), round 5) the whole network
    is ONE launch: the 1x1 conv 128 -> 64 epilogue (BN folded, no ReLU) writes [n, 64 from,
    64 to] fp16 = the logits in from*64 + to order, and there is no GEMM."""

    def __init__(self, net: PolicyValueNetwork, device="cuda"):
        import torch
        self.tower = MfmaValueNetwork(net.value_network(), device)
        self.conv_head = getattr(net, "head_kind", "linear") == "conv"
        if self.conv_head:
            folded = _fold(net.policy[0], net.policy[1])
            wf = folded.weight.detach().float().reshape(folded.out_channels, -1)   # [h*w, C]
            if wf.shape != (64, 128):
                raise ValueError("the fused convolutional head is 128 -> 64 channels (an 8x8 board)")
            self.fused = True
            self.pw = pack_policy_1x1(wf).to(device, torch.float16)
            self.pb = folded.bias.detach().float().contiguous().to(device)
            self._pout = {}
            return
        conv, bn, lin = net.policy[0], net.policy[1], net.policy[4]
        folded = _fold(conv, bn)
        P = conv.out_channels
        wf = folded.weight.detach().float().reshape(P, -1)                      # [P, C]
        self.w1 = wf.t().contiguous().to(device, torch.float16)  # [C, P]
        self.b1 = folded.bias.detach().float().to(device, torch.float16)
        self.fused = P == 32 and wf.shape[1] == 128
        if self.fused:
            self.pw = pack_policy_1x1(wf).to(device, torch.float16)
            self.pb = folded.bias.detach().float().contiguous().to(device)
        hw = lin.in_features // P
        # torch flattens [P, h, w] channel-major; the NHWC activation is pixel-major
        wl = lin.weight.detach().float().reshape(lin.out_features, P, hw).permute(0, 2, 1).reshape(lin.out_features, -1)
        self.w2 = wl.t().contiguous().to(device, torch.float16)  # [hw*P, n_logits]
        self.b2 = lin.bias.detach().float().to(device, torch.float16)
        self._pout = {}

    def replica(self) -> "MfmaPolicyValueNetwork":
        """Weights shared, buffers (tower activations, policy conv output) of its own."""
        r = copy.copy(self)
        r.tower = self.tower.replica()
        r._pout = {}
        return r

    def __call__(self, planes, fused: bool = True):
        import torch
        if planes.dim() == 3:   # NHWC planes in the tower's input layout (ChessPuctSearch(planes_nhwc=True))
            if not self.conv_head:
                raise ValueError("NHWC planes need the convolutional head")
            n, h, w = planes.shape[0], 8, 8
        else:
            n, _, h, w = planes.shape
        if self.conv_head:   # the logits straight from the tower launch: [n, 64 from, 64 to]
            key = (n, h * w)
            if key not in self._pout:
                self._pout[key] = torch.empty((n, h * w, 64), dtype=torch.float16, device=self.tower.dev)
            p = self._pout[key]
            vals = self.tower.tower_policy(planes, self.pw, self.pb, p, relu=False)
            return vals, p.view(n, h * w * 64)
        if fused and self.fused:
            key = (n, h * w)
            if key not in self._pout:
                self._pout[key] = torch.empty((n, h * w, 32), dtype=torch.float16, device=self.tower.dev)
            p = self._pout[key]
            vals = self.tower.tower_policy(planes, self.pw, self.pb, p)
            return vals, torch.addmm(self.b2, p.view(n, -1), self.w2)
        a, vals = self.tower.tower(planes, head=True)  # the activation and the values, one launch
        hw = a.shape[1]
        p = torch.relu(torch.addmm(self.b1, a.reshape(n * hw, -1), self.w1)).reshape(n, -1)
        logits = torch.addmm(self.b2, p, self.w2)
        return vals, logits
