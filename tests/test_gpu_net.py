"""The value network on this package's MFMA kernels (csrc/net_conv.hip) against the same
folded network in PyTorch fp32 on the GPU (tolerance: fp16 activations and weights,
fp32 accumulation)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _net(in_planes, seed, channels=128, blocks=8):
    from zeroclone_amd.nets import ValueNetwork
    torch.manual_seed(seed)
    net = ValueNetwork(channels, blocks, in_planes=in_planes)
    for m in net.modules():   # non-trivial folded BN
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.1, 0.1)
    return net.eval()


@pytest.mark.parametrize("shape", [(17, 8, 8), (2, 6, 7)])
@pytest.mark.parametrize("n", [1, 7, 301])
def test_mfma_network_matches_torch(shape, n):
    from zeroclone_amd.nets import FoldedValueNetwork, MfmaValueNetwork
    c, h, w = shape
    net = _net(c, seed=n)
    ref = FoldedValueNetwork(net).cuda().float().eval()
    x = (torch.rand(n, c, h, w, device="cuda") < 0.3).half()
    with torch.no_grad():
        want = ref(x.float()).reshape(-1).double()
    got = MfmaValueNetwork(net)(x).clone()
    torch.cuda.synchronize()
    assert got.dtype == torch.float64 and got.shape == (n,)
    np.testing.assert_allclose(got.cpu().numpy(), want.cpu().numpy(), rtol=0, atol=2e-2)


@pytest.mark.parametrize("mf", ["32", "16"])
def test_single_conv_layer_exactness(mf, monkeypatch):
    """One conv layer with small-integer data is exact in fp32 accumulation: checks the
    MFMA operand/accumulator layouts, the tap shifts and the board edges bit for bit (the
    packed form in both MFMA forms)."""
    from zeroclone_amd import _native
    monkeypatch.setenv("ZC_TOWER_MF", mf)
    L = _native.lib()
    for (h, w, cin) in [(8, 8, 128), (6, 7, 32), (8, 8, 32), (6, 7, 128)]:
        n = 13
        g = torch.Generator().manual_seed(h * 100 + cin)
        x = torch.randint(-2, 3, (n, h, w, cin), generator=g).half().cuda()
        wt = torch.randint(-2, 3, (128, cin, 3, 3), generator=g).float()
        bias = torch.randint(-3, 4, (128,), generator=g).float().cuda()
        res = torch.randint(-2, 3, (n, h, w, 128), generator=g).half().cuda()
        wk = wt.permute(2, 3, 0, 1).reshape(9, 128, cin).contiguous().half().cuda()
        out = torch.empty((n, h, w, 128), dtype=torch.float16, device="cuda")
        _native.check(L.zc_net_conv3x3_async(n, h, w, cin, x.data_ptr(), wk.data_ptr(), bias.data_ptr(),
                                             res.data_ptr(), out.data_ptr(), 1, None))
        torch.cuda.synchronize()
        ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float().cpu(), wt, bias.cpu(), padding=1)
        ref = torch.relu(ref + res.permute(0, 3, 1, 2).float().cpu()).permute(0, 2, 3, 1)
        assert torch.equal(out.float().cpu(), ref), (h, w, cin)
        # the packed, streamed-weight form on the same layer
        wp = torch.empty_like(wk)
        _native.check(L.zc_net_conv3x3_pack_async(cin, wk.data_ptr(), wp.data_ptr(), None))
        out2 = torch.empty_like(out)
        _native.check(L.zc_net_conv3x3_packed_async(n, h, w, cin, x.data_ptr(), wp.data_ptr(), bias.data_ptr(),
                                                    res.data_ptr(), out2.data_ptr(), 1, None))
        torch.cuda.synchronize()
        assert torch.equal(out2.float().cpu(), ref), ("packed", h, w, cin)


def test_packed_conv_is_bit_identical_to_the_staged_form():
    """Random fp16 data, ragged board counts, with and without residual / ReLU: the packed
    streamed-weight kernel accumulates in the staged kernels' order, so outputs agree bitwise."""
    from zeroclone_amd import _native
    L = _native.lib()
    g = torch.Generator(device="cuda").manual_seed(7)
    for (h, w, cin, n) in [(8, 8, 128, 1001), (6, 7, 128, 777), (8, 8, 32, 3), (6, 7, 32, 130)]:
        x = torch.randn(n, h, w, cin, device="cuda", generator=g).half()
        wk = (torch.randn(9, 128, cin, device="cuda", generator=g) * 0.05).half()
        bias = torch.randn(128, device="cuda", generator=g) * 0.1
        res = torch.randn(n, h, w, 128, device="cuda", generator=g).half()
        wp = torch.empty_like(wk)
        _native.check(L.zc_net_conv3x3_pack_async(cin, wk.data_ptr(), wp.data_ptr(), None))
        for use_res, relu in ((False, 1), (True, 1), (True, 0)):
            a = torch.empty((n, h, w, 128), dtype=torch.float16, device="cuda")
            b = torch.empty_like(a)
            rp = res.data_ptr() if use_res else None
            _native.check(L.zc_net_conv3x3_async(n, h, w, cin, x.data_ptr(), wk.data_ptr(), bias.data_ptr(), rp,
                                                 a.data_ptr(), relu, None))
            _native.check(L.zc_net_conv3x3_packed_async(n, h, w, cin, x.data_ptr(), wp.data_ptr(), bias.data_ptr(), rp,
                                                        b.data_ptr(), relu, None))
            torch.cuda.synchronize()
            assert torch.equal(a.view(torch.int16), b.view(torch.int16)), (h, w, cin, n, use_res, relu)


@pytest.mark.parametrize("mf", ["32", "16"])
@pytest.mark.parametrize("shape", [(17, 8, 8), (2, 6, 7)])
@pytest.mark.parametrize("n", [1, 7, 301, 4099])
def test_fused_tower_is_bit_identical_to_layered(shape, n, mf, monkeypatch):
    """zc_net_tower_async (the whole tower in one launch, activations on chip) against the
    layer-by-layer packed launches: the tower's output activation bit for bit, ragged last
    tiles included — in both MFMA forms (ZC_TOWER_MF selects the form of both launches)."""
    from zeroclone_amd.nets import MfmaValueNetwork
    monkeypatch.setenv("ZC_TOWER_MF", mf)
    c, h, w = shape
    net = MfmaValueNetwork(_net(c, seed=100 + n))
    x = (torch.rand(n, c, h, w, device="cuda") < 0.3).half()
    a, _ = net.tower(x, fused=False)
    want = a.clone()
    a.fill_(0)
    got, _ = net.tower(x, fused=True)
    torch.cuda.synchronize()
    assert got.shape == (n, h * w, 128)
    assert torch.equal(got, want)
    assert want.abs().sum().item() > 0


def _integer_net(c, blocks, seed, density=0.002):
    """A ValueNetwork whose folded convs are sparse small integers and whose BN is the identity
    (eps 0): every activation of the tower is a small integer, so any fp32 summation order gives
    the exact result — the MFMA forms' operand / accumulator layouts, tap shifts, board edges,
    residual adds and ragged tiles are checked bit for bit against float64."""
    from zeroclone_amd.nets import ValueNetwork
    g = torch.Generator().manual_seed(seed)
    net = ValueNetwork(128, blocks, in_planes=c).eval()
    for m in net.modules():
        if isinstance(m, torch.nn.Conv2d):
            keep = torch.rand(m.weight.shape, generator=g) < (density if m.in_channels == 128 else 0.02)
            m.weight.data = torch.randint(-2, 3, m.weight.shape, generator=g).float() * keep
        elif isinstance(m, torch.nn.BatchNorm2d):
            m.eps = 0.0
            m.running_mean.zero_()
            m.running_var.fill_(1.0)
            m.weight.data.fill_(1.0)
            m.bias.data = torch.randint(-1, 3, m.bias.shape, generator=g).float()
    return net


@pytest.mark.parametrize("mf", ["32", "16", "16e"])
@pytest.mark.parametrize("shape", [(17, 8, 8), (2, 6, 7)])
def test_tower_forms_exact_on_integers(mf, shape, monkeypatch):
    """Both MFMA forms of the fused tower (ZC_TOWER_MF: 32x32x16, 16x16x32; "16e": the
    16x16x32 form with the swap epilogue, ZC_TOWER_EPI=1) on an integer network, 2 residual
    blocks, ragged board counts: equal to float64 exactly."""
    from zeroclone_amd.nets import FoldedValueNetwork, MfmaValueNetwork
    monkeypatch.setenv("ZC_TOWER_MF", mf[:2])
    monkeypatch.setenv("ZC_TOWER_EPI", "1" if mf.endswith("e") else "0")
    c, h, w = shape
    vnet = _integer_net(c, 2, seed=h * 10 + int(mf[:2]))
    net = MfmaValueNetwork(vnet)
    f = FoldedValueNetwork(vnet).double()
    for n in (1, 5, 131):
        x = (torch.rand(n, c, h, w) < 0.3).half()
        got, _ = net.tower(x.cuda(), fused=True)
        torch.cuda.synchronize()
        with torch.no_grad():
            want = f.res(torch.relu(f.stem(x.double()))).permute(0, 2, 3, 1).reshape(n, h * w, 128)
        assert want.abs().max().item() < 2048 and want.abs().sum().item() > 0
        assert torch.equal(got.double().cpu(), want), (mf, shape, n)


def test_fused_tower_rejects_unsupported_shapes():
    from zeroclone_amd import _native
    L = _native.lib()
    buf = torch.zeros(1024, dtype=torch.float16, device="cuda")
    bias = torch.zeros(128, dtype=torch.float32, device="cuda")
    for (h, w, cin0, nconv) in [(5, 5, 32, 17), (8, 8, 128, 17), (8, 8, 32, 16), (8, 8, 32, 0)]:
        rc = L.zc_net_tower_async(1, h, w, cin0, nconv, buf.data_ptr(), buf.data_ptr(), bias.data_ptr(),
                                  buf.data_ptr(), None, 0.0, None, None)
        assert rc != 0, (h, w, cin0, nconv)


@pytest.mark.parametrize("shape", [(17, 8, 8), (2, 6, 7)])
@pytest.mark.parametrize("n", [1, 5, 1003])
def test_fused_value_head_is_bit_identical(shape, n):
    """The value head inside the tower launch (on the on-chip activation) against the layered
    tower + zc_net_value_head_async: the fp64 values bit for bit."""
    from zeroclone_amd.nets import MfmaValueNetwork
    c, h, w = shape
    net = MfmaValueNetwork(_net(c, seed=200 + n))
    x = (torch.rand(n, c, h, w, device="cuda") < 0.3).half()
    want = net(x, fused=False).clone()
    got = net(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    assert want.abs().sum().item() > 0
