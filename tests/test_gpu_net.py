"""The value network on this package's MFMA kernels (csrc/net_conv.hip) against the same
folded network in PyTorch fp32 on the GPU (tolerance: fp16 activations and weights,
fp32 accumulation)."""
import numpy as np
import pytest
import torch


@pytest.fixture
def net_sw():
    """Set the network launches' switches (zc_debug_net_switch) for one test; restored after."""
    from zeroclone_amd import _native
    saved = {}

    def set_(name, value):
        old = _native.net_switch(name, value)
        saved.setdefault(name, old)
    yield set_
    for name, old in saved.items():
        _native.net_switch(name, old)


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


def _features32(ref, x):
    """Pooled tower features of a FoldedValueNetwork (fp32 on the GPU)."""
    with torch.no_grad():
        a = torch.relu(ref.stem(x.contiguous(memory_format=torch.channels_last)))
        return ref.res(a).mean(dim=(2, 3))


@pytest.mark.parametrize("shape", [(17, 8, 8), (2, 6, 7)])
@pytest.mark.parametrize("n", [1, 7, 301])
def test_mfma_network_matches_torch(shape, n):
    """The fp16 MFMA network against the same folded network in fp32 (torch on the GPU), with
    two heads: the network's own (outputs std ~0.01): atol 5e-4; and a wide head along the
    top principal direction of 64 calibration boards' fp32 features (outputs std ~0.65,
    most of tanh's range): atol 6e-3.  The CPU restatement of the fp16 storage points
    (tests/nn_check.py) predicts max errors <= 1.1e-4 / 3.5e-3 on these networks, whose
    non-trivial BN scales the activations' fp16 rounding.  Pearson >= 0.999 (n > 2)."""
    from nn_check import assert_tracks, wide_head
    from zeroclone_amd.nets import FoldedValueNetwork, MfmaValueNetwork
    c, h, w = shape
    net = _net(c, seed=n)
    g = torch.Generator(device="cuda").manual_seed(1000 + n)
    x = (torch.rand(n, c, h, w, device="cuda", generator=g) < 0.3).half()
    cal = (torch.rand(64, c, h, w, device="cuda", generator=g) < 0.3).float()
    for head, atol in (("own", 5e-4), ("wide", 6e-3)):
        if head == "wide":
            wv, bv = wide_head(_features32(FoldedValueNetwork(net).cuda().float().eval(), cal).cpu())
            with torch.no_grad():
                net.head[2].weight.copy_(wv.reshape(1, -1))
                net.head[2].bias.fill_(bv)
        ref = FoldedValueNetwork(net).cuda().float().eval()
        with torch.no_grad():
            want = ref(x.float()).reshape(-1).double()
        got = MfmaValueNetwork(net)(x).clone()
        torch.cuda.synchronize()
        assert got.dtype == torch.float64 and got.shape == (n,)
        assert_tracks(got.cpu().numpy(), want.cpu().numpy(), atol, min_r=0.999, what=f"{head} head {shape} n={n}")
        if head == "wide" and n > 2:
            assert want.std().item() > 0.3


@pytest.mark.parametrize("mf", ["32", "16"])
def test_single_conv_layer_exactness(mf, net_sw):
    """One conv layer with small-integer data is exact in fp32 accumulation: checks the
    MFMA operand/accumulator layouts, the tap shifts and the board edges bit for bit (the
    packed form in both MFMA forms)."""
    from zeroclone_amd import _native
    net_sw("tower_mf", int(mf))
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


@pytest.mark.parametrize("mf", ["32", "16", "default"])
@pytest.mark.parametrize("shape", [(17, 8, 8), (2, 6, 7)])
@pytest.mark.parametrize("n", [1, 7, 301, 4099])
def test_fused_tower_is_bit_identical_to_layered(shape, n, mf, net_sw):
    """zc_net_tower_async (the whole tower in one launch, activations on chip) against the
    layer-by-layer packed launches: the tower's output activation bit for bit, ragged last
    tiles included — in both MFMA forms (the "tower_mf" switch selects the form of both launches), and
    in the default pairing ("tower_mf" 0: the fused tower on 16x16x32, the layered
    launches on 32x32x16)."""
    from zeroclone_amd.nets import MfmaValueNetwork
    if mf == "default":
        net_sw("tower_mf", 0)
    else:
        net_sw("tower_mf", int(mf))
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
def test_tower_forms_exact_on_integers(mf, shape, net_sw):
    """Both MFMA forms of the fused tower ("tower_mf": 32x32x16, 16x16x32; "16e": the
    16x16x32 form with the swap epilogue, "tower_epi" 1) on an integer network, 2 residual
    blocks, ragged board counts: equal to float64 exactly."""
    from zeroclone_amd.nets import FoldedValueNetwork, MfmaValueNetwork
    net_sw("tower_mf", int(mf[:2]))
    net_sw("tower_epi", 1 if mf.endswith("e") else 0)
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


def _integer_head(vnet, hw, seed):
    """Integer value head on an integer tower: Linear weights k_c * hw / 64 (k_c in {-1, 0, 1},
    sparse) and a bias that is a multiple of 1/64.  The kernels' head sums each lane's
    channels (exact integers times hw / 64), divides by hw (exact: the quotient k / 64 is
    representable) and adds the lanes (multiples of 1/64), so the pre-tanh sum is exact:
    sum_c k_c * S_c / 64 + bias, S_c the channel's pixel sum."""
    g = torch.Generator().manual_seed(seed)
    k = torch.randint(-1, 2, (128,), generator=g).float() * (torch.rand(128, generator=g) < 0.25)
    with torch.no_grad():
        vnet.head[2].weight.copy_((k * hw / 64.0).reshape(1, -1))
        vnet.head[2].bias.fill_(-3.0 + 5.0 / 64.0)
    return vnet


@pytest.mark.parametrize("mf", ["32", "16"])
@pytest.mark.parametrize("shape", [(17, 8, 8), (2, 6, 7)])
def test_value_head_exact_on_integers(mf, shape, net_sw):
    """The value head (avg-pool, Linear(128, 1), + bias) on an integer network: its pre-tanh
    sum ("head_raw" 1) equals float64 exactly, in the fused tower launch and in the layered
    value_head_kernel, ragged tiles included (on 6x7 too: each lane's sum is a multiple of
    42/64, so the kernel's correctly rounded division by 42 is exact).  With the
    tanh (the product path) the values equal float64 tanh of that sum within tanhf's precision.
    A head without its bias or without its Linear would fail every one of these."""
    from zeroclone_amd.nets import FoldedValueNetwork, MfmaValueNetwork
    net_sw("tower_mf", int(mf))
    c, h, w = shape
    vnet = _integer_head(_integer_net(c, 2, seed=h * 7 + int(mf)), h * w, seed=int(mf) + h)
    xs = [(torch.rand(n, c, h, w) < 0.3).half() for n in (1, 5, 131)]

    def pre_tanh(x):
        # exact in float64: the channel sums S_c (integers), k_c = fcw_c * 64 / hw (integers),
        # sum_c S_c k_c / 64 + bias (a mean taken first would round S_c / 42)
        f = FoldedValueNetwork(vnet).double()
        with torch.no_grad():
            act = f.res(torch.relu(f.stem(x.double())))
            k = torch.round(f.fc.weight.detach().double().reshape(-1) * 64.0 / (h * w))
            return (act.sum(dim=(2, 3)) @ k) / 64.0 + f.fc.bias.detach().double()
    with torch.no_grad():   # centre the sums on tanh's active range (a multiple of 1/64)
        vnet.head[2].bias.fill_(0.0)
        vnet.head[2].bias.fill_(-float(torch.round(pre_tanh(xs[-1]).median() * 64)) / 64)
    net = MfmaValueNetwork(vnet)
    for x in xs:
        n = x.shape[0]
        pre = pre_tanh(x)
        assert pre.abs().max().item() < 2 ** 16
        if n > 1:
            assert pre.std().item() > 0
        net_sw("head_raw", 1)
        for fused in (True, False):
            got = net(x.cuda(), fused=fused).clone()
            torch.cuda.synchronize()
            assert torch.equal(got.cpu(), pre), (mf, shape, n, fused)
        net_sw("head_raw", 0)
        got = net(x.cuda()).clone()
        torch.cuda.synchronize()
        np.testing.assert_allclose(got.cpu().numpy(), np.tanh(pre.numpy()), rtol=0, atol=1e-6)


def _integer_pv_net(c, h, w, nl, seed, head="linear"):
    """PolicyValueNetwork with an integer tower (as _integer_net), an integer 1x1 policy conv,
    identity BN with integer biases and a sparse integer Linear: every policy value is a small
    integer, exact in fp16 and in any fp32 summation order."""
    from zeroclone_amd.nets import PolicyValueNetwork
    g = torch.Generator().manual_seed(seed)
    net = PolicyValueNetwork(in_planes=c, board=(h, w), n_logits=nl, head=head).eval()
    for m in net.modules():
        if isinstance(m, torch.nn.Conv2d):
            dens = 0.002 if m.in_channels == 128 and m.kernel_size == (3, 3) else 0.02
            keep = torch.rand(m.weight.shape, generator=g) < dens
            m.weight.data = torch.randint(-2, 3, m.weight.shape, generator=g).float() * keep
        elif isinstance(m, torch.nn.BatchNorm2d):
            m.eps = 0.0
            m.running_mean.zero_()
            m.running_var.fill_(1.0)
            m.weight.data.fill_(1.0)
            m.bias.data = torch.randint(-1, 3, m.bias.shape, generator=g).float()
        elif isinstance(m, torch.nn.Linear) and m.out_features == nl:
            keep = torch.rand(m.weight.shape, generator=g) < 0.004
            m.weight.data = torch.randint(-1, 2, m.weight.shape, generator=g).float() * keep
            m.bias.data = torch.randint(-4, 5, m.bias.shape, generator=g).float()
    net.res = net.res[:2]
    return net


@pytest.mark.parametrize("shape", [(37, 17, 8, 8, 4096), (53, 2, 6, 7, 7)])
def test_policy_head_exact_on_integers(shape):
    """TowerPolicy (the 1x1 policy conv fused into the tower launch, zc_net_tower_policy_async)
    and the policy Linear on an integer PolicyValueNetwork: the conv's ReLU output and the
    logits equal float64 exactly (2 residual blocks, ragged last tiles)."""
    from zeroclone_amd.nets import MfmaPolicyValueNetwork
    n, c, h, w, nl = shape
    net = _integer_pv_net(c, h, w, nl, seed=n)
    mnet = MfmaPolicyValueNetwork(net)
    assert mnet.fused
    x = (torch.rand(n, c, h, w) < 0.3).half()
    _, logits = mnet(x.cuda())
    pout = mnet._pout[(n, h * w)].double().cpu()
    torch.cuda.synchronize()
    from zeroclone_amd.nets import FoldedValueNetwork
    fv = FoldedValueNetwork(net.value_network()).double()
    conv, bn, lin = net.policy[0], net.policy[1], net.policy[4]
    with torch.no_grad():   # identity BN (eps 0): the folded form is the module's own algebra
        t = fv.res(torch.relu(fv.stem(x.double())))
        p = torch.relu(torch.nn.functional.conv2d(t, conv.weight.double()) + bn.bias.double().reshape(1, -1, 1, 1))
        want_logits = p.flatten(1) @ lin.weight.double().t() + lin.bias.double()
    want_p = p.permute(0, 2, 3, 1).reshape(n, h * w, 32)
    assert want_p.abs().max().item() < 2048 and want_p.abs().sum().item() > 0
    assert want_logits.abs().max().item() < 2048 and (want_logits != lin.bias.double()).any()
    assert torch.equal(pout, want_p)
    assert torch.equal(logits.double().cpu(), want_logits)


def test_convolutional_policy_head_exact_on_integers():
    """PolicyValueNetwork(head="conv") on an integer network: the logits the tower launch
    writes (1x1 conv 128 -> 64 + BN bias, no ReLU; pixel = from, channel = to) equal float64
    exactly, in from*64 + to order (ragged last tile)."""
    from zeroclone_amd.nets import FoldedValueNetwork, MfmaPolicyValueNetwork
    n = 37
    net = _integer_pv_net(17, 8, 8, 4096, seed=91, head="conv")
    mnet = MfmaPolicyValueNetwork(net)
    x = (torch.rand(n, 17, 8, 8) < 0.3).half()
    _, logits = mnet(x.cuda())
    logits = logits.double().cpu()
    fv = FoldedValueNetwork(net.value_network()).double()
    conv, bn = net.policy[0], net.policy[1]
    with torch.no_grad():
        t = fv.res(torch.relu(fv.stem(x.double())))
        p = torch.nn.functional.conv2d(t, conv.weight.double()) + bn.bias.double().reshape(1, -1, 1, 1)
        want = p.flatten(2).transpose(1, 2).reshape(n, 4096)       # [n, from, to]
        assert torch.equal(want.float().double(), want)
    assert want.abs().max().item() < 2048 and (want < 0).any() and (want > 0).any()
    assert torch.equal(logits, want)
