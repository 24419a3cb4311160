"""CPU checks for the stepwise (caller-valued) search and the value network:
the oracle's valued get_move against the reference's outputs (tests/golden/
c4_get_move_valued.json, made by driving the reference with c4_values.hash_value), and
zeroclone_amd.nets.ValueNetwork against the reference ValueNetwork's seeded outputs
(tests/golden/value_network.json)."""
import numpy as np
import pytest
import torch

import oracle
from c4_values import bits_from_rows, hash_value


def oracle_value(boards, turns):
    out = []
    for b, t in zip(boards, turns):
        s0, s1 = bits_from_rows(b)
        out.append(hash_value(s0, s1, t))
    return out


def test_oracle_valued_search_matches_reference(golden):
    g = golden("c4_get_move_valued.json")
    assert len(g["cases"]) >= 30
    for case in g["cases"]:
        mt = oracle.MT(case["seed"])
        col, na, order = oracle.get_move_valued(case["board"], case["turn"], mt, case["sims"], case["c"],
                                                case["bs"], oracle_value)
        assert order == case["order"]
        assert na == case["root_na"], case
        assert col == case["move"]
        assert mt.drawn == case["consumed"]
        assert mt.u32() == case["next_word"]


def test_hash_value_has_full_precision():
    vals = [hash_value(i * 977, i * 131, i & 1) for i in range(1, 200)]
    assert len(set(vals)) > 190
    assert all(-1.0 < v < 1.0 for v in vals)


def _inputs(g):
    bits = np.unpackbits(np.frombuffer(bytes.fromhex(g["inputs_packed_hex"]), np.uint8))
    n = int(np.prod(g["shape"]))
    return torch.from_numpy(bits[:n].astype(np.float32).reshape(g["shape"]))


def test_value_network_matches_reference_init_and_forward(golden):
    from zeroclone_amd.nets import ValueNetwork
    g = golden("value_network.json")
    torch.manual_seed(g["seed"])
    net = ValueNetwork().eval()
    assert [[k, list(v.shape)] for k, v in net.state_dict().items()] == g["state_dict"]
    with torch.no_grad():
        y = net(_inputs(g)).reshape(-1).double().numpy()
    np.testing.assert_allclose(y, np.array(g["outputs"]), rtol=0, atol=1e-6)


def test_folded_network_matches_unfolded_fp32():
    from zeroclone_amd.nets import ValueNetwork, for_inference
    torch.manual_seed(0)
    net = ValueNetwork(channels=32, blocks=2, in_planes=2)
    # non-trivial BN statistics
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.1, 0.1)
    net.eval()
    x = (torch.rand(16, 2, 6, 7) < 0.3).float()
    with torch.no_grad():
        ref = net(x)
        got = for_inference(net, "cpu", torch.float32)(x)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


def _seeded_net(g, wide):
    from zeroclone_amd.nets import ValueNetwork
    torch.manual_seed(g["seed"])
    net = ValueNetwork().eval()
    if wide:
        with torch.no_grad():
            net.head[2].weight.copy_(torch.tensor(g["head_weight_wide"]).reshape(1, -1))
            net.head[2].bias.fill_(g["head_bias_wide"])
    return net


def test_wide_head_golden_matches_this_package_in_fp32(golden):
    """The wide head (the pooled features' top principal direction, tests/golden/gen_golden_nn.py)
    loaded into this package's ValueNetwork reproduces the reference's fp32 outputs, and those
    outputs span most of tanh's range (a tolerance of 3e-3 is < 1 % of their spread)."""
    g = golden("value_network.json")
    y = np.array(g["outputs_wide"])
    assert y.std() > 0.5 and y.min() < -0.9 and y.max() > 0.9
    with torch.no_grad():
        got = _seeded_net(g, True)(_inputs(g)).reshape(-1).double().numpy()
    np.testing.assert_allclose(got, y, rtol=0, atol=1e-5)


@pytest.mark.parametrize("wide,atol", [(False, 2e-4), (True, 3e-3)])
def test_fp16_storage_error_fits_the_gpu_tolerance(golden, wide, atol):
    """The GPU test's tolerances are not guesses: the fp16 storage points of the MFMA path
    (fp16 weights, fp16 activations after every layer) restated in float64 stay inside them
    against the reference's fp32 outputs, with a margin; a head missing its bias, or a
    constant head, does not."""
    from nn_check import assert_tracks, fails_tracking, fp16_emulation_features
    from zeroclone_amd.nets import FoldedValueNetwork
    g = golden("value_network.json")
    want = np.array(g["outputs_wide" if wide else "outputs"])
    net = _seeded_net(g, wide)
    f = FoldedValueNetwork(net)
    feat = fp16_emulation_features(f, _inputs(g))
    w = f.fc.weight.detach().double().reshape(-1)
    b = f.fc.bias.detach().double().item()
    emu = torch.tanh(feat @ w + b).numpy()
    err = assert_tracks(emu, want, atol, what="fp16 emulation")
    assert err < atol / 2, err
    assert fails_tracking(torch.tanh(feat @ w).numpy(), want, atol)          # bias dropped
    assert fails_tracking(np.full_like(want, want.mean()), want, atol)       # constant head


def test_convolutional_policy_head_orders_logits_from_to():
    """PolicyValueNetwork(head="conv"): logit index from*64 + to = the 1x1 conv's channel `to`
    at pixel `from` (the order zc_chess_puct_backup reads)."""
    from zeroclone_amd.nets import PolicyValueNetwork
    torch.manual_seed(2)
    net = PolicyValueNetwork(head="conv").eval()
    x = (torch.rand(2, 17, 8, 8) < 0.3).float()
    with torch.no_grad():
        _, lg = net(x)
        t = net.res(net.stem(x))
        p = net.policy(t)   # [n, 64 to, 8, 8]
    for fr in (0, 9, 63):
        for to in (0, 17, 63):
            assert torch.equal(lg[:, fr * 64 + to], p[:, to, fr // 8, fr % 8])
    with pytest.raises(ValueError):
        PolicyValueNetwork(board=(6, 7), n_logits=7, in_planes=2, head="conv")
