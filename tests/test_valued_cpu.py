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
