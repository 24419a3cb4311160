"""Value-network checkpoints: the reference's on-disk format loads (weights_only=True).

The reference saves the whole module (scripts/train.py:143, torch.save(model, latest_path))
and loads it after registering its allowlist (models/chess_value/network.py:add_safe_globals,
engine/value_functions.py:101-130).  tests/golden/ref_value_net_c8b1.pth was written that way
by the reference's own class (tests/golden/gen_golden_ckpt.py); its fp32 outputs are in the
JSON next to it.
"""
import os

import numpy as np
import torch

from conftest import GOLDEN, load_golden
from zeroclone_amd import nets
from zeroclone_amd.engine import value_functions as vf


def _inputs(g):
    bits = np.unpackbits(np.frombuffer(bytes.fromhex(g["inputs_packed_hex"]), np.uint8))
    return torch.from_numpy(bits[: int(np.prod(g["shape"]))].astype(np.float32).reshape(g["shape"]))


def test_reference_whole_module_checkpoint_loads_weights_only():
    g = load_golden("ref_value_net_c8b1.json")
    net = vf.load_value_network(os.path.join(GOLDEN, g["file"]), "chess_value").eval()
    assert isinstance(net, nets.ValueNetwork)
    assert net.stem[0].out_channels == g["channels"] and len(net.res) == g["blocks"]
    with torch.no_grad():
        y = net(_inputs(g)).reshape(-1).double().numpy()
    np.testing.assert_allclose(y, g["outputs"], rtol=0, atol=1e-6)


def test_state_dict_and_own_module_checkpoints_load(tmp_path):
    torch.manual_seed(3)
    ref = nets.ValueNetwork(16, 2).eval()
    x = (torch.rand(4, 17, 8, 8) < 0.2).float()
    with torch.no_grad():
        want = ref(x)
    for i, obj in enumerate((ref.state_dict(), ref)):
        p = str(tmp_path / f"m{i}.pth")
        torch.save(obj, p)
        net = vf.load_value_network(p, "chess_value").eval()
        with torch.no_grad():
            assert torch.equal(net(x), want)


def test_missing_checkpoint_is_the_random_init(tmp_path):
    torch.manual_seed(5)
    a = vf.load_value_network(str(tmp_path / "none.pth"), "chess_value")
    torch.manual_seed(5)
    b = nets.ValueNetwork()
    assert all(torch.equal(u, v) for u, v in zip(a.state_dict().values(), b.state_dict().values()))
    assert vf.latest_path("chess_value", {"models_dir": "/x"}) == "/x/chess_value/latest.pth"
