"""Leaf evaluators with the reference's interface (engine/value_functions.py:8-130).

Inside `mcts.get_move` / `Engine` the value object selects the device path (_search.py):
`random_rollout` (Connect4) and `crude_chess_score` (chess) are evaluated inside the search
kernels; the network modes hand the device-built leaf planes to the model between the
select and backup kernels.  Called directly, `Value` behaves as the reference's:

* `random_rollout`: `batch(states, backend=)` rolls the states out IN ORDER on the GPU on a
  CPython-compatible MT19937 stream taken from (and returned to) Python's global `random`
  — the numbers the reference's `[self(s) for s in states]` would draw (:20-22, 35-45).
* `crude_chess_score` (:48-55): 1000 if check_win(state), else (turn*-2+1) * material.
* `network_latest` / `network_at_path` (:61-130): the reference's ValueNetwork template
  (zeroclone_amd.nets) for `model_type` (chess_value: 17 planes; connect4: 2 planes), in fp16
  on the GPU; weights from `path` / <models_dir>/<model_type>/latest.pth when present (the
  reference's whole-module pickle or a state_dict, loaded with weights_only=True through the
  reference's allowlist mapped onto this package's classes), else the random init.
"""
from __future__ import annotations

import os

from . import _device

SUPPORTED = ("random_rollout", "crude_chess_score", "network_latest", "network_at_path")
_PIECES = {"P": 1, "N": 3, "B": 3, "R": 5, "Q": 9, "p": -1, "n": -3, "b": -3, "r": -5, "q": -9}
MODEL_PLANES = {"chess_value": 17, "connect4_value": 2}


class Value:
    def __init__(self, name, **kwargs):
        self.name = name
        self.init_args = kwargs
        self.zc_model = None
        # as the reference (value_functions.py:9-14): an unknown name constructs, and fails
        # with AttributeError when called (:17-18)
        if name in SUPPORTED and name.startswith("network"):
            self._init_network()

    def __call__(self, state, **kwargs):
        return self.batch([state], **kwargs)[0]

    def batch(self, states, **kwargs):
        backend = (self.init_args | kwargs).get("backend")
        return getattr(self, self.name)(list(states), backend)

    # ---------------------------------------------------------------- random_rollout
    def random_rollout(self, states, backend):
        if getattr(backend, "ZC_GAME", None) != "connect4" and not _looks_like_c4(backend, states):
            from ._search import game_of
            game = game_of(backend, states[0]) if states else "generic"
            if game == "chess":
                return _chess_rollouts(states)
            return [_backend_rollout(s, backend) for s in states]
        from .games.connect4 import c4_backend as c4
        if not states:
            return []
        ge = _device.value_engine()
        with ge.lock:
            eng = ge.ensure(1, 1, 1)
            mt, idx, ver, gauss = _device.python_random_state()
            eng.set_rng_state(0, mt, idx)
            vals, _ = eng.c4_rollouts(_device.c4_roots(states, c4), game=0)
            mt, idx = eng.get_rng_state(0)
            _device.set_python_random_state(mt, idx, ver, gauss)
        return [int(v) for v in vals]

    # ---------------------------------------------------------------- crude_chess_score
    def crude_chess_score(self, states, backend):
        out = []
        for s in states:
            if backend.check_win(s):
                out.append(1000)
                continue
            factor = s.turn * -2 + 1
            out.append(factor * sum(_PIECES.get(chr(p), 0) for p in s.board))
        return out

    # ---------------------------------------------------------------- network modes
    def _init_network(self):
        import torch
        from ..nets import for_inference
        mt = self.init_args.get("model_type", "chess_value")
        path = self.init_args.get("path") if self.name == "network_at_path" else latest_path(mt, self.init_args)
        net = load_value_network(path, mt)
        self.zc_model = for_inference(net.eval(), "cuda", torch.float16)
        self.batch_size = self.init_args.get("batch_size", 1)

    def _network(self, states, backend):
        import numpy as np
        import torch
        if not states:
            return []
        x = torch.from_numpy(np.stack([backend.state_to_tensor(s) for s in states]).astype(np.float32))
        with torch.no_grad():
            return [float(v) for v in self.zc_model(x.cuda().half()).float().reshape(-1).cpu()]

    network_latest = _network
    network_at_path = _network


def models_dir(init_args=None) -> str:
    """Where `network_latest` looks for <model_type>/latest.pth.  The reference resolves it
    next to its models package (models/core.py:10-13); here: the `models_dir` value arg, else
    $ZC_MODELS_DIR, else zeroclone_amd/models (the package's own models directory)."""
    d = (init_args or {}).get("models_dir") or os.environ.get("ZC_MODELS_DIR")
    return d or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "models")


def latest_path(model_type: str, init_args=None) -> str:
    return os.path.join(models_dir(init_args), model_type, "latest.pth")


def _reference_safe_globals():
    """The allowlist the reference registers before loading (models/chess_value/network.py:
    add_safe_globals), with the reference's own classes mapped by qualified name to this
    package's mirror classes: a checkpoint written by scripts/train.py:143 (torch.save of the
    whole module) then loads with weights_only=True — nothing in the file is executed."""
    import torch.nn as nn
    from .. import nets
    ref = "models.{}.network"
    out = [nn.Conv2d, nn.BatchNorm2d, nn.ReLU, nn.AdaptiveAvgPool2d, nn.Linear, nn.Tanh, nn.Sequential, nn.Flatten,
           nets.ValueNetwork, nets.ResidualBlock]
    for mt in MODEL_PLANES:
        out += [(nets.ValueNetwork, ref.format(mt) + ".ValueNetwork"),
                (nets.ResidualBlock, ref.format(mt) + ".ResidualBlock")]
    return out


def load_value_network(path, model_type: str = "chess_value"):
    """value_functions.py:init_network_latest / init_network_at_path (:101-130): the model at
    `path` when it exists, else a random-init ValueNetwork.  Accepts both a whole pickled
    module (the reference's format) and a plain state_dict; always weights_only=True.
    Returns an fp32 CPU `nets.ValueNetwork` whose width and depth are the checkpoint's."""
    import torch
    from ..nets import ValueNetwork
    planes = MODEL_PLANES.get(model_type, 17)
    if not path or not os.path.exists(path):
        return ValueNetwork(in_planes=planes)
    with torch.serialization.safe_globals(_reference_safe_globals()):
        obj = torch.load(path, map_location="cpu", weights_only=True)
    sd = obj.state_dict() if isinstance(obj, torch.nn.Module) else obj
    if not isinstance(sd, dict) or "stem.0.weight" not in sd:
        raise ValueError(f"{path}: not a ValueNetwork checkpoint (no stem.0.weight)")
    channels, in_planes = int(sd["stem.0.weight"].shape[0]), int(sd["stem.0.weight"].shape[1])
    blocks = len({k.split(".")[1] for k in sd if k.startswith("res.")})
    net = ValueNetwork(channels, blocks, in_planes=in_planes)
    net.load_state_dict(sd)
    return net


def _backend_rollout(state, backend):
    """value_functions.py:35-45 for a backend the device does not know: its
    rules are the plugin's Python callables, so the playout calls them where the reference
    does, drawing from Python's global `random`."""
    import random
    initial = state.turn
    while not backend.check_win(state) and not backend.check_draw(state):
        state = backend.play_move(state, random.choice(list(backend.get_legal_moves(state))))
    if backend.check_win(state):
        return -1 if state.turn == initial else 1
    return 0


def _chess_rollouts(states):
    """value_functions.py:35-45 on the chess backend, for a direct Value.batch call: the
    states are rolled out IN ORDER on the GPU (zc_chess_rollouts_async: the chess rules, both
    sides' histories for the repetition draw) on a CPython-compatible MT19937 stream taken from
    (and returned to) Python's global `random`."""
    import numpy as np
    import torch
    from .games.chess import chess_backend as cb
    from ._search import chess_roots
    if not states:
        return []
    hist, hlen = cb.pack_histories(states)
    ge = _device.value_engine()
    with ge.lock:
        eng = ge.ensure(1, 1, 1)
        dev = torch.device("cuda", eng.device)
        rows = torch.from_numpy(chess_roots(states).view(np.uint8).reshape(len(states), 72).copy()).to(dev)
        h, n = torch.from_numpy(hist).to(dev), torch.from_numpy(hlen).to(dev)
        vals = torch.zeros(len(states), dtype=torch.float64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        mt, idx, ver, gauss = _device.python_random_state()
        eng.set_rng_state(0, mt, idx)
        s = torch.cuda.current_stream(dev)
        eng.chess_rollouts_async(0, len(states), rows.data_ptr(), h.data_ptr(), n.data_ptr(), hist.shape[2],
                                 vals.data_ptr(), status.data_ptr(), s.cuda_stream)
        s.synchronize()
        if int(status.item()):
            raise RuntimeError(f"chess rollout exceeded {_native_roll_cap()} moves per side in its history")
        mt, idx = eng.get_rng_state(0)
        _device.set_python_random_state(mt, idx, ver, gauss)
        return [int(v) for v in vals.cpu().tolist()]


def _native_roll_cap():
    from .. import _native
    return _native.CHESS_ROLL_CAP


def _looks_like_c4(backend, states):
    from .games.connect4 import c4_backend as c4
    return getattr(backend, "__name__", "").endswith("c4_backend") and all(c4.is_state(s) for s in states)
