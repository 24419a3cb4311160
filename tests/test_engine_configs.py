"""Every shipped YAML builds an Engine and makes a one-simulation search — the reference's
tests/test_engine_configs.py:17-22 (Engine(cfg); legal_moves non-empty; mcts.get_move(state,
values[0], policy, backend, 1, c_puct, 1)), restated over configs/*.yaml."""
import glob
import os
import random

import pytest
import yaml

from conftest import REPO

CONFIGS = sorted(glob.glob(os.path.join(REPO, "configs", "*.yaml")))
REFERENCE_CONFIGS = {"chess_value.yaml", "connect4.yaml", "crude_chess.yaml"}


def test_reference_config_set_is_shipped_with_its_keys():
    assert REFERENCE_CONFIGS <= {os.path.basename(c) for c in CONFIGS}
    for cfg in CONFIGS:
        with open(cfg) as fh:
            c = yaml.safe_load(fh)
        for key in ("game", "backend", "value_function", "threads", "mcts"):
            assert key in c, (cfg, key)
        assert {"simulations", "c_puct"} <= set(c["mcts"]), cfg


@pytest.mark.parametrize("cfg", [c for c in CONFIGS if "network" not in open(c).read()], ids=os.path.basename)
def test_engine_constructs_without_gpu(cfg):
    from zeroclone_amd.engine import Engine
    eng = Engine(cfg)   # chess rules run on the device: legal moves only for Connect4 here
    assert len(eng.states) == eng.config.get("threads", 1)
    if eng.config["game"] == "connect4":
        assert len(eng.legal_moves()) == 7


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", CONFIGS, ids=os.path.basename)
def test_engine_config_basic_move(cfg):
    from zeroclone_amd.engine import Engine, mcts
    eng = Engine(cfg)
    moves = eng.legal_moves()
    assert len(moves) > 0
    random.seed(0)
    mv = mcts.get_move(eng.get_state(), eng.values[0], eng.policy, eng.backend, 1, eng.config["mcts"]["c_puct"], 1)
    assert mv in moves or any(m[0] == mv[0] for m in moves)
