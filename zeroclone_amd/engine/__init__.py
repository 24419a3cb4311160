"""The reference's Python surface (engine/: Engine, mcts.get_move, Value, Policy, game
backends), backed by the HIP search in libzeroclone_amd.so."""
from . import mcts  # noqa: F401
from .engine import Engine, History  # noqa: F401
from .policy_functions import Policy  # noqa: F401
from .value_functions import Value  # noqa: F401
