"""zeroclone_amd — MI355X-native batched MCTS self-play engine (drop-in for ZeroClone's
engine/mcts + engine/games hot path).

Layers:
  include/zeroclone.h, zeroclone_amd/csrc/   HIP kernels for gfx950 + the C-ABI library
  zeroclone_amd/_native.py                   ctypes binding (no CPU fallback)
  zeroclone_amd/engine/                      the reference's Python surface: Engine,
                                             mcts.get_move, Value, Policy, game backends
"""
__version__ = "0.1.0"
