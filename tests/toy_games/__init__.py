"""Toy game backends for the any-backend search tests: modules with the six
functions of the reference's plugin contract (engine/README.md:17-24), unknown to the
device.  Shared by tests/golden/gen_golden_generic.py (run against the reference's compiled
get_move) and tests/test_gpu_generic.py."""
