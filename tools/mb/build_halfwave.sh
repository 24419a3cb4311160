#!/bin/bash
# Build the half-wave rollout A/B (tools/mb/halfwave.hip) for gfx950, with the search
# kernel's flags (zeroclone_amd/build.py: FLAGS + c4_search.hip's machine scheduler).
set -e
cd "$(dirname "$0")/../.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
    -mllvm -amdgpu-sched-strategy=iterative-ilp -I include -o tools/mb/halfwave tools/mb/halfwave.hip
