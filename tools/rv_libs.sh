#!/bin/bash
# Builds zeroclone_amd/lib_rv<k>.so for each ZC_RV mask given (c4_search.hip under -DZC_RV=k,
# linked with the other objects of the in-tree build) for tools/ab_search.py A/B runs.  The
# product source carries no ZC_RV variants: while experimenting, guard each candidate with
# `if (ZC_RV & bit)` (default ZC_RV 0 = the current kernel), A/B it, then bake in or drop it
# (DESIGN §4 "late rollout trims" lists what was measured).
set -e
cd "$(dirname "$0")/.."
objs=$(ls zeroclone_amd/build_obj/*.o | grep -v c4_search.o)
for k in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -mllvm -amdgpu-sched-strategy=iterative-ilp \
    -DZC_RV=$k -c zeroclone_amd/csrc/c4_search.hip -o /tmp/c4s_rv$k.o &
done
wait
for k in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o zeroclone_amd/lib_rv$k.so /tmp/c4s_rv$k.o $objs
done
