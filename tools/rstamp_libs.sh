#!/bin/bash
# Builds zeroclone_amd/lib_rs{1..6}.so: the library with c4_search.hip compiled under
# -DZC_RSTAMP=k (rollout region k's s_memtime cycles into the stamped build's "sub" phase:
# 1 leaf setup, 2 view, 3 first segment, 4 absorbed fill, 5 win test, 6 block tail), linked
# with the other objects of the in-tree build.  Run tools/rstamp_regions.py on the GPU box.
set -e
cd "$(dirname "$0")/.."
python zeroclone_amd/build.py > /dev/null
objs=$(ls zeroclone_amd/build_obj/*.o | grep -v c4_search.o)
for k in 1 2 3 4 5 6; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -mllvm -amdgpu-sched-strategy=iterative-ilp \
    -DZC_RSTAMP=$k -c zeroclone_amd/csrc/c4_search.hip -o /tmp/c4s_rs$k.o &
done
wait
for k in 1 2 3 4 5 6; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o zeroclone_amd/lib_rs$k.so /tmp/c4s_rs$k.o $objs
done
