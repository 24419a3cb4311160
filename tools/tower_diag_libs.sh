#!/bin/bash
# Builds zeroclone_amd/libzc_td<k>.so: net_conv.hip under -DZC_TOWER_STAMP=1 -DZC_TOWER_DIAG=k
# (k = 0: the product loop; 1: no weight reloads; 2: no B-operand LDS reads; 3: neither),
# linked with the other objects of the in-tree build, for tools/tower_stamps.py: the MFMA loop's
# cycles per wave (s_memtime, clock-independent) with each operand stream removed.
set -e
cd "$(dirname "$0")/.."
objs=$(ls zeroclone_amd/build_obj/*.o | grep -v net_conv.o)
for k in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -mllvm -amdgpu-sched-strategy=iterative-ilp \
    -DZC_TOWER_STAMP=1 -DZC_TOWER_DIAG=$k -c zeroclone_amd/csrc/net_conv.hip -o /tmp/nc_td$k.o &
done
wait
for k in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o zeroclone_amd/libzc_td$k.so /tmp/nc_td$k.o $objs
done
