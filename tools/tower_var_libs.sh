#!/bin/bash
# Builds zeroclone_amd/libzc_<name>.so: net_conv.hip with extra defines, linked with the other
# objects of the in-tree build (tower A/B variants):
#   bash tools/tower_var_libs.sh pf2 "-DZC_TOWER_PF2=1" pf2st "-DZC_TOWER_PF2=1 -DZC_TOWER_STAMP=1"
set -e
cd "$(dirname "$0")/.."
objs=$(ls zeroclone_amd/build_obj/*.o | grep -v net_conv.o)
args=("$@")
for ((i = 0; i < ${#args[@]}; i += 2)); do
  n=${args[i]}; f=${args[i+1]}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -mllvm -amdgpu-sched-strategy=iterative-ilp \
    $f -Rpass-analysis=kernel-resource-usage -c zeroclone_amd/csrc/net_conv.hip -o /tmp/nc_$n.o > /tmp/nc_$n.res 2>&1 &
done
wait
for ((i = 0; i < ${#args[@]}; i += 2)); do
  n=${args[i]}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o zeroclone_amd/libzc_$n.so /tmp/nc_$n.o $objs
done
