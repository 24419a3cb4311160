# A/B of conv library variants (ZC_LIB copies), same box: bash tools/abconv_libs.sh lib1.so lib2.so ...
set -e
mkdir -p gpurun_out
for l in "$@"; do
  ZC_LIB=$PWD/zeroclone_amd/$l timeout -k 10 300 python tools/ab_conv.py stream3 > gpurun_out/abc_$l.log 2>&1
done
