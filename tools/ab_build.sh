#!/bin/bash
# build kernel variants for tools/ab_bench.sh:  tools/ab_build.sh name1 "-DFLAG ..." name2 "..." ...
set -e
cd "$(dirname "$0")/../pupperv3-mjx_amd/csrc"
mkdir -p ../../ab
[ -n "$AB_KEEP" ] || rm -f ../../ab/*.so
while [ $# -gt 0 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I../../include -Wall -Wno-unused-result \
    -fno-hip-fp32-correctly-rounded-divide-sqrt -fgpu-flush-denormals-to-zero -fno-slp-vectorize $flags \
    -o ../../ab/$name.so pp3_env.hip pp3_policy.hip pp3_comm.hip $(ls pp3_render.hip 2>/dev/null) -ldl &
done
wait
ls -la ../../ab
