#!/bin/bash
# build the committed (HEAD) kernel as ab/base.so for A/B against the working tree
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
T=$(mktemp -d)
mkdir -p $T/csrc $T/include
for f in pp3_env.hip pp3_policy.hip pp3_comm.hip pp3_render.hip pp3_device.h pp3_diag.h pp3_mlp.h; do git -C $ROOT show HEAD:pupperv3-mjx_amd/csrc/$f > $T/csrc/$f 2>/dev/null || rm -f $T/csrc/$f; done
for f in pupper_hip.h pupper_hip_diag.h; do git -C $ROOT show HEAD:include/$f > $T/include/$f; done
mkdir -p $ROOT/ab
cd $T/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I../include -Wall -Wno-unused-result \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -fgpu-flush-denormals-to-zero -fno-slp-vectorize \
  -o $ROOT/ab/${1:-base}.so pp3_env.hip pp3_policy.hip pp3_comm.hip $(ls pp3_render.hip 2>/dev/null) -ldl
rm -rf $T
