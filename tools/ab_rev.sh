#!/bin/bash
# build the kernel at git revision REV as ab/NAME.so:  tools/ab_rev.sh REV NAME
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
REV=$1; NAME=${2:-$1}
T=$(mktemp -d)
mkdir -p $T/csrc $T/include
for f in pp3_env.hip pp3_policy.hip pp3_comm.hip pp3_render.hip pp3_device.h pp3_diag.h; do git -C $ROOT show $REV:pupperv3-mjx_amd/csrc/$f > $T/csrc/$f 2>/dev/null || rm -f $T/csrc/$f; done
git -C $ROOT show $REV:include/pupper_hip.h > $T/include/pupper_hip.h
mkdir -p $ROOT/ab
cd $T/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I../include -Wall -Wno-unused-result \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -fgpu-flush-denormals-to-zero -fno-slp-vectorize \
  -o $ROOT/ab/$NAME.so pp3_env.hip pp3_policy.hip pp3_comm.hip $(ls pp3_render.hip 2>/dev/null) -ldl
rm -rf $T
