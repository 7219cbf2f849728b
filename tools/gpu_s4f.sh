#!/bin/bash
# Session 4: phase breakdown of the driver's window vs steady state (diagnostic build), and the
# per-launch time over the first 300 steps after reset (regular build)
OUT=gpurun_out/s4f
mkdir -p $OUT
export PP3_REPORT_DIR=$OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread > $OUT/headline_tests.log 2>&1; rc=$?; echo headline_rc=$rc; grep -E "PASS|FAIL|Error" $OUT/headline_tests.log | tail -8
[ $rc -eq 0 ] || exit 1
PP3_DIAG_OUT=$OUT DIAG_WARMUP=5 timeout -k 10 200 python3 tests/diag_phases.py > $OUT/phases_w5.txt 2>&1 || exit 1
PP3_DIAG_OUT=$OUT DIAG_WARMUP=200 timeout -k 10 200 python3 tests/diag_phases.py > $OUT/phases_w200.txt 2>&1 || exit 1
timeout -k 10 200 python3 - > $OUT/launch_curve.txt 2>&1 <<'PY' || exit 1
import ctypes as C, os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "pupperv3-mjx_amd")]
import numpy as np, bench
from pupperv3_mjx import MODEL_XML, _abi, _lib, sharding
from pupperv3_mjx.environment import PupperV3Env
E = 4096
env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=E, device=0, pipeline_output=True)
st = env.reset(sharding.shard_keys(0, E, 1, 0)); rec = st._record.copy()
rec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3] = [0.5, 0.0, 0.0]; env._put(_abi.F_STATE, rec)
T = 300
acts = _lib.DeviceBuffer(T * E * 48, 0)
_lib.check(env._L.pp3_fill_uniform(env._h, acts.ptr, T * E * 12, 1234, 0, -1.0, 1.0, None))
ms = C.c_float(); rows = []
for i in range(T):
    _lib.check(env._L.pp3_set_pipeline_output(env._h, 0))
    _lib.check(env._L.pp3_step_timed(env._h, C.c_void_p(acts.ptr.value + i * E * 48), E * 12, 1, C.byref(ms)))
    t = ms.value
    # contacts of this step's state: re-run is not possible, so read z / contacts from the state record
    s = env._get(_abi.F_STATE)
    rows.append((i, t, float(s[:, 2].mean()), float(s[:, 2].min())))
for i in range(0, T, 10):
    blk = rows[i:i + 10]
    print(f"steps {i:3d}-{i+9:3d}: launch {np.mean([r[1] for r in blk]):.4f} ms  base z mean {np.mean([r[2] for r in blk]):.3f} min {np.min([r[3] for r in blk]):.3f}")
PY
cat $OUT/launch_curve.txt | head -32; head -24 $OUT/phases_w5.txt; head -24 $OUT/phases_w200.txt
