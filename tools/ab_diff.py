"""Run the bench workload for K steps with the library at PP3_LIB_PATH and save the state records
per step (A/B: which fields differ first between two builds)."""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]
import numpy as np
import bench
from pupperv3_mjx import MODEL_XML, _abi, _lib
from pupperv3_mjx.environment import PupperV3Env, make_keys
E, K = 256, int(sys.argv[2]) if len(sys.argv) > 2 else 3
env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=E, pipeline_output=True)
st = env.reset(make_keys(0, E))
rec = st._record.copy(); rec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3] = [0.5, 0, 0]
env._put(_abi.F_STATE, rec)
a = _lib.DeviceBuffer(K * E * 48, 0)
_lib.check(env._L.pp3_fill_uniform(env._h, a.ptr, K * E * 12, 1234, 0, -1.0, 1.0, None))
out = [env._get(_abi.F_STATE)]
pipes = []
FUSED = os.environ.get("AB_DIFF_FUSED") == "1"  # one fused rollout launch per step (the fused kernel)
for i in range(K):
    if FUSED:
        env.rollout_device(a.ptr.value + i * E * 48, E * 12, 2 if i == 0 else 1)  # (nsteps 1 takes the single-step kernel)
    else:
        env.step_device(a.ptr.value + i * E * 48)
    env.synchronize()
    out.append(env._get(_abi.F_STATE)); pipes.append(env._get(_abi.F_PIPELINE))
np.savez(sys.argv[1], states=np.array(out), pipes=np.array(pipes))
