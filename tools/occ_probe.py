"""Occupancy probe (verdict r05 item 1): how a SIMD's throughput scales with resident waves on the
real step code.  Built with -DPP3_AB_ALIAS=1 -DPP3_AB_WPE=w (pp3_env.hip), both halves of a wave
share one env block in LDS, so a two-env wave needs 9.9 KB and the register budget of w waves per
SIMD sets the occupancy.  That is only correct when a wave's two envs are identical, so every env
pair here gets the same reset key and the same actions (no DR); each wave then runs one env's
physics twice.  Timing only: the product kernel is not built this way.

  PP3_LIB_PATH=ab/alias3.so python tools/occ_probe.py N [N ...]   -> one JSON line per N
Each line: fused K-step rollout (HIP events) after a ~200 ms pre-warm and W warmup steps, the
end-state hash (equal across builds = the same trajectories), and the wave count per SIMD.
"""
import ctypes as C
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]
import bench  # noqa: E402
from pupperv3_mjx import MODEL_XML, _abi, _lib  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env, make_keys  # noqa: E402

K = int(os.environ.get("OCC_STEPS", "20"))
W = int(os.environ.get("OCC_WARMUP", "5"))
REPS = int(os.environ.get("OCC_REPS", "3"))


def probe(E: int) -> dict:
    env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=E, pipeline_output=False)
    L = env._L
    keys = make_keys(0, E // 2)
    st = env.reset(np.repeat(keys, 2, axis=0))  # env 2b+1 = env 2b
    rec = st._record.copy()
    rec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3] = [0.5, 0.0, 0.0]
    env._put(_abi.F_STATE, rec)
    total = W + K
    acts = np.random.RandomState(1234).uniform(-1, 1, size=(total, E // 2, 12)).astype(np.float32)
    acts = np.ascontiguousarray(np.repeat(acts, 2, axis=1))
    buf = _lib.DeviceBuffer(acts.nbytes, env.device)
    buf.upload(acts)
    at = lambda i: buf.ptr.value + i * E * 48  # noqa: E731
    snap_f = [_abi.F_STATE, _abi.F_OBS, _abi.F_REWARD, _abi.F_DONE]
    stream = L.pp3_stream(env._h)
    snaps = {f: _lib.DeviceBuffer(4 * E * env.device_field(f)[1], env.device) for f in snap_f}
    for f, b in snaps.items():
        _lib.check(L.pp3_memcpy_d2d(b.ptr, C.c_void_p(env.device_field(f)[0]), b.nbytes, stream))

    def restore():
        for f, b in snaps.items():
            _lib.check(L.pp3_memcpy_d2d(C.c_void_p(env.device_field(f)[0]), b.ptr, b.nbytes, stream))
    ms = C.c_float()
    times = []
    for _ in range(REPS):
        restore()
        t = time.perf_counter()
        while time.perf_counter() - t < 0.2:  # pre-warm (restored below)
            _lib.check(L.pp3_rollout(env._h, buf.ptr, E * 12, K, None, None, None, None))
            restore()
            env.synchronize()
        _lib.check(L.pp3_rollout(env._h, buf.ptr, E * 12, W, None, None, None, None))
        _lib.check(L.pp3_rollout_timed(env._h, C.c_void_p(at(W)), E * 12, K, None, None, None, C.byref(ms)))
        env.synchronize()
        times.append(ms.value / K)
    rec = env._get(_abi.F_STATE)
    pair_equal = bool(np.array_equal(rec[0::2], rec[1::2]))
    env.close()
    best = min(times)
    return {"envs": E, "waves_per_simd": E / 2 / 1024, "ms_per_step": [round(t, 5) for t in times],
            "env_steps_per_s": E / best * 1e3, "state_sha16": hashlib.sha256(rec.tobytes()).hexdigest()[:16],
            "pairs_equal": pair_equal, "lib": os.path.basename(_lib.LIB_PATH)}


if __name__ == "__main__":
    for n in sys.argv[1:]:
        print(json.dumps(probe(int(n))), flush=True)
