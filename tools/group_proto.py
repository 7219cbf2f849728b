"""Prototype: G independent env groups (own pp3 handle + stream each) vs one batch; same envs, same actions."""
import ctypes as C, os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]
import numpy as np
import bench
from pupperv3_mjx import MODEL_XML, _abi, _lib, sharding
from pupperv3_mjx.environment import PupperV3Env

def run(G, E=4096, warm=5, K=20, reps=3):
    envs, acts = [], []
    for g in range(G):
        n = E // G
        env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=n, pipeline_output=False)
        st = env.reset(sharding.shard_keys(0, E, G, g))
        rec = st._record.copy(); rec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3] = [0.5, 0, 0]
        env._put(_abi.F_STATE, rec)
        a = _lib.DeviceBuffer((warm + K * reps) * n * 48, 0)
        _lib.check(env._L.pp3_fill_uniform(env._h, a.ptr, (warm + K * reps) * n * 12, 1234 + g, 0, -1.0, 1.0, None))
        envs.append(env); acts.append(a)
    for e in envs: e.synchronize()
    for i in range(warm):
        for g, e in enumerate(envs): e.step_device(acts[g].ptr.value + i * (E // G) * 48)
    for e in envs: e.synchronize()
    out = []
    for r in range(reps):
        t0 = time.perf_counter()
        for i in range(K):
            for g, e in enumerate(envs): e.step_device(acts[g].ptr.value + (warm + r * K + i) * (E // G) * 48)
        for e in envs: e.synchronize()
        out.append((time.perf_counter() - t0) / K * 1e3)
    for a in acts: a.free()
    for e in envs: e.close()
    return out

if __name__ == "__main__":
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    for G in [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else (1, 2, 4, 8, 16):
        ms = run(G, warm=warm, K=K)
        print(json.dumps({"G": G, "K": K, "warm": warm, "ms_per_step": [round(x, 4) for x in ms],
                          "Msteps": [round(4096 / x / 1e3, 2) for x in ms], "hwq": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)
