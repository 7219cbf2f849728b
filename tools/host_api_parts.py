"""Where the host API's single-step launch spends its extra time (verdict r04 item 4): N back-to-back
one-step pp3_rollout launches at the bench's 4096 envs, queued without host work in between and timed
wall-clock around a final synchronize, for every combination of
  actions read from a device buffer | from page-locked host memory (zero copy),
  obs / reward / done stored into device buffers | into page-locked host memory (its device mapping),
  the Brax pipeline record written | not.

  python tools/host_api_parts.py [N]
"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from pupperv3_mjx import MODEL_XML, _abi, _lib, sharding  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env  # noqa: E402

E = 4096
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
for pipe in (True, False):
    env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=E, pipeline_output=pipe)
    L, h = env._raw, env._h
    D = env.observation_size
    acts = np.random.RandomState(3).uniform(-1, 1, size=(E, 12)).astype(np.float32)
    a_dev = _lib.DeviceBuffer(acts.nbytes, env.device)
    a_dev.upload(acts)
    a_pin = _lib.PinnedBlock(acts.nbytes)
    np.asarray(a_pin)[:] = acts.ravel()
    o_dev = _lib.DeviceBuffer(4 * E * (D + 2), env.device)
    o_pin = _lib.PinnedBlock(4 * E * (D + 2))
    for a_name, a_ptr in (("actions:device", a_dev.ptr.value), ("actions:host", a_pin.device_ptr())):
        for o_name, o_ptr in (("outputs:device", o_dev.ptr.value), ("outputs:host", o_pin.device_ptr())):
            env.reset(sharding.shard_keys(0, E, 1, 0))

            def launch():
                _lib.check(L.pp3_rollout(h, C.c_void_p(a_ptr), 0, 1, C.c_void_p(o_ptr + 4 * E * D),
                                         C.c_void_p(o_ptr + 4 * E * (D + 1)), C.c_void_p(o_ptr), None))
            for _ in range(20):
                launch()
            _lib.check(L.pp3_synchronize(h))
            t = time.perf_counter()
            for _ in range(N):
                launch()
            _lib.check(L.pp3_synchronize(h))
            dt = (time.perf_counter() - t) / N
            print(f"pipeline={int(pipe)} {a_name:15s} {o_name:15s} {dt * 1e6:7.1f} us/step", flush=True)
    a_dev.free()
    o_dev.free()
    a_pin.free()
    o_pin.free()
    env.close()
