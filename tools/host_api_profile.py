"""Where the host API's time goes (GPU box): env.step(state, a) at 4096 envs under cProfile, plus
the same step as bare device launches with one sync each, and the D2H copy of obs | reward | done
alone.   python tools/host_api_profile.py [pipeline_output 0|1]"""
import cProfile
import ctypes as C
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from pupperv3_mjx import MODEL_XML, _lib  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env, make_keys  # noqa: E402

from pupperv3_mjx import environment  # noqa: E402

E, N = 4096, 100
pipe = len(sys.argv) > 1 and sys.argv[1] == "1"
mode = sys.argv[2] if len(sys.argv) > 2 else "fused"
environment.OUTPUTS_BY_KERNEL = mode != "copy"
environment.STEP_WRITES_HOST = mode == "fused"
print("outputs:", mode, "pipeline_output:", pipe)
env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=E, pipeline_output=pipe)
acts = np.random.RandomState(3).uniform(-1, 1, size=(N + 10, E, 12)).astype(np.float32)
st = env.reset(make_keys(0, E))
for i in range(10):
    st = env.step(st, acts[i])
for rep in range(3):
    t = time.perf_counter()
    for i in range(N):
        st = env.step(st, acts[i])
    dt = time.perf_counter() - t
    print(f"env.step: {dt / N * 1e6:.1f} us/step = {E * N / dt / 1e6:.2f} M env-steps/s")
dbuf = _lib.DeviceBuffer(E * 48, env.device)
dbuf.upload(acts[0])
t = time.perf_counter()
for i in range(N):
    env.step_device(dbuf.ptr.value)
    env.synchronize()
dt = time.perf_counter() - t
print(f"step_device + sync: {dt / N * 1e6:.1f} us/step")
t = time.perf_counter()
for i in range(N):
    env.step_device(dbuf.ptr.value)
env.synchronize()
dt = time.perf_counter() - t
print(f"step_device queued: {dt / N * 1e6:.1f} us/step")
pin = _lib.PinnedBlock.take(4 * E * 74, env._pin_pool)
from pupperv3_mjx import _abi  # noqa: E402
t = time.perf_counter()
for i in range(N):
    _lib.check(env._L.pp3_copy_field_to_host_async(env._h, _abi.F_OBS, C.c_void_p(pin.ptr.value), 4 * E * 72))
    env.synchronize()
dt = time.perf_counter() - t
print(f"obs D2H (pinned) + sync: {dt / N * 1e6:.1f} us")
del pin
pr = cProfile.Profile()
pr.enable()
for i in range(N):
    st = env.step(st, acts[i])
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
K = 30
ra = np.random.RandomState(4).uniform(-1, 1, size=(K, E, 12)).astype(np.float32)
for rep in range(3):
    t = time.perf_counter()
    st, tr = env.rollout(st, ra)
    dt = time.perf_counter() - t
    print(f"env.rollout(K={K}): {dt / K * 1e6:.1f} us/step = {E * K / dt / 1e6:.2f} M env-steps/s")
from collections import OrderedDict  # noqa: E402
from types import SimpleNamespace  # noqa: E402

from pupperv3_mjx import export  # noqa: E402
rs = np.random.RandomState(7)
sizes = [env.observation_size, 256, 128, 128, 24]
layers = OrderedDict((f"hidden_{i}", {"kernel": rs.normal(scale=1 / np.sqrt(sizes[i]), size=(sizes[i], sizes[i + 1])),
                                      "bias": np.zeros(sizes[i + 1])}) for i in range(len(sizes) - 1))
pol = export.DevicePolicy(export.convert_params((SimpleNamespace(mean=np.zeros(sizes[0]), std=np.ones(sizes[0])),
                                                 {"params": layers}), "elu", 0.75, 5.0, 0.25, np.zeros(12), np.ones(12),
                                                -np.ones(12), True, 2, 30.0, 30.0), env.device)
for rep in range(3):
    t = time.perf_counter()
    st, tr = env.rollout_policy(st, pol, K)
    dt = time.perf_counter() - t
    print(f"env.rollout_policy(K={K}): {dt / K * 1e6:.1f} us/step = {E * K / dt / 1e6:.2f} M env-steps/s")
