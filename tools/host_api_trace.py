"""A plain env.step loop for rocprofv3 --kernel-trace --hip-trace --stats (verdict r04 item 4: where
the host API's time per step goes).  4096 envs (bench.py workload), 20 untimed steps, then `N`
timed env.step(state, numpy actions) calls; prints us/step.

  python tools/host_api_trace.py [N] [pipeline_output 0|1] [sync|async|async_zc|defer1|defer|defer_all|defer_read]

Modes: sync = every step synchronises before it returns (the round-4 host API); async = step()
returns at once, obs / reward / done wait for their own launch (environment.ASYNC_STEP); async_zc =
async, and the launch reads the actions straight from the page-locked staging block
(environment.ACTIONS_ZERO_COPY); defer = async_zc with each launch issued at the next call
(environment.DEFER_LAUNCH: no device snapshot of the state the caller has dropped) with one launch
per step (defer1) or the queued steps fused into launches of up to environment.STEP_BATCH (defer, the
default; defer_all: with every queued step's obs / reward / done stored to the host, not only the
last's, environment.LIVE_OUTPUTS_ONLY off); defer_read = defer, reading every step's observation
before the next step (a host policy).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from pupperv3_mjx import MODEL_XML, environment, sharding  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env  # noqa: E402

E = 4096
N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
pipe = (sys.argv[2] == "1") if len(sys.argv) > 2 else True
mode = sys.argv[3] if len(sys.argv) > 3 else "defer"
environment.ASYNC_STEP = mode != "sync"
environment.ACTIONS_ZERO_COPY = mode in ("async_zc", "defer1", "defer", "defer_all", "defer_read")
environment.DEFER_LAUNCH = mode in ("defer1", "defer", "defer_all", "defer_read")
environment.LIVE_OUTPUTS_ONLY = mode != "defer_all"
if mode == "defer1":
    environment.STEP_BATCH = 1
read = mode == "defer_read"
env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=E, pipeline_output=pipe)
acts = np.random.RandomState(3).uniform(-1, 1, size=(N + 20, E, 12)).astype(np.float32)
st = env.reset(sharding.shard_keys(0, E, 1, 0))
for i in range(20):
    st = env.step(st, acts[i])
_ = st.obs  # the last warmup step's outputs are on the host
t = time.perf_counter()
for i in range(N):
    st = env.step(st, acts[20 + i])
    if read:
        _ = st.obs[0, 0]
_ = np.asarray(st.obs).sum()
dt = time.perf_counter() - t
print(f"env.step x {N} (pipeline_output={pipe}, {mode}): {dt / N * 1e6:.1f} us/step = {E * N / dt / 1e6:.2f} M env-steps/s",
      flush=True)
env.close()
