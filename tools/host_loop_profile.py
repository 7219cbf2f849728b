"""Where a host policy's loop spends its time (verdict r05 items 3 / weak 6): `state = env.step(state,
a); state.obs` at the bench's env count, against the floors below it -- the same single-step launch
from C-ABI calls with a stream sync after each (no Python State), and the launch alone back to back.
Then cProfile of the host loop (top functions by own time).

  python tools/host_loop_profile.py [steps]
"""
import cProfile
import ctypes as C
import io
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]
import bench  # noqa: E402
from pupperv3_mjx import MODEL_XML, _lib  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env, make_keys  # noqa: E402

E = 4096
N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
PIPE = (sys.argv[2] != "0") if len(sys.argv) > 2 else True  # the constructor default: the pipeline record on


def main():
    env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=E, pipeline_output=PIPE)
    acts = np.random.RandomState(3).uniform(-1, 1, size=(N + 10, E, 12)).astype(np.float32)
    st = env.reset(make_keys(0, E))
    for i in range(10):
        st = env.step(st, acts[i])
        _ = st.obs[0, 0]

    def loop(n, a0):
        nonlocal st
        for i in range(n):
            st = env.step(st, acts[a0 + i])
            _ = st.obs[0, 0]

    L = env._L
    abuf = _lib.DeviceBuffer(acts[0].nbytes, env.device)
    abuf.upload(acts[0])
    D = env.observation_size
    blk = _lib.PinnedBlock(4 * E * (D + 2))
    dev = blk.device_ptr()
    R = _lib.load()

    def c_sync(n):  # the same single-step launch from C-ABI calls, a stream sync after each
        env.flush()
        env._before_launch()
        for _ in range(n):
            _lib.check(R.pp3_step(env._h, abuf.ptr, None))
            _lib.check(R.pp3_synchronize(env._h))

    def c_out(n):  # what env.step issues: a one-step pp3_rollout storing obs | reward | done into a
        env.flush()  # page-locked block through its device mapping, + sync
        env._before_launch()
        for _ in range(n):
            _lib.check(R.pp3_rollout(env._h, abuf.ptr, E * 12, 1, C.c_void_p(dev + 4 * E * D),
                                     C.c_void_p(dev + 4 * E * (D + 1)), C.c_void_p(dev), None))
            _lib.check(R.pp3_synchronize(env._h))

    def c_b2b(n):
        env.flush()
        env._before_launch()
        for _ in range(n):
            _lib.check(R.pp3_step(env._h, abuf.ptr, None))
        env.synchronize()

    # interleaved windows (the workload drifts as the robots fall), per-step wall clock
    res = {"host loop (step + obs read)": [], "C-ABI pp3_step + sync": [],
           "C-ABI 1-step pp3_rollout to page-locked outputs + sync": [], "C-ABI pp3_step back to back": []}
    n = max(10, N // 4)
    a0 = 0
    for rep in range(4):
        t = time.perf_counter(); loop(n, a0); res["host loop (step + obs read)"].append((time.perf_counter() - t) / n)
        a0 += n
        st = env._issue(False)
        t = time.perf_counter(); c_sync(n); res["C-ABI pp3_step + sync"].append((time.perf_counter() - t) / n)
        t = time.perf_counter(); c_out(n); res["C-ABI 1-step pp3_rollout to page-locked outputs + sync"].append((time.perf_counter() - t) / n)
        t = time.perf_counter(); c_b2b(n); res["C-ABI pp3_step back to back"].append((time.perf_counter() - t) / n)
        st = env._issue(False)
    # the host loop under cProfile
    pr = cProfile.Profile()
    pr.enable()
    loop(N, 0)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    for k, v in res.items():
        print(f"{k:58s} " + " ".join(f"{x * 1e6:6.1f}" for x in v) + f"  us/step (windows of {n} steps, interleaved)")
    print(s.getvalue())
    env.close()


if __name__ == "__main__":
    main()
