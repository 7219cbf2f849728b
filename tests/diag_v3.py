"""Diagnostic: per-env GPU-vs-oracle differences over re-synced env steps (prints the worst
field, step, env and index for each part of the state record)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd"), os.path.join(ROOT, "tests")]
import tempfile  # noqa: E402

import numpy as np  # noqa: E402

import common  # noqa: E402
import gpu_harness as G  # noqa: E402
from oracle import oracle as O  # noqa: E402
from pupperv3_mjx import _abi  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env, make_keys  # noqa: E402


def run(kw, n, steps, tag):
    e = PupperV3Env(**kw, num_envs=n)
    st = e.reset(make_keys(9, n))
    oe = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f32")
    o64 = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f64")
    ref = {}
    rs = np.random.RandomState(4)
    worst = {}
    for t in range(steps):
        a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
        prev = st
        st = e.step(prev, a)
        for i in range(n):
            o = oe.step(dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64)),
                        a[i].astype(np.float64))
            orec = G.oracle_state_to_record(o["state"])
            o2 = o64.step(dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64)),
                          a[i].astype(np.float64))
            dv64 = float(np.abs(o2["state"][19:37] - o["state"][19:37]).max())
            dvg = float(np.abs(st._record[i][19:37] - o2["state"][19:37]).max())
            if dvg > ref.get("gpu_vs_f64_qvel", (0,))[0]:
                ref["gpu_vs_f64_qvel"] = (dvg, t, i)
            if dv64 > ref.get("f32orc_vs_f64_qvel", (0,))[0]:
                ref["f32orc_vs_f64_qvel"] = (dv64, t, i)
            with np.errstate(invalid="ignore"):
                d = np.abs(st._record[i] - orec)
            d[_abi.S_RNG:_abi.S_RNG + 2] = 0
            for name, sl in (("qpos", slice(0, 19)), ("qvel", slice(19, 37)), ("qws", slice(37, 55)),
                             ("info", slice(55, _abi.S_ACT_BUF)), ("buf", slice(_abi.S_ACT_BUF, None))):
                v = d[sl].max()
                if v > worst.get(name, (0,))[0]:
                    worst[name] = (float(v), t, i, int(np.argmax(d[sl])))
            v = float(np.abs(st.obs[i] - o["obs"]).max())
            if v > worst.get("obs", (0,))[0]:
                worst["obs"] = (v, t, i, int(np.argmax(np.abs(st.obs[i] - o["obs"]))))
            v = float(abs(st.reward[i] - o["reward"]))
            if v > worst.get("reward", (0,))[0]:
                worst["reward"] = (v, t, i, -1)
    print(tag, worst, ref, flush=True)
    e.close()


if __name__ == "__main__":
    d = tempfile.mkdtemp()
    path = common.write_model(d, 10)
    run(common.fixture_kwargs(path), 16, 20, "default")
    run(common.fixture_kwargs(path, observation_history=15), 16, 20, "H15")
    run(common.fixture_kwargs(path, latency_distribution=[0.1, 0.2, 0.3, 0.4],
                              imu_latency_distribution=[0.2, 0.3, 0.5]), 16, 20, "lat")
    run(common.fixture_kwargs(path, observation_history=15, latency_distribution=[0.1, 0.2, 0.3, 0.4],
                              imu_latency_distribution=[0.2, 0.3, 0.5]), 16, 20, "both")
