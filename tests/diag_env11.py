"""Diagnostic: replay one env step (config 'lat', env 11, step 6) on GPU and oracle; print contacts."""
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

np.set_printoptions(precision=5, suppress=True, linewidth=200)
d = tempfile.mkdtemp()
path = common.write_model(d, 10)
kw = common.fixture_kwargs(path, latency_distribution=[0.1, 0.2, 0.3, 0.4], imu_latency_distribution=[0.2, 0.3, 0.5])
n = 16
for rep in range(2):
    e = PupperV3Env(**kw, num_envs=n)
    st = e.reset(make_keys(9, n))
    rs = np.random.RandomState(4)
    for t in range(7):
        a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
        prev = st
        st = e.step(prev, a)
    i = 11
    o64 = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f64")
    o = o64.step(dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64)),
                 a[i].astype(np.float64))
    gp = st.pipeline_state
    print("rep", rep, "qvel gpu", st._record[i, 19:37])
    print("      qvel orc", o["state"][19:37])
    pipe = e._get(_abi.F_PIPELINE)[i]
    print("ncon gpu", pipe[_abi.P_NCON], "orc", o["pipe"][_abi.P_NCON])
    ng, no = int(pipe[_abi.P_NCON]), int(o["pipe"][_abi.P_NCON])
    print("dist gpu", pipe[_abi.P_CON_DIST:_abi.P_CON_DIST + ng], "\n     orc", o["pipe"][_abi.P_CON_DIST:_abi.P_CON_DIST + no])
    print("geom gpu", pipe[_abi.P_CON_GEOM:_abi.P_CON_GEOM + 2 * ng], "\n     orc", o["pipe"][_abi.P_CON_GEOM:_abi.P_CON_GEOM + 2 * no])
    print("qacc gpu", pipe[_abi.P_QACC:_abi.P_QACC + 18], "\n     orc", o["pipe"][_abi.P_QACC:_abi.P_QACC + 18])
    # also: raw physics from the same pre-state (5 substeps, same ctrl as the env would compute?)
    e.close()

# ---- physics-only replay of the same env step, substep by substep ----
from pupperv3_mjx import rng as R  # noqa: E402
e = PupperV3Env(**kw, num_envs=n)
st = e.reset(make_keys(9, n))
rs = np.random.RandomState(4)
for t in range(7):
    a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
    prev = st
    st = e.step(prev, a)
i = 11
rec0 = prev._record[i]
rec1 = st._record[i]
La = e.config_struct.latency_len
key = rec0[_abi.S_RNG:_abi.S_RNG + 2].copy().view(np.uint32)
ks = R.split(key, 5)
li = int(R.choice_index(ks[4], np.array(kw["latency_distribution"], dtype=np.float32)))
buf = rec1[_abi.S_ACT_BUF:_abi.S_ACT_BUF + 12 * La].reshape(12, La)
ctrl = np.clip(np.array(kw["default_pose"]) + buf[:, li] * 0.75, e.lowers, e.uppers)
q0 = rec0[0:19].astype(np.float64)
v0 = rec0[19:37].astype(np.float64)
v0[0:2] += rec1[_abi.S_KICK:_abi.S_KICK + 2]
w0 = rec0[37:55].astype(np.float64)
e1 = PupperV3Env(**kw, num_envs=1)
for ns in range(1, 6):
    gq, gv, gw, gp = G.gpu_physics(e1, q0[None], v0[None], w0[None], ctrl[None], ns)
    oq, ov, ow, op = G.oracle_physics(e1.sys_model.struct, q0[None], v0[None], w0[None], ctrl[None], ns)
    fq, fv, fw, fp = G.oracle_physics(e1.sys_model.struct, q0[None], v0[None], w0[None], ctrl[None], ns, precision="f32")
    print(ns, "gpu-f64 qvel", np.abs(gv - ov).max(), "f32-f64", np.abs(fv - ov).max(), "ncon", gp[0, _abi.P_NCON],
          op[0, _abi.P_NCON], "qacc err", np.abs(gp[0, _abi.P_QACC:_abi.P_QACC + 18] - op[0, _abi.P_QACC:_abi.P_QACC + 18]).max())
print("env-step qvel vs replay", np.abs(rec1[19:37] - gv[0]).max())

print("---- single substep from the oracle's post-substep-1 state ----")
oq1, ov1, ow1, _ = G.oracle_physics(e1.sys_model.struct, q0[None], v0[None], w0[None], ctrl[None], 1)
for tag, w in (("ws", ow1), ("zero", np.zeros_like(ow1))):
    gq, gv, gw, gp = G.gpu_physics(e1, oq1, ov1, w, ctrl[None], 1)
    oq, ov, ow, op = G.oracle_physics(e1.sys_model.struct, oq1, ov1, w, ctrl[None], 1)
    print(tag, "qacc gpu", gp[0, _abi.P_QACC:_abi.P_QACC + 18])
    print(tag, "qacc orc", op[0, _abi.P_QACC:_abi.P_QACC + 18])
    print(tag, "err", np.abs(gp[0, _abi.P_QACC:_abi.P_QACC + 18] - op[0, _abi.P_QACC:_abi.P_QACC + 18]).max())
f = O.mj_forward(e1.sys_model.struct, oq1[0], ov1[0], ow1[0], ctrl)
print("oracle forward: nefc", f["nefc"], "qacc_smooth", f["qacc_smooth"])
print("qws", ow1[0])
qs = f["qacc_smooth"][None]
for tag, w in (("ws", ow1), ("smooth", qs)):
    gq, gv, gw, gp = G.gpu_physics(e1, oq1, ov1, w, ctrl[None], 1)
    oq, ov, ow, op = G.oracle_physics(e1.sys_model.struct, oq1, ov1, w, ctrl[None], 1)
    print(tag, "gpu qacc[:6]", gp[0, _abi.P_QACC:_abi.P_QACC + 6], "orc", op[0, _abi.P_QACC:_abi.P_QACC + 6])
