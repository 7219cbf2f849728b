"""Diagnostic (not a test): print GPU-vs-oracle error statistics for calibrating tolerances.

python tests/diag_parity.py   (GPU box)
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "pupperv3-mjx_amd")]

import numpy as np  # noqa: E402

import common  # noqa: E402
import gpu_harness as G  # noqa: E402
from oracle import oracle as O  # noqa: E402
from pupperv3_mjx import MODEL_XML, _abi  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env, make_keys  # noqa: E402


def rel(a, b):
    return np.abs(a - b).max() / max(1e-6, np.abs(b).max())


def main():
    tmp = os.path.join(HERE, "_tmp")
    os.makedirs(tmp, exist_ok=True)
    path = common.write_model(tmp, 0)
    kw = common.fixture_kwargs(path)
    n = 64
    env = PupperV3Env(**kw, num_envs=n)
    m = env.sys_model.struct
    qpos, qvel, qws, ctrl = common.random_physics_states(n, seed=1)
    for nsteps in (1, 5, 50):
        t = time.time()
        gq, gv, gw, gp = G.gpu_physics(env, qpos, qvel, qws, ctrl, nsteps)
        tg = time.time() - t
        oq, ov, ow, op = G.oracle_physics(m, qpos, qvel, qws, ctrl, nsteps)
        fq, fv, fw, fp = G.oracle_physics(m, qpos, qvel, qws, ctrl, nsteps, precision="f32")
        print(f"nsteps={nsteps} gpu {tg:.3f}s")
        for name, g, o, f in (("qpos", gq, oq, fq), ("qvel", gv, ov, fv), ("qacc", gw, ow, fw)):
            eg = np.abs(g - o).max(axis=1)
            ef = np.abs(f - o).max(axis=1)
            print(f"  {name}: gpu-vs-f64 max {eg.max():.3e} median {np.median(eg):.3e} | f32oracle-vs-f64 max {ef.max():.3e} median {np.median(ef):.3e}")
        print("  ncon gpu", gp[:8, _abi.P_NCON], "oracle", op[:8, _abi.P_NCON])
        worst = np.argsort(-np.abs(gv - ov).max(axis=1))[:4]
        print("  worst envs (qvel):", worst, np.abs(gv - ov).max(axis=1)[worst])
    # env reset/step parity vs oracle f32
    env2 = PupperV3Env(**common.fixture_kwargs(path), num_envs=16)
    keys = make_keys(0, 16)
    st = env2.reset(keys)
    oe = O.OracleEnv(env2.sys_model.struct, env2.config_struct, precision="f32")
    orecs = [oe.reset(keys[i]) for i in range(16)]
    orec = np.array([G.oracle_state_to_record(r["state"]) for r in orecs])
    oobs = np.array([r["obs"] for r in orecs])
    print("reset: state max diff", np.abs(st._record - orec).max(), "obs max diff", np.abs(st.obs - oobs).max())
    print("reset rng equal:", np.array_equal(st._record[:, 55:57].view(np.uint32), orec[:, 55:57].view(np.uint32)))
    rs = np.random.RandomState(0)
    for t in range(30):
        a = rs.uniform(-1, 1, size=(16, 12)).astype(np.float32)
        st = env2.step(st, a)
        orecs = [oe.step(orecs[i], a[i].astype(np.float64)) for i in range(16)]
        orec = np.array([G.oracle_state_to_record(r["state"]) for r in orecs])
        oobs = np.array([r["obs"] for r in orecs])
        orew = np.array([r["reward"] for r in orecs])
        odone = np.array([r["done"] for r in orecs])
        if t % 5 == 0 or t == 29:
            print(f"step {t}: qpos diff {np.abs(st._record[:, :19] - orec[:, :19]).max():.3e} obs diff "
                  f"{np.abs(st.obs - oobs).max():.3e} rew diff {np.abs(st.reward - orew).max():.3e} "
                  f"done mismatch {(st.done != odone).sum()} rng eq "
                  f"{np.array_equal(st._record[:, 55:57].view(np.uint32), orec[:, 55:57].view(np.uint32))}")
        # re-sync oracle to the GPU state to measure one-step error only
        orecs = [dict(r, state=G.record_to_oracle_state(st._record[i]), obs=st.obs[i].astype(np.float64))
                 for i, r in enumerate(orecs)]
    # throughput probe
    for N in (4096, 8192):
        envb = PupperV3Env(**common.fixture_kwargs(path), num_envs=N, pipeline_output=False)
        envb.reset(make_keys(0, N))
        act = np.zeros((N, 12), dtype=np.float32)
        from pupperv3_mjx import _lib
        buf = _lib.DeviceBuffer(N * 48)
        buf.upload(act)
        import ctypes as C
        ms = C.c_float()
        _lib.check(envb._L.pp3_step_timed(envb._h, buf.ptr, 0, 5, C.byref(ms)))
        _lib.check(envb._L.pp3_step_timed(envb._h, buf.ptr, 0, 20, C.byref(ms)))
        print(f"N={N}: {ms.value / 20:.3f} ms/step -> {N * 20 / (ms.value / 1e3) / 1e6:.2f} M env-steps/s")


if __name__ == "__main__":
    main()
