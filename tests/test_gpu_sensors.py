"""Site sensors (mjData.sensordata in the pipeline record, PP3_P_SENSOR) through the C ABI vs the
CPU oracle's restatement (tests/test_sensors.py pins that restatement by physics known answers).

Tolerances (fp32 kernel vs fp64 oracle), per sensor kind:
  frame quat / pos       : 1e-5 abs (kinematics)
  gyro / linvel / angvel : 5e-3 abs, or 5x the fp32 oracle's own error (velocities of the forward)
  accelerometer          : 0.05 abs, or 5x the fp32 oracle's own error (it carries qacc of the
                           constraint solve, whose fp32 error is ~qvel error / h)
Steps whose oracle run crossed a constraint switch point (FlipBudget) may exceed them.
"""
import numpy as np
import pytest

import common
import gpu_harness as G
from oracle import oracle as O
from pupperv3_mjx import _abi
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu

KIND = {0: ("quat", 4), 4: ("vel", 3), 7: ("acc", 3), 10: ("quat", 4), 14: ("pos", 3), 17: ("vel", 3), 20: ("vel", 3)}
TOL = {"quat": 1e-5, "pos": 1e-5, "vel": 5e-3, "acc": 0.05}


def _check(g, o, f):
    """g, o, f: sensordata rows of the GPU, fp64 oracle, fp32 oracle; True if every sensor is in tolerance."""
    ok = True
    for adr, (kind, dim) in KIND.items():
        sl = slice(adr, adr + dim)
        err = np.abs(g[sl] - o[sl]).max()
        ok = ok and err <= max(TOL[kind], 5 * np.abs(f[sl] - o[sl]).max())
    return ok


@pytest.fixture(scope="module")
def env64(require_gpu, tmp_path_factory):
    path = common.write_model(tmp_path_factory.mktemp("m"), 0)
    e = PupperV3Env(**common.fixture_kwargs(path), num_envs=64)
    yield e
    e.close()


@pytest.mark.parametrize("nsteps", [1, 3])
def test_sensor_parity_physics(env64, nsteps):
    m = env64.sys_model.struct
    qpos, qvel, qws, ctrl = common.random_physics_states(64, seed=30 + nsteps)
    _, _, _, gp = G.gpu_physics(env64, qpos, qvel, qws, ctrl, nsteps)
    fb = G.FlipBudget()
    S = slice(_abi.P_SENSOR, _abi.P_SENSOR + 23)
    for i in range(64):
        o = O.mj_step(m, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=nsteps)
        boundary = O.mj_step.last_boundary
        f = O.mj_step(m, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=nsteps, precision="f32")
        fb.check(_check(gp[i][S], o[3][S], f[3][S]), {"boundary": boundary}, f"env {i}")
        np.testing.assert_array_equal(gp[i][_abi.P_SENSOR + 23:], 0)  # padding
    fb.finish()


def test_sensor_parity_env_step_and_reset(tmp_path):
    """reset (mjx.forward: sensors of the start pose) and env steps (sensors of the last substep's
    forward) against the oracle env, state re-synced every step."""
    path = common.write_model(tmp_path, 0)
    n = 16
    e = PupperV3Env(**common.fixture_kwargs(path), num_envs=n)
    try:
        oe = O.OracleEnv(e.sys_model.struct, e.config_struct)
        oe32 = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f32")
        keys = make_keys(11, n)
        st = e.reset(keys)
        S = slice(_abi.P_SENSOR, _abi.P_SENSOR + 23)
        gp = e._get(_abi.F_PIPELINE)
        for i in range(n):
            o, f = oe.reset(keys[i]), oe32.reset(keys[i])
            assert _check(gp[i][S], o["pipe"][S], f["pipe"][S]), i
        rs = np.random.RandomState(3)
        fb = G.FlipBudget()
        for t in range(5):
            a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
            prev = st
            st = e.step(prev, a)
            gp = e._get(_abi.F_PIPELINE)
            for i in range(n):
                s_in = dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64))
                o = oe.step(s_in, a[i].astype(np.float64))
                f = oe32.step(s_in, a[i].astype(np.float64))
                fb.check(_check(gp[i][S], o["pipe"][S], f["pipe"][S]), o, f"step {t} env {i}")
        fb.finish()
    finally:
        e.close()
