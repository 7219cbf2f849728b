"""CPU oracle self-checks (physical invariants + reference env tests on the oracle)."""
import numpy as np
import pytest

import common
import gpu_harness as G
from oracle import oracle as O
from pupperv3_mjx import _abi
from pupperv3_mjx.environment import make_keys

DP = np.array(common.DEFAULT_POSE)


def test_free_fall_is_exact_gravity():
    m = common.pd_model().struct
    q = np.zeros(19)
    q[2] = 1.0
    q[3] = 1
    q[7:] = DP
    r = O.mj_forward(m, q, np.zeros(18), np.zeros(18), DP)
    np.testing.assert_allclose(r["qacc"][:3], [0, 0, -9.81], atol=1e-9)
    np.testing.assert_allclose(r["qacc"][3:], 0, atol=1e-9)
    assert r["nefc"] == 12  # frictionloss rows only, no contacts/limits


def test_com_falls_with_g_in_flight():
    """No contacts: the COM accelerates at exactly g whatever the joints do (internal forces cancel)."""
    m = common.pd_model().struct
    rs = np.random.RandomState(0)
    for _ in range(3):
        q = np.zeros(19)
        q[2] = 2.0
        qq = rs.normal(size=4)
        q[3:7] = qq / np.linalg.norm(qq)
        q[7:] = DP + rs.uniform(-0.3, 0.3, 12)
        v = rs.normal(scale=0.5, size=18)
        r = O.mj_forward(m, q, v, np.zeros(18), DP + rs.uniform(-0.5, 0.5, 12))
        from pupperv3_mjx import mjcf
        M, jacp, _, _ = mjcf.mass_matrix_and_jacobians(m, q)
        mass = np.array(m.body_mass[:])
        # d/dt(sum m_i v_i) = sum m_i (J_i qacc + Jdot_i qd); check via finite differences of momentum
        h = 1e-6
        p0 = sum(mass[b] * jacp[b] @ v for b in range(1, 14))
        q1 = q.copy()
        q1[:3] += h * v[:3]
        w = v[3:6]
        from pupperv3_mjx.mjcf import axis_angle_quat, quat_mul
        nw = np.linalg.norm(w)
        q1[3:7] = quat_mul(q[3:7], axis_angle_quat(w / nw, h * nw))
        q1[7:] += h * v[6:]
        v1 = v + h * r["qacc"]
        _, jacp1, _, _ = mjcf.mass_matrix_and_jacobians(m, q1)
        p1 = sum(mass[b] * jacp1[b] @ v1 for b in range(1, 14))
        np.testing.assert_allclose((p1 - p0) / h / mass[1:].sum(), [0, 0, -9.81], atol=2e-4)


def test_standing_settles_on_four_feet():
    m = common.pd_model().struct
    q = np.zeros(19)
    q[2] = 0.2
    q[3] = 1
    q[7:] = DP
    v = np.zeros(18)
    w = np.zeros(18)
    q, v, w, pipe, _ = O.mj_step(m, q, v, w, DP, nsteps=1000)
    assert pipe[_abi.P_NCON] == 4
    assert 0.14 < q[2] < 0.17
    assert np.abs(v).max() < 5e-3  # slow creep of the soft frictionloss rows
    assert np.all(pipe[_abi.P_CON_DIST:_abi.P_CON_DIST + 4] < 0)


def test_fp32_oracle_tracks_fp64_on_standing_hold():
    """Benign trajectory: fp32 vs fp64 relative qpos drift over 1000 substeps."""
    m = common.pd_model().struct
    q0 = np.zeros(19)
    q0[2] = 0.17
    q0[3] = 1
    q0[7:] = DP
    z = np.zeros(18)
    qa, _, _, _, _ = O.mj_step(m, q0, z, z, DP, nsteps=1000, precision="f64")
    qb, _, _, _, _ = O.mj_step(m, q0, z, z, DP, nsteps=1000, precision="f32")
    rel = np.abs(qa - qb).max() / np.abs(qa).max()
    assert rel < 1e-4, rel


def _oracle_env(precision="f64", **over):
    m, c, env = common.env_model_and_config(common.write_model(common.GOLDEN + "/../_tmp", 0), **over)
    return O.OracleEnv(m, c, precision=precision), env


def test_oracle_get_obs_shape_and_range():
    oe, env = _oracle_env()
    s = oe.reset(make_keys(0, 1)[0])
    assert s["obs"].shape == (env._observation_history * env.observation_dim,)
    assert np.all(s["obs"] >= -100) and np.all(s["obs"] <= 100)
    for _ in range(20):
        s = oe.step(s, np.ones(12))
        assert np.all(np.isfinite(s["obs"])) and np.all(np.abs(s["obs"]) <= 100)


def test_oracle_imu_sampling():
    """test_environment.py:136-156: latency [0,0,1] reads the column that was 2nd-newest."""
    oe, env = _oracle_env(imu_latency_distribution=[0, 0, 1])
    s = oe.reset(make_keys(0, 1)[0])
    La = len(env._latency_distribution)
    io = _abi.imu_buf_offset(La)
    buf = np.zeros((6, 3))
    buf[:, -2] = np.arange(6)
    s["state"][io:io + 18] = buf.reshape(-1)
    s2 = oe.step(s, np.zeros(12))
    np.testing.assert_allclose(s2["obs"][:6], np.arange(6), atol=1e-5)


def test_oracle_reset_command_and_pose_ranges():
    oe, env = _oracle_env()
    keys = make_keys(11, 64)
    for k in keys:
        s = oe.reset(k)
        st = s["state"]
        assert -1 <= st[0] <= 1 and -1 <= st[1] <= 1 and 0.18 <= st[2] <= 0.24
        c = st[_abi.S_COMMAND:_abi.S_COMMAND + 3]
        assert (-0.75 <= c[0] <= 0.75 and -0.5 <= c[1] <= 0.5 and -2 <= c[2] <= 2) or np.all(np.abs(c) <= 0.1)
        dz = st[_abi.S_DESIRED_Z:_abi.S_DESIRED_Z + 3]
        assert abs(np.linalg.norm(dz) - 1) < 1e-9 and dz[2] >= np.cos(np.radians(45))
