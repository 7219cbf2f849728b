"""The kernel on the constructor branches of test_env_branches.py (use_imu=False, nonzero
desired_abduction_angles, a non-default terminal_body_angle): each against its known answer and
in env-step parity with the oracle on 64 envs (test_gpu_rewards._rollout_parity: every reward term,
state-record field, obs, reward and done per step, 1 % constraint-flip budget)."""
import numpy as np
import pytest

import common
import test_env_branches as B
from pupperv3_mjx import _abi
from pupperv3_mjx.environment import PupperV3Env, make_keys
from test_gpu_rewards import _rollout_parity

pytestmark = pytest.mark.gpu
N = 64


def _make(**over):
    return PupperV3Env(**common.fixture_kwargs(common.MODEL_XML, **over), num_envs=N)


def _tilted(e, keys, angles, axes, spins=None):
    st = e.reset(keys)
    q = st.pipeline_state.q.copy()
    qd = np.zeros_like(st.pipeline_state.qd)
    q[:, 2] = 0.5
    for i in range(N):
        ax = np.asarray(axes[i % len(axes)], float)
        ax /= np.linalg.norm(ax)
        q[i, 3:7] = np.concatenate([[np.cos(angles[i] / 2)], np.sin(angles[i] / 2) * ax])
        if spins is not None:
            qd[i, 3:6] = spins[i]
    q[:, 7:] = common.DEFAULT_POSE
    st.pipeline_state.q = q
    st.pipeline_state.qd = qd
    e._write_state(st)
    return e._issue(False)


def test_kernel_use_imu_false(require_gpu):
    # known answer: IMU noise off -> the lagged channels are exactly (0,0,0, 0,0,-1) on tilted, spinning bodies
    e = _make(use_imu=False, angular_velocity_noise=0.0, gravity_noise=0.0)
    try:
        rs = np.random.RandomState(1)
        st = _tilted(e, make_keys(7, N), rs.uniform(-1.2, 1.2, N), [(1, 2, 0.5), (0, 1, 0), (1, 0, 1)],
                     rs.uniform(-5, 5, (N, 3)))
        out = e.step(st, np.zeros((N, 12), np.float32))
        np.testing.assert_array_equal(out.obs[:, 0:6], np.tile([0, 0, 0, 0, 0, -1], (N, 1)))
    finally:
        e.close()
    e = _make(use_imu=False)
    try:
        _rollout_parity(e, make_keys(8, N), 20, 11, "env_branch_use_imu_false")
    finally:
        e.close()


def test_kernel_desired_abduction_angles(require_gpu):
    e = _make(desired_abduction_angles=B.ABD)
    try:
        stats = _rollout_parity(e, make_keys(9, N), 20, 12, "env_branch_abduction")
        assert "abduction_angle" in stats.nonzero
        # oracle-free: the kernel's term from its own post-step joint angles
        st = e.reset(make_keys(10, N))
        st = e.step(st, np.random.RandomState(2).uniform(-1, 1, (N, 12)).astype(np.float32))
        q = st.pipeline_state.q[:, 7:].astype(np.float64)
        scale = e.config_struct.reward_scales[_abi.REWARD_NAMES.index("abduction_angle")]
        want = scale * np.sum((q[:, 1::3] - np.array(B.ABD)) ** 2, axis=1)
        np.testing.assert_allclose(st.metrics["abduction_angle"], want, rtol=1e-5, atol=1e-7)
    finally:
        e.close()


def test_kernel_terminal_body_angle(require_gpu):
    e = _make(terminal_body_angle=0.3, kick_probability=0.0)
    try:
        angles = np.where(np.arange(N) % 2 == 0, 0.25, 0.35)
        st = _tilted(e, make_keys(11, N), angles, [(1, 0, 0), (0, 1, 0), (1, -1, 0)])
        out = e.step(st, np.zeros((N, 12), np.float32))
        np.testing.assert_array_equal(out.done, (angles > 0.3).astype(np.float32))
    finally:
        e.close()
    e = _make(terminal_body_angle=0.3)
    try:
        _rollout_parity(e, make_keys(12, N), 20, 13, "env_branch_terminal_angle")
    finally:
        e.close()
