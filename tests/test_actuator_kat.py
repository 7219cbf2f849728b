"""Actuator known answer (the model's <general> defaults, assets/pupper_v3.xml:44-45: affine bias,
forcerange -3 3, forcelimited; the env's PD overrides Kp = 5, Kd = 0.25 as in
environment.py's position_control_kp / dof_damping): qfrc_actuator of hinge i is
clip(Kp (ctrl_i - q_i) - Kd qd_i, -3, 3) and zero on the free joint, written here from the XML
literals, on the oracle; test_gpu_actuator_kat.py runs the same states through the kernel."""
import numpy as np

import common
from oracle import oracle as O
from pupperv3_mjx import _abi

KP, KD, FMAX = 5.0, 0.25, 3.0


def actuator_states(n, seed):
    rs = np.random.RandomState(seed)
    q = np.zeros((n, 19))
    q[:, 2], q[:, 3] = 2.0, 1.0  # in flight
    q[:, 7:] = np.array(common.DEFAULT_POSE) + rs.uniform(-0.4, 0.4, (n, 12))
    v = np.zeros((n, 18))
    v[:, 6:] = rs.normal(scale=4.0, size=(n, 12))
    ctrl = q[:, 7:] + rs.uniform(-1.0, 1.0, (n, 12))  # about a third saturate at +-3 N m
    return q, v, ctrl


def expected(q, v, ctrl):
    return np.clip(KP * (ctrl - q[:, 7:]) - KD * v[:, 6:], -FMAX, FMAX)


def test_pd_torque_equals_closed_form():
    m = common.pd_model().struct
    q, v, ctrl = actuator_states(32, seed=0)
    want = expected(q, v, ctrl)
    sat = 0
    for i in range(32):
        _, _, _, pipe, _ = O.mj_step(m, q[i], v[i], np.zeros(18), ctrl[i], nsteps=1)
        f = pipe[_abi.P_QFRC_ACT:_abi.P_QFRC_ACT + 18]
        np.testing.assert_allclose(f[6:], want[i], atol=1e-12)
        assert np.all(f[:6] == 0)
        sat += int(np.sum(np.abs(want[i]) == FMAX))
    assert 32 * 12 // 8 < sat < 32 * 12 * 7 // 8, sat  # both the linear and the clamped branch
