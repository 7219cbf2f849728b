"""The kernel against the analytic known answers of test_physics_kat.py (not via the oracle).

Frictionloss (xml:55) on the HIP path: a torque below the threshold gives MuJoCo's documented
soft-constraint creep v = tau R / (b + damping R) (R = (1 - d)/d * dof_invweight0, d = impedance at
0, b = 2 / (dmax timeconst)); above it the joint accelerates at (tau - frictionloss - damping v) /
M_jj.  Tolerances are fp32-sized: 0.5 % on the creep velocity, 1.5 % on the slip acceleration.
"""
import numpy as np
import pytest

import common
import gpu_harness as G
import test_physics_kat as K
from oracle import oracle as O

pytestmark = pytest.mark.gpu
KNEE = 8


def _run(require_gpu, taus, nsteps):
    m = K._torque_model()
    n = 4
    e = G.env_with_model(common.MODEL_XML, m, n)
    try:
        q = np.zeros((n, 19))
        q[:, 3] = 1
        q[:, 7:] = K.DP
        ctrl = np.zeros((n, 12))
        ctrl[:, KNEE - 6] = taus
        out = [G.gpu_physics(e, q, np.zeros((n, 18)), np.zeros((n, 18)), ctrl, k) for k in nsteps]
        return m, ctrl, out
    finally:
        e.close()


def test_kernel_frictionloss_creep(require_gpu):
    m, ctrl, out = _run(require_gpu, [0.06, -0.06, 0.03, -0.1], [100])
    v = out[0][1][:, KNEE]
    si = np.array(m.dof_solimp[KNEE][:])
    d = K._imp(si, 0.0)
    b = 2.0 / (si[1] * m.dof_solref[KNEE][0])
    R = (1 - d) / d * m.dof_invweight0[KNEE]
    expect = ctrl[:, KNEE - 6] * R / (b + m.dof_damping[KNEE] * R)
    np.testing.assert_allclose(v, expect, rtol=5e-3)


def test_kernel_frictionloss_slip(require_gpu):
    # |tau| <= 0.25: the parent hinges' reaction stays below their frictionloss, so they hold and the
    # knee alone accelerates (from |tau| ~ 0.28 the parents slip too and the M_jj law no longer applies)
    m, ctrl, out = _run(require_gpu, [0.25, -0.25, 0.2, -0.18], [2, 8])
    v1, v2 = out[0][1][:, KNEE], out[1][1][:, KNEE]
    acc = (v2 - v1) / (6 * m.timestep)
    q = np.zeros(19)
    q[3] = 1
    q[7:] = K.DP
    Mkk = O.mj_forward(m, q, np.zeros(18), np.zeros(18), np.zeros(12))["M"][KNEE, KNEE]
    tau = ctrl[:, KNEE - 6]
    vm = 0.5 * (v1 + v2)
    expect = (tau - np.sign(tau) * m.dof_frictionloss[KNEE] - m.dof_damping[KNEE] * vm) / Mkk
    np.testing.assert_allclose(acc, expect, rtol=1.5e-2)
    assert np.all(np.abs(out[1][1][:, 6:8]).max(axis=1) < 1e-2 * np.abs(v2))  # parents held
