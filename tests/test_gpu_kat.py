"""The kernel against the analytic known answers of test_physics_kat.py (not via the oracle).

Frictionloss (xml:55) on the HIP path: a torque below the threshold gives MuJoCo's documented
soft-constraint creep v = tau R / (b + damping R) (R = (1 - d)/d * dof_invweight0, d = impedance at
0, b = 2 / (dmax timeconst)); above it the joint accelerates at (tau - frictionloss - damping v) /
M_jj.  Tolerances are fp32-sized: 0.5 % on the creep velocity, 1.5 % on the slip acceleration.
Joint limits: a hinge pushed into its range limit rests where the limit row's soft-constraint
force equals the torque (test_physics_kat._limit_rest_prediction).
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


# ------------------------------------------------------------------ pyramidal friction (ball)
import test_friction_kat as F  # noqa: E402


def _ball_gpu(m, nsteps, n=2):
    """The ball model (test_friction_kat.ball_model) on the kernel: n identical envs from rest."""
    e = G.env_with_model(common.MODEL_XML, m, n)
    try:
        q, v, w = F._rest_state()
        tile = lambda x: np.tile(x, (n, 1))  # noqa: E731
        out = [G.gpu_physics(e, tile(q), tile(v), tile(w), tile(F.DP), k) for k in nsteps]
        return [(o[0][0], o[1][0], o[2][0]) for o in out]
    finally:
        e.close()


@pytest.mark.parametrize("case", sorted(F.CASES))
def test_kernel_converged_qacc_equals_documented_soft_pyramid(require_gpu, case):
    """The kernel's pyramid edge rows, impratio regulariser and aref: with Newton run to convergence
    its qacc at a rolling / sliding state equals the exact minimiser of the documented problem
    (fp32: 2e-3 relative to g)."""
    theta, mu = F.CASES[case]
    m = F.ball_model(theta, mu, iterations=50)
    (q, v, w), = _ball_gpu(m, [150])
    e = G.env_with_model(common.MODEL_XML, m, 2)
    try:
        _, _, w2, _ = G.gpu_physics(e, np.tile(q, (2, 1)), np.tile(v, (2, 1)), np.tile(w, (2, 1)),
                                    np.tile(F.DP, (2, 1)), 1)
    finally:
        e.close()
    a, info = F.ball_qacc(m, q, v)
    assert info["dist"] < 0 and sum(info["active"]) >= 1
    err = np.abs(w2[0, 0:6] - a)
    assert np.all(err <= 2e-3 * F.G + 2e-3 * np.abs(a)), (w2[0, 0:6], a)
    G.report(f"friction_kat_converged_{case}", {"qacc_abs_err_max": float(err.max()), "qacc": a.tolist()})


def test_kernel_ball_rolls_at_five_sevenths_g_sin(require_gpu):
    """The reference's solver (iterations = 1) on the kernel: rolling at (5/7) g sin th, contact
    point creeping at < 0.1 % of the speed."""
    theta, mu = F.CASES["roll"]
    m = F.ball_model(theta, mu)
    (q1, v1, _), (q2, v2, _) = _ball_gpu(m, [100, 150])
    acc = (v2[0] - v1[0]) / (50 * m.timestep)
    np.testing.assert_allclose(acc, 5.0 / 7.0 * F.G * np.sin(np.radians(theta)), rtol=5e-3)
    assert abs(F._slip(q2, v2)[0]) < 1e-3 * v2[0]


def test_kernel_ball_slides_at_the_coulomb_bound(require_gpu):
    """mu below the stick threshold (converged Newton): the kernel's ball accelerates at
    g (sin th - mu cos th) over a long slide, spinning up from the friction torque."""
    theta, mu = F.CASES["slide"]
    m = F.ball_model(theta, mu, iterations=50)
    (q1, v1, _), (q2, v2, _) = _ball_gpu(m, [100, 500])
    acc = (v2[0] - v1[0]) / (400 * m.timestep)
    th = np.radians(theta)
    np.testing.assert_allclose(acc, F.G * (np.sin(th) - mu * np.cos(th)), rtol=5e-3)
    assert F._slip(q2, v2)[0] > 0.3 * v2[0]


def test_kernel_impratio_scales_the_creep(require_gpu):
    theta, mu = F.CASES["roll"]
    creep = {}
    for ir in (1.0, 10.0):
        m = F.ball_model(theta, mu)
        m.impratio = ir
        (q, v, _), = _ball_gpu(m, [150])
        creep[ir] = F._slip(q, v)[0]
    assert creep[1.0] > 0 and creep[10.0] > 0
    assert 5.0 < creep[1.0] / creep[10.0] < 15.0, creep


def test_kernel_joint_limit_rest_position(require_gpu):
    """The kernel's joint-limit rows at rest (test_physics_kat.test_joint_limit_rest_position): a
    hinge pushed into its range limit settles at the documented soft-limit equilibrium, beyond the
    solimp width and inside it, against upper and lower limits."""
    m = K._torque_model()
    n = len(K.LIMIT_CASES)
    e = G.env_with_model(common.MODEL_XML, m, n)
    try:
        q = np.zeros((n, 19))
        q[:, 3] = 1
        q[:, 7:] = K.DP
        ctrl = np.zeros((n, 12))
        want = []
        for i, (jnt, tau) in enumerate(K.LIMIT_CASES):
            side, x, q_expect = K._limit_rest_prediction(m, jnt, tau)
            q[i, m.jnt_qposadr[jnt]] = m.jnt_range[jnt][(side + 1) // 2] - side * 0.002
            ctrl[i, m.jnt_dofadr[jnt] - 6] = tau
            want.append((jnt, side, x, q_expect))
        q1, v1, w1, _ = G.gpu_physics(e, q, np.zeros((n, 18)), np.zeros((n, 18)), ctrl, 1500)
        q2, v2, _, _ = G.gpu_physics(e, q1, v1, w1, ctrl, 1)
        for i, (jnt, side, x, q_expect) in enumerate(want):
            a, dof = m.jnt_qposadr[jnt], m.jnt_dofadr[jnt]
            assert abs(v1[i, dof] + v2[i, dof]) < 1e-4, (jnt, v1[i, dof], v2[i, dof])  # fp32: a ~1e-5 rad/s creep
            rng = m.jnt_range[jnt][(side + 1) // 2]
            got = 0.5 * (q1[i, a] + q2[i, a]) - rng
            assert abs(got - (q_expect - rng)) <= 3e-3 * abs(x) + 2e-6, (jnt, got, q_expect - rng)
    finally:
        e.close()
