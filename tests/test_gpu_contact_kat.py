"""The kernel against the mixing and tangent-basis known answers of test_contact_kat.py (written
from MuJoCo's documentation in tests/contact_kat.py, not via the oracle).

Tolerances are fp32-sized: 1e-2 relative on the resting depth and the steady creep (a difference of
two ~2.4 m/s numbers at fp32 spacing, accumulated over 300 substeps), 2e-3 g on the converged
rolling qacc, 1e-3 of the largest acceleration on the sliding-contact qacc.  Every basis check also
asserts that turning the tangents by 30 / 45 degrees moves the known answer by at least 20 times
that tolerance."""
import math

import numpy as np
import pytest

import common
import contact_kat as C
import gpu_harness as G
import test_friction_kat as F
from pupperv3_mjx import _abi

pytestmark = pytest.mark.gpu
GRAV = 9.81


def _run(path, m, q, v, w, ctrl, nsteps, n=2):
    """n identical envs of model struct m on the kernel: (qpos, qvel, qacc, pipe) of env 0."""
    e = G.env_with_model(path, m, n)
    try:
        tile = lambda x: np.tile(x, (n, 1))  # noqa: E731
        q2, v2, w2, p2 = G.gpu_physics(e, tile(q), tile(v), tile(w), tile(ctrl), nsteps)
        return q2[0], v2[0], w2[0], p2[0]
    finally:
        e.close()


def test_kernel_ball_rests_at_the_mixed_impedance_depth(require_gpu):
    m = F.ball_model(0.0, None, mixed=True)
    q, v, w = F._rest_state()
    q2, v2, _, _ = _run(common.MODEL_XML, m, q, v, w, F.DP, 500)
    r = C.rest_penetration(C.mix_params(C.COLLISION_CLASS, C.FLOOR), F.M_BALL, GRAV, F.R_BALL, m.impratio, m.timestep)
    G.report("contact_kat_rest_depth", {"kernel": float(q2[2] - F.R_BALL), "known": r})
    np.testing.assert_allclose(q2[2] - F.R_BALL, r, rtol=1e-2)
    assert np.abs(v2[0:6]).max() < 1e-3


def test_kernel_ball_rolls_at_the_mixed_impedance_creep(require_gpu):
    m = F.ball_model(10.0, None, mixed=True)
    q, v, w = F._rest_state()
    q2, v2, _, _ = _run(common.MODEL_XML, m, q, v, w, F.DP, 300)
    s, r = C.steady_creep(C.mix_params(C.COLLISION_CLASS, C.FLOOR), F.M_BALL, F.R_BALL, math.radians(10.0), GRAV,
                          m.impratio, m.timestep)
    G.report("contact_kat_creep", {"kernel_slip": float(F._slip(q2, v2)[0]), "known_slip": s,
                                   "kernel_depth": float(q2[2] - F.R_BALL), "known_depth": r})
    np.testing.assert_allclose(F._slip(q2, v2)[0], s, rtol=1e-2)
    np.testing.assert_allclose(q2[2] - F.R_BALL, r, rtol=1e-2)


def test_kernel_rolling_ball_converged_qacc_with_mixed_parameters(require_gpu):
    m = F.ball_model(10.0, None, iterations=50, mixed=True)
    q, v, w = F._rest_state()
    q1, v1, w1, _ = _run(common.MODEL_XML, m, q, v, w, F.DP, 150)
    _, _, w2, _ = _run(common.MODEL_XML, m, q1, v1, w1, F.DP, 1)
    a, P = C.ball_qacc(q1, v1, C.mix_params(C.COLLISION_CLASS, C.FLOOR), F.M_BALL, F.R_BALL,
                       np.array(m.gravity[:]), m.impratio, m.timestep)
    assert P["dist"] < 0 and sum(P["active"]) >= 1
    err = np.abs(w2[0:6] - a)
    assert np.all(err <= 2e-3 * GRAV + 2e-3 * np.abs(a)), (w2[0:6], a)


def _check_basis(got, a, rotated, tol_frac=1e-3):
    scale = np.abs(a).max()
    err = np.abs(got - a).max()
    sens = min(np.abs(rotated(math.radians(x)) - a).max() for x in (30.0, 45.0))
    assert sens > 20 * tol_frac * scale, (sens, scale)
    assert err <= tol_frac * scale, (got, a, err, scale)
    return err / scale, sens / scale


@pytest.mark.parametrize("case", sorted(C.BOX_CASES))
def test_kernel_ball_sliding_on_tilted_box_uses_the_documented_frame(tmp_path, require_gpu, case):
    path = common.write_model(tmp_path, 1)
    m, q, v, box = C.tilted_box_case(path, case)
    _, _, w, pipe = _run(path, m, q, v, np.zeros(18), F.DP, 1)
    assert int(pipe[_abi.P_NCON]) == 1
    a, act, _ = C.box_known_answer(m, q, v, box)
    assert 0 < sum(act) < 4
    rel, sens = _check_basis(w[0:6], a, lambda ang: C.box_known_answer(
        m, q, v, box, lambda n: C.rotated_frame(C.make_frame(n), ang))[0])
    G.report(f"contact_kat_box_frame_{case}", {"rel_err": rel, "basis_sensitivity": sens})


@pytest.fixture(scope="module")
def leg_model():
    return C.leg_pair_model()


@pytest.mark.parametrize("branch", ["ty", "tz"])
def test_kernel_leg_spheres_sliding_use_the_documented_frame(require_gpu, leg_model, branch):
    """Two legs' spheres sliding on each other: the kernel's leg-leg Newton path (the contact
    couples two legs) with the documented frame of a normal off every axis."""
    m, invw = leg_model
    q, v, p = C.leg_pair_state(m, invw, branch, seed=3)
    _, _, w, pipe = _run(common.MODEL_XML, m, q, v, np.zeros(18), np.zeros(12), 1)
    assert int(pipe[_abi.P_NCON]) == 1
    a, act, _ = C.leg_pair_known_answer(m, q, v, p, invw)
    assert 0 < sum(act) < 4
    rel, sens = _check_basis(w, a, lambda ang: C.leg_pair_known_answer(
        m, q, v, p, invw, lambda n: C.rotated_frame(C.make_frame(n), ang))[0])
    G.report(f"contact_kat_leg_frame_{branch}", {"rel_err": rel, "basis_sensitivity": sens})
