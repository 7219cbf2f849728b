"""Contact-parameter mixing and the pyramid's tangent basis, pinned on the oracle against known
answers written from MuJoCo's documentation (tests/contact_kat.py; the kernel's side is
test_gpu_contact_kat.py).

Mixing (/root/reference/test/test_pupper_model.xml:50-52 collision class vs the floor's defaults,
xml:219): a solid ball that keeps its own compiled parameters runs every floor contact on the
solmix-mixed solimp (0.4575, 0.975, 0.016, 0.5, 2).  Known answers: the depth at which it rests
(the four edge rows' documented force carries m g), the slip velocity at which it rolls steadily
down a 10 degree slope (the documented minimiser gives neither slip nor normal acceleration), and
the converged qacc.  Either geom's parameters taken alone predict a depth 20x / 8.5x off and a creep
11x / 4.6x off, so an implementation that skipped or mis-weighted the mixing fails.

Tangent basis (xml:57 cone="pyramidal", mju_makeFrame): the pyramid is not isotropic, so a sliding
contact's friction force depends on which tangents the frame picks.  Known answers: the converged
qacc of a ball sliding on a tilted obstacle box (face with n_y inside and outside (-0.5, 0.5), an
edge, a corner: normals off every axis) and of two legs' spheres sliding on each other (M and the
contact Jacobian from the independent kinematics of test_physics_kat), each the documented
minimiser with the documented frame.  The same minimiser with the tangents turned by 30 or 45
degrees differs by 5-30 % of the largest acceleration, far outside the tolerance."""
import math

import numpy as np
import pytest

import common
import contact_kat as C
import test_friction_kat as F
from oracle import oracle as O
from pupperv3_mjx import _abi

G = 9.81


def test_compiled_geom_parameters_are_the_xml_literals(tmp_path):
    """The MJCF compiler's per-geom contact parameters are the XML literals with MuJoCo's
    documented defaults filled in: every collision sphere carries the collision class, the floor
    and the obstacle boxes the defaults (the inputs to the mixing both implementations do)."""
    m = common.pd_model(common.write_model(tmp_path, 2)).struct
    for g in range(m.ncgeom):
        want = C.COLLISION_CLASS if m.cgeom_bodyid[g] != 0 else C.FLOOR
        np.testing.assert_allclose(m.cgeom_solref[g][:], want["solref"])
        np.testing.assert_allclose(m.cgeom_solimp[g][:], want["solimp"])
        np.testing.assert_allclose(m.cgeom_friction[g][:], want["friction"])
        assert m.cgeom_solmix[g] == want["solmix"] and m.cgeom_priority[g] == want["priority"]
    pair = C.mix_params(C.COLLISION_CLASS, C.FLOOR)
    np.testing.assert_allclose(pair["solimp"], [0.4575, 0.975, 0.016, 0.5, 2.0])
    assert pair["mu"] == 1.0 and pair["mix"] == 0.5


def _mixed():
    return C.mix_params(C.COLLISION_CLASS, C.FLOOR)


def test_ball_rests_at_the_mixed_impedance_depth():
    """Flat floor, the reference solver (iterations = 1): after 2 s the ball rests at the depth
    where the mixed-impedance edge rows carry its weight (1e-3 relative), at rest."""
    m = F.ball_model(0.0, None, mixed=True)
    q, v, w = F._rest_state()
    q2, v2, _, _, _ = O.mj_step(m, q, v, w, F.DP.copy(), nsteps=500)
    r = C.rest_penetration(_mixed(), F.M_BALL, G, F.R_BALL, m.impratio, m.timestep)
    np.testing.assert_allclose(q2[2] - F.R_BALL, r, rtol=1e-3)
    assert np.abs(v2[0:6]).max() < 1e-5
    for p in (C.FLOOR, C.COLLISION_CLASS):  # the unmixed parameters predict a far different depth
        other = C.rest_penetration(C.unmixed(p), F.M_BALL, G, F.R_BALL, m.impratio, m.timestep)
        assert max(other / r, r / other) > 2.0, (other, r)


def test_ball_rolls_at_the_mixed_impedance_creep():
    """10 degree slope, mu = max(0.8, 1) = 1, the reference solver: after 1.2 s of rolling the
    contact point slips at the documented steady creep and sits at its steady depth (1e-3)."""
    m = F.ball_model(10.0, None, mixed=True)
    q, v, _, _, _ = F.run_oracle(m, 300)
    s, r = C.steady_creep(_mixed(), F.M_BALL, F.R_BALL, math.radians(10.0), G, m.impratio, m.timestep)
    np.testing.assert_allclose(F._slip(q, v)[0], s, rtol=1e-3)
    np.testing.assert_allclose(q[2] - F.R_BALL, r, rtol=1e-3)
    for p in (C.FLOOR, C.COLLISION_CLASS):
        s2, _ = C.steady_creep(C.unmixed(p), F.M_BALL, F.R_BALL, math.radians(10.0), G, m.impratio, m.timestep)
        assert max(s2 / s, s / s2) > 2.0, (s2, s)


def test_rolling_ball_converged_qacc_with_mixed_parameters():
    m = F.ball_model(10.0, None, iterations=50, mixed=True)
    q, v, w, _, _ = F.run_oracle(m, 150)
    _, _, w2, _, _ = O.mj_step(m, q, v, w, F.DP.copy(), nsteps=1)
    a, P = C.ball_qacc(q, v, _mixed(), F.M_BALL, F.R_BALL, np.array(m.gravity[:]), m.impratio, m.timestep)
    assert P["dist"] < 0 and sum(P["active"]) >= 1
    np.testing.assert_allclose(w2[0:6], a, atol=1e-7 * G, rtol=1e-6)


# ------------------------------------------------------------------ tangent basis
@pytest.fixture(scope="module")
def box_path(tmp_path_factory):
    return common.write_model(tmp_path_factory.mktemp("m"), 1)


def _basis_sensitivity(known, solve_rotated):
    """Largest change of the known answer when the tangents are turned by 30 / 45 degrees."""
    return min(np.abs(solve_rotated(math.radians(a)) - known).max() for a in (30.0, 45.0))


@pytest.mark.parametrize("case", sorted(C.BOX_CASES))
def test_ball_sliding_on_tilted_box_uses_the_documented_frame(box_path, case):
    m, q, v, box = C.tilted_box_case(box_path, case)
    _, _, w, pipe, _ = O.mj_step(m, q, v, np.zeros(18), F.DP.copy(), nsteps=1)
    a, act, P = C.box_known_answer(m, q, v, box)
    assert int(pipe[_abi.P_NCON]) == 1 and 0 < sum(act) < 4       # sliding: the pyramid is anisotropic
    assert np.abs(P["n"]).min() > 0.2                               # a normal off every axis
    scale = np.abs(a).max()
    np.testing.assert_allclose(w[0:6], a, atol=1e-6 * scale)
    sens = _basis_sensitivity(a, lambda ang: C.box_known_answer(
        m, q, v, box, lambda n: C.rotated_frame(C.make_frame(n), ang))[0])
    assert sens > 0.02 * scale, (sens, scale)


@pytest.fixture(scope="module")
def leg_model():
    return C.leg_pair_model()


def test_leg_pair_invweight_is_the_compiled_one(leg_model):
    """The independent body_invweight0 the leg-pair answer uses equals the compiled constant the
    implementations read (tran of the contact's regulariser)."""
    m, invw = leg_model
    np.testing.assert_allclose(np.array(m.body_invweight0[:]), invw, rtol=1e-6, atol=1e-15)


@pytest.mark.parametrize("branch", ["ty", "tz"])
def test_leg_spheres_sliding_use_the_documented_frame(leg_model, branch):
    m, invw = leg_model
    q, v, p = C.leg_pair_state(m, invw, branch, seed=3)
    _, _, w, pipe, _ = O.mj_step(m, q, v, np.zeros(18), np.zeros(12), nsteps=1)
    a, act, P = C.leg_pair_known_answer(m, q, v, p, invw)
    assert int(pipe[_abi.P_NCON]) == 1 and 0 < sum(act) < 4
    scale = np.abs(a).max()
    np.testing.assert_allclose(w, a, atol=1e-6 * scale)
    sens = _basis_sensitivity(a, lambda ang: C.leg_pair_known_answer(
        m, q, v, p, invw, lambda n: C.rotated_frame(C.make_frame(n), ang))[0])
    assert sens > 0.02 * scale, (sens, scale)
