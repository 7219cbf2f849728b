"""Collision known answers on the oracle: every contact distance the narrow phase reports
(oracle/pp3_oracle.c `collision`: plane-sphere, sphere-sphere, sphere-box) equals the closed-form
signed distance recomputed from the geom poses alone (tests/collision_geometry.py), and the contact
set is exactly the candidate pairs within the margin (the 8 or 16 deepest when more hit).  The
kernel's counterpart is tests/test_gpu_collision_kat.py.  The states straddle the obstacles.py
walls (test/test_environment.py:18-43 layout), stand on the floor, or fold two legs into each
other (leg-leg sphere pairs)."""
import numpy as np
import pytest

import collision_geometry as CG
import common
from oracle import oracle as O
from pupperv3_mjx import _abi, mjcf


@pytest.fixture(scope="module")
def box_model(tmp_path_factory):
    return mjcf.load(common.write_model(tmp_path_factory.mktemp("m"), 10))


# (cap, start heights): robots over the walls; low starts overflow the 8-contact cap
BOX_CASES = [(8, (0.085, 0.175)), (16, (0.085, 0.175)), (8, (0.04, 0.08))]


@pytest.mark.parametrize("cap,z_range", BOX_CASES)
def test_contact_distances_equal_closed_form_on_boxes(box_model, cap, z_range):
    m = box_model.struct
    qpos, qvel, qws, ctrl = common.states_on_boxes(m, 48, seed=cap + int(100 * z_range[0]), z_range=z_range)
    n_all = n_box = n_capped = 0
    for i in range(48):
        _, _, _, pipe, _ = O.mj_step(m, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=1, ncon_max=cap)
        n, nb, _ = CG.check_record(m, pipe, cap, tol=1e-12)
        n_all += n
        n_box += nb
        n_capped += int(pipe[_abi.P_NHIT]) > cap
    assert n_box >= 16 and n_all > n_box, (n_all, n_box)  # the sphere-box collider really ran
    assert n_capped >= (8 if z_range[0] < 0.08 else 0)  # the overflow case ranks by depth


def test_contact_distances_equal_closed_form_standing():
    cm = mjcf.load(common.MODEL_XML)
    m = cm.struct
    qpos, qvel, qws, ctrl = common.random_physics_states(32, seed=4, mode="stand")
    n_all = 0
    for i in range(32):
        _, _, _, pipe, _ = O.mj_step(m, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=1)
        n_all += CG.check_record(m, pipe, 8, tol=1e-12)[0]
    assert n_all >= 32


def test_leg_leg_sphere_pairs_equal_closed_form(box_model):
    m = box_model.struct
    qpos, qvel, qws, ctrl = common.states_with_self_contact(m, box_model.jnt_range, 4, seed=7)
    for i in range(4):
        _, _, _, pipe, _ = O.mj_step(m, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=1)
        CG.check_record(m, pipe, 8, tol=1e-12)


def test_sphere_box_regions():
    """The closed form itself, on a unit box: face, edge, corner and inside regions."""
    class M:  # a two-geom stand-in model: sphere (radius 0.1) on body 0, box of half sizes (1, 2, 3)
        cgeom_bodyid = [0, 0]
        cgeom_type = [2, 6]
        cgeom_size = [[0.1, 0, 0], [1.0, 2.0, 3.0]]
        cgeom_quat = [[1.0, 0, 0, 0], [1.0, 0, 0, 0]]
        cgeom_pos = [[0, 0, 0], [0, 0, 0]]
    pipe = np.zeros(400)
    for c, want in [((1.5, 0, 0), 0.4), ((1.5, 2.5, 0), np.hypot(0.5, 0.5) - 0.1),
                    ((2, 3, 4), np.sqrt(3.0) - 0.1), ((0.9, 0, 0), -0.1 - 0.1), ((0, 0, -2.5), -0.5 - 0.1)]:
        M.cgeom_pos = [list(c), [0, 0, 0]]
        assert CG.pair_distance(M, pipe, 0, 1) == pytest.approx(want, abs=1e-12)


@pytest.mark.parametrize("region", sorted(CG.REGIONS))
def test_sphere_box_normal_by_region(tmp_path, region):
    """The contact normal of each sphere-box region (collision_geometry.ball_box_model): one oracle
    substep from rest accelerates the ball along the region's outward normal only."""
    m, q, u = CG.ball_box_model(common.write_model(tmp_path, 1), region)
    out = O.mj_forward(m, q, np.zeros(18), np.zeros(18), np.zeros(12))
    assert int(out["pipe"][_abi.P_NCON]) == 1 and out["nefc"] == 12 + 4  # hinge frictionloss + 4 edges
    tang, ang, an = CG.normal_residuals(out["qacc"], u)
    # (the 1e-9 kg legs and their frictionloss rows leave ~1e-8 / 1e-5; a wrong normal gives O(g), O(g / r))
    assert tang <= 1e-5 and ang <= 1e-3, (tang, ang)
    assert an > -9.81 + 1.0, an  # the contact pushes back
