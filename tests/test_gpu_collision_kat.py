"""Collision known answers on the kernel (through the C ABI's raw physics step): every contact
distance in the kernel's pipeline record equals the closed-form signed distance recomputed from
the record's own body poses (tests/collision_geometry.py, MuJoCo's documented plane-sphere,
sphere-sphere and sphere-box semantics), and the contact set is exactly the candidate pairs within
the margin, the cap deepest when more hit.  This pins the kernel's narrow phase without the
oracle (test_collision_kat.py is the oracle's side).

Tolerance: 3e-6 m on distances (the record is fp32; geom centres sit up to ~5 m from the origin,
where an fp32 coordinate's spacing is 4.8e-7, and the closed form composes a body pose from the
recorded fp32 position and quaternion)."""
import numpy as np
import pytest

import collision_geometry as CG
import common
import gpu_harness as G
from pupperv3_mjx import _abi
from pupperv3_mjx.environment import PupperV3Env

pytestmark = pytest.mark.gpu
TOL = 3e-6


@pytest.fixture(scope="module")
def box_path(require_gpu, tmp_path_factory):
    return common.write_model(tmp_path_factory.mktemp("m"), 10)


@pytest.mark.parametrize("cap,z_range", [(8, (0.085, 0.175)), (16, (0.085, 0.175)), (8, (0.04, 0.08))])
def test_kernel_contact_distances_equal_closed_form_on_boxes(box_path, cap, z_range):
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=64, max_contacts=cap)
    try:
        m = e.sys_model.struct
        qpos, qvel, qws, ctrl = common.states_on_boxes(m, 64, seed=cap + int(100 * z_range[0]), z_range=z_range)
        _, _, _, pipes = G.gpu_physics(e, qpos, qvel, qws, ctrl, 1)
        n_all = n_box = n_capped = 0
        worst = 0.0
        for i in range(64):
            n, nb, err = CG.check_record(m, pipes[i], cap, tol=TOL)
            n_all += n
            n_box += nb
            n_capped += int(pipes[i][_abi.P_NHIT]) > cap
            worst = max(worst, err)
        assert n_box >= 16 and n_all > n_box, (n_all, n_box)
        assert n_capped >= (8 if z_range[0] < 0.08 else 0)
        print(f"collision KAT cap={cap} z={z_range}: {n_all} contacts ({n_box} sphere-box, "
              f"{n_capped} capped envs), worst |dist - closed form| {worst:.2e}")
    finally:
        e.close()


def test_kernel_leg_leg_sphere_pairs_equal_closed_form(box_path):
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=8)
    try:
        m = e.sys_model.struct
        qpos, qvel, qws, ctrl = common.states_with_self_contact(m, e.sys_model.jnt_range, 8, seed=7)
        _, _, _, pipes = G.gpu_physics(e, qpos, qvel, qws, ctrl, 1)
        for i in range(8):
            CG.check_record(m, pipes[i], 8, tol=TOL)
    finally:
        e.close()


@pytest.mark.parametrize("region", sorted(CG.REGIONS))
def test_kernel_sphere_box_normal_by_region(tmp_path, require_gpu, region):
    """The kernel's sphere-box normal per region (collision_geometry.ball_box_model): one substep
    from rest accelerates the ball along the region's outward normal only (fp32: tangential
    <= 1e-3 m/s^2 = 1e-4 g, angular <= 0.05 rad/s^2; a wrong normal gives O(g), O(g / r))."""
    path = common.write_model(tmp_path, 1)
    m, q, u = CG.ball_box_model(path, region)
    e = G.env_with_model(path, m, 2)
    try:
        qpos = np.tile(q, (2, 1))
        _, _, qacc, pipes = G.gpu_physics(e, qpos, np.zeros((2, 18)), np.zeros((2, 18)), np.zeros((2, 12)), 1)
        assert int(pipes[0][_abi.P_NCON]) == 1
        tang, ang, an = CG.normal_residuals(qacc[0], u)
        print(f"normal KAT {region}: tangential {tang:.2e} m/s^2, angular {ang:.2e} rad/s^2, a.u {an:.4f}")
        assert tang <= 1e-3 and ang <= 5e-2, (tang, ang)
        assert an > -9.81 + 1.0, an
    finally:
        e.close()
