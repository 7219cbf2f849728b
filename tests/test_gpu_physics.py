"""GPU physics parity: the HIP substep kernel vs the CPU oracle on identical seeded states.

Tolerances (fp32 kernel vs fp64 oracle), stated per quantity:
  one substep   : |dqpos| <= 2e-5, |dqvel| <= 3e-3 (abs), median |dqvel| <= 1e-4, contact counts equal
  reference bar : the same errors of the fp32 *oracle* vs the fp64 oracle (the kernel must not be
                  more than 5x worse than a plain fp32 restatement of the same algorithm)
  1000 substeps : standing PD hold, relative qpos drift <= 1e-4 (SURVEY 8d C1 benign trajectory)
"""
import numpy as np
import pytest

import common
import gpu_harness as G
from pupperv3_mjx import _abi
from pupperv3_mjx.environment import PupperV3Env

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env64(require_gpu, tmp_path_factory):
    path = common.write_model(tmp_path_factory.mktemp("m"), 0)
    e = PupperV3Env(**common.fixture_kwargs(path), num_envs=64)
    yield e
    e.close()


@pytest.mark.parametrize("nsteps", [1, 5])
def test_substep_parity_random_states(env64, nsteps):
    m = env64.sys_model.struct
    qpos, qvel, qws, ctrl = common.random_physics_states(64, seed=nsteps)
    gq, gv, gw, gp = G.gpu_physics(env64, qpos, qvel, qws, ctrl, nsteps)
    oq, ov, ow, op = G.oracle_physics(m, qpos, qvel, qws, ctrl, nsteps)
    fq, fv, fw, fp = G.oracle_physics(m, qpos, qvel, qws, ctrl, nsteps, precision="f32")
    assert np.all(np.isfinite(gq)) and np.all(np.isfinite(gv))
    eq, ev = np.abs(gq - oq).max(), np.abs(gv - ov).max()
    fq_e, fv_e = np.abs(fq - oq).max(), np.abs(fv - ov).max()
    assert eq <= max(2e-5 * nsteps, 5 * fq_e), (eq, fq_e)
    assert ev <= max(3e-3, 5 * fv_e), (ev, fv_e)
    assert np.median(np.abs(gv - ov)) <= 1e-4
    if nsteps == 1:
        np.testing.assert_array_equal(gp[:, _abi.P_NCON], op[:, _abi.P_NCON])


@pytest.mark.parametrize("nsteps", [1, 3])
def test_joint_limit_rows_parity(env64, nsteps):
    """Every hinge pushed 0.02-0.2 rad past one of its limits (alternating sides): 12 active
    limit rows per env (mj_instantiateLimit compaction, limit rows of the Newton solve and the
    limit-row branch of the Jacobian row products), against the oracle."""
    m = env64.sys_model.struct
    rng_ = np.ctypeslib.as_array(m.jnt_range)[1:]
    assert np.all(np.ctypeslib.as_array(m.jnt_limited)[1:])
    qpos, qvel, qws, ctrl = common.random_physics_states(64, seed=20 + nsteps)
    rs = np.random.RandomState(nsteps)
    for i in range(64):
        over = rs.uniform(0.02, 0.2, 12)
        hi = (np.arange(12) + i) % 2 == 1
        qpos[i, 7:] = np.where(hi, rng_[:, 1] + over, rng_[:, 0] - over)
        qpos[i, 2] = 0.5  # in the air: limit rows only (no contacts)
    qvel *= 0.1
    gq, gv, _, gp = G.gpu_physics(env64, qpos, qvel, qws, ctrl, nsteps)
    oq, ov, _, op = G.oracle_physics(m, qpos, qvel, qws, ctrl, nsteps)
    fq, fv, _, _ = G.oracle_physics(m, qpos, qvel, qws, ctrl, nsteps, precision="f32")
    assert np.all(np.isfinite(gq)) and np.all(np.isfinite(gv))
    eq, ev = np.abs(gq - oq).max(), np.abs(gv - ov).max()
    fq_e, fv_e = np.abs(fq - oq).max(), np.abs(fv - ov).max()
    assert eq <= max(2e-5 * nsteps, 5 * fq_e), (eq, fq_e)
    assert ev <= max(3e-3, 5 * fv_e), (ev, fv_e)
    # the limits push the joints back towards their ranges
    back = np.where((np.arange(12)[None, :] + np.arange(64)[:, None]) % 2 == 1, -1.0, 1.0)
    assert np.mean(back * (gq[:, 7:] - qpos[:, 7:]) > 0) > 0.9


def test_free_fall_exact(env64):
    n = 64
    qpos = np.zeros((n, 19))
    qpos[:, 2] = 1.0
    qpos[:, 3] = 1
    qpos[:, 7:] = common.DEFAULT_POSE
    ctrl = np.tile(common.DEFAULT_POSE, (n, 1))
    _, _, gw, gp = G.gpu_physics(env64, qpos, np.zeros((n, 18)), np.zeros((n, 18)), ctrl, 1)
    np.testing.assert_allclose(gw[:, :3], np.tile([0, 0, -9.81], (n, 1)), atol=1e-5)
    np.testing.assert_allclose(gw[:, 3:], 0, atol=1e-5)
    assert np.all(gp[:, _abi.P_NCON] == 0)


def test_standing_hold_1000_substeps(env64):
    n = 64
    qpos = np.zeros((n, 19))
    qpos[:, 2] = 0.17
    qpos[:, 3] = 1
    qpos[:, 7:] = common.DEFAULT_POSE
    z = np.zeros((n, 18))
    ctrl = np.tile(common.DEFAULT_POSE, (n, 1))
    gq, gv, _, gp = G.gpu_physics(env64, qpos, z, z, ctrl, 1000)
    oq, ov, _, op = G.oracle_physics(env64.sys_model.struct, qpos[:1], z[:1], z[:1], ctrl[:1], 1000)
    rel = np.abs(gq - oq[0]).max() / np.abs(oq[0]).max()
    assert rel <= 1e-4, rel
    assert np.all(gp[:, _abi.P_NCON] == 4)


def test_dr_substep_parity(env64):
    from pupperv3_mjx import domain_randomization as dr, rng
    m = env64.sys_model.struct
    out, _ = dr.domain_randomize(env64.sys, rng.split(rng.PRNGKey(3), 64))
    table = out.dr_table()
    env64.set_domain_randomization(out)
    try:
        qpos, qvel, qws, ctrl = common.random_physics_states(64, seed=9)
        gq, gv, _, _ = G.gpu_physics(env64, qpos, qvel, qws, ctrl, 2)
        oq, ov, _, _ = G.oracle_physics(m, qpos, qvel, qws, ctrl, 2, dr=table.astype(np.float64))
        assert np.abs(gq - oq).max() <= 5e-5
        assert np.abs(gv - ov).max() <= 5e-3
        assert np.median(np.abs(gv - ov)) <= 1e-4
    finally:
        env64.set_domain_randomization(None)
