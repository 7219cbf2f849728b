"""The sphere-box cull of the narrow phase (DevModel::cull_on, pp3_env.hip collision()) is exact.

With obstacle boxes the collision pass skips the pairs after the first 32 whose box lies out of the
robot's reach (body 1's origin farther than the reach outside one of the box's slabs).  Such a pair
cannot come within its margin, so mj_collision's contact set (obstacles.py boxes; reference
environment.py:366) is unchanged: every test below runs the same work with the cull and with every
pair through the narrow phase (PP3_NO_CULL=1 at env creation) and requires bit-identical results.
"""
import numpy as np
import pytest

import common
import gpu_harness as G
from pupperv3_mjx import _abi, obstacles
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def box_path(require_gpu, tmp_path_factory):
    return common.write_model(tmp_path_factory.mktemp("m"), 10)


def _pair(monkeypatch, path, n):
    """(culled env, un-culled env) of the same model."""
    monkeypatch.delenv("PP3_NO_CULL", raising=False)
    a = PupperV3Env(**common.fixture_kwargs(path), num_envs=n)
    monkeypatch.setenv("PP3_NO_CULL", "1")
    b = PupperV3Env(**common.fixture_kwargs(path), num_envs=n)
    monkeypatch.delenv("PP3_NO_CULL")
    assert a._L.pp3_narrow_cull(a._h) == 1 and b._L.pp3_narrow_cull(b._h) == 0
    return a, b


@pytest.mark.parametrize("terrain", [False, True])
def test_cull_physics_bit_identical(box_path, monkeypatch, terrain):
    n = 256
    a, b = _pair(monkeypatch, box_path, n)
    try:
        m = a.sys_model.struct
        qpos, qvel, qws, ctrl = common.states_on_boxes(m, n, seed=11)
        if terrain:
            t = common.terrain_under(qpos[:, 0:2], 10, seed=5)
            a.set_terrain(t)
            b.set_terrain(t)
        ra = G.gpu_physics(a, qpos, qvel, qws, ctrl, 5)
        rb = G.gpu_physics(b, qpos, qvel, qws, ctrl, 5)
        for x, y in zip(ra, rb):
            np.testing.assert_array_equal(x, y)
        assert sum(int(ra[3][i][_abi.P_NCON]) > 0 for i in range(n)) > n // 2  # the workload has contacts
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("terrain", [False, True])
def test_cull_env_steps_bit_identical(box_path, monkeypatch, terrain):
    """20 env steps of configs[4]'s workload (robots started over the rails), fused rollout."""
    n = 512
    a, b = _pair(monkeypatch, box_path, n)
    try:
        keys = make_keys(0, n)
        sa, sb = a.reset(keys), b.reset(keys)
        rows = common.model_terrain_rows(a.sys_model.struct)  # [x, y, z, quat, half] per box
        if terrain:
            t = common.terrain_under(np.zeros((n, 2)), 10, seed=2)
            a.set_terrain(t)
            b.set_terrain(t)
            rows = t[:, 0]  # every env over its own slot-0 rail
        specs = [obstacles.BoxSpec("", float(r[0]), float(r[1]), tuple(float(v) for v in r[3:7]),
                                   tuple(float(v) for v in r[7:10])) for r in rows]
        rec = sa._record.copy()
        rec[:, _abi.S_QPOS:_abi.S_QPOS + 2] = obstacles.rail_start_xy(specs, n, seed=4)
        for e in (a, b):
            e._put(_abi.F_STATE, rec)
        acts = np.random.RandomState(9).uniform(-1, 1, size=(20, n, 12)).astype(np.float32)
        _, ta = a.rollout(sa, acts)
        _, tb = b.rollout(sb, acts)
        np.testing.assert_array_equal(a._get(_abi.F_STATE), b._get(_abi.F_STATE))
        for k in ("obs", "reward", "done"):
            np.testing.assert_array_equal(ta[k], tb[k])
    finally:
        a.close()
        b.close()


def test_cull_policy_rollout_bit_identical(box_path, monkeypatch):
    """The fused policy rollout (8-wave workgroups, each wave's envs with their own cached near-box
    masks) on per-env terrain: the same actions and end state with and without the cull."""
    from pupperv3_mjx import export
    from test_gpu_policy import _policy
    n, K = 40, 10
    a, b = _pair(monkeypatch, box_path, n)
    dp = export.DevicePolicy(_policy([72, 256, 128, 128, 24], "elu"))
    try:
        keys = make_keys(4, n)
        sa, sb = a.reset(keys), b.reset(keys)
        t = common.terrain_under(sa._record[:, _abi.S_QPOS:_abi.S_QPOS + 2].astype(np.float64), 10, seed=5)
        a.set_terrain(t)
        b.set_terrain(t)
        sa, ta = a.rollout_policy(sa, dp, K)
        sb, tb = b.rollout_policy(sb, dp, K)
        np.testing.assert_array_equal(ta["action"], tb["action"])
        np.testing.assert_array_equal(sa._record, sb._record)
        assert sa.pipeline_state.contact.ncon.sum() > 0
    finally:
        dp.close()
        a.close()
        b.close()


@pytest.mark.parametrize("nboxes,want", [(0, 0), (1, 1), (16, 1), (17, 0)])
def test_cull_applies_up_to_160_pairs(require_gpu, tmp_path, nboxes, want):
    """The cull needs 1..32 boxes and at most 160 candidate pairs (16 boxes for the 8 spheres);
    other models evaluate every pair (flat ground: the one 32-pair batch)."""
    e = PupperV3Env(**common.fixture_kwargs(common.write_model(tmp_path, nboxes)), num_envs=2)
    try:
        assert e._L.pp3_narrow_cull(e._h) == want
    finally:
        e.close()
