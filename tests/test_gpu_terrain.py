"""Per-env terrain through the C ABI vs the oracle.

The reference's obstacle boxes (obstacles.py:16-57) are static geoms shared by every env.  With
pp3_set_terrain each env holds its own boxes in the model's box-geom slots (some slots absent, so
envs differ in box and contact counts).  The oracle sees env i's terrain as a model whose box
geoms are moved to env i's boxes (common.model_with_terrain), so the same restated mj_step is
the reference for every env.  Parity unpinned against MJX itself (no MJX here; the static-box
path it extends is pinned as in test_gpu_edge.py).

Tolerances as in test_gpu_edge.py: |dqpos| <= 2e-5 per substep (or 5x the fp32 oracle's own
error), |dqvel| <= 3e-3, contact geom pairs equal after one substep; env step obs <= 5e-3,
reward <= 1e-3 with the constraint-flip allowance (gpu_harness.FlipBudget).
"""
import numpy as np
import pytest

import common
import gpu_harness as G
from oracle import oracle as O
from pupperv3_mjx import _abi, obstacles
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def box_path(require_gpu, tmp_path_factory):
    return common.write_model(tmp_path_factory.mktemp("m"), 10)


def _contact_set(pipe):
    n = int(pipe[_abi.P_NCON])
    g = pipe[_abi.P_CON_GEOM:_abi.P_CON_GEOM + 2 * n].reshape(n, 2)
    return sorted(map(tuple, g.astype(int).tolist()))


def test_static_layout_as_terrain_matches_model_boxes(box_path):
    """Every env given the model's own boxes as terrain == the static-box path."""
    n = 64
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=n)
    try:
        m = e.sys_model.struct
        assert e.terrain_slots == 10
        qpos, qvel, qws, ctrl = common.states_on_boxes(m, n, seed=3)
        a = G.gpu_physics(e, qpos, qvel, qws, ctrl, 3)
        e.set_terrain(np.broadcast_to(common.model_terrain_rows(m), (n, 10, 10)))
        b = G.gpu_physics(e, qpos, qvel, qws, ctrl, 3)
        e.set_terrain(None)
        c = G.gpu_physics(e, qpos, qvel, qws, ctrl, 3)
        # same boxes; only the box rotation's rounding differs (f32 of the same f64 rotation, from
        # a quaternion rounded to f32 first), so the results agree to fp32 noise
        np.testing.assert_allclose(a[0], b[0], rtol=0, atol=2e-5)
        np.testing.assert_allclose(a[1], b[1], rtol=0, atol=1e-3)
        for x, y in zip(a[:3], c[:3]):
            np.testing.assert_array_equal(x, y)  # back to the static boxes exactly
        assert sum(_contact_set(a[3][i]) == _contact_set(b[3][i]) for i in range(n)) == n
    finally:
        e.close()


@pytest.mark.parametrize("nsteps", [1, 3])
def test_per_env_terrain_physics_parity(box_path, nsteps):
    n = 64
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=n)
    try:
        m = e.sys_model.struct
        qpos, qvel, qws, ctrl = common.random_physics_states(n, seed=20 + nsteps, mode="stand")
        rs = np.random.RandomState(nsteps)
        qpos[:, 0:2] = rs.uniform(-3, 3, size=(n, 2))
        qpos[:, 2] = rs.uniform(0.15, 0.175, size=n)
        qvel *= 0.3
        terrain = common.terrain_under(qpos[:, 0:2], 10, seed=nsteps)
        assert np.any(np.all(terrain[:, :, 7:10] == 0, axis=2))  # some envs have absent slots
        e.set_terrain(terrain)
        gq, gv, _, gp = G.gpu_physics(e, qpos, qvel, qws, ctrl, nsteps)
        box_ids = {int(m.cgeom_id[g]) for g in common.terrain_slots(m)}
        n_box = 0
        for i in range(n):
            mi = common.model_with_terrain(m, terrain[i])
            q, v, _, p, _ = O.mj_step(mi, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=nsteps)
            q32, v32, _, _, _ = O.mj_step(mi, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=nsteps, precision="f32")
            assert np.abs(gq[i] - q).max() <= max(2e-5 * nsteps, 5 * np.abs(q32 - q).max()), i
            assert np.abs(gv[i] - v).max() <= max(3e-3, 5 * np.abs(v32 - v).max()), i
            if nsteps == 1:
                gs, os_ = _contact_set(gp[i]), _contact_set(p)
                assert gs == os_, (i, gs, os_)
                n_box += sum(1 for a, b in gs if a in box_ids or b in box_ids)
        if nsteps == 1:
            assert n_box >= 16, n_box  # the per-env rails really are under the robots
    finally:
        e.close()


def test_per_env_terrain_env_step_parity(box_path):
    """reset -> per-env terrain around each robot -> env steps, each env against an oracle env
    built on its own terrain (state re-synced every step, as in test_gpu_env.py)."""
    n = 8
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=n)
    try:
        m = e.sys_model.struct
        st = e.reset(make_keys(7, n))
        terrain = common.terrain_under(st._record[:, _abi.S_QPOS:_abi.S_QPOS + 2].astype(np.float64), 10, seed=7)
        e.set_terrain(terrain)
        oes = [O.OracleEnv(common.model_with_terrain(m, terrain[i]), e.config_struct, precision="f32")
               for i in range(n)]
        rs = np.random.RandomState(8)
        fb = G.FlipBudget()
        for t in range(6):
            a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
            prev = st
            st = e.step(prev, a)
            for i in range(n):
                o = oes[i].step(dict(state=G.record_to_oracle_state(prev._record[i]),
                                     obs=prev.obs[i].astype(np.float64)), a[i].astype(np.float64))
                np.testing.assert_array_equal(st._record[i, _abi.S_RNG:_abi.S_RNG + 2].view(np.uint32),
                                              G.oracle_state_to_record(o["state"])[_abi.S_RNG:_abi.S_RNG + 2]
                                              .view(np.uint32))
                ok = np.abs(st.obs[i] - o["obs"]).max() <= 5e-3 and abs(st.reward[i] - o["reward"]) <= 1e-3
                fb.check(ok, o, f"step {t} env {i}")
                assert st.done[i] == o["done"], (t, i)
        fb.finish()
    finally:
        e.close()


def test_terrain_argument_errors(box_path):
    from pupperv3_mjx import _lib
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=4)
    try:
        with pytest.raises(ValueError):
            e.set_terrain(np.zeros((3, 10, 10), np.float32))
        with pytest.raises(_lib.PupperHipError):
            e.set_terrain(np.zeros((4, 9, 10), np.float32) + 1)
        e.set_terrain(obstacles.sample_terrain(4, 10, (-5, 5), (-5, 5), seed=1, min_boxes=0))
        e.set_terrain(None)
    finally:
        e.close()
