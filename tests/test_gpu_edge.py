"""GPU edge cases through the C ABI vs the oracle: obstacle (sphere-box) contacts, contact-cap
overflow ranking, masked reset, single-env / ragged batches, maximum history and latency lengths.

Tolerances as in test_gpu_physics.py / test_gpu_env.py (fp32 kernel vs fp64/fp32 oracle):
  physics  : |dqpos| <= 2e-5 per substep (or 5x the fp32 oracle's own error), |dqvel| <= 3e-3,
             contact counts and contact geom pairs equal after one substep
  env step : obs |d| <= 5e-3, reward |d| <= 1e-3, RNG words / command / step bit-exact
"""
import numpy as np
import pytest

import common
import gpu_harness as G
from oracle import oracle as O
from pupperv3_mjx import _abi
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def box_path(require_gpu, tmp_path_factory):
    return common.write_model(tmp_path_factory.mktemp("m"), 10)


def _box_ids(model):
    return {int(model.cgeom_id[g]) for g in range(model.ncgeom) if model.cgeom_type[g] == _abi.GEOM_BOX}


def _contact_set(pipe):
    n = int(pipe[_abi.P_NCON])
    g = pipe[_abi.P_CON_GEOM:_abi.P_CON_GEOM + 2 * n].reshape(n, 2)
    return sorted(map(tuple, g.astype(int).tolist()))


def _physics_compare(env, m, qpos, qvel, qws, ctrl, nsteps, ncon_max=0, spread=5):
    gq, gv, _, gp = G.gpu_physics(env, qpos, qvel, qws, ctrl, nsteps)
    oq, ov, op, fq, fv = [], [], [], [], []
    for i in range(qpos.shape[0]):
        q, v, _, p, _ = O.mj_step(m, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=nsteps, ncon_max=ncon_max)
        q32, v32, _, _, _ = O.mj_step(m, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=nsteps, ncon_max=ncon_max,
                                      precision="f32")
        oq.append(q); ov.append(v); op.append(p); fq.append(q32); fv.append(v32)
    oq, ov, op, fq, fv = map(np.array, (oq, ov, op, fq, fv))
    assert np.all(np.isfinite(gq)) and np.all(np.isfinite(gv))
    eq, ev = np.abs(gq - oq).max(), np.abs(gv - ov).max()
    assert eq <= max(2e-5 * nsteps, spread * np.abs(fq - oq).max()), eq
    assert ev <= max(3e-3, spread * np.abs(fv - ov).max()), ev
    return gp, op


@pytest.mark.parametrize("nsteps,cap", [(1, 0), (3, 0), (1, 16), (3, 16)])
def test_sphere_box_contact_parity(box_path, nsteps, cap):
    """cap 0 = default contact cap (8 deepest); 16 = the larger kernel instance."""
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=64, max_contacts=cap)
    try:
        m = e.sys_model.struct
        assert e.config_struct.ncon_max == cap
        qpos, qvel, qws, ctrl = common.states_on_boxes(m, 64, seed=nsteps)
        gp, op = _physics_compare(e, m, qpos, qvel, qws, ctrl, nsteps, ncon_max=cap)
        if nsteps == 1:
            boxes = _box_ids(m)
            n_box = 0
            for i in range(64):
                gs, os_ = _contact_set(gp[i]), _contact_set(op[i])
                assert gs == os_, (i, gs, os_)
                n_box += sum(1 for a, b in gs if a in boxes or b in boxes)
            assert n_box >= 16, n_box  # the states really exercise the sphere-box collider
    finally:
        e.close()


@pytest.mark.parametrize("z", [0.5, 0.16])
def test_self_contact_dense_hessian_path(box_path, z):
    """Leg-leg sphere contacts couple two legs: the Newton Hessian is no longer arrowhead in the
    usual order; the kernel counts one leg of the pair with the base block (ldl_arrow_solve_b) --
    in the air, z=0.5, and near the ground, z=0.16."""
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=32)
    try:
        m = e.sys_model.struct
        qpos, qvel, qws, ctrl = common.states_with_self_contact(m, e.sys_model.jnt_range, 32, seed=int(z * 100), z=z)
        for nsteps in (1, 3):
            gp, op = _physics_compare(e, m, qpos, qvel, qws, ctrl, nsteps)
            if nsteps == 1:
                for i in range(32):
                    assert _contact_set(gp[i]) == _contact_set(op[i]), i
    finally:
        e.close()


def test_disjoint_leg_pairs_dense_fallback(box_path):
    """Two disjoint pairs of legs in contact (e.g. front-right/back-right and front-left/back-left):
    no leg is common to every coupling, so moving one leg into the base block cannot restore the
    arrowhead structure and the kernel factors the Hessian densely (dense_search's fallback)."""
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=8)
    try:
        m = e.sys_model.struct
        # waves of two envs: (disjoint, disjoint) and (one pair, disjoint) -- either way the wave
        # falls back to the dense factorisation
        d = common.states_with_self_contact(m, e.sys_model.jnt_range, 6, seed=5, kind="disjoint")
        o = common.states_with_self_contact(m, e.sys_model.jnt_range, 2, seed=6)
        order = [0, 1, 2, 3, 6, 4, 7, 5]  # rows 6, 7 = the one-pair states, each paired with a disjoint one
        qpos, qvel, qws, ctrl = (np.concatenate([x, y])[order] for x, y in zip(d, o))
        # one of these states is ill-conditioned (the fp32 oracle itself drifts 2.5e-5 after one
        # step); the kernel's dense LDL^T orders its operations differently: 10x the fp32 spread
        for nsteps in (1, 3):
            gp, op = _physics_compare(e, m, qpos, qvel, qws, ctrl, nsteps, spread=10)
            if nsteps == 1:
                for i in range(8):
                    assert _contact_set(gp[i]) == _contact_set(op[i]), i
    finally:
        e.close()


def test_contact_cap_overflow_keeps_deepest(box_path):
    """More penetrating pairs than the cap: the kernel and the oracle keep the same deepest set."""
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=64, max_contacts=8)
    try:
        m = e.sys_model.struct
        qpos, qvel, qws, ctrl = common.states_on_boxes(m, 64, seed=11, z_range=(0.085, 0.10))
        qpos[:, 7:] = (np.array(common.DEFAULT_POSE) + np.tile([0, 0.0, 0.6, 0, 0.0, -0.6], 2)  # knees down
                       + np.random.RandomState(12).uniform(-0.1, 0.1, size=(64, 12)))  # no exact depth ties
        gp, op = _physics_compare(e, m, qpos, qvel, qws, ctrl, 1, ncon_max=8)
        full = [O.mj_step(m, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=1, ncon_max=16)[3] for i in range(64)]
        overflow = sum(1 for p in full if p[_abi.P_NCON] > 8)
        assert overflow >= 4, overflow
        for i in range(64):
            assert gp[i][_abi.P_NCON] == op[i][_abi.P_NCON] <= 8
            assert _contact_set(gp[i]) == _contact_set(op[i]), i
    finally:
        e.close()


def test_masked_reset_touches_only_masked_envs(box_path):
    from pupperv3_mjx import _lib
    n = 8
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=n)
    try:
        st = e.reset(make_keys(0, n))
        st = e.step(st, np.zeros((n, 12), dtype=np.float32))
        before = e._get(_abi.F_STATE)
        obs_before = st.obs.copy()
        mask = np.array([1, 0, 0, 1, 0, 1, 0, 0], dtype=np.uint8)
        keys = make_keys(5, n)
        kb = _lib.DeviceBuffer(keys.nbytes, e.device)
        mb = _lib.DeviceBuffer(n, e.device)
        kb.upload(keys)
        mb.upload(mask)
        e.reset_device(kb.ptr.value, mb.ptr.value)
        e.synchronize()
        after = e._get(_abi.F_STATE)
        obs_after = e._get(_abi.F_OBS)
        kb.free(); mb.free()
        full = e.reset(keys)
        for i in range(n):
            if mask[i]:
                np.testing.assert_array_equal(after[i], full._record[i])
                np.testing.assert_array_equal(obs_after[i], full.obs[i])
            else:
                np.testing.assert_array_equal(after[i], before[i])
                np.testing.assert_array_equal(obs_after[i], obs_before[i])
    finally:
        e.close()


@pytest.mark.parametrize("n", [1, 3])
def test_single_and_ragged_batches(box_path, n):
    e = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=n)
    try:
        keys = make_keys(2, n)
        st = e.reset(keys if n > 1 else keys[0])
        oe = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f32")
        rs = np.random.RandomState(3)
        fb = G.FlipBudget(max_frac=0.1)
        for _ in range(10):
            a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
            prev = st
            st = e.step(prev, a if n > 1 else a[0])
            rec_prev = prev._record.reshape(n, -1)
            for i in range(n):
                o = oe.step(dict(state=G.record_to_oracle_state(rec_prev[i]),
                                 obs=np.asarray(prev.obs).reshape(n, -1)[i].astype(np.float64)),
                            a[i].astype(np.float64))
                rec = st._record.reshape(n, -1)[i]
                orec = G.oracle_state_to_record(o["state"])
                np.testing.assert_array_equal(rec[_abi.S_RNG:_abi.S_RNG + 2].view(np.uint32),
                                              orec[_abi.S_RNG:_abi.S_RNG + 2].view(np.uint32))
                ok = (np.abs(np.asarray(st.obs).reshape(n, -1)[i] - o["obs"]).max() <= 5e-3
                      and abs(np.asarray(st.reward).reshape(n)[i] - o["reward"]) <= 1e-3)
                fb.check(ok, o)
        fb.finish()
    finally:
        e.close()


def test_max_history_and_latency_lengths(box_path):
    """observation_history 15 (environment.py:338 comment), 4-long action latency, 3-long IMU latency."""
    n = 16
    kw = common.fixture_kwargs(box_path, observation_history=15, latency_distribution=[0.1, 0.2, 0.3, 0.4],
                               imu_latency_distribution=[0.2, 0.3, 0.5])
    e = PupperV3Env(**kw, num_envs=n)
    try:
        assert e.stride == 98 + 12 * 4 + 6 * 3
        st = e.reset(make_keys(9, n))
        assert st.obs.shape == (n, 36 * 15)
        oe = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f32")
        rs = np.random.RandomState(4)
        fb = G.FlipBudget()
        for t in range(20):
            a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
            prev = st
            st = e.step(prev, a)
            for i in range(n):
                o = oe.step(dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64)),
                            a[i].astype(np.float64))
                orec = G.oracle_state_to_record(o["state"])
                ok = (np.abs(st.obs[i] - o["obs"]).max() <= 5e-3 and abs(st.reward[i] - o["reward"]) <= 1e-3
                      and np.abs(st._record[i, _abi.S_ACT_BUF:] - orec[_abi.S_ACT_BUF:]).max() <= 5e-3)
                fb.check(ok, o, f"step {t} env {i}")
        fb.finish()
    finally:
        e.close()


def test_results_independent_of_batch_layout(box_path):
    """Envs are independent: the same keys and actions give bit-identical records, obs, rewards
    and dones whether the envs run in one handle or split over two handles (the sharded
    multi-GPU layout; shards start at even env ids, so wave partners are unchanged).  An odd
    split changes wave partners; then an env whose partner has a leg-leg contact takes the dense
    factorisation with it and may differ at the rounding level ("Wave partners")."""
    n, split = 64, 32
    kw = common.fixture_kwargs(box_path, terminal_body_z=0.0, kick_probability=0.5)
    full = PupperV3Env(**kw, num_envs=n)
    a_part = PupperV3Env(**kw, num_envs=split)
    b_part = PupperV3Env(**kw, num_envs=n - split)
    try:
        keys = make_keys(11, n)
        s_full = full.reset(keys)
        s_a = a_part.reset(keys[:split])
        s_b = b_part.reset(keys[split:])
        rs = np.random.RandomState(7)
        for _ in range(12):
            act = rs.uniform(-2, 2, size=(n, 12)).astype(np.float32)
            s_full = full.step(s_full, act)
            s_a = a_part.step(s_a, act[:split])
            s_b = b_part.step(s_b, act[split:])
            rec = np.concatenate([s_a._record, s_b._record])
            np.testing.assert_array_equal(s_full._record.view(np.uint32), rec.view(np.uint32))
            np.testing.assert_array_equal(s_full.obs, np.concatenate([s_a.obs, s_b.obs]))
            np.testing.assert_array_equal(s_full.reward, np.concatenate([s_a.reward, s_b.reward]))
            np.testing.assert_array_equal(s_full.done, np.concatenate([s_a.done, s_b.done]))
    finally:
        full.close(); a_part.close(); b_part.close()


def test_create_rejects_two_sided_limit_margin(require_gpu):
    """The kernel keeps at most one limit row per hinge (NLMAX = 12): a model whose joint range is
    narrower than twice its margin (both sides could be violated at once) is rejected at create."""
    import common
    from pupperv3_mjx import _lib
    m = common.pd_model().struct
    m.jnt_margin[3] = 0.6 * (m.jnt_range[3][1] - m.jnt_range[3][0])
    with pytest.raises(_lib.PupperHipError, match="twice the margin"):
        G.env_with_model(common.MODEL_XML, m, 2)


def test_unallocated_field_copy_and_bad_create_fail_loudly(box_path):
    """Auto-reset fields exist only after pp3_set_auto_reset: copying one before raises instead of
    reading a null device pointer; a pp3_create that fails (bad contact cap) leaves nothing behind
    and the next create works."""
    from pupperv3_mjx import _lib
    env = PupperV3Env(**common.fixture_kwargs(box_path), num_envs=3)
    try:
        out = np.empty((3, _abi.EP_STRIDE), dtype=np.float32)
        with pytest.raises(_lib.PupperHipError, match="not allocated"):
            _lib.check(env._L.pp3_copy_field_to_host(env._h, _abi.F_EPISODE, out.ctypes.data_as(_lib.C.c_void_p),
                                                     out.nbytes))
    finally:
        env.close()
    with pytest.raises(_lib.PupperHipError, match="ncon_max"):
        PupperV3Env(**common.fixture_kwargs(box_path), num_envs=3, max_contacts=12)
    PupperV3Env(**common.fixture_kwargs(box_path), num_envs=3).close()
