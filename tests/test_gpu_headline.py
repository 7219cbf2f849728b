"""The kernel at the headline launch geometries of BASELINE.json (not just 1-64 envs).

configs[1]: 4096 envs (2048 one-wave workgroups: every CU holds a full generation), flat,
fixed command (0.5, 0, 0), no DR; the same with domain randomisation (configs[2]) and with the 10
obstacle boxes (configs[4] per GPU).  configs[3] per GPU: 8192 envs (two generations), commands
sampled at reset and resampled every 500 steps.  Plus an odd batch (4097: the last wave's
second half recomputes env N-1 and must store nothing).  configs[0] (1 env, zero command,
mj_step plumbing) runs as C1 below: 1000 free-running env steps against the fp64 oracle.

20 env steps of U(-1,1) actions each; property checks on every env (finite, obs within the clip,
shapes, done/reward ranges, RNG words advanced and pairwise distinct), then one further step
compared against the fp32 oracle (re-synced) on 64 envs sampled across the grid -- the first
and the last workgroup included -- with the same per-term tolerances as test_gpu_rewards.
"""
import numpy as np
import pytest

import common
import gpu_harness as G
from bench import bench_kwargs
from oracle import oracle as O
from pupperv3_mjx import MODEL_XML, _abi
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu


def _sample_ids(n, k=64, seed=0):
    rs = np.random.RandomState(seed)
    ids = set(rs.choice(n, size=k - 4, replace=False).tolist())
    ids.update({0, 1, n - 2, n - 1})  # first and last workgroup (both halves)
    return sorted(ids)


def _box_contacts(st, box_ids):
    """Per env: number of the last substep's contacts that involve a world box geom."""
    c = st.pipeline_state.contact
    live = np.arange(c.geom1.shape[1])[None, :] < c.ncon[:, None]
    isbox = np.isin(c.geom1, box_ids) | np.isin(c.geom2, box_ids)
    return (live & isbox).sum(axis=1)


def _run(require_gpu, n, random_commands, name, model_path=MODEL_XML, dr=False, start_xy=None, box_ids=None):
    env = PupperV3Env(**bench_kwargs(model_path, random_commands), num_envs=n)
    try:
        table = None
        if dr:  # configs[2]: a domain-randomised model per env (domain_randomization.py:11-18 ranges)
            from pupperv3_mjx import domain_randomization, rng
            sysb, _ = domain_randomization.domain_randomize(env.sys, rng.split(rng.PRNGKey(1000), n))
            env.set_domain_randomization(sysb)
            table = sysb.dr_table().astype(np.float64)
        keys = make_keys(7, n)
        st = env.reset(keys)
        if not random_commands:
            st.info["command"] = np.tile(np.float32([0.5, 0.0, 0.0]), (n, 1))
        if start_xy is not None:  # configs[4]: robots stood over the boxes
            q = st.pipeline_state.q.copy()
            q[:, 0:2] = start_xy
            st.pipeline_state.q = q
        rng0 = st.info["rng"].copy()
        rs = np.random.RandomState(1)
        box_steps = np.zeros(n, dtype=int)  # env steps (of 21) whose last substep touched a box
        for _ in range(20):
            st = env.step(st, rs.uniform(-1, 1, size=(n, 12)).astype(np.float32))
            if box_ids is not None:
                box_steps += _box_contacts(st, box_ids) > 0
        # properties over the whole grid
        assert st.obs.shape == (n, 72) and st.reward.shape == (n,) and st.done.shape == (n,)
        for arr in (st.obs, st.reward, st.done, st._record[:, :_abi.S_RNG], st._metrics_raw):
            assert np.all(np.isfinite(arr))
        assert np.all(np.abs(st.obs) <= 100.0)
        assert np.all((st.done == 0) | (st.done == 1))
        assert np.all((st.reward >= 0) & (st.reward <= 1e4))
        q = st.pipeline_state.q
        np.testing.assert_allclose(np.linalg.norm(q[:, 3:7], axis=1), 1.0, atol=1e-5)
        assert not np.any(np.all(st.info["rng"] == rng0, axis=1))  # every env's key advanced
        assert len({tuple(r) for r in st.info["rng"].tolist()}) == n  # and they stay distinct
        if not random_commands:
            assert np.all(st.info["command"] == np.float32([0.5, 0.0, 0.0]))
        # one more step, sampled envs against the oracle
        a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
        prev = st
        st = env.step(prev, a)
        base = O.OracleEnv(env.sys_model.struct, env.config_struct, precision="f32")
        scales = np.array(env.config_struct.reward_scales[:])
        fb = G.FlipBudget(max_frac=0.01, name=name)
        stats = G.TermStats()
        ids = _sample_ids(n)
        extra = {}
        if box_ids is not None:
            now = _box_contacts(st, box_ids)
            box_steps += now > 0
            extra = {"box_contact_envs_any_step": int((box_steps > 0).sum()),
                     "sampled_envs_with_box_contact": int((box_steps[ids] > 0).sum()),
                     "sampled_envs_box_contact_compared_step": int((now[ids] > 0).sum()),
                     "box_contacts_compared_step": int(now[ids].sum())}
            # the compared envs really are on the obstacle path (verdict r02: a start square
            # that put robots beside the boxes measured the flat workload)
            assert extra["sampled_envs_with_box_contact"] >= len(ids) // 4, extra
        for i in ids:
            oe = base if table is None else O.OracleEnv(env.sys_model.struct, env.config_struct, dr=table[i],
                                                         precision="f32")
            o = oe.step(dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64)),
                        a[i].astype(np.float64))
            orec = G.oracle_state_to_record(o["state"])
            np.testing.assert_array_equal(st._record[i, _abi.S_RNG:_abi.S_RNG + 2].view(np.uint32),
                                          orec[_abi.S_RNG:_abi.S_RNG + 2].view(np.uint32))
            errs = {**G.metric_errors(st._metrics_raw[i], o["metrics"], scales),
                    **G.state_errors(st._record[i], orec, env.config_struct.latency_len,
                                     env.config_struct.imu_latency_len),
                    "qpos": (float(np.abs(st._record[i, :19] - orec[:19]).max()), 1e-4),
                    "obs": (float(np.abs(st.obs[i] - o["obs"]).max()), 5e-3),
                    "done": (abs(float(st.done[i]) - o["done"]), 0.0)}
            bad = G.TermStats.failures(errs)
            if not bad:
                stats.add(errs)
            flip = o["boundary"] > 0 or G.foot_threshold_flip(o["pipe"], env.config_struct.foot_radius)
            fb.check(not bad, dict(o, boundary=int(flip)), f"env {i}: {bad}")
        G.report(name, {"envs": n, **extra, "worst": {k: float(f"{v:.3g}") for k, v in stats.worst.items()}})
        fb.finish()
    finally:
        env.close()


def test_configs1_4096_envs(require_gpu):
    _run(require_gpu, 4096, False, "headline_4096")


def test_configs3_8192_envs_random_commands(require_gpu):
    _run(require_gpu, 8192, True, "headline_8192")


def test_configs2_4096_envs_domain_randomised(require_gpu):
    _run(require_gpu, 4096, False, "headline_4096_dr", dr=True)


def test_configs4_4096_envs_obstacle_boxes(require_gpu, tmp_path):
    """configs[4] per GPU: the 10 obstacles.py boxes of the golden layout (seed 0,
    test_environment.py:18-43: x, y in (-5, 5), length 6) in the model, every robot started over a
    box (obstacles.rail_start_xy) so the sphere-box lanes, variable contact counts and the solver
    work they bring are what the 64 compared envs exercise; the sphere-box contacts are counted
    from the pipeline record and at least a quarter of the compared envs must have had one."""
    import xml.etree.ElementTree as ET
    from pupperv3_mjx import obstacles
    tree = ET.ElementTree(ET.fromstring(open(MODEL_XML).read()))
    kw = dict(n_boxes=10, x_range=(-5, 5), y_range=(-5, 5), height=0.02, length=6.0)
    obstacles.add_boxes_to_model(tree, **kw)
    path = str(tmp_path / "pupper_obstacles.xml")
    tree.write(path, encoding="unicode")
    specs = obstacles.sample_boxes(kw["n_boxes"], kw["x_range"], kw["y_range"], kw["height"], length=kw["length"])
    n = 4096
    _run(require_gpu, n, False, "headline_4096_obstacles", model_path=path,
         start_xy=obstacles.rail_start_xy(specs, n, seed=3), box_ids=_world_box_geoms(path))


def _world_box_geoms(path):
    env_model = common.env_model_and_config(path)[0]
    return np.array([int(env_model.cgeom_id[g]) for g in range(env_model.ncgeom)
                     if env_model.cgeom_type[g] == _abi.GEOM_BOX and env_model.cgeom_bodyid[g] == 0])


def test_odd_batch_4097_envs(require_gpu):
    _run(require_gpu, 4097, False, "headline_4097")


def test_configs0_c1_zero_command_1000_steps(require_gpu):
    """configs[0] at env level: 1 env, flat, command (0,0,0) fixed (zero
    ranges, no orientation command), observation noise, kick and latencies off (latency [1], IMU
    latency [1]), actions 0, 1000 env steps (5000 substeps) FREE-RUNNING on the kernel and on the
    fp64 oracle from the same reset key; qpos / qvel / obs compared at every step.  The fp32 oracle,
    run alongside, calibrates the tolerance: the kernel may drift from fp64 by at most 10x what a
    plain fp32 execution of the same algorithm drifts, floored at 1e-4 (qpos) / 1e-3 (qvel)."""
    kw = common.fixture_kwargs(MODEL_XML, angular_velocity_noise=0.0, gravity_noise=0.0, motor_angle_noise=0.0,
                               last_action_noise=0.0, kick_probability=0.0, latency_distribution=[1.0],
                               imu_latency_distribution=[1.0], linear_velocity_x_range=[0.0, 0.0],
                               linear_velocity_y_range=[0.0, 0.0], angular_velocity_range=[0.0, 0.0],
                               maximum_pitch_command=0.0, maximum_roll_command=0.0)
    env = PupperV3Env(**kw, num_envs=1)
    try:
        key = make_keys(0, 1)
        st = env.reset(key)
        o64 = O.OracleEnv(env.sys_model.struct, env.config_struct, precision="f64")
        o32 = O.OracleEnv(env.sys_model.struct, env.config_struct, precision="f32")
        s64, s32 = o64.reset(key[0]), o32.reset(key[0])
        np.testing.assert_allclose(st._record[0, :19], G.oracle_state_to_record(s64["state"])[:19], atol=1e-6)
        zero = np.zeros(12)
        worst = dict(qpos=0.0, qvel=0.0, obs=0.0, qpos32=0.0, qvel32=0.0)
        for t in range(1000):
            st = env.step(st, np.zeros((1, 12), dtype=np.float32))
            s64, s32 = o64.step(s64, zero), o32.step(s32, zero)
            g, r64 = st._record[0], G.oracle_state_to_record(s64["state"])
            r32 = G.oracle_state_to_record(s32["state"])
            qv = slice(_abi.S_QVEL, _abi.S_QVEL + 18)
            worst["qpos"] = max(worst["qpos"], float(np.abs(g[:19] - r64[:19]).max()))
            worst["qvel"] = max(worst["qvel"], float(np.abs(g[qv] - r64[qv]).max()))
            worst["obs"] = max(worst["obs"], float(np.abs(st.obs[0] - s64["obs"]).max()))
            worst["qpos32"] = max(worst["qpos32"], float(np.abs(r32[:19] - r64[:19]).max()))
            worst["qvel32"] = max(worst["qvel32"], float(np.abs(r32[qv] - r64[qv]).max()))
            assert st.done[0] == s64["done"] == 0, t  # it stands: no termination, no reset
            assert np.all(st.info["command"] == 0.0)
        G.report("configs0_c1", {"steps": 1000, "worst": {k: float(f"{v:.3g}") for k, v in worst.items()}})
        assert worst["qpos"] <= max(1e-4, 10 * worst["qpos32"]), worst
        assert worst["qvel"] <= max(1e-3, 10 * worst["qvel32"]), worst
        assert worst["obs"] <= 5e-3, worst
        # it stood up from the drop and stays standing: base height and tilt at the end
        q = st._record[0, :7]
        up_z = 1.0 - 2.0 * (q[4] ** 2 + q[5] ** 2)  # world z of the body z axis (quat w, x, y, z at 3..6)
        assert 0.1 < q[2] < 0.3 and up_z > 0.9, q
    finally:
        env.close()
