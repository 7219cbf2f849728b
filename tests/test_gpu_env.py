"""GPU env parity: reset/step of the fused kernel vs the oracle (fp32 build) + reference env tests.

RNG-derived quantities (keys, command, kick, desired orientation, latency choice) must be
bit-exact; physics-derived ones (obs, reward terms) agree to fp32 tolerance: obs |d| <= 5e-3,
reward |d| <= 1e-3 after one step from an identical state (the oracle is re-synced to the
GPU state every step so only one step of error is measured).  A step may exceed these only
where the oracle reports a constraint row on its state-switch point during that step (the
one-iteration Newton solve is discontinuous there), and at most 5% of steps may
(gpu_harness.FlipBudget).
"""
import numpy as np
import pytest

import common
import gpu_harness as G
from oracle import oracle as O
from pupperv3_mjx import _abi
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu
N = 32


@pytest.fixture(scope="module")
def model_path(require_gpu, tmp_path_factory):
    return common.write_model(tmp_path_factory.mktemp("m"), 10)


@pytest.fixture(scope="module")
def env(model_path):
    e = PupperV3Env(**common.fixture_kwargs(model_path), num_envs=N)
    yield e
    e.close()


def _rng_words(rec):
    return rec[:, _abi.S_RNG:_abi.S_RNG + 2].copy().view(np.uint32)


def test_reset_parity(env):
    keys = make_keys(0, N)
    st = env.reset(keys)
    oe = O.OracleEnv(env.sys_model.struct, env.config_struct, precision="f32")
    orr = [oe.reset(keys[i]) for i in range(N)]
    orec = np.array([G.oracle_state_to_record(r["state"]) for r in orr])
    np.testing.assert_array_equal(_rng_words(st._record), _rng_words(orec))
    np.testing.assert_array_equal(st.info["command"], orec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3])
    np.testing.assert_allclose(st.info["desired_world_z_in_body_frame"],
                               orec[:, _abi.S_DESIRED_Z:_abi.S_DESIRED_Z + 3], atol=1e-6)
    np.testing.assert_allclose(st.pipeline_state.q[:, :7], orec[:, :7], atol=1e-6)
    np.testing.assert_allclose(st.obs, np.array([r["obs"] for r in orr]), atol=2e-5)
    assert np.all(st.reward == 0) and np.all(st.done == 0)


def test_step_parity_resynced(env):
    keys = make_keys(1, N)
    st = env.reset(keys)
    oe = O.OracleEnv(env.sys_model.struct, env.config_struct, precision="f32")
    rs = np.random.RandomState(0)
    worst_obs = 0.0
    fb = G.FlipBudget()
    for t in range(40):
        a = rs.uniform(-1, 1, size=(N, 12)).astype(np.float32)
        prev = st
        st = env.step(prev, a)
        for i in range(N):
            o = oe.step(dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64)),
                        a[i].astype(np.float64))
            orec = G.oracle_state_to_record(o["state"])
            assert np.array_equal(_rng_words(st._record[i:i + 1]), _rng_words(orec[None]))
            np.testing.assert_array_equal(st._record[i, _abi.S_KICK:_abi.S_KICK + 2], orec[_abi.S_KICK:_abi.S_KICK + 2])
            np.testing.assert_array_equal(st._record[i, _abi.S_COMMAND:_abi.S_COMMAND + 3],
                                          orec[_abi.S_COMMAND:_abi.S_COMMAND + 3])
            assert st._record[i, _abi.S_STEP] == orec[_abi.S_STEP]
            err = np.abs(st.obs[i] - o["obs"]).max()
            ok = err <= 5e-3 and abs(st.reward[i] - o["reward"]) <= 1e-3 and st.done[i] == o["done"]
            fb.check(ok, o, f"step {t} env {i}")
            if ok:
                worst_obs = max(worst_obs, err)
    fb.finish()
    assert worst_obs <= 5e-3, worst_obs


def test_get_obs_shape_and_range(env):
    """test_environment.py:118-133."""
    st = env.reset(make_keys(0, N))
    assert st.obs.shape == (N, env._observation_history * env.observation_dim)
    assert np.all(st.obs >= -100) and np.all(st.obs <= 100)


def test_get_obs_imu_sampling(model_path):
    """test_environment.py:136-156 through the kernel: latency [0,0,1] reads the 2nd-newest column."""
    e = PupperV3Env(**common.fixture_kwargs(model_path, imu_latency_distribution=[0, 0, 1]), num_envs=4)
    try:
        st = e.reset(make_keys(0, 4))
        buf = np.zeros((4, 6, 3), dtype=np.float32)
        buf[:, :, -2] = np.arange(6)
        st.info["imu_buffer"] = buf
        st = e.step(st, np.zeros((4, 12), dtype=np.float32))
        np.testing.assert_allclose(st.obs[:, :6], np.tile(np.arange(6), (4, 1)), atol=1e-5)
    finally:
        e.close()


def test_rollout_200_steps_command_override(model_path):
    """test_environment.py:167-229 without the video: jit_reset, command [0.5,0,0], 200 steps of ones."""
    e = PupperV3Env(**common.fixture_kwargs(model_path), num_envs=1)
    try:
        st = e.reset(make_keys(0, 1)[0])
        st.info["command"] = np.array([0.5, 0, 0], dtype=np.float32)
        for _ in range(200):
            st = e.step(st, np.ones(12, dtype=np.float32))
            assert np.all(np.isfinite(st.obs)) and np.isfinite(st.reward)
            assert st.obs.shape == (72,)
            assert set(st.metrics) == {"total_dist", *_abi.REWARD_NAMES}
    finally:
        e.close()


def test_domain_randomized_step_parity(model_path):
    from pupperv3_mjx import domain_randomization as dr, rng
    n = 16
    e = PupperV3Env(**common.fixture_kwargs(model_path), num_envs=n)
    try:
        sysb, _ = dr.domain_randomize(e.sys, rng.split(rng.PRNGKey(2), n))
        e.set_domain_randomization(sysb)
        table = sysb.dr_table().astype(np.float64)
        keys = make_keys(4, n)
        st = e.reset(keys)
        a = np.random.RandomState(1).uniform(-1, 1, size=(n, 12)).astype(np.float32)
        st2 = e.step(st, a)
        fb = G.FlipBudget(max_frac=0.1)
        for i in range(n):
            oe = O.OracleEnv(e.sys_model.struct, e.config_struct, dr=table[i], precision="f32")
            o = oe.step(dict(state=G.record_to_oracle_state(st._record[i]), obs=st.obs[i].astype(np.float64)),
                        a[i].astype(np.float64))
            ok = np.abs(st2.obs[i] - o["obs"]).max() <= 5e-3 and abs(st2.reward[i] - o["reward"]) <= 1e-3
            fb.check(ok, o, f"env {i}")
        fb.finish()
    finally:
        e.close()


def test_legacy_rng_split_parity(model_path):
    """jax_threefry_partitionable=False (jax 0.5.0's legacy split/bits layout): reset + steps
    bit-exact in the RNG words and commands against the oracle."""
    n = 8
    e = PupperV3Env(**common.fixture_kwargs(model_path), num_envs=n, rng_partitionable=False)
    try:
        keys = make_keys(6, n, partitionable=False)
        st = e.reset(keys)
        oe = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f32")
        orr = [oe.reset(keys[i]) for i in range(n)]
        orec = np.array([G.oracle_state_to_record(r["state"]) for r in orr])
        np.testing.assert_array_equal(_rng_words(st._record), _rng_words(orec))
        np.testing.assert_array_equal(st.info["command"], orec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3])
        rs = np.random.RandomState(2)
        fb = G.FlipBudget(max_frac=0.1)
        for t in range(5):
            a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
            prev = st
            st = e.step(prev, a)
            for i in range(n):
                o = oe.step(dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64)),
                            a[i].astype(np.float64))
                orr_i = G.oracle_state_to_record(o["state"])
                np.testing.assert_array_equal(_rng_words(st._record[i:i + 1]), _rng_words(orr_i[None]))
                np.testing.assert_array_equal(st._record[i, _abi.S_KICK:_abi.S_KICK + 2], orr_i[_abi.S_KICK:_abi.S_KICK + 2])
                fb.check(np.abs(st.obs[i] - o["obs"]).max() <= 5e-3, o, f"step {t} env {i}")
        fb.finish()
    finally:
        e.close()


def test_collision_reward_terms(env):
    """Robots dropped onto their knees and torso: rewards.py's knee_collision / body_collision
    (geom_collision over the contacts with dist < 0; the kernel counts them from per-pair
    knee/torso counts the host precomputes) against the oracle, plus the other reward terms and
    obs under many simultaneous contacts (the contact cap's deepest-first ranking included)."""
    keys = make_keys(3, N)
    st = env.reset(keys)
    rs = np.random.RandomState(11)
    q = st.pipeline_state.q.copy()
    q[:, 2] = rs.uniform(0.0, 0.05, N)  # torso near the floor: torso and upper legs penetrate
    for i in range(N):  # small random tilt
        ax = rs.normal(size=3)
        ax /= np.linalg.norm(ax)
        ang = rs.uniform(0, 0.6)
        q[i, 3:7] = [np.cos(ang / 2), *(np.sin(ang / 2) * ax)]
    st.pipeline_state.q = q
    rec = st._record.copy()
    rec[:, _abi.S_QPOS:_abi.S_QPOS + 19] = q
    a = np.zeros((N, 12), np.float32)
    out = env.step(st, a)
    oe = O.OracleEnv(env.sys_model.struct, env.config_struct, precision="f32")
    ik = 1 + _abi.REWARD_NAMES.index("knee_collision")
    ib = 1 + _abi.REWARD_NAMES.index("body_collision")
    fb = G.FlipBudget(max_frac=0.1)
    hits_k = hits_b = 0
    for i in range(N):
        o = oe.step(dict(state=G.record_to_oracle_state(rec[i]), obs=st.obs[i].astype(np.float64)),
                    a[i].astype(np.float64))
        gk, gb = out.metrics["knee_collision"][i], out.metrics["body_collision"][i]
        hits_k += o["metrics"][ik] != 0
        hits_b += o["metrics"][ib] != 0
        ok = (gk == np.float32(o["metrics"][ik]) and gb == np.float32(o["metrics"][ib])
              and abs(out.reward[i] - o["reward"]) <= 1e-3 and out.done[i] == o["done"])
        fb.check(ok, o, f"env {i}: knee {gk} vs {o['metrics'][ik]}, body {gb} vs {o['metrics'][ib]}")
    fb.finish()
    # the knee term is exercised; body_collision stays 0 on both sides here: the test model's
    # only torso geom is a visual mesh (contype 0), so no torso pair exists
    assert hits_k >= N // 4 and hits_b == 0, (hits_k, hits_b)
