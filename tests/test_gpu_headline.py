"""The kernel at the headline launch geometries of BASELINE.json (not just 1-64 envs).

configs[1]: 4096 envs (2048 one-wave workgroups: every CU holds a full generation), flat,
fixed command (0.5, 0, 0), no DR.  configs[3] per GPU: 8192 envs (two generations), commands
sampled at reset and resampled every 500 steps.  Plus an odd batch (4097: the last wave's
second half recomputes env N-1 and must store nothing).

20 env steps of U(-1,1) actions each; property checks on every env (finite, obs within the clip,
shapes, done/reward ranges, RNG words advanced and pairwise distinct), then one further step
compared against the fp32 oracle (re-synced) on 64 envs sampled across the grid -- the first
and the last workgroup included -- with the same per-term tolerances as test_gpu_rewards.
"""
import numpy as np
import pytest

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


def _run(require_gpu, n, random_commands, name):
    env = PupperV3Env(**bench_kwargs(MODEL_XML, random_commands), num_envs=n)
    try:
        keys = make_keys(7, n)
        st = env.reset(keys)
        if not random_commands:
            st.info["command"][:] = [0.5, 0.0, 0.0]
        rng0 = st.info["rng"].copy()
        rs = np.random.RandomState(1)
        for _ in range(20):
            st = env.step(st, rs.uniform(-1, 1, size=(n, 12)).astype(np.float32))
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
        oe = O.OracleEnv(env.sys_model.struct, env.config_struct, precision="f32")
        scales = np.array(env.config_struct.reward_scales[:])
        fb = G.FlipBudget(max_frac=0.02, name=name)
        stats = G.TermStats()
        for i in _sample_ids(n):
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
        G.report(name, {"envs": n, "worst": {k: float(f"{v:.3g}") for k, v in stats.worst.items()}})
        fb.finish()
    finally:
        env.close()


def test_configs1_4096_envs(require_gpu):
    _run(require_gpu, 4096, False, "headline_4096")


def test_configs3_8192_envs_random_commands(require_gpu):
    _run(require_gpu, 8192, True, "headline_8192")


def test_odd_batch_4097_envs(require_gpu):
    _run(require_gpu, 4097, False, "headline_4097")
