"""Long horizon at the headline geometry: 4096 envs, random commands, on-device auto-reset
(episode length 500), U(-1,1) actions, 5000 env steps as fused 100-step rollouts -- ten episodes
per env slot, with falls, terminations and truncations along the way; flat, with configs[2]'s
domain randomisation, and with per-env terrain (10 box slots, 5-10 boxes per env; the oracle step
then runs on each sampled env's own DR row or boxes).

Per rollout, over every env and step of the trajectory: obs / reward / done finite, |obs| within
the clip, done in {0, 1}, reward in range.  At the end: the state record finite, base quaternions
unit, velocities bounded, episodes really restarted (terminations and truncations both seen), and
one further step on 64 sampled envs against the fp64 oracle from the same states (envs whose
episode ended in that step hold their reset state and are left out; constraint-boundary flips
are counted, bench.one_step_err).  Guards against slow drift, NaN blow-ups and state-record
corruption that a 20-step window cannot show.
"""
import numpy as np
import pytest

import gpu_harness as G
from bench import bench_kwargs, one_step_err
from pupperv3_mjx import MODEL_XML, _abi, wrappers
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu

N, K, CHUNKS, EPISODE = 4096, 100, 50, 500


@pytest.mark.parametrize("variant", ["flat", "dr", "terrain"])
def test_5000_steps_with_auto_reset(require_gpu, tmp_path, variant):
    model_path = MODEL_XML
    if variant == "terrain":  # per-env terrain: 10 box slots, 5-10 boxes of each env's own
        import xml.etree.ElementTree as ET
        from pupperv3_mjx import obstacles
        tree = ET.ElementTree(ET.fromstring(open(MODEL_XML).read()))
        obstacles.add_boxes_to_model(tree, n_boxes=10, x_range=(-5, 5), y_range=(-5, 5), height=0.02, length=6.0)
        model_path = str(tmp_path / "terrain.xml")
        tree.write(model_path, encoding="unicode")
    e = PupperV3Env(**bench_kwargs(model_path, True), num_envs=N)
    try:
        table = terrain = None
        if variant == "dr":  # configs[2]'s domain randomisation, one model row per env
            from pupperv3_mjx import domain_randomization, rng
            sysb, _ = domain_randomization.domain_randomize(e.sys, rng.split(rng.PRNGKey(1000), N))
            e.set_domain_randomization(sysb)
            table = sysb.dr_table().astype(np.float64)
        if variant == "terrain":
            from pupperv3_mjx import obstacles
            terrain = obstacles.sample_terrain(N, 10, (-5, 5), (-5, 5), height=0.02, length=6.0, seed=21, min_boxes=5)
            e.set_terrain(terrain)
        env = wrappers.wrap(e, episode_length=EPISODE)
        st = env.reset(make_keys(21, N))
        rs = np.random.RandomState(21)
        dones = 0
        for c in range(CHUNKS):
            acts = rs.uniform(-1, 1, size=(K, N, 12)).astype(np.float32)
            st, traj = env.rollout(st, acts)
            obs, rew, done = traj["obs"], traj["reward"], traj["done"]
            assert np.all(np.isfinite(obs)) and np.all(np.isfinite(rew)), c
            assert np.all(np.abs(obs) <= 100.0), c
            assert np.all((done == 0) | (done == 1)), c
            assert np.all((rew >= 0) & (rew <= 1e4)), c
            dones += int(done.sum())
        rec = e._get(_abi.F_STATE)
        assert np.all(np.isfinite(rec[:, :_abi.S_RNG]))
        np.testing.assert_allclose(np.linalg.norm(rec[:, 3:7], axis=1), 1.0, atol=1e-5)
        assert np.abs(rec[:, _abi.S_QVEL:_abi.S_QVEL + 18]).max() < 1e3
        ep = e._get(_abi.F_EPISODE)
        assert np.all(ep[:, _abi.EP_STEPS] <= EPISODE)  # every counter restarted within its episode
        # the 5000 steps crossed episode ends: terminations (falls) and truncations (length 500)
        assert dones > N, dones
        err, _ = one_step_err(e, n_sample=64, seed=7, dr_table=table, terrain=terrain, auto_reset=True)
        G.report("long_horizon_5000_" + variant, {"envs": N, "steps": K * CHUNKS, "episode_length": EPISODE, "done_env_steps": dones,
                                       "one_step_vs_fp64": {k: err[k] for k in ("envs", "constraint_flip_envs",
                                                                                "auto_reset_envs_excluded",
                                                                                "qpos_abs_max_unflagged",
                                                                                "qvel_abs_max_unflagged")}})
        assert err["envs"] >= 48, err
        assert err["constraint_flip_envs"] <= err["envs"] // 8, err
        assert err["qpos_abs_max_unflagged"] is not None and err["qpos_abs_max_unflagged"] < 1e-4, err
    finally:
        e.close()
