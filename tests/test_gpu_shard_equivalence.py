"""Sharding at configs[3]'s full size, checked on the kernel: 8192 envs stepped as
ONE batch and as contiguous shards built from the global key rows (sharding.shard_keys) end in
bit-identical state records, observations, rewards and dones -- the property the multi-GPU bench
rests on (a sharded run reproduces the single-GPU run env for env, with no collective in the step).

Shards are cut at wave pairs (sharding.shard_bounds: every shard starts at an even env id), so
each env keeps its wave partner: three ranks split 8192 envs as 2732 | 2730 | 2730.  (Cut at an odd
id -- 2731 | 2731 | 2730 -- 3 % of the state words differed after 25 steps, by <= 1e-4 relative:
a wave with a leg-leg contact in either env takes one Newton factorisation for both)
Random commands (resampled inside the step), 20 fused steps then 5 single-step launches.
"""
import numpy as np
import pytest

from bench import bench_kwargs
from pupperv3_mjx import MODEL_XML, sharding
from pupperv3_mjx.environment import PupperV3Env

pytestmark = pytest.mark.gpu

G_ENVS, K_FUSED, K_SINGLE = 8192, 20, 5


def _run(keys, acts):
    env = PupperV3Env(**bench_kwargs(MODEL_XML, True), num_envs=len(keys))
    try:
        st = env.reset(keys)
        st, traj = env.rollout(st, acts[:K_FUSED])
        for t in range(K_FUSED, K_FUSED + K_SINGLE):
            st = env.step(st, acts[t])
        return (np.array(st._record), np.array(st.obs), np.array(st.reward), np.array(st.done),
                np.array(traj["obs"]), np.array(traj["reward"]), np.array(traj["done"]))
    finally:
        env.close()


@pytest.mark.parametrize("world", [2, 3])
def test_shards_reproduce_the_full_batch(require_gpu, world):
    rs = np.random.RandomState(11)
    acts = rs.uniform(-1, 1, size=(K_FUSED + K_SINGLE, G_ENVS, 12)).astype(np.float32)
    full = _run(sharding.shard_keys(0, G_ENVS, 1, 0), acts)
    parts = []
    for r in range(world):
        start, n = sharding.shard_bounds(G_ENVS, world, r)
        parts.append(_run(sharding.shard_keys(0, G_ENVS, world, r), np.ascontiguousarray(acts[:, start:start + n])))
    names = ("state record", "obs", "reward", "done", "trajectory obs", "trajectory reward", "trajectory done")
    for k, name in enumerate(names):
        axis = 1 if name.startswith("trajectory") else 0
        joined = np.concatenate([p[k] for p in parts], axis=axis)
        np.testing.assert_array_equal(joined.view(np.uint32), full[k].view(np.uint32), err_msg=name)

