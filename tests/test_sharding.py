"""Multi-process env sharding on CPU (gloo, world_size 2): SURVEY.md 8(e).

Each rank takes its contiguous shard of a global batch (pupperv3_mjx.sharding), steps it with
the CPU oracle (the GPU kernel is not available here; the sharding logic is the same code the
bench uses), and the per-step learner gather (sharding.gather_batch) reassembles obs / reward /
done.  The gathered batch must equal a single-process run of the whole batch bit-for-bit:
envs are independent and keys depend only on the global env id.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import common
from oracle import oracle as O
from pupperv3_mjx import sharding
from pupperv3_mjx.environment import make_keys

G_ENVS, STEPS = 7, 3  # ragged: 4 + 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rollout(model, cfg, keys, actions):
    oe = O.OracleEnv(model, cfg)
    states = [oe.reset(k) for k in keys]
    out = []
    for t in range(actions.shape[0]):
        states = [oe.step(s, actions[t, i]) for i, s in enumerate(states)]
        out.append((np.array([s["obs"] for s in states]), np.array([s["reward"] for s in states]),
                    np.array([s["done"] for s in states])))
    return out


def _worker(rank, world, port, path, ret):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model, cfg, _ = common.env_model_and_config(path)
        start, n = sharding.shard_bounds(G_ENVS, world, rank)
        keys = sharding.shard_keys(0, G_ENVS, world, rank)
        acts = np.random.RandomState(5).uniform(-1, 1, size=(STEPS, G_ENVS, 12))[:, start:start + n]
        per_step = _rollout(model, cfg, keys, acts)
        if rank == 0:
            ret["gathered"] = []
        for obs, rew, done in per_step:
            o, r, d = sharding.gather_batch(torch.from_numpy(obs).float(), torch.from_numpy(rew).float(),
                                            torch.from_numpy(done).float(), G_ENVS)
            if rank == 0:
                ret["gathered"] = ret["gathered"] + [(o.numpy(), r.numpy(), d.numpy())]
    finally:
        dist.destroy_process_group()


def test_shard_bounds_cover_exactly_once():
    for g in (2, 7, 4096, 8193):
        for w in (1, 2, 3, 8):
            if g < w:
                continue
            spans = [sharding.shard_bounds(g, w, r) for r in range(w)]
            assert sum(c for _, c in spans) == g
            assert [s for s, _ in spans] == list(np.cumsum([0] + [c for _, c in spans[:-1]]))
    with pytest.raises(ValueError):
        sharding.shard_bounds(1, 2, 0)


def test_shard_keys_are_global_key_rows():
    full = make_keys(3, 10)
    rows = np.concatenate([sharding.shard_keys(3, 10, 4, r) for r in range(4)])
    np.testing.assert_array_equal(rows, full)


def test_two_rank_gloo_gather_matches_single_process(tmp_path):
    path = common.write_model(tmp_path, 0)
    with mp.Manager() as mgr:
        ret = mgr.dict()
        mp.spawn(_worker, args=(2, _free_port(), path, ret), nprocs=2, join=True)
        gathered = list(ret["gathered"])
    model, cfg, _ = common.env_model_and_config(path)
    acts = np.random.RandomState(5).uniform(-1, 1, size=(STEPS, G_ENVS, 12))
    ref = _rollout(model, cfg, make_keys(0, G_ENVS), acts)
    assert len(gathered) == STEPS
    for (go, gr, gd), (ro, rr, rd) in zip(gathered, ref):
        np.testing.assert_array_equal(go, ro.astype(np.float32))
        np.testing.assert_array_equal(gr, rr.astype(np.float32))
        np.testing.assert_array_equal(gd, rd.astype(np.float32))
