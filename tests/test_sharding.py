"""Multi-process env sharding on CPU (gloo, world_size 2): SURVEY.md 8(e).

Each rank takes its contiguous shard of a global batch (pupperv3_mjx.sharding), steps it with
the CPU oracle (the GPU kernel is not available here; the sharding logic is the same code the
bench uses), packs its learner rows exactly as pp3_gather's device pack does
(sharding.pack_rows), and a gloo all-gather stands in for the RCCL collective (torch is used by
this test only, as the CPU transport; the product path is torch-free).  sharding.unpack_gathered
must then give a single-process run of the whole batch bit-for-bit: envs are independent and
keys depend only on the global env id.  The communicator-id rendezvous (file based, no torch)
runs in real processes too.
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
        nmax = sharding.max_shard(G_ENVS, world)
        for obs, rew, done in per_step:
            local = torch.from_numpy(sharding.pack_rows(obs, rew, done, nmax))
            full = torch.empty((world * nmax, local.shape[1]), dtype=torch.float32)
            dist.all_gather_into_tensor(full, local)
            o, r, d = sharding.unpack_gathered(full.numpy(), G_ENVS, world)
            if rank == 0:
                ret["gathered"] = ret["gathered"] + [(o, r, d)]
        # the hand-over once per unroll (pp3_gather_rollout's layout): the K-step trajectory packed
        # as [K][nmax][D + 2] and ONE all-gather
        traj = sharding.pack_traj_rows(*(np.stack([p[i] for p in per_step]) for i in range(3)), nmax)
        local = torch.from_numpy(traj.reshape(STEPS * nmax, -1))
        full = torch.empty((world * STEPS * nmax, local.shape[1]), dtype=torch.float32)
        dist.all_gather_into_tensor(full, local)
        if rank == 0:
            ret["traj"] = sharding.unpack_gathered_rollout(full.numpy(), G_ENVS, world, STEPS)
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


def test_shards_start_at_wave_pairs():
    """Every shard starts at an even env id (the step kernel's wave pairs stay whole), rank 0's is
    the largest, and an even per-rank count E shards E * world envs as E each (the bench)."""
    for g in (3, 7, 11, 4097, 8192, 8193):
        for w in (1, 2, 3, 5, 8):
            if (g + 1) // 2 < w:
                continue
            spans = [sharding.shard_bounds(g, w, r) for r in range(w)]
            assert all(s % 2 == 0 for s, _ in spans), (g, w, spans)
            assert max(c for _, c in spans) == spans[0][1] == sharding.max_shard(g, w)
    for w in (1, 2, 3, 8):
        assert [sharding.shard_bounds(4096 * w, w, r)[1] for r in range(w)] == [4096] * w
    assert [sharding.shard_bounds(8192, 3, r) for r in range(3)] == [(0, 2732), (2732, 2730), (5462, 2730)]


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
        traj = ret["traj"]
    model, cfg, _ = common.env_model_and_config(path)
    acts = np.random.RandomState(5).uniform(-1, 1, size=(STEPS, G_ENVS, 12))
    ref = _rollout(model, cfg, make_keys(0, G_ENVS), acts)
    assert len(gathered) == STEPS
    for (go, gr, gd), (ro, rr, rd) in zip(gathered, ref):
        np.testing.assert_array_equal(go, ro.astype(np.float32))
        np.testing.assert_array_equal(gr, rr.astype(np.float32))
        np.testing.assert_array_equal(gd, rd.astype(np.float32))
    to, tr, td = traj
    for t, (ro, rr, rd) in enumerate(ref):
        np.testing.assert_array_equal(to[t], ro.astype(np.float32))
        np.testing.assert_array_equal(tr[t], rr.astype(np.float32))
        np.testing.assert_array_equal(td[t], rd.astype(np.float32))


def _rdzv_worker(rank, world, d, ret):
    os.environ["PP3_RDZV_DIR"] = d
    os.environ["MASTER_PORT"] = "4242"
    blob = sharding.rendezvous_id(rank, world, lambda: os.urandom(128), timeout_s=30)
    ret[rank] = blob


def test_rendezvous_id_file_exchange(tmp_path):
    """Rank 0's 128-byte communicator id reaches every rank (the RCCL init input), no torch."""
    import multiprocessing as mpc
    with mpc.Manager() as mgr:
        ret = mgr.dict()
        ps = [mpc.Process(target=_rdzv_worker, args=(r, 3, str(tmp_path), ret)) for r in (1, 2, 0)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(60)
            assert p.exitcode == 0
        blobs = [ret[r] for r in range(3)]
    assert len(blobs[0]) == 128 and blobs[0] == blobs[1] == blobs[2]


def test_pack_unpack_ragged():
    rs = np.random.RandomState(0)
    G, world, D = 11, 4, 72
    obs = rs.normal(size=(G, D)).astype(np.float32)
    rew, done = rs.uniform(size=G).astype(np.float32), (rs.uniform(size=G) < 0.3).astype(np.float32)
    nmax = sharding.max_shard(G, world)
    full = np.concatenate([sharding.pack_rows(obs[s:s + n], rew[s:s + n], done[s:s + n], nmax)
                           for s, n in (sharding.shard_bounds(G, world, r) for r in range(world))])
    assert full.shape == (world * nmax, D + 2)
    o, r, d = sharding.unpack_gathered(full, G, world)
    np.testing.assert_array_equal(o, obs)
    np.testing.assert_array_equal(r, rew)
    np.testing.assert_array_equal(d, done)


def test_pack_unpack_rollout_ragged():
    """pack_traj_rows per rank, concatenated in rank order (pp3_gather_rollout's [world][K][nmax][D + 2]),
    then unpack_gathered_rollout: the global K-step trajectory back in env order."""
    rs = np.random.RandomState(1)
    G, world, K, D = 11, 4, 5, 72
    obs = rs.normal(size=(K, G, D)).astype(np.float32)
    rew = rs.uniform(size=(K, G)).astype(np.float32)
    done = (rs.uniform(size=(K, G)) < 0.3).astype(np.float32)
    nmax = sharding.max_shard(G, world)
    full = np.concatenate([sharding.pack_traj_rows(obs[:, s:s + n], rew[:, s:s + n], done[:, s:s + n], nmax)
                           for s, n in (sharding.shard_bounds(G, world, r) for r in range(world))])
    assert full.shape == (world * K, nmax, D + 2)
    o, r, d = sharding.unpack_gathered_rollout(full, G, world, K)
    np.testing.assert_array_equal(o, obs)
    np.testing.assert_array_equal(r, rew)
    np.testing.assert_array_equal(d, done)


def test_sharding_module_is_torch_free():
    import ast
    import inspect
    src = inspect.getsource(sharding)
    names = {a.name for n in ast.walk(ast.parse(src)) if isinstance(n, (ast.Import, ast.ImportFrom))
             for a in n.names}
    mods = {n.module for n in ast.walk(ast.parse(src)) if isinstance(n, ast.ImportFrom) and n.module}
    assert not any(x.split(".")[0] == "torch" for x in names | mods)


def _rdzv_fail_worker(rank, world, d, ret):
    os.environ["PP3_RDZV_DIR"] = d
    os.environ["MASTER_PORT"] = "4343"

    def bad_id():
        raise RuntimeError("no librccl here")
    try:
        sharding.rendezvous_id(rank, world, bad_id, tag="_fail", timeout_s=30)
        ret[rank] = "ok"
    except Exception as exc:  # every rank must fail fast, not at its timeout
        ret[rank] = type(exc).__name__ + ":" + str(exc)


def test_rendezvous_failure_reaches_every_rank(tmp_path):
    """Rank 0's failure to create the id is published, so the other ranks raise at once (bench.py
    then falls back to FileComm on every rank instead of rank 0 waiting out the others' timeout)."""
    import multiprocessing as mpc
    import time
    t0 = time.monotonic()
    with mpc.Manager() as mgr:
        ret = mgr.dict()
        ps = [mpc.Process(target=_rdzv_fail_worker, args=(r, 2, str(tmp_path), ret)) for r in (1, 0)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(60)
        out = dict(ret)
    assert time.monotonic() - t0 < 20
    assert out[0].startswith("RuntimeError:") and "no librccl" in out[0]
    assert out[1].startswith("RuntimeError:") and "no librccl" in out[1]


def _filecomm_worker(rank, world, d, ret):
    fc = sharding.FileComm(rank, world, directory=d, timeout_s=30)
    res = []
    for k in range(5):
        res.append(fc.allreduce([rank + k, -rank], "max").tolist())
        fc.barrier()
        res.append(fc.allreduce([rank + k], "sum").tolist())
    fc.close()
    ret[rank] = res


def test_file_comm_barrier_and_reductions(tmp_path):
    """The host-file fallback of bench.py's barrier / max-over-ranks timing, 3 processes."""
    import multiprocessing as mpc
    world = 3
    with mpc.Manager() as mgr:
        ret = mgr.dict()
        ps = [mpc.Process(target=_filecomm_worker, args=(r, world, str(tmp_path), ret)) for r in (2, 0, 1)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(60)
            assert p.exitcode == 0
        out = [ret[r] for r in range(world)]
    expect = []
    for k in range(5):
        expect.append([world - 1 + k, 0.0])
        expect.append([sum(r + k for r in range(world))])
    for r in range(world):
        assert out[r] == expect
    # only the last round's files are left behind
    assert len(os.listdir(tmp_path)) == world
