"""The multi-GPU collective through the C ABI on one GPU.

pp3_gather on a one-rank RCCL communicator: the device pack of obs | reward | done (with padding
rows past the shard) must equal sharding.pack_rows of the env's own fields, for the gather to
a root and for the all-gather; the reductions the bench's max-over-ranks timing uses must
return their inputs.  Several ranks need several GPUs (RCCL allows one rank per device):
test_two_rank_gather_on_two_devices runs the grouped send/recv and the all-gather across two
processes when the box has two devices and is skipped otherwise; the N > 1 path also runs, with
its checksum check, in every multi-GPU bench (bench.py gather_check).  On the one-GPU pool,
test_gpu_multirank.py runs 2 and 3 rank processes through the same code above RCCL (the
loopback test transport); RCCL's own transport between devices stays unverified until a
multi-GPU node runs one of the above.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

import common
from pupperv3_mjx import _abi, _lib, sharding
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm(require_gpu, tmp_path_factory):
    import os
    os.environ["PP3_RDZV_DIR"] = str(tmp_path_factory.mktemp("rdzv"))
    c = sharding.Comm(0, 1, 0, tag="_test")
    yield c
    c.close()


@pytest.mark.parametrize("root", [0, -1])
def test_gather_packs_learner_rows(comm, root):
    n, nmax = 37, 40
    env = PupperV3Env(**common.fixture_kwargs(common.MODEL_XML), num_envs=n)
    try:
        st = env.reset(make_keys(3, n))
        st = env.step(st, np.random.RandomState(0).uniform(-1, 1, size=(n, 12)).astype(np.float32))
        width = env.observation_size + 2
        dst = _lib.DeviceBuffer(nmax * width * 4, env.device)
        # poison the destination so the padding rows are checked as written, not assumed
        dst.upload(np.full(nmax * width, np.nan, np.float32))
        comm.gather(env, nmax, dst.ptr.value, root=root)
        env.synchronize()
        got = np.empty((nmax, width), np.float32)
        dst.download(got)
        dst.free()
        np.testing.assert_array_equal(got, sharding.pack_rows(st.obs, st.reward, st.done, nmax))
        o, r, d = sharding.unpack_gathered(got, n, 1)
        np.testing.assert_array_equal(o, st.obs)
    finally:
        env.close()


@pytest.mark.parametrize("root", [0, -1])
def test_gather_rollout_packs_the_unroll(comm, root):
    """pp3_gather_rollout on a one-rank communicator: the K-step trajectory of one fused rollout
    (device buffers written by pp3_rollout), packed as [K][nmax][D + 2] with zero padding rows, must
    equal sharding.pack_traj_rows of the same trajectory -- and that trajectory equals K single
    steps (rollout() is bit-equal to step())."""
    n, nmax, K = 37, 40, 4
    env = PupperV3Env(**common.fixture_kwargs(common.MODEL_XML), num_envs=n)
    try:
        st = env.reset(make_keys(9, n))
        acts = np.random.RandomState(4).uniform(-1, 1, size=(K, n, 12)).astype(np.float32)
        D = env.observation_size
        W = D + 2
        tr = [_lib.DeviceBuffer(K * n * D * 4, env.device), _lib.DeviceBuffer(K * n * 4, env.device),
              _lib.DeviceBuffer(K * n * 4, env.device)]
        abuf = _lib.DeviceBuffer(acts.nbytes, env.device)
        abuf.upload(acts)
        env.rollout_device(abuf.ptr.value, n * 12, K, tr[1].ptr.value, tr[2].ptr.value, tr[0].ptr.value)
        dst = _lib.DeviceBuffer(K * nmax * W * 4, env.device)
        dst.upload(np.full(K * nmax * W, np.nan, np.float32))
        comm.gather_rollout(env, tr[0].ptr.value, tr[1].ptr.value, tr[2].ptr.value, K, nmax, dst.ptr.value, root=root)
        env.synchronize()
        got = np.empty((K, nmax, W), np.float32)
        dst.download(got)
        # the same K steps through the host API (a fresh env from the same keys)
        e2 = PupperV3Env(**common.fixture_kwargs(common.MODEL_XML), num_envs=n)
        try:
            s2 = e2.reset(make_keys(9, n))
            want = []
            for t in range(K):
                s2 = e2.step(s2, acts[t])
                want.append(sharding.pack_rows(s2.obs, s2.reward, s2.done, nmax))
        finally:
            e2.close()
        np.testing.assert_array_equal(got, np.stack(want))
        for b in tr + [abuf, dst]:
            b.free()
    finally:
        env.close()


def test_gather_rejects_short_nmax(comm):
    env = PupperV3Env(**common.fixture_kwargs(common.MODEL_XML), num_envs=8)
    try:
        env.reset(make_keys(0, 8))
        with pytest.raises(_lib.PupperHipError):
            comm.gather(env, 7, None, root=0)
    finally:
        env.close()


def test_allreduce_and_barrier(comm):
    np.testing.assert_array_equal(comm.allreduce([1.5, -2.0, 3.25], "max"), [1.5, -2.0, 3.25])
    np.testing.assert_array_equal(comm.allreduce([1.5, -2.0], "sum"), [1.5, -2.0])
    comm.barrier()
    assert comm._L.pp3_comm_world(comm._h) == 1 and comm._L.pp3_comm_rank(comm._h) == 0


def test_gather_at_configs3_shard_size(comm):
    """configs[3]'s per-GPU shard (8192 envs, random commands) after steps: the hand-over rows of
    every env equal the env's own obs | reward | done, bit for bit (pack + RCCL on the env stream,
    no host synchronisation between the step and the gather)."""
    from bench import bench_kwargs
    n = 8192
    env = PupperV3Env(**bench_kwargs(common.MODEL_XML, True), num_envs=n, pipeline_output=False)
    try:
        env.reset(make_keys(5, n))
        width = env.observation_size + 2
        dst = _lib.DeviceBuffer(n * width * 4, env.device)
        acts = _lib.DeviceBuffer(n * 12 * 4, env.device)
        rs = np.random.RandomState(2)
        for _ in range(3):
            env.synchronize()  # the previous step has consumed the action buffer
            acts.upload(rs.uniform(-1, 1, size=(n, 12)).astype(np.float32))
            env.step_device(acts.ptr.value)
            comm.gather(env, n, dst.ptr.value, root=0)
        env.synchronize()
        got = np.empty((n, width), np.float32)
        dst.download(got)
        obs, rew, done = env._get(_abi.F_OBS), env._get(_abi.F_REWARD), env._get(_abi.F_DONE)
        np.testing.assert_array_equal(got, sharding.pack_rows(obs, rew.reshape(n), done.reshape(n), n))
        dst.free()
        acts.free()
    finally:
        env.close()


def test_two_rank_gather_on_two_devices(require_gpu, tmp_path):
    """Two ranks on two devices (tests/_comm_worker.py): each steps its own shard and gathers to
    root 0 and then all-gathers; every receiver's slots must equal each rank's own pack_rows."""
    if _lib.load().pp3_device_count() < 2:
        pytest.skip("needs 2 GPUs: RCCL allows one rank per device")
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_comm_worker.py")
    env = dict(os.environ, PP3_LAUNCH_ID=f"test{os.getpid()}", PP3_RDZV_DIR=str(tmp_path))
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", str(tmp_path)], env=env) for r in range(2)]
    for p in procs:
        assert p.wait(timeout=120) == 0
    mine = [np.load(tmp_path / f"rows_{r}.npy") for r in range(2)]
    nmax = mine[0].shape[0]
    root = np.load(tmp_path / "gather_root_0.npy")
    for r in range(2):
        np.testing.assert_array_equal(root[r * nmax:(r + 1) * nmax], mine[r])
        ag = np.load(tmp_path / f"allgather_{r}.npy")
        np.testing.assert_array_equal(ag, np.concatenate(mine))
    tmine = [np.load(tmp_path / f"traj_rows_{r}.npy") for r in range(2)]
    K, W = tmine[0].shape[0], tmine[0].shape[2]
    troot = np.load(tmp_path / "traj_root_0_0.npy").reshape(2, K, nmax, W)
    for r in range(2):
        np.testing.assert_array_equal(troot[r], tmine[r])
        np.testing.assert_array_equal(np.load(tmp_path / f"traj_allgather_{r}.npy").reshape(2, K, nmax, W), troot)
