"""Multi-rank runs on ONE GPU through the loopback test transport.

RCCL allows one rank per device, so on the one-GPU pool the multi-rank code paths -- several rank
processes, pp3_gather's grouped send/recv to a root (its per-rank placement dst + r * count) and
its all-gather, the all-reduces behind the barrier and the max-over-ranks timing, bench.py's own
launcher and its gather_check -- would otherwise never run.  `make loopback` builds the same
sources as the product library with the collectives routed to tests/loopback/loopback_rccl.cpp
(RCCL's API over files, blocking, host-staged; every rank on device 0).  What this covers is the
callers' logic above RCCL; RCCL's own xGMI transport still needs a multi-GPU node (the driver's
scaling bench, test_gpu_comm.py::test_two_rank_gather_on_two_devices).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import common
from pupperv3_mjx import sharding
from pupperv3_mjx.environment import PupperV3Env

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LOOPBACK_LIB = os.path.join(HERE, "loopback", "libpupper_hip_loopback.so")


@pytest.fixture
def loopback_env(require_gpu, tmp_path):
    if not os.path.exists(LOOPBACK_LIB) or not os.path.exists(os.path.join(HERE, "loopback", "libpp3_loopback_rccl.so")):
        pytest.fail("loopback test build missing: make -C pupperv3-mjx_amd/csrc loopback (__graft_entry__.build)")
    d = tmp_path / "lb"
    d.mkdir()
    return dict(os.environ, PP3_LIB_PATH=LOOPBACK_LIB, PP3_ALLOW_DIAG_BUILD="1", PP3_LOOPBACK_DIR=str(d),
                PP3_RDZV_DIR=str(d), PP3_LAUNCH_ID=f"lb{os.getpid()}.{tmp_path.name}", PP3_WORKER_DEVICE="0",
                PP3_BENCH_DEVICE="0")


@pytest.mark.parametrize("world,G", [(2, 9), (3, 10)])
def test_gather_across_rank_processes(loopback_env, tmp_path, world, G):
    """`world` rank processes each step their ragged shard of a G-env batch and hand the learner
    rows to root 0 (grouped send/recv) and to everyone (all-gather).  Every slot must hold its
    rank's own pack_rows (padding rows zero), and the unpacked batch must equal ONE env of G envs
    stepped with the same keys and actions, bit for bit."""
    worker = os.path.join(HERE, "_comm_worker.py")
    procs = [subprocess.Popen([sys.executable, worker, str(r), str(world), str(tmp_path), str(G)], env=loopback_env)
             for r in range(world)]
    try:
        codes = [p.wait(timeout=150) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert codes == [0] * world, codes
    mine = [np.load(tmp_path / f"rows_{r}.npy") for r in range(world)]
    nmax = sharding.max_shard(G, world)
    root = np.load(tmp_path / "gather_root_0.npy")
    for r in range(world):
        assert mine[r].shape[0] == nmax
        np.testing.assert_array_equal(root[r * nmax:(r + 1) * nmax], mine[r])
        np.testing.assert_array_equal(np.load(tmp_path / f"allgather_{r}.npy"), np.concatenate(mine))
    # the K-step unroll handed over once (pp3_gather_rollout): rank r's [K][nmax][D + 2] block
    tmine = [np.load(tmp_path / f"traj_rows_{r}.npy") for r in range(world)]
    K, W = tmine[0].shape[0], tmine[0].shape[2]
    troot = np.load(tmp_path / "traj_root_0_0.npy").reshape(world, K, nmax, W)
    for r in range(world):
        np.testing.assert_array_equal(troot[r], tmine[r])
        np.testing.assert_array_equal(np.load(tmp_path / f"traj_allgather_{r}.npy").reshape(world, K, nmax, W), troot)
    # the sharded job reproduces the single-GPU batch env for env
    env = PupperV3Env(**common.fixture_kwargs(common.MODEL_XML), num_envs=G)
    try:
        st = env.reset(sharding.shard_keys(5, G, 1, 0))
        st = env.step(st, np.random.RandomState(2).uniform(-1, 1, size=(G, 12)).astype(np.float32))
        obs, rew, done = sharding.unpack_gathered(root, G, world)
        np.testing.assert_array_equal(obs, st.obs)
        np.testing.assert_array_equal(rew, st.reward)
        np.testing.assert_array_equal(done, st.done)
    finally:
        env.close()


def _bench(env, *extra, timeout=240):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2", "--envs", "512",
           "--no-cpu-baseline", "--no-latency-floor", "--no-extras", "--no-prewarm", *extra]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 alone prints the JSON line
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 3, 4])
def test_bench_launches_ranks_and_checks_the_gather(loopback_env, world):
    """`python bench.py --gpus N` as the driver runs it, without a launcher: the parent starts N
    rank processes, they join one communicator, time with barrier + max over ranks, and finish
    with gather_check (per-rank checksums of the packed rows vs what landed at the root and at
    every rank)."""
    d = _bench(loopback_env, "--gpus", str(world))
    assert d["n_gpus"] == world
    assert d["config"]["global_envs"] == 512 * world
    assert d["config"]["comm"] == "RCCL (pp3_comm)"
    gc = d["config"]["gather_check"]
    assert gc["root0"] == "ok" and gc["allgather"] == "ok" and gc["failing_receivers"] == 0, gc
    assert gc["ranks"] == world
    assert d["per_step_launch"]["bit_equal_to_rollout"]


@pytest.mark.parametrize("root", [0, -1])
def test_bench_per_step_gather(loopback_env, root):
    """configs[3]'s shape: the per-step hand-over of obs | reward | done to a learner rank (or to
    every rank) inside the timed loop of a 2-rank job."""
    d = _bench(loopback_env, "--gpus", "2", "--gather", "--gather-root", str(root), "--random-commands")
    assert d["n_gpus"] == 2
    g = d["config"]["gather"]
    assert g["root"] == root and g["rows_per_rank"] == 512 and g["ms_per_gather"] > 0
    assert d["config"]["gather_check"]["failing_receivers"] == 0


@pytest.mark.parametrize("root", [0, -1])
def test_bench_unroll_gather(loopback_env, root):
    """configs[3] with one hand-over per unroll (--gather-mode unroll): the K timed steps are ONE
    fused rollout and its K-step trajectory goes to the learner rank (or every rank) in one
    pp3_gather_rollout; the fused launch is still bit-equal to the single-step replay."""
    d = _bench(loopback_env, "--gpus", "2", "--gather", "--gather-mode", "unroll", "--gather-root", str(root),
               "--random-commands")
    assert d["n_gpus"] == 2
    g = d["config"]["gather"]
    assert g["mode"] == "unroll" and g["root"] == root and g["steps_per_gather"] == 4
    assert g["rows_per_rank"] == 4 * 512 and g["ms_per_gather"] > 0
    assert d["per_step_launch"]["bit_equal_to_rollout"]
    assert d["config"]["gather_check"]["failing_receivers"] == 0


def test_bench_under_torch_distributed_run(loopback_env):
    """The driver's multi-GPU command: `python -m torch.distributed.run --nnodes=1 --nproc-per-node 2
    --master-addr 127.0.0.1 --master-port P bench.py --gpus 2 ...` -- the launcher sets RANK /
    LOCAL_RANK / WORLD_SIZE, the ranks find each other through the launch key of their shared
    parent (sharding.launch_key) and report one JSON line."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in loopback_env.items() if k != "PP3_LAUNCH_ID"}  # keyed by the launcher
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--envs", "256", "--no-cpu-baseline", "--no-latency-floor", "--no-extras", "--no-prewarm"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=420, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["comm"] == "RCCL (pp3_comm)"
    assert d["config"]["gather_check"]["failing_receivers"] == 0
