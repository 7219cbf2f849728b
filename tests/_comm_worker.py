"""One rank of tests/test_gpu_comm.py::test_two_rank_gather_on_two_devices and
tests/test_gpu_multirank.py (not a test module):
  python tests/_comm_worker.py RANK WORLD OUTDIR [GLOBAL_ENVS]
Rank r steps its shard of a global batch (default 9 envs: ragged, 5 + 4 on two ranks) on device r
(PP3_WORKER_DEVICE: every rank on that device -- the loopback transport's one-GPU runs), then
gathers the learner rows to root 0 and all-gathers them; it saves its own pack_rows and what it
received."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import common  # noqa: E402
from pupperv3_mjx import _lib, sharding  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env  # noqa: E402

rank, world, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
G = int(sys.argv[4]) if len(sys.argv) > 4 else 9
device = int(os.environ.get("PP3_WORKER_DEVICE", rank))
start, n = sharding.shard_bounds(G, world, rank)
nmax = sharding.max_shard(G, world)
comm = sharding.Comm(rank, world, device)
env = PupperV3Env(**common.fixture_kwargs(common.MODEL_XML), num_envs=n, device=device)
st = env.reset(sharding.shard_keys(5, G, world, rank))
acts = np.random.RandomState(2).uniform(-1, 1, size=(G, 12)).astype(np.float32)[start:start + n]
st = env.step(st, acts)
mine = sharding.pack_rows(st.obs, st.reward, st.done, nmax)
np.save(os.path.join(out, f"rows_{rank}.npy"), mine)
W = env.observation_size + 2
dst = _lib.DeviceBuffer(world * nmax * W * 4, env.device)
comm.gather(env, nmax, dst.ptr.value if rank == 0 else None, root=0)
env.synchronize()
if rank == 0:
    full = np.empty((world * nmax, W), np.float32)
    dst.download(full)
    np.save(os.path.join(out, "gather_root_0.npy"), full)
comm.barrier()
comm.gather(env, nmax, dst.ptr.value, root=-1)
env.synchronize()
full = np.empty((world * nmax, W), np.float32)
dst.download(full)
np.save(os.path.join(out, f"allgather_{rank}.npy"), full)
comm.barrier()
# a K-step unroll (one fused rollout writing its trajectory on the device) handed over ONCE
# (pp3_gather_rollout), to root 0 and to everyone
K = 3
D = env.observation_size
tr = [_lib.DeviceBuffer(K * n * D * 4, env.device), _lib.DeviceBuffer(K * n * 4, env.device),
      _lib.DeviceBuffer(K * n * 4, env.device)]
ua = np.random.RandomState(7).uniform(-1, 1, size=(K, G, 12)).astype(np.float32)[:, start:start + n]
abuf = _lib.DeviceBuffer(ua.nbytes, env.device)
abuf.upload(np.ascontiguousarray(ua))
env.rollout_device(abuf.ptr.value, n * 12, K, tr[1].ptr.value, tr[2].ptr.value, tr[0].ptr.value)
env.synchronize()
got = [np.empty((K, n, D), np.float32), np.empty((K, n), np.float32), np.empty((K, n), np.float32)]
for b, a in zip(tr, got):
    b.download(a)
np.save(os.path.join(out, f"traj_rows_{rank}.npy"), sharding.pack_traj_rows(got[0], got[1], got[2], nmax))
tdst = _lib.DeviceBuffer(world * K * nmax * W * 4, env.device)
for root in (0, -1):
    comm.gather_rollout(env, tr[0].ptr.value, tr[1].ptr.value, tr[2].ptr.value, K, nmax,
                        tdst.ptr.value if (root < 0 or rank == 0) else None, root=root)
    env.synchronize()
    if root < 0 or rank == 0:
        full = np.empty((world * K * nmax, W), np.float32)
        tdst.download(full)
        np.save(os.path.join(out, f"traj_{'root_0' if root == 0 else 'allgather'}_{rank}.npy"), full)
    comm.barrier()
for b in tr + [abuf, tdst]:
    b.free()
dst.free()
env.close()
comm.close()
