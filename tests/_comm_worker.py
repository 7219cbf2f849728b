"""One rank of tests/test_gpu_comm.py::test_two_rank_gather_on_two_devices (not a test module):
  python tests/_comm_worker.py RANK WORLD OUTDIR
Rank r steps its shard of a 9-env global batch (ragged: 5 + 4) on device r, then gathers the
learner rows to root 0 and all-gathers them; it saves its own pack_rows and what it received."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import common  # noqa: E402
from pupperv3_mjx import _lib, sharding  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env  # noqa: E402

rank, world, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
G = 9
start, n = sharding.shard_bounds(G, world, rank)
nmax = sharding.max_shard(G, world)
comm = sharding.Comm(rank, world, rank)
env = PupperV3Env(**common.fixture_kwargs(common.MODEL_XML), num_envs=n, device=rank)
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
dst.free()
env.close()
comm.close()
