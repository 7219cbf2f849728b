"""Env sharding across GPUs (one process per GPU) and the learner-batch collective.

SURVEY.md 8(e): envs are independent, so a global batch of G envs is cut into contiguous
per-rank shards (at wave pairs: ``shard_bounds``) with no collective inside the step.  Env i of the global batch gets the same
PRNG key (``jax.random.split(PRNGKey(seed), G)[i]``) whatever the world size, so a sharded run
reproduces the single-GPU run env-for-env.  The only collective is the optional per-step
hand-over of ``obs | reward | done`` to the learner: ``Comm.gather`` -> ``pp3_gather`` (RCCL over
xGMI, on the env's stream, no host sync; include/pupper_hip.h).  No torch anywhere: the RCCL
communicator id is exchanged by a file rendezvous on the node (``rendezvous_id``).

Gathered layout (``pp3_gather``): rank r's ``nmax`` rows of width D + 2 at row r * nmax, rows past
the rank's env count zero; ``pack_rows`` is its numpy statement, ``unpack_gathered`` drops the
padding and returns the global [G, D] / [G] / [G] batch in env-id order.  For a K-step unroll
(``Comm.gather_rollout`` -> ``pp3_gather_rollout``: one collective per unroll, the trajectory of one
fused ``pp3_rollout``) rank r's block is [K][nmax][D + 2] at r * K * nmax rows (``pack_traj_rows``;
``unpack_gathered_rollout`` returns the global [K, G, D] / [K, G] / [K, G] trajectory).
"""
from __future__ import annotations

import ctypes as C
import os
import time
from typing import Callable, Optional, Tuple

import numpy as np

from . import rng


def shard_bounds(global_envs: int, world: int, rank: int) -> Tuple[int, int]:
    """(first env id, env count) of `rank`'s contiguous shard, cut at wave pairs: envs 2p and 2p + 1
    share one wave of the step kernel, and a wave with a leg-leg contact in either env takes one
    Newton factorisation for both, so an env's rounding can depend on its partner.
    Every shard therefore starts at an even env id: each env keeps the partner it has in the
    single-GPU batch and a sharded run reproduces that run bit for bit
    (tests/test_gpu_shard_equivalence.py).  Pairs are dealt with the remainder to the low ranks (rank
    0's shard is the largest); an odd batch's last pair is its lone last env.  With fewer pairs than
    ranks the cut falls back to single envs."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world {world}")
    if global_envs < world:
        raise ValueError(f"{global_envs} envs cannot be sharded over {world} ranks")
    pairs = (global_envs + 1) // 2
    if pairs >= world:
        base, rem = divmod(pairs, world)
        start = 2 * (rank * base + min(rank, rem))
        return start, min(2 * (base + (1 if rank < rem else 0)), global_envs - start)
    base, rem = divmod(global_envs, world)
    count = base + (1 if rank < rem else 0)
    start = rank * base + min(rank, rem)
    return start, count


def shard_keys(seed: int, global_envs: int, world: int, rank: int, partitionable: bool = True) -> np.ndarray:
    """Reset keys of this rank's shard: rows [start, start+count) of split(PRNGKey(seed), G)."""
    start, count = shard_bounds(global_envs, world, rank)
    keys = rng.split(rng.PRNGKey(seed), global_envs, partitionable=partitionable)
    return np.ascontiguousarray(keys[start:start + count])


def max_shard(global_envs: int, world: int) -> int:
    """Rows every rank contributes to the gather (the largest shard: rank 0's)."""
    return shard_bounds(global_envs, world, 0)[1]


def pack_rows(obs, reward, done, nmax: int) -> np.ndarray:
    """numpy statement of pp3_comm.hip's pack_kernel: [nmax, D + 2] = obs | reward | done, zero rows
    past the shard's env count."""
    obs = np.asarray(obs, dtype=np.float32)
    n, D = obs.shape
    out = np.zeros((nmax, D + 2), dtype=np.float32)
    out[:n, :D] = obs
    out[:n, D] = np.asarray(reward, dtype=np.float32).reshape(n)
    out[:n, D + 1] = np.asarray(done, dtype=np.float32).reshape(n)
    return out


def pack_traj_rows(obs, reward, done, nmax: int) -> np.ndarray:
    """numpy statement of pp3_comm.hip's pack_traj_kernel: a K-step trajectory (obs [K, n, D], reward
    / done [K, n]) -> [K, nmax, D + 2], zero rows past the shard's env count."""
    obs = np.asarray(obs, dtype=np.float32)
    return np.stack([pack_rows(obs[t], np.asarray(reward)[t], np.asarray(done)[t], nmax) for t in range(obs.shape[0])])


def unpack_gathered(full, global_envs: int, world: int):
    """[world * nmax, D + 2] gathered rows -> (obs [G, D], reward [G], done [G]) in global env order."""
    full = np.asarray(full)
    nmax = max_shard(global_envs, world)
    rows = [full[r * nmax:r * nmax + shard_bounds(global_envs, world, r)[1]] for r in range(world)]
    out = np.concatenate(rows, 0)
    D = out.shape[1] - 2
    return out[:, :D], out[:, D], out[:, D + 1]


def unpack_gathered_rollout(full, global_envs: int, world: int, nsteps: int):
    """pp3_gather_rollout's [world][K][nmax][D + 2] rows -> (obs [K, G, D], reward [K, G], done [K, G])
    in global env order."""
    nmax = max_shard(global_envs, world)
    full = np.asarray(full).reshape(world, nsteps, nmax, -1)
    rows = [full[r, :, :shard_bounds(global_envs, world, r)[1]] for r in range(world)]
    out = np.concatenate(rows, 1)
    D = out.shape[2] - 2
    return out[:, :, :D], out[:, :, D], out[:, :, D + 1]


# ------------------------------------------------------------------------------ rendezvous
_RDZV_ERR = b"PP3_RDZV_ERROR:"  # (an id is COMM_ID_BYTES of binary; this prefix marks rank 0's failure)


def _proc_start_ticks(pid: int) -> str:
    """Start time of process `pid` in clock ticks since boot (/proc/<pid>/stat field 22), or "0"."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[19]
    except (OSError, IndexError):
        return "0"


def launch_key() -> str:
    """A value every rank of ONE launch shares and no other launch does.  bench.py's own launcher
    exports PP3_LAUNCH_ID (a per-launch nonce); under torch.distributed.run every worker of a launch
    has the same parent (the elastic agent): its pid together with its start time (pids are reused,
    pid + start time are not), MASTER_PORT and TORCHELASTIC_RUN_ID key the launch."""
    explicit = os.environ.get("PP3_LAUNCH_ID")
    if explicit:
        return explicit
    ppid = os.getppid()
    port = os.environ.get("MASTER_PORT", "0")
    run = os.environ.get("TORCHELASTIC_RUN_ID", "none")
    return f"{ppid}.{_proc_start_ticks(ppid)}_{port}_{run}"


def _rdzv_path(tag: str) -> str:
    """Per-launch file name on the node (launch_key): a file left behind by an earlier launch can
    never be read by a later one.  Explicit PP3_RDZV_FILE wins (e.g. a shared file system for
    several nodes)."""
    explicit = os.environ.get("PP3_RDZV_FILE")
    if explicit:
        return explicit + tag
    base = os.environ.get("PP3_RDZV_DIR", "/tmp")
    return os.path.join(base, f"pp3_rdzv_{launch_key()}{tag}.bin")


def rendezvous_id(rank: int, world: int, make_id: Callable[[], bytes], tag: str = "",
                  timeout_s: float = 120.0) -> bytes:
    """Rank 0 creates the communicator id (``make_id``) and publishes it atomically in a file on
    the node; the other ranks poll for it.  Returns the id on every rank."""
    path = _rdzv_path(tag)
    if rank == 0:
        err = None
        try:
            blob = bytes(make_id())
        except Exception as exc:  # published too, so the other ranks fail now instead of at their timeout
            err = exc
            blob = _RDZV_ERR + str(exc).encode()
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(blob)
        os.replace(tmp, path)  # atomic publish
        if err is not None:
            raise err
        return blob
    t0 = time.monotonic()
    while True:
        try:
            with open(path, "rb") as f:
                blob = f.read()
            if blob.startswith(_RDZV_ERR):
                raise RuntimeError(f"rank 0 could not create the communicator id: {blob[len(_RDZV_ERR):].decode()}")
            if blob:
                return blob
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout_s:
            raise TimeoutError(f"rank {rank}: no communicator id at {path} after {timeout_s:.0f} s")
        time.sleep(0.01)


def rendezvous_cleanup(tag: str = "") -> None:
    try:
        os.remove(_rdzv_path(tag))
    except FileNotFoundError:
        pass


# ------------------------------------------------------------------------------ RCCL comm
class Comm:
    """One rank of the env-sharded job: an RCCL communicator created through the C ABI
    (pp3_comm_init), the learner gather, and the host-blocking barrier / reductions the bench's
    max-over-ranks timing uses."""

    def __init__(self, rank: int, world: int, device: int, tag: str = ""):
        from . import _abi, _lib
        self._lib = _lib
        self._L = L = _lib.load()
        self.rank, self.world, self.device = int(rank), int(world), int(device)

        def make_id():
            buf = (C.c_uint8 * _abi.COMM_ID_BYTES)()
            _lib.check_comm(L.pp3_comm_unique_id(buf))
            return bytes(buf)

        self._h = None
        try:
            uid = rendezvous_id(self.rank, self.world, make_id, tag)
            ubuf = (C.c_uint8 * len(uid)).from_buffer_copy(uid)
            h = C.c_void_p()
            _lib.check_comm(L.pp3_comm_init(ubuf, self.rank, self.world, self.device, C.byref(h)))
            self._h = h
            self._tag = tag
            self.barrier()  # every rank has read the id: rank 0 may remove the file
        finally:
            if self.rank == 0:  # (also when the init failed: no later launch may find it)
                rendezvous_cleanup(tag)

    @classmethod
    def from_env(cls, device: Optional[int] = None) -> "Comm":
        """RANK / WORLD_SIZE / LOCAL_RANK as set by torch.distributed.run (or any launcher)."""
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        dev = int(os.environ.get("LOCAL_RANK", "0")) if device is None else device
        return cls(rank, world, dev)

    def gather(self, env, nmax: int, dst_dev: Optional[int], root: int = 0, stream: Optional[int] = None) -> None:
        """Learner batch of every rank's shard into dst_dev (see module doc); root < 0 = all-gather."""
        if hasattr(env, "_flush"):
            env._flush()  # a step() launch still queued (environment.DEFER_LAUNCH) first
        self._lib.check_comm(self._L.pp3_gather(self._h, env._h, int(nmax), int(root),
                                                C.c_void_p(dst_dev) if dst_dev else None,
                                                C.c_void_p(stream) if stream else None))

    def gather_rollout(self, env, traj_obs: int, traj_reward: int, traj_done: int, nsteps: int, nmax: int,
                       dst_dev: Optional[int], root: int = 0, stream: Optional[int] = None) -> None:
        """The K-step unroll of one fused rollout (device trajectory buffers [K][n][D] / [K][n] /
        [K][n]) of every rank into dst_dev ([world][K][nmax][D + 2]): one collective per unroll."""
        if hasattr(env, "_flush"):
            env._flush()
        vp = C.c_void_p
        self._lib.check_comm(self._L.pp3_gather_rollout(self._h, env._h, vp(traj_obs), vp(traj_reward), vp(traj_done),
                                                        int(nsteps), int(nmax), int(root),
                                                        vp(dst_dev) if dst_dev else None,
                                                        vp(stream) if stream else None))

    def allreduce(self, values, op: str = "max") -> np.ndarray:
        from . import _abi
        v = np.ascontiguousarray(values, dtype=np.float64).ravel()
        out = np.empty_like(v)
        self._lib.check_comm(self._L.pp3_comm_allreduce(
            self._h, v.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p), v.size,
            _abi.REDUCE_MAX if op == "max" else _abi.REDUCE_SUM))
        return out

    def barrier(self) -> None:
        self._lib.check_comm(self._L.pp3_comm_barrier(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.pp3_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FileComm:
    """Host-only stand-in for ``Comm``'s barrier and reductions (no gather), through files in one
    directory on the node.  bench.py falls back to it when the RCCL communicator cannot be
    created, so a multi-GPU timing run still gets its barrier and max-over-ranks timing; the env
    shards themselves never exchange data.  Round k: every rank publishes its values atomically
    as ``<dir>/<k>.<rank>`` and polls until all ``world`` files of round k exist."""

    def __init__(self, rank: int, world: int, tag: str = "_file", timeout_s: float = 300.0,
                 directory: Optional[str] = None):
        self.rank, self.world = int(rank), int(world)
        self._dir = directory or (_rdzv_path(tag) + ".d")
        os.makedirs(self._dir, exist_ok=True)
        self._round = 0
        self._timeout = timeout_s

    def _exchange(self, values) -> np.ndarray:
        k = self._round
        self._round += 1
        v = np.ascontiguousarray(values, dtype=np.float64).ravel()
        path = os.path.join(self._dir, f"{k}.{self.rank}")
        with open(path + ".tmp", "wb") as f:
            f.write(v.tobytes())
        os.replace(path + ".tmp", path)
        out = np.empty((self.world, v.size))
        t0 = time.monotonic()
        for r in range(self.world):
            p = os.path.join(self._dir, f"{k}.{r}")
            while not os.path.exists(p):
                if time.monotonic() - t0 > self._timeout:
                    raise TimeoutError(f"rank {self.rank}: rank {r} missing from round {k} at {self._dir}")
                time.sleep(2e-5)
            with open(p, "rb") as f:
                out[r] = np.frombuffer(f.read(), dtype=np.float64)
        if k >= 2:  # every rank has finished round k - 1 (it published round k): drop own k - 2
            try:
                os.remove(os.path.join(self._dir, f"{k - 2}.{self.rank}"))
            except FileNotFoundError:
                pass
        return out

    def allreduce(self, values, op: str = "max") -> np.ndarray:
        a = self._exchange(values)
        return a.max(0) if op == "max" else a.sum(0)

    def barrier(self) -> None:
        self._exchange([0.0])

    def gather(self, *args, **kwargs) -> None:
        raise RuntimeError("FileComm has no device gather: --gather needs the RCCL communicator")

    def close(self) -> None:
        if self._dir is None:
            return
        # after this last round every rank has read the previous one: drop it; the last round's
        # files stay (a slower rank may still be reading them), a few bytes per rank in the directory
        self.barrier()
        try:
            os.remove(os.path.join(self._dir, f"{self._round - 2}.{self.rank}"))
        except FileNotFoundError:
            pass
        self._dir = None
