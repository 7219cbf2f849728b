"""ctypes binding of the C-ABI in include/pupper_hip.h (libpupper_hip.so, built in-tree).

This is the binding a maintainer adds on the reference side.  There is
no fallback: if the HIP library is missing or no GPU is visible, the product path raises.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PP3_LIB_PATH") or os.path.join(_HERE, "libpupper_hip.so")
_lib = None


class PupperHipError(RuntimeError):
    pass


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PupperHipError(
            f"HIP extension not built: {LIB_PATH} is missing (run __graft_entry__.build() or make -C "
            "pupperv3-mjx_amd/csrc); there is no CPU fallback for the environment step.")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, sz = C.c_void_p, C.c_int32, C.c_int64, C.c_size_t
    L.pp3_abi_version.restype = C.c_int
    L.pp3_struct_size.argtypes = [C.c_int]
    L.pp3_struct_size.restype = sz
    L.pp3_last_error.restype = C.c_char_p
    L.pp3_device_count.restype = C.c_int
    L.pp3_create.argtypes = [C.POINTER(_abi.Model), C.POINTER(_abi.EnvConfig), i32, i32, C.POINTER(vp)]
    L.pp3_destroy.argtypes = [vp]
    L.pp3_num_envs.argtypes = [vp]
    L.pp3_num_envs.restype = i32
    L.pp3_state_stride.argtypes = [vp]
    L.pp3_state_stride.restype = i32
    L.pp3_env_device.argtypes = [vp]
    L.pp3_env_device.restype = i32
    L.pp3_reset.argtypes = [vp, vp, vp, vp]
    L.pp3_step.argtypes = [vp, vp, vp]
    L.pp3_rollout.argtypes = [vp, vp, i64, i32, vp, vp, vp, vp]
    L.pp3_set_dr.argtypes = [vp, vp]
    L.pp3_set_pipeline_output.argtypes = [vp, i32]
    L.pp3_physics_step.argtypes = [vp, vp, i32, vp]
    L.pp3_field.argtypes = [vp, i32, C.POINTER(vp), C.POINTER(i64)]
    L.pp3_copy_field_to_host.argtypes = [vp, i32, vp, sz]
    L.pp3_copy_field_from_host.argtypes = [vp, i32, vp, sz]
    L.pp3_synchronize.argtypes = [vp]
    L.pp3_copy_field_to_host_async.argtypes = [vp, i32, vp, sz]
    L.pp3_host_malloc.argtypes = [sz, C.POINTER(vp)]
    L.pp3_memcpy_h2d_async.argtypes = [vp, vp, sz, vp]
    L.pp3_host_free.argtypes = [vp]
    L.pp3_device_malloc.argtypes = [i32, sz, C.POINTER(vp)]
    L.pp3_device_free.argtypes = [vp]
    L.pp3_memcpy_h2d.argtypes = [vp, vp, sz]
    L.pp3_memcpy_d2h.argtypes = [vp, vp, sz]
    L.pp3_outputs_to_host.argtypes = [vp, vp]
    L.pp3_host_device_ptr.argtypes = [vp, C.POINTER(vp)]
    L.pp3_memcpy_d2d.argtypes = [vp, vp, sz, vp]
    L.pp3_fill_uniform.argtypes = [vp, vp, i64, C.c_uint32, C.c_uint32, C.c_float, C.c_float, vp]
    L.pp3_step_timed.argtypes = [vp, vp, i64, i32, C.POINTER(C.c_float)]
    L.pp3_rollout_timed.argtypes = [vp, vp, i64, i32, vp, vp, vp, C.POINTER(C.c_float)]
    L.pp3_phase_profile.argtypes = [C.POINTER(C.c_uint64), i32, i32]
    L.pp3_wave_profile.argtypes = [C.POINTER(C.c_uint32), i32]
    if hasattr(L, "pp3_rollout_policy_fused"):  # (diagnostic query; absent from pre-round-5 builds used in A/B)
        L.pp3_rollout_policy_fused.argtypes = [vp]
        L.pp3_rollout_policy_fused.restype = i32
    if hasattr(L, "pp3_narrow_cull"):  # (diagnostic query; absent from pre-round-6 builds used in A/B)
        L.pp3_narrow_cull.argtypes = [vp]
        L.pp3_narrow_cull.restype = i32
    L.pp3_set_auto_reset.argtypes = [vp, i32]
    L.pp3_set_action_repeat.argtypes = [vp, i32]
    L.pp3_policy_create.argtypes = [i32, i32, i32, vp, vp, vp, C.POINTER(vp)]
    L.pp3_policy_act.argtypes = [vp, vp, i64, i32, vp, i64, vp]
    L.pp3_policy_out_dim.argtypes = [vp]
    L.pp3_policy_destroy.argtypes = [vp]
    L.pp3_rollout_policy.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp]
    L.pp3_rollout_policy_timed.argtypes = [vp, vp, i32, vp, vp, vp, vp, C.POINTER(C.c_float)]
    L.pp3_policy_last_error.restype = C.c_char_p
    L.pp3_stream.argtypes = [vp]
    L.pp3_stream.restype = vp
    if hasattr(L, "pp3_event_create"):  # (absent from pre-round-5 builds run in kernel A/B: no host-API step there)
        L.pp3_event_create.argtypes = [vp, C.POINTER(vp)]
        L.pp3_event_record.argtypes = [vp, vp]
        L.pp3_event_synchronize.argtypes = [vp]
        L.pp3_event_destroy.argtypes = [vp]
        for name in ("pp3_event_create", "pp3_event_record", "pp3_event_synchronize", "pp3_event_destroy"):
            getattr(L, name).restype = C.c_int
    L.pp3_set_terrain.argtypes = [vp, vp, i32]
    L.pp3_terrain_slots.argtypes = [vp]
    L.pp3_terrain_slots.restype = i32
    # multi-GPU (pp3_comm.hip; RCCL is dlopen'ed by the library on first use)
    L.pp3_comm_unique_id.argtypes = [vp]
    L.pp3_comm_init.argtypes = [vp, i32, i32, i32, C.POINTER(vp)]
    L.pp3_comm_destroy.argtypes = [vp]
    L.pp3_comm_rank.argtypes = [vp]
    L.pp3_comm_rank.restype = i32
    L.pp3_comm_world.argtypes = [vp]
    L.pp3_comm_world.restype = i32
    L.pp3_comm_last_error.restype = C.c_char_p
    L.pp3_gather.argtypes = [vp, vp, i32, i32, vp, vp]
    L.pp3_gather_rollout.argtypes = [vp, vp, vp, vp, vp, i32, i32, i32, vp, vp]
    L.pp3_render.argtypes = [i32, vp, vp, i32, vp, i32, vp, vp, i32, i32, i32, C.POINTER(C.c_float), vp, vp]
    L.pp3_render_last_error.restype = C.c_char_p
    L.pp3_comm_allreduce.argtypes = [vp, vp, vp, i32, i32]
    L.pp3_comm_barrier.argtypes = [vp]
    for name in ("pp3_create", "pp3_destroy", "pp3_reset", "pp3_step", "pp3_rollout", "pp3_rollout_timed", "pp3_set_dr", "pp3_set_pipeline_output",
                 "pp3_physics_step", "pp3_field", "pp3_copy_field_to_host", "pp3_copy_field_from_host",
                 "pp3_synchronize", "pp3_copy_field_to_host_async", "pp3_host_malloc", "pp3_host_free",
                 "pp3_memcpy_h2d_async",
                 "pp3_device_malloc", "pp3_device_free", "pp3_memcpy_h2d", "pp3_memcpy_d2h",
                 "pp3_outputs_to_host", "pp3_host_device_ptr", "pp3_memcpy_d2d", "pp3_fill_uniform", "pp3_step_timed", "pp3_phase_profile",
                 "pp3_wave_profile", "pp3_set_auto_reset", "pp3_set_action_repeat", "pp3_policy_create", "pp3_policy_act", "pp3_policy_destroy", "pp3_rollout_policy",
                 "pp3_rollout_policy_timed", "pp3_set_terrain", "pp3_comm_unique_id", "pp3_comm_init", "pp3_comm_destroy", "pp3_gather", "pp3_gather_rollout",
                 "pp3_comm_allreduce", "pp3_comm_barrier", "pp3_render"):
        getattr(L, name).restype = C.c_int
    if L.pp3_abi_version() != _abi.ABI_VERSION:
        raise PupperHipError("ABI version mismatch between libpupper_hip.so and pupperv3_mjx/_abi.py")
    if L.pp3_struct_size(0) != C.sizeof(_abi.Model) or L.pp3_struct_size(1) != C.sizeof(_abi.EnvConfig):
        raise PupperHipError("struct layout mismatch between include/pupper_hip.h and pupperv3_mjx/_abi.py")
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        msg = load().pp3_last_error().decode(errors="replace")
        raise PupperHipError(f"pupper_hip error {rc}: {msg}")


def check_comm(rc: int) -> None:
    if rc != 0:
        msg = load().pp3_comm_last_error().decode(errors="replace")
        raise PupperHipError(f"pupper_hip comm error {rc}: {msg}")


EXPORTED_SYMBOLS = (
    "pp3_abi_version", "pp3_struct_size", "pp3_last_error", "pp3_device_count", "pp3_create", "pp3_destroy",
    "pp3_num_envs", "pp3_state_stride", "pp3_env_device", "pp3_reset", "pp3_step", "pp3_rollout", "pp3_set_dr",
    "pp3_set_pipeline_output", "pp3_physics_step", "pp3_field", "pp3_copy_field_to_host", "pp3_copy_field_from_host", "pp3_synchronize",
    "pp3_copy_field_to_host_async", "pp3_host_malloc", "pp3_host_free", "pp3_memcpy_h2d_async",
    "pp3_device_malloc", "pp3_device_free", "pp3_memcpy_h2d", "pp3_memcpy_d2h", "pp3_outputs_to_host", "pp3_host_device_ptr", "pp3_memcpy_d2d",
    "pp3_fill_uniform", "pp3_step_timed", "pp3_rollout_timed", "pp3_set_auto_reset", "pp3_set_action_repeat",
    "pp3_policy_create", "pp3_policy_act", "pp3_policy_out_dim", "pp3_policy_destroy", "pp3_policy_last_error",
    "pp3_rollout_policy", "pp3_rollout_policy_timed",
    "pp3_stream", "pp3_event_create", "pp3_event_record", "pp3_event_synchronize", "pp3_event_destroy",
    "pp3_set_terrain", "pp3_terrain_slots",
    "pp3_comm_unique_id", "pp3_comm_init", "pp3_comm_destroy", "pp3_comm_rank", "pp3_comm_world",
    "pp3_comm_last_error", "pp3_gather", "pp3_gather_rollout", "pp3_comm_allreduce", "pp3_comm_barrier",
    "pp3_render", "pp3_render_last_error",
)

# include/pupper_hip_diag.h: diagnostic entry points (per-phase / per-wave clocks of a -DPP3_PHASE_PROF
# build; the product library exports them only to return PP3_ERR_ARG)
DIAG_SYMBOLS = ("pp3_phase_profile", "pp3_wave_profile", "pp3_rollout_policy_fused", "pp3_narrow_cull")


class BlockPool(list):
    """Free PinnedBlocks of one size.  A retired pool (an unroll length the env no longer uses, a
    closed env) frees its free blocks, and a leased block released into it later is freed at once
    instead of being kept: nothing waits for the cyclic garbage collector."""

    def __init__(self):
        super().__init__()
        self.retired = False

    def release(self, block: "PinnedBlock") -> None:
        if self.retired:
            block.free()
        else:
            self.append(block)

    def retire(self) -> None:
        self.retired = True
        while self:
            self.pop().free()


def _release(pool, block) -> None:
    """A released lease (_BlockRef.__del__): the block goes back to its pool (or is freed there)."""
    if isinstance(pool, BlockPool):
        pool.release(block)
    else:
        pool.append(block)


class PinnedBlock:
    """Page-locked host memory (pp3_host_malloc) exposed to numpy through __array_interface__:
    arrays made from it keep it alive, and when the last one dies the block goes back to its pool
    (BlockPool.release), so host-API output arrays never alias a block that a later step reuses.
    The block does not reference its pool (no reference cycle)."""

    def __init__(self, nbytes: int):
        self.ptr = C.c_void_p()
        self.nbytes = int(nbytes)
        check(load().pp3_host_malloc(max(self.nbytes, 4), C.byref(self.ptr)))
        self.__array_interface__ = {"shape": (self.nbytes // 4,), "typestr": "<f4", "version": 3,
                                    "data": (self.ptr.value, False)}
        # (a lease's arrays are read-only from the start: no per-view flag update)
        self._ro_interface = dict(self.__array_interface__, data=(self.ptr.value, True))
        self._dev = None

    def device_ptr(self) -> int:
        """The block's device address (pp3_host_device_ptr; cached): kernels store into it directly."""
        if self._dev is None:
            d = C.c_void_p()
            check(load().pp3_host_device_ptr(self.ptr, C.byref(d)))
            self._dev = d.value
        return self._dev

    @staticmethod
    def take(nbytes: int, pool: list) -> "_BlockRef":
        """A block from `pool` (a BlockPool of free blocks) or a new one, leased: it returns there when
        the lease and every array made from it have died.  The lease's arrays are read-only (the
        blocks hold launch outputs the host only reads)."""
        b = pool.pop() if pool else PinnedBlock(nbytes)
        return _BlockRef(b, pool)

    def free(self) -> None:
        if self.ptr:
            load().pp3_host_free(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class _BlockRef:
    """One lease of a PinnedBlock: numpy arrays made from it reference this object, whose death
    returns the block to its pool (__del__: reference counting releases it the moment the last
    array dies, without a weakref.finalize registration per lease)."""

    def __init__(self, block: PinnedBlock, pool: list):
        self.block = block
        self.ptr = block.ptr
        self._pool = pool
        self.__array_interface__ = block._ro_interface

    def __del__(self):
        pool, self._pool = self._pool, None
        if pool is not None:
            try:
                _release(pool, self.block)
            except Exception:  # (interpreter shutdown)
                pass

    def device_ptr(self) -> int:
        return self.block.device_ptr()


class DeviceBuffer:
    """Minimal owning device allocation (no torch needed)."""

    def __init__(self, nbytes: int, device: int = 0):
        L = load()
        self.ptr = C.c_void_p()
        self.nbytes = int(nbytes)
        check(L.pp3_device_malloc(device, max(self.nbytes, 4), C.byref(self.ptr)))

    def upload(self, arr) -> None:
        import numpy as np
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes
        check(load().pp3_memcpy_h2d(self.ptr, a.ctypes.data_as(C.c_void_p), a.nbytes))

    def download(self, arr) -> None:
        check(load().pp3_memcpy_d2h(arr.ctypes.data_as(C.c_void_p), self.ptr, arr.nbytes))

    def free(self) -> None:
        if self.ptr:
            load().pp3_device_free(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
