"""The C-ABI library loads without a GPU and exports every symbol include/pupper_hip.h declares."""
import ctypes as C
import os
import re

import pytest

from pupperv3_mjx import _abi, _lib

INCLUDE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
HEADER = os.path.join(INCLUDE, "pupper_hip.h")
DIAG_HEADER = os.path.join(INCLUDE, "pupper_hip_diag.h")


def _declared(path=HEADER):
    src = open(path).read()
    return sorted(set(re.findall(r"\b(pp3_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_what_python_binds():
    assert set(_declared()) == set(_lib.EXPORTED_SYMBOLS)


def test_diagnostic_entry_points_live_in_their_own_header():
    """The per-phase / per-wave profilers are not part of the drop-in boundary: declared in
    pupper_hip_diag.h only, exported by the library (refusing to run in the product build)."""
    assert set(_declared(DIAG_HEADER)) == set(_lib.DIAG_SYMBOLS)
    assert not set(_lib.DIAG_SYMBOLS) & set(_declared())
    L = _lib.load()
    for name in _lib.DIAG_SYMBOLS:
        assert hasattr(L, name), name
    buf = (C.c_uint64 * 16)()
    assert L.pp3_phase_profile(buf, 16, 0) != 0  # the product build has no profiler
    assert L.pp3_rollout_policy_fused(None) == -1
    assert L.pp3_narrow_cull(None) == -1


def test_library_loads_and_exports_all_symbols():
    L = _lib.load()
    for name in _declared():
        assert hasattr(L, name), name
    assert L.pp3_abi_version() == _abi.ABI_VERSION


def test_struct_layouts_match_ctypes():
    L = _lib.load()
    assert L.pp3_struct_size(0) == C.sizeof(_abi.Model)
    assert L.pp3_struct_size(1) == C.sizeof(_abi.EnvConfig)
    assert 0 < L.pp3_struct_size(3) <= 20 * 1024  # LDS per env (one workgroup)


def test_create_rejects_bad_config_without_gpu_work():
    """pp3_create validates model/config before touching the device."""
    import common
    m, c, _ = common.env_model_and_config(common.MODEL_XML)
    L = _lib.load()
    h = C.c_void_p()
    c.obs_history = 99
    rc = L.pp3_create(C.byref(m), C.byref(c), 4, 0, C.byref(h))
    assert rc == 1 and b"observation_history" in L.pp3_last_error()
    c.obs_history = 2
    m2 = _abi.Model.from_buffer_copy(m)
    m2.cone = 1
    rc = L.pp3_create(C.byref(m2), C.byref(c), 4, 0, C.byref(h))
    assert rc == 2


def test_state_layout_constants():
    assert _abi.state_stride(2, 2) == 98 + 24 + 12
    assert _abi.REWARD_NAMES[_abi.NREWARD - 1] == "body_collision"


def test_step_entry_points_reject_null_arguments_without_gpu_work():
    """pp3_step / pp3_rollout / pp3_rollout_timed validate their arguments before any HIP call."""
    L = _lib.load()
    assert L.pp3_step(None, None, None) == 1
    assert L.pp3_rollout(None, C.c_void_p(16), 0, 4, None, None, None, None) == 1
    assert b"pp3_rollout" in L.pp3_last_error()
    ms = C.c_float()
    assert L.pp3_rollout_timed(None, C.c_void_p(16), 0, 4, None, None, None, C.byref(ms)) == 1


def test_loopback_transport_exports_the_rccl_api():
    """The multi-rank test transport (tests/loopback, test_gpu_multirank.py) provides every RCCL
    entry point pp3_comm.hip binds, and the test build of the library is a separate file that
    refuses pp3_create without the diagnostic opt-in (pp3_diag.h)."""
    import ctypes as C
    here = os.path.dirname(os.path.abspath(__file__))
    lb = os.path.join(here, "loopback", "libpp3_loopback_rccl.so")
    if not os.path.exists(lb):
        pytest.skip("loopback test build absent (make -C pupperv3-mjx_amd/csrc loopback)")
    T = C.CDLL(lb)
    for name in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclAllGather", "ncclAllReduce",
                 "ncclSend", "ncclRecv", "ncclGroupStart", "ncclGroupEnd", "ncclGetErrorString"):
        assert hasattr(T, name), name
    src = open(os.path.join(here, "..", "pupperv3-mjx_amd", "csrc", "pp3_comm.hip")).read()
    assert "#ifdef PP3_TEST_RCCL_SONAME" in src  # the product build always loads librccl
