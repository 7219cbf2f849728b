"""INTEGRATION.md section 3's reference-side ctypes stub, checked as written.

CPU: every `_L.<fn>.argtypes` line of the stub matches the prototype in include/pupper_hip.h
(argument count, and pointer / int32 / int64 kind per argument).
GPU: the stub's code block, executed against the in-tree library, drives a handle of its own
(create, reset, step, unroll) to the same bits as PupperV3Env on the same structs, keys and actions.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOC = os.path.join(ROOT, "INTEGRATION.md")
HEADER = os.path.join(ROOT, "include", "pupper_hip.h")


def _stub_source() -> str:
    text = open(DOC).read()
    sec = text[text.index("## 3."):text.index("## 4.")]
    m = re.search(r"```python\n(.*?)```", sec, re.S)
    assert m, "no python block in INTEGRATION.md section 3"
    return m.group(1)


def _kind_c(param: str) -> str:
    p = param.strip()
    if "*" in p:
        return "ptr"
    if p.startswith("int64_t"):
        return "i64"
    if p.startswith("int32_t"):
        return "i32"
    raise AssertionError(f"unclassified parameter {p!r}")


def _kind_py(expr: str) -> str:
    e = expr.strip()
    if e.startswith("C.c_void_p") or e.startswith("C.POINTER") or e.startswith("C.c_char_p"):
        return "ptr"
    return {"C.c_int64": "i64", "C.c_int32": "i32"}[e]


def _split_top(s: str):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return out


def test_stub_argtypes_match_the_header():
    header = open(HEADER).read()
    src = _stub_source()
    bound = re.findall(r"_L\.(pp3_\w+)\.argtypes\s*=\s*\[(.*?)\]\n", src, re.S)
    assert len(bound) >= 6, bound
    for name, args in bound:
        m = re.search(r"\b" + name + r"\s*\(([^;]*?)\)\s*;", header, re.S)
        assert m, f"{name} not declared in pupper_hip.h"
        c_kinds = [_kind_c(p) for p in m.group(1).split(",")]
        py_kinds = [_kind_py(a) for a in _split_top(" ".join(args.split()))]
        assert py_kinds == c_kinds, (name, py_kinds, c_kinds)


@pytest.mark.gpu
def test_stub_drives_a_handle_to_the_env_bits(require_gpu):
    from bench import bench_kwargs
    from pupperv3_mjx import MODEL_XML, _abi, _lib
    from pupperv3_mjx.environment import PupperV3Env, make_keys

    ns = {}
    exec(_stub_source().replace('C.CDLL("libpupper_hip.so")', f'C.CDLL({_lib.LIB_PATH!r})'), ns)
    N, K = 256, 6
    env = PupperV3Env(**bench_kwargs(MODEL_XML, True), num_envs=N, pipeline_output=False)
    stub = ns["HipPupperBatch"](env.sys_model.struct, env.config_struct, N, env.device)
    bufs = []
    try:
        keys = make_keys(4, N)
        kbuf = _lib.DeviceBuffer(keys.nbytes, env.device)
        kbuf.upload(np.ascontiguousarray(keys))
        acts = np.random.RandomState(4).uniform(-1, 1, size=(K + 1, N, 12)).astype(np.float32)
        abuf = _lib.DeviceBuffer(acts.nbytes, env.device)
        abuf.upload(acts)
        bufs += [kbuf, abuf]
        stub.reset(kbuf.ptr.value)
        stub.step(abuf.ptr.value)
        stub.unroll(abuf.ptr.value + acts[0].nbytes, K)
        C.CDLL(_lib.LIB_PATH).pp3_synchronize(stub.h)
        st = env.reset(keys)
        st = env.step(st, acts[0])
        st, _ = env.rollout(st, acts[1:])
        env.synchronize()
        for fid in (_abi.F_STATE, _abi.F_OBS, _abi.F_REWARD, _abi.F_DONE, _abi.F_METRICS):
            ptr, n = stub.field(fid)
            got = np.empty((N, n), np.float32)
            _lib.check(_lib.load().pp3_memcpy_d2h(got.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), got.nbytes))
            want = env._get(fid).reshape(N, n)
            np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg=f"field {fid}")
    finally:
        ns["_L"].pp3_destroy(stub.h)
        for b in bufs:
            b.free()
        env.close()
