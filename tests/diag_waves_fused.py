"""Diagnostic: per-wave lifetimes of ONE fused rollout launch (PP3_PHASE_PROF build), by XCD.

PP3_LIB_PATH=pupperv3-mjx_amd/pupperv3_mjx/libpupper_hip_prof.so python tests/diag_waves_fused.py [steps]
A fused launch ends with the wave whose summed step times are largest; this prints how those sums
spread (chip-wide 100 MHz realtime clock, so XCDs compare fairly; the shader-clock cycles too) and
whether the slowest waves sit on particular XCDs (a static env -> wave mapping cannot move them).
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]
os.environ.setdefault("PP3_LIB_PATH", os.path.join(ROOT, "pupperv3-mjx_amd", "pupperv3_mjx", "libpupper_hip_prof.so"))
os.environ.setdefault("PP3_ALLOW_DIAG_BUILD", "1")

import numpy as np  # noqa: E402

import bench  # noqa: E402
from pupperv3_mjx import MODEL_XML, _abi, _lib  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env, make_keys  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    E, warm = 4096, int(os.environ.get("DIAG_WARMUP", "5"))
    env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=E, pipeline_output=False)
    st = env.reset(make_keys(0, E))
    rec = st._record.copy()
    rec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3] = [0.5, 0.0, 0.0]
    env._put(_abi.F_STATE, rec)
    L = env._L
    acts = _lib.DeviceBuffer((steps + warm) * E * 48)
    _lib.check(L.pp3_fill_uniform(env._h, acts.ptr, (steps + warm) * E * 12, 1234, 0, -1.0, 1.0, None))
    ms = C.c_float()
    _lib.check(L.pp3_step_timed(env._h, acts.ptr, E * 12, warm, C.byref(ms)))
    _lib.check(L.pp3_rollout_timed(env._h, C.c_void_p(acts.ptr.value + warm * E * 48), E * 12, steps,
                                   None, None, None, C.byref(ms)))
    W = E // 2
    wv = (C.c_uint32 * (288 * W))()
    _lib.check(L.pp3_wave_profile(wv, W))
    w = np.array(wv[:], dtype=np.uint64).reshape(W, 288)
    cyc = w[:, 0].astype(np.float64)
    rt = ((w[:, 30].astype(np.int64) - w[:, 29].astype(np.int64)) & 0xFFFFFFFF).astype(np.float64)  # 10 ns ticks
    rt0 = w[:, 29].astype(np.int64)
    xcc = (w[:, 7] & 0xF).astype(int)
    print(f"fused launch: {steps} steps, {ms.value:.3f} ms ({ms.value / steps * 1e3:.1f} us/step, prof build)")
    print(f"start spread: {(rt0.max() - rt0.min()) / 100:.1f} us")
    for name, v, unit in (("realtime", rt / 100.0, "us"), ("shader cycles", cyc, "cyc")):
        q = np.percentile(v, [50, 90, 99])
        print(f"{name}: mean {v.mean():.1f} p50 {q[0]:.1f} p90 {q[1]:.1f} p99 {q[2]:.1f} max {v.max():.1f} {unit}")
    print("per XCD: waves, mean / max realtime us, mean shader cycles, cycles per us (clock)")
    for x in range(8):
        sel = xcc == x
        if sel.any():
            print(f"  xcd {x}: {sel.sum():4d}  {rt[sel].mean() / 100:8.1f} / {rt[sel].max() / 100:8.1f}  "
                  f"{cyc[sel].mean():10.0f}  {cyc[sel].sum() / (rt[sel].sum() / 100):7.0f}")
    top = np.argsort(rt)[-40:]
    print("slowest 40 waves by XCD:", np.bincount(xcc[top], minlength=8).tolist(),
          f"dense substeps mean {w[top, 1].astype(float).mean():.1f} (all {w[:, 1].astype(float).mean():.2f})")


if __name__ == "__main__":
    main()
