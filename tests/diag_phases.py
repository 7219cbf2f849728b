"""Diagnostic: per-phase shader-clock breakdown of env_step_kernel (PP3_PHASE_PROF build).

PP3_LIB_PATH=pupperv3-mjx_amd/pupperv3_mjx/libpupper_hip_prof.so python tests/diag_phases.py
Stamps are s_memtime reads into per-wave registers (a few % overhead; each stamp drains the LDS
reads in flight).  DIAG_FUSED=1 times one fused pp3_rollout launch instead of single-step launches
(the per-wave stamp trace then holds the launch's second step; tools/trace_intervals.py).
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]
os.environ.setdefault("PP3_LIB_PATH", os.path.join(ROOT, "pupperv3-mjx_amd", "pupperv3_mjx", "libpupper_hip_prof.so"))
os.environ.setdefault("PP3_ALLOW_DIAG_BUILD", "1")  # pp3_diag.h: the prof library refuses to run otherwise

import numpy as np  # noqa: E402

import bench  # noqa: E402
from pupperv3_mjx import MODEL_XML, _abi, _lib  # noqa: E402
from pupperv3_mjx.environment import PupperV3Env, make_keys  # noqa: E402

NAMES = ["kinematics", "com/cinert/cdof", "limit/friction rows+actuation", "M+bias+contactJ", "LDL(M)+solve",
         "warmstart", "newton update+grad", "LDL(H)+solve", "line search", "integrate",
         "prologue", "write_obs (history)", "rewards+state", "bias+contact edge rows", "hessian build",
         "crb*cdof+rne chain", "collision", "obs rng draws", "imu + lag buffers"]
# stamps 21..23 split phases 8 (line search), 6 (newton update+grad) and 5 (warmstart)
SUBNAMES = ["  line-search setup", "  newton row update", "  warmstart row costs"]


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = 20
    warm = int(os.environ.get("DIAG_WARMUP", "5"))  # 5: the driver's window (robots landing); 200: steady state
    nobst = int(os.environ.get("DIAG_OBST", "0"))  # configs[4]: bench.py --obstacles N (robots started over the boxes)
    model_path = MODEL_XML
    if nobst:
        import tempfile
        import xml.etree.ElementTree as ET
        from pupperv3_mjx import obstacles
        tree = ET.ElementTree(ET.fromstring(open(MODEL_XML).read()))
        obstacles.add_boxes_to_model(tree, n_boxes=nobst, x_range=(-5, 5), y_range=(-5, 5), height=0.02, length=6.0)
        model_path = os.path.join(tempfile.mkdtemp(), "obstacles.xml")
        tree.write(model_path, encoding="unicode")
    env = PupperV3Env(**bench.bench_kwargs(model_path), num_envs=E, pipeline_output=False)
    st = env.reset(make_keys(0, E))
    rec = st._record.copy()
    rec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3] = [0.5, 0.0, 0.0]  # bench workload (configs[1])
    if nobst:
        from pupperv3_mjx import obstacles
        specs = obstacles.sample_boxes(nobst, (-5, 5), (-5, 5), 0.02, length=6.0)
        rec[:, _abi.S_QPOS:_abi.S_QPOS + 2] = obstacles.rail_start_xy(specs, E, seed=0)
    env._put(_abi.F_STATE, rec)
    L = env._L
    acts = _lib.DeviceBuffer((steps + warm) * E * 48)
    _lib.check(L.pp3_fill_uniform(env._h, acts.ptr, (steps + warm) * E * 12, 1, 0, -1.0, 1.0, None))
    ms = C.c_float()
    _lib.check(L.pp3_step_timed(env._h, acts.ptr, E * 12, warm, C.byref(ms)))
    buf = (C.c_uint64 * 25)()
    _lib.check(L.pp3_phase_profile(buf, 25, 1))
    if os.environ.get("DIAG_FUSED") == "1":  # one pp3_rollout launch (trace: its second step)
        _lib.check(L.pp3_rollout_timed(env._h, C.c_void_p(acts.ptr.value + warm * E * 48), E * 12, steps,
                                       None, None, None, C.byref(ms)))
    else:
        _lib.check(L.pp3_step_timed(env._h, C.c_void_p(acts.ptr.value + warm * E * 48), E * 12, steps, C.byref(ms)))
    _lib.check(L.pp3_phase_profile(buf, 25, 1))
    v = np.array(buf[:len(NAMES)], dtype=np.float64)
    sub = np.array(buf[21:24], dtype=np.float64)  # sub-phases split off phases 8, 6, 5
    tot = v.sum() + sub.sum()
    print(f"E={E}: {ms.value / steps:.3f} ms/step (prof build); cycles per env-step per env: {tot / (E * steps):.0f}")
    for n, x in zip(NAMES, v):
        print(f"  {n:32s} {100 * x / tot:6.2f}%   {x / (E * steps):10.0f} cyc/env-step")
    for n, x in zip(SUBNAMES, sub):
        print(f"  {n:32s} {100 * x / tot:6.2f}%   {x / (E * steps):10.0f} cyc/env-step")
    # per-wave record of the last launch: the kernel ends with its slowest wave
    W = (E + 1) // 2
    wv = (C.c_uint32 * (288 * W))()
    _lib.check(L.pp3_wave_profile(wv, W))
    w8 = np.array(wv[:], dtype=np.uint64).reshape(W, 288)
    np.save(os.path.join(os.environ.get("PP3_DIAG_OUT", "/tmp"), "waves.npy"), w8)
    w = w8[:, :4].astype(np.float64)
    life = w[:, 0]
    q = np.percentile(life, [50, 90, 99, 99.9])
    print(f"  wave lifetime (last launch): mean {life.mean():.0f} p50 {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} "
          f"p99.9 {q[3]:.0f} max {life.max():.0f} cycles")
    for name, col in (("dense substeps", 1), ("max contacts", 2), ("line-search evals", 3)):
        v = w[:, col]
        top = np.argsort(life)[-20:]
        print(f"  {name:18s}: mean {v.mean():.2f} max {v.max():.0f} | slowest 20 waves mean {v[top].mean():.2f}")
    # lifetime by dense / contacts
    for d in range(int(w[:, 1].max()) + 1):
        sel = w[:, 1] == d
        if sel.any():
            print(f"    dense={d}: {sel.sum():5d} waves, mean life {life[sel].mean():.0f}, max {life[sel].max():.0f}")
    for c in range(int(w[:, 2].max()) + 1):
        sel = w[:, 2] == c
        if sel.any():
            print(f"    ncmax={c}: {sel.sum():5d} waves, mean life {life[sel].mean():.0f}, max {life[sel].max():.0f}")
    # which phases grow with contacts: per-wave phase cycles regressed on contact-substeps
    ph = w8[:, 8:27].astype(np.float64)
    cs = w8[:, 27].astype(np.float64)
    s2 = w8[:, 28].astype(np.float64)
    print(f"  contact-substeps per wave: mean {cs.mean():.1f}; substeps with row slot 1: mean {s2.mean():.2f}")
    A = np.stack([np.ones_like(cs), cs, s2, w[:, 1], w[:, 3]], 1)
    coef_l = np.linalg.lstsq(A, life, rcond=None)[0]
    print(f"  lifetime ~ {coef_l[0]:.0f} + {coef_l[1]:.0f}*csum + {coef_l[2]:.0f}*slot2 + {coef_l[3]:.0f}*dense "
          f"+ {coef_l[4]:.0f}*evals")
    print(f"  {'phase':32s} {'mean':>8s} {'/csum':>7s} {'/slot2':>7s} {'/dense':>7s} {'/eval':>7s} {'slow20':>8s}")
    top = np.argsort(life)[-20:]
    for k, n in enumerate(NAMES):
        c = np.linalg.lstsq(A, ph[:, k], rcond=None)[0]
        print(f"  {n:32s} {ph[:, k].mean():8.0f} {c[1]:7.0f} {c[2]:7.0f} {c[3]:7.0f} {c[4]:7.0f} {ph[top, k].mean():8.0f}")
    nsub = steps * env.n_frames if hasattr(env, "n_frames") else steps * 5
    print(f"  line-search evaluations per substep: {buf[20] / (E * nsub):.2f} per env, "
          f"{buf[19] / (E / 2 * nsub):.2f} per wave (max of its two envs)")


if __name__ == "__main__":
    main()
