"""Per-step kernel time of the configs[1] rollout from reset (the start-height drop transient the
driver's --warmup 5 bench runs inside), with the active-contact count and the share of waves
holding a leg-leg contact (dense Hessian path) every few steps.

  python tools/step_trace.py [--steps 300] [--envs 4096] > gpurun_out/step_trace.json
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--every", type=int, default=5)
    ap.add_argument("--repeat", type=int, default=1,
                    help="rollouts from the same reset, back to back (the later ones run on a warm GPU clock)")
    args = ap.parse_args()
    import numpy as np
    from bench import bench_kwargs
    from pupperv3_mjx import MODEL_XML, _abi, _lib
    from pupperv3_mjx.environment import PupperV3Env, make_keys
    E = args.envs
    env = PupperV3Env(**bench_kwargs(MODEL_XML), num_envs=E, pipeline_output=False)
    st = env.reset(make_keys(0, E))
    rec = st._record.copy()
    rec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3] = [0.5, 0.0, 0.0]
    obs0 = st.obs.copy()
    acts = _lib.DeviceBuffer(args.steps * E * 48, 0)
    _lib.check(env._L.pp3_fill_uniform(env._h, acts.ptr, args.steps * E * 12, 1234, 0, -1.0, 1.0, None))
    env.synchronize()
    for rep in range(args.repeat):
        env._put(_abi.F_STATE, rec)
        env._put(_abi.F_OBS, obs0)
        rollout(env, args, acts, E, rep)
    env.close()


def rollout(env, args, acts, E, rep):
    import numpy as np
    from pupperv3_mjx import _abi, _lib
    ms = C.c_float()
    for i in range(args.steps):
        probe = i % args.every == 0
        if probe:
            _lib.check(env._L.pp3_set_pipeline_output(env._h, 1))
        _lib.check(env._L.pp3_step_timed(env._h, C.c_void_p(acts.ptr.value + i * E * 48), 0, 1, C.byref(ms)))
        r = {"rep": rep, "step": i, "ms": round(ms.value, 5)}
        if probe:
            p = env._get(_abi.F_PIPELINE)
            _lib.check(env._L.pp3_set_pipeline_output(env._h, 0))
            ncon = p[:, _abi.P_NCON].astype(int)
            g = p[:, _abi.P_CON_GEOM:_abi.P_CON_GEOM + 32].reshape(E, 16, 2).astype(int)
            # leg-leg contact: neither geom is the floor (cgeom id of the world geoms: body 0)
            m = env.sys_model.struct
            static = {int(m.cgeom_id[k]) for k in range(m.ncgeom) if m.cgeom_bodyid[k] == 0}
            selfc = np.array([any(a not in static and b not in static for a, b in g[e, :ncon[e]]) for e in range(E)])
            wave_dense = np.logical_or(selfc[0::2], selfc[1::2]) if E % 2 == 0 else selfc
            r.update(ncon_mean=round(float(ncon.mean()), 3), ncon_max=int(ncon.max()),
                     dense_waves=round(float(wave_dense.mean()), 4), z_mean=round(float(env._get(_abi.F_STATE)[:, 2].mean()), 4))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
