"""GPU-side helpers shared by the -m gpu tests and the smoke/diagnostic scripts."""
import ctypes as C

import numpy as np

from pupperv3_mjx import _abi, _lib
from pupperv3_mjx.environment import PupperV3Env


def gpu_physics(env: PupperV3Env, qpos, qvel, qws, ctrl, nsteps):
    """Run nsteps raw mj_step substeps on the GPU for all envs; returns (qpos, qvel, qws, pipe)."""
    n = env.num_envs
    rec = np.zeros((n, env.stride), dtype=np.float32)
    rec[:, _abi.S_QPOS:_abi.S_QPOS + 19] = qpos
    rec[:, _abi.S_QVEL:_abi.S_QVEL + 18] = qvel
    rec[:, _abi.S_QACC_WS:_abi.S_QACC_WS + 18] = qws
    env._put(_abi.F_STATE, rec)
    buf = _lib.DeviceBuffer(n * 12 * 4, env.device)
    buf.upload(np.ascontiguousarray(ctrl, dtype=np.float32))
    _lib.check(env._L.pp3_physics_step(env._h, buf.ptr, int(nsteps), None))
    env.synchronize()
    rec = env._get(_abi.F_STATE)
    pipe = env._get(_abi.F_PIPELINE)
    buf.free()
    return (rec[:, 0:19].astype(np.float64), rec[:, 19:37].astype(np.float64), rec[:, 37:55].astype(np.float64),
            pipe.astype(np.float64))


def oracle_physics(model, qpos, qvel, qws, ctrl, nsteps, precision="f64", dr=None):
    from oracle import oracle as O
    n = qpos.shape[0]
    out_q, out_v, out_w, out_p = [], [], [], []
    for i in range(n):
        q, v, w, p, _ = O.mj_step(model, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=nsteps, precision=precision,
                                  dr=None if dr is None else dr[i])
        out_q.append(q); out_v.append(v); out_w.append(w); out_p.append(p)
    return np.array(out_q), np.array(out_v), np.array(out_w), np.array(out_p)


def record_to_oracle_state(rec_f32: np.ndarray) -> np.ndarray:
    """Device f32 record (rng bit-cast) -> oracle double record (rng as integer values)."""
    with np.errstate(invalid="ignore"):
        out = rec_f32.astype(np.float64)
    out[..., _abi.S_RNG:_abi.S_RNG + 2] = rec_f32[..., _abi.S_RNG:_abi.S_RNG + 2].copy().view(np.uint32)
    return out


def oracle_state_to_record(st: np.ndarray) -> np.ndarray:
    out = st.astype(np.float32)
    out[..., _abi.S_RNG:_abi.S_RNG + 2] = st[..., _abi.S_RNG:_abi.S_RNG + 2].astype(np.uint32).view(np.float32)
    return out


class FlipBudget:
    """Env-step parity with an explicit allowance for constraint-state flips.

    MuJoCo's Newton solver (iterations=1) is discontinuous where a constraint row sits on its
    switch point (satisfied/active, or the frictionloss kink): the fp32 kernel and the oracle
    may then take different branches and legitimately produce different accelerations.  A
    step may exceed the tolerance only if the oracle flagged such a row during that step
    (OracleEnv.step()['boundary'] > 0), and at most `max_frac` of all compared steps may.
    """

    def __init__(self, max_frac=0.05):
        self.max_frac = max_frac
        self.n = 0
        self.flips = 0

    def check(self, ok: bool, oracle_out: dict, what: str = ""):
        self.n += 1
        if ok:
            return
        assert oracle_out.get("boundary", 0) > 0, f"parity failure without a constraint-state flip: {what}"
        self.flips += 1

    def finish(self):
        assert self.flips <= max(1, self.max_frac * self.n), (self.flips, self.n)
