"""GPU-side helpers shared by the -m gpu tests and the smoke/diagnostic scripts."""
import json
import os

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


def report(name: str, payload: dict) -> None:
    """Print a one-line JSON report and append it to $PP3_REPORT_DIR/gpu_reports.jsonl when set
    (the GPU runs point it at gpurun_out/ so the numbers come back with the run)."""
    line = json.dumps({"test": name, **payload})
    print("REPORT " + line)
    d = os.environ.get("PP3_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "gpu_reports.jsonl"), "a") as f:
            f.write(line + "\n")


class FlipBudget:
    """Env-step parity with an explicit allowance for constraint-state flips.

    MuJoCo's Newton solver (iterations=1) is discontinuous where a constraint row sits on its
    switch point (satisfied/active, or the frictionloss kink): the fp32 kernel and the oracle
    may then take different branches and legitimately produce different accelerations.  A
    step may exceed the tolerance only if the oracle flagged such a row during that step
    (OracleEnv.step()['boundary'] > 0), and at most `max_frac` (default 1 %) of all compared
    steps may.  The flip count is reported (``report``) whatever the outcome.
    """

    def __init__(self, max_frac=0.01, name=""):
        self.max_frac = max_frac
        self.name = name or os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0]
        self.n = 0
        self.flips = 0
        self.flagged = 0

    def check(self, ok: bool, oracle_out: dict, what: str = ""):
        self.n += 1
        self.flagged += oracle_out.get("boundary", 0) > 0
        if ok:
            return
        assert oracle_out.get("boundary", 0) > 0, f"parity failure without a constraint-state flip: {what}"
        self.flips += 1

    def finish(self):
        report(self.name or "flip_budget", {"steps": self.n, "flips": self.flips, "flagged_steps": self.flagged,
                                            "max_flips": max(1, int(self.max_frac * self.n))})
        assert self.flips <= max(1, self.max_frac * self.n), (self.name, self.flips, self.n)


# ---------------------------------------------------------------------------------------------
# per-term reward / state-record comparison (environment.py:390-482, rewards.py:9-138)
# ---------------------------------------------------------------------------------------------
# Tolerance of a scaled metric: |gpu - oracle| <= RTOL * |oracle| + ATOL[name] * |scale|.  The
# absolute floors are in the term's own (unscaled) units and sized from the one-step physics
# error of the fp32 kernel vs the fp32 oracle (qpos ~1e-6, qvel ~1e-4 after 5 substeps from an
# identical state); the count terms (termination, knee/body collision) must be exact.
RTOL = 2e-3
ATOL = {
    "tracking_lin_vel": 1e-4, "tracking_ang_vel": 1e-4, "tracking_orientation": 1e-5,
    "lin_vel_z": 1e-4, "ang_vel_xy": 1e-4, "orientation": 1e-5,
    "torques": 1e-3, "joint_acceleration": 2.0, "mechanical_work": 1e-3, "action_rate": 0.0,
    "stand_still": 1e-5, "stand_still_joint_velocity": 1e-3, "abduction_angle": 1e-6,
    "feet_air_time": 1e-6, "foot_slip": 1e-4, "termination": 0.0, "knee_collision": 0.0,
    "body_collision": 0.0,
}
EXACT_TERMS = ("termination", "knee_collision", "body_collision")
FOOT_Z_THRESHOLDS = (1e-3, 3e-2)  # environment.py:376-378 contact / contact_filt_cm heights


def foot_threshold_flip(oracle_pipe, foot_radius, band=2e-5) -> bool:
    """True when a foot height sits within `band` of one of the contact thresholds in the
    oracle: the fp32 kernel may then see the other side of the comparison (a discrete flip of
    contact / first_contact / air-time state, like a constraint-state flip)."""
    z = oracle_pipe[_abi.P_SITE_XPOS + 2:_abi.P_SITE_XPOS + 12:3] - foot_radius
    return any(abs(z - t).min() < band for t in FOOT_Z_THRESHOLDS)


def metric_errors(gpu_met, oracle_met, scales):
    """Per-term (abs error, allowed) for the 19 metrics (total_dist + 18 scaled terms)."""
    out = {"total_dist": (abs(float(gpu_met[0]) - oracle_met[0]), 1e-5 + RTOL * abs(oracle_met[0]))}
    for k, name in enumerate(_abi.REWARD_NAMES):
        g, o = float(gpu_met[1 + k]), float(oracle_met[1 + k])
        if name in EXACT_TERMS:
            out[name] = (abs(g - np.float32(o)), 0.0)
        else:
            out[name] = (abs(g - o), RTOL * abs(o) + ATOL[name] * abs(scales[k]) + 1e-7)
    return out


def state_errors(gpu_rec, oracle_rec, La, Li):
    """Per-field (abs error, allowed) of the env info in the state record (everything but
    qpos/qvel/qacc_warmstart, compared separately)."""
    io = _abi.imu_buf_offset(La)
    with np.errstate(invalid="ignore"):  # the RNG words are bit patterns (compared separately)
        g = gpu_rec.astype(np.float64)
        o = oracle_rec.astype(np.float64)

    def err(off, n, tol, rtol=0.0):
        return (float(np.abs(g[off:off + n] - o[off:off + n]).max()), tol + rtol * float(np.abs(o[off:off + n]).max()))

    return {
        "last_act": err(_abi.S_LAST_ACT, 12, 0.0),
        "last_vel": err(_abi.S_LAST_VEL, 12, 2e-3, 1e-3),  # joint velocities reach tens of rad/s
        "command": err(_abi.S_COMMAND, 3, 0.0),
        "desired_world_z": err(_abi.S_DESIRED_Z, 3, 1e-6),
        "feet_air_time": err(_abi.S_AIR_TIME, 4, 1e-6),
        "last_contact": err(_abi.S_LAST_CONTACT, 4, 0.0),
        "kick": err(_abi.S_KICK, 2, 0.0),
        "step": err(_abi.S_STEP, 1, 0.0),
        "action_buffer": err(_abi.S_ACT_BUF, 12 * La, 0.0),
        "imu_buffer": err(io, 6 * Li, 5e-3),
    }


class TermStats:
    """Worst error per term over a test, for the report line."""

    def __init__(self):
        self.worst = {}
        self.nonzero = set()  # terms seen nonzero on the GPU

    def add(self, errs):
        for k, (e, _) in errs.items():
            self.worst[k] = max(self.worst.get(k, 0.0), float(e))

    @staticmethod
    def failures(errs):
        return {k: (e, tol) for k, (e, tol) in errs.items() if not e <= tol}


def env_with_model(path, model_struct, n, **kw):
    """A device env built from an edited model struct (known-answer tests on modified physics):
    the env config comes from the reference fixture kwargs, the model from `model_struct`."""
    import ctypes as C
    import common
    e = PupperV3Env(**common.fixture_kwargs(path, **kw), num_envs=n, create_device=False)
    L = _lib.load()
    h = C.c_void_p()
    _lib.check(L.pp3_create(C.byref(model_struct), C.byref(e.config_struct), n, 0, C.byref(h)))
    e._h, e._L = h, L
    _lib.check(L.pp3_set_pipeline_output(h, 1))
    e._keys_buf = _lib.DeviceBuffer(n * 8, 0)
    e._act_buf = _lib.DeviceBuffer(n * _abi.NU * 4, 0)
    e._dr_buf = None
    e._init_host_state()
    return e
