"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py (its cpu_baseline leg and its untimed
accuracy checks one_step_err / qpos_rel_err) import this module, and only as the checker /
CPU baseline -- never as the product path.  See pp3_oracle.c
for what is restated from where and for the parity status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PIPE_STRIDE = 304  # PP3_PIPE_STRIDE of include/pupper_hip.h (pipeline record incl. sensordata)
_LIBS = {}


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib(precision: str = "f64") -> C.CDLL:
    name = {"f64": "liboracle64.so", "f32": "liboracle32.so"}[precision]
    if name not in _LIBS:
        # PP3_ORACLE_DIR: a sanitizer build of the same sources (tools/oracle_sanitize.sh)
        path = os.path.join(os.environ.get("PP3_ORACLE_DIR") or _HERE, name)
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        dp = C.POINTER(C.c_double)
        u32p = C.POINTER(C.c_uint32)
        L.orc_mj_step.argtypes = [C.c_void_p, dp, C.c_int, dp, dp, dp, dp, C.c_int, dp, dp]
        L.orc_mj_forward.argtypes = [C.c_void_p, dp, dp, dp, dp, dp, dp, dp, dp, C.POINTER(C.c_int), dp]
        L.orc_env_reset.argtypes = [C.c_void_p, C.c_void_p, dp, u32p, dp, dp, dp, dp, dp, dp]
        L.orc_env_step.argtypes = [C.c_void_p, C.c_void_p, dp, dp, dp, dp, dp, dp, dp, dp]
        L.orc_env_rollout.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, dp, dp, dp, dp, C.c_int]
        L.orc_env_rollout.restype = C.c_int
        L.orc_threefry2x32.argtypes = [C.c_uint32] * 4 + [u32p]
        L.orc_split.argtypes = [u32p, C.c_int, u32p]
        L.orc_uniform.argtypes = [u32p, C.c_int, C.c_float, C.c_float, C.POINTER(C.c_float)]
        L.orc_choice.argtypes = [u32p, dp, C.c_int]
        L.orc_choice.restype = C.c_int
        L.orc_set_partitionable.argtypes = [C.c_int]
        L.orc_set_ncon_max.argtypes = [C.c_int]
        L.orc_set_ls_noise.argtypes = [C.c_int]
        L.orc_ls_take.argtypes = [C.POINTER(C.c_long)]
        L.orc_data_size.restype = C.c_size_t
        L.orc_boundary_take.restype = C.c_int
        _LIBS[name] = L
    return _LIBS[name]


def _p(a):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _u(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def mj_step(model, qpos, qvel, qacc_ws, ctrl, nsteps=1, dr=None, precision="f64", ncon_max=0, want_pipe=True):
    """nsteps x mj_step with constant ctrl. Returns (qpos, qvel, qacc_ws, pipe, site_xpos)."""
    L = lib(precision)
    q = np.array(qpos, dtype=np.float64).copy()
    v = np.array(qvel, dtype=np.float64).copy()
    w = np.array(qacc_ws, dtype=np.float64).copy()
    c = np.ascontiguousarray(ctrl, dtype=np.float64)
    pipe = np.zeros(PIPE_STRIDE, dtype=np.float64) if want_pipe else None
    sites = np.zeros((8, 3), dtype=np.float64)
    d = None if dr is None else np.ascontiguousarray(dr, dtype=np.float64)
    L.orc_boundary_take()
    L.orc_mj_step(C.byref(model), _p(d), ncon_max, _p(q), _p(v), _p(w), _p(c), nsteps, _p(pipe), _p(sites))
    mj_step.last_boundary = L.orc_boundary_take()
    return q, v, w, pipe, sites


GEOM_BOX = 6  # mjGEOM_BOX (pupperv3_mjx._abi.GEOM_BOX)


def terrain_slots(model):
    """cgeom indices of the world box geoms, in slot order (pp3_set_terrain)."""
    return [g for g in range(model.ncgeom) if model.cgeom_bodyid[g] == 0 and model.cgeom_type[g] == GEOM_BOX]


def model_with_terrain(model, rows):
    """Copy of the model struct whose box geoms hold one env's terrain rows f32[n_boxes, 10]
    (pos, quat, half-size): the oracle's view of a per-env terrain.  Absent boxes (zero size) are
    parked below the floor with zero size, as on the device."""
    m = type(model).from_buffer_copy(model)
    for b, g in enumerate(terrain_slots(model)):
        r = np.asarray(rows[b], dtype=np.float64)
        if not np.any(r[7:10] > 0):
            pos, quat, size = (0.0, 0.0, -1e4), (1.0, 0.0, 0.0, 0.0), (0.0, 0.0, 0.0)
        else:
            q = r[3:7] / np.linalg.norm(r[3:7])
            pos, quat, size = r[0:3], q, r[7:10]
        for k in range(3):
            m.cgeom_pos[g][k] = pos[k]
            m.cgeom_size[g][k] = size[k]
        for k in range(4):
            m.cgeom_quat[g][k] = quat[k]
    return m


def mj_forward(model, qpos, qvel, qacc_ws, ctrl, precision="f64"):
    L = lib(precision)
    M = np.zeros((18, 18))
    qs = np.zeros(18)
    qa = np.zeros(18)
    qb = np.zeros(18)
    nefc = C.c_int()
    pipe = np.zeros(PIPE_STRIDE)
    args = [np.ascontiguousarray(x, dtype=np.float64) for x in (qpos, qvel, qacc_ws, ctrl)]
    L.orc_mj_forward(C.byref(model), *[_p(a) for a in args], _p(M), _p(qs), _p(qa), _p(qb), C.byref(nefc), _p(pipe))
    return dict(M=M, qacc_smooth=qs, qacc=qa, qfrc_bias=qb, nefc=nefc.value, pipe=pipe)


def ls_take(precision: str = "f64") -> dict:
    """Line-search counters of this thread since the last call (pp3_oracle.c orc_ls_take): Newton
    searches, their evaluations, the warm-start choice, and how each search ended -- converged
    (ls_converged), capped (ls_iterations evaluations spent first: the alpha then comes from the
    PrimalSearch exit rule, which MuJoCo's documentation does not specify) or stalled; of the capped,
    those capped in the bracketing phase (`capped_bracketing`; the rest, `capped_one_sided`, ran out
    in the one-sided Newton phase), and how many searches reached the bracketing phase at all."""
    out = (C.c_long * 9)()
    lib(precision).orc_ls_take(out)
    keys = ("evals", "searches", "smooth_starts", "starts", "converged", "capped", "stalled", "bracketing",
            "capped_bracketing")
    d = dict(zip(keys, (int(v) for v in out)))
    d["capped_one_sided"] = d["capped"] - d["capped_bracketing"]
    return d


def with_ls_iterations(model, n):
    """Copy of the model struct with ls_iterations = n (the reference's is 5, xml:57)."""
    m = type(model).from_buffer_copy(model)
    m.ls_iterations = n
    return m


class OracleEnv:
    """Single-env oracle of PupperV3Env.reset/step operating on the device state layout."""

    def __init__(self, model, cfg, dr=None, precision="f64"):
        self.L = lib(precision)
        self.model = model
        self.cfg = cfg
        self.dr = None if dr is None else np.ascontiguousarray(dr, dtype=np.float64)
        La, Li = cfg.latency_len, cfg.imu_latency_len
        self.stride = 98 + 12 * La + 6 * Li
        self.H = cfg.obs_history

    def reset(self, key):
        st = np.zeros(self.stride)
        obs = np.zeros(36 * self.H)
        rew = np.zeros(1)
        done = np.zeros(1)
        met = np.zeros(19)
        pipe = np.zeros(PIPE_STRIDE)
        k = np.ascontiguousarray(key, dtype=np.uint32)
        self.L.orc_env_reset(C.byref(self.model), C.byref(self.cfg), _p(self.dr), _u(k), _p(st), _p(obs),
                             _p(rew), _p(done), _p(met), _p(pipe))
        return dict(state=st, obs=obs, reward=rew[0], done=done[0], metrics=met, pipe=pipe)

    def step(self, s, action):
        st = s["state"].copy()
        obs = s["obs"].copy()
        rew = np.zeros(1)
        done = np.zeros(1)
        met = np.zeros(19)
        pipe = np.zeros(PIPE_STRIDE)
        a = np.ascontiguousarray(action, dtype=np.float64)
        self.L.orc_boundary_take()
        self.L.orc_env_step(C.byref(self.model), C.byref(self.cfg), _p(self.dr), _p(st), _p(obs), _p(a),
                            _p(rew), _p(done), _p(met), _p(pipe))
        # rows decided within rounding of a constraint-state switch during this step (see
        # pp3_oracle.c BOUNDARY_REL): there an fp32 kernel may legitimately take the other branch
        nb = self.L.orc_boundary_take()
        return dict(state=st, obs=obs, reward=rew[0], done=done[0], metrics=met, pipe=pipe, boundary=nb)


def rollout(model, cfg, states, obs, actions, nsteps, nthreads=0, precision="f64"):
    """Batched env rollout (CPU baseline).  Returns (states, obs, rewards, threads_used)."""
    L = lib(precision)
    n = states.shape[0]
    st = np.ascontiguousarray(states, dtype=np.float64).copy()
    ob = np.ascontiguousarray(obs, dtype=np.float64).copy()
    rew = np.zeros((nsteps, n))
    act = None if actions is None else np.ascontiguousarray(actions, dtype=np.float64)
    used = L.orc_env_rollout(C.byref(model), C.byref(cfg), n, nsteps, _p(st), _p(ob), _p(act), _p(rew), nthreads)
    return st, ob, rew, used
