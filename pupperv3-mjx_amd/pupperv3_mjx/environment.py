"""PupperV3Env: the reference's environment surface over the MI355X HIP kernels.

Same constructor knobs and defaults as environment.py:35-121, same reset/step/observation/
reward semantics (environment.py:314-543, rewards.py), executed by the fused HIP kernels in
csrc/pp3_env.hip through the C-ABI (include/pupper_hip.h).  Differences in *form* (not in
numbers), all forced by the device-resident design:

* the env is batched: ``PupperV3Env(..., num_envs=N)``; ``reset(rng)`` takes N keys [N, 2]
  (or one key [2] when N == 1) and ``step(state, action)`` takes actions [N, 12];
* ``State`` fields are numpy host arrays (``obs`` [N, 36H], ``reward`` [N], ``done`` [N],
  ``metrics``/``info`` dicts of [N, ...] arrays), read-only like the reference's immutable JAX
  arrays: a state is edited by assigning new arrays (``state.info["command"] = ...``, as
  test_environment.py:147,186 do), and ``step`` packs an edited state back into the device record;
* reset/step return a ``DeviceState``: obs / reward / done are copied to the host at once, the
  rest (info, metrics, pipeline_state) on first access; a state passed back to ``step`` unedited
  (the usual rollout loop) is not re-uploaded -- the device already holds it;
* the zero-copy path for training loops is ``step_device`` / ``device_fields`` (no host
  round trip); ``State.pipeline_state`` exposes q, qd, x, xd, site_xpos, qfrc_actuator and
  contacts of the last substep (brax State semantics, environment.py:367).
"""
from __future__ import annotations

import ctypes as C
import math
import weakref
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _abi, _lib, domain_randomization, mjcf
from . import rng as _rng


@dataclass
class Transform:
    pos: np.ndarray
    rot: np.ndarray


@dataclass
class Motion:
    vel: np.ndarray
    ang: np.ndarray


@dataclass
class Contact:
    dist: np.ndarray
    geom1: np.ndarray
    geom2: np.ndarray


@dataclass
class PipelineState:
    q: np.ndarray
    qd: np.ndarray
    qacc_warmstart: np.ndarray
    x: Optional[Transform] = None
    xd: Optional[Motion] = None
    site_xpos: Optional[np.ndarray] = None
    qfrc_actuator: Optional[np.ndarray] = None
    qacc: Optional[np.ndarray] = None
    contact: Optional[Contact] = None
    subtree_com: Optional[np.ndarray] = None
    sensordata: Optional[np.ndarray] = None  # mjData.sensordata (model <sensor> order)

    @property
    def qpos(self):
        return self.q

    @property
    def qvel(self):
        return self.qd


@dataclass
class State:
    pipeline_state: PipelineState
    obs: np.ndarray
    reward: np.ndarray
    done: np.ndarray
    metrics: Dict[str, np.ndarray] = field(default_factory=dict)
    info: Dict[str, Any] = field(default_factory=dict)


_LAZY = ("pipeline_state", "metrics", "info", "_record", "_metrics_raw")
_OUTS = ("obs", "reward", "done")


# how the host API's per-step outputs reach the host (host API): the step launch
# stores them into the page-locked block itself (STEP_WRITES_HOST), else a kernel after the launch
# (OUTPUTS_BY_KERNEL, pp3_outputs_to_host) or copy-engine transfers
STEP_WRITES_HOST = True
OUTPUTS_BY_KERNEL = True
# rollout(): trajectories up to this size are stored by the launch into page-locked host memory
TRAJ_PINNED_MAX_BYTES = 256 << 20
# step() returns before its launch completes (obs / reward / done wait for it on first access), with
# at most ASYNC_DEPTH steps in flight; False: every step synchronises before it returns
ASYNC_STEP = True
ASYNC_DEPTH = 2
# step(): the launch reads the actions straight from the page-locked staging block through its device
# mapping instead of after a copy-engine transfer into a device buffer
ACTIONS_ZERO_COPY = True
# step() (with ASYNC_STEP) queues its launch and issues it at the env's next device operation (a
# step from another state, any other call into the library, or the first read of a queued state's
# fields): by then the caller of `state = env.step(state, action)` has dropped the states the launch
# overwrites, so no device snapshot of them is taken (PupperV3Env._flush)
DEFER_LAUNCH = True
# steps queued from one another (each from the state the previous returned) run as ONE fused
# pp3_rollout launch of up to STEP_BATCH steps when they are issued -- bit-equal to single-step
# launches; a queued state still alive at issue ends a launch of its own, so its lazy fields
# (info, metrics, pipeline_state) exist on the device; 1 = one launch per step
STEP_BATCH = 16
# a launch of queued steps stores obs / reward / done into page-locked host memory for its last step
# only (the state that ends it): the states before it were dropped, so nothing can read their rows,
# and each row is 1.2 MB of PCIe stores at 4096 envs.  The steps before are one launch without
# trajectory outputs, the last a launch of its own (bit-equal: a fused launch equals single steps)
LIVE_OUTPUTS_ONLY = True
# cap on one queued batch's page-locked output block ([B][N][36H + 2] floats): the batch length B is
# STEP_BATCH or fewer, so that ASYNC_DEPTH + 1 such blocks stay within a few hundred MB of page-locked
# memory at long observation histories (H = 20 at 4096 envs: 11.8 MB per step row)
STEP_BLOCK_MAX_BYTES = 64 << 20


def _ro(a):
    """Read-only view of a host array handed out in a State (JAX arrays are immutable)."""
    a = np.asarray(a)
    a.flags.writeable = False
    return a


class DeviceState(State):
    """A State returned by PupperV3Env.reset / step (the host surface of the
    device-resident env).  step() returns before its launch has finished -- with DEFER_LAUNCH before
    it is even issued: the env issues it at its next device operation or when this state's fields
    are first read (PupperV3Env._flush).  obs / reward / done are views of the page-locked block
    the launch stores into, made (after waiting for that launch's completion event) on first
    access.  pipeline_state, metrics, info (and the raw record) are
    downloaded on first access -- from the env's live buffers while the env has not launched since,
    else from a device snapshot the env took just before its next launch
    (PupperV3Env._before_launch), so an old state always reads its own data.  Every array is
    read-only; ``unedited()`` tells the env whether the device still holds exactly this state (then
    step() skips the upload).

    Assigning a field is an edit (the next step uploads the state).  Assigning one of the lazy
    fields (pipeline_state, info, metrics) of a state not yet read first downloads the whole lazy
    part (a blocking copy of the state record, metrics and pipeline record, plus a stream sync for
    a snapshot), so the assigned value is what a later read sees; obs / reward / done likewise wait
    for their step first.  A wrapper that assigns state.info every step therefore pays one lazy
    download per step."""

    def __init__(self, env: "PupperV3Env", gen: int, single: bool, obs=None, reward=None, done=None, ready=None):
        d = dict(_env=env, _gen=gen, _single=single, _snap=None, _ids=None, _ready=ready)
        if ready is None:  # outputs already on the host
            d.update(obs=obs, reward=reward, done=done, _out=(obs, reward, done))
        else:  # (lease, completion event slot): views made on first access
            d.update(_out=None)
        self.__dict__.update(d)

    def __getattr__(self, name):
        if name in _OUTS and self.__dict__.get("_ready") is not None:
            self._wait_outputs()
            return self.__dict__[name]
        if name in _LAZY and "_env" in self.__dict__:
            self._materialize()
            return self.__dict__[name]
        raise AttributeError(name)

    @property
    def materialized(self) -> bool:
        return "info" in self.__dict__

    def __setattr__(self, name, value):
        # assigning a lazy field (pipeline_state, info, metrics, ...) of a state not yet read: fetch
        # the issued values first, so the assignment is an edit unedited() sees and nothing
        # downloaded later overwrites it (see the class docstring for the cost)
        if name in _OUTS and self.__dict__.get("_ready") is not None:
            self._wait_outputs()
        if name in _LAZY and "_env" in self.__dict__ and not self.materialized:
            self._materialize()
        object.__setattr__(self, name, value)

    def __copy__(self):
        """A shallow copy sharing this state's arrays.  The original is read in full first (its step
        issued, its outputs waited for, its lazy fields downloaded), so the copy depends on nothing
        the env later overwrites."""
        self._materialize()
        c = object.__new__(type(self))
        c.__dict__.update(self.__dict__)
        return c

    def _wait_outputs(self) -> None:
        """obs / reward / done of a state whose launch may still run (or still be queued): issue it,
        wait for its completion event, then view the page-locked block the launch stored them into."""
        ready = self.__dict__.get("_ready")
        if ready is None:
            return
        if isinstance(ready[0], _StepBatch):  # step j of a batch (STEP_BATCH)
            batch, j = ready
            # a batch still queued is issued now, whether or not this very object is one of its
            # tracked states (a shallow copy of a queued state carries the same _ready)
            if batch is self._env._qb:
                self._env._flush()
            if batch.error is not None:
                raise RuntimeError("the launch of this state's step failed") from batch.error
            if not batch.stored[j]:
                # the row was never written: this state's step ended no launch because every state
                # that could read it had been dropped when the queue was issued (e.g. a copy made
                # of a state that was then dropped); its outputs are gone, not stale
                raise RuntimeError("DeviceState: this step's obs/reward/done were not kept (the state it "
                                   "was copied from was dropped before its step was issued)")
            batch.slot.wait()
            obs, rew, done = batch.views(j, self._single)
        else:
            lease, slot = ready
            slot.wait()
            obs, rew, done = self._env._output_views(lease, self._single)
        self.__dict__.update(obs=obs, reward=rew, done=done, _out=(obs, rew, done), _ready=None)

    def _materialize(self) -> None:
        if self.materialized:
            return
        self._wait_outputs()  # (the launch has completed: its fields are final)
        env = self._env
        src = self._snap
        if src is None and env._gen != self._gen:
            raise RuntimeError("DeviceState: the env launched again without preserving this state (internal error)")
        if src is not None:
            _lib.check(env._raw.pp3_synchronize(env._h))  # the snapshot's d2d copies were queued on the env's stream
        fields = env._lazy_fields()
        got = {}
        for f in fields:  # (raw library calls: a step queued after this state stays queued, DEFER_LAUNCH)
            got[f] = env._download(f, src.ptr.value + env._snap_offsets[f] if src is not None else None, raw=True)
        lazy = env._unpack_lazy(self, got, self._single)
        for k, v in lazy.items():  # never over a value the caller already assigned
            self.__dict__.setdefault(k, v)
        self.__dict__["_ids"] = _identity(lazy["pipeline_state"], lazy["info"], self._out[0])
        if src is not None:
            env._snap_pool.append(src)
            self.__dict__["_snap"] = None

    def unedited(self) -> bool:
        """True when every array step() would upload is the very object this state was issued with."""
        if self.__dict__.get("_ready") is not None:  # outputs not yet viewed: nothing can have been assigned
            return True
        d, o = self.__dict__, self._out
        if d.get("obs") is not o[0] or d.get("reward") is not o[1] or d.get("done") is not o[2]:
            return False
        if not self.materialized:
            return True
        return _same(_identity(d["pipeline_state"], d["info"], d["obs"]), self._ids)


def _identity(ps, info, obs) -> tuple:
    """The objects a state was issued with (strong references, compared by identity: an id() of a
    freed object can be reused by a new one)."""
    return (ps, ps.q, ps.qd, ps.qacc_warmstart, info, tuple(info.items()), obs)


def _same(a: tuple, b: tuple) -> bool:
    if len(a) != len(b):
        return False
    for x, y in zip(a, b):
        if isinstance(x, tuple) and isinstance(y, tuple):
            if len(x) != len(y) or any(kx != ky or vx is not vy for (kx, vx), (ky, vy) in zip(x, y)):
                return False
        elif x is not y:
            return False
    return True


_DEFAULT_LOWER = [-1.220, -0.420, -2.790, -2.510, -3.140, -0.710, -1.220, -0.420, -2.790, -2.510, -3.140, -0.710]
_DEFAULT_UPPER = [2.510, 3.140, 0.710, 1.220, 0.420, 2.790, 2.510, 3.140, 0.710, 1.220, 0.420, 2.790]
_DEFAULT_POSE = [0.26, 0.0, -0.52, -0.26, 0.0, 0.52, 0.26, 0.0, -0.52, -0.26, 0.0, 0.52]


class PupperV3Env:
    """Environment for training the Pupper V3 joystick policy on MI355X."""

    def __init__(
        self,
        path: str,
        reward_config: Dict,
        action_scale: float,
        observation_history: int,
        joint_lower_limits: Sequence = tuple(_DEFAULT_LOWER),
        joint_upper_limits: Sequence = tuple(_DEFAULT_UPPER),
        dof_damping: float = 0.25,
        position_control_kp: float = 5.0,
        start_position_config: domain_randomization.StartPositionRandomization = (
            domain_randomization.StartPositionRandomization(
                x_min=-2.0, x_max=2.0, y_min=-2.0, y_max=2.0, z_min=0.15, z_max=0.20)),
        foot_site_names: Sequence[str] = ("leg_front_r_3_foot_site", "leg_front_l_3_foot_site",
                                          "leg_back_r_3_foot_site", "leg_back_l_3_foot_site"),
        torso_name: str = "base_link",
        upper_leg_body_names: Sequence[str] = ("leg_front_r_2", "leg_front_l_2", "leg_back_r_2", "leg_back_l_2"),
        lower_leg_body_names: Sequence[str] = ("leg_front_r_3", "leg_front_l_3", "leg_back_r_3", "leg_back_l_3"),
        resample_velocity_step: int = 500,
        linear_velocity_x_range: Tuple[float, float] = (-0.75, 0.75),
        linear_velocity_y_range: Tuple[float, float] = (-0.5, 0.5),
        angular_velocity_range: Tuple[float, float] = (-2.0, 2.0),
        zero_command_probability: float = 0.01,
        stand_still_command_threshold: float = 0.1,
        maximum_pitch_command: float = 0.0,
        maximum_roll_command: float = 0.0,
        default_pose: Sequence = tuple(_DEFAULT_POSE),
        desired_abduction_angles: Sequence = (0.0, 0.0, 0.0, 0.0),
        angular_velocity_noise: float = 0.3,
        gravity_noise: float = 0.1,
        motor_angle_noise: float = 0.1,
        last_action_noise: float = 0.01,
        kick_vel: float = 0.2,
        kick_probability: float = 0.02,
        terminal_body_z: float = 0.1,
        early_termination_step_threshold: int = 500,
        terminal_body_angle: float = 0.52,
        foot_radius: float = 0.02,
        environment_timestep: float = 0.02,
        physics_timestep: float = 0.004,
        latency_distribution: Sequence = (0.2, 0.8),
        imu_latency_distribution: Sequence = (0.5, 0.5),
        desired_world_z_in_body_frame: Sequence = (0.0, 0.0, 1.0),
        use_imu: bool = True,
        *,
        num_envs: int = 1,
        device: int = 0,
        rng_partitionable: bool = True,
        pipeline_output: bool = True,
        create_device: bool = True,
        max_contacts: int = 0,
    ):
        cm = mjcf.load(path)
        m = cm.struct
        # environment.py:165-180: dt override, PD gains, home keyframe, n_frames
        m.timestep = float(physics_timestep)
        for i in range(_abi.NU):
            m.actuator_gainprm[i][0] = position_control_kp
            m.actuator_biasprm[i][1] = -position_control_kp
            m.actuator_biasprm[i][2] = -dof_damping
        default_pose = np.asarray(default_pose, dtype=np.float64)
        m.key_qpos[7:] = list(default_pose)
        n_frames = int(environment_timestep // m.timestep)
        self.sys_model = cm
        self._dt = environment_timestep
        self._n_frames = n_frames
        self._reward_config = reward_config
        self._torso_idx = cm.body_id(torso_name)
        assert self._torso_idx != -1, "torso not found"
        self._torso_geom_ids = cm.body_geom_ids(torso_name)
        feet = [cm.site_id(f) for f in foot_site_names]
        assert not any(i == -1 for i in feet), "Site not found."
        self._feet_site_id = np.array(feet)
        lower = [cm.body_id(n) for n in lower_leg_body_names]
        assert not any(i == -1 for i in lower), "Body not found."
        self._lower_leg_body_id = np.array(lower)
        self._upper_leg_geom_ids = np.concatenate([cm.body_geom_ids(n) for n in upper_leg_body_names])
        self._default_pose = default_pose
        self._action_scale = float(action_scale)
        self._observation_history = int(observation_history)
        self.observation_dim = _abi.OBS_DIM
        self.lowers = np.asarray(joint_lower_limits, dtype=np.float64)
        self.uppers = np.asarray(joint_upper_limits, dtype=np.float64)
        self._latency_distribution = np.asarray(latency_distribution, dtype=np.float32)
        self._imu_latency_distribution = np.asarray(imu_latency_distribution, dtype=np.float32)
        self._use_imu = bool(use_imu)
        self._partitionable = bool(rng_partitionable)
        self.num_envs = int(num_envs)
        self.device = int(device)

        c = _abi.EnvConfig()
        c.n_frames = n_frames
        c.obs_history = self._observation_history
        c.use_imu = int(use_imu)
        c.latency_len = len(self._latency_distribution)
        c.imu_latency_len = len(self._imu_latency_distribution)
        c.resample_velocity_step = int(resample_velocity_step)
        c.early_termination_step_threshold = int(early_termination_step_threshold)
        c.torso_body = self._torso_idx
        c.feet_site[:] = [int(v) for v in feet]
        c.lower_leg_body[:] = [int(v) for v in lower]
        ul = [int(v) for v in self._upper_leg_geom_ids]
        c.n_upper_leg_geoms = len(ul)
        c.upper_leg_geoms[:len(ul)] = ul
        tg = [int(v) for v in self._torso_geom_ids]
        c.n_torso_geoms = len(tg)
        c.torso_geoms[:len(tg)] = tg
        c.rng_partitionable = int(rng_partitionable)
        c.ncon_max = int(max_contacts)  # contact cap, deepest kept: 0 = default 8; else 8 or 16
        c.latency_dist[:c.latency_len] = [float(v) for v in self._latency_distribution]
        c.imu_latency_dist[:c.imu_latency_len] = [float(v) for v in self._imu_latency_distribution]
        c.action_scale = float(action_scale)
        c.default_pose[:] = list(default_pose)
        c.joint_lower[:] = [float(v) for v in self.lowers]
        c.joint_upper[:] = [float(v) for v in self.uppers]
        c.desired_abduction[:] = [float(v) for v in desired_abduction_angles]
        sp = start_position_config
        c.start_pos_min[:] = [sp.x_min, sp.y_min, sp.z_min]
        c.start_pos_max[:] = [sp.x_max, sp.y_max, sp.z_max]
        c.lin_vel_x_range[:] = list(linear_velocity_x_range)
        c.lin_vel_y_range[:] = list(linear_velocity_y_range)
        c.ang_vel_range[:] = list(angular_velocity_range)
        c.zero_command_probability = zero_command_probability
        c.stand_still_command_threshold = stand_still_command_threshold
        c.max_pitch_command = maximum_pitch_command
        c.max_roll_command = maximum_roll_command
        c.ang_vel_noise = angular_velocity_noise
        c.gravity_noise = gravity_noise
        c.motor_angle_noise = motor_angle_noise
        c.last_action_noise = last_action_noise
        c.kick_vel = kick_vel
        c.kick_probability = kick_probability
        c.terminal_body_z = terminal_body_z
        c.terminal_body_angle = terminal_body_angle
        c.foot_radius = foot_radius
        c.env_dt = environment_timestep
        c.dt = m.timestep * n_frames
        c.desired_world_z[:] = [float(v) for v in desired_world_z_in_body_frame]
        scales = reward_config.rewards.scales
        c.reward_scales[:] = [float(scales[k]) for k in _abi.REWARD_NAMES]
        c.tracking_sigma = float(reward_config.rewards.tracking_sigma)
        self.config_struct = c
        self._reward_keys = list(scales.keys())
        self._sys = domain_randomization.System(
            geom_friction=cm.geom_friction.copy(),
            actuator_gainprm=np.pad(np.array(m.actuator_gainprm[:], dtype=np.float64), ((0, 0), (0, 7))),
            actuator_biasprm=np.pad(np.array(m.actuator_biasprm[:], dtype=np.float64), ((0, 0), (0, 7))),
            body_ipos=np.array(m.body_ipos[:], dtype=np.float64),
            body_inertia=np.array(m.body_inertia[:], dtype=np.float64),
            body_mass=np.array(m.body_mass[:], dtype=np.float64),
        )
        self._h = None
        self.stride = _abi.state_stride(c.latency_len, c.imu_latency_len)
        self._pipeline_output = bool(pipeline_output)
        if not create_device:  # host-only construction (tests/oracle tooling): structs, no GPU
            return

        L = _lib.load()
        h = C.c_void_p()
        _lib.check(L.pp3_create(C.byref(m), C.byref(c), self.num_envs, self.device, C.byref(h)))
        self._h = h
        self._raw = L
        self._qb = None
        self._L = _FlushingLib(self, L)  # every call into the library issues the queued steps first
        assert int(L.pp3_state_stride(h)) == self.stride
        _lib.check(L.pp3_set_pipeline_output(h, int(pipeline_output)))
        self._keys_buf = _lib.DeviceBuffer(self.num_envs * 8, self.device)
        self._act_buf = _lib.DeviceBuffer(self.num_envs * _abi.NU * 4, self.device)
        self._dr_buf = None
        self._init_host_state()

    def _init_host_state(self) -> None:
        """Bookkeeping of the lazy host surface (DeviceState): generation counter of the device
        buffers, the last issued state, and a pool of device snapshots of its lazy fields."""
        self._gen = 0
        self._issued = None
        self._qb = None  # the steps queued for the next device operation (_StepBatch; DEFER_LAUNCH)
        self._batch_pool = _lib.BlockPool()
        self._batch_spares = False  # the pool holds its spares (_step_queued)
        self._n_snapshots = 0  # device snapshots taken of issued states (_before_launch)
        self._snap_pool = []
        self._pin_pool = _lib.BlockPool()  # page-locked output blocks (obs | reward | done) of issued states
        self._traj_pool = {}   # page-locked rollout trajectory blocks, per unroll length
        # page-locked action staging: a ring of ASYNC_DEPTH blocks, each reused only after the launch
        # that read it has completed (its event)
        self._act_ring = [_ActSlot(self, max(1, STEP_BATCH) * self.num_envs * _abi.NU * 4)
                          for _ in range(max(1, ASYNC_DEPTH))]
        self._act_i = 0
        self._lazy_extra = {}  # field id -> info hook (wrappers.AutoResetEpisodeEnv: the episode record)
        self._issue_capture = None  # () -> host data a wrapper attaches to each state when it is issued
        self._field_elems = {f: self.device_field(f)[1] for f in (_abi.F_STATE, _abi.F_METRICS, _abi.F_PIPELINE)}
        self._field_elems[_abi.F_EPISODE] = _abi.EP_STRIDE
        off, self._snap_offsets = 0, {}
        for f in (_abi.F_STATE, _abi.F_METRICS, _abi.F_PIPELINE, _abi.F_EPISODE):
            self._snap_offsets[f] = off
            off += (self.num_envs * self._field_elems[f] * 4 + 255) // 256 * 256
        self._snap_bytes = off

    # ------------------------------------------------------------------ reference helpers
    def sample_command(self, rng) -> np.ndarray:
        """environment.py:246-272 on the host: one key [2] or a batch [..., 2] -> f32[..., 3]
        (lin_vel_x, lin_vel_y, ang_vel_yaw), near zero with probability zero_command_probability.
        The same jax.random draws as the device's reset / resample (env_step_kernel
        sample_command), so a key gives the identical command."""
        c, p = self.config_struct, self._partitionable
        k = _rng.split(np.asarray(rng, dtype=np.uint32), 6, p)
        f = np.float32
        vx = _rng.uniform(k[..., 1, :], (1,), f(c.lin_vel_x_range[0]), f(c.lin_vel_x_range[1]), p)[..., 0]
        vy = _rng.uniform(k[..., 2, :], (1,), f(c.lin_vel_y_range[0]), f(c.lin_vel_y_range[1]), p)[..., 0]
        wz = _rng.uniform(k[..., 3, :], (1,), f(c.ang_vel_range[0]), f(c.ang_vel_range[1]), p)[..., 0]
        pz = _rng.uniform(k[..., 4, :], (1,), partitionable=p)[..., 0]
        thr = f(c.stand_still_command_threshold)
        near_zero = _rng.uniform(k[..., 5, :], (3,), -thr, thr, p)
        cmd = np.stack([vx, vy, wz], axis=-1)
        return np.where((pz < f(c.zero_command_probability))[..., None], near_zero, cmd).astype(np.float32)

    def sample_body_orientation(self, rng) -> np.ndarray:
        """environment.py:274-298 on the host: the desired world z in the body frame rotated by a
        random roll / pitch (brax math.euler_to_quat in degrees, then math.rotate), f32[..., 3]."""
        c, p = self.config_struct, self._partitionable
        k = _rng.split(np.asarray(rng, dtype=np.uint32), 3, p)
        f = np.float32
        pitch = _rng.uniform(k[..., 1, :], (1,), f(-1), f(1), p)[..., 0] * f(c.max_pitch_command)
        roll = _rng.uniform(k[..., 2, :], (1,), f(-1), f(1), p)[..., 0] * f(c.max_roll_command)
        h1, h2 = roll * f(np.pi / 360), pitch * f(np.pi / 360)  # half angles (yaw 0)
        c1, s1, c2, s2 = np.cos(h1), np.sin(h1), np.cos(h2), np.sin(h2)
        q = np.stack([c1 * c2, s1 * c2, c1 * s2, s1 * s2], axis=-1).astype(np.float32)
        v = np.broadcast_to(np.asarray(c.desired_world_z[:], dtype=np.float32), q.shape[:-1] + (3,))
        s, u = q[..., :1], q[..., 1:]
        r = 2 * np.sum(u * v, -1, keepdims=True) * u + (s * s - np.sum(u * u, -1, keepdims=True)) * v
        return (r + 2 * s * np.cross(u, v)).astype(np.float32)

    def initial_action_buffer(self) -> np.ndarray:
        """environment.py:300-301: zeros [12, len(latency_distribution)]."""
        return np.zeros((_abi.NU, len(self._latency_distribution)), dtype=np.float32)

    def initial_imu_buffer(self) -> np.ndarray:
        """environment.py:303-312: [6, len(imu_latency_distribution)] zeros with gravity z = -1
        (rows: angular velocity xyz, gravity xyz)."""
        buf = np.zeros((6, len(self._imu_latency_distribution)), dtype=np.float32)
        buf[5, :] = -1.0
        return buf

    # ------------------------------------------------------------------ properties
    @property
    def dt(self) -> float:
        return self.sys_model.struct.timestep * self._n_frames

    @property
    def observation_size(self) -> int:
        return self.observation_dim * self._observation_history

    @property
    def action_size(self) -> int:
        return _abi.NU

    @property
    def sys(self) -> domain_randomization.System:
        return self._sys

    def render(self, trajectory, camera: Optional[str] = None, height: int = 240, width: int = 320,
               env_index: int = 0, meshdir: Optional[str] = None) -> List[np.ndarray]:
        """environment.py:545-547 (-> Brax PipelineEnv.render): one u8 [height, width, 3] frame per
        state of `trajectory` (States, PipelineStates or qpos arrays; batched ones give env
        `env_index`), rasterised on the GPU by render.py / pp3_render.  `camera` defaults to "track"
        as in the reference (the stock model defines only "tracking_cam"; an unknown name raises,
        as MuJoCo does); None after that default is not possible, -1 selects a free camera."""
        from . import render as _render
        camera = camera or "track"
        qs = []
        for st in trajectory:
            ps = getattr(st, "pipeline_state", st)
            q = np.asarray(getattr(ps, "q", ps), dtype=np.float64)
            qs.append(q[env_index] if q.ndim == 2 else q)
        key = meshdir
        if getattr(self, "_render_scene", None) is None or self._render_key != key:
            self._render_scene = _render.Scene(self.sys_model, meshdir)
            self._render_key = key
        cam = None if camera == -1 else camera
        return _render.render_qpos(self._render_scene, qs, cam, height, width, self.device)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.pp3_destroy(self._h)
            self._h = None
        for b in (getattr(self, "_roll_bufs", None) or (0, []))[1]:
            b.free()
        self._roll_bufs = None
        # free page-locked blocks go with their pools; leased ones are freed when their arrays die
        if getattr(self, "_pin_pool", None) is not None:
            self._pin_pool.retire()
        if getattr(self, "_batch_pool", None) is not None:
            self._batch_pool.retire()
        for pool in (getattr(self, "_traj_pool", None) or {}).values():
            pool.retire()
        for slot in getattr(self, "_act_ring", None) or ():
            slot.close()
        self._act_ring = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ DR
    def set_domain_randomization(self, sys_batched: Optional[domain_randomization.System]) -> None:
        """Upload the per-env parameters of a batched System (or None to disable DR)."""
        if sys_batched is None:
            _lib.check(self._L.pp3_set_dr(self._h, None))
            return
        table = np.ascontiguousarray(sys_batched.dr_table(), dtype=np.float32)
        if table.shape[0] != self.num_envs:
            raise ValueError("DR batch size must equal num_envs")
        _lib.check(self._L.pp3_copy_field_from_host(self._h, _abi.F_DR, table.ctypes.data_as(C.c_void_p), table.nbytes))

    # ------------------------------------------------------------------ terrain
    @property
    def terrain_slots(self) -> int:
        """World box geoms in the model (obstacles.add_boxes_to_model); each is a per-env slot."""
        return int(self._L.pp3_terrain_slots(self._h))

    def set_terrain(self, boxes: Optional[np.ndarray]) -> None:
        """Per-env terrain boxes f32[num_envs, terrain_slots, 10] (pos, quat wxyz, half sizes;
        all-zero half sizes = absent), or None for the model's static boxes (pp3_set_terrain)."""
        if boxes is None:
            _lib.check(self._L.pp3_set_terrain(self._h, None, 0))
            return
        b = np.ascontiguousarray(boxes, dtype=np.float32)
        if b.ndim != 3 or b.shape[0] != self.num_envs or b.shape[2] != _abi.TERRAIN_BOX:
            raise ValueError(f"terrain must be [num_envs, n_boxes, {_abi.TERRAIN_BOX}], got {b.shape}")
        _lib.check(self._L.pp3_set_terrain(self._h, b.ctypes.data_as(C.c_void_p), b.shape[1]))

    # ------------------------------------------------------------------ device API
    def device_field(self, field_id: int) -> Tuple[int, int]:
        """(device pointer, elements per env) of a PP3_F_* buffer."""
        p = C.c_void_p()
        n = C.c_int64()
        _lib.check(self._L.pp3_field(self._h, field_id, C.byref(p), C.byref(n)))
        return p.value, n.value

    def reset_device(self, keys_dev: int, mask_dev: Optional[int] = None, stream: Optional[int] = None) -> None:
        self._before_launch()
        _lib.check(self._L.pp3_reset(self._h, C.c_void_p(keys_dev), C.c_void_p(mask_dev) if mask_dev else None,
                                     C.c_void_p(stream) if stream else None))

    def step_device(self, actions_dev: int, stream: Optional[int] = None) -> None:
        self._before_launch()
        _lib.check(self._L.pp3_step(self._h, C.c_void_p(actions_dev), C.c_void_p(stream) if stream else None))

    def synchronize(self) -> None:
        _lib.check(self._L.pp3_synchronize(self._h))

    def _get(self, field_id: int, dtype=np.float32, raw: bool = False) -> np.ndarray:
        """A field of the device buffers (after the queued step, if any; `raw`: as they are now)."""
        L = self._raw if raw else self._L
        p, n = C.c_void_p(), C.c_int64()
        _lib.check(L.pp3_field(self._h, field_id, C.byref(p), C.byref(n)))
        out = np.empty((self.num_envs, n.value), dtype=np.float32)
        _lib.check(L.pp3_copy_field_to_host(self._h, field_id, out.ctypes.data_as(C.c_void_p), out.nbytes))
        return out

    def _put(self, field_id: int, arr: np.ndarray) -> None:
        self._before_launch()
        a = np.ascontiguousarray(arr, dtype=np.float32)
        _lib.check(self._L.pp3_copy_field_from_host(self._h, field_id, a.ctypes.data_as(C.c_void_p), a.nbytes))

    # ------------------------------------------------------------------ host API
    def _batch_keys(self, rng) -> Tuple[np.ndarray, bool]:
        k = np.asarray(rng, dtype=np.uint32)
        single = k.ndim == 1
        k = k.reshape(-1, 2)
        if k.shape[0] != self.num_envs:
            raise ValueError(f"reset expects {self.num_envs} keys, got {k.shape[0]}")
        return np.ascontiguousarray(k), single

    def reset(self, rng) -> State:
        keys, single = self._batch_keys(rng)
        self._keys_buf.upload(keys)
        self.reset_device(self._keys_buf.ptr.value)
        return self._issue(single)

    def step(self, state: State, action) -> State:
        if ASYNC_STEP and DEFER_LAUNCH and STEP_WRITES_HOST:
            return self._step_queued(state, action)
        self._flush()
        single = _single_of(state)
        act = np.ascontiguousarray(np.asarray(action, dtype=np.float32).reshape(self.num_envs, _abi.NU))
        if not self.holds(state):
            self._write_state(state)
        # actions through a page-locked staging block of the ring; the launch that last read this
        # block has completed once its event has (at most ASYNC_DEPTH steps in flight)
        slot = self._act_ring[self._act_i]
        self._act_i = (self._act_i + 1) % len(self._act_ring)
        slot.wait()
        np.copyto(slot.arr[:act.size], act.reshape(-1))
        if ACTIONS_ZERO_COPY:
            act_ptr = C.c_void_p(slot.block.device_ptr())
        else:  # copied on the env's stream ahead of the launch
            _lib.check(self._L.pp3_memcpy_h2d_async(self._act_buf.ptr, slot.block.ptr, act.nbytes,
                                                     self._L.pp3_stream(self._h)))
            act_ptr = self._act_buf.ptr
        if not STEP_WRITES_HOST:
            self.step_device(act_ptr.value)
            slot.record()
            return self._issue(single)
        # the step launch itself stores obs | reward | done into the page-locked output block (a
        # one-step pp3_rollout whose trajectory rows are the block's device mapping): no copy after it
        n, D = self.num_envs, self.observation_size
        lease = _lib.PinnedBlock.take(4 * n * (D + 2), self._pin_pool)
        dev = lease.device_ptr()
        self._before_launch()
        _lib.check(self._L.pp3_rollout(self._h, act_ptr, 0, 1, C.c_void_p(dev + 4 * n * D),
                                       C.c_void_p(dev + 4 * n * (D + 1)), C.c_void_p(dev), None))
        slot.record()
        if ASYNC_STEP:  # no host sync: the State's outputs wait for this event when first read
            return self._issue(single, lease, slot)
        return self._issue(single, lease)

    def rollout_device(self, actions_dev: int, action_stride: int, nsteps: int, reward_dev: Optional[int] = None,
                       done_dev: Optional[int] = None, obs_dev: Optional[int] = None,
                       stream: Optional[int] = None) -> None:
        """pp3_rollout: `nsteps` steps fused into one launch; step t reads actions_dev + t *
        action_stride floats; optional trajectory outputs reward/done f32[nsteps][N], obs
        f32[nsteps][N][36H] (device pointers)."""
        self._before_launch()
        vp = lambda p: C.c_void_p(p) if p else None  # noqa: E731
        _lib.check(self._L.pp3_rollout(self._h, C.c_void_p(actions_dev), int(action_stride), int(nsteps),
                                       vp(reward_dev), vp(done_dev), vp(obs_dev), vp(stream)))

    def _step_queued(self, state: State, action) -> State:
        """step() with DEFER_LAUNCH: the step joins the queued batch when `state` is the batch's last
        state (the loop `state = env.step(state, action)`), else the queue is issued first and a new
        batch starts from `state`.  Nothing is launched here (see _flush)."""
        single = _single_of(state)
        act = np.asarray(action, dtype=np.float32).reshape(self.num_envs, _abi.NU)
        qb = self._qb
        if qb is not None and (qb.n >= qb.cap or qb.tail() is not state):
            self._flush()
            qb = None
        if qb is None:
            if not self.holds(state):
                self._write_state(state)
            # a page-locked action block of the ring (reused once the launch that read it completed)
            slot = self._act_ring[self._act_i]
            self._act_i = (self._act_i + 1) % len(self._act_ring)
            slot.wait()
            n, D, B = self.num_envs, self.observation_size, self._step_batch_len()
            lease = _lib.PinnedBlock.take(4 * B * n * (D + 2), self._batch_pool)
            if not self._batch_spares:
                # a step loop cycles through ASYNC_DEPTH + 1 output blocks (the batch in flight, the
                # one queuing, the one whose tail state is still the caller's): allocated now, not
                # as a multi-millisecond page-locked allocation in the middle of the loop
                self._batch_spares = True
                for _ in range(max(1, ASYNC_DEPTH)):
                    self._batch_pool.append(_lib.PinnedBlock(4 * B * n * (D + 2)))
            qb = self._qb = _StepBatch(self, slot, lease, B)
        j = qb.n
        np.copyto(qb.act[j], act)
        st = DeviceState(self, qb.gen0 + j + 1, single, ready=(qb, j))
        st.__dict__["_capture"] = self._issue_capture() if self._issue_capture is not None else None
        qb.states.append(weakref.ref(st))
        qb.n += 1
        return st

    def _step_batch_len(self) -> int:
        """Steps per queued batch: STEP_BATCH, fewer where its output block would exceed
        STEP_BLOCK_MAX_BYTES."""
        row = 4 * self.num_envs * (self.observation_size + 2)
        return max(1, min(max(1, STEP_BATCH), STEP_BLOCK_MAX_BYTES // row))

    def flush(self) -> None:
        """Issue the steps step() has queued (DEFER_LAUNCH) onto the env's stream.  Needed only by
        callers that read the device buffers (device_field pointers) outside the library after a
        host-API step: the library's own calls and every State field read issue the queue first."""
        self._flush()

    def _flush(self) -> None:
        """Issue the steps queued by DEFER_LAUNCH (no-op when none are): fused pp3_rollout launches
        that end at every queued state still alive and at the last one (a dropped state's device
        fields are never needed; a live one's are snapshotted before the next launch overwrites
        them, _before_launch), each storing the obs | reward | done of the state that ends it (with
        LIVE_OUTPUTS_ONLY; else of all its steps) into the batch's page-locked block; then the
        completion event of the batch's action block."""
        qb = self._qb
        if qb is None:
            return
        self._qb = None  # (detached first: _before_launch and the library calls below flush again)
        if qb.n == 0:
            return
        n, D, B = self.num_envs, self.observation_size, qb.cap
        dev = qb.lease.device_ptr()
        act_dev = qb.slot.block.device_ptr()
        ends = [j for j, r in enumerate(qb.states) if j == qb.n - 1 or r() is not None]
        start = 0
        try:
            for e in ends:
                self._before_launch()
                # (device addresses as plain ints: the c_void_p argtypes convert them)
                if LIVE_OUTPUTS_ONLY and e > start:  # steps start .. e-1: dropped states, no host rows
                    _lib.check(self._raw.pp3_rollout(self._h, act_dev + 4 * start * n * _abi.NU,
                                                     n * _abi.NU, e - start, None, None, None, None))
                    start = e
                _lib.check(self._raw.pp3_rollout(
                    self._h, act_dev + 4 * start * n * _abi.NU, n * _abi.NU, e - start + 1,
                    dev + 4 * (B * n * D + start * n), dev + 4 * (B * n * (D + 1) + start * n),
                    dev + 4 * start * n * D, None))
                for j in range(start if not LIVE_OUTPUTS_ONLY else e, e + 1):
                    qb.stored[j] = True
                self._gen = qb.gen0 + e + 1
                self._issued = qb.states[e]
                start = e + 1
        except BaseException as exc:  # the queued states' reads re-raise this instead of viewing unwritten rows
            qb.error = exc
            raise
        qb.slot.record()

    def rollout(self, state: State, actions) -> Tuple[State, Dict[str, np.ndarray]]:
        """The unroll of brax's generate_unroll ([ext] brax 0.12.1 training/acting.py: a lax.scan of
        env.step) with the K actions given up front, as ONE fused launch: returns the state after
        the last step (what K step() calls return) and the per-step trajectory {"obs": [K, N, 36H],
        "reward": [K, N], "done": [K, N]} (single-env states: [K, 36H] / [K]).  Bit for bit the
        same as K step() calls."""
        self._flush()
        single = _single_of(state)
        n, D = self.num_envs, self.observation_size
        act = np.ascontiguousarray(np.asarray(actions, dtype=np.float32))
        if act.ndim < 2 or act.size % (n * _abi.NU):
            raise ValueError(f"actions must be [K, {n}, {_abi.NU}] (got {np.shape(actions)})")
        K = act.size // (n * _abi.NU)
        if not self.holds(state):
            self._write_state(state)
        blk = self._traj_block(K)
        bufs = self._rollout_buffers(K, outputs=blk is None)
        bufs[0].upload(act)
        if blk is not None:
            # the trajectory lands in one page-locked block that the fused launch stores into through
            # its device mapping (no copy after the launch; the arrays are views that keep it leased)
            lease, (p_obs, p_rew, p_done) = blk
            self.rollout_device(bufs[0].ptr.value, n * _abi.NU, K, p_rew, p_done, p_obs)
            self.synchronize()
            obs, rew, done = self._traj_views(lease, K)
        else:  # a long unroll: device buffers, copied out after the launch
            self.rollout_device(bufs[0].ptr.value, n * _abi.NU, K, bufs[1].ptr.value, bufs[2].ptr.value,
                                bufs[3].ptr.value)
            self.synchronize()
            rew = np.empty((K, n), np.float32)
            done = np.empty((K, n), np.float32)
            obs = np.empty((K, n, D), np.float32)
            for b, a in zip(bufs[1:], (rew, done, obs)):
                b.download(a)
        traj = {"obs": obs, "reward": rew, "done": done}
        if single:
            traj = {k: v[:, 0] for k, v in traj.items()}
        return self._issue(single), traj

    def rollout_policy(self, state: State, policy, nsteps: int) -> Tuple[State, Dict[str, np.ndarray]]:
        """brax's generate_unroll with the policy in the loop, on device (pp3_rollout_policy):
        `policy` (an `export.DevicePolicy` with 12 outputs) acts on the env's observation buffer
        before each of the `nsteps` steps; no host round trip until the end.  Returns the state
        after the last step and {"obs": [K, N, 36H], "action": [K, N, 12], "reward": [K, N],
        "done": [K, N]} (single-env states: without the N axis)."""
        self._flush()
        single = _single_of(state)
        n, D, K = self.num_envs, self.observation_size, int(nsteps)
        if K < 1:
            raise ValueError("nsteps must be >= 1")
        if not self.holds(state):
            self._write_state(state)
        blk = self._traj_block(K)  # obs / reward / done straight into page-locked memory (see rollout)
        bufs = self._rollout_buffers(K, outputs=blk is None)
        self._before_launch()
        outs = blk[1] if blk is not None else (bufs[3].ptr.value, bufs[1].ptr.value, bufs[2].ptr.value)
        _lib.check(self._L.pp3_rollout_policy(self._h, policy._h, K, bufs[0].ptr, C.c_void_p(outs[1]),
                                              C.c_void_p(outs[2]), C.c_void_p(outs[0]), None))
        self.synchronize()
        traj = {"action": np.empty((K, n, _abi.NU), np.float32)}  # (the actions stay on the device for the steps)
        bufs[0].download(traj["action"])
        if blk is not None:
            traj["obs"], traj["reward"], traj["done"] = self._traj_views(blk[0], K)
        else:
            traj.update(obs=np.empty((K, n, D), np.float32), reward=np.empty((K, n), np.float32),
                        done=np.empty((K, n), np.float32))
            for b, k in zip(bufs[1:], ("reward", "done", "obs")):
                b.download(traj[k])
        if single:
            traj = {k: v[:, 0] for k, v in traj.items()}
        return self._issue(single), traj

    def _traj_block(self, K: int):
        """A page-locked block for a K-step trajectory [obs K x N x 36H | reward K x N | done K x N] and
        the device addresses of its three parts, or None above TRAJ_PINNED_MAX_BYTES."""
        n, D = self.num_envs, self.observation_size
        nbytes = 4 * K * n * (D + 2)
        if nbytes > TRAJ_PINNED_MAX_BYTES:
            return None
        for k in [k for k in self._traj_pool if k != K]:  # keep free blocks of the current length only
            self._traj_pool.pop(k).retire()  # (its leased blocks are freed when released)
        if K not in self._traj_pool:
            self._traj_pool[K] = _lib.BlockPool()
        lease = _lib.PinnedBlock.take(nbytes, self._traj_pool[K])
        dev = lease.device_ptr()
        return lease, (dev, dev + 4 * K * n * D, dev + 4 * K * n * (D + 1))

    def _traj_views(self, lease, K: int):
        """(obs, reward, done) read-only views of a filled _traj_block."""
        n, D = self.num_envs, self.observation_size
        flat = np.asarray(lease)
        return (flat[:K * n * D].reshape(K, n, D), flat[K * n * D:K * n * (D + 1)].reshape(K, n),
                flat[K * n * (D + 1):].reshape(K, n))  # (read-only: a lease's arrays are)

    def _rollout_buffers(self, K: int, outputs: bool) -> list:
        """Device buffers of rollout(): actions for K steps, and with `outputs` the reward, done and
        obs trajectories (only for unrolls too long for the page-locked block); kept and grown."""
        cur = getattr(self, "_roll_bufs", None)
        n, D = self.num_envs, self.observation_size
        sizes = [4 * K * n * _abi.NU] + ([4 * K * n, 4 * K * n, 4 * K * n * D] if outputs else [])
        if cur is None or len(cur[1]) < len(sizes) or any(b.nbytes < s for b, s in zip(cur[1], sizes)):
            if cur is not None:
                for b in cur[1]:
                    b.free()
            cur = (K, [_lib.DeviceBuffer(sz, self.device) for sz in sizes])
            self._roll_bufs = cur
        return cur[1]

    def holds(self, state: State) -> bool:
        """The device buffers hold exactly `state`: the last state this env issued, unedited, and
        no launch or upload since."""
        qb = self._qb
        if qb is not None and qb.n and qb.tail() is state:
            return True  # the queued steps' last state (held once they are issued; never edited before)
        self._flush()  # (a queued step's state is held once its launch is issued)
        return (isinstance(state, DeviceState) and state.__dict__.get("_env") is self and state._gen == self._gen
                and state.unedited())

    # lazy host state: obs / reward / done now, the rest on first access (DeviceState)
    def _lazy_fields(self) -> Tuple[int, ...]:
        return ((_abi.F_STATE, _abi.F_METRICS) + ((_abi.F_PIPELINE,) if self._pipeline_output else ())
                + tuple(self._lazy_extra))

    def _download(self, field_id: int, src_dev: Optional[int] = None, raw: bool = False) -> np.ndarray:
        if src_dev is None:
            return self._get(field_id, raw=raw)
        n = self._field_elems[field_id]
        out = np.empty((self.num_envs, n), dtype=np.float32)
        _lib.check((self._raw if raw else self._L).pp3_memcpy_d2h(out.ctypes.data_as(C.c_void_p), C.c_void_p(src_dev),
                                                                 out.nbytes))
        return out

    def _output_views(self, lease, single: bool):
        """(obs, reward, done): read-only views of a filled page-locked output block; they keep it
        leased until the last of them dies."""
        n, D = self.num_envs, self.observation_size
        flat = np.asarray(lease)  # (read-only, and so every view of it)
        obs = flat[:n * D].reshape(n, D)
        rew = flat[n * D:n * (D + 1)]
        done = flat[n * (D + 1):]
        if single:
            obs, rew, done = obs[0], rew[0], done[0]
        return obs, rew, done

    def _issue(self, single: bool, lease=None, slot=None) -> DeviceState:
        # obs | reward | done land in one page-locked block (one sync); the arrays are views of it
        # and keep it leased until the last of them dies.  `lease`: a block the launch already fills;
        # with `slot` (its completion event) the state is returned at once and waits on first read
        n, D = self.num_envs, self.observation_size
        if slot is not None:
            st = DeviceState(self, self._gen, single, ready=(lease, slot))
            st.__dict__["_capture"] = self._issue_capture() if self._issue_capture is not None else None
            self._issued = weakref.ref(st)
            return st
        if lease is None:
            lease = _lib.PinnedBlock.take(4 * n * (D + 2), self._pin_pool)
            base = lease.ptr.value
            if OUTPUTS_BY_KERNEL:  # one kernel storing through the block's device mapping (pp3_outputs_to_host)
                _lib.check(self._L.pp3_outputs_to_host(self._h, C.c_void_p(base)))
            else:  # three copy-engine transfers
                for f, off, nb in ((_abi.F_OBS, 0, 4 * n * D), (_abi.F_REWARD, 4 * n * D, 4 * n),
                                   (_abi.F_DONE, 4 * n * (D + 1), 4 * n)):
                    _lib.check(self._L.pp3_copy_field_to_host_async(self._h, f, C.c_void_p(base + off), nb))
        self.synchronize()
        obs, rew, done = self._output_views(lease, single)
        st = DeviceState(self, self._gen, single, obs, rew, done)
        st.__dict__["_capture"] = self._issue_capture() if self._issue_capture is not None else None
        self._issued = weakref.ref(st)
        return st

    def _before_launch(self) -> None:
        """Called before anything changes the device buffers: the last issued state, if still alive
        and not yet downloaded, gets a device-side snapshot of its lazy fields (d2d copies on the
        env's stream, ordered before the launch), then the buffers' generation advances."""
        self._flush()  # a queued step launches first (its state is the one this launch overwrites)
        st = self._issued() if self._issued is not None else None
        if st is not None and not st.materialized and st._snap is None and st._gen == self._gen:
            buf = self._snap_pool.pop() if self._snap_pool else _lib.DeviceBuffer(self._snap_bytes, self.device)
            stream = self._L.pp3_stream(self._h)
            for f in self._lazy_fields():
                ptr, n = self.device_field(f)
                _lib.check(self._L.pp3_memcpy_d2d(C.c_void_p(buf.ptr.value + self._snap_offsets[f]), C.c_void_p(ptr),
                                                  self.num_envs * n * 4, C.c_void_p(stream)))
            st.__dict__["_snap"] = buf
            self._n_snapshots += 1
            weakref.finalize(st, _return_snapshot, self._snap_pool, st.__dict__)
        self._gen += 1

    # ------------------------------------------------------------------ packing
    def _unpack_info(self, rec: np.ndarray) -> Dict[str, Any]:
        La = len(self._latency_distribution)
        Li = len(self._imu_latency_distribution)
        io = _abi.imu_buf_offset(La)
        info = {
            "rng": rec[:, _abi.S_RNG:_abi.S_RNG + 2].copy().view(np.uint32),
            "last_act": rec[:, _abi.S_LAST_ACT:_abi.S_LAST_ACT + 12].copy(),
            "action_buffer": rec[:, _abi.S_ACT_BUF:_abi.S_ACT_BUF + 12 * La].reshape(-1, 12, La).copy(),
            "imu_buffer": rec[:, io:io + 6 * Li].reshape(-1, 6, Li).copy(),
            "last_vel": rec[:, _abi.S_LAST_VEL:_abi.S_LAST_VEL + 12].copy(),
            "command": rec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3].copy(),
            "last_contact": rec[:, _abi.S_LAST_CONTACT:_abi.S_LAST_CONTACT + 4] != 0,
            "feet_air_time": rec[:, _abi.S_AIR_TIME:_abi.S_AIR_TIME + 4].copy(),
            "kick": rec[:, _abi.S_KICK:_abi.S_KICK + 2].copy(),
            "step": rec[:, _abi.S_STEP].astype(np.int32),
            "desired_world_z_in_body_frame": rec[:, _abi.S_DESIRED_Z:_abi.S_DESIRED_Z + 3].copy(),
        }
        return info

    def _unpack_lazy(self, st: "DeviceState", got: Dict[int, np.ndarray], single: bool) -> Dict[str, Any]:
        """The lazy part of a DeviceState from its downloaded record / metrics / pipeline rows."""
        rec = got[_abi.F_STATE]
        met = got[_abi.F_METRICS]
        info = self._unpack_info(rec)
        info["rewards"] = {k: met[:, 1 + i] for i, k in enumerate(_abi.REWARD_NAMES)}
        metrics = {"total_dist": met[:, 0]}
        metrics.update(info["rewards"])
        ps = PipelineState(q=rec[:, _abi.S_QPOS:_abi.S_QPOS + 19].copy(), qd=rec[:, _abi.S_QVEL:_abi.S_QVEL + 18].copy(),
                           qacc_warmstart=rec[:, _abi.S_QACC_WS:_abi.S_QACC_WS + 18].copy())
        if self._pipeline_output:
            p = got[_abi.F_PIPELINE]
            nb = _abi.NBODY - 1
            ps.x = Transform(pos=p[:, _abi.P_XPOS:_abi.P_XPOS + 3 * nb].reshape(-1, nb, 3),
                             rot=p[:, _abi.P_XQUAT:_abi.P_XQUAT + 4 * nb].reshape(-1, nb, 4))
            ps.xd = Motion(vel=p[:, _abi.P_XD_VEL:_abi.P_XD_VEL + 3 * nb].reshape(-1, nb, 3),
                           ang=p[:, _abi.P_XD_ANG:_abi.P_XD_ANG + 3 * nb].reshape(-1, nb, 3))
            ps.site_xpos = p[:, _abi.P_SITE_XPOS:_abi.P_SITE_XPOS + 12].reshape(-1, 4, 3)
            ps.qfrc_actuator = p[:, _abi.P_QFRC_ACT:_abi.P_QFRC_ACT + 18]
            ps.qacc = p[:, _abi.P_QACC:_abi.P_QACC + 18]
            ncon = p[:, _abi.P_NCON].astype(np.int32)
            g = p[:, _abi.P_CON_GEOM:_abi.P_CON_GEOM + 32].reshape(-1, 16, 2).astype(np.int32)
            ps.contact = Contact(dist=p[:, _abi.P_CON_DIST:_abi.P_CON_DIST + 16], geom1=g[..., 0], geom2=g[..., 1])
            ps.contact.ncon = ncon
            ps.subtree_com = p[:, _abi.P_SUBTREE_COM:_abi.P_SUBTREE_COM + 3]
            ps.sensordata = p[:, _abi.P_SENSOR:_abi.P_SENSOR + self.sys_model.struct.nsensordata]
        if single:
            sq = _squeeze_tree
            ps, metrics, info = sq(ps), sq(metrics), sq(info)
        for fid, hook in self._lazy_extra.items():  # wrappers' info entries (wrappers.py)
            info.update(hook(st, got, single))
        _freeze(ps)
        _freeze(metrics)
        _freeze(info)
        return dict(pipeline_state=ps, metrics=metrics, info=info, _record=_ro(rec), _metrics_raw=_ro(met))

    def _write_state(self, state: State) -> None:
        rec = getattr(state, "_record", None)
        if rec is None:
            raise ValueError("state must come from this env's reset/step")
        rec = rec.copy()
        info = state.info
        ps = state.pipeline_state
        La = len(self._latency_distribution)
        Li = len(self._imu_latency_distribution)
        io = _abi.imu_buf_offset(La)
        n = self.num_envs

        def put(off, val, width):
            rec[:, off:off + width] = np.asarray(val, dtype=np.float32).reshape(n, width)

        put(_abi.S_QPOS, ps.q, 19)
        put(_abi.S_QVEL, ps.qd, 18)
        put(_abi.S_QACC_WS, ps.qacc_warmstart, 18)
        rec[:, _abi.S_RNG:_abi.S_RNG + 2] = np.asarray(info["rng"], dtype=np.uint32).reshape(n, 2).view(np.float32)
        put(_abi.S_LAST_ACT, info["last_act"], 12)
        put(_abi.S_LAST_VEL, info["last_vel"], 12)
        put(_abi.S_COMMAND, info["command"], 3)
        put(_abi.S_DESIRED_Z, info["desired_world_z_in_body_frame"], 3)
        put(_abi.S_AIR_TIME, info["feet_air_time"], 4)
        put(_abi.S_LAST_CONTACT, np.asarray(info["last_contact"], dtype=np.float32), 4)
        put(_abi.S_KICK, info["kick"], 2)
        put(_abi.S_STEP, np.asarray(info["step"], dtype=np.float32), 1)
        put(_abi.S_ACT_BUF, info["action_buffer"], 12 * La)
        put(io, info["imu_buffer"], 6 * Li)
        self._put(_abi.F_STATE, rec)
        self._put(_abi.F_OBS, np.asarray(state.obs, dtype=np.float32).reshape(n, -1))


def _single_of(state) -> bool:
    """A single-env state (reset with one key): from the DeviceState's flag when it has one, so a
    pending state's outputs are not waited for just to learn their shape."""
    d = getattr(state, "__dict__", {})
    if "_single" in d:
        return bool(d["_single"])
    return np.ndim(state.reward) == 0


class _StepBatch:
    """Steps queued by PupperV3Env.step (DEFER_LAUNCH): their actions in one page-locked block of the
    env's ring ([cap][N][12]) and their outputs in one page-locked block ([cap][N][36H] obs |
    [cap][N] reward | [cap][N] done), each queued state viewing its own rows."""

    def __init__(self, env: "PupperV3Env", slot, lease, cap: int):
        n = env.num_envs
        self.slot, self.lease, self.cap = slot, lease, cap
        self.act = slot.act_rows(cap, n)
        self.n_envs, self.D = n, env.observation_size
        self.gen0 = env._gen
        self.states = []  # weak references to the queued states, in order
        self.n = 0
        self.stored = [False] * cap  # row j's obs / reward / done were stored by an issued launch
        self.error = None  # the exception an issuing launch raised

    def tail(self):
        return self.states[-1]() if self.states else None

    def views(self, j: int, single: bool):
        """(obs, reward, done) read-only views of step j's rows; they keep the block leased."""
        n, D, B = self.n_envs, self.D, self.cap
        flat = np.asarray(self.lease)  # (read-only, and so every view of it)
        obs = flat[j * n * D:(j + 1) * n * D].reshape(n, D)
        rew = flat[B * n * D + j * n:B * n * D + (j + 1) * n]
        done = flat[B * n * (D + 1) + j * n:B * n * (D + 1) + (j + 1) * n]
        if single:
            obs, rew, done = obs[0], rew[0], done[0]
        return obs, rew, done


class _FlushingLib:
    """The library as PupperV3Env._L: each call first issues the env's queued step() launch
    (DEFER_LAUNCH), so whatever reads or changes the device sees the state step() returned."""

    def __init__(self, env: "PupperV3Env", lib):
        self._env = weakref.ref(env)
        self._lib = lib

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        env_ref = self._env

        def call(*args):
            env = env_ref()
            if env is not None and env.__dict__.get("_qb") is not None:
                env._flush()
            return fn(*args)
        call.__name__ = name
        return call


class _ActSlot:
    """One page-locked action staging block of PupperV3Env.step's ring and the completion event of
    the last launch that read it (pp3_event_*)."""

    def __init__(self, env: "PupperV3Env", nbytes: int):
        self._L = getattr(env, "_raw", None) or env._L  # (events never wait for a queued step launch)
        self._h = env._h
        self.block = _lib.PinnedBlock(nbytes)
        self.arr = np.asarray(self.block)
        ev = C.c_void_p()
        _lib.check(self._L.pp3_event_create(env._h, C.byref(ev)))
        self.ev = ev
        self.pending = False  # recorded and not yet seen complete
        self._rows = {}

    def act_rows(self, cap: int, n: int) -> np.ndarray:
        """The block as [cap][n][12] action rows (one view per shape, reused by every batch)."""
        v = self._rows.get((cap, n))
        if v is None:
            v = self._rows[(cap, n)] = self.arr[:cap * n * _abi.NU].reshape(cap, n, _abi.NU)
        return v

    def record(self) -> None:
        _lib.check(self._L.pp3_event_record(self._h, self.ev))
        self.pending = True

    def wait(self) -> None:
        """Until the recorded launch has completed (no library call when a wait already saw it)."""
        if self.pending and self.ev:
            _lib.check(self._L.pp3_event_synchronize(self.ev))
            self.pending = False

    def close(self) -> None:
        if self.ev:
            self._L.pp3_event_destroy(self.ev)
            self.ev = C.c_void_p()
        self.block.free()


def _squeeze_tree(v):
    """Drop the leading batch axis of a 1-env result (single-key reset API)."""
    if isinstance(v, np.ndarray):
        return v[0] if v.ndim >= 1 and v.shape[0] == 1 else v
    if isinstance(v, dict):
        return {k: _squeeze_tree(x) for k, x in v.items()}
    if isinstance(v, (PipelineState, Transform, Motion, Contact)):
        for k, x in list(vars(v).items()):
            setattr(v, k, _squeeze_tree(x))
        return v
    return v


def _freeze(v):
    """Every array of a State tree read-only (in place)."""
    if isinstance(v, np.ndarray):
        v.flags.writeable = False
    elif isinstance(v, dict):
        for x in v.values():
            _freeze(x)
    elif isinstance(v, (PipelineState, Transform, Motion, Contact)):
        for x in vars(v).values():
            _freeze(x)


def _return_snapshot(pool, d) -> None:
    """weakref finalizer of a DeviceState: its device snapshot (if any) goes back to the env's pool."""
    buf = d.get("_snap")
    if buf is not None:
        pool.append(buf)


def make_keys(seed: int, n: int, partitionable: bool = True) -> np.ndarray:
    """N per-env reset keys = jax.random.split(PRNGKey(seed), N)."""
    return _rng.split(_rng.PRNGKey(seed), n, partitionable)
