"""Per-env parameter randomisation and start-pose randomisation.

Mirrors domain_randomization.py:8-210 of the reference with its exact jax.random key
schedule (restated in rng.py), so the same keys give the same randomised parameters:

* ``domain_randomize(sys, rng[N,2], ...) -> (sys_batched, in_axes)``: friction (one scalar
  for every geom), Kp/Kd multipliers, torso COM shift, elementwise inertia and mass scales.
  The batched ``System`` carries the same field shapes as the reference's vmapped MJX
  model ((N,23,3), (N,12,10), ...); ``System.dr_table()`` packs the 62 free scalars per env
  (PP3_DR_* layout) that the HIP kernel consumes as on-device per-env perturbations.
* ``randomize_qpos`` / ``random_z_rotation_quaternion`` (the device reset kernel draws the
  same numbers; this host version is used by tests and host tooling).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple

import numpy as np

from . import _abi
from . import rng as _rng


@dataclass
class StartPositionRandomization:
    x_min: float
    x_max: float
    y_min: float
    y_max: float
    z_min: float
    z_max: float


@dataclass
class System:
    """The model fields domain randomisation touches (shapes as in mjx.Model), plus nominal ids."""

    geom_friction: np.ndarray     # (ngeom, 3) or (N, ngeom, 3)
    actuator_gainprm: np.ndarray  # (nu, 10) or (N, nu, 10)
    actuator_biasprm: np.ndarray  # (nu, 10) or (N, nu, 10)
    body_ipos: np.ndarray         # (nbody, 3) or (N, nbody, 3)
    body_inertia: np.ndarray      # (nbody, 3) or (N, nbody, 3)
    body_mass: np.ndarray         # (nbody,) or (N, nbody)
    extra: Dict = field(default_factory=dict)

    @property
    def batched(self) -> bool:
        return self.body_mass.ndim == 2

    def tree_replace(self, params: Dict) -> "System":
        kw = dict(self.__dict__)
        kw.update(params)
        return System(**kw)

    def dr_table(self) -> np.ndarray:
        """Pack a batched System into the kernel's f32[N][62] DR record."""
        if not self.batched:
            raise ValueError("dr_table() needs a batched System from domain_randomize")
        n = self.body_mass.shape[0]
        fr = self.geom_friction[:, :, 0]
        if not np.all(fr == fr[:, :1]):
            raise ValueError("the kernel's DR record holds one friction scalar per env (domain_randomization.py:29)")
        kp = self.actuator_gainprm[:, :, 0]
        kd = -self.actuator_biasprm[:, :, 2]
        if not (np.all(kp == kp[:, :1]) and np.all(kd == kd[:, :1])):
            raise ValueError("the kernel's DR record holds one Kp and one Kd per env")
        t = np.zeros((n, _abi.NDR), dtype=np.float32)
        t[:, _abi.DR_FRICTION] = fr[:, 0]
        t[:, _abi.DR_KP] = kp[:, 0]
        t[:, _abi.DR_KD] = kd[:, 0]
        t[:, _abi.DR_BASE_IPOS:_abi.DR_BASE_IPOS + 3] = self.body_ipos[:, 1, :]
        t[:, _abi.DR_INERTIA:_abi.DR_INERTIA + 3 * _abi.NBODY] = self.body_inertia.reshape(n, -1)
        t[:, _abi.DR_MASS:_abi.DR_MASS + _abi.NBODY] = self.body_mass
        return t


def domain_randomize(sys: System, rng, friction_range: Tuple = (0.6, 1.4), kp_multiplier_range: Tuple = (0.75, 1.25),
                     kd_multiplier_range: Tuple = (0.5, 2.0), body_com_x_shift_range: Tuple = (-0.03, 0.03),
                     body_com_y_shift_range: Tuple = (-0.01, 0.01), body_com_z_shift_range: Tuple = (-0.02, 0.02),
                     body_inertia_scale_range: Tuple = (0.7, 1.3), body_mass_scale_range: Tuple = (0.7, 1.3),
                     partitionable: bool = True):
    """Randomise friction, Kp, Kd, torso COM, inertia and mass for each key in `rng` [N, 2]."""
    keys = np.asarray(rng, dtype=np.uint32).reshape(-1, 2)
    p = partitionable
    f32 = np.float32
    # key schedule of domain_randomization.py:27-80
    s1 = _rng.split(keys, 2, p)
    r1, k_fric = s1[:, 0], s1[:, 1]
    s2 = _rng.split(r1, 3, p)
    r2, k_kp, k_kd = s2[:, 0], s2[:, 1], s2[:, 2]
    s3 = _rng.split(r2, 2, p)
    r3, k_com = s3[:, 0], s3[:, 1]
    s4 = _rng.split(r3, 2, p)
    r4, k_inert = s4[:, 0], s4[:, 1]
    s5 = _rng.split(r4, 2, p)
    k_mass = s5[:, 1]

    fric = _rng.uniform(k_fric, (1,), friction_range[0], friction_range[1], p)  # (N,1)
    kp_mul = _rng.uniform(k_kp, (1,), kp_multiplier_range[0], kp_multiplier_range[1], p)
    kd_mul = _rng.uniform(k_kd, (1,), kd_multiplier_range[0], kd_multiplier_range[1], p)
    lo = np.array([body_com_x_shift_range[0], body_com_y_shift_range[0], body_com_z_shift_range[0]], dtype=f32)
    hi = np.array([body_com_x_shift_range[1], body_com_y_shift_range[1], body_com_z_shift_range[1]], dtype=f32)
    com = _rng.uniform(k_com, (3,), lo, hi, p)
    inert = _rng.uniform(k_inert, sys.body_inertia.shape, body_inertia_scale_range[0], body_inertia_scale_range[1], p)
    mass = _rng.uniform(k_mass, sys.body_mass.shape, body_mass_scale_range[0], body_mass_scale_range[1], p)

    n = keys.shape[0]
    friction = np.broadcast_to(sys.geom_friction.astype(f32), (n,) + sys.geom_friction.shape).copy()
    friction[:, :, 0] = fric
    kp = (kp_mul * sys.actuator_gainprm[:, 0].astype(f32)).astype(f32)     # (N, nu)
    kd = (kd_mul * (-sys.actuator_biasprm[:, 2]).astype(f32)).astype(f32)
    gain = np.broadcast_to(sys.actuator_gainprm.astype(f32), (n,) + sys.actuator_gainprm.shape).copy()
    gain[:, :, 0] = kp
    bias = np.broadcast_to(sys.actuator_biasprm.astype(f32), (n,) + sys.actuator_biasprm.shape).copy()
    bias[:, :, 1] = -kp
    bias[:, :, 2] = -kd
    ipos = np.broadcast_to(sys.body_ipos.astype(f32), (n,) + sys.body_ipos.shape).copy()
    ipos[:, 1] = (sys.body_ipos[1].astype(f32) + com).astype(f32)
    inertia = (sys.body_inertia.astype(f32) * inert).astype(f32)
    body_mass = (sys.body_mass.astype(f32) * mass).astype(f32)

    in_axes = {k: None for k in ("geom_friction", "actuator_gainprm", "actuator_biasprm", "body_ipos",
                                 "body_inertia", "body_mass")}
    in_axes.update({k: 0 for k in in_axes})
    out = System(friction, gain, bias, ipos, inertia, body_mass, dict(sys.extra))
    return out, in_axes


def small_quaternion(rng, max_angle_deg: float = 30, max_yaw_deg: float = 180, partitionable: bool = True):
    """Random roll/pitch in +-max_angle_deg and yaw in +-max_yaw_deg as a unit quaternion (w,x,y,z)."""
    k = _rng.split(rng, 4, partitionable)
    pitch = (_rng.uniform(k[1], ()) * 2 - 1) * max_angle_deg
    roll = (_rng.uniform(k[2], ()) * 2 - 1) * max_angle_deg
    yaw = (_rng.uniform(k[3], ()) * 2 - 1) * max_yaw_deg
    hr, hp, hy = (np.float32(v) * np.float32(math.pi) / np.float32(180.0) / 2 for v in (roll, pitch, yaw))
    cr, sr, cp, sp, cy, sy = np.cos(hr), np.sin(hr), np.cos(hp), np.sin(hp), np.cos(hy), np.sin(hy)
    q = np.array([cr * cp * cy + sr * sp * sy, sr * cp * cy - cr * sp * sy,
                  cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy], dtype=np.float32)
    return q / np.linalg.norm(q)


def random_z_rotation_quaternion(rng, partitionable: bool = True) -> np.ndarray:
    yaw = _rng.uniform(rng, (1,), -np.float32(np.pi), np.float32(np.pi), partitionable)
    half = yaw / np.float32(2)
    return np.concatenate([np.cos(half), np.zeros(2, dtype=np.float32), np.sin(half)]).astype(np.float32)


def randomize_qpos(qpos, start_position_config: StartPositionRandomization, rng, partitionable: bool = True):
    """qpos with the base xyz drawn in the configured box and a random yaw (domain_randomization.py:188-210)."""
    q = np.array(qpos, dtype=np.float32).copy()
    k = _rng.split(rng, 3, partitionable)
    c = start_position_config
    lo = np.array([c.x_min, c.y_min, c.z_min], dtype=np.float32)
    hi = np.array([c.x_max, c.y_max, c.z_max], dtype=np.float32)
    q[:3] = _rng.uniform(k[1], (3,), lo, hi, partitionable)
    q[3:7] = random_z_rotation_quaternion(k[2], partitionable)
    return q
