"""Reward terms of rewards.py:9-138 as host (numpy) functions over PupperV3Env's state types.

The env step computes every term on the device (csrc/pp3_env.hip, epilogue) and returns them
scaled in ``state.metrics`` / ``state.info["rewards"]``; this module is the reference's public
``pupperv3_mjx.rewards`` surface for code that evaluates a term itself (reward shaping, logging,
analysis of recorded ``pipeline_state``\\ s).  Same names, arguments and meaning as the
reference; every function also accepts a leading batch dimension (the reference's functions are
per env and batched by ``jax.vmap``).  ``x`` / ``xd`` are ``environment.Transform`` /
``environment.Motion`` with the world body dropped (Brax convention: index 0 = the torso).
"""
from __future__ import annotations

import numpy as np


# ------------------------------------------------------------------ brax.math (batched)
def quat_inv(q):
    q = np.asarray(q)
    return q * np.array([1, -1, -1, -1], dtype=q.dtype)


def rotate(vec, quat):
    """brax math.rotate: vec rotated by the unit quaternion quat (w, x, y, z)."""
    vec, quat = np.asarray(vec), np.asarray(quat)
    s, u = quat[..., :1], quat[..., 1:]
    r = 2 * np.sum(u * vec, -1, keepdims=True) * u + (s * s - np.sum(u * u, -1, keepdims=True)) * vec
    return r + 2 * s * np.cross(u, vec)


def _norm(v):
    return np.sqrt(np.sum(np.square(v), -1))


# ------------------------------------------------------------------ reward functions
def reward_lin_vel_z(xd):
    """rewards.py:9: squared z velocity of the base."""
    return np.square(xd.vel[..., 0, 2])


def reward_ang_vel_xy(xd):
    """rewards.py:14: squared x/y angular velocity of the base."""
    return np.sum(np.square(xd.ang[..., 0, :2]), -1)


def reward_tracking_orientation(desired_world_z_in_body_frame, x, tracking_sigma: float):
    """rewards.py:19: exp(-|world z in the body frame - desired|^2 / sigma)."""
    world_z = np.array([0.0, 0.0, 1.0], dtype=np.asarray(x.rot).dtype)
    z_body = rotate(world_z, quat_inv(x.rot[..., 0, :]))
    error = np.sum(np.square(z_body - np.asarray(desired_world_z_in_body_frame)), -1)
    return np.exp(-error / tracking_sigma)


def reward_orientation(x):
    """rewards.py:29: squared x/y of the body up axis in the world."""
    up = np.array([0.0, 0.0, 1.0], dtype=np.asarray(x.rot).dtype)
    rot_up = rotate(up, x.rot[..., 0, :])
    return np.sum(np.square(rot_up[..., :2]), -1)


def reward_torques(torques):
    """rewards.py:36: sum of squared actuator forces."""
    return np.sum(np.square(torques), -1)


def reward_joint_acceleration(joint_vel, last_joint_vel, dt: float):
    """rewards.py:44: sum of squared finite-difference joint accelerations."""
    return np.sum(np.square((np.asarray(joint_vel) - np.asarray(last_joint_vel)) / dt), -1)


def reward_mechanical_work(torques, velocities):
    """rewards.py:48: sum |torque * velocity|."""
    return np.sum(np.abs(np.asarray(torques) * np.asarray(velocities)), -1)


def reward_action_rate(act, last_act):
    """rewards.py:53: sum of squared action changes."""
    return np.sum(np.square(np.asarray(act) - np.asarray(last_act)), -1)


def reward_tracking_lin_vel(commands, x, xd, tracking_sigma):
    """rewards.py:58: exp(-|cmd_xy - base velocity_xy in the body frame|^2 / sigma)."""
    local_vel = rotate(xd.vel[..., 0, :], quat_inv(x.rot[..., 0, :]))
    err = np.sum(np.square(np.asarray(commands)[..., :2] - local_vel[..., :2]), -1)
    return np.exp(-err / tracking_sigma)


def reward_tracking_ang_vel(commands, x, xd, tracking_sigma):
    """rewards.py:66: exp(-(cmd_yaw - base yaw rate in the body frame)^2 / sigma)."""
    base_ang = rotate(xd.ang[..., 0, :], quat_inv(x.rot[..., 0, :]))
    err = np.square(np.asarray(commands)[..., 2] - base_ang[..., 2])
    return np.exp(-err / tracking_sigma)


def reward_feet_air_time(air_time, first_contact, commands, minimum_airtime: float = 0.1):
    """rewards.py:73: air time beyond the minimum at first contact; zero for a (near) zero command."""
    rew = np.sum((np.asarray(air_time) - minimum_airtime) * np.asarray(first_contact), -1)
    return rew * (_norm(np.asarray(commands)[..., :3]) > 0.05)


def reward_abduction_angle(joint_angles, desired_abduction_angles=np.zeros(4)):
    """rewards.py:85: squared deviation of the four abduction joints (every third joint)."""
    return np.sum(np.square(np.asarray(joint_angles)[..., 1::3] - np.asarray(desired_abduction_angles)), -1)


def reward_stand_still(commands, joint_angles, default_pose, command_threshold: float):
    """rewards.py:90: sum |joint_angles - default_pose| while |command| < threshold."""
    dev = np.sum(np.abs(np.asarray(joint_angles) - np.asarray(default_pose)), -1)
    return dev * (_norm(np.asarray(commands)[..., :3]) < command_threshold)


def reward_foot_slip(pipeline_state, contact_filt, feet_site_id, lower_leg_body_id):
    """rewards.py:109: squared horizontal velocity of the feet in contact.  A foot's velocity is
    its lower leg's Brax motion moved to the foot site (vel + ang x offset); MuJoCo body ids
    count the world body, Brax arrays do not (index id - 1)."""
    feet_site_id = np.asarray(feet_site_id)
    legs = np.asarray(lower_leg_body_id) - 1
    ps = pipeline_state
    site = np.asarray(ps.site_xpos)
    if site.shape[-2] != len(feet_site_id):  # full site table: pick the feet
        site = site[..., feet_site_id, :]
    offset = site - np.asarray(ps.x.pos)[..., legs, :]
    vel = np.asarray(ps.xd.vel)[..., legs, :] + np.cross(np.asarray(ps.xd.ang)[..., legs, :], offset)
    return np.sum(np.square(vel[..., :2]) * np.asarray(contact_filt)[..., None], (-1, -2))


def reward_termination(done, step, step_threshold: int):
    """rewards.py:127: done before the step threshold."""
    return np.logical_and(np.asarray(done).astype(bool), np.asarray(step) < step_threshold)


def reward_geom_collision(pipeline_state, geom_ids):
    """rewards.py:131: penetrating contacts (dist < 0) that involve any of geom_ids.  Contact
    slots past the env's contact count (``contact.ncon``, when the state carries it) are empty."""
    con = pipeline_state.contact
    g1, g2, dist = np.asarray(con.geom1), np.asarray(con.geom2), np.asarray(con.dist)
    live = dist < 0.0
    ncon = getattr(con, "ncon", None)
    if ncon is not None:
        live = live & (np.arange(dist.shape[-1]) < np.asarray(ncon)[..., None])
    total = np.zeros(dist.shape[:-1])
    for gid in np.asarray(geom_ids).ravel():
        total = total + np.sum(((g1 == gid) | (g2 == gid)) & live, -1)
    return total
