"""Reward configuration: ``get_config()`` with the reference's scales and tracking sigma.

Mirrors config.py:4-75 of the reference (an ml_collections ConfigDict there; ml_collections
is not available here, so a small attribute-access dict with the same access patterns is
used: ``cfg.rewards.scales.tracking_lin_vel``, ``cfg.rewards.scales[k]``, ``.keys()``).
"""
from __future__ import annotations


class ConfigDict(dict):
    """dict with attribute access (the subset of ml_collections.ConfigDict the env uses)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


# (name, scale) in config.py order; comments there explain each term.
_SCALES = (
    ("tracking_lin_vel", 1.5),
    ("tracking_ang_vel", 0.8),
    ("lin_vel_z", -2.0),
    ("ang_vel_xy", -0.05),
    ("orientation", -5.0),
    ("tracking_orientation", 1.0),
    ("torques", -0.0002),
    ("joint_acceleration", -1e-6),
    ("mechanical_work", -0.00),
    ("action_rate", -0.01),
    ("feet_air_time", 0.2),
    ("stand_still", -0.5),
    ("stand_still_joint_velocity", -0.1),
    ("abduction_angle", -0.1),
    ("termination", -100.0),
    ("foot_slip", -0.1),
    ("knee_collision", -1.0),
    ("body_collision", -1.0),
)


def get_config() -> ConfigDict:
    """Reward config for the Pupper joystick task (scales + tracking_sigma=0.25)."""
    scales = ConfigDict((k, v) for k, v in _SCALES)
    rewards = ConfigDict(scales=scales, tracking_sigma=0.25)
    return ConfigDict(rewards=rewards)
