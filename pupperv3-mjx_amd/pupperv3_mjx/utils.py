"""Host helpers mirroring the env-path parts of the reference's utils.py.

* latency ring buffers (utils.py:19-69) -- numpy restatements used by the host API and by
  tests; the device kernel implements the same push-front + categorical-column rule;
* MJCF editors ``set_mjx_custom_options`` / ``set_robot_starting_position`` (utils.py:145-199);
* ``activation_fn_map`` (utils.py:296-313) over numpy, for policy-export consumers.

Training UX (wandb/orbax/plotting/video) is out of scope.
"""
from __future__ import annotations

import re
import xml.etree.ElementTree as ET
from typing import List, Optional, Tuple

import numpy as np

from . import rng as _rng


def circular_buffer_push_back(buffer: np.ndarray, new_value: np.ndarray) -> np.ndarray:
    """Shift columns left by one; newest value goes to column -1."""
    out = np.empty_like(buffer)
    out[:, :-1] = buffer[:, 1:]
    out[:, -1] = new_value
    return out


def circular_buffer_push_front(buffer: np.ndarray, new_value: np.ndarray) -> np.ndarray:
    """Shift columns right by one; newest value goes to column 0."""
    out = np.empty_like(buffer)
    out[:, 1:] = buffer[:, :-1]
    out[:, 0] = new_value
    return out


def sample_lagged_value(key, buffer_newest_first: np.ndarray, new_value: np.ndarray, distribution,
                        partitionable: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """Push `new_value` to the front, then return the column drawn from `distribution`."""
    buf = circular_buffer_push_front(buffer_newest_first, new_value)
    idx = int(_rng.choice_index(key, np.asarray(distribution, dtype=np.float32), partitionable))
    return buf[:, idx], buf


def set_mjx_custom_options(tree: ET.ElementTree, max_contact_points: int, max_geom_pairs: int):
    """Rewrite the <custom><numeric> collision caps; returns None when there is no <custom>."""
    custom = tree.getroot().find("custom")
    if custom is None:
        return None
    values = {"max_contact_points": max_contact_points, "max_geom_pairs": max_geom_pairs}
    for numeric in custom.findall("numeric"):
        if numeric.get("name") in values:
            numeric.set("data", str(values[numeric.get("name")]))
    return tree


def set_robot_starting_position(tree: ET.ElementTree, starting_pos: List, starting_quat: Optional[List] = None):
    """Move base_link (body pos/quat) and the 'home' keyframe's free-joint qpos."""
    body = tree.find(".//worldbody/body[@name='base_link']")
    body.set("pos", " ".join(str(v) for v in starting_pos[:3]))
    if starting_quat is not None:
        body.set("quat", " ".join(str(v) for v in starting_quat[:4]))
    key = tree.find(".//keyframe/key[@name='home']")
    q = [float(v) for v in re.split(r"\s+", key.get("qpos").strip())]
    q[:3] = list(starting_pos)
    if starting_quat is not None:
        q[3:7] = list(starting_quat)
    key.set("qpos", " ".join(map(str, q)))
    return tree


def activation_fn_map(activation_name: str):
    name = activation_name.lower()

    def softmax(x):
        e = np.exp(x - np.max(x, axis=-1, keepdims=True))
        return e / e.sum(axis=-1, keepdims=True)

    table = {
        "relu": lambda x: np.maximum(x, 0),
        "sigmoid": lambda x: 1.0 / (1.0 + np.exp(-x)),
        "elu": lambda x: np.where(x > 0, x, np.expm1(np.minimum(x, 0))),
        "tanh": np.tanh,
        "softmax": softmax,
    }
    return table[name]
