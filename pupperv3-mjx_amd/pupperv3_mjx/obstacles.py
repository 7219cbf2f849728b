"""Static obstacle boxes ("rails") added to the MJCF worldbody.

Behavioural mirror of obstacles.py:16-57: the stdlib Mersenne-Twister ``random`` module is
seeded once with ``seed`` and, per box, draws x, y and a yaw in that order, so a given seed
produces the same boxes (pinned against a fixture generated from the reference module in
tests/golden/obstacles_golden.json, made by tests/golden/make_golden.py).  Boxes are static world geoms shared by all envs; the
HIP kernel collides every robot sphere against each of them (sphere-box narrow phase).
"""
from __future__ import annotations

import math
import random
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from typing import List, Sequence, Tuple


@dataclass
class BoxSpec:
    name: str
    x: float
    y: float
    quat: Tuple[float, int, int, float]
    half_sizes: Tuple[float, float, float]


def random_z_rotation_quaternion(seed: int = 0):
    """(w, 0, 0, z) for a yaw drawn uniformly in [-pi, pi] from the global `random` stream.

    As in the reference, `seed` is accepted but not used (the stream is seeded by the caller).
    """
    half = random.uniform(-math.pi, math.pi) / 2
    return [math.cos(half), 0, 0, math.sin(half)]


def sample_boxes(n_boxes: int, x_range: Sequence[float], y_range: Sequence[float], height: float = 0.02,
                 depth: float = 0.02, length: float = 3.0, seed: int = 0) -> List[BoxSpec]:
    random.seed(seed)
    specs = []
    for i in range(n_boxes):
        x = random.uniform(x_range[0], x_range[1])
        y = random.uniform(y_range[0], y_range[1])
        q = random_z_rotation_quaternion(seed=seed)
        specs.append(BoxSpec(f"box_geom_{i}", x, y, tuple(q), (depth / 2.0, length / 2.0, height)))
    return specs


def add_boxes_to_model(tree: ET.ElementTree, n_boxes: int, x_range: Tuple, y_range: Tuple, height: float = 0.02,
                       depth: float = 0.02, length: float = 3.0, group: str = "0", seed: int = 0) -> ET.ElementTree:
    """Append `n_boxes` box geoms to <worldbody>; returns the (mutated) tree."""
    world = tree.getroot().find("worldbody")
    for b in sample_boxes(n_boxes, x_range, y_range, height, depth, length, seed):
        attrs = {
            "name": b.name,
            "pos": f"{b.x} {b.y} 0",
            "quat": " ".join(str(v) for v in b.quat),
            "type": "box",
            "size": " ".join(str(v) for v in b.half_sizes),
            "rgba": "0.1 0.5 0.8 1",
            "conaffinity": "1",
            "contype": "1",
            "condim": "3",
            "group": group,
        }
        ET.SubElement(world, "geom", attrs)
    return tree


def rail_start_xy(specs: Sequence[BoxSpec], num_envs: int, seed: int = 0, offset: float = 0.06,
                  along: float = 0.8):
    """Start positions ON the boxes, for workloads that must exercise the sphere-box contacts
    (BASELINE configs[4]): env i stands over box i % len(specs), at a uniform point of the middle
    `along` fraction of its long axis (local y, half length half_sizes[1]) and a uniform lateral
    offset within +-`offset` of its centre line, so its feet land on or beside the rail.  Returns
    [num_envs, 2] world x, y (numpy Generator seeded with `seed`)."""
    import numpy as np
    g = np.random.default_rng(seed)
    out = np.zeros((num_envs, 2))
    for i in range(num_envs):
        b = specs[i % len(specs)]
        yaw = 2.0 * math.atan2(b.quat[3], b.quat[0])
        u = g.uniform(-along, along) * b.half_sizes[1]
        v = g.uniform(-offset, offset)
        # local y (the rail's length) -> world (-sin, cos); local x (its width) -> (cos, sin)
        out[i] = [b.x - u * math.sin(yaw) + v * math.cos(yaw), b.y + u * math.cos(yaw) + v * math.sin(yaw)]
    return out


# --------------------------------------------------------------------------- per-env terrain
# the reference's boxes are static and shared; here every env may hold its
# own boxes in the model's box-geom slots (PupperV3Env.set_terrain / pp3_set_terrain).  A row
# is pos[3], quat[4] (w,x,y,z), half sizes[3]; all-zero half sizes mark an absent box.

def terrain_from_specs(specs: Sequence[BoxSpec], num_envs: int):
    """Every env gets the same boxes (the reference's static layout, as per-env rows)."""
    import numpy as np
    row = np.array([[b.x, b.y, 0.0, *b.quat, *b.half_sizes] for b in specs], dtype=np.float32)
    return np.ascontiguousarray(np.broadcast_to(row, (num_envs,) + row.shape))


def sample_terrain(num_envs: int, n_boxes: int, x_range: Sequence[float], y_range: Sequence[float],
                   height: float = 0.02, depth: float = 0.02, length: float = 3.0, seed: int = 0,
                   min_boxes: int = None):
    """Independent boxes per env, each drawn like obstacles.py:16-57 draws one box (x, y
    uniform, yaw uniform in [-pi, pi], half sizes (depth/2, length/2, height)), from a numpy
    Generator seeded with `seed`.  With `min_boxes`, env i keeps a uniform number of boxes in
    [min_boxes, n_boxes] and the rest of its slots are absent (variable contact counts)."""
    import numpy as np
    g = np.random.default_rng(seed)
    x = g.uniform(x_range[0], x_range[1], size=(num_envs, n_boxes))
    y = g.uniform(y_range[0], y_range[1], size=(num_envs, n_boxes))
    half = g.uniform(-math.pi, math.pi, size=(num_envs, n_boxes)) / 2
    t = np.zeros((num_envs, n_boxes, 10), dtype=np.float32)
    t[..., 0], t[..., 1] = x, y
    t[..., 3], t[..., 6] = np.cos(half), np.sin(half)
    t[..., 7], t[..., 8], t[..., 9] = depth / 2.0, length / 2.0, height
    if min_boxes is not None:
        keep = g.integers(min_boxes, n_boxes + 1, size=num_envs)
        t[np.arange(n_boxes)[None, :] >= keep[:, None], 7:10] = 0.0
    return t
