"""PupperV3Env.render on the GPU (csrc/pp3_render.hip) against the CPU restatement
(oracle/render_ref.py) on the same scene, poses and camera; and the env-level API.

Pixels on triangle edges can round differently (fused multiply-adds on the GPU), so the check is
that >= 99 % of pixels are identical and every frame has the same set of colours."""
import struct

import numpy as np
import pytest

import common
from oracle import render_ref
from pupperv3_mjx import MODEL_XML, mjcf, render
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu


def _poses():
    q = np.zeros((3, 19))
    q[:, 3] = 1.0
    q[:, 7:] = common.DEFAULT_POSE
    q[:, 2] = [0.17, 0.2, 0.12]
    q[1, 0:2] = [0.2, 0.1]
    q[1, 3:7] = mjcf.axis_angle_quat(np.array([0.0, 0, 1]), 0.7)
    q[2, 7:] += np.linspace(-0.4, 0.4, 12)
    return list(q)


def _compare(sc, H, W):
    qs = _poses()
    gpu = render.render_qpos(sc, qs, "tracking_cam", H, W)
    cpu = render_ref.render(sc, qs, "tracking_cam", H, W)
    for g, c in zip(gpu, cpu):
        assert g.shape == (H, W, 3) and g.dtype == np.uint8
        same = np.all(g == c, axis=-1).mean()
        assert same >= 0.99, same
    return gpu


def test_render_matches_cpu_restatement_proxies(require_gpu):
    sc = render.Scene(mjcf.load(MODEL_XML), meshdir="/nonexistent")
    frames = _compare(sc, 48, 64)
    assert not np.array_equal(frames[0], frames[1])  # the pose moved the robot


def _write_box_stl(path, half):
    t = render._box(half)
    with open(path, "wb") as f:
        f.write(b"\0" * 80 + struct.pack("<I", len(t)))
        for tri in t:
            f.write(struct.pack("<3f", 0, 0, 0) + tri.astype(np.float32).tobytes() + b"\0\0")


def test_render_mesh_geoms_matches_cpu_restatement(require_gpu, tmp_path):
    """The mesh-geom path (asset scale, geom pose in the body) with small synthetic STL files in
    place of the robot's meshes (not shipped)."""
    cm = mjcf.load(MODEL_XML)
    for name, a in cm.visual["meshes"].items():
        _write_box_stl(tmp_path / a["file"], [0.03, 0.015, 0.01])
    sc = render.Scene(cm, meshdir=str(tmp_path))
    assert not sc.proxies and len(sc.items) == len(cm.visual["meshes"])
    _compare(sc, 60, 80)


def test_env_render_api(require_gpu):
    e = PupperV3Env(**common.fixture_kwargs(MODEL_XML), num_envs=2)
    try:
        st = e.reset(make_keys(0, 2))
        traj = [st]
        for _ in range(3):
            st = e.step(st, np.zeros((2, 12), np.float32))
            traj.append(st)
        frames = e.render(traj, camera="tracking_cam", height=60, width=80, env_index=1)
        assert len(frames) == 4 and all(f.shape == (60, 80, 3) and f.dtype == np.uint8 for f in frames)
        with pytest.raises(ValueError, match="does not exist"):
            e.render(traj[:1])  # the reference's default camera "track" is not in the stock model
        free = e.render(traj[:1], camera=-1, height=30, width=40)
        assert free[0].shape == (30, 40, 3)
    finally:
        e.close()
