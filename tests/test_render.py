"""PupperV3Env.render host side (render.py): STL loading, scene assembly from the MJCF visual
description, MuJoCo camera rules, and the CPU restatement of the rasteriser on a known pose.
(The kernel itself is compared with that restatement in test_gpu_render.py.)"""
import os
import struct

import numpy as np
import pytest

import common
from oracle import render_ref
from pupperv3_mjx import MODEL_XML, mjcf, render

REF_MESHES = "/root/reference/meshes/stl"  # present in the build container only (skipped elsewhere)


def _home_q():
    q = np.zeros(19)
    q[2], q[3] = 0.17, 1.0
    q[7:] = common.DEFAULT_POSE
    return q


def test_stl_binary_and_ascii(tmp_path):
    tri = np.array([[[0, 0, 0], [1, 0, 0], [0, 1, 0]], [[0, 0, 1], [1, 0, 1], [0, 1, 1]]], np.float32)
    b = tmp_path / "t.stl"
    with open(b, "wb") as f:
        f.write(b"\0" * 80 + struct.pack("<I", 2))
        for t in tri:
            f.write(struct.pack("<3f", 0, 0, 1) + t.tobytes() + b"\0\0")
    np.testing.assert_array_equal(render.load_stl(str(b)), tri)
    a = tmp_path / "a.stl"
    lines = ["solid x"]
    for t in tri:
        lines += ["facet normal 0 0 1", "outer loop"] + [f"vertex {v[0]} {v[1]} {v[2]}" for v in t]
        lines += ["endloop", "endfacet"]
    a.write_text("\n".join(lines + ["endsolid x"]))
    np.testing.assert_array_equal(render.load_stl(str(a)), tri)


@pytest.mark.skipif(not os.path.isdir(REF_MESHES), reason="reference mesh files not present")
def test_reference_meshes_load_and_replace_proxies():
    t = render.load_stl(os.path.join(REF_MESHES, "BodyV4v70_001.stl"))
    with open(os.path.join(REF_MESHES, "BodyV4v70_001.stl"), "rb") as f:
        f.seek(80)
        n = struct.unpack("<I", f.read(4))[0]
    assert t.shape == (n, 3, 3) and np.isfinite(t).all()
    sc = render.Scene(mjcf.load(MODEL_XML), meshdir=REF_MESHES)
    assert not sc.proxies and len(sc.items) == 13  # the 13 visual meshes
    # the mirrored leg meshes carry their asset scale
    assert (sc.tris.reshape(-1, 3, 3)[:, :, 1].min() < 0) and len(sc.tris) > 10 * n // 10


def test_scene_without_meshes_uses_proxies():
    cm = mjcf.load(MODEL_XML)
    sc = render.Scene(cm, meshdir="/nonexistent")
    assert sc.proxies
    nsph = sum(1 for g in cm.visual["geoms"] if g["type"] == mjcf.GEOM_TYPES["sphere"] and g["body"] > 0)
    assert len(sc.items) == nsph + 12 + 1  # spheres, one capsule per leg link, torso box
    f = sc.floor  # floor_visual: material "grid" = builtin checker, texuniform, texrepeat 1
    assert f["on"] and f["check"] == 0.5
    np.testing.assert_allclose(f["rgb1"], [0.2, 0.4, 0.6])
    np.testing.assert_allclose(f["rgb2"], [0.4, 0.6, 0.8])
    np.testing.assert_allclose(sc.sky_top, [0.3, 0.5, 0.7])
    xf = sc.transforms(_home_q())
    assert xf.shape == (len(sc.items), 12)
    R = xf[:, :9].reshape(-1, 3, 3)
    np.testing.assert_allclose(R @ R.transpose(0, 2, 1), np.broadcast_to(np.eye(3), R.shape), atol=1e-5)


def test_tracking_camera_follows_mujoco_targetbody_rules():
    sc = render.Scene(mjcf.load(MODEL_XML), meshdir="/nonexistent")
    q = _home_q()
    q[0:2] = [0.3, -0.2]
    c = sc.camera("tracking_cam", q, 240)
    pos, right, up, fwd, fpx = c[0:3], c[3:6], c[6:9], c[9:12], c[12]
    np.testing.assert_allclose(pos, [0.5, -0.5, 0.5])  # fixed in the world (parent = world)
    target = np.array([0.3, -0.2, 0.17])  # the target body's origin
    np.testing.assert_allclose(fwd, (target - pos) / np.linalg.norm(target - pos), atol=1e-6)
    assert abs(right[2]) < 1e-7  # x axis orthogonal to world z
    B = np.stack([right, up, fwd])
    np.testing.assert_allclose(B @ B.T, np.eye(3), atol=1e-6)
    assert np.cross(right, up) @ fwd < 0  # right-handed camera frame looking along -z
    np.testing.assert_allclose(fpx, 120 / np.tan(np.radians(22.5)), rtol=1e-6)
    with pytest.raises(ValueError, match="does not exist"):
        sc.camera("track", q, 240)  # the reference's default name is not in the stock model


def test_cpu_restatement_draws_robot_floor_and_sky():
    sc = render.Scene(mjcf.load(MODEL_XML), meshdir="/nonexistent")
    H, W = 48, 64
    img = render_ref.render(sc, [_home_q()], "tracking_cam", H, W)[0]
    assert img.shape == (H, W, 3) and img.dtype == np.uint8
    # the camera aims at the base: the centre pixel is a robot fragment (grey proxies), not floor
    c = img[H // 2, W // 2].astype(int)
    assert abs(c[0] - c[2]) < 12, c
    # below the robot: checker floor in the two grid colours (blue-dominant)
    low = img[-2].astype(int)
    assert np.all(low[:, 2] > low[:, 0])
