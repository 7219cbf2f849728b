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


def _model_with_cameras(tmp_path):
    """The stock model plus a fixed camera nested in base_link, a track camera and a targetbodycom
    camera (advisor r02: cameras inside bodies must move with them)."""
    import xml.etree.ElementTree as ET
    tree = ET.parse(MODEL_XML)
    root = tree.getroot()
    base = next(b for b in root.iter("body") if b.get("name") == "base_link")
    ET.SubElement(base, "camera", {"name": "nested_fixed", "pos": "0.1 0 0.05", "quat": "1 0 0 0"})
    ET.SubElement(base, "camera", {"name": "nested_track", "mode": "track", "pos": "0 -0.5 0.3",
                                   "xyaxes": "1 0 0 0 0.5 1"})
    wb = root.find("worldbody")
    ET.SubElement(wb, "camera", {"name": "com_cam", "mode": "targetbodycom", "target": "base_link",
                                 "pos": "1 1 1"})
    path = str(tmp_path / "cams.xml")
    tree.write(path)
    return render.Scene(mjcf.load(path), meshdir="/nonexistent")


def test_nested_and_tracking_cameras_follow_mujoco_rules(tmp_path):
    sc = _model_with_cameras(tmp_path)
    q0 = _home_q()
    q1 = q0.copy()
    q1[0:3] += [0.4, -0.3, 0.1]
    half = np.radians(30) / 2
    q1[3:7] = [np.cos(half), 0, 0, np.sin(half)]  # base yawed 30 deg
    R1 = mjcf.quat_to_mat(q1[3:7])
    # fixed camera in base_link: rigidly attached (position and axes turn with the base)
    c0, c1 = sc.camera("nested_fixed", q0, 240), sc.camera("nested_fixed", q1, 240)
    np.testing.assert_allclose(c1[0:3], q1[0:3] + R1 @ np.array([0.1, 0, 0.05]), atol=1e-6)
    np.testing.assert_allclose(c1[3:6], R1 @ np.array([1.0, 0, 0]), atol=1e-6)
    np.testing.assert_allclose(c1[9:12], R1 @ np.array([0, 0, -1.0]), atol=1e-6)
    # track: constant world offset to the body and constant world orientation (those at qpos0)
    t0, t1 = sc.camera("nested_track", q0, 240), sc.camera("nested_track", q1, 240)
    np.testing.assert_allclose(t1[0:3] - t0[0:3], q1[0:3] - q0[0:3], atol=1e-6)
    np.testing.assert_allclose(t1[3:12], t0[3:12], atol=1e-7)
    # targetbodycom: looks at base_link's subtree centre of mass (the whole robot), not its origin
    m = sc.cm.struct
    xpos, R, sub = sc._frames(q1)
    c = sc.camera("com_cam", q1, 240)
    fwd = (sub[1] - np.array([1.0, 1, 1])) / np.linalg.norm(sub[1] - np.array([1.0, 1, 1]))
    np.testing.assert_allclose(c[9:12], fwd, atol=1e-6)
    assert np.linalg.norm(sub[1] - xpos[1]) > 1e-3 and m.body_mass[1] > 0


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
