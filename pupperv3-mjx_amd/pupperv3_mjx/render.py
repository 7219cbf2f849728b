"""PupperV3Env.render on the GPU (environment.py:545-547).

The reference delegates to Brax ``PipelineEnv.render`` ([ext] brax 0.12.1), i.e. MuJoCo's OpenGL
renderer on mjData rebuilt from each pipeline state's q, and uses it only for the policy videos
of ``utils.visualize_policy`` (utils.py:214-293, camera "tracking_cam", 240 x 320).  Here the same
call rasterises the model's visual geoms with the HIP kernels of ``csrc/pp3_render.hip``:

* geometry: every geom of the visible groups (MuJoCo's default 0, 1, 2) -- the robot's STL meshes
  (with the mesh asset's ``scale``) when the mesh files are found under ``meshdir`` (the MJCF
  ``<compiler meshdir>`` relative to the model file, or an explicit directory), primitives
  (sphere / box / capsule / cylinder) tessellated; without the mesh files, proxies: the
  collision spheres, a capsule per leg link between its joint anchor and the next, a torso box;
* per frame: forward kinematics from q (the MJCF compiler's float64 ``mjcf._kinematics``), the
  named camera by MuJoCo's rules (``mode="targetbody"``: fixed position, z axis from the target
  body's origin, x axis orthogonal to world z), ``fovy``;
* floor: the plane's builtin checker material (``texuniform``: squares of 1 / (2 texrepeat) m),
  skybox: the builtin gradient (rgb1 at the zenith, rgb2 at the nadir); headlight Lambert shading.

This is not MuJoCo's renderer (no shadows, reflections or light sources beyond the headlight);
it gives the same kind of video of the same scene from the same camera.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import struct
from typing import List, Optional, Sequence

import numpy as np

from . import _lib, mjcf

GROUPS_VISIBLE = (0, 1, 2)


def load_stl(path: str) -> np.ndarray:
    """Triangles [n, 3, 3] (float32) of a binary or ASCII STL file."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) >= 84:
        n = struct.unpack_from("<I", data, 80)[0]
        if 84 + 50 * n == len(data):
            rec = np.frombuffer(data, dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]),
                                count=n, offset=84)
            return rec["v"].astype(np.float32)
    verts = [list(map(float, line.split()[1:4])) for line in data.decode("ascii", "replace").splitlines()
             if line.strip().startswith("vertex")]
    if not verts or len(verts) % 3:
        raise ValueError(f"{path}: not an STL file")
    return np.asarray(verts, dtype=np.float32).reshape(-1, 3, 3)


# ---------------------------------------------------------------------------- tessellation
def _sphere(r: float, nlat: int = 8, nlon: int = 12) -> np.ndarray:
    th = np.linspace(0, math.pi, nlat + 1)
    ph = np.linspace(0, 2 * math.pi, nlon + 1)
    p = np.stack([np.outer(np.sin(th), np.cos(ph)), np.outer(np.sin(th), np.sin(ph)),
                  np.outer(np.cos(th), np.ones_like(ph))], -1) * r
    tris = []
    for i in range(nlat):
        for j in range(nlon):
            a, b, c, d = p[i, j], p[i + 1, j], p[i + 1, j + 1], p[i, j + 1]
            if i > 0:
                tris.append([a, b, d])
            if i < nlat - 1:
                tris.append([b, c, d])
    return np.asarray(tris, dtype=np.float32)


def _box(half: Sequence[float]) -> np.ndarray:
    hx, hy, hz = half
    v = np.array([[x, y, z] for x in (-hx, hx) for y in (-hy, hy) for z in (-hz, hz)], dtype=np.float32)
    faces = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    return np.asarray([[v[a], v[b], v[c]] for a, b, c, d in faces] + [[v[a], v[c], v[d]] for a, b, c, d in faces],
                      dtype=np.float32)


def _capsule(r: float, half_len: float, nlon: int = 12, caps: bool = True) -> np.ndarray:
    """Along z; `caps=False` gives a closed cylinder."""
    ph = np.linspace(0, 2 * math.pi, nlon + 1)
    ring = np.stack([r * np.cos(ph), r * np.sin(ph)], -1)
    tris = []
    for j in range(nlon):
        a0, a1 = ring[j], ring[j + 1]
        p00, p01 = [a0[0], a0[1], -half_len], [a1[0], a1[1], -half_len]
        p10, p11 = [a0[0], a0[1], half_len], [a1[0], a1[1], half_len]
        tris += [[p00, p01, p11], [p00, p11, p10]]
        if not caps:
            tris += [[[0, 0, -half_len], p01, p00], [[0, 0, half_len], p10, p11]]
    out = np.asarray(tris, dtype=np.float32)
    if caps:
        s = _sphere(r)
        top, bot = s.copy(), s.copy()
        top[..., 2] += half_len
        bot[..., 2] -= half_len
        out = np.concatenate([out, top, bot])
    return out


def _segment(p0: np.ndarray, p1: np.ndarray, r: float):
    """Capsule between two points: local triangles, local pose (pos, quat)."""
    d = p1 - p0
    L = float(np.linalg.norm(d))
    z = d / L if L > 1e-9 else np.array([0.0, 0, 1])
    axis = np.cross([0.0, 0, 1], z)
    s = float(np.linalg.norm(axis))
    ang = math.atan2(s, float(z[2]))
    q = mjcf.axis_angle_quat(axis / s, ang) if s > 1e-9 else (np.array([1.0, 0, 0, 0]) if z[2] > 0 else
                                                              np.array([0.0, 1, 0, 0]))
    return _capsule(r, 0.5 * L), 0.5 * (p0 + p1), q


# ---------------------------------------------------------------------------- scene
class Scene:
    """Triangle soup of a compiled model's visual geoms, in geom-local frames."""

    def __init__(self, cm: "mjcf.CompiledModel", meshdir: Optional[str] = None, groups=GROUPS_VISIBLE):
        vis = cm.visual
        self.cm = cm
        if meshdir is None and vis.get("meshdir") is not None:
            meshdir = os.path.normpath(os.path.join(vis.get("source_dir", "."), vis["meshdir"]))
        self.meshdir = meshdir
        self.items: List[dict] = []  # draw items: body, local pos, local quat, rgb
        tris, owner = [], []
        self.floor = None
        missing = False

        def add(t: np.ndarray, body: int, pos, quat, rgb):
            self.items.append(dict(body=int(body), pos=np.asarray(pos, float), quat=np.asarray(quat, float),
                                   rgb=np.asarray(rgb[:3], np.float32)))
            tris.append(t.reshape(-1, 9))
            owner.append(np.full(len(t), len(self.items) - 1, np.int32))

        for g in vis["geoms"]:
            if g["type"] == mjcf.GEOM_TYPES["plane"]:
                if g["group"] in groups and self.floor is None:
                    self.floor = self._floor_params(g)
                continue
            if g["group"] not in groups:
                continue
            rgb = g["rgba"]
            if g["material"] and g["material"] in vis["materials"]:
                rgb = vis["materials"][g["material"]]["rgba"]
            if g["type"] == mjcf.GEOM_TYPES["mesh"]:
                asset = vis["meshes"].get(g["mesh"])
                path = os.path.join(meshdir, asset["file"]) if (asset and meshdir) else None
                if not path or not os.path.exists(path):
                    missing = True
                    continue
                t = load_stl(path) * asset["scale"].astype(np.float32)
            elif g["type"] == mjcf.GEOM_TYPES["sphere"]:
                t = _sphere(g["size"][0])
            elif g["type"] == mjcf.GEOM_TYPES["box"]:
                t = _box(g["size"])
            elif g["type"] == mjcf.GEOM_TYPES["capsule"]:
                t = _capsule(g["size"][0], g["size"][1])
            elif g["type"] == mjcf.GEOM_TYPES["cylinder"]:
                t = _capsule(g["size"][0], g["size"][1], caps=False)
            else:
                continue
            add(t, g["body"], g["pos"], g["quat"], rgb)
        self.proxies = missing
        if missing:
            self._add_proxies(add)
        if self.floor is None:
            self.floor = dict(rgb1=np.zeros(3), rgb2=np.zeros(3), check=1.0, z=0.0, on=False)
        sky = vis.get("skybox")
        self.sky_top = sky["rgb1"] if sky else np.array([0.3, 0.5, 0.7])
        self.sky_bottom = sky["rgb2"] if sky else np.zeros(3)
        self.tris = np.ascontiguousarray(np.concatenate(tris) if tris else np.zeros((0, 9), np.float32), np.float32)
        self.tri_owner = np.ascontiguousarray(np.concatenate(owner) if owner else np.zeros(0, np.int32))
        self.rgb = np.ascontiguousarray(np.array([it["rgb"] for it in self.items], np.float32).reshape(-1, 3))

    def _floor_params(self, g) -> dict:
        vis = self.cm.visual
        mat = vis["materials"].get(g["material"]) if g["material"] else None
        tex = vis["textures"].get(mat["texture"]) if mat and mat.get("texture") else None
        if tex is not None and tex["builtin"] == "checker":
            rep = float(mat["texrepeat"][0]) if mat["texuniform"] else 1.0
            return dict(rgb1=tex["rgb1"], rgb2=tex["rgb2"], check=0.5 / max(rep, 1e-9), z=float(g["pos"][2]), on=True)
        rgb = g["rgba"][:3]
        return dict(rgb1=rgb, rgb2=rgb, check=1.0, z=float(g["pos"][2]), on=True)

    def _add_proxies(self, add):
        """No mesh files: the collision spheres, a capsule per leg link (joint anchor to the next
        anchor or the foot sphere) and a torso box (the commented-out torso box of the model)."""
        cm, m = self.cm, self.cm.struct
        vis = cm.visual
        grey, dark = np.array([0.75, 0.75, 0.78]), np.array([0.25, 0.25, 0.3])
        for g in vis["geoms"]:
            if g["type"] == mjcf.GEOM_TYPES["sphere"] and g["body"] > 0:
                add(_sphere(g["size"][0]), g["body"], g["pos"], g["quat"], dark)
        nb = len(cm.body_names)
        children = {b: [c for c in range(nb) if m.body_parentid[c] == b] for b in range(nb)}
        for b in range(2, nb):
            p0 = np.zeros(3)
            kids = children[b]
            if kids:
                p1 = np.array(m.body_pos[kids[0]][:])
            else:
                sph = [g for g in vis["geoms"] if g["body"] == b and g["type"] == mjcf.GEOM_TYPES["sphere"]]
                p1 = np.asarray(sph[-1]["pos"]) if sph else p0 + [0, 0, -0.05]
            t, pos, q = _segment(p0, p1, 0.012)
            add(t, b, pos, q, grey)
        add(_box([0.04507, 0.06379, 0.129715]), 1, [0.02146, 0.0, 0.03345], [1.0, 0, 0, 0], grey)

    def transforms(self, qpos: np.ndarray) -> np.ndarray:
        """[n_items][12] world rotation (row-major) + translation for one configuration."""
        xpos, xquat, _, _ = mjcf._kinematics(self.cm.struct, np.asarray(qpos, np.float64))
        out = np.zeros((len(self.items), 12), np.float32)
        for i, it in enumerate(self.items):
            Rb = mjcf.quat_to_mat(xquat[it["body"]])
            out[i, :9] = (Rb @ mjcf.quat_to_mat(it["quat"])).reshape(-1)
            out[i, 9:] = xpos[it["body"]] + Rb @ it["pos"]
        return out

    def _frames(self, qpos):
        """Body origins, rotations and subtree centres of mass at qpos (mj_kinematics, mj_comPos)."""
        m = self.cm.struct
        xpos, xquat, _, _ = mjcf._kinematics(m, np.asarray(qpos, np.float64))
        R = np.array([mjcf.quat_to_mat(q) for q in xquat])
        nb = len(xpos)
        mass = np.array(m.body_mass[:nb], float)
        xipos = np.array([xpos[b] + R[b] @ np.array(m.body_ipos[b][:]) for b in range(nb)])
        com = np.zeros((nb, 3))
        msum = np.zeros(nb)
        for b in range(nb - 1, 0, -1):  # children have larger ids than their parents
            com[b] += mass[b] * xipos[b]
            msum[b] += mass[b]
            p = m.body_parentid[b]
            if p > 0:
                com[p] += com[b]
                msum[p] += msum[b]
        subtree = np.where(msum[:, None] > 0, com / np.maximum(msum, 1e-300)[:, None], xipos)
        return xpos, R, subtree

    def camera(self, name, qpos: np.ndarray, height: int) -> np.ndarray:
        """[16]: position, right, up, forward, focal length in pixels, by MuJoCo's camera rules
        (mj_camlight): the camera's pose is given in its parent body's frame; "fixed" moves with
        that body, "track" / "trackcom" keep the world offset to the body / its subtree COM and the
        world orientation they have at qpos0, "targetbody" / "targetbodycom" sit where "fixed" puts
        them and look at the target body's origin / subtree COM."""
        vis = self.cm.visual
        xpos, R, subtree = self._frames(qpos)
        if name is None or (isinstance(name, int) and name < 0):  # MuJoCo's free camera: look at the base
            target = xpos[1]
            pos = target + np.array([0.0, -1.0, 0.6])
            fovy = 45.0
            z = pos - target
        else:
            if name not in vis["cameras"]:
                raise ValueError(f'The camera "{name}" does not exist.')
            cam = vis["cameras"][name]
            fovy = cam["fovy"]
            b = cam["parent"]
            mode = cam["mode"]
            lpos, lR = np.array(cam["pos"], float), mjcf.quat_to_mat(cam["quat"])
            frame = None  # the camera frame's world axes, where the mode fixes them
            if mode in ("track", "trackcom"):
                x0, R0, c0 = self._frames(np.array(self.cm.struct.qpos0[:]))
                anchor0 = (c0 if mode == "trackcom" else x0)[b]
                anchor = (subtree if mode == "trackcom" else xpos)[b]
                pos = anchor + (x0[b] + R0[b] @ lpos - anchor0)
                frame = R0[b] @ lR
            elif mode in ("fixed", "targetbody", "targetbodycom"):
                pos = xpos[b] + R[b] @ lpos
                frame = R[b] @ lR
                if mode != "fixed" and cam["target"] >= 0:
                    tgt = (subtree if mode == "targetbodycom" else xpos)[cam["target"]]
                    frame = None
                    z = pos - tgt
            else:
                raise NotImplementedError(f'camera mode "{mode}"')
            if frame is not None:
                fpx = 0.5 * height / math.tan(math.radians(fovy) / 2)
                return np.concatenate([pos, frame[:, 0], frame[:, 1], -frame[:, 2], [fpx, 0, 0, 0]]).astype(np.float32)
        z = z / np.linalg.norm(z)
        x = np.cross([0.0, 0.0, 1.0], z)
        if np.linalg.norm(x) < 1e-9:
            x = np.array([1.0, 0, 0])
        x = x / np.linalg.norm(x)
        y = np.cross(z, x)
        fpx = 0.5 * height / math.tan(math.radians(fovy) / 2)
        return np.concatenate([pos, x, y, -z, [fpx, 0, 0, 0]]).astype(np.float32)

    def scene_params(self, ambient: float = 0.35, diffuse: float = 0.65) -> np.ndarray:
        f = self.floor
        return np.concatenate([f["rgb1"], f["rgb2"], [f["check"], f["z"]], self.sky_top, self.sky_bottom,
                               [ambient, diffuse, 1.0 if f["on"] else 0.0]]).astype(np.float32)


def render_qpos(scene: Scene, qposes: Sequence[np.ndarray], camera="tracking_cam", height: int = 240,
                width: int = 320, device: int = 0, chunk: int = 64) -> List[np.ndarray]:
    """Frames [height, width, 3] u8, one per configuration."""
    L = _lib.load()
    qposes = [np.asarray(q, np.float64).reshape(-1) for q in qposes]
    frames: List[np.ndarray] = []
    if not qposes:
        return frames
    tri_b = _lib.DeviceBuffer(max(scene.tris.nbytes, 4), device)
    own_b = _lib.DeviceBuffer(max(scene.tri_owner.nbytes, 4), device)
    rgb_b = _lib.DeviceBuffer(max(scene.rgb.nbytes, 4), device)
    if len(scene.tris):
        tri_b.upload(scene.tris)
        own_b.upload(scene.tri_owner)
        rgb_b.upload(scene.rgb)
    sp = scene.scene_params()
    ng = max(len(scene.items), 1)
    try:
        for c0 in range(0, len(qposes), chunk):
            qs = qposes[c0:c0 + chunk]
            F = len(qs)
            xf = np.zeros((F, ng, 12), np.float32)
            cams = np.zeros((F, 16), np.float32)
            for i, q in enumerate(qs):
                if scene.items:
                    xf[i] = scene.transforms(q)
                cams[i] = scene.camera(camera, q, height)
            xf_b = _lib.DeviceBuffer(xf.nbytes, device)
            cam_b = _lib.DeviceBuffer(cams.nbytes, device)
            out_b = _lib.DeviceBuffer(F * height * width * 3, device)
            try:
                xf_b.upload(xf)
                cam_b.upload(cams)
                rc = L.pp3_render(device, tri_b.ptr, own_b.ptr, len(scene.tris), rgb_b.ptr, ng, xf_b.ptr, cam_b.ptr, F,
                                  height, width, sp.ctypes.data_as(C.POINTER(C.c_float)), out_b.ptr, None)
                if rc != 0:
                    raise _lib.PupperHipError(f"pp3_render error {rc}: {L.pp3_render_last_error().decode()}")
                img = np.empty((F, height, width, 3), np.uint8)
                out_b.download(img)
                frames += list(img)
            finally:
                xf_b.free()
                cam_b.free()
                out_b.free()
    finally:
        tri_b.free()
        own_b.free()
        rgb_b.free()
    return frames
