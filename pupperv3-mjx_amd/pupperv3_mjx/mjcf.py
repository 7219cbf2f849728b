"""MJCF-subset compiler: test_pupper_model.xml (+ obstacles.py boxes) -> pp3_model_t.

Replaces the model-construction half of ``brax.io.mjcf.load`` / ``mujoco.MjModel``
([ext] mujoco 3.2.7, called at environment.py:165) for exactly the MJCF features the
reference model uses:

* ``<default>`` classes (nested, ``class=``) for geom / joint / general / site;
* bodies with pos/quat (or axisangle), ``<inertial pos quat mass diaginertia>``,
  ``<freejoint>`` (MuJoCo's shortcut: no armature/damping/frictionloss/limits),
  hinge ``<joint>`` (pos, axis, range, limited, armature, damping, frictionloss);
* sphere / plane / box geoms (meshes are visual only here: contype=conaffinity=0 and
  density=0 in test_pupper_model.xml:89-90 etc., so they only reserve geom ids);
* sites, ``<general>`` joint actuators (gain/bias/forcerange), ``<option>``,
  ``<keyframe name="home">`` and ``<custom><numeric>``.

Derived constants follow MuJoCo's ``mj_setConst`` (engine_setconst.c, [ext]):
``dof_invweight0`` = diag(M^-1) at qpos0 (averaged over the 3 translational / 3
rotational dofs of the free joint), ``body_invweight0`` = mean diagonal of the
translational / rotational blocks of J_com M^-1 J_com^T, ``meaninertia`` = mean
diag(M).  Everything here is float64 numpy and runs once on the host.
"""
from __future__ import annotations

import copy
import ctypes
import math
import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple, Union

import numpy as np

from . import _abi

GEOM_TYPES = {"plane": 0, "hfield": 1, "sphere": 2, "capsule": 3, "ellipsoid": 4,
              "cylinder": 5, "box": 6, "mesh": 7}
JNT_FREE, JNT_HINGE = 0, 3

# MuJoCo built-in defaults (mjs_defaultGeom / mjs_defaultJoint / mjs_defaultActuator).
_GEOM_DEFAULTS = dict(type="sphere", size="0 0 0", pos="0 0 0", quat="1 0 0 0", contype="1",
                      conaffinity="1", condim="3", group="0", priority="0",
                      friction="1 0.005 0.0001", solmix="1", solref="0.02 1",
                      solimp="0.9 0.95 0.001 0.5 2", margin="0", gap="0", density="1000")
_JOINT_DEFAULTS = dict(type="hinge", pos="0 0 0", axis="0 0 1", range="0 0", limited="auto",
                       armature="0", damping="0", frictionloss="0", margin="0",
                       solreflimit="0.02 1", solimplimit="0.9 0.95 0.001 0.5 2",
                       solreffriction="0.02 1", solimpfriction="0.9 0.95 0.001 0.5 2", ref="0")
_ACT_DEFAULTS = dict(gainprm="1 0 0", biasprm="0 0 0", biastype="none", gaintype="fixed",
                     forcerange="0 0", forcelimited="auto", ctrlrange="0 0", ctrllimited="auto",
                     gear="1 0 0 0 0 0", dyntype="none")
_SITE_DEFAULTS = dict(pos="0 0 0", quat="1 0 0 0")


def _vec(s: str, n: Optional[int] = None, fill: Optional[List[float]] = None) -> np.ndarray:
    vals = [float(x) for x in s.split()]
    if n is not None and len(vals) < n:
        base = list(fill) if fill is not None else [0.0] * n
        vals = vals + base[len(vals):n]
    return np.array(vals, dtype=np.float64)


def quat_normalize(q: np.ndarray) -> np.ndarray:
    n = np.linalg.norm(q)
    return q / n if n > 0 else np.array([1.0, 0, 0, 0])


def quat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return np.array([
        a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
        a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
        a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
        a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0],
    ])


def quat_to_mat(q: np.ndarray) -> np.ndarray:
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def axis_angle_quat(axis: np.ndarray, angle: float) -> np.ndarray:
    a = np.asarray(axis, dtype=np.float64)
    a = a / np.linalg.norm(a)
    return np.concatenate([[math.cos(angle / 2)], a * math.sin(angle / 2)])


class _Defaults:
    """Tree of <default> classes; attribute lookup walks class -> parents."""

    def __init__(self):
        self.classes: Dict[str, Dict[str, Dict[str, str]]] = {"main": {}}
        self.parent: Dict[str, Optional[str]] = {"main": None}

    def parse(self, node: ET.Element, name: str, parent: Optional[str]):
        self.classes.setdefault(name, {})
        self.parent[name] = parent
        for child in node:
            if child.tag == "default":
                self.parse(child, child.get("class", name), name)
            else:
                self.classes[name].setdefault(child.tag, {}).update(child.attrib)

    def resolve(self, tag: str, cls: str, builtin: Dict[str, str]) -> Dict[str, str]:
        chain = []
        c: Optional[str] = cls
        while c is not None:
            chain.append(c)
            c = self.parent.get(c)
        out = dict(builtin)
        for c in reversed(chain):
            out.update(self.classes.get(c, {}).get(tag, {}))
        return out


@dataclass
class _Body:
    name: str
    parent: int
    pos: np.ndarray
    quat: np.ndarray
    ipos: np.ndarray = field(default_factory=lambda: np.zeros(3))
    iquat: np.ndarray = field(default_factory=lambda: np.array([1.0, 0, 0, 0]))
    mass: float = 0.0
    inertia: np.ndarray = field(default_factory=lambda: np.zeros(3))
    joints: List[int] = field(default_factory=list)
    geoms: List[int] = field(default_factory=list)
    sites: List[int] = field(default_factory=list)
    childclass: Optional[str] = None


@dataclass
class CompiledModel:
    """Host-side compiled model (float64) + name tables; `.struct` is the ABI blob."""

    struct: "_abi.Model"
    body_names: List[str]
    joint_names: List[str]
    geom_names: List[str]
    site_names: List[str]
    sensor_names: List[str]
    actuator_names: List[str]
    body_geomadr: np.ndarray
    body_geomnum: np.ndarray
    geom_bodyid: np.ndarray
    geom_type: np.ndarray
    geom_friction: np.ndarray
    jnt_range: np.ndarray
    xml: str
    # rendering-only description (render.py): visual geoms, mesh assets, materials, cameras
    visual: Dict = field(default_factory=dict)

    # --- name -> id helpers (mujoco.mj_name2id equivalents, environment.py:17-29) ---
    def body_id(self, name: str) -> int:
        return self.body_names.index(name) if name in self.body_names else -1

    def site_id(self, name: str) -> int:
        return self.site_names.index(name) if name in self.site_names else -1

    def body_geom_ids(self, name: str) -> np.ndarray:
        b = self.body_id(name)
        return self.body_geomadr[b] + np.arange(self.body_geomnum[b])

    @property
    def nq(self) -> int:
        return _abi.NQ

    @property
    def nv(self) -> int:
        return _abi.NV

    @property
    def nu(self) -> int:
        return _abi.NU

    @property
    def ngeom(self) -> int:
        return int(self.struct.ngeom)

    @property
    def nbody(self) -> int:
        return _abi.NBODY

    def copy(self) -> "CompiledModel":
        c = copy.copy(self)
        c.struct = _abi.Model.from_buffer_copy(self.struct)
        return c


def load(path_or_xml: Union[str, "ET.ElementTree"], is_string: bool = False) -> CompiledModel:
    """Compile an MJCF file/string/ElementTree into a CompiledModel."""
    if isinstance(path_or_xml, ET.ElementTree):
        root = path_or_xml.getroot()
        xml = ET.tostring(root, encoding="unicode")
    elif is_string or path_or_xml.lstrip().startswith("<"):
        xml = path_or_xml
        root = ET.fromstring(xml)
    else:
        with open(path_or_xml) as f:
            xml = f.read()
        root = ET.fromstring(xml)
        cm = _compile(root, xml)
        cm.visual["source_dir"] = os.path.dirname(os.path.abspath(path_or_xml))
        return cm
    return _compile(root, xml)


def _orientation(attrs: Dict[str, str], angle_deg: bool) -> np.ndarray:
    if "quat" in attrs and "axisangle" not in attrs:
        return quat_normalize(_vec(attrs["quat"]))
    if "axisangle" in attrs:
        v = _vec(attrs["axisangle"])
        ang = math.radians(v[3]) if angle_deg else v[3]
        return axis_angle_quat(v[:3], ang)
    if "xyaxes" in attrs:  # x axis, then y made orthogonal to it; z = x cross y (MJCF spec)
        v = _vec(attrs["xyaxes"])
        x = v[:3] / np.linalg.norm(v[:3])
        y = v[3:6] - (v[3:6] @ x) * x
        y = y / np.linalg.norm(y)
        return _mat_to_quat(np.stack([x, y, np.cross(x, y)], axis=1))
    if "zaxis" in attrs:  # the minimal rotation taking (0, 0, 1) to the given axis
        z = _vec(attrs["zaxis"])
        z = z / np.linalg.norm(z)
        axis = np.cross([0.0, 0.0, 1.0], z)
        s, c = np.linalg.norm(axis), z[2]
        if s < 1e-12:
            return np.array([1.0, 0, 0, 0]) if c > 0 else np.array([0.0, 1.0, 0, 0])
        return axis_angle_quat(axis / s, math.atan2(s, c))
    if "euler" in attrs:
        raise NotImplementedError("MJCF orientation 'euler' is not used by the Pupper model")
    return np.array([1.0, 0, 0, 0])


def _mat_to_quat(R: np.ndarray) -> np.ndarray:
    """Unit quaternion (w, x, y, z) of a rotation matrix (columns = the frame's axes)."""
    t = np.trace(R)
    if t > 0:
        w = math.sqrt(1.0 + t) / 2
        q = [w, (R[2, 1] - R[1, 2]) / (4 * w), (R[0, 2] - R[2, 0]) / (4 * w), (R[1, 0] - R[0, 1]) / (4 * w)]
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        r = math.sqrt(max(1.0 + R[i, i] - R[j, j] - R[k, k], 1e-300))
        q = [0.0, 0.0, 0.0, 0.0]
        q[1 + i] = r / 2
        q[0] = (R[k, j] - R[j, k]) / (2 * r)
        q[1 + j] = (R[j, i] + R[i, j]) / (2 * r)
        q[1 + k] = (R[k, i] + R[i, k]) / (2 * r)
    q = np.array(q)
    return q / np.linalg.norm(q)


def _compile(root: ET.Element, xml: str) -> CompiledModel:
    defaults = _Defaults()
    for d in root.findall("default"):
        defaults.parse(d, d.get("class", "main"), None if d.get("class", "main") == "main" else "main")
    compiler = root.find("compiler")
    angle_deg = not (compiler is not None and compiler.get("angle", "degree") == "radian")
    autolimits = not (compiler is not None and compiler.get("autolimits", "true") == "false")

    bodies: List[_Body] = [_Body("world", -1, np.zeros(3), np.array([1.0, 0, 0, 0]))]
    joints: List[dict] = []
    geoms: List[dict] = []
    sites: List[dict] = []

    def add_geoms_sites(node: ET.Element, bid: int, cls: str):
        for g in node.findall("geom"):
            a = defaults.resolve("geom", g.get("class", cls), _GEOM_DEFAULTS)
            a.update(g.attrib)
            gtype = a["type"]
            if gtype not in GEOM_TYPES:
                raise NotImplementedError(f"geom type {gtype}")
            geoms.append(dict(
                name=a.get("name", ""), body=bid, type=GEOM_TYPES[gtype],
                size=_vec(a["size"], 3), pos=_vec(a["pos"], 3),
                quat=_orientation(a, angle_deg), contype=int(a["contype"]),
                conaffinity=int(a["conaffinity"]), condim=int(a["condim"]),
                priority=int(a["priority"]),
                friction=_vec(a["friction"], 3, [1, 0.005, 0.0001]), solmix=float(a["solmix"]),
                solref=_vec(a["solref"], 2, [0.02, 1]),
                solimp=_vec(a["solimp"], 5, [0.9, 0.95, 0.001, 0.5, 2]),
                margin=float(a["margin"]), gap=float(a["gap"]),
                group=int(a.get("group", "0")), mesh=a.get("mesh"), material=a.get("material"),
                rgba=_vec(a.get("rgba", "0.5 0.5 0.5 1"), 4)))
            bodies[bid].geoms.append(len(geoms) - 1)
        for s in node.findall("site"):
            a = defaults.resolve("site", s.get("class", cls), _SITE_DEFAULTS)
            a.update(s.attrib)
            sites.append(dict(name=a.get("name", ""), body=bid, pos=_vec(a["pos"], 3),
                              quat=_orientation(a, angle_deg)))
            bodies[bid].sites.append(len(sites) - 1)

    def walk(node: ET.Element, parent: int, cls: str):
        for b in node.findall("body"):
            bcls = b.get("childclass", cls)
            body = _Body(b.get("name", f"body{len(bodies)}"), parent, _vec(b.get("pos", "0 0 0")),
                         _orientation(b.attrib, angle_deg))
            bid = len(bodies)
            bodies.append(body)
            inert = b.find("inertial")
            if inert is None:
                raise NotImplementedError("bodies must carry an explicit <inertial> (inertiafromgeom unsupported)")
            body.ipos = _vec(inert.get("pos", "0 0 0"))
            body.iquat = _orientation(inert.attrib, angle_deg)
            body.mass = float(inert.get("mass"))
            if "fullinertia" in inert.attrib:
                raise NotImplementedError("fullinertia")
            body.inertia = _vec(inert.get("diaginertia"))
            for child in b:
                if child.tag == "freejoint":
                    # MuJoCo: <freejoint> ignores joint defaults (no damping/armature/frictionloss).
                    joints.append(dict(name=child.get("name", ""), type=JNT_FREE, body=bid,
                                       pos=np.zeros(3), axis=np.array([0.0, 0, 1]), range=np.zeros(2),
                                       limited=0, armature=0.0, damping=0.0, frictionloss=0.0,
                                       margin=0.0, solreflimit=np.array([0.02, 1]),
                                       solimplimit=np.array([0.9, 0.95, 0.001, 0.5, 2]),
                                       solreffriction=np.array([0.02, 1]),
                                       solimpfriction=np.array([0.9, 0.95, 0.001, 0.5, 2])))
                    body.joints.append(len(joints) - 1)
                elif child.tag == "joint":
                    explicit = defaults.resolve("joint", child.get("class", bcls), {})
                    explicit.update(child.attrib)
                    a = dict(_JOINT_DEFAULTS)
                    a.update(explicit)
                    jt = a["type"]
                    if jt == "free":
                        jtype = JNT_FREE
                    elif jt == "hinge":
                        jtype = JNT_HINGE
                    else:
                        raise NotImplementedError(f"joint type {jt}")
                    rng = _vec(a["range"], 2)
                    if rng[0] != 0 or rng[1] != 0:
                        if angle_deg and jtype == JNT_HINGE:
                            rng = np.radians(rng)
                    lim = a["limited"]
                    limited = 1 if lim == "true" else 0 if lim == "false" else int(autolimits and "range" in explicit)
                    if float(a.get("ref", "0")) != 0.0:
                        raise NotImplementedError("joint ref")
                    axis = _vec(a["axis"], 3)
                    joints.append(dict(name=a.get("name", ""), type=jtype, body=bid, pos=_vec(a["pos"], 3),
                                       axis=axis / np.linalg.norm(axis), range=rng, limited=limited,
                                       armature=float(a["armature"]), damping=float(a["damping"]),
                                       frictionloss=float(a["frictionloss"]), margin=float(a["margin"]),
                                       solreflimit=_vec(a["solreflimit"], 2, [0.02, 1]),
                                       solimplimit=_vec(a["solimplimit"], 5, [0.9, 0.95, 0.001, 0.5, 2]),
                                       solreffriction=_vec(a["solreffriction"], 2, [0.02, 1]),
                                       solimpfriction=_vec(a["solimpfriction"], 5, [0.9, 0.95, 0.001, 0.5, 2])))
                    body.joints.append(len(joints) - 1)
            add_geoms_sites(b, bid, bcls)
            walk(b, bid, bcls)

    worldbody = root.find("worldbody")
    # MuJoCo numbers objects body by body (world first), children in document order.
    add_geoms_sites(worldbody, 0, "main")
    walk(worldbody, 0, "main")
    # Re-number geoms/sites in body order (world geoms were appended first already; the
    # depth-first walk appends per body, which is MuJoCo's order).
    geom_order = [g for b in bodies for g in b.geoms]
    site_order = [s for b in bodies for s in b.sites]
    geoms = [geoms[i] for i in geom_order]
    sites = [sites[i] for i in site_order]
    gid = 0
    for b in bodies:
        b.geoms = list(range(gid, gid + len(b.geoms)))
        gid += len(b.geoms)
    sid = 0
    for b in bodies:
        b.sites = list(range(sid, sid + len(b.sites)))
        sid += len(b.sites)

    # ---------------- topology check: free base + 4 chains of 3 hinges -------------
    if len(bodies) != _abi.NBODY or len(joints) != _abi.NJNT:
        raise ValueError(f"unsupported topology: nbody={len(bodies)} njnt={len(joints)}")
    if joints[0]["type"] != JNT_FREE or joints[0]["body"] != 1 or bodies[1].parent != 0:
        raise ValueError("model must start with a free-floating base body")
    for leg in range(4):
        for k in range(3):
            b = 2 + 3 * leg + k
            if bodies[b].parent != (1 if k == 0 else b - 1) or len(bodies[b].joints) != 1:
                raise ValueError("legs must be serial chains of 3 single-hinge bodies")
            if joints[bodies[b].joints[0]]["type"] != JNT_HINGE:
                raise ValueError("leg joints must be hinges")

    m = _abi.Model()
    # ---------------- <option> ---------------
    opt = root.find("option")
    oa = opt.attrib if opt is not None else {}
    m.timestep = float(oa.get("timestep", "0.002"))
    m.gravity[:] = list(_vec(oa.get("gravity", "0 0 -9.81")))
    m.impratio = float(oa.get("impratio", "1"))
    m.tolerance = float(oa.get("tolerance", "1e-8"))
    m.ls_tolerance = float(oa.get("ls_tolerance", "0.01"))
    m.iterations = int(oa.get("iterations", "100"))
    m.ls_iterations = int(oa.get("ls_iterations", "50"))
    if oa.get("cone", "pyramidal") != "pyramidal":
        raise NotImplementedError("only pyramidal cones (xml:57)")
    if oa.get("solver", "Newton") != "Newton":
        raise NotImplementedError("only the Newton solver (MuJoCo default)")
    if oa.get("integrator", "Euler") != "Euler":
        raise NotImplementedError("only the Euler integrator")
    if int(oa.get("noslip_iterations", "0")) != 0:
        raise NotImplementedError("noslip")
    m.cone = 0
    eulerdamp = 1
    if opt is not None:
        fl = opt.find("flag")
        if fl is not None and fl.get("eulerdamp", "enable") == "disable":
            eulerdamp = 0
    m.eulerdamp = eulerdamp

    # ---------------- bodies / joints / dofs ----------------
    dof = 0
    qadr = 0
    dof_body, dof_jnt, dof_parent = [], [], []
    last_dof_of_body = {0: -1}
    for bi, b in enumerate(bodies):
        m.body_parentid[bi] = b.parent
        m.body_pos[bi][:] = list(b.pos)
        m.body_quat[bi][:] = list(b.quat)
        m.body_ipos[bi][:] = list(b.ipos)
        m.body_iquat[bi][:] = list(b.iquat)
        m.body_mass[bi] = b.mass
        m.body_inertia[bi][:] = list(b.inertia)
        m.body_jntadr[bi] = b.joints[0] if b.joints else -1
        m.body_dofadr[bi] = dof if b.joints else -1
        parent_last = last_dof_of_body.get(b.parent, -1)
        nd = 0
        for j in b.joints:
            jj = joints[j]
            ndj = 6 if jj["type"] == JNT_FREE else 1
            m.jnt_type[j] = jj["type"]
            m.jnt_bodyid[j] = bi
            m.jnt_qposadr[j] = qadr
            m.jnt_dofadr[j] = dof
            m.jnt_limited[j] = jj["limited"]
            m.jnt_pos[j][:] = list(jj["pos"])
            m.jnt_axis[j][:] = list(jj["axis"])
            m.jnt_range[j][:] = list(jj["range"])
            m.jnt_margin[j] = jj["margin"]
            m.jnt_solref[j][:] = list(jj["solreflimit"])
            m.jnt_solimp[j][:] = list(jj["solimplimit"])
            for k in range(ndj):
                d = dof + k
                dof_body.append(bi)
                dof_jnt.append(j)
                dof_parent.append(parent_last if (k == 0 and nd == 0) else d - 1)
                m.dof_armature[d] = jj["armature"]
                m.dof_damping[d] = jj["damping"]
                m.dof_frictionloss[d] = jj["frictionloss"]
                m.dof_solref[d][:] = list(jj["solreffriction"])
                m.dof_solimp[d][:] = list(jj["solimpfriction"])
            if jj["type"] == JNT_FREE:
                m.qpos0[qadr:qadr + 3] = list(b.pos)
                m.qpos0[qadr + 3:qadr + 7] = list(b.quat)
                qadr += 7
            else:
                m.qpos0[qadr] = 0.0
                qadr += 1
            dof += ndj
            nd += ndj
        m.body_dofnum[bi] = nd
        last_dof_of_body[bi] = dof - 1 if nd else parent_last
    for d in range(dof):
        m.dof_bodyid[d] = dof_body[d]
        m.dof_jntid[d] = dof_jnt[d]
        m.dof_parentid[d] = dof_parent[d]

    # keyframe "home"
    key_q = np.array(m.qpos0[:])
    kf = root.find("keyframe")
    if kf is not None:
        for k in kf.findall("key"):
            if k.get("name") == "home" and "qpos" in k.attrib:
                key_q = _vec(k.get("qpos"))
    m.key_qpos[:] = list(key_q)

    # ---------------- geoms / pairs ----------------
    m.ngeom = len(geoms)
    cg = [i for i, g in enumerate(geoms) if g["contype"] or g["conaffinity"]]
    if len(cg) > _abi.MAX_CGEOM:
        raise ValueError("too many collidable geoms")
    for k, gi in enumerate(cg):
        g = geoms[gi]
        if g["type"] not in (0, 2, 6):
            raise NotImplementedError(f"collidable geom type {g['type']} (only plane/sphere/box)")
        if g["condim"] != 3:
            raise NotImplementedError("only condim=3 contacts (xml:47)")
        m.cgeom_id[k] = gi
        m.cgeom_type[k] = g["type"]
        m.cgeom_bodyid[k] = g["body"]
        m.cgeom_condim[k] = g["condim"]
        m.cgeom_priority[k] = g["priority"]
        m.cgeom_size[k][:] = list(g["size"])
        m.cgeom_pos[k][:] = list(g["pos"])
        m.cgeom_quat[k][:] = list(g["quat"])
        m.cgeom_friction[k][:] = list(g["friction"])
        m.cgeom_solref[k][:] = list(g["solref"])
        m.cgeom_solimp[k][:] = list(g["solimp"])
        m.cgeom_solmix[k] = g["solmix"]
        m.cgeom_margin[k] = g["margin"]
        m.cgeom_gap[k] = g["gap"]
    m.ncgeom = len(cg)
    pairs = []
    for a in range(len(cg)):
        for b in range(a + 1, len(cg)):
            ga, gb = geoms[cg[a]], geoms[cg[b]]
            ba, bb = ga["body"], gb["body"]
            if ba == bb:
                continue
            if not ((ga["contype"] & gb["conaffinity"]) or (gb["contype"] & ga["conaffinity"])):
                continue
            if ba == 0 and bb == 0:
                continue  # both static
            # filterparent: parent-child bodies do not collide unless the parent is the world
            if (bodies[ba].parent == bb and bb != 0) or (bodies[bb].parent == ba and ba != 0):
                continue
            i1, i2 = (a, b) if ga["type"] <= gb["type"] else (b, a)
            pairs.append((i1, i2))
    # grouped by geom-type pair (plane-sphere, sphere-sphere, sphere-box), geom order within a
    # group: the robot's own 32 candidates come first whatever boxes follow, so the kernel's first
    # (prefetched) 32-pair batch is the same with and without obstacles and the box pairs after it
    # are culled by box (pp3_env.hip collision()).  The order only decides the contacts' (and their
    # constraint rows') order -- rounding, and ties of the contact cap; the oracle follows it too.
    pairs.sort(key=lambda ab: (geoms[cg[ab[0]]]["type"], geoms[cg[ab[1]]]["type"]))
    if len(pairs) > _abi.MAX_PAIR:
        raise ValueError("too many collision pairs")
    m.npair = len(pairs)
    for k, (a, b) in enumerate(pairs):
        m.pair_g1[k] = a
        m.pair_g2[k] = b

    # ---------------- sites ----------------
    if len(sites) > _abi.MAX_SITE:
        raise ValueError("too many sites")
    m.nsite = len(sites)
    for k, s in enumerate(sites):
        m.site_bodyid[k] = s["body"]
        m.site_pos[k][:] = list(s["pos"])
        m.site_quat[k][:] = list(s["quat"])

    # ---------------- actuators ----------------
    act_nodes = []
    act = root.find("actuator")
    if act is not None:
        for a in act:
            if a.tag != "general":
                raise NotImplementedError(f"actuator <{a.tag}>")
            act_nodes.append(a)
    if len(act_nodes) != _abi.NU:
        raise ValueError("expected 12 actuators")
    jnames = [j["name"] for j in joints]
    act_names = []
    for k, node in enumerate(act_nodes):
        explicit = defaults.resolve("general", node.get("class", "main"), {})
        explicit.update(node.attrib)
        a = dict(_ACT_DEFAULTS)
        a.update(explicit)
        act_names.append(a.get("name", ""))
        if a.get("dyntype", "none") != "none" or a.get("gaintype", "fixed") != "fixed":
            raise NotImplementedError("only fixed-gain, no-dynamics actuators")
        jid = jnames.index(a["joint"])
        m.actuator_trnid[k] = jid
        bt = a["biastype"]
        m.actuator_biastype[k] = 1 if bt == "affine" else 0
        fl = a["forcelimited"]
        fr = _vec(a["forcerange"], 2)
        m.actuator_forcelimited[k] = 1 if fl == "true" else 0 if fl == "false" else int(autolimits and "forcerange" in explicit)
        cl = a["ctrllimited"]
        cr = _vec(a["ctrlrange"], 2)
        m.actuator_ctrllimited[k] = 1 if cl == "true" else 0 if cl == "false" else int(autolimits and "ctrlrange" in explicit)
        m.actuator_gear[k] = _vec(a["gear"])[0]
        m.actuator_gainprm[k][:] = list(_vec(a["gainprm"], 3)[:3])
        m.actuator_biasprm[k][:] = list(_vec(a["biasprm"], 3)[:3])
        m.actuator_forcerange[k][:] = list(fr)
        m.actuator_ctrlrange[k][:] = list(cr)

    # ---------------- custom numerics ----------------
    m.max_contact_points = -1
    m.max_geom_pairs = -1
    custom = root.find("custom")
    if custom is not None:
        for n in custom.findall("numeric"):
            if n.get("name") == "max_contact_points":
                m.max_contact_points = int(float(n.get("data")))
            elif n.get("name") == "max_geom_pairs":
                m.max_geom_pairs = int(float(n.get("data")))

    # ---------------- sensors (site-attached types; mjData.sensordata layout) ----------------
    sens_types = {"accelerometer": (_abi.SENS_ACCELEROMETER, 3), "velocimeter": (_abi.SENS_VELOCIMETER, 3),
                  "gyro": (_abi.SENS_GYRO, 3), "framepos": (_abi.SENS_FRAMEPOS, 3),
                  "framequat": (_abi.SENS_FRAMEQUAT, 4), "framelinvel": (_abi.SENS_FRAMELINVEL, 3),
                  "frameangvel": (_abi.SENS_FRAMEANGVEL, 3)}
    site_names = [s["name"] for s in sites]
    m.nsensor = 0
    m.nsensordata = 0
    sensor_names = []
    for sec in root.findall("sensor"):
        for e in sec:
            if e.tag not in sens_types:
                raise NotImplementedError(f"sensor <{e.tag}>")
            if e.tag.startswith("frame"):
                if e.get("objtype") != "site" or e.get("reftype") or e.get("refname"):
                    raise NotImplementedError(f"<{e.tag}>: only objtype=\"site\" without a reference frame")
                site = e.get("objname")
            else:
                site = e.get("site")
            if site not in site_names:
                raise ValueError(f"sensor <{e.tag}>: unknown site {site!r}")
            typ, dim = sens_types[e.tag]
            k = m.nsensor
            if k >= _abi.MAX_SENSOR or m.nsensordata + dim > _abi.MAX_SENSORDATA:
                raise ValueError("too many sensors")
            m.sensor_type[k] = typ
            m.sensor_objid[k] = site_names.index(site)
            m.sensor_adr[k] = m.nsensordata
            m.sensor_dim[k] = dim
            m.sensor_cutoff[k] = float(e.get("cutoff", "0"))
            m.nsensor += 1
            m.nsensordata += dim
            sensor_names.append(e.get("name", f"sensor{k}"))

    # ---------------- set0: invweight0, meaninertia ----------------
    _set_const(m)

    body_geomadr = np.array([b.geoms[0] if b.geoms else -1 for b in bodies])
    body_geomnum = np.array([len(b.geoms) for b in bodies])
    visual = _visual(root, geoms, [b.name for b in bodies], angle_deg)
    return CompiledModel(
        struct=m,
        body_names=[b.name for b in bodies],
        joint_names=jnames,
        geom_names=[g["name"] for g in geoms],
        site_names=[s["name"] for s in sites],
        sensor_names=sensor_names,
        actuator_names=act_names,
        body_geomadr=body_geomadr,
        body_geomnum=body_geomnum,
        geom_bodyid=np.array([g["body"] for g in geoms]),
        geom_type=np.array([g["type"] for g in geoms]),
        geom_friction=np.array([g["friction"] for g in geoms]),
        jnt_range=np.array([joints[j]["range"] for j in range(len(joints))]),
        xml=xml,
        visual=visual,
    )


def _visual(root: ET.Element, geoms: List[dict], body_names: List[str], angle_deg: bool) -> Dict:
    """What render.py needs: every geom's shape/pose/group/colour, the mesh assets (file, scale),
    materials and textures (rgba / builtin checker and gradient colours), the cameras."""
    compiler = root.find("compiler")
    vis: Dict = {"meshdir": compiler.get("meshdir", "") if compiler is not None else "",
                 "meshes": {}, "materials": {}, "textures": {}, "cameras": {}, "skybox": None}
    for asset in root.findall("asset"):
        for m in asset.findall("mesh"):
            name = m.get("name") or os.path.splitext(os.path.basename(m.get("file", "")))[0]
            vis["meshes"][name] = dict(file=m.get("file"), scale=_vec(m.get("scale", "1 1 1"), 3))
        for t in asset.findall("texture"):
            tex = dict(type=t.get("type", "cube"), builtin=t.get("builtin", "none"),
                       rgb1=_vec(t.get("rgb1", "0.8 0.8 0.8"), 3), rgb2=_vec(t.get("rgb2", "0.5 0.5 0.5"), 3))
            if tex["type"] == "skybox":
                vis["skybox"] = tex
            if t.get("name"):
                vis["textures"][t.get("name")] = tex
        for mt in asset.findall("material"):
            vis["materials"][mt.get("name")] = dict(
                rgba=_vec(mt.get("rgba", "1 1 1 1"), 4), texture=mt.get("texture"),
                texrepeat=_vec(mt.get("texrepeat", "1 1"), 2), texuniform=mt.get("texuniform", "false") == "true")
    vis["geoms"] = [dict(type=g["type"], size=g["size"], pos=g["pos"], quat=g["quat"], body=g["body"],
                         group=g["group"], mesh=g["mesh"], material=g["material"], rgba=g["rgba"], name=g["name"])
                    for g in geoms]
    wb = root.find("worldbody")
    parent_of = {child: parent for parent in wb.iter() for child in parent}
    for c in wb.iter("camera"):
        par = parent_of.get(c, wb)
        parent = 0 if par is wb else (body_names.index(par.get("name")) if par.get("name") in body_names else -1)
        if parent < 0:
            raise NotImplementedError("camera inside an unnamed body")
        vis["cameras"][c.get("name", f"camera{len(vis['cameras'])}")] = dict(
            mode=c.get("mode", "fixed"), target=body_names.index(c.get("target")) if c.get("target") in body_names else -1,
            pos=_vec(c.get("pos", "0 0 0"), 3), quat=_orientation(c.attrib, angle_deg),
            fovy=float(c.get("fovy", "45")), parent=parent)
    return vis


# ----------------------------------------------------------------------------------
# mj_setConst restatement (float64): kinematics + mass matrix + body Jacobians at qpos0
# ----------------------------------------------------------------------------------
def _kinematics(m, qpos: np.ndarray):
    nb = _abi.NBODY
    xpos = np.zeros((nb, 3))
    xquat = np.zeros((nb, 4))
    xquat[0] = [1, 0, 0, 0]
    xanchor = np.zeros((_abi.NJNT, 3))
    xaxis = np.zeros((_abi.NJNT, 3))
    for b in range(1, nb):
        p = m.body_parentid[b]
        j = m.body_jntadr[b]
        if m.jnt_type[j] == JNT_FREE:
            a = m.jnt_qposadr[j]
            xpos[b] = qpos[a:a + 3]
            xquat[b] = quat_normalize(qpos[a + 3:a + 7])
            xanchor[j] = xpos[b]
            xaxis[j] = np.array(m.jnt_axis[j][:])
            continue
        Rp = quat_to_mat(xquat[p])
        xpos[b] = xpos[p] + Rp @ np.array(m.body_pos[b][:])
        q = quat_mul(xquat[p], np.array(m.body_quat[b][:]))
        R = quat_to_mat(q)
        jp_ = np.array(m.jnt_pos[j][:])
        ax = np.array(m.jnt_axis[j][:])
        xaxis[j] = R @ ax
        xanchor[j] = R @ jp_ + xpos[b]
        q = quat_mul(q, axis_angle_quat(ax, qpos[m.jnt_qposadr[j]] - m.qpos0[m.jnt_qposadr[j]]))
        q = quat_normalize(q)
        xpos[b] = xanchor[j] - quat_to_mat(q) @ jp_
        xquat[b] = q
    return xpos, xquat, xanchor, xaxis


def mass_matrix_and_jacobians(m, qpos: np.ndarray):
    """Return (M, jacp[nb,3,nv], jacr[nb,3,nv], xipos) at qpos (world-frame Jacobians at body coms)."""
    nb, nv = _abi.NBODY, _abi.NV
    xpos, xquat, xanchor, xaxis = _kinematics(m, qpos)
    xipos = np.zeros((nb, 3))
    jacp = np.zeros((nb, 3, nv))
    jacr = np.zeros((nb, 3, nv))
    M = np.zeros((nv, nv))
    for b in range(1, nb):
        R = quat_to_mat(xquat[b])
        xipos[b] = xpos[b] + R @ np.array(m.body_ipos[b][:])
    for b in range(1, nb):
        # walk up the chain collecting dofs
        c = b
        while c > 0:
            j = m.body_jntadr[c]
            d0 = m.jnt_dofadr[j]
            if m.jnt_type[j] == JNT_FREE:
                Rb = quat_to_mat(xquat[c])
                for k in range(3):
                    jacp[b, k, d0 + k] = 1.0
                for k in range(3):
                    ax = Rb[:, k]
                    jacr[b, :, d0 + 3 + k] = ax
                    jacp[b, :, d0 + 3 + k] = np.cross(ax, xipos[b] - xanchor[j])
            else:
                ax = xaxis[j]
                jacr[b, :, d0] = ax
                jacp[b, :, d0] = np.cross(ax, xipos[b] - xanchor[j])
            c = m.body_parentid[c]
        R = quat_to_mat(quat_mul(xquat[b], np.array(m.body_iquat[b][:])))
        Iw = R @ np.diag(np.array(m.body_inertia[b][:])) @ R.T
        M += m.body_mass[b] * jacp[b].T @ jacp[b] + jacr[b].T @ Iw @ jacr[b]
    M += np.diag(np.array(m.dof_armature[:]))
    return M, jacp, jacr, xipos


def _set_const(m) -> None:
    q0 = np.array(m.qpos0[:])
    M, jacp, jacr, _ = mass_matrix_and_jacobians(m, q0)
    Minv = np.linalg.inv(M)
    dinv = np.diag(Minv).copy()
    for j in range(_abi.NJNT):
        d0 = m.jnt_dofadr[j]
        if m.jnt_type[j] == JNT_FREE:
            dinv[d0:d0 + 3] = dinv[d0:d0 + 3].mean()
            dinv[d0 + 3:d0 + 6] = dinv[d0 + 3:d0 + 6].mean()
    m.dof_invweight0[:] = list(dinv)
    m.body_invweight0[0][:] = [0.0, 0.0]
    for b in range(1, _abi.NBODY):
        J = np.concatenate([jacp[b], jacr[b]], axis=0)
        A = J @ Minv @ J.T
        m.body_invweight0[b][:] = [np.trace(A[:3, :3]) / 3.0, np.trace(A[3:, 3:]) / 3.0]
    m.meaninertia = float(np.trace(M) / _abi.NV)


def recompute_constants(cm: CompiledModel) -> None:
    """Re-run set0 after editing the model struct (e.g. tests that change masses)."""
    _set_const(cm.struct)
