"""Independent closed-form contact geometry for the collision known answers
(test_collision_kat.py on the oracle, test_gpu_collision_kat.py on the kernel).

Both the oracle (oracle/pp3_oracle.c `collision` / `sphere_box`) and the kernel compute contact
distances with their own narrow phase; a mistake shared by the two would be invisible to parity.
This module recomputes every candidate pair's signed distance from the geom poses alone, written
from MuJoCo's documented collision semantics (mjCOLLISION: dist < 0 is penetration):

* plane-sphere: the sphere centre's height along the plane normal minus the radius;
* sphere-sphere: centre distance minus both radii;
* sphere-box: the distance from the sphere centre to the box (clamped point in the box frame)
  minus the radius, or, with the centre inside the box, minus the depth to the nearest face
  minus the radius.

Geom poses come from the body poses in the Brax pipeline record (x.pos / x.rot of bodies 1..13,
the frames the step's collision ran on) composed with the model's body-frame geom pos / quat."""
import numpy as np

from pupperv3_mjx import _abi, mjcf


def geom_pose(m, pipe, g):
    """World centre and rotation of collidable geom g (cgeom index) from a pipeline record."""
    b = int(m.cgeom_bodyid[g])
    if b == 0:
        x0, R = np.zeros(3), np.eye(3)
    else:
        x0 = pipe[_abi.P_XPOS + 3 * (b - 1):_abi.P_XPOS + 3 * b]
        R = mjcf.quat_to_mat(np.asarray(pipe[_abi.P_XQUAT + 4 * (b - 1):_abi.P_XQUAT + 4 * b], float))
    return x0 + R @ np.array(m.cgeom_pos[g][:]), R @ mjcf.quat_to_mat(np.array(m.cgeom_quat[g][:]))


def pair_distance(m, pipe, g1, g2):
    """Signed distance of the candidate pair (g1, g2) (cgeom indices, type(g1) <= type(g2))."""
    t1, t2 = int(m.cgeom_type[g1]), int(m.cgeom_type[g2])
    c1, R1 = geom_pose(m, pipe, g1)
    c2, R2 = geom_pose(m, pipe, g2)
    if t1 == _abi.GEOM_PLANE and t2 == _abi.GEOM_SPHERE:
        return float((c2 - c1) @ R1[:, 2] - m.cgeom_size[g2][0])
    if t1 == _abi.GEOM_SPHERE and t2 == _abi.GEOM_SPHERE:
        return float(np.linalg.norm(c2 - c1) - m.cgeom_size[g1][0] - m.cgeom_size[g2][0])
    if t1 == _abi.GEOM_SPHERE and t2 == _abi.GEOM_BOX:
        h = np.array(m.cgeom_size[g2][:])
        local = R2.T @ (c1 - c2)
        outside = np.maximum(np.abs(local) - h, 0.0)
        d = np.linalg.norm(outside) if outside.any() else -np.min(h - np.abs(local))
        return float(d - m.cgeom_size[g1][0])
    raise ValueError(f"pair type ({t1}, {t2}) not in the model's collider table")


def margin(m, g1, g2):
    return max(m.cgeom_margin[g1], m.cgeom_margin[g2])


def check_record(m, pipe, cap, tol):
    """Every contact's distance equals the closed form, and the contact set is exactly the
    candidate pairs within the margin (the `cap` deepest, ties by pair order, when more hit).
    Returns (number of contacts, number of sphere-box contacts, worst distance error)."""
    gid2cg = {int(m.cgeom_id[g]): g for g in range(m.ncgeom)}
    pairs = [(int(m.pair_g1[p]), int(m.pair_g2[p])) for p in range(m.npair)]
    d_all = np.array([pair_distance(m, pipe, a, b) for a, b in pairs])
    hits = [p for p, (a, b) in enumerate(pairs) if d_all[p] <= margin(m, a, b)]
    n = int(pipe[_abi.P_NCON])
    geo = pipe[_abi.P_CON_GEOM:_abi.P_CON_GEOM + 2 * n].reshape(n, 2).astype(int)
    dist = pipe[_abi.P_CON_DIST:_abi.P_CON_DIST + n]
    got = [pairs.index((gid2cg[a], gid2cg[b])) for a, b in geo]
    # a hit within tol of the margin may go either way in fp32: compare the sets away from it
    sure = [p for p in hits if d_all[p] <= margin(m, *pairs[p]) - tol]
    maybe = set(hits) | {p for p, (a, b) in enumerate(pairs) if abs(d_all[p] - margin(m, a, b)) <= tol}
    assert int(pipe[_abi.P_NHIT]) >= len(sure)
    if len(hits) <= cap:
        assert set(sure) <= set(got) <= maybe, (sorted(sure), sorted(got))
    else:  # capped: the kept contacts are the deepest
        assert n == cap and set(got) <= maybe
        worst_kept = max(d_all[p] for p in got)
        dropped = [d_all[p] for p in sure if p not in got]
        assert not dropped or min(dropped) >= worst_kept - tol, (worst_kept, min(dropped))
    err = np.abs(dist - d_all[got]) if n else np.zeros(0)
    assert np.all(err <= tol), (err.max(), tol)
    nbox = sum(1 for p in got if int(m.cgeom_type[pairs[p][1]]) == _abi.GEOM_BOX)
    return n, nbox, float(err.max()) if n else 0.0


# ------------------------------------------------------------------ contact normal known answer
# A solid ball pressed into a box by a gravity vector along the outward normal u of the box region
# it touches (face: the face normal; edge: the bisector; corner: the diagonal), from rest.  The
# contact problem is then symmetric under the reflections t1 -> -t1 and t2 -> -t2 of the contact
# frame (the pyramid edges J_n +- mu J_t swap in pairs, a0 = g has no tangential part, the ball's
# inertia is isotropic), so the exact minimiser and every Newton iterate of it have linear
# acceleration parallel to u and zero angular acceleration, and the contact pushes back (a.u > -g).
# A wrong normal (a face normal in the edge region, a box rotation applied the wrong way) gives a
# tangential or angular component.
BALL_R, BALL_M = 0.05, 1.0
REGIONS = {"face": (1.0, 0.0, 0.0), "edge": (1.0, 0.0, 1.0), "corner": (1.0, 1.0, 1.0)}


def ball_box_model(path, region, pen=1e-3):
    """(model struct, qpos) of the ball touching the first box geom of the model at `path` in
    `region`, penetrating by `pen`; gravity along -u.  Returns (struct, qpos[19], u_world)."""
    import math
    cm = mjcf.load(path)
    m = cm.struct
    m.timestep = 0.004
    for b in range(2, _abi.NBODY):
        m.body_mass[b] = 1e-9
        for k in range(3):
            m.body_inertia[b][k] = 1e-13
    m.body_mass[1] = BALL_M
    m.body_inertia[1][:] = [0.4 * BALL_M * BALL_R ** 2] * 3
    m.body_ipos[1][:] = [0.0, 0.0, 0.0]
    m.body_iquat[1][:] = [1.0, 0.0, 0.0, 0.0]
    box = next(g for g in range(m.ncgeom) if m.cgeom_type[g] == _abi.GEOM_BOX)
    ball = next(g for g in range(m.ncgeom) if m.cgeom_bodyid[g] != 0 and m.cgeom_type[g] == _abi.GEOM_SPHERE)
    m.cgeom_bodyid[ball] = 1
    m.cgeom_pos[ball][:] = [0.0, 0.0, 0.0]
    m.cgeom_size[ball][0] = BALL_R
    m.npair = 1
    m.pair_g1[0], m.pair_g2[0] = ball, box
    h = np.array(m.cgeom_size[box][:])
    d = np.array(REGIONS[region])
    u_loc = d / np.linalg.norm(d)
    closest = h * d  # the face centre line / edge / corner point on the box surface
    Rb = mjcf.quat_to_mat(np.array(m.cgeom_quat[box][:]))
    u = Rb @ u_loc
    centre = np.array(m.cgeom_pos[box][:]) + Rb @ (closest + u_loc * (BALL_R - pen))
    m.gravity[:] = list(-9.81 * u)
    mjcf.recompute_constants(cm)
    q = np.zeros(19)
    q[0:3], q[3] = centre, 1.0
    q[7:] = [0.26, 0.0, -0.52, -0.26, 0.0, 0.52] * 2  # the legs (1e-9 kg) at the default pose
    assert math.isclose(np.linalg.norm(u), 1.0)
    return m, q, u


def normal_residuals(qacc, u):
    """(tangential part of the linear acceleration, |angular acceleration|, a.u) in m/s^2, rad/s^2."""
    a, w = np.asarray(qacc[0:3]), np.asarray(qacc[3:6])
    an = float(a @ u)
    return float(np.linalg.norm(a - an * u)), float(np.linalg.norm(w)), an
