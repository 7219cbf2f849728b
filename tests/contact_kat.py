"""Known answers for the two contact-model pieces the kernel and the oracle still shared after
round 3: solref/solimp MIXING of a pair's parameters and the pyramid's TANGENT BASIS for contact
normals off the vertical (test_contact_kat.py on the oracle, test_gpu_contact_kat.py on the
kernel).  Everything here is written from MuJoCo's documentation and the MJCF literals, not from
either restatement and not from pupperv3_mjx/mjcf.py:

* parameters (MuJoCo XML reference, <geom>): the defaults solref "0.02 1", solimp
  "0.9 0.95 0.001 0.5 2", solmix "1", friction "1 0.005 0.0001", priority 0; the model's collision
  class (/root/reference/test/test_pupper_model.xml:50-52) sets solimp="0.015 1 0.031" (midpoint and
  power keep their defaults) and friction="0.8 0.02 0.01"; the floor (xml:219) and the obstacle
  boxes (obstacles.py:44-52) set none;
* mixing (Computation / Contact parameters, mj_contactParam): equal priorities -> mix = s1/(s1+s2)
  (0.5 if both solmix are ~0, 0 or 1 if one is); solref = mix r1 + (1-mix) r2 when both time
  constants are positive (standard form), else the element-wise minimum; solimp = mix i1 + (1-mix)
  i2; friction = the element-wise max.  Higher priority: that geom's parameters alone;
* the soft constraint (Computation / Solver parameters): impedance d(r) from solimp (dmin, dmax
  clamped to [1e-4, 0.9999]), R = (1-d)/d * A, reference acceleration aref = -b J v - k d r with
  b = 2/(dmax tc), k = 1/(dmax^2 tc^2 dr^2), tc >= 2 timestep; pyramidal rows J_n +- mu J_t_i with
  A = (tran + mu^2 tran) 2 mu^2 / impratio and tran = the two bodies' body_invweight0;
* the contact frame (mju_makeFrame): t1 = normalize(y - (y.n) n) with y = (0,1,0) when
  -0.5 < n_y < 0.5 and (0,0,1) otherwise; t2 = n x t1;
* MuJoCo's primal problem: qacc minimises 1/2 (a - a0)' M (a - a0) + sum_active 1/2 D (J a - aref)^2,
  D = 1/R, a row active where J a - aref < 0 (a convex piecewise quadratic: the minimiser is found
  by enumerating the rows' active sets).  With Newton iterated to convergence the implementations'
  qacc must equal it.
"""
import itertools

import numpy as np

import test_physics_kat as K

# ------------------------------------------------------------------ documented parameters
GEOM_DEFAULT = dict(solref=(0.02, 1.0), solimp=(0.9, 0.95, 0.001, 0.5, 2.0), solmix=1.0,
                    friction=(1.0, 0.005, 0.0001), priority=0)
COLLISION_CLASS = dict(GEOM_DEFAULT, solimp=(0.015, 1.0, 0.031, 0.5, 2.0), friction=(0.8, 0.02, 0.01))
FLOOR = GEOM_DEFAULT
MINVAL = 1e-15


def mix_params(p1, p2):
    """A contact's (solref, solimp, mu) from its two geoms' parameters (module docstring)."""
    if p1["priority"] != p2["priority"]:
        g = p1 if p1["priority"] > p2["priority"] else p2
        return dict(solref=np.array(g["solref"], float), solimp=np.array(g["solimp"], float), mu=g["friction"][0])
    s1, s2 = p1["solmix"], p2["solmix"]
    if s1 >= MINVAL and s2 >= MINVAL:
        mix = s1 / (s1 + s2)
    elif s1 < MINVAL and s2 < MINVAL:
        mix = 0.5
    else:
        mix = 0.0 if s1 < MINVAL else 1.0
    r1, r2 = np.array(p1["solref"], float), np.array(p2["solref"], float)
    solref = mix * r1 + (1 - mix) * r2 if (r1[0] > 0 and r2[0] > 0) else np.minimum(r1, r2)
    solimp = mix * np.array(p1["solimp"], float) + (1 - mix) * np.array(p2["solimp"], float)
    return dict(solref=solref, solimp=solimp, mu=max(p1["friction"][0], p2["friction"][0]), mix=mix)


def unmixed(p):
    """One geom's parameters taken alone (what an implementation that skipped the mixing would use)."""
    return dict(solref=np.array(p["solref"], float), solimp=np.array(p["solimp"], float), mu=p["friction"][0])


def impedance(solimp, r):
    si = np.array(solimp, float)
    si[0] = min(max(si[0], 1e-4), 0.9999)
    si[1] = min(max(si[1], 1e-4), 0.9999)
    return K._imp(si, r)


def kb(pair, timestep):
    solref, solimp = pair["solref"], pair["solimp"]
    dmax = min(max(solimp[1], 1e-4), 0.9999)
    tc, dr = max(solref[0], 2 * timestep), solref[1]
    return 1.0 / (dmax * dmax * tc * tc * dr * dr), 2.0 / (dmax * tc)


def make_frame(n):
    """mju_makeFrame of a contact normal: rows n, t1, t2."""
    n = np.asarray(n, float) / np.linalg.norm(n)
    y = np.array([0.0, 1.0, 0.0]) if -0.5 < n[1] < 0.5 else np.array([0.0, 0.0, 1.0])
    t1 = y - (y @ n) * n
    t1 /= np.linalg.norm(t1)
    return np.array([n, t1, np.cross(n, t1)])


def rotated_frame(frame, ang):
    """The same normal with the tangent pair turned by `ang` about it (a wrong basis)."""
    n, t1, t2 = frame
    c, s = np.cos(ang), np.sin(ang)
    u1 = c * t1 + s * t2
    return np.array([n, u1, np.cross(n, u1)])


def edge_rows(frame, J3, mu):
    """The four pyramid edges J_n +- mu J_t1, J_n +- mu J_t2 of one contact (J3: 3 x nv Jacobian of
    the relative velocity of body 2's contact point w.r.t. body 1's, world frame)."""
    Jn, Jt1, Jt2 = frame @ J3
    return np.array([Jn + mu * Jt1, Jn - mu * Jt1, Jn + mu * Jt2, Jn - mu * Jt2])


def contact_terms(rows, qvel, dist, pair, tran, impratio, timestep):
    """(D, aref) of a contact's edge rows."""
    mu = pair["mu"]
    d = impedance(pair["solimp"], dist)
    A = (tran + mu * mu * tran) * 2 * mu * mu / impratio
    D = 1.0 / max(MINVAL, (1 - d) / d * A)
    k, b = kb(pair, timestep)
    return np.full(len(rows), D), -b * (rows @ qvel) - k * d * dist


def minimise(M, a0, rows, D, aref):
    """Exact minimiser of the Gauss + soft-constraint cost (module docstring).  Returns (qacc, active)."""
    nr = len(rows)
    for act in itertools.product([0, 1], repeat=nr):
        Da = D * np.array(act, float)
        H = M + rows.T @ (Da[:, None] * rows)
        a = np.linalg.solve(H, M @ a0 + rows.T @ (Da * aref))
        x = rows @ a - aref
        if all((x[i] < 0) == bool(act[i]) or abs(x[i]) < 1e-9 * (1 + abs(aref[i])) for i in range(nr)):
            return a, act
    raise AssertionError("no consistent active set (the cost is convex: one must exist)")


# ------------------------------------------------------------------ a ball on a floor (mixing)
def ball_problem(qpos, qvel, pair, mass, radius, gravity, impratio, timestep, frame_fn=make_frame):
    """The solid ball's (6 free dofs) contact problem on the plane z = 0 with the pair parameters
    `pair`: tran = 1/m (a lone free body's body_invweight0, test_physics_kat pins it)."""
    R = K._qmat(qpos[3:7])
    inertia = 0.4 * mass * radius ** 2
    M = np.diag([mass] * 3 + [inertia] * 3)
    a0 = np.concatenate([np.asarray(gravity, float), np.zeros(3)])
    dist = qpos[2] - radius
    if dist > 0:
        return dict(M=M, a0=a0, rows=None, dist=dist)
    n = np.array([0.0, 0.0, 1.0])                     # plane normal, from the plane (geom1) to the ball
    pos = qpos[0:3] - (radius + 0.5 * dist) * n
    rc = pos - qpos[0:3]
    rx = np.array([[0, -rc[2], rc[1]], [rc[2], 0, -rc[0]], [-rc[1], rc[0], 0]])
    J3 = np.hstack([np.eye(3), -rx @ R])              # ball point velocity (the plane is static)
    rows = edge_rows(frame_fn(n), J3, pair["mu"])
    D, aref = contact_terms(rows, qvel[0:6], dist, pair, 1.0 / mass, impratio, timestep)
    return dict(M=M, a0=a0, rows=rows, D=D, aref=aref, dist=dist)


def ball_qacc(qpos, qvel, pair, mass, radius, gravity, impratio, timestep, frame_fn=make_frame):
    P = ball_problem(qpos, qvel, pair, mass, radius, gravity, impratio, timestep, frame_fn)
    if P["rows"] is None:
        return P["a0"], P
    a, act = minimise(P["M"], P["a0"], P["rows"], P["D"], P["aref"])
    P["active"] = act
    return a, P


def rest_penetration(pair, mass, g_normal, radius, impratio, timestep):
    """Depth r < 0 at which a ball at rest (a = v = 0) on a plane carries m g_n: every edge row is
    active with force D k d(r) (-r), and the four edges' normal parts sum to the load:
    4 k d(r)^2 (-r) / ((1 - d(r)) A) = m g_n.  Solved by bisection (the left side grows with -r)."""
    mu = pair["mu"]
    tran = 1.0 / mass
    A = (tran + mu * mu * tran) * 2 * mu * mu / impratio
    k, _ = kb(pair, timestep)

    def load(r):
        d = impedance(pair["solimp"], r)
        return 4 * k * d * d * (-r) / ((1 - d) * A)

    lo, hi = -1e-9, -1e-9
    while load(hi) < mass * g_normal:
        hi *= 2
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if mid == lo or mid == hi:  # the bracket is one ulp wide: further halvings change nothing
            break
        lo, hi = (mid, hi) if load(mid) < mass * g_normal else (lo, mid)
    return 0.5 * (lo + hi)


def steady_creep(pair, mass, radius, theta, g, impratio, timestep):
    """Steady rolling down a slope of angle theta (gravity tilted, the plane z = 0): the contact
    point's slip velocity s and the depth r at which the documented minimiser gives neither slip
    acceleration nor normal acceleration.  The ball's edge rows see only (s, r) (J_n v = 0 in the
    steady state, the ball has no velocity-product forces), so this is a 2-D root, found by nested
    bisection: the slip acceleration falls with s (more friction), the normal acceleration grows
    with the depth -r (more push).  Returns (s, r)."""
    grav = np.array([g * np.sin(theta), 0.0, -g * np.cos(theta)])

    def accel(s, r):
        q = np.zeros(7)
        q[2], q[3] = radius + r, 1.0
        lever = radius + 0.5 * r
        v = np.zeros(6)
        v[0] = 1.0                                    # any rolling speed: the rows see the slip only
        v[4] = (v[0] - s) / lever                     # slip = v_x - lever w_y
        a, _ = ball_qacc(q, v, pair, mass, radius, grav, impratio, timestep)
        return a[0] - lever * a[4], a[2]

    def bisect(f, lo, hi):
        """Root of a decreasing f, brackets grown from [lo, hi] (lo < hi)."""
        while f(lo) < 0:
            lo -= 2 * (hi - lo)
        while f(hi) > 0:
            hi += 2 * (hi - lo)
        for _ in range(200):
            mid = 0.5 * (lo + hi)
            if mid == lo or mid == hi:  # (one ulp wide: the same result as the full 200 halvings)
                break
            lo, hi = (mid, hi) if f(mid) > 0 else (lo, mid)
        return 0.5 * (lo + hi)

    r0 = abs(rest_penetration(pair, mass, g * np.cos(theta), radius, impratio, timestep))
    slip_at = lambda r: bisect(lambda s: accel(s, r)[0], -r0, r0)  # noqa: E731
    r = bisect(lambda r: accel(slip_at(r), r)[1], -2 * r0, -0.5 * r0)
    return slip_at(r), r


# ------------------------------------------------------------------ a ball on a tilted box face
def ball_box_problem(m, qpos, qvel, box, pair, mass, radius, frame_fn=make_frame):
    """The ball (free body, COM at the origin, mass / radius) pressed into world box `box`
    (geom2; the normal points from the sphere into the box, MuJoCo's sphere-box convention): the
    contact found by the closed-form distance of the ball centre to the box, the rows of the
    documented frame of that normal.  Returns the problem dict."""
    c = qpos[0:3]
    Rb = K._qmat(np.array(m.cgeom_quat[box][:]))
    p = np.array(m.cgeom_pos[box][:])
    h = np.array(m.cgeom_size[box][:])
    loc = Rb.T @ (c - p)
    cl = np.clip(loc, -h, h)
    assert np.any(cl != loc), "ball centre inside the box"
    v = cl - loc
    length = np.linalg.norm(v)
    dist = length - radius
    n = Rb @ (v / length)                              # sphere -> box
    pos = c + n * (radius + 0.5 * dist)
    rc = pos - c
    rx = np.array([[0, -rc[2], rc[1]], [rc[2], 0, -rc[0]], [-rc[1], rc[0], 0]])
    J3 = -np.hstack([np.eye(3), -rx @ K._qmat(qpos[3:7])])   # box (static) minus the ball's point
    frame = frame_fn(n)
    rows = edge_rows(frame, J3, pair["mu"])
    inertia = 0.4 * mass * radius ** 2
    M = np.diag([mass] * 3 + [inertia] * 3)
    a0 = np.concatenate([np.array(m.gravity[:]), np.zeros(3)])
    D, aref = contact_terms(rows, qvel[0:6], dist, pair, 1.0 / mass, m.impratio, m.timestep)
    return dict(M=M, a0=a0, rows=rows, D=D, aref=aref, dist=dist, n=n, frame=frame)


def box_rotation(normal_world, local_dir):
    """A box quaternion that turns the unit local direction `local_dir` onto `normal_world`
    (shortest arc), so the ball can touch that face with a chosen world normal."""
    a = np.asarray(local_dir, float) / np.linalg.norm(local_dir)
    b = np.asarray(normal_world, float) / np.linalg.norm(normal_world)
    axis = np.cross(a, b)
    s, c = np.linalg.norm(axis), a @ b
    if s < 1e-12:
        return np.array([1.0, 0.0, 0.0, 0.0])
    ang = np.arctan2(s, c)
    return np.concatenate([[np.cos(ang / 2)], np.sin(ang / 2) * axis / s])


# ------------------------------------------------------------------ two leg spheres (articulated)
def body_poses(m, q):
    """Body ORIGIN frames (xpos, xquat) of the tree written from the MJCF alone (the same recursion
    as test_physics_kat.body_frames, which returns COM frames)."""
    from pupperv3_mjx import _abi, mjcf
    nb = _abi.NBODY
    xpos, xquat = np.zeros((nb, 3)), np.zeros((nb, 4))
    xquat[0] = [1, 0, 0, 0]
    for b in range(1, nb):
        j = m.body_jntadr[b]
        if m.jnt_type[j] == mjcf.JNT_FREE:
            xpos[b] = q[0:3]
            xquat[b] = q[3:7] / np.linalg.norm(q[3:7])
        else:
            p = m.body_parentid[b]
            xpos[b] = xpos[p] + K._qmat(xquat[p]) @ np.array(m.body_pos[b][:])
            a = m.jnt_qposadr[j]
            xquat[b] = K._qmul(K._qmul(xquat[p], np.array(m.body_quat[b][:])),
                               K._qaxis(m.jnt_axis[j][:], q[a] - m.qpos0[a]))
    return xpos, xquat


def geom_centre(m, q, g, poses=None):
    xpos, xquat = poses if poses is not None else body_poses(m, q)
    b = int(m.cgeom_bodyid[g])
    return xpos[b] + K._qmat(xquat[b]) @ np.array(m.cgeom_pos[g][:])


def point_jacobian(m, q, b, pos, eps=1e-6):
    """3 x nv Jacobian of the world velocity of the point `pos` carried by body b (central
    differences of the independent kinematics along MuJoCo's velocity coordinates)."""
    from pupperv3_mjx import _abi
    xpos, xquat = body_poses(m, q)
    loc = K._qmat(xquat[b]).T @ (pos - xpos[b])
    J = np.zeros((3, _abi.NV))
    for i in range(_abi.NV):
        out = []
        for s in (eps, -eps):
            xp, xq = body_poses(m, K._perturb(q, i, s))
            out.append(xp[b] + K._qmat(xq[b]) @ loc)
        J[:, i] = (out[0] - out[1]) / (2 * eps)
    return J


def sphere_pair_problem(m, q, qvel, pair_index, pair, invweight, frame_fn=make_frame):
    """The articulated contact problem of sphere-sphere pair `pair_index` (MuJoCo: normal from
    geom1's centre to geom2's, dist = |c2 - c1| - r1 - r2, position the midpoint between the
    surfaces, J = J_body2(pos) - J_body1(pos)) with no other force than the joint damping: M from
    the kinetic energy (test_physics_kat.energy_mass_matrix), a0 = M^-1 (-damping qvel), tran the
    two bodies' body_invweight0 from that M (`invweight`).  Velocity-product forces are left out:
    the caller makes every moving body negligible (1e-9 kg), so the joints' armature carries the
    inertia and they are ~1e-9 of the contact forces."""
    g1, g2 = int(m.pair_g1[pair_index]), int(m.pair_g2[pair_index])
    b1, b2 = int(m.cgeom_bodyid[g1]), int(m.cgeom_bodyid[g2])
    poses = body_poses(m, q)
    c1, c2 = geom_centre(m, q, g1, poses), geom_centre(m, q, g2, poses)
    r1, r2 = m.cgeom_size[g1][0], m.cgeom_size[g2][0]
    axis = c2 - c1
    length = np.linalg.norm(axis)
    n = axis / length
    dist = length - r1 - r2
    pos = c1 + n * (r1 + 0.5 * dist)
    J3 = point_jacobian(m, q, b2, pos) - point_jacobian(m, q, b1, pos)
    M, _, _ = K.energy_mass_matrix(m, q)
    a0 = np.linalg.solve(M, -np.array(m.dof_damping[:]) * qvel)
    frame = frame_fn(n)
    rows = edge_rows(frame, J3, pair["mu"])
    tran = invweight[b1, 0] + invweight[b2, 0]
    D, aref = contact_terms(rows, qvel, dist, pair, tran, m.impratio, m.timestep)
    return dict(M=M, a0=a0, rows=rows, D=D, aref=aref, dist=dist, n=n, frame=frame, J3=J3, b=(b1, b2))


# ------------------------------------------------------------------ the test set-ups
BALL_R, BALL_M = 0.05, 1.0
# world outward normal u of the box region the ball touches, and that region's local direction
# (face centre / edge / corner of the box, collision_geometry.REGIONS); the contact normal (sphere ->
# box) is -u: n_y inside (-0.5, 0.5) takes t1 from y, outside from z (mju_makeFrame's two branches)
BOX_CASES = {"face_ty": ((0.3, 0.35, 0.89), (0, 0, 1)), "face_tz": ((0.45, -0.8, 0.4), (1, 0, 0)),
             "edge": ((-0.6, 0.3, 0.74), (1, 0, 1)), "corner": ((-0.5, 0.45, 0.74), (1, 1, 1))}
SLIDE_ANGLE = np.radians(25.0)   # sliding direction measured from the documented t1
SLIDE_SPEED = 0.4


def tilted_box_case(path, case, pen=1e-3, iterations=50):
    """The robot turned into a solid ball (legs 1e-9 kg) touching the first box geom of the model at
    `path` in the region of BOX_CASES[case], the box turned so that region's outward normal is the
    case's world direction u, gravity -g u pressing the ball in, the ball sliding at SLIDE_SPEED in
    the contact plane at SLIDE_ANGLE from the documented t1.  The ball geom and the box keep their
    compiled contact parameters (the collision class against the box's defaults: a mixed pair).
    Returns (model struct, qpos, qvel, box cgeom index)."""
    from pupperv3_mjx import _abi, mjcf
    u, d = (np.asarray(x, float) for x in BOX_CASES[case])
    u /= np.linalg.norm(u)
    cm = mjcf.load(path)
    m = cm.struct
    m.timestep = 0.004
    m.iterations = iterations
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
    bq = box_rotation(u, d)
    m.cgeom_quat[box][:] = list(bq)
    h = np.array(m.cgeom_size[box][:])
    centre = np.array(m.cgeom_pos[box][:]) + K._qmat(bq) @ (h * d + d / np.linalg.norm(d) * (BALL_R - pen))
    m.gravity[:] = list(-9.81 * u)
    mjcf.recompute_constants(cm)
    q = np.zeros(19)
    q[0:3], q[3] = centre, 1.0
    q[7:] = K.DP
    frame = make_frame(-u)
    v = np.zeros(18)
    v[0:3] = SLIDE_SPEED * (np.cos(SLIDE_ANGLE) * frame[1] + np.sin(SLIDE_ANGLE) * frame[2])
    return m, q, v, box


def box_known_answer(m, q, v, box, frame_fn=make_frame):
    pair = mix_params(COLLISION_CLASS, GEOM_DEFAULT)
    P = ball_box_problem(m, q, v, box, pair, BALL_M, BALL_R, frame_fn)
    a, act = minimise(P["M"], P["a0"], P["rows"], P["D"], P["aref"])
    return a, act, P


def leg_pair_model():
    """Base pinned (1e9 kg), legs negligible (1e-9 kg: the joints' armature carries the inertia, so
    velocity-product forces vanish), gravity off, actuators off, frictionloss 1e-9 N m (the kernel
    requires it positive; its force is bounded by it), Newton to convergence.  Returns (model
    struct, independent body_invweight0 [nbody, 2] from the kinetic-energy M at qpos0)."""
    cm = __import__("common").pd_model()
    m = cm.struct
    m.gravity[:] = [0.0, 0.0, 0.0]
    m.body_mass[1] = 1e9
    for k in range(3):
        m.body_inertia[1][k] = 1e9
    for i in range(12):
        m.actuator_gainprm[i][0] = 0.0
        m.actuator_biasprm[i][:] = [0.0, 0.0, 0.0]
    for i in range(6, 18):
        m.dof_frictionloss[i] = 1e-9
    m.iterations = 50
    m = K._negligible_legs(cm)
    M0, Jp0, Jr0 = K.energy_mass_matrix(m, np.array(m.qpos0[:]))
    return m, K._invweight_from(M0, Jp0, Jr0, m)[1]


def leg_pair_state(m, invweight, branch, seed=0):
    """A pose (joint angles uniform in their ranges, base at z = 0.5) in which exactly one
    sphere-sphere pair of two legs penetrates (0.5 to 5 mm, every other pair 2 mm clear), its
    normal off every axis (|n_k| > 0.2) with n_y in the makeFrame branch asked for ("ty": |n_y| <
    0.5, "tz": |n_y| >= 0.5); the two legs' joints spinning at random with the normal relative
    velocity removed, so the contact slides.  Found by rejection sampling on the independent
    kinematics.  Returns (qpos, qvel, pair index)."""
    from pupperv3_mjx import _abi
    rs = np.random.RandomState(seed)
    jr = np.array(m.jnt_range[:])
    pairs = [(int(m.pair_g1[p]), int(m.pair_g2[p])) for p in range(m.npair)]
    ss = [p for p, (a, b) in enumerate(pairs)
          if m.cgeom_type[a] == _abi.GEOM_SPHERE and m.cgeom_type[b] == _abi.GEOM_SPHERE]
    for _ in range(100000):
        q = np.zeros(19)
        q[2], q[3] = 0.5, 1.0
        q[7:] = rs.uniform(jr[1:, 0], jr[1:, 1])
        poses = body_poses(m, q)
        hit = []
        for p in ss:
            g1, g2 = pairs[p]
            c = geom_centre(m, q, g2, poses) - geom_centre(m, q, g1, poses)
            dist = np.linalg.norm(c) - m.cgeom_size[g1][0] - m.cgeom_size[g2][0]
            if dist < 2e-3:
                hit.append((dist, p, c / np.linalg.norm(c)))
        if len(hit) != 1:
            continue
        dist, p, n = hit[0]
        if -5e-3 < dist < -5e-4 and np.abs(n).min() > 0.2 and (abs(n[1]) < 0.5) == (branch == "ty"):
            break
    else:
        raise AssertionError("no pose found")
    P = sphere_pair_problem(m, q, np.zeros(18), p, mix_params(COLLISION_CLASS, COLLISION_CLASS), invweight)
    v = np.zeros(18)
    for b in P["b"]:
        leg = (b - 2) // 3
        v[6 + 3 * leg:9 + 3 * leg] = rs.normal(scale=2.0, size=3)
    Jn = P["n"] @ P["J3"]
    v -= Jn * (Jn @ v) / (Jn @ Jn)
    return q, v, p


def leg_pair_known_answer(m, q, v, p, invweight, frame_fn=make_frame):
    pair = mix_params(COLLISION_CLASS, COLLISION_CLASS)
    P = sphere_pair_problem(m, q, v, p, pair, invweight, frame_fn)
    a, act = minimise(P["M"], P["a0"], P["rows"], P["D"], P["aref"])
    return a, act, P
