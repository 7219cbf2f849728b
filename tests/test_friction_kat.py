"""Known answers for pyramidal contact friction with impratio (xml:57 cone="pyramidal" impratio="10",
floor friction xml:52), on a body that cannot tip: a solid ball rolling or sliding down a slope.

Every GPU parity test compares the kernel with oracle/pp3_oracle.c, and both build the contact rows
the same way (pyramid edges, their regulariser, the Newton solve), so an error there would be
common-mode.  This file pins that part without either restatement:

* the model: the robot's base becomes a solid ball (mass m, radius r, inertia 2/5 m r^2 about its
  centre, COM at the free joint's origin), the legs are made negligible (1e-9 kg), and one of the
  robot's collision spheres is moved onto the base as the ball's geom; the only collision pair is
  ball-floor.  The slope is a tilted gravity vector g (sin th, 0, -cos th), so the contact frame
  is MuJoCo's mju_makeFrame of the floor normal (z; tangents +y and -x) and the ball slides along
  a pyramid axis;
* the answer for one substep (`ball_qacc`, numpy, written from MuJoCo's documented constraint
  model, not from either implementation): contact point and dist of a sphere on a plane, the
  Jacobian of the contact point in free-joint coordinates (world linear velocity, body angular
  velocity), the four pyramid edges J_n +- mu J_t (efc_pos = dist), impedance d(dist) from solimp,
  R = (1 - d)/d * A, A = (tran + mu^2 tran) 2 mu^2 / impratio with tran = body_invweight0 of the
  ball (1/m), aref = -b J v - k d dist (b = 2/(dmax tc), k = 1/(dmax tc dr)^2), and qacc = the
  exact minimiser of the convex Gauss + soft-constraint cost, found by enumerating the edge rows'
  active sets.  One Newton iteration with its exact line search reaches this minimiser whenever the
  warm start's active set is the final one (steady rolling / sliding), so the oracle's and the
  kernel's qacc must equal it;
* physics limits that hold whatever the regulariser: rolling without slip at (5/7) g sin th when
  mu > (2/7) tan th (contact point at rest to within the soft-constraint creep), sliding when mu is
  below it, with the tangential force never above mu times the normal force (the pyramid's
  Coulomb bound along an axis) and the ball spun up by the friction torque.
"""
import itertools
import math

import numpy as np
import pytest

import common
from oracle import oracle as O
from pupperv3_mjx import _abi, mjcf

G = 9.81
R_BALL, M_BALL = 0.05, 1.0
DP = np.array(common.DEFAULT_POSE)


def ball_model(theta_deg, mu, iterations=None, mixed=False):
    """The Pupper tree turned into a ball on a slope (see module docstring).  `iterations` overrides
    the Newton iteration count (the reference's is 1, xml:57).  mixed=True keeps each geom's own
    compiled contact parameters (the ball's collision class, xml:51, against the floor's defaults,
    xml:219), so the pair runs on the solmix-mixed solref / solimp (tests/test_contact_kat.py);
    `mu` is then ignored."""
    cm = common.pd_model()
    m = cm.struct
    if iterations is not None:
        m.iterations = iterations
    for b in range(2, _abi.NBODY):
        m.body_mass[b] = 1e-9
        for k in range(3):
            m.body_inertia[b][k] = 1e-13
    inertia = 0.4 * M_BALL * R_BALL ** 2
    m.body_mass[1] = M_BALL
    m.body_inertia[1][:] = [inertia] * 3
    m.body_ipos[1][:] = [0.0, 0.0, 0.0]
    m.body_iquat[1][:] = [1.0, 0.0, 0.0, 0.0]
    floor = next(g for g in range(m.ncgeom) if m.cgeom_type[g] == _abi.GEOM_PLANE)
    ball = next(g for g in range(m.ncgeom) if m.cgeom_bodyid[g] != 0)
    m.cgeom_bodyid[ball] = 1
    m.cgeom_pos[ball][:] = [0.0, 0.0, 0.0]
    m.cgeom_size[ball][0] = R_BALL
    if not mixed:
        for g in (floor, ball):
            m.cgeom_friction[g][0] = mu
        m.cgeom_solref[ball][:] = m.cgeom_solref[floor][:]  # pair parameters = the floor's: no mixing
        m.cgeom_solimp[ball][:] = m.cgeom_solimp[floor][:]
        m.cgeom_solmix[ball] = m.cgeom_solmix[floor]
    m.npair = 1
    m.pair_g1[0], m.pair_g2[0] = floor, ball
    th = math.radians(theta_deg)
    m.gravity[:] = [G * math.sin(th), 0.0, -G * math.cos(th)]
    mjcf.recompute_constants(cm)
    return m


def _quat_mat(q):
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _imp(si, x):
    dmin, dmax, width, mid, p = si
    x = min(abs(x) / width, 1.0)
    y = x ** p / mid ** (p - 1) if x <= mid else 1 - (1 - x) ** p / (1 - mid) ** (p - 1)
    return dmin + y * (dmax - dmin)


def ball_problem(m, qpos, qvel):
    """The ball's constraint problem at (qpos, qvel): M, the unconstrained qacc a0, the edge rows J,
    their D = 1/R and aref (module docstring).  rows is None when the ball is off the floor."""
    p, R = qpos[0:3], _quat_mat(qpos[3:7])
    v = qvel[0:6]
    inertia = 0.4 * M_BALL * R_BALL ** 2
    Mb = np.diag([M_BALL] * 3 + [inertia] * 3)
    grav = np.array(m.gravity[:])
    # qfrc_bias = -m g (COM at the origin; w x I w = 0 for a ball); free-joint damping, if any
    qfrc = np.concatenate([M_BALL * grav, np.zeros(3)]) - np.array(m.dof_damping[0:6]) * v
    a0 = np.linalg.solve(Mb, qfrc)
    dist = p[2] - R_BALL
    if dist > 0:
        return dict(M=Mb, a0=a0, rows=None, dist=dist)
    n = np.array([0.0, 0.0, 1.0])
    t1 = np.array([0.0, 1.0, 0.0])           # mju_makeFrame(z): y axis first ...
    t2 = np.cross(n, t1)                     # ... then x = n x t1 = -x
    pos = p - (R_BALL + 0.5 * dist) * n      # mid-point between the surfaces
    rc = pos - p
    rx = np.array([[0, -rc[2], rc[1]], [rc[2], 0, -rc[0]], [-rc[1], rc[0], 0]])
    Jp = np.hstack([np.eye(3), -rx @ R])     # point velocity = v + (R w) x rc
    mu = m.cgeom_friction[0][0] if m.cgeom_type[0] == _abi.GEOM_PLANE else None
    floor = next(g for g in range(m.ncgeom) if m.cgeom_type[g] == _abi.GEOM_PLANE)
    mu = m.cgeom_friction[floor][0]
    solref, solimp = np.array(m.cgeom_solref[floor][:]), np.array(m.cgeom_solimp[floor][:])
    Jn, Jt1, Jt2 = n @ Jp, t1 @ Jp, t2 @ Jp
    rows = np.array([Jn + mu * Jt1, Jn - mu * Jt1, Jn + mu * Jt2, Jn - mu * Jt2])
    d = _imp(solimp, dist)
    tran = 1.0 / M_BALL
    A = (tran + mu * mu * tran) * 2 * mu * mu / m.impratio
    Rr = max(1e-15, (1 - d) / d * A)
    D = 1.0 / Rr
    tc, dr = max(solref[0], 2 * m.timestep), solref[1]
    dmax = solimp[1]
    b, k = 2.0 / (dmax * tc), 1.0 / (dmax * dmax * tc * tc * dr * dr)
    aref = -b * (rows @ v) - k * d * dist
    return dict(M=Mb, a0=a0, rows=rows, D=D, aref=aref, dist=dist, mu=mu)


def cost(P, a):
    """MuJoCo's primal cost: Gauss term + the active rows' quadratic penalty."""
    c = 0.5 * (a - P["a0"]) @ P["M"] @ (a - P["a0"])
    if P["rows"] is not None:
        x = P["rows"] @ a - P["aref"]
        c += 0.5 * P["D"] * np.sum(np.where(x < 0, x * x, 0.0))
    return c


def ball_qacc(m, qpos, qvel):
    """Exact qacc of the ball's 6 free dofs at (qpos, qvel): the minimiser of `cost` (enumerated
    active sets; the cost is convex).  Returns (qacc[6], info)."""
    P = ball_problem(m, qpos, qvel)
    if P["rows"] is None:
        return P["a0"], dict(active=(), dist=P["dist"])
    Mb, a0, rows, D, aref, mu = P["M"], P["a0"], P["rows"], P["D"], P["aref"], P["mu"]
    best = None
    for act in itertools.product([0, 1], repeat=4):
        Da = D * np.array(act, float)
        H = Mb + rows.T @ (Da[:, None] * rows)
        a = np.linalg.solve(H, Mb @ a0 + rows.T @ (Da * aref))
        x = rows @ a - aref
        if all((x[i] < 0) == bool(act[i]) or abs(x[i]) < 1e-9 * (1 + abs(aref[i])) for i in range(4)):
            best = (a, act, x)
            break
    assert best is not None, "no consistent active set (the cost is convex: one must exist)"
    a, act, x = best
    f = -D * np.array(act, float) * x  # edge forces
    fn = f.sum()
    ft = mu * np.array([f[0] - f[1], f[2] - f[3]])  # along t1 (y), t2 (-x)
    return a, dict(active=act, dist=P["dist"], fn=fn, ft=ft, D=D, aref=aref)


def newton_step(m, qpos, qvel, qws):
    """One Newton iteration of mj_solNewton on the ball's cost, restated from its documented steps:
    start from the cheaper of qacc_warmstart and qacc_smooth, gradient and Hessian M + J_A' D J_A
    of the rows active there, direction d = -H^-1 grad; returns (x0, d, the exact minimum of the
    cost along x0 + alpha d over alpha >= 0)."""
    P = ball_problem(m, qpos, qvel)
    xs, xw = P["a0"], np.asarray(qws[0:6], float)
    x0 = xs if cost(P, xw) > cost(P, xs) else xw
    Mb, a0 = P["M"], P["a0"]
    g = Mb @ (x0 - a0)
    H = Mb.copy()
    if P["rows"] is not None:
        x = P["rows"] @ x0 - P["aref"]
        act = (x < 0).astype(float)
        g = g + P["rows"].T @ (P["D"] * act * x)
        H = H + P["rows"].T @ ((P["D"] * act)[:, None] * P["rows"])
    d = -np.linalg.solve(H, g)
    # exact 1-D minimum of the piecewise quadratic: on each piece between consecutive switch points
    # the active set is fixed and the cost is c0 + c1 a + c2 a^2 with these coefficients
    e = x0 - a0
    g0, g1, g2 = 0.5 * e @ Mb @ e, d @ Mb @ e, 0.5 * d @ Mb @ d
    br = [0.0]
    x = jd = np.zeros(0)
    if P["rows"] is not None:
        jd = P["rows"] @ d
        x = P["rows"] @ x0 - P["aref"]
        br += [float(-xi / ji) for xi, ji in zip(x, jd) if ji != 0 and -xi / ji > 0]
    br = sorted(set(br)) + [np.inf]
    best = np.inf
    for lo, hi in zip(br[:-1], br[1:]):
        mid = lo + 1.0 if hi == np.inf else 0.5 * (lo + hi)
        on = (x + mid * jd) < 0
        c0 = g0 + 0.5 * P.get("D", 0.0) * np.sum(on * x * x)
        c1 = g1 + P.get("D", 0.0) * np.sum(on * x * jd)
        c2 = g2 + 0.5 * P.get("D", 0.0) * np.sum(on * jd * jd)
        cands = [lo] + ([hi] if hi != np.inf else [])
        am = -c1 / (2 * c2)
        if lo <= am <= hi:
            cands.append(am)
        best = min(best, min(c0 + c1 * a + c2 * a * a for a in cands))
    return x0, d, best, P


def _rest_state():
    q = np.zeros(19)
    q[2], q[3] = R_BALL, 1.0
    q[7:] = DP
    return q, np.zeros(18), np.zeros(18)


def run_oracle(m, nsteps, precision="f64"):
    q, v, w = _rest_state()
    return O.mj_step(m, q, v, w, DP.copy(), nsteps=nsteps, precision=precision)


CASES = {"roll": (10.0, 1.0), "slide": (20.0, 0.05)}


@pytest.mark.parametrize("case", sorted(CASES))
def test_converged_qacc_equals_documented_soft_pyramid(case):
    """Newton run to convergence (50 iterations): after 0.6 s of rolling / sliding, one more oracle
    substep's qacc (its qacc_warmstart output) is the exact minimiser of the documented soft-pyramid
    problem at that state -- this pins the edge rows, their regulariser with impratio and aref."""
    theta, mu = CASES[case]
    m = ball_model(theta, mu, iterations=50)
    q, v, w, _, _ = run_oracle(m, 150)
    _, _, w2, _, _ = O.mj_step(m, q, v, w, DP.copy(), nsteps=1)
    a, info = ball_qacc(m, q, v)
    assert info["dist"] < 0 and sum(info["active"]) >= 1
    np.testing.assert_allclose(w2[0:6], a, atol=1e-7 * G, rtol=1e-6)


@pytest.mark.parametrize("case", sorted(CASES))
def test_one_newton_iteration_is_a_line_searched_newton_step(case):
    """The reference's iterations=1 (xml:57): the oracle's qacc lies on the Newton direction from
    the cheaper of warm start / smooth acceleration (cosine 1 - 1e-9) and never costs more than
    that start; on the smooth rolling contact the line search reaches the line's exact minimum.
    (On the chattering sliding contact MuJoCo's PrimalSearch can exhaust ls_iterations = 5 on a
    bracket and keep alpha = 0 -- then the step is the warm start itself, still consistent.)"""
    theta, mu = CASES[case]
    m = ball_model(theta, mu)
    for n in (150, 151, 157):
        q, v, w, _, _ = run_oracle(m, n)
        _, _, w2, _, _ = O.mj_step(m, q, v, w, DP.copy(), nsteps=1)
        x0, d, cmin, P = newton_step(m, q, v, w)
        step = w2[0:6] - x0
        if np.linalg.norm(step) > 1e-6 * np.linalg.norm(x0):  # (alpha = 0 or a converged warm start: no step)
            cosang = step @ d / (np.linalg.norm(step) * np.linalg.norm(d))
            assert cosang > 1 - 1e-9, cosang
        c = cost(P, w2[0:6])
        assert c <= cost(P, x0) * (1 + 1e-12) + 1e-12
        if case == "roll":
            assert cmin - 1e-12 <= c <= cmin + 1e-6 * max(abs(cmin), 1e-3), (c, cmin)


def _slip(q, v):
    """Tangential velocity (along the slope, x) of the ball's material point at the contact."""
    wy = (_quat_mat(q[3:7]) @ v[3:6])[1]
    dist = q[2] - R_BALL
    return v[0] - (R_BALL + 0.5 * dist) * wy, wy


def test_ball_rolls_without_slip_at_five_sevenths_g_sin():
    """mu = 1 > (2/7) tan 10 deg (the reference's solver, iterations = 1): the ball rolls; its centre
    accelerates at (5/7) g sin th along the slope and the contact point creeps at < 0.1 % of the
    speed (the soft constraint's regularised stick)."""
    theta, mu = CASES["roll"]
    m = ball_model(theta, mu)
    q1, v1, w1, _, _ = run_oracle(m, 100)
    q2, v2, _, _, _ = O.mj_step(m, q1, v1, w1, DP.copy(), nsteps=50)
    acc = (v2[0] - v1[0]) / (50 * m.timestep)
    expect = 5.0 / 7.0 * G * math.sin(math.radians(theta))
    np.testing.assert_allclose(acc, expect, rtol=5e-3)
    slip, _ = _slip(q2, v2)
    assert abs(slip) < 1e-3 * v2[0], (slip, v2[0])
    assert abs(v2[1]) < 1e-9 and abs(q2[2] - R_BALL) < 2e-3  # no sideways motion, rests on the floor


def test_ball_slides_below_the_stick_threshold():
    """mu = 0.05 < (2/7) tan 20 deg = 0.104 (Newton converged, 50 iterations): the ball slides.  The
    friction never exceeds the pyramid's Coulomb bound mu F_n along the slide axis, so over a long
    window the centre accelerates at g (sin th - mu cos th) or a little more (the soft pyramid's
    side edges carry part of the normal load at low slip); the friction torque spins the ball up at
    5 F_t / (2 m r) while the contact point keeps slipping."""
    theta, mu = CASES["slide"]
    m = ball_model(theta, mu, iterations=50)
    th = math.radians(theta)
    q1, v1, w1, _, _ = run_oracle(m, 100)
    q2, v2, w2, _, _ = O.mj_step(m, q1, v1, w1, DP.copy(), nsteps=400)
    acc = (v2[0] - v1[0]) / (400 * m.timestep)
    lo = G * (math.sin(th) - mu * math.cos(th))
    np.testing.assert_allclose(acc, lo, rtol=2e-3)
    spin = (_slip(q2, v2)[1] - _slip(q1, v1)[1]) / (400 * m.timestep)
    # torque F_t (r - |dist|/2) on 2/5 m r^2 (the contact point sits half the penetration inside)
    np.testing.assert_allclose(spin, 5.0 * M_BALL * (G * math.sin(th) - acc) / (2.0 * M_BALL * R_BALL), rtol=5e-3)
    assert _slip(q2, v2)[0] > 0.3 * v2[0]  # still slipping
    # instantaneous Coulomb bound on every contact substep of a stretch of the slide
    q, v, w = q2, v2, w2
    for _ in range(40):
        _, info = ball_qacc(m, q, v)
        if info["dist"] < 0 and info["fn"] > 0:
            assert abs(info["ft"][0]) < 1e-9 * info["fn"]  # no friction across the slope
            assert abs(info["ft"][1]) <= mu * info["fn"] * (1 + 1e-12)
        q, v, w, _, _ = O.mj_step(m, q, v, w, DP.copy(), nsteps=1)


def test_impratio_hardens_the_friction_rows():
    """impratio divides the edge rows' regulariser (A = (tran + mu^2 tran) 2 mu^2 / impratio): rolling,
    the contact point's creep shrinks about in proportion when impratio goes from 1 to 10, and the
    converged qacc still equals the documented minimiser at both values."""
    theta, mu = CASES["roll"]
    creep = {}
    for ir in (1.0, 10.0):
        m = ball_model(theta, mu)
        m.impratio = ir
        q, v, w, _, _ = run_oracle(m, 150)
        creep[ir] = _slip(q, v)[0]
        m50 = ball_model(theta, mu, iterations=50)
        m50.impratio = ir
        a, _ = ball_qacc(m50, q, v)
        _, _, w2, _, _ = O.mj_step(m50, q, v, w, DP.copy(), nsteps=1)
        np.testing.assert_allclose(w2[0:6], a, atol=1e-7 * G, rtol=1e-6)
    assert creep[1.0] > 0 and creep[10.0] > 0
    assert 5.0 < creep[1.0] / creep[10.0] < 15.0, creep
