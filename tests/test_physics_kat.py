"""Analytic / independent known answers for the physics pieces the kernel and the oracle SHARE.

Every GPU parity test compares the kernel with oracle/pp3_oracle.c, and both consume the same
model constants from pupperv3_mjx/mjcf.py (invweight0, meaninertia, solref/solimp mixing).  A
mistake there would be common-mode and invisible to parity, so these CPU tests pin them against
answers derived without either restatement (SURVEY.md 7 hard part 1; MuJoCo itself is absent, so
the answers come from mechanics and from MuJoCo's documented constraint model):

* the joint-space inertia M: an independent forward kinematics written here, body velocities by
  central finite differences, M = sum_b m J_p'J_p + J_r' I_w J_r + diag(armature) (kinetic energy);
  it must equal the oracle's CRB mass matrix and mjcf's analytic-Jacobian one;
* invweight0 / meaninertia (mjcf.py:676-692, MuJoCo mj_setConst): recomputed from that M, and for a
  lone free body (legs made negligible) the closed forms 1/m and trace(I_com^-1)/3; for a hinge
  pendulum on a pinned base, 1/(armature + I_axis + m d^2);
* frictionloss (xml:55, 0.125 on every hinge): below the threshold a joint creeps at MuJoCo's
  documented soft-constraint steady state v = tau R / b (R = (1 - d) / d * dof_invweight0, d = the
  solimp impedance at 0, b = 2 / (dmax timeconst)); above it the joint accelerates at
  (tau - 0.125 - damping v) / M_jj;
* soft-contact resting state: the weight is carried (qfrc_bias of the vertical dof = total weight
  = the summed normal force at rest) and every foot penetrates by the documented equilibrium depth
  sign (r < 0, |r| below the solimp width where the impedance saturates).

Pyramidal contact friction with impratio (the edge rows' regulariser and the one-Newton-iteration
response) is pinned in tests/test_friction_kat.py on a body that cannot tip (a solid ball on a
slope: the exact soft-pyramid minimiser, rolling at 5/7 g sin, the Coulomb bound, impratio creep),
and on the kernel by tests/test_gpu_kat.py.  solref/solimp MIXING (the collision class, xml:51,
against the floor's defaults, xml:219: resting depth, steady rolling creep, converged qacc) and the
pyramid's TANGENT BASIS for normals off the vertical (mju_makeFrame on tilted box faces, edges,
corners and between two legs' spheres) are pinned in tests/test_contact_kat.py (oracle) and
tests/test_gpu_contact_kat.py (kernel), from MuJoCo's documentation (tests/contact_kat.py).  What stays unpinned is MuJoCo's own implementation
(both restatements are checked against its documented constraint model, not its C source).
"""
import numpy as np
import pytest

import common
from oracle import oracle as O
from pupperv3_mjx import _abi, mjcf

DP = np.array(common.DEFAULT_POSE)


# ------------------------------------------------------------------ independent kinematics / M
def _qmul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def _qmat(q):
    q = q / np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _qaxis(axis, ang):
    axis = np.asarray(axis, float)
    return np.concatenate([[np.cos(ang / 2)], np.sin(ang / 2) * axis / np.linalg.norm(axis)])


def body_frames(m, q):
    """World position of every body's COM and the world rotation of its inertia frame, written
    from the MJCF tree alone: free base, then hinge chains (xquat_b = xquat_p * body_quat_b *
    rot(axis, q - q0), xpos_b = xpos_p + R_p body_pos_b)."""
    nb = _abi.NBODY
    xpos, xquat = np.zeros((nb, 3)), np.zeros((nb, 4))
    xquat[0] = [1, 0, 0, 0]
    com, rot = np.zeros((nb, 3)), np.zeros((nb, 3, 3))
    for b in range(1, nb):
        j = m.body_jntadr[b]
        if m.jnt_type[j] == mjcf.JNT_FREE:
            xpos[b] = q[0:3]
            xquat[b] = q[3:7] / np.linalg.norm(q[3:7])
        else:
            p = m.body_parentid[b]
            xpos[b] = xpos[p] + _qmat(xquat[p]) @ np.array(m.body_pos[b][:])
            a = m.jnt_qposadr[j]
            xquat[b] = _qmul(_qmul(xquat[p], np.array(m.body_quat[b][:])),
                             _qaxis(m.jnt_axis[j][:], q[a] - m.qpos0[a]))
        R = _qmat(xquat[b])
        com[b] = xpos[b] + R @ np.array(m.body_ipos[b][:])
        rot[b] = _qmat(_qmul(xquat[b], np.array(m.body_iquat[b][:])))
    return com, rot


def _perturb(q, i, eps):
    """q (+) eps * e_i in MuJoCo's velocity coordinates: free translation in world, free rotation
    in the body frame (quat * exp), hinges additive."""
    q = q.copy()
    if i < 3:
        q[i] += eps
    elif i < 6:
        q[3:7] = _qmul(q[3:7], _qaxis(np.eye(3)[i - 3], eps))
    else:
        q[i + 1] += eps
    return q


def fd_jacobians(m, q, eps=1e-6):
    """COM Jacobians (translation, rotation) of every body by central differences."""
    nb, nv = _abi.NBODY, _abi.NV
    Jp, Jr = np.zeros((nb, 3, nv)), np.zeros((nb, 3, nv))
    for i in range(nv):
        cp, rp = body_frames(m, _perturb(q, i, eps))
        cm, rm = body_frames(m, _perturb(q, i, -eps))
        Jp[:, :, i] = (cp - cm) / (2 * eps)
        for b in range(1, nb):
            dR = rp[b] @ rm[b].T
            Jr[b, :, i] = np.array([dR[2, 1] - dR[1, 2], dR[0, 2] - dR[2, 0], dR[1, 0] - dR[0, 1]]) / (4 * eps)
    return Jp, Jr


def energy_mass_matrix(m, q):
    """M from the kinetic energy T = 1/2 qd' M qd = 1/2 sum_b (m_b |v_b|^2 + w_b' I_b,world w_b)."""
    Jp, Jr = fd_jacobians(m, q)
    _, rot = body_frames(m, q)
    M = np.diag(np.array(m.dof_armature[:]))
    for b in range(1, _abi.NBODY):
        Iw = rot[b] @ np.diag(np.array(m.body_inertia[b][:])) @ rot[b].T
        M = M + m.body_mass[b] * Jp[b].T @ Jp[b] + Jr[b].T @ Iw @ Jr[b]
    return M, Jp, Jr


def _random_q(rs):
    q = np.zeros(19)
    q[:3] = rs.uniform(-1, 1, 3)
    qq = rs.normal(size=4)
    q[3:7] = qq / np.linalg.norm(qq)
    q[7:] = DP + rs.uniform(-0.6, 0.6, 12)
    return q


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_mass_matrix_equals_kinetic_energy_hessian(seed):
    m = common.pd_model().struct
    q = np.array(m.qpos0[:]) if seed == 0 else _random_q(np.random.RandomState(seed))
    M_fd, _, _ = energy_mass_matrix(m, q)
    M_oracle = O.mj_forward(m, q, np.zeros(18), np.zeros(18), DP)["M"]
    M_mjcf = mjcf.mass_matrix_and_jacobians(m, q)[0]
    scale = np.abs(M_fd).max()
    np.testing.assert_allclose(M_oracle, M_fd, atol=1e-7 * scale)
    np.testing.assert_allclose(M_mjcf, M_fd, atol=1e-7 * scale)
    assert np.all(np.linalg.eigvalsh(M_fd) > 0)


def _invweight_from(M, Jp, Jr, m):
    Minv = np.linalg.inv(M)
    d = np.diag(Minv).copy()
    d[0:3] = d[0:3].mean()
    d[3:6] = d[3:6].mean()
    body = np.zeros((_abi.NBODY, 2))
    for b in range(1, _abi.NBODY):
        body[b] = [np.trace(Jp[b] @ Minv @ Jp[b].T) / 3, np.trace(Jr[b] @ Minv @ Jr[b].T) / 3]
    return d, body, np.trace(M) / _abi.NV


def test_invweight0_and_meaninertia_from_independent_M():
    cm = common.pd_model()
    m = cm.struct
    M, Jp, Jr = energy_mass_matrix(m, np.array(m.qpos0[:]))
    d, body, mi = _invweight_from(M, Jp, Jr, m)
    np.testing.assert_allclose(np.array(m.dof_invweight0[:]), d, rtol=1e-6)
    np.testing.assert_allclose(np.array(m.body_invweight0[:]), body, rtol=1e-6, atol=1e-12)
    assert abs(m.meaninertia - mi) <= 1e-7 * mi


def _negligible_legs(cm, keep=()):
    """Legs reduced to 1e-9 kg / 1e-13 kg m^2 (bodies in `keep` untouched), constants recomputed."""
    m = cm.struct
    for b in range(2, _abi.NBODY):
        if b in keep:
            continue
        m.body_mass[b] = 1e-9
        for k in range(3):
            m.body_inertia[b][k] = 1e-13
    mjcf.recompute_constants(cm)
    return m


def test_lone_free_body_invweight_closed_form():
    """A free body alone: COM mobility 1/m and angular mobility trace(I_com^-1)/3 exactly
    (independent of where the free joint's origin sits relative to the COM)."""
    cm = common.pd_model()
    m = _negligible_legs(cm)
    mass = m.body_mass[1]
    I = np.array(m.body_inertia[1][:])
    np.testing.assert_allclose(m.body_invweight0[1][0], 1.0 / mass, rtol=1e-5)
    np.testing.assert_allclose(m.body_invweight0[1][1], np.mean(1.0 / I), rtol=1e-5)
    # free translational dofs move the body ORIGIN: 1/m + the COM-offset coupling, averaged
    c = np.array(m.body_ipos[1][:])
    Rc = _qmat(np.array(m.body_iquat[1][:]))
    Ic = Rc @ np.diag(I) @ Rc.T                       # inertia about the COM, body axes
    cx = np.array([[0, -c[2], c[1]], [c[2], 0, -c[0]], [-c[1], c[0], 0]])
    Mfree = np.block([[mass * np.eye(3), -mass * cx], [mass * cx, Ic - mass * cx @ cx]])  # qpos0: R = I
    Minv = np.linalg.inv(Mfree)
    np.testing.assert_allclose(np.array(m.dof_invweight0[0:3]), np.trace(Minv[:3, :3]) / 3, rtol=1e-5)
    np.testing.assert_allclose(np.array(m.dof_invweight0[3:6]), np.trace(Minv[3:, 3:]) / 3, rtol=1e-5)
    # hinges with negligible links: only their armature resists
    np.testing.assert_allclose(np.array(m.dof_invweight0[6:]), 1.0 / np.array(m.dof_armature[6:]), rtol=1e-4)


def test_hinge_pendulum_invweight_closed_form():
    """Base pinned (1e9 kg), the hip hinge of leg 0 locked (armature 1e9), the leg's second link
    real and everything else negligible: that link's hinge is a compound pendulum with an offset
    COM, invweight0 = 1/(armature + I_axis + m d_perp^2)."""
    cm = common.pd_model()
    m = cm.struct
    m.body_mass[1] = 1e9
    for k in range(3):
        m.body_inertia[1][k] = 1e9
    m.dof_armature[6] = 1e9
    m = _negligible_legs(cm, keep=(3,))
    b, j, dof = 3, 2, 7
    q0 = np.array(m.qpos0[:])
    com, rot = body_frames(m, q0)
    # the hinge's world anchor (jnt_pos = 0: the body origin) and axis, from the tree
    xq = _qmul(_qmul(q0[3:7] / np.linalg.norm(q0[3:7]), np.array(m.body_quat[2][:])), np.array(m.body_quat[b][:]))
    anchor = q0[0:3] + _qmat(q0[3:7]) @ np.array(m.body_pos[2][:]) + \
        _qmat(_qmul(q0[3:7] / np.linalg.norm(q0[3:7]), np.array(m.body_quat[2][:]))) @ np.array(m.body_pos[b][:])
    axis = _qmat(xq) @ np.array(m.jnt_axis[j][:])
    Iw = rot[b] @ np.diag(np.array(m.body_inertia[b][:])) @ rot[b].T
    r = com[b] - anchor
    d_perp2 = r @ r - (r @ axis) ** 2
    assert d_perp2 > 1e-4  # a real offset pendulum
    expect = 1.0 / (m.dof_armature[dof] + axis @ Iw @ axis + m.body_mass[b] * d_perp2)
    np.testing.assert_allclose(m.dof_invweight0[dof], expect, rtol=1e-5)


# ------------------------------------------------------------------ frictionloss stick / slip
def _torque_model(pin_base=True):
    """Gravity off, base pinned, actuators as pure torque sources (force = ctrl)."""
    cm = common.pd_model()
    m = cm.struct
    m.gravity[:] = [0.0, 0.0, 0.0]
    if pin_base:
        m.body_mass[1] = 1e9
        for k in range(3):
            m.body_inertia[1][k] = 1e9
    for i in range(12):
        m.actuator_gainprm[i][0] = 1.0
        m.actuator_biasprm[i][:] = [0.0, 0.0, 0.0]
    m.npair = 0  # no contacts: the joint rows alone
    mjcf.recompute_constants(cm)
    return m


def _imp(si, x):
    """MuJoCo's documented impedance sigmoid d(x) (solimp = dmin, dmax, width, midpoint, power)."""
    dmin, dmax, width, mid, p = si
    x = min(abs(x) / width, 1.0)
    y = x ** p / mid ** (p - 1) if x <= mid else 1 - (1 - x) ** p / (1 - mid) ** (p - 1)
    return dmin + y * (dmax - dmin)


def test_frictionloss_creep_below_threshold():
    """|tau| < frictionloss: the joint creeps at the documented soft-constraint steady state.  The
    row is in its quadratic zone with f = -D (J a - aref), aref = -b v (pos = 0), D = 1/R,
    R = (1 - d)/d * dof_invweight0, d = impedance at 0; steady state (a = 0) with the joint damping:
    D b v + damping v = tau  ->  v = tau R / (b + damping R)."""
    m = _torque_model()
    knee = 8  # dof of leg 0's distal hinge (actuator 2): nothing hangs below it
    tau = 0.06
    q = np.zeros(19)
    q[3] = 1
    q[7:] = DP
    ctrl = np.zeros(12)
    ctrl[knee - 6] = tau
    qn, vn, wn, _, _ = O.mj_step(m, q, np.zeros(18), np.zeros(18), ctrl, nsteps=100)
    si = np.array(m.dof_solimp[knee][:])
    tc = m.dof_solref[knee][0]
    d = _imp(si, 0.0)
    b = 2.0 / (si[1] * tc)
    R = (1 - d) / d * m.dof_invweight0[knee]
    v_expect = tau * R / (b + m.dof_damping[knee] * R)
    np.testing.assert_allclose(vn[knee], v_expect, rtol=2e-3)
    # settled (no acceleration): a soft hold, not a slow slide
    _, vn2, _, _, _ = O.mj_step(m, qn, vn, wn, ctrl, nsteps=50)
    np.testing.assert_allclose(vn2[knee], vn[knee], rtol=1e-4)
    # the parent joints stay held (their reaction torques are below the frictionloss)
    assert np.abs(vn[6:8]).max() < 1e-3 * vn[knee]


def test_frictionloss_slips_above_threshold():
    """|tau| > frictionloss: the friction row saturates at exactly the frictionloss and the joint
    accelerates at (tau - frictionloss - damping v) / M_jj (parent joints held)."""
    m = _torque_model()
    knee = 8
    tau = 0.25
    q = np.zeros(19)
    q[3] = 1
    q[7:] = DP
    ctrl = np.zeros(12)
    ctrl[knee - 6] = tau
    M = O.mj_forward(m, q, np.zeros(18), np.zeros(18), ctrl)["M"]
    q1, v1, w1, _, _ = O.mj_step(m, q, np.zeros(18), np.zeros(18), ctrl, nsteps=2)
    _, v2, _, _, _ = O.mj_step(m, q1, v1, w1, ctrl, nsteps=6)
    acc = (v2[knee] - v1[knee]) / (6 * m.timestep)
    vm = 0.5 * (v1[knee] + v2[knee])
    expect = (tau - m.dof_frictionloss[knee] - m.dof_damping[knee] * vm) / M[knee, knee]
    np.testing.assert_allclose(acc, expect, rtol=0.01)
    assert np.abs(v2[6:8]).max() < 1e-2 * v2[knee]


# ------------------------------------------------------------------ soft contact at rest
def _stand(mu, nsteps=2000):
    """The robot PD-held at its default pose, settled on flat ground (fp64 oracle)."""
    cm = common.pd_model()
    m = cm.struct
    for g in range(m.ncgeom):
        m.cgeom_friction[g][0] = mu
    q = np.zeros(19)
    q[2], q[3], q[7:] = 0.16, 1.0, DP
    q, v, w, _, _ = O.mj_step(m, q, np.zeros(18), np.zeros(18), DP, nsteps=nsteps)
    return m, q, v, w


def test_resting_robot_carries_its_weight():
    """At rest the contact rows carry the robot: the constraint force on the vertical free dof,
    qfrc_constraint[2] = (M qacc)[2] + qfrc_bias[2] (no actuator or passive force acts on a free
    dof), equals the total weight, with every foot penetrating by less than the mixed solimp width
    (0.016 m: collision class 0.031 averaged with the floor's default 0.001 at solmix 0.5)."""
    m, q, v, w = _stand(0.8)
    out = O.mj_forward(m, q, v, w, DP)
    weight = 9.81 * sum(m.body_mass[1:])
    assert np.abs(v[:6]).max() < 1e-4 and np.abs(v).max() < 1e-3  # settled (joints creep at 1e-4)
    fc_z = (out["M"] @ out["qacc"])[2] + out["qfrc_bias"][2]
    np.testing.assert_allclose(fc_z, weight, rtol=2e-3)
    p = out["pipe"]
    ncon = int(p[_abi.P_NCON])
    dist = p[_abi.P_CON_DIST:_abi.P_CON_DIST + ncon]
    assert ncon >= 3 and np.all(dist < 0)
    assert np.all(-dist < 0.016), dist


# ------------------------------------------------------------------ joint-limit rows at rest
def _limit_rest_prediction(m, jnt, tau):
    """Where a hinge pushed by a constant torque tau comes to rest against its limit (MuJoCo's
    documented soft-constraint model, not either implementation): the side the torque pushes into,
    and x = pos - margin of that limit row (pos = side (range - q) < 0 when violated).  At rest
    (a = v = 0) the row force is f = D aref = -(k d(x) / R(x)) x with R = (1 - d)/d * A,
    A = dof_invweight0, k = 1/(dmax tc dr)^2 (tc >= 2 timestep, REFSAFE); the joint-space balance
    -side f + tau = 0 gives x = -|tau| A (1 - d(x)) / (k d(x)^2), solved by bisection (d from
    solimp on |x|)."""
    side = 1 if tau > 0 else -1
    dof = m.jnt_dofadr[jnt]
    si = np.array(m.jnt_solimp[jnt][:])
    tc, dr = m.jnt_solref[jnt][0], m.jnt_solref[jnt][1]
    tc = max(tc, 2 * m.timestep)
    k = 1.0 / (si[1] * tc * dr) ** 2
    A = m.dof_invweight0[dof]

    def resid(x):
        d = _imp(si, x)
        return x + abs(tau) * A * (1 - d) / (k * d * d)
    lo, hi = -1.0, 0.0  # resid(-1) < 0 < resid(0)
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if resid(mid) < 0:
            lo = mid
        else:
            hi = mid
    x = 0.5 * (lo + hi)
    rng = m.jnt_range[jnt][(side + 1) // 2]
    # pos = side (rng - q) = x + margin  ->  q = rng - side (x + margin)
    return side, x, rng - side * (x + m.jnt_margin[jnt])


LIMIT_CASES = [(3, 0.3), (3, -0.3), (3, 0.01), (1, -0.25)]  # (joint, torque): knee both sides, in the solimp width, hip


@pytest.mark.parametrize("jnt,tau", LIMIT_CASES)
def test_joint_limit_rest_position(jnt, tau):
    """A hinge driven into its range limit by a constant torque settles at the documented soft-limit
    equilibrium: beyond the solimp width (d = dmax) and inside it (d on the sigmoid); the limit row
    then carries exactly the torque (the frictionloss row carries nothing at rest)."""
    m = _torque_model()
    dof = m.jnt_dofadr[jnt]
    side, x, q_expect = _limit_rest_prediction(m, jnt, tau)
    assert (abs(x) > m.jnt_solimp[jnt][2]) == (abs(tau) > 0.1)  # the cases cover both impedance zones
    q = np.zeros(19)
    q[3] = 1
    q[7:] = DP
    q[m.jnt_qposadr[jnt]] = m.jnt_range[jnt][(side + 1) // 2] - side * 0.002  # just inside the limit
    ctrl = np.zeros(12)
    ctrl[dof - 6] = tau
    qn, vn, wn, _, _ = O.mj_step(m, q, np.zeros(18), np.zeros(18), ctrl, nsteps=1500)
    q2, v2, _, _, _ = O.mj_step(m, qn, vn, wn, ctrl, nsteps=1)
    # at rest over a substep pair: against a lower limit the folded leg's parent hinges keep a
    # period-2 chatter (v flips sign every substep; one Newton iteration with the frictionloss rows
    # at their kinks), which leaves the mean motion and the pushed joint's position at rest
    assert abs(vn[dof] + v2[dof]) < 1e-8 and np.abs(vn[6:] + v2[6:]).max() < 2e-5, (vn[dof], v2[dof])
    qa = 0.5 * (qn[m.jnt_qposadr[jnt]] + q2[m.jnt_qposadr[jnt]])
    rng = m.jnt_range[jnt][(side + 1) // 2]
    np.testing.assert_allclose(qa - rng, q_expect - rng, rtol=2e-3)
