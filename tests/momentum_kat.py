"""Angular-momentum known answer for the articulated dynamics (mj_rne's Coriolis / gyroscopic
terms, the CRB mass matrix and the free joint's conventions), shared by test_momentum_kat.py (the
oracle) and test_gpu_momentum_kat.py (the kernel).

In flight (no contact), with uniform gravity and only joint-space internal forces (PD actuators,
hinge damping, frictionloss and limit rows act between parent and child bodies), the system's
angular momentum about its centre of mass is conserved and its linear momentum changes at
M_total g.  Both are evaluated here from the bodies alone (an independent forward kinematics,
mjcf.mass_matrix_and_jacobians) and differentiated in time by a central finite difference along
(qvel, qacc), so a wrong velocity-product term in either restatement shows up as a torque.
Armature (reflected rotor inertia belongs to no body) and free-joint damping (an external force)
are zeroed in the model used here."""
import numpy as np

import common
from pupperv3_mjx import _abi, mjcf


def flight_model():
    cm = common.pd_model()
    m = cm.struct
    for d in range(_abi.NV):
        m.dof_armature[d] = 0.0
    for d in range(6):
        m.dof_damping[d] = 0.0
    mjcf.recompute_constants(cm)
    return m


def flight_states(n, seed):
    rs = np.random.RandomState(seed)
    out = []
    for _ in range(n):
        q = np.zeros(19)
        q[2] = 2.0
        qq = rs.normal(size=4)
        q[3:7] = qq / np.linalg.norm(qq)
        q[7:] = np.array(common.DEFAULT_POSE) + rs.uniform(-0.3, 0.3, 12)
        v = np.concatenate([rs.normal(scale=0.5, size=3), rs.normal(scale=3.0, size=3), rs.normal(scale=3.0, size=12)])
        ctrl = np.array(common.DEFAULT_POSE) + rs.uniform(-0.5, 0.5, 12)
        out.append((q, v, ctrl))
    return out


def _advance(q, v, h):
    """qpos after moving along qvel for time h (free joint: world linear, body-frame angular)."""
    q1 = q.copy()
    q1[:3] += h * v[:3]
    w = v[3:6]
    nw = np.linalg.norm(w)
    q1[3:7] = mjcf.quat_mul(q[3:7], mjcf.axis_angle_quat(w / nw, h * nw))
    q1[7:] += h * v[6:]
    return q1


def momenta(m, q, v):
    """(linear momentum, angular momentum about the system COM) from the bodies alone."""
    _, jacp, jacr, xipos = mjcf.mass_matrix_and_jacobians(m, q)
    _, xquat, _, _ = mjcf._kinematics(m, q)
    mass = np.array(m.body_mass[:])
    xc = sum(mass[b] * xipos[b] for b in range(1, _abi.NBODY)) / mass[1:].sum()
    P = np.zeros(3)
    L = np.zeros(3)
    for b in range(1, _abi.NBODY):
        vb, wb = jacp[b] @ v, jacr[b] @ v
        R = mjcf.quat_to_mat(mjcf.quat_mul(xquat[b], np.array(m.body_iquat[b][:])))
        Iw = R @ np.diag(np.array(m.body_inertia[b][:])) @ R.T
        P += mass[b] * vb
        L += mass[b] * np.cross(xipos[b] - xc, vb) + Iw @ wb
    return P, L


def momentum_rates(m, q, v, qacc, h=1e-5):
    """(dP/dt, dL/dt, dL/dt with qacc = 0) by central differences along (v, qacc)."""
    def at(t, a):
        return momenta(m, _advance(q, v, t), v + t * a)
    (P1, L1), (P0, L0) = at(h, qacc), at(-h, qacc)
    (_, L1z), (_, L0z) = at(h, 0 * qacc), at(-h, 0 * qacc)
    return (P1 - P0) / (2 * h), (L1 - L0) / (2 * h), (L1z - L0z) / (2 * h)


def dr_rows(n, seed):
    """n domain-randomisation rows: domain_randomization.domain_randomize (the reference's ranges)
    on the nominal PD model's System, built as PupperV3Env builds `env.sys`."""
    from pupperv3_mjx import domain_randomization as dr, rng
    cm = common.pd_model()
    m = cm.struct
    nominal = dr.System(
        geom_friction=cm.geom_friction.copy(),
        actuator_gainprm=np.pad(np.array(m.actuator_gainprm[:], dtype=np.float64), ((0, 0), (0, 7))),
        actuator_biasprm=np.pad(np.array(m.actuator_biasprm[:], dtype=np.float64), ((0, 0), (0, 7))),
        body_ipos=np.array(m.body_ipos[:], dtype=np.float64),
        body_inertia=np.array(m.body_inertia[:], dtype=np.float64),
        body_mass=np.array(m.body_mass[:], dtype=np.float64))
    out, _ = dr.domain_randomize(nominal, rng.split(rng.PRNGKey(seed), n))
    return out


def dr_edited(m, row):
    """A copy of model struct m with one DR row written into the reference's fields
    (domain_randomization.py: body_mass, body_inertia, body_ipos[1]; sys.tree_replace)."""
    e = type(m).from_buffer_copy(m)
    for b in range(_abi.NBODY):
        e.body_mass[b] = float(row[_abi.DR_MASS + b])
        for k in range(3):
            e.body_inertia[b][k] = float(row[_abi.DR_INERTIA + 3 * b + k])
    for k in range(3):
        e.body_ipos[1][k] = float(row[_abi.DR_BASE_IPOS + k])
    return e
