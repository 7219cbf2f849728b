"""Momentum known answers on the oracle (tests/momentum_kat.py): in flight the articulated body's
angular momentum about its COM is conserved and its linear momentum changes at M_total g, for
random poses, spins and PD targets; the kernel's counterpart is test_gpu_momentum_kat.py."""
import numpy as np

import momentum_kat as K
from oracle import oracle as O


def test_flight_conserves_angular_momentum_and_falls_at_g():
    m = K.flight_model()
    mass = np.array(m.body_mass[1:]).sum()
    for q, v, ctrl in K.flight_states(6, seed=1):
        r = O.mj_forward(m, q, v, np.zeros(18), ctrl)
        assert r["nefc"] >= 12  # frictionloss rows active (internal), no contacts
        dP, dL, dL0 = K.momentum_rates(m, q, v, r["qacc"])
        np.testing.assert_allclose(dP / mass, np.array(m.gravity[:]), atol=1e-6)
        # the velocity-product terms qacc must cancel are O(|dL0|): a wrong term leaves O(1) of it
        assert np.linalg.norm(dL0) > 1e-3
        assert np.linalg.norm(dL) <= 1e-6 * np.linalg.norm(dL0) + 1e-9, (dL, dL0)


def test_domain_randomised_flight_uses_the_rows_fields():
    """With a DR row (domain_randomization.py semantics: body_mass, body_inertia, body_ipos[1],
    Kp / Kd) the step's dynamics are those of the model with the row written into those fields:
    momentum computed on the edited model is conserved / falls at g, and the PD torque uses the
    row's Kp and Kd."""
    import test_actuator_kat as A
    from pupperv3_mjx import _abi
    m = K.flight_model()
    table = K.dr_rows(6, seed=5).dr_table().astype(np.float64)
    for i, (q, v, ctrl) in enumerate(K.flight_states(6, seed=3)):
        _, _, qacc, pipe, _ = O.mj_step(m, q, v, np.zeros(18), ctrl, nsteps=1, dr=table[i])
        me = K.dr_edited(m, table[i])
        dP, dL, dL0 = K.momentum_rates(me, q, v, qacc)
        np.testing.assert_allclose(dP / np.array(me.body_mass[1:]).sum(), np.array(m.gravity[:]), atol=1e-6)
        assert np.linalg.norm(dL) <= 1e-6 * np.linalg.norm(dL0) + 1e-9, (dL, dL0)
        kp, kd = table[i, _abi.DR_KP], table[i, _abi.DR_KD]
        want = np.clip(kp * (ctrl - q[7:]) - kd * v[6:], -A.FMAX, A.FMAX)
        np.testing.assert_allclose(pipe[_abi.P_QFRC_ACT + 6:_abi.P_QFRC_ACT + 18], want, atol=1e-9)
