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
