"""Momentum known answers on the kernel (tests/momentum_kat.py): one raw substep from random
flight states (random poses, spins up to ~3 rad/s per dof, PD targets) gives a qacc whose angular
momentum rate about the COM is zero and whose linear momentum rate is M_total g.  fp32 tolerance:
|dL/dt| <= 2e-3 |dL0/dt| (dL0 = the velocity-product part the solve must cancel; dropping it leaves
all of it) and |dP/dt / M - g| <= 1e-3 m/s^2."""
import numpy as np
import pytest

import common
import gpu_harness as G
import momentum_kat as K

pytestmark = pytest.mark.gpu


def test_kernel_flight_conserves_angular_momentum_and_falls_at_g(require_gpu):
    m = K.flight_model()
    st = K.flight_states(16, seed=2)
    e = G.env_with_model(common.MODEL_XML, m, len(st))
    try:
        qpos = np.array([s[0] for s in st])
        qvel = np.array([s[1] for s in st])
        ctrl = np.array([s[2] for s in st])
        _, _, qacc, _ = G.gpu_physics(e, qpos, qvel, np.zeros_like(qvel), ctrl, 1)
        mass = np.array(m.body_mass[1:]).sum()
        worst = 0.0
        for i in range(len(st)):
            dP, dL, dL0 = K.momentum_rates(m, qpos[i], qvel[i], qacc[i])
            assert np.abs(dP / mass - np.array(m.gravity[:])).max() <= 1e-3, dP / mass
            assert np.linalg.norm(dL0) > 1e-3
            worst = max(worst, np.linalg.norm(dL) / np.linalg.norm(dL0))
        print(f"momentum KAT: worst |dL/dt| / |dL0/dt| = {worst:.2e} over {len(st)} flight states")
        assert worst <= 2e-3, worst
    finally:
        e.close()
