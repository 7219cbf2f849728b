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


def test_kernel_domain_randomised_flight_uses_the_rows_fields(require_gpu):
    """The DR known answer (test_momentum_kat.py) on the kernel: each env's step is the dynamics
    of the model with its DR row written into body_mass / body_inertia / body_ipos[1], and its PD
    torque uses the row's Kp / Kd (fp32: as above, torques 2e-6 N m)."""
    import test_actuator_kat as A
    from pupperv3_mjx import _abi
    m = K.flight_model()
    st = K.flight_states(16, seed=4)
    out = K.dr_rows(16, seed=6)
    table = out.dr_table().astype(np.float64)
    e = G.env_with_model(common.MODEL_XML, m, len(st))
    try:
        e.set_domain_randomization(out)
        qpos = np.array([s[0] for s in st])
        qvel = np.array([s[1] for s in st])
        ctrl = np.array([s[2] for s in st])
        _, _, qacc, pipes = G.gpu_physics(e, qpos, qvel, np.zeros_like(qvel), ctrl, 1)
        worst = worst_f = 0.0
        for i in range(len(st)):
            me = K.dr_edited(m, table[i])
            dP, dL, dL0 = K.momentum_rates(me, qpos[i], qvel[i], qacc[i])
            assert np.abs(dP / np.array(me.body_mass[1:]).sum() - np.array(m.gravity[:])).max() <= 1e-3
            worst = max(worst, np.linalg.norm(dL) / np.linalg.norm(dL0))
            kp, kd = table[i, _abi.DR_KP], table[i, _abi.DR_KD]
            want = np.clip(kp * (ctrl[i] - qpos[i, 7:]) - kd * qvel[i, 6:], -A.FMAX, A.FMAX)
            worst_f = max(worst_f, np.abs(pipes[i, _abi.P_QFRC_ACT + 6:_abi.P_QFRC_ACT + 18] - want).max())
        print(f"DR KAT: worst |dL/dt| / |dL0/dt| = {worst:.2e}, worst torque error {worst_f:.2e} N m")
        assert worst <= 2e-3 and worst_f <= 2e-6, (worst, worst_f)
    finally:
        e.close()
