"""The actuator known answer (test_actuator_kat.py) through the kernel: qfrc_actuator in the
pipeline record equals clip(Kp (ctrl - q) - Kd qd, -3, 3) on every hinge (fp32: 2e-6 N m)."""
import numpy as np
import pytest

import common
import gpu_harness as G
import test_actuator_kat as A
from pupperv3_mjx import _abi

pytestmark = pytest.mark.gpu


def test_kernel_pd_torque_equals_closed_form(require_gpu):
    m = common.pd_model().struct
    q, v, ctrl = A.actuator_states(64, seed=1)
    e = G.env_with_model(common.MODEL_XML, m, 64)
    try:
        _, _, _, pipes = G.gpu_physics(e, q, v, np.zeros((64, 18)), ctrl, 1)
        f = pipes[:, _abi.P_QFRC_ACT:_abi.P_QFRC_ACT + 18]
        err = np.abs(f[:, 6:] - A.expected(q, v, ctrl)).max()
        print(f"actuator KAT: worst |qfrc_actuator - closed form| = {err:.2e} N m")
        assert err <= 2e-6 and np.all(f[:, :6] == 0)
    finally:
        e.close()
