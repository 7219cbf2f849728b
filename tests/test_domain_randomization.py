"""test_domain_randomization.py:15-102 re-expressed (ranges, shapes) + DR record packing."""
import numpy as np

import common
from pupperv3_mjx import _abi, domain_randomization as dr, rng


def _sys():
    _, _, env = common.env_model_and_config(common.MODEL_XML)
    return env.sys


def test_randomize_qpos():
    cfg = dr.StartPositionRandomization(x_min=-0.5, x_max=0.5, y_min=-0.5, y_max=0.5, z_min=-0.5, z_max=0.5)
    key = rng.PRNGKey(0)
    for _ in range(100):
        key, sub = rng.split(key)
        q = dr.randomize_qpos(np.arange(11, dtype=np.float32), cfg, sub)
        assert -0.5 <= q[0] <= 0.5 and -0.5 <= q[1] <= 0.5 and -0.5 <= q[2] <= 0.5
        assert abs(np.linalg.norm(q[3:7]) - 1) < 1e-6 and q[4] == 0 and q[5] == 0


def test_domain_randomize_shapes_and_ranges():
    sys = _sys()
    kp0 = sys.actuator_gainprm[:, 0]
    kd0 = -sys.actuator_biasprm[:, 2]
    rngs = rng.split(rng.PRNGKey(0), 10)
    out, in_axes = dr.domain_randomize(sys, rngs, friction_range=(2.0, 10.0), kp_multiplier_range=(1.1, 1.25),
                                       kd_multiplier_range=(1.5, 2.0), body_com_x_shift_range=(0.02, 0.04),
                                       body_com_y_shift_range=(0.02, 0.04), body_com_z_shift_range=(0.02, 0.04),
                                       body_inertia_scale_range=(1.5, 2.0), body_mass_scale_range=(1.5, 2.0))
    assert out.geom_friction.shape == (10, 23, 3)
    assert out.actuator_gainprm.shape == (10, 12, 10) and out.actuator_biasprm.shape == (10, 12, 10)
    assert np.all((out.geom_friction[:, :, 0] >= 2.0) & (out.geom_friction[:, :, 0] <= 10.0))
    assert np.all(out.actuator_gainprm[:, :, 0] >= 1.1 * kp0 - 1e-6) and np.all(out.actuator_gainprm[:, :, 0] <= 1.25 * kp0 + 1e-6)
    assert np.all(-out.actuator_biasprm[:, :, 2] >= 1.5 * kd0 - 1e-6) and np.all(-out.actuator_biasprm[:, :, 2] <= 2.0 * kd0 + 1e-6)
    assert np.all(out.body_inertia[:, 1] >= 1.5 * sys.body_inertia[1] - 1e-9)
    assert np.all(out.body_inertia[:, 1] <= 2.0 * sys.body_inertia[1] + 1e-9)
    assert np.all(out.body_mass[:, 1] >= 1.5 * sys.body_mass[1] - 1e-6) and np.all(out.body_mass[:, 1] <= 2.0 * sys.body_mass[1] + 1e-6)
    d = out.body_ipos[:, 1] - sys.body_ipos[1]
    assert np.all(d >= 0.02 - 1e-6) and np.all(d <= 0.04 + 1e-6)
    assert all(v == 0 for v in in_axes.values()) and len(in_axes) == 6
    # every env got its own draw, and the kp multiplier is shared by all 12 actuators
    assert len(np.unique(out.geom_friction[:, 0, 0])) == 10
    assert np.allclose(out.actuator_gainprm[:, :, 0], out.actuator_gainprm[:, :1, 0])


def test_dr_table_layout_and_determinism():
    sys = _sys()
    keys = rng.split(rng.PRNGKey(5), 7)
    out, _ = dr.domain_randomize(sys, keys)
    t = out.dr_table()
    assert t.shape == (7, _abi.NDR) and t.dtype == np.float32
    np.testing.assert_array_equal(t[:, _abi.DR_FRICTION], out.geom_friction[:, 0, 0])
    np.testing.assert_array_equal(t[:, _abi.DR_MASS:_abi.DR_MASS + 14], out.body_mass)
    np.testing.assert_array_equal(t[:, _abi.DR_BASE_IPOS:_abi.DR_BASE_IPOS + 3], out.body_ipos[:, 1])
    out2, _ = dr.domain_randomize(sys, keys)
    np.testing.assert_array_equal(out2.dr_table(), t)
    # defaults of domain_randomization.py:11-18
    assert np.all((t[:, 0] >= 0.6) & (t[:, 0] <= 1.4))
    assert np.all((t[:, 1] >= 0.75 * 5.0) & (t[:, 1] <= 1.25 * 5.0))
    assert np.all((t[:, 2] >= 0.5 * 0.25) & (t[:, 2] <= 2.0 * 0.25))
