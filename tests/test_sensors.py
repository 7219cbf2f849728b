"""Site sensors of test_pupper_model.xml (xml:14-23) in the CPU oracle.

MuJoCo is absent, so the restated mj_sensorPos/Vel/Acc are pinned by physics known answers:
  * free fall (no contact, no motion): accelerometer = 0, gyro = 0;
  * robot settled on the floor: accelerometer = R^T (0, 0, 9.81) (gravity reaction), gyro ~ 0;
  * spinning free flight: the accelerometer equals the finite difference of the site's world
    velocity (framelinvel) over one substep, rotated into the site frame, plus the gravity term;
  * frame sensors equal the kinematics the pipeline record already carries.
"""
import numpy as np

import common
from oracle import oracle as O
from pupperv3_mjx import MODEL_XML, _abi, mjcf

ADR = dict(body_quat=0, body_gyro=4, body_acc=7, orientation=10, global_position=14, global_linvel=17,
           global_angvel=20)


def _sens(pipe, name, n=3):
    a = _abi.P_SENSOR + ADR[name]
    return pipe[a:a + n]


def _quat2mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def test_sensor_table_compiled():
    cm = mjcf.load(MODEL_XML)
    m = cm.struct
    assert cm.sensor_names == list(ADR)
    assert m.nsensordata == 23
    assert [m.sensor_adr[i] for i in range(7)] == list(ADR.values())
    assert [m.sensor_type[i] for i in range(7)] == [_abi.SENS_FRAMEQUAT, _abi.SENS_GYRO, _abi.SENS_ACCELEROMETER,
                                                   _abi.SENS_FRAMEQUAT, _abi.SENS_FRAMEPOS, _abi.SENS_FRAMELINVEL,
                                                   _abi.SENS_FRAMEANGVEL]
    assert O.PIPE_STRIDE == _abi.PIPE_STRIDE


def _home(z):
    q = np.zeros(19)
    q[2], q[3] = z, 1.0
    q[7:] = common.DEFAULT_POSE
    return q


def test_free_fall_reads_zero():
    m = mjcf.load(MODEL_XML).struct
    q = _home(1.0)
    _, _, _, p, _ = O.mj_step(m, q, np.zeros(18), np.zeros(18), q[7:].copy(), nsteps=1)
    np.testing.assert_allclose(_sens(p, "body_acc"), 0, atol=1e-9)
    np.testing.assert_allclose(_sens(p, "body_gyro"), 0, atol=1e-12)


def test_resting_robot_reads_gravity_reaction():
    m = mjcf.load(MODEL_XML).struct
    q, v, w = _home(0.2), np.zeros(18), np.zeros(18)
    for _ in range(10):  # 2 s of PD standing: settles on the floor
        q, v, w, p, _ = O.mj_step(m, q, v, w, np.array(common.DEFAULT_POSE), nsteps=50)
    R = _quat2mat(_sens(p, "body_quat", 4))
    np.testing.assert_allclose(_sens(p, "body_acc"), R.T @ np.array([0, 0, 9.81]), atol=0.05)
    assert np.abs(_sens(p, "body_gyro")).max() < 0.02


def test_accelerometer_matches_finite_difference_in_free_flight():
    m = mjcf.load(MODEL_XML).struct
    rs = np.random.RandomState(0)
    h = m.timestep
    for trial in range(3):
        q = _home(2.0)
        v = np.zeros(18)
        v[0:3] = rs.uniform(-1, 1, 3)
        v[3:6] = rs.uniform(-3, 3, 3)  # spinning: centripetal + rotating-frame terms
        ctrl = q[7:].copy()
        q1, v1, w1, p0, _ = O.mj_step(m, q, v, np.zeros(18), ctrl, nsteps=1)
        _, _, _, p1, _ = O.mj_step(m, q1, v1, w1, ctrl, nsteps=1)
        a_fd = (_sens(p1, "global_linvel") - _sens(p0, "global_linvel")) / h
        R0 = _quat2mat(_sens(p0, "body_quat", 4))
        a_sensor = R0 @ _sens(p0, "body_acc") - np.array([0, 0, 9.81])
        np.testing.assert_allclose(a_sensor, a_fd, atol=0.01 * (1 + np.abs(a_fd).max()))  # O(h) agreement


def test_frame_sensors_match_kinematics():
    m = mjcf.load(MODEL_XML).struct
    qpos, qvel, qws, ctrl = common.random_physics_states(8, seed=4)
    for i in range(8):
        _, _, _, p, sites = O.mj_step(m, qpos[i], qvel[i], qws[i], ctrl[i], nsteps=1)
        quat = p[_abi.P_XQUAT:_abi.P_XQUAT + 4]  # body 1 (the IMU site's body; identity site quat)
        np.testing.assert_allclose(_sens(p, "body_quat", 4), quat, atol=1e-12)
        np.testing.assert_allclose(_sens(p, "orientation", 4), quat, atol=1e-12)
        w = p[_abi.P_XD_ANG:_abi.P_XD_ANG + 3]
        np.testing.assert_allclose(_sens(p, "global_angvel"), w, atol=1e-12)
        R = _quat2mat(quat)
        np.testing.assert_allclose(_sens(p, "body_gyro"), R.T @ w, atol=1e-9)
        # site velocity = body-origin velocity + w x (site - body origin)
        xb = p[_abi.P_XPOS:_abi.P_XPOS + 3]
        sp = _sens(p, "global_position")
        vb = p[_abi.P_XD_VEL:_abi.P_XD_VEL + 3]
        np.testing.assert_allclose(_sens(p, "global_linvel"), vb + np.cross(w, sp - xb), atol=1e-9)
        np.testing.assert_allclose(sp, xb + R @ np.array([0.09, 0, 0.032]), atol=1e-12)
