"""Known answers for three constructor branches of PupperV3Env (/root/reference/pupperv3_mjx/
environment.py:35-121) that no other test sets, on the oracle (test_gpu_env_branches.py runs the
kernel against the oracle with the same kwargs):

* use_imu=False (environment.py:491-496): the angular-velocity channel is the noise alone and the
  gravity channel is normalize((0,0,-1) + noise) with the identity rotation, whatever the body's
  orientation and spin; with the IMU noise off the lagged channels are exactly (0,0,0, 0,0,-1);
* desired_abduction_angles (rewards.py:85-87, environment.py:420-423): the abduction term is
  scale * sum((q[7:][1::3] - desired)^2) on the post-step joint angles;
* terminal_body_angle (environment.py:384-385): done exactly when the torso's up axis is tilted by
  more than the angle (robots in the air, inside their joint limits, above terminal_body_z).
"""
import numpy as np

import common
from oracle import oracle as O
from pupperv3_mjx import _abi
from pupperv3_mjx.environment import make_keys

ABD = (0.1, -0.1, 0.05, 0.0)


def oracle_env(**over):
    m, cfg, env = common.env_model_and_config(common.MODEL_XML, **over)
    return O.OracleEnv(m, cfg, precision="f64"), env


def tilted(s, angle, axis=(1.0, 0.0, 0.0), spin=(0.0, 0.0, 0.0), z=0.5):
    """The reset state lifted into the air, its base turned by `angle` about `axis` and spinning
    at `spin` (body frame), joints at rest."""
    st = s["state"].copy()
    ax = np.asarray(axis, float) / np.linalg.norm(axis)
    st[_abi.S_QPOS + 2] = z
    st[_abi.S_QPOS + 3:_abi.S_QPOS + 7] = np.concatenate([[np.cos(angle / 2)], np.sin(angle / 2) * ax])
    st[_abi.S_QVEL:_abi.S_QVEL + 18] = 0.0
    st[_abi.S_QVEL + 3:_abi.S_QVEL + 6] = spin
    return dict(state=st, obs=s["obs"].copy())


def test_use_imu_false_channels_are_noise_only():
    oe, _ = oracle_env(use_imu=False, angular_velocity_noise=0.0, gravity_noise=0.0)
    s = oe.reset(make_keys(3, 1)[0])
    np.testing.assert_array_equal(s["obs"][0:6], [0, 0, 0, 0, 0, -1])
    for ang, spin in ((0.7, (3.0, -2.0, 1.0)), (-1.2, (0.0, 5.0, 0.0))):
        out = oe.step(tilted(s, ang, axis=(1, 2, 0.5), spin=spin), np.zeros(12))
        np.testing.assert_array_equal(out["obs"][0:6], [0, 0, 0, 0, 0, -1])


def test_use_imu_false_is_independent_of_the_body_motion():
    """With the IMU noise on, the channels are the noise draws alone: two bodies with different
    orientations and spins, stepped from the same RNG state, read the same IMU channels; the
    angular-velocity part stays inside the noise bound and the gravity part is a unit vector
    within the noise of -z."""
    oe, env = oracle_env(use_imu=False)
    s = oe.reset(make_keys(4, 1)[0])
    a = oe.step(tilted(s, 0.9, axis=(0, 1, 0), spin=(4.0, 0.0, -2.0)), np.zeros(12))
    b = oe.step(tilted(s, -0.4, axis=(1, 0, 1), spin=(0.0, -3.0, 1.0)), np.zeros(12))
    np.testing.assert_array_equal(a["obs"][0:6], b["obs"][0:6])
    imu_a = a["state"][_abi.imu_buf_offset(env.config_struct.latency_len):][:6 * env.config_struct.imu_latency_len]
    imu_a = imu_a.reshape(6, -1)[:, 0]   # the newest (unlagged) IMU sample of this step
    assert np.all(np.abs(imu_a[0:3]) <= 0.3) and np.any(imu_a[0:3] != 0)
    g = imu_a[3:6]
    assert abs(np.linalg.norm(g) - 1) < 1e-12 and np.all(np.abs(g - [0, 0, -1]) <= 0.12)
    # with the IMU on, the same two bodies read different channels (the test can tell)
    oi, _ = oracle_env(use_imu=True)
    si = oi.reset(make_keys(4, 1)[0])
    ai = oi.step(tilted(si, 0.9, axis=(0, 1, 0), spin=(4.0, 0.0, -2.0)), np.zeros(12))
    bi = oi.step(tilted(si, -0.4, axis=(1, 0, 1), spin=(0.0, -3.0, 1.0)), np.zeros(12))
    newest = lambda o: o["state"][_abi.imu_buf_offset(env.config_struct.latency_len):][:12].reshape(6, -1)[:, 0]  # noqa: E731
    assert np.abs(newest(ai) - newest(bi)).max() > 0.5


def test_desired_abduction_angles_term():
    oe, env = oracle_env(desired_abduction_angles=ABD)
    scale = env.config_struct.reward_scales[_abi.REWARD_NAMES.index("abduction_angle")]
    rs = np.random.RandomState(0)
    for i in range(6):
        s = oe.reset(make_keys(10 + i, 1)[0])
        for _ in range(3):
            s = oe.step(s, rs.uniform(-1, 1, 12))
            q = s["state"][_abi.S_QPOS + 7:_abi.S_QPOS + 19]
            want = scale * np.sum((q[1::3] - np.array(ABD)) ** 2)
            got = s["metrics"][1 + _abi.REWARD_NAMES.index("abduction_angle")]
            np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15)
            # the default (zero) targets would give a different value: the kwarg is in effect
            assert abs(scale * np.sum(q[1::3] ** 2) - want) > 1e-6


def test_terminal_body_angle():
    """terminal_body_angle = 0.3 rad: bodies tilted 0.25 rad stay alive, 0.35 rad are done (in the
    air, at rest, default joint pose: no other done condition applies); at the default 0.52 both
    stay alive."""
    for thr, expect in ((0.3, {0.25: 0.0, 0.35: 1.0}), (0.52, {0.25: 0.0, 0.35: 0.0})):
        oe, _ = oracle_env(terminal_body_angle=thr, kick_probability=0.0)
        s = oe.reset(make_keys(5, 1)[0])
        for ang, want in expect.items():
            for axis in ((1, 0, 0), (0, 1, 0), (1, -1, 0)):
                out = oe.step(tilted(s, ang, axis=axis), np.zeros(12))
                assert out["done"] == want, (thr, ang, axis, out["done"])
