"""PupperV3Env's public helpers other than reset/step (environment.py:246-312): sample_command,
sample_body_orientation, initial_action_buffer, initial_imu_buffer, on the host.

The commands and orientations must be the draws the reset makes from its command / orientation
keys (environment.py:315-321: split(rng, 4)[1] and [2]); the oracle's reset restates that
(pp3_oracle.c sample_command / sample_orientation) and the GPU reset parity tests pin the device
to the oracle, so host == oracle here closes host == device."""
import numpy as np
import pytest

import common
from oracle import oracle as O
from pupperv3_mjx import _abi, rng
from pupperv3_mjx.environment import make_keys


@pytest.fixture(scope="module")
def model_path(tmp_path_factory):
    return common.write_model(tmp_path_factory.mktemp("helpers"))


@pytest.mark.parametrize("zero_p", [0.01, 1.0])
def test_sample_command_and_orientation_match_reset_draws(model_path, zero_p):
    m, cfg, env = common.env_model_and_config(model_path, zero_command_probability=zero_p,
                                              maximum_pitch_command=30, maximum_roll_command=20)
    keys = make_keys(3, 24)
    sub = rng.split(keys, 4)                      # reset: rng, command key, orientation key, pose key
    cmd = env.sample_command(sub[:, 1])
    dz = env.sample_body_orientation(sub[:, 2])
    assert cmd.shape == (24, 3) and cmd.dtype == np.float32 and dz.shape == (24, 3)
    oe = O.OracleEnv(m, cfg)
    for i, k in enumerate(keys):
        st = oe.reset(k)["state"]
        np.testing.assert_array_equal(cmd[i], st[_abi.S_COMMAND:_abi.S_COMMAND + 3].astype(np.float32))
        np.testing.assert_allclose(dz[i], st[_abi.S_DESIRED_Z:_abi.S_DESIRED_Z + 3], atol=2e-7)
    # one key at a time gives the batch's rows
    np.testing.assert_array_equal(env.sample_command(sub[5, 1]), cmd[5])
    if zero_p == 1.0:
        assert np.abs(cmd).max() <= 0.1
    else:
        lo = np.array([-0.75, -0.5, -2.0])
        assert np.all(cmd >= lo) and np.all(cmd <= -lo)
    np.testing.assert_allclose(np.linalg.norm(dz, axis=-1), 1.0, atol=1e-6)
    tilt = np.degrees(np.arccos(np.clip(dz[:, 2], -1, 1)))
    assert tilt.max() <= np.hypot(30, 20) + 1e-3


def test_initial_buffers(model_path):
    _, _, env = common.env_model_and_config(model_path, latency_distribution=[0.2, 0.5, 0.3],
                                            imu_latency_distribution=[0.5, 0.5])
    a = env.initial_action_buffer()
    assert a.shape == (12, 3) and not a.any()
    b = env.initial_imu_buffer()
    assert b.shape == (6, 2)
    np.testing.assert_array_equal(b[5], [-1, -1])
    assert not b[:5].any()


@pytest.mark.gpu
def test_device_reset_draws_equal_host_helpers(require_gpu, model_path):
    """The kernel's reset (env_reset_kernel) draws the same command (bit-exact) and orientation as
    env.sample_command / env.sample_body_orientation on the reset's sub-keys."""
    from pupperv3_mjx.environment import PupperV3Env
    n = 33
    env = PupperV3Env(**common.fixture_kwargs(model_path, maximum_pitch_command=30, maximum_roll_command=20),
                      num_envs=n)
    try:
        keys = make_keys(11, n)
        st = env.reset(keys)
        sub = rng.split(keys, 4)
        np.testing.assert_array_equal(st.info["command"], env.sample_command(sub[:, 1]))
        np.testing.assert_allclose(st.info["desired_world_z_in_body_frame"], env.sample_body_orientation(sub[:, 2]),
                                   atol=1e-6)
    finally:
        env.close()
