"""On-device policy (csrc/pp3_policy.hip, f32 MFMA) vs the numpy meaning of the exported JSON
(export.policy_forward, float64).  Tolerance: |d| <= 2e-5 * (1 + |y|) (fp32 products and
accumulation, K <= 540)."""
import ctypes as C

import numpy as np
import pytest

import common
from pupperv3_mjx import _abi, _lib, export
from pupperv3_mjx.environment import PupperV3Env, make_keys
from test_export import _brax_like_params

pytestmark = pytest.mark.gpu


def _policy(sizes, act, seed=0):
    rs = np.random.RandomState(seed)
    return export.convert_params(_brax_like_params(rs, sizes), act, 0.75, 5.0, 0.25, np.zeros(12), np.ones(12),
                                 -np.ones(12), True, (sizes[0] // 36), 30.0, 30.0)


@pytest.mark.parametrize("sizes,act,n", [([72, 256, 128, 128, 24], "elu", 37), ([540, 512, 256, 24], "relu", 64),
                                         ([72, 64, 24], "sigmoid", 16), ([72, 128, 128, 24], "tanh", 1)])
def test_device_policy_matches_numpy(require_gpu, sizes, act, n):
    pol = _policy(sizes, act)
    dp = export.DevicePolicy(pol)
    x = np.random.RandomState(1).normal(size=(n, sizes[0])).astype(np.float32)
    xb = _lib.DeviceBuffer(x.nbytes)
    yb = _lib.DeviceBuffer(n * 12 * 4)
    try:
        xb.upload(x)
        dp.act(xb.ptr.value, sizes[0], n, yb.ptr.value, 12)
        y = np.zeros((n, 12), dtype=np.float32)
        _lib.check(_lib.load().pp3_memcpy_d2h(y.ctypes.data_as(C.c_void_p), yb.ptr, y.nbytes))
        want = export.policy_forward(pol, x.astype(np.float64))
        assert np.all(np.abs(y - want) <= 2e-5 * (1 + np.abs(want))), np.abs(y - want).max()
    finally:
        xb.free(); yb.free(); dp.close()


def test_policy_env_rollout_on_device(require_gpu, tmp_path):
    """policy(obs buffer) -> actions -> env step, 20 times without host round trips."""
    path = common.write_model(tmp_path, 0)
    n = 32
    e = PupperV3Env(**common.fixture_kwargs(path), num_envs=n)
    pol = _policy([72, 128, 128, 24], "elu")
    dp = export.DevicePolicy(pol)
    ab = _lib.DeviceBuffer(n * 12 * 4)
    try:
        st = e.reset(make_keys(0, n))
        dp.act_env(e, ab.ptr.value)
        a = np.zeros((n, 12), dtype=np.float32)
        e.synchronize()
        _lib.check(_lib.load().pp3_memcpy_d2h(a.ctypes.data_as(C.c_void_p), ab.ptr, a.nbytes))
        assert np.all(np.abs(a - export.policy_forward(pol, st.obs)) <= 2e-5 * (1 + np.abs(a)))
        for _ in range(20):
            dp.act_env(e, ab.ptr.value)
            e.step_device(ab.ptr.value)
        e.synchronize()
        assert np.all(np.isfinite(e._get(_abi.F_OBS))) and np.all(np.isfinite(e._get(_abi.F_REWARD)))
    finally:
        ab.free(); dp.close(); e.close()


@pytest.mark.parametrize("n,sizes,H", [(48, [72, 128, 128, 24], 2), (37, [72, 256, 128, 128, 24], 2),
                                       (1, [72, 128, 128, 24], 2), (20, [540, 256, 128, 24], 15)])
def test_rollout_policy_equals_act_then_step(require_gpu, tmp_path, n, sizes, H):
    """pp3_rollout_policy (policy in the loop, ONE fused launch for the K steps: 8-wave workgroups of
    16 envs run the MLP before every step) equals the Python loop DevicePolicy.act_env (the
    stand-alone policy kernel) + step, bit for bit, with auto-reset inside the window; batches that
    fill no whole workgroup (37, 1 envs) and observation_history 15 (540 inputs) included."""
    from pupperv3_mjx import wrappers
    path = common.write_model(tmp_path, 0)
    K = 12
    envs = [PupperV3Env(**common.fixture_kwargs(path, terminal_body_z=0.25, observation_history=H), num_envs=n)
            for _ in range(2)]
    pol = _policy(sizes, "elu")
    dp = export.DevicePolicy(pol)
    ab = _lib.DeviceBuffer(n * 12 * 4)
    try:
        ws = [wrappers.wrap(e, episode_length=5) for e in envs]
        s1, s2 = ws[0].reset(make_keys(2, n)), ws[1].reset(make_keys(2, n))
        s1, tr = ws[0].rollout_policy(s1, dp, K)
        acts, obs, rew, done = [], [], [], []
        for _ in range(K):
            dp.act_env(envs[1], ab.ptr.value)
            a = np.zeros((n, 12), dtype=np.float32)
            envs[1].synchronize()
            _lib.check(_lib.load().pp3_memcpy_d2h(a.ctypes.data_as(C.c_void_p), ab.ptr, a.nbytes))
            s2 = ws[1].step(s2, a)
            acts.append(a); obs.append(np.array(s2.obs)); rew.append(np.array(s2.reward)); done.append(np.array(s2.done))
        np.testing.assert_array_equal(tr["action"], np.stack(acts))
        np.testing.assert_array_equal(tr["obs"], np.stack(obs))
        np.testing.assert_array_equal(tr["reward"], np.stack(rew))
        np.testing.assert_array_equal(tr["done"], np.stack(done))
        assert tr["done"].sum() > 0 or n == 1
        np.testing.assert_array_equal(s1._record, s2._record)
    finally:
        ab.free(); dp.close()
        for e in envs:
            e.close()


def test_rollout_policy_with_dr_and_terrain_equals_act_then_step(require_gpu, tmp_path):
    """The fused policy rollout on domain-randomised envs (each env its own DR row) standing on
    per-env terrain (the sphere-box lanes index the terrain rows by env, with 16 envs per
    workgroup here): bit-equal to the per-step policy + step launches."""
    from pupperv3_mjx import domain_randomization, rng
    path = common.write_model(tmp_path, 10)
    n, K = 40, 10
    envs = [PupperV3Env(**common.fixture_kwargs(path), num_envs=n) for _ in range(2)]
    pol = _policy([72, 256, 128, 128, 24], "elu")
    dp = export.DevicePolicy(pol)
    ab = _lib.DeviceBuffer(n * 12 * 4)
    try:
        sysb, _ = domain_randomization.domain_randomize(envs[0].sys, rng.split(rng.PRNGKey(3), n))
        states = []
        for e in envs:
            e.set_domain_randomization(sysb)
            st = e.reset(make_keys(4, n))
            xy = st._record[:, _abi.S_QPOS:_abi.S_QPOS + 2].astype(np.float64)
            e.set_terrain(common.terrain_under(xy, 10, seed=5))
            states.append(st)
        s1, tr = envs[0].rollout_policy(states[0], dp, K)
        s2 = states[1]
        acts = []
        for _ in range(K):
            dp.act_env(envs[1], ab.ptr.value)
            a = np.zeros((n, 12), dtype=np.float32)
            envs[1].synchronize()
            _lib.check(_lib.load().pp3_memcpy_d2h(a.ctypes.data_as(C.c_void_p), ab.ptr, a.nbytes))
            s2 = envs[1].step(s2, a)
            acts.append(a)
        np.testing.assert_array_equal(tr["action"], np.stack(acts))
        np.testing.assert_array_equal(s1._record, s2._record)
        np.testing.assert_array_equal(s1.obs, s2.obs)
        assert s1.pipeline_state.contact.ncon.sum() > 0
    finally:
        ab.free(); dp.close()
        for e in envs:
            e.close()
