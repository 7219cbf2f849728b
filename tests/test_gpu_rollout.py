"""Fused rollout (pp3_rollout / PupperV3Env.rollout): K env steps in one launch, the unroll of
brax's generate_unroll ([ext] brax 0.12.1 training/acting.py, a lax.scan of env.step) with the
actions given up front.  The contract is bit equality with K single-step launches (pp3_step /
PupperV3Env.step, environment.py:348-483): same end state, and per-step trajectories equal to the
reward / done / obs each step() returned -- with kicks, latency, DR and the on-device
EpisodeWrapper + AutoResetWrapper (resets inside the rollout) all on.
"""
import ctypes as C

import numpy as np
import pytest

import common
from pupperv3_mjx import MODEL_XML, _abi, _lib, domain_randomization, wrappers
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu
N = 64


def _env(**kw):
    return PupperV3Env(**common.fixture_kwargs(MODEL_XML, **kw), num_envs=N)


def _steps(env, st, acts):
    obs, rew, done = [], [], []
    for a in acts:
        st = env.step(st, a)
        obs.append(np.array(st.obs))
        rew.append(np.array(st.reward))
        done.append(np.array(st.done))
    return st, {"obs": np.stack(obs), "reward": np.stack(rew), "done": np.stack(done)}


def _check(tr1, tr2, s1, s2):
    for k in ("obs", "reward", "done"):
        np.testing.assert_array_equal(tr1[k], tr2[k], err_msg=k)
    np.testing.assert_array_equal(s1._record, s2._record)
    np.testing.assert_array_equal(s1._metrics_raw, s2._metrics_raw)


def test_rollout_equals_single_steps(require_gpu):
    acts = np.random.RandomState(0).uniform(-1, 1, size=(9, N, 12)).astype(np.float32)
    e1, e2 = _env(kick_probability=0.3), _env(kick_probability=0.3)
    try:
        s1, s2 = e1.reset(make_keys(3, N)), e2.reset(make_keys(3, N))
        s1, tr1 = e1.rollout(s1, acts)
        s2, tr2 = _steps(e2, s2, acts)
        _check(tr1, tr2, s1, s2)
        assert e1.holds(s1)
        # and on from there: a rollout continues a stepped env (and vice versa) seamlessly
        s1, tr1 = e1.rollout(s1, acts[:4])
        s2, tr2 = _steps(e2, s2, acts[:4])
        _check(tr1, tr2, s1, s2)
    finally:
        e1.close()
        e2.close()


def test_rollout_with_dr_and_auto_reset(require_gpu):
    acts = np.random.RandomState(1).uniform(-1, 1, size=(14, N, 12)).astype(np.float32)
    envs = [_env(terminal_body_z=0.3), _env(terminal_body_z=0.3)]
    try:
        ws = []
        for e in envs:
            sys_b, _ = domain_randomization.domain_randomize(e.sys, make_keys(11, N))
            e.set_domain_randomization(sys_b)
            ws.append(wrappers.wrap(e, episode_length=5))
        s1, s2 = ws[0].reset(make_keys(12, N)), ws[1].reset(make_keys(12, N))
        s1, tr1 = ws[0].rollout(s1, acts)
        tr2 = {"obs": [], "reward": [], "done": []}
        for a in acts:
            s2 = ws[1].step(s2, a)
            for k in tr2:
                tr2[k].append(np.array(getattr(s2, k)))
        tr2 = {k: np.stack(v) for k, v in tr2.items()}
        assert tr2["done"].sum() >= N  # every env was reset at least once inside the window
        _check(tr1, tr2, s1, s2)
        for k in ("steps", "truncation"):
            np.testing.assert_array_equal(s1.info[k], s2.info[k])
    finally:
        for e in envs:
            e.close()


def test_rollout_action_repeat_keeps_per_step_launches(require_gpu):
    acts = np.random.RandomState(2).uniform(-1, 1, size=(6, N, 12)).astype(np.float32)
    envs = [_env(), _env()]
    try:
        ws = [wrappers.wrap(e, episode_length=4, action_repeat=2) for e in envs]
        s1, s2 = ws[0].reset(make_keys(13, N)), ws[1].reset(make_keys(13, N))
        s1, tr1 = ws[0].rollout(s1, acts)
        tr2 = {"obs": [], "reward": [], "done": []}
        for a in acts:
            s2 = ws[1].step(s2, a)
            for k in tr2:
                tr2[k].append(np.array(getattr(s2, k)))
        _check(tr1, {k: np.stack(v) for k, v in tr2.items()}, s1, s2)
    finally:
        for e in envs:
            e.close()


def test_rollout_device_stride_zero_and_partial_outputs(require_gpu):
    """action_stride 0 = the same action every step; a NULL trajectory output is skipped."""
    e1, e2 = _env(), _env()
    try:
        s1, s2 = e1.reset(make_keys(14, N)), e2.reset(make_keys(14, N))
        a = np.random.RandomState(3).uniform(-1, 1, size=(N, 12)).astype(np.float32)
        buf = _lib.DeviceBuffer(a.nbytes, e1.device)
        rew = _lib.DeviceBuffer(4 * 5 * N, e1.device)
        try:
            buf.upload(a)
            e1.rollout_device(buf.ptr.value, 0, 5, reward_dev=rew.ptr.value)
            e1.synchronize()
            r = np.empty((5, N), np.float32)
            rew.download(r)
        finally:
            buf.free()
            rew.free()
        _, tr2 = _steps(e2, s2, [a] * 5)
        np.testing.assert_array_equal(r, tr2["reward"])
        np.testing.assert_array_equal(e1._get(_abi.F_STATE), e2._get(_abi.F_STATE))
        with pytest.raises(_lib.PupperHipError):
            _lib.check(e1._L.pp3_rollout(e1._h, C.c_void_p(1), 0, 0, None, None, None, None))
        with pytest.raises(ValueError):
            e1.rollout(s1, np.zeros((3, N, 11), np.float32))
    finally:
        e1.close()
        e2.close()


@pytest.mark.parametrize("cap", [8, 16])
def test_rollout_terrain_pipeline_and_odd_batch(require_gpu, tmp_path, cap):
    """Both kernel instances (contact cap 8 / 16) with per-env terrain under the robots, the
    Brax pipeline record on, and an odd env count (the last wave's second half stores nothing)."""
    n = 65
    path = common.write_model(tmp_path, 10)
    kw = dict(num_envs=n, max_contacts=cap, pipeline_output=True)
    e1, e2 = PupperV3Env(**common.fixture_kwargs(path), **kw), PupperV3Env(**common.fixture_kwargs(path), **kw)
    acts = np.random.RandomState(4).uniform(-1, 1, size=(6, n, 12)).astype(np.float32)
    try:
        s1, s2 = e1.reset(make_keys(15, n)), e2.reset(make_keys(15, n))
        terrain = common.terrain_under(np.asarray(s1.pipeline_state.q)[:, 0:2], 10, seed=5)
        e1.set_terrain(terrain)
        e2.set_terrain(terrain)
        s1, tr1 = e1.rollout(s1, acts)
        s2, tr2 = _steps(e2, s2, acts)
        _check(tr1, tr2, s1, s2)
        np.testing.assert_array_equal(e1._get(_abi.F_PIPELINE), e2._get(_abi.F_PIPELINE))
        ncon = e1._get(_abi.F_PIPELINE)[:, _abi.P_NCON]
        assert ncon.max() > 0
    finally:
        e1.close()
        e2.close()


def test_rollout_long_history_and_latency_buffers(require_gpu):
    """H = 15 (the history window shifts over itself in place, read back across fused steps) with
    4-long action and 3-long IMU latency buffers."""
    kw = common.fixture_kwargs(MODEL_XML, observation_history=15, latency_distribution=[0.1, 0.2, 0.3, 0.4],
                               imu_latency_distribution=[0.2, 0.3, 0.5])
    e1, e2 = PupperV3Env(**kw, num_envs=N), PupperV3Env(**kw, num_envs=N)
    acts = np.random.RandomState(5).uniform(-1, 1, size=(18, N, 12)).astype(np.float32)
    try:
        s1, s2 = e1.reset(make_keys(16, N)), e2.reset(make_keys(16, N))
        assert s1.obs.shape == (N, 36 * 15)
        s1, tr1 = e1.rollout(s1, acts)
        s2, tr2 = _steps(e2, s2, acts)
        _check(tr1, tr2, s1, s2)
    finally:
        e1.close()
        e2.close()
