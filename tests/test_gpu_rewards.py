"""GPU parity of every reward term, the env state record and the info-update branches.

Reference: environment.py:374-482 (contacts, done, the 18-term rewards_dict, info update incl.
the command/orientation resample branch with its shared cmd_rng), rewards.py:9-138.

Each compared step starts from the GPU's own previous state (the oracle is re-synced), so one
step of fp32 error is measured.  Every one of the 18 scaled terms of ``state.metrics`` (and
``total_dist``) is compared on its own with the tolerance of ``gpu_harness.metric_errors``
(relative 2e-3 plus a per-term absolute floor; termination and the collision counts exact), as
is every info field of the state record (``gpu_harness.state_errors``: last_act, command, kick,
step, action buffer and last_contact exact; air time 1e-6; last_vel 2e-3 + 1e-3 relative; IMU
buffer 5e-3).
A step may fail only where the oracle flagged a constraint row on its switch point or a foot
height sits on a contact threshold (both discrete flips), at most 1 % of steps.  The worst error
per term is reported (``REPORT`` lines / $PP3_REPORT_DIR/gpu_reports.jsonl).
"""
import numpy as np
import pytest

import common
import gpu_harness as G
from oracle import oracle as O
from pupperv3_mjx import _abi, config
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu
N = 32


@pytest.fixture(scope="module")
def model_path(require_gpu, tmp_path_factory):
    return common.write_model(tmp_path_factory.mktemp("m"), 0)


def all_ones_config():
    """Every reward scale 1.0 (mechanical_work included): every term is visible in the metrics
    and, all raw terms being >= 0, in the clipped total (no clip at 0)."""
    cfg = config.get_config()
    for k in list(cfg.rewards.scales.keys()):
        cfg.rewards.scales[k] = 1.0
    return cfg


def _make(model_path, n=N, **over):
    return PupperV3Env(**common.fixture_kwargs(model_path, **over), num_envs=n)


def _compare_step(env, oe, prev, st, a, i, stats):
    """Compare env i of GPU step prev -> st with the oracle step from prev; returns
    (ok, oracle output, failure description)."""
    o = oe.step(dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64)),
                a[i].astype(np.float64))
    orec = G.oracle_state_to_record(o["state"])
    # RNG-decided fields are bit-exact always (no physics in them)
    np.testing.assert_array_equal(st._record[i, _abi.S_RNG:_abi.S_RNG + 2].view(np.uint32),
                                  orec[_abi.S_RNG:_abi.S_RNG + 2].view(np.uint32))
    np.testing.assert_array_equal(st._record[i, _abi.S_KICK:_abi.S_KICK + 2], orec[_abi.S_KICK:_abi.S_KICK + 2])
    scales = np.array(env.config_struct.reward_scales[:])
    merr = G.metric_errors(st._metrics_raw[i], o["metrics"], scales)
    serr = G.state_errors(st._record[i], orec, env.config_struct.latency_len, env.config_struct.imu_latency_len)
    allowed_r = env.dt * sum(tol for k, (_, tol) in merr.items() if k != "total_dist") + 1e-6
    extra = {"reward": (abs(float(st.reward[i]) - o["reward"]), allowed_r),
             "done": (abs(float(st.done[i]) - o["done"]), 0.0),
             "obs": (float(np.abs(st.obs[i] - o["obs"]).max()), 5e-3)}
    errs = {**merr, **serr, **extra}
    stats.nonzero.update(k for k in _abi.REWARD_NAMES if st.metrics[k][i] != 0)
    bad = G.TermStats.failures(errs)
    if not bad:
        stats.add(errs)
    flip = o["boundary"] > 0 or G.foot_threshold_flip(o["pipe"], env.config_struct.foot_radius)
    return not bad, dict(o, boundary=int(flip)), bad


def _rollout_parity(env, keys, steps, seed, name, prep=None, max_frac=0.01):
    st = env.reset(keys)
    oe = O.OracleEnv(env.sys_model.struct, env.config_struct, precision="f32")
    rs = np.random.RandomState(seed)
    stats = G.TermStats()
    fb = G.FlipBudget(max_frac=max_frac, name=name)
    n = env.num_envs
    for t in range(steps):
        if prep is not None:  # edit the info, then re-read so the oracle starts from the edited record
            prep(t, st)
            env._write_state(st)
            st = env._issue(False)
        a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
        prev = st
        st = env.step(prev, a)
        for i in range(n):
            ok, o, bad = _compare_step(env, oe, prev, st, a, i, stats)
            fb.check(ok, o, f"step {t} env {i}: {bad}")
    G.report(name, {"worst": {k: float(f"{v:.3g}") for k, v in stats.worst.items()}})
    fb.finish()
    return stats


def test_reward_terms_and_state_record(model_path):
    """Fixture config (test_environment.py:64-113): 40 steps x 32 envs, every term and field."""
    e = _make(model_path)
    try:
        stats = _rollout_parity(e, make_keys(21, N), 40, 3, "reward_terms_fixture")
        # the rollout must actually exercise the terms it claims to compare: every term with a
        # nonzero fixture scale is nonzero on at least one env.  Excepted: body_collision (the test
        # model's torso is a visual mesh, no pair can exist), termination (test_termination_gate)
        # and the two stand_still terms (they need a near-zero command, which the fixture's
        # sampled commands do not give: test_all_reward_scales_one zeroes a third of them)
        scales = dict(zip(_abi.REWARD_NAMES, e.config_struct.reward_scales[:]))
        expected = {k for k, v in scales.items() if v != 0} - {"body_collision", "termination", "stand_still",
                                                                "stand_still_joint_velocity"}
        missing = expected - stats.nonzero
        assert not missing, f"terms never nonzero in the rollout: {sorted(missing)}"
    finally:
        e.close()


def test_all_reward_scales_one(model_path):
    """Every scale 1.0 (mechanical_work included), so no term hides under another's scale or
    under the clip at 0: per-term parity and the unclipped total."""
    e = _make(model_path, reward_config=all_ones_config())

    def prep(t, st):
        # zero command on a third of the envs: the stand_still terms are active there
        c = st.info["command"].copy()  # (State arrays are read-only, like the reference's jax arrays)
        c[::3] = 0.0
        st.info["command"] = c

    try:
        stats = _rollout_parity(e, make_keys(22, N), 30, 4, "reward_terms_scales_one", prep=prep)
        silent = [k for k in _abi.REWARD_NAMES if k not in stats.nonzero]
        # body_collision: the test model's torso geom is a visual mesh (no pair can exist);
        # termination: no env falls within 30 steps here (pinned by test_termination_gate)
        assert set(silent) <= {"body_collision", "termination"}, silent
    finally:
        e.close()


def test_resample_branch_shared_cmd_rng(model_path):
    """environment.py:455-474: when step+1 > resample_velocity_step the command AND the desired
    orientation are redrawn from the SAME cmd_rng, and step restarts at 0.  Half the envs sit
    at step = resample_velocity_step (resample), half one below (no resample)."""
    rvs = 100
    e = _make(model_path, resample_velocity_step=rvs)
    try:
        st = e.reset(make_keys(31, N))
        st.info["step"] = np.where(np.arange(N) % 2 == 0, rvs, rvs - 1).astype(st.info["step"].dtype)
        old_cmd = st.info["command"].copy()
        a = np.random.RandomState(5).uniform(-1, 1, size=(N, 12)).astype(np.float32)
        e._write_state(st)
        prev = e._issue(False)
        out = e.step(prev, a)
        oe = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f32")
        for i in range(N):
            o = oe.step(dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64)),
                        a[i].astype(np.float64))
            orec = G.oracle_state_to_record(o["state"])
            np.testing.assert_array_equal(out._record[i, _abi.S_COMMAND:_abi.S_COMMAND + 3],
                                          orec[_abi.S_COMMAND:_abi.S_COMMAND + 3])
            np.testing.assert_allclose(out._record[i, _abi.S_DESIRED_Z:_abi.S_DESIRED_Z + 3],
                                       orec[_abi.S_DESIRED_Z:_abi.S_DESIRED_Z + 3], atol=1e-6)
            assert out._record[i, _abi.S_STEP] == orec[_abi.S_STEP]
        resampled = np.arange(N) % 2 == 0
        assert np.all(out.info["step"][resampled] == 0)
        assert np.all(out.info["step"][~resampled & (out.done == 0)] == rvs)
        assert np.all(np.any(out.info["command"][resampled] != old_cmd[resampled], axis=1))
        np.testing.assert_array_equal(out.info["command"][~resampled], old_cmd[~resampled])
        # max pitch/roll 30 deg in the fixture: the new desired orientation is not the default
        assert np.all(np.abs(out.info["desired_world_z_in_body_frame"][resampled, 2] - 1.0) > 0)
    finally:
        e.close()


def _tilted_state(e, keys, steps_info):
    st = e.reset(keys)
    q = st.pipeline_state.q.copy()
    q[:, 2] = 0.5                                         # in the air: no contacts
    q[:, 3:7] = [np.cos(np.pi / 4), np.sin(np.pi / 4), 0, 0]  # rolled 90 deg: done by tilt (:384-385)
    st.pipeline_state.q = q
    st.pipeline_state.qd = np.zeros_like(st.pipeline_state.qd)
    st.info["step"] = (np.zeros_like(st.info["step"]) + steps_info).astype(st.info["step"].dtype)
    return st


def test_termination_gate(model_path):
    """rewards.py:127-128: termination = done & (step < early_termination_step_threshold) with
    the step BEFORE the increment; the counter restarts at 0 on done (environment.py:471-474)."""
    thr = 500
    e = _make(model_path, early_termination_step_threshold=thr, resample_velocity_step=10 ** 6)
    try:
        steps = np.where(np.arange(N) % 2 == 0, thr - 1, thr)
        st = _tilted_state(e, make_keys(41, N), steps)
        a = np.zeros((N, 12), np.float32)
        e._write_state(st)
        prev = e._issue(False)
        out = e.step(prev, a)
        oe = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f32")
        it = 1 + _abi.REWARD_NAMES.index("termination")
        for i in range(N):
            o = oe.step(dict(state=G.record_to_oracle_state(prev._record[i]), obs=prev.obs[i].astype(np.float64)),
                        a[i].astype(np.float64))
            assert out.done[i] == o["done"] == 1.0
            assert out.metrics["termination"][i] == np.float32(o["metrics"][it])
            assert out.info["step"][i] == 0
        np.testing.assert_array_equal(out.metrics["termination"], np.where(steps < thr, -100.0, 0.0))
        # the clipped total reward is 0 where the -100 term applies
        assert np.all(out.reward[steps < thr] == 0.0)
    finally:
        e.close()


def test_zero_command_probability(model_path):
    """environment.py:262-270: with probability zero_command_probability the command is
    U(+-stand_still_command_threshold)^3 instead of the ranges; at p = 1 every reset and every
    resample takes that branch, bit-exact against the oracle, and the stand_still terms act."""
    e = _make(model_path, zero_command_probability=1.0, resample_velocity_step=3)
    try:
        keys = make_keys(51, N)
        st = e.reset(keys)
        oe = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f32")
        for i in range(N):
            orr = G.oracle_state_to_record(oe.reset(keys[i])["state"])
            np.testing.assert_array_equal(st.info["command"][i], orr[_abi.S_COMMAND:_abi.S_COMMAND + 3])
        assert np.all(np.abs(st.info["command"]) <= 0.1)
        stats = _rollout_parity(e, keys, 8, 6, "reward_terms_zero_command")
        assert "stand_still" in stats.worst
    finally:
        e.close()


def test_obs_pointer_stable_across_steps(model_path):
    """pp3_field(PP3_F_OBS) returns one buffer updated in place (include/pupper_hip.h): a
    pointer taken before two steps reads the newest observation after them."""
    import ctypes as C
    from pupperv3_mjx import _lib
    e = _make(model_path, n=4)
    try:
        st = e.reset(make_keys(61, 4))
        ptr0, n_per = e.device_field(_abi.F_OBS)
        a = np.zeros((4, 12), np.float32)
        st = e.step(st, a)
        st = e.step(st, a)
        assert e.device_field(_abi.F_OBS)[0] == ptr0
        # step() returns before its launch completes: a raw read of the device buffer (not through
        # the State) synchronises with the env's stream first
        e.synchronize()
        host = np.empty((4, n_per), np.float32)
        _lib.check(e._L.pp3_memcpy_d2h(host.ctypes.data_as(C.c_void_p), C.c_void_p(ptr0), host.nbytes))
        np.testing.assert_array_equal(host, st.obs)
        # history: the second frame is the previous step's newest frame
        assert np.all(np.isfinite(host))
    finally:
        e.close()
