"""On-device Brax EpisodeWrapper + AutoResetWrapper (pupperv3_mjx.wrappers)
against a restatement of the same wrapper logic ([ext] brax 0.12.1 brax/envs/wrappers/
training.py, not vendored: parity unpinned against Brax itself) over the CPU oracle env.

Checks per step (oracle re-synced to the GPU state every step):
  * episode counter, truncation flag, done (env done | counter >= episode_length): exact;
  * on done steps qpos|qvel|qacc_warmstart and obs are the env's first (reset) state: exact;
  * episode sum_reward / length (reset after a done step): reward tolerance 1e-3 per step;
  * the env's own info keeps running (rng words follow the env step, exact).
"""
import numpy as np
import pytest

import common
import gpu_harness as G
from oracle import oracle as O
from pupperv3_mjx import _abi, wrappers
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu


def _oracle_wrapped_step(oe, rec, obs, action, ep, prev_done, first_state, first_obs, L):
    keep = 1.0 - prev_done
    o = oe.step(dict(state=G.record_to_oracle_state(rec), obs=obs.astype(np.float64)), action.astype(np.float64))
    steps = ep[_abi.EP_STEPS] * keep + 1.0
    hit = steps >= L
    done = bool(o["done"]) or hit
    trunc = 1.0 if (hit and not o["done"]) else 0.0
    out_rec = G.oracle_state_to_record(o["state"])
    out_obs = o["obs"].astype(np.float32)
    if done:
        out_rec[0:_abi.FIRST_STRIDE] = first_state
        out_obs = first_obs.copy()
    ep_new = np.array([steps, trunc, (ep[_abi.EP_SUM_REWARD] + o["reward"]) * keep, (ep[_abi.EP_LENGTH] + 1) * keep])
    return out_rec, out_obs, float(done), ep_new, o


@pytest.mark.parametrize("episode_length,terminal_z,nsteps", [(7, 0.1, 16), (1000, 0.3, 16), (1000, 0.12, 40)])
def test_auto_reset_episode_semantics(require_gpu, tmp_path, episode_length, terminal_z, nsteps):
    """(7, 0.1): truncations; (1000, 0.3): every env terminates at every step (terminal height above
    every start height), so only the reset path is compared; (1000, 0.12): terminations mixed with
    surviving envs, whose obs / reward are compared on the non-done path (at least 50 env steps)."""
    path = common.write_model(tmp_path, 0)
    n = 8
    e = PupperV3Env(**common.fixture_kwargs(path, terminal_body_z=terminal_z), num_envs=n)
    try:
        env = wrappers.wrap(e, episode_length=episode_length)
        st = env.reset(make_keys(3, n))
        first_state = e._get(_abi.F_FIRST_STATE)
        first_obs = e._get(_abi.F_FIRST_OBS)
        np.testing.assert_array_equal(first_state, st._record[:, 0:_abi.FIRST_STRIDE])
        np.testing.assert_array_equal(first_obs, st.obs)
        assert np.all(st.info["steps"] == 0) and np.all(st.info["truncation"] == 0)
        oe = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f32")
        rs = np.random.RandomState(5)
        n_done = n_trunc = 0
        fb = G.FlipBudget()
        for t in range(nsteps):
            a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
            prev = st
            ep_prev = e._get(_abi.F_EPISODE)
            st = env.step(prev, a)
            ep = e._get(_abi.F_EPISODE)
            for i in range(n):
                orec, oobs, odone, oep, o = _oracle_wrapped_step(
                    oe, prev._record[i], prev.obs[i], a[i], ep_prev[i], float(prev.done[i]), first_state[i],
                    first_obs[i], episode_length)
                assert st.done[i] == odone, (t, i)
                np.testing.assert_array_equal(ep[i, :2], oep[:2].astype(np.float32))
                assert abs(ep[i, _abi.EP_LENGTH] - oep[3]) == 0
                np.testing.assert_array_equal(st._record[i, _abi.S_RNG:_abi.S_RNG + 2].view(np.uint32),
                                              orec[_abi.S_RNG:_abi.S_RNG + 2].view(np.uint32))
                if odone:
                    n_done += 1
                    n_trunc += int(oep[1])
                    np.testing.assert_array_equal(st._record[i, 0:_abi.FIRST_STRIDE], first_state[i])
                    np.testing.assert_array_equal(st.obs[i], first_obs[i])
                else:
                    ok = np.abs(st.obs[i] - oobs).max() <= 5e-3 and abs(st.reward[i] - o["reward"]) <= 1e-3
                    fb.check(ok, o, f"step {t} env {i}")
                assert abs(ep[i, _abi.EP_SUM_REWARD] - oep[2]) <= 1e-3 * (t + 1)
        fb.finish()
        assert n_done > 0
        if episode_length == 7:
            assert n_trunc > 0
        if terminal_z < 0.2:  # the robots survive some steps: the non-done path is compared
            assert fb.n >= 50, fb.n
    finally:
        e.close()


def _oracle_repeat_step(oe, rec, obs, action, ep, prev_done, first_state, first_obs, L, k):
    """brax EpisodeWrapper.step with action_repeat k (lax.scan of env.step, rewards summed), then
    AutoResetWrapper: counters restart after a done step, the last repeat's env done decides."""
    keep = 1.0 - prev_done
    st = dict(state=G.record_to_oracle_state(rec), obs=obs.astype(np.float64))
    rsum, flagged = 0.0, False
    for _ in range(k):
        o = oe.step(st, action.astype(np.float64))
        st = dict(state=o["state"], obs=o["obs"])
        rsum += o["reward"]
        flagged = flagged or o["boundary"] > 0
    steps = ep[_abi.EP_STEPS] * keep + k
    hit = steps >= L
    done = bool(o["done"]) or hit
    trunc = 1.0 if (hit and not o["done"]) else 0.0
    out_obs = o["obs"].astype(np.float32)
    if done:
        out_obs = first_obs.copy()
    ep_new = np.array([steps, trunc, (ep[_abi.EP_SUM_REWARD] + rsum) * keep, (ep[_abi.EP_LENGTH] + k) * keep])
    return out_obs, float(done), ep_new, rsum, dict(o, boundary=1 if flagged else 0)


def test_action_repeat(require_gpu, tmp_path):
    """wrap(env, episode_length=8, action_repeat=3): every step() is 3 env steps with the same
    action; reward = their sum, counters advance by 3 (a truncation at step 9), done and the
    auto-reset follow the last repeat -- against the restated wrapper over the oracle."""
    path = common.write_model(tmp_path, 0)
    n, k, L = 8, 3, 8
    e = PupperV3Env(**common.fixture_kwargs(path, terminal_body_z=0.1), num_envs=n)
    try:
        env = wrappers.wrap(e, episode_length=L, action_repeat=k)
        st = env.reset(make_keys(4, n))
        first_state = e._get(_abi.F_FIRST_STATE)
        first_obs = e._get(_abi.F_FIRST_OBS)
        oe = O.OracleEnv(e.sys_model.struct, e.config_struct, precision="f32")
        rs = np.random.RandomState(6)
        fb = G.FlipBudget()
        n_trunc = 0
        for t in range(6):
            a = rs.uniform(-1, 1, size=(n, 12)).astype(np.float32)
            prev = st
            ep_prev = e._get(_abi.F_EPISODE)
            st = env.step(prev, a)
            ep = e._get(_abi.F_EPISODE)
            for i in range(n):
                oobs, odone, oep, rsum, o = _oracle_repeat_step(
                    oe, prev._record[i], prev.obs[i], a[i], ep_prev[i], float(prev.done[i]), first_state[i],
                    first_obs[i], L, k)
                ok = st.done[i] == odone and abs(st.reward[i] - rsum) <= 3e-3
                if odone:
                    ok = ok and np.array_equal(st._record[i, 0:_abi.FIRST_STRIDE], first_state[i])
                    ok = ok and np.array_equal(st.obs[i], first_obs[i])
                else:
                    ok = ok and np.abs(st.obs[i] - oobs).max() <= 5e-3
                fb.check(ok, o, f"step {t} env {i}")
                np.testing.assert_array_equal(ep[i, _abi.EP_STEPS], oep[0])
                if st.done[i] == odone:
                    np.testing.assert_array_equal(ep[i, _abi.EP_TRUNCATION], oep[1])
                n_trunc += int(ep[i, _abi.EP_TRUNCATION])
        fb.finish()
        assert n_trunc > 0  # 3 + 3 + 3 = 9 >= 8 steps
    finally:
        e.close()


def test_action_repeat_needs_auto_reset(require_gpu):
    from pupperv3_mjx import _lib
    e = PupperV3Env(**common.fixture_kwargs(common.MODEL_XML), num_envs=2)
    try:
        with pytest.raises(_lib.PupperHipError, match="auto-reset"):
            _lib.check(e._L.pp3_set_action_repeat(e._h, 2))
    finally:
        e.close()
