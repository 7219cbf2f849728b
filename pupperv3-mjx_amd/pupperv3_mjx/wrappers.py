"""Brax training wrappers for the HIP env, on device.

Brax PPO does not step PupperV3Env directly: `brax.training.agents.ppo.train` wraps it with
`brax.envs.training.wrap(env, episode_length, action_repeat, randomization_fn)` =
(DomainRandomization)VmapWrapper -> EpisodeWrapper -> AutoResetWrapper ([ext] brax 0.12.1,
pinned in requirements.txt:3; not vendored in the reference).  `wrap` below gives the same
reset()/step() surface with the episode bookkeeping and the auto-reset done inside the fused
step kernel (pp3_set_auto_reset), so a rollout never leaves the GPU:

  * EpisodeWrapper: info['steps'] counts env steps; done |= steps >= episode_length;
    info['truncation'] = 1 where the episode length, not the env, ended the episode;
    info['episode_metrics'] = {'sum_reward', 'length'} (reset to 0 after a done step).
  * AutoResetWrapper: at the start of a step, steps := 0 where the previous step was done;
    after it, pipeline_state (qpos, qvel, qacc_warmstart) and obs := the env's first state
    (the state its last reset produced) where done.  The env's own info (rng, command, last
    action, latency buffers, ...) carries over, as in Brax.

  * action_repeat k (EpisodeWrapper.step's lax.scan over env.step with the same action): every
    step() is k launches of the env step; reward = the sum over the k repeats, info['steps'] and
    the episode length advance by k, and done / truncation / the auto-reset follow the last
    repeat (pp3_set_action_repeat).

Domain randomisation (the DomainRandomizationVmapWrapper role) is PupperV3Env.
set_domain_randomization.
"""
from __future__ import annotations

import numpy as np

from . import _abi, _lib
from .environment import PupperV3Env, State


class AutoResetEpisodeEnv:
    """EpisodeWrapper + AutoResetWrapper semantics over a batched PupperV3Env."""

    def __init__(self, env: PupperV3Env, episode_length: int = 1000, action_repeat: int = 1):
        if episode_length <= 0:
            raise ValueError("episode_length must be positive")
        if action_repeat < 1:
            raise ValueError("action_repeat must be >= 1")
        self.env = env
        self.episode_length = int(episode_length)
        self.action_repeat = int(action_repeat)
        _lib.check(env._L.pp3_set_auto_reset(env._h, self.episode_length))
        _lib.check(env._L.pp3_set_action_repeat(env._h, self.action_repeat))
        env._lazy_extra = {_abi.F_EPISODE: self._extra_info}  # info entries of the env's DeviceStates
        env._issue_capture = lambda: (self._first_ps, self._first_obs)  # each state keeps its own
        self._first_ps, self._first_obs = None, None

    # brax Env surface
    @property
    def observation_size(self) -> int:
        return self.env.observation_size

    @property
    def action_size(self) -> int:
        return self.env.action_size

    @property
    def dt(self) -> float:
        return self.env.dt

    @property
    def unwrapped(self) -> PupperV3Env:
        return self.env

    def _extra_info(self, st, got, single: bool) -> dict:
        """The wrapper's info entries of a DeviceState, built when its lazy part is downloaded: the
        episode record rides along as one more lazy field (snapshotted with the rest); the first
        state / obs change only at reset: cached on the host then, and captured by each state when
        it is issued (st._capture), so a state read after a later reset still reports its own."""
        ep = got[_abi.F_EPISODE]
        first_ps, first_obs = st.__dict__.get("_capture") or (None, None)
        sq = (lambda v: v[0]) if single else (lambda v: v)
        return {"steps": sq(ep[:, _abi.EP_STEPS].copy()),
                "truncation": sq(ep[:, _abi.EP_TRUNCATION].copy()),
                "episode_metrics": {"sum_reward": sq(ep[:, _abi.EP_SUM_REWARD].copy()),
                                    "length": sq(ep[:, _abi.EP_LENGTH].copy())},
                "episode_done": np.array(st.done, dtype=np.float32),
                "first_pipeline_state": None if first_ps is None else dict(first_ps),
                "first_obs": first_obs}

    def reset(self, rng) -> State:
        st = self.env.reset(rng)
        sq = (lambda v: v[0]) if np.ndim(st.reward) == 0 else (lambda v: v)
        first = self.env._get(_abi.F_FIRST_STATE)
        fobs = self.env._get(_abi.F_FIRST_OBS)
        self._first_ps = {"q": sq(first[:, 0:19].copy()), "qd": sq(first[:, 19:37].copy()),
                          "qacc_warmstart": sq(first[:, 37:55].copy())}
        self._first_obs = sq(fobs.copy())
        st.__dict__["_capture"] = (self._first_ps, self._first_obs)  # (issued before they were read)
        return st

    def step(self, state: State, action) -> State:
        self._prepare(state)
        return self.env.step(state, action)

    def rollout(self, state: State, actions):
        """K wrapper steps as one fused launch (PupperV3Env.rollout; action_repeat > 1 keeps its
        k launches per step): (state after the last step, {"obs", "reward", "done"} per step)."""
        self._prepare(state)
        return self.env.rollout(state, actions)

    def rollout_policy(self, state: State, policy, nsteps: int):
        """K wrapper steps with the on-device policy in the loop (PupperV3Env.rollout_policy)."""
        self._prepare(state)
        return self.env.rollout_policy(state, policy, nsteps)

    def _prepare(self, state: State) -> None:
        n = self.env.num_envs
        if not self.env.holds(state):
            # an edited (or foreign) state: its episode record and done go back with it (env.step
            # then uploads the rest); the rollout loop's unedited states skip all of this
            info = state.info
            if "steps" in info:
                ep = np.zeros((n, _abi.EP_STRIDE), dtype=np.float32)
                ep[:, _abi.EP_STEPS] = np.asarray(info["steps"], dtype=np.float32).reshape(n)
                ep[:, _abi.EP_TRUNCATION] = np.asarray(info["truncation"], dtype=np.float32).reshape(n)
                ep[:, _abi.EP_SUM_REWARD] = np.asarray(info["episode_metrics"]["sum_reward"], dtype=np.float32).reshape(n)
                ep[:, _abi.EP_LENGTH] = np.asarray(info["episode_metrics"]["length"], dtype=np.float32).reshape(n)
                self.env._put(_abi.F_EPISODE, ep)
            self.env._put(_abi.F_DONE, np.asarray(state.done, dtype=np.float32).reshape(n, 1))


def wrap(env: PupperV3Env, episode_length: int = 1000, action_repeat: int = 1,
         randomization_fn=None, rng=None) -> AutoResetEpisodeEnv:
    """brax.envs.training.wrap for the HIP env.  `randomization_fn(sys, rng) -> (sys_batched,
    in_axes)` (domain_randomization.domain_randomize) is applied once with `rng` [N, 2]."""
    if randomization_fn is not None:
        if rng is None:
            raise ValueError("randomization_fn needs rng (one key per env)")
        sys_b, _ = randomization_fn(env.sys, rng)
        env.set_domain_randomization(sys_b)
    return AutoResetEpisodeEnv(env, episode_length, action_repeat)
