"""The drop-in host surface (environment.py:314,348 reset/step returning a State) over
the device-resident env: DeviceState semantics.

* an unedited state passed back to step() is not re-uploaded, and the rollout equals one in which
  every state is re-uploaded from the host, bit for bit;
* old states keep their own data after the env has stepped on (device snapshots of the lazy part);
* an edited state (a new array assigned, as test_environment.py:147,186 do) is uploaded and
  honoured; in-place edits are refused (read-only arrays, as JAX arrays are immutable);
* the same through wrappers.wrap (EpisodeWrapper + AutoResetWrapper on device).
"""
import numpy as np
import pytest

import common
from pupperv3_mjx import MODEL_XML, _abi, wrappers
from pupperv3_mjx.environment import PupperV3Env, make_keys

pytestmark = pytest.mark.gpu
N = 64


def _env(**kw):
    return PupperV3Env(**common.fixture_kwargs(MODEL_XML, **kw), num_envs=N)


def _count_uploads(env):
    calls = []
    orig = env._write_state

    def spy(st):
        calls.append(1)
        return orig(st)
    env._write_state = spy
    return calls


def test_unedited_states_are_not_reuploaded_and_match_forced_uploads(require_gpu):
    acts = np.random.RandomState(0).uniform(-1, 1, size=(12, N, 12)).astype(np.float32)
    e1, e2 = _env(), _env()
    try:
        uploads = _count_uploads(e1)
        s1, s2 = e1.reset(make_keys(4, N)), e2.reset(make_keys(4, N))
        for t in range(12):
            s1 = e1.step(s1, acts[t])
            if t % 3 == 0:
                _ = s1.info["rng"]  # materialised states stay "held" while unedited
            e2._write_state(s2)  # forced host round trip of every state
            s2 = e2.step(e2._issue(False), acts[t])
        assert not uploads
        np.testing.assert_array_equal(s1.obs, s2.obs)
        np.testing.assert_array_equal(s1.reward, s2.reward)
        np.testing.assert_array_equal(s1._record, s2._record)
    finally:
        e1.close()
        e2.close()


def test_old_states_keep_their_data(require_gpu):
    e = _env()
    try:
        st = e.reset(make_keys(5, N))
        rs = np.random.RandomState(1)
        kept, eager = [], []
        for t in range(6):
            st = e.step(st, rs.uniform(-1, 1, size=(N, 12)).astype(np.float32))
            kept.append(st)
            eager.append((e._get(_abi.F_STATE).copy(), e._get(_abi.F_METRICS).copy(), e._get(_abi.F_PIPELINE).copy()))
        for st, (rec, met, pipe) in zip(kept, eager):  # read only now, after the env moved on
            np.testing.assert_array_equal(st._record, rec)
            np.testing.assert_array_equal(st._metrics_raw, met)
            np.testing.assert_array_equal(st.pipeline_state.q, rec[:, :19])
            np.testing.assert_array_equal(st.pipeline_state.qacc, pipe[:, _abi.P_QACC:_abi.P_QACC + 18])
            assert np.all(st.info["step"] == rec[:, _abi.S_STEP].astype(np.int32))
        # stepping an OLD state rewinds the env to it (it is uploaded from its snapshot)
        a = np.zeros((N, 12), dtype=np.float32)
        r1 = e.step(kept[2], a)
        r2 = e.step(kept[2], a)
        np.testing.assert_array_equal(r1._record, r2._record)
    finally:
        e.close()


def test_edited_state_is_uploaded_and_inplace_edits_refused(require_gpu):
    e = _env(resample_velocity_step=10 ** 9)
    try:
        st = e.reset(make_keys(6, N))
        with pytest.raises(ValueError):
            st.info["command"][0, 0] = 9.0  # read-only, as the reference's jax arrays
        with pytest.raises(ValueError):
            st.obs[0, 0] = 1.0
        st.info["command"] = np.tile(np.float32([0.3, -0.2, 0.1]), (N, 1))
        assert not e.holds(st)
        out = e.step(st, np.zeros((N, 12), dtype=np.float32))
        np.testing.assert_array_equal(out.info["command"], np.tile(np.float32([0.3, -0.2, 0.1]), (N, 1)))
        assert e.holds(out)
    finally:
        e.close()


def test_wrapper_rollout_without_uploads_matches_forced(require_gpu):
    acts = np.random.RandomState(2).uniform(-1, 1, size=(20, N, 12)).astype(np.float32)
    e1, e2 = _env(terminal_body_z=0.3), _env(terminal_body_z=0.3)
    try:
        w1, w2 = wrappers.wrap(e1, episode_length=7), wrappers.wrap(e2, episode_length=7)
        uploads = _count_uploads(e1)
        s1, s2 = w1.reset(make_keys(8, N)), w2.reset(make_keys(8, N))
        for t in range(20):
            s1 = w1.step(s1, acts[t])
            s2 = dict_roundtrip(w2, s2)
            s2 = w2.step(s2, acts[t])
            np.testing.assert_array_equal(s1.done, s2.done)
        assert not uploads
        np.testing.assert_array_equal(s1.obs, s2.obs)
        for k in ("steps", "truncation"):
            np.testing.assert_array_equal(s1.info[k], s2.info[k])
        np.testing.assert_array_equal(s1.info["episode_metrics"]["sum_reward"], s2.info["episode_metrics"]["sum_reward"])
    finally:
        e1.close()
        e2.close()


def dict_roundtrip(w, st):
    """A state rebuilt on the host (every array a fresh copy): the wrapper must upload it."""
    info = {k: (dict(v) if isinstance(v, dict) else np.array(v)) for k, v in st.info.items()}
    st.info = info
    assert not w.env.holds(st)
    return st


@pytest.mark.parametrize("mode", ["fused", "kernel", "copy"])
def test_output_paths_return_the_device_outputs(require_gpu, mode):
    """env.step's obs / reward / done reach the host three ways: stored by the step launch itself
    into the page-locked block (a one-step pp3_rollout whose trajectory rows are the block's device
    mapping, the default), by pp3_outputs_to_host after the launch, or by copy-engine transfers.
    Each must return exactly the env's device buffers, with auto-reset and action_repeat too (the
    trajectory rows are written at the last repeat; a done env's rows are its reset obs)."""
    from pupperv3_mjx import environment, wrappers
    saved = environment.STEP_WRITES_HOST, environment.OUTPUTS_BY_KERNEL
    environment.STEP_WRITES_HOST, environment.OUTPUTS_BY_KERNEL = mode == "fused", mode != "copy"
    try:
        for wrapped in (False, True):
            N = 67
            env = PupperV3Env(**common.fixture_kwargs(common.MODEL_XML), num_envs=N)
            try:
                api = wrappers.wrap(env, episode_length=4, action_repeat=2) if wrapped else env
                st = api.reset(make_keys(2, N))
                rs = np.random.RandomState(5)
                for _ in range(6):
                    st = api.step(st, rs.uniform(-1, 1, size=(N, 12)).astype(np.float32))
                    np.testing.assert_array_equal(st.obs, env._get(_abi.F_OBS))
                    np.testing.assert_array_equal(st.reward, env._get(_abi.F_REWARD)[:, 0])
                    np.testing.assert_array_equal(st.done, env._get(_abi.F_DONE)[:, 0])
                if wrapped:  # truncation at 4 steps: every env went through an auto-reset
                    assert np.all(st.info["steps"] <= 4)
            finally:
                env.close()
    finally:
        environment.STEP_WRITES_HOST, environment.OUTPUTS_BY_KERNEL = saved


def test_reassigned_outputs_and_unread_fields_are_uploaded(require_gpu):
    """Assigning a new obs / done array (N > 1) or a pipeline_state / info to a state nobody has
    read yet is an edit: step() uploads it instead of failing or skipping it, and nothing
    downloaded later overwrites the assignment."""
    e = _env()
    try:
        uploads = _count_uploads(e)
        st = e.reset(make_keys(5, N))
        st.obs = np.full_like(st.obs, 0.5)            # N > 1: a tuple != of arrays used to raise here
        st.done = np.zeros(N, np.float32)
        out = e.step(st, np.zeros((N, 12), np.float32))
        assert len(uploads) == 1
        np.testing.assert_array_equal(out.obs[:, 36:72], np.full((N, 36), 0.5, np.float32))  # history frame
        # a pipeline_state assigned before anything was read (the lazy part not downloaded)
        fresh = e.step(out, np.zeros((N, 12), np.float32))
        assert not fresh.materialized
        from pupperv3_mjx.environment import PipelineState
        q = np.zeros((N, 19), np.float32)
        q[:, 2], q[:, 3] = 0.8, 1.0
        q[:, 7:] = common.DEFAULT_POSE
        fresh.pipeline_state = PipelineState(q=q, qd=np.zeros((N, 18), np.float32),
                                             qacc_warmstart=np.zeros((N, 18), np.float32))
        assert fresh.materialized and fresh.pipeline_state.q is q  # the download did not overwrite it
        n0 = len(uploads)
        up = e.step(fresh, np.zeros((N, 12), np.float32))
        assert len(uploads) == n0 + 1
        assert np.all(up.pipeline_state.q[:, 2] > 0.7)  # the lifted pose was stepped, not the old one
        # info assigned before the lazy part was read: no KeyError, uploaded
        nxt = e.step(up, np.zeros((N, 12), np.float32))
        info = dict(nxt.info)
        info["command"] = np.zeros((N, 3), np.float32)
        nxt.info = info
        after = e.step(nxt, np.zeros((N, 12), np.float32))
        np.testing.assert_array_equal(after.info["command"], np.zeros((N, 3), np.float32))
    finally:
        e.close()


def test_old_state_read_after_device_launches(require_gpu):
    """An unread state whose env has since launched on its own stream (step_device, no host
    synchronisation) reads its own snapshot, not the next state's data."""
    e = _env()
    try:
        st = e.reset(make_keys(6, N))
        st = e.step(st, np.zeros((N, 12), np.float32))
        want = e._get(_abi.F_STATE).copy()
        from pupperv3_mjx import _lib
        buf = _lib.DeviceBuffer(N * 12 * 4, e.device)
        buf.upload(np.random.RandomState(1).uniform(-1, 1, (N, 12)).astype(np.float32))
        for _ in range(5):
            e.step_device(buf.ptr.value)
        np.testing.assert_array_equal(st._record, want)
        buf.free()
    finally:
        e.close()


def test_wrapper_states_keep_their_first_state(require_gpu):
    """info['first_obs'] / ['first_pipeline_state'] of a wrapper state read after a later reset
    are those of the reset the state descends from."""
    w = wrappers.wrap(_env(), episode_length=50)
    try:
        s1 = w.reset(make_keys(7, N))
        s1 = w.step(s1, np.zeros((N, 12), np.float32))
        first1 = np.array(w._first_obs)
        s2 = w.reset(make_keys(8, N))
        assert np.any(np.array(w._first_obs) != first1)
        np.testing.assert_array_equal(s1.info["first_obs"], first1)
        np.testing.assert_array_equal(s2.info["first_obs"], w._first_obs)
    finally:
        w.env.close()


@pytest.mark.parametrize("zero_copy", [False, True])
def test_async_steps_match_synchronous_steps(require_gpu, zero_copy):
    """step() returns before its launch completes (ASYNC_STEP): states issued back to back and read
    only afterwards hold their own step's obs / reward / done / record, bit for bit the same as a
    loop that synchronises every step; with the actions read by the launch straight from the
    page-locked staging ring too (ACTIONS_ZERO_COPY), and through the wrapper."""
    from pupperv3_mjx import environment
    saved = environment.ASYNC_STEP, environment.ACTIONS_ZERO_COPY
    acts = np.random.RandomState(9).uniform(-1, 1, size=(7, N, 12)).astype(np.float32)
    try:
        for wrapped in (False, True):
            ref = []
            environment.ASYNC_STEP, environment.ACTIONS_ZERO_COPY = False, False
            e = _env()
            api = wrappers.wrap(e, episode_length=5) if wrapped else e
            st = api.reset(make_keys(11, N))
            for t in range(7):
                st = api.step(st, acts[t])
                ref.append((np.array(st.obs), np.array(st.reward), np.array(st.done), np.array(st._record)))
            e.close()
            environment.ASYNC_STEP, environment.ACTIONS_ZERO_COPY = True, zero_copy
            e = _env()
            api = wrappers.wrap(e, episode_length=5) if wrapped else e
            st = api.reset(make_keys(11, N))
            kept = []
            for t in range(7):
                st = api.step(st, acts[t])
                kept.append(st)
            assert all(k.__dict__.get("_ready") is not None for k in kept[-2:])  # returned unread
            for k, (o, r, d, rec) in zip(kept, ref):
                np.testing.assert_array_equal(k.obs, o)
                np.testing.assert_array_equal(k.reward, r)
                np.testing.assert_array_equal(k.done, d)
                np.testing.assert_array_equal(k._record, rec)
            e.close()
    finally:
        environment.ASYNC_STEP, environment.ACTIONS_ZERO_COPY = saved


def test_deferred_step_loop_takes_no_snapshots(require_gpu):
    """`state = env.step(state, action)` with DEFER_LAUNCH: the steps queue and run as fused launches
    once a queued state's fields are read, after the caller has dropped the states they overwrite,
    so the loop takes no device snapshot and ends bit for bit where the synchronous loop does; a
    state the caller keeps ends a launch of its own, is snapshotted before the next one and reads
    its own record."""
    from pupperv3_mjx import environment
    saved = environment.ASYNC_STEP, environment.DEFER_LAUNCH
    acts = np.random.RandomState(12).uniform(-1, 1, size=(9, N, 12)).astype(np.float32)
    try:
        environment.ASYNC_STEP, environment.DEFER_LAUNCH = False, False
        e = _env()
        st = e.reset(make_keys(13, N))
        recs = []
        for t in range(9):
            st = e.step(st, acts[t])
            recs.append(np.array(st._record))
        ref_obs = np.array(st.obs)
        e.close()
        environment.ASYNC_STEP, environment.DEFER_LAUNCH = True, True
        e = _env()
        st = e.reset(make_keys(13, N))
        for t in range(6):
            st = e.step(st, acts[t])
        assert e._n_snapshots == 0 and e._qb is not None and e._qb.n == 6  # queued, nothing launched
        kept = st
        for t in range(6, 9):
            st = e.step(st, acts[t])
        assert e._n_snapshots == 0 and e._qb.n == 9
        np.testing.assert_array_equal(kept._record, recs[5])  # (issues the queue: launches end at 5 and 8)
        assert e._qb is None and e._n_snapshots == 1
        np.testing.assert_array_equal(st.obs, ref_obs)
        np.testing.assert_array_equal(st._record, recs[8])
        e.close()
    finally:
        environment.ASYNC_STEP, environment.DEFER_LAUNCH = saved


@pytest.mark.parametrize("keep", ["states", "batches"])
@pytest.mark.parametrize("wrapped", [False, True])
def test_step_batches_match_synchronous_steps(require_gpu, keep, wrapped):
    """Queued steps issued as fused launches (STEP_BATCH = 4: 11 steps are batches of 4, 4 and 3)
    give every step's obs / reward / done, and every kept state's record, bit for bit as the
    synchronous loop: with every state kept (each ends a launch of its own: one-step launches) and
    with the states dropped (three- and two-step launches without host outputs, then the batch's
    last step storing its rows into the batch's page-locked block, read here), also through the
    wrapper (on-device auto-reset inside the fused launches)."""
    from pupperv3_mjx import environment
    saved = environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.STEP_BATCH
    acts = np.random.RandomState(14).uniform(-1, 1, size=(11, N, 12)).astype(np.float32)
    try:
        environment.ASYNC_STEP, environment.DEFER_LAUNCH = False, False
        e = _env()
        api = wrappers.wrap(e, episode_length=5) if wrapped else e
        st = api.reset(make_keys(15, N))
        ref = []
        for t in range(11):
            st = api.step(st, acts[t])
            ref.append((np.array(st.obs), np.array(st.reward), np.array(st.done), np.array(st._record)))
        e.close()
        environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.STEP_BATCH = True, True, 4
        e = _env()
        api = wrappers.wrap(e, episode_length=5) if wrapped else e
        st = api.reset(make_keys(15, N))
        kept, batches = [], []
        for t in range(11):
            st = api.step(st, acts[t])
            if keep == "states":
                kept.append(st)
            elif e._qb is not None and (not batches or batches[-1] is not e._qb):
                batches.append(e._qb)
        np.testing.assert_array_equal(st._record, ref[-1][3])  # (issues the last batch)
        e.synchronize()
        if keep == "states":
            for k, (o, r, d, rec) in zip(kept, ref):
                np.testing.assert_array_equal(k.obs, o)
                np.testing.assert_array_equal(k.reward, r)
                np.testing.assert_array_equal(k.done, d)
                np.testing.assert_array_equal(k._record, rec)
        else:
            # (LIVE_OUTPUTS_ONLY: a batch's block holds the rows of the state that ended its launch,
            # the batch's last; the dropped states' rows are not stored)
            assert [b.n for b in batches] == [4, 4, 3] and e._n_snapshots == 0
            t = -1
            for b in batches:
                t += b.n
                go, gr, gd = b.views(b.n - 1, False)
                np.testing.assert_array_equal(go, ref[t][0])
                np.testing.assert_array_equal(gr, ref[t][1])
                np.testing.assert_array_equal(gd, ref[t][2])
        e.close()
    finally:
        environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.STEP_BATCH = saved


def test_step_batches_capped_by_block_bytes(require_gpu):
    """STEP_BLOCK_MAX_BYTES bounds a queued batch's page-locked output block ([B][N][36H + 2]
    floats): with room for three rows, 8 queued steps run as batches of 3, 3 and 2 steps, still bit
    for bit the synchronous loop (advisor r05: long observation histories at 4096 envs)."""
    from pupperv3_mjx import environment
    saved = (environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.STEP_BATCH,
             environment.STEP_BLOCK_MAX_BYTES)
    acts = np.random.RandomState(16).uniform(-1, 1, size=(8, N, 12)).astype(np.float32)
    try:
        environment.ASYNC_STEP, environment.DEFER_LAUNCH = False, False
        e = _env()
        st = e.reset(make_keys(17, N))
        ref = []
        for t in range(8):
            st = e.step(st, acts[t])
            ref.append((np.array(st.obs), np.array(st.reward), np.array(st.done), np.array(st._record)))
        e.close()
        environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.STEP_BATCH = True, True, 16
        e = _env()
        environment.STEP_BLOCK_MAX_BYTES = 3 * 4 * N * (e.observation_size + 2) + 1
        st = e.reset(make_keys(17, N))
        batches = []
        for t in range(8):
            st = e.step(st, acts[t])
            if not batches or batches[-1] is not e._qb:
                batches.append(e._qb)
        np.testing.assert_array_equal(st._record, ref[-1][3])
        assert [b.cap for b in batches] == [3, 3, 3] and [b.n for b in batches] == [3, 3, 2]
        t = -1
        for b in batches:
            t += b.n
            go, gr, gd = b.views(b.n - 1, False)
            np.testing.assert_array_equal(go, ref[t][0])
            np.testing.assert_array_equal(gr, ref[t][1])
            np.testing.assert_array_equal(gd, ref[t][2])
        e.close()
    finally:
        (environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.STEP_BATCH,
         environment.STEP_BLOCK_MAX_BYTES) = saved


def test_dropped_states_get_no_host_rows(require_gpu):
    """LIVE_OUTPUTS_ONLY: a queue of steps whose states the caller dropped is issued as one launch
    without trajectory outputs plus a one-step launch that stores the last state's obs / reward /
    done into host memory; a state the caller kept ends a launch of its own and gets its rows."""
    from pupperv3_mjx import environment
    saved = environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.LIVE_OUTPUTS_ONLY
    acts = np.random.RandomState(19).uniform(-1, 1, size=(6, N, 12)).astype(np.float32)
    calls = []

    class Spy:
        def __init__(self, lib):
            self._lib = lib

        def __getattr__(self, name):
            fn = getattr(self._lib, name)
            if name != "pp3_rollout":
                return fn

            def call(*args):
                calls.append((int(args[3]), all(a is None or not getattr(a, "value", a) for a in args[4:7])))
                return fn(*args)
            return call
    try:
        environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.LIVE_OUTPUTS_ONLY = True, True, True
        e = _env()
        st = e.reset(make_keys(20, N))
        e._raw = Spy(e._raw)
        kept = None
        for t in range(6):
            st = e.step(st, acts[t])
            if t == 2:
                kept = st
        _ = st.obs
        # steps 0-1 (dropped): no outputs; step 2 (kept): its own launch with rows; steps 3-4
        # (dropped): no outputs; step 5: its own launch with rows
        assert calls == [(2, True), (1, False), (2, True), (1, False)], calls
        assert np.isfinite(kept.obs).all() and np.isfinite(st.obs).all()
        e.close()
    finally:
        environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.LIVE_OUTPUTS_ONLY = saved


def test_copies_of_queued_states_and_unstored_rows(require_gpu):
    """Copies and restores of queued states (advisor r05): copy.copy of a queued state reads its own
    step's outputs even after the original is dropped; an object restored from a queued state's
    __dict__ whose original was dropped before the queue was issued raises instead of viewing
    unwritten rows; env.flush() issues the queue so device_field buffers hold the last step."""
    import copy
    import gc
    acts = np.random.RandomState(23).uniform(-1, 1, size=(5, N, 12)).astype(np.float32)
    e, ref = _env(), _env()
    try:
        st, sr = e.reset(make_keys(21, N)), ref.reset(make_keys(21, N))
        want = []
        for t in range(5):
            sr = ref.step(sr, acts[t])
            want.append((np.array(sr.obs), np.array(sr.reward)))
        st = e.step(st, acts[0])
        st = e.step(st, acts[1])
        c = copy.copy(st)  # a copy of the queued step 1
        st = e.step(st, acts[2])
        restored = object.__new__(type(st))
        restored.__dict__.update(st.__dict__)  # (bypasses __copy__: untracked by the queue)
        st = e.step(st, acts[3])
        st = e.step(st, acts[4])
        gc.collect()
        np.testing.assert_array_equal(c.obs, want[1][0])
        np.testing.assert_array_equal(c.reward, want[1][1])
        with pytest.raises(RuntimeError, match="not kept"):
            _ = restored.obs
        e.flush()
        assert e._qb is None
        np.testing.assert_array_equal(st.obs, want[4][0])
        ptr, n = e.device_field(_abi.F_REWARD)
        e.synchronize()
        got = e._get(_abi.F_REWARD, raw=True).reshape(-1)
        np.testing.assert_array_equal(got, want[4][1])
    finally:
        e.close()
        ref.close()


def test_step_queue_mixed_with_rollout_branch_and_reset(require_gpu):
    """The step queue (DEFER_LAUNCH, STEP_BATCH) between other calls: a rollout() from the queued
    tail, a step from an older kept state (a branch: the queue is issued, the old state re-uploaded
    from its snapshot), a reset() while steps are queued, and reads in between -- every state's
    obs / reward / done / record bit for bit the synchronous sequence's."""
    from pupperv3_mjx import environment
    saved = environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.STEP_BATCH
    acts = np.random.RandomState(16).uniform(-1, 1, size=(16, N, 12)).astype(np.float32)

    def run(e):
        out = {}
        st = e.reset(make_keys(17, N))
        st = e.step(st, acts[0])
        s1 = st                                  # kept, read only at the end
        st = e.step(st, acts[1])
        st = e.step(st, acts[2])
        st, tr = e.rollout(st, acts[3:6])        # from the queued tail
        out["traj"] = tr
        st = e.step(st, acts[6])
        st = e.step(st, acts[7])
        out["mid_obs"] = np.array(st.obs)        # read between queued steps
        st = e.step(st, acts[8])
        b = e.step(s1, acts[9])                  # branch from an old state
        b = e.step(b, acts[10])
        st = e.step(st, acts[11])                # and back to the main line
        r = e.reset(make_keys(18, N))            # reset with steps queued
        r = e.step(r, acts[12])
        r = e.step(r, acts[13])
        for name, x in (("s1", s1), ("main", st), ("branch", b), ("reset", r)):
            out[name] = (np.array(x.obs), np.array(x.reward), np.array(x.done), np.array(x._record))
        return out

    try:
        environment.ASYNC_STEP, environment.DEFER_LAUNCH = False, False
        e = _env()
        ref = run(e)
        e.close()
        environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.STEP_BATCH = True, True, 4
        e = _env()
        got = run(e)
        e.close()
        for k in ref["traj"]:
            np.testing.assert_array_equal(got["traj"][k], ref["traj"][k])
        np.testing.assert_array_equal(got["mid_obs"], ref["mid_obs"])
        for name in ("s1", "main", "branch", "reset"):
            for g, r in zip(got[name], ref[name]):
                np.testing.assert_array_equal(g, r)
    finally:
        environment.ASYNC_STEP, environment.DEFER_LAUNCH, environment.STEP_BATCH = saved


def test_retired_pools_free_their_blocks(require_gpu):
    """A page-locked block leased from a pool the env has retired (a trajectory length no longer
    used, or a closed env) is freed when released, not parked in the orphaned pool (advisor r04)."""
    from pupperv3_mjx import _lib
    e = _env()
    try:
        st = e.reset(make_keys(3, N))
        st, tr3 = e.rollout(st, np.zeros((3, N, 12), np.float32))
        pool3 = e._traj_pool[3]
        st, tr4 = e.rollout(st, np.zeros((4, N, 12), np.float32))
        assert 3 not in e._traj_pool and pool3.retired and len(pool3) == 0
        blk = tr3["obs"].base
        while blk is not None and not isinstance(blk, _lib._BlockRef):
            blk = getattr(blk, "base", None)
        block = blk.block if blk is not None else None
        del tr3, blk
        import gc
        gc.collect()
        assert len(pool3) == 0
        if block is not None:
            assert not block.ptr  # freed on release
    finally:
        e.close()
    assert e._pin_pool.retired
