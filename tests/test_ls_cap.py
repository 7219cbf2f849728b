"""The truncated line search: where the reference's ls_iterations = 5 cap binds, and what it moves.

The model runs Newton with iterations="1" ls_iterations="5" (test_pupper_model.xml:57), so every
substep's qacc is ONE line-searched Newton step.  When the 5-evaluation budget runs out before the
search converges, the returned alpha is set by PrimalSearch's exit rule (engine_solver.c), which
MuJoCo's documentation does not specify; the oracle (pp3_oracle.c line_search) and the kernel
(pp3_env.hip) restate it identically, so no parity test can pin it.  These CPU tests pin the
oracle's exit counters (orc_ls_take) that bench.py's `ls_cap` block reports, on cases where the
answer is known:

* the sliding ball of test_friction_kat.py (mu = 0.05 on a 20 degree slope, the chattering contact
  its docstring describes): the cap provably binds, and a capped substep's qacc differs from the
  converged search's (ls_iterations = 50) by tens of m/s^2, while a substep whose search converged
  inside the budget is bit-identical under the larger budget (same evaluations, same exit);
* the rolling ball: the cap binds too (the derivative never gets under MuJoCo's gtol), but the
  smooth contact's search has reached the 1-D minimum by then: a 50-evaluation search moves qacc
  by < 1e-6 of g;
* bench.ls_cap_stats on env states: its counters add up (every substep one search; converged +
  capped + stalled = searches; the converged replay never caps).
"""
import numpy as np

import test_friction_kat as F
from oracle import oracle as O


def _substeps(case, n=12, warm=150):
    theta, mu = F.CASES[case]
    m = F.ball_model(theta, mu)
    m50 = O.with_ls_iterations(m, 50)
    assert m.ls_iterations == 5 and m.iterations == 1  # the reference's solver (xml:57)
    q, v, w, _, _ = F.run_oracle(m, warm)
    O.ls_take()
    rows = []
    for _ in range(n):
        q2, v2, w2, _, _ = O.mj_step(m, q, v, w, F.DP.copy(), nsteps=1)
        c5 = O.ls_take()
        _, v3, w3, _, _ = O.mj_step(m50, q, v, w, F.DP.copy(), nsteps=1)
        c50 = O.ls_take()
        rows.append(dict(c5=c5, c50=c50, dqacc=np.abs(w2[0:6] - w3[0:6]).max(), dqvel=np.abs(v2[0:6] - v3[0:6]).max()))
        q, v, w = q2, v2, w2
    return rows


def test_cap_binds_on_the_sliding_ball():
    rows = _substeps("slide")
    capped = [r for r in rows if r["c5"]["capped"]]
    free = [r for r in rows if not r["c5"]["capped"]]
    for r in rows:
        assert r["c5"]["searches"] == 1 and r["c50"]["searches"] == 1
        assert r["c5"]["converged"] + r["c5"]["capped"] + r["c5"]["stalled"] == 1
        assert r["c50"]["capped"] == 0  # 50 evaluations always suffice here
        assert r["c5"]["evals"] <= 5 + 2  # the bracket loop may finish its round (p1next / p2next)
        # the capped searches split by the phase they ran out in (bench ls_cap)
        c = r["c5"]
        assert c["capped_one_sided"] + c["capped_bracketing"] == c["capped"]
        assert c["capped_one_sided"] >= 0 and c["capped_bracketing"] <= c["bracketing"] <= c["searches"]
    assert len(capped) >= 4 and len(free) >= 2, [r["c5"] for r in rows]
    # a capped search returns a different step: by up to tens of m/s^2 on this contact
    assert max(r["dqacc"] for r in capped) > 10.0
    assert all(r["dqacc"] > 1e-3 for r in capped)
    # a search that converged inside the budget is unchanged by a larger budget, bit for bit
    assert all(r["dqacc"] == 0.0 and r["dqvel"] == 0.0 for r in free)


def test_cap_binds_harmlessly_on_the_rolling_ball():
    rows = _substeps("roll")
    assert all(r["c5"]["capped"] == 1 for r in rows)  # gtol is never met within 5 evaluations ...
    # with 50 evaluations nearly every search converges (one may still spend all 50 on rounding noise)
    assert sum(r["c50"]["converged"] for r in rows) >= len(rows) - 2
    assert max(r["dqacc"] for r in rows) < 1e-6 * F.G  # ... but the search already sits at the minimum


def test_bench_ls_cap_stats_counts_add_up():
    import bench
    from pupperv3_mjx import MODEL_XML, _abi, sharding
    from pupperv3_mjx.environment import PupperV3Env
    n = 24
    env = PupperV3Env(**bench.bench_kwargs(MODEL_XML), num_envs=n, create_device=False)
    m, cfg = env.sys_model.struct, env.config_struct
    keys = sharding.shard_keys(0, n, 1, 0)
    oe = O.OracleEnv(m, cfg)
    sts, obs = [], []
    for i in range(n):
        r = oe.reset(keys[i])
        r["state"][_abi.S_COMMAND:_abi.S_COMMAND + 3] = [0.5, 0.0, 0.0]
        sts.append(r["state"])
        obs.append(r["obs"])
    rs = np.random.RandomState(0)
    st, ob, _, _ = O.rollout(m, cfg, np.array(sts), np.array(obs), rs.uniform(-1, 1, size=(25, n, 12)), 25, 2)
    recs = st.astype(np.float32)  # the device record layout: RNG words as float bit patterns
    recs[:, _abi.S_RNG:_abi.S_RNG + 2] = st[:, _abi.S_RNG:_abi.S_RNG + 2].astype(np.uint32).view(np.float32)
    res = bench.ls_cap_stats(env, recs, ob.astype(np.float32), rs.uniform(-1, 1, size=(n, 12)).astype(np.float32),
                             np.arange(n))
    c = res["counts"]
    for p in ("f64", "f32"):
        assert c[p]["searches"] == n * env._n_frames
        assert c[p]["converged"] + c[p]["capped"] + c[p]["stalled"] == c[p]["searches"]
    assert c["f64_converged_run"]["searches"] == n * env._n_frames and c["f64_converged_run"]["capped"] == 0
    assert 0.0 <= res["frac_capped"] <= 1.0 and res["ls_iterations"] == 5
    assert res["frac_capped"] == round(c["f64"]["capped"] / c["f64"]["searches"], 5)
    d = res["vs_converged_search"]
    assert d["qpos_abs"]["p50"] <= d["qpos_abs"]["p99"] <= d["qpos_abs"]["max"]
    # landing robots: some searches cap, and then the step differs from the converged one
    assert c["f64"]["capped"] > 0 and d["qpos_abs"]["max"] > 0.0
