#!/usr/bin/env python
"""bench.py -- env-steps/sec of the fused PupperV3Env.step HIP kernel (BASELINE.json metric).

One "step" = one batched env step of E envs per GPU (E = 4096, BASELINE configs[1]): action
latency + kick + 5 MuJoCo-semantics physics substeps + observation + 18 reward terms +
termination, all inside ONE kernel launch (csrc/pp3_env.hip).  Workload: test_pupper_model.xml,
flat terrain, the reference test fixture's env kwargs (test_environment.py:64-113, H=2),
fixed forward command (0.5, 0, 0), no domain randomisation, actions U(-1,1) pre-generated in
HBM (synthetic).  Multi-GPU: one process per GPU (torch.distributed.run), envs sharded with no
data-path collective (weak scaling); barrier + max-over-ranks timing over RCCL.

  python bench.py [--gpus N --steps K --warmup W --envs E --dr --gather --no-cpu-baseline]

Multi-GPU: `python bench.py --gpus N` starts N rank processes itself (launch_ranks: RANK /
LOCAL_RANK / WORLD_SIZE set per child, before this process touches HIP) and relays rank 0's JSON
line; under torch.distributed.run (WORLD_SIZE already set) the process is one rank and --gpus
must equal WORLD_SIZE.  No torch: ranks talk through the library's own RCCL communicator
(pp3_comm_*: barrier, max-over-ranks timing, the --gather collective), created from an id
exchanged by a file rendezvous on the node.  With N > 1 every run also checks the multi-rank
gather once, untimed (gather_check: per-rank checksums of the packed rows vs what landed at the
root and in the all-gather).
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]

METRIC = "env-steps/sec at N_envs=4096/GPU, 1/2/4/8 MI355X; qpos rel-err vs mj_step"
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TFLOPS = 157.3    # vector FP32 (spec)
# 256 CUs x 4 SIMDs; peak engine clock; a wave64 VALU instruction occupies a SIMD-32 for 2 cycles
# when the SIMD is fed by >= 2 waves (MI355X_MICROARCH.md "Wave scheduling"; one wave alone
# sustains one per 4 cycles).  Transcendentals are counted at the plain rate (a lower bound).
N_SIMD, CLOCK_HZ, VALU_CYC = 1024, 2.4e9, 2
KERNEL_SOURCES = ("pupperv3-mjx_amd/csrc/pp3_env.hip", "pupperv3-mjx_amd/csrc/pp3_device.h",
                  "pupperv3-mjx_amd/csrc/pp3_mlp.h", "pupperv3-mjx_amd/csrc/Makefile")
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic_current.json")


def algorithmic_bytes_per_env_step(stride: int, H: int, dr: bool, trajectory: bool = False) -> int:
    """HBM bytes one env step must move (DESIGN.md 'Roofline'): state record read+write,
    obs history read (36(H-1)) + write (36H), actions in, reward/done/metrics out, DR params;
    a fused rollout also writes the step's trajectory row (reward, done, obs 36H)."""
    words = 2 * stride + 36 * (H - 1) + 36 * H + 12 + 2 + 19 + (62 if dr else 0) + ((2 + 36 * H) if trajectory else 0)
    return 4 * words


def bench_kwargs(model_path, random_commands=False):
    from pupperv3_mjx import config, domain_randomization
    return dict(
        path=model_path, reward_config=config.get_config(), action_scale=0.75, observation_history=2,
        joint_lower_limits=[-1.22, -0.42, -2.79, -2.51, -3.14, -0.71, -1.22, -0.42, -2.79, -2.51, -3.14, -0.71],
        joint_upper_limits=[2.51, 3.14, 0.71, 1.22, 0.42, 2.79, 2.51, 3.14, 0.71, 1.22, 0.42, 2.79],
        dof_damping=0.25, position_control_kp=5.0,
        # fixed command (configs[1]); configs[3]: the reference's default resampling every 500 steps
        resample_velocity_step=500 if random_commands else 2 ** 30,
        maximum_pitch_command=30, maximum_roll_command=30,
        start_position_config=domain_randomization.StartPositionRandomization(
            x_min=-1.0, x_max=1.0, y_min=-1.0, y_max=1.0, z_min=0.18, z_max=0.24),
        kick_vel=1.0, kick_probability=0.04, terminal_body_z=0.1, early_termination_step_threshold=500,
    )


def kernel_source_sha16() -> str:
    """Hash of the sources the step kernel is built from: a PMC profile (profiles/traffic_current.json)
    is only used for the kernel it was measured on."""
    import hashlib
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update(open(os.path.join(ROOT, f), "rb").read())
    return h.hexdigest()[:16]


def _oracle_record(rec):
    """Device f32 state record (RNG words bit-cast) -> the oracle's float64 record."""
    import numpy as np
    from pupperv3_mjx import _abi
    with np.errstate(invalid="ignore"):
        out = rec.astype(np.float64)
    out[..., _abi.S_RNG:_abi.S_RNG + 2] = rec[..., _abi.S_RNG:_abi.S_RNG + 2].copy().view(np.uint32)
    return out


def one_step_err(env, n_sample=256, seed=0, dr_table=None, terrain=None, auto_reset=False):
    """SURVEY 7 hard part 2: one env step (n_frames substeps) of the fp32 kernel vs the fp64 oracle
    restatement from IDENTICAL states, on the workload's own states after the timed run.  Each
    sampled env is checked against an oracle env built on ITS model: its domain-randomisation row
    (`dr_table`) and its terrain (`terrain`).  With auto-reset on, envs that ended their episode in
    this step hold the episode's first state, not a physics step: they are left out (counted).
    Returns (one_step_err, ls_cap): ls_cap = ls_cap_stats on the same states and actions."""
    import numpy as np
    from pupperv3_mjx import _abi, _lib
    from oracle import oracle as O
    E = env.num_envs
    rec0 = env._get(_abi.F_STATE)
    obs0 = env._get(_abi.F_OBS)
    a = np.random.RandomState(seed).uniform(-1, 1, size=(E, 12)).astype(np.float32)
    buf = _lib.DeviceBuffer(a.nbytes, env.device)
    buf.upload(a)
    env.step_device(buf.ptr.value)
    env.synchronize()
    rec1 = env._get(_abi.F_STATE)
    done = env._get(_abi.F_DONE).reshape(E) != 0
    buf.free()
    ids = np.random.RandomState(seed + 1).choice(E, size=min(n_sample, E), replace=False)
    n_reset = int(done[ids].sum()) if auto_reset else 0
    if auto_reset:
        ids = ids[~done[ids]]
    base = O.OracleEnv(env.sys_model.struct, env.config_struct, precision="f64")
    dq, dv, rq, flagged = [], [], [], []
    for i in ids:
        oe = base
        if dr_table is not None or terrain is not None:
            m = env.sys_model.struct if terrain is None else O.model_with_terrain(env.sys_model.struct, terrain[i])
            oe = O.OracleEnv(m, env.config_struct, dr=None if dr_table is None else dr_table[i], precision="f64")
        o = oe.step(dict(state=_oracle_record(rec0[i]), obs=obs0[i].astype(np.float64)), a[i].astype(np.float64))
        q_o, v_o = o["state"][0:19], o["state"][19:37]
        dq.append(np.abs(rec1[i, 0:19] - q_o).max())
        dv.append(np.abs(rec1[i, 19:37] - v_o).max())
        rq.append(np.abs(rec1[i, 0:19] - q_o).max() / max(np.abs(q_o).max(), 1e-9))
        flagged.append(o["boundary"] > 0)
    dq, dv, rq, flagged = map(np.array, (dq, dv, rq, flagged))

    def st(x):
        return {"max": float(x.max()), "median": float(np.median(x)), "p99": float(np.percentile(x, 99))}

    ok = ~flagged
    err = {"envs": int(len(ids)), "substeps": int(env._n_frames), "vs": "fp64 oracle restatement, identical start state",
           "qpos_abs": st(dq), "qvel_abs": st(dv), "qpos_rel": st(rq),
           "constraint_flip_envs": int(flagged.sum()),
           "per_env_model": {"dr": dr_table is not None, "terrain": terrain is not None},
           "auto_reset_envs_excluded": n_reset,
           "qpos_abs_max_unflagged": float(dq[ok].max()) if ok.any() else None,
           "qvel_abs_max_unflagged": float(dv[ok].max()) if ok.any() else None}
    return err, ls_cap_stats(env, rec0[ids], obs0[ids], a[ids], ids, dr_table, terrain)


def ls_cap_stats(env, recs, obs, acts, ids, dr_table=None, terrain=None, converged_iters=50):
    """How much of the hot path rests on the unpinned truncated line search (verdict r04 item 1).
    The model runs Newton with iterations=1, ls_iterations=5 (test_pupper_model.xml:57): every
    substep's qacc is ONE line-searched Newton step.  Where the search ends by its 5-evaluation cap
    instead of by convergence, the returned alpha comes from PrimalSearch's exit rule, which MuJoCo's
    documentation does not specify (the oracle and the kernel restate it identically).  On the given
    post-window states (the same states and actions as one_step_err), one env step of the oracle is
    replayed (a) as the reference runs it, counting how each Newton search ended, in fp64 and in fp32
    (the kernel's arithmetic, same exit rule), and (b) in fp64 with the search run to convergence
    (ls_iterations = `converged_iters`) from the identical state: the (a)-(b) one-step qpos / qvel
    differences bound what the undocumented exit rule can move."""
    import numpy as np
    from oracle import oracle as O
    cfg = env.config_struct

    def model_of(i, iters):
        m = env.sys_model.struct if terrain is None else O.model_with_terrain(env.sys_model.struct, terrain[i])
        return O.with_ls_iterations(m, iters) if iters else m

    counts = {p: {"searches": 0, "evals": 0, "converged": 0, "capped": 0, "stalled": 0, "bracketing": 0,
                  "capped_one_sided": 0, "capped_bracketing": 0} for p in ("f64", "f32")}
    counts["f64_converged_run"] = {"searches": 0, "capped": 0, "stalled": 0}
    capped_env = []
    dq, dv, rq = [], [], []
    cap_iters = int(env.sys_model.struct.ls_iterations)
    for p in ("f64", "f32"):
        O.ls_take(p)
    for j, i in enumerate(ids):
        dr = None if dr_table is None else dr_table[i]
        s0 = dict(state=_oracle_record(recs[j]), obs=obs[j].astype(np.float64))
        act = acts[j].astype(np.float64)
        outs = {}
        for p in ("f64", "f32"):
            o = O.OracleEnv(model_of(i, 0), cfg, dr=dr, precision=p).step(s0, act)
            c = O.ls_take(p)
            for k in counts[p]:
                counts[p][k] += c[k]
            if p == "f64":
                outs["cap"] = o
                capped_env.append(c["capped"] > 0)
        o50 = O.OracleEnv(model_of(i, converged_iters), cfg, dr=dr, precision="f64").step(s0, act)
        c50 = O.ls_take("f64")
        for k in ("searches", "capped", "stalled"):
            counts["f64_converged_run"][k] += c50[k]
        q5, v5 = outs["cap"]["state"][0:19], outs["cap"]["state"][19:37]
        q50, v50 = o50["state"][0:19], o50["state"][19:37]
        dq.append(np.abs(q5 - q50).max())
        dv.append(np.abs(v5 - v50).max())
        rq.append(np.abs(q5 - q50).max() / max(np.abs(q50).max(), 1e-9))
    dq, dv, rq = map(np.array, (dq, dv, rq))

    def st(x):
        return {"p50": float(np.median(x)), "p99": float(np.percentile(x, 99)), "max": float(x.max())}

    def frac(c, k):
        return round(c[k] / max(c["searches"], 1), 5)

    return {"envs": int(len(ids)), "substeps_per_env_step": int(env._n_frames), "ls_iterations": cap_iters,
            "frac_capped": frac(counts["f64"], "capped"), "frac_stalled": frac(counts["f64"], "stalled"),
            "frac_converged": frac(counts["f64"], "converged"),
            "frac_capped_f32": frac(counts["f32"], "capped"),
            # where the capped searches ended: the one-sided Newton phase returns its last point (it
            # depends only on the one-sided exit), the bracketing phase the better end of the bracket
            # (it depends on updateBracket's candidate rules as restated): DESIGN.md 5
            "capped_one_sided": frac(counts["f64"], "capped_one_sided"),
            "capped_bracketing": frac(counts["f64"], "capped_bracketing"),
            "frac_reaching_bracketing": frac(counts["f64"], "bracketing"),
            "evals_per_search": round(counts["f64"]["evals"] / max(counts["f64"]["searches"], 1), 3),
            "frac_env_steps_with_a_capped_search": round(float(np.mean(capped_env)), 4),
            "counts": counts,
            "vs_converged_search": {"ls_iterations": converged_iters, "qpos_abs": st(dq), "qvel_abs": st(dv),
                                    "qpos_rel": st(rq)},
            "note": "oracle replay of one env step from the post-window states: the fraction of Newton searches "
                    "ended by the ls_iterations cap (alpha from PrimalSearch's undocumented exit rule) and the "
                    "one-step state difference against the same step with the search run to convergence"}


def contact_cap_stats(env, acts_ptr, steps):
    """Untimed: `steps` env steps with the pipeline record on; counts env steps whose penetrating
    pairs exceed the contact cap (PP3_P_NHIT > the kernel's cap): where the cap binds, the kernel
    (like the oracle) keeps the deepest and departs from MuJoCo-CPU's keep-all.  With
    obstacle boxes it also counts the sphere-box contacts (box_contacts: env steps whose last
    substep had one, and their total), i.e. how much of the workload is on the obstacle path."""
    import numpy as np
    from pupperv3_mjx import _abi, _lib
    m = env.sys_model.struct
    boxes = np.array([int(m.cgeom_id[g]) for g in range(m.ncgeom)
                      if m.cgeom_type[g] == _abi.GEOM_BOX and m.cgeom_bodyid[g] == 0])
    cap = env.config_struct.ncon_max or 8
    _lib.check(env._L.pp3_set_pipeline_output(env._h, 1))
    over = 0
    max_hit = 0
    hist = None
    box_env_steps, box_total = 0, 0
    for i in range(steps):
        env.step_device(acts_ptr + i * env.num_envs * 48)
        p = env._get(_abi.F_PIPELINE)
        nhit = p[:, _abi.P_NHIT].astype(int)
        over += int((nhit > cap).sum())
        max_hit = max(max_hit, int(nhit.max()))
        ncon = p[:, _abi.P_NCON].astype(int)
        hist = np.bincount(ncon, minlength=cap + 1).tolist()
        if boxes.size:
            g = p[:, _abi.P_CON_GEOM:_abi.P_CON_GEOM + 32].reshape(-1, 16, 2).astype(int)
            live = np.arange(16)[None, :] < ncon[:, None]
            nb = (live & (np.isin(g[..., 0], boxes) | np.isin(g[..., 1], boxes))).sum(axis=1)
            box_env_steps += int((nb > 0).sum())
            box_total += int(nb.sum())
    _lib.check(env._L.pp3_set_pipeline_output(env._h, 0))
    out = {"cap": int(cap), "env_steps": int(steps * env.num_envs), "overflow_env_steps": over,
           "max_penetrating_pairs": max_hit, "active_contact_hist_last_step": hist}
    if boxes.size:
        out["box_contacts"] = {"env_steps_with_box_contact": box_env_steps, "box_contacts_total": box_total,
                               "frac_env_steps": round(box_env_steps / (steps * env.num_envs), 4)}
    return out


def host_api_rates(model_path, E, device, keys, steps=30, loop_steps=96, warmup=3):
    """Untimed extra (verdict r02 item 5): the drop-in host surface -- `env.step(state, action)` and
    `wrappers.wrap(env).step` with numpy actions and the State returned to the host every step
    (obs / reward / done stored by the step launch into page-locked memory, the rest lazily; an
    unedited state is not re-uploaded) --
    at the bench's env count, with the constructor's default pipeline record and without it; and
    `rollout(state, actions[K])` (one fused launch for K steps, the trajectory returned to the
    host).  Each rate is the better of two windows (host jitter): `steps` steps for rollout (K =
    `steps`, a PPO unroll), `loop_steps` for the step loops (six queued-step batches: a loop's
    steady state rather than its first batch's start-up)."""
    import numpy as np
    from pupperv3_mjx import wrappers
    from pupperv3_mjx.environment import PupperV3Env
    acts = np.random.RandomState(3).uniform(-1, 1, size=(warmup + 2 * max(steps, loop_steps), E, 12)).astype(np.float32)
    out = {}
    for pipe in (True, False):
        for wrapped in (False, True):
            for roll in ((False, True) if not pipe else (False,)):
                env = PupperV3Env(**bench_kwargs(model_path), num_envs=E, device=device, pipeline_output=pipe)
                api = wrappers.wrap(env, episode_length=1000) if wrapped else env
                st = api.reset(keys)
                for i in range(warmup):
                    st = api.step(st, acts[i])
                if roll:  # a loop's first two unrolls allocate its two page-locked trajectory blocks
                    for _ in range(2):
                        st, _tr = api.rollout(st, acts[warmup:warmup + steps])
                    del _tr
                best = 0.0
                n = steps if roll else loop_steps
                for w in range(2):
                    a0 = warmup + w * n
                    t = time.perf_counter()
                    if roll:
                        st, _ = api.rollout(st, acts[a0:a0 + n])
                    else:
                        for i in range(n):
                            st = api.step(st, acts[a0 + i])
                        _ = st.obs[0, 0]  # the window ends when the last step's outputs are on the host
                    best = max(best, E * n / (time.perf_counter() - t))
                name = ("wrap(env)" if wrapped else "env") + (f".rollout(K={steps})" if roll else ".step")
                out[name + ("" if pipe else " [pipeline_output=False]")] = round(best, 1)
                if not roll and not wrapped and pipe:
                    # a host policy's loop: the caller reads every step's observation before the next
                    best = 0.0
                    for w in range(2):
                        a0 = warmup + w * loop_steps
                        t = time.perf_counter()
                        for i in range(loop_steps):
                            st = api.step(st, acts[a0 + i])
                            _ = st.obs[0, 0]
                        best = max(best, E * loop_steps / (time.perf_counter() - t))
                    out["env.step, obs read every step"] = round(best, 1)
                env.close()
    out["per_step_pcie_bytes"] = {"h2d_actions": E * 12 * 4, "d2h_obs_reward_done": E * (72 + 2) * 4,
                                  "d2h_note": "per state read; a step loop reads only its last state's rows"}
    out["note"] = ("env-steps/s through the host API (numpy in, numpy out; step: asynchronous, the launches "
                   "issued when a queued state is read or the queue holds environment.STEP_BATCH steps, "
                   "consecutive steps fused into one launch, obs / reward / done of the states the "
                   "caller still holds (here the last) stored by it into page-locked host memory, the "
                   "window closed by reading the last step's obs; "
                   "'obs read every step': the loop reads each step's observation before the next step, as "
                   "a host policy does; rollout: one launch and one sync per K steps, the K-step trajectory "
                   "stored into page-locked host memory); the device path is `value`")
    return out


def host_cores() -> dict:
    """What the host offers this process: the machine's CPUs, the ones this process may run on,
    and the OpenMP thread count the pool sets (OMP_NUM_THREADS is the GPU box's per-GPU CPU share;
    the box's rules say to leave it)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return {"os_cpu_count": os.cpu_count(), "affinity": aff, "omp_num_threads": omp or None,
            "threads": omp or aff}


def cpu_baseline(model, cfg, states, obs, seconds_target=12.0):
    """Time the oracle (C fp64 restatement of the same step, OpenMP over envs) on every host core
    this process may use (sched_getaffinity, or OMP_NUM_THREADS where the pool sets it), 64 envs
    per thread."""
    import numpy as np
    from oracle import oracle as O
    hc = host_cores()
    threads = hc["threads"]
    n = min(states.shape[0], 64 * threads)
    if n < 64 * threads:  # more cores than the GPU workload has envs: tile the states
        reps = -(-64 * threads // states.shape[0])
        states, obs = np.concatenate([states] * reps)[:64 * threads], np.concatenate([obs] * reps)[:64 * threads]
        n = 64 * threads
    st = states[:n].copy()
    ob = obs[:n].copy()
    rs = np.random.RandomState(0)
    # calibrate on 2 steps, then size the sample to ~seconds_target of wall time (bounded)
    t = time.time()
    st, ob, _, used = O.rollout(model, cfg, st, ob, rs.uniform(-1, 1, size=(2, n, 12)), 2, threads)
    per = (time.time() - t) / 2
    k = int(max(2, min(20000, seconds_target / max(per, 1e-6))))
    acts = rs.uniform(-1, 1, size=(k, n, 12))
    t = time.time()
    st, ob, _, used = O.rollout(model, cfg, st, ob, acts, k, threads)
    dt = time.time() - t
    return {"value": n * k / dt, "unit": "env-steps/s", "cores": int(used), "kind": "port", "host_cores": hc,
            "sample": f"{n} envs x {k} steps of the fp64 C oracle (pp3_oracle.c restatement of mj_step + env, "
                      f"not MuJoCo), OpenMP {used} threads = "
                      + ("OMP_NUM_THREADS (the pool's CPU share per GPU)" if hc["omp_num_threads"] else
                         "every CPU in this process's affinity mask")
                      + f", {dt:.1f} s wall"}


def qpos_drift(env, nsub=1000, dr_row=None, terrain_row=None):
    """Standing PD hold: GPU fp32 vs fp64 oracle relative qpos drift after nsub substeps
    (env 0, against an oracle on env 0's model: its DR row and terrain when the workload has them)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from pupperv3_mjx import _abi, _lib
    from oracle import oracle as O
    dp = [0.26, 0.0, -0.52, -0.26, 0.0, 0.52, 0.26, 0.0, -0.52, -0.26, 0.0, 0.52]
    n = env.num_envs
    rec = np.zeros((n, env.stride), dtype=np.float32)
    rec[:, 2] = 0.17
    rec[:, 3] = 1
    rec[:, 7:19] = dp
    env._put(_abi.F_STATE, rec)
    ctrl = np.tile(np.array(dp, dtype=np.float32), (n, 1))
    buf = _lib.DeviceBuffer(ctrl.nbytes, env.device)
    buf.upload(ctrl)
    _lib.check(env._L.pp3_physics_step(env._h, buf.ptr, nsub, None))
    env.synchronize()
    g = env._get(_abi.F_STATE)[0, :19].astype(np.float64)
    q0 = np.zeros(19)
    q0[2], q0[3], q0[7:] = 0.17, 1, dp
    m = env.sys_model.struct if terrain_row is None else O.model_with_terrain(env.sys_model.struct, terrain_row)
    o, _, _, _, _ = O.mj_step(m, q0, np.zeros(18), np.zeros(18), np.array(dp), nsteps=nsub, dr=dr_row)
    buf.free()
    return float(np.abs(g - o).max() / np.abs(o).max())


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (this script, RANK / LOCAL_RANK /
    WORLD_SIZE set, one GPU each), wait for them and return the job's exit status (rank 0 prints
    the JSON line; its stdout is this process's).  This parent never touches HIP or the GPU and
    never execs: it only spawns children.  If one rank fails, the others are stopped (they would
    otherwise wait in the next barrier) and the job fails."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    nonce = f"bench{os.getpid()}.{time.time_ns()}"
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PP3_LAUNCH_ID=nonce)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(range(n))
    while live:
        for r in list(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.remove(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py launcher: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    return rc


def gather_check(env, comm, world, rank, nmax):
    """Untimed check of the multi-rank hand-over (pp3_gather), run once per N > 1 job: each rank's
    checksum of its OWN packed rows (sharding.pack_rows of its obs / reward / done), all-reduced,
    must equal the checksum of rank r's slot of what arrived at the root (root 0, grouped send /
    recv) and at every rank (root -1, all-gather); each receiver's own slot must equal its rows bit
    for bit.  Returns the report; every rank learns the verdict (one all-reduce)."""
    import numpy as np
    from pupperv3_mjx import _abi, _lib, sharding
    env.synchronize()
    mine = sharding.pack_rows(env._get(_abi.F_OBS), env._get(_abi.F_REWARD), env._get(_abi.F_DONE), nmax)
    W = mine.shape[1]
    wts = 1.0 + (np.arange(mine.size, dtype=np.float64) % 1021) / 1021.0  # position-sensitive

    def csum(rows):
        return float(np.dot(rows.astype(np.float64).ravel(), wts))
    vec = np.zeros(world)
    vec[rank] = csum(mine)
    expect = comm.allreduce(vec, "sum")  # one nonzero term per entry: exact
    dst = _lib.DeviceBuffer(world * nmax * W * 4, env.device)
    bad = 0
    report = {}
    for root in (0, -1):
        recv = root < 0 or rank == root
        comm.gather(env, nmax, dst.ptr.value if recv else None, root=root)
        env.synchronize()
        if recv:
            full = np.empty((world * nmax, W), dtype=np.float32)
            dst.download(full)
            got = [csum(full[r * nmax:(r + 1) * nmax]) for r in range(world)]
            ok = all(g == e for g, e in zip(got, expect)) and np.array_equal(full[rank * nmax:(rank + 1) * nmax], mine)
            bad += 0 if ok else 1
            if rank == 0:
                report["root0" if root == 0 else "allgather"] = "ok" if ok else "MISMATCH"
    dst.free()
    nbad = int(comm.allreduce([float(bad)], "sum")[0])
    report.update(ranks=world, rows_per_rank=nmax, row_floats=W, failing_receivers=nbad,
                  check="per-rank float64 checksums of pack_rows vs the received slots")
    return report


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks) of the job; default WORLD_SIZE under a launcher, else 1")
    ap.add_argument("--dry-launch", action="store_true",
                    help="ranks report RANK / LOCAL_RANK / WORLD_SIZE as a JSON line and exit before any HIP call")
    ap.add_argument("--no-gather-check", action="store_true", help="skip the N > 1 gather_check")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=200,
                    help="untimed steps first: the drop from the start height settles (steady state)")
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--dr", action="store_true", help="domain randomisation on (configs[2])")
    ap.add_argument("--obstacles", type=int, default=0, help="obstacles.py boxes (configs[4])")
    ap.add_argument("--terrain", action="store_true",
                    help="per-env terrain (SURVEY 8f rank 3): every env gets its own random boxes in the --obstacles slots")
    ap.add_argument("--flat-start", action="store_true",
                    help="with --obstacles: keep the flat start square instead of starting every robot over a box")
    ap.add_argument("--random-commands", action="store_true",
                    help="keep the reset's sampled velocity commands (configs[3]) instead of the fixed (0.5,0,0)")
    ap.add_argument("--gather", action="store_true",
                    help="per-step RCCL hand-over of obs|reward|done to the learner rank (configs[3])")
    ap.add_argument("--gather-root", type=int, default=0, help="learner rank of --gather; -1 = all-gather")
    ap.add_argument("--gather-mode", choices=("step", "unroll"), default="step",
                    help="--gather: hand over every step (single-step launches, one pp3_gather each), or the K "
                         "timed steps as ONE fused rollout whose trajectory is handed over once "
                         "(pp3_gather_rollout: Brax's generate_unroll + one learner hand-over per unroll)")
    ap.add_argument("--auto-reset", type=int, default=0, metavar="EPISODE_LENGTH",
                    help="on-device EpisodeWrapper+AutoResetWrapper (brax training wrap) with this episode length")
    ap.add_argument("--policy", type=str, default="", metavar="H1,H2,...",
                    help="policy-in-the-loop rollout: an exported-format MLP (random weights, elu) computes the "
                         "actions from the observation buffer on device before every env step")
    ap.add_argument("--launch", choices=("rollout", "step"), default="rollout",
                    help="rollout: the K timed steps as ONE fused launch (pp3_rollout, brax generate_unroll's "
                         "lax.scan with the actions given up front; per-step reward/done/obs trajectories written), "
                         "then the same K steps as K single-step launches from the same start state, timed too and "
                         "checked bit-equal; step: K single-step launches only (pp3_step)")
    ap.add_argument("--no-prewarm", action="store_true",
                    help="skip the ~200 ms untimed GPU pre-warm (state restored after it) before the warmup steps")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency-floor", action="store_true",
                    help="skip the E/2-envs latency-floor launches (keeps rocprof stats to E-env launches)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the untimed accuracy / contact-cap measurements (profiling runs)")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus))  # this process only spawns the ranks (no HIP here)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.dry_launch:
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world": world, "pid": os.getpid(),
                          "launch": os.environ.get("PP3_LAUNCH_ID")}), flush=True)
        return
    # rehearsal knob for the multi-rank code on one GPU (never used by the driver): every rank on
    # this device
    device = int(os.environ.get("PP3_BENCH_DEVICE", local_rank))
    import numpy as np
    from pupperv3_mjx import MODEL_XML, _abi, _lib, sharding
    from pupperv3_mjx.environment import PupperV3Env

    comm, comm_kind = None, None
    if world > 1:
        try:
            comm, comm_kind = sharding.Comm(rank, world, device), "RCCL (pp3_comm)"
        except Exception as exc:  # timing still needs a barrier + max over ranks; the shards never exchange data
            if args.gather:
                raise
            print(f"rank {rank}: RCCL communicator unavailable ({exc}); barrier/max-over-ranks through files",
                  file=sys.stderr, flush=True)
            comm, comm_kind = sharding.FileComm(rank, world), "host files (RCCL init failed)"

    model_path = MODEL_XML
    if args.obstacles:
        import xml.etree.ElementTree as ET
        from pupperv3_mjx import obstacles
        tree = ET.ElementTree(ET.fromstring(open(MODEL_XML).read()))
        obstacles.add_boxes_to_model(tree, n_boxes=args.obstacles, x_range=(-5, 5), y_range=(-5, 5), height=0.02,
                                     length=6.0)
        model_path = os.path.join(ROOT, "gpurun_out", f"bench_obstacles_{rank}.xml")
        os.makedirs(os.path.dirname(model_path), exist_ok=True)
        tree.write(model_path, encoding="unicode")

    E = args.envs
    env = PupperV3Env(**bench_kwargs(model_path, args.random_commands), num_envs=E, device=device, pipeline_output=False)
    L = env._L
    dr_table, terrain = None, None
    if args.dr:
        from pupperv3_mjx import domain_randomization as dr, rng
        sysb, _ = dr.domain_randomize(env.sys, rng.split(rng.PRNGKey(1000 + rank), E))
        env.set_domain_randomization(sysb)
        dr_table = sysb.dr_table().astype(np.float64)
    if args.terrain:
        from pupperv3_mjx import obstacles
        if not args.obstacles:
            raise SystemExit("--terrain needs --obstacles N (the box-geom slots)")
        terrain = obstacles.sample_terrain(E, args.obstacles, (-5, 5), (-5, 5), height=0.02, length=6.0,
                                           seed=args.seed * 1000 + rank, min_boxes=args.obstacles // 2)
        env.set_terrain(terrain)
    if args.auto_reset > 0:
        _lib.check(L.pp3_set_auto_reset(env._h, args.auto_reset))
    # global env ids: rank r steps envs [r E, (r + 1) E) of the job's E * world (weak scaling: E per
    # rank, whatever E's parity; sharding.shard_bounds cuts the same ranges when E is even)
    from pupperv3_mjx import rng as _rng
    keys = np.ascontiguousarray(_rng.split(_rng.PRNGKey(args.seed), E * world)[rank * E:(rank + 1) * E])
    st = env.reset(keys)
    rec = st._record.copy()
    if not args.random_commands:
        rec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3] = [0.5, 0.0, 0.0]
    if args.obstacles and not args.flat_start:
        # configs[4]: every robot starts over a box (its own first box with --terrain), so the
        # workload runs the sphere-box contacts it exists to measure (contact_cap.box_contacts)
        from pupperv3_mjx import obstacles
        if terrain is None:
            specs = obstacles.sample_boxes(args.obstacles, (-5, 5), (-5, 5), 0.02, length=6.0)
        else:
            specs = [obstacles.BoxSpec("", float(t[0, 0]), float(t[0, 1]), tuple(float(v) for v in t[0, 3:7]),
                                       tuple(float(v) for v in t[0, 7:10])) for t in terrain]
        xy = obstacles.rail_start_xy(specs, E, seed=args.seed * 1000 + rank)
        rec[:, _abi.S_QPOS:_abi.S_QPOS + 2] = xy
    env._put(_abi.F_STATE, rec)
    init_obs = st.obs.copy()

    total = args.warmup + args.steps
    acts = _lib.DeviceBuffer(total * E * 12 * 4, device)
    _lib.check(L.pp3_fill_uniform(env._h, acts.ptr, total * E * 12, 1234 + rank, 0, -1.0, 1.0, None))
    env.synchronize()
    act_at = lambda i: acts.ptr.value + i * E * 48  # noqa: E731  (actions of step i)
    ms = C.c_float()
    gather_dst, nmax = None, 0
    if args.gather:
        nmax = E  # equal shards: every rank contributes E rows of width 36H + 2
        width = env.observation_size + 2
        if args.gather_root < 0 or rank == args.gather_root:
            per = args.steps if args.gather_mode == "unroll" else 1  # (unroll: [world][K][nmax][width])
            gather_dst = _lib.DeviceBuffer(world * per * nmax * width * 4, device)
        if comm is None:  # one rank: the gather is a pack (a one-rank communicator still runs it)
            comm = sharding.Comm(0, 1, device, tag="_solo")

    def barrier():
        if comm is not None and comm.world > 1:
            comm.barrier()

    policy = None
    if args.policy:
        from types import SimpleNamespace
        from collections import OrderedDict
        from pupperv3_mjx import export
        rs = np.random.RandomState(7)
        sizes = [env.observation_size] + [int(v) for v in args.policy.split(",")] + [2 * _abi.NU]
        layers = OrderedDict((f"hidden_{i}", {"kernel": rs.normal(scale=1 / np.sqrt(sizes[i]), size=(sizes[i], sizes[i + 1])),
                                              "bias": np.zeros(sizes[i + 1])}) for i in range(len(sizes) - 1))
        norm = SimpleNamespace(mean=np.zeros(sizes[0]), std=np.ones(sizes[0]))
        pol = export.convert_params((norm, {"params": layers}), "elu", 0.75, 5.0, 0.25, np.zeros(12), np.ones(12),
                                    -np.ones(12), True, env._observation_history, 30.0, 30.0)
        policy = export.DevicePolicy(pol, device)

    # --launch rollout (the default for the plain env-step workloads): the timed K steps are one
    # fused launch writing per-step trajectories; the start state is kept to replay the same K
    # steps as single-step launches afterwards (timed, and checked bit-equal)
    unroll_gather = args.gather and args.gather_mode == "unroll"
    rollout = args.launch == "rollout" and policy is None and (not args.gather or unroll_gather)
    traj, snap = None, None
    if rollout or policy is not None:
        D = env.observation_size
        traj = [_lib.DeviceBuffer(4 * args.steps * E, device), _lib.DeviceBuffer(4 * args.steps * E, device),
                _lib.DeviceBuffer(4 * args.steps * E * D, device)]
    # device-side snapshots of the env's state buffers (D2D copies queued on the env's stream, no
    # host round trip): the pre-warm and the single-step replay restore them
    snap_fields = [_abi.F_STATE, _abi.F_OBS, _abi.F_REWARD, _abi.F_DONE] + ([_abi.F_EPISODE] if args.auto_reset else [])
    stream = L.pp3_stream(env._h)

    def dev_snapshot(bufs=None):
        bufs = bufs or {f: _lib.DeviceBuffer(4 * E * env.device_field(f)[1], device) for f in snap_fields}
        for f, b in bufs.items():
            _lib.check(L.pp3_memcpy_d2d(b.ptr, C.c_void_p(env.device_field(f)[0]), b.nbytes, stream))
        return bufs

    def dev_restore(bufs):
        env._before_launch()
        for f, b in bufs.items():
            _lib.check(L.pp3_memcpy_d2d(C.c_void_p(env.device_field(f)[0]), b.ptr, b.nbytes, stream))

    # GPU pre-warm (untimed; the env's state is restored afterwards): ~200 ms of the same launches,
    # so the timed window runs at the clocks of a busy GPU.  After a host-side pause of 0.2 s the
    # same 20-step window measured 6-7 % slower than right after continuous work;
    # a training loop keeps the GPU busy.  --no-prewarm measures from the idle state.
    prewarm_ms = 0.0
    if not args.no_prewarm:
        s0 = dev_snapshot()
        t_pw = time.perf_counter()
        n_pw = 0
        while time.perf_counter() - t_pw < 0.2:
            _lib.check(L.pp3_rollout(env._h, acts.ptr, E * 12, min(total, 20), None, None, None, None))
            dev_restore(s0)
            n_pw += 1
            if n_pw % 4 == 0:
                env.synchronize()
        prewarm_ms = (time.perf_counter() - t_pw) * 1e3
    # the W untimed warmup steps, right before the timed window
    if args.warmup:
        if policy is not None:
            _lib.check(L.pp3_rollout_policy(env._h, policy._h, args.warmup, acts.ptr, None, None, None, None))
        else:
            _lib.check(L.pp3_step_timed(env._h, acts.ptr, E * 12, args.warmup, C.byref(ms)))
    if rollout or policy is not None:
        snap = dev_snapshot()  # the timed window's start state

    env.synchronize()
    barrier()
    t0 = time.perf_counter()
    if policy is not None:
        # generate_unroll with the policy in the loop: pp3_rollout_policy, ONE fused launch (per
        # step the workgroup's MLP on its envs' observations, then the env step; action / reward /
        # done / obs trajectories written), HIP events around it
        _lib.check(L.pp3_rollout_policy_timed(env._h, policy._h, args.steps, C.c_void_p(act_at(args.warmup)),
                                              traj[0].ptr, traj[1].ptr, traj[2].ptr, C.byref(ms)))
        kernel_ms = ms.value
    elif rollout:
        _lib.check(L.pp3_rollout_timed(env._h, C.c_void_p(act_at(args.warmup)), E * 12, args.steps,
                                       traj[0].ptr, traj[1].ptr, traj[2].ptr, C.byref(ms)))
        kernel_ms = ms.value
        if unroll_gather:  # the unroll's trajectory to the learner: one collective, on the env stream
            comm.gather_rollout(env, traj[2].ptr.value, traj[0].ptr.value, traj[1].ptr.value, args.steps, nmax,
                                gather_dst.ptr.value if gather_dst else None, root=args.gather_root)
    elif not args.gather:
        _lib.check(L.pp3_step_timed(env._h, C.c_void_p(act_at(args.warmup)), E * 12, args.steps, C.byref(ms)))
        kernel_ms = ms.value
    else:
        # step kernel, then the RCCL hand-over of its outputs, both on the env's stream: no host sync
        for i in range(args.steps):
            env.step_device(act_at(args.warmup + i))
            comm.gather(env, nmax, gather_dst.ptr.value if gather_dst else None, root=args.gather_root)
        kernel_ms = None
    env.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    per_step, idle_start = None, None
    if rollout:
        # the same K steps again as K single-step launches (HIP events) from the kept start state,
        # queued right behind the timed window (the rollout's end state kept on the device first)
        K, D = args.steps, env.observation_size
        end_dev = dev_snapshot()
        dev_restore(snap)
        _lib.check(L.pp3_step_timed(env._h, C.c_void_p(act_at(args.warmup)), E * 12, K, C.byref(ms)))
        step_ms = ms.value
        end = {f: np.empty((E, env.device_field(f)[1]), np.float32) for f in snap_fields}
        for f, a in end.items():
            end_dev[f].download(a)
        # the trajectories' last row against the rollout's outputs
        last_r, last_d, last_o = np.empty(E, np.float32), np.empty(E, np.float32), np.empty(E * D, np.float32)
        _lib.check(L.pp3_memcpy_d2h(last_r.ctypes.data_as(C.c_void_p), C.c_void_p(traj[0].ptr.value + 4 * (K - 1) * E), 4 * E))
        _lib.check(L.pp3_memcpy_d2h(last_d.ctypes.data_as(C.c_void_p), C.c_void_p(traj[1].ptr.value + 4 * (K - 1) * E), 4 * E))
        _lib.check(L.pp3_memcpy_d2h(last_o.ctypes.data_as(C.c_void_p), C.c_void_p(traj[2].ptr.value + 4 * (K - 1) * E * D), 4 * E * D))
        traj_ok = (np.array_equal(last_r, end[_abi.F_REWARD][:, 0]) and np.array_equal(last_d, end[_abi.F_DONE][:, 0])
                   and np.array_equal(last_o.reshape(E, D), end[_abi.F_OBS]))
        # bitwise (the state record holds the rng key words as float bit patterns, some of them NaNs)
        differ = [int(f) for f, v in end.items() if not np.array_equal(env._get(f).view(np.uint32), v.view(np.uint32))]
        same = not differ
        for b in end_dev.values():
            b.free()
        per_step = {"launches": K, "avg_launch_ms": round(step_ms / K, 4),
                    "kernel_env_steps_per_s": round(E * K / (step_ms / 1e3), 1),
                    "bit_equal_to_rollout": bool(same), "trajectory_last_row_equals_outputs": bool(traj_ok)}
        if differ:
            per_step["differing_fields"] = differ
        if not (same and traj_ok):
            print(f"rank {rank}: fused rollout differs from single-step launches: {per_step}", file=sys.stderr, flush=True)
        # idle start (verdict r04 item 5): the same fused window from the same start state after a
        # 0.2 s host pause, so the GPU starts it from the clock state of an idle device instead of
        # behind the pre-warm; HIP events, like the timed window's kernel_ms.  Not `value`.  (Not in
        # --no-extras profiling runs: their kernel stats keep to the timed launch.)
    if rollout and not args.no_extras:
        dev_restore(snap)
        env.synchronize()
        time.sleep(0.2)
        _lib.check(L.pp3_rollout_timed(env._h, C.c_void_p(act_at(args.warmup)), E * 12, K, traj[0].ptr, traj[1].ptr,
                                       traj[2].ptr, C.byref(ms)))
        idle_ms = ms.value
        idle_same = np.array_equal(env._get(_abi.F_STATE).view(np.uint32), end[_abi.F_STATE].view(np.uint32))
        idle_start = {"pause_s": 0.2, "ms_per_step": round(idle_ms / K, 4),
                      "env_steps_per_s": round(E * K / (idle_ms / 1e3), 1),
                      "prewarmed_ms_per_step": round(kernel_ms / K, 4),
                      "prewarmed_env_steps_per_s": round(E * K / (kernel_ms / 1e3), 1),
                      "idle_over_prewarmed": round(idle_ms / kernel_ms, 4), "bit_equal_to_rollout": bool(idle_same),
                      "note": "the timed window replayed from its saved start state after a 0.2 s host pause "
                              "(HIP events around the fused launch) vs the same launch right behind the pre-warm "
                              "and warmup (events); value is the wall clock of the latter"}
        if not idle_same:
            print(f"rank {rank}: idle-start replay differs from the timed rollout", file=sys.stderr, flush=True)
    if rollout:
        for b in snap.values():
            b.free()
        if not unroll_gather:  # (the unroll hand-over is timed alone below, on these buffers)
            for b in traj:
                b.free()
    if policy is not None:
        # the same K steps again as the unfused loop (per step a pp3_policy_act launch on the obs
        # buffer, then a single-step launch) from the kept start state: actions and end state must
        # be bit-equal to the fused launch's
        K = args.steps
        end_dev = dev_snapshot()
        a_fused = np.empty((K, E, 12), np.float32)
        _lib.check(L.pp3_memcpy_d2h(a_fused.ctypes.data_as(C.c_void_p), C.c_void_p(act_at(args.warmup)), a_fused.nbytes))
        dev_restore(snap)
        rbuf = _lib.DeviceBuffer(4 * K * E * 12, device)
        obs_ptr = env.device_field(_abi.F_OBS)[0]
        env.synchronize()
        tr0 = time.perf_counter()
        for t in range(K):
            policy.act(obs_ptr, env.observation_size, E, rbuf.ptr.value + 4 * t * E * 12, 12, stream=stream)
            _lib.check(L.pp3_step(env._h, C.c_void_p(rbuf.ptr.value + 4 * t * E * 12), None))
        env.synchronize()
        unfused_ms = (time.perf_counter() - tr0) * 1e3
        a_unf = np.empty_like(a_fused)
        rbuf.download(a_unf)
        rbuf.free()
        end = {f: np.empty((E, env.device_field(f)[1]), np.float32) for f in snap_fields}
        for f, a in end.items():
            end_dev[f].download(a)
        differ = [int(f) for f, v in end.items() if not np.array_equal(env._get(f).view(np.uint32), v.view(np.uint32))]
        per_step = {"launches": 2 * K, "ms_per_step": round(unfused_ms / K, 4),
                    "env_steps_per_s": round(E * K / (unfused_ms / 1e3), 1),
                    "note": "the same steps as the unfused loop: per step a pp3_policy_act launch, then a pp3_step "
                            "launch (host loop, wall clock)",
                    "actions_bit_equal": bool(np.array_equal(a_fused.view(np.uint32), a_unf.view(np.uint32))),
                    "bit_equal_to_rollout": not differ}
        if differ:
            per_step["differing_fields"] = differ
        if differ or not per_step["actions_bit_equal"]:
            print(f"rank {rank}: fused policy rollout differs from the unfused loop: {per_step}", file=sys.stderr, flush=True)
        for b in list(end_dev.values()) + list(snap.values()):
            b.free()
        for b in traj:
            b.free()
    # the timed window's end state (rank 0's shard; after the replay when it is bit-equal): equal
    # hashes across kernel builds mean the A/B variants ran the same trajectories, so a timing
    # difference is code speed, not a changed workload
    import hashlib
    state_sha16 = hashlib.sha256((end[_abi.F_STATE] if (rollout or policy is not None) else env._get(_abi.F_STATE)).tobytes()).hexdigest()[:16]
    gather_info = None
    if args.gather and not unroll_gather:
        # untimed: the same K steps' kernels alone (events), then the gather alone
        _lib.check(L.pp3_step_timed(env._h, C.c_void_p(act_at(args.warmup)), E * 12, args.steps, C.byref(ms)))
        kernel_ms = ms.value
        env.synchronize()
        barrier()
        tg = time.perf_counter()
        for i in range(args.steps):
            comm.gather(env, nmax, gather_dst.ptr.value if gather_dst else None, root=args.gather_root)
        env.synchronize()
        barrier()
        gather_s = (time.perf_counter() - tg) / args.steps
        gather_info = {"mode": "step", "root": args.gather_root, "rows_per_rank": nmax,
                       "row_floats": env.observation_size + 2, "bytes_per_rank": nmax * (env.observation_size + 2) * 4,
                       "ms_per_gather": round(gather_s * 1e3, 4), "transport": "RCCL (pp3_gather), env stream"}
    elif unroll_gather:
        # untimed: the unroll's hand-over alone (the trajectory buffers still hold the timed unroll)
        env.synchronize()
        barrier()
        tg = time.perf_counter()
        comm.gather_rollout(env, traj[2].ptr.value, traj[0].ptr.value, traj[1].ptr.value, args.steps, nmax,
                            gather_dst.ptr.value if gather_dst else None, root=args.gather_root)
        env.synchronize()
        barrier()
        gather_s = time.perf_counter() - tg
        for b in traj:
            b.free()
        gather_info = {"mode": "unroll", "root": args.gather_root, "steps_per_gather": args.steps,
                       "rows_per_rank": args.steps * nmax, "row_floats": env.observation_size + 2,
                       "bytes_per_rank": args.steps * nmax * (env.observation_size + 2) * 4,
                       "ms_per_gather": round(gather_s * 1e3, 4), "transport": "RCCL (pp3_gather_rollout), env stream"}
    if comm is not None and comm.world > 1:
        wall_max, kernel_ms_max = (float(v) for v in comm.allreduce([wall, kernel_ms], "max"))
    else:
        wall_max, kernel_ms_max = wall, kernel_ms
    n_gpus = comm.world if comm is not None else 1  # the ranks that actually joined the job
    gcheck = None
    if world > 1 and not args.no_gather_check:
        if isinstance(comm, sharding.Comm):
            gcheck = gather_check(env, comm, world, rank, E)
            if gcheck["failing_receivers"]:
                print(f"rank {rank}: gather_check failed: {gcheck}", file=sys.stderr, flush=True)
        else:
            gcheck = {"skipped": f"no RCCL communicator ({comm_kind})"}

    # sanity on the produced batch
    rew = env._get(_abi.F_REWARD)
    obs = env._get(_abi.F_OBS)
    assert np.all(np.isfinite(rew)) and np.all(np.isfinite(obs)), "non-finite env outputs"

    if rank == 0:
        K = args.steps
        value = E * world * K / wall_max
        launch_s = kernel_ms_max / 1e3 / K  # kernel time per env step of the batch
        # the library reports which path pp3_rollout_policy took (fused only at cap 8, action_repeat 1,
        # PP3_POLICY_UNFUSED unset and in a product build)
        fused_policy = policy is not None and L.pp3_rollout_policy_fused(env._h) == 1
        # the step kernels' sphere-box cull (obstacle models): the CULL = true instantiation
        cull = "true" if hasattr(L, "pp3_narrow_cull") and L.pp3_narrow_cull(env._h) == 1 else "false"
        spl = K if (rollout or fused_policy) else 1  # env steps per launch
        bpe = algorithmic_bytes_per_env_step(env.stride, env._observation_history, args.dr,
                                             trajectory=rollout or policy is not None)
        achieved = bpe * E / launch_s / 1e9
        traffic, valu, epw, tsrc, flops, fsrc = None, None, 2, None, None, None
        if os.path.exists(TRAFFIC_FILE):
            # PMC figures of this kernel build and launch shape, per env step of the batch
            # (profiles/traffic_current.json: per-launch values over steps_per_launch)
            tj = json.load(open(TRAFFIC_FILE))
            if (tj.get("src_sha16") == kernel_source_sha16() and tj.get("envs") == E
                    and tj.get("dr", False) == args.dr and not args.obstacles
                    and tj.get("launch", "step") == ("rollout" if rollout else "step")):
                tspl = tj.get("steps_per_launch", 1)
                traffic = tj.get("hbm_bytes_per_launch") / tspl * spl
                valu = tj.get("valu_insts_per_wave") / tspl
                epw = tj.get("envs_per_wave", 2)
                tsrc = tj.get("source")
                if tj.get("fp32_flops_per_launch"):
                    flops, fsrc = tj.get("fp32_flops_per_launch") / tspl, tj.get("fp32_flops_source")
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": n_gpus,
            "steps": K,
            "warmup": args.warmup,
            "gpu_prewarm_ms": round(prewarm_ms, 1),
            "ms_per_step": round(wall_max / K * 1e3, 4),
            "state_sha16": state_sha16,
            # the step kernel's sources (profiles/README.md names each version by this hash)
            "kernel_src_sha16": kernel_source_sha16(),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (actions U(-1,1) pre-generated in HBM; reset keys = jax.random.split(PRNGKey(seed), E))",
            "config": {"workload": ("configs[1]: test_pupper_model.xml, %d envs/GPU, %s, %s, %s"
                                    % (E, "flat terrain" if not args.obstacles else
                                       f"{args.obstacles} obstacle boxes" + ("" if args.flat_start else ", robots started over the boxes"),
                                       "random commands" if args.random_commands else "fixed command (0.5,0,0)",
                                       "domain randomisation" if args.dr else "no DR")),
                       "envs_per_gpu": E, "global_envs": E * world, "obs_history": env._observation_history,
                       "n_frames": env._n_frames, "parallelism": f"env-sharded x{world} (no data-path collective)"
                       if not args.gather else (f"env-sharded x{world} + per-step RCCL gather to rank {args.gather_root}"
                                                if not unroll_gather else
                                                f"env-sharded x{world} + one RCCL gather of the {args.steps}-step unroll "
                                                f"to rank {args.gather_root}"),
                       "per_env_terrain": bool(args.terrain),
                       "commands": "reset-sampled, resampled every 500 steps" if args.random_commands else "fixed (0.5,0,0)",
                       "gather": gather_info, "gather_check": gcheck, "comm": comm_kind, "auto_reset_episode_length": args.auto_reset or None,
                       "policy_in_loop": args.policy or None},
            "launch": (f"rollout: the {K} timed steps fused into one pp3_rollout launch (per-step reward/done/obs "
                       "trajectories written); per_step_launch = the same steps as single-step launches"
                       if rollout else
                       ("policy: pp3_rollout_policy, the K steps as ONE fused launch (8-wave workgroups of 16 envs run "
                        "the MLP before each step; action/reward/done/obs trajectories written); per_step_launch = "
                        "the same steps as per-step policy + step launches"
                        if policy is not None else "step: one pp3_step launch per env step")),
            "per_step_launch": per_step,
            "idle_start": idle_start,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "kernel": ("pp3::env_step_kernel<8, true, 8, %s> (policy MLP fused)" % cull if fused_policy else
                                    "pp3::env_step_kernel<%d, %s, 1, %s>" % (env.config_struct.ncon_max or 8, "true" if rollout else "false",
                                                                             cull)),
                         "steps_per_launch": spl, "bytes_per_env_step": bpe,
                         "algorithmic_bytes_per_launch": bpe * E * spl,
                         "launch_ms": round(launch_s * spl * 1e3, 4),
                         "avg_launch_ms": round(launch_s * 1e3, 4),
                         "traffic_source": tsrc or "none for this kernel build (profiles/traffic_current.json "
                                                   "src_sha16 != the kernel sources' hash)"},
        }
        if valu:
            # Compute-side bound: VALU issue.  One wave = `epw` envs; E/epw waves over
            # 1024 SIMDs; a wave64 VALU instruction holds its SIMD for VALU_CYC cycles at 2.4 GHz.
            ceil_s = valu * VALU_CYC * (E / epw) / (N_SIMD * CLOCK_HZ)
            out["roofline"]["valu_issue"] = {"valu_insts_per_wave": valu, "envs_per_wave": epw,
                                             "cycles_per_valu": VALU_CYC,
                                             "ceiling_ms": round(ceil_s * 1e3, 4),
                                             "frac": round(ceil_s / launch_s, 4),
                                             "source": "profiles/traffic_current.json (rocprofv3 SQ_INSTS_VALU)"}
        if flops:
            # Arithmetic side: executed FP32 VALU operations per launch from the PMC
            # instruction mix (64 lanes x (2 FMA + ADD + MUL + TRANS)), over this run's launch time,
            # against the FP32 vector peak.  Every lane counts, masked or replicated: an upper bound.
            out["roofline"]["fp32_vector"] = {"executed_flops_per_env_step": round(flops / E, 1),
                                              "achieved": round(flops / launch_s / 1e12, 3),
                                              "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                                              "frac": round(flops / launch_s / 1e12 / FP32_PEAK_TFLOPS, 5),
                                              "source": fsrc}
        if (world == 1 and policy is None and not args.gather and E == 4096 and not args.dr and not args.obstacles
                and not args.auto_reset and not args.no_latency_floor):
            # Latency floor: the same step at E/2 envs puts ONE wave (two envs)
            # on each SIMD; the kernel then takes one wave's critical path.  ratio = launch time at E
            # / launch time at E/2 (1.0 = the second wave per SIMD is free: latency-bound).
            half = PupperV3Env(**bench_kwargs(model_path, args.random_commands), num_envs=E // 2, device=device,
                               pipeline_output=False)
            hst = half.reset(keys[: E // 2])
            hrec = hst._record.copy()
            hrec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3] = rec[: E // 2, _abi.S_COMMAND:_abi.S_COMMAND + 3]
            half._put(_abi.F_STATE, hrec)
            _lib.check(L.pp3_step_timed(half._h, acts.ptr, E // 2 * 12, args.warmup or 5, C.byref(ms)))
            hk = min(args.steps, 100)
            if rollout:  # the same launch shape as the measured one
                _lib.check(L.pp3_rollout_timed(half._h, acts.ptr, E // 2 * 12, hk, None, None, None, C.byref(ms)))
            else:
                _lib.check(L.pp3_step_timed(half._h, acts.ptr, E // 2 * 12, hk, C.byref(ms)))
            half_s = ms.value / 1e3 / hk
            half.close()
            out["roofline"]["latency"] = {"envs": E // 2, "waves_per_simd": (E // 2) / 2 / N_SIMD,
                                          "avg_launch_ms": round(half_s * 1e3, 4),
                                          "ratio": round(launch_s / half_s, 4),
                                          "note": "launch time at E / at E/2 envs (one wave per SIMD)"}
        lat, vi = out["roofline"].get("latency"), out["roofline"].get("valu_issue")
        # what binds the launch: the HBM traffic of the contract's `bound` is ~1 % of
        # peak; the step is one wave's dependency chain (second wave per SIMD ~free, VALU issue ~1/3)
        out["roofline"]["binding"] = {
            "resource": "latency",
            "valu_issue_frac": vi["frac"] if vi else None,
            "latency_ratio": lat["ratio"] if lat else None,
            "note": "the contract's bound field is the HBM roofline; the kernel is bound by the slowest "
                    "wave's dependency chain (exposed LDS / memory latency), not by HBM or VALU issue"}
        if world == 1 and not args.no_extras:
            if not (args.dr or args.obstacles or args.auto_reset or args.policy or args.gather):
                out["host_api"] = host_api_rates(model_path, E, device, keys)
            out["contact_cap"] = contact_cap_stats(env, acts.ptr.value, min(K, 50))
            out["one_step_err"], out["ls_cap"] = one_step_err(env, dr_table=dr_table, terrain=terrain,
                                                              auto_reset=args.auto_reset > 0)
            out["qpos_rel_err"] = {"value": qpos_drift(env, dr_row=None if dr_table is None else dr_table[0],
                                                       terrain_row=None if terrain is None else terrain[0]),
                                   "substeps": 1000,
                                   "vs": "fp64 oracle restatement (MuJoCo absent; parity unpinned vs mj_step)",
                                   "trajectory": "standing PD hold"}
            if not args.no_cpu_baseline:
                states = _oracle_record(rec)
                out["cpu_baseline"] = cpu_baseline(env.sys_model.struct, env.config_struct, states,
                                                   init_obs.astype(np.float64))
        print(json.dumps(out), flush=True)
    if gather_dst is not None:
        gather_dst.free()
    env.close()
    if comm is not None:
        comm.close()
    if gcheck and gcheck.get("failing_receivers"):
        sys.exit(3)


if __name__ == "__main__":
    main()
