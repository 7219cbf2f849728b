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
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pupperv3-mjx_amd")]

METRIC = "env-steps/sec at N_envs=4096/GPU, 1/2/4/8 MI355X; qpos rel-err vs mj_step"
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TFLOPS = 157.3    # vector FP32 (spec)
N_SIMD, CLOCK_HZ, VALU_CYC = 1024, 2.4e9, 4   # 256 CUs x 4 SIMDs; peak engine clock; wave64 VALU issue


def algorithmic_bytes_per_env_step(stride: int, H: int, dr: bool) -> int:
    """HBM bytes one env step must move (DESIGN.md 'Roofline'): state record read+write,
    obs history read (36(H-1)) + write (36H), actions in, reward/done/metrics out, DR params."""
    words = 2 * stride + 36 * (H - 1) + 36 * H + 12 + 2 + 19 + (62 if dr else 0)
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


def cpu_baseline(model, cfg, states, obs, seconds_target=12.0):
    """Time the oracle (C fp64 restatement of the same step, OpenMP over envs) on host cores."""
    import numpy as np
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    n = min(states.shape[0], 64 * threads)
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
    return {"value": n * k / dt, "unit": "env-steps/s", "cores": int(used), "kind": "port",
            "sample": f"{n} envs x {k} steps of the fp64 C oracle (pp3_oracle.c restatement of mj_step + env, "
                      f"not MuJoCo), OpenMP {used} threads, {dt:.1f} s wall"}


def qpos_drift(env, nsub=1000):
    """Standing PD hold: GPU fp32 vs fp64 oracle relative qpos drift after nsub substeps."""
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
    o, _, _, _, _ = O.mj_step(env.sys_model.struct, q0, np.zeros(18), np.zeros(18), np.array(dp), nsteps=nsub)
    buf.free()
    return float(np.abs(g - o).max() / np.abs(o).max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=200,
                    help="untimed steps first: the drop from the start height settles (steady state)")
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--dr", action="store_true", help="domain randomisation on (configs[2])")
    ap.add_argument("--obstacles", type=int, default=0, help="obstacles.py boxes (configs[4])")
    ap.add_argument("--terrain", action="store_true",
                    help="per-env terrain (SURVEY 8f rank 3): every env gets its own random boxes in the --obstacles slots")
    ap.add_argument("--random-commands", action="store_true",
                    help="keep the reset's sampled velocity commands (configs[3]) instead of the fixed (0.5,0,0)")
    ap.add_argument("--gather", action="store_true", help="RCCL all_gather of obs|reward|done per step (configs[3])")
    ap.add_argument("--auto-reset", type=int, default=0, metavar="EPISODE_LENGTH",
                    help="on-device EpisodeWrapper+AutoResetWrapper (brax training wrap) with this episode length")
    ap.add_argument("--policy", type=str, default="", metavar="H1,H2,...",
                    help="policy-in-the-loop rollout: an exported-format MLP (random weights, elu) computes the "
                         "actions from the observation buffer on device before every env step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency-floor", action="store_true",
                    help="skip the E/2-envs latency-floor launches (keeps rocprof stats to E-env launches)")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for the multi-rank path on a single GPU (never used by the driver):
    # PP3_BENCH_DEVICE pins every rank to one device, PP3_BENCH_BACKEND=gloo avoids RCCL's
    # one-rank-per-GPU rule
    device = int(os.environ.get("PP3_BENCH_DEVICE", local_rank))
    backend = os.environ.get("PP3_BENCH_BACKEND", "nccl")
    # torch first: its bundled libamdhip64.so.7 then also serves libpupper_hip.so (one HIP runtime)
    import torch
    import torch.distributed as dist
    import numpy as np
    torch.cuda.set_device(device)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)

    from pupperv3_mjx import MODEL_XML, _abi, _lib, sharding
    from pupperv3_mjx.environment import PupperV3Env

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
    if args.dr:
        from pupperv3_mjx import domain_randomization as dr, rng
        sysb, _ = dr.domain_randomize(env.sys, rng.split(rng.PRNGKey(1000 + rank), E))
        env.set_domain_randomization(sysb)
    if args.terrain:
        from pupperv3_mjx import obstacles
        if not args.obstacles:
            raise SystemExit("--terrain needs --obstacles N (the box-geom slots)")
        env.set_terrain(obstacles.sample_terrain(E, args.obstacles, (-5, 5), (-5, 5), height=0.02, length=6.0,
                                                 seed=args.seed * 1000 + rank, min_boxes=args.obstacles // 2))
    if args.auto_reset > 0:
        _lib.check(L.pp3_set_auto_reset(env._h, args.auto_reset))
    keys = sharding.shard_keys(args.seed, E * world, world, rank)  # global env ids, contiguous shards
    st = env.reset(keys)
    rec = st._record.copy()
    if not args.random_commands:
        rec[:, _abi.S_COMMAND:_abi.S_COMMAND + 3] = [0.5, 0.0, 0.0]
    env._put(_abi.F_STATE, rec)
    init_obs = st.obs.copy()

    total = args.warmup + args.steps
    acts = _lib.DeviceBuffer(total * E * 12 * 4, device)
    _lib.check(L.pp3_fill_uniform(env._h, acts.ptr, total * E * 12, 1234 + rank, 0, -1.0, 1.0, None))
    env.synchronize()
    ms = C.c_float()
    if args.warmup:
        _lib.check(L.pp3_step_timed(env._h, acts.ptr, E * 12, args.warmup, C.byref(ms)))
    gather_buf = None
    if args.gather and world > 1:
        obs_n = env.device_field(_abi.F_OBS)[1]
        gather_buf = (torch.empty((E, obs_n), device="cuda"), torch.empty(E, device="cuda"),
                      torch.empty(E, device="cuda"))

    def barrier():
        if world > 1:
            dist.barrier()

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
        for _ in range(args.warmup):
            policy.act_env(env, acts.ptr.value)
            env.step_device(acts.ptr.value)

    barrier()
    torch.cuda.synchronize()
    env.synchronize()
    t0 = time.perf_counter()
    if policy is not None:
        for i in range(args.steps):
            policy.act_env(env, acts.ptr.value)
            env.step_device(acts.ptr.value)
        env.synchronize()
        kernel_ms = (time.perf_counter() - t0) * 1e3  # policy + env step per iteration (no per-kernel events)
    elif gather_buf is None:
        _lib.check(L.pp3_step_timed(env._h, C.c_void_p(acts.ptr.value + args.warmup * E * 12 * 4), E * 12,
                                    args.steps, C.byref(ms)))
        kernel_ms = ms.value
    else:
        kernel_ms = 0.0
        obs_t, rew_t, done_t = gather_buf
        for i in range(args.steps):
            _lib.check(L.pp3_step_timed(env._h, C.c_void_p(acts.ptr.value + (args.warmup + i) * E * 48), 0, 1,
                                        C.byref(ms)))
            kernel_ms += ms.value
            env.synchronize()  # step ran on the handle's stream; copies + gather go on torch's (null) stream
            for fid, t in ((_abi.F_OBS, obs_t), (_abi.F_REWARD, rew_t), (_abi.F_DONE, done_t)):
                ptr, _ = env.device_field(fid)
                _lib.check(L.pp3_memcpy_d2d(C.c_void_p(t.data_ptr()), C.c_void_p(ptr), t.numel() * 4, None))
            sharding.gather_batch(obs_t, rew_t, done_t, E * world)
    env.synchronize()
    torch.cuda.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall, kernel_ms], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max, kernel_ms_max = float(t[0]), float(t[1])

    # sanity on the produced batch
    rew = env._get(_abi.F_REWARD)
    obs = env._get(_abi.F_OBS)
    assert np.all(np.isfinite(rew)) and np.all(np.isfinite(obs)), "non-finite env outputs"
    # active-contact histogram of one further (untimed) step, from the Brax-pipeline record
    _lib.check(L.pp3_set_pipeline_output(env._h, 1))
    env.step_device(acts.ptr.value)
    env.synchronize()
    ncon = env._get(_abi.F_PIPELINE)[:, _abi.P_NCON].astype(int)
    contact_hist = np.bincount(ncon, minlength=9).tolist()

    if rank == 0:
        K = args.steps
        value = E * world * K / wall_max
        launch_s = kernel_ms_max / 1e3 / K
        bpe = algorithmic_bytes_per_env_step(env.stride, env._observation_history, args.dr)
        achieved = bpe * E / launch_s / 1e9
        traffic, valu, epw = None, None, 1
        tpath = os.path.join(ROOT, "profiles", "traffic_r01.json")
        if os.path.exists(tpath):
            tj = json.load(open(tpath))
            if tj.get("envs") == E and tj.get("dr", False) == args.dr and not args.obstacles:
                traffic = tj.get("hbm_bytes_per_launch")
                valu = tj.get("valu_insts_per_wave")
                epw = tj.get("envs_per_wave", 1)
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (actions U(-1,1) pre-generated in HBM; reset keys = jax.random.split(PRNGKey(seed), E))",
            "config": {"workload": ("configs[1]: test_pupper_model.xml, %d envs/GPU, %s, %s, %s"
                                    % (E, "flat terrain" if not args.obstacles else f"{args.obstacles} obstacle boxes",
                                       "random commands" if args.random_commands else "fixed command (0.5,0,0)",
                                       "domain randomisation" if args.dr else "no DR")),
                       "envs_per_gpu": E, "global_envs": E * world, "obs_history": env._observation_history,
                       "n_frames": env._n_frames, "parallelism": f"env-sharded x{world} (no data-path collective)",
                       "per_env_terrain": bool(args.terrain),
                       "commands": "reset-sampled, resampled every 500 steps" if args.random_commands else "fixed (0.5,0,0)",
                       "gather": bool(gather_buf is not None), "auto_reset_episode_length": args.auto_reset or None,
                       "policy_in_loop": args.policy or None},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "kernel": "pp3::env_step_kernel", "bytes_per_env_step": bpe,
                         "avg_launch_ms": round(launch_s * 1e3, 4)},
            "active_contacts": {"hist": contact_hist, "mean": round(float(np.mean(ncon)), 3),
                                "note": "contacts per env after the run (rank 0's shard)"},
        }
        if valu:
            # Compute-side bound (DESIGN.md 'Roofline'): VALU issue.  One wave = `epw` envs; a wave64
            # VALU instruction occupies its SIMD for 4 cycles; 1024 SIMDs at 2.4 GHz.
            ceil_s = valu * VALU_CYC * (E / epw) / (N_SIMD * CLOCK_HZ)
            out["roofline"]["valu_issue"] = {"valu_insts_per_wave": valu, "envs_per_wave": epw,
                                             "ceiling_ms": round(ceil_s * 1e3, 4),
                                             "frac": round(ceil_s / launch_s, 4),
                                             "source": "profiles/traffic_r01.json (rocprofv3 SQ_INSTS_VALU)"}
        if (world == 1 and policy is None and gather_buf is None and E == 4096 and not args.dr and not args.obstacles
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
            _lib.check(L.pp3_step_timed(half._h, acts.ptr, E // 2 * 12, hk, C.byref(ms)))
            half_s = ms.value / 1e3 / hk
            half.close()
            out["roofline"]["latency"] = {"envs": E // 2, "waves_per_simd": (E // 2) / 2 / N_SIMD,
                                          "avg_launch_ms": round(half_s * 1e3, 4),
                                          "ratio": round(launch_s / half_s, 4),
                                          "note": "launch time at E / at E/2 envs (one wave per SIMD)"}
        if world == 1:
            out["qpos_rel_err"] = {"value": qpos_drift(env), "substeps": 1000,
                                   "vs": "fp64 oracle restatement (MuJoCo absent; parity unpinned vs mj_step)",
                                   "trajectory": "standing PD hold"}
            if not args.no_cpu_baseline:
                with np.errstate(invalid="ignore"):  # RNG words are bit-cast uint32 in the f32 record
                    states = rec.astype(np.float64)
                states[:, _abi.S_RNG:_abi.S_RNG + 2] = rec[:, _abi.S_RNG:_abi.S_RNG + 2].copy().view(np.uint32)
                out["cpu_baseline"] = cpu_baseline(env.sys_model.struct, env.config_struct, states,
                                                   init_obs.astype(np.float64))
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
