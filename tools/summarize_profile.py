"""Summarise a tools/gpu_profile.sh output directory (kernel stats + PMC passes) for env_step_kernel.

  python tools/summarize_profile.py gpurun_out/<tag> [--commit profiles/r01_vN] [--launch step]

The bench's default launch is a fused rollout (pp3_rollout, `env_step_kernel<8, true>`, one
dispatch of --steps env steps); its single-step replay and the warmup are `env_step_kernel<8,
false>` dispatches, kept apart here.  --launch step summarises the single-step kernel instead
(a `bench.py --launch step` profile).  Per-launch figures are also given per env step.

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KB; per MI355X_MICROARCH.md (HBM /
rocprofv3 section) FETCH_SIZE on gfx950 reports half the bytes of wide coalesced reads, so it is
doubled here; WRITE_SIZE is taken as-is.  SQ_* instruction counts are per dispatch, summed over
waves (one wave = one env).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

KERNEL = "env_step_kernel<8, true, 1, false>"  # (the fused policy rollout is <8, true, 8, false>)


def _arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


def _kernel():
    launch = _arg("--launch", "rollout")
    return {"step": "env_step_kernel<8, false, 1, false>", "policy": "env_step_kernel<8, true, 8, false>"}.get(launch, KERNEL)


def _pmc(d):
    """Counters of the summarised kernel: for the fused rollout the LAST dispatch of
    env_step_kernel<8, true> (the timed window; the bench's untimed GPU pre-warm launches the same
    kernel for 20-step rollouts before it), for single-step launches the mean over dispatches."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(float))
    for f in files:
        for r in csv.DictReader(open(f)):
            if _kernel() in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        return {}
    if _arg("--launch", "rollout") in ("rollout", "policy"):
        return dict(per[max(per)])
    agg = defaultdict(list)
    for c in per.values():
        for k, v in c.items():
            agg[k].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def _trace_last(d):
    """Duration (ns) of the last dispatch of the summarised kernel in the kernel trace."""
    files = glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True)
    last = None
    for f in files:
        for r in csv.DictReader(open(f)):
            if _kernel() in r["Kernel_Name"]:
                did = int(r["Dispatch_Id"])
                if last is None or did > last[0]:
                    last = (did, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return None if last is None else float(last[1])


def main():
    d = sys.argv[1]
    launch = _arg("--launch", "rollout")
    spl = int(_arg("--steps-per-launch", 50 if launch in ("rollout", "policy") else 1))  # gpu_profile.sh: --steps 50
    out = {"kernel": _kernel(), "launch": launch, "steps_per_launch": spl}
    stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        for r in csv.DictReader(open(stats[0])):
            if _kernel() in r["Name"]:
                out["kernel_avg_ns"] = float(r["AverageNs"])
                out["kernel_calls"] = int(r["Calls"])
    if launch in ("rollout", "policy"):
        t = _trace_last(d)
        if t is not None:  # the timed window's launch (the stats' average includes the pre-warm's)
            out["kernel_avg_ns"] = t
            out["timed_launch_ns"] = t
    sq = _pmc(os.path.join(d, "pmc_sq"))
    if sq:
        waves = sq.get("SQ_WAVES", 1.0)
        out["per_wave"] = {k: v / waves for k, v in sq.items() if k != "SQ_WAVES"}
        out["waves"] = waves
    f = _pmc(os.path.join(d, "pmc_fetch")).get("FETCH_SIZE")
    w = _pmc(os.path.join(d, "pmc_write")).get("WRITE_SIZE")
    if f is not None and w is not None:
        out["fetch_bytes_per_launch"] = 2 * f * 1024   # gfx950 FETCH_SIZE x2 correction
        out["write_bytes_per_launch"] = w * 1024
        out["hbm_bytes_per_launch"] = out["fetch_bytes_per_launch"] + out["write_bytes_per_launch"]
        out["hbm_bytes_per_env_step"] = out["hbm_bytes_per_launch"] / spl / 4096
    if "per_wave" in out:
        out["per_wave_per_step"] = {k: v / spl for k, v in out["per_wave"].items()}
    print(json.dumps(out, indent=1))
    if "--commit" in sys.argv:
        dst = sys.argv[sys.argv.index("--commit") + 1]
        if stats:
            shutil.copy(stats[0], dst + "_kernel_stats.csv")
        traces = glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True)
        if traces:  # every env_step_kernel dispatch: the pre-warm's, the timed window's, the replay's
            with open(dst + "_env_step_dispatches.csv", "w") as fo:
                fo.write("dispatch_id,kernel,duration_ns\n")
                for r in csv.DictReader(open(traces[0])):
                    if "env_step_kernel" in r["Kernel_Name"]:
                        fo.write(f'{r["Dispatch_Id"]},"{r["Kernel_Name"]}",{int(r["End_Timestamp"]) - int(r["Start_Timestamp"])}\n')
        json.dump(out, open(dst + "_pmc_summary.json", "w"), indent=1)
        # the bench's roofline.traffic / valu_issue source, keyed to the kernel sources it was measured on
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import bench
        if "hbm_bytes_per_launch" in out and "per_wave" in out:
            json.dump({"source": dst + "_pmc_summary.json (tools/gpu_profile.sh on MI355X, bench.py --steps 50 --warmup 5 "
                                     "--no-latency-floor --no-extras)",
                       "src_sha16": bench.kernel_source_sha16(), "envs": 4096, "dr": False,
                       "kernel": out["kernel"], "launch": launch, "steps_per_launch": spl,
                       "hbm_bytes_per_launch": out["hbm_bytes_per_launch"],
                       "fetch_bytes_per_launch": out["fetch_bytes_per_launch"],
                       "write_bytes_per_launch": out["write_bytes_per_launch"],
                       "valu_insts_per_wave": out["per_wave"]["SQ_INSTS_VALU"], "envs_per_wave": 2,
                       "waves": out.get("waves"), "kernel_avg_ns": out.get("kernel_avg_ns")},
                      open(os.path.join(root, "profiles", "traffic_current.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
