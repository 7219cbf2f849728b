"""One-line summary of a bench.py JSON output file (the last line of the file)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
r = d["roofline"]
ps = d.get("per_step_launch") or {}
out = {"value": d["value"], "ms_per_step": d["ms_per_step"], "avg_launch_ms": r.get("avg_launch_ms"),
       "per_step": ps.get("avg_launch_ms") or ps.get("ms_per_step"), "per_step_rate": ps.get("kernel_env_steps_per_s") or ps.get("env_steps_per_s"),
       "bit_equal": ps.get("bit_equal_to_rollout"), "actions_bit_equal": ps.get("actions_bit_equal"),
       "sha": d.get("state_sha16"), "frac": r.get("frac"), "kernel": r.get("kernel")}
if d.get("idle_start"):
    out["idle"] = {k: d["idle_start"][k] for k in ("env_steps_per_s", "idle_over_prewarmed", "bit_equal_to_rollout")}
if d.get("ls_cap"):
    lc = d["ls_cap"]
    out["ls_cap"] = {"frac_capped": lc["frac_capped"], "frac_capped_f32": lc["frac_capped_f32"],
                     "qpos_abs": lc["vs_converged_search"]["qpos_abs"]}
if d.get("host_api"):
    out["host_api"] = {k: v for k, v in d["host_api"].items() if isinstance(v, float)}
if d.get("one_step_err"):
    out["one_step_qpos_max"] = d["one_step_err"]["qpos_abs"]["max"]
print(json.dumps(out))
