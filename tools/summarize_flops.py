"""Summarise tools/gpu_flops.sh (FP32 instruction-mix PMC pass) for env_step_kernel.

  python tools/summarize_flops.py gpurun_out/<tag> [--commit profiles/r02_vN]

Executed FP32 operations per launch = 64 x (2 FMA + ADD + MUL + TRANS) wave-instructions (the
rocprofv3 FLOPS expression restricted to FP32 VALU; every lane of a wave64 instruction is counted,
so lanes masked off by EXEC and work replicated across lanes count too: an upper bound on the
arithmetic the step needs).  --commit writes <dst>_flops_pmc.json and adds the per-launch figure
to profiles/traffic_current.json (bench.py's roofline.fp32_vector), keyed like the rest of that
file to the kernel sources' hash.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profile import _arg, _kernel, _pmc  # noqa: E402

ENVS = 4096


def main():
    d = sys.argv[1]
    c = _pmc(os.path.join(d, "pmc_flops"))
    if not c:
        raise SystemExit(f"no {_kernel()} counters under {d}/pmc_flops")
    spl = int(_arg("--steps-per-launch", 50 if _arg("--launch", "rollout") == "rollout" else 1))
    fma, add, mul, trans = (c.get("SQ_INSTS_VALU_%s_F32" % k, 0.0) for k in ("FMA", "ADD", "MUL", "TRANS"))
    flops = 64.0 * (2 * fma + add + mul + trans)
    out = {"kernel": _kernel(), "steps_per_launch": spl, "counters_per_launch": c, "fp32_flops_per_launch": flops,
           "envs": ENVS, "fp32_flops_per_env_step": flops / ENVS / spl,
           "fp32_share_of_valu": (fma + add + mul + trans) / max(c.get("SQ_INSTS_VALU", 1.0), 1.0)}
    print(json.dumps(out, indent=1))
    if "--commit" in sys.argv:
        dst = sys.argv[sys.argv.index("--commit") + 1]
        json.dump(out, open(dst + "_flops_pmc.json", "w"), indent=1)
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import bench
        tf = os.path.join(root, "profiles", "traffic_current.json")
        tj = json.load(open(tf))
        if tj.get("src_sha16") != bench.kernel_source_sha16() or tj.get("steps_per_launch", 1) != spl:
            raise SystemExit("traffic_current.json is for another kernel build: re-run tools/gpu_profile.sh first")
        tj["fp32_flops_per_launch"] = flops
        tj["fp32_flops_source"] = dst + "_flops_pmc.json (tools/gpu_flops.sh on MI355X)"
        json.dump(tj, open(tf, "w"), indent=1)


if __name__ == "__main__":
    main()
