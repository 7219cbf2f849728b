"""Per-kernel register / scratch / LDS counts of the step library, keyed by the kernel source hash
(bench.kernel_source_sha16) -- verdict r05 item 1.  Compiles pp3_env.hip for gfx950 with the
product flags (plus any extra -D flags given): the compiler's kernel-resource-usage remarks give
VGPRs, SGPRs, SGPR / VGPR spills, scratch bytes per lane, LDS bytes per workgroup and occupancy;
the assembly gives the static count of scratch loads / stores in each function body.

  python tools/resource_usage.py [-DFLAG ...] >> profiles/r06_resource_usage.txt
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

CSRC = os.path.join(ROOT, "pupperv3-mjx_amd", "csrc")
BASE = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
        "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-fgpu-flush-denormals-to-zero", "-fno-slp-vectorize"]
KEYS = {"VGPRs": "vgpr", "TotalSGPRs": "sgpr", "ScratchSize [bytes/lane]": "scratch", "Occupancy [waves/SIMD]": "occ",
        "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill", "LDS Size [bytes/block]": "lds"}


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.split("\n")
    return dict(zip(names, out))


def main(extra):
    src = os.path.join(CSRC, "pp3_env.hip")
    with tempfile.TemporaryDirectory() as td:
        rem = subprocess.run(BASE + list(extra) + ["--cuda-device-only", "-c", "-Rpass-analysis=kernel-resource-usage",
                                                   "-o", os.path.join(td, "k.o"), src],
                             check=True, capture_output=True, text=True).stderr
        asm = os.path.join(td, "k.s")
        subprocess.run(BASE + list(extra) + ["--cuda-device-only", "-S", "-o", asm, src], check=True, capture_output=True)
        text = open(asm).read().split("\n")
    funcs, cur = {}, None
    for line in rem.split("\n"):
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = funcs.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z \[\]/]+?): (\d+) \[", line)
        if m and cur is not None and m.group(1).strip() in KEYS:
            cur[KEYS[m.group(1).strip()]] = int(m.group(2))
    body = None
    for line in text:
        m = re.match(r"^(\S+):\s+; @", line)
        if m:
            body = funcs.get(m.group(1))
            if body is not None:
                body.setdefault("scr_ld", 0)
                body.setdefault("scr_st", 0)
            continue
        if body is None:
            continue
        s = line.strip()
        if s.startswith("scratch_load"):
            body["scr_ld"] += 1
        elif s.startswith("scratch_store"):
            body["scr_st"] += 1
    names = demangle(list(funcs))
    print(f"# src_sha16 {bench.kernel_source_sha16()}  flags {' '.join(extra) or '(product)'}")
    print(f"# {'function':62s} {'VGPR':>4s} {'SGPR':>4s} {'spill s/v':>9s} {'scratch':>7s} {'LDS B':>6s} {'occ':>3s} {'scr ld/st':>9s}")
    for n, f in funcs.items():
        if "vgpr" not in f:
            continue
        print(f"  {names.get(n, n)[:62]:62s} {f['vgpr']:4d} {f.get('sgpr', 0):4d} {f.get('sgpr_spill', 0):4d}/{f.get('vgpr_spill', 0):<4d}"
              f" {f.get('scratch', 0):7d} {f.get('lds', 0):6d} {f.get('occ', 0):3d} {f.get('scr_ld', 0):4d}/{f.get('scr_st', 0):<4d}")


if __name__ == "__main__":
    main(sys.argv[1:])
