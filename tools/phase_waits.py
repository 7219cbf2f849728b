"""Per-phase global-load / vmcnt-wait counts of env_step_kernel<8> (prof build asm).

  python tools/phase_waits.py [asm]   (default: builds /tmp/pp3_prof.s)
A phase whose vector-memory loads each get their own `s_waitcnt vmcnt` pays one L1/L2 round
trip per load; batched loads show many loads per wait.
"""
import os
import re
import subprocess
import sys
from collections import Counter

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pupperv3-mjx_amd", "csrc")


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/pp3_prof.s"
    if len(sys.argv) == 1:
        subprocess.run(["make", "-s", "-C", CSRC, "asm-prof"], check=True)
    s = open(path).read()
    a = s.index("_ZN3pp315env_step_kernelILi8EEEvNS_8StepArgsE:")
    body = s[a:s.index(".Lfunc_end", a)].split("\n")
    seg = Counter()
    tot = Counter()
    for line in body:
        t = line.strip()
        m = re.search(r"PP3PHASE (\d+)", t)
        if m:
            print(f"{m.group(1):>4} " + " ".join(f"{k}={seg[k]}" for k in ("vmem_ld", "wait_vm", "ds", "wait_lgkm")))
            tot.update(seg)
            seg = Counter()
            continue
        if not t or t.startswith((".", ";")):
            continue
        op = t.split()[0]
        if op.startswith(("global_load", "buffer_load")):
            seg["vmem_ld"] += 1
        elif op.startswith("ds_"):
            seg["ds"] += 1
        elif op == "s_waitcnt":
            seg["wait_vm"] += "vmcnt" in t
            seg["wait_lgkm"] += "lgkmcnt" in t
    print("total " + " ".join(f"{k}={tot[k]}" for k in ("vmem_ld", "wait_vm", "ds", "wait_lgkm")))


if __name__ == "__main__":
    main()
