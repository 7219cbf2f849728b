"""Static instruction / LDS-wait counts per PHASE segment of env_step_kernel<8> (prof build asm).

  python tools/phase_waits_static.py [asm]   (default: builds /tmp/pp3_prof.s via make asm-prof)
A segment ends at the `; PP3PHASE k` marker of the phase it closes.
"""
import os
import re
import subprocess
import sys
from collections import Counter

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pupperv3-mjx_amd", "csrc")
NAMES = {0: "kinematics", 1: "com", 2: "limit rows", 3: "M+bias+J", 4: "LDL(M)", 5: "warmstart", 6: "newton grad",
         7: "LDL(H)", 8: "linesearch", 9: "integrate", 10: "prologue", 11: "write_obs", 12: "rewards",
         13: "edge rows", 14: "hess build", 15: "crb+rne", 16: "collision", 17: "obs rng", 18: "imu"}


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/pp3_prof.s"
    if len(sys.argv) == 1:
        subprocess.run(["make", "-s", "-C", CSRC, "asm-prof"], check=True, stderr=subprocess.DEVNULL)
    s = open(path).read()
    a = s.index("_ZN3pp315env_step_kernelILi8ELb1EEEvNS_8StepArgsE:")
    body = s[a:s.index(".Lfunc_end", a)].split("\n")
    seg = Counter()
    tot = Counter()
    for L in body:
        t = L.strip()
        m = re.search(r"PP3PHASE (\d+)", t)
        if m:
            k = int(m.group(1))
            print(f"{NAMES[k]:12s} " + " ".join(f"{n}={seg[n]:5d}" for n in ("all", "valu", "ds", "lgkm", "vm", "nop", "salu", "br")))
            tot.update(seg)
            seg = Counter()
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        seg["all"] += 1
        seg["valu"] += op.startswith("v_")
        seg["ds"] += op.startswith("ds_")
        if op == "s_waitcnt":
            seg["lgkm"] += "lgkmcnt" in t
            seg["vm"] += "vmcnt" in t
        seg["nop"] += op == "s_nop"
        seg["br"] += op.startswith("s_cbranch") or op == "s_branch"
        seg["salu"] += op.startswith("s_") and op not in ("s_nop", "s_waitcnt")
    print("total        " + " ".join(f"{n}={tot[n]:5d}" for n in ("all", "valu", "ds", "lgkm", "vm", "nop", "salu", "br")))


if __name__ == "__main__":
    main()
