"""Static instruction mix of env_step_kernel<8> per PHASE segment (prof build asm).

  python tools/phase_static.py [asm]   (default: builds /tmp/pp3_prof.s)
Segments end at the `; PP3PHASE k` marker of the phase they close.
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
    a = s.index("_ZN3pp315env_step_kernelILi8ELb1ELi1EEEvNSt11conditionalIXgtT1_Li1EENS_14PolicyStepArgsENS_8StepArgsEE4typeE:")
    body = s[a:s.index(".Lfunc_end", a)].split("\n")
    seg = Counter()
    out = []
    for line in body:
        t = line.strip()
        m = re.search(r"PP3PHASE (\d+)", t)
        if m:
            out.append((int(m.group(1)), seg))
            seg = Counter()
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        seg["valu"] += op.startswith("v_")
        seg["readlane"] += op.startswith(("v_readlane", "v_writelane", "v_readfirstlane"))
        seg["mov/cnd"] += op.startswith(("v_mov", "v_cndmask"))
        seg["ds"] += op.startswith("ds_")
        seg["nop"] += op.startswith("s_nop")
        seg["salu"] += op.startswith("s_") and not op.startswith(("s_nop", "s_waitcnt", "s_cbranch"))
    out.append(("tail", seg))
    for k, c in out:
        print(f"{str(k):>5} " + " ".join(f"{n}={c[n]}" for n in ("valu", "readlane", "mov/cnd", "ds", "nop", "salu")))


if __name__ == "__main__":
    main()
