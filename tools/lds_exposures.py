"""Static count of exposed LDS round trips per PHASE segment (prof-build asm): an `s_waitcnt lgkmcnt`
that follows its LDS read within K instructions (nothing issued meanwhile to cover ~50+ cycles).

  python tools/lds_exposures.py [asm] [K]
"""
import re
import sys
from collections import Counter

NAMES = {0: "kinematics", 1: "com", 2: "limit rows", 3: "M+bias+J", 4: "LDL(M)", 5: "warmstart", 6: "newton grad",
         7: "LDL(H)", 8: "linesearch", 9: "integrate", 10: "prologue", 11: "write_obs", 12: "rewards",
         13: "edge rows", 14: "hess build", 15: "crb+rne", 16: "collision", 17: "obs rng", 18: "imu"}
path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/pp3_prof.s"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
s = open(path).read()
a = re.search(r"^_ZN3pp315env_step_kernelILi8ELb1E(?:Li1E)?(?:Lb0E)?EEv\S*:", s, re.M).start()
body = [L.strip() for L in s[a:s.index(".Lfunc_end", a)].split("\n")]
seg, exp = [], Counter()
tot = 0
for L in body:
    m = re.search(r"PP3PHASE (\d+)", L)
    if m:
        n = 0
        last_read = -100
        idx = 0
        for t in seg:
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            if t.startswith("ds_read") or t.startswith("ds_bpermute"):
                last_read = idx
            if t.startswith("s_waitcnt") and "lgkmcnt" in t and idx - last_read <= K:
                n += 1
            idx += 1
        print(f"{NAMES[int(m.group(1))]:12s} exposed={n}")
        tot += n
        seg = []
        continue
    seg.append(L)
print("total", tot)
