"""Serial LDS load chains per PHASE segment of the prof-build asm: a ds_read, a wait on lgkmcnt
within 4 instructions, the next ds_read within 4 instructions of the wait, and so on.  A chain of
length >= N usually means the compiler reused one register (pair) for a gather under register
pressure and waited after each load; loading the operands into an array and pinning them
(PIN(...)) turns it into one round (round 4: +1.4 % for the M entries, +3.0 % for CRB x cdof,
the base RNE terms, the bias subtree rows and the limit / actuation reads).

  make -C pupperv3-mjx_amd/csrc asm-prof && python tools/lds_chains.py [/tmp/pp3_prof.s] [N]
"""
import re
import sys

NAMES = {0: "kinematics", 1: "com", 2: "limit rows", 3: "M+bias+J", 4: "LDL(M)", 5: "warmstart", 6: "newton grad",
         7: "LDL(H)", 8: "linesearch", 9: "integrate", 10: "prologue", 11: "write_obs", 12: "rewards",
         13: "edge rows", 14: "hess build", 15: "crb+rne", 16: "collision", 17: "obs rng", 18: "imu"}


def main(path, nmin):
    s = open(path).read()
    a = re.search(r"^_ZN3pp315env_step_kernelILi8ELb1E(?:Li1E)?(?:Lb0E)?EEv\S*:", s, re.M).start()
    body = [L.strip() for L in s[a:s.index(".Lfunc_end", a)].split("\n")]
    seg = []
    for L in body:
        m = re.search(r"PP3PHASE (\d+)", L)
        if not m:
            if L and not L.startswith((".", ";")) and not L.endswith(":"):
                seg.append(L)
            continue
        chains, i = [], 0
        while i < len(seg):
            if seg[i].startswith("ds_read"):
                j, n, start = i, 1, i
                while True:
                    w = next((k for k in range(j + 1, min(j + 5, len(seg)))
                              if seg[k].startswith("s_waitcnt") and "lgkmcnt" in seg[k]), None)
                    if w is None:
                        break
                    r = next((k for k in range(w + 1, min(w + 5, len(seg))) if seg[k].startswith("ds_read")), None)
                    if r is None:
                        break
                    n, j = n + 1, r
                if n >= nmin:
                    chains.append((start, n))
                i = j + 1
            else:
                i += 1
        print(f"{NAMES.get(int(m.group(1)), m.group(1)):12s} chains (start, length): {chains}")
        seg = []


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/pp3_prof.s", int(sys.argv[2]) if len(sys.argv) > 2 else 3)
