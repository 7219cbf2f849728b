"""Static instruction mix of one kernel in a hipcc -S output (spill traffic, loads, waits)."""
import re
import sys
from collections import Counter

path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/pp3_env.s"
pat = sys.argv[2] if len(sys.argv) > 2 else "env_step_kernelILi8"
s = open(path).read()
starts = [m for m in re.finditer(r"^(_Z\w+):", s, re.M)]
for i, m in enumerate(starts):
    if pat not in m.group(1):
        continue
    end = s.find(".Lfunc_end", m.start())
    body = s[m.start():end].splitlines()
    ops = Counter()
    for L in body:
        t = L.strip().split()
        if t and not t[0].startswith((";", ".")) and not t[0].endswith(":"):
            ops[t[0]] += 1
    tot = sum(ops.values())
    print(m.group(1), "instructions", tot)
    for k in ("v_writelane_b32", "v_readlane_b32", "v_readfirstlane_b32", "s_waitcnt", "s_nop", "ds_read_b32",
              "ds_write_b32", "ds_read2_b32", "ds_write2_b32", "ds_read_b128", "ds_read_b64", "s_load_dword",
              "s_load_dwordx2", "s_load_dwordx4", "s_load_dwordx8", "global_load_dword", "scratch_load_dword",
              "scratch_store_dword", "v_cndmask_b32_e32", "v_cndmask_b32_e64", "s_cbranch_execz", "s_and_saveexec_b64"):
        print(f"  {k:24s} {ops.get(k, 0)}")
    print("  top:", ops.most_common(25))
