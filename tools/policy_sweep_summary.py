"""Per-config average duration of mlp_kernel from a policy_sweep.py kernel trace."""
import csv
import glob
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from policy_sweep import CONFIGS, REPS  # noqa: E402

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "mlp_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for i, c in enumerate(CONFIGS):
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[i * REPS:(i + 1) * REPS]][5:]
    flops = 2 * 4096 * sum(c[j] * c[j + 1] for j in range(len(c) - 1))
    us = sum(d) / len(d) / 1e3
    print(f"{str(c):28s} {us:8.2f} us  {flops / us / 1e6:7.2f} TFLOP/s")
