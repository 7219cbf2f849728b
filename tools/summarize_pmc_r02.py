"""Per-wave means of every counter in a tools/gpu_pmc_r02.sh output dir, env_step_kernel only."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
out = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    agg = defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "env_step_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out[k] = sum(v) / len(v)
waves = out.get("SQ_WAVES", 2048.0)
per_wave = {k: (v / waves if k.startswith("SQ_") and k != "SQ_WAVES" else v) for k, v in sorted(out.items())}
print(json.dumps(per_wave, indent=1))
