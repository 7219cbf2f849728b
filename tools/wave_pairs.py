"""Per-SIMD wave-pair analysis of a diag_phases.py waves.npy (prof build): lifetime of the older and
the younger wave of each SIMD (same CU counter), by HW_ID wave slot.

  python tools/wave_pairs.py gpurun_out/<tag>/waves.npy
"""
import sys
from collections import defaultdict

import numpy as np

w = np.load(sys.argv[1]).astype(np.int64)
life, dense, ncm, ev, t0, t1, hw, xcc = [w[:, k] for k in range(8)]
slot, simd, cu, se = hw & 0xF, (hw >> 4) & 3, (hw >> 8) & 0xF, (hw >> 13) & 7
key = (xcc << 16) | (se << 8) | (cu << 2) | simd
g = defaultdict(list)
for i in range(len(w)):
    g[key[i]].append(i)
old, young, pmax = [], [], []
for v in g.values():
    if len(v) != 2:
        continue
    a, b = sorted(v, key=lambda i: t0[i])
    old.append(life[a]); young.append(life[b]); pmax.append(max(t1[a], t1[b]) - min(t0[a], t0[b]))
for name, x in (("older", old), ("younger", young), ("pair span", pmax)):
    x = np.array(x)
    print(f"{name:9s} mean {x.mean():8.0f} p50 {np.median(x):8.0f} p90 {np.percentile(x, 90):8.0f} max {x.max():8.0f}")
for s in (0, 1):
    print(f"slot {s}: mean life {life[slot == s].mean():.0f}")
