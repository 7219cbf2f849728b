"""Mean duration of each stamped interval in a diag_phases.py waves.npy, by phase id and by its
occurrence in the wave's trace (the trace holds a wave's first 128 stamps: the launch's first
step and part of the second).

  python tools/trace_intervals.py waves.npy [ids, comma-separated]
"""
import sys
from collections import defaultdict

import numpy as np


def main(path, ids):
    w = np.load(path).astype(np.int64)
    tr, kk = w[:, 32:160], w[:, 160:288]
    acc = defaultdict(list)
    for r in range(len(w)):
        seen = defaultdict(int)
        for i in range(1, 128):
            k = kk[r, i]
            if k == 0xffffffff or kk[r, i - 1] == 0xffffffff:
                break
            d = (tr[r, i] - tr[r, i - 1]) & 0xffffffff
            acc[(int(k), seen[k])].append(d)
            seen[k] += 1
    for (k, o), v in sorted(acc.items()):
        if ids and k not in ids:
            continue
        v = np.array(v, dtype=np.float64)
        print(f"id {k:3d} occurrence {o:2d}: waves {len(v):5d} mean {v.mean():9.0f} p50 {np.median(v):9.0f} max {v.max():9.0f}")


if __name__ == "__main__":
    main(sys.argv[1], [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [])
