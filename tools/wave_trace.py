"""Stamp-trace analysis of a diag_phases.py waves.npy (prof build, 288 words per wave).

  python tools/wave_trace.py gpurun_out/<tag>/waves.npy

Each wave carries up to 128 (s_memtime stamp, phase id) pairs in kernel order.  For every phase
interval the script compares the wave's duration with the median of that interval over all waves
(same position in the sequence); an "excess" is a duration above median + 5k cycles.  It prints
where the slowest waves lost their time, and whether excess intervals of different waves overlap
in absolute time on the same SQC (CU pair), the same XCD, or not at all.
"""
import sys

import numpy as np

NAMES = ["kin", "com", "lim", "Mbias", "LDLM", "warm", "grad", "LDLH", "LS", "integ", "prol", "wobs", "rew",
         "edge", "hess", "rne", "coll", "rng", "imu"]


def main(path):
    w = np.load(path).astype(np.int64)
    W = len(w)
    t0 = w[:, 4]
    life = w[:, 0]
    hw, xcc = w[:, 6], w[:, 7]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    sqc = ((xcc * 8 + se) * 2 + sh) * 8 + (cu >> 1)
    tr = w[:, 32:160]
    kk = w[:, 160:288]
    n = (kk != 0xFFFFFFFF).sum(1)
    print(f"waves {W}; stamps per wave: min {n.min()} max {n.max()}")
    # interval j: from stamp j-1 (or wave start) to stamp j, labelled by phase kk[:, j]
    prev = np.concatenate([t0[:, None], tr[:, :-1]], 1)
    dur = (tr - prev) & 0xFFFFFFFF
    valid = kk != 0xFFFFFFFF
    # waves with the modal sequence length (no dense substeps) share positions
    L = np.bincount(n).argmax()
    same = n == L
    med = np.zeros(128)
    for j in range(L):
        med[j] = np.median(dur[same, j])
    print(f"modal sequence length {L} ({same.sum()} waves); median lifetime {np.median(life):.0f}")
    exc = np.where(same[:, None] & valid & (np.arange(128)[None] < L), dur - med[None], 0)
    top = np.argsort(life)[::-1][:15]
    for i in top:
        if not same[i]:
            print(f"wave {i:5d} life {life[i]} (sequence length {n[i]}, dense path)")
            continue
        big = np.argsort(exc[i])[::-1][:4]
        s = ", ".join(f"#{j} {NAMES[kk[i, j]]} +{exc[i, j] // 1000}k@{(tr[i, j] - t0.min()) // 1000}k" for j in big)
        print(f"wave {i:5d} life {life[i]} xcc {xcc[i]} sqc {sqc[i]} simd {simd[i]} slot {hw[i] & 15}: "
              f"excess total {exc[i].clip(0).sum() // 1000}k; {s}")
    # excess events: (wave, start, end) for exc > 5k
    ev = [(i, int(prev[i, j]), int(tr[i, j]), int(exc[i, j]), j) for i in range(W) if same[i]
          for j in range(L) if exc[i, j] > 5000]
    print(f"excess events (> median + 5k): {len(ev)}, {sum(e[3] for e in ev) / 1e6:.1f} M cycles; "
          f"per interval position:")
    pos = np.bincount([e[4] for e in ev], minlength=L)
    amt = np.bincount([e[4] for e in ev], weights=[e[3] for e in ev], minlength=L)
    for j in np.argsort(amt)[::-1][:12]:
        ph = np.bincount(kk[same, j]).argmax()
        print(f"   #{j:3d} {NAMES[ph]:6s} median {med[j]:7.0f}  events {pos[j]:5d}  excess {amt[j] / 1e6:6.2f} M")
    # co-occurrence: for each event, fraction of overlapping events on the same SQC / other SQC same XCD
    ev = sorted(ev, key=lambda e: e[1])
    if ev:
        st = np.array([e[1] for e in ev])
        en = np.array([e[2] for e in ev])
        wv = np.array([e[0] for e in ev])
        same_sqc = other = 0
        for a in range(len(ev)):
            ov = (st < en[a]) & (en > st[a]) & (wv != wv[a])
            same_sqc += (ov & (sqc[wv] == sqc[wv[a]])).any()
            other += (ov & (xcc[wv] == xcc[wv[a]]) & (sqc[wv] != sqc[wv[a]])).any()
        print(f"events overlapping another wave's event on the same SQC: {same_sqc / len(ev):.2f}, "
              f"on another SQC of the same XCD: {other / len(ev):.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
