"""Host side of the host-API step (verdict r05 item 3 / weak 6): how long the per-step copy of the
4096 x 12 actions (196 KB) into the page-locked staging block takes, by allocation kind --
pageable numpy, hipHostMalloc default (what PinnedBlock uses) and write-combined -- and reading a
step's obs rows (1.2 MB) back from a page-locked block.  Timing only; run on the GPU box.

  python tools/pinned_copy_microbench.py
"""
import ctypes as C
import time

import numpy as np

hip = C.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipHostFree.argtypes = [C.c_void_p]
FLAGS = {"default": 0x0, "coherent": 0x40000000, "noncoherent": 0x80000000, "writecombined": 0x4}


def block(nbytes, flags):
    p = C.c_void_p()
    rc = hip.hipHostMalloc(C.byref(p), nbytes, flags)
    if rc != 0:
        raise RuntimeError(f"hipHostMalloc flags {flags:#x}: {rc}")
    return p, np.ctypeslib.as_array((C.c_float * (nbytes // 4)).from_address(p.value))


def t_us(fn, n=2000):
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(n):
            fn()
        best = min(best, (time.perf_counter() - t) / n * 1e6)
    return best


def main():
    E = 4096
    a = np.random.RandomState(0).uniform(-1, 1, size=(E, 12)).astype(np.float32)
    obs_n = E * 74
    print(f"actions {a.nbytes} B, obs rows {obs_n * 4} B")
    dst = np.empty(E * 12, np.float32)
    print(f"  pageable numpy      copy-in {t_us(lambda: np.copyto(dst, a.reshape(-1))):7.2f} us")
    for name, fl in FLAGS.items():
        try:
            p, arr = block(16 * E * 12 * 4 + obs_n * 4, fl)
        except RuntimeError as e:
            print(f"  {name:18s} {e}")
            continue
        view = arr[:E * 12]
        cin = t_us(lambda: np.copyto(view, a.reshape(-1)))
        rows = arr[16 * E * 12:16 * E * 12 + obs_n]
        out = np.empty_like(rows)
        cout = t_us(lambda: np.copyto(out, rows), n=300)
        s = t_us(lambda: float(rows[::37].sum()), n=300)
        print(f"  {name:18s} copy-in {cin:7.2f} us   obs read-out {cout:8.2f} us   strided sum {s:7.2f} us")
        hip.hipHostFree(p)


if __name__ == "__main__":
    main()
