"""Time the MLP policy kernel on a sweep of layer shapes (run under rocprofv3 --kernel-trace;
kernel launches are in config order, 40 per config)."""
import ctypes as C
import sys
import os

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pupperv3-mjx_amd"))
from pupperv3_mjx import _lib  # noqa: E402

CONFIGS = [[72, 32], [72, 256], [72, 256, 128], [72, 256, 128, 128], [72, 256, 128, 128, 24], [256, 256], [256, 256, 256]]
N, REPS = 4096, 40


def main():
    L = _lib.load()
    rs = np.random.RandomState(0)
    obs = _lib.DeviceBuffer(N * 512 * 4, 0)
    obs.upload(rs.normal(size=N * 512).astype(np.float32))
    out = _lib.DeviceBuffer(N * 512 * 4, 0)
    for sizes in CONFIGS:
        outs = np.array(sizes[1:], dtype=np.int32)
        acts = np.full(len(outs), 2, dtype=np.int32)  # elu
        w = np.concatenate([np.concatenate([rs.normal(scale=0.1, size=sizes[i] * sizes[i + 1]), np.zeros(sizes[i + 1])])
                            for i in range(len(outs))]).astype(np.float32)
        h = C.c_void_p()
        _lib.check(L.pp3_policy_create(0, sizes[0], len(outs), outs.ctypes.data_as(C.c_void_p),
                                       acts.ctypes.data_as(C.c_void_p), w.ctypes.data_as(C.c_void_p), C.byref(h)))
        for _ in range(REPS):
            L.pp3_policy_act(h, obs.ptr, sizes[0], N, out.ptr, sizes[-1], None)
        L.pp3_memcpy_d2h(C.c_void_p(w.ctypes.data), out.ptr, 4)
        L.pp3_policy_destroy(h)
        print(sizes, flush=True)


if __name__ == "__main__":
    main()
