"""jax.random restatement (rng.py host, pp3_oracle.c oracle, and the kernel's copy) pinned by KATs.

Known answers: Random123 threefry2x32-20 vectors (the same ones jax's random_test.py
checks), and jax's documented outputs for PRNGKey(0) with the pre-0.5 counter layout.
"""
import numpy as np
import pytest

from pupperv3_mjx import rng


@pytest.mark.parametrize("key,ctr,expected", [
    ((0, 0), (0, 0), (0x6B200159, 0x99BA4EFE)),
    ((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF), (0x1CB996FC, 0xBB002BE7)),
    ((0x13198A2E, 0x03707344), (0x243F6A88, 0x85A308D3), (0xC4923A9C, 0x483DF7A0)),
])
def test_threefry_random123_kat(key, ctr, expected):
    y = rng.threefry2x32(key[0], key[1], ctr[0], ctr[1])
    assert (int(y[0]), int(y[1])) == expected


def test_oracle_threefry_kat():
    import ctypes as C
    from oracle import oracle as O
    out = (C.c_uint32 * 2)()
    O.lib("f64").orc_threefry2x32(0x13198A2E, 0x03707344, 0x243F6A88, 0x85A308D3, out)
    assert (out[0], out[1]) == (0xC4923A9C, 0x483DF7A0)


def test_prngkey_and_original_split_known_values():
    assert rng.PRNGKey(0).tolist() == [0, 0]
    assert rng.PRNGKey(42).tolist() == [0, 42]
    # jax.random.split(jax.random.PRNGKey(0)) with jax_threefry_partitionable=False
    assert rng.split(rng.PRNGKey(0), 2, partitionable=False).tolist() == [[4146024105, 967050713],
                                                                          [2718843009, 1272950319]]
    # jax.random.uniform(jax.random.PRNGKey(0)) with the original layout
    assert np.float32(rng.uniform(rng.PRNGKey(0), (), partitionable=False)) == np.float32(0.41845703)


def test_partitionable_split_is_foldlike():
    k = rng.PRNGKey(7)
    s6 = rng.split(k, 6)
    s3 = rng.split(k, 3)
    assert np.array_equal(s6[:3], s3)  # split(k, n)[i] independent of n (threefry(k, (0, i)))
    y = rng.threefry2x32(k[0], k[1], 0, 4)
    assert s6[4].tolist() == [int(y[0]), int(y[1])]


@pytest.mark.parametrize("part", [True, False])
def test_host_and_oracle_rng_agree(part):
    import ctypes as C
    from oracle import oracle as O
    L = O.lib("f32")
    L.orc_set_partitionable(int(part))
    try:
        for seed in range(5):
            key = rng.split(rng.PRNGKey(seed), 3, part)[1]
            kk = np.ascontiguousarray(key, dtype=np.uint32)
            for n in (1, 2, 3, 5, 6, 12):
                out = np.zeros(2 * n, dtype=np.uint32)
                L.orc_split(kk.ctypes.data_as(C.POINTER(C.c_uint32)), n, out.ctypes.data_as(C.POINTER(C.c_uint32)))
                assert np.array_equal(out.reshape(n, 2), rng.split(key, n, part))
                u = np.zeros(n, dtype=np.float32)
                L.orc_uniform(kk.ctypes.data_as(C.POINTER(C.c_uint32)), n, -0.3, 0.7,
                              u.ctypes.data_as(C.POINTER(C.c_float)))
                assert np.array_equal(u, rng.uniform(key, (n,), -0.3, 0.7, part))
            for p in ([0.2, 0.8], [0.5, 0.5], [0, 0, 1], [0.1, 0.2, 0.3, 0.4]):
                pa = np.asarray(p, dtype=np.float64)
                i = L.orc_choice(kk.ctypes.data_as(C.POINTER(C.c_uint32)), pa.ctypes.data_as(C.POINTER(C.c_double)), len(p))
                assert i == int(rng.choice_index(key, p, part))
    finally:
        L.orc_set_partitionable(1)


def test_uniform_range_and_bernoulli_rate():
    keys = rng.split(rng.PRNGKey(1), 20000)
    u = rng.uniform(keys, (1,), -2.0, 3.0)[:, 0]
    assert u.min() >= -2.0 and u.max() < 3.0
    assert abs(u.mean() - 0.5) < 0.05
    b = rng.bernoulli(keys, 0.04, (1,))
    assert abs(b.mean() - 0.04) < 0.006


def test_choice_distribution():
    keys = rng.split(rng.PRNGKey(3), 4000)
    idx = np.array([rng.choice_index(k, [0.2, 0.8]) for k in keys])
    assert abs((idx == 1).mean() - 0.8) < 0.03
    assert all(rng.choice_index(k, [0, 0, 1]) == 2 for k in keys[:50])
