"""JAX-compatible threefry-2x32 PRNG on the host (numpy, vectorised over keys).

The reference draws every random number through ``jax.random`` ([ext] jax 0.5.0,
requirements.txt:2): ``split`` (environment.py:315,349,506; domain_randomization.py:27-80),
``uniform`` (environment.py:257-269,292-293,352,508-511), ``bernoulli`` (:353) and
``choice(p=...)`` (utils.py:67).  This module restates those primitives bit-for-bit:

* threefry2x32 with 20 rounds (Salmon et al. 2011; rotations (13,15,26,6)/(17,29,16,24),
  key-schedule parity constant 0x1BD11BDA), pinned by the Random123 known-answer vectors in
  tests/test_rng.py;
* ``PRNGKey(seed)`` = (0, seed & 0xffffffff) for 32-bit seeds;
* ``jax_threefry_partitionable=True`` (the jax 0.5.0 default): ``split(k, n)[i]`` =
  threefry(k, (0, i)) and the 32-bit ``random_bits`` element i = x0 ^ x1 of threefry(k, (0, i));
  ``partitionable=False`` selects the pre-0.5 counter layout instead;
* ``uniform``: bits >> 9 | 0x3f800000 reinterpreted as f32, minus 1, scaled, max(minval, .);
  ``bernoulli(p)`` = uniform < p; ``choice(p)`` = searchsorted_left(cumsum(p), cumsum[-1]*(1-u)).

All float arithmetic here is float32 to match JAX with x64 disabled.
"""
from __future__ import annotations

import numpy as np

_ROT = ((13, 15, 26, 6), (17, 29, 16, 24))
M32 = np.uint64(0xFFFFFFFF)


def _rotl(x: np.ndarray, r: int) -> np.ndarray:
    return ((x << np.uint32(r)) | (x >> np.uint32(32 - r))).astype(np.uint32)


def threefry2x32(k0, k1, x0, x1):
    """Threefry-2x32-20 on uint32 arrays (broadcast).  Returns (y0, y1)."""
    k0 = np.asarray(k0, dtype=np.uint32)
    k1 = np.asarray(k1, dtype=np.uint32)
    x0 = np.asarray(x0, dtype=np.uint32).copy()
    x1 = np.asarray(x1, dtype=np.uint32).copy()
    k0, k1, x0, x1 = np.broadcast_arrays(k0, k1, x0, x1)
    x0 = x0.astype(np.uint32).copy()
    x1 = x1.astype(np.uint32).copy()
    ks = (k0, k1, (k0 ^ k1 ^ np.uint32(0x1BD11BDA)).astype(np.uint32))
    with np.errstate(over="ignore"):
        x0 = (x0 + ks[0]).astype(np.uint32)
        x1 = (x1 + ks[1]).astype(np.uint32)
        for i in range(5):
            for r in _ROT[i % 2]:
                x0 = (x0 + x1).astype(np.uint32)
                x1 = _rotl(x1, r)
                x1 = (x1 ^ x0).astype(np.uint32)
            x0 = (x0 + ks[(i + 1) % 3]).astype(np.uint32)
            x1 = (x1 + ks[(i + 2) % 3] + np.uint32(i + 1)).astype(np.uint32)
    return x0, x1


def PRNGKey(seed: int) -> np.ndarray:
    s = int(seed)
    return np.array([(s >> 32) & 0xFFFFFFFF if s >= 0 else 0xFFFFFFFF, s & 0xFFFFFFFF], dtype=np.uint32)


def _keys(key):
    key = np.asarray(key, dtype=np.uint32)
    return key[..., 0], key[..., 1]


def split(key, num: int = 2, partitionable: bool = True) -> np.ndarray:
    """jax.random.split for one key [2] or a batch [..., 2] -> [..., num, 2]."""
    k0, k1 = _keys(key)
    k0 = k0[..., None]
    k1 = k1[..., None]
    if partitionable:
        i = np.arange(num, dtype=np.uint32)
        y0, y1 = threefry2x32(k0, k1, np.zeros_like(i), i)
        return np.stack([y0, y1], axis=-1)
    cnt = np.arange(2 * num, dtype=np.uint32)
    y0, y1 = threefry2x32(k0, k1, cnt[:num], cnt[num:])
    out = np.concatenate([y0, y1], axis=-1)  # [..., 2n]
    return out.reshape(out.shape[:-1] + (num, 2))


def random_bits32(key, count: int, partitionable: bool = True) -> np.ndarray:
    """32-bit random_bits for `count` elements -> [..., count] uint32."""
    k0, k1 = _keys(key)
    k0 = k0[..., None]
    k1 = k1[..., None]
    if partitionable:
        i = np.arange(count, dtype=np.uint32)
        y0, y1 = threefry2x32(k0, k1, np.zeros_like(i), i)
        return (y0 ^ y1).astype(np.uint32)
    n = count + (count % 2)
    cnt = np.arange(n, dtype=np.uint32)
    if count % 2:
        cnt[-1] = 0
        cnt[: count] = np.arange(count, dtype=np.uint32)
    y0, y1 = threefry2x32(k0, k1, cnt[: n // 2], cnt[n // 2:])
    out = np.concatenate([y0, y1], axis=-1)
    return out[..., :count]


def bits_to_unit_float(bits: np.ndarray) -> np.ndarray:
    fb = ((bits >> np.uint32(9)) | np.uint32(0x3F800000)).astype(np.uint32)
    return fb.view(np.float32) - np.float32(1.0)


def uniform(key, shape, minval=0.0, maxval=1.0, partitionable: bool = True) -> np.ndarray:
    shape = (shape,) if isinstance(shape, int) else tuple(shape)
    count = int(np.prod(shape)) if shape else 1
    u = bits_to_unit_float(random_bits32(key, count, partitionable))
    lead = np.asarray(key).shape[:-1]
    u = u.reshape(lead + shape)
    lo = np.asarray(minval, dtype=np.float32)
    hi = np.asarray(maxval, dtype=np.float32)
    out = (u * (hi - lo) + lo).astype(np.float32)
    return np.maximum(lo, out).astype(np.float32)


def bernoulli(key, p: float, shape=(), partitionable: bool = True) -> np.ndarray:
    return uniform(key, shape, partitionable=partitionable) < np.float32(p)


def choice_index(key, p, partitionable: bool = True) -> np.ndarray:
    """Index drawn by jax.random.choice(key, n, p=p) (replace=True, shape=())."""
    p = np.asarray(p, dtype=np.float32)
    cum = np.cumsum(p, dtype=np.float32)
    u = uniform(key, (), partitionable=partitionable)
    r = (cum[-1] * (np.float32(1.0) - u)).astype(np.float32)
    return np.searchsorted(cum, r, side="left") if np.ndim(r) == 0 else np.array(
        [np.searchsorted(cum, x, side="left") for x in np.ravel(r)]).reshape(np.shape(r))
