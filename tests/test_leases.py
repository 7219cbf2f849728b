"""Page-locked output leases (pupperv3_mjx._lib: PinnedBlock.take / _BlockRef / BlockPool), on CPU
with a stand-in block: the arrays of a lease are read-only, keep the lease alive, and the block
returns to its pool the moment the last of them dies (reference counting, no finalizer
registration); a retired pool frees a block released into it."""
import ctypes as C
import gc

import numpy as np
import pytest

from pupperv3_mjx import _lib


class _FakeBlock:
    """The attributes of a PinnedBlock a lease uses, over ordinary host memory."""

    def __init__(self, n):
        self.buf = np.arange(n, dtype=np.float32)
        self.ptr = C.c_void_p(self.buf.ctypes.data)
        self.__array_interface__ = {"shape": (n,), "typestr": "<f4", "version": 3, "data": (self.ptr.value, False)}
        self._ro_interface = dict(self.__array_interface__, data=(self.ptr.value, True))
        self.freed = False

    def free(self):
        self.freed = True


def test_lease_arrays_are_read_only_views_of_the_block():
    pool = _lib.BlockPool()
    blk = _FakeBlock(64)
    pool.append(blk)
    lease = _lib.PinnedBlock.take(256, pool)
    assert len(pool) == 0 and lease.block is blk
    flat = np.asarray(lease)
    obs = flat[:32].reshape(4, 8)
    assert not flat.flags.writeable and not obs.flags.writeable
    np.testing.assert_array_equal(obs.ravel(), np.arange(32, dtype=np.float32))
    with pytest.raises(ValueError):
        obs[0, 0] = 1.0
    blk.buf[0] = 7.0  # (a view, not a copy: the launch's stores show through)
    assert obs[0, 0] == 7.0


def test_block_returns_when_the_last_array_dies():
    pool = _lib.BlockPool()
    blk = _FakeBlock(64)
    pool.append(blk)
    lease = _lib.PinnedBlock.take(256, pool)
    obs = np.asarray(lease)[:32].reshape(4, 8)
    rew = np.asarray(lease)[32:36]
    del lease
    assert len(pool) == 0  # the arrays still hold it
    del obs
    assert len(pool) == 0
    del rew  # no gc.collect(): reference counting releases it
    assert len(pool) == 1 and pool[0] is blk and not blk.freed


def test_retired_pool_frees_a_block_released_later():
    pool = _lib.BlockPool()
    blk = _FakeBlock(16)
    pool.append(blk)
    arr = np.asarray(_lib.PinnedBlock.take(64, pool))
    pool.retire()
    del arr
    gc.collect()
    assert blk.freed and len(pool) == 0


def test_action_slot_waits_once_per_record():
    """An action staging slot synchronizes its completion event once per record: a wait that
    already saw the launch complete is not repeated (the host loop's ring reuse)."""
    from pupperv3_mjx.environment import _ActSlot
    calls = []

    class FakeLib:
        def pp3_event_record(self, h, ev):
            calls.append("record")
            return 0

        def pp3_event_synchronize(self, ev):
            calls.append("sync")
            return 0

    slot = object.__new__(_ActSlot)
    slot._L, slot._h, slot.ev, slot.pending = FakeLib(), None, C.c_void_p(1), False
    slot.wait()
    assert calls == []  # never recorded: nothing to wait for
    slot.record()
    slot.wait()
    slot.wait()
    assert calls == ["record", "sync"]
    slot.record()
    slot.wait()
    assert calls == ["record", "sync", "record", "sync"]
