"""device.Context reuses the WAL replay's records array only when no earlier
result still refers to it (host logic; no GPU)."""
import numpy as np

from lsm_storage_engine_amd.device import WAL_REC16_DTYPE, WAL_REC_DTYPE, Context


class _Ctx(Context):
    def __init__(self):  # no device: only the buffer logic
        self._wal_recs = {}
        self.handle = None

    def replay(self, cap=100, dtype=WAL_REC_DTYPE):
        recs = self._wal_recs_buffer(cap, dtype)
        return recs[:10].view(np.recarray), 0

    def cur(self, dtype=WAL_REC_DTYPE):
        return self._wal_recs[dtype.str]


def test_records_array_reused_only_when_released():
    c = _Ctx()
    r1, _ = c.replay()
    id1 = id(c.cur())
    r2, _ = c.replay()
    assert id(c.cur()) != id1  # r1 still alive: a fresh array
    id2 = id(c.cur())
    del r1, r2
    r3, _ = c.replay()
    assert id(c.cur()) == id2  # nothing refers to it: reused
    r3[0]["crc"] = 5
    r4, _ = c.replay()
    assert id(c.cur()) != id2 and r3[0]["crc"] == 5  # r3 untouched by the next replay
    r5, _ = c.replay(cap=10**6)
    assert len(c.cur()) >= 10**6  # grows when a larger log needs it


def test_compact_records_have_their_own_array():
    c = _Ctx()
    r1, _ = c.replay()
    r2, _ = c.replay(dtype=WAL_REC16_DTYPE)
    assert c.cur(WAL_REC16_DTYPE).dtype.itemsize == 16 and c.cur().dtype.itemsize == 32
    del r1, r2
    i16 = id(c.cur(WAL_REC16_DTYPE))
    c.replay(dtype=WAL_REC16_DTYPE)
    assert id(c.cur(WAL_REC16_DTYPE)) == i16  # reused within its own dtype


def test_multicontext_replay_takes_the_context_options():
    """MultiContext.wal_replay_verify (the tree's WAL on the first device)
    accepts every option Context.wal_replay_verify does: MemTable.from_log
    calls it with compact=True on either."""
    import inspect

    from lsm_storage_engine_amd.device import MultiContext

    one = inspect.signature(Context.wal_replay_verify).parameters
    multi = inspect.signature(MultiContext.wal_replay_verify).parameters
    assert list(multi) == list(one)
    assert all(multi[k].default == one[k].default for k in one)
