"""device.Context reuses the WAL replay's records array only when no earlier
result still refers to it (host logic; no GPU)."""
import numpy as np

from lsm_storage_engine_amd.device import Context


class _Ctx(Context):
    def __init__(self):  # no device: only the buffer logic
        self._wal_recs = None
        self.handle = None

    def replay(self, cap=100):
        recs = self._wal_recs_buffer(cap)
        return recs[:10].view(np.recarray), 0


def test_records_array_reused_only_when_released():
    c = _Ctx()
    r1, _ = c.replay()
    id1 = id(c._wal_recs)
    r2, _ = c.replay()
    assert id(c._wal_recs) != id1  # r1 still alive: a fresh array
    id2 = id(c._wal_recs)
    del r1, r2
    r3, _ = c.replay()
    assert id(c._wal_recs) == id2  # nothing refers to it: reused
    r3[0]["crc"] = 5
    r4, _ = c.replay()
    assert id(c._wal_recs) != id2 and r3[0]["crc"] == 5  # r3 untouched by the next replay
    r5, _ = c.replay(cap=10**6)
    assert len(c._wal_recs) >= 10**6  # grows when a larger log needs it
