"""Write-ahead log framing and replay -- the host-side mirror of src/wal.rs.

Same names, argument meaning and error behaviour as the reference:

* ``CommandLog.log`` frames a record exactly as wal.rs:165-196 and checksums
  its payload through the scalar CRC entry point (one record = one call).
* ``CommandLog.next_record`` / iteration restate wal.rs:68-84,122-163: a header
  cut short by end-of-file ends the iteration, an Insert whose CRC does not match
  raises ``CorruptedData``, a Remove whose CRC does not match is a panic in the
  reference (``WalPanic`` here), an unknown type byte raises
  ``InvalidCommandType``.
* ``CommandLog.replay_verify(ctx)`` is the batch form: the
  whole log's payload CRCs are checked in one GPU batch
  (lsmck_wal_replay_verify) and the same first error in log order is raised.
"""
import os
import struct
from dataclasses import dataclass

from . import _lib
from .crc32 import checksum_ieee

INSERT = 1
REMOVE = 2


class WalError(Exception):
    """wal.rs:14-22 WalError."""


class InvalidCommandType(WalError):
    def __init__(self, type_code):
        self.type_code = type_code
        super().__init__(f"invalid command type: {type_code}")


class CorruptedData(WalError):
    def __init__(self, checksum, expected):
        self.checksum = checksum
        self.expected = expected
        super().__init__(f"data corruption encountered ({checksum:08x}) != {expected:08x}")


class WalPanic(RuntimeError):
    """Where the reference panics (wal.rs:154-159, Remove checksum mismatch)."""


@dataclass(frozen=True)
class Insert:
    key: bytes
    val: bytes


@dataclass(frozen=True)
class Remove:
    key: bytes


class LogRecord:
    """wal.rs:41-45 LogRecord::{Insert, Remove}."""
    Insert = Insert
    Remove = Remove


class _Eof(Exception):
    pass


class CommandLog:
    """wal.rs:47-50.  ``file`` is any binary file object (or BytesIO)."""

    def __init__(self, file, path=None):
        self.file = file
        self.path = path

    # --- constructors -----------------------------------------------------
    @classmethod
    def new(cls, path):
        """wal.rs:86-101: create parent dirs, open read+append, seek to 0."""
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        f = open(path, "a+b")
        f.seek(0)
        return cls(f, path)

    @classmethod
    def new_in_memory(cls, vec=b""):
        """wal.rs:205-213 (test helper)."""
        import io
        b = io.BytesIO(bytes(vec))
        b.seek(0)
        return cls(b, None)

    def inner(self):
        return self.file.getvalue()

    def close(self):
        """wal.rs:103-108: closing the log deletes the file."""
        if self.path is not None:
            self.file.close()
            os.remove(self.path)

    # --- append -----------------------------------------------------------
    def insert(self, key, val):
        return self.log(Insert(bytes(key), bytes(val)))

    def remove(self, key):
        return self.log(Remove(bytes(key)))

    def log(self, record):
        """wal.rs:165-196.  Returns data_len + 5 / key_len + 5 as the reference
        does (the header is 13 / 9 bytes; the value is unused by callers)."""
        if isinstance(record, Insert):
            data = record.key + record.val
            crc = checksum_ieee(data)
            self.file.write(struct.pack("<BIII", INSERT, crc, len(record.key), len(record.val)) + data)
            self.file.flush()
            return len(data) + 5
        crc = checksum_ieee(record.key)
        self.file.write(struct.pack("<BII", REMOVE, crc, len(record.key)) + record.key)
        self.file.flush()
        return len(record.key) + 5

    # --- replay -----------------------------------------------------------
    def _read_exact(self, n):
        b = self.file.read(n)
        if len(b) < n:
            raise _Eof()
        return b

    def next_record(self):
        """wal.rs:122-163; raises EOFError at a truncated header."""
        try:
            t = self._read_exact(1)[0]
            if t not in (INSERT, REMOVE):
                raise InvalidCommandType(t)
            saved = struct.unpack("<I", self._read_exact(4))[0]
            if t == INSERT:
                klen, vlen = struct.unpack("<II", self._read_exact(8))
            else:
                klen, vlen = struct.unpack("<I", self._read_exact(4))[0], 0
        except _Eof:
            raise EOFError("UnexpectedEof")
        dlen = (klen + vlen) & 0xFFFFFFFF
        data = self.file.read(dlen)  # read_to_end on take(): short at EOF, no error
        crc = checksum_ieee(data)
        if crc != saved:
            if t == INSERT:
                raise CorruptedData(crc, saved)
            raise WalPanic(f"data corruption encountered ({crc:08x}) != {saved:08x}")
        if t == INSERT:
            if len(data) < klen:  # cut at EOF inside the key: data.split_off(key_len) panics (wal.rs:142)
                raise WalPanic(_split_off_msg(klen, len(data)))
            return Insert(data[:klen], data[klen:])
        return Remove(data)

    def __iter__(self):
        """wal.rs:68-84: UnexpectedEof ends the iteration, other errors surface."""
        while True:
            try:
                yield self.next_record()
            except EOFError:
                return

    def replay_verify(self, ctx):
        """Batch replay of the whole log from its current position: every
        payload CRC checked in one GPU batch.  Returns the records in log
        order; raises the error the iterator would raise first."""
        pos = self.file.tell()
        img = self.file.read()
        records, status, bad = ctx.wal_replay_verify(img, compact=True)  # 16-byte records: all from_log needs
        if status == _lib.WAL_CORRUPTED:
            raise CorruptedData(bad[1], bad[2])
        if status == _lib.WAL_REMOVE_PANIC:
            raise WalPanic(f"data corruption encountered ({bad[1]:08x}) != {bad[2]:08x}")
        if status == _lib.WAL_BAD_TYPE:
            raise InvalidCommandType(bad[1])
        out = []
        consumed = 0
        from .device import decode_rec16
        r = decode_rec16(records)
        for k0, kl, vl, t in zip(r["payload_off"].tolist(), r["klen"].tolist(), r["vlen"].tolist(), r["type"].tolist()):
            # the payload actually read: u32 data_len (wal.rs:129), short at EOF
            # (read_to_end on take(), :132) -- the same bytes the CRC covered
            data = img[k0:k0 + ((kl + vl) & 0xFFFFFFFF)]
            if t == INSERT:
                if len(data) < kl:  # cut at EOF inside the key: split_off panics (wal.rs:142)
                    raise WalPanic(_split_off_msg(kl, len(data)))
                out.append(Insert(data[:kl], data[kl:]))  # data.split_off(key_len), wal.rs:142
            else:
                out.append(Remove(data))
            consumed = k0 + len(data)
        self.file.seek(pos + consumed)
        return out


def _split_off_msg(at, length):
    """Vec::split_off's panic message (the reference's wal.rs:142 on a key cut at EOF)."""
    return f"`at` split index (is {at}) should be <= len (is {length})"


class MemTable:
    """The replay consumer, src/memtable.rs:9-47 (BTreeMap + byte count)."""

    def __init__(self):
        self.data = {}
        self.bytes = 0

    @classmethod
    def from_log(cls, log, ctx=None):
        """memtable.rs:28-47.  With ``ctx`` the log is verified in one GPU batch."""
        t = cls()
        recs = log.replay_verify(ctx) if ctx is not None else log
        for rec in recs:
            if isinstance(rec, Insert):
                t.data[rec.key] = rec.val
                t.bytes += len(rec.key) + len(rec.val)
            else:
                v = t.data.pop(rec.key, None)
                t.bytes -= (len(v) + len(rec.key)) if v is not None else 0
        return t

    def get(self, key):
        return self.data.get(bytes(key))

    def insert(self, key, val):
        key, val = bytes(key), bytes(val)
        prev = self.data.get(key)
        self.data[key] = val
        self.bytes = self.bytes + len(key) + len(val) - ((len(prev) + len(key)) if prev is not None else 0)
        return prev

    def remove(self, key):
        key = bytes(key)
        prev = self.data.pop(key, None)
        self.bytes -= (len(prev) + len(key)) if prev is not None else 0
        return prev

    def size(self):
        return len(self.data)

    def size_in_bytes(self):
        return self.bytes

    def __iter__(self):
        return iter(sorted(self.data.items()))
