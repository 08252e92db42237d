"""lsm_storage_engine_amd -- MI355X-native checksum path of lsm_storage_engine.

The hot path of the reference's integrity checks, rebuilt for gfx950:
  * CRC-32/ISO-HDLC per WAL record (src/wal.rs, crate crc ^1.7) and
  * SHA-256 + base64 per SSTable file (src/checksums.rs, sha2 ^0.10),
batched over HBM-resident records by hand-written HIP kernels behind the C ABI
of include/lsmck.h (liblsmck.so, built in-tree).

Modules mirror the reference's interface: ``crc32`` (checksum_ieee),
``wal`` (CommandLog, LogRecord, WalError, MemTable.from_log), ``checksums``
(Checksums), ``sstable_metadata`` (SsTableMetadata); ``device`` holds the GPU
context and batch entry points.
"""
from . import _lib  # noqa: F401

__all__ = ["crc32", "wal", "checksums", "sstable_metadata", "device"]
