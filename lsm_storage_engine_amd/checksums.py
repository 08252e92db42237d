"""SSTable file checksums -- the host-side mirror of src/checksums.rs.

``Checksums.calculate_checksum`` / ``verify`` / ``write_checksums`` keep the
reference's three signatures (checksums.rs:20, :40, :64) and semantics:
SHA-256 of the whole file, base64 STANDARD, the JSON record
{"index_checksum": ..., "data_checksum": ...}; verify fails (the reference
panics) naming the data file first, then the index file.

``Checksums.verify_many(ctx, metadatas)`` is the batch form used at engine load
and compaction: every data and index file of the tree hashed
in one GPU batch (lsmck_checksums_verify_many).
"""
import ctypes as C

from . import _lib


class ChecksumPanic(RuntimeError):
    """Where the reference panics (checksums.rs:25, :46, :49-60)."""


class ChecksumJsonError(OSError, ValueError):
    """The checksum file is not JSON of the Checksums shape: serde_json's error
    mapped to io::Error and returned as Err (checksums.rs:47-48), not a panic."""


class Checksums:
    def __init__(self, index_checksum, data_checksum):
        self.index_checksum = index_checksum
        self.data_checksum = data_checksum

    @staticmethod
    def calculate_checksum(path) -> str:
        """checksums.rs:20-38."""
        out = C.create_string_buffer(45)
        rc = _lib.load().lsmck_checksum_file(str(path).encode(), out)
        if rc == _lib.PANIC_OPEN_FILE:  # .expect at :25
            raise ChecksumPanic(f"Can't open file to calculate checksum: {_lib.last_error()}")
        if rc < 0:  # read error: Err (the `?` at :30)
            raise OSError(-rc, _lib.last_error())
        return out.value.decode()

    @staticmethod
    def verify(metadata):
        """checksums.rs:40-62."""
        rc = _lib.load().lsmck_checksums_verify(metadata.data_path().encode(), metadata.index_path().encode(),
                                               metadata.checksum_path().encode())
        _raise_for(rc, metadata)

    @staticmethod
    def write_checksums(metadata):
        """checksums.rs:64-80."""
        rc = _lib.load().lsmck_checksums_write(metadata.data_path().encode(), metadata.index_path().encode(),
                                              metadata.checksum_path().encode())
        if rc in (_lib.PANIC_OPEN_FILE, _lib.PANIC_OPEN_INDEX):  # calculate_checksum's .expect (:25)
            raise ChecksumPanic(f"Can't open file to calculate checksum: {_lib.last_error()}")
        if rc < 0:  # read error, or the checksum file cannot be opened / written: Err (:78-79)
            raise OSError(-rc, _lib.last_error())

    @staticmethod
    def verify_many(ctx, metadatas):
        """Batch verify of many SSTables; returns per-table status codes
        (0 ok, DATA_MISMATCH, INDEX_MISMATCH, PANIC_OPEN_*, -errno, EJSON);
        ``_raise_for`` turns one into the reference's panic or Err."""
        return ctx.checksums_verify_many([(m.data_path(), m.index_path(), m.checksum_path()) for m in metadatas])


def _raise_for(rc, metadata):
    """A verify status as the reference surfaces it: panics (checksums.rs:25,
    :46, :49-60) as ChecksumPanic, Err(io::Error) (:30, :48) as OSError."""
    if rc == 0:
        return
    if rc == _lib.DATA_MISMATCH:
        raise ChecksumPanic(f"Can't load SSTable from {metadata.data_filename}. Checksum is not correct")
    if rc == _lib.INDEX_MISMATCH:
        raise ChecksumPanic(f"Can't load SSTable from {metadata.index_filename}. Checksum is not correct")
    if rc in (_lib.PANIC_OPEN_FILE, _lib.PANIC_OPEN_INDEX):
        raise ChecksumPanic("Can't open file to calculate checksum")
    if rc == _lib.PANIC_OPEN_CHECKSUM:
        raise ChecksumPanic("Can't open checksum file")
    if rc == _lib.EJSON:
        raise ChecksumJsonError(_lib.last_error())
    raise OSError(-rc, _lib.last_error())
