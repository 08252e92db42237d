"""Paths of one SSTable's files -- mirror of src/sstable_metadata.rs.

Only what the checksum path needs: the file naming scheme
``<base>/level-<n>/{metadata,data,index,checksum,bloom}_<ms>.db``
(sstable_metadata.rs:20-68) and the JSON metadata record (:70-85).
"""
import json
import os
import time


class SsTableMetadata:
    FIELDS = ("base_path", "id", "level", "metadata_filename", "checksum_filename", "data_filename",
              "index_filename", "bloom_filter_filename")

    def __init__(self, base_path, id, level, metadata_filename, checksum_filename, data_filename, index_filename,
                 bloom_filter_filename):
        self.base_path = base_path
        self.id = id
        self.level = level
        self.metadata_filename = metadata_filename
        self.checksum_filename = checksum_filename
        self.data_filename = data_filename
        self.index_filename = index_filename
        self.bloom_filter_filename = bloom_filter_filename

    @classmethod
    def new(cls, base_path, level, timestamp_ms=None):
        """sstable_metadata.rs:20-42 (id = milliseconds since the epoch)."""
        ts = int(time.time() * 1000) if timestamp_ms is None else int(timestamp_ms)
        return cls(base_path, ts, level, f"metadata_{ts}.db", f"checksum_{ts}.db", f"data_{ts}.db",
                   f"index_{ts}.db", f"bloom_{ts}.db")

    def construct_path(self, filename):
        return os.path.join(self.base_path, f"level-{self.level}", filename)

    def data_path(self):
        return self.construct_path(self.data_filename)

    def index_path(self):
        return self.construct_path(self.index_filename)

    def checksum_path(self):
        return self.construct_path(self.checksum_filename)

    def metadata_path(self):
        return self.construct_path(self.metadata_filename)

    def bloom_filter_path(self):
        return self.construct_path(self.bloom_filter_filename)

    @classmethod
    def load(cls, metadata_path):
        with open(metadata_path) as f:
            d = json.load(f)
        return cls(**{k: d[k] for k in cls.FIELDS})

    def write_to_file(self):
        """serde_json::to_writer in struct declaration order (:7-17, :79-85)."""
        order = ("base_path", "id", "level", "metadata_filename", "checksum_filename", "data_filename",
                 "index_filename", "bloom_filter_filename")
        s = json.dumps({k: getattr(self, k) for k in order}, separators=(",", ":"))
        fd = os.open(self.metadata_path(), os.O_WRONLY | os.O_CREAT, 0o644)  # no truncate, as the reference
        try:
            os.write(fd, s.encode())
        finally:
            os.close(fd)
