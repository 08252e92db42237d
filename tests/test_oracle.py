"""The CPU restatement (oracle/) pinned against the golden vectors.

Golden vectors: published KATs (CRC-32 check value, FIPS 180-2 SHA-256,
RFC 4648 base64) plus fixtures made by tests/golden/make_golden.py with
zlib/hashlib/base64 in the reference's byte layouts (wal.rs, datafile.rs,
sstable_index.rs, checksums.rs).  The reference's own tests carry no literal
checksum values, so these are what pins parity.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_crc32_text_kats(golden):
    for e in golden["crc32_text"]:
        assert O.crc32(e["text"].encode()) == e["crc"], e
    assert O.crc32(b"123456789") == 0xCBF43926
    assert O.crc32(b"") == 0


def test_crc32_slices(golden, blob):
    B = np.frombuffer(blob, dtype=np.uint8)
    off = np.array([e["off"] for e in golden["crc32_slices"]], dtype=np.uint64)
    ln = np.array([e["len"] for e in golden["crc32_slices"]], dtype=np.uint32)
    want = np.array([e["crc"] for e in golden["crc32_slices"]], dtype=np.uint32)
    assert np.array_equal(O.crc32_batch(B, off, ln), want)
    assert np.array_equal(O.crc32_batch(B, off, ln, threads=4), want)


def test_sha256_kats(golden, blob):
    for e in golden["sha256_text"]:
        assert O.sha256(e["text"].encode()).hex() == e["sha256"]
        assert O.base64(O.sha256(e["text"].encode())) == e["b64"]
    B = np.frombuffer(blob, dtype=np.uint8)
    off = np.array([e["off"] for e in golden["sha256_slices"]], dtype=np.uint64)
    ln = np.array([e["len"] for e in golden["sha256_slices"]], dtype=np.uint32)
    got = O.sha256_batch(B, off, ln, threads=4)
    for i, e in enumerate(golden["sha256_slices"]):
        assert got[i].tobytes().hex() == e["sha256"], e


def test_base64_rfc4648(golden):
    for e in golden["base64"]:
        assert O.base64(bytes.fromhex(e["hex"])) == e["b64"]


def test_wal_framing_matches_reference_tests(golden):
    # wal.rs:219-242 write_insert_log_record / write_remove_log_record
    assert O.wal_insert(b"key", b"value").hex() == golden["wal"]["insert_key_value"]
    assert O.wal_remove(b"key").hex() == golden["wal"]["remove_key"]
    # memtable.rs:113-134 restore_from_log
    img = (O.wal_insert(b"key", b"value") + O.wal_insert(b"key1", b"value1") + O.wal_insert(b"key2", b"value2") +
           O.wal_remove(b"key2"))
    assert img.hex() == golden["wal"]["restore_from_log"]
    st, recs, _ = O.wal_replay(img)
    assert st == 0 and [r.type for r in recs] == [1, 1, 1, 2]


def test_wal_replay_2000(golden):
    img = open(os.path.join(GOLDEN, golden["wal_2000"]["file"]), "rb").read()
    st, recs, _ = O.wal_replay(img)
    want = golden["wal_2000"]["records"]
    assert st == 0 and len(recs) == len(want)
    for r, w in zip(recs, want):
        assert (r.type, r.rec_off, r.klen, r.vlen, r.crc) == (w["type"], w["off"], w["klen"], w["vlen"], w["crc"])


def test_wal_replay_error_semantics(golden):
    img = bytearray(open(os.path.join(GOLDEN, golden["wal_2000"]["file"]), "rb").read())
    recs = golden["wal_2000"]["records"]
    ins = next(i for i, r in enumerate(recs) if r["type"] == 1 and r["klen"] + r["vlen"] > 0 and i > 10)
    rem = next(i for i, r in enumerate(recs) if r["type"] == 2 and r["klen"] > 0 and i > ins)
    # corrupt an Insert payload -> CorruptedData at that record (wal.rs:136-141)
    b = bytearray(img)
    b[recs[ins]["off"] + 13] ^= 0x40
    st, got, bad = O.wal_replay(bytes(b))
    assert st == 1 and bad[0] == ins and len(got) == ins and bad[2] == recs[ins]["crc"]
    # corrupt a Remove payload -> panic (wal.rs:154-159)
    b = bytearray(img)
    b[recs[rem]["off"] + 9] ^= 0x01
    st, got, bad = O.wal_replay(bytes(b))
    assert st == 2 and bad[0] == rem
    # bad type byte -> InvalidCommandType (wal.rs:36)
    b = bytearray(img)
    b[recs[5]["off"]] = 7
    st, got, bad = O.wal_replay(bytes(b))
    assert st == 3 and bad == (5, 7, bad[2]) and len(got) == 5
    # header truncated -> clean end (wal.rs:76-77)
    cut = recs[100]["off"] + 6
    st, got, _ = O.wal_replay(bytes(img[:cut]))
    assert st == 0 and len(got) == 100
    # payload truncated -> checksum of the short read mismatches
    cut = recs[100]["off"] + 13 + 1 if recs[100]["type"] == 1 else recs[100]["off"] + 9 + 1
    if recs[100]["klen"] + recs[100]["vlen"] > 1:
        st, got, bad = O.wal_replay(bytes(img[:cut]))
        assert st in (1, 2) and bad[0] == 100


def test_sstable_test_checksum_file(golden):
    g = golden["sstable_test"]
    d = O.file_checksum(os.path.join(GOLDEN, g["data"]))
    i = O.file_checksum(os.path.join(GOLDEN, g["index"]))
    assert O.checksums_json(i, d) == g["json"]
    assert open(os.path.join(GOLDEN, g["checksum"])).read() == g["json"]


def test_generators():
    # byte b of the stream = byte b%8 of splitmix64(seed ^ b//8)
    seed = 0x5EED0002
    s = O.gen_stream(seed, 8 * 1000 + 3, 64)
    for i, b in enumerate(s):
        pos = 8 * 1000 + 3 + i
        w = O.lib().oracle_splitmix64(seed ^ (pos // 8))
        assert b == (w >> (8 * (pos % 8))) & 0xFF
    L = O.gen_zipf_lengths(0x5EED0003, 1 << 16)
    assert L.min() >= 64 and L.max() <= 65536
    assert 1200 < L.mean() < 1900  # mean ~1538 B at s = 1.5
    assert abs((L == 64).mean() - 0.38) < 0.03


# BASELINE config 1: 2^20 x 256 B records of the splitmix64 stream,
# seed 0x5EED0001.  Summary digest = CRC-32 of the little-endian output array,
# for cross-run comparison (bench.py reports the GPU's as "summary_crc32").
CONFIG1_SUMMARY_CRC32 = 0x727D43C0


def test_config1_full_size_oracle_vs_zlib():
    """The oracle's Sarwate CRC at BASELINE config 1's full size against zlib's
    crc32 (an independent implementation of CRC-32/ISO-HDLC), record by record."""
    import zlib
    n = 1 << 20
    data = O.gen_stream(0x5EED0001, 0, n * 256)
    out = O.crc32_fixed(data, 256, 256, n, threads=8)
    mv = memoryview(data)
    z = np.fromiter((zlib.crc32(mv[i * 256:(i + 1) * 256]) for i in range(n)), dtype=np.uint32, count=n)
    assert np.array_equal(out, z)
    assert zlib.crc32(out.astype("<u4").tobytes()) == CONFIG1_SUMMARY_CRC32


# The oracle against independent implementations on arbitrary inputs
# (hypothesis): zlib.crc32 and hashlib.sha256, one record and a batch.
from hypothesis import given, settings, strategies as st  # noqa: E402


@settings(max_examples=200, deadline=None)
@given(st.lists(st.binary(max_size=700), min_size=1, max_size=40))
def test_property_oracle_batches_vs_stdlib(recs):
    import hashlib
    import zlib
    data = np.frombuffer(b"".join(recs) + b"\0" * 8, dtype=np.uint8)
    ln = np.array([len(r) for r in recs], dtype=np.uint32)
    off = np.zeros(len(recs), dtype=np.uint64)
    np.cumsum(ln[:-1].astype(np.uint64), out=off[1:])
    assert list(O.crc32_batch(data, off, ln)) == [zlib.crc32(r) for r in recs]
    got = np.asarray(O.sha256_batch(data, off, ln)).reshape(-1, 32)
    assert [bytes(g) for g in got] == [hashlib.sha256(r).digest() for r in recs]
    assert O.crc32(recs[0]) == zlib.crc32(recs[0])
