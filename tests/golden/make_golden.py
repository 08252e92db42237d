#!/usr/bin/env python3
"""Generate the committed golden fixtures for the checksum path.

The reference (Rust) cannot be built or imported here and its own tests hold
no literal checksum values, so the vectors come from
independent standard implementations of the algorithms its crates implement:

  * zlib.crc32            == crc 1.x crc32::checksum_ieee (CRC-32/ISO-HDLC)
  * hashlib.sha256        == sha2 0.10 Sha256 (FIPS 180-4)
  * base64.b64encode      == base64 0.13 encode (STANDARD, padded)

laid out exactly as the reference's byte formats:

  * WAL records, CommandLog::log             src/wal.rs:165-196
  * SSTable data file, write_key_value       src/datafile.rs:27-35
  * SSTable index, bincode 1.x fixint map    src/sstable_index.rs:42-46
  * checksum file, serde_json of Checksums   src/checksums.rs:13-17,75-79

Run:  python3 tests/golden/make_golden.py   (writes next to this script)
"""
import base64
import hashlib
import json
import os
import struct
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))


def blob(n, seed=b"lsmck-golden"):
    """Deterministic pseudo-random bytes (SHA-256 counter mode)."""
    out = bytearray()
    i = 0
    while len(out) < n:
        out += hashlib.sha256(seed + struct.pack("<Q", i)).digest()
        i += 1
    return bytes(out[:n])


def crc(b):
    return zlib.crc32(b) & 0xFFFFFFFF


# --- wal.rs framing ---------------------------------------------------------
def wal_insert(key, val):
    data = key + val
    return struct.pack("<BIII", 1, crc(data), len(key), len(val)) + data


def wal_remove(key):
    return struct.pack("<BII", 2, crc(key), len(key)) + key


# --- datafile.rs / sstable_index.rs ----------------------------------------
def sstable_files(entries, index_step=100):
    """entries: iterable of (key, val) already in BTreeMap order."""
    data = bytearray()
    index = []
    pos = 0
    for i, (k, v) in enumerate(entries):
        rec = struct.pack("<II", len(k), len(v)) + k + v
        if i % index_step == 0:
            index.append((k, pos))
        data += rec
        pos += len(rec)
    idx = bytearray(struct.pack("<Q", len(index)))
    for k, p in index:
        idx += struct.pack("<Q", len(k)) + k + struct.pack("<Q", p)
    return bytes(data), bytes(idx)


def b64sha(b):
    return base64.b64encode(hashlib.sha256(b).digest()).decode()


def checksum_json(index_b64, data_b64):
    return json.dumps({"index_checksum": index_b64, "data_checksum": data_b64}, separators=(",", ":"))


def main():
    fx = {}
    B = blob(1 << 17)
    with open(os.path.join(HERE, "blob.bin"), "wb") as f:
        f.write(B)

    # CRC-32 known answers
    kat = [
        ("", 0x00000000),
        ("123456789", 0xCBF43926),  # the CRC-32/ISO-HDLC check value
        ("keyvalue", None),
        ("key", None),
        ("a", None),
        ("abc", None),
        ("The quick brown fox jumps over the lazy dog", 0x414FA339),
    ]
    fx["crc32_text"] = []
    for s, want in kat:
        c = crc(s.encode())
        if want is not None:
            assert c == want, (s, hex(c))
        fx["crc32_text"].append({"text": s, "crc": c})
    # slices of the blob: every length 0..300 at 4 alignments, and big ones
    sl = []
    for ln in range(0, 301):
        for a in (0, 1, 2, 3):
            o = 1000 + 37 * ln + a
            sl.append((o, ln))
    for ln in (383, 384, 385, 511, 512, 513, 1000, 4095, 4096, 4097, 8191, 8192, 8193, 65535, 65536, 65537):
        for a in (0, 3, 5, 16):
            sl.append((a, ln))
    assert all(o + l <= len(B) for o, l in sl)
    fx["crc32_slices"] = [{"off": o, "len": l, "crc": crc(B[o:o + l])} for o, l in sl]

    # SHA-256 known answers (FIPS 180-2 appendix B) + base64
    fips = [
        ("", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
        ("abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
        ("abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
         "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
        ("abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu",
         "cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"),
    ]
    fx["sha256_text"] = []
    for s, want in fips:
        d = hashlib.sha256(s.encode()).hexdigest()
        assert d == want
        fx["sha256_text"].append({"text": s, "sha256": d, "b64": b64sha(s.encode())})
    assert b64sha(b"") == "47DEQpj8HBSa+/TImW+5JCeuQeRkm5NMpJWZG3hSuFU="
    ssl = []
    for ln in list(range(0, 200)) + [447, 448, 449, 1023, 1024, 1025, 4095, 4096, 4097, 65536, 100001]:
        for a in (0, 1, 2, 3):
            ssl.append(((7 * ln) % (len(B) - ln - 8) + a, ln))
    assert all(o + l <= len(B) for o, l in ssl)
    fx["sha256_slices"] = [{"off": o, "len": l, "sha256": hashlib.sha256(B[o:o + l]).hexdigest()} for o, l in ssl]

    # base64 (RFC 4648 section 10)
    fx["base64"] = [{"hex": s.encode().hex(), "b64": base64.b64encode(s.encode()).decode()}
                    for s in ("", "f", "fo", "foo", "foob", "fooba", "foobar")]

    # WAL images: wal.rs tests and memtable.rs restore_from_log
    ins = wal_insert(b"key", b"value")
    rem = wal_remove(b"key")
    assert ins.hex() == "01e6f355c603000000050000006b657976616c7565", ins.hex()
    assert rem.hex() == "02a9ab908a030000006b6579", rem.hex()
    restore = (wal_insert(b"key", b"value") + wal_insert(b"key1", b"value1") + wal_insert(b"key2", b"value2")
               + wal_remove(b"key2"))
    assert len(restore) == 80
    fx["wal"] = {
        "insert_key_value": ins.hex(),
        "remove_key": rem.hex(),
        "restore_from_log": restore.hex(),
    }
    # a bigger deterministic WAL: 2000 records, mixed insert/remove, sizes 0..700
    recs = []
    img = bytearray()
    rnd = blob(20000, b"wal-shape")
    for i in range(2000):
        kl = rnd[4 * i] % 40
        vl = (rnd[4 * i + 1] | (rnd[4 * i + 2] << 8)) % 700
        key = B[(i * 97) % 60000:(i * 97) % 60000 + kl]
        if rnd[4 * i + 3] % 7 == 0:
            r = wal_remove(key)
            recs.append({"type": 2, "off": len(img), "klen": kl, "vlen": 0, "crc": crc(key)})
        else:
            val = B[(i * 389) % 60000:(i * 389) % 60000 + vl]
            r = wal_insert(key, val)
            recs.append({"type": 1, "off": len(img), "klen": kl, "vlen": vl, "crc": crc(key + val)})
        img += r
    with open(os.path.join(HERE, "wal_2000.bin"), "wb") as f:
        f.write(img)
    fx["wal_2000"] = {"file": "wal_2000.bin", "records": recs}

    # SSTable of sync/sstable.rs sstable_test: keys i.to_string(), values (i*100).to_string(), i in 0..500,
    # in BTreeMap (bytewise) order
    ents = sorted(((str(i).encode(), str(i * 100).encode()) for i in range(500)), key=lambda kv: kv[0])
    data, index = sstable_files(ents)
    assert len(data) == 7778 and len(index) == 101, (len(data), len(index))
    with open(os.path.join(HERE, "sstable_test_data.db"), "wb") as f:
        f.write(data)
    with open(os.path.join(HERE, "sstable_test_index.db"), "wb") as f:
        f.write(index)
    cj = checksum_json(b64sha(index), b64sha(data))
    assert cj == ('{"index_checksum":"zqWNuAB4Nq6qUFyuUxqUno+n1MTst0tK2hPBdmppD+s=",'
                  '"data_checksum":"O0gfuQX131pwnlEuXSMuxBMZ0vGJNsVJ2cmtPery5fU="}'), cj
    with open(os.path.join(HERE, "sstable_test_checksum.db"), "w") as f:
        f.write(cj)
    fx["sstable_test"] = {"data": "sstable_test_data.db", "index": "sstable_test_index.db",
                          "checksum": "sstable_test_checksum.db", "json": cj,
                          "index_keys": [k.decode() for k, _ in ents[::100]]}

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(fx, f, indent=0, sort_keys=True)
    print("wrote", len(fx["crc32_slices"]), "crc slices,", len(fx["sha256_slices"]), "sha slices")


if __name__ == "__main__":
    main()
