"""ctypes wrapper of the CPU restatement (oracle/liblsmck_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.  See
lsmck_oracle.h for what it restates and how it is pinned.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liblsmck_oracle.so")
_lib = None


class WalRec(C.Structure):
    _fields_ = [("rec_off", C.c_uint64), ("payload_off", C.c_uint64), ("klen", C.c_uint32),
                ("vlen", C.c_uint32), ("crc", C.c_uint32), ("type", C.c_uint8)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp, sz = C.c_void_p, C.c_size_t
        L.oracle_crc32_ieee.restype = C.c_uint32
        L.oracle_crc32_ieee.argtypes = [vp, sz]
        L.oracle_crc32_batch.argtypes = [vp, vp, vp, sz, vp, C.c_int]
        L.oracle_crc32_fixed.argtypes = [vp, sz, sz, sz, vp, C.c_int]
        L.oracle_sha256.argtypes = [vp, sz, vp]
        L.oracle_sha256_batch.argtypes = [vp, vp, vp, sz, vp, C.c_int]
        L.oracle_base64_std.restype = sz
        L.oracle_base64_std.argtypes = [vp, sz, C.c_char_p]
        L.oracle_file_checksum.argtypes = [C.c_char_p, C.c_char_p]
        L.oracle_checksums_json.restype = sz
        L.oracle_checksums_json.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, sz]
        L.oracle_wal_encode_insert.restype = sz
        L.oracle_wal_encode_insert.argtypes = [vp, C.c_uint32, vp, C.c_uint32, vp]
        L.oracle_wal_encode_remove.restype = sz
        L.oracle_wal_encode_remove.argtypes = [vp, C.c_uint32, vp]
        L.oracle_wal_replay.argtypes = [vp, sz, C.POINTER(WalRec), sz, C.POINTER(sz), C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.oracle_splitmix64.restype = C.c_uint64
        L.oracle_splitmix64.argtypes = [C.c_uint64]
        L.oracle_gen_stream.argtypes = [C.c_uint64, C.c_uint64, sz, vp]
        L.oracle_gen_zipf_lengths.argtypes = [C.c_uint64, C.c_double, C.c_int, C.c_uint32, sz, vp]
        L.oracle_gen_zipf_lengths_at.argtypes = [C.c_uint64, C.c_double, C.c_int, C.c_uint32, C.c_uint64, sz, vp]
        _lib = L
    return _lib


def _u8(b):
    return np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b


def crc32(b):
    a = _u8(b)
    return lib().oracle_crc32_ieee(a.ctypes.data, len(a))


def crc32_batch(data, off, length, threads=1):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    out = np.empty(len(off), dtype=np.uint32)
    lib().oracle_crc32_batch(data.ctypes.data, off.ctypes.data, length.ctypes.data, len(off), out.ctypes.data, threads)
    return out


def crc32_fixed(data, stride, length, n, threads=1):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.empty(n, dtype=np.uint32)
    lib().oracle_crc32_fixed(data.ctypes.data, stride, length, n, out.ctypes.data, threads)
    return out


def sha256(b):
    a = _u8(b)
    out = np.empty(32, dtype=np.uint8)
    lib().oracle_sha256(a.ctypes.data, len(a), out.ctypes.data)
    return out.tobytes()


def sha256_batch(data, off, length, threads=1):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    out = np.empty((len(off), 32), dtype=np.uint8)
    lib().oracle_sha256_batch(data.ctypes.data, off.ctypes.data, length.ctypes.data, len(off), out.ctypes.data,
                              threads)
    return out


def base64(b):
    a = _u8(b)
    out = C.create_string_buffer(4 * (len(a) // 3 + 2) + 1)
    lib().oracle_base64_std(a.ctypes.data, len(a), out)
    return out.value.decode()


def file_checksum(path):
    out = C.create_string_buffer(45)
    rc = lib().oracle_file_checksum(str(path).encode(), out)
    if rc:
        raise OSError(-rc, path)
    return out.value.decode()


def checksums_json(index_b64, data_b64):
    out = C.create_string_buffer(256)
    lib().oracle_checksums_json(index_b64.encode(), data_b64.encode(), out, 256)
    return out.value.decode()


def wal_insert(key, val):
    k, v = _u8(key), _u8(val)
    out = np.empty(13 + len(k) + len(v), dtype=np.uint8)
    n = lib().oracle_wal_encode_insert(k.ctypes.data, len(k), v.ctypes.data, len(v), out.ctypes.data)
    return out[:n].tobytes()


def wal_remove(key):
    k = _u8(key)
    out = np.empty(9 + len(k), dtype=np.uint8)
    n = lib().oracle_wal_encode_remove(k.ctypes.data, len(k), out.ctypes.data)
    return out[:n].tobytes()


def wal_replay(image):
    a = _u8(image)
    cap = len(a) // 9 + 1
    recs = (WalRec * cap)()
    nrec = C.c_size_t()
    bi, bc, be = C.c_uint64(), C.c_uint32(), C.c_uint32()
    st = lib().oracle_wal_replay(a.ctypes.data, len(a), recs, cap, C.byref(nrec), C.byref(bi), C.byref(bc),
                                 C.byref(be))
    return st, list(recs[:nrec.value]), (bi.value, bc.value, be.value)


def gen_stream(seed, byte_off, n):
    out = np.empty(n, dtype=np.uint8)
    lib().oracle_gen_stream(seed, byte_off, n, out.ctypes.data)
    return out


def gen_zipf_lengths(seed, n, s=1.5, kmax=1024, lmin=64, first=0):
    """lengths of records [first, first + n) of the config-3 length stream"""
    out = np.empty(n, dtype=np.uint32)
    lib().oracle_gen_zipf_lengths_at(seed, s, kmax, lmin, first, n, out.ctypes.data)
    return out
