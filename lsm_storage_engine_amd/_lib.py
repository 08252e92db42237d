"""ctypes binding of liblsmck.so (the C ABI declared in include/lsmck.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C lsm_storage_engine_amd/csrc``).  There is no fallback: if the library
is missing this module raises on import, and the batch (GPU) entry points
return LSMCK_ENODEV when no MI355X is visible.

HIP runtime note: the torch wheel bundles its own libamdhip64 (soname
libamdhip64.so.7, same as /opt/rocm's).  A process that uses both torch and
this library must import torch FIRST, so that liblsmck resolves to the runtime
torch already loaded (one HIP runtime per process).  ``load()`` checks that.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblsmck.so")

# error / status codes (include/lsmck.h)
EINVAL = -22
ENOMEM = -12
EIO = -5
ENODEV = -19
EHIP = -1000
EJSON = -74
DATA_MISMATCH = 1
INDEX_MISMATCH = 2
WAL_CORRUPTED = 1
WAL_REMOVE_PANIC = 2
WAL_BAD_TYPE = 3
META_PANIC = 3  # lsmck_tree_verify status: metadata file unreadable / not SsTableMetadata JSON
PANIC_OPEN_FILE = 4      # checksums.rs:25 "Can't open file to calculate checksum" (the data file in verify/write)
PANIC_OPEN_INDEX = 5     # the same panic on the index file
PANIC_OPEN_CHECKSUM = 6  # checksums.rs:46 "Can't open checksum file"
SSTABLE_MAX_LEVEL = 5

DEVICE = 0x1
HOST = 0x0
HOST_PINNED = 0x2
SORTED = 0x4  # LSMCK_SORTED: device descriptors sorted inside one readable span (include/lsmck.h)
RECS_PINNED = 0x8  # LSMCK_RECS_PINNED: lsmck_wal_replay_verify's records array is page-locked
RECS_DEVICE = 0x10  # LSMCK_RECS_DEVICE: the records array is device memory (include/lsmck.h)

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
vp = C.c_void_p
sz = C.c_size_t


class Sha256Ctx(C.Structure):
    _fields_ = [("h", C.c_uint32 * 8), ("nbytes", C.c_uint64), ("buf", C.c_uint8 * 64), ("nbuf", C.c_uint32)]


class WalRec(C.Structure):
    _fields_ = [("rec_off", C.c_uint64), ("payload_off", C.c_uint64), ("klen", C.c_uint32),
                ("vlen", C.c_uint32), ("crc", C.c_uint32), ("type", C.c_uint32)]


class WalRec16(C.Structure):
    """lsmck_wal_rec16: payload offset with the type in bit 63 (set: Remove), klen, vlen."""
    _fields_ = [("payload_type", C.c_uint64), ("klen", C.c_uint32), ("vlen", C.c_uint32)]


WAL_REC16_REMOVE = 1 << 63


class TreeReport(C.Structure):
    _fields_ = [("tables", C.c_uint64), ("table_bytes", C.c_uint64), ("bad_tables", C.c_uint64),
                ("first_index", C.c_uint64), ("first_status", C.c_int), ("reserved", C.c_int),
                ("list_seconds", C.c_double), ("verify_seconds", C.c_double), ("stat_seconds", C.c_double),
                ("read_seconds", C.c_double), ("gpu_wait_seconds", C.c_double), ("compare_seconds", C.c_double),
                ("rounds", C.c_uint64), ("fds_cached", C.c_uint64),
                ("first_metadata_path", C.c_char * 4096)]


class TableEntry(C.Structure):
    _fields_ = [("metadata_path", C.c_char_p), ("data_path", C.c_char_p), ("index_path", C.c_char_p),
                ("checksum_path", C.c_char_p), ("id", C.c_char_p), ("level", C.c_uint), ("status", C.c_int)]


LISTED_FN = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(TableEntry), C.c_size_t)


# (name, restype, argtypes) for every symbol of include/lsmck.h
SIGNATURES = [
    ("lsmck_crc32_ieee", C.c_uint32, [vp, sz]),
    ("lsmck_crc32_update", C.c_uint32, [C.c_uint32, vp, sz]),
    ("lsmck_crc32_combine", C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint64]),
    ("lsmck_sha256_init", None, [C.POINTER(Sha256Ctx)]),
    ("lsmck_sha256_update", None, [C.POINTER(Sha256Ctx), vp, sz]),
    ("lsmck_sha256_final", None, [C.POINTER(Sha256Ctx), vp]),
    ("lsmck_sha256", None, [vp, sz, vp]),
    ("lsmck_base64_encode", sz, [vp, sz, C.c_char_p]),
    ("lsmck_checksum_file", C.c_int, [C.c_char_p, C.c_char_p]),
    ("lsmck_checksums_write", C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p]),
    ("lsmck_checksums_verify", C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p]),
    ("lsmck_wal_encode_insert", sz, [vp, C.c_uint32, vp, C.c_uint32, vp]),
    ("lsmck_wal_encode_remove", sz, [vp, C.c_uint32, vp]),
    ("lsmck_ctx_create", vp, [C.c_int]),
    ("lsmck_ctx_destroy", None, [vp]),
    ("lsmck_last_error", C.c_char_p, []),
    ("lsmck_device_count", C.c_int, []),
    ("lsmck_ctx_set_option", C.c_int, [vp, C.c_char_p, C.c_long]),
    ("lsmck_ctx_get_stat", C.c_int, [vp, C.c_char_p, C.POINTER(C.c_long)]),
    ("lsmck_crc32_batch", C.c_int, [vp, vp, vp, vp, sz, vp, C.c_uint, vp]),
    ("lsmck_crc32_batch_fixed", C.c_int, [vp, vp, sz, C.c_uint32, sz, vp, C.c_uint, vp]),
    ("lsmck_crc32_verify_batch", C.c_int, [vp, vp, vp, vp, vp, sz, C.c_uint, vp, u64p, u64p]),
    ("lsmck_sha256_batch", C.c_int, [vp, vp, vp, vp, sz, vp, C.c_uint, vp]),
    ("lsmck_sha256_batch_fixed", C.c_int, [vp, vp, sz, C.c_uint32, sz, vp, C.c_uint, vp]),
    ("lsmck_wal_replay_verify", C.c_int,
     [vp, vp, sz, C.c_uint, vp, sz, C.POINTER(sz), u64p, u32p, u32p]),  # recs: lsmck_wal_rec[cap]
    ("lsmck_wal_replay_verify16", C.c_int,
     [vp, vp, sz, C.c_uint, vp, sz, C.POINTER(sz), u64p, u32p, u32p]),  # recs: lsmck_wal_rec16[cap]
    ("lsmck_wal_frame_insert_device", C.c_int, [vp, vp, vp, vp, vp, sz, C.c_uint32, vp]),
    ("lsmck_checksums_verify_many", C.c_int,
     [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), sz, C.POINTER(C.c_int)]),
    ("lsmck_tree_verify", C.c_int, [vp, C.c_char_p, C.POINTER(TreeReport)]),
    ("lsmck_tree_verify_listed", C.c_int, [vp, C.c_char_p, C.POINTER(TreeReport), LISTED_FN, vp]),
    ("lsmck_tree_verify_multi", C.c_int, [C.POINTER(vp), sz, C.c_char_p, C.POINTER(TreeReport)]),
    ("lsmck_checksums_verify_many_multi", C.c_int,
     [C.POINTER(vp), sz, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), sz,
      C.POINTER(C.c_int)]),
    ("lsmck_dev_alloc", vp, [vp, sz]),
    ("lsmck_dev_free", None, [vp, vp]),
    ("lsmck_host_alloc_pinned", vp, [vp, sz]),
    ("lsmck_host_free_pinned", None, [vp, vp]),
    ("lsmck_memcpy_h2d", C.c_int, [vp, vp, vp, sz, vp]),
    ("lsmck_memcpy_d2h", C.c_int, [vp, vp, vp, sz, vp]),
    ("lsmck_memset_dev", C.c_int, [vp, vp, C.c_int, sz, vp]),
    ("lsmck_stream_sync", C.c_int, [vp, vp]),
    ("lsmck_gen_stream", C.c_int, [vp, vp, C.c_uint64, C.c_uint64, sz, vp]),
    ("lsmck_gen_zipf_lengths", None, [C.c_uint64, C.c_double, C.c_int, C.c_uint32, sz, vp]),
    ("lsmck_gen_zipf_lengths_at", None, [C.c_uint64, C.c_double, C.c_int, C.c_uint32, C.c_uint64, sz, vp]),
]

_lib = None


def _foreign_hip_runtime_loaded():
    """Path of a libamdhip64 already mapped into this process, if any."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    return line.split()[-1]
    except OSError:
        pass
    return None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built; run __graft_entry__.build() or "
                          f"make -C {os.path.join(_HERE, 'csrc')}")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error():
    msg = load().lsmck_last_error()
    return msg.decode(errors="replace") if msg else ""


class LsmckError(RuntimeError):
    def __init__(self, rc, what=""):
        self.rc = rc
        super().__init__(f"{what}: rc={rc} {last_error()}".strip())


def check(rc, what=""):
    if rc < 0:
        raise LsmckError(rc, what)
    return rc


def buf_ptr(b):
    """Pointer to a bytes-like object's memory without copying where possible."""
    import numpy as np
    if isinstance(b, np.ndarray):
        return b.ctypes.data
    if isinstance(b, (bytes, bytearray, memoryview)):
        a = np.frombuffer(b, dtype=np.uint8)
        return a.ctypes.data
    raise TypeError(type(b))
