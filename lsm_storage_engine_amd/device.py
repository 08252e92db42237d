"""GPU context and batch entry points (include/lsmck.h sections 2-4).

``Context`` owns one liblsmck context (one MI355X).  Host-array methods take
numpy arrays and return numpy arrays (the library stages them through pinned
memory); ``*_device`` methods take raw device pointers (ints) and run
asynchronously on ``stream`` (a hipStream_t as int, or None for the context's
stream) -- that is the device-resident hot path the bench times.

There is no CPU fallback: constructing a Context without a usable gfx950 GPU
raises.
"""
import ctypes as C
import sys

import numpy as np

from . import _lib
from .shard import shard_by_bytes, shard_fixed


def _p(a):
    return None if a is None else a.ctypes.data


class DeviceBuffer:
    def __init__(self, ctx, nbytes):
        self.ctx = ctx
        self.nbytes = nbytes
        self.ptr = _lib.load().lsmck_dev_alloc(ctx.handle, nbytes)
        if not self.ptr:
            raise MemoryError(f"hipMalloc({nbytes}): {_lib.last_error()}")

    def free(self):
        if self.ptr:
            _lib.load().lsmck_dev_free(self.ctx.handle, self.ptr)
            self.ptr = None

    def upload(self, arr, offset=0):
        a = np.ascontiguousarray(arr)
        assert offset + a.nbytes <= self.nbytes
        _lib.check(_lib.load().lsmck_memcpy_h2d(self.ctx.handle, self.ptr + offset, a.ctypes.data, a.nbytes, None),
                   "h2d")

    def download(self, dtype=np.uint8, count=None, offset=0):
        dt = np.dtype(dtype)
        count = (self.nbytes - offset) // dt.itemsize if count is None else count
        out = np.empty(count, dtype=dt)
        _lib.check(_lib.load().lsmck_memcpy_d2h(self.ctx.handle, out.ctypes.data, self.ptr + offset, out.nbytes, None),
                   "d2h")
        return out

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedBuffer:
    """Page-locked host memory (hipHostMalloc through liblsmck); ``array`` is a
    uint8 numpy view.  Batch calls given these arrays with pinned=True DMA
    straight from / to them (LSMCK_HOST_PINNED)."""

    def __init__(self, ctx, nbytes):
        self.ctx = ctx
        self.nbytes = nbytes
        self.ptr = _lib.load().lsmck_host_alloc_pinned(ctx.handle, max(1, nbytes))
        if not self.ptr:
            raise MemoryError(f"hipHostMalloc({nbytes}): {_lib.last_error()}")
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(1, nbytes)).from_address(self.ptr))[:nbytes]

    def free(self):
        if self.ptr:
            self.array = None
            _lib.load().lsmck_host_free_pinned(self.ctx.handle, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class _PinnedRecords:
    """numpy's view of a PinnedBuffer as lsmck_wal_rec[n] (or another record
    dtype): the arrays made from it keep it (and the page-locked memory) alive."""

    def __init__(self, pb, n, dtype):
        self.pb = pb
        self.__array_interface__ = {"data": (pb.ptr, False), "shape": (n,), "typestr": dtype.str,
                                    "descr": dtype.descr, "version": 3}


class Context:
    def __init__(self, device=0):
        lib = _lib.load()
        self.lib = lib
        self.handle = lib.lsmck_ctx_create(device)
        if not self.handle:
            raise RuntimeError(f"lsmck_ctx_create({device}) failed: {_lib.last_error()}")
        self.device = device
        # records arrays of the last WAL replays per record dtype (pageable, page-locked),
        # reused once nothing refers to them
        self._wal_recs = {}
        self._wal_pinned = {}

    def _wal_recs_buffer(self, cap, dtype=None):
        """An uninitialised record array (WAL_REC_DTYPE, or WAL_REC16_DTYPE) of
        at least cap entries: the last replay's array again when no result
        refers to it any more (its pages are already mapped: a fresh worst-case
        n/9-entry array cost ~1 ms per 0.24 GB replay in allocation,
        first-touch faults and unmapping), else a new one."""
        dtype = WAL_REC_DTYPE if dtype is None else dtype
        buf = self._wal_recs.get(dtype.str)
        # references: the dict's, `buf`, getrefcount's argument -- any more is
        # a returned view still alive
        if buf is not None and len(buf) >= cap and sys.getrefcount(buf) <= 3:
            return buf
        buf = np.empty(cap, dtype=dtype)  # uninitialised: no zeroing of every slot
        self._wal_recs[dtype.str] = buf
        return buf

    def _wal_recs_pinned(self, cap, dtype=None):
        """A page-locked record array of at least cap entries (grow-only,
        reused once no result refers to it): the replay DMAs the records into it
        (LSMCK_RECS_PINNED).  The array's base is a holder of its PinnedBuffer,
        so the pinned memory lives as long as any view of it."""
        dtype = WAL_REC_DTYPE if dtype is None else dtype
        arr = self._wal_pinned.get(dtype.str)
        if arr is not None and len(arr) >= cap and sys.getrefcount(arr) <= 3:
            return arr
        arr = np.asarray(_PinnedRecords(PinnedBuffer(self, max(1, cap) * dtype.itemsize), max(1, cap), dtype))
        self._wal_pinned[dtype.str] = arr
        return arr

    def close(self):
        self._wal_pinned = {}
        if self.handle:
            self.lib.lsmck_ctx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, key, value):
        _lib.check(self.lib.lsmck_ctx_set_option(self.handle, key.encode(), int(value)), f"set_option({key})")

    def get_stat(self, key):
        v = C.c_long()
        _lib.check(self.lib.lsmck_ctx_get_stat(self.handle, key.encode(), C.byref(v)), f"get_stat({key})")
        return v.value

    # --- memory -------------------------------------------------------------
    def alloc(self, nbytes):
        return DeviceBuffer(self, nbytes)

    def alloc_pinned(self, nbytes):
        return PinnedBuffer(self, nbytes)

    def memcpy_d2h(self, dst_ptr, src_ptr, nbytes, stream=None):
        _lib.check(self.lib.lsmck_memcpy_d2h(self.handle, dst_ptr, src_ptr, nbytes, stream), "d2h")

    def sync(self, stream=None):
        _lib.check(self.lib.lsmck_stream_sync(self.handle, stream), "sync")

    def memset(self, ptr, value, nbytes, stream=None):
        _lib.check(self.lib.lsmck_memset_dev(self.handle, ptr, value, nbytes, stream), "memset")

    def gen_stream(self, dst_ptr, seed, byte_off, nbytes, stream=None):
        _lib.check(self.lib.lsmck_gen_stream(self.handle, dst_ptr, seed, byte_off, nbytes, stream), "gen_stream")

    # --- CRC-32, host arrays ------------------------------------------------
    def crc32(self, data, off, length, pinned=False):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        n = len(off)
        out = np.empty(n, dtype=np.uint32)
        flags = _lib.HOST_PINNED if pinned else _lib.HOST
        _lib.check(self.lib.lsmck_crc32_batch(self.handle, data.ctypes.data, off.ctypes.data, length.ctypes.data, n,
                                              out.ctypes.data, flags, None), "crc32_batch")
        return out

    def crc32_fixed(self, data, stride, length, n, pinned=False):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        out = np.empty(n, dtype=np.uint32)
        flags = _lib.HOST_PINNED if pinned else _lib.HOST
        _lib.check(self.lib.lsmck_crc32_batch_fixed(self.handle, data.ctypes.data, stride, length, n, out.ctypes.data,
                                                    flags, None), "crc32_batch_fixed")
        return out

    def crc32_verify(self, data, off, length, expected):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        expected = np.ascontiguousarray(expected, dtype=np.uint32)
        nb, fb = C.c_uint64(), C.c_uint64()
        rc = _lib.check(self.lib.lsmck_crc32_verify_batch(self.handle, data.ctypes.data, off.ctypes.data,
                                                          length.ctypes.data, expected.ctypes.data, len(off),
                                                          _lib.HOST, None, C.byref(nb), C.byref(fb)), "verify")
        return rc, nb.value, fb.value

    # --- CRC-32, device pointers (async on stream) ----------------------------
    def crc32_device(self, base, off, length, n, out, stream=None, sorted_span=False):
        """sorted_span: LSMCK_SORTED, the caller asserts its records are sorted inside one readable span"""
        flags = _lib.DEVICE | (_lib.SORTED if sorted_span else 0)
        _lib.check(self.lib.lsmck_crc32_batch(self.handle, base, off, length, n, out, flags, stream),
                   "crc32_batch(device)")

    def crc32_fixed_device(self, base, stride, length, n, out, stream=None):
        _lib.check(self.lib.lsmck_crc32_batch_fixed(self.handle, base, stride, length, n, out, _lib.DEVICE, stream),
                   "crc32_batch_fixed(device)")

    def crc32_verify_device(self, base, off, length, expected, n, stream=None):
        nb, fb = C.c_uint64(), C.c_uint64()
        rc = _lib.check(self.lib.lsmck_crc32_verify_batch(self.handle, base, off, length, expected, n, _lib.DEVICE,
                                                          stream, C.byref(nb), C.byref(fb)), "verify(device)")
        return rc, nb.value, fb.value

    # --- SHA-256 --------------------------------------------------------------
    def sha256(self, data, off, length):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        n = len(off)
        out = np.empty((n, 32), dtype=np.uint8)
        _lib.check(self.lib.lsmck_sha256_batch(self.handle, data.ctypes.data, off.ctypes.data, length.ctypes.data, n,
                                               out.ctypes.data, _lib.HOST, None), "sha256_batch")
        return out

    def sha256_fixed(self, data, stride, length, n):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        out = np.empty((n, 32), dtype=np.uint8)
        _lib.check(self.lib.lsmck_sha256_batch_fixed(self.handle, data.ctypes.data, stride, length, n,
                                                     out.ctypes.data, _lib.HOST, None), "sha256_batch_fixed")
        return out

    def sha256_device(self, base, off, length, n, out, stream=None):
        _lib.check(self.lib.lsmck_sha256_batch(self.handle, base, off, length, n, out, _lib.DEVICE, stream),
                   "sha256_batch(device)")

    def sha256_fixed_device(self, base, stride, length, n, out, stream=None):
        _lib.check(self.lib.lsmck_sha256_batch_fixed(self.handle, base, stride, length, n, out, _lib.DEVICE, stream),
                   "sha256_batch_fixed(device)")

    # --- WAL / SSTable batch verify ---------------------------------------------
    def wal_frame_insert_device(self, img_ptr, off_ptr, len_ptr, crc_ptr, n, kmax=16, stream=None):
        """lsmck_wal_frame_insert_device: Insert headers in front of n payloads
        of a device-resident log (all device pointers)."""
        _lib.check(self.lib.lsmck_wal_frame_insert_device(self.handle, img_ptr, off_ptr, len_ptr, crc_ptr, n, kmax,
                                                           stream), "wal_frame_insert_device")

    def wal_replay_verify(self, image, device_ptr=None, cap=None, pinned_recs=False, compact=False):
        """Returns (records, status, (bad_index, bad_crc, bad_expected)).
        cap: records to return at most (default: the n/9 + 1 a log of n
        bytes can hold; a very large log whose record count is known can ask
        for fewer -- the status and the count cover the whole log).
        pinned_recs: the records land in a page-locked array by DMA
        (LSMCK_RECS_PINNED; cap entries stay pinned for the context's life).
        compact: 16-byte records (lsmck_wal_replay_verify16, WAL_REC16_DTYPE;
        decode_rec16 gives the 32-byte form's fields)."""
        if device_ptr is None:
            # any buffer (bytes, bytearray, memoryview, a read-only mmap of the
            # log file) is read in place: no copy of the image
            img = np.frombuffer(image, dtype=np.uint8) if len(image) else np.zeros(1, dtype=np.uint8)[:0]
            ptr, n, flags = img.ctypes.data, len(img), _lib.HOST
        else:
            ptr, n, flags = device_ptr, image, _lib.DEVICE
        cap = n // 9 + 1 if cap is None else cap  # a record is at least 9 bytes (Remove of an empty key)
        dtype = WAL_REC16_DTYPE if compact else WAL_REC_DTYPE
        if pinned_recs:
            recs = self._wal_recs_pinned(cap, dtype)
            flags |= _lib.RECS_PINNED
        else:
            recs = self._wal_recs_buffer(cap, dtype)
        nrec = C.c_size_t()
        bi, bc, be = C.c_uint64(), C.c_uint32(), C.c_uint32()
        fn = self.lib.lsmck_wal_replay_verify16 if compact else self.lib.lsmck_wal_replay_verify
        rc = _lib.check(fn(self.handle, ptr, n, flags, recs.ctypes.data, cap, C.byref(nrec), C.byref(bi),
                           C.byref(bc), C.byref(be)), "wal_replay_verify")
        # np.recarray: record fields read as attributes (r.payload_off), like the ctypes struct
        # nrec counts the whole log's accepted records; at most cap of them were written
        return recs[:min(nrec.value, cap)].view(np.recarray), rc, (bi.value, bc.value, be.value)

    def wal_replay_verify_to_device(self, image, recs_ptr, cap, device_ptr=None, compact=False):
        """The replay with its records left in device memory (LSMCK_RECS_DEVICE):
        recs_ptr is a device array of cap lsmck_wal_rec entries (32 bytes each,
        WAL_REC_DTYPE; compact: lsmck_wal_rec16, 16 bytes, WAL_REC16_DTYPE).
        Returns (nrec, status, (bad_index, bad_crc, bad_expected)); min(nrec, cap)
        records were written."""
        if device_ptr is None:
            img = np.frombuffer(image, dtype=np.uint8) if len(image) else np.zeros(1, dtype=np.uint8)[:0]
            ptr, n, flags = img.ctypes.data, len(img), _lib.HOST
        else:
            ptr, n, flags = device_ptr, image, _lib.DEVICE
        nrec = C.c_size_t()
        bi, bc, be = C.c_uint64(), C.c_uint32(), C.c_uint32()
        fn = self.lib.lsmck_wal_replay_verify16 if compact else self.lib.lsmck_wal_replay_verify
        rc = _lib.check(fn(self.handle, ptr, n, flags | _lib.RECS_DEVICE, recs_ptr, cap, C.byref(nrec), C.byref(bi),
                           C.byref(bc), C.byref(be)), "wal_replay_verify")
        return nrec.value, rc, (bi.value, bc.value, be.value)

    def checksums_verify_many(self, triples):
        n = len(triples)
        arr = C.c_char_p * max(n, 1)
        d = arr(*[str(t[0]).encode() for t in triples])
        i = arr(*[str(t[1]).encode() for t in triples])
        c = arr(*[str(t[2]).encode() for t in triples])
        status = (C.c_int * max(n, 1))()
        _lib.check(self.lib.lsmck_checksums_verify_many(self.handle, d, i, c, n, status), "checksums_verify_many")
        return list(status[:n])

    def tree_verify(self, base, listed=None):
        """lsmck_tree_verify: Db::load's table scan + batch verify of the tree
        under ``base``.  Returns a dict of the report (first_* describe the
        first failing table in load order, or are None).  ``listed``: a list
        that receives the verify's listing (lsmck_tree_verify_listed), one
        dict per table in load order, before the tables are hashed."""
        rep = _lib.TreeReport()
        if listed is None:
            rc = self.lib.lsmck_tree_verify(self.handle, str(base).encode(), C.byref(rep))
        else:
            def on_listed(_user, e, n):
                for i in range(n):
                    t = e[i]
                    dec = lambda b: b.decode(errors="surrogateescape") if b is not None else None  # noqa: E731
                    listed.append({"metadata_path": dec(t.metadata_path), "data_path": dec(t.data_path),
                                   "index_path": dec(t.index_path), "checksum_path": dec(t.checksum_path),
                                   "id": dec(t.id), "level": t.level, "status": t.status})
            fn = _lib.LISTED_FN(on_listed)
            rc = self.lib.lsmck_tree_verify_listed(self.handle, str(base).encode(), C.byref(rep), fn, None)
        return _tree_report(rep, _lib.check(rc, "tree_verify"))


def _tree_report(rep, rc):
    """lsmck_tree_report as a dict (first_* are None when every table verified)."""
    bad = rc != 0
    return {"tables": rep.tables, "table_bytes": rep.table_bytes, "bad_tables": rep.bad_tables,
            "first_index": rep.first_index if bad else None, "first_status": rep.first_status if bad else None,
            "first_metadata_path": rep.first_metadata_path.decode(errors="surrogateescape") if bad else None,
            "list_seconds": rep.list_seconds, "verify_seconds": rep.verify_seconds,
            "stat_seconds": rep.stat_seconds, "read_seconds": rep.read_seconds,
            "gpu_wait_seconds": rep.gpu_wait_seconds, "compare_seconds": rep.compare_seconds,
            "rounds": rep.rounds, "fds_cached": rep.fds_cached}


def _path_arrays(triples):
    n = len(triples)
    arr = C.c_char_p * max(n, 1)
    return (arr(*[str(t[0]).encode() for t in triples]), arr(*[str(t[1]).encode() for t in triples]),
            arr(*[str(t[2]).encode() for t in triples]))


class MultiContext:
    """Host-resident batches split over several GPUs in one process (SURVEY
    8e): one Context per device, one host thread each (the ctypes calls drop
    the GIL), contiguous record ranges -- by bytes for variable-length records
    (shard.shard_by_bytes), by count for fixed ones -- and no data exchange
    between devices: each device's results land in its slice of the output.
    Each device's host path streams its share through its own pinned slots,
    so the PCIe links of the devices work in parallel."""

    def __init__(self, devices=None, contexts=None):
        if contexts is None:
            devices = range(device_count()) if devices is None else devices
            contexts = [Context(d) for d in devices]
        if not contexts:
            raise _lib.LsmckError(_lib.ENODEV, "MultiContext: no device")
        self.ctxs = list(contexts)

    def _parallel(self, bounds, fn):
        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(len(self.ctxs)) as ex:
            for f in [ex.submit(fn, k, int(bounds[k]), int(bounds[k + 1])) for k in range(len(self.ctxs))]:
                f.result()

    def _var(self, data, off, length, width, call):
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        out = np.empty((len(off), width) if width > 1 else len(off), dtype=np.uint8 if width > 1 else np.uint32)
        b = shard_by_bytes(length, len(self.ctxs))

        def part(k, r0, r1):
            if r1 > r0:
                out[r0:r1] = call(self.ctxs[k], data, off[r0:r1], length[r0:r1])
        self._parallel(b, part)
        return out

    def _fixed(self, data, stride, length, n, width, call):
        out = np.empty((n, width) if width > 1 else n, dtype=np.uint8 if width > 1 else np.uint32)
        b = [shard_fixed(n, len(self.ctxs), k)[0] for k in range(len(self.ctxs))] + [n]
        data = np.ascontiguousarray(data, dtype=np.uint8)

        def part(k, r0, r1):
            if r1 > r0:
                out[r0:r1] = call(self.ctxs[k], data[r0 * stride:], stride, length, r1 - r0)
        self._parallel(b, part)
        return out

    def crc32(self, data, off, length):
        return self._var(np.ascontiguousarray(data, dtype=np.uint8), off, length, 1, Context.crc32)

    def crc32_fixed(self, data, stride, length, n):
        return self._fixed(data, stride, length, n, 1, Context.crc32_fixed)

    def sha256(self, data, off, length):
        return self._var(np.ascontiguousarray(data, dtype=np.uint8), off, length, 32, Context.sha256)

    def sha256_fixed(self, data, stride, length, n):
        return self._fixed(data, stride, length, n, 32, Context.sha256_fixed)

    # --- SSTable verify over every device's PCIe link (lsmck_*_multi) ---------
    def _handles(self):
        return (C.c_void_p * len(self.ctxs))(*[c.handle for c in self.ctxs])

    def checksums_verify_many(self, triples):
        n = len(triples)
        d, i, c = _path_arrays(triples)
        status = (C.c_int * max(n, 1))()
        lib = _lib.load()
        _lib.check(lib.lsmck_checksums_verify_many_multi(self._handles(), len(self.ctxs), d, i, c, n, status),
                   "checksums_verify_many_multi")
        return list(status[:n])

    def tree_verify(self, base):
        rep = _lib.TreeReport()
        lib = _lib.load()
        rc = _lib.check(lib.lsmck_tree_verify_multi(self._handles(), len(self.ctxs), str(base).encode(),
                                                    C.byref(rep)), "tree_verify_multi")
        return _tree_report(rep, rc)

    def wal_replay_verify(self, image, device_ptr=None, cap=None, pinned_recs=False, compact=False):
        """The WAL is one log: replayed on the first device (Context.wal_replay_verify)."""
        return self.ctxs[0].wal_replay_verify(image, device_ptr, cap=cap, pinned_recs=pinned_recs, compact=compact)


# include/lsmck.h lsmck_wal_rec (32 bytes, no padding)
WAL_REC_DTYPE = np.dtype([("rec_off", "<u8"), ("payload_off", "<u8"), ("klen", "<u4"), ("vlen", "<u4"),
                          ("crc", "<u4"), ("type", "<u4")])
assert WAL_REC_DTYPE.itemsize == C.sizeof(_lib.WalRec)
# include/lsmck.h lsmck_wal_rec16 (16 bytes): lsmck_wal_replay_verify16's compact records
WAL_REC16_DTYPE = np.dtype([("payload_type", "<u8"), ("klen", "<u4"), ("vlen", "<u4")])
assert WAL_REC16_DTYPE.itemsize == C.sizeof(_lib.WalRec16)


def decode_rec16(recs):
    """Compact records as the 32-byte form's fields: a dict of arrays rec_off,
    payload_off, klen, vlen, type (the stored CRC is not kept: it is the
    computed one for every accepted record)."""
    pt = np.asarray(recs["payload_type"], dtype=np.uint64)
    remove = (pt >> np.uint64(63)).astype(bool)
    payload = pt & np.uint64(_lib.WAL_REC16_REMOVE - 1)
    typ = np.where(remove, 2, 1).astype(np.uint32)
    return {"rec_off": payload - np.where(remove, 9, 13).astype(np.uint64), "payload_off": payload,
            "klen": np.asarray(recs["klen"]), "vlen": np.asarray(recs["vlen"]), "type": typ}


def device_count():
    return _lib.load().lsmck_device_count()


def gen_zipf_lengths(seed, n, s=1.5, kmax=1024, lmin=64, first=0):
    """lengths of records [first, first + n) of the config-3 length stream"""
    out = np.empty(n, dtype=np.uint32)
    _lib.load().lsmck_gen_zipf_lengths_at(seed, s, kmax, lmin, first, n, out.ctypes.data)
    return out
