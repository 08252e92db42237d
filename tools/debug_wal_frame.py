"""Debug: config-3w framing + device replay at a given record count."""
import sys, zlib, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lsm_storage_engine_amd.device import Context, gen_zipf_lengths

n = int(sys.argv[1])
part = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ctx = Context(0)
ln = gen_zipf_lengths(0x5EED0003, n)
off = np.full(n, 13, dtype=np.uint64)
off[1:] += ln[:-1].astype(np.uint64)
off = np.cumsum(off, dtype=np.uint64)
total = int(off[-1]) + int(ln[-1])
print("n", n, "total", total, "off[:3]", off[:3], "ln[:3]", ln[:3], flush=True)
d = ctx.alloc(total + 64)
d_o, d_l, out = ctx.alloc(off.nbytes), ctx.alloc(ln.nbytes), ctx.alloc(4 * n)
ctx.gen_stream(d.ptr, 0x5EED0003, 0, total)
d_o.upload(off)
d_l.upload(ln)
ctx.crc32_device(d.ptr, d_o.ptr, d_l.ptr, n, out.ptr)
ctx.sync()
crc = out.download(np.uint32)
print("crc[:3]", [hex(x) for x in crc[:3]], flush=True)
ctx.wal_frame_insert_device(d.ptr, d_o.ptr, d_l.ptr, out.ptr, n, 16)
ctx.sync()
head = d.download(np.uint8, count=int(off[1]) + 16)
print("hdr0", head[:13].tobytes().hex(), "hdr1", head[int(off[1]) - 13:int(off[1])].tobytes().hex(), flush=True)
if part:
    ctx.set_option("wal_part_bytes", part)
recs, st, bad = ctx.wal_replay_verify(total, device_ptr=d.ptr, cap=n)
print("status", st, "bad", bad, "nrec", len(recs), flush=True)
if len(recs):
    print("rec0", recs[0], flush=True)
