"""Wrong-guess repairs of the segment walk on the host model (tools/segwalk_sim.cpp),
the shipped rules against the later-start rule at every segment size: logs like
tools/wal_diag.py's, binary-payload logs, Zipf config-3-like records; segments
of 512 B to 64 KiB.  Builds both models with g++ into /tmp.
  python3 tools/segwalk_repairs.py"""
import ctypes as C, os, subprocess, sys, struct, zlib
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CSRC = os.path.join(ROOT, "lsm_storage_engine_amd", "csrc")
for so, extra in (("/tmp/segwalk_sim_shipped.so", []), ("/tmp/segwalk_sim_later.so", ["-DLSMCK_DIAG", "-DLSMCK_SEG_LATER_ALWAYS"])):
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I", CSRC, *extra, "-o", so,
                    os.path.join(ROOT, "tools", "segwalk_sim.cpp")], check=True)
from oracle import oracle as O
u64p = C.POINTER(C.c_uint64)
def load(path):
    lib = C.CDLL(path)
    lib.segwalk_sim.restype = C.c_int
    lib.segwalk_sim.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, u64p, C.c_size_t, u64p,
                                C.POINTER(C.c_uint32), u64p, C.POINTER(C.c_int), u64p, C.POINTER(C.c_uint32)]
    return lib
libs = {"skip": load("/tmp/segwalk_sim_shipped.so"), "c2": load("/tmp/segwalk_sim_later.so")}
def run(lib, img, S):
    a = np.frombuffer(img, np.uint8)
    cap = 4
    offs = (C.c_uint64 * cap)()
    m, code, pos, rep, K, nf = C.c_uint64(), C.c_uint32(), C.c_uint64(), C.c_int(), C.c_uint64(), C.c_uint32()
    rc = lib.segwalk_sim(a.ctypes.data, len(img), 0, S, 1 << 20, offs, cap, C.byref(m), C.byref(code), C.byref(pos), C.byref(rep), C.byref(K), C.byref(nf))
    return rc, rep.value, nf.value, K.value
def wal_diag_like(n, seed):
    rng = np.random.default_rng(seed); pool = rng.bytes(1 << 20)
    kl = rng.integers(1, 40, size=n); vl = rng.integers(0, 1000, size=n); rm = rng.random(n) < 0.1
    out = bytearray()
    for i in range(n):
        o = (i * 7919) % ((1 << 20) - 1100)
        key = pool[o:o + int(kl[i])]
        d = key if rm[i] else key + pool[o + 40:o + 40 + int(vl[i])]
        out += (struct.pack("<BII", 2, zlib.crc32(d), len(key)) if rm[i] else struct.pack("<BIII", 1, zlib.crc32(d), len(key), int(vl[i]))) + d
    return bytes(out)
def binary_like(n, seed, hi=600):
    rng = np.random.default_rng(seed); blob = O.gen_stream(seed, 0, 1 << 21)
    parts = []
    for i in range(n):
        kl = int(rng.integers(1, 40)); vl = int(rng.integers(0, hi))
        o = int(rng.integers(0, (1 << 21) - 40 - vl))
        k = blob[o:o + kl].tobytes(); v = blob[o + 40:o + 40 + vl].tobytes()
        parts.append(O.wal_remove(k) if i % 9 == 0 else O.wal_insert(k, v))
    return b"".join(parts)
def zipf_like(n, seed):
    from lsm_storage_engine_amd.device import gen_zipf_lengths
    ln = gen_zipf_lengths(seed, n); blob = O.gen_stream(seed, 0, int(ln.sum()))
    out = bytearray(); p = 0
    for L in ln:
        L = int(L); d = blob[p:p+L].tobytes(); p += L
        k = min(L, 16)
        out += struct.pack("<BIII", 1, zlib.crc32(d), k, L - k) + d
    return bytes(out)
logs = {"wal_diag 500k": wal_diag_like(500000, 5), "binary 60k": binary_like(60000, 61), "binary 60k s2": binary_like(60000, 99)}
try:
    logs["zipf 200k"] = zipf_like(200000, 3)
except Exception as e:
    print("zipf skipped", e)
for name, img in logs.items():
    for S in (512, 4096, 8192, 65536):
        res = {k: run(l, img, S) for k, l in libs.items()}
        print(f"{name:14s} {len(img)/1e6:7.1f} MB S={S:6d} K={res['skip'][3]:7d} repairs skip={res['skip'][1]:3d} (first-round fails {res['skip'][2]:4d}) c2={res['c2'][1]:3d} ({res['c2'][2]:4d}) rc={res['skip'][0]},{res['c2'][0]}", flush=True)
