// lsmck_crc32.hip -- batched CRC-32/ISO-HDLC ("checksum_ieee") for gfx950 (MI355X).
//
// Replaces, in bulk, the per-record `crc::crc32::checksum_ieee(&[u8]) -> u32`
// that the reference calls on every WAL record (src/wal.rs:135,153 on replay,
// :177,187 on append).  Bit-exact with crc 1.x: reflected poly 0xEDB88320,
// init 0xFFFFFFFF, xorout 0xFFFFFFFF.
//
// Design (DESIGN.md section 3 has the derivation and the measurements behind it):
//   * Every record is cut into 128-byte SEGMENTS aligned to the record's END;
//     only the record's first segment can be short, and it is front-padded with
//     zeros (leading zeros do not change a CRC whose register starts at 0).
//   * One lane owns one segment and streams it from HBM itself: lane-contiguous
//     128-B segments measured 6.42 TB/s on MI355X (tools/microbench.hip), better
//     than the wave-coalesced 16 B/lane pattern.  Loads are dword-aligned
//     dwordx4 (byte-misaligned vector loads measured 3x slower) and a
//     v_alignbyte funnel produces the byte stream; loads never touch a dword
//     that does not intersect the record (no over-read past either end).
//   * The lane runs a raw (init 0) slicing-by-4 CRC over its 32 words.  The four
//     256-entry tables live in LDS replicated 32x so that lane l only ever reads
//     bank l%32: conflict-free random lookups (17 lookups/clk/CU measured vs
//     9.8 for plain tables); the LDS byte address of entry e is
//     256*e + 4*(lane%32) (+128, +64 KiB for the other tables), formed by ONE
//     v_perm_b32 from the state word and a per-lane constant.
//   * Segment results are combined with the CRC combination law
//        raw(A||B) = raw(A) (x) x^(8|B|)  xor  raw(B)   (GF(2)[x] mod P)
//     Each lane multiplies by x^(8*128*k) (k = segments after it; table in HBM,
//     L2-resident), the record's first segment also folds in the init term
//     0xFFFFFFFF (x) x^(8*len0), and a segmented XOR across the wave's lanes
//     collects each record at its first lane.  Records entirely inside one
//     wave tile are stored directly; records spanning tiles XOR their partial
//     results into a zeroed output with atomics (XOR is order independent, so
//     the result is deterministic).
//   * Persistent grid: one 1024-thread workgroup per CU (the 128 KiB of tables
//     are built once per CU), 16 waves per CU, each wave walks 64-segment tiles.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsmck_device.h"

namespace lsmck {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define LDS_TABLE_BYTES 131072u  // slicing-by-4 tables, 32x bank-replicated
#define LDS_SHIFT_OFF 131072u    // chain-combine tables: shift by 32, 64, 96 bytes (3 x 4 x 256 x 4 B)
#define LDS_SHIFT_BYTES 12288u
#define LDS_COLS_OFF (LDS_SHIFT_OFF + LDS_SHIFT_BYTES)  // fixed records: per-lane columns of x^(8*128*k)
#define LDS_COLS_BYTES 8192u                               // [32/4][64 lanes][4] u32
#define LDS_KHI_OFF (LDS_COLS_OFF + LDS_COLS_BYTES)  // khi[0..511]: x^(8*128*65536*j), j = k >> 16 (len < 2^32)
#define LDS_KHI_BYTES 2048u
// per-segment factor K = x^(8*128*k) = klo[k & 511] (x) kmid[(k >> 9) & 127] (x) khi[k >> 16],
// and the init terms tinit[len0]: all from LDS, so the issue path gathers no tables
#define LDS_KLO_OFF (LDS_KHI_OFF + LDS_KHI_BYTES)
#define LDS_KMID_OFF (LDS_KLO_OFF + 2048u)
#define LDS_TINIT_OFF (LDS_KMID_OFF + 512u)
#define LDS_SCRATCH_OFF (LDS_TINIT_OFF + 544u)
#define WAVE_SCRATCH_BYTES 256u
// ring kernel, ORDER 4: each wave's CRCs of 16 tiles (<= 4 records per tile)
// gathered in LDS behind the kernel's tables, then stored by one instruction
#define LDS_WOUT_OFF LDS_SCRATCH_OFF
#define LDS_WOUT_BYTES 4096u
// stream kernel, LM: per wave 64 chunks x {first, second} boundary byte + 1
// (0 = none), written by the window lanes, read and cleared by the chunk lanes
#define LDS_SMAP_OFF LDS_SCRATCH_OFF
#define LDS_SMAP_BYTES 2048u
#ifndef LSMCK_DEFAULT_CHAINS
#define LSMCK_DEFAULT_CHAINS 2       // fixed records (A/B: profiles/r01)
#endif
#ifndef LSMCK_DEFAULT_BUFLOADS
#define LSMCK_DEFAULT_BUFLOADS 1     // fixed records: raw buffer loads (A/B: profiles/r01)
#endif
#ifndef LSMCK_DEFAULT_RING
#define LSMCK_DEFAULT_RING 2         // fixed percol records: whole-tile ring slots (1 = two-slot kernel; A/B: profiles/r01)
#endif
#ifndef LSMCK_DEFAULT_DESC_CHAINS
#define LSMCK_DEFAULT_DESC_CHAINS 2  // descriptor records (A/B: profiles/r01)
#endif

// ---------------------------------------------------------------------------
// GF(2) polynomial product modulo the reflected CRC-32 polynomial.
// Same function as zlib's multmodp; branch-free, 32 steps.
__device__ __forceinline__ uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    uint32_t m = (uint32_t)((int32_t)(a << i) >> 31);
    p ^= b & m;
    b = (b >> 1) ^ (0xEDB88320u & (0u - (b & 1u)));
  }
  return p;
}

// x^(8*128*k) mod P for any 32-bit k, from two 64 Ki-entry tables.
__device__ __forceinline__ uint32_t seg_shift_factor(const uint32_t* __restrict__ kseg,
                                                     const uint32_t* __restrict__ khi, uint32_t k) {
  uint32_t f = kseg[k & 0xFFFFu];
  if (k >> 16) f = gf2_mulmod(f, khi[k >> 16]);
  return f;
}

// The kernels declare no static LDS, so the dynamic region starts at LDS
// address 0: index an address_space(3) pointer directly (indexing smem + a
// costs a v_add of the relocated base per lookup).
typedef __attribute__((address_space(3))) const uint32_t lds_u32_t;
typedef __attribute__((address_space(3))) const u32x4 lds_u32x4_t;
__device__ __forceinline__ uint32_t lds_ld(const unsigned char* smem, uint32_t a) {
  (void)smem;
  return *(lds_u32_t*)(size_t)a;
}
__device__ __forceinline__ u32x4 lds_ld128(uint32_t a) { return *(lds_u32x4_t*)(size_t)a; }

// ---------------------------------------------------------------------------
// LDS tables.  Byte address of T_t[e], replica r:
//   256*e + 4*r + 128*(t&1) + 65536*(t>>1)
// T0 = Sarwate table, T_k[n] = (T_{k-1}[n] >> 8) ^ T0[T_{k-1}[n] & 0xFF].
__device__ __forceinline__ void build_lds_tables(unsigned char* smem, const CrcParams& P) {
  const uint32_t* __restrict__ master = P.master;
  uint32_t* s32 = (uint32_t*)smem;
  for (uint32_t i = threadIdx.x; i < LDS_TABLE_BYTES / 4; i += blockDim.x) {
    uint32_t t = ((i >> 14) << 1) | ((i >> 5) & 1u);
    uint32_t e = (i >> 6) & 255u;
    s32[i] = master[t * 256u + e];
  }
  // shift tables ST_m[j][b] = (b << 8j) (x) x^(8*32m) mod P, m = 1..3, plain layout
  for (uint32_t i = threadIdx.x; i < LDS_SHIFT_BYTES / 4; i += blockDim.x) s32[LDS_SHIFT_OFF / 4 + i] = master[1024u + i];
  // segment factors of records over 2^16 segments (8 MiB): from LDS, so the
  // checksum loop issues no global load of its own (its waits would also
  // wait for the next tile's prefetch)
  for (uint32_t i = threadIdx.x; i < LDS_KHI_BYTES / 4; i += blockDim.x) s32[LDS_KHI_OFF / 4 + i] = P.khi[i];
  for (uint32_t i = threadIdx.x; i < 512u; i += blockDim.x) s32[LDS_KLO_OFF / 4 + i] = P.kseg[i];
  for (uint32_t i = threadIdx.x; i < 128u; i += blockDim.x) s32[LDS_KMID_OFF / 4 + i] = P.kseg[512u * i];
  for (uint32_t i = threadIdx.x; i < 130u; i += blockDim.x) s32[LDS_TINIT_OFF / 4 + i] = P.tinit[i];
}

// raw CRC register s advanced over 32*m zero bytes (m = 1..3): 4 plain-table lookups
template <int M>
__device__ __forceinline__ uint32_t shift_bytes32(const unsigned char* smem, uint32_t s) {
  constexpr uint32_t base = LDS_SHIFT_OFF + (M - 1) * 4096u;
  return lds_ld(smem, base + ((s & 0xFFu) << 2)) ^ lds_ld(smem, base + 1024u + (((s >> 8) & 0xFFu) << 2)) ^
         lds_ld(smem, base + 2048u + (((s >> 16) & 0xFFu) << 2)) ^ lds_ld(smem, base + 3072u + ((s >> 24) << 2));
}


// One slicing-by-4 step of the raw CRC register: s' = F(s ^ w).
// lo = lane4, hi = lane4 | 0x10000 (region of T2/T3).
__device__ __forceinline__ uint32_t crc_word(const unsigned char* smem, uint32_t s, uint32_t w, uint32_t lo,
                                             uint32_t hi) {
  uint32_t x = s ^ w;
  uint32_t a0 = __builtin_amdgcn_perm(x, hi, 0x0c020400u);  // byte0 -> T3
  uint32_t a1 = __builtin_amdgcn_perm(x, hi, 0x0c020500u);  // byte1 -> T2
  uint32_t a2 = __builtin_amdgcn_perm(x, lo, 0x0c0c0600u);  // byte2 -> T1
  uint32_t a3 = __builtin_amdgcn_perm(x, lo, 0x0c0c0700u);  // byte3 -> T0
  return lds_ld(smem, a0 + 128u) ^ lds_ld(smem, a1) ^ lds_ld(smem, a2 + 128u) ^ lds_ld(smem, a3);
}

// The same step on x = s ^ w already formed, folding in the NEXT word:
// returns F(x) ^ w_next, the next step's x, as two v_bitop3_b32 (xor3) --
// instead of three v_xor for F and one for the next s ^ w.
__device__ __forceinline__ uint32_t crc_step_x(const unsigned char* smem, uint32_t x, uint32_t w_next, uint32_t lo,
                                               uint32_t hi) {
  uint32_t a0 = __builtin_amdgcn_perm(x, hi, 0x0c020400u);  // byte0 -> T3
  uint32_t a1 = __builtin_amdgcn_perm(x, hi, 0x0c020500u);  // byte1 -> T2
  uint32_t a2 = __builtin_amdgcn_perm(x, lo, 0x0c0c0600u);  // byte2 -> T1
  uint32_t a3 = __builtin_amdgcn_perm(x, lo, 0x0c0c0700u);  // byte3 -> T0
  const uint32_t l2 = lds_ld(smem, a2 + 128u), l3 = lds_ld(smem, a3);
  const uint32_t t = __builtin_amdgcn_bitop3_b32(l2, l3, w_next, 0x96);
  return __builtin_amdgcn_bitop3_b32(lds_ld(smem, a0 + 128u), lds_ld(smem, a1), t, 0x96);
}

// ---------------------------------------------------------------------------
// Segment loading.
//
// A segment's byte stream is the 128 bytes [E-128, E) (absolute addresses),
// of which only [B, E) are record bytes (B = E-128 except for a record's short
// first segment).  Dwords D_i live at base4 + 4i, base4 = floor4(E-128),
// i = 0..32; stream word j = alignbyte(D_{j+1}, D_j, (E-128)&3).
// Dword i is loaded only if it intersects [B, E): i >= lo_i, and D_32 only if
// (E-128) is not dword aligned.  Nothing outside the record's dwords is read.
__device__ __forceinline__ uint32_t ld32(const unsigned char* p) { return *(const uint32_t*)p; }
__device__ __forceinline__ u32x4 ld128(const unsigned char* p) { return *(const u32x4*)p; }

// Keep a load's address VGPRs live past the segment's loads.  Otherwise hipcc
// lets the last load of a segment write its data over the address register
// (e.g. `buffer_load_dwordx4 v[34:37], v34, ... offset:112`), and that form
// streams 14-20% slower on gfx950: tools/microbench_policy.hip measured 12.4
// vs 10.75 ms for 64 GB with the same addresses, and 13.0 vs 10.76 ms for
// eight per-load offsets whose registers the next tile's loads overwrite
// (profiles/r01/ablations.md, "Load instruction form").
template <typename T>
__device__ __forceinline__ void keep_live(const T& x) {
  asm volatile("" ::"v"(x));
}

struct SegInfo {
  uint32_t rec;       // record index
  uint32_t q;         // segment index from the record's front
  uint32_t k;         // segments after this one
  uint64_t rec_off;   // record offset from base
  uint32_t rec_len;
  bool valid;
};

// In-flight loads of one segment (issued one tile ahead of their use).
struct SegLoad {
  uint32_t d[33];  // dwords D_0..D_32 (D_32 only when the stream start is not dword aligned)
  // the segment's coordinates, copied at issue time (when they are resident):
  // finish needs no SegInfo, so the map of a later tile may still be in flight
  uint32_t rec, k;
  uint32_t fl;     // packed SegLoad.fl fields below
};
// FL_SH: (E-128) & 3.  FL_BST: B - floor4(E-128).  FL_VALID: lane holds a
// real segment.  FL_FIRST: q == 0.  FL_M: the load window was moved up by
// m dwords to the start of B's page (see seg_issue); seg_finish moves the
// registers back.
#define FL_SH(f) ((f) & 3u)
#define FL_BST(f) (((f) >> 2) & 0xFFu)
#define FL_VALID 0x400u
#define FL_FIRST 0x800u
#define FL_M(f) (((f) >> 12) & 0x3Fu)

// Issue every global load of a segment; consumes nothing.  FAST: full
// segment whose stream start is dword aligned (ALIGNED16: 16-byte aligned).
// Buffer resource over the 2 GiB window at `b` (wave-uniform): raw buffer
// loads take a 32-bit lane offset from one SGPR base, and hipcc issues them in
// program order (address-ascending per lane); see BUF below.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t window_rsrc(const unsigned char* b) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(b), (short)0, 0x7FFFFFFF, 0x00020000);
}

// BUF (FAST only): the eight 16-byte loads are raw buffer loads from the
// wave-uniform tile base `tbase` (offset from P.base; the host guarantees the
// tile's segments lie within 2^31 bytes of it).  tools/microbench_policy.hip:
// this load shape streams at 6.43 TB/s as buffer loads and 5.39 TB/s as
// global loads, which hipcc issues out of address order (48,32,0,16,112,...).
template <bool FAST, int ABLATE = 0, bool BUF = false>
__device__ __forceinline__ void seg_issue(const CrcParams& P, const SegInfo& si, SegLoad& L, uint64_t tbase = 0) {
  const uint64_t E = si.rec_off + si.rec_len - 128ull * si.k;  // segment end (offset from base)
  const uint32_t seglen = (si.q == 0) ? si.rec_len - 128u * si.k : 128u;
  const uint32_t lead = 128u - seglen;  // stream bytes in front of the record (first segment only)
  L.rec = si.rec;
  L.k = si.k;
  const uint32_t flv = (si.valid ? FL_VALID : 0u) | (si.q == 0 ? FL_FIRST : 0u);
  L.fl = flv;
  // pointer arithmetic on the kernel-argument pointer keeps these global_load (not flat_load)
  const unsigned char* s0 = P.base + (E - 128);
  if (ABLATE == 2 || (ABLATE >= 8 && ABLATE <= 11)) {  // diagnostic: no payload loads (compute-only timing; results invalid)
#pragma unroll
    for (int j = 0; j < 33; ++j) L.d[j] = (uint32_t)E * 0x9E3779B1u + j;
    return;
  }
  if (FAST && BUF) {
    const __amdgpu_buffer_rsrc_t r = window_rsrc(P.base + tbase);
    const uint32_t vo = (uint32_t)(E - 128 - tbase);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16u * g, 0, 0);
      L.d[4 * g + 0] = v[0];
      L.d[4 * g + 1] = v[1];
      L.d[4 * g + 2] = v[2];
      L.d[4 * g + 3] = v[3];
    }
    keep_live(vo);
    L.d[32] = 0;
    return;
  }
  if (FAST) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      u32x4 v = ld128(s0 + 16 * g);
      L.d[4 * g + 0] = v.x;
      L.d[4 * g + 1] = v.y;
      L.d[4 * g + 2] = v.z;
      L.d[4 * g + 3] = v.w;
    }
    keep_live(s0);
    L.d[32] = 0;
    return;
  }
  // General path: one base pointer per lane, eight 16-byte loads at
  // immediate offsets (per-group addresses cost ~30% of the load path:
  // crc_ablate 3 vs 6), straight-line (a divergent branch here makes hipcc
  // wait for the loads and the prefetch is lost).
  //  - window [p, p+128), p = floor4(E-128): it never passes E.  Bytes of it
  //    in front of B (first segments) are zeroed in seg_finish;
  //  - they are on B's page unless a page boundary lies in (p, B].  A page
  //    boundary is dword aligned, so it can only fall in front of B's dword,
  //    never inside the stream of a non-first segment.  Then the window starts
  //    at the boundary instead (m = 1..32 dwords higher; it ends at most 131
  //    bytes into B's page) and seg_finish shifts the registers back up;
  //  - D_32 (stream bytes only when the stream start is not dword aligned)
  //    is the dword at p+128, which holds E-1 when it is needed; otherwise a
  //    dword inside the window is loaded and ignored;
  //  - an empty segment (empty record, pad lane) reads a zero buffer.
  const uint32_t sh = (uint32_t)((uintptr_t)s0 & 3);
  const unsigned char* p = s0 - sh;  // floor4(E-128)
  const uint32_t bstart = sh + lead; // B - p
  const bool empty = lead >= 128u;
  const uintptr_t pa = (uintptr_t)p;
  const uintptr_t pg = (pa + bstart) & ~(uintptr_t)4095;  // B's page
  const bool cross = !empty & (pg > pa);
  const uint32_t m = cross ? (uint32_t)(pg - pa) >> 2 : 0u;  // 1..32
  L.fl = flv | sh | (bstart << 2) | (m << 12);
  // pointer arithmetic from the kernel-argument pointers keeps these global_load
  const unsigned char* w = empty ? (const unsigned char*)P.zero : p + 4u * m;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    u32x4 v = ld128(w + 16 * g);
    L.d[4 * g + 0] = v.x;
    L.d[4 * g + 1] = v.y;
    L.d[4 * g + 2] = v.z;
    L.d[4 * g + 3] = v.w;
  }
  if (ABLATE == 7) {  // diagnostic: no D_32 load
    L.d[32] = sh;
    return;
  }
  L.d[32] = ld32(w + ((sh != 0u && m == 0u) ? 128 : 124));
  keep_live(w);
}

// Diagnostic load form (crc_ablate 13 / 14, packed batches only: record r+1
// starts where r ends): the general form's window, zero-lane and page rules as
// raw buffer loads, in program order, from a wave-uniform tile base (lane 0's
// window start less 512 B; every later window of a packed tile starts at or
// after it) instead of per-lane 64-bit global_load pointers.  Empty lanes load
// from an out-of-range offset (zeros, no access).  The range ends 4 bytes past
// the batch's last byte, inside the last dword.
__device__ __forceinline__ void seg_issue_pk(const CrcParams& P, const SegInfo& si, SegLoad& L, uint64_t data_end) {
  const uint64_t E = si.rec_off + si.rec_len - 128ull * si.k;
  const uint32_t seglen = (si.q == 0) ? si.rec_len - 128u * si.k : 128u;
  const uint32_t lead = 128u - seglen;
  L.rec = si.rec;
  L.k = si.k;
  const uint32_t flv = (si.valid ? FL_VALID : 0u) | (si.q == 0 ? FL_FIRST : 0u);
  const uint64_t w0 = E - 128;
  const uint32_t sh = (uint32_t)(((uintptr_t)P.base + w0) & 3);
  const uint64_t pw = w0 - sh;
  const uint32_t bstart = sh + lead;
  const bool empty = lead >= 128u;
  const uintptr_t pa = (uintptr_t)P.base + pw;
  const uintptr_t pg = (pa + bstart) & ~(uintptr_t)4095;
  const bool cross = !empty & (pg > pa);
  const uint32_t m = cross ? (uint32_t)(pg - pa) >> 2 : 0u;
  L.fl = flv | sh | (bstart << 2) | (m << 12);
  const uint32_t e_lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pw);
  const uint32_t e_hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pw >> 32));
  const uint64_t tb = (((uint64_t)e_hi << 32) | e_lo) - 512u;
  const uint64_t span = data_end + 4u - tb;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(P.base + tb), (short)0, (int)(span < 0x7FFFFFFFull ? span : 0x7FFFFFFFull), 0x00020000);
  const uint32_t vo = empty ? 0x80000000u : (uint32_t)(pw + 4u * m - tb);
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16u * g, 0, 0);
    L.d[4 * g + 0] = v[0];
    L.d[4 * g + 1] = v[1];
    L.d[4 * g + 2] = v[2];
    L.d[4 * g + 3] = v[3];
  }
  L.d[32] = __builtin_amdgcn_raw_buffer_load_b32(r, vo + ((sh != 0u && m == 0u) ? 128u : 124u), 0, 0);
  keep_live(vo);
}

// Funnel, mask, raw slicing-by-4 CRC, init term, shift to the record's end.
// CHAINS independent register chains per lane (the segment's 128 bytes cut in
// CHAINS pieces) hide the LDS lookup latency; they are recombined with the
// shift-by-32m-bytes tables: raw(A||B) = shift_|B|(raw(A)) ^ raw(B).
template <bool FAST, int CHAINS, int ABLATE = 0, bool PERCOL = false, bool RAW = false>
__device__ __forceinline__ uint32_t seg_finish(const unsigned char* smem, const CrcParams& P, const SegLoad& L,
                                               uint32_t lo, uint32_t hi) {
  if (ABLATE == 1 || (ABLATE >= 3 && ABLATE <= 7) || ABLATE == 12 || ABLATE == 13) {  // diagnostic: loads only (results invalid)
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 33; ++j) x ^= L.d[j];
    return x ^ L.k ^ L.fl;
  }
  uint32_t w[32];
  if (FAST) {
#pragma unroll
    for (int j = 0; j < 32; ++j) w[j] = L.d[j];
  } else {
    uint32_t d[33];
#pragma unroll
    for (int j = 0; j < 33; ++j) d[j] = L.d[j];
    const uint32_t sh = FL_SH(L.fl), bstart = FL_BST(L.fl), lo_i = bstart >> 2;
    const uint32_t bm = 0xFFFFFFFFu << (8u * (bstart & 3u));  // keep-mask of B's dword
    const uint32_t m = FL_M(L.fl);
    if (__any(m != 0u)) {  // rare: the window started at B's page, m dwords up: shift back
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        const int s = 1 << b;
        const bool on = (m >> b) & 1u;
#pragma unroll
        for (int j = 32; j >= 0; --j) d[j] = on ? (j >= s ? d[j - s] : 0u) : d[j];
      }
    }
    if (ABLATE != 9 && __any(bstart != 0u)) {  // (9: diagnostic, compute without the masks)
      // zero the window in front of B: the groups before B's group and the
      // bytes of B's group in front of B (with lead = 0 this only clears bytes
      // of D_0 in front of the stream start, which the funnel drops anyway)
      const uint32_t r = lo_i & 3u, gb = lo_i >> 2;
      uint32_t mk[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) mk[k] = ((uint32_t)k < r) ? 0u : (((uint32_t)k == r) ? bm : 0xFFFFFFFFu);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const bool before = (uint32_t)g < gb, here = (uint32_t)g == gb;
#pragma unroll
        for (int k = 0; k < 4; ++k) d[4 * g + k] &= before ? 0u : (here ? mk[k] : 0xFFFFFFFFu);
      }
      d[32] &= (lo_i == 32u) ? bm : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int j = 0; j < 32; ++j) w[j] = ABLATE == 10 ? d[j] : __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
  }
  constexpr int WPC = 32 / CHAINS;  // words per chain
  // each chain carries x = state ^ (its next word); the state starts at 0, so
  // the first x is the first word, and the last step folds in 0
  uint32_t c[CHAINS];
#pragma unroll
  for (int h = 0; h < CHAINS; ++h) c[h] = w[h * WPC];
#pragma unroll
  for (int j = 0; j < WPC; ++j) {
#pragma unroll
    for (int h = 0; h < CHAINS; ++h) c[h] = crc_step_x(smem, c[h], j + 1 < WPC ? w[h * WPC + j + 1] : 0u, lo, hi);
  }
  uint32_t s;
  if constexpr (CHAINS == 1) {
    s = c[0];
  } else if constexpr (CHAINS == 2) {
    s = shift_bytes32<2>(smem, c[0]) ^ c[1];
  } else {
    s = shift_bytes32<3>(smem, c[0]) ^ shift_bytes32<2>(smem, c[1]) ^ shift_bytes32<1>(smem, c[2]) ^ c[3];
  }
  // init term of a record's first segment: 0xFFFFFFFF (x) x^(8*len0), len0 = 128 - lead
  const uint32_t lead0 = FL_BST(L.fl) - FL_SH(L.fl);
  s ^= (L.fl & FL_FIRST) ? lds_ld(smem, LDS_TINIT_OFF + ((128u - lead0) << 2)) : 0u;
  if constexpr (RAW) return s;  // walking kernel: shifted by the caller (Horner within the tile)
  if constexpr (PERCOL) {
    // s (x) K with the lane's 32 precomputed columns K*x^i: p ^= col_i if bit 31-i of s
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t p = 0;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      u32x4 c = lds_ld128(LDS_COLS_OFF + g * 1024u + lane * 16u);
      // p ^= col & mask as one v_bitop3_b32 (truth table 0x78: a ^ (b & c))
      p = __builtin_amdgcn_bitop3_b32(p, c.x, (uint32_t)((int32_t)(s << (4 * g + 0)) >> 31), 0x78);
      p = __builtin_amdgcn_bitop3_b32(p, c.y, (uint32_t)((int32_t)(s << (4 * g + 1)) >> 31), 0x78);
      p = __builtin_amdgcn_bitop3_b32(p, c.z, (uint32_t)((int32_t)(s << (4 * g + 2)) >> 31), 0x78);
      p = __builtin_amdgcn_bitop3_b32(p, c.w, (uint32_t)((int32_t)(s << (4 * g + 3)) >> 31), 0x78);
    }
    return p;
  }
  if (ABLATE == 8) return s;  // diagnostic: compute without the segment-factor multiply
  uint32_t K = lds_ld(smem, LDS_KLO_OFF + ((L.k & 511u) << 2));
  if (__any(L.k >= 512u)) {  // records over 64 KiB (identity factors for the other lanes)
    K = gf2_mulmod(K, lds_ld(smem, LDS_KMID_OFF + (((L.k >> 9) & 127u) << 2)));
    if (__any(L.k >= 65536u)) K = gf2_mulmod(K, lds_ld(smem, LDS_KHI_OFF + ((L.k >> 16) << 2)));
  }
  return gf2_mulmod(s, K);
}

// Per-lane columns K*x^i (i = 0..31) of the shift factor K = x^(8*128*k_lane)
// for fixed records whose segment count divides 64: every tile starts on a
// record boundary, so lane l always holds segment k = nsegr-1 - l%nsegr.
__device__ __forceinline__ void build_lds_cols(const CrcParams& P, uint32_t nsegr) {
  if (threadIdx.x >= 64) return;
  const uint32_t lane = threadIdx.x;
  uint32_t b = P.kseg[nsegr - 1u - lane % nsegr];
  uint32_t* s32 = (uint32_t*)0;
  (void)s32;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    *(__attribute__((address_space(3))) uint32_t*)(size_t)(LDS_COLS_OFF + (i >> 2) * 1024u + lane * 16u + (i & 3) * 4u) = b;
    b = (b >> 1) ^ (0xEDB88320u & (0u - (b & 1u)));
  }
}

// ---------------------------------------------------------------------------
// Segmented XOR over a wave, for record heads: XOR of lanes [lane, run_end]
// = X[run_end] ^ X[lane-1] with X the inclusive prefix XOR of the wave.  The
// prefix runs on the VALU through DPP (row_shr 1/2/4/8 inside each 16-lane
// row, then row_bcast 15/31 across rows); only the gather of X[run_end] uses
// the LDS crossbar (one ds_bpermute instead of six shuffles): the LDS pipe is
// the checksum's bottleneck, the VALU has room.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {  // lanes without a source (or masked rows) read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_prefix_xor(uint32_t x) {
  x ^= dpp0<0x111, 0xF>(x);  // row_shr:1
  x ^= dpp0<0x112, 0xF>(x);  // row_shr:2
  x ^= dpp0<0x114, 0xF>(x);  // row_shr:4
  x ^= dpp0<0x118, 0xF>(x);  // row_shr:8
  x ^= dpp0<0x142, 0xA>(x);  // row_bcast:15 -> rows 1, 3
  x ^= dpp0<0x143, 0xC>(x);  // row_bcast:31 -> rows 2, 3
  return x;
}
__device__ __forceinline__ uint32_t run_xor(uint32_t v, uint32_t run_end) {
  const uint32_t X = wave_prefix_xor(v);
  const uint32_t Xe = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(run_end << 2), (int)X);
  return Xe ^ dpp0<0x138, 0xF>(X);  // wave_shr:1 -> X[lane-1], 0 for lane 0
}

__device__ __forceinline__ void emit_record(const CrcParams& P, uint32_t v, const SegLoad& L, uint32_t lane,
                                            bool head) {
  if (!(L.fl & FL_VALID) || !head) return;
  bool has_last = (lane + L.k) <= 63u;  // this tile holds the record's final segment
  if ((L.fl & FL_FIRST) && has_last) {
    P.out[L.rec] = ~v;
  } else {
    atomicXor(&P.out[L.rec], has_last ? ~v : v);
  }
}

template <bool FAST, int CHAINS, int ABLATE = 0, bool PERCOL = false>
__device__ __forceinline__ void finish_tile(const unsigned char* smem, const CrcParams& P, const SegLoad& L,
                                            uint32_t lane, uint32_t lo, uint32_t hi) {
  uint32_t v = seg_finish<FAST, CHAINS, ABLATE, PERCOL>(smem, P, L, lo, hi);
  if ((ABLATE >= 3 && ABLATE <= 7) || ABLATE == 12 || ABLATE == 13) {  // no reduction, no store (unless a magic value: keeps the loads alive)
    if (v == 0x9E3779B1u) P.out[0] = v;
    return;
  }
  v = (L.fl & FL_VALID) ? v : 0u;
  v = run_xor(v, min(63u, lane + L.k));
  if (ABLATE == 14) {  // diagnostic: everything but the output store (results invalid)
    if (v == 0x9E3779B1u) P.out[0] = v;
    return;
  }
  if (ABLATE == 15) {  // diagnostic: the store, but every tile of a wave to the same 8 bytes (an L2 hit)
    if ((L.fl & FL_VALID) && (L.fl & FL_FIRST)) P.out[((blockIdx.x * 16u + (threadIdx.x >> 6)) * 2u + (lane >> 5)) & 1023u] = ~v;
    return;
  }
  emit_record(P, v, L, lane, lane == 0 || (L.fl & FL_FIRST));
}

// ---------------------------------------------------------------------------
// Fixed-size records: record r = [r*stride, r*stride + len).
__device__ __forceinline__ SegInfo fixed_map(const CrcParams& P, uint32_t t, uint32_t lane, uint32_t nsegr,
                                             uint32_t total) {
  uint32_t g = t * 64u + lane;
  SegInfo si;
  si.valid = g < total;
  uint32_t gg = si.valid ? g : total - 1u;
  si.rec = gg / nsegr;
  si.q = gg - si.rec * nsegr;
  si.k = nsegr - 1u - si.q;
  si.rec_off = (uint64_t)si.rec * P.stride;
  si.rec_len = P.flen;
  return si;
}

// Software pipelined: the loads of tile t+nwaves are in flight while tile t is
// checksummed (sched_barrier keeps the compiler from sinking them to their use).
// Fixed records whose segment count divides 64 (PERCOL), buffer loads: every
// tile starts on a record boundary, so a lane's byte offset from its tile's
// first record, (lane/nsegr)*stride + 128*(lane%nsegr), is the same in every
// tile.  The eight load offsets are computed once, before the loop, and kept
// in eight VGPRs (hidden from the compiler, which would otherwise fold them
// into one VGPR + immediate offsets): tools/microbench_policy.hip measured this
// load shape at 6.39 TB/s, the same loads with offset:16..112 immediates at
// 5.53 TB/s, and with the offsets recomputed per tile at 5.45 TB/s.
// Pad lanes of the last tile fall past the batch's end: the descriptor's
// range check returns zeros for them (their results are dropped).
struct PercolMap {
  uint32_t voff[8];  // lane offsets of the eight 16-byte loads
  uint32_t lsh;      // log2(nsegr)
  uint64_t tstride;  // bytes per tile (64/nsegr records)
  uint64_t end;      // bytes from P.base to the last record's end
};
__device__ __forceinline__ PercolMap percol_map(const CrcParams& P, uint32_t lane, uint32_t nsegr) {
  PercolMap M;
  M.lsh = __builtin_ctz(nsegr);
  const uint32_t lo = (uint32_t)((lane >> M.lsh) * P.stride) + 128u * (lane & (nsegr - 1u));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t o = lo + 16u * j;
    asm volatile("" : "+v"(o));
    M.voff[j] = o;
  }
  M.tstride = (uint64_t)(64u >> M.lsh) * P.stride;
  M.end = (uint64_t)(P.nrec - 1) * P.stride + P.flen;
  return M;
}
__device__ __forceinline__ void seg_issue_percol(const CrcParams& P, const PercolMap& M, uint32_t t, uint32_t lane,
                                                 uint32_t nsegr, uint32_t total, SegLoad& L) {
  const uint64_t tb = (uint64_t)t * M.tstride;
  const uint64_t left = M.end - tb;  // t < ntiles: > 0
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(P.base + tb), (short)0, (int)(left < 0x7FFFFFFFull ? left : 0x7FFFFFFFull), 0x00020000);
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, M.voff[g], 0, 0);
    L.d[4 * g + 0] = v[0];
    L.d[4 * g + 1] = v[1];
    L.d[4 * g + 2] = v[2];
    L.d[4 * g + 3] = v[3];
  }
  L.d[32] = 0;
  const uint32_t gi = t * 64u + lane;
  const uint32_t q = gi & (nsegr - 1u);
  L.rec = gi >> M.lsh;
  L.k = nsegr - 1u - q;
  L.fl = (gi < total ? FL_VALID : 0u) | (q == 0u ? FL_FIRST : 0u);
}

// wave-uniform base of tile t for buffer loads: the start of the record
// holding the tile's first segment
__device__ __forceinline__ uint64_t fixed_tile_base(const CrcParams& P, uint32_t t, uint32_t nsegr) {
  return (uint64_t)((t * 64u) / nsegr) * P.stride;
}

template <bool FAST, int CHAINS, int ABLATE = 0, bool PERCOL = false, bool BUF = false>
__global__ __launch_bounds__(1024) void crc32_fixed_kernel(CrcParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  build_lds_tables(smem, P);
  if (PERCOL) build_lds_cols(P, (P.flen + 127u) >> 7);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lo = (lane & 31u) * 4u, hi = lo | 0x10000u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);  // uniform: scalar loop control
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t nsegr = (P.flen + 127u) >> 7;
  const uint32_t total = nsegr * (uint32_t)P.nrec;  // host keeps this < 2^32 - 64
  const uint32_t ntiles = (total + 63u) >> 6;
  // ping-pong between two load slots A/B: a loaded register is never copied
  // (a copy would force s_waitcnt vmcnt(0) on the prefetch).  The loop has one
  // exit, at the bottom, with a precomputed trip count: a break between the
  // halves gives the CFG a second path into the header on which the other
  // slot's loads are still outstanding, and the wait-count merge then waits
  // for the prefetch at the top of every iteration.
  const uint32_t t0 = wave;
  if (t0 >= ntiles) return;
  const uint32_t niter = (ntiles - t0 + nwaves - 1u) / nwaves;  // tiles of this wave, >= 1
  uint32_t t = t0;
  SegLoad A, B;
  if constexpr (FAST && PERCOL && BUF) {
    const PercolMap M = percol_map(P, lane, nsegr);
    seg_issue_percol(P, M, t, lane, nsegr, total, A);
    for (uint32_t j = 2; j <= niter; j += 2) {
      seg_issue_percol(P, M, t + nwaves, lane, nsegr, total, B);
      __builtin_amdgcn_sched_barrier(0);
      finish_tile<FAST, CHAINS, ABLATE, PERCOL>(smem, P, A, lane, lo, hi);
      const uint32_t ta = (t + 2u * nwaves < ntiles) ? t + 2u * nwaves : t;  // past the end: reload, unused
      seg_issue_percol(P, M, ta, lane, nsegr, total, A);
      __builtin_amdgcn_sched_barrier(0);
      finish_tile<FAST, CHAINS, ABLATE, PERCOL>(smem, P, B, lane, lo, hi);
      t += 2u * nwaves;
    }
    if (niter & 1u) finish_tile<FAST, CHAINS, ABLATE, PERCOL>(smem, P, A, lane, lo, hi);
    return;
  }
  seg_issue<FAST, ABLATE, BUF>(P, fixed_map(P, t, lane, nsegr, total), A, fixed_tile_base(P, t, nsegr));
  for (uint32_t j = 2; j <= niter; j += 2) {
    const uint32_t tb = t + nwaves;
    seg_issue<FAST, ABLATE, BUF>(P, fixed_map(P, tb, lane, nsegr, total), B, fixed_tile_base(P, tb, nsegr));
    __builtin_amdgcn_sched_barrier(0);
    finish_tile<FAST, CHAINS, ABLATE, PERCOL>(smem, P, A, lane, lo, hi);
    const uint32_t ta = (t + 2u * nwaves < ntiles) ? t + 2u * nwaves : t;  // past the end: reload, unused
    seg_issue<FAST, ABLATE, BUF>(P, fixed_map(P, ta, lane, nsegr, total), A, fixed_tile_base(P, ta, nsegr));
    __builtin_amdgcn_sched_barrier(0);
    finish_tile<FAST, CHAINS, ABLATE, PERCOL>(smem, P, B, lane, lo, hi);
    t += 2u * nwaves;
  }
  if (niter & 1u) finish_tile<FAST, CHAINS, ABLATE, PERCOL>(smem, P, A, lane, lo, hi);
}

// ---------------------------------------------------------------------------
// Whole-tile ring: R slots of a whole segment (SegLoad), R-1 tiles in flight
// while one is checksummed (the two-slot kernel is R = 2 with eight offset
// VGPRs).  One offset VGPR per lane (the eight loads use immediate offsets,
// the register kept live past them: keep_live) so that three slots fit in the
// 128 VGPRs of a 16-wave workgroup.  The checksum is the two-slot kernel's
// finish_tile, unchanged.
__device__ __forceinline__ void issue_whole(const CrcParams& P, const PercolMap& M, uint32_t vo, uint32_t t,
                                            uint32_t lane, uint32_t nsegr, uint32_t total, SegLoad& L) {
  const uint64_t tb = (uint64_t)t * M.tstride;
  const uint64_t left = M.end - tb;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(P.base + tb), (short)0, (int)(left < 0x7FFFFFFFull ? left : 0x7FFFFFFFull), 0x00020000);
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16u * g, 0, 0);
    L.d[4 * g + 0] = v[0];
    L.d[4 * g + 1] = v[1];
    L.d[4 * g + 2] = v[2];
    L.d[4 * g + 3] = v[3];
  }
  keep_live(vo);
  L.d[32] = 0;
  const uint32_t gi = t * 64u + lane;
  const uint32_t q = gi & (nsegr - 1u);
  L.rec = gi >> M.lsh;
  L.k = nsegr - 1u - q;
  L.fl = (gi < total ? FL_VALID : 0u) | (q == 0u ? FL_FIRST : 0u);
}
// ORDER: which tiles a wave walks.  0 = strided (tile t -> wave t mod nwaves);
// 1 = one contiguous range per wave; 2 = blocks of WRING_BLOCK tiles claimed
// from an atomic counter (P.work, zeroed by the host), each walked in order.
// tools/microbench_walk.hip measured the load stream at 10.69 / 10.65 / 10.52
// ms for 64 GiB in these orders (profiles/r02/mb/mb_walk64.log).
#define WRING_BLOCK 16u
// QST (ORDER 1 only: a wave's records are consecutive): the CRCs are queued in
// one VGPR (lane p: record qb + p) and stored as whole 256-byte blocks, as in
// the stream kernel.  The per-tile store of a tile's two 4 KiB records (8
// bytes) cost 0.68 of 11.96 ms on config 2 (crc_ablate 14:
// profiles/r02/q/ab_r02c2s.log) and 0.94 GB of fetches per launch.
template <int R, int ABLATE = 0, int BLOCK = 1024, int ORDER = 0, bool QST = false>
__global__ __launch_bounds__(BLOCK) void crc32_wring_kernel(CrcParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t nsegr = P.flen >> 7;
  build_lds_tables(smem, P);
  build_lds_cols(P, nsegr);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lo = (lane & 31u) * 4u, hi = lo | 0x10000u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t total = nsegr * (uint32_t)P.nrec;
  const uint32_t ntiles = (total + 63u) >> 6;
  PercolMap M;
  M.lsh = __builtin_ctz(nsegr);
  M.tstride = (uint64_t)(64u >> M.lsh) * P.stride;
  M.end = (uint64_t)(P.nrec - 1) * P.stride + P.flen;
  const uint32_t vo = (uint32_t)((lane >> M.lsh) * P.stride) + 128u * (lane & (nsegr - 1u));
  const uint32_t m = 64u >> M.lsh;  // records per tile
  uint32_t qv = 0, qs = 0, qf = 0;
  uint64_t qb = 0;
  auto qstore = [&](bool on) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)(P.out + qb), (short)0, 256, 0x00020000);
    if (ABLATE == 14) on = on && qv == 0x9E3779B1u;  // diagnostic: no output store
    if (on) __builtin_amdgcn_raw_buffer_store_b32(qv, r, lane << 2, 0, 0);
  };
  // the tile's records (head lanes 0, nsegr, ...; cnt of them valid) onto the queue
  auto qpush = [&](uint32_t v, uint32_t cnt) {
    const uint32_t k = (lane - qf) & 63u;  // the queue lane's record within the tile
    const uint32_t val = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((k << M.lsh) & 63u) << 2), (int)v);
    const uint32_t end = qf + cnt;  // cnt <= 64: at most one block completes
    qv = (lane >= qf && lane < end) ? val : qv;
    if (end >= 64u) {
      qstore(lane >= qs);
      qb += 64u;
      qs = 0u;
      qf = end - 64u;
      qv = lane < qf ? val : qv;
    } else {
      qf = end;
    }
  };
  // walk tiles t0, t0 + step, ... (mine of them) through the R-slot ring
  auto run = [&](uint32_t t0, uint32_t mine, uint32_t step) {
    const uint32_t iters = (mine + R - 1u) / R;
    // slots past the run's last tile reload its first tile (in bounds) and are
    // marked invalid (no store)
    auto tile_of = [&](uint32_t i) -> uint32_t { return i < mine ? t0 + i * step : t0; };
    SegLoad S[R];
    // ORDER 5 / QST: the previous tile's CRCs, stored (pushed) only after the
    // next tile's loads are issued -- no work between a tile's checksum and
    // the next issue (profiles/r02/q: a store or queue push there cost
    // 1.2-1.5 ms of 12.2 on config 2, whatever its address)
    uint32_t dv = 0, drec = 0, dcnt = 0;
    bool dst = false;
#pragma unroll
    for (int k = 0; k < R - 1; ++k) {
      issue_whole(P, M, vo, tile_of(k), lane, nsegr, (k < (int)mine) ? total : 0u, S[k]);
      __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t n0 = 0;
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const uint32_t ni = n0 + k + R - 1;
        issue_whole(P, M, vo, tile_of(ni), lane, nsegr, ni < mine ? total : 0u, S[(k + R - 1) % R]);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (ORDER == 5) {
          if (dst) P.out[drec] = dv;
          uint32_t v = seg_finish<true, 2, ABLATE, true>(smem, P, S[k % R], lo, hi);
          v = (S[k % R].fl & FL_VALID) ? v : 0u;
          v = run_xor(v, min(63u, lane + S[k % R].k));
          dv = ~v;
          drec = S[k % R].rec;
          dst = (S[k % R].fl & FL_VALID) && (S[k % R].fl & FL_FIRST);  // tiles start on records: heads end in the tile
        } else if constexpr (ORDER == 4) {
          // the tile's head lanes write their CRCs to the wave's LDS rows; every
          // 16 tiles the rows go out in one store (lane l: tile l / m, record l % m)
          const uint32_t ti = n0 + k;
          uint32_t v = seg_finish<true, 2, ABLATE, true>(smem, P, S[k % R], lo, hi);
          v = (S[k % R].fl & FL_VALID) ? v : 0u;
          v = ~run_xor(v, min(63u, lane + S[k % R].k));
          const uint32_t wb = LDS_WOUT_OFF + (threadIdx.x >> 6) * 256u;
          if ((lane & (nsegr - 1u)) == 0u)
            *(__attribute__((address_space(3))) uint32_t*)(size_t)(wb + (((ti & 15u) * m + (lane >> M.lsh)) << 2)) = v;
          if (ti < mine && ((ti & 15u) == 15u || ti + 1u == mine)) {
            const uint32_t j = lane >> __builtin_ctz(m), tj = (ti & ~15u) + j;
            const uint32_t w = *(__attribute__((address_space(3))) const uint32_t*)(size_t)(wb + (lane << 2));
            const uint64_t rec = (uint64_t)(t0 + tj * step) * m + (lane & (m - 1u));
            if (lane < 16u * m && tj <= ti && rec < P.nrec) P.out[rec] = w;  // tj <= ti < mine
          }
        } else if constexpr (QST) {
          if (dcnt) qpush(dv, dcnt);
          const uint32_t ti = n0 + k;  // this slot's tile, valid if ti < mine
          uint32_t v = seg_finish<true, 2, ABLATE, true>(smem, P, S[k % R], lo, hi);
          v = (S[k % R].fl & FL_VALID) ? v : 0u;
          dv = ~run_xor(v, min(63u, lane + S[k % R].k));
          const uint64_t r0 = (uint64_t)(t0 + ti) * m;  // the tile's first record
          dcnt = ti < mine ? (uint32_t)min((uint64_t)m, (uint64_t)P.nrec - r0) : 0u;
        } else {
          finish_tile<true, 2, ABLATE, true>(smem, P, S[k % R], lane, lo, hi);
        }
      }
      n0 += R;
    }
    if constexpr (ORDER == 5) {
      if (dst) P.out[drec] = dv;
    }
    if constexpr (QST) {
      if (dcnt) qpush(dv, dcnt);
    }
  };
  if constexpr (ORDER == 0 || ORDER == 4 || ORDER == 5) {
    if (wave >= ntiles) return;
    run(wave, (ntiles - wave + nwaves - 1u) / nwaves, nwaves);
  } else if constexpr (ORDER == 1) {
    const uint32_t per = (ntiles + nwaves - 1u) / nwaves, t0 = wave * per;
    if (t0 >= ntiles) return;
    if constexpr (QST) {
      qb = ((uint64_t)t0 * m) & ~63ull;
      qs = qf = (uint32_t)(((uint64_t)t0 * m) & 63u);
    }
    run(t0, min(per, ntiles - t0), 1u);
    if constexpr (QST) qstore(lane >= qs && lane < qf);
  } else {
    const uint32_t nb = (ntiles + WRING_BLOCK - 1u) / WRING_BLOCK;
    for (;;) {
      uint32_t b = 0;
      if (lane == 0) b = atomicAdd(P.work, 1u);
      b = __builtin_amdgcn_readfirstlane(b);
      if (b >= nb) break;
      run(b * WRING_BLOCK, min(WRING_BLOCK, ntiles - b * WRING_BLOCK), 1u);
    }
  }
}

// ---------------------------------------------------------------------------
// Descriptor records (offset u64, len u32), arbitrary alignment and order.
// Prep (scan kernels below): every record owns nseg = max(1, ceil(len/128))
// consecutive segments (an empty record owns one empty segment, so every
// record has a start lane); seg_start[r] = exclusive prefix of nseg; per
// 64-segment tile, tile_info[t] = {r0 = record holding segment 64t,
// q0 = its segment index there, 64-bit mask of record starts in the tile}.
// A wave maps its lanes from that one 16-byte record (a scalar load):
//   rec = r0 + (record starts at positions 1..lane)
//   q   = lane - (last start <= lane), or q0 + lane if none.
// stage 0 (three tiles ahead): the tile's 16-byte record.  A vector load
// (lane l holds dword l&3), not a scalar one: it then retires in order with
// the payload loads (vmcnt), while an s_load would share lgkmcnt with the LDS
// lookups and force lgkmcnt(0) waits in the checksum loop.  Tiles outside
// [0, ntiles) read a clamped entry (their lanes are all pad lanes).
template <int ABLATE = 0>
__device__ __forceinline__ uint32_t desc_tile(const CrcParams& P, int32_t x, int32_t nt, uint32_t lane) {
  const int32_t c = x < 0 ? 0 : (x < nt ? x : nt - 1);
  if (ABLATE >= 4 && ABLATE <= 6) {  // diagnostic, config-2 layout only (4 KiB records): synthesized, not loaded
    const uint32_t q = lane & 3u;
    return q == 0 ? 2u * (uint32_t)c : (q == 1 ? 0u : 1u);
  }
  return P.tile_info[4ull * (uint32_t)c + (lane & 3u)];
}

// stage 1 (two tiles ahead): lane -> (rec, q); issues the off/len gathers
template <int ABLATE = 0>
__device__ __forceinline__ SegInfo desc_map_issue(const CrcParams& P, uint32_t tv, int32_t x, uint32_t lane,
                                                  uint32_t total) {
  // (readlane returns int: go through uint32_t, a direct widening would sign-extend)
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane(tv, 0), q0 = (uint32_t)__builtin_amdgcn_readlane(tv, 1);
  const uint32_t mlo = (uint32_t)__builtin_amdgcn_readlane(tv, 2), mhi = (uint32_t)__builtin_amdgcn_readlane(tv, 3);
  const uint64_t mask = (uint64_t)mlo | ((uint64_t)mhi << 32);
  const uint64_t below = mask & ((lane == 63u) ? ~0ull : ((2ull << lane) - 1ull));
  const uint32_t cnt = (uint32_t)__builtin_popcountll(below & ~1ull);
  SegInfo si;
  si.valid = (x >= 0) & ((uint32_t)x * 64u + lane < total);
  uint32_t rec = r0 + cnt;
  rec = (si.valid && rec < P.nrec) ? rec : (uint32_t)P.nrec - 1u;
  si.q = below ? lane - (63u - (uint32_t)__builtin_clzll(below)) : q0 + lane;
  si.rec = rec;
  if (ABLATE == 5 || ABLATE == 6) {  // diagnostic, config-2 layout only: synthesized descriptors
    si.rec_off = (uint64_t)rec * 4096u;
    si.rec_len = 4096u;
  } else {
    si.rec_off = P.off[rec];
    si.rec_len = P.len[rec];
  }
  si.k = 0;
  return si;
}

// stage 2 (one tile ahead, once the gathers have landed): segments after this one
__device__ __forceinline__ void desc_map_complete(SegInfo& si) {
  const uint32_t nseg = si.rec_len ? (si.rec_len + 127u) >> 7 : 1u;
  si.k = nseg - 1u - si.q;
  if (!si.valid) {  // pad lanes: an empty first segment (loads only the zero buffer; no store)
    si.q = 0;
    si.k = 0;
    si.rec_len = 0;
  }
}

// Three-stage software pipeline per wave (tile stride n = nwaves):
//   tile_info(c+3n) | off/len gathers(c+2n) | payload loads(c+n) | checksum(c)
// Each wait is for loads issued one half-iteration earlier, which are older
// than the payload of tile c+n (vmcnt retires in order), so no dependent
// gather round trip is exposed.  Unrolled 2x so that every stage alternates
// between two register sets and no in-flight register is copied.  There is
// no prologue and no skipped stage: the loop starts three tiles early on
// virtual tiles (all pad lanes: zero-buffer loads, checksum computed and
// dropped), so the loop header is only ever entered with the same loads in
// flight in the same order -- a differently scheduled prologue, or a branch
// around a stage, makes the wait-count merge at the header conservative.
template <int CHAINS, int ABLATE = 0, int BLOCK = 1024>
__global__ __launch_bounds__(BLOCK) void crc32_desc_kernel(CrcParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  build_lds_tables(smem, P);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lo = (lane & 31u) * 4u, hi = lo | 0x10000u;
  const int32_t wave = (int32_t)__builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int32_t n = (int32_t)((gridDim.x * blockDim.x) >> 6);
  const uint32_t total = (uint32_t)*P.total_segs;  // host checked < 2^32
  const int32_t nt = (int32_t)((total + 63u) >> 6);  // < 2^26
  if (wave >= nt) return;
  const uint64_t data_end = (ABLATE == 13 || ABLATE == 14) ? P.off[P.nrec - 1] + P.len[P.nrec - 1] : 0;
  uint32_t T0 = 0, T1 = 0;  // virtual tiles: no loads needed, all lanes pad
  SegInfo M0, M1;
  M0.valid = M1.valid = false;
  M0.q = M1.q = 0;
  M0.rec = M1.rec = 0;
  // (the general loads send an empty segment to the zero buffer; the aligned
  // loads of diagnostic 6 read [E-128, E) and need E >= 128)
  M0.rec_off = M1.rec_off = (ABLATE == 6 || ABLATE == 12) ? 128u : 0u;
  M0.rec_len = M1.rec_len = 0;
  M0.k = M1.k = 0;
  SegLoad A, B;
  A.fl = 0;  // first virtual tile: no valid lane, nothing stored
  A.k = 0;
  A.rec = 0;
  // half-steps: 3 virtual + the wave's real tiles; one bottom exit (see the
  // fixed kernel), the odd last half-step after the loop only checksums
  const int32_t H = 3 + (nt - wave + n - 1) / n;
  int32_t c = wave - 3 * n;
  for (int32_t j = 2; j <= H; j += 2) {
    // in flight: A = payload(c), M1 = gathers(c+n), T0 = tile_info(c+2n)
    M0 = desc_map_issue<ABLATE>(P, T0, c + 2 * n, lane, total);
    T1 = desc_tile<ABLATE>(P, c + 3 * n, nt, lane);
    desc_map_complete(M1);
    if constexpr (ABLATE == 13 || ABLATE == 14)
      seg_issue_pk(P, M1, B, data_end);
    else
      seg_issue<(ABLATE == 6 || ABLATE == 12), ABLATE>(P, M1, B);
    __builtin_amdgcn_sched_barrier(0);
    finish_tile<false, CHAINS, ABLATE>(smem, P, A, lane, lo, hi);  // virtual tiles: pad lanes, no store
    c += n;
    // in flight: B = payload(c), M0 = gathers(c+n), T1 = tile_info(c+2n)
    M1 = desc_map_issue<ABLATE>(P, T1, c + 2 * n, lane, total);
    T0 = desc_tile<ABLATE>(P, c + 3 * n, nt, lane);
    desc_map_complete(M0);
    if constexpr (ABLATE == 13 || ABLATE == 14)
      seg_issue_pk(P, M0, A, data_end);
    else
      seg_issue<(ABLATE == 6 || ABLATE == 12), ABLATE>(P, M0, A);
    __builtin_amdgcn_sched_barrier(0);
    finish_tile<false, CHAINS, ABLATE>(smem, P, B, lane, lo, hi);
    c += n;
  }
  if (H & 1) finish_tile<false, CHAINS, ABLATE>(smem, P, A, lane, lo, hi);
}

// ---------------------------------------------------------------------------
// Prep kernels for the descriptor path.  Every record owns
// nseg = max(1, ceil(len/128)) consecutive segments; the checksum kernel only
// needs tile_info (record starts per 64-segment tile), so no per-record
// prefix array is materialised: phase 1 reduces nseg per 4096-record block,
// phase 2 scans the block sums (u64: a batch may exceed 2^32 segments, which
// the host rejects after reading the total), phase 3 re-reads len, rescans
// inside its block and writes tile_info.  HBM traffic: len twice + tile_info.
// Four records per thread (one 16-byte load): the kernels are bound by wave
// launches and the cross-lane steps, not by bytes; scans run on DPP.
#define SCAN_BLOCK 1024
#define SCAN_ITEMS 4
#define SCAN_RECS (SCAN_BLOCK * SCAN_ITEMS)
__device__ __forceinline__ uint32_t rec_nseg(uint32_t len) { return len ? (len + 127u) >> 7 : 1u; }

// the thread's four lengths (records >= n read as "absent": own = false)
__device__ __forceinline__ void load_len4(const uint32_t* __restrict__ len, uint64_t n, uint64_t r0, uint32_t l[4]) {
  if (r0 + 3 < n) {
    u32x4 v = *(const u32x4*)(len + r0);  // dword-aligned 16-byte load
    l[0] = v.x;
    l[1] = v.y;
    l[2] = v.z;
    l[3] = v.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) l[j] = (r0 + j < n) ? len[r0 + j] : 0u;
  }
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int dppv(int old, int x) {
  return __builtin_amdgcn_update_dpp(old, x, CTRL, ROW_MASK, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_prefix_add(uint32_t x) {  // inclusive
  x += (uint32_t)dppv<0x111, 0xF>(0, (int)x);
  x += (uint32_t)dppv<0x112, 0xF>(0, (int)x);
  x += (uint32_t)dppv<0x114, 0xF>(0, (int)x);
  x += (uint32_t)dppv<0x118, 0xF>(0, (int)x);
  x += (uint32_t)dppv<0x142, 0xA>(0, (int)x);
  x += (uint32_t)dppv<0x143, 0xC>(0, (int)x);
  return x;
}
__device__ __forceinline__ int wave_prefix_max(int x) {  // inclusive, identity -1
  x = max(x, dppv<0x111, 0xF>(-1, x));
  x = max(x, dppv<0x112, 0xF>(-1, x));
  x = max(x, dppv<0x114, 0xF>(-1, x));
  x = max(x, dppv<0x118, 0xF>(-1, x));
  x = max(x, dppv<0x142, 0xA>(-1, x));
  x = max(x, dppv<0x143, 0xC>(-1, x));
  return x;
}

__global__ __launch_bounds__(SCAN_BLOCK) void scan_phase1(const uint32_t* __restrict__ len, uint64_t n,
                                                           uint64_t* __restrict__ block_sum) {
  __shared__ uint64_t wsum[SCAN_BLOCK / 64];
  const uint64_t r0 = (uint64_t)blockIdx.x * SCAN_RECS + (uint64_t)threadIdx.x * SCAN_ITEMS;
  uint32_t l[4];
  load_len4(len, n, r0, l);
  uint64_t x = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) x += (r0 + j < n) ? rec_nseg(l[j]) : 0u;
  // a wave may hold 256 x 2^25 segments: reduce in u64
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  if ((threadIdx.x & 63u) == 0) wsum[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
#pragma unroll
    for (int i = 0; i < SCAN_BLOCK / 64; ++i) t += wsum[i];
    block_sum[blockIdx.x] = t;
  }
}

// single workgroup: exclusive scan of the block sums in place, total in *total.
// Thread i owns the contiguous chunk [i*C, (i+1)*C).
// skip: the stream kernel's flag -- set when it took the batch, so the walking
// kernel's segment prefix is not needed (nullptr: always run)
__global__ __launch_bounds__(1024) void scan_phase2(uint64_t* __restrict__ block_sum, uint32_t nblocks,
                                                     uint64_t* __restrict__ total, const uint32_t* skip = nullptr) {
  if (skip && *skip) return;
  __shared__ uint64_t wsum[16];
  const uint32_t C = (nblocks + 1023u) / 1024u;
  const uint32_t b0 = threadIdx.x * C, b1 = min(nblocks, b0 + C);
  uint64_t mine = 0;
  for (uint32_t b = b0; b < b1; ++b) mine += block_sum[b];
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t x = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t o = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += o;
  }
  if (lane == 63u) wsum[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t acc = 0;
    for (int i = 0; i < 16; ++i) {
      uint64_t v = wsum[i];
      wsum[i] = acc;
      acc += v;
    }
    *total = acc;
  }
  __syncthreads();
  uint64_t run = wsum[threadIdx.x >> 6] + x - mine;  // exclusive prefix of this chunk
  for (uint32_t b = b0; b < b1; ++b) {
    uint64_t v = block_sum[b];
    block_sum[b] = run;
    run += v;
  }
}

// Start masks: records of one tile are a run of consecutive records (ss is
// non-decreasing), so each run ORs its start bits into an LDS slot owned by
// the run's first record (per wave: 256 records, 256 slots), and that record
// stores the tile's mask: a plain store, or atomicOr for the wave's first and
// last tile, which a neighbouring wave may share (tile_info is zeroed first).
__global__ __launch_bounds__(SCAN_BLOCK) void scan_phase3(const uint32_t* __restrict__ len, uint64_t n,
                                                           const uint64_t* __restrict__ block_sum,
                                                           uint32_t* __restrict__ tile_info) {
  __shared__ uint32_t wsum[SCAN_BLOCK / 64];
  __shared__ unsigned long long slot[SCAN_BLOCK / 64][64 * SCAN_ITEMS];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t r0 = (uint64_t)blockIdx.x * SCAN_RECS + (uint64_t)threadIdx.x * SCAN_ITEMS;
  uint32_t l[4], ns[4], e[4];
  load_len4(len, n, r0, l);
  uint32_t tsum = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ns[j] = (r0 + j < n) ? rec_nseg(l[j]) : 0u;
    e[j] = tsum;
    tsum += ns[j];
  }
  // block-exclusive prefix of the thread sums (u32: the host launches this
  // only when the whole batch has < 2^32 segments)
  const uint32_t x = wave_prefix_add(tsum);
  if (lane == 63u) wsum[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < SCAN_BLOCK / 64; ++i) {
      uint32_t v = wsum[i];
      wsum[i] = acc;
      acc += v;
    }
  }
  __syncthreads();
  const uint64_t wr0 = (uint64_t)blockIdx.x * SCAN_RECS + (uint64_t)w * 64u * SCAN_ITEMS;  // wave's first record
  if (wr0 >= n) return;  // whole wave past the end (wave-uniform, after the barriers)
  const uint32_t base = (uint32_t)block_sum[blockIdx.x] + wsum[w] + (x - tsum);
  uint32_t ss[4], T[4];
  bool own[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ss[j] = base + e[j];
    T[j] = ss[j] >> 6;
    own[j] = r0 + j < n;
  }
  // run heads: a record whose tile differs from its predecessor's (record 0 of
  // the wave always); h[j] = index in the wave of the head of j's run
  const uint32_t prevT3 = (uint32_t)dppv<0x138, 0xF>(-1, (int)T[3]);  // wave_shr:1: lane-1's last tile
  bool head[4];
  head[0] = own[0] && (lane == 0 || prevT3 != T[0]);
#pragma unroll
  for (int j = 1; j < 4; ++j) head[j] = own[j] && T[j] != T[j - 1];
  int lasth = -1;
#pragma unroll
  for (int j = 0; j < 4; ++j) lasth = head[j] ? (int)(lane * 4u + j) : lasth;
  const int before = dppv<0x138, 0xF>(-1, wave_prefix_max(lasth));  // last head in lanes < lane
  int h[4];
  int cur = before;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    cur = head[j] ? (int)(lane * 4u + j) : cur;
    h[j] = cur;
  }
  unsigned long long* sl = slot[w];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (head[j]) sl[h[j]] = 0ull;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (own[j]) atomicOr(&sl[h[j]], 1ull << (ss[j] & 63u));
  // the wave's first and last tiles (last own record: index min(255, n-1-wr0))
  const uint32_t nown = (uint32_t)min((uint64_t)(64 * SCAN_ITEMS), n - wr0);
  const uint32_t firstT = (uint32_t)__builtin_amdgcn_readfirstlane((int)T[0]);
  const uint32_t ll = (nown - 1u) >> 2, lj = (nown - 1u) & 3u;
  const uint32_t Tl = lj == 0 ? T[0] : (lj == 1 ? T[1] : (lj == 2 ? T[2] : T[3]));
  const uint32_t lastT = (uint32_t)__builtin_amdgcn_readlane((int)Tl, (int)ll);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (head[j]) {
      const unsigned long long m = sl[h[j]];
      unsigned long long* gm = (unsigned long long*)(tile_info + 4ull * T[j] + 2);
      if (T[j] == firstT || T[j] == lastT)
        atomicOr(gm, m);
      else
        *gm = m;
    }
  }
  // tiles whose first segment lies in record r: r0 = r, q0 = 64t - ss
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!own[j]) continue;
    const uint32_t t0 = (ss[j] + 63u) >> 6, t1 = (ss[j] + ns[j] - 1u) >> 6;
    for (uint32_t t = t0; t <= t1; ++t) {
      tile_info[4ull * t + 0] = (uint32_t)(r0 + j);
      tile_info[4ull * t + 1] = t * 64u - ss[j];
    }
  }
}


// ===========================================================================
// Walking descriptor kernel (the default for descriptor batches).
//
// Every wave owns ONE contiguous run of records -- whole superblocks of
// WALK_SB records, cut so that every wave gets about the same number of
// 128-byte segments (walk_phase1 + scan_phase2 give the segment prefix per
// superblock; a wave binary-searches its cut points) -- and walks the run's
// segments in order, 64 per tile.  So:
//  * no record is split between waves: every CRC is stored once, with a plain
//    store (no zeroing of `out`, no atomics);
//  * a record spanning tiles carries its partial value to the next tile in a
//    wave-uniform register (Horner: carry (x) x^(8*128*m) ^ the next tile's
//    part), so a lane only shifts its segment to the record's last lane IN THE
//    TILE, d < 64 segments: 32 precomputed LDS columns per d (8 ds_read_b128 +
//    32 v_bitop3) instead of the 32-step generic GF(2) multiply;
//  * the segment -> record map comes from windows of 64 records (one per lane:
//    off, len, prefix of segment counts) held in registers, three windows deep
//    (current, next, prefetched): no per-tile map in HBM.  The only scratch is
//    one u64 per superblock, sized by the record count, so the host never has
//    to read a device total back to size anything: the batch is asynchronous
//    on its stream;
//  * contiguous per-wave runs stream as fast as the strided tile order of the
//    fixed kernels (tools/microbench_walk.hip: 6.56 against 6.42 TB/s over
//    96 GiB, profiles/r02/mb/mb_walk96.log).
#define WALK_SB 256u
#define LDS_WCOLS_OFF LDS_COLS_OFF  // [8 groups][65 d][4 u32] columns of x^(8*128*d), d = 0..64 (8320 B)

__global__ __launch_bounds__(1024) void walk_phase1(const uint32_t* __restrict__ len, uint64_t n,
                                                     uint64_t* __restrict__ sb_sum, const uint32_t* skip) {
  if (skip && *skip) return;  // the stream kernel took the batch
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t sb = (uint64_t)blockIdx.x * 16u + (threadIdx.x >> 6);
  if (sb * WALK_SB >= n) return;  // wave-uniform
  const uint64_t r0 = sb * WALK_SB + lane * 4u;
  uint32_t l[4];
  load_len4(len, n, r0, l);
  uint64_t x = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) x += (r0 + j < n) ? rec_nseg(l[j]) : 0u;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  if (lane == 0) sb_sum[sb] = x;
}

// columns K*x^i (i = 0..31) of K = x^(8*128*d), d = 0..64, for the Horner shifts
__device__ __forceinline__ void build_walk_cols(const CrcParams& P) {
  if (threadIdx.x > 64) return;
  const uint32_t d = threadIdx.x;
  uint32_t b = P.kseg[d];
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    *(__attribute__((address_space(3))) uint32_t*)(size_t)(LDS_WCOLS_OFF + ((i >> 2) * 65u + d) * 16u + (i & 3) * 4u) = b;
    b = (b >> 1) ^ (0xEDB88320u & (0u - (b & 1u)));
  }
}

// v (x) x^(8*128*d), d = 0..64, from the LDS columns
__device__ __forceinline__ uint32_t walk_mulcol(uint32_t v, uint32_t d) {
  uint32_t p = 0;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const u32x4 c = lds_ld128(LDS_WCOLS_OFF + (g * 65u + d) * 16u);
    p = __builtin_amdgcn_bitop3_b32(p, c.x, (uint32_t)((int32_t)(v << (4 * g + 0)) >> 31), 0x78);
    p = __builtin_amdgcn_bitop3_b32(p, c.y, (uint32_t)((int32_t)(v << (4 * g + 1)) >> 31), 0x78);
    p = __builtin_amdgcn_bitop3_b32(p, c.z, (uint32_t)((int32_t)(v << (4 * g + 2)) >> 31), 0x78);
    p = __builtin_amdgcn_bitop3_b32(p, c.w, (uint32_t)((int32_t)(v << (4 * g + 3)) >> 31), 0x78);
  }
  return p;
}

// the same for a wave-uniform v and d = 1..64, spread over the lanes: lane i
// < 32 contributes column i if bit 31-i of v is set; XOR over lanes 0..31
// OPQ: the lane's column offset is recomputed at each use rather than held
// across the tile loop (in the stream kernel's short-path form it spilled)
template <bool OPQ = false>
__device__ __forceinline__ uint32_t walk_mulcol_uniform(uint32_t v, uint32_t d, uint32_t lane) {
  uint32_t i = lane & 31u;
  if (OPQ) asm volatile("" : "+v"(i));
  const uint32_t col = lds_ld(nullptr, LDS_WCOLS_OFF + ((i >> 2) * 65u + d) * 16u + (i & 3u) * 4u);
  const uint32_t t = (lane < 32u && ((v >> (31u - i)) & 1u)) ? col : 0u;
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_prefix_xor(t), 31);
}

__device__ __forceinline__ uint32_t wave_or_u32(uint32_t x) {  // OR over the wave (uniform)
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
  x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// a window: records w0 + lane of the run (lane-held), absent past the run's end
struct WalkWin {
  uint64_t off;
  uint32_t len;
  uint32_t p;    // exclusive prefix of the segment counts inside the window
  uint32_t ok;   // the record exists (in the run)
};
__device__ __forceinline__ void walk_win_issue(const CrcParams& P, uint64_t w0, uint64_t r1, uint32_t lane, WalkWin& W) {
  const uint64_t r = w0 + lane;
  W.ok = r < r1;
  const uint64_t rr = W.ok ? r : (r1 - 1u);  // r1 > 0 whenever a window is loaded
  W.off = P.off[rr];
  W.len = P.len[rr];
}
// segment prefix of a landed window; returns the window's segment total (uniform)
__device__ __forceinline__ uint32_t walk_win_scan(WalkWin& W) {
  const uint32_t ns = W.ok ? rec_nseg(W.len) : 0u;
  const uint32_t inc = wave_prefix_add(ns);
  W.p = inc - ns;
  return (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
}
__device__ __forceinline__ uint64_t start_bit(const WalkWin& W, int64_t rel) {
  // rel = position of the window's first segment relative to the tile start
  const int64_t s = rel + (int64_t)W.p;
  return (W.ok && s >= 1 && s <= 63) ? (1ull << s) : 0ull;
}

// OPQ: the continuing record's uniform multiply recomputes its lane column
// offset (else hipcc kept it in two VGPRs that spilled, reloaded in the tile
// loop behind an s_waitcnt vmcnt(0) on the payload prefetch)
template <int CHAINS, int ABLATE = 0, bool OPQ = false>
__global__ __launch_bounds__(1024) void crc32_walk_kernel(CrcParams P) {
  if (P.sflag && *P.sflag) return;  // a packed batch of >= 64-byte records: crc32_stream_kernel took it
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  build_lds_tables(smem, P);
  __syncthreads();  // the column table reuses the khi/klo area the table build fills
  build_walk_cols(P);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lo = (lane & 31u) * 4u, hi = lo | 0x10000u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
  const uint64_t n = P.nrec;
  const uint64_t nsb = (n + WALK_SB - 1u) / WALK_SB;
  const uint64_t S = *P.total_segs;
  // this wave's superblocks [b0, b1): the first superblock whose segment
  // prefix reaches S*w/nw (lower bound), for w and w+1
  auto cut = [&](uint32_t w) -> uint64_t {
    if (w >= nw) return nsb;
    const uint64_t target = (S / nw) * w + (S % nw) * w / nw;  // floor(S*w/nw) without overflow
    uint64_t a = 0, b = nsb;
    while (a < b) {
      const uint64_t m = (a + b) >> 1;
      if (P.sb_prefix[m] < target) a = m + 1; else b = m;
    }
    return a;
  };
  const uint64_t b0 = cut(wave), b1 = cut(wave + 1);
  if (b0 >= b1) return;
  const uint64_t r0 = b0 * WALK_SB, r1 = min(n, b1 * WALK_SB);
  const uint64_t segs = (b1 < nsb ? P.sb_prefix[b1] : S) - P.sb_prefix[b0];
  const uint64_t ntile = (segs + 63u) >> 6;
  // windows: records [r0 + 64*wc, +64) (cur), the next (nxt), the one after (pre, in flight)
  WalkWin cur, nxt, pre;
  walk_win_issue(P, r0, r1, lane, cur);
  walk_win_issue(P, r0 + 64u, r1, lane, nxt);
  walk_win_issue(P, r0 + 128u, r1, lane, pre);
  uint64_t wc0 = r0;                      // first record of cur
  uint64_t Bc = 0;                         // run segment of cur's first segment
  const uint32_t totc0 = walk_win_scan(cur);
  uint64_t Bn = Bc + totc0;                // run segment of nxt's first segment
  uint32_t totn = walk_win_scan(nxt);
  uint64_t G = 0;                          // run segment at lane 0 of the tile being mapped
  uint64_t rg = r0;                        // record holding segment G
  uint32_t qg = 0;                         //   and its segment index there
  uint32_t carry = 0;                      // partial value of the record continuing across tiles
  SegLoad A, B;
  A.fl = 0;  // virtual tile before the first: no valid lane, nothing stored
  A.k = 0;
  A.rec = 0;

  // map the tile at G onto (record, segment) per lane, advance the cursor and the windows
  auto map_tile = [&]() -> SegInfo {
    const uint64_t m = start_bit(cur, (int64_t)(Bc - G)) | start_bit(nxt, (int64_t)(Bn - G));
    const uint64_t M = (uint64_t)wave_or_u32((uint32_t)m) | ((uint64_t)wave_or_u32((uint32_t)(m >> 32)) << 32);
    const uint64_t below = M & ((lane == 63u) ? ~0ull : ((2ull << lane) - 1ull));
    SegInfo si;
    const uint64_t rec = rg + (uint64_t)__builtin_popcountll(below);
    si.q = below ? lane - (63u - (uint32_t)__builtin_clzll(below)) : qg + lane;
    // pad lanes: past the run's last segment (no start bit marks the end of
    // the run's last record, so the record index alone cannot tell)
    si.valid = G + lane < segs;
    const uint32_t idx = (uint32_t)(si.valid ? rec - wc0 : 0u);  // < 128
    const int src = (int)((idx & 63u) << 2);
    const uint32_t ol_c = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)cur.off);
    const uint32_t oh_c = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(cur.off >> 32));
    const uint32_t ln_c = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)cur.len);
    const uint32_t ol_n = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)nxt.off);
    const uint32_t oh_n = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(nxt.off >> 32));
    const uint32_t ln_n = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)nxt.len);
    const bool in_c = idx < 64u;
    si.rec = (uint32_t)rec;
    si.rec_off = in_c ? (((uint64_t)oh_c << 32) | ol_c) : (((uint64_t)oh_n << 32) | ol_n);
    si.rec_len = in_c ? ln_c : ln_n;
    si.k = 0;
    // (defensive: a lane never addresses a segment its record does not have)
    si.valid = si.valid && si.q < (si.rec_len ? (si.rec_len + 127u) >> 7 : 1u);
    desc_map_complete(si);  // k; pad lanes become empty first segments
    // cursor for the next tile: the record holding segment G + 64
    const uint32_t rec63 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(rec - wc0), 63);
    const uint32_t q63 = (uint32_t)__builtin_amdgcn_readlane((int)si.q, 63);
    const uint32_t k63 = (uint32_t)__builtin_amdgcn_readlane((int)si.k, 63);
    rg = wc0 + rec63 + (k63 ? 0u : 1u);
    qg = k63 ? q63 + 1u : 0u;
    G += 64u;
    // one window step when the cursor left cur (at most one per tile: a full
    // window holds >= 64 segments); branch-free, pre is reloaded every tile
    const bool rot = rg >= wc0 + 64u;
    cur.off = rot ? nxt.off : cur.off;
    cur.len = rot ? nxt.len : cur.len;
    cur.p = rot ? nxt.p : cur.p;
    cur.ok = rot ? nxt.ok : cur.ok;
    nxt.off = rot ? pre.off : nxt.off;
    nxt.len = rot ? pre.len : nxt.len;
    nxt.ok = rot ? pre.ok : nxt.ok;
    wc0 = rot ? wc0 + 64u : wc0;
    Bc = rot ? Bn : Bc;
    const uint32_t tn = walk_win_scan(nxt);
    Bn = Bc + (rot ? totn : (Bn - Bc));
    totn = tn;
    walk_win_issue(P, wc0 + 128u, r1, lane, pre);
    return si;
  };

  auto finish = [&](const SegLoad& L) {
    if (!__builtin_amdgcn_readfirstlane((int)(L.fl & FL_VALID))) return;  // virtual tile (lane 0 valid otherwise)
    uint32_t v = seg_finish<false, CHAINS, ABLATE, false, true>(smem, P, L, lo, hi);
    if (ABLATE == 3) {  // loads only (no reduction or store, unless a magic value keeps the loads alive)
      if (v == 0x9E3779B1u) P.out[0] = v;
      return;
    }
    const bool valid = (L.fl & FL_VALID) != 0;
    v = valid ? v : 0u;
    const uint32_t d = min(63u - lane, L.k);
    v = walk_mulcol(v, d);
    const uint32_t run_end = min(63u, lane + L.k);
    const uint32_t X = wave_prefix_xor(v);
    const uint32_t Xe = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(run_end << 2), (int)X);
    uint32_t total = Xe ^ dpp0<0x138, 0xF>(X);  // lanes [lane, run_end]
    const bool head = valid && (lane == 0u || (L.fl & FL_FIRST));
    // lane 0 continuing a record from the previous tile: Horner step
    const bool cont0 = !__builtin_amdgcn_readfirstlane((int)(L.fl & FL_FIRST));
    const uint32_t re0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)run_end);
    const uint32_t cm = cont0 ? walk_mulcol_uniform<OPQ>(carry, re0 + 1u, lane) : 0u;
    total ^= (lane == 0u) ? cm : 0u;
    const bool ends = head && (lane + L.k <= 63u);
    if (ends) P.out[L.rec] = ~total;
    const uint64_t cb = __ballot(head && lane + L.k > 63u);
    carry = cb ? (uint32_t)__builtin_amdgcn_readlane((int)total, __builtin_ctzll(cb)) : 0u;
  };

  // half-steps: map + issue tile t, then finish tile t-1; one bottom exit with
  // a precomputed trip count (see crc32_fixed_kernel)
  uint64_t t = 0;
  for (; t + 2 <= ntile; t += 2) {
    seg_issue<false, ABLATE>(P, map_tile(), B);
    __builtin_amdgcn_sched_barrier(0);
    finish(A);
    seg_issue<false, ABLATE>(P, map_tile(), A);
    __builtin_amdgcn_sched_barrier(0);
    finish(B);
  }
  if (t < ntile) {
    seg_issue<false, ABLATE>(P, map_tile(), B);
    __builtin_amdgcn_sched_barrier(0);
    finish(A);
    finish(B);
  } else {
    finish(A);
  }
}

// ===========================================================================
// Stream kernel: packed batches (record r+1 starts where r ends) of records of
// at least 64 bytes -- config 3's shape.  The lanes read the batch as ALIGNED
// 128-byte chunks of the byte stream, the fixed ring kernel's load shape
// (buffer loads from a wave-uniform tile base, no per-lane address from the
// descriptors: tools/microbench_c3.hip, 16.2 against 18.2 ms for config 3's
// per-record segment windows), and record boundaries inside a chunk are CRC
// register resets.  tools/stream_sim.py is the lane-level model of the
// algebra below, checked against zlib:
//  * a chunk is 32 words in two chains of 16; a boundary at chunk byte j lies
//    in chain h = j >= 64 (>= 64-byte records: at most one per chain).  At its
//    word the chain computes A = F(c ^ (u & ~mlo)) -- the chain's bytes before
//    j, zero-extended to the word end -- and xors A ^ I into its register,
//    I = 0xFFFFFFFF (x) x^(8s), s = bytes from j to the word end: the register
//    then holds the new record's bytes from j with the CRC's init folded in;
//  * the chunk's tail T (the last piece, aligned to the chunk end) is carried
//    Horner-wise to the chunk before the record's end chunk: T (x) x^(1024 d)
//    from the LDS columns, a prefix XOR over the wave, a wave-uniform carry
//    across tiles;
//  * a record ending at byte j of chunk c: CRC = ~(P (x) x^(8m) ^ A (x)
//    x^(-8s)), P = Hprev (chain 0) or shift64(Hprev) ^ R0 (chain 1), m = j -
//    64h -- computed by the window lane of its end boundary, so every CRC is
//    one plain, coalesced store.
// Boundaries are read from off[] in windows of 128 (a tile holds at most 128:
// records >= 64 bytes), one tile ahead.  Each wave owns the boundaries
// [cut_w, cut_w+1] (stream_cuts: balanced by bytes) and the tiles that hold
// them; a record belongs to the wave of its end boundary.  Eligibility is
// decided on the device (stream_check); the walking kernel, launched after
// this one, exits when the batch was taken here.
#define STREAM_MIN_LEN 64u
// LDS columns K (x) x^i, i = 0..31 (128 B per factor K) of the finish factors,
// in areas this kernel does not otherwise use: x^(8m) for m = 0..31 over the
// shift-by-32-bytes table, m = 32..63 over the shift-by-96-bytes table (only
// shift-by-64 is used here), x^(-8(4-t)) for t = 0..3 in the klo area
#define LDS_XMC_OFF(m) ((m) < 32u ? LDS_SHIFT_OFF + (m) * 128u : LDS_SHIFT_OFF + 8192u + ((m) - 32u) * 128u)
#define LDS_XIC_OFF(t) (LDS_KLO_OFF + (t) * 128u)

// v (x) K from K's 32 LDS columns at `base` (8 ds_read_b128 + 32 v_bitop3).
// (The generic gf2_mulmod here had its factor folded into 32 hoisted shifted
// copies: ~70 spilled VGPRs.)
__device__ __forceinline__ uint32_t stream_mulcol(uint32_t v, uint32_t base) {
  uint32_t p = 0;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const u32x4 c = lds_ld128(base + g * 16u);
    p = __builtin_amdgcn_bitop3_b32(p, c.x, (uint32_t)((int32_t)(v << (4 * g + 0)) >> 31), 0x78);
    p = __builtin_amdgcn_bitop3_b32(p, c.y, (uint32_t)((int32_t)(v << (4 * g + 1)) >> 31), 0x78);
    p = __builtin_amdgcn_bitop3_b32(p, c.z, (uint32_t)((int32_t)(v << (4 * g + 2)) >> 31), 0x78);
    p = __builtin_amdgcn_bitop3_b32(p, c.w, (uint32_t)((int32_t)(v << (4 * g + 3)) >> 31), 0x78);
  }
  return p;
}

// The exact capture at a boundary at byte t of word u: the register s before
// the word advanced over the word's t bytes before the boundary (the ending
// record's last bytes), slicing-by-t from cx = s ^ u:
// (s >> 8t) ^ XOR_{i<t} T_{t-1-i}[cx byte i].  Run once per chunk after the
// chains, off their dependency path.
__device__ __forceinline__ uint32_t stream_capture(const unsigned char* smem, uint32_t cx, uint32_t u, uint32_t t,
                                                   uint32_t lo) {
  const uint32_t b0 = t == 1u ? lo : (t == 2u ? lo + 128u : (lo | 0x10000u));  // T_{t-1}
  const uint32_t b1 = t == 2u ? lo : lo + 128u;                                // T_{t-2}
  const uint32_t l0 = lds_ld(smem, __builtin_amdgcn_perm(cx, b0, 0x0c020400u));  // byte 0
  const uint32_t l1 = lds_ld(smem, __builtin_amdgcn_perm(cx, b1, 0x0c020500u));  // byte 1
  const uint32_t l2 = lds_ld(smem, __builtin_amdgcn_perm(cx, lo, 0x0c020600u));  // byte 2 (T0)
  return ((cx ^ u) >> (t << 3)) ^ (t >= 1u ? l0 : 0u) ^ (t >= 2u ? l1 : 0u) ^ (t >= 3u ? l2 : 0u);
}

__device__ __forceinline__ uint32_t stream_xinv(uint32_t t) {  // x^(-8(4-t))
  return t == 0u ? 0x5b358fd3u : (t == 1u ? 0x1f81b6e1u : (t == 2u ? 0xd7125358u : 0x6567cb95u));
}

__global__ __launch_bounds__(1024) void stream_check(const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
                                                     uint64_t n, uint32_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = false;
  if (i < n) {
    const uint32_t l = len[i];
    bad = l < STREAM_MIN_LEN || (i + 1 < n && off[i + 1] != off[i] + l);
  }
  if (__any(bad) && (threadIdx.x & 63u) == 0u) *flag = 0u;  // plain stores of one value: no atomic needed
}

// boundary b = 0..n: the start of record b (b = n: the end of the last record)
__device__ __forceinline__ uint64_t stream_pos(const CrcParams& P, uint64_t b, uint64_t dend) {
  return b < P.nrec ? P.off[b] : dend;
}

// cut w, w = 0..W: the first boundary at or after off[0] + total*w/W
__global__ __launch_bounds__(256) void stream_cuts(CrcParams P, uint32_t W) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w > W || !*P.sflag) return;
  const uint64_t n = P.nrec, o0 = P.off[0], dend = P.off[n - 1] + P.len[n - 1];
  const uint64_t target = o0 + (dend - o0) * w / W;
  uint64_t a = 0, b = n;
  while (a < b) {
    const uint64_t m = (a + b) >> 1;
    if (stream_pos(P, m, dend) < target) a = m + 1; else b = m;
  }
  P.scuts[w] = a;
}

struct StreamWin {
  uint64_t a, b;  // off[] of boundaries bt + lane and bt + 64 + lane (clamped to n - 1; fixed up at use)
};
template <int WIN>
__device__ __forceinline__ void stream_win_issue(const CrcParams& P, uint64_t bt, uint32_t lane, StreamWin& W) {
  const uint64_t n = P.nrec, ia = bt + lane, ib = bt + 64u + lane;
  W.a = P.off[ia < n ? ia : n - 1];
  if (WIN == 0) W.b = P.off[ib < n ? ib : n - 1];
}

// the tile's 64 chunks: bytes [tb, tb + 8192) from P.base (tb >= -127, the
// chunk grid is 128-byte aligned in memory); the buffer range ends in the
// dword holding the batch's last byte, so loads past it read zeros and touch
// nothing
template <int ABLATE>
__device__ __forceinline__ void stream_issue(const CrcParams& P, int64_t tb, uintptr_t end4, uint32_t lane,
                                             uint32_t (&u)[32]) {
  const uintptr_t t0 = (uintptr_t)P.base + (uintptr_t)tb;
  const uint64_t span = end4 - t0;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(P.base + tb), (short)0, (int)(span < 0x7FFFFFFFull ? span : 0x7FFFFFFFull), 0x00020000);
  const uint32_t vo = lane * 128u;
  if (ABLATE == 2) {  // diagnostic: compute only (no payload loads; results invalid)
#pragma unroll
    for (int j = 0; j < 32; ++j) u[j] = (uint32_t)tb * 0x9E3779B1u + lane + j;
    return;
  }
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16u * g, 0, 0);
    u[4 * g + 0] = v[0];
    u[4 * g + 1] = v[1];
    u[4 * g + 2] = v[2];
    u[4 * g + 3] = v[3];
  }
  keep_live(vo);
}

__device__ __forceinline__ uint64_t wave_or_u64(uint64_t x) {
  return (uint64_t)wave_or_u32((uint32_t)x) | ((uint64_t)wave_or_u32((uint32_t)(x >> 32)) << 32);
}

// WIN: how the boundary window is read.  0: both halves (boundaries bt..bt+127)
// reloaded every tile; 1: the second half only for a tile whose 64 first
// boundaries all lie in it (no tile of config 3: at most 58); 2 (default): as
// 1, and the first half slides -- the next tile's window is this one shifted by
// the tile's boundary count (ds_bpermute), only the new entries loaded.  A tile
// of config 3 ends ~5 records, so 0 requested 1 KiB of off[] per 8 KiB tile.
// DQ (with QST): a tile's first-half records are pushed onto the queue at the
// next tile, after its payload loads are issued (as the ring kernel's order 3).
// SEL: a word's boundary branch only selects the two chains' step inputs; both
// steps follow the branch, so their eight lookups issue together (else the
// compiler split them over the branch's blocks: 1.9 ms of 21 on config 3,
// crc_ablate 9 against 4 in profiles/r02/q).
// SEL 2: no branch at all.  The boundary word's step input is known before
// the chain runs: ~(u | mlo) ^ Finv(mlo) (Finv(mlo): the word step's inverse
// of the t-byte mask, so that F of it is the step's F(~(u | mlo)) ^ mlo), with
// u the lane's word kb picked by a 16-way select; each step then selects its
// input (and the capture) on kb == k, 3 VALU per chain step.
// Z0: a tile in which no record ends (43% of config 3's tiles: records of
// 8 KiB and more) takes a short path -- straight chains, the Horner shift to
// the tile end, the carry -- without the boundary map, the word branches and
// the finish.
// LM: the chunk lanes' boundaries through LDS bytes (window lanes write, chunk
// lanes read and clear) instead of four DPP OR reductions, popcounts and
// bpermutes.
// FSP: a half with at most 16 records spreads each record's finish multiply
// over 8 lanes (4 LDS columns each, then a 3-step DPP XOR), 8 records per
// round, instead of one 32-column multiply issued for the whole wave.
template <int ABLATE = 0, int BLOCK = 1024, int SLOTS = 2, bool BATCH = false, bool QST = true, int WIN = 2,
          bool DQ = false, int SEL = 0, bool Z0 = false, bool LM = false, bool FSP = false>
__global__ __launch_bounds__(BLOCK) void crc32_stream_kernel(CrcParams P) {
  if (!*P.sflag) return;  // not a packed batch of >= 64-byte records: the walking kernel takes it
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  build_lds_tables(smem, P);
  __syncthreads();  // the walk columns reuse the khi area, x^(8m) the klo area
  build_walk_cols(P);
  if (threadIdx.x >= 128u && threadIdx.x < 196u) {  // the finish factors' columns
    const uint32_t f = threadIdx.x - 128u;
    uint32_t K, base;
    if (f < 64u) {  // x^(8m): m zero-byte steps of the register from x^0
      K = 0x80000000u;
      for (uint32_t i = 0; i < f; ++i) K = (K >> 8) ^ P.master[K & 0xFFu];
      base = LDS_XMC_OFF(f);
    } else {
      K = stream_xinv(f - 64u);
      base = LDS_XIC_OFF(f - 64u);
    }
    for (uint32_t i = 0; i < 32u; ++i) {
      *(__attribute__((address_space(3))) uint32_t*)(size_t)(base + 4u * i) = K;
      K = (K >> 1) ^ (0xEDB88320u & (0u - (K & 1u)));
    }
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lo = (lane & 31u) * 4u, hi = lo | 0x10000u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint32_t smap = LDS_SMAP_OFF + (threadIdx.x >> 6) * 128u;  // LM: this wave's boundary bytes
  if (LM && lane < 32u) *(__attribute__((address_space(3))) uint32_t*)(size_t)(smap + 4u * lane) = 0u;
  const uint64_t n = P.nrec;
  const uint64_t b_lo = P.scuts[wave], b_hi = P.scuts[wave + 1];
  if (b_lo >= b_hi) return;  // no record ends in this wave's range
  const uint64_t dend = P.off[n - 1] + P.len[n - 1];
  const uintptr_t end4 = ((uintptr_t)P.base + dend + 3u) & ~(uintptr_t)3;
  // chunk grid origin, relative to P.base (128-byte aligned in memory)
  const int64_t a0 = (int64_t)((((uintptr_t)P.base + P.off[0]) & ~(uintptr_t)127) - (uintptr_t)P.base);
  const uint64_t t_first = (uint64_t)((int64_t)stream_pos(P, b_lo, dend) - a0) >> 13;
  const uint64_t t_last = (uint64_t)((int64_t)stream_pos(P, b_hi, dend) - a0) >> 13;
  const uint64_t ntile = t_last - t_first + 1u;
  auto tbase = [&](uint64_t t) -> int64_t { return a0 + (int64_t)(t << 13); };

  StreamWin Wn;
  uint64_t bt = b_lo;  // the first boundary of the tile being mapped
  uint32_t carry = 0;  // the record crossing into the next tile, aligned to this tile's end
  // BATCH: records finished in batches of up to 64 (one per lane) instead of
  // per tile: H, R0 of the end chunk, the exact capture, j, the output index
  uint32_t qH = 0, qR = 0, qA = 0, qJ = 0, qI = 0xFFFFFFFFu, qn = 0;
  auto flush = [&]() {
    if (lane < qn && qI != 0xFFFFFFFFu) {  // per active lane: LDS reads in the record lanes only
      const bool h = qJ >= 64u;
      const uint32_t Pv = h ? (shift_bytes32<2>(smem, qH) ^ qR) : qH;
      P.out[qI] = ~(stream_mulcol(Pv, LDS_XMC_OFF(qJ & 63u)) ^ qA);
    }
    qn = 0;
  };
  // QST: the CRCs are queued in one VGPR (lane p: record qb + p, qb a
  // multiple of 64) and stored as whole 256-byte blocks.  A wave's records are
  // consecutive, so only its first and last blocks are partial.  Per-tile
  // stores of the ~5 records a tile ends wrote partial 128-byte lines: the
  // config-3 PMC counted 5.9 GB of fetches (and 2x the output's bytes written)
  // for the 0.27 GB output (profiles/r02/official_b, a3 against c0).
  uint32_t qv = 0;
  uint64_t qb = b_lo & ~63ull;
  uint32_t qs = (uint32_t)(b_lo & 63u), qf = qs;  // first valid lane of the block, next lane to fill
  auto qstore = [&](uint32_t v, bool on) {  // block qb from a uniform base: no 64-bit lane address to keep
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)(P.out + qb), (short)0, 256, 0x00020000);
    if (on) __builtin_amdgcn_raw_buffer_store_b32(v, r, lane << 2, 0, 0);
  };
  auto qpush = [&](uint32_t v, uint32_t i0, uint32_t cnt) {  // window lanes i0 .. i0+cnt-1: the next cnt records
    const uint32_t src = (lane - qf + i0) & 63u;
    const uint32_t val = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
    const uint32_t end = qf + cnt;  // cnt <= 64 - i0: at most one block completes
    qv = (lane >= qf && lane < end) ? val : qv;
    if (end >= 64u) {
      qstore(qv, lane >= qs);
      qb += 64u;
      qs = 0u;
      qf = end - 64u;
      qv = lane < qf ? val : qv;
    } else {
      qf = end;
    }
  };
  uint32_t dqv = 0, dqi0 = 0, dqcnt = 0;  // DQ: the deferred push
  stream_win_issue<WIN>(P, bt, lane, Wn);

  auto process = [&](const uint32_t (&U)[32], uint64_t t, auto&& issue_next) {
    const int64_t tb = tbase(t);
    // --- map: this tile's boundaries, bt .. bt+cnt-1 (window lanes); ra/rb:
    // tile-relative byte of boundary bt+lane / bt+64+lane (chunk = r >> 7)
    const uint64_t ia = bt + lane, ib = bt + 64u + lane;
    const int64_t ra64 = (int64_t)(ia < n ? Wn.a : dend) - tb;
    const bool ina = ia <= b_hi && ra64 < 8192;
    const uint64_t bal_a = __ballot(ina);
    int64_t rb64 = 8192;
    bool inb = false;
    if constexpr (WIN == 0) {
      rb64 = (int64_t)(ib < n ? Wn.b : dend) - tb;
      inb = ib <= b_hi && rb64 < 8192;
    } else if (bal_a == ~0ull) {  // the first 64 boundaries all end here: the next 64 may too
      const uint64_t wb = P.off[ib < n ? ib : n - 1];
      rb64 = (int64_t)(ib < n ? wb : dend) - tb;
      inb = ib <= b_hi && rb64 < 8192;
    }
    const uint32_t ra = (uint32_t)ra64 & 8191u, rb = (uint32_t)rb64 & 8191u;
    const uint64_t bal_b = __ballot(inb);
    const uint32_t na = (uint32_t)__builtin_popcountll(bal_a), nb = (uint32_t)__builtin_popcountll(bal_b);
    const uint32_t cnt = na + nb;
    const uint64_t bt0 = bt;
    bt += cnt;
    // the next tile's window (lands while this tile is checksummed)
    if constexpr (WIN == 2) {
      const uint32_t src = lane + cnt;  // lanes whose entry this window holds take it from there
      const int sp = (int)((src & 63u) << 2);
      const uint32_t wlo = (uint32_t)__builtin_amdgcn_ds_bpermute(sp, (int)(uint32_t)Wn.a);
      const uint32_t whi = (uint32_t)__builtin_amdgcn_ds_bpermute(sp, (int)(uint32_t)(Wn.a >> 32));
      Wn.a = ((uint64_t)whi << 32) | wlo;
      if (src >= 64u) {  // the new entries only
        const uint64_t i2 = bt + lane;
        Wn.a = P.off[i2 < n ? i2 : n - 1];
      }
    } else {
      stream_win_issue<WIN>(P, bt, lane, Wn);
    }
    // then the payload SLOTS-1 tiles ahead: after the window, so that waiting
    // for the window at the next tile never waits for that payload
    issue_next();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (QST && DQ) {
      if (dqcnt) qpush(dqv, dqi0, dqcnt);
      dqcnt = 0;
    }
    if constexpr (Z0 && ABLATE == 0 && !BATCH) {
      if (cnt == 0u) {  // (uniform) no boundary in the tile
        // the carry (the record's raw CRC up to this tile, aligned to its start)
        // enters as lane 0's initial register: the Horner shift of lane 0 then
        // carries it to the tile end with the chunk (no separate multiply)
        uint32_t z0 = U[0] ^ (lane == 0u ? carry : 0u), z1 = U[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          z0 = crc_step_x(smem, z0, k + 1 < 16 ? U[k + 1] : 0u, lo, hi);
          z1 = crc_step_x(smem, z1, k + 1 < 16 ? U[17 + k] : 0u, lo, hi);
        }
        uint32_t dz = 63u - lane;
        asm volatile("" : "+v"(dz));  // not hoisted: eight loop-invariant column addresses spilled
        const uint32_t XZ = wave_prefix_xor(walk_mulcol(shift_bytes32<2>(smem, z0) ^ z1, dz));
        carry = (uint32_t)__builtin_amdgcn_readlane((int)XZ, 63);
        return;
      }
    }
    uint64_t M1, M2;
    bool any2;
    uint32_t jc0, jc1;
    if constexpr (LM) {
      const uint32_t ca = ra >> 7, cb = rb >> 7;
      const uint32_t ca63 = (uint32_t)__builtin_amdgcn_readlane((int)ca, 63);
      const uint32_t pca = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ca, 0x138, 0xF, 0xF, false);  // wave_shr:1
      const uint32_t pcb0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cb, 0x138, 0xF, 0xF, false);
      const uint32_t pcb = lane ? pcb0 : ca63;
      const bool seca = ina && lane > 0u && pca == ca;
      const bool secb = inb && pcb == cb && (lane > 0u || (bal_a >> 63));
      typedef __attribute__((address_space(3))) unsigned char lds_u8w_t;
      typedef __attribute__((address_space(3))) unsigned short lds_u16w_t;
      if (ina) *(lds_u8w_t*)(size_t)(smap + 2u * ca + (seca ? 1u : 0u)) = (unsigned char)((ra & 127u) + 1u);
      if (inb) *(lds_u8w_t*)(size_t)(smap + 2u * cb + (secb ? 1u : 0u)) = (unsigned char)((rb & 127u) + 1u);
      const uint32_t e = *(lds_u16w_t*)(size_t)(smap + 2u * lane);
      if (e) *(lds_u16w_t*)(size_t)(smap + 2u * lane) = (unsigned short)0;
      const uint32_t e1 = e & 0xFFu, e2 = e >> 8;
      M1 = __ballot(e1 != 0u);
      M2 = __ballot(e2 != 0u);
      any2 = M2 != 0ull;
      const uint32_t j1 = e1 - 1u;
      jc0 = (e1 && j1 < 64u) ? j1 : 128u;
      jc1 = e2 ? e2 - 1u : ((e1 && j1 >= 64u) ? j1 : 128u);
    } else {
      const uint32_t ca = ra >> 7, cb = rb >> 7;
      const uint32_t ca63 = (uint32_t)__builtin_amdgcn_readlane((int)ca, 63);
      const uint32_t pca = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ca, 0x138, 0xF, 0xF, false);  // wave_shr:1
      const uint32_t pcb0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cb, 0x138, 0xF, 0xF, false);
      const uint32_t pcb = lane ? pcb0 : ca63;
      const bool seca = ina && lane > 0u && pca == ca;
      const bool secb = inb && pcb == cb && (lane > 0u || (bal_a >> 63));
      M1 = wave_or_u64(((ina && !seca) ? (1ull << ca) : 0ull) | ((inb && !secb) ? (1ull << cb) : 0ull));
      any2 = __any(seca || secb);
      M2 = any2 ? wave_or_u64((seca ? (1ull << ca) : 0ull) | (secb ? (1ull << cb) : 0ull)) : 0ull;
    }
    // --- chunk-lane view: this chunk's boundaries jc0 (chain 0), jc1 (chain 1); 128 = none
    if constexpr (!LM) {
      const uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
      const uint32_t k1 = (uint32_t)__builtin_popcountll(M1 & below) + (uint32_t)__builtin_popcountll(M2 & below);
      const bool b1 = (M1 >> lane) & 1ull, b2 = (M2 >> lane) & 1ull;
      const int s1 = (int)((k1 & 63u) << 2);
      const uint32_t j1a = (uint32_t)__builtin_amdgcn_ds_bpermute(s1, (int)ra);
      const uint32_t j1b = (uint32_t)__builtin_amdgcn_ds_bpermute(s1, (int)rb);
      const uint32_t j1 = (k1 < 64u ? j1a : j1b) & 127u;
      uint32_t j2 = 128u;
      if (any2) {
        const uint32_t k2 = k1 + 1u;
        const int s2 = (int)((k2 & 63u) << 2);
        const uint32_t j2a = (uint32_t)__builtin_amdgcn_ds_bpermute(s2, (int)ra);
        const uint32_t j2b = (uint32_t)__builtin_amdgcn_ds_bpermute(s2, (int)rb);
        j2 = b2 ? ((k2 < 64u ? j2a : j2b) & 127u) : 128u;
      }
      jc0 = (b1 && j1 < 64u) ? j1 : 128u;
      jc1 = b2 ? j2 : ((b1 && j1 >= 64u) ? j1 : 128u);
    }
    // (ABLATE 4, diagnostic: no boundary bodies; results invalid)
    // (ABLATE 9, diagnostic: the boundary branches kept, never taken; results invalid)
    const uint32_t kz = ABLATE == 9 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(P.nrec >> 62)) : 0u;
    // the words holding a boundary, chain 0 in bits 0-15 and chain 1 in bits
    // 16-31: one OR over the window's boundaries (at most one per chain and
    // chunk) instead of one per chain over the chunk lanes
    const uint32_t Kw = (ABLATE == 4 || ABLATE == 9 || SEL == 2)
                            ? 0u
                            : wave_or_u32((ina ? (1u << ((ra & 127u) >> 2)) : 0u) | (inb ? (1u << ((rb & 127u) >> 2)) : 0u));
    const uint32_t Km0 = ABLATE == 4 ? 0u : ABLATE == 9 ? kz
                         : SEL == 2 ? (uint32_t)(__ballot(jc0 < 128u) != 0ull) : (Kw & 0xFFFFu);
    const uint32_t Km1 = ABLATE == 4 ? 0u : ABLATE == 9 ? kz
                         : SEL == 2 ? (uint32_t)(__ballot(jc1 < 128u) != 0ull) : (Kw >> 16);
    if (ABLATE == 3) {  // diagnostic: payload loads only
      uint32_t x = 0;
#pragma unroll
      for (int k = 0; k < 32; ++k) x ^= U[k];
      if (x == 0x9E3779B1u) P.out[0] = x ^ jc0 ^ jc1;
      return;
    }
    // --- the chunk's two chains, with the register resets at its boundaries.
    // A record starting at byte t of word u resets the chain: the register
    // after the word is F(~(u | mlo)) ^ mlo (mlo: the t bytes before the
    // boundary; the 0xFFFFFFFF init folded in), so the boundary lane only
    // swaps the input of its ordinary word step -- no extra lookups -- and
    // keeps c ^ u and u of that word for its capture.
    // Z0 (carry in): the carry enters as lane 0's initial register here too.
    // Up to the tile's first boundary it then rides in lane 0's chain: into
    // the capture (a boundary in chain 0 of chunk 0), R0 (one in chain 1), or
    // the Horner value of chunk 0; a reset drops it after the boundary, so no
    // record but the carried one sees it
    uint32_t c0 = U[0] ^ ((Z0 && lane == 0u) ? carry : 0u), c1 = U[16], x0 = 0u, x1 = 0u, ub0 = 0u, ub1 = 0u;
    const uint32_t Km = Km0 | Km1;
    uint32_t kb0 = 32u, kb1 = 32u, s0 = 0u, s1 = 0u;
    if constexpr (SEL == 2) {
      // U[base + kb], kb < 16, as a tree of bitwise selects (v_bitop3 0xCA:
      // m ? a : b per bit): written as ?: selects, hipcc turned the tree into
      // an indexed scratch array of the payload registers
      auto pick16 = [&](uint32_t kb, int base) -> uint32_t {
        auto bsel = [](uint32_t m, uint32_t a, uint32_t b) { return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA); };
        const uint32_t m1 = 0u - (kb & 1u), m2 = 0u - ((kb >> 1) & 1u), m4 = 0u - ((kb >> 2) & 1u),
                       m8 = 0u - ((kb >> 3) & 1u);
        uint32_t a[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) a[q] = bsel(m1, U[base + 2 * q + 1], U[base + 2 * q]);
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = bsel(m2, a[2 * q + 1], a[2 * q]);
#pragma unroll
        for (int q = 0; q < 2; ++q) a[q] = bsel(m4, a[2 * q + 1], a[2 * q]);
        return bsel(m8, a[1], a[0]);
      };
      auto finv = [](uint32_t t) -> uint32_t {  // Finv of the t-byte mask (1 << 8t) - 1
        return t == 1u ? 0x0f6a70d9u : (t == 2u ? 0x65e39d90u : (t == 3u ? 0x5c2e2681u : 0u));
      };
      kb0 = jc0 >> 2;          // 32: no boundary in chain 0
      kb1 = (jc1 >> 2) - 16u;  // 16: none in chain 1
      ub0 = pick16(kb0 & 15u, 0);
      ub1 = pick16(kb1 & 15u, 16);
      const uint32_t t0 = jc0 & 3u, t1 = jc1 & 3u;
      s0 = ~(ub0 | ((1u << (t0 << 3)) - 1u)) ^ finv(t0);
      s1 = ~(ub1 | ((1u << (t1 << 3)) - 1u)) ^ finv(t1);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t w0 = k + 1 < 16 ? U[k + 1] : 0u, w1 = k + 1 < 16 ? U[17 + k] : 0u;
      if constexpr (SEL == 2) {
        const bool m0 = kb0 == (uint32_t)k, m1 = kb1 == (uint32_t)k;
        x0 = m0 ? c0 : x0;
        x1 = m1 ? c1 : x1;
        c0 = crc_step_x(smem, m0 ? s0 : c0, w0, lo, hi);
        c1 = crc_step_x(smem, m1 ? s1 : c1, w1, lo, hi);
        continue;
      }
      if constexpr (SEL == 1) {
        uint32_t i0 = c0, i1 = c1, n0 = w0, n1 = w1;
        if (Km & (1u << k)) {  // wave-uniform: some lane's chain has a boundary in word k
          uint32_t j0 = jc0, j1 = jc1;
          asm volatile("" : "+v"(j0), "+v"(j1));
          const bool m0 = (j0 >> 2) == (uint32_t)k, m1 = (j1 >> 2) == (uint32_t)(16 + k);
          const uint32_t mlo0 = (1u << ((j0 & 3u) << 3)) - 1u, mlo1 = (1u << ((j1 & 3u) << 3)) - 1u;
          x0 = m0 ? c0 : x0;
          ub0 = m0 ? U[k] : ub0;
          x1 = m1 ? c1 : x1;
          ub1 = m1 ? U[16 + k] : ub1;
          i0 = m0 ? ~(U[k] | mlo0) : c0;
          n0 = m0 ? (w0 ^ mlo0) : w0;
          i1 = m1 ? ~(U[16 + k] | mlo1) : c1;
          n1 = m1 ? (w1 ^ mlo1) : w1;
        }
        c0 = crc_step_x(smem, i0, n0, lo, hi);
        c1 = crc_step_x(smem, i1, n1, lo, hi);
        continue;
      }
      if (Km & (1u << k)) {  // wave-uniform: some lane's chain has a boundary in word k
        uint32_t j0 = jc0, j1 = jc1;
        asm volatile("" : "+v"(j0), "+v"(j1));  // recomputed here, not hoisted: fewer VGPRs through the loop
        const bool m0 = (j0 >> 2) == (uint32_t)k, m1 = (j1 >> 2) == (uint32_t)(16 + k);
        const uint32_t mlo0 = (1u << ((j0 & 3u) << 3)) - 1u, mlo1 = (1u << ((j1 & 3u) << 3)) - 1u;
        x0 = m0 ? c0 : x0;
        ub0 = m0 ? U[k] : ub0;
        x1 = m1 ? c1 : x1;
        ub1 = m1 ? U[16 + k] : ub1;
        c0 = crc_step_x(smem, m0 ? ~(U[k] | mlo0) : c0, m0 ? (w0 ^ mlo0) : w0, lo, hi);
        c1 = crc_step_x(smem, m1 ? ~(U[16 + k] | mlo1) : c1, m1 ? (w1 ^ mlo1) : w1, lo, hi);
      } else {
        c0 = crc_step_x(smem, c0, w0, lo, hi);
        c1 = crc_step_x(smem, c1, w1, lo, hi);
      }
    }
    const uint32_t cap0 = Km0 ? stream_capture(smem, x0, ub0, jc0 & 3u, lo) : 0u;
    const uint32_t cap1 = Km1 ? stream_capture(smem, x1, ub1, jc1 & 3u, lo) : 0u;
    const uint32_t R0 = c0;
    const uint32_t T = (jc1 < 128u) ? c1 : (shift_bytes32<2>(smem, c0) ^ c1);
    // --- Horner inside the tile: T to the chunk before the next boundary's chunk
    const uint64_t above = lane == 63u ? 0ull : (M1 >> (lane + 1u)) << (lane + 1u);
    const uint32_t cn = above ? (uint32_t)__builtin_ctzll(above) : 64u;
    // (ABLATE 6, diagnostic: no per-lane Horner shift)
    const uint32_t X = wave_prefix_xor(ABLATE == 6 ? (T ^ cn) : walk_mulcol(T, cn - 1u - lane));
    // --- records: window lane i finishes the record that ends at boundary bt0 + i
    const uint32_t ca = ra >> 7, cb = rb >> 7;
    const uint32_t c00 = (uint32_t)__builtin_amdgcn_readfirstlane((int)ca);
    const uint32_t cterm = (Z0 || !na) ? 0u : walk_mulcol_uniform<Z0>(carry, c00, lane);
    // Y = X[c-1] of the window lane's end chunk c; the record began at the
    // previous window lane's chunk, whose Y is one DPP shift away (lane 0:
    // `first`, the carry term or the other half's last Y)
    auto finish = [&](bool in, uint32_t r, uint32_t first, uint64_t bidx, uint32_t i0, uint32_t cnt,
                      bool half_b) -> uint32_t {
      const uint32_t c = r >> 7, j = r & 127u;
      const uint32_t Xc = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((c - 1u) & 63u) << 2), (int)X);
      const uint32_t Y = c ? Xc : 0u;
      const uint32_t Yp = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)Y, 0x138, 0xF, 0xF, false);  // wave_shr:1
      const uint32_t H = Y ^ (lane ? Yp : first);
      const int sc = (int)(c << 2);
      const uint32_t R0c = (uint32_t)__builtin_amdgcn_ds_bpermute(sc, (int)R0);
      const uint32_t A0c = (uint32_t)__builtin_amdgcn_ds_bpermute(sc, (int)cap0);
      const uint32_t A1c = (uint32_t)__builtin_amdgcn_ds_bpermute(sc, (int)cap1);
      if constexpr (BATCH) {
        // append this half's record lanes (window lanes 0..m-1) to the queue
        const uint32_t m = (uint32_t)__builtin_popcountll(__ballot(in));
        if (qn + m > 64u) flush();
        const int sh = (int)(((lane - qn) & 63u) << 2);
        const uint32_t sH = (uint32_t)__builtin_amdgcn_ds_bpermute(sh, (int)H);
        const uint32_t sR = (uint32_t)__builtin_amdgcn_ds_bpermute(sh, (int)R0c);
        const uint32_t sA = (uint32_t)__builtin_amdgcn_ds_bpermute(sh, (int)(j >= 64u ? A1c : A0c));
        const uint32_t sJ = (uint32_t)__builtin_amdgcn_ds_bpermute(sh, (int)j);
        const uint32_t sI = (uint32_t)__builtin_amdgcn_ds_bpermute(
            sh, (int)((in && bidx > b_lo) ? (uint32_t)(bidx - 1u) : 0xFFFFFFFFu));
        const bool take = lane >= qn && lane < qn + m;
        qH = take ? sH : qH;
        qR = take ? sR : qR;
        qA = take ? sA : qA;
        qJ = take ? sJ : qJ;
        qI = take ? sI : qI;
        qn += m;
        return Y;
      }
      // only the lanes holding a record from here on (a few per tile): the LDS
      // reads below cost per active lane, and all 64 lanes doing them cost
      // 4.8 of 25.6 ms (crc_ablate 5); the bpermutes above need every lane
      uint32_t fv = 0u;
      if (FSP && ABLATE == 0 && cnt <= 16u) {  // (uniform)
        uint32_t pv = 0u, av = 0u, mf = 0u;
        if (in && bidx > b_lo) {
          const bool h = j >= 64u;
          pv = h ? (shift_bytes32<2>(smem, H) ^ R0c) : H;
          av = h ? A1c : A0c;
          mf = LDS_XMC_OFF(j & 63u);  // the factor x^(8m)'s 32 columns
        }
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));  // lane-derived offsets recomputed here, not held across the tile loop (spilled)
        for (uint32_t q = 0; q < cnt; q += 8u) {
          // lane L works on record lane i0 + q + L/8, columns 4(L%8) .. +3
          const int src = (int)(((i0 + q + (ln >> 3)) & 63u) << 2);
          const uint32_t p = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pv);
          const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)mf);
          const uint32_t g = ln & 7u;
          const u32x4 c = lds_ld128(b + g * 16u);
          const uint32_t ps = p << (g << 2);
          uint32_t x = c.x & (uint32_t)((int32_t)ps >> 31);
          x = __builtin_amdgcn_bitop3_b32(x, c.y, (uint32_t)((int32_t)(ps << 1) >> 31), 0x78);
          x = __builtin_amdgcn_bitop3_b32(x, c.z, (uint32_t)((int32_t)(ps << 2) >> 31), 0x78);
          x = __builtin_amdgcn_bitop3_b32(x, c.w, (uint32_t)((int32_t)(ps << 3) >> 31), 0x78);
          x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
          x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
          x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4: group total at L%8 >= 4
          const uint32_t d = ln - i0 - q;  // this round's record lanes: d < 8
          const uint32_t got = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((((d << 3) + 4u) & 63u) << 2), (int)x);
          fv = (d < 8u && d < cnt - q) ? ~(got ^ av) : fv;
        }
      } else if (in && bidx > b_lo) {
        const bool h = j >= 64u;
        const uint32_t Pv = h ? (shift_bytes32<2>(smem, H) ^ R0c) : H;
        uint32_t v;
        if (ABLATE == 8) {  // diagnostic: no finish multiply (results invalid)
          v = Pv ^ (h ? A1c : A0c);
        } else if (ABLATE == 7) {  // A/B: the multiplies on the VALU (factors from LDS column 0)
          v = gf2_mulmod(Pv, lds_ld(smem, LDS_XMC_OFF(j & 63u))) ^ gf2_mulmod(h ? A1c : A0c, lds_ld(smem, LDS_XIC_OFF(j & 3u)));
        } else {
          // the capture is exact (the chain's bytes before j): one multiply
          v = stream_mulcol(Pv, LDS_XMC_OFF(j & 63u)) ^ (h ? A1c : A0c);
        }
        fv = ~v;
        if constexpr (!QST) P.out[bidx - 1u] = fv;
      }
      if constexpr (QST && DQ) {
        if (half_b) {  // (rare) the first half's records go first
          if (dqcnt) qpush(dqv, dqi0, dqcnt);
          dqcnt = 0;
          if (cnt) qpush(fv, i0, cnt);
        } else {
          dqv = fv;
          dqi0 = i0;
          dqcnt = cnt;
        }
      } else if constexpr (QST) {
        if (cnt) qpush(fv, i0, cnt);
      }
      return Y;
    };
    if (ABLATE == 5) {  // diagnostic: no record finish (one store keeps the tile's work alive)
      if (X == 0x9E3779B1u) P.out[0] = X ^ R0 ^ cap0 ^ cap1;
    } else {
      // record lanes: window lanes with a boundary after b_lo (only lane 0 of
      // the wave's first tile is not one)
      const uint32_t i0 = bt0 == b_lo ? 1u : 0u;
      const uint32_t Ya = finish(ina, ra, cterm, bt0 + lane, i0, na > i0 ? na - i0 : 0u, false);
      if (nb) finish(inb, rb, (uint32_t)__builtin_amdgcn_readlane((int)Ya, 63), bt0 + 64u + lane, 0u, nb, true);
    }
    // --- carry: the record active at the tile's end
    const uint32_t X63 = (uint32_t)__builtin_amdgcn_readlane((int)X, 63);
    if (cnt) {
      const uint32_t cl = nb ? (uint32_t)__builtin_amdgcn_readlane((int)cb, (int)(nb - 1u))
                             : (uint32_t)__builtin_amdgcn_readlane((int)ca, (int)(na - 1u));
      carry = X63 ^ (cl ? (uint32_t)__builtin_amdgcn_readlane((int)X, (int)(cl - 1u)) : 0u);
    } else {
      carry = X63 ^ (Z0 ? 0u : walk_mulcol_uniform<Z0>(carry, 64u, lane));
    }
  };

  // payload slots: SLOTS - 1 tiles in flight while one is checksummed; tiles
  // past the run reload its last tile (in bounds, unused)
  auto tcl = [&](uint64_t x) -> int64_t { return tbase(x < ntile ? t_first + x : t_last); };
  auto none = [] {};
  uint32_t U0[32], U1[32];
  stream_issue<ABLATE>(P, tcl(0), end4, lane, U0);
  uint64_t i = 0;
  if constexpr (SLOTS == 3) {
    uint32_t U2[32];
    stream_issue<ABLATE>(P, tcl(1), end4, lane, U1);
    for (; i + 3 <= ntile; i += 3) {
      process(U0, t_first + i, [&] { stream_issue<ABLATE>(P, tcl(i + 2), end4, lane, U2); });
      process(U1, t_first + i + 1, [&] { stream_issue<ABLATE>(P, tcl(i + 3), end4, lane, U0); });
      process(U2, t_first + i + 2, [&] { stream_issue<ABLATE>(P, tcl(i + 4), end4, lane, U1); });
    }
    if (i < ntile) process(U0, t_first + i, none);
    if (i + 1 < ntile) process(U1, t_first + i + 1, none);
  } else {
    for (; i + 2 <= ntile; i += 2) {
      process(U0, t_first + i, [&] { stream_issue<ABLATE>(P, tcl(i + 1), end4, lane, U1); });
      process(U1, t_first + i + 1, [&] { stream_issue<ABLATE>(P, tcl(i + 2), end4, lane, U0); });
    }
    if (i < ntile) process(U0, t_first + i, none);
  }
  if constexpr (BATCH) flush();
  if constexpr (QST && !BATCH) {
    if constexpr (DQ) {
      if (dqcnt) qpush(dqv, dqi0, dqcnt);
    }
    qstore(qv, lane >= qs && lane < qf);
  }
}
}  // namespace lsmck

// ---------------------------------------------------------------------------
// Launchers (C linkage inside the library; the public C ABI is lsmck_api.cpp)
using namespace lsmck;


template <bool FAST, int CHAINS, int ABLATE = 0, bool PERCOL = false, bool BUF = false>
static int launch_fixed(const CrcParams* P, int ncu, hipStream_t st) {
  size_t lds = LDS_SCRATCH_OFF;
  hipError_t e = hipFuncSetAttribute((const void*)crc32_fixed_kernel<FAST, CHAINS, ABLATE, PERCOL, BUF>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  hipLaunchKernelGGL((crc32_fixed_kernel<FAST, CHAINS, ABLATE, PERCOL, BUF>), dim3(ncu), dim3(1024), lds, st, *P);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

template <int R, int ABLATE = 0, int BLOCK = 1024, int ORDER = 0, bool QST = false>
static int launch_wring(const CrcParams* P, int ncu, hipStream_t st) {
  size_t lds = LDS_SCRATCH_OFF + (ORDER == 4 ? LDS_WOUT_BYTES : 0u);
  hipError_t e = hipFuncSetAttribute((const void*)crc32_wring_kernel<R, ABLATE, BLOCK, ORDER, QST>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  if (ORDER == 2) {
    if (!P->work) return -(int)hipErrorInvalidValue;
    e = hipMemsetAsync(P->work, 0, 4, st);
    if (e != hipSuccess) return -(int)e;
  }
  hipLaunchKernelGGL((crc32_wring_kernel<R, ABLATE, BLOCK, ORDER, QST>), dim3(ncu), dim3(BLOCK), lds, st, *P);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

// variant: number of independent CRC chains per lane (1, 2, 4); 0 = default
extern "C" int lsmk_launch_crc32_fixed(const CrcParams* P, int ncu, int variant, hipStream_t st) {
  bool fast = ((uintptr_t)P->base % 4 == 0) && (P->stride % 4 == 0) && (P->flen % 128 == 0);
  int ch = (variant & 0xF) ? (variant & 0xF) : LSMCK_DEFAULT_CHAINS;
  int ablate = (variant >> 8) & 0xF;  // diagnostic ablations (results invalid): 1 loads only, 2 compute only
  if (fast && ablate == 1) return launch_fixed<true, 2, 1>(P, ncu, st);
  if (fast && ablate == 2) return launch_fixed<true, 2, 2>(P, ncu, st);
  // per-lane shift columns when every tile starts on a record boundary (and k < 2^16)
  const uint32_t nsegr = (P->flen + 127u) >> 7;
  const bool percol = (64u % nsegr) == 0 && !(variant & 0x10);  // 0x10: force the generic multiply (A/B)
  // buffer loads: every tile's segments within 2^31 bytes of its first record
  // (64 records of the stride); 0x40 forces global loads, 0x80 buffer loads
  const bool buf_ok = (uint64_t)P->stride * 65u + P->flen < (1ull << 31);
  // default: buffer loads with loop-invariant offsets where every tile starts on
  // a record boundary (percol); per-tile offsets measured no faster than global
  // loads (profiles/r01/ablations.md), so the other layouts keep global loads
  const bool buf = buf_ok && ((variant & 0x80) || (LSMCK_DEFAULT_BUFLOADS && percol && !(variant & 0x40)));
  // ring kernel (variant bits 12-15: 1 = the two-slot kernel below, 2 or 3 =
  // whole-tile ring of that many slots; 0 = LSMCK_DEFAULT_RING)
  const int ring = ((variant >> 12) & 0xF) ? ((variant >> 12) & 0xF) : LSMCK_DEFAULT_RING;
  if (fast && percol && buf && ring >= 2 && (ablate == 0 || ablate == 3 || ablate == 14 || ablate == 15)) {
    const int osel14 = (variant >> 24) & 7, order14 = osel14 ? osel14 - 1 : LSMCK_DEFAULT_ORDER;
    if (ablate == 14 && order14 == 0) return launch_wring<2, 14>(P, ncu, st);  // diagnostic: no output store
    if (ablate == 15 && order14 == 0) return launch_wring<2, 15>(P, ncu, st);  // diagnostic: L2-hit stores
    if (ablate == 14 && order14 == 3) return launch_wring<2, 14, 1024, 1, true>(P, ncu, st);
    if (variant & 0x20) {  // 12-wave workgroups (168 VGPRs per lane): A/B of the 3-slot ring
      if (ring == 2) return launch_wring<2, 0, 768>(P, ncu, st);
      return ablate ? launch_wring<3, 3, 768>(P, ncu, st) : launch_wring<3, 0, 768>(P, ncu, st);
    }
    // tile order (variant bits 24-25): 0 strided, 1 contiguous per wave, 2 claimed blocks
    const int osel = (variant >> 24) & 7, order = osel ? osel - 1 : LSMCK_DEFAULT_ORDER;
    if (ring == 2 && order == 1 && ablate == 14) return launch_wring<2, 14, 1024, 1>(P, ncu, st);
    if (ring == 2 && order == 1) return ablate ? launch_wring<2, 3, 1024, 1>(P, ncu, st) : launch_wring<2, 0, 1024, 1>(P, ncu, st);
    if (ring == 2 && order == 5) return ablate ? launch_wring<2, 3>(P, ncu, st) : launch_wring<2, 0, 1024, 5>(P, ncu, st);
    if (ring == 2 && order == 4 && (P->flen >> 7) >= 16u)  // <= 4 records per tile
      return ablate ? launch_wring<2, 3, 1024, 4>(P, ncu, st) : launch_wring<2, 0, 1024, 4>(P, ncu, st);
    if (ring == 2 && order == 3) return ablate ? launch_wring<2, 3, 1024, 1>(P, ncu, st) : launch_wring<2, 0, 1024, 1, true>(P, ncu, st);
    if (ring == 2 && order == 2) return ablate ? launch_wring<2, 3, 1024, 2>(P, ncu, st) : launch_wring<2, 0, 1024, 2>(P, ncu, st);
    if (ring == 2) return ablate ? launch_wring<2, 3>(P, ncu, st) : launch_wring<2, 0>(P, ncu, st);
    return ablate ? launch_wring<3, 3>(P, ncu, st) : launch_wring<3, 0>(P, ncu, st);
  }
  if (fast && ablate == 3 && buf && percol) return launch_fixed<true, 2, 3, true, true>(P, ncu, st);
  if (fast && ablate == 3 && buf) return launch_fixed<true, 2, 3, false, true>(P, ncu, st);
  if (fast && ablate == 3) return launch_fixed<true, 2, 3>(P, ncu, st);
  if (fast && percol && buf) {
    if (ch == 1) return launch_fixed<true, 1, 0, true, true>(P, ncu, st);
    if (ch == 2) return launch_fixed<true, 2, 0, true, true>(P, ncu, st);
    return launch_fixed<true, 4, 0, true, true>(P, ncu, st);
  }
  if (fast && percol) {
    if (ch == 1) return launch_fixed<true, 1, 0, true>(P, ncu, st);
    if (ch == 2) return launch_fixed<true, 2, 0, true>(P, ncu, st);
    return launch_fixed<true, 4, 0, true>(P, ncu, st);
  }
  if (fast && buf) {
    if (ch == 1) return launch_fixed<true, 1, 0, false, true>(P, ncu, st);
    if (ch == 2) return launch_fixed<true, 2, 0, false, true>(P, ncu, st);
    return launch_fixed<true, 4, 0, false, true>(P, ncu, st);
  }
  if (fast) {
    if (ch == 1) return launch_fixed<true, 1>(P, ncu, st);
    if (ch == 2) return launch_fixed<true, 2>(P, ncu, st);
    return launch_fixed<true, 4>(P, ncu, st);
  }
  if (ch == 1) return launch_fixed<false, 1>(P, ncu, st);
  if (ch == 2) return launch_fixed<false, 2>(P, ncu, st);
  return launch_fixed<false, 4>(P, ncu, st);
}

extern "C" uint64_t lsmk_scan_block_count(uint64_t n) { return (n + SCAN_RECS - 1) / SCAN_RECS; }

// phase 1+2: block sums and the total segment count (device, u64)
extern "C" int lsmk_launch_crc32_scan(const CrcParams* P, uint64_t* block_sum, hipStream_t st) {
  uint64_t n = P->nrec;
  uint32_t nb = (uint32_t)lsmk_scan_block_count(n);
  hipLaunchKernelGGL(scan_phase1, dim3(nb), dim3(SCAN_BLOCK), 0, st, P->len, n, block_sum);
  hipLaunchKernelGGL(scan_phase2, dim3(1), dim3(1024), 0, st, block_sum, nb, P->total_segs, (const uint32_t*)nullptr);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

// phase 3 (tile_info) and the checksum kernel; tile_info must hold
// ceil(total/64) zeroed 16-byte entries and total < 2^32
extern "C" int lsmk_launch_crc32_desc(const CrcParams* P, const uint64_t* block_sum, int ncu, int variant,
                                      hipStream_t st) {
  uint64_t n = P->nrec;
  hipLaunchKernelGGL(scan_phase3, dim3((unsigned)lsmk_scan_block_count(n)), dim3(SCAN_BLOCK), 0, st, P->len, n,
                     block_sum, P->tile_info);
  size_t lds = LDS_SCRATCH_OFF;
  int ch = (variant & 0xF) ? (variant & 0xF) : LSMCK_DEFAULT_DESC_CHAINS;
  int ablate = (variant >> 8) & 0xF;
  // 0x20: 12-wave workgroups (168 VGPRs per lane instead of 128)
  const bool w12 = (variant & 0x20) != 0;
  const int block = w12 ? 768 : 1024;
  const void* fn = w12 ? (ablate == 1 ? (const void*)crc32_desc_kernel<1, 1, 768>
                          : ablate == 3 ? (const void*)crc32_desc_kernel<1, 3, 768>
                          : ablate == 2 ? (const void*)crc32_desc_kernel<1, 2, 768>
                          : ch == 1 ? (const void*)crc32_desc_kernel<1, 0, 768>
                          : ch == 2 ? (const void*)crc32_desc_kernel<2, 0, 768> : (const void*)crc32_desc_kernel<4, 0, 768>)
                       : (ablate == 1 ? (const void*)crc32_desc_kernel<1, 1>
                          : ablate == 3 ? (const void*)crc32_desc_kernel<1, 3>
                          : ablate == 4 ? (const void*)crc32_desc_kernel<1, 4>
                          : ablate == 5 ? (const void*)crc32_desc_kernel<1, 5>
                          : ablate == 6 ? (const void*)crc32_desc_kernel<1, 6>
                          : ablate == 7 ? (const void*)crc32_desc_kernel<1, 7>
                          : ablate == 2 ? (const void*)crc32_desc_kernel<1, 2>
                          : ablate == 8 ? (const void*)crc32_desc_kernel<2, 8>
                          : ablate == 9 ? (const void*)crc32_desc_kernel<2, 9>
                          : ablate == 10 ? (const void*)crc32_desc_kernel<2, 10>
                          : ablate == 11 ? (const void*)crc32_desc_kernel<2, 2>
                          : ablate == 12 ? (const void*)crc32_desc_kernel<1, 12>
                          : ablate == 13 ? (const void*)crc32_desc_kernel<2, 13>
                          : ablate == 14 ? (const void*)crc32_desc_kernel<2, 14>
                          : ch == 1 ? (const void*)crc32_desc_kernel<1>
                          : ch == 2 ? (const void*)crc32_desc_kernel<2> : (const void*)crc32_desc_kernel<4>);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  void* args[] = {(void*)P};
  e = hipLaunchKernel(fn, dim3(ncu), dim3(block), args, lds, st);
  if (e != hipSuccess) return -(int)e;
  e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}


extern "C" uint32_t lsmk_stream_waves(int ncu) { return (uint32_t)ncu * 16u; }

// stream kernel: eligibility flag, per-wave cuts, the kernel.  The walking
// kernel launched after it on the same stream exits when the flag is set.
extern "C" int lsmk_launch_crc32_stream(const CrcParams* P, int ncu, int variant, int variant2, hipStream_t st) {
  const uint64_t n = P->nrec;
  if (n == 0) return 0;
  hipError_t e = hipMemsetAsync(P->sflag, 1, 4, st);
  if (e != hipSuccess) return -(int)e;
  hipLaunchKernelGGL(stream_check, dim3((unsigned)((n + 1023) / 1024)), dim3(1024), 0, st, P->off, P->len, n, P->sflag);
  // 0x20: 12-wave workgroups (168 VGPRs per lane instead of 128)
  const bool w12 = (variant & 0x20) != 0;
  const int block = w12 ? 768 : 1024;
  const uint32_t W = (uint32_t)ncu * (uint32_t)(block / 64);
  hipLaunchKernelGGL(stream_cuts, dim3((W + 1u + 255u) / 256u), dim3(256), 0, st, *P, W);
  const int ablate = (variant >> 8) & 0xF;
  const bool batch = (variant & 0x800000) != 0;  // A/B: batched record finish
  const bool tstore = (variant & 0x20000000) != 0;  // A/B: per-tile stores instead of queued 256-B blocks
  const int win = 2 - (int)((variant >> 27) & 3u);  // A/B: boundary window form (crc_stream_window)
  const bool dq = (variant & 0x40000000) == 0;       // deferred queue push (A/B: crc_stream_qstore 1 = at once)
  const bool sel = (variant & 0x40000) == 0;          // boundary branches select the step inputs (A/B: crc_stream_sel 0)
  const bool sel2 = (variant & 0x80000) != 0;         // A/B: branch-free boundary steps (crc_stream_sel 2)
  const bool z0 = (variant & 0x20000) == 0;           // short path for tiles without a boundary (A/B: crc_stream_z0 0)
  const bool lm = (variant2 & 0x1) == 0;              // chunk boundaries through LDS bytes (A/B: crc_stream_lm 0)
  const bool fsp = (variant2 & 0x2) != 0;             // A/B: finish multiplies spread over 8 lanes (crc_stream_fsp)
  const void* fn = batch ? (w12 ? (const void*)crc32_stream_kernel<0, 768, 2, true>
                                : (const void*)crc32_stream_kernel<0, 1024, 2, true>)
                 : (tstore && !w12 && ablate == 0) ? (const void*)crc32_stream_kernel<0, 1024, 2, false, false>
                 : (win == 1 && !w12 && ablate == 0) ? (const void*)crc32_stream_kernel<0, 1024, 2, false, true, 1>
                 : (win == 0 && !w12 && ablate == 0) ? (const void*)crc32_stream_kernel<0, 1024, 2, false, true, 0>
                 : (dq && !w12 && ablate == 0 && sel2) ? (const void*)crc32_stream_kernel<0, 1024, 2, false, true, 2, true, 2>
                 : (dq && !w12 && ablate == 0 && sel && z0 && lm && fsp) ? (const void*)crc32_stream_kernel<0, 1024, 2, false, true, 2, true, 1, true, true, true>
                 : (dq && !w12 && ablate == 0 && sel && z0 && lm) ? (const void*)crc32_stream_kernel<0, 1024, 2, false, true, 2, true, 1, true, true>
                 : (dq && !w12 && ablate == 0 && sel && z0) ? (const void*)crc32_stream_kernel<0, 1024, 2, false, true, 2, true, 1, true>
                 : (dq && !w12 && ablate == 0 && sel) ? (const void*)crc32_stream_kernel<0, 1024, 2, false, true, 2, true, 1>
                 : (dq && !w12 && ablate == 0) ? (const void*)crc32_stream_kernel<0, 1024, 2, false, true, 2, true>
                 : (ablate >= 4 && ablate <= 9 && !w12)
                       ? (ablate == 4 ? (const void*)crc32_stream_kernel<4>
                          : ablate == 5 ? (const void*)crc32_stream_kernel<5>
                          : ablate == 6 ? (const void*)crc32_stream_kernel<6>
                          : ablate == 7 ? (const void*)crc32_stream_kernel<7>
                          : ablate == 8 ? (const void*)crc32_stream_kernel<8> : (const void*)crc32_stream_kernel<9>)
                 : (w12 && ((variant >> 12) & 0xF) == 3) ? (const void*)crc32_stream_kernel<0, 768, 3>  // crc_ring 3
                 : w12 ? (ablate == 3 ? (const void*)crc32_stream_kernel<3, 768>
                          : ablate == 2 ? (const void*)crc32_stream_kernel<2, 768> : (const void*)crc32_stream_kernel<0, 768>)
                       : (ablate == 3 ? (const void*)crc32_stream_kernel<3>
                          : ablate == 2 ? (const void*)crc32_stream_kernel<2> : (const void*)crc32_stream_kernel<0>);
  const size_t lds = LDS_SCRATCH_OFF + (lm ? LDS_SMAP_BYTES : 0u);
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  void* args[] = {(void*)P};
  e = hipLaunchKernel(fn, dim3(ncu), dim3(block), args, lds, st);
  if (e != hipSuccess) return -(int)e;
  e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

extern "C" uint64_t lsmk_walk_sb_count(uint64_t n) { return (n + WALK_SB - 1) / WALK_SB; }

// walking descriptor kernel: superblock sums, their scan (total at
// P->total_segs), the kernel; sb_prefix holds lsmk_walk_sb_count(n) u64.
// Nothing is read back: asynchronous on st.
extern "C" int lsmk_launch_crc32_walk(const CrcParams* P, uint64_t* sb_prefix, int ncu, int variant,
                                      hipStream_t st) {
  const uint64_t n = P->nrec;
  if (n == 0) return 0;
  const uint64_t nsb = lsmk_walk_sb_count(n);
  hipLaunchKernelGGL(walk_phase1, dim3((unsigned)((nsb + 15) / 16)), dim3(1024), 0, st, P->len, n, sb_prefix,
                     (const uint32_t*)P->sflag);
  hipLaunchKernelGGL(scan_phase2, dim3(1), dim3(1024), 0, st, sb_prefix, (uint32_t)nsb, P->total_segs,
                     (const uint32_t*)P->sflag);
  CrcParams Q = *P;
  Q.sb_prefix = sb_prefix;
  const int ch = (variant & 0xF) ? (variant & 0xF) : LSMCK_DEFAULT_DESC_CHAINS;
  const int ablate = (variant >> 8) & 0xF;
  const void* fn = ablate == 3 ? (const void*)crc32_walk_kernel<2, 3>
                 : ch == 1 ? (const void*)crc32_walk_kernel<1>
                 : ch == 4 ? (const void*)crc32_walk_kernel<4>
                 : (variant & (int)0x80000000u) ? (const void*)crc32_walk_kernel<2, 0, true>  // A/B: crc_walk_opq 1
                                                : (const void*)crc32_walk_kernel<2>;
  size_t lds = LDS_SCRATCH_OFF;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  void* args[] = {(void*)&Q};
  e = hipLaunchKernel(fn, dim3(ncu), dim3(1024), args, lds, st);
  if (e != hipSuccess) return -(int)e;
  e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

// ---------------------------------------------------------------------------
// Verify: n_bad += (crc[i] != expected[i]); first_bad = min i with a mismatch.
namespace lsmck {
__global__ __launch_bounds__(256) void crc32_compare_kernel(const uint32_t* __restrict__ crc,
                                                             const uint32_t* __restrict__ expected, uint64_t n,
                                                             unsigned long long* __restrict__ n_bad,
                                                             unsigned long long* __restrict__ first_bad) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long bad = 0, first = ~0ull;
  for (; i < n; i += stride) {
    if (crc[i] != expected[i]) {
      ++bad;
      if (i < first) first = i;
    }
  }
  if (bad) {
    atomicAdd(n_bad, bad);
    atomicMin(first_bad, first);
  }
}
}  // namespace lsmck

extern "C" int lsmk_launch_crc32_compare(const uint32_t* crc, const uint32_t* expected, uint64_t n,
                                          unsigned long long* n_bad, unsigned long long* first_bad, hipStream_t st) {
  if (n == 0) return 0;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(crc32_compare_kernel, dim3((unsigned)blocks), dim3(256), 0, st, crc, expected, n, n_bad,
                     first_bad);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}
