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

#define LDS_TABLE_BYTES 131072u
#define WAVE_SCRATCH_BYTES 256u

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

// ---------------------------------------------------------------------------
// LDS tables.  Byte address of T_t[e], replica r:
//   256*e + 4*r + 128*(t&1) + 65536*(t>>1)
// T0 = Sarwate table, T_k[n] = (T_{k-1}[n] >> 8) ^ T0[T_{k-1}[n] & 0xFF].
__device__ __forceinline__ void build_lds_tables(unsigned char* smem, const uint32_t* __restrict__ master) {
  uint32_t* s32 = (uint32_t*)smem;
  for (uint32_t i = threadIdx.x; i < LDS_TABLE_BYTES / 4; i += blockDim.x) {
    uint32_t t = ((i >> 14) << 1) | ((i >> 5) & 1u);
    uint32_t e = (i >> 6) & 255u;
    s32[i] = master[t * 256u + e];
  }
}

__device__ __forceinline__ uint32_t lds_ld(const unsigned char* smem, uint32_t a) {
  return *(const uint32_t*)(smem + a);
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
  uint32_t K;      // x^(8*128*k) mod P for this segment (k < 2^16; larger k finish in seg_finish)
  uint32_t TI;     // init term 0xFFFFFFFF (x) x^(8*len0) for a record's first segment, else 0
  uint32_t sh;     // (E-128) & 3
  uint32_t lead;   // stream bytes in front of the record (first segment only)
};

// Issue every global load of a segment; consumes nothing.  FAST: full
// segment whose stream start is dword aligned (ALIGNED16: 16-byte aligned).
template <bool FAST>
__device__ __forceinline__ void seg_issue(const CrcParams& P, const SegInfo& si, SegLoad& L) {
  const uint64_t E = si.rec_off + si.rec_len - 128ull * si.k;  // segment end (offset from base)
  const uint32_t seglen = (si.q == 0) ? si.rec_len - 128u * si.k : 128u;
  L.lead = 128u - seglen;
  L.K = P.kseg[si.k & 0xFFFFu];
  L.TI = (si.q == 0) ? P.tinit[seglen] : 0u;
  // pointer arithmetic on the kernel-argument pointer keeps these global_load (not flat_load)
  const unsigned char* s0 = P.base + (E - 128);
  if (FAST) {
    L.sh = 0;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      u32x4 v = ld128(s0 + 16 * g);
      L.d[4 * g + 0] = v.x;
      L.d[4 * g + 1] = v.y;
      L.d[4 * g + 2] = v.z;
      L.d[4 * g + 3] = v.w;
    }
    L.d[32] = 0;
    return;
  }
  L.sh = (uint32_t)((uintptr_t)s0 & 3);
  const unsigned char* p = s0 - L.sh;                                         // floor4(E-128)
  const uint32_t lo_i = (L.sh + L.lead) >> 2;                                 // first dword to load
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    u32x4 v;
    if (4u * g >= lo_i) {
      v = ld128(p + 16 * g);
    } else {
      v.x = (4u * g + 0 >= lo_i) ? ld32(p + 16 * g + 0) : 0u;
      v.y = (4u * g + 1 >= lo_i) ? ld32(p + 16 * g + 4) : 0u;
      v.z = (4u * g + 2 >= lo_i) ? ld32(p + 16 * g + 8) : 0u;
      v.w = (4u * g + 3 >= lo_i) ? ld32(p + 16 * g + 12) : 0u;
    }
    L.d[4 * g + 0] = v.x;
    L.d[4 * g + 1] = v.y;
    L.d[4 * g + 2] = v.z;
    L.d[4 * g + 3] = v.w;
  }
  L.d[32] = L.sh ? ld32(p + 128) : 0u;
}

// Funnel, mask, raw slicing-by-4 CRC, init term, shift to the record's end.
template <bool FAST>
__device__ __forceinline__ uint32_t seg_finish(const unsigned char* smem, const CrcParams& P, const SegInfo& si,
                                               const SegLoad& L, uint32_t lo, uint32_t hi) {
  uint32_t w[32];
  if (FAST) {
#pragma unroll
    for (int j = 0; j < 32; ++j) w[j] = L.d[j];
  } else {
#pragma unroll
    for (int j = 0; j < 32; ++j) w[j] = __builtin_amdgcn_alignbyte(L.d[j + 1], L.d[j], L.sh);
    // zero the stream bytes in front of the record: bytes of B's dword that
    // belong to the previous record, and the slots of dwords never loaded
    if (__any(L.lead != 0)) {
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        int c = (int)L.lead - 4 * j;
        uint32_t m = (c >= 4) ? 0u : ((c > 0) ? (0xFFFFFFFFu << (8 * c)) : 0xFFFFFFFFu);
        w[j] &= m;
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 32; ++j) s = crc_word(smem, s, w[j], lo, hi);
  s ^= L.TI;
  uint32_t K = L.K;
  if (si.k >> 16) K = gf2_mulmod(K, P.khi[si.k >> 16]);
  return gf2_mulmod(s, K);
}

// ---------------------------------------------------------------------------
// Segmented XOR over a wave: each lane ends with the XOR of lanes [lane, run_end].
__device__ __forceinline__ uint32_t seg_suffix_xor(uint32_t v, uint32_t lane, uint32_t run_end) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_down(v, d, 64);
    v ^= (lane + d <= run_end) ? o : 0u;
  }
  return v;
}


__device__ __forceinline__ void emit_record(const CrcParams& P, uint32_t v, const SegInfo& si, uint32_t lane,
                                            uint32_t run_end, bool head) {
  if (!si.valid || !head) return;
  bool has_last = (lane + si.k) <= 63u;  // this tile holds the record's final segment
  if (si.q == 0 && has_last) {
    P.out[si.rec] = ~v;
  } else {
    atomicXor(&P.out[si.rec], has_last ? ~v : v);
  }
}

template <bool FAST>
__device__ __forceinline__ void finish_tile(const unsigned char* smem, const CrcParams& P, const SegInfo& si,
                                            const SegLoad& L, uint32_t lane, uint32_t lo, uint32_t hi) {
  uint32_t v = seg_finish<FAST>(smem, P, si, L, lo, hi);
  v = si.valid ? v : 0u;
  uint32_t run_end = min(63u, lane + si.k);
  v = seg_suffix_xor(v, lane, run_end);
  emit_record(P, v, si, lane, run_end, lane == 0 || si.q == 0);
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
template <bool FAST>
__global__ __launch_bounds__(1024) void crc32_fixed_kernel(CrcParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  build_lds_tables(smem, P.master);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lo = (lane & 31u) * 4u, hi = lo | 0x10000u;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  const uint32_t nsegr = (P.flen + 127u) >> 7;
  const uint32_t total = nsegr * (uint32_t)P.nrec;  // host keeps this < 2^32 - 64
  const uint32_t ntiles = (total + 63u) >> 6;
  // ping-pong between two load slots A/B: a loaded register is never copied
  // (a copy would force s_waitcnt vmcnt(0) on the prefetch)
  uint32_t t = wave;
  if (t >= ntiles) return;
  SegInfo sa = fixed_map(P, t, lane, nsegr, total), sb;
  SegLoad A, B;
  seg_issue<FAST>(P, sa, A);
  for (;;) {
    uint32_t tb = (t + nwaves < ntiles) ? t + nwaves : t;  // always issue: exact vmcnt counting
    sb = fixed_map(P, tb, lane, nsegr, total);
    seg_issue<FAST>(P, sb, B);
    __builtin_amdgcn_sched_barrier(0);
    finish_tile<FAST>(smem, P, sa, A, lane, lo, hi);
    t += nwaves;
    if (t >= ntiles) break;
    uint32_t ta = (t + nwaves < ntiles) ? t + nwaves : t;
    sa = fixed_map(P, ta, lane, nsegr, total);
    seg_issue<FAST>(P, sa, A);
    __builtin_amdgcn_sched_barrier(0);
    finish_tile<FAST>(smem, P, sb, B, lane, lo, hi);
    t += nwaves;
    if (t >= ntiles) break;
  }
}

// ---------------------------------------------------------------------------
// Descriptor records (offset u64, len u32), arbitrary alignment.
// Prep: seg_start[r] = exclusive prefix of nseg(r) = ceil(len/128);
//       tile_first[t] = record holding segment 64t.
__device__ __forceinline__ SegInfo desc_map(const CrcParams& P, int* R, uint32_t t, uint32_t lane, uint32_t total) {
  const uint32_t g = t * 64u + lane;
  const uint32_t r0 = P.tile_first[t];
  // lane -> record: the largest r with seg_start[r] <= g (empty records own nothing)
  R[lane] = -1;
  __builtin_amdgcn_wave_barrier();
  uint64_t chunk = 0;
  for (;;) {
    uint64_t r = (uint64_t)r0 + chunk + lane;
    uint32_t ss = r < P.nrec ? P.seg_start[r] : 0xFFFFFFFFu;
    int64_t st = (int64_t)ss - (int64_t)t * 64;
    if (ss != 0xFFFFFFFFu && st < 64) atomicMax(&R[st < 0 ? 0 : (int)st], (int)(chunk + lane));
    // continue while the 64th record of this chunk still starts inside the tile
    uint32_t last_ss = __shfl(ss, 63, 64);
    chunk += 64;
    if (last_ss == 0xFFFFFFFFu || (int64_t)last_ss - (int64_t)t * 64 >= 64) break;
  }
  __builtin_amdgcn_wave_barrier();
  int mine = R[lane];
  uint64_t starts = __ballot(mine >= 0);
  uint64_t below = starts & ((lane == 63) ? ~0ull : ((2ull << lane) - 1ull));
  uint32_t p = 63u - (uint32_t)__builtin_clzll(below | 1ull);
  int jrec = __shfl(mine, (int)p, 64);
  __builtin_amdgcn_wave_barrier();
  SegInfo si;
  si.valid = g < total;
  si.rec = r0 + (uint32_t)(jrec < 0 ? 0 : jrec);
  uint32_t rs = P.seg_start[si.rec];
  si.rec_off = P.off[si.rec];
  si.rec_len = P.len[si.rec];
  uint32_t nseg = (si.rec_len + 127u) >> 7;
  si.q = g - rs;
  si.k = nseg - 1u - si.q;
  if (!si.valid) {  // pad lanes: a harmless full segment of the last record (result discarded)
    si.q = 1;
    si.k = 0;
    si.rec_len = si.rec_len < 128u ? 128u : si.rec_len;
  }
  return si;
}

__global__ __launch_bounds__(1024) void crc32_desc_kernel(CrcParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  build_lds_tables(smem, P.master);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lo = (lane & 31u) * 4u, hi = lo | 0x10000u;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  int* R = (int*)(smem + LDS_TABLE_BYTES + (threadIdx.x >> 6) * WAVE_SCRATCH_BYTES);
  const uint32_t total = *P.total_segs;
  const uint32_t ntiles = (total + 63u) >> 6;
  uint32_t t = wave;
  if (t >= ntiles) return;
  SegInfo sa = desc_map(P, R, t, lane, total), sb;
  SegLoad A, B;
  seg_issue<false>(P, sa, A);
  for (;;) {
    uint32_t tb = (t + nwaves < ntiles) ? t + nwaves : t;
    sb = desc_map(P, R, tb, lane, total);
    seg_issue<false>(P, sb, B);
    __builtin_amdgcn_sched_barrier(0);
    finish_tile<false>(smem, P, sa, A, lane, lo, hi);
    t += nwaves;
    if (t >= ntiles) break;
    uint32_t ta = (t + nwaves < ntiles) ? t + nwaves : t;
    sa = desc_map(P, R, ta, lane, total);
    seg_issue<false>(P, sa, A);
    __builtin_amdgcn_sched_barrier(0);
    finish_tile<false>(smem, P, sb, B, lane, lo, hi);
    t += nwaves;
    if (t >= ntiles) break;
  }
}

// ---------------------------------------------------------------------------
// Prep kernels for the descriptor path: three-phase exclusive scan of
// nseg(r) = ceil(len/128), then tile_first.
#define SCAN_ITEMS 4
#define SCAN_BLOCK 1024
__global__ __launch_bounds__(SCAN_BLOCK) void scan_phase1(const uint32_t* __restrict__ len, uint64_t n,
                                                           uint32_t* __restrict__ seg_start,
                                                           uint32_t* __restrict__ block_sum) {
  __shared__ uint32_t wsum[SCAN_BLOCK / 64];
  uint64_t base = (uint64_t)blockIdx.x * SCAN_BLOCK * SCAN_ITEMS + (uint64_t)threadIdx.x * SCAN_ITEMS;
  uint32_t v[SCAN_ITEMS], acc = 0;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    uint64_t r = base + i;
    uint32_t l = r < n ? len[r] : 0u;
    v[i] = acc;
    acc += (l + 127u) >> 7;
  }
  // wave inclusive scan of acc
  uint32_t lane = threadIdx.x & 63u, x = acc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += o;
  }
  if (lane == 63) wsum[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x < 64) {
    uint32_t y = threadIdx.x < SCAN_BLOCK / 64 ? wsum[threadIdx.x] : 0u;
    uint32_t z = y;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      uint32_t o = __shfl_up(z, d, 64);
      if (threadIdx.x >= (uint32_t)d) z += o;
    }
    if (threadIdx.x < SCAN_BLOCK / 64) wsum[threadIdx.x] = z - y;  // exclusive
    if (threadIdx.x == SCAN_BLOCK / 64 - 1) block_sum[blockIdx.x] = z;
  }
  __syncthreads();
  uint32_t excl = x - acc + wsum[threadIdx.x >> 6];
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    uint64_t r = base + i;
    if (r < n) seg_start[r] = excl + v[i];
  }
}

__global__ __launch_bounds__(1024) void scan_phase2(uint32_t* __restrict__ block_sum, uint32_t nblocks,
                                                     uint32_t* __restrict__ total) {
  // single workgroup: exclusive scan of block sums in place
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nblocks; b0 += 1024) {
    uint32_t i = b0 + threadIdx.x;
    uint32_t y = i < nblocks ? block_sum[i] : 0u;
    uint32_t lane = threadIdx.x & 63u, x = y;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      uint32_t o = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += o;
    }
    if (lane == 63) wsum[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
      uint32_t a = threadIdx.x < 16 ? wsum[threadIdx.x] : 0u, z = a;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = __shfl_up(z, d, 64);
        if (threadIdx.x >= (uint32_t)d) z += o;
      }
      if (threadIdx.x < 16) wsum[threadIdx.x] = z - a;
    }
    __syncthreads();
    uint32_t c = carry;
    uint32_t ex = c + wsum[threadIdx.x >> 6] + x - y;
    if (i < nblocks) block_sum[i] = ex;
    __syncthreads();
    if (threadIdx.x == 1023) carry = ex + y;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(1024) void scan_phase3(const uint32_t* __restrict__ len, uint64_t n,
                                                     uint32_t* __restrict__ seg_start,
                                                     const uint32_t* __restrict__ block_sum,
                                                     uint32_t* __restrict__ tile_first) {
  uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  uint32_t ss = seg_start[r] + block_sum[r / (SCAN_BLOCK * SCAN_ITEMS)];
  seg_start[r] = ss;
  uint32_t ns = (len[r] + 127u) >> 7;
  if (ns == 0) return;
  uint32_t t0 = (ss + 63u) >> 6, t1 = (ss + ns - 1u) >> 6;
  for (uint32_t t = t0; t <= t1; ++t) tile_first[t] = (uint32_t)r;
}

}  // namespace lsmck

// ---------------------------------------------------------------------------
// Launchers (C linkage inside the library; the public C ABI is lsmck_api.cpp)
using namespace lsmck;


extern "C" int lsmk_launch_crc32_fixed(const CrcParams* P, int ncu, hipStream_t st) {
  size_t lds = LDS_TABLE_BYTES;
  bool fast = ((uintptr_t)P->base % 4 == 0) && (P->stride % 4 == 0) && (P->flen % 128 == 0);
  const void* fn = fast ? (const void*)crc32_fixed_kernel<true> : (const void*)crc32_fixed_kernel<false>;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  if (fast)
    hipLaunchKernelGGL((crc32_fixed_kernel<true>), dim3(ncu), dim3(1024), lds, st, *P);
  else
    hipLaunchKernelGGL((crc32_fixed_kernel<false>), dim3(ncu), dim3(1024), lds, st, *P);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

extern "C" uint64_t lsmk_scan_block_count(uint64_t n) {
  uint64_t per = (uint64_t)SCAN_BLOCK * SCAN_ITEMS;
  return (n + per - 1) / per;
}

// phase 1+2: seg_start (block-local) and the total segment count (device)
extern "C" int lsmk_launch_crc32_scan(const CrcParams* P, uint32_t* block_sum, hipStream_t st) {
  uint64_t n = P->nrec;
  uint32_t nb = (uint32_t)lsmk_scan_block_count(n);
  hipLaunchKernelGGL(scan_phase1, dim3(nb), dim3(SCAN_BLOCK), 0, st, P->len, n, P->seg_start, block_sum);
  hipLaunchKernelGGL(scan_phase2, dim3(1), dim3(1024), 0, st, block_sum, nb, P->total_segs);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

// phase 3 (+tile_first) and the checksum kernel; tile_first must hold
// ceil(total/64) entries
extern "C" int lsmk_launch_crc32_desc(const CrcParams* P, const uint32_t* block_sum, int ncu, hipStream_t st) {
  uint64_t n = P->nrec;
  hipLaunchKernelGGL(scan_phase3, dim3((unsigned)((n + 1023) / 1024)), dim3(1024), 0, st, P->len, n, P->seg_start,
                     block_sum, P->tile_first);
  size_t lds = LDS_TABLE_BYTES + 16 * WAVE_SCRATCH_BYTES;
  hipError_t e = hipFuncSetAttribute((const void*)crc32_desc_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  hipLaunchKernelGGL(crc32_desc_kernel, dim3(ncu), dim3(1024), lds, st, *P);
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
