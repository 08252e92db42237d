// lsmck_wal.hip -- WAL replay header walk on the GPU (gfx950).
//
// The reference reads the log record by record (src/wal.rs:68-84, 122-163):
// each header's position comes from the previous header's lengths, a serial
// chain.  Here the chain is found in parallel, without reading the image back
// to the host:
//   1. every byte position p whose byte is a command type (1 Insert, 2 Remove)
//      and whose header fits in the log is a CANDIDATE record start (a bitmap,
//      one u64 per 64 bytes, and per-word candidate counts);
//   2. an exclusive scan of the counts ranks the candidates;
//   3. every candidate gets its successor -- the position after its header and
//      payload (the payload cut at EOF as read_to_end on take() does) -- as a
//      candidate rank, or a terminal: clean END (EOF at or inside the next
//      header) or BAD (the next byte is not a command type, at position q);
//   4. pointer doubling J_{k+1} = J_k o J_k (terminals absorb) over the
//      candidates, every level kept;
//   5. the chain from position 0 is unrolled by doubling too: knowing records
//      0..L-1, records L..2L-1 are J_k of them (k = log2 L);
//   6. the chain's records become payload descriptors for the CRC batch
//      (crc32_walk_kernel) and the GPU compare.
// Candidates are positions, so bogus ones (type bytes inside payloads) only
// cost work: a chain that starts at position 0 follows real headers only.
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef LSMCK_SEG_CLOCK  // diagnostic builds only: the segment walk's clock marks per segment
#ifndef LSMCK_DIAG
#define LSMCK_DIAG  // (lsmck_segwalk.h then takes its marks from lsmck_diag.h)
#endif
__device__ uint64_t g_seg_clock[3 * 131072];
#define LSMCK_SEG_CLOCK_MARK(k, slot) \
  do {                                  \
    if ((k) < 131072u) g_seg_clock[3u * (k) + (slot)] = wall_clock64(); \
  } while (0)
#endif

#include "lsmck.h"
#include "lsmck_device.h"
#include "lsmck_segwalk.h"

namespace lsmck {

#define WAL_END 0xFFFFFFFFu  // chain ends cleanly (EOF at or inside the next header)
#define WAL_BAD 0xFFFFFFFEu  // the next byte is not a command type
// prefix walks (lim < n: only the bytes before lim are on the device yet)
#define WAL_STOP 0xFFFFFFFDu      // the next record starts at badpos[c]: resume the walk there
#define WAL_STOPSELF 0xFFFFFFFCu  // this record does not end by lim: resume the walk at its own position
#define WAL_TERM_MIN 0xFFFFFFFCu  // entries >= this are terminals (absorbing)

__device__ __forceinline__ uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t hdr_len(uint8_t t) { return t == 1 ? 13u : 9u; }

// 1. candidate bitmap: thread per 64-byte word of positions (16-byte loads
// when the image is 16-byte aligned, byte loads otherwise)
__global__ __launch_bounds__(256) void wal_mark(const uint8_t* __restrict__ img, uint64_t n, int aligned,
                                                 uint64_t* __restrict__ bits, uint32_t* __restrict__ cnt, uint64_t w0,
                                                 uint64_t w1) {
  const uint64_t w = w0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // words [w0, w1)
  if (w >= w1) return;
  const uint64_t p0 = w << 6;
  uint64_t m = 0;
  if (aligned && p0 + 64 <= n) {
    const uint4* q = (const uint4*)(img + p0);  // the image is 16-byte aligned by the caller
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint4 v = q[g];
      const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t b = (d[j >> 2] >> (8 * (j & 3))) & 0xFFu;
        const uint64_t p = p0 + 16 * g + j;
        if ((b == 1u || b == 2u) && p + hdr_len((uint8_t)b) <= n) m |= 1ull << (16 * g + j);
      }
    }
  } else {
    const uint64_t pe = p0 + 64 < n ? p0 + 64 : n;
    for (uint64_t p = p0; p < pe; ++p) {
      const uint8_t b = img[p];
      if ((b == 1 || b == 2) && p + hdr_len(b) <= n) m |= 1ull << (p - p0);
    }
  }
  bits[w] = m;
  cnt[w] = (uint32_t)__popcll(m);
}

// 2. exclusive scan of cnt (u32) in place: per-block sums, one-block scan of
// those, per-block rescan.  1024 threads x 4 words per block.
#define WSCAN_ITEMS 4u
#define WSCAN_BLOCK 1024u
__global__ __launch_bounds__(WSCAN_BLOCK) void wal_scan_a(const uint32_t* __restrict__ cnt, uint64_t nw,
                                                            uint32_t* __restrict__ bsum) {
  __shared__ uint32_t s[WSCAN_BLOCK / 64];
  const uint64_t i0 = ((uint64_t)blockIdx.x * WSCAN_BLOCK + threadIdx.x) * WSCAN_ITEMS;
  uint32_t x = 0;
  for (uint32_t j = 0; j < WSCAN_ITEMS; ++j) x += (i0 + j < nw) ? cnt[i0 + j] : 0u;
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  if ((threadIdx.x & 63u) == 0) s[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t k = 0; k < WSCAN_BLOCK / 64; ++k) t += s[k];
    bsum[blockIdx.x] = t;
  }
}
__global__ __launch_bounds__(1024) void wal_scan_b(uint32_t* __restrict__ bsum, uint32_t nb,
                                                     uint32_t* __restrict__ total) {
  __shared__ uint32_t ws[16];
  const uint32_t C = (nb + 1023u) / 1024u, b0 = threadIdx.x * C, b1 = min(nb, b0 + C);
  uint32_t mine = 0;
  for (uint32_t b = b0; b < b1; ++b) mine += bsum[b];
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t x = mine;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += o;
  }
  if (lane == 63u) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < 16; ++i) {
      const uint32_t v = ws[i];
      ws[i] = acc;
      acc += v;
    }
    *total = acc;
  }
  __syncthreads();
  uint32_t run = ws[threadIdx.x >> 6] + x - mine;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t v = bsum[b];
    bsum[b] = run;
    run += v;
  }
}
__global__ __launch_bounds__(WSCAN_BLOCK) void wal_scan_c(uint32_t* __restrict__ cnt, uint64_t nw,
                                                            const uint32_t* __restrict__ bsum) {
  __shared__ uint32_t s[WSCAN_BLOCK / 64];
  const uint64_t i0 = ((uint64_t)blockIdx.x * WSCAN_BLOCK + threadIdx.x) * WSCAN_ITEMS;
  uint32_t v[WSCAN_ITEMS], x = 0;
  for (uint32_t j = 0; j < WSCAN_ITEMS; ++j) {
    v[j] = (i0 + j < nw) ? cnt[i0 + j] : 0u;
    x += v[j];
  }
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t inc = x;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += o;
  }
  if (lane == 63u) s[threadIdx.x >> 6] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (uint32_t k = 0; k < WSCAN_BLOCK / 64; ++k) {
      const uint32_t t = s[k];
      s[k] = acc;
      acc += t;
    }
  }
  __syncthreads();
  uint32_t run = bsum[blockIdx.x] + s[threadIdx.x >> 6] + inc - x;
  for (uint32_t j = 0; j < WSCAN_ITEMS; ++j)
    if (i0 + j < nw) {
      cnt[i0 + j] = run;  // now: candidates before word i0 + j
      run += v[j];
    }
}

// rank of candidate position q (q must be a candidate)
__device__ __forceinline__ uint32_t cand_rank(const uint64_t* __restrict__ bits, const uint32_t* __restrict__ pre,
                                              uint64_t q) {
  const uint64_t w = q >> 6;
  const uint32_t b = (uint32_t)(q & 63u);
  return pre[w] + (uint32_t)__popcll(bits[w] & ((1ull << b) - 1ull));
}

// 3. positions and successors of the candidates of words [w0, w1) (their
// ranks: pre, scanned over the same words): thread per 64-byte word.  A prefix
// walk (lim < n) takes a record only when its header and payload end by lim,
// and stops at a next header that does not start 13 bytes before lim.
__global__ __launch_bounds__(256) void wal_succ(const uint8_t* __restrict__ img, uint64_t n,
                                                 const uint64_t* __restrict__ bits, const uint32_t* __restrict__ pre,
                                                 uint64_t* __restrict__ pos, uint32_t* __restrict__ J0,
                                                 uint64_t* __restrict__ badpos, uint64_t w0, uint64_t w1, uint64_t lim) {
  const uint64_t w = w0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= w1) return;
  uint64_t m = bits[w];
  uint32_t c = pre[w];
  while (m) {
    const uint32_t b = (uint32_t)__builtin_ctzll(m);
    m &= m - 1;
    const uint64_t p = (w << 6) + b;
    pos[c] = p;
    if (lim < n && p + 13u > lim) {  // (a header not yet readable in full)
      J0[c] = WAL_STOPSELF;
      ++c;
      continue;
    }
    const uint8_t t = img[p];
    const uint32_t h = hdr_len(t);
    const uint32_t klen = rd32(img + p + 5);
    const uint32_t vlen = t == 1 ? rd32(img + p + 9) : 0u;
    const uint32_t dlen = klen + vlen;  // u32, as wal.rs:129
    const uint64_t avail = n - (p + h);
    const uint64_t q = p + h + (dlen <= avail ? (uint64_t)dlen : avail);
    uint32_t s;
    if (lim < n && p + h + (uint64_t)dlen > lim) {
      s = WAL_STOPSELF;
    } else if (lim < n && q + 13u > lim) {
      s = WAL_STOP;
      badpos[c] = q;
    } else if (q >= n) {
      s = WAL_END;  // wal.rs:76-77: EOF on the next header's type byte
    } else {
      const uint8_t t2 = img[q];
      if (t2 != 1 && t2 != 2) {
        s = WAL_BAD;
        badpos[c] = q;
      } else if (q + hdr_len(t2) > n) {
        s = WAL_END;  // UnexpectedEof inside the next header
      } else {
        s = cand_rank(bits, pre, q);
      }
    }
    J0[c] = s;
    ++c;
  }
}

// the chain's first entry: the candidate at position `start` when it is one;
// otherwise the log ends there: empty (END) or a bad type byte at start
__global__ void wal_chain_init(const uint8_t* __restrict__ img, uint64_t n, const uint64_t* __restrict__ bits,
                               const uint32_t* __restrict__ pre, uint64_t start, uint32_t* __restrict__ chain,
                               unsigned long long* __restrict__ info) {
  const bool cand = start < n && ((bits[start >> 6] >> (start & 63u)) & 1ull);
  const bool bad = start < n && img[start] != 1 && img[start] != 2;
  chain[0] = cand ? cand_rank(bits, pre, start) : (bad ? WAL_BAD : WAL_END);
  info[0] = 0;
  info[1] = bad ? WAL_BAD : WAL_END;
  info[2] = start;  // bad position
}

// 4. one doubling level: Jn[c] = J[J[c]] (terminals absorb)
__global__ __launch_bounds__(256) void wal_double(const uint32_t* __restrict__ J, uint32_t* __restrict__ Jn,
                                                   uint32_t nc) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  const uint32_t s = J[c];
  Jn[c] = s >= WAL_TERM_MIN ? s : J[s];
}

// 5. chain unrolling, one level: chain[L + i] = J_k(chain[i]) for i < L = 2^k
// (an entry is a candidate rank or a terminal; a terminal absorbs).
__global__ __launch_bounds__(256) void wal_unroll(const uint32_t* __restrict__ Jk, uint32_t* __restrict__ chain,
                                                   uint32_t L) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L) return;
  const uint32_t c = chain[i];
  chain[L + i] = c >= WAL_TERM_MIN ? c : Jk[c];
}

// the chain's length and how it ends: the first terminal entry (entries are
// ranks up to it, terminals after); out[0] = records, out[1] = terminal code,
// out[2] = the BAD position, or where a prefix walk resumes (STOP: the next
// header; STOPSELF: the record that did not end by the limit, not counted)
__global__ __launch_bounds__(256) void wal_chain_end(const uint32_t* __restrict__ chain, uint32_t len,
                                                      const uint32_t* __restrict__ J0, const uint64_t* __restrict__ badpos,
                                                      const uint64_t* __restrict__ pos, unsigned long long* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len) return;
  const bool here = chain[i] < WAL_TERM_MIN && (i + 1 == len || chain[i + 1] >= WAL_TERM_MIN);
  if (!here) return;  // exactly one entry: the chain's last record
  const uint32_t c = chain[i];
  const uint32_t code = J0[c];
  out[0] = code == WAL_STOPSELF ? i : i + 1;
  out[1] = code;
  out[2] = (code == WAL_BAD || code == WAL_STOP) ? badpos[c] : (code == WAL_STOPSELF ? pos[c] : 0ull);
}

// 6. records -> lsmck_wal_rec entries, CRC descriptors and stored CRCs
__global__ __launch_bounds__(256) void wal_emit(const uint8_t* __restrict__ img, uint64_t n,
                                                 const uint32_t* __restrict__ chain, const uint64_t* __restrict__ pos,
                                                 const unsigned long long* __restrict__ info,
                                                 lsmck_wal_rec* __restrict__ recs, uint64_t* __restrict__ poff,
                                                 uint32_t* __restrict__ plen, uint32_t* __restrict__ pcrc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint32_t)info[0]) return;
  const uint64_t p = pos[chain[i]];
  const uint8_t t = img[p];
  const uint32_t h = hdr_len(t);
  const uint32_t klen = rd32(img + p + 5), vlen = t == 1 ? rd32(img + p + 9) : 0u;
  const uint32_t dlen = klen + vlen;
  const uint64_t avail = n - (p + h);
  lsmck_wal_rec r;
  r.rec_off = p;
  r.payload_off = p + h;
  r.klen = klen;
  r.vlen = vlen;
  r.crc = rd32(img + p + 1);
  r.type = t;
  recs[i] = r;
  poff[i] = p + h;
  plen[i] = dlen <= avail ? dlen : (uint32_t)avail;
  pcrc[i] = r.crc;
}

// Batch framing of Insert records in place (CommandLog::log, wal.rs:165-196):
// payload i = key || value already lies at img + off[i]; its 13-byte header
// goes in front of it: type 1, crc[i], klen = min(len[i], kmax), vlen = the rest.
// Byte stores (headers start at any offset); a thread per record.
__global__ __launch_bounds__(256) void wal_frame_insert(uint8_t* __restrict__ img, const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ len,
                                                         const uint32_t* __restrict__ crc, uint64_t n, uint32_t kmax) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* h = img + off[i] - 13u;
  const uint32_t l = len[i], k = l < kmax ? l : kmax, v = l - k, c = crc[i];
  h[0] = 1;
  for (int b = 0; b < 4; ++b) {
    h[1 + b] = (uint8_t)(c >> (8 * b));
    h[5 + b] = (uint8_t)(k >> (8 * b));
    h[9 + b] = (uint8_t)(v >> (8 * b));
  }
}

// --- the segment walk (lsmck_segwalk.h) ------------------------------------
// Thread per segment.  The walks are chains of dependent header reads, so
// the launch wants as many segments in flight as the chip holds: the host
// sizes segments for ~2^16 of them (lsmk_wal_seg_bytes).
__global__ __launch_bounds__(256) void wal_seg_walk(seg::SegArgs a) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < a.K) seg::seg_walk_thread(a, k);
}

// The guess by a group of G consecutive lanes: lane j of the group scans the
// segment's scan chunks j, j + G, ... in rounds, each taking the first start
// in its chunk that accept() takes; after each round the group keeps the
// lowest one found (all chunks before it held none), so the result is the
// one seg::guess finds -- before its later-start rule, which the group's
// first lane then runs.  A wave's time in the guess is its slowest lane's
// (a segment that starts inside a long record scans tens of KB at about one
// wave per SIMD); G lanes cut that lane's serial candidate iterations G-fold.
template <int G>
__device__ __forceinline__ uint64_t guess_group(const seg::SegArgs& a, uint32_t k, uint32_t j) {
  using namespace seg;
  const uint64_t b = seg_begin(a, k), e = seg_end(a, k), hop = seg_hop(a);
  constexpr uint64_t CH = 64u * kScanBlocks;
  const uintptr_t base = (uintptr_t)a.img;
  const uintptr_t A0 = (base + b) & ~(uintptr_t)(CH - 1);
  for (uint32_t r = 0;; ++r) {
    const int64_t cs = (int64_t)(A0 + ((uint64_t)r * G + j) * CH - base);
    const bool act = cs < (int64_t)e;
    uint64_t f = kNoGuess;
    if (act) {
      const uint64_t lo = cs > (int64_t)b ? (uint64_t)cs : b;
      const uint64_t hi = (uint64_t)(cs + (int64_t)CH) < e ? (uint64_t)(cs + (int64_t)CH) : e;
      Scan S;
      for (uint64_t c = next_cand(S, a.img, a.n, lo, hi); c != kNoGuess; c = next_cand(S, a.img, a.n, c + 1, hi))
        if (accept(a.img, a.n, c, hop)) {
          f = c;
          break;
        }
    }
    uint32_t any = act ? 1u : 0u;
#pragma unroll
    for (int s = 1; s < G; s <<= 1) {  // (the group's lanes run these rounds together)
      const uint32_t lo32 = (uint32_t)__shfl_xor((int)(uint32_t)f, s), hi32 = (uint32_t)__shfl_xor((int)(uint32_t)(f >> 32), s);
      const uint64_t o = ((uint64_t)hi32 << 32) | lo32;
      f = o < f ? o : f;
      any |= (uint32_t)__shfl_xor((int)any, s);
    }
    if (f != kNoGuess || !any) return f;
  }
}

// seg::later_rule by the same group of G lanes: lane j scans chunks j, j + G,
// ... of the window after the accepted start c for the first candidate whose
// chain reaches c's first record's end; the group keeps the lowest found in a
// round (every chunk before it held none), so each step takes the start the
// one-lane rule takes.  The rule's scan (up to kLaterScan bytes) runs G-fold
// shorter on the wave's slowest lane -- in a log of MiB records every true
// guess scans its whole window.
template <int G>
__device__ __forceinline__ uint64_t later_group(const seg::SegArgs& a, uint32_t k, uint32_t j, uint64_t c) {
  using namespace seg;
  const uint64_t e = seg_end(a, k), later_min = seg_later_min(a);
  constexpr uint64_t CH = 64u * kScanBlocks;
  const uintptr_t base = (uintptr_t)a.img;
  for (;;) {
    bool whole;
    const Head hc = head(a.img, a.n, c);
    const uint64_t q1 = next_of(hc, a.n, c, &whole);
    uint64_t lim = q1 < e ? q1 : e;
    if (later_min) {
      if (q1 - c - hdr_len(hc.t) <= later_min) return c;  // (kLaterMin)
      if (lim > c + 1 + kLaterScan) lim = c + 1 + kLaterScan;  // (kLaterScan)
    }
    const uint64_t b = c + 1;
    const uintptr_t A0 = (base + b) & ~(uintptr_t)(CH - 1);
    uint64_t found = kNoGuess;
    for (uint32_t r = 0;; ++r) {
      const int64_t cs = (int64_t)(A0 + ((uint64_t)r * G + j) * CH - base);
      const bool act = cs < (int64_t)lim;
      uint64_t f = kNoGuess;
      if (act) {
        const uint64_t lo = cs > (int64_t)b ? (uint64_t)cs : b;
        const uint64_t hi = (uint64_t)(cs + (int64_t)CH) < lim ? (uint64_t)(cs + (int64_t)CH) : lim;
        Scan S;
        for (uint64_t c2 = next_cand(S, a.img, a.n, lo, hi); c2 != kNoGuess; c2 = next_cand(S, a.img, a.n, c2 + 1, hi))
          if (reaches(a.img, a.n, c2, q1)) {
            f = c2;
            break;
          }
      }
      uint32_t any = act ? 1u : 0u;
#pragma unroll
      for (int s = 1; s < G; s <<= 1) {
        const uint32_t lo32 = (uint32_t)__shfl_xor((int)(uint32_t)f, s), hi32 = (uint32_t)__shfl_xor((int)(uint32_t)(f >> 32), s);
        const uint64_t o = ((uint64_t)hi32 << 32) | lo32;
        f = o < f ? o : f;
        any |= (uint32_t)__shfl_xor((int)any, s);
      }
      if (f != kNoGuess || !any) {
        found = f;
        break;
      }
    }
    if (found == kNoGuess) return c;
    c = found;
  }
}

template <int G>
__global__ __launch_bounds__(256) void wal_seg_walk_group(seg::SegArgs a) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, k = t / G, j = t % G;
  if (k >= a.K) return;  // (the whole group)
  if (j == 0) LSMCK_SEG_CLOCK_MARK(k, 0);
  if (k == 0) {
    if (j == 0) seg::seg_forced(a, 0, a.start);
    return;
  }
  uint64_t c = guess_group<G>(a, k, j);
  if (c != seg::kNoGuess && seg::seg_later(a)) c = later_group<G>(a, k, j, c);  // (c: the group's, in every lane)
  if (j != 0) return;
  LSMCK_SEG_CLOCK_MARK(k, 1);
  seg::seg_take_guess(a, k, c);
  LSMCK_SEG_CLOCK_MARK(k, 2);
}

__global__ __launch_bounds__(256) void wal_seg_jterm(seg::SegArgs a) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < a.K && (a.code[k] == seg::kEnd || a.code[k] == seg::kBad))
    atomicMin((unsigned int*)(a.info + seg::kInfoJterm), k);
}

// exclusive scan of the placement words into pre[0..K] (three passes: block
// sums, one block over those, per-block rescan), 1024 threads x 4 segments
#define SSCAN_ITEMS 4u
#define SSCAN_BLOCK 1024u
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x, uint32_t lane) {
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += o;
  }
  return x;
}
__global__ __launch_bounds__(SSCAN_BLOCK) void wal_seg_scan_a(seg::SegArgs a, uint64_t* __restrict__ bsum) {
  __shared__ uint64_t s[SSCAN_BLOCK / 64];
  const uint32_t jterm = (uint32_t)a.info[seg::kInfoJterm];
  const uint64_t i0 = ((uint64_t)blockIdx.x * SSCAN_BLOCK + threadIdx.x) * SSCAN_ITEMS;
  uint64_t x = 0;
  for (uint32_t j = 0; j < SSCAN_ITEMS; ++j)
    if (i0 + j < a.K) x += seg::seg_word(a, (uint32_t)(i0 + j), jterm);
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  if ((threadIdx.x & 63u) == 0) s[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (uint32_t k = 0; k < SSCAN_BLOCK / 64; ++k) t += s[k];
    bsum[blockIdx.x] = t;
  }
}
__global__ __launch_bounds__(1024) void wal_seg_scan_b(uint64_t* __restrict__ bsum, uint32_t nb) {
  __shared__ uint64_t ws[16];
  const uint32_t C = (nb + 1023u) / 1024u, b0 = threadIdx.x * C, b1 = min(nb, b0 + C);
  uint64_t mine = 0;
  for (uint32_t b = b0; b < b1; ++b) mine += bsum[b];
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t x = wave_incl_scan(mine, lane);
  if (lane == 63u) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t acc = 0;
    for (int i = 0; i < 16; ++i) {
      const uint64_t v = ws[i];
      ws[i] = acc;
      acc += v;
    }
  }
  __syncthreads();
  uint64_t run = ws[threadIdx.x >> 6] + x - mine;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint64_t v = bsum[b];
    bsum[b] = run;
    run += v;
  }
}
__global__ __launch_bounds__(SSCAN_BLOCK) void wal_seg_scan_c(seg::SegArgs a, const uint64_t* __restrict__ bsum) {
  __shared__ uint64_t s[SSCAN_BLOCK / 64];
  const uint32_t jterm = (uint32_t)a.info[seg::kInfoJterm];
  const uint64_t i0 = ((uint64_t)blockIdx.x * SSCAN_BLOCK + threadIdx.x) * SSCAN_ITEMS;
  uint64_t v[SSCAN_ITEMS], x = 0;
  for (uint32_t j = 0; j < SSCAN_ITEMS; ++j) {
    v[j] = i0 + j < a.K ? seg::seg_word(a, (uint32_t)(i0 + j), jterm) : 0ull;
    x += v[j];
  }
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t inc = wave_incl_scan(x, lane);
  if (lane == 63u) s[threadIdx.x >> 6] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t acc = 0;
    for (uint32_t k = 0; k < SSCAN_BLOCK / 64; ++k) {
      const uint64_t t = s[k];
      s[k] = acc;
      acc += t;
    }
  }
  __syncthreads();
  uint64_t run = bsum[blockIdx.x] + s[threadIdx.x >> 6] + inc - x;
  for (uint32_t j = 0; j < SSCAN_ITEMS; ++j)
    if (i0 + j <= a.K) {  // (pre[K]: the total)
      a.pre[i0 + j] = run;
      run += v[j];
    }
}

__global__ __launch_bounds__(256) void wal_seg_check(seg::SegArgs a) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t jterm = (uint32_t)a.info[seg::kInfoJterm];
  if (k < a.K && seg::seg_check_fails(a, k, jterm)) {
    atomicMin((unsigned int*)(a.info + seg::kInfoFail), k);
    atomicAdd((unsigned int*)(a.info + seg::kInfoNFail), 1u);
  }
  // the chain's way out of a prefix (lim < n): the last guessed segment whose
  // exit lies at or past lim (once the check passes, the only one)
  if (k < a.K && k < jterm && a.code[k] == seg::kExit && a.x[k] >= a.lim)
    atomicMax((unsigned int*)(a.info + seg::kInfoLast), k + 1u);
}

// the round's outcome into info (one thread)
__global__ void wal_seg_finalize(seg::SegArgs a) {
  const uint32_t jterm = (uint32_t)a.info[seg::kInfoJterm], fail = (uint32_t)a.info[seg::kInfoFail];
  a.info[seg::kInfoRecs] = a.pre[a.K] & seg::kRecMask;
  const bool jt = jterm < a.K;
  const uint32_t last = (uint32_t)a.info[seg::kInfoLast];  // (no chain end in the prefix: its way out)
  a.info[seg::kInfoCode] = jt ? a.code[jterm] : (last ? seg::kExit : 0u);
  a.info[seg::kInfoPos] = jt ? a.x[jterm] : (last ? a.x[last - 1u] : 0ull);
  a.info[seg::kInfoFailX] = fail < a.K ? a.x[fail] : 0ull;
}

// a new round: jterm and fail back to "none"
__global__ void wal_seg_reset(seg::SegArgs a) {
  a.info[seg::kInfoJterm] = seg::kNoSeg;
  a.info[seg::kInfoFail] = seg::kNoSeg;
  a.info[seg::kInfoNFail] = 0;
  a.info[seg::kInfoLast] = 0;
}

// a parallel repair round (seg::seg_prepair) from the snapshot g0 / x0 / code0
__global__ __launch_bounds__(256) void wal_seg_prepair(seg::SegArgs a, const uint64_t* __restrict__ g0,
                                                        const uint64_t* __restrict__ x0,
                                                        const uint32_t* __restrict__ code0) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < a.K) seg::seg_prepair(a, t, g0, x0, code0);
}

__global__ void wal_seg_repair(seg::SegArgs a, uint32_t budget) {
  const uint32_t j = (uint32_t)a.info[seg::kInfoFail];
  if (j < a.K) seg::seg_repair(a, j, budget);
}

template <class Rec>
__global__ __launch_bounds__(256) void wal_seg_emit(seg::SegArgs a, uint64_t at, Rec* __restrict__ recs,
                                                     uint64_t* __restrict__ poff, uint32_t* __restrict__ plen,
                                                     uint32_t* __restrict__ pcrc) {
  // one thread per sub-segment (a.nsub per segment; 1: per segment)
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t k = (uint32_t)(t / a.nsub), j = (uint32_t)(t % a.nsub);
  if (k < a.K) seg::seg_emit_thread(a, k, (uint32_t)a.info[seg::kInfoJterm], at, recs, poff, plen, pcrc, j);
}

// the CRC-32 slicing tables T0..T3 in LDS (T0 bitwise, Tk[b] = T(k-1)[b] >> 8
// ^ T0[T(k-1)[b] & 0xFF]), by a 256-thread block, for seg::hdr_reg
__device__ __forceinline__ void build_crc_tables(uint32_t* T) {
  const uint32_t b = threadIdx.x;
  uint32_t c = b;
#pragma unroll
  for (int q = 0; q < 8; ++q) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  T[b] = c;
  __syncthreads();
#pragma unroll
  for (int q = 1; q < 4; ++q) {
    c = (c >> 8) ^ T[c & 0xFFu];
    T[q * 256 + b] = c;
  }
  __syncthreads();
}

// The same with packed CRC spans (seg::Pack): the expected CRC of each span
// from its record's stored CRC and the next header (seg::pack_crc).
template <class Rec>
__global__ __launch_bounds__(256) void wal_seg_emit_packed(seg::SegArgs a, uint64_t at, Rec* __restrict__ recs,
                                                            uint64_t* __restrict__ poff, uint32_t* __restrict__ plen,
                                                            uint32_t* __restrict__ pcrc, uint64_t iend) {
  __shared__ uint32_t T[1024];
  build_crc_tables(T);
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t k = (uint32_t)(t / a.nsub), j = (uint32_t)(t % a.nsub);
  const seg::Pack pk{iend, T};
  if (k < a.K) seg::seg_emit_thread(a, k, (uint32_t)a.info[seg::kInfoJterm], at, recs, poff, plen, pcrc, j, &pk);
}

// The staged segments' records out (seg::seg_place_rec): one wave per
// segment, four per workgroup, its slots read in order -- instead of the
// second walk of the headers seg_emit_thread makes for a segment with more
// records than slots.  A lane takes the next record's header fields from the
// next lane (lane 63 and the segment's last record read them).
template <bool PACK, class Rec>
__global__ __launch_bounds__(256) void wal_seg_place(seg::SegArgs a, uint64_t at, Rec* __restrict__ recs,
                                                     uint64_t* __restrict__ poff, uint32_t* __restrict__ plen,
                                                     uint32_t* __restrict__ pcrc, uint64_t iend) {
  __shared__ uint32_t T[1024];
  if (PACK) build_crc_tables(T);
  const uint32_t k = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (k >= a.K) return;
  const uint32_t jterm = (uint32_t)a.info[seg::kInfoJterm];
  if (k > jterm || a.code[k] == seg::kNone) return;
  const uint32_t cnt = a.recs[k];
  if (cnt > a.scap) return;  // (emitted by wal_seg_emit*)
  const seg::StageRec* st = a.srec + (uint64_t)k * a.scap;
  const uint64_t i0 = at + (a.pre[k] & seg::kRecMask);
  const seg::Pack pk{iend, T};
  // The slots two windows of 64 ahead are loaded while a window is placed (a
  // wave walks its segment's slots in ~20 windows); the record after a
  // window's lane 63 is the next window's lane 0, already loaded.  Three
  // buffers in turn (the loop unrolled by three), so no register copy of a
  // window still in flight makes the wave wait for it a window early.
  // The loads are not branched around (a lane past the segment's records
  // re-reads its last slot, and never uses what it reads): a load into a
  // register that keeps its old value on the other path is a copy the wave
  // waits for at once.
  if (cnt == 0) return;
  const uint32_t last = cnt - 1u;
  seg::StageRec W0 = st[lane < last ? lane : last], W1 = st[64u + lane < last ? 64u + lane : last], W2;
  // window r0: its records R, the next window N (lane 0: the record after
  // lane 63's), and L, free since the window before, refilled with window r0 + 128
  auto window = [&](uint32_t r0, const seg::StageRec& R, const seg::StageRec& N, seg::StageRec& L) {
    const uint32_t r = r0 + lane;
    L = st[r + 128u < last ? r + 128u : last];
    seg::Head nh{};
    if (PACK) {
      const bool l63 = lane == 63u;  // (the next window's lane 0)
      const uint32_t nrel = (uint32_t)__shfl_down(R.rel_t, 1), frel = (uint32_t)__shfl(N.rel_t, 0);
      const uint32_t ncrc = (uint32_t)__shfl_down(R.crc, 1), fcrc = (uint32_t)__shfl(N.crc, 0);
      const uint32_t nkl = (uint32_t)__shfl_down(R.klen, 1), fkl = (uint32_t)__shfl(N.klen, 0);
      const uint32_t nvl = (uint32_t)__shfl_down(R.vlen, 1), fvl = (uint32_t)__shfl(N.vlen, 0);
      nh.t = seg::stage_type(seg::StageRec{l63 ? frel : nrel, 0u, 0u, 0u});
      nh.crc = l63 ? fcrc : ncrc;
      nh.klen = l63 ? fkl : nkl;
      nh.vlen = l63 ? fvl : nvl;
      // the segment's last record: the header at its exit (another segment's first)
      if (r < cnt && r + 1u == cnt && i0 + r + 1u < iend) nh = seg::seg_place_next_head(a, k, r);
    }
    if (r < cnt) seg::seg_place_rec(a, k, i0, recs, poff, plen, pcrc, r, R, nh, PACK ? &pk : nullptr);
  };
  for (uint32_t r0 = 0; r0 < cnt; r0 += 192u) {  // (wave-uniform)
    window(r0, W0, W1, W2);
    if (r0 + 64u >= cnt) break;
    window(r0 + 64u, W1, W2, W0);
    if (r0 + 128u >= cnt) break;
    window(r0 + 128u, W2, W0, W1);
  }
}

// 32-byte records -> the compact form (seg::put_rec), for the walks that
// emit the wide layout (candidate doubling) when the caller asked for lsmck_wal_rec16
__global__ __launch_bounds__(256) void wal_recs_compact(const lsmck_wal_rec* __restrict__ in,
                                                        seg::Compact16* __restrict__ out, uint64_t m) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) {
    const lsmck_wal_rec r = in[i];
    seg::put_rec(out + i, r.rec_off, r.payload_off, r.klen, r.vlen, r.crc, r.type);
  }
}

}  // namespace lsmck

using namespace lsmck;

static int launch_err();

// Segment bytes for a walk over `len` bytes: a power of two from 512 B to
// 16 MiB giving about 2^16 segments (one thread each; same-box sweeps, profiles/r04/j:
// 2 MiB segments walk the 97.8 GiB log in 34.7 ms against 43.1 at 256 KiB and
// 38.0 at 4 MiB, 4 KiB the 0.24 GB one in 0.41 ms against 0.56 at 512 B --
// fewer, longer segments pay the per-segment scan to the first record fewer
// times); `want` overrides.
extern "C" uint64_t lsmk_wal_seg_bytes(uint64_t len, uint64_t want) {
  if (want) return want;
  uint64_t S = 512;
  while (S < (16ull << 20) && (len + S - 1) / S > (1ull << 16)) S <<= 1;
  return S;
}
extern "C" uint64_t lsmk_wal_seg_scan_blocks(uint32_t K) {
  return ((uint64_t)K + 1 + SSCAN_BLOCK * SSCAN_ITEMS - 1) / (SSCAN_BLOCK * SSCAN_ITEMS);
}

// steps 1-2: every segment's guess and walk (a round follows)
#if defined(LSMCK_SEG_CLOCK) && !defined(LSMCK_SEG_GUESS_LANES)
#define LSMCK_SEG_GUESS_LANES 1  // (the clock marks are in the one-lane walk)
#endif
#ifndef LSMCK_SEG_GUESS_LANES
#define LSMCK_SEG_GUESS_LANES 8  // (round 5: four lanes with four-block scan steps before)
#endif
extern "C" int lsmk_wal_seg_walk(const seg::SegArgs* a, hipStream_t st) {
  constexpr int G = LSMCK_SEG_GUESS_LANES;
  if (G == 1) {
    hipLaunchKernelGGL(wal_seg_walk, dim3((a->K + 255) / 256), dim3(256), 0, st, *a);
  } else {
    const uint64_t threads = (uint64_t)a->K * G;
    hipLaunchKernelGGL(wal_seg_walk_group<G>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, *a);
  }
  return launch_err();
}

// one check round: jterm, the placement scan, the check, the outcome in info
// (bsum: lsmk_wal_seg_scan_blocks(K) u64)
extern "C" int lsmk_wal_seg_round(const seg::SegArgs* a, uint64_t* bsum, hipStream_t st) {
  const unsigned g = (a->K + 255) / 256;
  const uint32_t nb = (uint32_t)lsmk_wal_seg_scan_blocks(a->K);
  hipLaunchKernelGGL(wal_seg_reset, dim3(1), dim3(1), 0, st, *a);
  hipLaunchKernelGGL(wal_seg_jterm, dim3(g), dim3(256), 0, st, *a);
  hipLaunchKernelGGL(wal_seg_scan_a, dim3(nb), dim3(SSCAN_BLOCK), 0, st, *a, bsum);
  hipLaunchKernelGGL(wal_seg_scan_b, dim3(1), dim3(1024), 0, st, bsum, nb);
  hipLaunchKernelGGL(wal_seg_scan_c, dim3(nb), dim3(SSCAN_BLOCK), 0, st, *a, (const uint64_t*)bsum);
  hipLaunchKernelGGL(wal_seg_check, dim3(g), dim3(256), 0, st, *a);
  hipLaunchKernelGGL(wal_seg_finalize, dim3(1), dim3(1), 0, st, *a);
  return launch_err();
}

// a parallel repair round: snapshot (K entries of each array) then one thread per segment
extern "C" int lsmk_wal_seg_prepair(const seg::SegArgs* a, uint64_t* g0, uint64_t* x0, uint32_t* code0,
                                    hipStream_t st) {
  if (!a->K) return 0;
  hipError_t e;
  if ((e = hipMemcpyAsync(g0, a->g, (size_t)a->K * 8, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
      (e = hipMemcpyAsync(x0, a->x, (size_t)a->K * 8, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
      (e = hipMemcpyAsync(code0, a->code, (size_t)a->K * 4, hipMemcpyDeviceToDevice, st)) != hipSuccess)
    return -(int)e;
  hipLaunchKernelGGL(wal_seg_prepair, dim3((a->K + 255) / 256), dim3(256), 0, st, *a, (const uint64_t*)g0,
                     (const uint64_t*)x0, (const uint32_t*)code0);
  return launch_err();
}

extern "C" int lsmk_wal_seg_repair(const seg::SegArgs* a, uint32_t budget, hipStream_t st) {
  hipLaunchKernelGGL(wal_seg_repair, dim3(1), dim3(1), 0, st, *a, budget);
  return launch_err();
}

// recs: lsmck_wal_rec[] or, compact, lsmck_wal_rec16[] (seg::Compact16)
extern "C" int lsmk_wal_seg_emit(const seg::SegArgs* a, uint64_t at, void* recs, int compact, uint64_t* poff,
                                 uint32_t* plen, uint32_t* pcrc, hipStream_t st) {
  const dim3 g((unsigned)(((uint64_t)a->K * a->nsub + 255) / 256));
  if (compact)
    hipLaunchKernelGGL(wal_seg_emit<seg::Compact16>, g, dim3(256), 0, st, *a, at, (seg::Compact16*)recs, poff, plen,
                       pcrc);
  else
    hipLaunchKernelGGL(wal_seg_emit<lsmck_wal_rec>, g, dim3(256), 0, st, *a, at, (lsmck_wal_rec*)recs, poff, plen,
                       pcrc);
  return launch_err();
}

extern "C" int lsmk_wal_seg_emit_packed(const seg::SegArgs* a, uint64_t at, void* recs, int compact, uint64_t* poff,
                                        uint32_t* plen, uint32_t* pcrc, uint64_t iend, hipStream_t st) {
  const dim3 g((unsigned)(((uint64_t)a->K * a->nsub + 255) / 256));
  if (compact)
    hipLaunchKernelGGL(wal_seg_emit_packed<seg::Compact16>, g, dim3(256), 0, st, *a, at, (seg::Compact16*)recs, poff,
                       plen, pcrc, iend);
  else
    hipLaunchKernelGGL(wal_seg_emit_packed<lsmck_wal_rec>, g, dim3(256), 0, st, *a, at, (lsmck_wal_rec*)recs, poff,
                       plen, pcrc, iend);
  return launch_err();
}

template <bool PACK, class Rec>
static void seg_place_launch(const seg::SegArgs* a, uint64_t at, Rec* recs, uint64_t* poff, uint32_t* plen,
                             uint32_t* pcrc, uint64_t iend, hipStream_t st) {
  hipLaunchKernelGGL((wal_seg_place<PACK, Rec>), dim3((a->K + 3u) / 4u), dim3(256), 0, st, *a, at, recs, poff, plen,
                     pcrc, iend);
}
extern "C" int lsmk_wal_seg_place(const seg::SegArgs* a, uint64_t at, void* recs, int compact, uint64_t* poff,
                                  uint32_t* plen, uint32_t* pcrc, uint64_t iend, int packed, hipStream_t st) {
  if (!a->scap || !a->K) return 0;
  if (compact) {
    if (packed)
      seg_place_launch<true>(a, at, (seg::Compact16*)recs, poff, plen, pcrc, iend, st);
    else
      seg_place_launch<false>(a, at, (seg::Compact16*)recs, poff, plen, pcrc, iend, st);
  } else {
    if (packed)
      seg_place_launch<true>(a, at, (lsmck_wal_rec*)recs, poff, plen, pcrc, iend, st);
    else
      seg_place_launch<false>(a, at, (lsmck_wal_rec*)recs, poff, plen, pcrc, iend, st);
  }
  return launch_err();
}

extern "C" int lsmk_wal_recs_compact(const lsmck_wal_rec* in, void* out, uint64_t m, hipStream_t st) {
  if (m == 0) return 0;
  hipLaunchKernelGGL(wal_recs_compact, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, in, (seg::Compact16*)out,
                     m);
  return launch_err();
}

extern "C" int lsmk_wal_frame_insert(uint8_t* img, const uint64_t* off, const uint32_t* len, const uint32_t* crc,
                                     uint64_t n, uint32_t kmax, hipStream_t st) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(wal_frame_insert, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, img, off, len, crc, n,
                     kmax);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

static int launch_err() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

extern "C" uint64_t lsmk_wal_words(uint64_t n) { return (n + 63) >> 6; }
extern "C" uint64_t lsmk_wal_scan_blocks(uint64_t n) {
  const uint64_t nw = lsmk_wal_words(n);
  return (nw + WSCAN_BLOCK * WSCAN_ITEMS - 1) / (WSCAN_BLOCK * WSCAN_ITEMS);
}

// phase 1 over the words of bytes [b0, b1) (b0 a multiple of 64): candidate
// bitmap and counts.  A word reads only its own 64 bytes, so an image uploaded
// in 64-byte-aligned chunks is marked chunk by chunk behind its copies.
extern "C" int lsmk_wal_mark_range(const uint8_t* img, uint64_t n, uint64_t b0, uint64_t b1, uint64_t* bits,
                                   uint32_t* pre, hipStream_t st) {
  const uint64_t w0 = b0 >> 6, w1 = lsmk_wal_words(b1 < n ? b1 : n);
  if (w1 <= w0) return 0;
  const int aligned = ((uintptr_t)img & 15) == 0;
  hipLaunchKernelGGL(wal_mark, dim3((unsigned)((w1 - w0 + 255) / 256)), dim3(256), 0, st, img, n, aligned, bits, pre,
                     w0, w1);
  return launch_err();
}

// phase 1-2: bitmap, counts (unless `marked`: lsmk_wal_mark_range ran over the
// whole image), their exclusive scan over words [w0, w1) (ranks relative to
// word w0); *total = candidates there
extern "C" int lsmk_wal_mark(const uint8_t* img, uint64_t n, uint64_t* bits, uint32_t* pre, uint32_t* bsum,
                             uint32_t* total, int marked, uint64_t w0, uint64_t w1, hipStream_t st) {
  if (w1 <= w0) return 0;
  if (!marked) {
    const int rc = lsmk_wal_mark_range(img, n, 0, n, bits, pre, st);
    if (rc) return rc;
  }
  const uint64_t nw = w1 - w0;
  const uint64_t nb = (nw + WSCAN_BLOCK * WSCAN_ITEMS - 1) / (WSCAN_BLOCK * WSCAN_ITEMS);
  hipLaunchKernelGGL(wal_scan_a, dim3((unsigned)nb), dim3(WSCAN_BLOCK), 0, st, pre + w0, nw, bsum);
  hipLaunchKernelGGL(wal_scan_b, dim3(1), dim3(1024), 0, st, bsum, (uint32_t)nb, total);
  hipLaunchKernelGGL(wal_scan_c, dim3((unsigned)nb), dim3(WSCAN_BLOCK), 0, st, pre + w0, nw, bsum);
  return launch_err();
}

// phase 3-5 for the nc candidates of words [w0, w1) (read back by the host),
// the chain from position `start` (a multiple-of-64 prefix [0, lim) when lim <
// n): levels = bit length of nc (2^levels > nc >= the chain's length), J holds
// levels * nc u32, chain 2^levels u32, info 4 u64 (device): records,
// terminal code, bad / resume position
extern "C" int lsmk_wal_chain(const uint8_t* img, uint64_t n, const uint64_t* bits, const uint32_t* pre, uint32_t nc,
                              int levels, uint64_t* pos, uint32_t* J, uint64_t* badpos, uint32_t* chain,
                              unsigned long long* info, uint64_t w0, uint64_t w1, uint64_t start, uint64_t lim,
                              hipStream_t st) {
  hipLaunchKernelGGL(wal_chain_init, dim3(1), dim3(1), 0, st, img, n, bits, pre, start, chain, info);
  if (nc == 0) return launch_err();
  hipLaunchKernelGGL(wal_succ, dim3((unsigned)((w1 - w0 + 255) / 256)), dim3(256), 0, st, img, n, bits, pre, pos, J,
                     badpos, w0, w1, lim);
  for (int k = 0; k + 1 < levels; ++k)
    hipLaunchKernelGGL(wal_double, dim3((nc + 255) / 256), dim3(256), 0, st, J + (uint64_t)k * nc,
                       J + (uint64_t)(k + 1) * nc, nc);
  for (int k = 0; k < levels; ++k) {
    const uint32_t L = 1u << k;
    hipLaunchKernelGGL(wal_unroll, dim3((L + 255) / 256), dim3(256), 0, st, J + (uint64_t)k * nc, chain, L);
  }
  const uint32_t len = 1u << levels;
  hipLaunchKernelGGL(wal_chain_end, dim3((len + 255) / 256), dim3(256), 0, st, chain, len, J, badpos, pos, info);
  return launch_err();
}

// records, descriptors and stored CRCs of the first info[0] chain entries
// (m: their count, read back by the host)
extern "C" int lsmk_wal_emit(const uint8_t* img, uint64_t n, const uint32_t* chain, const uint64_t* pos,
                             const unsigned long long* info, uint32_t m, lsmck_wal_rec* recs, uint64_t* poff,
                             uint32_t* plen, uint32_t* pcrc, hipStream_t st) {
  if (m == 0) return 0;
  hipLaunchKernelGGL(wal_emit, dim3((m + 255) / 256), dim3(256), 0, st, img, n, chain, pos, info, recs, poff, plen,
                     pcrc);
  return launch_err();
}

#ifdef LSMCK_SEG_CLOCK
// (diagnostic) the last segment walk's marks: 3 per segment (start, after
// the guess, after the walk), wall_clock64 ticks (100 MHz)
extern "C" int lsmck_diag_seg_clock(uint64_t* out, size_t n) {
  if (n > 3u * 131072u) n = 3u * 131072u;
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_seg_clock), n * 8, 0, hipMemcpyDeviceToHost);
  return e == hipSuccess ? 0 : -(int)e;
}
#endif
