// lsmck_segwalk.h -- the WAL header walk by segments: the per-thread logic of
// the kernels in lsmck_wal.hip (wal_seg_*), written once for the device and
// for the host model the CPU tests run (tools/segwalk_sim.cpp).
//
// The reference reads the log record by record (src/wal.rs:68-84, 122-163):
// a header's position is the previous record's end, a serial chain.  Here the
// log [start, n) is cut into K segments of S bytes and one GPU thread takes
// each segment:
//   1. its ENTRY -- the first record of the chain that starts in it -- is
//      guessed: segment 0's is `start`; any other scans its bytes for command
//      type bytes (1 Insert, 2 Remove) whose header fits, and takes the first
//      whose own walk is plausible (kAccept complete records, or a clean end
//      of the log; a bogus start inside a payload reads a random length and
//      lands on a non-type byte within a step or two);
//   2. from the guess it walks the headers (one 16-byte load per record, not
//      the payloads) to the first record start at or past the segment's end:
//      its EXIT -- or to the chain's end (EOF, or a bad type byte);
//   3. the guesses are checked all at once: with segment 0 right, every
//      segment before the first one that ends the chain (jterm) must have its
//      exit's segment t's guess equal to that exit, and no guessed segment
//      strictly between them.  By induction along the chain that makes every
//      guessed segment up to jterm a true entry (and the rest of the log past
//      jterm irrelevant: the chain ended there).  The first failure is at a
//      segment whose own entry is right, so its exit is the true entry of t:
//      a repair rewalks t from it and the check runs again.  After too many
//      repairs the caller takes the candidate-doubling walk instead;
//   4. an exclusive scan of the per-segment record counts of the checked
//      segments places each segment's records; each thread walks its segment
//      again and emits them.
// The chain found is the reference's exactly: a record is the one at the
// previous record's end, its payload cut at EOF as read_to_end on take()
// does, the chain ending at EOF (or in a truncated header: UnexpectedEof) or
// at a byte that is not a command type (InvalidCommandType, wal.rs:36).
#ifndef LSMCK_SEGWALK_H
#define LSMCK_SEGWALK_H
#include <stdint.h>
#include <string.h>
#include <assert.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define LSMCK_HD __host__ __device__ __forceinline__
#else
#define LSMCK_HD static inline
#endif

// Diagnostic builds (-DLSMCK_DIAG: tools/build_ab.sh A/B builds, the host
// models of tools/segwalk_repairs.py, clock-mark builds) take the tuning
// values and the per-segment clock marks from lsmck_diag.h; the product build
// has these and no marks.
#ifdef LSMCK_DIAG
#include "lsmck_diag.h"
#else
#define LSMCK_SEG_CLOCK_MARK(k, slot)
namespace lsmck {
namespace seg {
namespace tune {
constexpr uint64_t kLaterSkipTo = 131072;  // kLaterSkipTo below
constexpr uint64_t kLaterMin = 65536;      // kLaterMin below
constexpr uint64_t kLaterScan = 65536;     // kLaterScan below
constexpr int kScanBlocks = 1;             // kScanBlocks below
constexpr bool kLaterAlways = false;       // (host-model A/B: the later-start rule everywhere)
}  // namespace tune
}  // namespace seg
}  // namespace lsmck
#endif

namespace lsmck {
namespace seg {

// a segment's outcome (its walk from the guessed entry)
constexpr uint32_t kNone = 0;  // no entry: the chain passes over the segment (or the guess found none)
constexpr uint32_t kExit = 1;  // the walk left the segment at a record start `pos`
constexpr uint32_t kEnd = 2;   // the chain ends in the segment: EOF (or a truncated header)
constexpr uint32_t kBad = 3;   // the chain ends in the segment: `pos` holds a byte that is not a command type
constexpr uint64_t kNoGuess = ~0ull;
constexpr uint32_t kNoSeg = 0xFFFFFFFFu;
// a guessed entry must lead to this many complete records (or to a clean
// end of the log) before it is taken: a bogus one passes its first step only
// with a first record of at most the hop (below), and then each further one
// with ~1/128 odds on random payloads -- ~1e-11 per candidate for a 64 KiB
// hop.  (Six ran the 0.24 GB log's walk 3% slower and caught nothing more,
// profiles/r04/o; a wrong guess that passes is caught by the check anyway.)
constexpr uint32_t kAccept = 4;
// ... and its first record must end within this many bytes (or the segment
// length, if longer).  A bogus start reads a random 32-bit length; on a log
// past 4 GiB it lands inside the log, and exactly on a true record with odds
// of (records / bytes), ~1/1,500 for config 3w -- a merge with the true
// chain that the acceptance test cannot see, and with ~100 bogus starts
// scanned before a segment's first true record, one segment in ~13 would
// be guessed wrong.  A first record of at most kHop bytes cuts that by
// 4 GiB / 64 KiB.  A true first record longer than this is refused and
// repaired by the check (or the walk re-segments, with longer hops).
constexpr uint64_t kHop = 65536;
// The later-start rule (guess()) is skipped for segments of 4 KiB up to (not
// including) 128 KiB: there a wrong guess that merges with the chain is rare
// (none in the host model's logs: tools/segwalk_sim.cpp over wal_diag-like,
// binary-payload and Zipf logs, 4 to 64 KiB segments), and the rule's scan of
// the accepted record's payload is most of a small segment's guess (0.24 GB
// log: 0.33 vs 0.42 ms, profiles/r04/o).  Segments shorter than records
// (under 4 KiB) often hold no true start, and long hops (2 MiB segments)
// let bogus lengths land on a true record: the rule stays for both.
constexpr uint64_t kLaterSkipFrom = 4096, kLaterSkipTo = tune::kLaterSkipTo;
// From kLaterSkipTo on, the rule runs only for a guess whose first record is
// longer than kHop payload bytes.  A bogus start whose random 32-bit length is
// at most kHop lands on a true record with odds ~(records / bytes) * 2^-16
// (~1e-8 per candidate for config 3w); a longer one is the merge the rule is
// for.  A true first record of at most kHop (every record of config 3w) then
// costs no scan of its payload: 7.72 -> ~6.2 ms of walk for the 97.8 GiB log
// (without the rule at all: 6.21 ms and three repairs of 0.87 ms each,
// profiles/r04/v).  A wrong guess is caught by the check either way.
constexpr uint64_t kLaterMin = tune::kLaterMin;
// ... and then scans at most kLaterScan bytes past the guess for the later
// start.  The rule scanned the whole first record, and a true first record of
// a MiB -- in a log of MiB values, every segment's -- cost the 97.8 GiB log
// 216 ms of walk (profiles/r05/d).  A bogus merge's true entry is the first
// true start after it, within one true record: every one of them in a log of
// records of at most kLaterScan (config 3w) is still found.  Capping the
// first record's length instead (at 256 KiB) left config 3w's bogus merges
// to the check: a parallel repair round of ~1 ms in every replay
// (profiles/r05/kt).  A longer-range merge is caught by the check and
// repaired (seg_prepair).
constexpr uint64_t kLaterScan = tune::kLaterScan;
// 64-byte blocks the guess scan loads per iteration.  One (round 5): the
// walk kernel then needs 63 VGPRs instead of 123 -- eight waves a SIMD, so
// twice the segments' groups in flight -- and each guess takes eight lanes
// (97.8 GiB config-3w log 25.0-25.15 -> 24.8-24.9 ms in HBM, ~1 MiB values
// 40.8 -> 35.3 ms; profiles/r05/sb/)
constexpr int kScanBlocks = tune::kScanBlocks;
// per-segment record counts and the guessed-segment count share one u64 in
// the placement scan: guessed segments in the top 24 bits, records below
constexpr int kSegShift = 40;
constexpr uint64_t kRecMask = (1ull << kSegShift) - 1;

struct WalkOut {
  uint32_t code;  // kExit / kEnd / kBad
  uint32_t recs;  // records of the chain that start in the segment
  uint64_t pos;   // kExit: the next record (at or past the segment end); kBad: the bad byte
};

LSMCK_HD uint32_t hdr_len(uint32_t t) { return t == 1 ? 13u : 9u; }
// bytes s .. s+3 of the 8-byte little-endian pair lo, hi (s = 0..3: v_alignbyte)
LSMCK_HD uint32_t fsh(uint32_t hi, uint32_t lo, uint32_t s) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * s));
}

// The header at q, read at once: whether q starts a record (cl: 0), or ends
// the chain -- EOF at or inside the header (kEnd, wal.rs:76-77) or a byte that
// is not a command type (kBad) -- and the header's fields.  One 16-byte load
// of the four dwords holding bytes q .. q+12 (address-aligned to 4; the
// dwords at the image's two ends are read byte by byte instead): a lane's
// loads are what the walk's time goes to, so one per record, not one per byte.
struct Head {
  uint32_t cl;
  uint32_t t, crc, klen, vlen;  // vlen 0 for Remove
};
// head() in two halves, so that a walk can issue the next header's load,
// then the stores of the record it has passed, and only then wait for the
// load (head_dec's first use): on gfx950 one counter covers loads and stores
// and completes in issue order, so a store issued before the load would be
// waited for with it.
struct RawHead {
  uint32_t d0, d1, d2, d3;  // the four dwords holding bytes q .. q+15 (from byte s of d0)
  uint32_t s;
  uint32_t end;  // q at or past EOF
};
LSMCK_HD RawHead head_raw(const uint8_t* img, uint64_t n, uint64_t q) {
  RawHead r{};
  if (q >= n) {
    r.end = 1;
    return r;
  }
  const uintptr_t A = ((uintptr_t)img + q) & ~(uintptr_t)3;
  const int64_t a0 = (int64_t)(A - (uintptr_t)img);
  if (a0 >= 0 && (uint64_t)a0 + 16 <= n) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
    const u32x4a4 v = *(const __attribute__((address_space(1))) u32x4a4*)A;  // global_load_dwordx4
    r.d0 = v.x;
    r.d1 = v.y;
    r.d2 = v.z;
    r.d3 = v.w;
#else
    uint32_t d[4];
    memcpy(d, (const void*)A, 16);
    r.d0 = d[0];
    r.d1 = d[1];
    r.d2 = d[2];
    r.d3 = d[3];
#endif
    r.s = (uint32_t)(((uintptr_t)img + q) & 3u);
  } else {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < 16u; ++i)
      if (q + i < n) w[i >> 2] |= (uint32_t)img[q + i] << (8u * (i & 3u));
    r.d0 = w[0];
    r.d1 = w[1];
    r.d2 = w[2];
    r.d3 = w[3];
  }
  return r;
}
LSMCK_HD Head head_dec(const RawHead& r, uint64_t n, uint64_t q) {
  Head h{};
  if (r.end) {
    h.cl = kEnd;
    return h;
  }
  const uint32_t e0 = fsh(r.d1, r.d0, r.s), e1 = fsh(r.d2, r.d1, r.s), e2 = fsh(r.d3, r.d2, r.s),
                 e3 = fsh(0u, r.d3, r.s);
  h.t = e0 & 0xFFu;
  if (h.t != 1u && h.t != 2u) {
    h.cl = kBad;
    return h;
  }
  if (q + hdr_len(h.t) > n) {
    h.cl = kEnd;
    return h;
  }
  h.crc = (e0 >> 8) | (e1 << 24);
  h.klen = (e1 >> 8) | (e2 << 24);
  h.vlen = h.t == 1u ? ((e2 >> 8) | (e3 << 24)) : 0u;
  return h;
}
LSMCK_HD Head head(const uint8_t* img, uint64_t n, uint64_t q) { return head_dec(head_raw(img, n, q), n, q); }

// the record at p with header h: where the next one starts -- its payload cut
// at EOF (wal.rs:130-133) -- and whether the payload is whole.  The length is
// key_len + val_len in u32, as wal.rs:129 (wrapping).
LSMCK_HD uint64_t next_of(const Head& h, uint64_t n, uint64_t p, bool* whole) {
  const uint32_t hl = hdr_len(h.t);
  const uint32_t dlen = h.klen + h.vlen;
  const uint64_t avail = n - (p + hl);
  *whole = dlen <= avail;
  return p + hl + (*whole ? (uint64_t)dlen : avail);
}

// A record as the walk stages it: segment k's walk writes its records to its
// own slots [k * scap, k * scap + scap) as it passes them, so the records need
// no second walk of the headers when they all fit (seg_place_thread copies
// them out); a segment with more records than slots is emitted by its second
// walk as before (seg_emit_thread).  16 bytes: the record's offset from its
// segment's start (bits 0-30; a segment's records start inside it, and the
// walk stages only for segments of at most kStageMaxSeg bytes), Remove in bit
// 31, then the header's CRC and lengths.
struct StageRec {
  uint32_t rel_t, crc, klen, vlen;
};
static_assert(sizeof(StageRec) == 16, "the staging budget and the place kernel assume 16-byte slots");
constexpr uint64_t kStageMaxSeg = 1ull << 31;
LSMCK_HD uint32_t stage_type(const StageRec& R) { return (R.rel_t >> 31) ? 2u : 1u; }
LSMCK_HD uint64_t stage_off(const StageRec& R, uint64_t b0) { return b0 + (R.rel_t & 0x7FFFFFFFu); }
// b0: the segment's start.  Staged (S) walks store every record: past the
// segment's cap slots the last slot is overwritten, harmlessly -- a segment
// with more records than slots is emitted by its second walk and its slots are
// not read -- so the store is not branched around, and the wait for the next
// header's load (issued before it) need not cover it (head_raw).
template <bool S>
LSMCK_HD void stage_put(StageRec* st, uint32_t cap, uint32_t cnt, uint64_t p, const Head& h, uint64_t b0) {
  if (S) {
#if !defined(__HIP_DEVICE_COMPILE__)
    assert(st && cap && p >= b0 && p - b0 < kStageMaxSeg);  // (the host model's runs check the layout's premise)
#endif
    StageRec R;
    R.rel_t = (uint32_t)(p - b0) | (h.t == 2u ? 0x80000000u : 0u);
    R.crc = h.crc;
    R.klen = h.klen;
    R.vlen = h.vlen;
    st[cnt < cap ? cnt : cap - 1] = R;
  }
}

// The segment's outcome from its entry c (a record start on the chain, or
// the guess; h its header): the walk through the segment ending at e, to the
// first record start at or past e (kExit) or to the chain's end (kEnd / kBad).
// st: the segment's staging slots (scap of them), or none.
template <bool S>
LSMCK_HD void walk_t(const uint8_t* img, uint64_t n, uint64_t c, Head h, uint64_t e, WalkOut* o, StageRec* st,
                     uint32_t scap, uint64_t b0) {
  uint64_t p = c;
  uint32_t cnt = 0;
  for (;;) {
    if (p >= e) {
      o->code = kExit;
      o->pos = p;
      o->recs = cnt;
      return;
    }
    bool whole;
    const uint64_t q = next_of(h, n, p, &whole);
    const RawHead r = head_raw(img, n, q);  // (issued before the record's store: head_raw)
    stage_put<S>(st, scap, cnt, p, h, b0);
    ++cnt;
    h = head_dec(r, n, q);
    if (h.cl) {  // the chain ends after the record at p
      o->code = h.cl;
      o->pos = q;
      o->recs = cnt;
      return;
    }
    p = q;
  }
}
LSMCK_HD void walk(const uint8_t* img, uint64_t n, uint64_t c, Head h, uint64_t e, WalkOut* o,
                   StageRec* st = nullptr, uint32_t scap = 0, uint64_t b0 = 0) {
  if (st) walk_t<true>(img, n, c, h, e, o, st, scap, b0);
  else walk_t<false>(img, n, c, h, e, o, st, scap, b0);
}

// Whether a candidate start c (a type byte whose header fits) is plausible:
// its first record ends within `hop` bytes, and its chain holds kAccept whole
// records, or ends cleanly at EOF before that.
// At most kAccept + 1 headers are read, so the lanes of a wave that test
// candidates stay together; the long walk through the segment runs after the
// guess, in step across the wave.
LSMCK_HD bool accept(const uint8_t* img, uint64_t n, uint64_t c, uint64_t hop) {
  uint64_t p = c;
  Head h = head(img, n, c);
  for (uint32_t good = 0;;) {
    bool whole;
    const uint64_t q = next_of(h, n, p, &whole);
    if (p == c && q - c > hop) return false;  // a first record this long: not taken (kHop)
    good += whole;
    if (good >= kAccept) return true;
    h = head(img, n, q);
    if (h.cl) return whole && h.cl == kEnd;
    p = q;
  }
}
// bit 8j+7 set where byte j of v is 1 or 2 (exact, no cross-byte carries)
LSMCK_HD uint32_t type_bytes(uint32_t v) {
  const uint32_t hi = v & 0xFCFCFCFCu;  // zero iff the byte is < 4
  const uint32_t z = ~(((hi & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | hi | 0x7F7F7F7Fu);
  const uint32_t lo = v & 0x03030303u;  // the byte's low two bits: 1 or 2, not 0 or 3
  return z & (((lo ^ (lo >> 1)) & 0x01010101u) << 7);
}
// 16 bytes at an address aligned to 16 (device: one vector load)
LSMCK_HD void load16(const uint8_t* a, uint32_t w[4]) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)(uintptr_t)a;
  w[0] = v.x;
  w[1] = v.y;
  w[2] = v.z;
  w[3] = v.w;
#else
  memcpy(w, a, 16);
#endif
}
// The scan's current chunk: kScanBlocks 64-byte blocks, aligned in the
// address space, and their type-byte masks.  A lane steps through the
// candidates of a chunk without loading it again.
constexpr int64_t kNoChunk = INT64_MIN;
struct Scan {
  int64_t p0 = kNoChunk;  // image position of the chunk's first byte (< 0: before the image)
  uint64_t m[kScanBlocks];
};
// The first type byte c in [from, e) whose header fits, or kNoGuess.  The
// chunk holding `from` comes from S when it is the one already loaded (vector
// loads inside the image, byte loads at its two ends); then the ones after it.
LSMCK_HD uint64_t next_cand(Scan& S, const uint8_t* img, uint64_t n, uint64_t from, uint64_t e) {
  // all the chunk's loads are in flight together, so a lane that starts
  // inside a long record waits on a quarter as many dependent loads (the
  // wave waits for its slowest lane)
  const uintptr_t base = (uintptr_t)img;
  for (uintptr_t A = (base + from) & ~(uintptr_t)(64 * kScanBlocks - 1);; A += 64 * kScanBlocks) {
    const int64_t p0 = (int64_t)(A - base);
    if (p0 >= (int64_t)e) return kNoGuess;
    if (p0 != S.p0) {
      S.p0 = p0;
      if (p0 >= 0 && (uint64_t)p0 + 64 * kScanBlocks <= n) {
        uint32_t w[16 * kScanBlocks];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int q = 0; q < 4 * kScanBlocks; ++q) load16((const uint8_t*)A + 16 * q, w + 4 * q);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int j = 0; j < kScanBlocks; ++j) {
          uint64_t mj = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
          for (int d = 0; d < 16; ++d) {
            const uint32_t f = type_bytes(w[16 * j + d]);
            const uint64_t nib = ((f >> 7) & 1u) | ((f >> 14) & 2u) | ((f >> 21) & 4u) | ((f >> 28) & 8u);
            mj |= nib << (4 * d);
          }
          S.m[j] = mj;
        }
      } else {
        for (int j = 0; j < kScanBlocks; ++j) {
          uint64_t mj = 0;
          for (int i = 0; i < 64; ++i) {
            const int64_t p = p0 + 64 * j + i;
            if (p >= 0 && (uint64_t)p < n) {
              const uint32_t t = img[p];
              if (t == 1 || t == 2) mj |= 1ull << i;
            }
          }
          S.m[j] = mj;
        }
      }
    }
    for (int j = 0; j < kScanBlocks; ++j) {
      // only positions in [from, e)
      const int64_t pj = p0 + 64 * j;
      const int64_t lo = (int64_t)from - pj, hi = (int64_t)e - pj;
      if (hi <= 0) return kNoGuess;
      if (lo >= 64) continue;
      uint64_t mj = S.m[j];
      if (lo > 0) mj &= ~0ull << lo;
      if (hi < 64) mj &= (1ull << hi) - 1ull;
      while (mj) {
        const int i = __builtin_ctzll(mj);
        mj &= mj - 1;
        const uint64_t c = (uint64_t)(pj + i);
        if (c + 13u <= n || c + hdr_len(img[c]) <= n) return c;  // (the byte is read only at the image's end)
      }
    }
  }
}
// whether the chain from the record start c passes through position q > c
// (q is at most a hop past the candidate that asks: a bounded walk)
LSMCK_HD bool reaches(const uint8_t* img, uint64_t n, uint64_t c, uint64_t q) {
  uint64_t p = c;
  Head h = head(img, n, c);
  while (p < q) {
    bool whole;
    p = next_of(h, n, p, &whole);
    if (p >= q) break;
    h = head(img, n, p);
    if (h.cl) return false;
  }
  return p == q;
}
// The guess of a segment [b, e) (b > start): the first type byte c in it
// whose header fits and which accept() takes -- unless a later start inside
// c's first record has a chain through that record's end, which is then
// preferred (the same test again from it).  The common wrong guess is a
// bogus start before the segment's first true record whose random length
// happens to land on a later true record: its chains merge with the true
// one, so its walk is taken, but its first "record" covers the true entry,
// whose chain reaches the merge point (`later`: the rule runs; see
// kLaterSkipFrom).  kNoGuess: no start taken.
// the later-start rule from an accepted start c (see guess())
LSMCK_HD uint64_t later_rule(Scan& S, const uint8_t* img, uint64_t n, uint64_t c, uint64_t e, uint64_t later_min) {
  for (;;) {
    bool whole;
    const Head hc = head(img, n, c);
    const uint64_t q1 = next_of(hc, n, c, &whole);
    uint64_t lim = q1 < e ? q1 : e;
    if (later_min) {
      if (q1 - c - hdr_len(hc.t) <= later_min) return c;  // (kLaterMin)
      if (lim > c + 1 + kLaterScan) lim = c + 1 + kLaterScan;  // (kLaterScan)
    }
    uint64_t c2 = next_cand(S, img, n, c + 1, lim);
    while (c2 != kNoGuess && !reaches(img, n, c2, q1)) c2 = next_cand(S, img, n, c2 + 1, lim);
    if (c2 == kNoGuess) return c;
    c = c2;
  }
}
LSMCK_HD uint64_t guess(const uint8_t* img, uint64_t n, uint64_t b, uint64_t e, uint64_t hop, bool later = true,
                        uint64_t later_min = 0) {
  Scan S;
  for (uint64_t c = next_cand(S, img, n, b, e); c != kNoGuess; c = next_cand(S, img, n, c + 1, e)) {
    if (!accept(img, n, c, hop)) continue;
    if (!later) return c;
    return later_rule(S, img, n, c, e, later_min);
  }
  return kNoGuess;
}
// --- the per-thread steps of the kernels ------------------------------------
// Per segment k: g[k] (the guessed entry), x[k] (kExit: the exit; kBad: the
// bad byte), code[k], recs[k].  info: u64 words, see kInfo*.
enum : int {
  kInfoJterm = 0,  // u32 at info word 0: the first segment whose walk ends the chain (atomic min)
  kInfoFail = 1,   // u32 at info word 1: the first segment failing the check (atomic min)
  kInfoRecs = 2,   // finalize: records of segments 0..jterm
  kInfoCode = 3,   // finalize: jterm's code (kEnd / kBad)
  kInfoPos = 4,    // finalize: jterm's bad byte
  kInfoFailX = 5,  // finalize: the failing segment's exit
  kInfoNFail = 6,  // u32 at info word 6: how many segments fail the check (atomic add)
  kInfoLast = 7,   // u32 at info word 7: 1 + the last guessed segment whose exit is at or past lim (atomic max)
  kInfoWords = 8
};

// The walk covers the records that start in [start, lim) (lim <= n: a prefix
// of the rest of the log; the next prefix resumes at the first record start
// at or past lim, its records emitted after these).
struct SegArgs {
  const uint8_t* img;
  uint64_t n;
  uint64_t start;  // the chain's first record
  uint64_t S;      // segment bytes
  uint32_t K;      // segments: ceil((lim - start) / S)
  uint64_t* g;
  uint64_t* x;
  uint32_t* code;
  uint32_t* recs;
  uint64_t* pre;  // K + 1: exclusive scan of the placement words
  unsigned long long* info;
  uint64_t lim;   // the prefix end
  // emit checkpoints (nsub > 1): segment k's walk notes, for each of its
  // nsub sub-segments j (bytes [begin + j*sub, ..)), the first chain record
  // starting at or past the sub-segment's start (cpp) and how many of the
  // segment's records come before it (cpc) -- the emit then runs one thread
  // per sub-segment instead of one per segment
  uint32_t nsub;
  uint64_t sub;
  uint64_t* cpp;  // K * nsub
  uint32_t* cpc;
  // walk-time staging (StageRec): scap slots per segment, 0 = none
  StageRec* srec;
  uint32_t scap;
};
LSMCK_HD StageRec* seg_stage(const SegArgs& a, uint32_t k) {
  return a.scap ? a.srec + (uint64_t)k * a.scap : nullptr;
}

LSMCK_HD uint64_t seg_begin(const SegArgs& a, uint32_t k) { return a.start + (uint64_t)k * a.S; }
LSMCK_HD uint64_t seg_end(const SegArgs& a, uint32_t k) {
  const uint64_t e = a.start + (uint64_t)(k + 1) * a.S;
  return e < a.lim ? e : a.lim;
}
// the segment holding pos; K for a position at or past lim (beyond the prefix)
LSMCK_HD uint32_t seg_of(const SegArgs& a, uint64_t pos) {
  return pos >= a.lim ? a.K : (uint32_t)((pos - a.start) / a.S);
}

// the forced walk of segment k from its entry c (a position on the chain)
// walk() of segment k from its entry c (header h), noting the emit
// checkpoints as it passes each sub-segment's start
template <bool S>
LSMCK_HD void walk_cp_t(const SegArgs& a, uint32_t k, uint64_t c, Head h, WalkOut* o) {
  const uint8_t* img = a.img;
  const uint64_t n = a.n, e = seg_end(a, k), b0 = seg_begin(a, k);
  uint64_t* cpp = a.cpp + (uint64_t)k * a.nsub;
  uint32_t* cpc = a.cpc + (uint64_t)k * a.nsub;
  StageRec* st = seg_stage(a, k);
  uint32_t j = 0;
  uint64_t p = c;
  uint32_t cnt = 0;
  for (;;) {
    for (; j < a.nsub && b0 + j * a.sub <= p; ++j) {  // sub-segments whose start p is the first record at or past
      cpp[j] = p;
      cpc[j] = cnt;
    }
    if (p >= e) {
      o->code = kExit;
      o->pos = p;
      o->recs = cnt;
      break;
    }
    bool whole;
    const uint64_t q = next_of(h, n, p, &whole);
    const RawHead r = head_raw(img, n, q);  // (issued before the record's store: head_raw)
    stage_put<S>(st, a.scap, cnt, p, h, b0);
    ++cnt;
    h = head_dec(r, n, q);
    if (h.cl) {
      o->code = h.cl;
      o->pos = q;
      o->recs = cnt;
      p = q;
      break;
    }
    p = q;
  }
  for (; j < a.nsub; ++j) {  // past the chain's end or the exit: no records there
    cpp[j] = p;
    cpc[j] = cnt;
  }
}
LSMCK_HD void walk_cp(const SegArgs& a, uint32_t k, uint64_t c, Head h, WalkOut* o) {
  if (a.scap) walk_cp_t<true>(a, k, c, h, o);
  else walk_cp_t<false>(a, k, c, h, o);
}

LSMCK_HD void seg_forced(const SegArgs& a, uint32_t k, uint64_t c) {
  WalkOut o;
  const Head h = head(a.img, a.n, c);
  if (h.cl) {
    o.code = h.cl;
    o.pos = c;
    o.recs = 0;
    for (uint32_t j = 0; a.nsub > 1 && j < a.nsub; ++j) {  // no records in any sub-segment
      a.cpp[(uint64_t)k * a.nsub + j] = c;
      a.cpc[(uint64_t)k * a.nsub + j] = 0;
    }
  } else if (a.nsub > 1) {
    walk_cp(a, k, c, h, &o);
  } else {
    walk(a.img, a.n, c, h, seg_end(a, k), &o, seg_stage(a, k), a.scap, seg_begin(a, k));
  }
  a.g[k] = c;
  a.x[k] = o.pos;
  a.code[k] = o.code;
  a.recs[k] = o.recs;
}

// step 1-2 for segment k
// the guess's parameters for the walk's segments
LSMCK_HD uint64_t seg_hop(const SegArgs& a) { return a.S > kHop ? a.S : kHop; }
LSMCK_HD bool seg_later(const SegArgs& a) {
  return tune::kLaterAlways || a.S < kLaterSkipFrom || a.S >= kLaterSkipTo;
}
LSMCK_HD uint64_t seg_later_min(const SegArgs& a) {
  return !tune::kLaterAlways && a.S >= kLaterSkipTo ? kLaterMin : 0;
}
LSMCK_HD void seg_take_guess(const SegArgs& a, uint32_t k, uint64_t c);
LSMCK_HD void seg_walk_thread(const SegArgs& a, uint32_t k) {
  LSMCK_SEG_CLOCK_MARK(k, 0);
  if (k == 0) {
    seg_forced(a, 0, a.start);
    return;
  }
  const uint64_t c = guess(a.img, a.n, seg_begin(a, k), seg_end(a, k), seg_hop(a), seg_later(a), seg_later_min(a));
  LSMCK_SEG_CLOCK_MARK(k, 1);
  seg_take_guess(a, k, c);
  LSMCK_SEG_CLOCK_MARK(k, 2);
}
// segment k from its guess c: its walk, or no entry
LSMCK_HD void seg_take_guess(const SegArgs& a, uint32_t k, uint64_t c) {
  if (c == kNoGuess) {
    a.g[k] = c;
    a.x[k] = 0;
    a.code[k] = kNone;
    a.recs[k] = 0;
  } else {
    seg_forced(a, k, c);  // the walk from the guess (every lane of the wave at once)
  }
}

// placement word of segment k (the scan's input): guessed segments up to jterm
LSMCK_HD uint64_t seg_word(const SegArgs& a, uint32_t k, uint32_t jterm) {
  return (a.code[k] != kNone && k <= jterm) ? ((1ull << kSegShift) | a.recs[k]) : 0ull;
}

// step 3 for segment k: whether it fails the check (after the scan)
LSMCK_HD bool seg_check_fails(const SegArgs& a, uint32_t k, uint32_t jterm) {
  if (k >= jterm || a.code[k] == kNone) return false;
  if (a.code[k] != kExit) return true;  // (cannot happen: jterm is the first chain end)
  const uint32_t t = seg_of(a, a.x[k]);
  const uint64_t between = (a.pre[t] >> kSegShift) - (a.pre[k + 1] >> kSegShift);
  return between != 0 || (t < a.K && a.g[t] != a.x[k]);  // (t == K: the exit leaves the prefix)
}

// repair after a failure at segment j (whose entry is right): the segments
// strictly inside its exit's span are cleared, the exit's segment t is walked
// from that exit, and so on while t's own exit does not meet a consistent
// guess -- at most `budget` segments rewalked.  One thread.
LSMCK_HD void seg_repair(const SegArgs& a, uint32_t j, uint32_t budget) {
  for (uint32_t step = 0; step < budget; ++step) {
    if (a.code[j] != kExit) return;
    const uint64_t xe = a.x[j];
    const uint32_t t = seg_of(a, xe);
    bool clean = t == a.K || a.g[t] == xe;  // (t == K: the exit leaves the prefix)
    for (uint32_t u = j + 1; u < t; ++u) {
      if (a.code[u] != kNone) clean = false;
      a.g[u] = kNoGuess;
      a.code[u] = kNone;
      a.recs[u] = 0;
    }
    if (clean) return;
    seg_forced(a, t, xe);
    j = t;
  }
}

// A parallel repair round (after a check with several failures), from a
// snapshot g0 / x0 / code0 of the round's arrays: segment t takes its entry
// from the exit of the nearest guessed segment k before it (at most
// kPrepairBack back) -- walked from that exit when the exit lies in t and t
// guessed otherwise, cleared when the exit passes over t.  Every segment at
// once, one thread each, each writing only its own arrays.  The serial
// repair above fixes one run of failures per launch from the first failing
// segment on; a log whose payloads are framed records (a log of logs: the
// guesses inside a value follow the value's own chain, which ends where the
// value does, at the log's next header) fails at every segment, yet every
// walk's exit is right -- the guessed chain merges with the log's before
// leaving the segment -- so one such round repairs them all.  Nothing here
// is trusted: the check runs again after it, and a wrong predecessor exit
// only costs another round (the caller bounds them, then repairs serially).
constexpr uint32_t kPrepairBack = 256;
LSMCK_HD void seg_prepair(const SegArgs& a, uint32_t t, const uint64_t* g0, const uint64_t* x0,
                          const uint32_t* code0) {
  if (t == 0 || t >= a.K) return;
  uint32_t k = t - 1;
  for (uint32_t s = 0; s < kPrepairBack && k > 0 && code0[k] == kNone; ++s) --k;
  if (code0[k] != kExit) return;  // (kNone: too far back; kEnd / kBad: the chain ends before t)
  const uint64_t e = x0[k];
  const uint32_t te = seg_of(a, e);
  if (te > t) {  // t lies inside k's last record: no entry
    if (code0[t] != kNone) {
      a.g[t] = kNoGuess;
      a.x[t] = 0;
      a.code[t] = kNone;
      a.recs[t] = 0;
    }
  } else if (te == t && (code0[t] == kNone || g0[t] != e)) {
    seg_forced(a, t, e);
  }
}

// The raw CRC-32 register after a header's bytes [t][crc][klen]([vlen]) fed
// from register 0, by the four slicing tables T (T0..T3, 256 words each).
LSMCK_HD uint32_t hdr_reg(const Head& h, const uint32_t* T) {
  auto sl4 = [T](uint32_t x) {
    return T[768 + (x & 0xFFu)] ^ T[512 + ((x >> 8) & 0xFFu)] ^ T[256 + ((x >> 16) & 0xFFu)] ^ T[x >> 24];
  };
  uint32_t r = T[h.t & 0xFFu];
  r = sl4(r ^ h.crc);
  r = sl4(r ^ h.klen);
  if (h.t == 1) r = sl4(r ^ h.vlen);
  return r;
}

// Packed CRC spans (Pack non-null): record i's CRC-pass span is its payload
// and the NEXT record's header, [payload_i | header_i+1), so the spans tile
// the log and the stream kernel runs on them as on config 3's packed objects.
// The last record of the emit (iend: at + records walked) keeps its payload
// alone, and so does a payload within a header of 4 GiB (pack_fits).  The
// expected CRC written for a packed span is the stored CRC carried over the
// next header by linearity (pack_crc), so the compare is the plain one; a
// bad record's computed CRC is taken back to its payload's (unpack_crc) for
// the report.
struct Pack {
  uint64_t iend;
  const uint32_t* T;  // CRC-32 slicing tables T0..T3 (hdr_reg)
};
LSMCK_HD bool pack_fits(uint32_t got, uint32_t hl) { return got <= 0xFFFFFFFFu - hl; }

// c(x) * b(x) mod P(x), reflected (bit 31 is x^0): 32 steps, no branch
LSMCK_HD uint32_t gf2_mul(uint32_t c, uint32_t b) {
  uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    p ^= b & (0u - ((c >> i) & 1u));
    b = (b >> 1) ^ (0xEDB88320u & (0u - (b & 1u)));
  }
  return p;
}
// The CRC of a payload P from the CRC c of its packed span P | H, H the next
// record's header nh:  crc(P) = ~( x^(-8|H|) * (~c ^ hdr_reg(H)) ) mod P(x),
// x^-104 and x^-72 the constants (tests/test_segwalk_model.py checks them).
LSMCK_HD uint32_t unpack_crc(uint32_t c, const Head& nh, const uint32_t* T) {
  return ~gf2_mul(~c ^ hdr_reg(nh, T), nh.t == 1 ? 0x525983aau : 0x2fb98a7du);
}
// ... and the other way: what crc(P | H) is when crc(P) is the stored CRC
// `crc` -- the expected value the emit writes for a packed span, so that the
// compare is the plain one:  ~( x^(8|H|) * ~crc ^ hdr_reg(H) ),  x^104 / x^72.
LSMCK_HD uint32_t pack_crc(uint32_t crc, const Head& nh, const uint32_t* T) {
  return ~(gf2_mul(~crc, nh.t == 1 ? 0xe6050901u : 0x1eb014d8u) ^ hdr_reg(nh, T));
}

// The records the emit writes: the 32-byte lsmck_wal_rec layout (any struct
// with its fields), or the 16-byte compact one (lsmck_wal_rec16, include/
// lsmck.h): the payload offset with the type in bit 63 (set: Remove), klen,
// vlen -- what MemTable::from_log takes from a record (src/memtable.rs:28-47);
// the header offset is the payload's less hdr_len, and the stored CRC is the
// computed one for every accepted record.
struct Compact16 {
  uint64_t payload_type;
  uint32_t klen, vlen;
};
constexpr uint64_t kRemoveBit = 1ull << 63;
static_assert(sizeof(Compact16) == 16, "Compact16 is lsmck_wal_rec16 (include/lsmck.h)");
#ifdef LSMCK_H  // (the host side: the public layout is in scope -- tie the two together)
static_assert(sizeof(Compact16) == sizeof(lsmck_wal_rec16) &&
                  offsetof(Compact16, payload_type) == offsetof(lsmck_wal_rec16, payload_type) &&
                  offsetof(Compact16, klen) == offsetof(lsmck_wal_rec16, klen) &&
                  offsetof(Compact16, vlen) == offsetof(lsmck_wal_rec16, vlen) &&
                  kRemoveBit == LSMCK_WAL_REC16_REMOVE,
              "seg::Compact16 and lsmck_wal_rec16 must share one layout");
#endif
LSMCK_HD void put_rec(Compact16* r, uint64_t rec_off, uint64_t payload_off, uint32_t klen, uint32_t vlen,
                      uint32_t crc, uint32_t type) {
  (void)rec_off;
  (void)crc;
  Compact16 O;
  O.payload_type = payload_off | (type == 2u ? kRemoveBit : 0ull);
  O.klen = klen;
  O.vlen = vlen;
  *r = O;
}
template <class Rec>
LSMCK_HD void put_rec(Rec* r, uint64_t rec_off, uint64_t payload_off, uint32_t klen, uint32_t vlen, uint32_t crc,
                      uint32_t type) {
  Rec O;
  O.rec_off = rec_off;
  O.payload_off = payload_off;
  O.klen = klen;
  O.vlen = vlen;
  O.crc = crc;
  O.type = type;
  *r = O;
}

// step 4 for segment k (after the check passed): its records at `at` + its
// place, as lsmck_wal_rec entries, CRC descriptors and stored CRCs
// (sub-segment j of segment k when a.nsub > 1: its records only, from the
// checkpoint the walk noted)
template <class Rec>
LSMCK_HD void seg_emit_thread(const SegArgs& a, uint32_t k, uint32_t jterm, uint64_t at, Rec* recs, uint64_t* poff,
                              uint32_t* plen, uint32_t* pcrc, uint32_t j = 0, const Pack* pk = nullptr) {
  if (k > jterm || a.code[k] == kNone) return;
  if (a.scap && a.recs[k] <= a.scap) return;  // staged: seg_place_thread
  uint32_t r = 0, rend = a.recs[k];
  uint64_t p = a.g[k], pend = ~0ull;
  if (a.nsub > 1) {
    const uint64_t t = (uint64_t)k * a.nsub + j;
    p = a.cpp[t];
    r = a.cpc[t];
    if (j + 1 < a.nsub) pend = seg_begin(a, k) + (uint64_t)(j + 1) * a.sub;
  }
  uint64_t i = at + (a.pre[k] & kRecMask) + r;
  const uint8_t* img = a.img;
  uint64_t pi = ~0ull;  // packed: the previous record, its span closed by this one's header
  uint32_t pgot = 0, pcv = 0;
  for (; r < rend && p < pend; ++r, ++i) {
    const Head h = head(img, a.n, p);
    const uint32_t hl = hdr_len(h.t);
    const uint32_t dlen = h.klen + h.vlen;
    const uint64_t avail = a.n - (p + hl);
    const uint32_t got = dlen <= avail ? dlen : (uint32_t)avail;
    if (pk && pi != ~0ull) {
      const bool fit = pack_fits(pgot, hl);
      plen[pi] = fit ? pgot + hl : pgot;
      pcrc[pi] = fit ? pack_crc(pcv, h, pk->T) : pcv;
    }
    put_rec(recs + i, p, p + hl, h.klen, h.vlen, h.crc, h.t);
    poff[i] = p + hl;
    if (pk) {
      pi = i;
      pgot = got;
      pcv = h.crc;
    } else {
      plen[i] = got;
      pcrc[i] = h.crc;
    }
    p += hl + got;
  }
  if (pk && pi != ~0ull) {  // the last record here: the next one's header is at p (another thread's first)
    bool fit = false;
    Head h{};
    if (i < pk->iend) {
      h = head(img, a.n, p);
      fit = pack_fits(pgot, hdr_len(h.t));
    }
    plen[pi] = fit ? pgot + hdr_len(h.t) : pgot;
    pcrc[pi] = fit ? pack_crc(pcv, h, pk->T) : pcv;
  }
}

// Record r of staged segment k (every record it walked fit its slots), R
// its staged form: the record to its place, its CRC span -- packed
// (pk; its expected CRC then pack_crc's) or the payload alone -- and its
// expected CRC.  nh: the header of the record after it (the next slot's, or
// the one at the segment's exit for its last record), used only when the
// walk has a record after it.  The payload is cut at EOF only for the walk's
// last record.
template <class Rec>
// i0: the segment's first record's index in recs (at + its placement prefix,
// read once by the caller rather than per window)
LSMCK_HD void seg_place_rec(const SegArgs& a, uint32_t k, uint64_t i0, Rec* recs, uint64_t* poff, uint32_t* plen,
                            uint32_t* pcrc, uint32_t r, const StageRec& R, const Head& nh, const Pack* pk) {
  const uint64_t i = i0 + r;
  const uint32_t t = stage_type(R);
  const uint64_t rec_off = stage_off(R, seg_begin(a, k)), payload_off = rec_off + hdr_len(t);
  put_rec(recs + i, rec_off, payload_off, R.klen, R.vlen, R.crc, t);
  poff[i] = payload_off;
  const uint32_t dlen = R.klen + R.vlen;
  const uint64_t avail = a.n - payload_off;
  const uint32_t got = dlen <= avail ? dlen : (uint32_t)avail;
  const bool fit = pk && i + 1 < pk->iend && pack_fits(got, hdr_len(nh.t));
  plen[i] = fit ? got + hdr_len(nh.t) : got;
  pcrc[i] = fit ? pack_crc(R.crc, nh, pk->T) : R.crc;
}
// the header of the record after record r of staged segment k (see above)
LSMCK_HD Head seg_place_next_head(const SegArgs& a, uint32_t k, uint32_t r) {
  if (r + 1 < a.recs[k]) {
    const StageRec& N = a.srec[(uint64_t)k * a.scap + r + 1];
    Head h{};
    h.t = stage_type(N);
    h.crc = N.crc;
    h.klen = N.klen;
    h.vlen = N.vlen;
    return h;
  }
  return head(a.img, a.n, a.x[k]);
}

}  // namespace seg
}  // namespace lsmck
#endif
