// segwalk_sim.cpp -- the segment walk of lsmck_segwalk.h run on the host:
// the same per-thread functions the wal_seg_* kernels run, called in loops in
// the order lsmck_api.cpp's wal_seg_walk launches them.  Test infrastructure
// (tests/test_segwalk_model.py builds it with g++): it checks the walk's logic
// -- guesses, the check, repairs, placement -- against a plain chain walk on
// logs the GPU suite cannot afford many of (adversarial payloads, tiny
// segments, every cut position).  Not part of liblsmck.
#include <stdint.h>
#include <stddef.h>

#include <algorithm>
#include <vector>

#include "lsmck_segwalk.h"

namespace sg = lsmck::seg;

struct SimRec {
  uint64_t rec_off, payload_off;
  uint32_t klen, vlen, crc, type;
};

static uint64_t* g_dbg = nullptr;  // debug: the first round's guesses
extern "C" void segwalk_sim_debug(uint64_t* g) { g_dbg = g; }
static uint32_t g_nsub = 1;  // emit checkpoints: sub-segments per segment (1 = none)
extern "C" void segwalk_sim_set_nsub(uint32_t v) { g_nsub = v ? v : 1; }
static uint32_t g_scap = 0;  // walk-time staging: slots per segment (0 = none)
static int g_prepair = 2;    // parallel repair rounds before the serial repairs (wal_seg_prepair)
extern "C" void segwalk_sim_set_prepair(int v) { g_prepair = v; }
static int g_prepairs = 0;   // the last walk's parallel repair rounds
extern "C" int segwalk_sim_prepairs() { return g_prepairs; }
extern "C" void segwalk_sim_set_stage(uint32_t v) { g_scap = v; }
// packed CRC spans (seg::Pack): when set, the next walk emits them here --
// span offsets, lengths and expected CRCs
static uint64_t* g_poff = nullptr;
static uint32_t *g_plen = nullptr, *g_pexp = nullptr;
static size_t g_pcap = 0;
extern "C" void segwalk_sim_pack(uint64_t* poff, uint32_t* plen, uint32_t* pexp, size_t cap) {
  g_poff = poff;
  g_plen = plen;
  g_pexp = pexp;
  g_pcap = poff ? cap : 0;
}
// seg::unpack_crc with wal_compare_packed's tables: the payload CRC from a
// packed span's CRC c and the next header's fields
static const uint32_t* crc_tables4() {  // T0..T3, as build_crc_tables (lsmck_wal.hip) makes them in LDS
  static uint32_t T[1024];
  static bool done = false;
  if (!done) {
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t c = b;
      for (int i = 0; i < 8; ++i) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
      T[b] = c;
    }
    for (int q = 1; q < 4; ++q)
      for (uint32_t b = 0; b < 256; ++b) T[q * 256 + b] = (T[(q - 1) * 256 + b] >> 8) ^ T[T[(q - 1) * 256 + b] & 0xFFu];
    done = true;
  }
  return T;
}
extern "C" uint32_t segwalk_sim_unpack(uint32_t c, uint32_t t, uint32_t crc, uint32_t klen, uint32_t vlen) {
  sg::Head h{};
  h.t = t;
  h.crc = crc;
  h.klen = klen;
  h.vlen = vlen;
  return sg::unpack_crc(c, h, crc_tables4());
}

// the records starting in [start, lim): code_out kExit with pos_out the first
// record start at or past lim when the chain goes on past the prefix
extern "C" int segwalk_sim_prefix(const uint8_t* img, uint64_t n, uint64_t start, uint64_t lim, uint64_t S,
                                  int max_rounds, uint64_t* rec_off, size_t cap, uint64_t* m_out, uint32_t* code_out,
                                  uint64_t* pos_out, int* repairs, uint64_t* segments, uint32_t* first_fails) {
  *first_fails = 0;
  *repairs = 0;
  *segments = 0;
  if (start >= n) {
    *m_out = 0;
    *code_out = sg::kEnd;
    *pos_out = 0;
    return 0;
  }
  if (lim > n || lim <= start) lim = n;
  const uint32_t K = (uint32_t)((lim - start + S - 1) / S);
  *segments = K;
  std::vector<uint64_t> g(K + 1), x(K + 1), pre(K + 1);
  std::vector<uint32_t> code(K + 1), recs(K + 1);
  unsigned long long info[sg::kInfoWords] = {};
  std::vector<uint64_t> cpp((size_t)K * g_nsub);
  std::vector<uint32_t> cpc((size_t)K * g_nsub);
  const uint32_t scap = (uint32_t)std::min<uint64_t>(g_scap, S / 9 + 1);  // (as wal_seg_walk caps it)
  std::vector<sg::StageRec> st((size_t)K * scap);
  sg::SegArgs a{img, n, start, S, K, g.data(), x.data(), code.data(), recs.data(), pre.data(), info, lim,
                g_nsub, (S + g_nsub - 1) / g_nsub, cpp.data(), cpc.data(), scap ? st.data() : nullptr, scap};
  for (uint32_t k = 0; k < K; ++k) sg::seg_walk_thread(a, k);
  if (g_dbg) std::copy(g.begin(), g.begin() + K, g_dbg);
  g_prepairs = 0;
  int serial = 0;
  for (int round = 0;; ++round) {
    uint32_t jterm = sg::kNoSeg, fail = sg::kNoSeg;
    for (uint32_t k = 0; k < K; ++k)
      if (code[k] == sg::kEnd || code[k] == sg::kBad) jterm = std::min(jterm, k);
    uint64_t run = 0;
    for (uint32_t k = 0; k <= K; ++k) {
      pre[k] = run;
      if (k < K) run += sg::seg_word(a, k, jterm);
    }
    uint32_t nfail = 0;
    for (uint32_t k = 0; k < K; ++k)
      if (sg::seg_check_fails(a, k, jterm)) fail = std::min(fail, k), ++nfail;
    if (round == 0) *first_fails = nfail;
    info[sg::kInfoJterm] = jterm;
    info[sg::kInfoFail] = fail;
    if (fail == sg::kNoSeg) {
      *m_out = pre[K] & sg::kRecMask;
      if (jterm != sg::kNoSeg) {
        *code_out = code[jterm];
        *pos_out = x[jterm];
        break;
      }
      uint32_t last = 0;  // the chain's way out of the prefix (wal_seg_check's kInfoLast)
      for (uint32_t k = 0; k < K; ++k)
        if (code[k] == sg::kExit && x[k] >= lim) last = k + 1;
      if (!last) return 2;  // (cannot happen: the chain ends in the prefix or leaves it)
      *code_out = sg::kExit;
      *pos_out = x[last - 1];
      break;
    }
    if (nfail >= 2 && g_prepairs < g_prepair) {  // a parallel round (wal_seg_prepair), from a snapshot
      const std::vector<uint64_t> g0(g), x0(x);
      const std::vector<uint32_t> c0(code);
      for (uint32_t t = 0; t < K; ++t) sg::seg_prepair(a, t, g0.data(), x0.data(), c0.data());
      ++g_prepairs;
      continue;
    }
    if (serial >= max_rounds) return 1;  // declined: the caller walks by candidate doubling
    sg::seg_repair(a, fail, 4096);
    *repairs = ++serial;
  }
  const uint64_t m = *m_out;
  std::vector<SimRec> R(m);
  std::vector<uint64_t> poff(m);
  std::vector<uint32_t> plen(m), pcrc(m);
  const sg::Pack pk{m, crc_tables4()};
  for (uint32_t k = 0; k < K; ++k)
    for (uint32_t j = 0; j < a.nsub; ++j)
      sg::seg_emit_thread(a, k, (uint32_t)info[sg::kInfoJterm], 0, R.data(), poff.data(), plen.data(), pcrc.data(), j,
                          g_pcap ? &pk : nullptr);
  const uint32_t jt = (uint32_t)info[sg::kInfoJterm];
  for (uint32_t k = 0; scap && k < K; ++k)  // wal_seg_place: the staged segments
    if (k <= jt && code[k] != sg::kNone && recs[k] <= scap)
      for (uint32_t r = 0; r < recs[k]; ++r) {
        const uint64_t i = (pre[k] & sg::kRecMask) + r;
        const sg::Head nh = i + 1 < m ? sg::seg_place_next_head(a, k, r) : sg::Head{};
        sg::seg_place_rec(a, k, pre[k] & sg::kRecMask, R.data(), poff.data(), plen.data(), pcrc.data(), r,
                          st[(size_t)k * scap + r], nh,
                          g_pcap ? &pk : nullptr);
      }
  for (uint64_t i = 0; i < m && i < cap; ++i) rec_off[i] = R[i].rec_off;
  for (uint64_t i = 0; i < m && i < g_pcap; ++i) {
    g_poff[i] = poff[i];
    g_plen[i] = plen[i];
    g_pexp[i] = pcrc[i];
  }
  return 0;
}

extern "C" int segwalk_sim(const uint8_t* img, uint64_t n, uint64_t start, uint64_t S, int max_rounds,
                           uint64_t* rec_off, size_t cap, uint64_t* m_out, uint32_t* code_out, uint64_t* pos_out,
                           int* repairs, uint64_t* segments, uint32_t* first_fails) {
  return segwalk_sim_prefix(img, n, start, n, S, max_rounds, rec_off, cap, m_out, code_out, pos_out, repairs, segments,
                            first_fails);
}
