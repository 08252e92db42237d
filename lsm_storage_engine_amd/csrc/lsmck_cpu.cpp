// lsmck_cpu.cpp -- scalar CPU entry points of liblsmck.so (include/lsmck.h section 1).
//
// These are the per-record latency path: one WAL append checksums one small
// record (src/wal.rs:177,187) and one SSTable flush hashes two files
// (src/checksums.rs:64-80); launching a GPU kernel for either would cost more
// than the work.  Bulk work goes through the batch entry points (GPU only).
//
// CRC-32 here is PCLMULQDQ folding for the 16-byte-multiple head of records
// of 64 B and more, slicing-by-8 (8 KiB of static const tables) for the rest
// and where the CPU lacks PCLMULQDQ; SHA-256 is a portable FIPS 180-4
// implementation with an x86 SHA-NI fast path.  Both are selected once at
// load time.
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>

#include "lsmck.h"
#include "lsmck_internal.h"

#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
#endif

namespace {

// ---------------------------------------------------------------------------
// CRC-32/ISO-HDLC tables (reflected 0xEDB88320), slicing-by-8.
struct CrcTables {
  uint32_t t[8][256];
  CrcTables() {
    for (uint32_t n = 0; n < 256; ++n) {
      uint32_t c = n;
      for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
      t[0][n] = c;
    }
    for (int s = 1; s < 8; ++s)
      for (uint32_t n = 0; n < 256; ++n) t[s][n] = (t[s - 1][n] >> 8) ^ t[0][t[s - 1][n] & 0xFFu];
  }
};
const CrcTables kCrc;

#if defined(__x86_64__)
// Carry-less-multiply folding (x86 PCLMULQDQ) over n bytes, n >= 64 and a
// multiple of 16; v is the inverted register, as in crc_reg_update.  Four
// 128-bit lanes are folded forward by 512 bits per 64-byte block (constants
// x^(512±32) mod P, bit-reflected), then folded into one lane (x^(128±32)),
// reduced to 64 bits (x^64) and Barrett-reduced to 32 (P and
// floor(x^64 / P)) -- the published folding scheme for a reflected CRC-32.
__attribute__((target("pclmul,sse4.1"))) inline __m128i fold(__m128i x, __m128i k, __m128i next) {
  return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), next);
}
__attribute__((target("pclmul,sse4.1"))) uint32_t crc_fold_pclmul(uint32_t v, const uint8_t* p, size_t n) {
  const __m128i k1k2 = _mm_set_epi64x(0x1c6e41596ll, 0x154442bd4ll);
  const __m128i k3k4 = _mm_set_epi64x(0x0ccaa009ell, 0x1751997d0ll);
  const __m128i k5 = _mm_set_epi64x(0, 0x163cd6124ll);
  const __m128i pmu = _mm_set_epi64x(0x1f7011641ll, 0x1db710641ll);
  const __m128i lo32 = _mm_setr_epi32(-1, 0, -1, 0);
  __m128i a = _mm_xor_si128(_mm_loadu_si128((const __m128i*)p), _mm_cvtsi32_si128((int)v));
  __m128i b = _mm_loadu_si128((const __m128i*)(p + 16));
  __m128i c = _mm_loadu_si128((const __m128i*)(p + 32));
  __m128i d = _mm_loadu_si128((const __m128i*)(p + 48));
  p += 64;
  n -= 64;
  for (; n >= 64; p += 64, n -= 64) {
    a = fold(a, k1k2, _mm_loadu_si128((const __m128i*)p));
    b = fold(b, k1k2, _mm_loadu_si128((const __m128i*)(p + 16)));
    c = fold(c, k1k2, _mm_loadu_si128((const __m128i*)(p + 32)));
    d = fold(d, k1k2, _mm_loadu_si128((const __m128i*)(p + 48)));
  }
  a = fold(a, k3k4, b);
  a = fold(a, k3k4, c);
  a = fold(a, k3k4, d);
  for (; n >= 16; p += 16, n -= 16) a = fold(a, k3k4, _mm_loadu_si128((const __m128i*)p));
  // 128 -> 64 bits
  __m128i t = _mm_clmulepi64_si128(a, k3k4, 0x10);
  a = _mm_xor_si128(_mm_srli_si128(a, 8), t);
  t = _mm_srli_si128(a, 4);
  a = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(a, lo32), k5, 0x00), t);
  // Barrett: 64 -> 32 bits
  t = _mm_clmulepi64_si128(_mm_and_si128(a, lo32), pmu, 0x10);
  t = _mm_clmulepi64_si128(_mm_and_si128(t, lo32), pmu, 0x00);
  return (uint32_t)_mm_extract_epi32(_mm_xor_si128(a, t), 1);
}

bool cpu_has_pclmul() {
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  return ((c >> 1) & 1) && ((c >> 19) & 1);  // PCLMULQDQ, SSE4.1
}
const bool kPclmul = cpu_has_pclmul();
#endif

// raw register update, register already inverted
uint32_t crc_reg_update(uint32_t v, const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  if (kPclmul && n >= 64) {
    const size_t m = n & ~(size_t)15;
    v = crc_fold_pclmul(v, p, m);
    p += m;
    n -= m;
  }
#endif
  const auto& T = kCrc.t;
  while (n && ((uintptr_t)p & 7)) {
    v = T[0][(v ^ *p++) & 0xFFu] ^ (v >> 8);
    --n;
  }
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= v;
    v = T[7][lo & 0xFF] ^ T[6][(lo >> 8) & 0xFF] ^ T[5][(lo >> 16) & 0xFF] ^ T[4][lo >> 24] ^ T[3][hi & 0xFF] ^
        T[2][(hi >> 8) & 0xFF] ^ T[1][(hi >> 16) & 0xFF] ^ T[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) v = T[0][(v ^ *p++) & 0xFFu] ^ (v >> 8);
  return v;
}

// ---------------------------------------------------------------------------
// SHA-256
const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void sha_blocks_portable(uint32_t h[8], const uint8_t* p, size_t nblocks) {
  for (; nblocks; --nblocks, p += 64) {
    uint32_t w[64];
    for (int t = 0; t < 16; ++t)
      w[t] = ((uint32_t)p[4 * t] << 24) | ((uint32_t)p[4 * t + 1] << 16) | ((uint32_t)p[4 * t + 2] << 8) | p[4 * t + 3];
    for (int t = 16; t < 64; ++t)
      w[t] = w[t - 16] + (ror(w[t - 15], 7) ^ ror(w[t - 15], 18) ^ (w[t - 15] >> 3)) + w[t - 7] +
             (ror(w[t - 2], 17) ^ ror(w[t - 2], 19) ^ (w[t - 2] >> 10));
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int t = 0; t < 64; ++t) {
      uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K256[t] + w[t];
      uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
    h[5] += f;
    h[6] += g;
    h[7] += hh;
  }
}

#if defined(__x86_64__)
// Intel SHA extensions (what sha2 0.10 selects at run time on such CPUs).
__attribute__((target("sha,sse4.1"))) void sha_blocks_shani(uint32_t h[8], const uint8_t* p, size_t nblocks) {
  const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i TMP = _mm_loadu_si128((const __m128i*)&h[0]);
  __m128i STATE1 = _mm_loadu_si128((const __m128i*)&h[4]);
  TMP = _mm_shuffle_epi32(TMP, 0xB1);
  STATE1 = _mm_shuffle_epi32(STATE1, 0x1B);
  __m128i STATE0 = _mm_alignr_epi8(TMP, STATE1, 8);
  STATE1 = _mm_blend_epi16(STATE1, TMP, 0xF0);
  for (; nblocks; --nblocks, p += 64) {
    __m128i ABEF_SAVE = STATE0, CDGH_SAVE = STATE1;
    __m128i M[4];
    for (int i = 0; i < 4; ++i) M[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * i)), MASK);
    for (int r = 0; r < 16; ++r) {
      __m128i& Mi = M[r & 3];
      if (r >= 4) {
        // message schedule for the 4 words of group r
        __m128i t = _mm_alignr_epi8(M[(r - 1) & 3], M[(r - 2) & 3], 4);
        Mi = _mm_sha256msg1_epu32(Mi, M[(r - 3) & 3]);
        Mi = _mm_add_epi32(Mi, t);
        Mi = _mm_sha256msg2_epu32(Mi, M[(r - 1) & 3]);
      }
      __m128i K = _mm_loadu_si128((const __m128i*)&K256[4 * r]);
      __m128i MSG = _mm_add_epi32(Mi, K);
      STATE1 = _mm_sha256rnds2_epu32(STATE1, STATE0, MSG);
      MSG = _mm_shuffle_epi32(MSG, 0x0E);
      STATE0 = _mm_sha256rnds2_epu32(STATE0, STATE1, MSG);
    }
    STATE0 = _mm_add_epi32(STATE0, ABEF_SAVE);
    STATE1 = _mm_add_epi32(STATE1, CDGH_SAVE);
  }
  TMP = _mm_shuffle_epi32(STATE0, 0x1B);
  STATE1 = _mm_shuffle_epi32(STATE1, 0xB1);
  STATE0 = _mm_blend_epi16(TMP, STATE1, 0xF0);
  STATE1 = _mm_alignr_epi8(STATE1, TMP, 8);
  _mm_storeu_si128((__m128i*)&h[0], STATE0);
  _mm_storeu_si128((__m128i*)&h[4], STATE1);
}

bool cpu_has_shani() {
  unsigned a, b, c, d;
  if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
  bool sha = (b >> 29) & 1;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  bool sse41 = (c >> 19) & 1;
  return sha && sse41;
}
#endif

typedef void (*sha_blocks_fn)(uint32_t*, const uint8_t*, size_t);
sha_blocks_fn pick_sha() {
#if defined(__x86_64__)
  if (cpu_has_shani()) return sha_blocks_shani;
#endif
  return sha_blocks_portable;
}
const sha_blocks_fn kShaBlocks = pick_sha();

}  // namespace

// ---------------------------------------------------------------------------
namespace lsmck_host {
uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
  // zlib multmodp: a(x) * b(x) mod P(x), reflected
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
  }
  return p;
}
uint32_t x_pow_8n(uint64_t n) {
  // x^(8n) mod P by square-and-multiply on x^(2^k)
  uint32_t p = 1u << 31;       // x^0
  uint32_t sq = 1u << 23;      // x^8
  while (n) {
    if (n & 1) p = gf2_mulmod(sq, p);
    sq = gf2_mulmod(sq, sq);
    n >>= 1;
  }
  return p;
}
const uint32_t* crc_tables() { return &kCrc.t[0][0]; }
}  // namespace lsmck_host

extern "C" {

uint32_t lsmck_crc32_ieee(const uint8_t* p, size_t n) {
  if (n == 0) return 0;
  return ~crc_reg_update(0xFFFFFFFFu, p, n);
}

uint32_t lsmck_crc32_update(uint32_t crc_a, const uint8_t* p, size_t n) {
  if (n == 0) return crc_a;
  return ~crc_reg_update(~crc_a, p, n);
}

uint32_t lsmck_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  if (len_b == 0) return crc_a;
  return lsmck_host::gf2_mulmod(lsmck_host::x_pow_8n(len_b), crc_a) ^ crc_b;
}

void lsmck_sha256_init(lsmck_sha256_ctx* c) {
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(c->h, iv, sizeof iv);
  c->nbytes = 0;
  c->nbuf = 0;
}

void lsmck_sha256_update(lsmck_sha256_ctx* c, const uint8_t* p, size_t n) {
  c->nbytes += n;
  if (c->nbuf) {
    size_t take = 64 - c->nbuf;
    if (take > n) take = n;
    memcpy(c->buf + c->nbuf, p, take);
    c->nbuf += (uint32_t)take;
    p += take;
    n -= take;
    if (c->nbuf < 64) return;
    kShaBlocks(c->h, c->buf, 1);
    c->nbuf = 0;
  }
  size_t nb = n / 64;
  if (nb) kShaBlocks(c->h, p, nb);
  p += nb * 64;
  n -= nb * 64;
  if (n) {
    memcpy(c->buf, p, n);
    c->nbuf = (uint32_t)n;
  }
}

void lsmck_sha256_final(lsmck_sha256_ctx* c, uint8_t out[32]) {
  uint64_t bits = c->nbytes * 8;
  uint8_t tail[128];
  memset(tail, 0, sizeof tail);
  memcpy(tail, c->buf, c->nbuf);
  tail[c->nbuf] = 0x80;
  size_t tn = (c->nbuf + 9 <= 64) ? 64 : 128;
  for (int i = 0; i < 8; ++i) tail[tn - 1 - i] = (uint8_t)(bits >> (8 * i));
  kShaBlocks(c->h, tail, tn / 64);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(c->h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(c->h[i] >> 8);
    out[4 * i + 3] = (uint8_t)c->h[i];
  }
}

void lsmck_sha256(const uint8_t* p, size_t n, uint8_t out[32]) {
  lsmck_sha256_ctx c;
  lsmck_sha256_init(&c);
  lsmck_sha256_update(&c, p, n);
  lsmck_sha256_final(&c, out);
}

size_t lsmck_base64_encode(const uint8_t* p, size_t n, char* out) {
  static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  size_t o = 0, i = 0;
  for (; i + 3 <= n; i += 3) {
    uint32_t v = ((uint32_t)p[i] << 16) | ((uint32_t)p[i + 1] << 8) | p[i + 2];
    out[o++] = A[v >> 18];
    out[o++] = A[(v >> 12) & 63];
    out[o++] = A[(v >> 6) & 63];
    out[o++] = A[v & 63];
  }
  size_t r = n - i;
  if (r) {
    uint32_t v = (uint32_t)p[i] << 16;
    if (r == 2) v |= (uint32_t)p[i + 1] << 8;
    out[o++] = A[v >> 18];
    out[o++] = A[(v >> 12) & 63];
    out[o++] = r == 2 ? A[(v >> 6) & 63] : '=';
    out[o++] = '=';
  }
  out[o] = 0;
  return o;
}

int lsmck_checksum_file(const char* path, char out[45]) {
  if (!path || !out) return lsmck_host::set_error(LSMCK_EINVAL, "null argument");
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {  // the reference panics here (checksums.rs:25)
    int e = errno;
    std::string m = std::string("Can't open file to calculate checksum ") + path + ": " + strerror(e);
    return lsmck_host::set_error(LSMCK_PANIC_OPEN_FILE, m.c_str());
  }
  lsmck_sha256_ctx c;
  lsmck_sha256_init(&c);
  uint8_t buf[1 << 16];
  for (;;) {
    ssize_t k = read(fd, buf, sizeof buf);
    if (k < 0) {
      if (errno == EINTR) continue;
      int e = errno;
      close(fd);
      return lsmck_host::set_errno_error(e, "read", path);
    }
    if (k == 0) break;
    lsmck_sha256_update(&c, buf, (size_t)k);
  }
  close(fd);
  uint8_t d[32];
  lsmck_sha256_final(&c, d);
  lsmck_base64_encode(d, 32, out);
  return 0;
}

// the index file is hashed second: its open panic is LSMCK_PANIC_OPEN_INDEX
static int checksum_index_file(const char* index_path, char out[45]) {
  int rc = lsmck_checksum_file(index_path, out);
  if (rc == LSMCK_PANIC_OPEN_FILE) {
    std::string m = lsmck_last_error();
    return lsmck_host::set_error(LSMCK_PANIC_OPEN_INDEX, m.c_str());
  }
  return rc;
}

int lsmck_checksums_write(const char* data_path, const char* index_path, const char* checksum_path) {
  char db[45], ib[45];
  int rc = lsmck_checksum_file(data_path, db);
  if (rc) return rc;
  rc = checksum_index_file(index_path, ib);
  if (rc) return rc;
  return lsmck_host::write_checksum_json(checksum_path, ib, db);
}

int lsmck_checksums_verify(const char* data_path, const char* index_path, const char* checksum_path) {
  char db[45], ib[45];
  int rc = lsmck_checksum_file(data_path, db);
  if (rc) return rc;
  rc = checksum_index_file(index_path, ib);
  if (rc) return rc;
  std::string want_index, want_data;
  rc = lsmck_host::read_checksum_json(checksum_path, &want_index, &want_data);
  if (rc) return rc;
  if (want_data != db) return lsmck_host::set_error(LSMCK_DATA_MISMATCH, "data checksum mismatch");
  if (want_index != ib) return lsmck_host::set_error(LSMCK_INDEX_MISMATCH, "index checksum mismatch");
  return 0;
}

static void put_u32le(uint8_t* o, uint32_t v) {
  o[0] = (uint8_t)v;
  o[1] = (uint8_t)(v >> 8);
  o[2] = (uint8_t)(v >> 16);
  o[3] = (uint8_t)(v >> 24);
}

size_t lsmck_wal_encode_insert(const uint8_t* key, uint32_t klen, const uint8_t* val, uint32_t vlen, uint8_t* out) {
  uint8_t* pay = out + 13;
  if (klen) memcpy(pay, key, klen);
  if (vlen) memcpy(pay + klen, val, vlen);
  out[0] = 1;
  put_u32le(out + 1, lsmck_crc32_ieee(pay, (size_t)klen + vlen));
  put_u32le(out + 5, klen);
  put_u32le(out + 9, vlen);
  return 13 + (size_t)klen + vlen;
}

size_t lsmck_wal_encode_remove(const uint8_t* key, uint32_t klen, uint8_t* out) {
  if (klen) memcpy(out + 9, key, klen);
  out[0] = 2;
  put_u32le(out + 1, lsmck_crc32_ieee(out + 9, klen));
  put_u32le(out + 5, klen);
  return 9 + (size_t)klen;
}

void lsmck_gen_zipf_lengths(uint64_t seed, double s, int kmax, uint32_t lmin, size_t n, uint32_t* out) {
  lsmck_host::gen_zipf_lengths(seed, s, kmax, lmin, 0, n, out);
}

void lsmck_gen_zipf_lengths_at(uint64_t seed, double s, int kmax, uint32_t lmin, uint64_t first, size_t n,
                               uint32_t* out) {
  lsmck_host::gen_zipf_lengths(seed, s, kmax, lmin, first, n, out);
}

}  // extern "C"
