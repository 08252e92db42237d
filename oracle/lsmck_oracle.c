/*
 * lsmck_oracle.c -- CPU restatement of the reference checksum path.
 * TEST INFRASTRUCTURE ONLY (see lsmck_oracle.h for scope and pinning).
 * Deliberately simple, scalar code: it is the checker, not a product path.
 */
#define _GNU_SOURCE
#include "lsmck_oracle.h"

#include <errno.h>
#include <fcntl.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------------ */
/* CRC-32/ISO-HDLC, as crc 1.x crc32::checksum_ieee computes it:
 *   make_table(IEEE): reflected table of 0xEDB88320;
 *   update(!0, table, bytes): value = table[(value ^ b) & 0xFF] ^ (value >> 8);
 *   result = !value.
 * Call sites: src/wal.rs:135,153,177,187. */
static uint32_t g_crc_table[256];
static pthread_once_t g_crc_once = PTHREAD_ONCE_INIT;

static void crc_table_init(void) {
  for (uint32_t n = 0; n < 256; ++n) {
    uint32_t c = n;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
    g_crc_table[n] = c;
  }
}

uint32_t oracle_crc32_ieee(const uint8_t* p, size_t n) {
  pthread_once(&g_crc_once, crc_table_init);
  uint32_t v = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) v = g_crc_table[(v ^ p[i]) & 0xFFu] ^ (v >> 8);
  return ~v;
}

typedef struct {
  const uint8_t* base;
  const uint64_t* off;
  const uint32_t* len;
  size_t stride, flen;
  size_t lo, hi;
  uint32_t* out;
  uint8_t* out32;
  int sha;
} job_t;

static void* crc_worker(void* a) {
  job_t* j = (job_t*)a;
  for (size_t i = j->lo; i < j->hi; ++i) {
    const uint8_t* p;
    size_t n;
    if (j->off) {
      p = j->base + j->off[i];
      n = j->len[i];
    } else {
      p = j->base + i * j->stride;
      n = j->flen;
    }
    if (j->sha)
      oracle_sha256(p, n, j->out32 + 32 * i);
    else
      j->out[i] = oracle_crc32_ieee(p, n);
  }
  return NULL;
}

static void run_jobs(job_t proto, size_t n, int nthreads, const uint32_t* len) {
  pthread_once(&g_crc_once, crc_table_init);
  if (nthreads <= 1 || n < 2) {
    proto.lo = 0;
    proto.hi = n;
    crc_worker(&proto);
    return;
  }
  if (nthreads > 256) nthreads = 256;
  /* byte-balanced partition (SURVEY 8d "byte-balanced partition") */
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += len ? len[i] : proto.flen;
  pthread_t th[256];
  job_t jobs[256];
  size_t start = 0;
  uint64_t acc = 0;
  for (int t = 0; t < nthreads; ++t) {
    uint64_t target = total * (uint64_t)(t + 1) / (uint64_t)nthreads;
    size_t end = start;
    while (end < n && (t == nthreads - 1 || acc < target)) {
      acc += len ? len[end] : proto.flen;
      ++end;
    }
    jobs[t] = proto;
    jobs[t].lo = start;
    jobs[t].hi = end;
    start = end;
    pthread_create(&th[t], NULL, crc_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

void oracle_crc32_batch(const uint8_t* base, const uint64_t* off, const uint32_t* len, size_t n,
                        uint32_t* out, int nthreads) {
  job_t j;
  memset(&j, 0, sizeof j);
  j.base = base;
  j.off = off;
  j.len = len;
  j.out = out;
  run_jobs(j, n, nthreads, len);
}

void oracle_crc32_fixed(const uint8_t* base, size_t stride, size_t len, size_t n, uint32_t* out,
                        int nthreads) {
  job_t j;
  memset(&j, 0, sizeof j);
  j.base = base;
  j.stride = stride;
  j.flen = len;
  j.out = out;
  run_jobs(j, n, nthreads, NULL);
}

/* ------------------------------------------------------------------------ */
/* SHA-256, FIPS 180-4 section 6.2 (what sha2 0.10's Sha256 computes). */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t h[8], const uint8_t* p) {
  uint32_t w[64];
  for (int t = 0; t < 16; ++t)
    w[t] = ((uint32_t)p[4 * t] << 24) | ((uint32_t)p[4 * t + 1] << 16) | ((uint32_t)p[4 * t + 2] << 8) |
           (uint32_t)p[4 * t + 3];
  for (int t = 16; t < 64; ++t) {
    uint32_t s0 = ROR(w[t - 15], 7) ^ ROR(w[t - 15], 18) ^ (w[t - 15] >> 3);
    uint32_t s1 = ROR(w[t - 2], 17) ^ ROR(w[t - 2], 19) ^ (w[t - 2] >> 10);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 64; ++t) {
    uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + K256[t] + w[t];
    uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
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

void oracle_sha256_init(oracle_sha256_ctx* c) {
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(c->h, iv, sizeof iv);
  c->nbytes = 0;
  c->nbuf = 0;
}

void oracle_sha256_update(oracle_sha256_ctx* c, const uint8_t* p, size_t n) {
  c->nbytes += n;
  while (n) {
    size_t take = 64 - c->nbuf;
    if (take > n) take = n;
    memcpy(c->buf + c->nbuf, p, take);
    c->nbuf += (uint32_t)take;
    p += take;
    n -= take;
    if (c->nbuf == 64) {
      sha256_block(c->h, c->buf);
      c->nbuf = 0;
    }
  }
}

void oracle_sha256_final(oracle_sha256_ctx* c, uint8_t out[32]) {
  uint64_t bits = c->nbytes * 8;
  uint8_t pad = 0x80;
  uint64_t saved = c->nbytes;
  oracle_sha256_update(c, &pad, 1);
  uint8_t z = 0;
  while (c->nbuf != 56) oracle_sha256_update(c, &z, 1);
  uint8_t lb[8];
  for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
  oracle_sha256_update(c, lb, 8);
  c->nbytes = saved;
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(c->h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(c->h[i] >> 8);
    out[4 * i + 3] = (uint8_t)c->h[i];
  }
}

void oracle_sha256(const uint8_t* p, size_t n, uint8_t out[32]) {
  oracle_sha256_ctx c;
  oracle_sha256_init(&c);
  oracle_sha256_update(&c, p, n);
  oracle_sha256_final(&c, out);
}

void oracle_sha256_batch(const uint8_t* base, const uint64_t* off, const uint32_t* len, size_t n,
                         uint8_t* out32, int nthreads) {
  job_t j;
  memset(&j, 0, sizeof j);
  j.base = base;
  j.off = off;
  j.len = len;
  j.out32 = out32;
  j.sha = 1;
  run_jobs(j, n, nthreads, len);
}

/* ------------------------------------------------------------------------ */
/* base64 0.13 `encode` = STANDARD config: A-Z a-z 0-9 + /, '=' padding. */
size_t oracle_base64_std(const uint8_t* p, size_t n, char* out) {
  static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  size_t o = 0, i = 0;
  for (; i + 3 <= n; i += 3) {
    uint32_t v = ((uint32_t)p[i] << 16) | ((uint32_t)p[i + 1] << 8) | p[i + 2];
    out[o++] = A[(v >> 18) & 63];
    out[o++] = A[(v >> 12) & 63];
    out[o++] = A[(v >> 6) & 63];
    out[o++] = A[v & 63];
  }
  if (n - i == 1) {
    uint32_t v = (uint32_t)p[i] << 16;
    out[o++] = A[(v >> 18) & 63];
    out[o++] = A[(v >> 12) & 63];
    out[o++] = '=';
    out[o++] = '=';
  } else if (n - i == 2) {
    uint32_t v = ((uint32_t)p[i] << 16) | ((uint32_t)p[i + 1] << 8);
    out[o++] = A[(v >> 18) & 63];
    out[o++] = A[(v >> 12) & 63];
    out[o++] = A[(v >> 6) & 63];
    out[o++] = '=';
  }
  out[o] = 0;
  return o;
}

/* checksums.rs:20-38: open (panics on failure in the reference, :25), read in
 * 1 KiB chunks (:28-35), Sha256 update per chunk, finalize, base64. */
int oracle_file_checksum(const char* path, char out[45]) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return -errno;
  oracle_sha256_ctx c;
  oracle_sha256_init(&c);
  uint8_t buf[1024];
  for (;;) {
    ssize_t k = read(fd, buf, sizeof buf);
    if (k < 0) {
      int e = errno;
      close(fd);
      return -e;
    }
    if (k == 0) break;
    oracle_sha256_update(&c, buf, (size_t)k);
  }
  close(fd);
  uint8_t d[32];
  oracle_sha256_final(&c, d);
  oracle_base64_std(d, 32, out);
  return 0;
}

/* serde_json::to_writer(&Checksums{index_checksum, data_checksum})
 * (checksums.rs:13-17 field order, :79 compact writer).  base64 output needs
 * no JSON escaping. */
size_t oracle_checksums_json(const char* index_b64, const char* data_b64, char* out, size_t cap) {
  size_t n = strlen("{\"index_checksum\":\"\",\"data_checksum\":\"\"}") + strlen(index_b64) + strlen(data_b64);
  if (n + 1 > cap) return 0;
  char* o = out;
  const char* parts[5] = {"{\"index_checksum\":\"", index_b64, "\",\"data_checksum\":\"", data_b64, "\"}"};
  for (int i = 0; i < 5; ++i) {
    size_t l = strlen(parts[i]);
    memcpy(o, parts[i], l);
    o += l;
  }
  *o = 0;
  return n;
}

/* ------------------------------------------------------------------------ */
static void put_u32le(uint8_t* o, uint32_t v) {
  o[0] = (uint8_t)v;
  o[1] = (uint8_t)(v >> 8);
  o[2] = (uint8_t)(v >> 16);
  o[3] = (uint8_t)(v >> 24);
}
static uint32_t get_u32le(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* wal.rs:168-185: tmp = key ++ val; crc = checksum_ieee(tmp); write
 * u8 Insert(1), u32 crc, u32 klen, u32 vlen, tmp (all little endian). */
size_t oracle_wal_encode_insert(const uint8_t* key, uint32_t klen, const uint8_t* val, uint32_t vlen,
                                uint8_t* out) {
  uint8_t* payload = out + 13;
  if (klen) memcpy(payload, key, klen);
  if (vlen) memcpy(payload + klen, val, vlen);
  uint32_t crc = oracle_crc32_ieee(payload, (size_t)klen + vlen);
  out[0] = 1;
  put_u32le(out + 1, crc);
  put_u32le(out + 5, klen);
  put_u32le(out + 9, vlen);
  return 13 + (size_t)klen + vlen;
}

/* wal.rs:186-194: crc = checksum_ieee(key); u8 Remove(2), u32 crc, u32 klen, key. */
size_t oracle_wal_encode_remove(const uint8_t* key, uint32_t klen, uint8_t* out) {
  if (klen) memcpy(out + 9, key, klen);
  out[0] = 2;
  put_u32le(out + 1, oracle_crc32_ieee(out + 9, klen));
  put_u32le(out + 5, klen);
  return 9 + (size_t)klen;
}

/* wal.rs:122-163 next_record + Iterator (wal.rs:68-84).  Any UnexpectedEof
 * inside a header ends iteration cleanly.  A truncated payload: read_to_end
 * on `take(len)` returns the short data (wal.rs:132), debug_assert is off in
 * release, and the CRC of the short data is compared -> mismatch (or, by
 * chance, a match).  We restate that literally. */
int oracle_wal_replay(const uint8_t* buf, size_t n, oracle_wal_rec* recs, size_t cap, size_t* nrec,
                      uint64_t* bad_index, uint32_t* bad_crc, uint32_t* bad_expected) {
  size_t pos = 0, k = 0;
  *nrec = 0;
  for (;;) {
    if (pos + 1 > n) break; /* read_u8 EOF */
    uint8_t t = buf[pos];
    if (t != 1 && t != 2) {
      *bad_index = k;
      *bad_crc = t;
      *nrec = k;
      return 3;
    }
    if (pos + 5 > n) break; /* read_u32 crc EOF */
    uint32_t saved = get_u32le(buf + pos + 1);
    uint32_t klen, vlen = 0;
    size_t hdr;
    if (t == 1) {
      if (pos + 13 > n) break;
      klen = get_u32le(buf + pos + 5);
      vlen = get_u32le(buf + pos + 9);
      hdr = 13;
    } else {
      if (pos + 9 > n) break;
      klen = get_u32le(buf + pos + 5);
      hdr = 9;
    }
    /* data_len = key_len + val_len in u32 (wal.rs:129); overflow panics in
     * debug, wraps in release.  Treat it as wrapping. */
    uint32_t dlen = klen + vlen;
    size_t avail = n - (pos + hdr);
    size_t got = dlen <= avail ? dlen : avail;
    uint32_t c = oracle_crc32_ieee(buf + pos + hdr, got);
    if (c != saved) {
      *bad_index = k;
      *bad_crc = c;
      *bad_expected = saved;
      *nrec = k;
      return t == 1 ? 1 : 2;
    }
    if (k < cap) {
      recs[k].rec_off = pos;
      recs[k].payload_off = pos + hdr;
      recs[k].klen = klen;
      recs[k].vlen = vlen;
      recs[k].crc = saved;
      recs[k].type = t;
    }
    ++k;
    pos += hdr + got;
  }
  *nrec = k;
  return 0;
}

/* ------------------------------------------------------------------------ */
uint64_t oracle_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void oracle_gen_stream(uint64_t seed, uint64_t byte_off, size_t n, uint8_t* out) {
  for (size_t i = 0; i < n; ++i) {
    uint64_t b = byte_off + i;
    uint64_t w = oracle_splitmix64(seed ^ (b >> 3));
    out[i] = (uint8_t)(w >> (8 * (b & 7)));
  }
}

/* records [first, first + n) of the counter-based length stream (record r's
 * length depends on (seed, r) alone: a rank's share of one global stream is
 * generated without the records before it) */
void oracle_gen_zipf_lengths_at(uint64_t seed, double s, int kmax, uint32_t lmin, uint64_t first, size_t n,
                                uint32_t* out) {
  double* cdf = (double*)malloc(sizeof(double) * (size_t)kmax);
  double tot = 0.0;
  for (int k = 1; k <= kmax; ++k) tot += pow((double)k, -s);
  double acc = 0.0;
  for (int k = 1; k <= kmax; ++k) {
    acc += pow((double)k, -s);
    cdf[k - 1] = acc / tot;
  }
  cdf[kmax - 1] = 1.0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t r = first + i;
    uint64_t u1 = oracle_splitmix64(seed ^ (2 * r));
    uint64_t u2 = oracle_splitmix64(seed ^ (2 * r + 1));
    double u = (double)(u1 >> 11) * 0x1.0p-53;
    int lo = 0, hi = kmax - 1;
    while (lo < hi) {
      int mid = (lo + hi) / 2;
      if (u < cdf[mid])
        hi = mid;
      else
        lo = mid + 1;
    }
    int64_t L = 64 * (int64_t)(lo + 1) - (int64_t)(u2 & 63);
    out[i] = L < (int64_t)lmin ? lmin : (uint32_t)L;
  }
  free(cdf);
}

void oracle_gen_zipf_lengths(uint64_t seed, double s, int kmax, uint32_t lmin, size_t n, uint32_t* out) {
  oracle_gen_zipf_lengths_at(seed, s, kmax, lmin, 0, n, out);
}
