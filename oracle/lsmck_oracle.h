/*
 * lsmck_oracle.h -- CPU restatement of the reference's checksum path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (lsm_storage_engine_amd/,
 * liblsmck.so) links, loads or calls this code.  Only tests/, the smoke() of
 * __graft_entry__.py and the cpu_baseline leg of bench.py use it, and only as
 * the checker / the timed CPU baseline.
 *
 * The reference (myroslavlisniak/lsm_storage_engine, Rust) cannot be built in
 * this image (no rustc/cargo, no crate sources, no Cargo.lock), so this is a
 * restatement of the algorithms its hot path delegates to:
 *   - crc  ^1.7 (resolves to 1.8.1), crc::crc32::checksum_ieee  [Cargo.toml:14]
 *       called at src/wal.rs:135,153 (replay) and :177,187 (append):
 *       CRC-32/ISO-HDLC, reflected poly 0xEDB88320, init/xorout 0xFFFFFFFF,
 *       Sarwate byte-at-a-time table update (crc 1.x `update`).
 *   - sha2 ^0.10.1, Sha256  [Cargo.toml:11]  used by src/checksums.rs:20-38
 *       (FIPS 180-4 SHA-256 over the whole file, streamed in 1 KiB reads).
 *   - base64 ^0.13, base64::encode  [Cargo.toml:12]  src/checksums.rs:37
 *       (STANDARD alphabet, '=' padded).
 *   - serde_json ^1 to_writer of struct Checksums  src/checksums.rs:13-17,79
 *       -> {"index_checksum":"...","data_checksum":"..."} (declaration order).
 *
 * Parity pinning: the reference's own tests hold no literal checksum values
 * (SURVEY.md section 4/8c), so this oracle is pinned by the published
 * known-answer vectors of those algorithms (CRC-32 check "123456789" ->
 * 0xCBF43926, FIPS 180-2 SHA-256 "abc"/"" vectors, RFC 4648 base64 vectors)
 * and by fixtures produced with independent implementations (Python zlib,
 * hashlib, base64) laid out exactly as the reference's byte formats
 * (tests/golden/make_golden.py).  Reference-level parity is therefore
 * "pinned to the crates' published algorithms", not to reference outputs.
 */
#ifndef LSMCK_ORACLE_H
#define LSMCK_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- CRC-32/ISO-HDLC (crc 1.x checksum_ieee) ---------------------------- */
uint32_t oracle_crc32_ieee(const uint8_t* p, size_t n);
/* one record per descriptor; nthreads<=1 -> single thread */
void oracle_crc32_batch(const uint8_t* base, const uint64_t* off, const uint32_t* len, size_t n,
                        uint32_t* out, int nthreads);
void oracle_crc32_fixed(const uint8_t* base, size_t stride, size_t len, size_t n, uint32_t* out,
                        int nthreads);

/* ---- SHA-256 (sha2 0.10) -------------------------------------------------- */
typedef struct {
  uint32_t h[8];
  uint64_t nbytes;
  uint8_t buf[64];
  uint32_t nbuf;
} oracle_sha256_ctx;
void oracle_sha256_init(oracle_sha256_ctx* c);
void oracle_sha256_update(oracle_sha256_ctx* c, const uint8_t* p, size_t n);
void oracle_sha256_final(oracle_sha256_ctx* c, uint8_t out[32]);
void oracle_sha256(const uint8_t* p, size_t n, uint8_t out[32]);
void oracle_sha256_batch(const uint8_t* base, const uint64_t* off, const uint32_t* len, size_t n,
                         uint8_t* out32, int nthreads);

/* ---- base64 STANDARD padded (base64 0.13 encode) ----------------------- */
size_t oracle_base64_std(const uint8_t* p, size_t n, char* out); /* writes NUL, returns strlen */

/* ---- checksums.rs restatement ------------------------------------------- */
/* calculate_checksum(path): SHA-256 of the whole file (1 KiB reads), base64.
 * returns 0 ok, -errno on I/O failure. out must hold 45 bytes. */
int oracle_file_checksum(const char* path, char out[45]);
/* JSON text exactly as serde_json::to_writer(&Checksums) writes it. */
size_t oracle_checksums_json(const char* index_b64, const char* data_b64, char* out, size_t cap);

/* ---- wal.rs record framing ----------------------------------------------- */
/* CommandLog::log Insert (wal.rs:168-185): [u8 1][u32 crc][u32 klen][u32 vlen][key][val] */
size_t oracle_wal_encode_insert(const uint8_t* key, uint32_t klen, const uint8_t* val, uint32_t vlen,
                                uint8_t* out);
/* CommandLog::log Remove (wal.rs:186-194): [u8 2][u32 crc][u32 klen][key] */
size_t oracle_wal_encode_remove(const uint8_t* key, uint32_t klen, uint8_t* out);

/* Replay (wal.rs:68-84, 122-163).  Fills up to cap entries of the record
 * table; returns the status of the scan:
 *   0  clean end (header EOF / UnexpectedEof, wal.rs:76-77)
 *   1  CorruptedData on an Insert (wal.rs:136-141) -> *bad_index, *bad_crc, *bad_expected
 *   2  Remove checksum mismatch -> reference panics (wal.rs:154-159)
 *   3  InvalidCommandType (wal.rs:36) -> *bad_index = record index, *bad_crc = type byte
 * *nrec = number of records returned before the stop. */
typedef struct {
  uint64_t rec_off;     /* offset of the header byte */
  uint64_t payload_off; /* offset of key */
  uint32_t klen, vlen;  /* vlen = 0 for Remove */
  uint32_t crc;         /* stored checksum */
  uint8_t type;         /* 1 insert, 2 remove */
} oracle_wal_rec;
int oracle_wal_replay(const uint8_t* buf, size_t n, oracle_wal_rec* recs, size_t cap, size_t* nrec,
                      uint64_t* bad_index, uint32_t* bad_crc, uint32_t* bad_expected);

/* ---- synthetic inputs shared with the bench (counter-based) ------------- */
uint64_t oracle_splitmix64(uint64_t x);
/* byte i of the stream = byte (i%8) (little endian) of splitmix64(seed ^ (i/8)) */
void oracle_gen_stream(uint64_t seed, uint64_t byte_off, size_t n, uint8_t* out);
/* Zipf(s) over k in 1..kmax, L = max(lmin, 64k - j), j ~ U{0..63}; SURVEY 8d config 3 */
void oracle_gen_zipf_lengths(uint64_t seed, double s, int kmax, uint32_t lmin, size_t n, uint32_t* out);
void oracle_gen_zipf_lengths_at(uint64_t seed, double s, int kmax, uint32_t lmin, uint64_t first, size_t n,
                                uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif
