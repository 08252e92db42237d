/*
 * lsmck.h -- C ABI of liblsmck.so, the MI355X-native checksum path of the
 * lsm_storage_engine reference (myroslavlisniak/lsm_storage_engine).
 *
 * The reference has no plugin/FFI API; its checksum path sits behind two Rust
 * seams:
 *   (i)  crc::crc32::checksum_ieee(&[u8]) -> u32, crate `crc` ^1.7
 *        (Cargo.toml:14), called at src/wal.rs:135,153 (replay verify) and
 *        src/wal.rs:177,187 (append);
 *   (ii) the crate-private Checksums API of src/checksums.rs:
 *        calculate_checksum (:20-38), verify (:40-62), write_checksums (:64-80),
 *        called from src/sync/sstable.rs:119,139,210 and
 *        src/tokio/sstable.rs:34,88,189.
 * Every entry point below names the reference item it replaces.  The Rust
 * bindings a maintainer would add are in INTEGRATION.md.
 *
 * Conventions
 *   - Plain pointers and sizes only.  The caller owns every buffer; the library
 *     never retains a caller pointer after the call returns (synchronous calls)
 *     or after the work on `stream` completes (LSMCK_DEVICE calls).
 *   - Return values: 0 = ok; < 0 = error (-EINVAL, -ENOMEM, -EIO, or
 *     LSMCK_EHIP - hipError_t); > 0 = an integrity verdict documented at the
 *     function.  lsmck_last_error() holds a thread-local message.
 *   - Scalar entry points (section 1) run on the calling CPU thread.  They are
 *     the per-record latency path (one WAL append = one call; a kernel launch
 *     costs microseconds), are reentrant and keep no mutable global state.
 *   - Batch entry points (section 3) run on the GPU and FAIL (return
 *     LSMCK_ENODEV) when no GPU / HIP runtime is usable: there is no CPU
 *     fallback for a batch.
 */
#ifndef LSMCK_H
#define LSMCK_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSMCK_ABI_VERSION 1

/* error codes (negative) */
#define LSMCK_EINVAL (-22)
#define LSMCK_ENOMEM (-12)
#define LSMCK_EIO (-5)
#define LSMCK_ENODEV (-19)
#define LSMCK_EHIP (-1000) /* LSMCK_EHIP - hipError_t */

/* flags for batch calls */
#define LSMCK_DEVICE 0x1u      /* base/off/len/out are device pointers; async on `stream` */
#define LSMCK_HOST 0x0u        /* host (pageable) pointers; staged through pinned memory; synchronous */
#define LSMCK_HOST_PINNED 0x2u /* host pointers already pinned (hipHostMalloc); DMA without a copy */
/* with LSMCK_DEVICE, descriptor CRC batches only: the caller asserts that its
 * records are sorted by offset, do not overlap, and that every byte between
 * the first record's start and the last record's end lies in memory it may
 * read (one buffer, e.g. a WAL image or a data file).  The stream kernel then
 * takes the batch without the device-side check of its descriptors (one pass
 * over them; lsmck_wal_replay_verify does the same for its own payloads). */
#define LSMCK_SORTED 0x4u

/* ======================================================================== */
/* 1. Scalar CPU entry points                                                */
/* ======================================================================== */

/* Replaces crc::crc32::checksum_ieee (crc ^1.7) at src/wal.rs:135,153,177,187.
 * CRC-32/ISO-HDLC: reflected 0xEDB88320, init/xorout 0xFFFFFFFF.
 * n == 0 accepts any p (an empty Rust slice passes a dangling non-null pointer)
 * and returns 0. */
uint32_t lsmck_crc32_ieee(const uint8_t* p, size_t n);

/* crc of (A || B) from crc(A) and the bytes of B (zlib crc32() convention);
 * lsmck_crc32_update(0, p, n) == lsmck_crc32_ieee(p, n). */
uint32_t lsmck_crc32_update(uint32_t crc_a, const uint8_t* p, size_t n);

/* crc of (A || B) from crc(A), crc(B) and |B|. */
uint32_t lsmck_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* SHA-256 (sha2 ^0.10.1 Sha256, src/checksums.rs:21,34,36). */
typedef struct {
  uint32_t h[8];
  uint64_t nbytes;
  uint8_t buf[64];
  uint32_t nbuf;
} lsmck_sha256_ctx;
void lsmck_sha256_init(lsmck_sha256_ctx* c);
void lsmck_sha256_update(lsmck_sha256_ctx* c, const uint8_t* p, size_t n);
void lsmck_sha256_final(lsmck_sha256_ctx* c, uint8_t out[32]);
void lsmck_sha256(const uint8_t* p, size_t n, uint8_t out[32]);

/* base64 ^0.13 `encode` (STANDARD alphabet, '=' padded), src/checksums.rs:37.
 * Writes 4*ceil(n/3) chars plus a NUL; returns the char count. */
size_t lsmck_base64_encode(const uint8_t* p, size_t n, char* out);

/* Positive status codes mark the places where the reference PANICS; negative
 * ones (-errno, LSMCK_EJSON) the places where it returns Err(io::Error).
 *   LSMCK_PANIC_OPEN_FILE      calculate_checksum's .expect("Can't open file to
 *                              calculate checksum") (src/checksums.rs:22-25), on the
 *                              file given (lsmck_checksum_file) or on the data file
 *                              (verify / write_checksums: it is hashed first, :41, :65)
 *   LSMCK_PANIC_OPEN_INDEX     the same panic on the index file (:42, :66)
 *   LSMCK_PANIC_OPEN_CHECKSUM  verify's .expect("Can't open checksum file") (:43-46)
 * A read error after a successful open is -errno (the `?` at :30). */
#define LSMCK_PANIC_OPEN_FILE 4
#define LSMCK_PANIC_OPEN_INDEX 5
#define LSMCK_PANIC_OPEN_CHECKSUM 6

/* Replaces Checksums::calculate_checksum(path) (src/checksums.rs:20-38):
 * SHA-256 of the whole file, base64 -> out (44 chars + NUL).  Returns 0,
 * LSMCK_PANIC_OPEN_FILE when the file cannot be opened (the reference panics,
 * :25), or -errno on a read error (Err, :30). */
int lsmck_checksum_file(const char* path, char out[45]);

/* Replaces Checksums::write_checksums(&SsTableMetadata) (src/checksums.rs:64-80):
 * hashes the data and index files and writes
 * {"index_checksum":"<b64>","data_checksum":"<b64>"} to checksum_path, opened
 * write+create WITHOUT truncate exactly as the reference opens it (:75-78).
 * Returns 0, LSMCK_PANIC_OPEN_FILE / LSMCK_PANIC_OPEN_INDEX (a data / index
 * file cannot be opened: panic), or -errno (a read error, or the checksum
 * file cannot be opened or written: Err, :78-79). */
int lsmck_checksums_write(const char* data_path, const char* index_path, const char* checksum_path);

/* Replaces Checksums::verify(&SsTableMetadata) (src/checksums.rs:40-62).
 * Returns, in the reference's order of checks:
 *   LSMCK_PANIC_OPEN_FILE / -errno      data file: cannot be opened (panic) / read error (Err)
 *   LSMCK_PANIC_OPEN_INDEX / -errno     index file: the same
 *   LSMCK_PANIC_OPEN_CHECKSUM           checksum file cannot be opened (panic, :46)
 *   LSMCK_EJSON / -errno                checksum file is not JSON of the Checksums
 *                                       shape, or cannot be read (Err, :48)
 *   LSMCK_DATA_MISMATCH / LSMCK_INDEX_MISMATCH   digest mismatch (panic, :49-60;
 *                                       data is checked first)
 *   0                                   both digests match */
#define LSMCK_DATA_MISMATCH 1
#define LSMCK_INDEX_MISMATCH 2
#define LSMCK_EJSON (-74)
int lsmck_checksums_verify(const char* data_path, const char* index_path, const char* checksum_path);

/* WAL record framing, CommandLog::log (src/wal.rs:165-196).
 * Insert: [u8 1][u32 crc LE][u32 klen][u32 vlen][key][val], crc over key||val.
 * Remove: [u8 2][u32 crc LE][u32 klen][key], crc over key.
 * Return the record size (13+klen+vlen / 9+klen); out must hold that much. */
size_t lsmck_wal_encode_insert(const uint8_t* key, uint32_t klen, const uint8_t* val, uint32_t vlen,
                               uint8_t* out);
size_t lsmck_wal_encode_remove(const uint8_t* key, uint32_t klen, uint8_t* out);

/* ======================================================================== */
/* 2. Device context                                                          */
/* ======================================================================== */
typedef struct lsmck_ctx lsmck_ctx;

/* Binds a context to HIP device `device` (one context per GPU; thread-safe:
 * concurrent calls on one context are serialised on its scratch). NULL on
 * failure (see lsmck_last_error). */
lsmck_ctx* lsmck_ctx_create(int device);
void lsmck_ctx_destroy(lsmck_ctx* ctx);
const char* lsmck_last_error(void);
int lsmck_device_count(void);

/* Tuning knobs of a context (no effect on results, only on speed):
 *   "crc_stream"  descriptor CRC batches: 1 = the stream kernel for sorted
 *                 batches (default), 0 = the walking kernel only (A/B),
 *                 2 = the stream kernel only (DIAGNOSTIC: a caller batch it
 *                 declines gets no CRCs).
 *   "crc_ablate"  DIAGNOSTIC ONLY, results are invalid while set: 3 = payload
 *                 loads only (ring, stream and walking kernels: the bench's
 *                 loads-only ceiling); 0 = off.  2 (the stream kernel without
 *                 payload loads) and 4..10 (stream kernel ablations,
 *                 DESIGN.md 3.1 items 10-11) only in A/B builds
 *                 (-DLSMCK_AB_ABLATIONS, tools/build_ab.sh).
 *   "sha_order"   variable-length SHA-256 batches of >= 2048 messages run in
 *                 decreasing length order (1, default) or batch order (0).
 *                 A/B switch; digests are identical either way.
 *   "sha_bucket_shift" / "sha_bucket_from"  that order's length key: messages
 *                 of from..1023 compression blocks share a bucket per
 *                 2^shift blocks (defaults 2 and 128; shift 0 = exact block
 *                 counts).  A/B switch; digests are identical either way.
 *   "sha_short_blocks"  in that order, messages of at most this many
 *                 compression blocks run on a lean kernel with more waves per
 *                 SIMD (default 12; 0 = every message on the window kernel).
 *                 Digests are identical either way.
 *   "sha_pair"    the window kernel loads two blocks (a 128-B line) per window
 *                 (1, default) or one (0); 2 and 3 are diagnostics (no payload
 *                 loads: digests invalid / line-aligned loads realigned
 *                 through LDS).
 *   "tree_active_files" / "tree_slice_bytes"  lsmck_checksums_verify_many's
 *                 files in flight (0 = 8192) and bytes of a file per round
 *                 (0 = 128 KiB; a multiple of 64).  Tests use small values.
 *   "tree_list_threads"  lsmck_tree_verify's metadata parsing threads (0 = 8).
 *   "tree_cpu_file_bytes"  whole-tree verify: files of at least this many
 *                 bytes are hashed on 4 host threads (SHA-NI where present)
 *                 instead of a GPU lane (0 = 16 MiB).
 *   "wal_prefetch"  bytes lsmck_wal_replay_verify's header walk prefetches
 *                 ahead of its position (default 4096; 0 = off).  A/B switch.
 *   "stage_numa"  where host-memory batches stage: -2 (default) the
 *                 device's NUMA node when the host has several -- pinned
 *                 buffers allocated there (lsmck_host_alloc_pinned too) and the
 *                 copy threads on its CPUs; -1 HIP's default placement and
 *                 unpinned threads; >= 0 that node.  Applies to buffers
 *                 allocated after the call.
 *   "stage_threads"  host-memory batches: threads that copy a pageable chunk
 *                 into its pinned staging slot (default 8; 1 = one memcpy).
 *   "wal_gpu_walk"  lsmck_wal_replay_verify of a device image: 1 = header walk
 *                 on the GPU (default), 0 = read back and walk on the host.
 *   "wal_upload_min"  host images of at least this many bytes are uploaded and
 *                 walked on the GPU (default 1 MiB; 0 = always the host walk).
 *   "wal_split"   an uploaded host image is walked in two parts, the first
 *                 behind the upload of the second (1, default; taken when each
 *                 half holds one "wal_stage_bytes" chunk), or whole after it (0).
 *   "wal_stage_bytes"  an uploaded host WAL image moves in chunks of this many
 *                 bytes (pageable: copied into a pinned slot, then DMA'd; each
 *                 chunk's candidate marking runs behind its DMA); a multiple
 *                 of 64 KiB in [1 MiB, 64 MiB], default 16 MiB.
 *   "wal_register"  1 = an uploaded host WAL image is DMA'd from the caller's
 *                 own pages, pinned in place for the call (hipHostRegister),
 *                 instead of through the pinned staging copy (default 0).  A/B.
 *   "wal_chunk_bytes"  lsmck_wal_replay_verify of a host image: CRC batches
 *                 of this many payload bytes run on a helper thread while the
 *                 walk goes on (default 32 MiB; 0 = one batch after the walk).
 *   "tree_overlap"  lsmck_tree_verify reads the highest level's directory
 *                 first and, when it holds at least this many tables (default
 *                 2048; 0 = never), verifies them while the lower levels are
 *                 listed -- its first 8x this many as soon as they are
 *                 parsed, the rest once the level is read -- then the lower
 *                 levels' tables.  The report is the same either way (the
 *                 first failure in read_dir order).
 *   "tree_list_batch"  lsmck_tree_verify: metadata names per listing batch
 *                 (0 = 1024).  Tests use small values.
 *   "tree_json_threads"  whole-tree verify: threads reading the tables'
 *                 checksum files beside the stream (0 = default: 2, or 4 for
 *                 a batch of 16k tables or more).
 *   "tree_stages"  whole-tree verify: pinned slots its rounds cycle through
 *                 (3, default: a round is read while the two before it upload
 *                 and hash; 2 = round 4's double buffering).  A/B.
 *   "tree_open_files"  files kept open from their first slice to their last
 *                 (-1 = default: as many as RLIMIT_NOFILE leaves after a
 *                 1024-descriptor reserve; the rest reopen per slice).
 *   "wal_part_bytes"  the candidate-doubling GPU walk goes in parts of this
 *                 many bytes (0 = whole, default; otherwise >= 1 MiB; a
 *                 nonzero value also skips the segment walk).  Tests / A/B.
 *   "wal_seg_walk"  the GPU header walk: 1 = the segment walk (default;
 *                 lsmck_segwalk.h), falling back to candidate doubling when
 *                 its check keeps failing; 0 = candidate doubling only.
 *   "wal_seg_bytes"  segment walk: bytes per segment (0 = auto, default:
 *                 ~2^16 segments; else 64..2^30).  Tests use small segments.
 *   "wal_seg_rounds"  segment walk: check failures repaired before it
 *                 declines to candidate doubling (default 16).
 *   "wal_seg_prepair"  segment walk: parallel repair rounds (every segment
 *                 walked again from its predecessor's exit at once) after a
 *                 check with several failures, before the serial repairs
 *                 (default 2; 0 = none).
 *   "wal_seg_pack"  segment walk: 1 = the CRC pass runs over packed spans,
 *                 each payload with the next record's header, the header
 *                 then taken back out of the CRC (default); 0 = over the
 *                 payloads alone.  A/B; results are the same.
 *   "wal_seg_stage"  segment walk: the walk stages the records it passes so
 *                 they need no second walk of the headers: 1 = auto slots
 *                 per segment (default), 0 = off (A/B), N >= 2 = N slots
 *                 (tests).  A segment with more records is walked again.
 *   "wal_dma_engines"  device replays whose records go to the host: the
 *                 read-back is dealt over this many SDMA engines through HSA
 *                 (default 4; 1..16), beside the CRC pass and off the compute
 *                 units; 0 = hipMemcpyAsync on a staging stream (A/B).
 *   "wal_dma_chunks"  ... cut in this many pieces (default 32; 1..64); a
 *                 pageable records array is filled piece by piece as they land.
 *   "wal_pipe"    device replays of at least "wal_pipe_min" bytes (default
 *                 1 GiB): the log is walked in this many parts (2..64) on a
 *                 CU-masked stream while the previous part's CRC pass runs
 *                 on the other CUs; 0 or 1 = off (default 0: measured slower,
 *                 DESIGN.md 8).  "wal_pipe_first" the first part in 64ths
 *                 of the log (1..63, default 4), "wal_pipe_cus" the walk's
 *                 CUs (default 32), "wal_pipe_layout" which ones (0 the last,
 *                 1 spread), "wal_pipe_seg" the parts' segment bytes (0 =
 *                 sized to the walk's CUs).  A/B; results are the same.
 *   "tree_readers"  whole-tree verify: reader threads per context (default
 *                 16; 1..64).  A/B.
 *   "crc_ablate"  diagnostic: 3 = the stream kernel with payload loads only
 *                 (the bench's loads-only ceiling; results are garbage); 2,
 *                 4..12 only in A/B libraries built with -DLSMCK_AB_ABLATIONS.
 * Returns 0, or LSMCK_EINVAL for an unknown key / value. */
int lsmck_ctx_set_option(lsmck_ctx* ctx, const char* key, long value);

/* What the context's last call of a kind did (diagnostics for tests and
 * tools; no effect on results):
 *   "wal_walk_path"  the last lsmck_wal_replay_verify that walked on the GPU
 *                    or the host: 1 = segment walk, 2 = candidate doubling,
 *                    3 = host walk.
 *   "wal_seg_repairs"  its segment walk's repaired check failures.
 *   "wal_segments"   its segment walk's segment count.
 *   "wal_seg_prepairs"  its segment walk's parallel repair rounds.
 *   "wal_recs_dma"   its records' read-back to the host: the SDMA engines it
 *                    was dealt over, 0 = hipMemcpyAsync (or none read back).
 *   "wal_pipe_parts"  its pipelined parts ("wal_pipe"; 0 = one walk, one pass).
 *   "numa_node"      the device's NUMA node (sysfs of its PCI function; -1
 *                    unknown), and "stage_numa_node" the node the context's
 *                    pinned buffers and copy threads are placed on (-1: none).
 * Returns 0 and *value, or LSMCK_EINVAL for an unknown key. */
int lsmck_ctx_get_stat(lsmck_ctx* ctx, const char* key, long* value);

/* ======================================================================== */
/* 3. Batch GPU entry points                                                  */
/* ======================================================================== */

/* CRC-32 of n records: record i = base[off[i] .. off[i]+len[i]).  The batch
 * form of checksum_ieee for WAL replay / bulk append (src/wal.rs:135,153,177).
 * Any offsets, lengths and order.  A device batch whose records are sorted,
 * do not overlap, lie at most 64 bytes apart (a WAL's 13- / 9-byte headers)
 * and whose empty records sit at their predecessor's end runs on the stream
 * kernel (decided on the device, nothing read back); any other batch on the
 * walking kernel.  Host batches are staged in order and always take the
 * stream kernel.  stream: hipStream_t (NULL = the context's default stream). */
int lsmck_crc32_batch(lsmck_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint32_t* len, size_t n,
                      uint32_t* out, unsigned flags, void* stream);

/* Fixed-size records: record i = base[i*stride .. i*stride+len). */
int lsmck_crc32_batch_fixed(lsmck_ctx* ctx, const uint8_t* base, size_t stride, uint32_t len, size_t n,
                            uint32_t* out, unsigned flags, void* stream);

/* Verify: compares against expected[i].  Host-visible results: *n_bad and
 * *first_bad (index of the first mismatching record in batch order, or n).
 * Synchronous.  Returns 0 when every record matches, 1 otherwise. */
int lsmck_crc32_verify_batch(lsmck_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint32_t* len,
                             const uint32_t* expected, size_t n, unsigned flags, void* stream, uint64_t* n_bad,
                             uint64_t* first_bad);

/* SHA-256 of n messages -> out32[32*i .. 32*i+32).  The batch form of
 * calculate_checksum's digest (src/checksums.rs:20-38). */
int lsmck_sha256_batch(lsmck_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint32_t* len, size_t n,
                       uint8_t* out32, unsigned flags, void* stream);
int lsmck_sha256_batch_fixed(lsmck_ctx* ctx, const uint8_t* base, size_t stride, uint32_t len, size_t n,
                             uint8_t* out32, unsigned flags, void* stream);

/* WAL replay verify: the batch form of the CommandLog iterator + MemTable::from_log
 * (src/wal.rs:68-84,122-163; src/memtable.rs:28-47) over an in-memory WAL image.
 * Each record's length lives in its own header, so the walk is a dependent
 * chain.  On the GPU (lsmck_wal.hip) it is a speculative parallel parse: the
 * segment walk (lsmck_segwalk.h: one thread per segment of the log guesses
 * the segment's first record and walks the headers to the next segment; the
 * guesses are checked against each other and wrong ones repaired), or, when
 * its check keeps failing, candidate doubling (every byte that could start a
 * header is a candidate, candidate -> successor links followed by pointer
 * doubling from offset 0); the accepted chain's payload CRCs are checked in
 * one batch with the GPU compare.  A device image
 * never leaves the device; a host image of at least "wal_upload_min" bytes
 * (default 1 MiB) is uploaded whole and walked there; smaller host images
 * (and "wal_upload_min" 0) take the serial host walk with the CRC batches on
 * the GPU.  Results are the same on every path.
 * recs (optional, cap entries) receives the parsed records in log order.
 * Returns
 *   0                      clean end of log (header EOF ends iteration, wal.rs:76-77)
 *   LSMCK_WAL_CORRUPTED    first bad record is an Insert: WalError::CorruptedData
 *                          {checksum=*bad_crc, expected=*bad_expected} (wal.rs:136-141)
 *   LSMCK_WAL_REMOVE_PANIC first bad record is a Remove: the reference panics (wal.rs:154-159)
 *   LSMCK_WAL_BAD_TYPE     InvalidCommandType(*bad_crc) at record *bad_index (wal.rs:36)
 * *nrec = records accepted before the stop.  flags: LSMCK_HOST (optionally
 * | LSMCK_HOST_PINNED) or LSMCK_DEVICE for `wal`, optionally
 * | LSMCK_RECS_PINNED: `recs` is page-locked (lsmck_host_alloc_pinned), and
 * the records are DMA'd into it straight from the device (no staging copy),
 * or | LSMCK_RECS_DEVICE: `recs` is device memory (cap entries) and the
 * records stay there -- for a device-resident log whose consumer runs on the
 * GPU; the segment walk writes them in place when all of them fit, and no
 * record crosses the host link (any path that walks on the host copies its
 * records up).  In either array, entries past *nrec up to the walked record
 * count (records after a failed CRC) may be written too.  Synchronous. */
#define LSMCK_RECS_PINNED 0x8u
#define LSMCK_RECS_DEVICE 0x10u
#define LSMCK_WAL_CORRUPTED 1
#define LSMCK_WAL_REMOVE_PANIC 2
#define LSMCK_WAL_BAD_TYPE 3
typedef struct {
  uint64_t rec_off;     /* header offset */
  uint64_t payload_off; /* key offset */
  uint32_t klen, vlen;  /* vlen = 0 for Remove */
  uint32_t crc;         /* stored checksum */
  uint32_t type;        /* 1 Insert, 2 Remove */
} lsmck_wal_rec;
int lsmck_wal_replay_verify(lsmck_ctx* ctx, const uint8_t* wal, size_t n, unsigned flags, lsmck_wal_rec* recs,
                            size_t cap, size_t* nrec, uint64_t* bad_index, uint32_t* bad_crc,
                            uint32_t* bad_expected);

/* The same replay with compact records: 16 bytes each instead of 32 -- what
 * MemTable::from_log takes from a record (src/memtable.rs:28-47: the key and
 * value bytes and the command type).  The header offset is payload_off less
 * the header (13 bytes for Insert, 9 for Remove), and the stored CRC is not
 * kept: every accepted record's stored CRC equals its payload's CRC (a bad
 * one's comes back in *bad_expected).  Half the bytes cross the link when
 * the records go to the host (LSMCK_RECS_PINNED or a pageable array); with
 * LSMCK_RECS_DEVICE `recs` is a device array of lsmck_wal_rec16.  Flags,
 * returns and the other outputs as lsmck_wal_replay_verify.  Replaces the
 * same reference items. */
typedef struct {
  uint64_t payload_type; /* bits 0..62: payload (key) offset; bit 63: set for Remove, clear for Insert */
  uint32_t klen, vlen;   /* vlen = 0 for Remove */
} lsmck_wal_rec16;
#define LSMCK_WAL_REC16_REMOVE 0x8000000000000000ull
#define LSMCK_WAL_REC16_OFF_MASK 0x7FFFFFFFFFFFFFFFull
int lsmck_wal_replay_verify16(lsmck_ctx* ctx, const uint8_t* wal, size_t n, unsigned flags, lsmck_wal_rec16* recs,
                              size_t cap, size_t* nrec, uint64_t* bad_index, uint32_t* bad_crc,
                              uint32_t* bad_expected);

/* Batch framing of Insert records in a device-resident log, in place: payload
 * i (key || value, len[i] bytes) already lies at img + off[i], and its
 * 13-byte header (CommandLog::log, src/wal.rs:165-196) is written to
 * img + off[i] - 13 -- type 1, crc[i], klen = min(len[i], kmax), vlen = the
 * rest.  The batch form of lsmck_wal_encode_insert for logs built on the
 * GPU (a log of many GiB is framed in one launch); crc[i] is normally
 * lsmck_crc32_batch's output for the same payloads.  img, off, len, crc:
 * device pointers; asynchronous on `stream` (NULL = the context's stream).
 * Returns 0 or a negative hipError_t. */
int lsmck_wal_frame_insert_device(lsmck_ctx* ctx, uint8_t* img, const uint64_t* off, const uint32_t* len,
                                  const uint32_t* crc, size_t n, uint32_t kmax, void* stream);

/* Whole-tree SSTable verify: the batch form of Checksums::verify over many
 * tables (Db::load, src/tokio/db.rs:37-59 -> src/tokio/sstable.rs:34).
 * Streams every data/index file in slices: 8192 files in flight (largest
 * first), 128 KiB of each per round, 16 reader threads filling one pinned slot
 * while the GPU hashes the previous round (per-file SHA-256 state carried on
 * the device), then compares with each checksum file.  Files of 16 MiB and
 * more are hashed on host threads meanwhile (one file is one sequential
 * SHA-256: a GPU lane would take ~1 s per 16 MB).  status[i] gets table i's
 * lsmck_checksums_verify status (0, the LSMCK_PANIC_OPEN_* codes,
 * LSMCK_DATA_MISMATCH / LSMCK_INDEX_MISMATCH, -errno, LSMCK_EJSON; -EAGAIN: a
 * file shrank while it was read).  Returns the number of tables whose status
 * is not 0. */
int lsmck_checksums_verify_many(lsmck_ctx* ctx, const char* const* data_paths, const char* const* index_paths,
                                const char* const* checksum_paths, size_t n, int* status);

/* Db::load's whole checksum scan of a tree (src/tokio/db.rs:37-59): for
 * level-0 .. level-4 under `base` (created if missing, fs::create_dir_all),
 * every directory entry whose UTF-8 name contains "metadata" is parsed as
 * SsTableMetadata JSON (sstable_metadata.rs:76-83) and the table it names --
 * base_path/level-<level>/{data,index,checksum}_filename -- is verified as by
 * lsmck_checksums_verify_many.  Metadata parsing runs on 8 host threads.  Returns 0 when every table verifies, 1 when some table
 * does not (rep->first_* names the first one in load order: level, then
 * read_dir order -- the table where the reference's loop panics or errors),
 * or a negative error (creating or listing a level directory failed).
 * first_status is a lsmck_checksums_verify_many status or LSMCK_META_PANIC:
 * the metadata file is unreadable or not valid SsTableMetadata JSON, where
 * the reference panics with "Can't open metadata file" / "Can't read metadata
 * file, file with unknown format" (sstable_metadata.rs:77-83). */
#define LSMCK_SSTABLE_MAX_LEVEL 5 /* src/tokio/db.rs:17 */
#define LSMCK_META_PANIC 3
typedef struct {
  uint64_t tables;      /* metadata entries found */
  uint64_t table_bytes; /* data + index bytes hashed */
  uint64_t bad_tables;  /* tables with a non-zero status */
  uint64_t first_index; /* load-order index of the first bad table (UINT64_MAX: none) */
  int first_status;
  int reserved;
  double list_seconds;   /* listing + metadata parsing */
  double verify_seconds; /* the lsmck_checksums_verify_many part, split as: */
  double stat_seconds;   /*   sizing the files */
  double read_seconds;   /*   reader threads filling the pinned slots */
  double gpu_wait_seconds; /* waiting for a slot's copy + kernels, final digest copy */
  double compare_seconds;  /*  reading the checksum files, comparing */
  uint64_t rounds;         /*  slice rounds */
  uint64_t fds_cached;     /*  files kept open between slices (RLIMIT_NOFILE bound) */
  char first_metadata_path[4096];
} lsmck_tree_report;
int lsmck_tree_verify(lsmck_ctx* ctx, const char* base, lsmck_tree_report* rep);

/* The same verify, handing the caller the listing it made: `fn` is called once,
 * after every metadata file is parsed and before the tables are hashed, with
 * the tables in load order (per level, read_dir order).  The entries live until
 * lsmck_tree_verify_listed returns, so the caller can load the tables' read
 * path (their sparse indexes) beside the verify instead of opening every
 * metadata file again -- Db::load's other half (src/tokio/db.rs:40-55 ->
 * SsTable::load).  fn may be NULL. */
typedef struct {
  const char* metadata_path;
  const char* data_path;     /* construct_path: base_path/level-<level>/data_filename (sstable_metadata.rs:43-48) */
  const char* index_path;
  const char* checksum_path;
  const char* id;            /* the metadata's u128 id, decimal */
  unsigned level;
  int status;                /* 0, or LSMCK_META_PANIC: not SsTableMetadata JSON (paths and id "") */
} lsmck_table_entry;
typedef void (*lsmck_tree_listed_fn)(void* user, const lsmck_table_entry* tables, size_t n);
int lsmck_tree_verify_listed(lsmck_ctx* ctx, const char* base, lsmck_tree_report* rep, lsmck_tree_listed_fn fn,
                             void* user);

/* The same over several devices of one node: the tables are split
 * into contiguous runs balanced by bytes, one per context (one host thread,
 * one set of pinned slots and one PCIe link each), verified concurrently; no
 * data moves between devices.  Statuses and the report are those of the
 * single-context call (timings: the slowest device's). */
int lsmck_tree_verify_multi(lsmck_ctx* const* ctxs, size_t nctx, const char* base, lsmck_tree_report* rep);
int lsmck_checksums_verify_many_multi(lsmck_ctx* const* ctxs, size_t nctx, const char* const* data_paths,
                                      const char* const* index_paths, const char* const* checksum_paths, size_t n,
                                      int* status);

/* ======================================================================== */
/* 4. Plumbing for hosts without their own HIP bindings (tests, bench)        */
/* ======================================================================== */
void* lsmck_dev_alloc(lsmck_ctx* ctx, size_t bytes);       /* hipMalloc */
void lsmck_dev_free(lsmck_ctx* ctx, void* p);
void* lsmck_host_alloc_pinned(lsmck_ctx* ctx, size_t bytes); /* hipHostMalloc */
void lsmck_host_free_pinned(lsmck_ctx* ctx, void* p);
int lsmck_memcpy_h2d(lsmck_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream);
int lsmck_memcpy_d2h(lsmck_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream);
int lsmck_memset_dev(lsmck_ctx* ctx, void* dst, int value, size_t bytes, void* stream);
int lsmck_stream_sync(lsmck_ctx* ctx, void* stream);
/* Synthetic records: device byte stream, byte b = byte (b%8) of
 * splitmix64(seed ^ (b/8)) for b in [byte_off, byte_off+n). */
int lsmck_gen_stream(lsmck_ctx* ctx, uint8_t* dst_dev, uint64_t seed, uint64_t byte_off, size_t n, void* stream);
/* Zipf(s) lengths on k=1..kmax, L = max(lmin, 64k - j), j ~ U{0..63} (host). */
void lsmck_gen_zipf_lengths(uint64_t seed, double s, int kmax, uint32_t lmin, size_t n, uint32_t* out);
/* records [first, first + n) of the same stream (record r's length depends on
 * (seed, r) alone): one rank's share of a global config-3 stream */
void lsmck_gen_zipf_lengths_at(uint64_t seed, double s, int kmax, uint32_t lmin, uint64_t first, size_t n,
                               uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* LSMCK_H */
