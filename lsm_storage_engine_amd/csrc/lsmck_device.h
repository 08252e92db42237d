// lsmck_device.h -- parameter blocks shared by the HIP kernels and the host
// dispatcher (lsmck_api.cpp).  Internal to liblsmck.so; not part of the C ABI.
#ifndef LSMCK_DEVICE_H
#define LSMCK_DEVICE_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsmck.h"

namespace lsmck {

// CRC-32 batch job.  Records are either fixed ([r*stride, r*stride+flen)) or
// described by (off[r], len[r]) relative to `base`.
struct CrcParams {
  const unsigned char* base;
  const uint64_t* off;        // descriptor mode
  const uint32_t* len;        // descriptor mode
  uint64_t stride;            // fixed mode
  uint32_t flen;              // fixed mode
  uint64_t nrec;
  uint64_t* total_segs;       // walking kernel scratch: total segments (device)
  uint32_t* out;              // nrec CRCs
  const uint32_t* kseg;       // x^(8*128*k) mod P, k < 2^16
  const uint32_t* khi;        // x^(8*128*65536*k) mod P, k < 2^16
  const uint32_t* tinit;      // 0xFFFFFFFF (x) x^(8*m) mod P, m = 0..128; [129] = 0
  const uint32_t* master;     // slicing-by-4 tables T0..T3 (4 x 256), then shift tables ST_1..ST_3 (3 x 4 x 256)
  const uint32_t* zero;       // 256 zero bytes (16-aligned): the load window of empty segments
  const uint64_t* sb_prefix;  // walking descriptor kernel: exclusive segment prefix per WALK_SB-record superblock
  uint32_t* sflag;            // stream kernel: nonzero = it takes the batch (the walking kernel then exits)
  uint64_t* scuts;            // stream kernel: first record of each wave's range (waves + 1 entries)
};

// SHA-256 batch job (lane per message).
struct ShaParams {
  const unsigned char* base;
  const uint64_t* off;        // null -> fixed mode
  const uint32_t* len;
  uint64_t stride;
  uint32_t flen;
  uint64_t nmsg;
  const uint32_t* order;      // optional permutation (longest first), may be null
  unsigned char* out;         // 32 bytes per message
  uint32_t pair;              // 1: two blocks per load window (A/B, lsmck_sha256.hip ShaWin2)
  const uint64_t* split;      // device: order index where the short tail starts (lean kernel), null = none
};

// One slice of a message streamed through sha256_slices_kernel.
#define SHA_SLICE_FIRST 1u
#define SHA_SLICE_LAST 2u
struct ShaSlice {
  uint64_t off;    // slice bytes at base + off
  uint64_t total;  // the message's length (used on its last slice)
  uint32_t len;    // slice bytes: a multiple of 64 unless it is the message's last slice
  uint32_t slot;   // state slot (8 u32) carrying the message between slices
  uint32_t msg;    // message index: digest at out + 32 * msg
  uint32_t flags;  // SHA_SLICE_FIRST | SHA_SLICE_LAST
};
struct ShaSliceParams {
  const unsigned char* base;
  const ShaSlice* slices;
  uint64_t nslices;
  uint32_t* state;
  unsigned char* out;
};

}  // namespace lsmck

extern "C" {
int lsmk_launch_crc32_fixed(const lsmck::CrcParams* P, int ncu, int variant, hipStream_t st);
int lsmk_launch_sha256(const lsmck::ShaParams* P, hipStream_t st);
int lsmk_launch_sha256_slices(const lsmck::ShaSliceParams* P, hipStream_t st);
uint64_t lsmk_walk_sb_count(uint64_t n);
int lsmk_launch_crc32_walk(const lsmck::CrcParams* P, uint64_t* sb_prefix, int ncu, int variant, hipStream_t st);
// stream kernel for sorted, non-overlapping batches (packed or with small gaps;
// a caller's batch is checked on the device unless `trusted`: P->sflag;
// P->scuts holds lsmk_stream_waves(ncu) + 1 entries)
uint32_t lsmk_stream_waves(int ncu);
int lsmk_ab_ablations(void);  // 1: built with -DLSMCK_AB_ABLATIONS (tools/build_ab.sh)
int lsmk_launch_crc32_stream(const lsmck::CrcParams* P, int ncu, int variant, int trusted, hipStream_t st);
uint64_t lsmk_wal_words(uint64_t n);
uint64_t lsmk_wal_scan_blocks(uint64_t n);
int lsmk_wal_mark_range(const uint8_t* img, uint64_t n, uint64_t b0, uint64_t b1, uint64_t* bits, uint32_t* pre,
                        hipStream_t st);
int lsmk_wal_mark(const uint8_t* img, uint64_t n, uint64_t* bits, uint32_t* pre, uint32_t* bsum, uint32_t* total,
                  int marked, uint64_t w0, uint64_t w1, hipStream_t st);
int lsmk_wal_chain(const uint8_t* img, uint64_t n, const uint64_t* bits, const uint32_t* pre, uint32_t nc, int levels,
                   uint64_t* pos, uint32_t* J, uint64_t* badpos, uint32_t* chain, unsigned long long* info, uint64_t w0,
                   uint64_t w1, uint64_t start, uint64_t lim, hipStream_t st);
int lsmk_wal_frame_insert(uint8_t* img, const uint64_t* off, const uint32_t* len, const uint32_t* crc, uint64_t n,
                          uint32_t kmax, hipStream_t st);
int lsmk_wal_emit(const uint8_t* img, uint64_t n, const uint32_t* chain, const uint64_t* pos,
                  const unsigned long long* info, uint32_t m, lsmck_wal_rec* recs, uint64_t* poff, uint32_t* plen,
                  uint32_t* pcrc, hipStream_t st);
// the segment walk (lsmck_segwalk.h; lsmck_wal.hip wal_seg_*)
namespace lsmck { namespace seg { struct SegArgs; } }
uint64_t lsmk_wal_seg_bytes(uint64_t len, uint64_t want);
uint64_t lsmk_wal_seg_scan_blocks(uint32_t K);
int lsmk_wal_seg_walk(const lsmck::seg::SegArgs* a, hipStream_t st);
int lsmk_wal_seg_round(const lsmck::seg::SegArgs* a, uint64_t* bsum, hipStream_t st);
int lsmk_wal_seg_repair(const lsmck::seg::SegArgs* a, uint32_t budget, hipStream_t st);
// a parallel repair round (seg::seg_prepair): g0 / x0 / code0 hold K entries (the snapshot)
int lsmk_wal_seg_prepair(const lsmck::seg::SegArgs* a, uint64_t* g0, uint64_t* x0, uint32_t* code0, hipStream_t st);
// recs: lsmck_wal_rec[] or, compact != 0, lsmck_wal_rec16[]
int lsmk_wal_seg_emit(const lsmck::seg::SegArgs* a, uint64_t at, void* recs, int compact, uint64_t* poff,
                      uint32_t* plen, uint32_t* pcrc, hipStream_t st);
int lsmk_wal_seg_emit_packed(const lsmck::seg::SegArgs* a, uint64_t at, void* recs, int compact, uint64_t* poff,
                             uint32_t* plen, uint32_t* pcrc, uint64_t iend, hipStream_t st);
int lsmk_wal_seg_place(const lsmck::seg::SegArgs* a, uint64_t at, void* recs, int compact, uint64_t* poff,
                       uint32_t* plen, uint32_t* pcrc, uint64_t iend, int packed, hipStream_t st);
// m wide records -> lsmck_wal_rec16 (out)
int lsmk_wal_recs_compact(const lsmck_wal_rec* in, void* out, uint64_t m, hipStream_t st);
int lsmk_launch_crc32_compare(const uint32_t* crc, const uint32_t* expected, uint64_t n,
                               unsigned long long* n_bad, unsigned long long* first_bad, hipStream_t st);
int lsmk_sha_order(const uint32_t* len, size_t n, uint16_t* keys_out, uint32_t* order, void* tmp, size_t* tmp_bytes,
                   int coarse, int from, hipStream_t st);
int lsmk_sha_split(const uint16_t* keys, size_t n, uint32_t t, uint64_t* split, hipStream_t st);
int lsmk_launch_gen_stream(unsigned char* dst, uint64_t seed, uint64_t byte_off, uint64_t n, hipStream_t st);
}
#endif
