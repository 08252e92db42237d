// lsmck_order.hip -- dispatch order for variable-length SHA-256 batches.
//
// sha256_kernel runs one message per lane (SHA-256 is sequential inside a
// message), so a wave costs as much as its longest message.  For a batch of
// mixed lengths (SSTable data + index files of every level, src/checksums.rs
// over a whole tree; or config 3's Zipf records) in batch order, most lanes of
// a wave sit idle: measured 55.6 GiB/s on config 3 against 1,316 GiB/s for
// equal 4 KiB records.  This file builds a permutation that visits messages by
// decreasing compression-block count, so every wave holds messages of nearly
// equal length and the longest go first (longest-processing-time order for
// the tail).  Exact block counts below 128 (8 KiB); 4-block buckets from 128
// to 1023 blocks; above that, 16 log-spaced buckets per octave (lengths within
// 1/16 of each other).  The 4-block buckets trade a little lane divergence for
// locality: equal-key messages are 4x denser in the batch, so a wave's lanes
// read messages closer together (config 3 SHA-256: 83.8 -> 72.0 ms; exact
// keys stay available, option "sha_bucket_shift" 0).  The key is 11 bits,
// sorted with rocPRIM's device radix sort (stable, two passes).
// Results do not depend on the order: the kernel writes message m's digest to
// out[32*m].
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>
#include <stdint.h>

namespace lsmck {

struct ShaBucket {
  // coarse (A/B, option "sha_bucket_shift"): block counts from..1023 share a
  // bucket per 2^coarse blocks, so equal-key messages lie closer in memory
  uint32_t coarse = 2, from = 128;
  __host__ __device__ uint16_t operator()(uint32_t len) const {
    const uint32_t nb = (uint32_t)(((uint64_t)len + 72u) >> 6);  // compression blocks: ceil((len + 9) / 64)
    if (coarse == 0) {
      if (nb < 1024u) return (uint16_t)nb;
      const uint32_t e = 31u - (uint32_t)__builtin_clz(nb);  // 10..26
      return (uint16_t)(1024u + 16u * (e - 10u) + ((nb >> (e - 4u)) & 15u));
    }
    if (nb < from) return (uint16_t)nb;
    if (nb < 1024u) return (uint16_t)(from + ((nb - from) >> coarse));
    const uint32_t e = 31u - (uint32_t)__builtin_clz(nb);
    return (uint16_t)(from + ((1024u - from) >> coarse) + 16u * (e - 10u) + ((nb >> (e - 4u)) & 15u));
  }
};

}  // namespace lsmck

// order[0..n) = message indices by decreasing block-count bucket.  With
// tmp == nullptr only *tmp_bytes is set (rocPRIM's two-call protocol).
extern "C" int lsmk_sha_order(const uint32_t* len, size_t n, uint16_t* keys_out, uint32_t* order, void* tmp,
                              size_t* tmp_bytes, int coarse, int from, hipStream_t st) {
  lsmck::ShaBucket b;
  b.coarse = (uint32_t)coarse;
  b.from = (uint32_t)from;
  auto keys = rocprim::make_transform_iterator(len, b);
  rocprim::counting_iterator<uint32_t> idx(0u);
  hipError_t e = rocprim::radix_sort_pairs_desc(tmp, *tmp_bytes, keys, keys_out, idx, order, n, 0, 11, st);
  return e == hipSuccess ? 0 : -(int)e;
}

// The first position in the order whose key is at most `t` blocks (keys are
// sorted descending; below sha_bucket_from a key is the exact block count):
// where the short messages start.  One thread, binary search.
__global__ void sha_split_kernel(const uint16_t* keys, uint64_t n, uint32_t t, uint64_t* split) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (keys[mid] > t) lo = mid + 1; else hi = mid;
  }
  *split = lo;
}

extern "C" int lsmk_sha_split(const uint16_t* keys, size_t n, uint32_t t, uint64_t* split, hipStream_t st) {
  hipLaunchKernelGGL(sha_split_kernel, dim3(1), dim3(1), 0, st, keys, (uint64_t)n, t, split);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}
