// lsmck_sha256.hip -- batched SHA-256 (FIPS 180-4) over independent messages,
// gfx950.  This is the digest src/checksums.rs:20-38 computes over a whole
// SSTable data / index file (sha2 ^0.10.1, Cargo.toml:11); the host side
// (lsmck_api.cpp) adds base64 (checksums.rs:37) and the JSON record.
//
// Merkle-Damgard is sequential inside one message, so parallelism is across
// messages: one lane owns one message and runs all of its compression blocks.
// The kernel is int32-VALU bound (~1.4k VALU ops per 64-B block, rotates are
// v_alignbit, Ch/Maj are v_bitop3), not HBM bound; DESIGN.md prices it
// against the VALU roof.  Loads are dword-aligned with a v_alignbyte funnel
// and never touch a dword outside the message.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lsmck_device.h"

namespace lsmck {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__constant__ uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
// a ^ b ^ c in one v_bitop3_b32 (truth table 0x96): hipcc emits two v_xor_b32
// for the Sigma/sigma functions otherwise (1,716 -> ~1,490 VALU per block)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// Ch(e, f, g) = e ? f : g and Maj(a, b, c) in one v_bitop3_b32 each (truth
// tables 0xCA, 0xE8; bit (x<<2 | y<<1 | z) of the table for inputs x, y, z).
// hipcc builds Maj as v_xor + v_and + v_bitop3 otherwise: 128 VALU per block.
__device__ __forceinline__ uint32_t ch3(uint32_t e, uint32_t f, uint32_t g) {
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

__device__ __forceinline__ void sha256_compress(uint32_t (&h)[8], uint32_t (&w)[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
      w[t & 15] = wt;
    }
    uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    uint32_t ch = ch3(e, f, g);
    uint32_t t1 = hh + S1 + ch + kSha256K[t] + wt;
    uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    uint32_t mj = maj3(a, b, c);
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + mj;
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

__device__ __forceinline__ uint32_t ld32(const unsigned char* p) { return *(const uint32_t*)p; }
__device__ __forceinline__ u32x4 ld128(const unsigned char* p) { return *(const u32x4*)p; }

// Loads the 64 message bytes [p0, p0+64) of a message starting at absolute
// address A with length len, as 16 little-endian words; only dwords that
// intersect [A, A+len) are read (others are 0; the caller masks and pads).
__device__ __forceinline__ void load_block(uintptr_t A, uint64_t len, uint64_t p0, uint32_t (&wle)[16]) {
  const uintptr_t s = A + p0;
  const uintptr_t a4 = s & ~(uintptr_t)3;
  const uint32_t sh = (uint32_t)(s & 3);
  // one past the last dword touching the message (an empty message touches none)
  const uintptr_t end4 = len ? ((A + len + 3) & ~(uintptr_t)3) : (A & ~(uintptr_t)3);
  const unsigned char* p = (const unsigned char*)a4;
  uint32_t d[17];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    u32x4 v;
    uintptr_t ga = a4 + 16 * g;
    if (ga + 16 <= end4) {
      v = ld128(p + 16 * g);
    } else {
      v.x = (ga + 0 < end4) ? ld32(p + 16 * g + 0) : 0u;
      v.y = (ga + 4 < end4) ? ld32(p + 16 * g + 4) : 0u;
      v.z = (ga + 8 < end4) ? ld32(p + 16 * g + 8) : 0u;
      v.w = (ga + 12 < end4) ? ld32(p + 16 * g + 12) : 0u;
    }
    d[4 * g + 0] = v.x;
    d[4 * g + 1] = v.y;
    d[4 * g + 2] = v.z;
    d[4 * g + 3] = v.w;
  }
  d[16] = (sh && a4 + 64 < end4) ? ld32(p + 64) : 0u;
#pragma unroll
  for (int j = 0; j < 16; ++j) wle[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
}

// One whole 64-byte block of message data whose 68-byte dword window
// [a4, a4 + 68) lies inside the message's dwords: unconditional loads (the
// software-pipelined main loop below issues them one block ahead).
struct ShaWin {
  uint32_t d[17];
};
__device__ __forceinline__ void issue_win(const unsigned char* base, uint64_t off, uint64_t p0, ShaWin& W) {
  const unsigned char* s = base + off + p0;  // from the kernel-argument pointer: global_load
  const unsigned char* p = s - ((uintptr_t)s & 3);
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    u32x4 v = ld128(p + 16 * g);
    W.d[4 * g + 0] = v.x;
    W.d[4 * g + 1] = v.y;
    W.d[4 * g + 2] = v.z;
    W.d[4 * g + 3] = v.w;
  }
  // the funnel dword only when the message is not dword aligned; otherwise a
  // dword inside the window (unused): a load past the window pulls in the
  // next line early, and it is fetched again when its own block comes
  W.d[16] = ld32(p + (s != p ? 64 : 60));
  asm volatile("" ::"v"(p));  // keep the address live: no load overwrites it (lsmck_crc32.hip keep_live)
}
// Funnel shift by sh bytes and big-endian byte swap in one v_perm_b32 per
// word: result byte k = byte (3 - k + sh) of {W.d[j+1]:W.d[j]} (selector
// 0x00010203 + sh * 0x01010101) -- instead of v_alignbyte + v_perm.
__device__ __forceinline__ void compress_win(uint32_t (&h)[8], const ShaWin& W, uint32_t sh) {
  const uint32_t sel = 0x00010203u + sh * 0x01010101u;
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_perm(W.d[j + 1], W.d[j], sel);
  sha256_compress(h, w);
}

// Two whole blocks per window (PAIR): 128 message bytes + the funnel dword,
// [a4, a4 + 132).  A lane then reads each 128-B line of its message at once; a
// 68-byte window per block reads half a line per block, and the other half is
// fetched again when the line has left L2 in between (FETCH_SIZE 1.6x the
// payload for config 2, profiles/pmc_traffic.json).  Costs 32 more VGPRs.
struct ShaWin2 {
  uint32_t d[33];
};
template <int ABL = 0>
__device__ __forceinline__ void issue_win2(const unsigned char* base, uint64_t off, uint64_t p0, ShaWin2& W) {
  // ABL 1 (option sha_pair 2, diagnostic): every window reloads the message's
  // first one (in bounds, cache resident after the first), so almost no HBM
  // traffic -- digests invalid
  const unsigned char* s = base + off + (ABL == 1 ? 0u : p0);
  const unsigned char* p = s - ((uintptr_t)s & 3);
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    u32x4 v = ld128(p + 16 * g);
    W.d[4 * g + 0] = v.x;
    W.d[4 * g + 1] = v.y;
    W.d[4 * g + 2] = v.z;
    W.d[4 * g + 3] = v.w;
  }
  W.d[32] = ld32(p + (s != p ? 128 : 124));  // as issue_win: no next-line dword when aligned
  asm volatile("" ::"v"(p));
}
__device__ __forceinline__ void compress_win2(uint32_t (&h)[8], const ShaWin2& W, uint32_t sh) {
  const uint32_t sel = 0x00010203u + sh * 0x01010101u;
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_perm(W.d[j + 1], W.d[j], sel);
  sha256_compress(h, w);
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_perm(W.d[j + 17], W.d[j + 16], sel);
  sha256_compress(h, w);
}

// Line-aligned windows (MODE 2, option sha_pair 3; A/B): a 132-byte window at
// a message's own offset straddles two 128-B lines, and a lane's next window
// starts in the second of them -- when that line has left L2 in between it is
// fetched twice (config 3: 1.37x the payload).  Here every load
// is one whole aligned line L_k = (A & ~127) + 128k, each line is loaded once,
// and pair p (message bytes [128p, 128p+128) + the funnel dword) is realigned
// through the lane's own 272-byte LDS row: L_p and L_{p+1} are written to it
// and the 33 dwords from byte (A & 127) & ~3 read back.  Lines stay in
// registers for two pairs (X = L_p, Y = L_{p+1}, Z = L_{p+2} in flight), so the
// loop is unrolled by three to rotate them without copies.
struct ShaLine {
  u32x4 v[8];
};
__device__ __forceinline__ void issue_line(const unsigned char* L0, uint64_t k, ShaLine& X) {
  const unsigned char* q = L0 + (k << 7);
#pragma unroll
  for (int g = 0; g < 8; ++g) X.v[g] = ld128(q + 16 * g);
  asm volatile("" ::"v"(q));
}
__device__ __forceinline__ void compress_lines(uint32_t (&h)[8], const ShaLine& X, const ShaLine& Y, uint32_t* row,
                                               uint32_t cd, uint32_t sh) {
#pragma unroll
  for (int g = 0; g < 8; ++g) *(u32x4*)(row + 4 * g) = X.v[g];
#pragma unroll
  for (int g = 0; g < 8; ++g) *(u32x4*)(row + 32 + 4 * g) = Y.v[g];
  ShaWin2 W;
  const uint32_t* r = row + cd;
#pragma unroll
  for (int j = 0; j < 33; ++j) W.d[j] = r[j];
  compress_win2(h, W, sh);
}

// Runs the compression over `len` bytes at base + off into h.  last: these are
// the message's final bytes -- pad and append the bit length `bits` of the
// whole message (the slice starts on a 64-byte boundary of the message).  Not
// last: len is a multiple of 64 and no padding is added (a slice of a message
// streamed through sha256_slices_kernel).
template <bool PAIR = false, int ABL = 0>
__device__ __forceinline__ void sha256_run(uint32_t (&h)[8], const unsigned char* base, uint64_t off, uint64_t len,
                                           bool last, uint64_t bits) {
  const uintptr_t A = (uintptr_t)(base + off);
  const uint64_t nb = last ? (len + 9 + 63) >> 6 : len >> 6;
  // Main loop: blocks entirely of message data whose dword window stays inside
  // the message (no masking, no padding), software pipelined: the next block's
  // loads are in flight while this one is compressed.  A lane-per-message
  // kernel otherwise waits a full memory round trip per block (measured 49% of
  // the VALU roof without).  Slots A/B alternate so that no
  // loaded register is copied; the loads past the lane's last main block
  // reload that block (in bounds, unused).
  const uint32_t sh = (uint32_t)(A & 3);
  const uintptr_t end4 = (A + len + 3) & ~(uintptr_t)3;
  const uintptr_t a40 = A & ~(uintptr_t)3;
  // blocks b with p0 + 64 <= len and a4(b) + 68 <= end4 (a4(b) = a40 + 64b)
  uint64_t nmain = len >> 6;
  if (len && end4 >= a40 + 68) {
    const uint64_t nsafe = (end4 - a40 - 68) / 64 + 1;
    nmain = nmain < nsafe ? nmain : nsafe;
  } else {
    nmain = 0;
  }
  uint64_t b = 0;
  if (PAIR && ABL == 2 && nmain >= 2) {
    const uint64_t npair = nmain >> 1;
    const unsigned char* L0 = (const unsigned char*)(A & ~(uintptr_t)127);
    const uint32_t c = (uint32_t)(A & 127u), cd = c >> 2;
    // the last line any pair needs (pair p uses L_p, and L_{p+1} unless the
    // message is line aligned); loads past it reload it (in bounds, unused)
    const uint64_t kmax = npair - 1 + (c != 0u);
    extern __shared__ __attribute__((aligned(16))) uint32_t sha_rows[];
    uint32_t* row = sha_rows + threadIdx.x * 68u;  // 272-B rows: lanes 4 banks apart
    ShaLine X, Y, Z;
    issue_line(L0, 0, X);
    issue_line(L0, kmax < 1 ? kmax : 1, Y);
    uint64_t p = 0;
    for (; p + 3 <= npair; p += 3) {
      issue_line(L0, kmax < p + 2 ? kmax : p + 2, Z);
      __builtin_amdgcn_sched_barrier(0);
      compress_lines(h, X, Y, row, cd, sh);
      issue_line(L0, kmax < p + 3 ? kmax : p + 3, X);
      __builtin_amdgcn_sched_barrier(0);
      compress_lines(h, Y, Z, row, cd, sh);
      issue_line(L0, kmax < p + 4 ? kmax : p + 4, Y);
      __builtin_amdgcn_sched_barrier(0);
      compress_lines(h, Z, X, row, cd, sh);
    }
    if (p < npair) {
      issue_line(L0, kmax < p + 2 ? kmax : p + 2, Z);
      compress_lines(h, X, Y, row, cd, sh);
      if (p + 1 < npair) compress_lines(h, Y, Z, row, cd, sh);
    }
    b = npair << 1;
  } else if (PAIR && nmain >= 2) {
    // pairs (2p, 2p+1), p < nmain/2: their 132-byte windows stay inside the
    // message's dwords; an odd last main block goes through the loader below
    const uint64_t npair = nmain >> 1;
    ShaWin2 WA, WB;
    issue_win2<ABL>(base, off, 0, WA);
    uint64_t p = 0;
    for (; p + 1 < npair; p += 2) {
      issue_win2<ABL>(base, off, (p + 1) << 7, WB);
      __builtin_amdgcn_sched_barrier(0);
      compress_win2(h, WA, sh);
      issue_win2<ABL>(base, off, (p + 2 < npair ? p + 2 : p + 1) << 7, WA);
      __builtin_amdgcn_sched_barrier(0);
      compress_win2(h, WB, sh);
    }
    if (p < npair) compress_win2(h, WA, sh);
    b = npair << 1;
  } else if (!PAIR && nmain) {
    ShaWin WA, WB;
    issue_win(base, off, 0, WA);
    for (; b + 1 < nmain; b += 2) {
      issue_win(base, off, (b + 1) << 6, WB);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the compression
      compress_win(h, WA, sh);
      issue_win(base, off, (b + 2 < nmain ? b + 2 : b + 1) << 6, WA);
      __builtin_amdgcn_sched_barrier(0);
      compress_win(h, WB, sh);
    }
    if (b < nmain) {  // odd count: the last main block is in WA
      compress_win(h, WA, sh);
      ++b;
    }
  }
  for (; b < nb; ++b) {
    const uint64_t p0 = b << 6;
    uint32_t w[16];
    load_block(A, len, p0, w);
    if (p0 + 64 > len) {
      // tail: mask bytes past the end, append 0x80, and the bit length in the final block
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        int64_t c = (int64_t)len - (int64_t)(p0 + 4 * t);  // data bytes in this word
        uint32_t mask = c >= 4 ? 0xFFFFFFFFu : (c <= 0 ? 0u : ((1u << (8 * c)) - 1u));
        uint32_t pad = (c >= 0 && c < 4) ? (0x80u << (8 * c)) : 0u;
        w[t] = (w[t] & mask) | pad;
      }
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = __builtin_bswap32(w[t]);
    if (last && b == nb - 1) {
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
    sha256_compress(h, w);
  }
}

__device__ __forceinline__ void sha256_iv(uint32_t (&h)[8]) {
  h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}

__device__ __forceinline__ void store_digest(unsigned char* out, const uint32_t (&h)[8]) {
  u32x4* o = (u32x4*)out;
  u32x4 o0 = {__builtin_bswap32(h[0]), __builtin_bswap32(h[1]), __builtin_bswap32(h[2]), __builtin_bswap32(h[3])};
  u32x4 o1 = {__builtin_bswap32(h[4]), __builtin_bswap32(h[5]), __builtin_bswap32(h[6]), __builtin_bswap32(h[7])};
  o[0] = o0;
  o[1] = o1;
}

template <bool PAIR, int ABL = 0>
__global__ __launch_bounds__(256) void sha256_kernel(ShaParams P) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.nmsg || (P.split && i >= *P.split)) return;  // (the short tail: sha256_short_kernel)
  uint64_t m = P.order ? P.order[i] : i;
  uint64_t off = P.off ? P.off[m] : m * P.stride;
  uint64_t len = P.len ? P.len[m] : P.flen;
  uint32_t h[8];
  sha256_iv(h);
  sha256_run<PAIR, ABL>(h, P.base, off, len, true, len << 3);
  store_digest(P.out + 32 * m, h);
}

// The short tail of a length-ordered batch (a few blocks per message): no
// load windows in flight, so few VGPRs (102: 4 waves per SIMD against the
// window kernel's 3) to cover each message's dependent round trips (order ->
// descriptor -> payload).  Config 3 (same box, ms): every message on the
// window kernel 65.3; messages of <= 3 / 6 / 12 / 16 / 32 blocks here 64.6 /
// 64.4 / 64.2 / 64.3 / 64.9 (default 12: "sha_short_blocks").  Compiled for 5
// waves (96 VGPRs, 4 spilled) it ran 64.4 against 64.2.
__global__ __launch_bounds__(256) void sha256_short_kernel(ShaParams P) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.nmsg || i < *P.split) return;
  const uint64_t m = P.order[i];
  const uint64_t off = P.off ? P.off[m] : m * P.stride;
  const uint64_t len = P.len[m];
  const uintptr_t A = (uintptr_t)(P.base + off);
  const uint64_t nb = (len + 9 + 63) >> 6;
  uint32_t h[8];
  sha256_iv(h);
  for (uint64_t b = 0; b < nb; ++b) {
    const uint64_t p0 = b << 6;
    uint32_t w[16];
    load_block(A, len, p0, w);
    if (p0 + 64 > len) {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        int64_t c = (int64_t)len - (int64_t)(p0 + 4 * t);
        uint32_t mask = c >= 4 ? 0xFFFFFFFFu : (c <= 0 ? 0u : ((1u << (8 * c)) - 1u));
        uint32_t pad = (c >= 0 && c < 4) ? (0x80u << (8 * c)) : 0u;
        w[t] = (w[t] & mask) | pad;
      }
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = __builtin_bswap32(w[t]);
    if (b == nb - 1) {
      w[14] = (uint32_t)(len >> 29);
      w[15] = (uint32_t)(len << 3);
    }
    sha256_compress(h, w);
  }
  store_digest(P.out + 32 * m, h);
}

// Many messages streamed in slices (whole-tree verify, lsmck_api.cpp): slice i
// continues message D[i].msg from its state slot (or from the IV on the
// message's first slice) over D[i].len bytes, then either stores the state
// back or, on the message's last slice, finishes it and writes its digest.
// One lane per slice, one 64-lane wave per workgroup: a round holds at most a
// few thousand slices, spread over as many CUs as possible.
__global__ __launch_bounds__(64) void sha256_slices_kernel(ShaSliceParams P) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.nslices) return;
  const ShaSlice d = P.slices[i];
  uint32_t h[8];
  if (d.flags & SHA_SLICE_FIRST) {
    sha256_iv(h);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = P.state[8u * d.slot + k];
  }
  const bool last = (d.flags & SHA_SLICE_LAST) != 0;
  sha256_run(h, P.base, d.off, d.len, last, d.total << 3);
  if (last) {
    store_digest(P.out + 32ull * d.msg, h);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) P.state[8u * d.slot + k] = h[k];
  }
}

// ---------------------------------------------------------------------------
// Synthetic input generator (bench / tests): byte b of the stream is byte
// (b % 8) of splitmix64(seed ^ (b / 8)); same definition as the oracle's
// oracle_gen_stream, so host and device see identical records without a copy.
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void gen_stream_kernel(unsigned char* dst, uint64_t seed, uint64_t byte_off,
                                                         uint64_t n) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  if ((byte_off & 7) == 0 && ((uintptr_t)dst & 15) == 0) {
    uint64_t n16 = n >> 4;
    uint64_t w0 = byte_off >> 3;
    for (uint64_t i = tid; i < n16; i += stride) {
      uint64_t a = splitmix64(seed ^ (w0 + 2 * i)), b = splitmix64(seed ^ (w0 + 2 * i + 1));
      u32x4 v = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
      *(u32x4*)(dst + 16 * i) = v;
    }
    for (uint64_t i = (n16 << 4) + tid; i < n; i += stride) {
      uint64_t bb = byte_off + i;
      dst[i] = (unsigned char)(splitmix64(seed ^ (bb >> 3)) >> (8 * (bb & 7)));
    }
  } else {
    for (uint64_t i = tid; i < n; i += stride) {
      uint64_t bb = byte_off + i;
      dst[i] = (unsigned char)(splitmix64(seed ^ (bb >> 3)) >> (8 * (bb & 7)));
    }
  }
}

}  // namespace lsmck

using namespace lsmck;

extern "C" int lsmk_launch_sha256(const ShaParams* P, hipStream_t st) {
  if (P->nmsg == 0) return 0;
  uint64_t blocks = (P->nmsg + 255) / 256;
  if (P->pair == 2)  // diagnostic: the pair kernel without its payload loads
    hipLaunchKernelGGL((sha256_kernel<true, 1>), dim3((unsigned)blocks), dim3(256), 0, st, *P);
  else if (P->pair == 3)  // line-aligned windows realigned through LDS rows (A/B)
    hipLaunchKernelGGL((sha256_kernel<true, 2>), dim3((unsigned)blocks), dim3(256), 256 * 272, st, *P);
  else if (P->pair)
    hipLaunchKernelGGL(sha256_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, *P);
  else
    hipLaunchKernelGGL(sha256_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, *P);
  if (P->split && P->order && P->len)  // the short tail of the order (its start on the device)
    hipLaunchKernelGGL(sha256_short_kernel, dim3((unsigned)blocks), dim3(256), 0, st, *P);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

extern "C" int lsmk_launch_sha256_slices(const ShaSliceParams* P, hipStream_t st) {
  if (P->nslices == 0) return 0;
  uint64_t blocks = (P->nslices + 63) / 64;
  hipLaunchKernelGGL(sha256_slices_kernel, dim3((unsigned)blocks), dim3(64), 0, st, *P);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

extern "C" int lsmk_launch_gen_stream(unsigned char* dst, uint64_t seed, uint64_t byte_off, uint64_t n,
                                       hipStream_t st) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(gen_stream_kernel, dim3(8192), dim3(256), 0, st, dst, seed, byte_off, n);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}
