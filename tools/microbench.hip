// Design-space microbenchmarks for the CRC-32 kernel on gfx950 (MI355X).
// Not part of the product: answers three questions before the kernel is written.
//   1. streaming-read peak (coalesced 16 B/lane) -> the "measured" HBM denominator
//   2. lane-contiguous segment loads (each lane reads S contiguous bytes)
//   3. LDS table-lookup rate for slicing-by-4 with bank-replicated vs plain tables,
//      and ds_bpermute (register-resident 64-entry tables) as the alternative.
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench.hip -o tools/microbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(uint64_t* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

// 1. coalesced stream read: each lane 16 B per load, 4 loads in flight
__global__ __launch_bounds__(256) void k_stream(const u32x4* __restrict__ p, size_t n16, uint32_t* out) {
  size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  u32x4 acc = {0, 0, 0, 0};
  size_t i = tid;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a ^ b ^ c ^ d;
  }
  for (; i < n16; i += stride) acc ^= p[i];
  out[tid] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// 2. lane-contiguous segments of S bytes: lane g handles segments g, g+G, ...
template <int S, int MIS>
__global__ __launch_bounds__(256) void k_laneseg(const unsigned char* __restrict__ base, size_t nseg, uint32_t* out) {
  size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  u32x4 acc = {0, 0, 0, 0};
  constexpr int NL = S / 16 + (MIS ? 1 : 0);
  for (size_t s = tid; s < nseg; s += stride) {
    const u32x4* q = (const u32x4*)(base + s * S + MIS);
#pragma unroll
    for (int j = 0; j < NL; ++j) acc ^= q[j];
  }
  out[tid] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// 3a. slicing-by-4 chain, tables replicated 32x so lane l only touches bank l%32.
//     entry e of table t for replica r at byte 256*e + 4*r + 128*(t&1) + 65536*(t>>1)
//     -> address = v_perm(x, lane4|(t>>1)<<16, sel) : one VALU per lookup.
__global__ __launch_bounds__(1024) void k_lds_rep(const uint32_t* __restrict__ tab, int iters, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* s32 = (uint32_t*)smem;
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) {
    int r = i & 31, t = (i >> 5) & 1, e = (i >> 6) & 255, h = i >> 14;
    s32[i] = tab[(h * 2 + t) * 256 + e] ^ r * 0;
  }
  __syncthreads();
  unsigned lane4 = (threadIdx.x & 31) * 4;
  unsigned lo = lane4, hi = lane4 | 0x10000u;
  uint32_t s0 = threadIdx.x * 0x9E3779B9u + blockIdx.x, s1 = s0 ^ 0x12345678u;
  uint32_t w = 0x2545F491u * (threadIdx.x + 1);
  for (int it = 0; it < iters; ++it) {
    w = w * 1664525u + 1013904223u;
    uint32_t x0 = s0 ^ w, x1 = s1 ^ (w >> 3);
    uint32_t a0 = __builtin_amdgcn_perm(x0, lo, 0x0c0c0400u);
    uint32_t a1 = __builtin_amdgcn_perm(x0, lo, 0x0c0c0500u);
    uint32_t a2 = __builtin_amdgcn_perm(x0, hi, 0x0c020600u);
    uint32_t a3 = __builtin_amdgcn_perm(x0, hi, 0x0c020700u);
    uint32_t b0 = __builtin_amdgcn_perm(x1, lo, 0x0c0c0400u);
    uint32_t b1 = __builtin_amdgcn_perm(x1, lo, 0x0c0c0500u);
    uint32_t b2 = __builtin_amdgcn_perm(x1, hi, 0x0c020600u);
    uint32_t b3 = __builtin_amdgcn_perm(x1, hi, 0x0c020700u);
    s0 = *(uint32_t*)(smem + a0) ^ *(uint32_t*)(smem + a1 + 128) ^ *(uint32_t*)(smem + a2) ^ *(uint32_t*)(smem + a3 + 128);
    s1 = *(uint32_t*)(smem + b0) ^ *(uint32_t*)(smem + b1 + 128) ^ *(uint32_t*)(smem + b2) ^ *(uint32_t*)(smem + b3 + 128);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1;
}

// 3b. plain 4 x 1 KiB tables (bank conflicts on random indices)
__global__ __launch_bounds__(1024) void k_lds_plain(const uint32_t* __restrict__ tab, int iters, uint32_t* out) {
  __shared__ uint32_t T[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) T[i] = tab[i];
  __syncthreads();
  uint32_t s0 = threadIdx.x * 0x9E3779B9u + blockIdx.x, s1 = s0 ^ 0x12345678u;
  uint32_t w = 0x2545F491u * (threadIdx.x + 1);
  for (int it = 0; it < iters; ++it) {
    w = w * 1664525u + 1013904223u;
    uint32_t x0 = s0 ^ w, x1 = s1 ^ (w >> 3);
    s0 = T[768 + (x0 & 255)] ^ T[512 + ((x0 >> 8) & 255)] ^ T[256 + ((x0 >> 16) & 255)] ^ T[x0 >> 24];
    s1 = T[768 + (x1 & 255)] ^ T[512 + ((x1 >> 8) & 255)] ^ T[256 + ((x1 >> 16) & 255)] ^ T[x1 >> 24];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1;
}

// 3c. ds_bpermute with 6-bit fields: 6 lookups per 32-bit word, tables in VGPRs
__global__ __launch_bounds__(1024) void k_bperm(const uint32_t* __restrict__ tab, int iters, uint32_t* out) {
  int lane = threadIdx.x & 63;
  uint32_t t0 = tab[lane], t1 = tab[64 + lane], t2 = tab[128 + lane], t3 = tab[192 + lane], t4 = tab[256 + lane], t5 = tab[320 + lane];
  uint32_t s0 = threadIdx.x * 0x9E3779B9u + blockIdx.x, s1 = s0 ^ 0x12345678u;
  uint32_t w = 0x2545F491u * (threadIdx.x + 1);
  for (int it = 0; it < iters; ++it) {
    w = w * 1664525u + 1013904223u;
    uint32_t x0 = s0 ^ w, x1 = s1 ^ (w >> 3);
    s0 = __builtin_amdgcn_ds_bpermute((x0 << 2) & 0xfc, t0) ^ __builtin_amdgcn_ds_bpermute((x0 >> 4) & 0xfc, t1) ^
         __builtin_amdgcn_ds_bpermute((x0 >> 10) & 0xfc, t2) ^ __builtin_amdgcn_ds_bpermute((x0 >> 16) & 0xfc, t3) ^
         __builtin_amdgcn_ds_bpermute((x0 >> 22) & 0xfc, t4) ^ __builtin_amdgcn_ds_bpermute((x0 >> 28) << 2, t5);
    s1 = __builtin_amdgcn_ds_bpermute((x1 << 2) & 0xfc, t0) ^ __builtin_amdgcn_ds_bpermute((x1 >> 4) & 0xfc, t1) ^
         __builtin_amdgcn_ds_bpermute((x1 >> 10) & 0xfc, t2) ^ __builtin_amdgcn_ds_bpermute((x1 >> 16) & 0xfc, t3) ^
         __builtin_amdgcn_ds_bpermute((x1 >> 22) & 0xfc, t4) ^ __builtin_amdgcn_ds_bpermute((x1 >> 28) << 2, t5);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1;
}

static float time_ms(hipEvent_t a, hipEvent_t b) { float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }

int main(int argc, char** argv) {
  size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 8ull) << 30;
  int dev; CK(hipGetDevice(&dev));
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, dev));
  printf("device %s CUs %d clock %d kHz\n", pr.gcnArchName, pr.multiProcessorCount, pr.clockRate);
  unsigned char* buf; CK(hipMalloc(&buf, bytes + 4096));
  uint32_t* out; CK(hipMalloc(&out, 64ull << 20));
  uint32_t* tab; CK(hipMalloc(&tab, 4096 * 4));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)buf, (bytes + 4096) / 8);
  hipLaunchKernelGGL(k_fill, dim3(16), dim3(256), 0, 0, (uint64_t*)tab, 2048);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int REP = 10;
  for (int grid : {2048, 4096, 8192}) {
    hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, (const u32x4*)buf, bytes / 16, out);
    CK(hipEventRecord(e0));
    for (int r = 0; r < REP; ++r) hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, (const u32x4*)buf, bytes / 16, out);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    double ms = time_ms(e0, e1) / REP;
    printf("stream_read grid=%d : %.3f ms  %.1f GB/s\n", grid, ms, bytes / ms / 1e6);
  }
#define LANESEG(S, MIS)                                                                         \
  {                                                                                             \
    size_t nseg = bytes / S - 1;                                                                \
    for (int grid : {2048, 8192}) {                                                             \
      hipLaunchKernelGGL((k_laneseg<S, MIS>), dim3(grid), dim3(256), 0, 0, buf, nseg, out);     \
      CK(hipEventRecord(e0));                                                                   \
      for (int r = 0; r < REP; ++r)                                                             \
        hipLaunchKernelGGL((k_laneseg<S, MIS>), dim3(grid), dim3(256), 0, 0, buf, nseg, out);   \
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                                      \
      double ms = time_ms(e0, e1) / REP;                                                        \
      printf("laneseg S=%d mis=%d grid=%d : %.3f ms  %.1f GB/s (useful)\n", S, MIS, grid, ms,  \
             nseg * (double)S / ms / 1e6);                                                      \
    }                                                                                           \
  }
  LANESEG(64, 0) LANESEG(128, 0) LANESEG(256, 0) LANESEG(128, 4) LANESEG(128, 1) LANESEG(64, 4)
  int ncu = pr.multiProcessorCount;
  int iters = 20000;
  {
    CK(hipFuncSetAttribute((const void*)k_lds_rep, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    hipLaunchKernelGGL(k_lds_rep, dim3(ncu), dim3(1024), 131072, 0, tab, 100, out);
    CK(hipGetLastError());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_lds_rep, dim3(ncu), dim3(1024), 131072, 0, tab, iters, out);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    double ms = time_ms(e0, e1);
    double lk = (double)ncu * 1024 * iters * 8;
    printf("lds_rep32 : %.3f ms  %.2f Glookups/s  %.2f lookups/clk/CU @2.4GHz\n", ms, lk / ms / 1e6, lk / (ms * 1e-3) / ncu / 2.4e9);
  }
  {
    hipLaunchKernelGGL(k_lds_plain, dim3(ncu), dim3(1024), 0, 0, tab, 100, out);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_lds_plain, dim3(ncu), dim3(1024), 0, 0, tab, iters, out);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    double ms = time_ms(e0, e1);
    double lk = (double)ncu * 1024 * iters * 8;
    printf("lds_plain : %.3f ms  %.2f Glookups/s  %.2f lookups/clk/CU @2.4GHz\n", ms, lk / ms / 1e6, lk / (ms * 1e-3) / ncu / 2.4e9);
  }
  {
    hipLaunchKernelGGL(k_bperm, dim3(ncu), dim3(1024), 0, 0, tab, 100, out);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_bperm, dim3(ncu), dim3(1024), 0, 0, tab, iters, out);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    double ms = time_ms(e0, e1);
    double lk = (double)ncu * 1024 * iters * 12;
    printf("bpermute6 : %.3f ms  %.2f Glookups/s  %.2f lookups/clk/CU @2.4GHz (=%.2f B/clk/CU at 1.5 lookups/B)\n", ms,
           lk / ms / 1e6, lk / (ms * 1e-3) / ncu / 2.4e9, lk / (ms * 1e-3) / ncu / 2.4e9 / 1.5);
  }
  CK(hipFree(buf)); CK(hipFree(out)); CK(hipFree(tab));
  return 0;
}
