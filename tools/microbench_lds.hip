// LDS table-lookup rate on gfx950 for the CRC main loop's access pattern:
// is the slicing-by-4 chain bound by LDS throughput, bank conflicts of the
// 32-way replicated tables, or the dependent chain's latency?
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/microbench_lds tools/microbench_lds.hip
//   tools/microbench_lds
//
// Every variant runs 256 workgroups x 1024 threads (one per CU, 16 waves, as
// the CRC kernels) and reports table lookups (lane reads) per clock per CU at
// 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef __attribute__((address_space(3))) const uint32_t lds_u32_t;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const u32x2 lds_u64_t;
__device__ __forceinline__ uint32_t L32(uint32_t a) { return *(lds_u32_t*)(size_t)a; }
__device__ __forceinline__ u32x2 L64(uint32_t a) { return *(lds_u64_t*)(size_t)a; }

// MODE 0: 32 replicas (lane & 31), 4 tables, dependent slicing-by-4 chains (CHAINS per lane)
// MODE 1: the same addresses, but the next address does not depend on the loaded value
// MODE 2: 64 replicas (lane), 2 tables (T0/T1, 128 KiB), dependent slicing-by-2 chains
// MODE 3: 64 replicas, independent addresses
// MODE 4: 32 replicas, 8-byte entries (ds_read_b64, 2 values per lane read), dependent
// MODE 5: MODE 0's tables, but the upper half-wave reads the other table of each
//         256-B row (T2 where the lower half reads T3, ...): 64 distinct banks per
//         read instead of two lanes per bank (x's bytes swapped in pairs there)
// MODE 6: MODE 5, independent addresses
template <int MODE, int CHAINS>
__global__ __launch_bounds__(1024) void k(int iters, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* s32 = (uint32_t*)smem;
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) s32[i] = i * 0x9E3779B9u ^ (i >> 7);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t s[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s[c] = threadIdx.x * 0x9E3779B9u + blockIdx.x + c * 0x1234567u;
  uint32_t w = 0x2545F491u * (threadIdx.x + 1);
  uint32_t acc = 0;
  const uint32_t lo = (lane & 31u) * 4u, hi = lo | 0x10000u;
  const uint32_t l64 = lane * 4u;  // 64 replicas: 256 B rows hold one entry of 64 replicas
  const uint32_t u = lane >> 5;
  const uint32_t B0 = hi + 128u * (1u - u), B1 = hi + 128u * u, B2 = lo + 128u * (1u - u), B3 = lo + 128u * u;
  const uint32_t swp = u ? 0x02030001u : 0x03020100u;
  for (int it = 0; it < iters; ++it) {
    w = w * 1664525u + 1013904223u;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      const uint32_t x = (MODE == 1 || MODE == 3 || MODE == 6) ? (w + c * 0x9E3779B9u) : (s[c] ^ (w >> c));
      if (MODE == 0 || MODE == 1) {
        const uint32_t a0 = __builtin_amdgcn_perm(x, hi, 0x0c020400u);
        const uint32_t a1 = __builtin_amdgcn_perm(x, hi, 0x0c020500u);
        const uint32_t a2 = __builtin_amdgcn_perm(x, lo, 0x0c0c0600u);
        const uint32_t a3 = __builtin_amdgcn_perm(x, lo, 0x0c0c0700u);
        const uint32_t v = L32(a0 + 128u) ^ L32(a1) ^ L32(a2 + 128u) ^ L32(a3);
        if (MODE == 0) s[c] = v; else acc ^= v;
      } else if (MODE == 2 || MODE == 3) {
        // two tables of 256 x 64 replicas: T_t[e] at 32768*t + 256*e + 4*lane (e < 128 per 32 KiB
        // half: index 8 bits -> row e, table t in the 64 KiB halves)
        const uint32_t a0 = ((x & 0xFFu) << 8) | l64;
        const uint32_t a1 = (((x >> 8) & 0xFFu) << 8) | l64 | 0x10000u;
        const uint32_t v = L32(a0) ^ L32(a1);
        if (MODE == 2) s[c] = (s[c] >> 16) ^ v; else acc ^= v;
      } else if (MODE == 5 || MODE == 6) {
        const uint32_t xs = __builtin_amdgcn_perm(x, x, swp);
        const uint32_t a0 = __builtin_amdgcn_perm(xs, B0, 0x0c020400u);
        const uint32_t a1 = __builtin_amdgcn_perm(xs, B1, 0x0c020500u);
        const uint32_t a2 = __builtin_amdgcn_perm(xs, B2, 0x0c0c0600u);
        const uint32_t a3 = __builtin_amdgcn_perm(xs, B3, 0x0c0c0700u);
        const uint32_t v = L32(a0) ^ L32(a1) ^ L32(a2) ^ L32(a3);
        if (MODE == 5) s[c] = v; else acc ^= v;
      } else if (MODE == 4) {
        // 8-byte entries, 32 replicas x 8 B = 256 B rows: byte e -> row e of 2 tables (64 KiB)
        const uint32_t r8 = (lane & 31u) * 8u;
        const u32x2 p0 = L64(((x & 0xFFu) << 8) | r8);
        const u32x2 p1 = L64((((x >> 8) & 0xFFu) << 8) | r8 | 0x10000u);
        s[c] = p0.x ^ p0.y ^ p1.x ^ p1.y ^ (s[c] >> 16);
      }
    }
  }
  uint32_t r = acc;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) r ^= s[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int MODE, int CHAINS>
static void run(const char* name, int ncu, uint32_t* out, double lookups_per_chain_iter) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int lds = 131072;
  CK(hipFuncSetAttribute((const void*)k<MODE, CHAINS>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const int iters = 20000;
  hipLaunchKernelGGL((k<MODE, CHAINS>), dim3(ncu), dim3(1024), lds, 0, 100, out);
  CK(hipGetLastError());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k<MODE, CHAINS>), dim3(ncu), dim3(1024), lds, 0, iters, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double lk = (double)ncu * 1024 * iters * CHAINS * lookups_per_chain_iter;
  printf("%-34s chains %d : %8.3f ms  %6.2f lookups/clk/CU  (%.1f B/clk/CU of CRC input at 1 lookup/B)\n", name, CHAINS,
         best, lk / (best * 1e-3) / ncu / 2.4e9, lk / (best * 1e-3) / ncu / 2.4e9);
}

int main() {
  int dev;
  CK(hipGetDevice(&dev));
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, dev));
  printf("device %s CUs %d\n", pr.gcnArchName, pr.multiProcessorCount);
  uint32_t* out;
  CK(hipMalloc(&out, (size_t)pr.multiProcessorCount * 1024 * 4));
  const int ncu = pr.multiProcessorCount;
  run<0, 2>("rep32 slicing-4, dependent", ncu, out, 4);
  run<0, 4>("rep32 slicing-4, dependent", ncu, out, 4);
  run<1, 2>("rep32 slicing-4, independent", ncu, out, 4);
  run<1, 4>("rep32 slicing-4, independent", ncu, out, 4);
  run<2, 2>("rep64 slicing-2, dependent", ncu, out, 2);
  run<2, 4>("rep64 slicing-2, dependent", ncu, out, 2);
  run<3, 4>("rep64 slicing-2, independent", ncu, out, 2);
  run<5, 2>("rep32 half-wave table swap, dep", ncu, out, 4);
  run<5, 4>("rep32 half-wave table swap, dep", ncu, out, 4);
  run<6, 2>("rep32 half-wave table swap, indep", ncu, out, 4);
  run<6, 4>("rep32 half-wave table swap, indep", ncu, out, 4);
  run<4, 2>("rep32 b64 pairs, dependent (2/read)", ncu, out, 4);
  run<4, 4>("rep32 b64 pairs, dependent (2/read)", ncu, out, 4);
  CK(hipFree(out));
  return 0;
}
