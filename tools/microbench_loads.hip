// Load-loop structure microbenchmark for the CRC kernel's constraints:
// one 1024-thread workgroup per CU (LDS 144 KiB reserved), lane-contiguous
// 128-B segments, 64-segment tiles per wave.  Which tile order / prefetch
// depth / workgroup shape reaches the HBM streaming peak?
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench_loads.hip -o tools/microbench_loads
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(uint64_t* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) p[i] = i * 0x9E3779B97F4A7C15ull;
}

struct Seg { u32x4 v[8]; };
__device__ __forceinline__ void issue(const unsigned char* base, uint32_t tile, uint32_t lane, Seg& S) {
  const u32x4* q = (const u32x4*)(base + ((size_t)tile * 64 + lane) * 128);
#pragma unroll
  for (int j = 0; j < 8; ++j) S.v[j] = q[j];
}
__device__ __forceinline__ uint32_t eat(const Seg& S) {
  u32x4 a = S.v[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) a ^= S.v[j];
  return a.x ^ a.y ^ a.z ^ a.w;
}

// ORDER 0: tile = wave + k*nwaves   (current kernel)
// ORDER 1: block-contiguous: block b owns tiles [b*T/nb, (b+1)*T/nb), its waves interleave inside
// ORDER 2: XCD-contiguous: tiles split in 8 ranges by blockIdx%8, then wave-strided inside
// DEPTH: tiles in flight per wave beyond the one being consumed (1 or 2)
template <int ORDER, int DEPTH>
__global__ __launch_bounds__(1024) void k_tiles(const unsigned char* __restrict__ base, uint32_t ntiles, uint32_t* out) {
  extern __shared__ unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63, wib = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  uint32_t first, step, end;
  if (ORDER == 0) {
    first = blockIdx.x * wpb + wib; step = gridDim.x * wpb; end = ntiles;
  } else if (ORDER == 1) {
    uint32_t per = (ntiles + gridDim.x - 1) / gridDim.x;
    first = blockIdx.x * per + wib; step = wpb; end = min(ntiles, (blockIdx.x + 1) * per);
  } else {
    uint32_t x = blockIdx.x & 7, bx = blockIdx.x >> 3, nbx = gridDim.x >> 3;
    uint32_t per = (ntiles + 7) / 8;
    first = x * per + bx * wpb + wib; step = nbx * wpb; end = min(ntiles, (x + 1) * per);
  }
  uint32_t acc = 0;
  if (DEPTH == 1) {
    Seg A, B;
    uint32_t t = first;
    if (t >= end) return;
    issue(base, t, lane, A);
    for (;;) {
      uint32_t tb = t + step < end ? t + step : t;
      issue(base, tb, lane, B);
      __builtin_amdgcn_sched_barrier(0);
      acc ^= eat(A);
      t += step;
      if (t >= end) break;
      uint32_t ta = t + step < end ? t + step : t;
      issue(base, ta, lane, A);
      __builtin_amdgcn_sched_barrier(0);
      acc ^= eat(B);
      t += step;
      if (t >= end) break;
    }
  } else {
    Seg A, B, C;
    uint32_t t = first;
    if (t >= end) return;
    issue(base, t, lane, A);
    issue(base, t + step < end ? t + step : t, lane, B);
    for (;;) {
      uint32_t tc = t + 2 * step < end ? t + 2 * step : t;
      issue(base, tc, lane, C);
      __builtin_amdgcn_sched_barrier(0);
      acc ^= eat(A);
      t += step;
      if (t >= end) break;
      uint32_t ta = t + 2 * step < end ? t + 2 * step : t;
      issue(base, ta, lane, A);
      __builtin_amdgcn_sched_barrier(0);
      acc ^= eat(B);
      t += step;
      if (t >= end) break;
      uint32_t tb = t + 2 * step < end ? t + 2 * step : t;
      issue(base, tb, lane, B);
      __builtin_amdgcn_sched_barrier(0);
      acc ^= eat(C);
      t += step;
      if (t >= end) break;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (acc == 0x12345678u) smem[threadIdx.x] = 1;
}

int main(int argc, char** argv) {
  size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 32ull) << 30;
  uint32_t ntiles = (uint32_t)(bytes / 8192);
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
  int ncu = pr.multiProcessorCount;
  unsigned char* buf; CK(hipMalloc(&buf, bytes));
  uint32_t* out; CK(hipMalloc(&out, 64 << 20));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)buf, bytes / 8);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, const void* fn, int blocks, int threads, size_t lds) {
    CK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    void* args[] = {&buf, &ntiles, &out};
    CK(hipLaunchKernel(fn, dim3(blocks), dim3(threads), args, lds, 0));
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      CK(hipLaunchKernel(fn, dim3(blocks), dim3(threads), args, lds, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("%-44s blocks=%5d thr=%4d lds=%6zu : %8.3f ms  %7.1f GB/s\n", name, blocks, threads, lds, best, bytes / best / 1e6);
  };
  size_t L = 147456;
  run("order0 depth1 (current)", (const void*)k_tiles<0, 1>, ncu, 1024, L);
  run("order1 depth1 (block-contiguous)", (const void*)k_tiles<1, 1>, ncu, 1024, L);
  run("order2 depth1 (xcd-contiguous)", (const void*)k_tiles<2, 1>, ncu, 1024, L);
  run("order0 depth2", (const void*)k_tiles<0, 2>, ncu, 1024, L);
  run("order1 depth2", (const void*)k_tiles<1, 2>, ncu, 1024, L);
  run("order0 depth1, no LDS, 2 WG/CU of 1024", (const void*)k_tiles<0, 1>, 2 * ncu, 1024, 0);
  run("order0 depth1, no LDS, 4 WG/CU of 512", (const void*)k_tiles<0, 1>, 4 * ncu, 512, 0);
  run("order0 depth1, 512 thr, 70KB LDS (2/CU)", (const void*)k_tiles<0, 1>, 2 * ncu, 512, 70000);
  run("order0 depth2, no LDS, 2 WG/CU", (const void*)k_tiles<0, 2>, 2 * ncu, 1024, 0);
  return 0;
}
