// Tile-order microbenchmark for a "walking" CRC kernel (one wave walks a run
// of consecutive tiles, carrying record state from tile to tile) against the
// strided order of the committed kernels (tile t -> wave t mod nwaves).
// Same load shape as crc32_wring_kernel: one 1024-thread workgroup per CU,
// 150 KiB LDS reserved, each lane streams one 128-B segment per 64-segment
// tile (8 x buffer_load_dwordx4 at a loop-invariant lane offset, address
// register kept live), one tile in flight while the previous one is consumed.
//   ORDER 0: strided            t = wave + i*nwaves            (committed kernels)
//   ORDER 1: contiguous ranges  wave w takes tiles [w*per, (w+1)*per)
//   ORDER 2: blocks of S tiles, block b -> wave b mod nwaves (S = 16)
//   ORDER 3: blocks of S tiles claimed from an atomic counter (S = 16)
//   ORDER 4: blocks of S tiles claimed from an atomic counter (S = 64)
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench_walk.hip -o tools/microbench_walk
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(uint64_t* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

struct Seg { u32x4 v[8]; };

__device__ __forceinline__ void issue(const unsigned char* base, uint32_t t, uint32_t vo, Seg& S) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(base + (size_t)t * 8192),
                                                               (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16u * j, 0, 0);
    S.v[j] = *(u32x4*)&v;
  }
  asm volatile("" ::"v"(vo));
}
__device__ __forceinline__ uint32_t eat(const Seg& S) {
  u32x4 a = S.v[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) a ^= S.v[j];
  return a.x ^ a.y ^ a.z ^ a.w;
}

// run tiles [t0, t0 + cnt*stride) step `stride`, two slots
__device__ __forceinline__ uint32_t run(const unsigned char* base, uint32_t t0, uint32_t cnt, uint32_t stride,
                                        uint32_t vo) {
  if (cnt == 0) return 0;
  uint32_t acc = 0, t = t0;
  Seg A, B;
  issue(base, t, vo, A);
  for (uint32_t j = 2; j <= cnt; j += 2) {
    issue(base, t + stride, vo, B);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= eat(A);
    const uint32_t ta = (j + 1 <= cnt) ? t + 2 * stride : t;
    issue(base, ta, vo, A);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= eat(B);
    t += 2 * stride;
  }
  if (cnt & 1) acc ^= eat(A);
  return acc;
}

template <int ORDER>
__global__ __launch_bounds__(1024) void k_order(const unsigned char* __restrict__ base, uint32_t ntiles, uint32_t* out,
                                               uint32_t* counter) {
  extern __shared__ unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
  const uint32_t vo = lane * 128u;
  uint32_t acc = 0;
  if (ORDER == 0) {
    if (wave < ntiles) acc = run(base, wave, (ntiles - wave + nw - 1) / nw, nw, vo);
  } else if (ORDER == 1) {
    const uint32_t per = (ntiles + nw - 1) / nw, t0 = wave * per;
    if (t0 < ntiles) acc = run(base, t0, min(per, ntiles - t0), 1, vo);
  } else if (ORDER == 2) {
    constexpr uint32_t S = 16;
    const uint32_t nb = (ntiles + S - 1) / S;
    for (uint32_t b = wave; b < nb; b += nw) acc ^= run(base, b * S, min(S, ntiles - b * S), 1, vo);
  } else {
    constexpr uint32_t S = ORDER == 3 ? 16 : 64;
    const uint32_t nb = (ntiles + S - 1) / S;
    for (;;) {
      uint32_t b = 0;
      if (lane == 0) b = atomicAdd(counter, 1u);
      b = __builtin_amdgcn_readfirstlane(b);
      if (b >= nb) break;
      acc ^= run(base, b * S, min(S, ntiles - b * S), 1, vo);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (acc == 0x12345678u) smem[threadIdx.x] = 1;
}

int main(int argc, char** argv) {
  size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 64ull) << 30;
  int reps = argc > 2 ? atoi(argv[2]) : 4;
  uint32_t ntiles = (uint32_t)(bytes / 8192);
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
  int ncu = pr.multiProcessorCount;
  printf("device %s CUs %d, %zu GiB\n", pr.gcnArchName, ncu, bytes >> 30);
  unsigned char* buf; CK(hipMalloc(&buf, bytes));
  uint32_t* out; CK(hipMalloc(&out, 64 << 20));
  uint32_t* counter; CK(hipMalloc(&counter, 64));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)buf, bytes / 8);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* names[] = {"strided (committed)", "contiguous per wave", "16-tile blocks round robin",
                         "16-tile blocks, atomic claim", "64-tile blocks, atomic claim"};
  const void* fns[] = {(const void*)k_order<0>, (const void*)k_order<1>, (const void*)k_order<2>,
                       (const void*)k_order<3>, (const void*)k_order<4>};
  size_t L = 153600;
  float best[5], sum[5];
  for (int i = 0; i < 5; ++i) best[i] = 1e30f, sum[i] = 0;
  for (int r = 0; r < reps; ++r) {
    for (int i = 0; i < 5; ++i) {
      CK(hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize, (int)L));
      CK(hipMemset(counter, 0, 64));
      void* args[] = {&buf, &ntiles, &out, &counter};
      CK(hipEventRecord(e0));
      CK(hipLaunchKernel(fns[i], dim3(ncu), dim3(1024), args, L, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) { if (ms < best[i]) best[i] = ms; sum[i] += ms; }
    }
  }
  for (int i = 0; i < 5; ++i)
    printf("%-32s : best %8.3f ms  mean %8.3f ms  %7.1f GB/s\n", names[i], best[i], sum[i] / (reps - 1),
           bytes / best[i] / 1e6);
  return 0;
}
