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

// Descriptor-path features, one at a time, on the order0/depth1 loop:
//  FEAT 1: segment start dword-aligned, not 16-B aligned (+4 B)
//  FEAT 2: + three gathers per tile and lane (off u64, len u32, tile_info u32)
//  FEAT 4: + a 9th dword load (D_32) per segment
//  FEAT 8: lanes with (lane % 8 == 0) read groups 0..3 from a 64-B zero buffer
//          (first segments of records: zero padding in front of the record)
template <int FEAT>
__global__ __launch_bounds__(1024) void k_desc_like(const unsigned char* __restrict__ base, uint32_t ntiles,
                                                    const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
                                                    const uint32_t* __restrict__ tinfo,
                                                    const unsigned char* __restrict__ zero, uint32_t* out) {
  extern __shared__ unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
  const uint32_t first = blockIdx.x * wpb + (threadIdx.x >> 6), step = gridDim.x * wpb;
  const uint32_t mis = (FEAT & 1) ? 4u : 0u;
  uint32_t acc = 0;
  struct S { u32x4 v[8]; uint32_t d32, g0, g1, g2; uint64_t o; };
  auto issue = [&](uint32_t t, S& x) {
    const unsigned char* p = base + ((size_t)t * 64 + lane) * 128 + mis;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned char* q = p + 16 * j;
      if ((FEAT & 8) && j < 4) q = ((lane & 7) == 0) ? zero + 16 * j : q;
      x.v[j] = *(const u32x4*)q;
    }
    if (FEAT & 4) x.d32 = *(const uint32_t*)(p + 128 - mis + (mis ? 0 : 0));
    if (FEAT & 16) asm volatile("" ::"v"(p));  // keep the address live (no load overwrites it)
    if (FEAT & 2) {
      uint32_t r = (t * 64 + lane) >> 3;
      x.o = off[r];
      x.g1 = len[r];
      x.g2 = tinfo[4 * t + (lane & 3)];
    }
  };
  auto eat = [&](const S& x) {
    u32x4 a = x.v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) a ^= x.v[j];
    uint32_t r = a.x ^ a.y ^ a.z ^ a.w;
    if (FEAT & 4) r ^= x.d32;
    if (FEAT & 2) r ^= (uint32_t)x.o ^ x.g1 ^ x.g2;
    return r;
  };
  uint32_t t = first;
  if (t >= ntiles) return;
  const uint32_t niter = (ntiles - t + step - 1) / step;
  S A, B;
  issue(t, A);
  for (uint32_t j = 2; j <= niter; j += 2) {
    issue(t + step, B);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= eat(A);
    uint32_t ta = t + 2 * step < ntiles ? t + 2 * step : t;
    issue(ta, A);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= eat(B);
    t += 2 * step;
  }
  if (niter & 1) acc ^= eat(A);
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
  // descriptor-path features (ntiles-1 tiles so +4 B misalignment stays in bounds)
  uint32_t nrec = ntiles * 8;
  uint64_t* off; uint32_t* len; uint32_t* tinfo; unsigned char* zero;
  CK(hipMalloc(&off, nrec * 8ull)); CK(hipMalloc(&len, nrec * 4ull)); CK(hipMalloc(&tinfo, ntiles * 16ull));
  CK(hipMalloc(&zero, 64)); CK(hipMemset(zero, 0, 64));
  CK(hipMemset(off, 0, nrec * 8ull)); CK(hipMemset(len, 0, nrec * 4ull)); CK(hipMemset(tinfo, 0, ntiles * 16ull));
  uint32_t nt1 = ntiles - 1;
  auto rund = [&](const char* name, const void* fn) {
    CK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L));
    void* args[] = {&buf, &nt1, &off, &len, &tinfo, &zero, &out};
    CK(hipLaunchKernel(fn, dim3(ncu), dim3(1024), args, L, 0));
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      CK(hipLaunchKernel(fn, dim3(ncu), dim3(1024), args, L, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("%-44s : %8.3f ms  %7.1f GB/s\n", name, best, (double)nt1 * 8192 / best / 1e6);
  };
  rund("desc-like: keep-live baseline (16-B aligned)", (const void*)k_desc_like<16>);
  rund("desc-like: keep-live dword aligned", (const void*)k_desc_like<17>);
  rund("desc-like: keep-live + gathers", (const void*)k_desc_like<18>);
  rund("desc-like: keep-live dword aligned + D32", (const void*)k_desc_like<21>);
  rund("desc-like: keep-live zero-buffer groups", (const void*)k_desc_like<24>);
  rund("desc-like: keep-live all", (const void*)k_desc_like<31>);
  rund("desc-like: baseline (16-B aligned)", (const void*)k_desc_like<0>);
  rund("desc-like: dword aligned", (const void*)k_desc_like<1>);
  rund("desc-like: + gathers", (const void*)k_desc_like<2>);
  rund("desc-like: dword aligned + gathers", (const void*)k_desc_like<3>);
  rund("desc-like: dword aligned + D32", (const void*)k_desc_like<5>);
  rund("desc-like: zero-buffer groups", (const void*)k_desc_like<8>);
  rund("desc-like: all", (const void*)k_desc_like<15>);
  return 0;
}
