// Load-alignment microbenchmark for the descriptor CRC kernel's load shape:
// each lane streams one 128-B window per 64-lane tile (8 KiB per tile, one
// tile in flight while the previous one is consumed), one 1024-thread
// workgroup per CU with 144 KiB of LDS reserved, like the checksum kernels.
// Question: what does a window that is dword- but not 16-byte aligned cost?
// (config 3's records are packed at arbitrary byte offsets, so the descriptor
// kernel's per-segment windows start at floor4(E-128).)
//   FORM 0: buffer_load x8 at lane*128 + SH (SH runtime: 0 = aligned)
//   FORM 1: global_load x8 at the same addresses
//   FORM 2: buffer_load x9 at floor16(lane*128 + SH): 16-byte aligned loads
//           covering the shifted window (144 B per lane)
//   FORM 3: FORM 0 plus the kernel's extra D_32 dword load at window end
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench_misalign.hip -o tools/microbench_misalign
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(uint64_t* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) p[i] = i * 0x9E3779B97F4A7C15ull;
}

struct Seg { u32x4 v[9]; uint32_t x; };

template <typename T>
__device__ __forceinline__ void keep_live(const T& x) { asm volatile("" ::"v"(x)); }

template <int FORM>
__device__ __forceinline__ void issue(const unsigned char* base, uint64_t bytes, uint32_t tile, uint32_t lane,
                                      uint32_t sh, Seg& S) {
  const uint64_t tb = (uint64_t)tile * 8192;
  const uint64_t left = bytes - tb;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(base + tb), (short)0, (int)(left < 0x7FFFFFFFull ? left : 0x7FFFFFFFull), 0x00020000);
  if (FORM == 0 || FORM == 3) {
    const uint32_t vo = lane * 128u + sh;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16u * j, 0, 0);
      S.v[j] = *(u32x4*)&v;
    }
    S.v[8] = 0;
    S.x = FORM == 3 ? __builtin_amdgcn_raw_buffer_load_b32(r, vo + 128u, 0, 0) : 0u;
    keep_live(vo);
  } else if (FORM == 1) {
    const unsigned char* p = base + tb + lane * 128u + sh;
#pragma unroll
    for (int j = 0; j < 8; ++j) S.v[j] = *(const u32x4*)(p + 16 * j);
    S.v[8] = 0;
    S.x = 0;
    keep_live(p);
  } else {
    const uint32_t vo = (lane * 128u + sh) & ~15u;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16u * j, 0, 0);
      S.v[j] = *(u32x4*)&v;
    }
    S.x = 0;
    keep_live(vo);
  }
}
__device__ __forceinline__ uint32_t eat(const Seg& S) {
  u32x4 a = S.v[0];
#pragma unroll
  for (int j = 1; j < 9; ++j) a ^= S.v[j];
  return a.x ^ a.y ^ a.z ^ a.w ^ S.x;
}

template <int FORM>
__global__ __launch_bounds__(1024) void k_tiles(const unsigned char* __restrict__ base, uint64_t bytes, uint32_t ntiles,
                                                uint32_t sh, uint32_t* out) {
  extern __shared__ unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
  const uint32_t first = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  const uint32_t step = gridDim.x * wpb;
  uint32_t acc = 0;
  uint32_t t = first;
  if (t >= ntiles) return;
  const uint32_t niter = (ntiles - t + step - 1) / step;
  Seg A, B;
  issue<FORM>(base, bytes, t, lane, sh, A);
  for (uint32_t j = 2; j <= niter; j += 2) {
    issue<FORM>(base, bytes, t + step, lane, sh, B);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= eat(A);
    uint32_t ta = t + 2 * step < ntiles ? t + 2 * step : t;
    issue<FORM>(base, bytes, ta, lane, sh, A);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= eat(B);
    t += 2 * step;
  }
  if (niter & 1) acc ^= eat(A);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (acc == 0x12345678u) smem[threadIdx.x] = 1;
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 32ull) << 30;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  const uint32_t ntiles = (uint32_t)(bytes / 8192) - 1;  // the shifted windows stay inside the buffer
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int ncu = pr.multiProcessorCount;
  printf("device %s CUs %d, %zu GiB\n", pr.gcnArchName, ncu, bytes >> 30);
  unsigned char* buf;
  CK(hipMalloc(&buf, bytes));
  uint32_t* out;
  CK(hipMalloc(&out, 64 << 20));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)buf, bytes / 8);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const void* fns[] = {(const void*)k_tiles<0>, (const void*)k_tiles<1>, (const void*)k_tiles<2>,
                       (const void*)k_tiles<3>};
  const char* names[] = {"buffer x8 at +sh", "global x8 at +sh", "buffer x9 aligned (144 B)", "buffer x8 +sh, +D_32"};
  const uint32_t shs[] = {0, 4, 8, 12, 64};
  const size_t L = 147456;
  for (int f = 0; f < 4; ++f) CK(hipFuncSetAttribute(fns[f], hipFuncAttributeMaxDynamicSharedMemorySize, (int)L));
  for (uint32_t sh : shs) {
    for (int f = 0; f < 4; ++f) {
      float best = 1e30f;
      for (int r = 0; r < reps; ++r) {
        uint32_t s = sh;
        uint64_t b = bytes;
        uint32_t nt = ntiles;
        void* args[] = {&buf, &b, &nt, &s, &out};
        CK(hipEventRecord(e0));
        CK(hipLaunchKernel(fns[f], dim3(ncu), dim3(1024), args, L, 0));
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && ms < best) best = ms;
      }
      const double useful = (double)ntiles * 8192.0;
      printf("sh %3u  %-28s : %8.3f ms  %7.1f GB/s (window bytes)\n", sh, names[f], best, useful / best / 1e6);
      fflush(stdout);
    }
  }
  return 0;
}
