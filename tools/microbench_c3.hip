// Load-shape ceiling of config 3 (2^26 packed Zipf records, 64 B-64 KiB):
// what do the descriptor kernels' per-segment windows stream at when the
// window addresses cost nothing to find?
//   MODE 0: each lane loads its segment's 128-B window at a precomputed
//           address (u64 per segment, read one tile ahead): the exact windows
//           crc32_walk_kernel reads (128-B segments aligned to each record's
//           end, dword floor, the first one reaching into the previous record)
//   MODE 1: the same payload bytes as aligned 128-B chunks of the packed
//           stream (no address array): the fixed ring kernel's shape
//   MODE 2: MODE 0's address reads only
// Strided tiles, one tile of loads in flight while the previous one is XOR-
// folded, one 1024-thread workgroup per CU with 144 KiB LDS reserved, as in
// the checksum kernels.  Lengths come from a file (u32 per record, written by
// lsm_storage_engine_amd.device.gen_zipf_lengths) so the shape is bench.py's.
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench_c3.hip -o tools/microbench_c3
// Run:   tools/microbench_c3 lens.u32 [reps]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(uint64_t* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) p[i] = i * 0x9E3779B97F4A7C15ull;
}

struct Win { u32x4 v[8]; };

template <typename T>
__device__ __forceinline__ void keep_live(const T& x) { asm volatile("" ::"v"(x)); }

template <int MODE>
__device__ __forceinline__ void issue(const unsigned char* img, const uint64_t* addr, uint64_t nseg, uint64_t t,
                                      uint32_t lane, Win& W) {
  const uint64_t s = t * 64 + lane;
  if (MODE == 1) {
    const unsigned char* p = img + (s < nseg ? s : nseg - 1) * 128;
#pragma unroll
    for (int j = 0; j < 8; ++j) W.v[j] = *(const u32x4*)(p + 16 * j);
    keep_live(p);
  } else {
    const uint64_t a = addr[s < nseg ? s : nseg - 1];
    if (MODE == 0) {
      const unsigned char* p = img + a;
#pragma unroll
      for (int j = 0; j < 8; ++j) W.v[j] = *(const u32x4*)(p + 16 * j);
      keep_live(p);
    } else {
      W.v[0] = u32x4{(uint32_t)a, (uint32_t)(a >> 32), 0u, 0u};
#pragma unroll
      for (int j = 1; j < 8; ++j) W.v[j] = 0;
    }
  }
}

__device__ __forceinline__ uint32_t fold(const Win& W) {
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) x ^= W.v[j].x ^ W.v[j].y ^ W.v[j].z ^ W.v[j].w;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_stream(const unsigned char* img, const uint64_t* addr, uint64_t nseg,
                                                 uint32_t* out) {
  extern __shared__ uint32_t lds[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  const uint64_t ntile = (nseg + 63) / 64;
  uint32_t acc = 0;
  if (threadIdx.x == 0) lds[0] = 0;
  uint64_t t = wave;
  if (t < ntile) {
    Win A, B;
    issue<MODE>(img, addr, nseg, t, lane, A);
    for (;;) {
      const uint64_t t1 = t + nw;
      const bool more = t1 < ntile;
      issue<MODE>(img, addr, nseg, more ? t1 : t, lane, B);
      __builtin_amdgcn_sched_barrier(0);
      acc ^= fold(A);
      if (!more) break;
      t = t1;
      const uint64_t t2 = t + nw;
      const bool more2 = t2 < ntile;
      issue<MODE>(img, addr, nseg, more2 ? t2 : t, lane, A);
      __builtin_amdgcn_sched_barrier(0);
      acc ^= fold(B);
      if (!more2) break;
      t = t2;
    }
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc + lds[0];
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s lens.u32 [reps]\n", argv[0]);
    return 2;
  }
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  const size_t n = (size_t)ftell(f) / 4;
  fseek(f, 0, SEEK_SET);
  std::vector<uint32_t> len(n);
  if (fread(len.data(), 4, n, f) != n) return 2;
  fclose(f);
  uint64_t bytes = 0, nseg = 0;
  for (size_t i = 0; i < n; ++i) {
    bytes += len[i];
    nseg += len[i] ? (len[i] + 127) / 128 : 1;
  }
  std::vector<uint64_t> addr(nseg);
  uint64_t O = 0, s = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t E = O + len[i];
    const uint64_t k = len[i] ? (len[i] + 127) / 128 : 1;
    for (uint64_t q = 0; q < k; ++q) {  // record order: first (short) segment first
      const int64_t w = (int64_t)E - 128 * (int64_t)(k - q);
      addr[s++] = (uint64_t)(w < 0 ? 0 : w) & ~3ull;
    }
    O = E;
  }
  const uint64_t alloc = ((bytes > nseg * 128 ? bytes : nseg * 128) + 4096 + 4095) & ~4095ull;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  unsigned char* img;
  uint64_t* daddr;
  uint32_t* out;
  CK(hipMalloc(&img, alloc));
  CK(hipMalloc(&daddr, nseg * 8));
  CK(hipMalloc(&out, (size_t)cus * 1024 * 4));
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (uint64_t*)img, alloc / 8);
  CK(hipMemcpy(daddr, addr.data(), nseg * 8, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  printf("records %zu  payload %.3f GB  segments %llu (%.2f per record)  address array %.3f GB\n", n, bytes / 1e9,
         (unsigned long long)nseg, (double)nseg / n, nseg * 8 / 1e9);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t lds = 144 * 1024;
  CK(hipFuncSetAttribute((const void*)k_stream<0>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void*)k_stream<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void*)k_stream<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const char* names[3] = {"segment windows at precomputed addresses", "aligned 128-B chunks of the packed stream",
                          "address array only"};
  const uint64_t chunks = (bytes + 127) / 128;
  for (int mode = 0; mode < 3; ++mode) {
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps + 1; ++r) {
      CK(hipEventRecord(e0, 0));
      if (mode == 0) hipLaunchKernelGGL(k_stream<0>, dim3(cus), dim3(1024), lds, 0, img, daddr, nseg, out);
      if (mode == 1) hipLaunchKernelGGL(k_stream<1>, dim3(cus), dim3(1024), lds, 0, img, daddr, chunks, out);
      if (mode == 2) hipLaunchKernelGGL(k_stream<2>, dim3(cus), dim3(1024), lds, 0, img, daddr, nseg, out);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r == 0) continue;  // cold
      best = ms < best ? ms : best;
      sum += ms;
    }
    printf("%-44s: best %8.3f ms  mean %8.3f ms  %7.1f GB/s of payload\n", names[mode], best, sum / reps,
           bytes / 1e6 / best);
    fflush(stdout);
  }
  return 0;
}
