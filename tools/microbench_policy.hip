// Cache-policy microbenchmark for the CRC kernels' load shape: one 1024-thread
// workgroup per CU (144 KiB LDS reserved, like the checksum kernels), each lane
// streams one contiguous 128-B segment per tile (8 x dwordx4), 64-segment tiles
// per wave, one tile in flight while the previous one is consumed.
// Which load instruction / cache-policy bits stream fastest on gfx950?
//   POL 0: plain global_load_dwordx4
//   POL 1: __builtin_nontemporal_load (nt)
//   POL 6: global_load, saddr form (SGPR tile base + 32-bit VGPR offset)
//   POL 7 / 8: plain / saddr global_load, issued in ascending address order
//   POL 2..5: raw buffer load, aux = 0 / 1 (sc0) / 2 (nt) / 3 (sc0|nt) [aux passed as POL-2]
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench_policy.hip -o tools/microbench_policy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// MODE 0: i * golden (low entropy); MODE 1: splitmix64(i) (random bytes, like gen_stream)
__global__ void k_fill(uint64_t* p, size_t n, int mode) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    if (mode) {
      z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
      z ^= z >> 27; z *= 0x94D049BB133111EBull;
      z ^= z >> 31;
    }
    p[i] = z;
  }
}

struct Seg { u32x4 v[8]; };

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7FFFFFFF, 0x00020000);
}

template <int POL>
__device__ __forceinline__ void issue(const unsigned char* base, uint32_t tile, uint32_t lane, Seg& S) {
  if (POL == 0) {
    const u32x4* q = (const u32x4*)(base + ((size_t)tile * 64 + lane) * 128);
#pragma unroll
    for (int j = 0; j < 8; ++j) S.v[j] = q[j];
  } else if (POL == 1) {
    const u32x4* q = (const u32x4*)(base + ((size_t)tile * 64 + lane) * 128);
#pragma unroll
    for (int j = 0; j < 8; ++j) S.v[j] = __builtin_nontemporal_load(q + j);
  } else if (POL == 6) {
    // global_load saddr form: uniform tile base in SGPRs + 32-bit lane offset
    const unsigned char* tb = base + (size_t)__builtin_amdgcn_readfirstlane(tile) * 8192;
    const uint32_t o = lane * 128u;
#pragma unroll
    for (int j = 0; j < 8; ++j) S.v[j] = *(const u32x4*)(tb + o + 16 * j);
  } else if (POL == 7 || POL == 8) {
    // global_load in ascending address order (sched_group_barrier pins the order)
    const u32x4* q = (const u32x4*)(base + ((size_t)tile * 64 + lane) * 128);
    const unsigned char* tb = base + (size_t)__builtin_amdgcn_readfirstlane(tile) * 8192;
    const uint32_t o = lane * 128u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      S.v[j] = POL == 7 ? q[j] : *(const u32x4*)(tb + o + 16 * j);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    // buffer resource per 8 KiB tile (base + tile*8192), voffset = lane*128
    const unsigned char* tb = base + (size_t)tile * 8192;
    __amdgpu_buffer_rsrc_t r = make_rsrc(tb);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 128 + 16 * j, 0, POL - 2);
      S.v[j] = *(u32x4*)&v;
    }
  }
}
__device__ __forceinline__ uint32_t eat(const Seg& S) {
  u32x4 a = S.v[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) a ^= S.v[j];
  return a.x ^ a.y ^ a.z ^ a.w;
}

template <int POL>
__global__ __launch_bounds__(1024) void k_tiles(const unsigned char* __restrict__ base, uint32_t ntiles, uint32_t* out) {
  extern __shared__ unsigned char smem[];
  const uint32_t lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
  const uint32_t first = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  const uint32_t step = gridDim.x * wpb;
  uint32_t acc = 0;
  uint32_t t = first;
  if (t >= ntiles) return;
  const uint32_t niter = (ntiles - t + step - 1) / step;
  Seg A, B;
  issue<POL>(base, t, lane, A);
  for (uint32_t j = 2; j <= niter; j += 2) {
    issue<POL>(base, t + step, lane, B);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= eat(A);
    uint32_t ta = t + 2 * step < ntiles ? t + 2 * step : t;
    issue<POL>(base, ta, lane, A);
    __builtin_amdgcn_sched_barrier(0);
    acc ^= eat(B);
    t += 2 * step;
  }
  if (niter & 1) acc ^= eat(A);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (acc == 0x12345678u) smem[threadIdx.x] = 1;
}

// Bisection of the checksum kernel's loads-only ablation (crc_ablate 3, buffer
// loads) against k_tiles<2>: FEAT bit 0 = 128 KiB LDS table build from global
// memory + barrier before the loop; bit 1 = the kernel's per-lane address map
// (record = g / nsegr with a runtime nsegr, E = rec*stride + flen - 128k,
// tile base = (64t / nsegr) * stride); bit 2 = the in-loop magic-value store.
struct MapP { uint32_t nsegr, flen; uint64_t stride; const uint32_t* tab; };
template <int FEAT>
__global__ __launch_bounds__(1024) void k_bisect(const unsigned char* __restrict__ base, uint32_t ntiles, uint32_t* out,
                                                 MapP M) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (FEAT & 1) {
    uint32_t* s32 = (uint32_t*)smem;
    for (uint32_t i = threadIdx.x; i < 32768u; i += blockDim.x) s32[i] = M.tab[(i >> 6) & 1023u];
    __syncthreads();
  }
  const uint32_t lane = threadIdx.x & 63;
  uint32_t first = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  uint32_t step = (gridDim.x * blockDim.x) >> 6;
  const uint32_t total = ntiles * 64u;
  uint32_t tile0 = 0;
  if (FEAT & 32) {  // XCD-contiguous: workgroup b runs on XCD b % 8 (round-robin placement)
    const uint32_t x = blockIdx.x & 7u, wpb = blockDim.x >> 6;
    const uint32_t per = (ntiles + 7u) / 8u;
    tile0 = x * per;
    const uint32_t tend = min(ntiles, tile0 + per);
    first = tile0 + __builtin_amdgcn_readfirstlane((blockIdx.x >> 3) * wpb + (threadIdx.x >> 6));
    step = (gridDim.x >> 3) * wpb;
    ntiles = tend;
  }
  auto issue = [&](uint32_t t, Seg& S) {
    uint64_t tb;
    uint32_t vo;
    if (FEAT & 2) {
      uint32_t g = t * 64u + lane;
      uint32_t gg = g < total ? g : total - 1u;
      uint32_t rec = gg / M.nsegr, q = gg - rec * M.nsegr, k = M.nsegr - 1u - q;
      uint64_t E = (uint64_t)rec * M.stride + M.flen - 128ull * k;
      tb = (uint64_t)((t * 64u) / M.nsegr) * M.stride;
      vo = (uint32_t)(E - 128 - tb);
    } else {
      tb = (size_t)t * 8192;
      vo = lane * 128u;
    }
    __amdgpu_buffer_rsrc_t r = make_rsrc(base + tb);
    if (FEAT & 16) asm volatile("" : "+v"(vo));  // hide the base: offsets fold to offset:16..112
    if (FEAT & 64) {  // eight offsets computed first, then eight back-to-back loads, no immediates
      uint32_t o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = vo + 16 * j;
      asm volatile("" : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]), "+v"(o[4]), "+v"(o[5]), "+v"(o[6]), "+v"(o[7]));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(r, o[j], 0, 0);
        S.v[j] = *(u32x4*)&v;
      }
      if (FEAT & 128)  // keep the offset VGPRs live past the loads: no load overwrites an address register
        asm volatile("" :: "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "v"(o[4]), "v"(o[5]), "v"(o[6]), "v"(o[7]));
      return;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t o = vo + 16 * j;
      if (FEAT & 8) asm volatile("" : "+v"(o));  // one VGPR offset per load, no immediate offset
      auto v = __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0);
      S.v[j] = *(u32x4*)&v;
    }
    if (FEAT & 128) asm volatile("" :: "v"(vo));
  };
  uint32_t acc = 0;
  uint32_t t = first;
  if (t >= ntiles) return;
  const uint32_t niter = (ntiles - t + step - 1) / step;
  Seg A, B;
  auto consume = [&](const Seg& S) {
    uint32_t v = eat(S);
    if (FEAT & 4) {
      if (v == 0x9E3779B1u) out[0] = v;
    } else {
      acc ^= v;
    }
  };
  issue(t, A);
  for (uint32_t j = 2; j <= niter; j += 2) {
    issue(t + step, B);
    __builtin_amdgcn_sched_barrier(0);
    consume(A);
    uint32_t ta = t + 2 * step < ntiles ? t + 2 * step : t;
    issue(ta, A);
    __builtin_amdgcn_sched_barrier(0);
    consume(B);
    t += 2 * step;
  }
  if (niter & 1) consume(A);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (acc == 0x12345678u) smem[threadIdx.x] = 1;
}

int main(int argc, char** argv) {
  size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 32ull) << 30;
  int reps = argc > 2 ? atoi(argv[2]) : 3;
  uint32_t ntiles = (uint32_t)(bytes / 8192);
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
  int ncu = pr.multiProcessorCount;
  printf("device %s CUs %d\n", pr.gcnArchName, ncu);
  unsigned char* buf; CK(hipMalloc(&buf, bytes));
  uint32_t* out; CK(hipMalloc(&out, 64 << 20));
  int fill_mode = getenv("MB_RANDOM") ? 1 : 0;
  printf("fill: %s\n", fill_mode ? "splitmix64 (random)" : "i * golden");
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)buf, bytes / 8, fill_mode);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* names[] = {"global_load plain", "global_load nt (builtin)", "buffer_load aux0", "buffer_load aux1 (sc0)",
                         "buffer_load aux2 (nt)", "buffer_load aux3 (sc0|nt)", "global_load saddr", "global_load ascending", "global_load saddr ascending"};
  const void* fns[] = {(const void*)k_tiles<0>, (const void*)k_tiles<1>, (const void*)k_tiles<2>,
                       (const void*)k_tiles<3>, (const void*)k_tiles<4>, (const void*)k_tiles<5>, (const void*)k_tiles<6>,
                       (const void*)k_tiles<7>, (const void*)k_tiles<8>};
  size_t L = 147456;
  float best[9];
  for (int i = 0; i < 9; ++i) best[i] = 1e30f;
  for (int r = 0; r < reps; ++r) {  // interleaved rounds
    for (int i = 0; i < 9; ++i) {
      if (i == 1 || i == 4 || i == 5) continue;  // nt: 2.3-2.7 TB/s (measured), skipped
      CK(hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize, (int)L));
      void* args[] = {&buf, &ntiles, &out};
      CK(hipEventRecord(e0));
      CK(hipLaunchKernel(fns[i], dim3(ncu), dim3(1024), args, L, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < best[i]) best[i] = ms;
      if (getenv("MB_TRACE")) printf("round %d %-30s %8.3f ms\n", r, names[i], ms);
    }
  }
  for (int i = 0; i < 9; ++i)
    if (best[i] < 1e29f) printf("%-30s : %8.3f ms  %7.1f GB/s\n", names[i], best[i], bytes / best[i] / 1e6);
  // bisection of the kernel's loads-only ablation
  uint32_t* tab; CK(hipMalloc(&tab, 4096 * 4)); CK(hipMemset(tab, 0, 4096 * 4));
  MapP M{32u, 4096u, 4096ull, tab};
  const void* bf[] = {(const void*)k_bisect<0>, (const void*)k_bisect<16 | 128>, (const void*)k_bisect<2 | 128>,
                      (const void*)k_bisect<66 | 128>, (const void*)k_bisect<80 | 128>};
  const char* bn[] = {"bisect: none", "bisect: imm offsets, addr kept", "bisect: +address map, addr kept",
                      "bisect: +map, 8 offsets, kept", "bisect: 8 offsets then 8 loads, kept"};
  size_t LB = 156704;
  float bb[5] = {1e30f, 1e30f, 1e30f, 1e30f, 1e30f};
  for (int r = 0; r < reps; ++r) {
    for (int i = 0; i < 5; ++i) {
      CK(hipFuncSetAttribute(bf[i], hipFuncAttributeMaxDynamicSharedMemorySize, (int)LB));
      void* args[] = {&buf, &ntiles, &out, &M};
      CK(hipEventRecord(e0));
      CK(hipLaunchKernel(bf[i], dim3(ncu), dim3(1024), args, LB, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0 && ms < bb[i]) bb[i] = ms;
    }
  }
  for (int i = 0; i < 5; ++i) printf("%-30s : %8.3f ms  %7.1f GB/s\n", bn[i], bb[i], bytes / bb[i] / 1e6);
  return 0;
}
