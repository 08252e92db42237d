// Dependent-load latency with many walkers at once: what one step of the WAL
// segment walk's header chain costs (round 5).  K walkers, one
// lane of every G (the walk's group), each follows a chain of `steps`
// dependent 16-byte loads through its own region of R bytes, `stride` apart
// (wrapping inside the region); the next address depends on the loaded value
// (the buffer is zero, so the chain is a fixed walk the compiler cannot
// lift).  Walker k's region starts at (k mod M) * R: M = K spreads the
// walkers over K * R bytes (the 97.8 GiB log, one 2 MiB segment each), a
// small M packs the same walks into M regions (fewer distinct pages, same
// per-walker access pattern, start offsets staggered by 4 KiB).
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_chase.hip -o /tmp/mb_chase && /tmp/mb_chase
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int G>
__global__ __launch_bounds__(256) void chase(const uint8_t* __restrict__ buf, uint32_t K, uint32_t M, uint64_t R,
                                             uint32_t stride, uint32_t steps, uint32_t* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, k = t / G;
  if (k >= K || t % G) return;
  const uint8_t* base = buf + (uint64_t)(k % M) * R;
  uint64_t p = ((uint64_t)(k / M) * 4096u) % R;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < steps; ++i) {
    const uint4 v = *(const uint4*)(base + p);
    acc ^= v.x ^ v.w;
    p = (p + stride + v.y) & (R - 16);  // (v.y is zero: the dependency, not the value; R a power of two)
  }
  out[k] = acc;
}

int main(int argc, char** argv) {
  const uint64_t R = 2ull << 20;
  const uint32_t stride = argc > 1 ? (uint32_t)atoi(argv[1]) : 1600, steps = argc > 2 ? (uint32_t)atoi(argv[2]) : 1300;
  const uint32_t Kmax = 50176;  // the 97.8 GiB log in 2 MiB segments: ~50k
  const uint64_t bytes = (uint64_t)Kmax * R;
  CK(hipSetDevice(0));
  uint8_t* buf = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 0, bytes));
  CK(hipMalloc(&out, 4ull * Kmax));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Case {
    uint32_t K, M;
  } cases[] = {{Kmax, Kmax}, {Kmax, 512}, {Kmax, 64}, {16384, 16384}, {16384, 512}, {4096, 4096}, {4096, 512},
               {1024, 1024}};
  printf("stride %u B, %u dependent 16-B loads per walker, region 2 MiB, one walker per 8 lanes\n", stride, steps);
  for (const Case& c : cases) {
    const uint32_t threads = c.K * 8;
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(chase<8>, dim3((threads + 255) / 256), dim3(256), 0, 0, buf, c.K, c.M, R, stride, steps, out);
      CK(hipGetLastError());
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep && ms < best) best = ms;  // (rep 0 warms)
    }
    printf("walkers %6u over %6u regions (%7.2f GiB): %.3f ms, %.0f ns per dependent load\n", c.K, c.M,
           (double)c.M * R / (1ull << 30), best, 1e6 * best / steps);
  }
  CK(hipFree(out));
  CK(hipFree(buf));
  return 0;
}
