// Pinned host memory for the tree verify's staging slots: what a fresh
// process pays for 1 GiB (round 5).  Three ways, each timed
// from the call to pages the DMA can use:
//   host_malloc   hipHostMalloc, then one write per page (the readers' first touch)
//   malloc_pop    hipHostMalloc, then madvise(MADV_POPULATE_WRITE) (the prewarm's form)
//   huge_register mmap, madvise(MADV_HUGEPAGE), MADV_POPULATE_WRITE, hipHostRegister
// and an H2D copy of the whole buffer from each, to check the rate it feeds.
//   hipcc -O2 --offload-arch=gfx950 tools/microbench_pin.hip -o /tmp/mb_pin && /tmp/mb_pin [GiB]
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double h2d_gbps(void* dev, const void* host, size_t bytes) {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s));  // warm
  CK(hipStreamSynchronize(s));
  const double t = now();
  for (int i = 0; i < 3; ++i) CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s));
  CK(hipStreamSynchronize(s));
  const double dt = now() - t;
  CK(hipStreamDestroy(s));
  return 3.0 * bytes / dt / 1e9;
}

int main(int argc, char** argv) {
  const size_t gib = argc > 1 ? (size_t)atoi(argv[1]) : 1;
  const size_t bytes = gib << 30;
  CK(hipSetDevice(0));
  void* dev = nullptr;
  CK(hipMalloc(&dev, bytes));
  CK(hipDeviceSynchronize());
  for (int round = 0; round < 2; ++round) {
    {  // hipHostMalloc + first touch
      const double t = now();
      void* p = nullptr;
      CK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
      const double ta = now() - t;
      for (size_t o = 0; o < bytes; o += 4096) ((volatile char*)p)[o] = 0;
      const double tt = now() - t;
      printf("round %d host_malloc   %zu GiB: alloc %.3f s, + touch %.3f s, H2D %.1f GB/s\n", round, gib, ta, tt,
             h2d_gbps(dev, p, bytes));
      const double tf = now();
      CK(hipHostFree(p));
      printf("round %d host_malloc   free %.3f s\n", round, now() - tf);
    }
    {  // hipHostMalloc + MADV_POPULATE_WRITE
      const double t = now();
      void* p = nullptr;
      CK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
      const int rc = madvise(p, bytes, 23 /* MADV_POPULATE_WRITE */);
      printf("round %d malloc_pop    %zu GiB: %.3f s (madvise rc %d), H2D %.1f GB/s\n", round, gib, now() - t, rc,
             h2d_gbps(dev, p, bytes));
      CK(hipHostFree(p));
    }
    {  // anonymous huge pages, populated, registered
      const double t = now();
      void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (p == MAP_FAILED) {
        perror("mmap");
        return 1;
      }
      const int rh = madvise(p, bytes, MADV_HUGEPAGE);
      const int rp = madvise(p, bytes, 23 /* MADV_POPULATE_WRITE */);
      const double tp = now() - t;
      CK(hipHostRegister(p, bytes, hipHostRegisterDefault));
      const double tr = now() - t;
      printf("round %d huge_register %zu GiB: populate %.3f s (hugepage rc %d, populate rc %d), + register %.3f s, "
             "H2D %.1f GB/s\n", round, gib, tp, rh, rp, tr, h2d_gbps(dev, p, bytes));
      const double tf = now();
      CK(hipHostUnregister(p));
      munmap(p, bytes);
      printf("round %d huge_register unregister + unmap %.3f s\n", round, now() - tf);
    }
  }
  CK(hipFree(dev));
  return 0;
}
