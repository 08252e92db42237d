// Table files from the page cache to the GPU, three ways (the
// tree verify's readers): what a 100 GiB Db::load / compaction tick could
// save by not copying the files into pinned staging on host CPUs.
//
//   A  pread into a pinned slot, 128 KiB per file per call (the verify's
//      readers), then one H2D DMA of the slot
//   B  mmap (MAP_POPULATE) + hipHostRegister of the mapping, one H2D DMA
//      straight from the page-cache pages, hipHostUnregister + munmap
//   C  mmap (MAP_POPULATE) + memcpy into the pinned slot (no syscall per
//      128 KiB), then the DMA
//
// Files: <dir>/f<i>, made here (sizes cycling over 64 KiB .. 1 MiB, like the
// synthetic tree's upper levels).  T threads, each its own files and its own
// 32 MiB pinned slot and stream (a batch of files per DMA, as the verify's rounds).  Prints GB/s per mode and thread count.
//
//   hipcc -O2 -std=c++17 -o tools/microbench_pagecache tools/microbench_pagecache.cpp -lpthread
//   tools/microbench_pagecache /dev/shm/pcbench 4096 16
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/dev/shm/pcbench";
  const int nfiles = argc > 2 ? atoi(argv[2]) : 4096;
  const int maxT = argc > 3 ? atoi(argv[3]) : 16;
  mkdir(dir.c_str(), 0755);
  std::vector<size_t> sz(nfiles);
  size_t total = 0;
  {
    std::vector<char> buf(1 << 20);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = (char)(i * 131 + 7);
    for (int i = 0; i < nfiles; ++i) {
      sz[i] = (size_t)(64 << 10) << (i % 5);  // 64 KiB .. 1 MiB
      total += sz[i];
      const std::string p = dir + "/f" + std::to_string(i);
      int fd = open(p.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
      if (fd < 0 || write(fd, buf.data(), sz[i]) != (ssize_t)sz[i]) {
        perror("write");
        return 1;
      }
      close(fd);
    }
  }
  printf("files %d, %.2f GB in %s\n", nfiles, total / 1e9, dir.c_str());
  void* dev = nullptr;
  CK(hipMalloc(&dev, (size_t)64 << 20));
  for (int mode = 0; mode < 3; ++mode) {
    for (int T : {1, 4, 8, maxT}) {
      if (T > maxT) continue;
      std::atomic<int> next{0};
      std::atomic<long> reg_us{0};
      const double t0 = now();
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t]() {
          (void)t;
          CK(hipSetDevice(0));
          hipStream_t s;
          CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
          uint8_t* slot = nullptr;
          const size_t cap = (size_t)32 << 20;  // a batch of files per DMA round, as the verify's rounds
          CK(hipHostMalloc((void**)&slot, cap, hipHostMallocDefault));
          struct M {
            void* p;
            size_t n;
          };
          std::vector<M> maps;
          size_t used = 0;
          auto flush = [&]() {  // the batch's DMA(s), then its mappings released
            if (mode != 1 && used) CK(hipMemcpyAsync(dev, slot, used, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            for (auto& x : maps) {
              if (mode == 1) {
                const double u0 = now();
                CK(hipHostUnregister(x.p));
                reg_us += (long)((now() - u0) * 1e6);
              }
              munmap(x.p, x.n);
            }
            maps.clear();
            used = 0;
          };
          for (int i; (i = next.fetch_add(1)) < nfiles;) {
            const std::string p = dir + "/f" + std::to_string(i);
            int fd = open(p.c_str(), O_RDONLY);
            if (fd < 0) {
              perror("open");
              exit(1);
            }
            const size_t n = sz[i];
            if (used + n > cap) flush();
            if (mode == 0) {
              for (size_t o = 0; o < n; o += 128 << 10) {
                const size_t k = std::min<size_t>(128 << 10, n - o);
                if (pread(fd, slot + used + o, k, (off_t)o) != (ssize_t)k) {
                  perror("pread");
                  exit(1);
                }
              }
            } else {
              void* m = mmap(nullptr, n, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
              if (m == MAP_FAILED) {
                perror("mmap");
                exit(1);
              }
              maps.push_back({m, n});
              if (mode == 1) {
                const double r0 = now();
                hipError_t e = hipHostRegister(m, n, hipHostRegisterReadOnly);
                if (e != hipSuccess) e = hipHostRegister(m, n, hipHostRegisterDefault);
                reg_us += (long)((now() - r0) * 1e6);
                if (e != hipSuccess) {
                  fprintf(stderr, "hipHostRegister: %s\n", hipGetErrorString(e));
                  exit(2);
                }
                CK(hipMemcpyAsync((uint8_t*)dev + used, m, n, hipMemcpyHostToDevice, s));
              } else {
                memcpy(slot + used, m, n);
              }
            }
            used += n;
            close(fd);
          }
          flush();
          CK(hipHostFree(slot));
          CK(hipStreamDestroy(s));
        });
      for (auto& x : th) x.join();
      const double dt = now() - t0;
      printf("%s T=%2d: %.3f s, %.1f GB/s%s\n",
             mode == 0 ? "A pread -> pinned slot -> DMA     " : mode == 1 ? "B mmap + hipHostRegister -> DMA   "
                                                                          : "C mmap + memcpy -> pinned -> DMA  ",
             T, dt, total / dt / 1e9,
             mode == 1 ? (" (register+unregister " + std::to_string(reg_us.load() / 1000) + " thread-ms)").c_str()
                       : "");
      fflush(stdout);
    }
  }
  for (int i = 0; i < nfiles; ++i) unlink((dir + "/f" + std::to_string(i)).c_str());
  rmdir(dir.c_str());
  return 0;
}
