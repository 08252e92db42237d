// Device -> pinned-host read-back beside an HBM-streaming kernel: which
// transfer leaves the compute units to the stream?  (the WAL
// replay's records to the host.)
//   A  hipMemcpyAsync D2H on a second stream (what the replay does now)
//   B  hsa_amd_memory_async_copy, dst agent = the CPU (SDMA)
//   C  hsa_amd_memory_async_copy_on_engine, forced SDMA engine
//   D  a kernel on 8 workgroups storing straight into the pinned array
//   E, F  A and B into a hipHostMallocNumaUser array (the library's pinned
//         memory on a multi-node host: stage_numa, lsmck_api.cpp host_malloc_near)
// Each alone, then each beside the streaming kernel (a 64 GiB xor read).
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench_d2h.hip -lhsa-runtime64 -o tools/microbench_d2h
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <sys/syscall.h>
#include <unistd.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)
#define HK(x) do { hsa_status_t s = (x); if (s != HSA_STATUS_SUCCESS) { const char* m = ""; hsa_status_string(s, &m); \
  fprintf(stderr, "HSA error %d (%s) at %s:%d\n", (int)s, m, __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(uint64_t* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) p[i] = i * 0x9E3779B97F4A7C15ull;
}

// the stand-in for the CRC pass: every CU streams its share of the buffer
__global__ __launch_bounds__(1024) void k_stream(const u32x4* __restrict__ p, size_t n16, uint32_t* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  u32x4 a = {0, 0, 0, 0};
  for (; i + 3 * s < n16; i += 4 * s) {
    u32x4 x0 = p[i], x1 = p[i + s], x2 = p[i + 2 * s], x3 = p[i + 3 * s];
    a ^= x0 ^ x1 ^ x2 ^ x3;
  }
  for (; i < n16; i += s) a ^= p[i];
  const uint32_t v = a.x ^ a.y ^ a.z ^ a.w;
  if (v == 0x12345678u) out[0] = v;
}

// D: the records stored straight into host memory by a few workgroups
__global__ __launch_bounds__(256) void k_store_host(const u32x4* __restrict__ src, u32x4* dst, size_t n16) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n16; i += s) dst[i] = src[i];
}

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t find_agents(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
  if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
  return HSA_STATUS_SUCCESS;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t rec_bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : 1024) << 20;  // MiB
  const size_t big = (size_t)(argc > 2 ? strtoull(argv[2], 0, 0) : 64) << 30;    // GiB streamed
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  CK(hipSetDevice(0));
  uint8_t *d_big, *d_rec, *h_rec;
  uint32_t* d_out;
  CK(hipMalloc(&d_big, big));
  CK(hipMalloc(&d_rec, rec_bytes));
  CK(hipMalloc(&d_out, 64));
  uint8_t *h_def, *h_numa;
  CK(hipHostMalloc(&h_def, rec_bytes, hipHostMallocDefault));
  {
    int node = 0;
    char bus[64] = {0};
    CK(hipDeviceGetPCIBusId(bus, sizeof bus, 0));
    for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
    FILE* f = fopen((std::string("/sys/bus/pci/devices/") + bus + "/numa_node").c_str(), "r");
    if (f) { if (fscanf(f, "%d", &node) != 1) node = 0; fclose(f); }
    if (node < 0) node = 0;
    unsigned long mask[16] = {0};
    mask[node / 64] |= 1ul << (node % 64);
    const bool set = syscall(SYS_set_mempolicy, 1, mask, 16 * 64) == 0;
    CK(hipHostMalloc(&h_numa, rec_bytes, set ? hipHostMallocNumaUser : hipHostMallocDefault));
    syscall(SYS_set_mempolicy, 0, nullptr, 0);
    printf("device node %d, NumaUser array %s\n", node, set ? "on it" : "(policy failed: default)");
  }
  memset(h_def, 0, rec_bytes);
  memset(h_numa, 0, rec_bytes);
  h_rec = h_def;
  k_fill<<<4096, 256>>>((uint64_t*)d_big, big / 8);
  k_fill<<<4096, 256>>>((uint64_t*)d_rec, rec_bytes / 8);
  CK(hipDeviceSynchronize());
  HK(hsa_init());
  HK(hsa_iterate_agents(find_agents, nullptr));
  uint32_t emask = 0, pmask = 0;
  hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &emask);
  hsa_amd_memory_get_preferred_copy_engine(g_cpu, g_gpu, &pmask);
  printf("engines to split over:"); for (int i = 0; i < 16; ++i) if ((emask >> i) & 1) printf(" %d", i); printf("\n");
  printf("gpu agent %lx cpu agent %lx sdma engines avail 0x%x preferred 0x%x HSA_ENABLE_SDMA=%s\n",
         (unsigned long)g_gpu.handle, (unsigned long)g_cpu.handle, emask, pmask,
         getenv("HSA_ENABLE_SDMA") ? getenv("HSA_ENABLE_SDMA") : "(unset)");
  hsa_signal_t sig;
  HK(hsa_signal_create(1, 0, nullptr, &sig));
  hipStream_t s1, s2, sx[4];
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  for (auto& q : sx) CK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
  hipEvent_t xe[4];
  for (auto& ev : xe) CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  hipEvent_t e0, e1, c0, c1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&c0)); CK(hipEventCreate(&c1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));

  // engines to split over: the preferred ones first, then the other available ones
  uint32_t engs[16];
  int neng = 0;
  for (int pass = 0; pass < 2; ++pass)
    for (int b = 0; b < 16; ++b) {
      const uint32_t m = 1u << b;
      if ((pass == 0 ? (pmask & m) : ((emask & m) && !(pmask & m)))) engs[neng++] = m;
    }
  hipEvent_t dep;
  CK(hipEventCreateWithFlags(&dep, hipEventDisableTiming));
  auto hsa_split = [&](int parts, bool h2d = false) {
    hsa_signal_store_relaxed(sig, parts);
    const size_t per = (rec_bytes / parts + 4095) & ~(size_t)4095;
    for (int i = 0; i < parts; ++i) {
      const size_t o = per * i, c = o >= rec_bytes ? 0 : std::min(per, rec_bytes - o);
      if (h2d)
        HK(hsa_amd_memory_async_copy_on_engine(d_rec + o, g_gpu, h_rec + o, g_cpu, c, 0, nullptr, sig,
                                               (hsa_amd_sdma_engine_id_t)engs[i % neng], true));
      else
        HK(hsa_amd_memory_async_copy_on_engine(h_rec + o, g_cpu, d_rec + o, g_gpu, c, 0, nullptr, sig,
                                               (hsa_amd_sdma_engine_id_t)engs[i % neng], true));
    }
  };
  auto hip_split = [&](int parts, hipMemcpyKind kind) {  // one hipMemcpyAsync per stream, joined on s2
    const size_t per = (rec_bytes / parts + 4095) & ~(size_t)4095;
    CK(hipEventRecord(c0, s2));
    for (int i = 0; i < parts; ++i) {
      CK(hipStreamWaitEvent(sx[i], c0, 0));
      const size_t o = per * i, c = std::min(per, rec_bytes - o);
      if (kind == hipMemcpyDeviceToHost) CK(hipMemcpyAsync(h_rec + o, d_rec + o, c, kind, sx[i]));
      else CK(hipMemcpyAsync(d_rec + o, h_rec + o, c, kind, sx[i]));
      CK(hipEventRecord(xe[i], sx[i]));
      CK(hipStreamWaitEvent(s2, xe[i], 0));
    }
    CK(hipEventRecord(c1, s2));
  };
  // variants: 0 hip D2H, 1 hsa auto, 2/3 hsa split over 2/4 engines, 4 kernel stores,
  // 5 hip D2H behind a cross-stream event, 6 hip D2H NumaUser, 7 hsa split 2 NumaUser
  auto is_hsa = [](int how) { return how == 1 || how == 2 || how == 3 || how == 7 || how == 11; };
  auto copy = [&](int how) {
    h_rec = how >= 6 ? h_numa : h_def;
    if (how == 0 || how == 6) {
      CK(hipEventRecord(c0, s2));
      CK(hipMemcpyAsync(h_rec, d_rec, rec_bytes, hipMemcpyDeviceToHost, s2));
      CK(hipEventRecord(c1, s2));
    } else if (how == 5) {
      CK(hipStreamWaitEvent(s2, dep, 0));
      CK(hipEventRecord(c0, s2));
      CK(hipMemcpyAsync(h_rec, d_rec, rec_bytes, hipMemcpyDeviceToHost, s2));
      CK(hipEventRecord(c1, s2));
    } else if (how == 1) {
      hsa_signal_store_relaxed(sig, 1);
      HK(hsa_amd_memory_async_copy(h_rec, g_cpu, d_rec, g_gpu, rec_bytes, 0, nullptr, sig));
    } else if (how == 2 || how == 7) {
      hsa_split(2);
    } else if (how == 3) {
      hsa_split(4);
    } else if (how == 8) {
      hip_split(4, hipMemcpyDeviceToHost);
    } else if (how == 9) {
      CK(hipEventRecord(c0, s2));
      CK(hipMemcpyAsync(d_rec, h_rec, rec_bytes, hipMemcpyHostToDevice, s2));
      CK(hipEventRecord(c1, s2));
    } else if (how == 10) {
      hip_split(4, hipMemcpyHostToDevice);
    } else if (how == 11) {
      hsa_split(4, true);
    } else {
      CK(hipEventRecord(c0, s2));
      k_store_host<<<8, 256, 0, s2>>>((const u32x4*)d_rec, (u32x4*)h_rec, rec_bytes / 16);
      CK(hipEventRecord(c1, s2));
    }
  };
  auto wait_copy = [&](int how) -> double {  // ms of the copy (events), -1 for HSA copies (host clock)
    if (is_hsa(how)) {
      while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) != 0) {
      }
      return -1;
    }
    CK(hipEventSynchronize(c1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, c0, c1));
    return ms;
  };
  auto check = [&]() {
    // spot-check the landed bytes against a device re-read
    uint64_t probe[4];
    const size_t at[4] = {0, rec_bytes / 3 & ~(size_t)7, rec_bytes / 2 & ~(size_t)7, rec_bytes - 8};
    for (int i = 0; i < 4; ++i) {
      CK(hipMemcpy(&probe[i], d_rec + at[i], 8, hipMemcpyDeviceToHost));
      if (memcmp(&probe[i], h_rec + at[i], 8)) { printf("  MISMATCH at %zu\n", at[i]); return false; }
    }
    return true;
  };
  const char* names[] = {"hipMemcpyAsync D2H", "hsa async copy (cpu dst agent)", "hsa split over 2 sdma engines",
                         "hsa split over 4 sdma engines", "kernel stores to host (8 WG)",
                         "hipMemcpyAsync D2H after an event", "hipMemcpyAsync D2H, NumaUser array",
                         "hsa split 2 engines, NumaUser array", "hipMemcpyAsync D2H over 4 streams",
                         "hipMemcpyAsync H2D", "hipMemcpyAsync H2D over 4 streams", "hsa H2D split over 4 engines"};
  for (int rep = 0; rep < reps; ++rep) {
    // the stream alone
    CK(hipEventRecord(e0, s1));
    k_stream<<<ncu * 4, 1024, 0, s1>>>((const u32x4*)d_big, big / 16, d_out);
    CK(hipEventRecord(e1, s1));
    CK(hipEventSynchronize(e1));
    float ms_alone = 0;
    CK(hipEventElapsedTime(&ms_alone, e0, e1));
    printf("rep %d stream alone %.3f ms (%.2f TB/s)\n", rep, ms_alone, big / ms_alone / 1e9);
    for (int how = 0; how < 12; ++how) {
      memset(h_rec, 0, 4096);
      double t0 = now_ms();
      copy(how);
      double ms = wait_copy(how);
      double wall = now_ms() - t0;
      bool ok = check();
      printf("rep %d %-34s alone: %.3f ms wall%s (%.1f GB/s)%s\n", rep, names[how], wall,
             ms >= 0 ? (" " + std::to_string(ms) + " ev").c_str() : "", rec_bytes / wall / 1e6, ok ? "" : " BAD");
      // beside the stream: the stream first, the copy right behind it
      CK(hipEventRecord(e0, s1));
      CK(hipEventRecord(dep, s1));
      k_stream<<<ncu * 4, 1024, 0, s1>>>((const u32x4*)d_big, big / 16, d_out);
      CK(hipEventRecord(e1, s1));
      std::this_thread::sleep_for(std::chrono::microseconds(200));
      t0 = now_ms();
      copy(how);
      ms = wait_copy(how);
      wall = now_ms() - t0;
      CK(hipEventSynchronize(e1));
      float ms_s = 0;
      CK(hipEventElapsedTime(&ms_s, e0, e1));
      ok = check();
      printf("rep %d %-34s beside: copy %.3f ms wall (%.1f GB/s), stream %.3f ms (%.2f TB/s, x%.3f)%s\n", rep,
             names[how], wall, rec_bytes / wall / 1e6, ms_s, big / ms_s / 1e9, ms_s / ms_alone, ok ? "" : " BAD");
    }
  }
  hsa_signal_destroy(sig);
  return 0;
}
