// lsmck_api.cpp -- device context and batch dispatch of liblsmck.so
// (include/lsmck.h sections 2-4).
//
// A context owns, per GPU: the CRC combination tables (x^(8*128*k) mod P,
// init terms, slicing tables; ~0.5 MiB, resident in HBM and L2), the scratch
// of the descriptor path (segment prefix sums, tile -> first record), and two
// pinned staging slots for host-resident batches (H2D / kernel / D2H of chunk
// c overlap the host-side packing of chunk c+1).
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <time.h>
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "lsmck.h"
#include "lsmck_device.h"
#include "lsmck_dma.h"
#include "lsmck_internal.h"
#include "lsmck_pool.h"
#include "lsmck_segwalk.h"

using lsmck::CrcParams;
using lsmck::ShaParams;

namespace {

constexpr uint64_t kMaxSegsPerLaunch = (1ull << 32) - 64;  // 32-bit segment indices in the kernels
constexpr int kVariantNoStream = 0x200000;  // descriptor batches: no stream kernel for packed >= 64-byte records (A/B)
constexpr int kVariantStreamOnly = 0x400000;  // diagnostic: the stream kernel alone (ineligible batches get no CRCs)
constexpr size_t kChunkBytes = 64ull << 20;                // host staging chunk (payload)
constexpr size_t kChunkRecs = 1u << 20;                    // host staging chunk (records)
constexpr int kWalHostWalk = 0x7FFF0001;  // internal: the GPU header walk declined the log; walk it on the host
constexpr int kWalTooBig = 0x7FFF0003;    // internal: one walk's jump tables would not fit; walk in smaller parts

struct HipFail {
  hipError_t e;
};

int hip_error(hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return lsmck_host::set_error(LSMCK_EHIP - (int)e, m.c_str());
}

#define HIPCHK(expr)                                  \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) return hip_error(_e, #expr); \
  } while (0)

int launch_rc(int rc, const char* what) {
  if (rc == 0) return 0;
  return hip_error((hipError_t)(-rc), what);
}

template <typename T>
int ensure_dev(T** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return 0;
  size_t want = std::max(need, *cap * 3 / 2);
  if (want == 0) want = 1;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HIPCHK(hipMalloc((void**)p, want * sizeof(T)));
  *cap = want;
  return 0;
}

// --- NUMA: the staging buffers and threads next to the device --
// On a node with several sockets each GPU hangs off one socket's PCIe root;
// pinned staging on the other socket's memory, or copy threads on its cores,
// cross the socket link on the way to the device.
int read_int_file(const std::string& path, int dflt) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return dflt;
  int v = dflt;
  if (fscanf(f, "%d", &v) != 1) v = dflt;
  fclose(f);
  return v;
}
// the device's NUMA node (sysfs of its PCI function), -1 if unknown
int device_numa_node(int dev) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, dev) != hipSuccess) return -1;
  std::string b(bus);
  for (auto& c : b) c = (char)tolower((unsigned char)c);
  return read_int_file("/sys/bus/pci/devices/" + b + "/numa_node", -1);
}
int numa_node_count() {
  int n = 0;
  while (n < 1024 && access(("/sys/devices/system/node/node" + std::to_string(n)).c_str(), F_OK) == 0) ++n;
  return n;
}
// the CPUs of a node ("0-7,16-23" in sysfs)
bool node_cpus(int node, cpu_set_t* set) {
  FILE* f = fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
  if (!f) return false;
  char buf[4096] = {0};
  const bool got = fgets(buf, sizeof buf, f) != nullptr;
  fclose(f);
  if (!got) return false;
  CPU_ZERO(set);
  int n = 0;
  for (char* s = buf; *s && *s != '\n';) {
    char* e = nullptr;
    const long a = strtol(s, &e, 10);
    if (e == s) break;
    long b = a;
    if (*e == '-') b = strtol(e + 1, &e, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET((int)c, set), ++n;
    s = *e == ',' ? e + 1 : e;
  }
  return n > 0;
}
constexpr int kMpolDefault = 0, kMpolPreferred = 1;

// Large pinned buffers are anonymous huge pages, populated and then
// registered (hipHostRegister): 1 GiB costs a fresh process ~0.04 s that way
// against ~0.2 s through hipHostMalloc, and ~0.04 s against ~0.13 s to free,
// at the same upload rate (tools/microbench_pin.hip, profiles/r05/pin; the
// tree verify's three ~1 GiB slots are allocated while the tree is listed).
// The registry tells host_free which way a pointer came.
constexpr size_t kHugePinMin = 2u << 20;
struct HugePins {
  std::mutex mu;
  std::vector<std::pair<void*, size_t>> v;
};
HugePins& huge_pins() {
  static HugePins h;
  return h;
}
hipError_t host_malloc_huge(void** p, size_t bytes, int node) {
  const size_t len = (bytes + kHugePinMin - 1) & ~(kHugePinMin - 1);
  void* q = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (q == MAP_FAILED) return hipErrorOutOfMemory;
  (void)madvise(q, len, MADV_HUGEPAGE);
  if (node >= 0 && node < 1024) {  // pages on the device's node, as hipHostMallocNumaUser places them
    unsigned long mask[16] = {0};
    mask[node / 64] |= 1ul << (node % 64);
    (void)syscall(SYS_mbind, q, len, kMpolPreferred, mask, 16 * 64, 0);
  }
  (void)madvise(q, len, 23 /* MADV_POPULATE_WRITE; hipHostRegister faults in what it leaves */);
  const hipError_t e = hipHostRegister(q, len, hipHostRegisterPortable | hipHostRegisterMapped);
  if (e != hipSuccess) {
    munmap(q, len);
    return e;
  }
  {
    std::lock_guard<std::mutex> lk(huge_pins().mu);
    huge_pins().v.emplace_back(q, len);
  }
  *p = q;
  return hipSuccess;
}
// frees what host_malloc_near (or hipHostMalloc) gave
void host_free(void* p) {
  if (!p) return;
  size_t len = 0;
  {
    std::lock_guard<std::mutex> lk(huge_pins().mu);
    auto& v = huge_pins().v;
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i].first == p) {
        len = v[i].second;
        v[i] = v.back();
        v.pop_back();
        break;
      }
  }
  if (len) {
    (void)hipHostUnregister(p);
    munmap(p, len);
  } else {
    (void)hipHostFree(p);
  }
}

// pinned host memory, on NUMA node `node` when one is given (the context's pin_node): the
// calling thread's policy prefers that node while HIP allocates and pins
// the pages (hipHostMallocNumaUser), then goes back to what it was
// huge: large buffers as registered huge pages (the tree verify's slots;
// not the buffers the SDMA read-back of lsmck_dma lands in, which take
// HIP's own pinned allocations)
hipError_t host_malloc_near(void** p, size_t bytes, int node, bool huge = false) {
  if (huge && bytes >= kHugePinMin) {
    const hipError_t e = host_malloc_huge(p, bytes, node);
    if (e == hipSuccess) return e;
    (void)hipGetLastError();  // (then as before)
  }
  if (node < 0 || node >= 1024) return hipHostMalloc(p, bytes, hipHostMallocDefault);
  int old_mode = kMpolDefault;
  unsigned long old_mask[16] = {0};
  const bool have_old = syscall(SYS_get_mempolicy, &old_mode, old_mask, 16 * 64, nullptr, 0) == 0;
  unsigned long mask[16] = {0};
  mask[node / 64] |= 1ul << (node % 64);
  const bool set = syscall(SYS_set_mempolicy, kMpolPreferred, mask, 16 * 64) == 0;
  const hipError_t e = hipHostMalloc(p, bytes, set ? hipHostMallocNumaUser : hipHostMallocDefault);
  if (set) {
    if (have_old && old_mode != kMpolDefault)
      (void)syscall(SYS_set_mempolicy, old_mode, old_mask, 16 * 64);
    else
      (void)syscall(SYS_set_mempolicy, kMpolDefault, nullptr, 0);
  }
  return e;
}

template <typename T>
int ensure_pinned(int node, T** p, size_t* cap, size_t need, bool huge = false) {
  if (*cap >= need && *p) return 0;
  size_t want = std::max(need, *cap * 3 / 2);
  if (want == 0) want = 1;
  if (*p) host_free(*p);
  *p = nullptr;
  *cap = 0;
  HIPCHK(host_malloc_near((void**)p, want * sizeof(T), node, huge));
  *cap = want;
  return 0;
}

// ensure_dev that keeps the first `keep` elements (copied on st)
template <typename T>
int ensure_dev_keep(T** p, size_t* cap, size_t need, size_t keep, hipStream_t st) {
  if (*cap >= need && *p) return 0;
  if (!keep || !*p) return ensure_dev(p, cap, need);
  const size_t want = std::max(need, *cap * 3 / 2);
  T* q = nullptr;
  HIPCHK(hipMalloc((void**)&q, want * sizeof(T)));
  HIPCHK(hipMemcpyAsync(q, *p, keep * sizeof(T), hipMemcpyDeviceToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  (void)hipFree(*p);
  *p = q;
  *cap = want;
  return 0;
}

// Scratch of the descriptor CRC path (one per in-flight launch).
struct DescScratch {
  uint64_t* block_sum = nullptr;  // per 1024-record block
  size_t cap_bs = 0;
  uint64_t* total = nullptr;  // device, 1 u64
  // SHA-256 dispatch order (lsmck_order.hip)
  uint16_t* sha_keys = nullptr;
  size_t cap_keys = 0;
  uint32_t* sha_order = nullptr;
  size_t cap_order = 0;
  unsigned char* sort_tmp = nullptr;
  size_t cap_tmp = 0;
  uint64_t* sha_split = nullptr;  // device, 1 u64: where the order's short tail starts
  size_t cap_split = 0;
  // stream kernel (lsmck_crc32.hip): eligibility flag, per-wave boundary cuts
  uint32_t* sflag = nullptr;
  uint64_t* scuts = nullptr;
  size_t cap_cuts = 0;
  void release() {
    if (sflag) (void)hipFree(sflag);
    if (scuts) (void)hipFree(scuts);
    if (block_sum) (void)hipFree(block_sum);
    if (total) (void)hipFree(total);
    if (sha_keys) (void)hipFree(sha_keys);
    if (sha_order) (void)hipFree(sha_order);
    if (sort_tmp) (void)hipFree(sort_tmp);
    if (sha_split) (void)hipFree(sha_split);
    *this = DescScratch();
  }
};

// One pinned staging slot of the host-resident pipeline.
struct Stage {
  hipStream_t s = nullptr;
  hipEvent_t done = nullptr;
  bool busy = false;
  // host (pinned)
  uint8_t* h_pay = nullptr;
  size_t cap_h_pay = 0;
  uint64_t* h_off = nullptr;
  size_t cap_h_off = 0;
  uint32_t* h_len = nullptr;
  size_t cap_h_len = 0;
  uint8_t* h_out = nullptr;
  size_t cap_h_out = 0;
  // device
  uint8_t* d_pay = nullptr;
  size_t cap_d_pay = 0;
  uint64_t* d_off = nullptr;
  size_t cap_d_off = 0;
  uint32_t* d_len = nullptr;
  size_t cap_d_len = 0;
  uint8_t* d_out = nullptr;
  size_t cap_d_out = 0;
  DescScratch scratch;
  // whole-tree verify: slice descriptors of the round in this slot
  lsmck::ShaSlice* h_slices = nullptr;
  size_t cap_h_slices = 0;
  lsmck::ShaSlice* d_slices = nullptr;
  size_t cap_d_slices = 0;
  // bookkeeping of the chunk in flight
  size_t rec0 = 0, nrec = 0;
  void release() {
    if (h_pay) host_free(h_pay);
    if (h_off) host_free(h_off);
    if (h_len) host_free(h_len);
    if (h_out) host_free(h_out);
    if (d_pay) (void)hipFree(d_pay);
    if (d_off) (void)hipFree(d_off);
    if (d_len) (void)hipFree(d_len);
    if (d_out) (void)hipFree(d_out);
    if (h_slices) host_free(h_slices);
    if (d_slices) (void)hipFree(d_slices);
    scratch.release();
    if (done) (void)hipEventDestroy(done);
    if (s) (void)hipStreamDestroy(s);
    *this = Stage();
  }
};
constexpr int kHostSlots = 2;  // slots the host batches and the WAL upload alternate

}  // namespace

struct lsmck_ctx {
  int dev = 0;
  int ncu = 0;
  hipStream_t stream0 = nullptr;
  uint32_t* d_master = nullptr;  // 4 x 256 slicing tables
  uint32_t* d_kseg = nullptr;    // 65536
  uint32_t* d_khi = nullptr;     // 65536
  uint32_t* d_tinit = nullptr;   // 129
  uint32_t* d_zero = nullptr;    // 256 zero bytes
  std::mutex mu;
  DescScratch scratch;           // device-mode descriptor scratch
  hipEvent_t scratch_ev = nullptr;
  unsigned long long* d_verify = nullptr;  // [n_bad, first_bad]
  unsigned long long* h_verify = nullptr;  // pinned
  // device verify / device WAL replay (grow-only; part of the scratch, ordered by scratch_ev)
  uint32_t* d_vcrc = nullptr;  // computed CRCs
  size_t cap_vcrc = 0;
  uint64_t* d_woff = nullptr;  // WAL payload descriptors and stored CRCs
  size_t cap_woff = 0;
  uint32_t* d_wlen = nullptr;
  size_t cap_wlen = 0;
  uint32_t* d_wexp = nullptr;
  size_t cap_wexp = 0;
  // device WAL walk (lsmck_wal.hip): candidate bitmap, ranks, successor levels, chain
  struct {
    uint64_t* bits = nullptr;
    size_t cap_bits = 0;
    uint32_t* pre = nullptr;
    size_t cap_pre = 0;
    uint32_t* bsum = nullptr;
    size_t cap_bsum = 0;
    uint64_t* pos = nullptr;
    size_t cap_pos = 0;
    uint32_t* J = nullptr;
    size_t cap_J = 0;
    uint64_t* badpos = nullptr;
    size_t cap_badpos = 0;
    uint32_t* chain = nullptr;
    size_t cap_chain = 0;
    lsmck_wal_rec* recs = nullptr;
    size_t cap_recs = 0;
    lsmck::seg::Compact16* recs16 = nullptr;  // the records in the compact layout (lsmck_wal_replay_verify16)
    size_t cap_recs16 = 0;
    unsigned long long* info = nullptr;  // [records, terminal, bad position, candidates (u32 at info+3)]
    unsigned long long* h_info = nullptr;  // pinned
    // the segment walk (lsmck_segwalk.h): per segment guess, exit, outcome,
    // records, placement scan; its round outcome (info words, and pinned)
    uint64_t* sg = nullptr;
    uint64_t* sx = nullptr;
    uint64_t* spre = nullptr;
    uint32_t* scode = nullptr;
    uint32_t* srecs = nullptr;
    size_t cap_seg = 0;
    uint64_t* sbsum = nullptr;
    size_t cap_sbsum = 0;
    unsigned long long* sinfo = nullptr;
    unsigned long long* h_sinfo = nullptr;
    uint64_t* scpp = nullptr;  // the emit's checkpoints (segments of 128 KiB and more)
    uint32_t* scpc = nullptr;
    size_t cap_cp = 0;
    lsmck::seg::StageRec* sst = nullptr;  // walk-time staged records (K * scap)
    size_t cap_sst = 0;
    uint64_t* sg0 = nullptr;  // the parallel repair's snapshot of sg / sx / scode
    uint64_t* sx0 = nullptr;
    uint32_t* scode0 = nullptr;
    size_t cap_seg0 = 0;
  } wd;
  bool wal_recs_direct = false;  // this replay's records go by DMA into the caller's pinned array (under wal_mu)
  bool wal_compact = false;      // this replay's records are lsmck_wal_rec16 (under wal_mu)
  // LSMCK_RECS_DEVICE (under wal_mu): the caller's device array and its capacity
  // (the segment walk emits straight into it when every record fits), and
  // whether this replay's emit did
  void* wal_recs_dev = nullptr;  // lsmck_wal_rec[] or, wal_compact, lsmck_wal_rec16[]
  size_t wal_recs_dev_cap = 0;
  bool wal_recs_dev_emitted = false;
  int wal_seg = 1;           // device WAL walk: 1 = the segment walk first (default), 0 = candidate doubling only
  uint64_t wal_seg_bytes = 0;  // segment walk: bytes per segment (0 = auto, ~2^16 segments)
  bool wal_seg_pack = true;  // segment walk: packed CRC spans (seg::Pack) for the CRC pass
  long wal_seg_stage = 1;    // segment walk: staged records (seg::StageRec): 0 off, 1 auto slots, else slots per segment
  int wal_seg_rounds = 16;   // segment walk: repairs before it declines to the candidate-doubling walk
  int wal_seg_prepair = 2;   // segment walk: parallel repair rounds before the serial repairs (0 = none)
  // The pipelined device replay (wal_replay_pipelined): the log walked in
  // wal_pipe parts, each part's CRC pass on a CU-masked stream beside the next
  // part's walk on the CUs left over (0 = off: the walk, then one CRC pass)
  int wal_pipe = 0;
  int wal_pipe_first = 4;   // the first part, in 64ths of the log (walked on every CU, nothing beside it)
  int wal_pipe_cus = 32;    // CUs the walk keeps; the CRC passes take the rest
  int wal_pipe_layout = 0;  // which CUs the walk keeps: 0 the last wal_pipe_cus, 1 spread (every ncu/cus-th)
  size_t wal_pipe_min = (size_t)1 << 30;  // logs from this size take the pipeline (when wal_pipe is on)
  uint64_t wal_pipe_seg = 0;  // the walk parts' segment bytes (0: sized to the walk CUs' resident lanes)
  uint64_t wal_seg_auto = 0;  // (set by the pipeline) the segment bytes of an auto-sized walk, 0: lsmk_wal_seg_bytes
  hipStream_t wal_pw = nullptr;  // the walk's CU-masked stream
  hipStream_t wal_pc = nullptr;  // the CRC passes' CU-masked stream
  int wal_pipe_key = -1;         // (cus, layout) the two streams were made for
  std::vector<hipEvent_t> wal_pipe_ev;  // per part: its records emitted (the CRC pass waits for it)
  // set while a pipelined replay runs: called before the walk grows the record
  // arrays, so nothing beside it still reads the old ones
  std::function<int()> wal_grow_hook;
  std::atomic<int> last_pipe_parts{0};  // the last device replay's parts (0: not pipelined)
  int numa_node = -1;    // the device's NUMA node (sysfs), -1 unknown
  int stage_numa = -2;   // option "stage_numa": -2 the device's node on a multi-node host, -1 off, >= 0 that node
  int pin_node = -1;     // in effect: pinned buffers and copy threads on this node (-1: none)
  // what the last device-walked replay did (lsmck_ctx_get_stat "wal_walk_path" / "wal_seg_repairs" / "wal_segments")
  // (atomic: lsmck_ctx_get_stat reads them under ctx->mu while a replay runs under wal_mu)
  std::atomic<int> last_walk_path{0};
  std::atomic<int> last_seg_repairs{0};
  std::atomic<uint64_t> last_segments{0};
  std::atomic<int> last_seg_prepairs{0};
  uint8_t* h_wrecs = nullptr;  // device WAL replay: the records' pinned landing buffer (bytes; grow-only)
  size_t cap_hwrecs = 0;
  // the records' read-back on the SDMA engines (lsmck_dma.h): created on first
  // use; "wal_dma_engines" engines (0: hipMemcpyAsync on the staging stream,
  // the round-4 path), the copy cut in "wal_dma_chunks" pieces
  lsmck_dma::Copier* dma = nullptr;
  bool dma_tried = false;
  std::atomic<int> last_recs_dma{0};  // the last read-back: SDMA engines used (0: hipMemcpyAsync)
  int wal_dma_engines = 4;
  int wal_dma_chunks = 32;
  hipEvent_t wal_emit_ev = nullptr;  // the emit's end: the records' read-back beside the CRC pass waits for it
  uint8_t* h_wrecs1 = nullptr;  // split host-image replay: the first part's records (pinned bytes, grow-only)
  size_t cap_hwrecs1 = 0;
  hipStream_t wal_rs = nullptr;       // ... read back on their own stream while the second part uploads
  hipEvent_t wal_emit1_ev = nullptr;
  std::unique_ptr<lsmck_host::HostPool> pool;  // staging copy threads (created on first use)
  uint64_t* h_woff = nullptr;  // pinned staging of the same
  size_t cap_hwoff = 0;
  uint32_t* h_wlen = nullptr;
  size_t cap_hwlen = 0;
  uint32_t* h_wexp = nullptr;
  size_t cap_hwexp = 0;
  // the host-batch pipelines alternate over slots 0 and 1; the whole-tree
  // verify cycles through the first tree_stages of them
  Stage stage[3];  // host batches and the WAL upload alternate 0 and 1 (kHostSlots); the tree verify uses all 3
  uint32_t tree_stages = 3;
  unsigned tree_json_threads = 0;  // whole-tree verify: checksum-file reader threads (0 = 2, 4 from 16k tables)
  size_t tree_list_batch = 0;  // lsmck_tree_verify: metadata names per listing batch (0 = 1024)
  long tree_overlap = 2048;  // lsmck_tree_verify: the top level's tables verified while the lower levels are
                             // listed, when it holds at least this many (0 = never)
  int variant = 0;  // A/B and diagnostic bits (crc_ablate, crc_stream, sha_order); 0 = default
  uint32_t tree_active = 0;  // whole-tree verify: files in flight (0 = kTreeActive)
  uint32_t tree_slice = 0;   // whole-tree verify: bytes of a file per round (0 = kTreeSlice)
  long tree_open = -1;       // whole-tree verify: files kept open between slices (-1 = RLIMIT_NOFILE budget)
  uint64_t tree_cpu_file = 0;  // whole-tree verify: files of at least this many bytes go to host threads (0 = 16 MiB)
  int sha_bucket_shift = 2;  // SHA order key: 2^shift-block buckets for from..1023 blocks (0 = exact; A/B: DESIGN.md 3.2)
  int sha_bucket_from = 128;
  int sha_pair = 1;  // SHA-256 batches: two blocks per load window (A/B: DESIGN.md 3.2)
  int sha_short_blocks = 12;  // SHA-256 ordered batches: messages of at most this many blocks on the lean kernel (0 = off)
  unsigned tree_list_threads = 0;  // lsmck_tree_verify: metadata parsing threads (0 = kListThreads)
  unsigned tree_readers = 16;      // whole-tree verify: threads reading a round's slices into its pinned slot
  size_t wal_prefetch = 4096;  // lsmck_wal_replay_verify: host walk's prefetch distance in bytes (0 = off)
  uint8_t* wal_host = nullptr;  // lsmck_wal_replay_verify of a device image: pinned host copy (grow-only)
  size_t wal_host_cap = 0;
  std::mutex wal_mu;  // guards wal_host for the duration of one device-image replay
  size_t wal_chunk = 32u << 20;
  int wal_gpu_walk = 1;  // lsmck_wal_replay_verify of a device image: header walk on the GPU (0 = copy back, host walk)
  // the GPU walk's scratch budget: this many bytes per log byte + 256 MiB (and
  // at most half the free device memory); over it the log takes the host walk
  size_t wal_walk_budget_per_byte = 8;
  int wal_register = 0;  // host WAL images: hipHostRegister the caller's pages instead of the staging copy (A/B)
  size_t wal_part_bytes = 0;  // GPU WAL walk: bytes per part (0 = the whole log, parts only when it does not fit)
  int wal_split = 1;     // host WAL images of two upload chunks or more: walk the first half during the second's upload
  // host WAL image upload: bytes per staged / DMA'd chunk.  16 MiB: 6.3 ms
  // for the 0.24 GB wal_diag image against 6.5 at 64 MiB (the first copy and
  // the last DMA are not overlapped), 10.7 at 4 MiB (per-chunk costs);
  // profiles/r03/h/wal_diag_r03h.json
  size_t wal_stage_bytes = 16u << 20;
  // host images of at least this many bytes are uploaded whole and walked on
  // the GPU (0 = always the host walk)
  size_t wal_upload_min = 1u << 20;
  uint8_t* d_wimg = nullptr;  // the uploaded host image (grow-only), guarded by wal_mu
  size_t cap_wimg = 0;
  unsigned stage_threads = 8;  // host batches: threads copying a pageable chunk into its pinned slot (1 = memcpy)  // lsmck_wal_replay_verify, host image: payload bytes per overlapped CRC batch (0 = one batch)
  struct {
    uint32_t* state = nullptr;  // 8 u32 per active slot
    size_t cap_state = 0;
    unsigned char* digests = nullptr;  // 32 B per file of the call
    size_t cap_digests = 0;
    hipEvent_t kernel_done = nullptr;
  } tree;
};

namespace {

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DevGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

hipStream_t pick_stream(lsmck_ctx* ctx, void* s) { return s ? (hipStream_t)s : ctx->stream0; }

// Every use of the context's device scratch (ctx->scratch, d_vcrc, d_verify,
// the WAL descriptor buffers) is ordered across streams by scratch_ev: the
// stream waits for the previous user's work, and the event is re-recorded
// after this call's work is enqueued (the host mutex only orders the enqueue).
struct ScratchOrder {
  lsmck_ctx* ctx;
  hipStream_t st;
  hipError_t e;
  ScratchOrder(lsmck_ctx* c, hipStream_t s) : ctx(c), st(s), e(hipStreamWaitEvent(s, c->scratch_ev, 0)) {}
  ~ScratchOrder() { (void)hipEventRecord(ctx->scratch_ev, st); }
};

int ensure_scratch(DescScratch& sc, size_t nblocks) {
  int rc;
  if ((rc = ensure_dev(&sc.block_sum, &sc.cap_bs, nblocks))) return rc;
  if (!sc.total) HIPCHK(hipMalloc((void**)&sc.total, 16));
  return 0;
}

void fill_tables(lsmck_ctx* ctx, CrcParams* P) {
  P->kseg = ctx->d_kseg;
  P->khi = ctx->d_khi;
  P->tinit = ctx->d_tinit;
  P->master = ctx->d_master;
  P->zero = ctx->d_zero;
}

// Fixed-size CRC on device pointers, split so each launch has < 2^32 segments.
int crc_fixed_device(lsmck_ctx* ctx, const uint8_t* base, size_t stride, uint32_t len, size_t n, uint32_t* out,
                     hipStream_t st) {
  if (n == 0) return 0;
  if (len == 0) {
    HIPCHK(hipMemsetAsync(out, 0, n * 4, st));
    return 0;
  }
  uint64_t nsegr = (len + 127u) / 128u;
  uint64_t per = kMaxSegsPerLaunch / nsegr;
  // every record is stored whole by one lane when no record straddles a
  // 64-segment tile; otherwise partial results are XOR-accumulated into zeros
  bool straddle = (64 % nsegr) != 0;
  if (straddle) HIPCHK(hipMemsetAsync(out, 0, n * 4, st));
  for (size_t r0 = 0; r0 < n; r0 += per) {
    size_t cnt = std::min<uint64_t>(per, n - r0);
    CrcParams P{};
    P.base = base + r0 * stride;
    P.stride = stride;
    P.flen = len;
    P.nrec = cnt;
    P.out = out + r0;
    fill_tables(ctx, &P);
    int rc = lsmk_launch_crc32_fixed(&P, ctx->ncu, ctx->variant, st);
    if (rc) return launch_rc(rc, "crc32_fixed kernel");
  }
  return 0;
}

// Descriptor CRC on device pointers with known (host) total segment count
// (host staging path) or unknown (device path: read back after the scan).
// trusted: the library's own batch (host-staged chunks, WAL payloads): sorted,
// not overlapping, the bytes between records inside the same buffer -- the
// stream kernel takes it without the device check or the walking kernel.
// ncu: the stream kernel's grid in workgroups (0: every CU; the pipelined WAL
// replay runs it on a CU-masked stream of fewer)
int crc_desc_device(lsmck_ctx* ctx, DescScratch& sc, const uint8_t* base, const uint64_t* off, const uint32_t* len,
                    size_t n, uint32_t* out, hipStream_t st, bool trusted = false, int ncu = 0) {
  if (n == 0) return 0;
  if (n >= (1ull << 32)) return lsmck_host::set_error(LSMCK_EINVAL, "more than 2^32-1 records in one batch");
  // walking kernel: scratch sized by the record count, nothing read back,
  // every CRC stored once -- asynchronous on st
  int rc = ensure_scratch(sc, (size_t)lsmk_walk_sb_count(n));
  if (rc) return rc;
  CrcParams P{};
  P.base = base;
  P.off = off;
  P.len = len;
  P.nrec = n;
  P.total_segs = sc.total;
  P.out = out;
  fill_tables(ctx, &P);
  if (!(ctx->variant & kVariantNoStream)) {
    // sorted batches, packed or with small gaps: the stream kernel (a
    // caller's batch is checked on the device; when it is not eligible the
    // walking kernel below takes it, else that kernel exits at once)
    if (!sc.sflag) HIPCHK(hipMalloc((void**)&sc.sflag, 16));
    const int g = ncu > 0 && ncu < ctx->ncu ? ncu : ctx->ncu;
    if ((rc = ensure_dev(&sc.scuts, &sc.cap_cuts, (size_t)lsmk_stream_waves(ctx->ncu) + 1))) return rc;
    P.sflag = sc.sflag;
    P.scuts = sc.scuts;
    rc = lsmk_launch_crc32_stream(&P, g, ctx->variant, trusted ? 1 : 0, st);
    if (rc) return launch_rc(rc, "crc32_stream kernel");
    if (trusted || (ctx->variant & kVariantStreamOnly)) return 0;
  }
  rc = lsmk_launch_crc32_walk(&P, sc.block_sum, ctx->ncu, ctx->variant, st);
  return rc ? launch_rc(rc, "crc32_walk kernel") : 0;
}

// Variable-length batches of at least this many messages run in decreasing
// length order (lsmck_order.hip); below it the sort costs more than the
// divergence it removes.
constexpr size_t kShaSortMin = 2048;

int sha_device(lsmck_ctx* ctx, DescScratch& sc, const uint8_t* base, const uint64_t* off, const uint32_t* len,
               size_t stride, uint32_t flen, size_t n, uint8_t* out32, hipStream_t st) {
  const uint32_t* order = nullptr;
  if (len && n >= kShaSortMin && !(ctx->variant & 0x10000)) {  // 0x10000: batch order (A/B)
    if (n >= (1ull << 32)) return lsmck_host::set_error(LSMCK_EINVAL, "more than 2^32-1 messages in one batch");
    int rc;
    if ((rc = ensure_dev(&sc.sha_keys, &sc.cap_keys, n))) return rc;
    if ((rc = ensure_dev(&sc.sha_order, &sc.cap_order, n))) return rc;
    size_t tmp = 0;
    rc = lsmk_sha_order(len, n, sc.sha_keys, sc.sha_order, nullptr, &tmp, ctx->sha_bucket_shift, ctx->sha_bucket_from, st);
    if (rc) return launch_rc(rc, "sha order (size query)");
    if ((rc = ensure_dev(&sc.sort_tmp, &sc.cap_tmp, std::max<size_t>(tmp, 1)))) return rc;
    rc = lsmk_sha_order(len, n, sc.sha_keys, sc.sha_order, sc.sort_tmp, &tmp, ctx->sha_bucket_shift, ctx->sha_bucket_from, st);
    if (rc) return launch_rc(rc, "sha order (radix sort)");
    order = sc.sha_order;
    if (ctx->sha_short_blocks > 0) {
      if ((rc = ensure_dev(&sc.sha_split, &sc.cap_split, 1))) return rc;
      rc = lsmk_sha_split(sc.sha_keys, n, (uint32_t)ctx->sha_short_blocks, sc.sha_split, st);
      if (rc) return launch_rc(rc, "sha split");
    }
  }
  ShaParams P{};
  P.base = base;
  P.off = off;
  P.len = len;
  P.stride = stride;
  P.flen = flen;
  P.nmsg = n;
  P.order = order;
  P.out = out32;
  P.pair = (uint32_t)ctx->sha_pair;
  P.split = (order && ctx->sha_short_blocks > 0) ? sc.sha_split : nullptr;
  int rc = lsmk_launch_sha256(&P, st);
  return rc ? launch_rc(rc, "sha256 kernel") : 0;
}

// ---------------------------------------------------------------------------
// Host-resident batches: chunked, double-buffered pipeline through pinned slots.
enum Kind { CRC = 0, SHA = 1 };

struct HostJob {
  Kind kind;
  const uint8_t* base;
  const uint64_t* off;  // null -> fixed
  const uint32_t* len;
  size_t stride;
  uint32_t flen;
  size_t n;
  uint8_t* out;  // 4 or 32 bytes per record
  bool pinned;   // base is pinned: DMA straight from it (contiguous spans only)
};

int stage_init(Stage& S) {
  if (!S.s) HIPCHK(hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking));
  if (!S.done) HIPCHK(hipEventCreateWithFlags(&S.done, hipEventDisableTiming));
  return 0;
}

// Pageable payload into a pinned slot.  One thread copies at ~20 GiB/s, below
// the PCIe link the slot then feeds; large chunks are split over `threads`
// (contiguous byte ranges, 4 KiB-aligned cuts).
lsmck_host::HostPool& host_pool(lsmck_ctx* ctx) {
  if (!ctx->pool) {
    ctx->pool.reset(new lsmck_host::HostPool());
    cpu_set_t set;
    if (ctx->pin_node >= 0 && node_cpus(ctx->pin_node, &set)) ctx->pool->set_cpus(set);
  }
  return *ctx->pool;
}

// the context's NUMA placement from its option (ctx->mu held or not yet shared)
void apply_numa(lsmck_ctx* ctx) {
  ctx->pin_node = ctx->stage_numa == -2 ? (numa_node_count() > 1 ? ctx->numa_node : -1) : ctx->stage_numa;
  if (ctx->pool) {
    cpu_set_t set;
    if (ctx->pin_node >= 0 && node_cpus(ctx->pin_node, &set))
      ctx->pool->set_cpus(set);
    else
      ctx->pool->clear_cpus();
  }
}

void stage_copy(lsmck_ctx* ctx, uint8_t* dst, const uint8_t* src, size_t n, unsigned threads) {
  if (threads <= 1 || n < (8u << 20)) {
    memcpy(dst, src, n);
    return;
  }
  const size_t part = ((n / threads) + 4095) & ~(size_t)4095;
  host_pool(ctx).run(threads, [=](unsigned t) {
    const size_t a = std::min(n, t * part), b = std::min(n, (t + 1) * part);
    if (a < b) memcpy(dst + a, src + a, b - a);
  });
}

// Wait for a slot's previous chunk and hand its results to the caller.
int stage_retire(Stage& S, const HostJob& J) {
  if (!S.busy) return 0;
  HIPCHK(hipEventSynchronize(S.done));
  size_t esz = J.kind == CRC ? 4 : 32;
  memcpy(J.out + S.rec0 * esz, S.h_out, S.nrec * esz);
  S.busy = false;
  return 0;
}

// On any early return of run_host_job: wait for both staging streams (no DMA
// from the caller's memory may still run after the call returns) and drop the
// slots' bookkeeping, so that the next call never retires a stale chunk into
// its own output.
struct StageGuard {
  lsmck_ctx* ctx;
  bool ok = false;
  ~StageGuard() {
    if (ok) return;
    for (auto& S : ctx->stage) {
      if (S.s) (void)hipStreamSynchronize(S.s);
      S.busy = false;
    }
  }
};

int run_host_job(lsmck_ctx* ctx, const HostJob& J) {
  size_t esz = J.kind == CRC ? 4 : 32;
  int rc;
  StageGuard guard{ctx};
  for (int k = 0; k < kHostSlots; ++k) {  // (the batches alternate slots 0 and 1; slot 2 is the tree verify's)
    Stage& S = ctx->stage[k];
    if ((rc = stage_init(S))) return rc;
    if (S.busy) {  // left by a call that failed before its guard existed: never retire it here
      HIPCHK(hipStreamSynchronize(S.s));
      S.busy = false;
    }
  }
  // Fixed records far apart (stride well above len) are gathered into a packed
  // layout instead of shipping their whole span: a span of cnt*stride bytes
  // would cost stride/len times the PCIe traffic (and the staging memory).
  const bool sparse = !J.off && (uint64_t)J.stride * 4 > (uint64_t)J.flen * 5 + 256;
  size_t r = 0;
  int slot = 0;
  while (r < J.n) {
    // choose the chunk [r, r1)
    size_t r1 = r;
    uint64_t bytes = 0;
    uint64_t span_lo = UINT64_MAX, span_hi = 0;
    bool mono = true;
    uint64_t prev_end = 0;
    while (r1 < J.n && (r1 - r) < kChunkRecs) {
      uint64_t o = J.off ? J.off[r1] : (uint64_t)r1 * J.stride;
      uint64_t l = J.off ? J.len[r1] : J.flen;
      if (r1 > r && bytes + l > kChunkBytes) break;
      if (r1 > r && o < prev_end) mono = false;
      prev_end = o + l;
      span_lo = std::min(span_lo, o);
      span_hi = std::max(span_hi, o + l);
      bytes += l;
      ++r1;
    }
    size_t cnt = r1 - r;
    if (span_lo == UINT64_MAX) span_lo = span_hi = 0;
    // dense fixed-stride records ship as their span (the kernel indexes by stride)
    bool use_span = !J.off ? !sparse : (mono && (span_hi - span_lo) <= bytes + bytes / 4 + 4096);
    Stage& S = ctx->stage[slot];
    if ((rc = stage_retire(S, J))) return rc;
    // descriptors (rebased) and payload
    size_t pay_bytes = use_span ? (size_t)(span_hi - span_lo) : (size_t)bytes;
    if ((rc = ensure_pinned(ctx->pin_node, &S.h_out, &S.cap_h_out, cnt * esz))) return rc;
    if ((rc = ensure_dev(&S.d_out, &S.cap_d_out, cnt * esz))) return rc;
    if ((rc = ensure_dev(&S.d_pay, &S.cap_d_pay, pay_bytes + 16))) return rc;
    const uint8_t* h_src = nullptr;
    if (J.off) {
      if ((rc = ensure_pinned(ctx->pin_node, &S.h_off, &S.cap_h_off, cnt))) return rc;
      if ((rc = ensure_pinned(ctx->pin_node, &S.h_len, &S.cap_h_len, cnt))) return rc;
      if ((rc = ensure_dev(&S.d_off, &S.cap_d_off, cnt))) return rc;
      if ((rc = ensure_dev(&S.d_len, &S.cap_d_len, cnt))) return rc;
      uint64_t pos = 0;
      for (size_t i = 0; i < cnt; ++i) {
        uint64_t o = J.off[r + i];
        S.h_len[i] = J.len[r + i];
        S.h_off[i] = use_span ? o - span_lo : pos;
        pos += J.len[r + i];
      }
    }
    if (use_span && J.pinned) {
      h_src = J.base + span_lo;
    } else {
      if ((rc = ensure_pinned(ctx->pin_node, &S.h_pay, &S.cap_h_pay, pay_bytes + 16))) return rc;
      if (use_span) {
        stage_copy(ctx, S.h_pay, J.base + span_lo, pay_bytes, ctx->stage_threads);
      } else if (!J.off) {
        // sparse fixed records: record r+i lands at i*flen
        const unsigned T = pay_bytes >= (8u << 20) ? std::max(1u, ctx->stage_threads) : 1u;
        auto gather = [&](size_t i0, size_t i1) {
          for (size_t i = i0; i < i1; ++i) memcpy(S.h_pay + i * J.flen, J.base + (r + i) * J.stride, J.flen);
        };
        host_pool(ctx).run(T, [&](unsigned t) { gather(cnt * t / T, cnt * (t + 1) / T); });
      } else {
        // gather: record i lands at its packed position S.h_off[i]; large
        // chunks split the records over stage_threads threads
        const unsigned T = pay_bytes >= (8u << 20) ? std::max(1u, ctx->stage_threads) : 1u;
        auto gather = [&](size_t i0, size_t i1) {
          for (size_t i = i0; i < i1; ++i) memcpy(S.h_pay + S.h_off[i], J.base + J.off[r + i], J.len[r + i]);
        };
        host_pool(ctx).run(T, [&](unsigned t) { gather(cnt * t / T, cnt * (t + 1) / T); });
      }
      h_src = S.h_pay;
    }
    HIPCHK(hipMemcpyAsync(S.d_pay, h_src, pay_bytes, hipMemcpyHostToDevice, S.s));
    if (J.off) {
      HIPCHK(hipMemcpyAsync(S.d_off, S.h_off, cnt * 8, hipMemcpyHostToDevice, S.s));
      HIPCHK(hipMemcpyAsync(S.d_len, S.h_len, cnt * 4, hipMemcpyHostToDevice, S.s));
    }
    if (J.kind == CRC) {
      if (J.off) {
        // the staged chunk is sorted by construction: its whole span (sorted,
        // not overlapping: `mono`), or the records packed in order
        rc = crc_desc_device(ctx, S.scratch, S.d_pay, S.d_off, S.d_len, cnt, (uint32_t*)S.d_out, S.s, true);
      } else {
        // fixed records: the span starts at record r (gathered: packed at stride flen)
        rc = crc_fixed_device(ctx, S.d_pay, use_span ? J.stride : J.flen, J.flen, cnt, (uint32_t*)S.d_out, S.s);
      }
    } else {
      if (J.off)
        rc = sha_device(ctx, S.scratch, S.d_pay, S.d_off, S.d_len, 0, 0, cnt, S.d_out, S.s);
      else
        rc = sha_device(ctx, S.scratch, S.d_pay, nullptr, nullptr, use_span ? J.stride : J.flen, J.flen, cnt,
                        S.d_out, S.s);
    }
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(S.h_out, S.d_out, cnt * esz, hipMemcpyDeviceToHost, S.s));
    HIPCHK(hipEventRecord(S.done, S.s));
    S.busy = true;
    S.rec0 = r;
    S.nrec = cnt;
    r = r1;
    slot ^= 1;
  }
  for (int k = 0; k < kHostSlots; ++k)
    if ((rc = stage_retire(ctx->stage[k], J))) return rc;
  guard.ok = true;
  return 0;
}

int check_ctx(lsmck_ctx* ctx) {
  if (!ctx) return lsmck_host::set_error(LSMCK_EINVAL, "null context");
  return 0;
}

// CRC batch + GPU compare with expected[] (all device pointers) on st, into the
// context's pooled buffers; synchronous (the counts come back to the host).
// Caller holds ctx->mu and orders st on the scratch.
// while_running: host work done after the launches, before the wait (the
// WAL replay copies its records out meanwhile)
int device_verify(lsmck_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint32_t* len,
                  const uint32_t* expected, size_t n, hipStream_t st, uint64_t* n_bad, uint64_t* first_bad,
                  bool trusted = false, const std::function<int()>& while_running = {}) {
  int rc = ensure_dev(&ctx->d_vcrc, &ctx->cap_vcrc, std::max<size_t>(n, 1));
  if (rc) return rc;
  rc = crc_desc_device(ctx, ctx->scratch, base, off, len, n, ctx->d_vcrc, st, trusted);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(ctx->d_verify, 0, 8, st));         // n_bad
  HIPCHK(hipMemsetAsync(ctx->d_verify + 1, 0xFF, 8, st));  // first_bad = ~0
  rc = lsmk_launch_crc32_compare(ctx->d_vcrc, expected, n, ctx->d_verify, ctx->d_verify + 1, st);
  if (rc) return launch_rc(rc, "compare kernel");
  HIPCHK(hipMemcpyAsync(ctx->h_verify, ctx->d_verify, 16, hipMemcpyDeviceToHost, st));
  const int hrc = while_running ? while_running() : 0;
  HIPCHK(hipStreamSynchronize(st));
  if (hrc) return hrc;
  if (n_bad) *n_bad = ctx->h_verify[0];
  if (first_bad) *first_bad = ctx->h_verify[0] ? ctx->h_verify[1] : n;
  return ctx->h_verify[0] ? 1 : 0;
}

}  // namespace

// ===========================================================================
extern "C" {

int lsmck_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

lsmck_ctx* lsmck_ctx_create(int device) {
  int n = lsmck_device_count();
  if (n <= 0) {
    lsmck_host::set_error(LSMCK_ENODEV, "no HIP device available");
    return nullptr;
  }
  if (device < 0 || device >= n) {
    lsmck_host::set_error(LSMCK_EINVAL, "device index out of range");
    return nullptr;
  }
  DevGuard g(device);
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, device) != hipSuccess) {
    lsmck_host::set_error(LSMCK_ENODEV, "hipGetDeviceProperties failed");
    return nullptr;
  }
  if (strncmp(pr.gcnArchName, "gfx950", 6) != 0) {
    std::string m = std::string("liblsmck is built for gfx950 (MI355X); device is ") + pr.gcnArchName;
    lsmck_host::set_error(LSMCK_ENODEV, m.c_str());
    return nullptr;
  }
  lsmck_ctx* ctx = new lsmck_ctx();
  ctx->dev = device;
  ctx->ncu = pr.multiProcessorCount;
#ifdef LSMCK_DIAG
  if (const char* e = getenv("LSMCK_CUS")) {  // diagnostic builds only: the persistent kernels on fewer CUs
    const int c = atoi(e);
    if (c > 0 && c < ctx->ncu) ctx->ncu = c;
  }
#endif
  ctx->numa_node = device_numa_node(device);
  apply_numa(ctx);
  // combination tables
  std::vector<uint32_t> master(4096), kseg(65536), khi(65536), tinit(130, 0u);
  const uint32_t* T = lsmck_host::crc_tables();
  for (int t = 0; t < 4; ++t)
    for (int e = 0; e < 256; ++e) master[t * 256 + e] = T[t * 256 + e];
  for (int m = 1; m <= 3; ++m) {  // shift tables: register advanced over 32*m zero bytes
    uint32_t X = lsmck_host::x_pow_8n(32 * m);
    for (int j = 0; j < 4; ++j)
      for (int b = 0; b < 256; ++b) master[1024 * m + 256 * j + b] = lsmck_host::gf2_mulmod(X, (uint32_t)b << (8 * j));
  }
  uint32_t X = lsmck_host::x_pow_8n(128);  // one segment
  kseg[0] = 1u << 31;
  for (int k = 1; k < 65536; ++k) kseg[k] = lsmck_host::gf2_mulmod(kseg[k - 1], X);
  uint32_t Y = lsmck_host::gf2_mulmod(kseg[65535], X);  // 65536 segments
  khi[0] = 1u << 31;
  for (int k = 1; k < 65536; ++k) khi[k] = lsmck_host::gf2_mulmod(khi[k - 1], Y);
  for (int m = 0; m <= 128; ++m) tinit[m] = lsmck_host::gf2_mulmod(lsmck_host::x_pow_8n(m), 0xFFFFFFFFu);
  bool ok = hipStreamCreateWithFlags(&ctx->stream0, hipStreamNonBlocking) == hipSuccess &&
            hipMalloc((void**)&ctx->d_master, 4096 * 4) == hipSuccess &&
            hipMalloc((void**)&ctx->d_kseg, 65536 * 4) == hipSuccess &&
            hipMalloc((void**)&ctx->d_khi, 65536 * 4) == hipSuccess &&
            hipMalloc((void**)&ctx->d_tinit, 130 * 4) == hipSuccess &&
            hipMalloc((void**)&ctx->d_zero, 256) == hipSuccess && hipMemset(ctx->d_zero, 0, 256) == hipSuccess &&
            hipMemcpy(ctx->d_master, master.data(), 4096 * 4, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(ctx->d_kseg, kseg.data(), 65536 * 4, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(ctx->d_khi, khi.data(), 65536 * 4, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(ctx->d_tinit, tinit.data(), 130 * 4, hipMemcpyHostToDevice) == hipSuccess &&
            hipEventCreateWithFlags(&ctx->scratch_ev, hipEventDisableTiming) == hipSuccess &&
            hipHostMalloc((void**)&ctx->h_verify, 64, hipHostMallocDefault) == hipSuccess &&
            hipMalloc((void**)&ctx->d_verify, 64) == hipSuccess;
  if (!ok) {
    lsmck_host::set_error(LSMCK_ENOMEM, "context allocation failed");
    lsmck_ctx_destroy(ctx);
    return nullptr;
  }
  return ctx;
}

int lsmck_ctx_set_option(lsmck_ctx* ctx, const char* key, long value) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!key) return lsmck_host::set_error(LSMCK_EINVAL, "null key");
  if (!strcmp(key, "crc_ablate")) {  // diagnostic only (results are garbage): 3 = payload loads only (the
                                     // bench's loads-only ceiling), 2 = stream kernel without payload loads
    if (value != 0 && value != 3 && (!lsmk_ab_ablations() || value < 2 || value > 12))
      return lsmck_host::set_error(LSMCK_EINVAL, lsmk_ab_ablations() ? "crc_ablate must be 0 or 2..12"
                                                                     : "crc_ablate must be 0 or 3 (2, 4..12: an A/B "
                                                                       "library built with -DLSMCK_AB_ABLATIONS)");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->variant = (ctx->variant & ~0xF00) | ((int)value << 8);
    return 0;
  }
  if (!strcmp(key, "tree_active_files")) {  // whole-tree verify: files in flight (0 = 8192); tests use few
    if (value < 0 || value > (1l << 20)) return lsmck_host::set_error(LSMCK_EINVAL, "tree_active_files: 0..2^20");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->tree_active = (uint32_t)value;
    return 0;
  }
  if (!strcmp(key, "tree_slice_bytes")) {  // whole-tree verify: bytes per file per round (0 = 128 KiB)
    if (value < 0 || value % 64 || value > (1l << 30))
      return lsmck_host::set_error(LSMCK_EINVAL, "tree_slice_bytes: a multiple of 64, <= 2^30");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->tree_slice = (uint32_t)value;
    return 0;
  }
  if (!strcmp(key, "tree_list_batch")) {  // lsmck_tree_verify: metadata names per listing batch (0 = 1024; tests)
    if (value < 0 || value > (1l << 20)) return lsmck_host::set_error(LSMCK_EINVAL, "tree_list_batch: 0 .. 2^20");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->tree_list_batch = (size_t)value;
    return 0;
  }
  if (!strcmp(key, "tree_overlap")) {  // lsmck_tree_verify: the top level verified while the others are listed
    if (value < 0 || value > (1l << 30)) return lsmck_host::set_error(LSMCK_EINVAL, "tree_overlap: 0 .. 2^30");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->tree_overlap = (long)value;
    return 0;
  }
  if (!strcmp(key, "tree_json_threads")) {  // whole-tree verify: threads reading the checksum files (0 = auto)
    if (value < 0 || value > 64) return lsmck_host::set_error(LSMCK_EINVAL, "tree_json_threads: 0..64");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->tree_json_threads = (unsigned)value;
    return 0;
  }
  if (!strcmp(key, "tree_stages")) {  // whole-tree verify: pinned slots the rounds cycle through (A/B: 2 or 3)
    if (value < 2 || value > 3) return lsmck_host::set_error(LSMCK_EINVAL, "tree_stages: 2 or 3");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->tree_stages = (uint32_t)value;
    return 0;
  }
  if (!strcmp(key, "tree_open_files")) {  // whole-tree verify: cap on files kept open (-1 = rlimit budget)
    if (value < -1) return lsmck_host::set_error(LSMCK_EINVAL, "tree_open_files: -1 or >= 0");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->tree_open = value;
    return 0;
  }
  if (!strcmp(key, "tree_cpu_file_bytes")) {  // whole-tree verify: host-thread SHA-256 for files >= this (0 = 16 MiB)
    if (value < 0) return lsmck_host::set_error(LSMCK_EINVAL, "tree_cpu_file_bytes: >= 0");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->tree_cpu_file = (uint64_t)value;
    return 0;
  }
  if (!strcmp(key, "tree_list_threads")) {  // A/B: metadata parsing threads of lsmck_tree_verify (0 = 8)
    if (value < 0 || value > 256) return lsmck_host::set_error(LSMCK_EINVAL, "tree_list_threads: 0..256");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->tree_list_threads = (unsigned)value;
    return 0;
  }
  if (!strcmp(key, "tree_readers")) {  // A/B: whole-tree verify's slice reader threads
    if (value < 1 || value > 64) return lsmck_host::set_error(LSMCK_EINVAL, "tree_readers: 1..64");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->tree_readers = (unsigned)value;
    return 0;
  }
  if (!strcmp(key, "stage_threads")) {  // A/B: threads of the pageable -> pinned staging copy (1 = one memcpy)
    if (value < 1 || value > 64) return lsmck_host::set_error(LSMCK_EINVAL, "stage_threads: 1..64");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->stage_threads = (unsigned)value;
    return 0;
  }
  if (!strcmp(key, "wal_chunk_bytes")) {  // A/B: WAL replay CRC batches overlapped with the walk (0 = one batch after it)
    if (value < 0) return lsmck_host::set_error(LSMCK_EINVAL, "wal_chunk_bytes: >= 0");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_chunk = (size_t)value;
    return 0;
  }
  if (!strcmp(key, "wal_gpu_walk")) {  // A/B: device-image WAL replay, 1 = GPU header walk (default), 0 = host walk
    if (value != 0 && value != 1) return lsmck_host::set_error(LSMCK_EINVAL, "wal_gpu_walk must be 0 or 1");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_gpu_walk = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_stage_bytes")) {  // A/B: host WAL image upload chunk (a multiple of 64 KiB, 1..64 MiB)
    if (value < (1 << 20) || value > (long)kChunkBytes || (value & 0xFFFF))
      return lsmck_host::set_error(LSMCK_EINVAL, "wal_stage_bytes: a multiple of 64 KiB in [1 MiB, 64 MiB]");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_stage_bytes = (size_t)value;
    return 0;
  }
  if (!strcmp(key, "wal_part_bytes")) {  // GPU WAL walk in parts of this many bytes (0 = whole; tests / A/B)
    if (value < 0 || (value && value < (1l << 20)))
      return lsmck_host::set_error(LSMCK_EINVAL, "wal_part_bytes: 0 or >= 1 MiB");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_part_bytes = (size_t)value;
    return 0;
  }
  if (!strcmp(key, "wal_split")) {  // A/B: host WAL image walked in two parts behind its upload (0 = whole)
    if (value != 0 && value != 1) return lsmck_host::set_error(LSMCK_EINVAL, "wal_split must be 0 or 1");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_split = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_register")) {  // A/B: host WAL image uploaded by DMA from its own pages, pinned in place
    if (value != 0 && value != 1) return lsmck_host::set_error(LSMCK_EINVAL, "wal_register must be 0 or 1");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_register = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_upload_min")) {  // A/B: host WAL images from this size go to the GPU walk (0 = never)
    if (value < 0) return lsmck_host::set_error(LSMCK_EINVAL, "wal_upload_min: >= 0");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_upload_min = (size_t)value;
    return 0;
  }
  if (!strcmp(key, "wal_seg_walk")) {  // A/B: device WAL walk, 1 = segment walk first (default), 0 = doubling only
    if (value != 0 && value != 1) return lsmck_host::set_error(LSMCK_EINVAL, "wal_seg_walk must be 0 or 1");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_seg = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_dma_engines")) {  // WAL records to the host: SDMA engines (0 = hipMemcpyAsync; A/B)
    if (value < 0 || value > 16) return lsmck_host::set_error(LSMCK_EINVAL, "wal_dma_engines: 0..16");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_dma_engines = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_dma_chunks")) {  // WAL records to the host: pieces of the SDMA copy
    if (value < 1 || value > lsmck_dma::kMaxChunks)
      return lsmck_host::set_error(LSMCK_EINVAL, "wal_dma_chunks: 1..64");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_dma_chunks = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_seg_bytes")) {  // segment walk: bytes per segment (0 = auto; tests force small segments)
    if (value < 0 || (value && (value < 64 || value > (1l << 30))))
      return lsmck_host::set_error(LSMCK_EINVAL, "wal_seg_bytes: 0 or 64..2^30");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_seg_bytes = (uint64_t)value;
    return 0;
  }
  if (!strcmp(key, "stage_numa")) {  // pinned staging and copy threads: -2 auto (device's node), -1 off, >= 0 a node
    if (value < -2 || value > 1023) return lsmck_host::set_error(LSMCK_EINVAL, "stage_numa: -2..1023");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->stage_numa = (int)value;
    apply_numa(ctx);
    return 0;
  }
  if (!strcmp(key, "wal_seg_stage")) {  // segment walk: records staged by the walk (1 auto, 0 off, >= 2 slots/segment)
    if (value < 0 || value > (1l << 24)) return lsmck_host::set_error(LSMCK_EINVAL, "wal_seg_stage: 0..2^24");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_seg_stage = value;
    return 0;
  }
  if (!strcmp(key, "wal_seg_pack")) {  // A/B: the segment walk's packed CRC spans (1, default) or payloads alone (0)
    if (value != 0 && value != 1) return lsmck_host::set_error(LSMCK_EINVAL, "wal_seg_pack: 0 or 1");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_seg_pack = value != 0;
    return 0;
  }
  if (!strcmp(key, "wal_seg_prepair")) {  // segment walk: parallel repair rounds before serial repairs (0 = none)
    if (value < 0 || value > 64) return lsmck_host::set_error(LSMCK_EINVAL, "wal_seg_prepair: 0..64");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_seg_prepair = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_seg_rounds")) {  // segment walk: repair rounds before declining (0 = decline on any failure)
    if (value < 0 || value > 1024) return lsmck_host::set_error(LSMCK_EINVAL, "wal_seg_rounds: 0..1024");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_seg_rounds = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_pipe")) {  // device WAL replay: parts walked beside the CRC passes (0 = off)
    if (value < 0 || value > 64) return lsmck_host::set_error(LSMCK_EINVAL, "wal_pipe: 0..64");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_pipe = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_pipe_first")) {  // the pipeline's first part, in 64ths of the log
    if (value < 1 || value > 63) return lsmck_host::set_error(LSMCK_EINVAL, "wal_pipe_first: 1..63");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_pipe_first = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_pipe_cus")) {  // the pipeline's walk CUs (the CRC passes take the rest)
    if (value < 1 || value >= ctx->ncu) return lsmck_host::set_error(LSMCK_EINVAL, "wal_pipe_cus: 1..ncu-1");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_pipe_cus = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_pipe_min")) {  // the pipeline's smallest log (tests: small logs through every part)
    if (value < 0) return lsmck_host::set_error(LSMCK_EINVAL, "wal_pipe_min: >= 0");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_pipe_min = (size_t)value;
    return 0;
  }
  if (!strcmp(key, "wal_pipe_seg")) {  // the pipeline walk parts' segment bytes (0 = sized to the walk's CUs)
    if (value < 0 || (value && (value < 4096 || value > (1l << 30))))
      return lsmck_host::set_error(LSMCK_EINVAL, "wal_pipe_seg: 0 or 4096..2^30");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_pipe_seg = (uint64_t)value;
    return 0;
  }
  if (!strcmp(key, "wal_pipe_layout")) {  // which CUs the walk keeps: 0 the last ones, 1 spread
    if (value != 0 && value != 1) return lsmck_host::set_error(LSMCK_EINVAL, "wal_pipe_layout: 0 or 1");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_pipe_layout = (int)value;
    return 0;
  }
  if (!strcmp(key, "wal_prefetch")) {  // A/B: bytes the WAL header walk prefetches ahead (0 = off)
    if (value < 0 || value > (1l << 24)) return lsmck_host::set_error(LSMCK_EINVAL, "wal_prefetch: 0..16 MiB");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->wal_prefetch = (size_t)value;
    return 0;
  }
  if (!strcmp(key, "sha_bucket_from")) {  // A/B: first block count of the coarse SHA buckets
    if (value < 2 || value > 1024) return lsmck_host::set_error(LSMCK_EINVAL, "sha_bucket_from: 2..1024");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->sha_bucket_from = (int)value;
    return 0;
  }
  if (!strcmp(key, "sha_bucket_shift")) {  // A/B: coarser SHA length buckets (0 = exact block counts)
    if (value < 0 || value > 6) return lsmck_host::set_error(LSMCK_EINVAL, "sha_bucket_shift: 0..6");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->sha_bucket_shift = (int)value;
    return 0;
  }
  if (!strcmp(key, "sha_short_blocks")) {  // A/B: the lean kernel takes an ordered batch's messages of <= N blocks
    if (value < 0 || value > 127) return lsmck_host::set_error(LSMCK_EINVAL, "sha_short_blocks: 0..127");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->sha_short_blocks = (int)value;
    return 0;
  }



  if (!strcmp(key, "sha_pair")) {  // A/B: SHA-256 batch kernel loads two blocks (a 128-B line) per window
    // 2: diagnostic, the pair kernel's main loop without payload loads (digests invalid);
    // 3: line-aligned loads realigned through LDS rows
    if (value < 0 || value > 3) return lsmck_host::set_error(LSMCK_EINVAL, "sha_pair must be 0..3");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->sha_pair = (int)value;
    return 0;
  }
  if (!strcmp(key, "sha_order")) {  // A/B: 1 = variable-length SHA batches in decreasing length order (default)
    if (value != 0 && value != 1) return lsmck_host::set_error(LSMCK_EINVAL, "sha_order must be 0 or 1");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->variant = (ctx->variant & ~0x10000) | (value ? 0 : 0x10000);
    return 0;
  }
  if (!strcmp(key, "crc_stream")) {  // A/B: descriptor batches, 1 = stream kernel for sorted batches (default),
                                     // 0 = walking kernel only, 2 = stream kernel only (diagnostic: a declined
                                     // caller batch gets no CRCs)
    if (value < 0 || value > 2) return lsmck_host::set_error(LSMCK_EINVAL, "crc_stream must be 0, 1 or 2");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->variant = (ctx->variant & ~(kVariantNoStream | kVariantStreamOnly)) |
                   (value == 0 ? kVariantNoStream : value == 2 ? kVariantStreamOnly : 0);
    return 0;
  }
  return lsmck_host::set_error(LSMCK_EINVAL, "unknown option");
}

int lsmck_ctx_get_stat(lsmck_ctx* ctx, const char* key, long* value) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!key || !value) return lsmck_host::set_error(LSMCK_EINVAL, "null key or value");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!strcmp(key, "wal_walk_path")) {
    *value = ctx->last_walk_path.load();
  } else if (!strcmp(key, "wal_seg_repairs")) {
    *value = ctx->last_seg_repairs.load();
  } else if (!strcmp(key, "wal_segments")) {
    *value = (long)ctx->last_segments.load();
  } else if (!strcmp(key, "wal_seg_prepairs")) {  // the last segment walk's parallel repair rounds
    *value = ctx->last_seg_prepairs.load();
  } else if (!strcmp(key, "wal_pipe_parts")) {  // the last device replay's pipelined parts (0: one walk, one pass)
    *value = ctx->last_pipe_parts.load();
  } else if (!strcmp(key, "wal_recs_dma")) {  // the last records read-back: SDMA engines (0: hipMemcpyAsync)
    *value = ctx->last_recs_dma.load();
  } else if (!strcmp(key, "numa_node")) {
    *value = ctx->numa_node;
  } else if (!strcmp(key, "stage_numa_node")) {
    *value = ctx->pin_node;
  } else {
    return lsmck_host::set_error(LSMCK_EINVAL, "unknown stat");
  }
  return 0;
}

void lsmck_ctx_destroy(lsmck_ctx* ctx) {
  if (!ctx) return;
  DevGuard g(ctx->dev);
  (void)hipDeviceSynchronize();
  for (auto& S : ctx->stage) S.release();
  ctx->scratch.release();
  if (ctx->tree.state) (void)hipFree(ctx->tree.state);
  if (ctx->tree.digests) (void)hipFree(ctx->tree.digests);
  if (ctx->tree.kernel_done) (void)hipEventDestroy(ctx->tree.kernel_done);
  if (ctx->d_master) (void)hipFree(ctx->d_master);
  if (ctx->d_kseg) (void)hipFree(ctx->d_kseg);
  if (ctx->d_khi) (void)hipFree(ctx->d_khi);
  if (ctx->d_tinit) (void)hipFree(ctx->d_tinit);
  if (ctx->d_zero) (void)hipFree(ctx->d_zero);
  if (ctx->d_verify) (void)hipFree(ctx->d_verify);
  for (void* p : {(void*)ctx->wd.bits, (void*)ctx->wd.pre, (void*)ctx->wd.bsum, (void*)ctx->wd.pos, (void*)ctx->wd.J,
                  (void*)ctx->wd.badpos, (void*)ctx->wd.chain, (void*)ctx->wd.recs, (void*)ctx->wd.info})
    if (p) (void)hipFree(p);
  if (ctx->wd.h_info) host_free(ctx->wd.h_info);
  for (void* p : {(void*)ctx->wd.sg, (void*)ctx->wd.sx, (void*)ctx->wd.spre, (void*)ctx->wd.scode,
                  (void*)ctx->wd.srecs, (void*)ctx->wd.sbsum, (void*)ctx->wd.sinfo, (void*)ctx->wd.scpp,
                  (void*)ctx->wd.scpc, (void*)ctx->wd.sst, (void*)ctx->wd.sg0, (void*)ctx->wd.sx0,
                  (void*)ctx->wd.scode0})
    if (p) (void)hipFree(p);
  if (ctx->wd.h_sinfo) host_free(ctx->wd.h_sinfo);
  for (void* p : {(void*)ctx->d_vcrc, (void*)ctx->d_woff, (void*)ctx->d_wlen, (void*)ctx->d_wexp})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)ctx->h_woff, (void*)ctx->h_wlen, (void*)ctx->h_wexp})
    if (p) host_free(p);
  if (ctx->h_verify) host_free(ctx->h_verify);
  if (ctx->h_wrecs) host_free(ctx->h_wrecs);
  if (ctx->wd.recs16) (void)hipFree(ctx->wd.recs16);
  lsmck_dma::destroy(ctx->dma);
  if (ctx->wal_emit_ev) (void)hipEventDestroy(ctx->wal_emit_ev);
  if (ctx->h_wrecs1) host_free(ctx->h_wrecs1);
  if (ctx->wal_emit1_ev) (void)hipEventDestroy(ctx->wal_emit1_ev);
  if (ctx->wal_rs) (void)hipStreamDestroy(ctx->wal_rs);
  if (ctx->wal_pw) (void)hipStreamDestroy(ctx->wal_pw);
  if (ctx->wal_pc) (void)hipStreamDestroy(ctx->wal_pc);
  for (hipEvent_t e : ctx->wal_pipe_ev) (void)hipEventDestroy(e);
  if (ctx->wal_host) host_free(ctx->wal_host);
  if (ctx->d_wimg) (void)hipFree(ctx->d_wimg);
  if (ctx->scratch_ev) (void)hipEventDestroy(ctx->scratch_ev);
  if (ctx->stream0) (void)hipStreamDestroy(ctx->stream0);
  delete ctx;
}

int lsmck_crc32_batch(lsmck_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint32_t* len, size_t n,
                      uint32_t* out, unsigned flags, void* stream) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (n && (!off || !len || !out)) return lsmck_host::set_error(LSMCK_EINVAL, "null descriptor or output");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DevGuard g(ctx->dev);
  if (flags & LSMCK_DEVICE) {
    ScratchOrder so(ctx, pick_stream(ctx, stream));
    if (so.e != hipSuccess) return hip_error(so.e, "hipStreamWaitEvent(scratch)");
    return crc_desc_device(ctx, ctx->scratch, base, off, len, n, out, so.st, (flags & LSMCK_SORTED) != 0);
  }
  HostJob J{CRC, base, off, len, 0, 0, n, (uint8_t*)out, (flags & LSMCK_HOST_PINNED) != 0};
  return run_host_job(ctx, J);
}

int lsmck_crc32_batch_fixed(lsmck_ctx* ctx, const uint8_t* base, size_t stride, uint32_t len, size_t n,
                            uint32_t* out, unsigned flags, void* stream) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (n && !out) return lsmck_host::set_error(LSMCK_EINVAL, "null output");
  if (n > 1 && stride < len) return lsmck_host::set_error(LSMCK_EINVAL, "stride < len");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DevGuard g(ctx->dev);
  if (flags & LSMCK_DEVICE) return crc_fixed_device(ctx, base, stride, len, n, out, pick_stream(ctx, stream));
  HostJob J{CRC, base, nullptr, nullptr, stride, len, n, (uint8_t*)out, (flags & LSMCK_HOST_PINNED) != 0};
  return run_host_job(ctx, J);
}

int lsmck_crc32_verify_batch(lsmck_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint32_t* len,
                             const uint32_t* expected, size_t n, unsigned flags, void* stream, uint64_t* n_bad,
                             uint64_t* first_bad) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (flags & LSMCK_DEVICE) {
    if (n && (!off || !len || !expected)) return lsmck_host::set_error(LSMCK_EINVAL, "null descriptor or expected");
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard g(ctx->dev);
    ScratchOrder so(ctx, pick_stream(ctx, stream));
    if (so.e != hipSuccess) return hip_error(so.e, "hipStreamWaitEvent(scratch)");
    rc = device_verify(ctx, base, off, len, expected, n, so.st, n_bad, first_bad, (flags & LSMCK_SORTED) != 0);
    return rc;
  }
  std::vector<uint32_t> crc(n);
  rc = lsmck_crc32_batch(ctx, base, off, len, n, crc.data(), flags, stream);
  if (rc) return rc;
  uint64_t bad = 0, first = n;
  for (size_t i = 0; i < n; ++i)
    if (crc[i] != expected[i]) {
      if (!bad) first = i;
      ++bad;
    }
  if (n_bad) *n_bad = bad;
  if (first_bad) *first_bad = first;
  return bad ? 1 : 0;
}

int lsmck_sha256_batch(lsmck_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint32_t* len, size_t n,
                       uint8_t* out32, unsigned flags, void* stream) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (n && (!off || !len || !out32)) return lsmck_host::set_error(LSMCK_EINVAL, "null descriptor or output");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DevGuard g(ctx->dev);
  if (flags & LSMCK_DEVICE) {
    ScratchOrder so(ctx, pick_stream(ctx, stream));
    if (so.e != hipSuccess) return hip_error(so.e, "hipStreamWaitEvent(scratch)");
    return sha_device(ctx, ctx->scratch, base, off, len, 0, 0, n, out32, so.st);
  }
  HostJob J{SHA, base, off, len, 0, 0, n, out32, (flags & LSMCK_HOST_PINNED) != 0};
  return run_host_job(ctx, J);
}

int lsmck_sha256_batch_fixed(lsmck_ctx* ctx, const uint8_t* base, size_t stride, uint32_t len, size_t n,
                             uint8_t* out32, unsigned flags, void* stream) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (n && !out32) return lsmck_host::set_error(LSMCK_EINVAL, "null output");
  std::lock_guard<std::mutex> lk(ctx->mu);
  DevGuard g(ctx->dev);
  if (flags & LSMCK_DEVICE) {
    ScratchOrder so(ctx, pick_stream(ctx, stream));
    if (so.e != hipSuccess) return hip_error(so.e, "hipStreamWaitEvent(scratch)");
    return sha_device(ctx, ctx->scratch, base, nullptr, nullptr, stride, len, n, out32, so.st);
  }
  HostJob J{SHA, base, nullptr, nullptr, stride, len, n, out32, (flags & LSMCK_HOST_PINNED) != 0};
  return run_host_job(ctx, J);
}

// ---------------------------------------------------------------------------
// WAL replay verify (src/wal.rs:68-84, 122-163; src/memtable.rs:28-47)
static uint32_t rd_u32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

}  // extern "C"

// WAL replay of a device-resident image with the header walk on the GPU
// (lsmck_wal.hip): nothing of the image comes back to the host, only the
// accepted records (32 B each) and a few counters.
static int wal_bitmap_ensure(lsmck_ctx* ctx, size_t n) {
  auto& W = ctx->wd;
  int rc;
  const size_t nw = (size_t)lsmk_wal_words(n), nb = (size_t)lsmk_wal_scan_blocks(n);
  if ((rc = ensure_dev(&W.bits, &W.cap_bits, std::max<size_t>(nw, 1))) ||
      (rc = ensure_dev(&W.pre, &W.cap_pre, std::max<size_t>(nw, 1))) ||
      (rc = ensure_dev(&W.bsum, &W.cap_bsum, nb + 1)))
    return rc;
  return 0;
}

// LSMCK_WAL_TRACE=1: the replay's phases on stderr (seconds since the call began)
struct WalTrace {
  bool on = getenv("LSMCK_WAL_TRACE") != nullptr;
  timespec t0{};
  WalTrace() { clock_gettime(CLOCK_MONOTONIC, &t0); }
  void mark(const char* what) const {
    if (!on) return;
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    fprintf(stderr, "wal_trace %-24s %.6f\n", what, (double)(t.tv_sec - t0.tv_sec) + 1e-9 * (double)(t.tv_nsec - t0.tv_nsec));
  }
};

// One header walk over the candidates of words [w0, w1), from position
// `start` (a prefix walk when lim < n: lsmck_wal.hip wal_succ), its records
// emitted at index `at` of the record / descriptor arrays.  Caller holds
// ctx->mu; st is ordered after the scratch users.
struct WalPart {
  size_t m = 0;        // records
  uint32_t term = 0;   // terminal code (WAL_END / BAD / STOP / STOPSELF, lsmck_wal.hip)
  uint64_t tpos = 0;   // BAD position, or where a prefix walk resumes
  double over = 0;     // kWalTooBig: the scratch it needed over the budget (ratio)
  bool packed = false; // the segment walk emitted packed CRC spans (seg::Pack) from `at` on
};
constexpr uint32_t kWalBad = 0xFFFFFFFEu, kWalStop = 0xFFFFFFFDu, kWalStopSelf = 0xFFFFFFFCu;

static int wal_walk_part(lsmck_ctx* ctx, const uint8_t* img, size_t n, uint64_t w0, uint64_t w1, uint64_t start,
                         uint64_t lim, bool marked, size_t at, hipStream_t st, WalPart* out, const WalTrace& tr) {
  auto& W = ctx->wd;
  int rc;
  uint32_t* d_total = (uint32_t*)(W.info + 3);
  HIPCHK(hipMemsetAsync(d_total, 0, 4, st));
  rc = lsmk_wal_mark(img, n, W.bits, W.pre, W.bsum, d_total, marked ? 1 : 0, w0, w1, st);
  if (rc) return launch_rc(rc, "wal mark/scan kernels");
  HIPCHK(hipMemcpyAsync(W.h_info + 3, d_total, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  tr.mark("mark+scan (sync)");
  const uint64_t nc64 = W.h_info[3] & 0xFFFFFFFFull;
  // The jump tables grow with the CANDIDATE count -- every 0x01/0x02 byte
  // that could start a header -- not with the record count: a valid log whose
  // payloads are dense in those bytes needs up to ~120x its size (levels x nc
  // x 4 B of J alone), and past 2^31 candidates the u32 ranks would reach the
  // terminal codes.  Over a budget, or when an allocation fails, this walk
  // declines (kWalTooBig) and the caller walks the log in smaller parts.
  if (nc64 >= (1ull << 31)) {
    out->over = (double)nc64 / (double)(1ull << 30);
    return kWalTooBig;
  }
  const uint32_t nc = (uint32_t)nc64;
  int levels = 0;
  while ((1ull << levels) <= nc) ++levels;  // 2^levels > nc, levels <= 31
  const size_t need = (size_t)nc * (8 + 8 + 4 * (size_t)levels) + ((size_t)4 << levels);
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
  const size_t budget = std::min(free_b / 2, ctx->wal_walk_budget_per_byte * n + ((size_t)256 << 20));
  if (need > budget) {
    out->over = (double)need / (double)std::max<size_t>(budget, 1);
    return kWalTooBig;
  }
  if (ensure_dev(&W.pos, &W.cap_pos, std::max<size_t>(nc, 1)) ||
      ensure_dev(&W.J, &W.cap_J, std::max<size_t>((size_t)levels * nc, 1)) ||
      ensure_dev(&W.badpos, &W.cap_badpos, std::max<size_t>(nc, 1)) ||
      ensure_dev(&W.chain, &W.cap_chain, (size_t)1 << levels)) {
    (void)hipGetLastError();  // the failed hipMalloc's sticky error
    out->over = 2.0;
    return kWalTooBig;
  }
  rc = lsmk_wal_chain(img, n, W.bits, W.pre, nc, levels, W.pos, W.J, W.badpos, W.chain, W.info, w0, w1, start, lim,
                      st);
  if (rc) return launch_rc(rc, "wal chain kernels");
  HIPCHK(hipMemcpyAsync(W.h_info, W.info, 24, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  tr.mark("chain (sync)");
  out->m = (size_t)W.h_info[0];
  out->term = (uint32_t)W.h_info[1];
  out->tpos = W.h_info[2];
  if (out->m) {  // records -> lsmck_wal_rec, payload descriptors, stored CRCs (after the first `at`)
    const size_t tot = at + out->m;
    if ((rc = ensure_dev_keep(&W.recs, &W.cap_recs, tot, at, st)) ||
        (rc = ensure_dev_keep(&ctx->d_woff, &ctx->cap_woff, tot, at, st)) ||
        (rc = ensure_dev_keep(&ctx->d_wlen, &ctx->cap_wlen, tot, at, st)) ||
        (rc = ensure_dev_keep(&ctx->d_wexp, &ctx->cap_wexp, tot, at, st)) ||
        (rc = ensure_dev_keep(&ctx->d_vcrc, &ctx->cap_vcrc, tot, at, st)))
      return rc;
    rc = lsmk_wal_emit(img, n, W.chain, W.pos, W.info, (uint32_t)out->m, W.recs + at, ctx->d_woff + at,
                       ctx->d_wlen + at, ctx->d_wexp + at, st);
    if (rc) return launch_rc(rc, "wal emit kernel");
    if (ctx->wal_compact) {  // the caller's layout: lsmck_wal_rec16 (the segment walk emits it directly)
      if ((rc = ensure_dev_keep(&W.recs16, &W.cap_recs16, tot, at, st))) return rc;
      if ((rc = lsmk_wal_recs_compact(W.recs + at, W.recs16 + at, out->m, st)))
        return launch_rc(rc, "wal record compaction kernel");
    }
  }
  return 0;
}

// The CRC pass over records [at, at + m): their spans in log order (the
// stream kernel, no eligibility check), CRCs into d_vcrc + at.  (Packed spans,
// seg::Pack, are taken apart by the compare, wal_finish.)  Asynchronous.
static int wal_crc_part(lsmck_ctx* ctx, const uint8_t* img, size_t at, size_t m, hipStream_t st, int ncu = 0) {
  if (!m) return 0;
  return crc_desc_device(ctx, ctx->scratch, img, ctx->d_woff + at, ctx->d_wlen + at, m, ctx->d_vcrc + at, st, true,
                         ncu);
}

// This replay's record layout: bytes per record (lsmck_wal_rec, or
// lsmck_wal_rec16 for lsmck_wal_replay_verify16).
static size_t wal_rec_size(const lsmck_ctx* ctx) {
  return ctx->wal_compact ? sizeof(lsmck_wal_rec16) : sizeof(lsmck_wal_rec);
}

// the context's SDMA copier (lsmck_dma.h), made on first use; nullptr: none
static lsmck_dma::Copier* dma_copier(lsmck_ctx* ctx) {
  if (!ctx->dma_tried) {
    ctx->dma_tried = true;
    ctx->dma = lsmck_dma::create(ctx->d_verify);  // (any allocation of the device names its agent)
  }
  return ctx->dma;
}

// Record i of this replay as an lsmck_wal_rec, read from the device array src
// (compact: its 16 bytes, and the stored CRC from its header in the image).
static int wal_dev_rec(lsmck_ctx* ctx, const uint8_t* img, const uint8_t* src, size_t i, lsmck_wal_rec* r) {
  if (!ctx->wal_compact) {
    HIPCHK(hipMemcpy(r, src + i * sizeof(lsmck_wal_rec), sizeof *r, hipMemcpyDeviceToHost));
    return 0;
  }
  lsmck_wal_rec16 c;
  HIPCHK(hipMemcpy(&c, src + i * sizeof c, sizeof c, hipMemcpyDeviceToHost));
  r->type = (c.payload_type & LSMCK_WAL_REC16_REMOVE) ? 2u : 1u;
  r->payload_off = c.payload_type & LSMCK_WAL_REC16_OFF_MASK;
  r->rec_off = r->payload_off - lsmck::seg::hdr_len(r->type);
  r->klen = c.klen;
  r->vlen = c.vlen;
  uint8_t h[4];
  HIPCHK(hipMemcpy(h, img + r->rec_off + 1, 4, hipMemcpyDeviceToHost));
  r->crc = (uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 24);
  return 0;
}

// The records' read-back beside the CRC pass: `bytes` of the device array
// src into the page-locked `land` once the emit is done (ctx->wal_emit_ev),
// dealt over "wal_dma_engines" SDMA engines (lsmck_dma.h) -- no copy kernel
// on the CUs beside the CRC pass -- or, without them, by hipMemcpyAsync on
// the staging stream.  out (pageable, or null): where the records go from
// `land`, copied on host threads piece by piece as the pieces land.
// Returns once all of it is in place.
static int wal_read_back(lsmck_ctx* ctx, uint8_t* land, const uint8_t* src, size_t bytes, uint8_t* out) {
  HIPCHK(hipEventSynchronize(ctx->wal_emit_ev));
  auto copy_out = [&](size_t a, size_t b) {  // land [a, b) -> out, several threads for large pieces
    const size_t len = b - a;
    const unsigned T = len >= (4u << 20) ? std::max(1u, std::min(ctx->stage_threads, 8u)) : 1u;
    host_pool(ctx).run(T, [&](unsigned t) {
      const size_t x = a + (len * t / T & ~(size_t)4095), y = t + 1 == T ? b : a + (len * (t + 1) / T & ~(size_t)4095);
      if (y > x) memcpy(out + x, land + x, y - x);
    });
  };
  lsmck_dma::Copier* dc = ctx->wal_dma_engines ? dma_copier(ctx) : nullptr;
  lsmck_dma::Job job;
  if (dc && lsmck_dma::d2h(dc, land, src, bytes, ctx->wal_dma_engines, ctx->wal_dma_chunks, &job) == 0) {
    const int E = std::max(1, std::min(ctx->wal_dma_engines, lsmck_dma::engines(dc)));
    ctx->last_recs_dma = E;
    int werr = 0;
    for (int i = 0; i < job.n;) {  // (a round: the next piece of every engine)
      const int i1 = std::min(job.n, i + E);
      for (int k = i; k < i1; ++k)
        if (lsmck_dma::wait(dc, job, k) && !werr) werr = 1;
      if (out && !werr) copy_out(job.off[i], job.off[i1]);
      i = i1;
    }
    if (werr) return lsmck_host::set_error(LSMCK_EIO, "SDMA copy of the WAL records failed");
    return 0;
  }
  ctx->last_recs_dma = 0;
  int rc;
  if ((rc = stage_init(ctx->stage[0]))) return rc;
  HIPCHK(hipMemcpyAsync(land, src, bytes, hipMemcpyDeviceToHost, ctx->stage[0].s));
  HIPCHK(hipStreamSynchronize(ctx->stage[0].s));
  if (out) copy_out(0, bytes);
  return 0;
}

// After the CRC pass of all m records: the compare, the records to the caller
// (read back beside the compare and copied out on host threads), and the
// replay's outcome (the first bad record in log order, or a bad type byte
// after the last record at badq).
// done: records [0, done) are already in the caller's array (the split
// replay's first part); the rest are read back from the device.
// emit_recorded: ctx->wal_emit_ev marks the end of the emit (the segment
// walk); otherwise the read-back waits for everything queued on st so far.
// pack_from: records [pack_from, m) have packed CRC spans (the segment walk's
// emit, seg::Pack): their expected CRCs are the spans' (seg::pack_crc), and a
// bad one's computed CRC is taken back to its payload's for the report.
static int wal_finish(lsmck_ctx* ctx, const uint8_t* img, size_t m, uint32_t term, uint64_t badq, void* recs,
                      size_t cap, size_t* nrec, uint64_t* bad_index, uint32_t* bad_crc, uint32_t* bad_expected,
                      hipStream_t st, const WalTrace& tr, size_t done = 0, bool emit_recorded = false,
                      size_t pack_from = ~(size_t)0, const std::vector<size_t>* unpacked = nullptr) {
  auto& W = ctx->wd;
  int rc;
  uint64_t nbad = 0, first = m;
  const size_t rsz = wal_rec_size(ctx);
  ctx->last_recs_dma = 0;
  // the device array that holds records [0, m): the caller's when the emit wrote them there
  const uint8_t* dsrc = ctx->wal_recs_dev && ctx->wal_recs_dev_emitted ? (const uint8_t*)recs
                        : ctx->wal_compact                             ? (const uint8_t*)W.recs16
                                                                       : (const uint8_t*)W.recs;
  if (m) {
    const size_t ntake = std::min(m, cap) > done ? std::min(m, cap) - done : 0;  // records for the caller's array
    uint8_t* const rb = (uint8_t*)recs;
    uint8_t* land = nullptr;  // the read-back's page-locked landing: the caller's array or ctx->h_wrecs
    if (ctx->wal_recs_dev) {
      // LSMCK_RECS_DEVICE: the records stay on the device (emitted there, or
      // copied from the walk's own array); nothing crosses the link
      if (recs && ntake && !ctx->wal_recs_dev_emitted)
        HIPCHK(hipMemcpyAsync(rb + done * rsz, dsrc + done * rsz, ntake * rsz, hipMemcpyDeviceToDevice, st));
    } else if (recs && ntake) {
      if (ctx->wal_recs_direct) {
        land = rb + done * rsz;  // page-locked (LSMCK_RECS_PINNED): straight in
      } else {
        if ((rc = ensure_pinned(ctx->pin_node, &ctx->h_wrecs, &ctx->cap_hwrecs, ntake * rsz))) return rc;
        land = ctx->h_wrecs;
      }
      if (!ctx->wal_emit_ev) HIPCHK(hipEventCreateWithFlags(&ctx->wal_emit_ev, hipEventDisableTiming));
      if (!emit_recorded) HIPCHK(hipEventRecord(ctx->wal_emit_ev, st));
    }
    HIPCHK(hipMemsetAsync(ctx->d_verify, 0, 8, st));         // n_bad
    HIPCHK(hipMemsetAsync(ctx->d_verify + 1, 0xFF, 8, st));  // first_bad = ~0
    rc = lsmk_launch_crc32_compare(ctx->d_vcrc, ctx->d_wexp, m, ctx->d_verify, ctx->d_verify + 1, st);
    if (rc) return launch_rc(rc, "compare kernel");
    HIPCHK(hipMemcpyAsync(ctx->h_verify, ctx->d_verify, 16, hipMemcpyDeviceToHost, st));
    const int hrc = land ? wal_read_back(ctx, land, dsrc + done * rsz, ntake * rsz,
                                         ctx->wal_recs_direct ? nullptr : rb + done * rsz)
                         : 0;
    HIPCHK(hipStreamSynchronize(st));
    if (hrc) return hrc;
    nbad = ctx->h_verify[0];
    first = nbad ? ctx->h_verify[1] : m;
  }
  tr.mark("crc+compare+records (sync)");
  const size_t accepted = nbad ? (size_t)first : m;
  if (nrec) *nrec = accepted;
  if (nbad) {  // the report, from the device's copy of the records
    lsmck_wal_rec r;
    uint32_t got = 0;
    if ((rc = wal_dev_rec(ctx, img, dsrc, first, &r))) return rc;
    HIPCHK(hipMemcpy(&got, ctx->d_vcrc + first, 4, hipMemcpyDeviceToHost));
    // (unpacked: the pipelined parts' last records, whose spans are their payloads alone)
    const bool alone = unpacked && std::binary_search(unpacked->begin(), unpacked->end(), (size_t)first);
    if (first >= pack_from && first + 1 < m && !alone) {  // a packed span's CRC: the next header taken back out
      namespace sg = lsmck::seg;
      lsmck_wal_rec rn;
      if ((rc = wal_dev_rec(ctx, img, dsrc, first + 1, &rn))) return rc;
      if (sg::pack_fits(r.klen + r.vlen, sg::hdr_len(rn.type))) {
        sg::Head nh{};
        nh.t = rn.type;
        nh.crc = rn.crc;
        nh.klen = rn.klen;
        nh.vlen = rn.vlen;
        got = sg::unpack_crc(got, nh, lsmck_host::crc_tables());
      }
    }
    if (bad_index) *bad_index = first;
    if (bad_expected) *bad_expected = r.crc;
    if (bad_crc) *bad_crc = got;
    return r.type == 1 ? LSMCK_WAL_CORRUPTED : LSMCK_WAL_REMOVE_PANIC;
  }
  if (term == kWalBad) {  // InvalidCommandType at the record after the last one
    uint8_t t = 0;
    HIPCHK(hipMemcpy(&t, img + badq, 1, hipMemcpyDeviceToHost));
    if (bad_index) *bad_index = m;
    if (bad_crc) *bad_crc = t;
    return LSMCK_WAL_BAD_TYPE;
  }
  return 0;
}

static int wal_walk_setup(lsmck_ctx* ctx, size_t n) {
  auto& W = ctx->wd;
  int rc;
  if ((rc = wal_bitmap_ensure(ctx, n))) return rc;
  if (!W.info) HIPCHK(hipMalloc((void**)&W.info, 64));
  if (!W.h_info) HIPCHK(hipHostMalloc((void**)&W.h_info, 64, hipHostMallocDefault));
  return 0;
}

// The walk from position r to the end of the image in parts: each part is a
// prefix walk over [r, a) (a = r + part, or the end) that resumes where the
// previous one stopped, its records emitted after the `at` already there and
// their CRC pass launched.  part 0: the whole rest in one walk first.  A part
// whose jump tables do not fit (kWalTooBig) is cut to fit and walked again; a
// record longer than the part doubles the part.  So the walk's scratch stays
// within its budget and the log may exceed the u32 candidate ranks.  Marks
// each part's words first unless `marked` (the whole image is marked).
static int wal_walk_from(lsmck_ctx* ctx, const uint8_t* img, size_t n, uint64_t r, size_t at, size_t part,
                         bool marked, hipStream_t st, const WalTrace& tr, WalPart* out) {
  auto& W = ctx->wd;
  int rc;
  const uint64_t nw = lsmk_wal_words(n);
  constexpr size_t kMinPart = 1u << 20;
  if (!part && n - r >= (1ull << 32)) part = (size_t)1 << 31;  // (per-part ranks are u32)
  for (;;) {
    const uint64_t a = (part && n - r > part) ? ((r + part) & ~(uint64_t)63) : n;
    if (!marked && (rc = lsmk_wal_mark_range(img, n, r & ~(uint64_t)63, a, W.bits, W.pre, st)))
      return launch_rc(rc, "wal mark kernel");
    WalPart P;
    rc = wal_walk_part(ctx, img, n, r >> 6, a == n ? nw : a >> 6, r, a, true, at, st, &P, tr);
    if (rc == kWalTooBig) {
      const size_t cur = (size_t)(a - r);
      size_t next = (size_t)((double)cur / (2.0 * std::max(P.over, 1.0)));
      next &= ~(size_t)(kMinPart - 1);
      if (next < kMinPart) {
        if (cur <= kMinPart) return kWalHostWalk;  // even a 1 MiB part is too dense: the host walk
        next = kMinPart;
      }
      part = next;
      marked = false;  // (the scan of the declined part replaced its words' counts)
      continue;
    }
    if (rc) return rc;
    if ((rc = wal_crc_part(ctx, img, at, P.m, st))) return rc;
    at += P.m;
    if (a == n || (P.term != kWalStop && P.term != kWalStopSelf)) {
      out->m = at;
      out->term = P.term;
      out->tpos = P.tpos;
      return 0;
    }
    if (P.term == kWalStopSelf && P.tpos == r) {  // a record longer than the part: a longer part
      part = std::min<size_t>((size_t)(n - r), part * 2);
      marked = false;
      continue;
    }
    r = P.tpos;
    marked = false;  // the next part re-marks its words: the scan replaced the counts of [r, a)
  }
}

// The segment walk (lsmck_segwalk.h) of the chain from `start`: the records
// that start in [start, lim) (lim = n: to the end of the image) -- every
// segment's guess and walk, check rounds (one host sync each; a failure is
// repaired on the device and checked again), then the records emitted after
// the `at` already there, the emit's completion recorded on
// ctx->wal_emit_ev (the records' read-back waits for that, not for the CRC
// pass behind it).  out->term: END / kWalBad where the chain ends, or
// kWalStop with out->tpos = the first record start at or past lim (the next
// prefix starts there).  kWalSegDecline: more failures than wal_seg_rounds --
// payloads that look like framed records along the chain; the caller walks
// by candidate doubling instead.
constexpr int kWalSegDecline = 0x7FFF0004;
// internal: a pipelined part's records no longer fit the caller's device array
// the earlier parts were emitted into (the replay starts over, not pipelined)
constexpr int kWalPipeRestart = 0x7FFF0005;
static int wal_seg_walk(lsmck_ctx* ctx, const uint8_t* img, size_t n, uint64_t start, uint64_t lim, size_t at,
                        hipStream_t st, const WalTrace& tr, WalPart* out) {
  namespace sg = lsmck::seg;
  auto& W = ctx->wd;
  int rc;
  ctx->last_walk_path = 1;
  ctx->last_seg_repairs = 0;
  ctx->last_segments = 0;
  if (start >= n) {
    out->m = at;
    out->term = 0xFFFFFFFFu;  // END
    out->tpos = 0;
    return 0;
  }
  if (lim > n || lim <= start) lim = n;
  uint64_t S = lsmk_wal_seg_bytes(lim - start, ctx->wal_seg_bytes ? ctx->wal_seg_bytes : ctx->wal_seg_auto);
  sg::SegArgs a{};
  int resegs = 0, prepairs = 0, repairs = 0;
  ctx->last_seg_prepairs = 0;
  for (bool walk = true;;) {
    if (walk) {  // (re)segment and walk every segment
      walk = false;
      prepairs = repairs = 0;
      const uint64_t K64 = (lim - start + S - 1) / S;
      if (K64 >= (1ull << 31)) return kWalSegDecline;  // (tiny forced segments over a huge log)
      const uint32_t K = (uint32_t)K64;
      ctx->last_segments = K;
      // The walk's own arrays (~40 B per segment).  An allocation that fails
      // (a log that nearly fills HBM) declines to the candidate-doubling walk,
      // whose scratch is budgeted against the free memory, instead of failing
      // the replay: the failed hipMalloc's sticky error is cleared first.
      auto alloc_fail = [&]() {
        (void)hipGetLastError();
        return kWalSegDecline;
      };
      if (ensure_dev(&W.sbsum, &W.cap_sbsum, (size_t)lsmk_wal_seg_scan_blocks(K) + 1)) return alloc_fail();
      if (W.cap_seg < (size_t)K + 1) {
        for (void* p : {(void*)W.sg, (void*)W.sx, (void*)W.spre, (void*)W.scode, (void*)W.srecs})
          if (p) (void)hipFree(p);
        const size_t c = std::max<size_t>((size_t)K + 1, W.cap_seg * 3 / 2);
        W.sg = W.sx = W.spre = nullptr;
        W.scode = W.srecs = nullptr;
        W.cap_seg = 0;
        if (hipMalloc((void**)&W.sg, c * 8) != hipSuccess || hipMalloc((void**)&W.sx, c * 8) != hipSuccess ||
            hipMalloc((void**)&W.spre, c * 8) != hipSuccess || hipMalloc((void**)&W.scode, c * 4) != hipSuccess ||
            hipMalloc((void**)&W.srecs, c * 4) != hipSuccess) {
          for (void** p : {(void**)&W.sg, (void**)&W.sx, (void**)&W.spre, (void**)&W.scode, (void**)&W.srecs}) {
            if (*p) (void)hipFree(*p);
            *p = nullptr;
          }
          return alloc_fail();
        }
        W.cap_seg = c;
      }
      if (!W.sinfo && hipMalloc((void**)&W.sinfo, sg::kInfoWords * 8) != hipSuccess) {
        W.sinfo = nullptr;
        return alloc_fail();
      }
      if (!W.h_sinfo && hipHostMalloc((void**)&W.h_sinfo, sg::kInfoWords * 8, hipHostMallocDefault) != hipSuccess) {
        W.h_sinfo = nullptr;
        return alloc_fail();
      }
      // the emit from checkpoints every 64 KiB (up to 32 per segment): its
      // walks run 32x as many threads, each a 32nd as long
      const uint32_t nsub = S >= (128u << 10) ? (uint32_t)std::min<uint64_t>(32, S >> 16) : 1u;
      if (nsub > 1 && W.cap_cp < (size_t)K * nsub) {
        for (void* p : {(void*)W.scpp, (void*)W.scpc})
          if (p) (void)hipFree(p);
        W.scpp = nullptr;
        W.scpc = nullptr;
        W.cap_cp = 0;
        const size_t c = (size_t)K * nsub;
        if (hipMalloc((void**)&W.scpp, c * 8) != hipSuccess || hipMalloc((void**)&W.scpc, c * 4) != hipSuccess) {
          if (W.scpp) (void)hipFree(W.scpp);
          if (W.scpc) (void)hipFree(W.scpc);
          W.scpp = nullptr;
          W.scpc = nullptr;
          return alloc_fail();
        }
        W.cap_cp = c;
      }
      // the walk stages each segment's records in scap slots (auto: an
      // eighth of the walked bytes, 64 MiB .. 8 GiB, over the segments, and
      // at most a quarter of the free device memory (less the records'
      // arrays still to come); at most the records a segment can hold); a
      // segment with more is emitted by a second walk of its headers, and so
      // is every segment when the slots cannot be had (scap 0)
      uint32_t scap = 0;
      if (ctx->wal_seg_stage && S <= sg::kStageMaxSeg) {  // (a staged record keeps its offset in 31 bits)
        const uint64_t most = S / 9 + 1;
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
        const uint64_t have = W.sst ? (uint64_t)W.cap_sst * sizeof(sg::StageRec) : 0;  // (reused, not new)
        const uint64_t budget = std::min<uint64_t>(
            std::min<uint64_t>(std::max<uint64_t>((lim - start) / 8, 64ull << 20), 8ull << 30),
            (uint64_t)free_b / 4 + have);
        const uint64_t c = std::min<uint64_t>(most, ctx->wal_seg_stage >= 2 ? (uint64_t)ctx->wal_seg_stage
                                                                               : budget / (sizeof(sg::StageRec) * K));
        if (c >= 1) {
          scap = (uint32_t)c;
          if (ensure_dev(&W.sst, &W.cap_sst, (size_t)K * scap)) {
            (void)hipGetLastError();  // no slots: every segment is emitted by its second walk
            scap = 0;
          }
        }
      }
      a = sg::SegArgs{img, n, start, S, K, W.sg, W.sx, W.scode, W.srecs, W.spre, W.sinfo, lim,
                      nsub, S / nsub, nsub > 1 ? W.scpp : nullptr, nsub > 1 ? W.scpc : nullptr,
                      scap ? W.sst : nullptr, scap};
      if ((rc = lsmk_wal_seg_walk(&a, st))) return launch_rc(rc, "wal segment walk kernel");
    }
    if ((rc = lsmk_wal_seg_round(&a, W.sbsum, st))) return launch_rc(rc, "wal segment check kernels");
    HIPCHK(hipMemcpyAsync(W.h_sinfo, W.sinfo, sg::kInfoWords * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    tr.mark("segment walk round (sync)");
    if ((uint32_t)W.h_sinfo[sg::kInfoFail] == sg::kNoSeg) break;
    const uint32_t nfail = (uint32_t)W.h_sinfo[sg::kInfoNFail];
    // Several failures: a parallel repair round first (seg::seg_prepair:
    // every segment from its predecessor's exit at once -- a log of logs
    // fails at every segment and is whole after one), then check again
    if (nfail >= 2 && prepairs < ctx->wal_seg_prepair) {
      if (W.cap_seg0 < W.cap_seg) {
        for (void** p : {(void**)&W.sg0, (void**)&W.sx0, (void**)&W.scode0}) {
          if (*p) (void)hipFree(*p);
          *p = nullptr;
        }
        W.cap_seg0 = 0;
        if (hipMalloc((void**)&W.sg0, W.cap_seg * 8) != hipSuccess ||
            hipMalloc((void**)&W.sx0, W.cap_seg * 8) != hipSuccess ||
            hipMalloc((void**)&W.scode0, W.cap_seg * 4) != hipSuccess) {
          (void)hipGetLastError();  // (no room for the snapshot: the serial repairs below)
        } else {
          W.cap_seg0 = W.cap_seg;
        }
      }
      if (W.cap_seg0 >= a.K) {
        if ((rc = lsmk_wal_seg_prepair(&a, W.sg0, W.sx0, W.scode0, st)))
          return launch_rc(rc, "wal segment parallel repair");
        ++prepairs;
        ctx->last_seg_prepairs = ctx->last_seg_prepairs + 1;
        continue;
      }
    }
    // Many failures still: records longer than the segments (a segment
    // inside one has no true entry, and a bogus start there is taken) --
    // segments 16x longer, once or twice, unless the caller fixed the size
    if (repairs == 0 && !ctx->wal_seg_bytes && resegs < 2 && nfail > std::max<uint32_t>(64, a.K / 512) &&
        S < (1ull << 30)) {
      S <<= 4;
      ++resegs;
      walk = true;
      continue;
    }
    if (repairs >= ctx->wal_seg_rounds) {
      ctx->last_seg_repairs = repairs;
      return kWalSegDecline;
    }
    // the failing segment's entry is right: rewalk from its exit (and on, for
    // up to 4096 segments of consecutive failures), then check again
    if ((rc = lsmk_wal_seg_repair(&a, 4096, st))) return launch_rc(rc, "wal segment repair kernel");
    ctx->last_seg_repairs = ++repairs;
  }
  const uint64_t m = W.h_sinfo[sg::kInfoRecs];
  out->m = at + m;
  const uint64_t code = W.h_sinfo[sg::kInfoCode];
  out->term = code == sg::kBad ? kWalBad : (code == sg::kExit ? kWalStop : 0xFFFFFFFFu);
  out->tpos = W.h_sinfo[sg::kInfoPos];
  if (m) {
    const size_t tot = at + m;
    // LSMCK_RECS_DEVICE with room for every record: emitted into the caller's
    // array (a pipelined part after the first: when the parts before it were)
    const bool dev = ctx->wal_recs_dev && (at == 0 || ctx->wal_recs_dev_emitted) && tot <= ctx->wal_recs_dev_cap;
    if (ctx->wal_recs_dev_emitted && at > 0 && !dev) return kWalPipeRestart;
    const bool c16 = ctx->wal_compact;
    if (ctx->wal_grow_hook) {  // (a pipelined replay: the CRC passes and read-backs beside it let go first)
      const size_t rcap = dev ? tot : c16 ? W.cap_recs16 : W.cap_recs;
      if ((rcap < tot || ctx->cap_woff < tot || ctx->cap_wlen < tot || ctx->cap_wexp < tot || ctx->cap_vcrc < tot) &&
          (rc = ctx->wal_grow_hook()))
        return rc;
    }
    if ((!dev && !c16 && (rc = ensure_dev_keep(&W.recs, &W.cap_recs, tot, at, st))) ||
        (!dev && c16 && (rc = ensure_dev_keep(&W.recs16, &W.cap_recs16, tot, at, st))) ||
        (rc = ensure_dev_keep(&ctx->d_woff, &ctx->cap_woff, tot, at, st)) ||
        (rc = ensure_dev_keep(&ctx->d_wlen, &ctx->cap_wlen, tot, at, st)) ||
        (rc = ensure_dev_keep(&ctx->d_wexp, &ctx->cap_wexp, tot, at, st)) ||
        (rc = ensure_dev_keep(&ctx->d_vcrc, &ctx->cap_vcrc, tot, at, st)))
      return rc;
    void* to = dev ? ctx->wal_recs_dev : c16 ? (void*)W.recs16 : (void*)W.recs;
    if (ctx->wal_seg_pack) {
      rc = lsmk_wal_seg_emit_packed(&a, at, to, c16, ctx->d_woff, ctx->d_wlen, ctx->d_wexp, tot, st);
    } else {
      rc = lsmk_wal_seg_emit(&a, at, to, c16, ctx->d_woff, ctx->d_wlen, ctx->d_wexp, st);
    }
    if (rc) return launch_rc(rc, "wal segment emit kernel");
    if ((rc = lsmk_wal_seg_place(&a, at, to, c16, ctx->d_woff, ctx->d_wlen, ctx->d_wexp, tot,
                                 ctx->wal_seg_pack ? 1 : 0, st)))
      return launch_rc(rc, "wal segment place kernel");
    out->packed = ctx->wal_seg_pack;
    ctx->wal_recs_dev_emitted = dev;
  }
  if (!ctx->wal_emit_ev) HIPCHK(hipEventCreateWithFlags(&ctx->wal_emit_ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(ctx->wal_emit_ev, st));
  return 0;
}

// The pipelined replay's two CU-masked streams: the walk keeps wal_pipe_cus
// CUs (the last ones, or spread over the chip), the CRC passes get the rest.
// A persistent stream kernel sized to the rest's CU count keeps each of its
// CUs to itself, so neither side's workgroups wait for the other's.
static int wal_pipe_streams(lsmck_ctx* ctx) {
  const int N = ctx->ncu, cus = std::min(ctx->wal_pipe_cus, N - 1);
  const int key = cus * 2 + ctx->wal_pipe_layout;
  if (ctx->wal_pw && ctx->wal_pc && ctx->wal_pipe_key == key) return 0;
  for (hipStream_t* s : {&ctx->wal_pw, &ctx->wal_pc})
    if (*s) {
      (void)hipStreamSynchronize(*s);
      (void)hipStreamDestroy(*s);
      *s = nullptr;
    }
  std::vector<uint32_t> mw((size_t)(N + 31) / 32, 0u), mc((size_t)(N + 31) / 32, 0u);
  std::vector<char> walk((size_t)N, 0);
  if (ctx->wal_pipe_layout == 0) {
    for (int i = N - cus; i < N; ++i) walk[(size_t)i] = 1;
  } else {
    for (int j = 0; j < cus; ++j) walk[(size_t)(((int64_t)j * N) / cus + N / cus - 1)] = 1;
  }
  for (int i = 0; i < N; ++i) (walk[(size_t)i] ? mw : mc)[(size_t)i / 32] |= 1u << (i % 32);
  HIPCHK(hipExtStreamCreateWithCUMask(&ctx->wal_pw, (uint32_t)mw.size(), mw.data()));
  HIPCHK(hipExtStreamCreateWithCUMask(&ctx->wal_pc, (uint32_t)mc.size(), mc.data()));
  ctx->wal_pipe_key = key;
  return 0;
}

// The device replay in parts ("wal_pipe" parts, logs of "wal_pipe_min" bytes
// and more): the segment walk of part k+1 runs on wal_pipe_cus CUs while the
// CRC pass of part k runs on the others.  The walk is latency-bound (HBM
// nearly idle, ~1.2 TB/s), the pass is bound by its compute at the clock the
// chip holds, so the walk's time hides inside the pass except for the first
// part's, which is walked on every CU before anything runs beside it.  Each
// part is a prefix walk (records that start in [start, lim); the next part
// starts at the first record at or past lim, exactly as the split host replay
// resumes), its records emitted after the parts before it.  A part's last
// record keeps its payload alone as its CRC span (the next header is the next
// part's), so the compare's report unpacks no header from it (`ends`).
// Records to the host are read back part by part on the SDMA engines as each
// part is emitted.  Returns kWalSegDecline / kWalPipeRestart, everything
// beside it drained, when a part's segment walk declines or its records
// outgrow the caller's device array: the caller then replays unpipelined.
static int wal_replay_pipelined(lsmck_ctx* ctx, const uint8_t* img, size_t n, void* recs, size_t cap, size_t* nrec,
                                uint64_t* bad_index, uint32_t* bad_crc, uint32_t* bad_expected, hipStream_t st,
                                const WalTrace& tr) {
  auto& Wd = ctx->wd;
  int rc;
  if ((rc = wal_pipe_streams(ctx))) return rc;
  const int P = ctx->wal_pipe;
  const int crc_cus = ctx->ncu - std::min(ctx->wal_pipe_cus, ctx->ncu - 1);
  hipStream_t W = ctx->wal_pw, C = ctx->wal_pc;
  while ((int)ctx->wal_pipe_ev.size() < P) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ctx->wal_pipe_ev.push_back(e);
  }
  const size_t rsz = wal_rec_size(ctx);
  const bool c16 = ctx->wal_compact;
  // records to the host, part by part on the SDMA engines (no engines: the
  // whole read-back in wal_finish, after the last part)
  const bool host_recs = !ctx->wal_recs_dev && recs && cap;
  lsmck_dma::Copier* dc = host_recs && ctx->wal_dma_engines ? dma_copier(ctx) : nullptr;
  const int E = dc ? std::max(1, std::min(ctx->wal_dma_engines, lsmck_dma::engines(dc))) : 0;
  const bool direct = ctx->wal_recs_direct;
  struct RB {
    lsmck_dma::Job job;
    size_t lo;    // its first record
    int cur = 0;  // pieces landed (and copied out)
  };
  std::vector<RB> jobs;
  int sig_next = 0, derr = 0;
  auto copy_out = [&](size_t a, size_t b) {  // the landing's bytes [a, b) -> the caller's pageable array
    const size_t len = b - a;
    const unsigned T = len >= (4u << 20) ? std::max(1u, std::min(ctx->stage_threads, 8u)) : 1u;
    host_pool(ctx).run(T, [&](unsigned t) {
      const size_t x = a + (len * t / T & ~(size_t)4095), y = t + 1 == T ? b : a + (len * (t + 1) / T & ~(size_t)4095);
      if (y > x) memcpy((uint8_t*)recs + x, ctx->h_wrecs + x, y - x);
    });
  };
  auto drain = [&](bool block) {  // landed pieces copied out, in order; block: all of them
    for (auto& J : jobs)
      for (; J.cur < J.job.n; ++J.cur) {
        if (!block && !lsmck_dma::landed(dc, J.job, J.cur)) return;
        if (lsmck_dma::wait(dc, J.job, J.cur) && !derr) derr = 1;
        if (!direct && !derr) copy_out(J.lo * rsz + J.job.off[J.cur], J.lo * rsz + J.job.off[J.cur + 1]);
      }
    jobs.clear();
    sig_next = 0;
  };
  auto quiesce = [&]() -> int {  // nothing beside the walk reads the record arrays any more
    HIPCHK(hipStreamSynchronize(C));
    HIPCHK(hipStreamSynchronize(W));
    if (dc) drain(true);
    return derr ? lsmck_host::set_error(LSMCK_EIO, "SDMA copy of the WAL records failed") : 0;
  };
  struct Hook {  // (cleared on every return)
    lsmck_ctx* c;
    ~Hook() {
      c->wal_grow_hook = nullptr;
      c->wal_seg_auto = 0;
    }
  } hook{ctx};
  ctx->wal_grow_hook = quiesce;
  auto readback = [&](size_t lo, size_t hi) -> int {  // records [lo, hi) to the host (hi <= cap)
    if (!dc || hi <= lo) return 0;
    uint8_t* land;
    if (direct) {
      land = (uint8_t*)recs + lo * rsz;
    } else {
      if (hi * rsz > ctx->cap_hwrecs) {  // (the landing grows only with nothing in flight)
        drain(true);
        if ((rc = ensure_pinned(ctx->pin_node, &ctx->h_wrecs, &ctx->cap_hwrecs, hi * rsz + hi * rsz / 4))) return rc;
      }
      land = ctx->h_wrecs + lo * rsz;
    }
    const int chunks = std::max(E, ctx->wal_dma_chunks / 4);
    if (sig_next + chunks > lsmck_dma::kMaxSignals) drain(true);
    const uint8_t* src = c16 ? (const uint8_t*)Wd.recs16 : (const uint8_t*)Wd.recs;
    RB J;
    J.lo = lo;
    if (lsmck_dma::d2h(dc, land, src + lo * rsz, (hi - lo) * rsz, E, chunks, &J.job, sig_next) != 0) {
      drain(true);  // (the engines refused: one plain copy of this part)
      HIPCHK(hipMemcpy(land, src + lo * rsz, (hi - lo) * rsz, hipMemcpyDeviceToHost));
      if (!direct) copy_out(lo * rsz, hi * rsz);
      return 0;
    }
    sig_next += J.job.n;
    jobs.push_back(J);
    return 0;
  };
  // part bounds: the first part on every CU (st), the rest in P - 1 parts on W
  const uint64_t a0 = std::max<uint64_t>(n * (uint64_t)ctx->wal_pipe_first / 64, 1);
  std::vector<size_t> ends;  // the parts' last records (their spans are their payloads alone)
  uint64_t start = 0;
  size_t at = 0;
  int parts = 0, repairs = 0, prepairs = 0;
  uint64_t segs = 0;
  WalPart Pk;
  for (int k = 0;; ++k) {
    const uint64_t lim = k + 1 >= P ? n : k == 0 ? a0 : a0 + (n - a0) * (uint64_t)k / (uint64_t)(P - 1);
    hipStream_t ws = k == 0 ? st : W;
    // the parts on W in segments for the lanes the walk CUs hold at once
    // (8 waves a SIMD, a segment per 8 lanes): one round of waves, each
    // chain as long as that allows; part 0 on every CU keeps the auto size
    if (k == 1) {
      const uint64_t lanes = (uint64_t)std::min(ctx->wal_pipe_cus, ctx->ncu - 1) * 4 * 8 * 64 / 8;
      uint64_t S = ctx->wal_pipe_seg;
      if (!S) {
        S = 4096;
        while (S < (16ull << 20) && ((n - a0) / (uint64_t)(P - 1) + S - 1) / S > lanes) S <<= 1;
      }
      ctx->wal_seg_auto = S;
    }
    rc = wal_seg_walk(ctx, img, n, start, lim, at, ws, tr, &Pk);
    repairs += ctx->last_seg_repairs;
    prepairs += ctx->last_seg_prepairs;
    segs += ctx->last_segments;
    if (rc) {
      const int q = quiesce();
      return q ? q : rc;
    }
    const size_t m = Pk.m - at;
    const bool more = Pk.term == kWalStop && Pk.tpos < n && lim < n;
    if (more && !m) {  // (no record started in the part: not expected, the plain replay instead)
      const int q = quiesce();
      return q ? q : kWalPipeRestart;
    }
    if (k == 0 && more && m) {
      // the record arrays sized once for the whole log from the first part's
      // density (+15 %), before anything runs beside the walk; a later part
      // that outgrows them drains first (wal_grow_hook)
      const size_t est = (size_t)((double)m * ((double)n / (double)std::max<uint64_t>(Pk.tpos, 1)) * 1.15) + 65536;
      const bool dev = ctx->wal_recs_dev_emitted;
      if ((!dev && !c16 && (rc = ensure_dev_keep(&Wd.recs, &Wd.cap_recs, est, m, st))) ||
          (!dev && c16 && (rc = ensure_dev_keep(&Wd.recs16, &Wd.cap_recs16, est, m, st))) ||
          (rc = ensure_dev_keep(&ctx->d_woff, &ctx->cap_woff, est, m, st)) ||
          (rc = ensure_dev_keep(&ctx->d_wlen, &ctx->cap_wlen, est, m, st)) ||
          (rc = ensure_dev_keep(&ctx->d_wexp, &ctx->cap_wexp, est, m, st)) ||
          (rc = ensure_dev_keep(&ctx->d_vcrc, &ctx->cap_vcrc, est, m, st)))
        return rc;
      if (dc && !direct && (rc = ensure_pinned(ctx->pin_node, &ctx->h_wrecs, &ctx->cap_hwrecs, std::min(est, cap) * rsz)))
        return rc;
    }
    hipEvent_t ev = ctx->wal_pipe_ev[(size_t)k % ctx->wal_pipe_ev.size()];
    HIPCHK(hipEventRecord(ev, ws));
    if (k == 0) HIPCHK(hipStreamWaitEvent(W, ev, 0));  // (the walk's arrays: part 0's place is done)
    HIPCHK(hipStreamWaitEvent(C, ev, 0));
    if ((rc = wal_crc_part(ctx, img, at, m, C, crc_cus))) {
      const int q = quiesce();
      return q ? q : rc;
    }
    ++parts;
    tr.mark(k == 0 ? "pipe: part 0 walked, its CRC pass queued" : "pipe: part walked, its CRC pass queued");
    if (dc && at < cap) {  // this part's records to the host once its emit is done
      HIPCHK(hipEventSynchronize(ev));
      if ((rc = readback(at, std::min(at + m, cap)))) return rc;
    }
    if (more && m) ends.push_back(at + m - 1);
    at += m;
    if (!more) break;
    start = Pk.tpos;
    if (dc) drain(false);
  }
  ctx->last_pipe_parts = parts;
  ctx->last_walk_path = 1;
  ctx->last_seg_repairs = repairs;
  ctx->last_seg_prepairs = prepairs;
  ctx->last_segments = segs;
  // the compare on st once the last pass is done
  hipEvent_t evc = ctx->wal_pipe_ev[(size_t)parts % ctx->wal_pipe_ev.size()];
  HIPCHK(hipEventRecord(evc, C));
  HIPCHK(hipStreamWaitEvent(st, evc, 0));
  const size_t done = dc ? std::min(at, cap) : 0;  // (read back already, or landing as wal_finish returns)
  rc = wal_finish(ctx, img, at, Pk.term, Pk.tpos, recs, cap, nrec, bad_index, bad_crc, bad_expected, st, tr, done, true,
                  Pk.packed ? 0 : ~(size_t)0, &ends);
  if (dc) {
    drain(true);
    if (dc) ctx->last_recs_dma = E;
    tr.mark("pipe: records read back");
    if (derr && rc >= 0) return lsmck_host::set_error(LSMCK_EIO, "SDMA copy of the WAL records failed");
  }
  return rc;
}

// A device-resident image (or an uploaded one: `marked`, its candidate bitmap
// is already in ctx->wd -- wal_upload marks each chunk behind its copy): the
// walk (in parts when its scratch would not fit), one CRC pass per part.
static int wal_replay_device(lsmck_ctx* ctx, const uint8_t* img, size_t n, void* recs, size_t cap,
                             size_t* nrec, uint64_t* bad_index, uint32_t* bad_crc, uint32_t* bad_expected,
                             bool marked = false) {
  std::lock_guard<std::mutex> lk(ctx->mu);
  DevGuard g(ctx->dev);
  const WalTrace tr;
  int rc;
  ScratchOrder so(ctx, ctx->stream0);
  if (so.e != hipSuccess) return hip_error(so.e, "hipStreamWaitEvent(scratch)");
  hipStream_t st = so.st;
  ctx->last_pipe_parts = 0;
  if (ctx->wal_pipe >= 2 && ctx->wal_seg && !ctx->wal_part_bytes && n >= ctx->wal_pipe_min && n >= 64) {
    rc = wal_replay_pipelined(ctx, img, n, recs, cap, nrec, bad_index, bad_crc, bad_expected, st, tr);
    if (rc != kWalSegDecline && rc != kWalPipeRestart) return rc;
    ctx->last_pipe_parts = 0;  // (a part declined, or outgrew the caller's array: the whole log, unpipelined)
    ctx->wal_recs_dev_emitted = false;
  }
  WalPart P;
  rc = ctx->wal_seg && !ctx->wal_part_bytes ? wal_seg_walk(ctx, img, n, 0, n, 0, st, tr, &P) : kWalSegDecline;
  if (rc == 0) {  // the CRC pass over every record, then the compare and the records
    if ((rc = wal_crc_part(ctx, img, 0, P.m, st))) return rc;
    return wal_finish(ctx, img, P.m, P.term, P.tpos, recs, cap, nrec, bad_index, bad_crc, bad_expected, st, tr, 0,
                      true, P.packed ? 0 : ~(size_t)0);
  }
  if (rc != kWalSegDecline) return rc;
  ctx->last_walk_path = 2;  // candidate doubling: its bitmap, ranks and jump tables
  if ((rc = wal_walk_setup(ctx, n))) return rc;
  if ((rc = wal_walk_from(ctx, img, n, 0, 0, ctx->wal_part_bytes, marked, st, tr, &P))) return rc;
  return wal_finish(ctx, img, P.m, P.term, P.tpos, recs, cap, nrec, bad_index, bad_crc, bad_expected, st, tr);
}

// Host WAL image upload into ctx->d_wimg, in chunks of "wal_stage_bytes"
// alternating over the two staging slots, each chunk's candidate marking
// queued behind its copy (the marking then overlaps the rest of the upload).
// Pageable images go through the slot's pinned buffer (copied on
// stage_threads threads while the other slot's DMA runs); pinned (or
// registered) ones are DMA'd straight from the caller's pages.  Bytes
// [lo, hi), lo a multiple of the chunk size.  Caller holds ctx->mu and a
// StageGuard; the slots' streams carry the work (wait on them).
struct WalUpload {
  const uint8_t* img;
  size_t n;
  bool direct;  // pinned or registered: no staging copy
  int slot = 0;
};
static int wal_upload_range(lsmck_ctx* ctx, WalUpload& U, size_t lo, size_t hi) {
  auto& W = ctx->wd;
  int rc;
  const size_t ch = ctx->wal_stage_bytes;
  for (size_t o = lo; o < hi; o += ch, U.slot ^= 1) {
    Stage& S = ctx->stage[U.slot];
    const size_t c = std::min(ch, hi - o);
    HIPCHK(hipEventSynchronize(S.done));  // the slot's previous DMA has drained
    if (U.direct) {
      HIPCHK(hipMemcpyAsync(ctx->d_wimg + o, U.img + o, c, hipMemcpyHostToDevice, S.s));
    } else {
      stage_copy(ctx, S.h_pay, U.img + o, c, ctx->stage_threads);
      HIPCHK(hipMemcpyAsync(ctx->d_wimg + o, S.h_pay, c, hipMemcpyHostToDevice, S.s));
    }
    HIPCHK(hipEventRecord(S.done, S.s));
    rc = lsmk_wal_mark_range(ctx->d_wimg, U.n, o, o + c, W.bits, W.pre, S.s);  // ch: a multiple of 64
    if (rc) return launch_rc(rc, "wal mark kernel");
  }
  return 0;
}

// the slots' work so far, ordered before stream st
static int wal_upload_fence(lsmck_ctx* ctx, hipStream_t st) {
  for (int k = 0; k < kHostSlots; ++k) {  // (the upload's slots)
    Stage& S = ctx->stage[k];
    HIPCHK(hipEventRecord(S.done, S.s));
    HIPCHK(hipStreamWaitEvent(st, S.done, 0));
  }
  return 0;
}

// "wal_register": pin the caller's pageable pages in place for the call
// (hipHostRegister) and DMA straight from them, instead of the staging copy.
struct HostRegistration {
  uint8_t* base = nullptr;
  bool on = false;
  HostRegistration(const uint8_t* img, size_t n) {
    const uintptr_t pa = (uintptr_t)img & ~(uintptr_t)4095, pe = ((uintptr_t)img + n + 4095) & ~(uintptr_t)4095;
    base = (uint8_t*)pa;
    on = hipHostRegister(base, pe - pa, hipHostRegisterDefault) == hipSuccess;
    if (!on) (void)hipGetLastError();
  }
  ~HostRegistration() {
    if (on) (void)hipHostUnregister(base);
  }
};

static int wal_upload_prepare(lsmck_ctx* ctx, size_t n, bool direct) {
  int rc;
  if ((rc = ensure_dev(&ctx->d_wimg, &ctx->cap_wimg, n + 16)) || (rc = wal_walk_setup(ctx, n))) return rc;
  for (int k = 0; k < kHostSlots; ++k) {  // (the upload alternates slots 0 and 1)
    Stage& S = ctx->stage[k];
    if ((rc = stage_init(S))) return rc;
    if (S.busy) {  // a failed host batch's slot: nothing to retire here
      HIPCHK(hipStreamSynchronize(S.s));
      S.busy = false;
    }
    if (!direct && (rc = ensure_pinned(ctx->pin_node, &S.h_pay, &S.cap_h_pay, std::min(n, ctx->wal_stage_bytes)))) return rc;
  }
  return 0;
}

// The whole host image uploaded (and marked) before the walk (caller holds wal_mu).
static int wal_upload(lsmck_ctx* ctx, const uint8_t* img, size_t n, bool pinned) {
  std::lock_guard<std::mutex> lk(ctx->mu);
  DevGuard g(ctx->dev);
  const WalTrace tr;
  std::unique_ptr<HostRegistration> reg;
  if (!pinned && ctx->wal_register && n >= (1u << 20)) reg.reset(new HostRegistration(img, n));
  WalUpload U{img, n, pinned || (reg && reg->on)};
  int rc;
  if ((rc = wal_upload_prepare(ctx, n, U.direct))) return rc;
  StageGuard guard{ctx};
  if ((rc = wal_upload_range(ctx, U, 0, n))) return rc;
  for (int k = 0; k < kHostSlots; ++k) HIPCHK(hipStreamSynchronize(ctx->stage[k].s));
  tr.mark("upload");
  guard.ok = true;
  return 0;
}

// The split replay's first m records (emitted on st) into the caller's array
// on this (helper) thread, through ctx->h_wrecs1 and the records' own stream.
static int wal_records_early(lsmck_ctx* ctx, size_t m, void* recs, size_t cap, hipStream_t st, size_t* done) {
  int rc;
  const size_t rsz = wal_rec_size(ctx);
  if ((rc = ensure_pinned(ctx->pin_node, &ctx->h_wrecs1, &ctx->cap_hwrecs1, m * rsz))) return rc;
  if (!ctx->wal_rs) HIPCHK(hipStreamCreateWithFlags(&ctx->wal_rs, hipStreamNonBlocking));
  if (!ctx->wal_emit1_ev) HIPCHK(hipEventCreateWithFlags(&ctx->wal_emit1_ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(ctx->wal_emit1_ev, st));
  HIPCHK(hipStreamWaitEvent(ctx->wal_rs, ctx->wal_emit1_ev, 0));
  const void* src = ctx->wal_compact ? (const void*)ctx->wd.recs16 : (const void*)ctx->wd.recs;
  HIPCHK(hipMemcpyAsync(ctx->h_wrecs1, src, m * rsz, hipMemcpyDeviceToHost, ctx->wal_rs));
  HIPCHK(hipStreamSynchronize(ctx->wal_rs));
  const size_t cnt = std::min(m, cap);
  memcpy(recs, ctx->h_wrecs1, cnt * rsz);  // (one thread: the pool is staging the upload)
  *done = m;
  return 0;
}

constexpr int kWalNoSplit = 0x7FFF0002;  // internal: the image is too small to upload in two parts

// A host image uploaded in two parts ("wal_split", default on; taken when each
// half holds at least one upload chunk -- images of two "wal_stage_bytes"
// chunks and more, 32 MiB at the default 16 MiB chunk):
// the prefix [0, a) is walked (lsmck_wal.hip's prefix walk: records that end
// by a) and its CRC pass launched on stream0, on a helper thread, while this
// thread uploads the rest; the walk then resumes where the prefix stopped
// (the next header, or the first record that did not end by a).  The walk's
// own time then hides behind the upload except for the second part's.
// Caller holds wal_mu.
static int wal_replay_split(lsmck_ctx* ctx, const uint8_t* img, size_t n, bool pinned, void* recs,
                            size_t cap, size_t* nrec, uint64_t* bad_index, uint32_t* bad_crc, uint32_t* bad_expected) {
  const size_t ch = ctx->wal_stage_bytes;
  const size_t a = (n / 2) / ch * ch;
  if (a < ch || n - a < ch || a >= (1ull << 32)) return kWalNoSplit;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DevGuard g(ctx->dev);
  const WalTrace tr;
  std::unique_ptr<HostRegistration> reg;
  if (!pinned && ctx->wal_register) reg.reset(new HostRegistration(img, n));
  // on every return: no DMA from the caller's pages still running (and none
  // from registered pages once they are unregistered, right after this)
  struct SyncStages {
    lsmck_ctx* c;
    ~SyncStages() {
      for (auto& S : c->stage)
        if (S.s) (void)hipStreamSynchronize(S.s);
    }
  } sync_stages{ctx};
  WalUpload U{img, n, pinned || (reg && reg->on)};
  int rc;
  if ((rc = wal_upload_prepare(ctx, n, U.direct))) return rc;
  ScratchOrder so(ctx, ctx->stream0);
  if (so.e != hipSuccess) return hip_error(so.e, "hipStreamWaitEvent(scratch)");
  hipStream_t st = so.st;
  const uint8_t* d = ctx->d_wimg;
  WalPart P1, P2;
  size_t done = 0;  // records already in the caller's array
  {
    StageGuard guard{ctx};
    if ((rc = wal_upload_range(ctx, U, 0, a)) || (rc = wal_upload_fence(ctx, st))) return rc;
    tr.mark("upload part 1 issued");
    auto prefix = std::async(std::launch::async, [&]() -> std::pair<int, std::string> {
      DevGuard gd(ctx->dev);  // (a new thread's current device is device 0)
      int r = wal_walk_part(ctx, d, n, 0, a >> 6, 0, a, true, 0, st, &P1, tr);
      if (!r) r = wal_crc_part(ctx, d, 0, P1.m, st);
      // the first part's records to the caller now, on their own stream, while
      // the second part uploads
      if (!r && recs && cap && P1.m) r = wal_records_early(ctx, P1.m, recs, cap, st, &done);
      return {r, r ? std::string(lsmck_last_error()) : std::string()};
    });
    rc = wal_upload_range(ctx, U, a, n);
    const auto pr = prefix.get();
    if (rc) return rc;
    if (pr.first == kWalTooBig) {  // the first half alone is too dense to walk in one part: all of it in parts
      if ((rc = wal_upload_fence(ctx, st))) return rc;
      guard.ok = true;
      WalPart PA;
      if ((rc = wal_walk_from(ctx, d, n, 0, 0, ctx->wal_part_bytes, false, st, tr, &PA))) return rc;
      return wal_finish(ctx, d, PA.m, PA.term, PA.tpos, recs, cap, nrec, bad_index, bad_crc, bad_expected, st, tr);
    }
    if (pr.first) {
      if (pr.first != kWalHostWalk) lsmck_host::set_error(pr.first, pr.second.c_str());
      for (int k = 0; k < kHostSlots; ++k) HIPCHK(hipStreamSynchronize(ctx->stage[k].s));
      guard.ok = true;
      return pr.first;  // (kWalHostWalk: the image is whole on the device; the caller walks it on the host)
    }
    if ((rc = wal_upload_fence(ctx, st))) return rc;
    tr.mark("upload part 2 issued");
    guard.ok = true;
  }
  if (P1.term != kWalStop && P1.term != kWalStopSelf)  // the log ended inside the prefix
    return wal_finish(ctx, d, P1.m, P1.term, P1.tpos, recs, cap, nrec, bad_index, bad_crc, bad_expected, st, tr, done);
  // resume at r: the segment walk of the rest (it needs no candidate marks);
  // when it declines, the words from r's to the prefix end lost their counts
  // to the prefix scan: mark them again, then walk words [r/64, end) from r
  // (in parts, when the rest's scratch would not fit)
  const uint64_t r = P1.tpos;
  if (ctx->wal_seg && !ctx->wal_part_bytes) {
    rc = wal_seg_walk(ctx, d, n, r, n, P1.m, st, tr, &P2);
    if (rc == 0) {
      if ((rc = wal_crc_part(ctx, d, P1.m, P2.m - P1.m, st))) return rc;
      return wal_finish(ctx, d, P2.m, P2.term, P2.tpos, recs, cap, nrec, bad_index, bad_crc, bad_expected, st, tr,
                        done, true, P2.packed ? P1.m : ~(size_t)0);
    }
    if (rc != kWalSegDecline) return rc;
  }
  ctx->last_walk_path = 2;
  if (r < a && (rc = lsmk_wal_mark_range(d, n, r & ~(uint64_t)63, a, ctx->wd.bits, ctx->wd.pre, st)))
    return launch_rc(rc, "wal mark kernel");
  if ((rc = wal_walk_from(ctx, d, n, r, P1.m, ctx->wal_part_bytes, true, st, tr, &P2))) return rc;
  return wal_finish(ctx, d, P2.m, P2.term, P2.tpos, recs, cap, nrec, bad_index, bad_crc, bad_expected, st, tr, done);
}

extern "C" {

int lsmck_wal_frame_insert_device(lsmck_ctx* ctx, uint8_t* img, const uint64_t* off, const uint32_t* len,
                                  const uint32_t* crc, size_t n, uint32_t kmax, void* stream) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  DevGuard g(ctx->dev);
  rc = lsmk_wal_frame_insert(img, off, len, crc, n, kmax, pick_stream(ctx, stream));
  return rc ? launch_rc(rc, "wal frame kernel") : 0;
}

}  // extern "C"

// internal flag: the GPU walk of this image already declined (kWalHostWalk): straight to the host walk
constexpr unsigned kWalNoGpuWalk = 0x40000000u;

// the call's record options on the context, set while wal_mu is held and
// cleared on every return (wal_finish and the walks read them)
struct WalCallRecs {
  lsmck_ctx* c;
  WalCallRecs(lsmck_ctx* c_, bool compact, bool direct, void* dev, size_t cap) : c(c_) {
    c->wal_compact = compact;
    c->wal_recs_direct = direct;
    c->wal_recs_dev = dev;
    c->wal_recs_dev_cap = dev ? cap : 0;
    c->wal_recs_dev_emitted = false;
  }
  ~WalCallRecs() {
    c->wal_compact = false;
    c->wal_recs_direct = false;
    c->wal_recs_dev = nullptr;
    c->wal_recs_dev_cap = 0;
    c->wal_recs_dev_emitted = false;
  }
};

// lsmck_wal_replay_verify (recs: lsmck_wal_rec[cap]) and
// lsmck_wal_replay_verify16 (compact: lsmck_wal_rec16[cap])
static int wal_replay_verify(lsmck_ctx* ctx, const uint8_t* wal, size_t n, unsigned flags, void* recs, bool compact,
                             size_t cap, size_t* nrec, uint64_t* bad_index, uint32_t* bad_crc,
                             uint32_t* bad_expected) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  const size_t rsz = compact ? sizeof(lsmck_wal_rec16) : sizeof(lsmck_wal_rec);
  // LSMCK_RECS_PINNED: the records go by DMA into the caller's pinned array
  // (read by wal_finish under wal_mu; the host walk ignores it)
  const bool recs_pinned = (flags & LSMCK_RECS_PINNED) != 0;
  const bool gpu_walk = (flags & LSMCK_DEVICE) && ctx->wal_gpu_walk && !(flags & kWalNoGpuWalk);
  if (flags & LSMCK_RECS_DEVICE) {
    if (recs_pinned) return lsmck_host::set_error(LSMCK_EINVAL, "LSMCK_RECS_DEVICE with LSMCK_RECS_PINNED");
    unsigned more = 0;
    if (gpu_walk) {
      std::lock_guard<std::mutex> wl(ctx->wal_mu);
      WalCallRecs wc(ctx, compact, false, recs, cap);
      rc = wal_replay_device(ctx, wal, n, recs, cap, nrec, bad_index, bad_crc, bad_expected);
      if (rc != kWalHostWalk) return rc;
      more = kWalNoGpuWalk;  // (the GPU walk declined: no second try below)
    }
    // any other path makes the records on the host: into a host array, then
    // copied to the caller's device array (uninitialised: only what the walk writes is copied)
    const size_t k0 = recs ? std::min<size_t>(cap, n / 9 + 1) : 0;
    std::unique_ptr<uint8_t[]> tmp(k0 ? new uint8_t[k0 * rsz] : nullptr);
    size_t got = 0;
    rc = wal_replay_verify(ctx, wal, n, (flags & ~LSMCK_RECS_DEVICE) | more, tmp.get(), compact, k0, &got, bad_index,
                           bad_crc, bad_expected);
    if (rc < 0) return rc;
    if (nrec) *nrec = got;
    const size_t k = std::min(got, k0);
    if (k) {
      DevGuard g(ctx->dev);
      HIPCHK(hipMemcpy(recs, tmp.get(), k * rsz, hipMemcpyHostToDevice));
    }
    return rc;
  }
  if (gpu_walk) {
    std::lock_guard<std::mutex> wl(ctx->wal_mu);  // the walk's bitmap (ctx->wd) is shared with the upload path
    WalCallRecs wc(ctx, compact, recs_pinned, nullptr, 0);
    rc = wal_replay_device(ctx, wal, n, recs, cap, nrec, bad_index, bad_crc, bad_expected);
    if (rc != kWalHostWalk) return rc;
    // (the GPU walk declined: the image is copied back and walked on the host below)
  } else if (!(flags & LSMCK_DEVICE) && ctx->wal_upload_min && n >= ctx->wal_upload_min) {
    // Host image: one upload (~36 GiB/s through the staging slots) and the GPU
    // header walk, instead of the serial host walk (~12 GiB/s) -- the records
    // and offsets are the same, they index the caller's image
    std::lock_guard<std::mutex> wl(ctx->wal_mu);
    WalCallRecs wc(ctx, compact, recs_pinned, nullptr, 0);
    const bool pinned = (flags & LSMCK_HOST_PINNED) != 0;
    rc = ctx->wal_split ? wal_replay_split(ctx, wal, n, pinned, recs, cap, nrec, bad_index, bad_crc, bad_expected)
                        : kWalNoSplit;
    if (rc == kWalNoSplit) {
      if ((rc = wal_upload(ctx, wal, n, pinned))) return rc;
      rc = wal_replay_device(ctx, ctx->d_wimg, n, recs, cap, nrec, bad_index, bad_crc, bad_expected, true);
    }
    if (rc != kWalHostWalk) return rc;
  }
  ctx->last_walk_path = 3;
  const uint8_t* h = wal;
  // Device image: the walk reads a host copy, made by DMA into a pinned
  // buffer the context keeps (grow-only).  Copying into fresh pageable memory
  // instead ran at 2.8 GiB/s for 0.24 GB: page faults plus HIP's bounce copy.
  std::unique_lock<std::mutex> wal_lk(ctx->wal_mu, std::defer_lock);
  if (flags & LSMCK_DEVICE) {
    wal_lk.lock();
    DevGuard g(ctx->dev);
    rc = ensure_pinned(ctx->pin_node, &ctx->wal_host, &ctx->wal_host_cap, n);
    if (rc) return rc;
    if (n) HIPCHK(hipMemcpy(ctx->wal_host, wal, n, hipMemcpyDeviceToHost));
    h = ctx->wal_host;
  }
  // 1. header walk (serial: each record's length is in its own header)
  std::vector<uint64_t> poff;
  std::vector<uint32_t> plen, pcrc;
  std::vector<uint8_t> ptype;
  std::vector<uint64_t> roff;
  std::vector<uint32_t> rk, rv;
  size_t pos = 0;
  int stop = 0;  // 0 clean, 3 bad type
  uint64_t stop_index = 0;
  uint32_t stop_type = 0;
  // The walk is a dependent chain -- each header's address comes from the
  // previous header's lengths -- so without help every header is one DRAM
  // round trip (~140 ns, 500k records in 72 ms, 1.7 GiB/s).  Every line up to
  // `dist` bytes ahead is prefetched, turning the chain into a stream.
  const size_t dist = ctx->wal_prefetch;
  size_t pf = 0;
  // Host image: the CRCs of the records walked so far run as a batch on a
  // helper thread while the walk goes on.  Each batch takes its own copy of
  // its descriptors (the vectors move as they grow), batches serialise on the
  // context's lock, and every helper is joined before the function returns
  // (a std::async future's destructor waits).
  const bool overlap = !(flags & LSMCK_DEVICE) && ctx->wal_chunk;
  struct Part {
    size_t r0, r1;
    struct Out {
      int rc;
      std::vector<uint32_t> crc;
      std::string err;  // lsmck_last_error() is thread-local: the helper's message travels back
    };
    std::future<Out> f;
  };
  std::vector<Part> parts;
  size_t chunk_r0 = 0;
  uint64_t chunk_bytes = 0;
  auto launch = [&](size_t r1) {
    std::vector<uint64_t> o(poff.begin() + chunk_r0, poff.begin() + r1);
    std::vector<uint32_t> l(plen.begin() + chunk_r0, plen.begin() + r1);
    parts.push_back({chunk_r0, r1, std::async(std::launch::async, [ctx, h, flags, o = std::move(o), l = std::move(l)]() {
                       Part::Out out{0, std::vector<uint32_t>(o.size()), {}};
                       out.rc = lsmck_crc32_batch(ctx, h, o.data(), l.data(), o.size(), out.crc.data(), flags, nullptr);
                       if (out.rc) out.err = lsmck_last_error();
                       return out;
                     })});
    chunk_r0 = r1;
    chunk_bytes = 0;
  };
  for (;;) {
    if (pos + 1 > n) break;
    if (dist) {
      const size_t lim = std::min(n, pos + dist);
      for (; pf < lim; pf += 64) __builtin_prefetch(h + pf, 0, 0);
    }
    uint8_t t = h[pos];
    if (t != 1 && t != 2) {
      stop = LSMCK_WAL_BAD_TYPE;
      stop_index = poff.size();
      stop_type = t;
      break;
    }
    size_t hdr = t == 1 ? 13 : 9;
    if (pos + hdr > n) break;  // UnexpectedEof inside a header: end of log
    uint32_t saved = rd_u32(h + pos + 1);
    uint32_t klen = rd_u32(h + pos + 5);
    uint32_t vlen = t == 1 ? rd_u32(h + pos + 9) : 0;
    uint32_t dlen = klen + vlen;  // u32 as wal.rs:129
    size_t avail = n - (pos + hdr);
    size_t got = dlen <= avail ? dlen : avail;  // read_to_end on take(): short read at EOF
    roff.push_back(pos);
    poff.push_back(pos + hdr);
    plen.push_back((uint32_t)got);
    pcrc.push_back(saved);
    ptype.push_back(t);
    rk.push_back(klen);
    rv.push_back(vlen);
    pos += hdr + got;
    if (overlap && (chunk_bytes += got) >= ctx->wal_chunk) launch(poff.size());
  }
  size_t m = poff.size();
  if (overlap && chunk_r0 < m) launch(m);
  // 2. every payload CRC in one GPU batch
  uint64_t nb = 0, first = m;
  if (m) {
    if (flags & LSMCK_DEVICE) {
      // descriptors + stored CRCs through pinned staging into pooled device
      // buffers, one CRC batch over the device image, and the GPU compare:
      // only the two counts come back
      std::lock_guard<std::mutex> lk(ctx->mu);
      DevGuard g(ctx->dev);
      if ((rc = ensure_pinned(ctx->pin_node, &ctx->h_woff, &ctx->cap_hwoff, m)) || (rc = ensure_pinned(ctx->pin_node, &ctx->h_wlen, &ctx->cap_hwlen, m)) ||
          (rc = ensure_pinned(ctx->pin_node, &ctx->h_wexp, &ctx->cap_hwexp, m)) || (rc = ensure_dev(&ctx->d_woff, &ctx->cap_woff, m)) ||
          (rc = ensure_dev(&ctx->d_wlen, &ctx->cap_wlen, m)) || (rc = ensure_dev(&ctx->d_wexp, &ctx->cap_wexp, m)))
        return rc;
      ScratchOrder so(ctx, ctx->stream0);
      if (so.e != hipSuccess) return hip_error(so.e, "hipStreamWaitEvent(scratch)");
      memcpy(ctx->h_woff, poff.data(), m * 8);
      memcpy(ctx->h_wlen, plen.data(), m * 4);
      memcpy(ctx->h_wexp, pcrc.data(), m * 4);
      HIPCHK(hipMemcpyAsync(ctx->d_woff, ctx->h_woff, m * 8, hipMemcpyHostToDevice, so.st));
      HIPCHK(hipMemcpyAsync(ctx->d_wlen, ctx->h_wlen, m * 4, hipMemcpyHostToDevice, so.st));
      HIPCHK(hipMemcpyAsync(ctx->d_wexp, ctx->h_wexp, m * 4, hipMemcpyHostToDevice, so.st));
      rc = device_verify(ctx, wal, ctx->d_woff, ctx->d_wlen, ctx->d_wexp, m, so.st, &nb, &first, true);
      if (rc < 0) return rc;
    } else if (overlap) {
      int prc = 0;
      std::string perr;
      for (auto& P : parts) {
        auto res = P.f.get();
        if (res.rc && !prc) {
          prc = res.rc;
          perr = res.err;
        }
        if (prc) continue;
        for (size_t i = P.r0; i < P.r1; ++i)
          if (res.crc[i - P.r0] != pcrc[i]) {
            if (!nb) first = i;
            ++nb;
          }
      }
      if (prc) return lsmck_host::set_error(prc, perr.c_str());
    } else {
      rc = lsmck_crc32_verify_batch(ctx, h, poff.data(), plen.data(), pcrc.data(), m, flags, nullptr, &nb, &first);
      if (rc < 0) return rc;
    }
  }
  // 3. the reference stops at the first failing record in log order
  size_t accepted = m;
  int result = 0;
  if (nb) {
    accepted = (size_t)first;
    result = ptype[first] == 1 ? LSMCK_WAL_CORRUPTED : LSMCK_WAL_REMOVE_PANIC;
    if (bad_index) *bad_index = first;
    if (bad_expected) *bad_expected = pcrc[first];
    if (bad_crc) *bad_crc = lsmck_crc32_ieee(h + poff[first], plen[first]);
  } else if (stop == LSMCK_WAL_BAD_TYPE) {
    result = LSMCK_WAL_BAD_TYPE;
    if (bad_index) *bad_index = stop_index;
    if (bad_crc) *bad_crc = stop_type;
  }
  if (recs)
    for (size_t i = 0; i < accepted && i < cap; ++i) {
      if (compact)
        lsmck::seg::put_rec((lsmck::seg::Compact16*)recs + i, roff[i], poff[i], rk[i], rv[i], pcrc[i], ptype[i]);
      else
        lsmck::seg::put_rec((lsmck_wal_rec*)recs + i, roff[i], poff[i], rk[i], rv[i], pcrc[i], ptype[i]);
    }
  if (nrec) *nrec = accepted;
  return result;
}

extern "C" {

int lsmck_wal_replay_verify(lsmck_ctx* ctx, const uint8_t* wal, size_t n, unsigned flags, lsmck_wal_rec* recs,
                            size_t cap, size_t* nrec, uint64_t* bad_index, uint32_t* bad_crc, uint32_t* bad_expected) {
  return wal_replay_verify(ctx, wal, n, flags & ~kWalNoGpuWalk, recs, false, cap, nrec, bad_index, bad_crc,
                           bad_expected);
}

int lsmck_wal_replay_verify16(lsmck_ctx* ctx, const uint8_t* wal, size_t n, unsigned flags, lsmck_wal_rec16* recs,
                              size_t cap, size_t* nrec, uint64_t* bad_index, uint32_t* bad_crc,
                              uint32_t* bad_expected) {
  return wal_replay_verify(ctx, wal, n, flags & ~kWalNoGpuWalk, recs, true, cap, nrec, bad_index, bad_crc,
                           bad_expected);
}

// ---------------------------------------------------------------------------
// Whole-tree SSTable verify (Db::load: src/tokio/db.rs:37-59 -> SsTable::load
// -> Checksums::verify, checksums.rs:40-62, for every table of the tree).
//
// SHA-256 is sequential inside a file, so the GPU's parallelism is the number
// of files hashed at once: one lane hashes ~16 MB/s, a whole tree needs
// thousands of files in flight.  The files are therefore streamed in SLICES:
// up to kTreeActive files are open at once, and each ROUND takes the next
// kTreeSlice bytes of every active file (its remaining bytes on its last
// round).  Reader threads pread a round's slices into one pinned slot while
// the GPU runs the previous round from the other; sha256_slices_kernel carries
// each file's SHA state between rounds in a device table (32 B per active
// slot) and writes the digest when the file's last slice is hashed.  A file
// that finishes frees its slot for the next file of the tree.  Host memory is
// two slots of kTreeActive * kTreeSlice bytes whatever the tree's size; the
// digests (32 B per file) come back in one copy at the end.
namespace {

constexpr uint32_t kTreeActive = 8192;        // files in flight
constexpr uint32_t kTreeSlice = 128u << 10;   // bytes of a file per round (multiple of 64; A/B: DESIGN.md 7a)
constexpr unsigned kTreeReaders = 16;  // the GPU box gives a process 16 CPUs
constexpr unsigned kListThreads = 8;   // lsmck_tree_verify's metadata parsing (A/B: DESIGN.md 7a)
constexpr uint64_t kTreeCpuFile = 16ull << 20;  // files this large are hashed on host threads, not a GPU lane
constexpr unsigned kTreeCpuThreads = 4;

// pread exactly n bytes at offset off of fd into dst
int pread_fd(int fd, uint8_t* dst, uint64_t off, uint64_t n) {
  uint64_t got = 0;
  while (got < n) {
    ssize_t k = pread(fd, dst + got, (size_t)std::min<uint64_t>(n - got, 1ull << 30), (off_t)(off + got));
    if (k < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (k == 0) break;
    got += (uint64_t)k;
  }
  return got == n ? 0 : -EAGAIN;  // the file shrank while the tree was read
}

// A file stays open from its first slice to its last: open(2)/close(2) in a
// multi-threaded process contend in the kernel (the fd table, the directory's
// dentry) and cost ~9 us each at 16 threads -- reopening per 64 KiB slice was
// most of the read phase.  Slots past the fd budget (RLIMIT_NOFILE minus a
// reserve) reopen per slice instead.
struct SlotFds {
  std::vector<int> fd;
  uint32_t cached = 0;  // slots [0, cached) keep their file open
  explicit SlotFds(uint32_t slots) : fd(slots, -1) {
    struct rlimit rl;
    uint64_t budget = 0;
    if (getrlimit(RLIMIT_NOFILE, &rl) == 0) {
      const uint64_t cur = rl.rlim_cur == RLIM_INFINITY ? (1ull << 30) : (uint64_t)rl.rlim_cur;
      budget = cur > 1024 ? cur - 1024 : 0;
    }
    cached = (uint32_t)std::min<uint64_t>(slots, budget);
  }
  ~SlotFds() {
    for (int f : fd)
      if (f >= 0) close(f);
  }
  void drop(uint32_t k) {
    if (fd[k] >= 0) close(fd[k]);
    fd[k] = -1;
  }
  // read one slice of `path` for slot k; `last` closes the file after it.
  // An open failure returns kOpenFailed (a panic site of the reference, not -errno)
  static constexpr int kOpenFailed = 1;
  int read(uint32_t k, const char* path, uint8_t* dst, uint64_t off, uint64_t n, bool last) {
    int f = fd[k];
    if (f < 0) {
      f = open(path, O_RDONLY | O_CLOEXEC);
      if (f < 0) return kOpenFailed;
    }
    int rc = pread_fd(f, dst, off, n);
    if (last || rc || k >= cached) {
      close(f);
      f = -1;
    }
    fd[k] = f;
    return rc;
  }
};

double seconds_since(const struct timespec& t0) {
  struct timespec t1;
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
struct Clock {
  struct timespec t;
  Clock() { clock_gettime(CLOCK_MONOTONIC, &t); }
  double lap() {  // seconds since the last lap
    double d = seconds_since(t);
    clock_gettime(CLOCK_MONOTONIC, &t);
    return d;
  }
};

// where verify_tables' wall time goes (lsmck_tree_report)
struct TreeTiming {
  double stat = 0, read = 0, wait = 0, compare = 0;
  uint64_t rounds = 0, bytes = 0;
  uint32_t fds_cached = 0;
};

// fn(i) for i in [0, n) on up to kTreeReaders threads (file-system metadata
// work: stat, small JSON reads -- latency bound, so run many at once)
extern "C++" template <class F>
void host_parallel(size_t n, F&& fn, unsigned max_threads = kTreeReaders) {
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t j; (j = next.fetch_add(1, std::memory_order_relaxed)) < n;) fn(j);
  };
  const unsigned nt = (unsigned)std::min<size_t>(std::max(1u, max_threads), n / 64 + 1);
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

}  // namespace

static int verify_tables(lsmck_ctx* ctx, const char* const* data_paths, const char* const* index_paths,
                         const char* const* checksum_paths, size_t n, int* status, TreeTiming* tm) {
  int rc = check_ctx(ctx);
  TreeTiming tdummy;
  if (!tm) tm = &tdummy;
  Clock clk;
  if (rc) return rc;
  if (n && (!data_paths || !index_paths || !checksum_paths || !status))
    return lsmck_host::set_error(LSMCK_EINVAL, "null path array or status");
  if (2 * n >= (1ull << 32)) return lsmck_host::set_error(LSMCK_EINVAL, "too many tables");
  // file 2i = table i's data file, 2i+1 its index file
  const size_t nf = 2 * n;
  std::vector<const char*> paths(nf);
  std::vector<uint64_t> fsize(nf, 0);
  std::vector<int> ferr(nf, 0);
  for (size_t i = 0; i < n; ++i) {
    paths[2 * i] = data_paths[i];
    paths[2 * i + 1] = index_paths[i];
  }
  // a file that cannot be opened is calculate_checksum's panic (checksums.rs:25):
  // LSMCK_PANIC_OPEN_FILE for the data file, _INDEX for the index file
  auto open_panic = [](size_t f) { return (f & 1) ? LSMCK_PANIC_OPEN_INDEX : LSMCK_PANIC_OPEN_FILE; };
  host_parallel(nf, [&](size_t f) {
    struct stat st;
    if (stat(paths[f], &st) != 0) ferr[f] = open_panic(f);
    else fsize[f] = (uint64_t)st.st_size;
  });
  tm->stat += clk.lap();
  // the checksum files are read by two background threads while the table
  // files stream (the readers leave the CPU idle while a slot's copy runs)
  std::vector<std::string> want_i(n), want_d(n);
  std::vector<int> want_rc(n, 0);
  std::atomic<size_t> want_next{0};
  struct Joiner {
    std::vector<std::thread> t;
    ~Joiner() {
      for (auto& x : t)
        if (x.joinable()) x.join();
    }
  } want_th;
  // (a compaction tick's 142k-table batch: 4 threads 0.82-0.86 s, 2 0.90-0.94 s, 8 0.84-0.99 s; profiles/r05/tk)
  const unsigned jt = ctx->tree_json_threads ? ctx->tree_json_threads : (n >= 16384 ? 4u : 2u);
  for (unsigned t = 0; t < (n >= 64 ? jt : n ? 1u : 0u); ++t)
    want_th.t.emplace_back([&]() {
      for (size_t i; (i = want_next.fetch_add(1, std::memory_order_relaxed)) < n;)
        want_rc[i] = lsmck_host::read_checksum_json(checksum_paths[i], &want_i[i], &want_d[i]);
    });
  const uint32_t active_max = ctx->tree_active ? ctx->tree_active : kTreeActive;
  const uint32_t slice = ctx->tree_slice ? ctx->tree_slice : kTreeSlice;
  std::vector<uint8_t> dig(32 * std::max<size_t>(nf, 1), 0);
  // Large files are hashed on host threads (SHA-NI where the CPU has it,
  // ~1.5-2 GB/s per thread) while the GPU streams the rest: SHA-256 is
  // sequential inside a file, so one file is one GPU lane at ~16 MB/s -- a
  // 230 MB table alone would hold the stream open for 14 s.  The GPU admits
  // the remaining files largest first, so no large file starts at the tail.
  const uint64_t cpu_min = ctx->tree_cpu_file ? ctx->tree_cpu_file : kTreeCpuFile;
  std::vector<size_t> gpu_order, cpu_files;
  for (size_t f = 0; f < nf; ++f) {
    if (ferr[f]) continue;
    (fsize[f] >= cpu_min ? cpu_files : gpu_order).push_back(f);
  }
  std::stable_sort(gpu_order.begin(), gpu_order.end(), [&](size_t a, size_t b) { return fsize[a] > fsize[b]; });
  std::atomic<size_t> cpu_next{0};
  struct CpuJoiner {
    std::vector<std::thread> t;
    ~CpuJoiner() {
      for (auto& x : t)
        if (x.joinable()) x.join();
    }
  } cpu_th;
  for (unsigned t = 0; t < std::min<size_t>(kTreeCpuThreads, cpu_files.size()); ++t)
    cpu_th.t.emplace_back([&]() {
      std::vector<uint8_t> buf(1u << 20);
      for (size_t j; (j = cpu_next.fetch_add(1)) < cpu_files.size();) {
        const size_t f = cpu_files[j];
        int fd = open(paths[f], O_RDONLY | O_CLOEXEC);
        if (fd < 0) {
          ferr[f] = open_panic(f);
          continue;
        }
        lsmck_sha256_ctx c;
        lsmck_sha256_init(&c);
        uint64_t off = 0;
        for (;;) {
          ssize_t k = pread(fd, buf.data(), buf.size(), (off_t)off);
          if (k < 0 && errno == EINTR) continue;
          if (k < 0) {
            ferr[f] = -errno;
            break;
          }
          if (k == 0) break;
          lsmck_sha256_update(&c, buf.data(), (size_t)k);
          off += (uint64_t)k;
        }
        close(fd);
        if (!ferr[f]) lsmck_sha256_final(&c, &dig[32 * f]);
      }
    });
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    DevGuard g(ctx->dev);
    for (auto& S : ctx->stage)
      if ((rc = stage_init(S))) return rc;
    auto& T = ctx->tree;
    if ((rc = ensure_dev(&T.state, &T.cap_state, 8ull * active_max))) return rc;
    if ((rc = ensure_dev(&T.digests, &T.cap_digests, 32 * std::max<size_t>(nf, 1)))) return rc;
    if (!T.kernel_done) HIPCHK(hipEventCreateWithFlags(&T.kernel_done, hipEventDisableTiming));
    // active slots: file index and bytes already scheduled
    std::vector<size_t> slot_file(active_max, SIZE_MAX);
    std::vector<uint64_t> slot_done(active_max, 0);
    std::vector<uint32_t> free_slots;
    for (uint32_t k = active_max; k-- > 0;) free_slots.push_back(k);
    size_t next_file = 0, active = 0;
    // the rounds cycle through ns slots: a round's reads wait for the round
    // ns back (its slot), so with three the reads of round r + 2 overlap the
    // upload and hashing of rounds r and r + 1
    const uint32_t ns = ctx->tree_stages;
    bool busy[3] = {false, false, false}, any_kernel = false;
    uint32_t sl = 0;
    std::vector<uint64_t> rd_off;  // per slice: offset inside its file
    SlotFds fds(active_max);
    if (ctx->tree_open >= 0) fds.cached = (uint32_t)std::min<long>(fds.cached, ctx->tree_open);
    tm->fds_cached = fds.cached;
    for (;;) {
      // admit files into free slots
      while (!free_slots.empty() && next_file < gpu_order.size()) {
        const size_t f = gpu_order[next_file++];
        if (ferr[f]) continue;
        const uint32_t k = free_slots.back();
        free_slots.pop_back();
        slot_file[k] = f;
        slot_done[k] = 0;
        ++active;
      }
      if (active == 0) break;
      // the round's slices: the next `slice` bytes of every active file
      Stage& S = ctx->stage[sl];
      if (busy[sl]) {
        clk.lap();
        HIPCHK(hipEventSynchronize(S.done));
        tm->wait += clk.lap();
        busy[sl] = false;
      }
      std::vector<lsmck::ShaSlice> sv;
      sv.reserve(active);
      rd_off.clear();
      uint64_t pay = 0;
      for (uint32_t k = 0; k < active_max; ++k) {
        if (slot_file[k] == SIZE_MAX) continue;
        const size_t f = slot_file[k];
        const uint64_t left = fsize[f] - slot_done[k];
        const uint32_t len = (uint32_t)std::min<uint64_t>(left, slice);
        lsmck::ShaSlice d{};
        pay = (pay + 15) & ~(uint64_t)15;  // 16-B aligned slices: no funnel, no next-line dword (lsmck_sha256.hip)
        d.off = pay;
        d.total = fsize[f];
        d.len = len;
        d.slot = k;
        d.msg = (uint32_t)f;
        d.flags = (slot_done[k] == 0 ? SHA_SLICE_FIRST : 0u) | (len == left ? SHA_SLICE_LAST : 0u);
        sv.push_back(d);
        rd_off.push_back(slot_done[k]);
        pay += len;
        slot_done[k] += len;
        if (len == left) {  // last slice scheduled: the slot is free for the next round
          slot_file[k] = SIZE_MAX;
          free_slots.push_back(k);
          --active;
        }
      }
      const size_t cnt = sv.size();
      if ((rc = ensure_pinned(ctx->pin_node, &S.h_pay, &S.cap_h_pay, pay + 16, true))) return rc;
      if ((rc = ensure_pinned(ctx->pin_node, &S.h_slices, &S.cap_h_slices, cnt, true))) return rc;
      if ((rc = ensure_dev(&S.d_pay, &S.cap_d_pay, pay + 16))) return rc;
      if ((rc = ensure_dev(&S.d_slices, &S.cap_d_slices, cnt))) return rc;
      memcpy(S.h_slices, sv.data(), cnt * sizeof(lsmck::ShaSlice));
      // read the slices (overlaps the other slot's GPU work, already queued)
      clk.lap();
      std::atomic<size_t> next{0};
      auto work = [&]() {
        for (size_t j; (j = next.fetch_add(1)) < cnt;) {
          const lsmck::ShaSlice& d = sv[j];
          if (ferr[d.msg]) {  // an earlier slice of this file failed: skip the rest
            if (d.flags & SHA_SLICE_LAST) fds.drop(d.slot);
            continue;
          }
          int e = fds.read(d.slot, paths[d.msg], S.h_pay + d.off, rd_off[j], d.len, d.flags & SHA_SLICE_LAST);
          if (e) ferr[d.msg] = e == SlotFds::kOpenFailed ? open_panic(d.msg) : e;
        }
      };
      const unsigned nt = (unsigned)std::min<size_t>(ctx->tree_readers, cnt);
      std::vector<std::thread> th;
      for (unsigned t = 1; t < nt; ++t) th.emplace_back(work);
      work();
      for (auto& t : th) t.join();
      {
        const double dt = clk.lap();
        tm->read += dt;
        static const bool trace = getenv("LSMCK_TREE_TRACE") != nullptr;  // diagnostic: per-round read times
        if (trace) fprintf(stderr, "tree round %llu slot %d: %zu slices, %.1f MB, read %.2f ms\n",
                           (unsigned long long)tm->rounds, sl, cnt, pay / 1e6, dt * 1e3);
      }
      ++tm->rounds;
      HIPCHK(hipMemcpyAsync(S.d_pay, S.h_pay, pay, hipMemcpyHostToDevice, S.s));
      HIPCHK(hipMemcpyAsync(S.d_slices, S.h_slices, cnt * sizeof(lsmck::ShaSlice), hipMemcpyHostToDevice, S.s));
      // the state carried between rounds orders the kernels across the two streams
      if (any_kernel) HIPCHK(hipStreamWaitEvent(S.s, T.kernel_done, 0));
      lsmck::ShaSliceParams P{};
      P.base = S.d_pay;
      P.slices = S.d_slices;
      P.nslices = cnt;
      P.state = T.state;
      P.out = T.digests;
      rc = lsmk_launch_sha256_slices(&P, S.s);
      if (rc) return launch_rc(rc, "sha256 slices kernel");
      HIPCHK(hipEventRecord(T.kernel_done, S.s));
      HIPCHK(hipEventRecord(S.done, S.s));
      busy[sl] = true;
      any_kernel = true;
      sl = sl + 1 < ns ? sl + 1 : 0;
    }
    clk.lap();
    for (uint32_t k = 0; k < ns; ++k)
      if (busy[k]) HIPCHK(hipEventSynchronize(ctx->stage[k].done));
    if (nf) {  // the GPU's digests land at their files' slots; the CPU threads write theirs in place
      std::vector<uint8_t> gd(32 * nf);
      HIPCHK(hipMemcpy(gd.data(), T.digests, 32 * nf, hipMemcpyDeviceToHost));
      for (size_t f : gpu_order) memcpy(&dig[32 * f], &gd[32 * f], 32);
    }
    tm->wait += clk.lap();
  }
  for (auto& x : want_th.t) x.join();
  want_th.t.clear();
  const double json_join = clk.lap();  // (the checksum-file readers still running after the last round)
  tm->compare += json_join;
  for (auto& x : cpu_th.t) x.join();
  cpu_th.t.clear();
  host_parallel(n, [&](size_t i) {
    status[i] = ferr[2 * i] ? ferr[2 * i] : ferr[2 * i + 1];
    if (status[i] == 0) {
      char db[45], ib[45];
      lsmck_base64_encode(&dig[64 * i], 32, db);
      lsmck_base64_encode(&dig[64 * i + 32], 32, ib);
      if (want_rc[i]) status[i] = want_rc[i];
      else if (want_d[i] != db) status[i] = LSMCK_DATA_MISMATCH;  // data first, as checksums.rs:49-60
      else if (want_i[i] != ib) status[i] = LSMCK_INDEX_MISMATCH;
    }
  });
  int bad = 0;
  for (size_t i = 0; i < n; ++i) bad += status[i] != 0;
  tm->bytes = std::accumulate(fsize.begin(), fsize.end(), (uint64_t)0);
  tm->compare += clk.lap();
  if (getenv("LSMCK_TREE_TRACE"))  // diagnostic: where the batch's time went
    fprintf(stderr,
            "tree verify: %zu tables, %.2f GB: stat %.3f s, read %.3f s, slot wait + last rounds %.3f s, "
            "checksum-file readers after the last round %.3f s, compare %.3f s, %llu rounds\n",
            n, tm->bytes / 1e9, tm->stat, tm->read, tm->wait, json_join, tm->compare - json_join,
            (unsigned long long)tm->rounds);
  return bad;
}

int lsmck_checksums_verify_many(lsmck_ctx* ctx, const char* const* data_paths, const char* const* index_paths,
                                const char* const* checksum_paths, size_t n, int* status) {
  return verify_tables(ctx, data_paths, index_paths, checksum_paths, n, status, nullptr);
}

}  // extern "C"

// The tables split over several devices (one host thread, one
// context and one set of pinned slots per device, no data exchange): contiguous
// runs of tables balanced by bytes, each verified by its own context in its
// own thread, so every device's PCIe link streams its share.  Statuses land in
// place; the timing fields are the slowest device's, byte and round counts sum.
static int verify_tables_multi(lsmck_ctx* const* ctxs, size_t nctx, const char* const* data_paths,
                               const char* const* index_paths, const char* const* checksum_paths, size_t n,
                               int* status, TreeTiming* tm) {
  if (!ctxs || nctx == 0) return lsmck_host::set_error(LSMCK_EINVAL, "no contexts");
  for (size_t k = 0; k < nctx; ++k)
    if (!ctxs[k]) return lsmck_host::set_error(LSMCK_EINVAL, "null context");
  if (nctx == 1 || n < 2) return verify_tables(ctxs[0], data_paths, index_paths, checksum_paths, n, status, tm);
  std::vector<uint64_t> bytes(n, 0);
  host_parallel(n, [&](size_t i) {
    struct stat st;
    if (stat(data_paths[i], &st) == 0) bytes[i] += (uint64_t)st.st_size;
    if (stat(index_paths[i], &st) == 0) bytes[i] += (uint64_t)st.st_size;
  });
  uint64_t total = 0;
  for (uint64_t b : bytes) total += b;
  std::vector<size_t> cut(nctx + 1, n);
  cut[0] = 0;
  uint64_t acc = 0;
  size_t k = 1;
  for (size_t i = 0; i < n && k < nctx; ++i) {
    acc += bytes[i];
    while (k < nctx && acc * nctx >= total * k) cut[k++] = i + 1;
  }
  std::vector<int> rc(nctx, 0);
  std::vector<TreeTiming> tms(nctx);
  std::vector<std::string> errs(nctx);
  std::vector<std::thread> th;
  for (size_t j = 0; j < nctx; ++j)
    th.emplace_back([&, j]() {
      const size_t a = cut[j], b = cut[j + 1];
      if (a >= b) return;
      rc[j] = verify_tables(ctxs[j], data_paths + a, index_paths + a, checksum_paths + a, b - a, status + a, &tms[j]);
      if (rc[j] < 0) errs[j] = lsmck_last_error();  // thread-local: carry it back
    });
  for (auto& t : th) t.join();
  int bad = 0;
  for (size_t j = 0; j < nctx; ++j) {
    if (rc[j] < 0) return lsmck_host::set_error(rc[j], errs[j].c_str());
    bad += rc[j];
  }
  if (tm) {
    for (auto& x : tms) {
      tm->stat = std::max(tm->stat, x.stat);
      tm->read = std::max(tm->read, x.read);
      tm->wait = std::max(tm->wait, x.wait);
      tm->compare = std::max(tm->compare, x.compare);
      tm->rounds += x.rounds;
      tm->bytes += x.bytes;
      tm->fds_cached += x.fds_cached;
    }
  }
  return bad;
}

extern "C" {

int lsmck_checksums_verify_many_multi(lsmck_ctx* const* ctxs, size_t nctx, const char* const* data_paths,
                                      const char* const* index_paths, const char* const* checksum_paths, size_t n,
                                      int* status) {
  if (n && (!data_paths || !index_paths || !checksum_paths || !status))
    return lsmck_host::set_error(LSMCK_EINVAL, "null path array or status");
  return verify_tables_multi(ctxs, nctx, data_paths, index_paths, checksum_paths, n, status, nullptr);
}

// ---------------------------------------------------------------------------
// Db::load's table scan (src/tokio/db.rs:37-59) in native code: per level
// create_dir_all + read_dir, every entry whose (UTF-8) name contains
// "metadata", SsTableMetadata::load (sstable_metadata.rs:76-83), then the
// tables' checksum verify as one lsmck_checksums_verify_many batch.  The
// reference verifies in read_dir order and stops at the first failure; the
// batch verifies every table and reports the first failure in that order.
namespace {

bool valid_utf8(const char* s) {
  const unsigned char* p = (const unsigned char*)s;
  while (*p) {
    unsigned c = *p, k;
    uint32_t cp;
    if (c < 0x80) {
      ++p;
      continue;
    } else if ((c & 0xE0) == 0xC0) k = 1, cp = c & 0x1F;
    else if ((c & 0xF0) == 0xE0) k = 2, cp = c & 0x0F;
    else if ((c & 0xF8) == 0xF0) k = 3, cp = c & 0x07;
    else return false;
    for (unsigned j = 1; j <= k; ++j) {
      if ((p[j] & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (p[j] & 0x3F);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000) || cp > 0x10FFFF ||
        (cp >= 0xD800 && cp <= 0xDFFF))
      return false;
    p += k + 1;
  }
  return true;
}

int mkdir_p(const std::string& path) {  // fs::create_dir_all
  struct stat st;
  if (stat(path.c_str(), &st) == 0) return S_ISDIR(st.st_mode) ? 0 : -EEXIST;
  size_t cut = path.find_last_of('/');
  if (cut != std::string::npos && cut > 0) {
    int rc = mkdir_p(path.substr(0, cut));
    if (rc) return rc;
  }
  if (mkdir(path.c_str(), 0777) != 0 && errno != EEXIST) return -errno;
  return 0;
}

}  // namespace

static int tree_verify_impl(lsmck_ctx* const* ctxs, size_t nctx, const char* base, lsmck_tree_report* rep,
                            lsmck_tree_listed_fn fn = nullptr, void* user = nullptr);

int lsmck_tree_verify_listed(lsmck_ctx* ctx, const char* base, lsmck_tree_report* rep, lsmck_tree_listed_fn fn,
                             void* user) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  lsmck_ctx* one[1] = {ctx};
  return tree_verify_impl(one, 1, base, rep, fn, user);
}

int lsmck_tree_verify(lsmck_ctx* ctx, const char* base, lsmck_tree_report* rep) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  return tree_verify_impl(&ctx, 1, base, rep);
}

int lsmck_tree_verify_multi(lsmck_ctx* const* ctxs, size_t nctx, const char* base, lsmck_tree_report* rep) {
  if (!ctxs || nctx == 0) return lsmck_host::set_error(LSMCK_EINVAL, "no contexts");
  for (size_t k = 0; k < nctx; ++k)
    if (!ctxs[k]) return lsmck_host::set_error(LSMCK_EINVAL, "null context");
  return tree_verify_impl(ctxs, nctx, base, rep);
}

}  // extern "C"

static int tree_verify_impl(lsmck_ctx* const* ctxs, size_t nctx, const char* base, lsmck_tree_report* rep,
                            lsmck_tree_listed_fn fn, void* user) {
  lsmck_ctx* ctx = ctxs[0];
  int rc = 0;
  if (!base || !rep) return lsmck_host::set_error(LSMCK_EINVAL, "null base path or report");
  memset(rep, 0, sizeof *rep);
  rep->first_index = UINT64_MAX;
  struct timespec t0;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  struct {
    std::vector<lsmck_table_entry> ents;
    std::vector<std::string> dps, ips, cps;
  } listed;  // lives until the verify returns (lsmck_tree_verify_listed's contract)
  // The metadata files are parsed while the level directories are still
  // being read: the scan hands batches of names to the parsing threads as it
  // goes (a readdir of the 1.1 M names of a 229k-table tree and the 229k
  // small-file opens cost about the same, and only the opens parallelise).
  // 8 threads: small-file system calls contend in the kernel (229k metadata
  // files: 1 thread 1.25 s, 4 1.01 s, 8 0.80 s, 16 0.89 s, 32 1.25 s)
  struct ListBatch {
    std::vector<std::string> path;
    std::vector<lsmck_host::TableMeta> meta;
    std::vector<int> st;
    bool done = false;  // parsed (under the lister's mutex)
  };
  struct Lister {
    std::vector<std::unique_ptr<ListBatch>> batches;  // load order
    std::mutex mu;
    std::condition_variable cv;
    size_t next = 0, parsed = 0;
    bool done = false;
    std::condition_variable cv_parsed;
    std::vector<std::thread> th;
    void finish() {
      {
        std::lock_guard<std::mutex> lk(mu);
        done = true;
      }
      cv.notify_all();
      for (auto& t : th)
        if (t.joinable()) t.join();
    }
    ~Lister() { finish(); }
  } lister;
  {
    const unsigned lthreads = ctx->tree_list_threads ? ctx->tree_list_threads : kListThreads;
    for (unsigned t = 0; t < lthreads; ++t)
      lister.th.emplace_back([&lister]() {
        for (;;) {
          ListBatch* b;
          {
            std::unique_lock<std::mutex> lk(lister.mu);
            lister.cv.wait(lk, [&] { return lister.next < lister.batches.size() || lister.done; });
            if (lister.next >= lister.batches.size()) return;
            b = lister.batches[lister.next++].get();
          }
          b->meta.resize(b->path.size());
          b->st.assign(b->path.size(), 0);
          for (size_t i = 0; i < b->path.size(); ++i)
            if (lsmck_host::read_metadata_json(b->path[i].c_str(), &b->meta[i])) b->st[i] = LSMCK_META_PANIC;
          {
            std::lock_guard<std::mutex> lk(lister.mu);
            ++lister.parsed;
            b->done = true;
          }
          lister.cv_parsed.notify_all();
        }
      });
  }
  std::unique_ptr<ListBatch> cur(new ListBatch);
  auto publish = [&]() {
    if (cur->path.empty()) return;
    {
      std::lock_guard<std::mutex> lk(lister.mu);
      lister.batches.push_back(std::move(cur));
    }
    lister.cv.notify_one();
    cur.reset(new ListBatch);
  };
  for (int lv = 0; lv < LSMCK_SSTABLE_MAX_LEVEL; ++lv) {  // fs::create_dir_all of every level, in order
    const std::string dir = lsmck_host::path_push(base, "level-" + std::to_string(lv));
    if ((rc = mkdir_p(dir))) return lsmck_host::set_errno_error(-rc, "create_dir_all", dir.c_str());
  }
  // read_dir of one level: its metadata names, in batches to the parsers;
  // hook(batches published so far) after each full batch
  const size_t list_batch = ctx->tree_list_batch ? ctx->tree_list_batch : 1024u;
  auto scan = [&](int lv, const std::function<void(size_t)>& hook) -> int {
    const std::string dir = lsmck_host::path_push(base, "level-" + std::to_string(lv));
    DIR* d = opendir(dir.c_str());
    if (!d) return lsmck_host::set_errno_error(errno, "read_dir", dir.c_str());
    for (;;) {
      errno = 0;
      struct dirent* e = readdir(d);
      if (!e) {
        if (errno) {
          int er = errno;
          closedir(d);
          return lsmck_host::set_errno_error(er, "read_dir", dir.c_str());
        }
        break;
      }
      if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
      if (strstr(e->d_name, "metadata") && valid_utf8(e->d_name)) {
        cur->path.push_back(dir + "/" + e->d_name);
        if (cur->path.size() >= list_batch) {
          publish();
          if (hook) {
            size_t nb;
            {
              std::lock_guard<std::mutex> lk(lister.mu);
              nb = lister.batches.size();
            }
            hook(nb);
          }
        }
      }
    }
    closedir(d);
    publish();
    return 0;
  };
  // Listing beside the verify (tree_overlap, default): the highest level is
  // read first -- an LSM tree keeps most of its bytes there (the synthetic
  // tree 85 %, in its largest tables) -- and its tables are verified while the
  // lower levels are listed; the lower levels' tables follow in a second
  // batch.  The verify order is free: statuses land per table and the report
  // takes the first failure in read_dir order (levels 0, 1, ...).
  // table paths: construct_path = base_path / level-<level> / file (sstable_metadata.rs:43-48)
  struct Part {
    std::vector<std::string> dp, ip, cp;
    std::vector<size_t> which;  // indices into the part's tables
    std::vector<int> vst;
    TreeTiming tm;
    int rc = 0;
    std::string err;
  };
  auto paths_of = [](const std::vector<lsmck_host::TableMeta>& meta, const std::vector<int>& st, size_t i0, size_t i1,
                     Part* P) {
    for (size_t i = i0; i < i1; ++i) {
      if (st[i]) continue;
      const std::string lvdir = lsmck_host::path_push(meta[i].base_path, "level-" + std::to_string(meta[i].level));
      P->dp.push_back(lsmck_host::path_push(lvdir, meta[i].data_filename));
      P->ip.push_back(lsmck_host::path_push(lvdir, meta[i].index_filename));
      P->cp.push_back(lsmck_host::path_push(lvdir, meta[i].checksum_filename));
      P->which.push_back(i);
    }
  };
  auto run_part = [ctxs, nctx](Part* P) {
    const size_t m = P->which.size();
    std::vector<const char*> dpp(m), ipp(m), cpp(m);
    for (size_t j = 0; j < m; ++j) dpp[j] = P->dp[j].c_str(), ipp[j] = P->ip[j].c_str(), cpp[j] = P->cp[j].c_str();
    P->vst.assign(std::max<size_t>(m, 1), 0);
    P->rc = verify_tables_multi(ctxs, nctx, dpp.data(), ipp.data(), cpp.data(), m, P->vst.data(), &P->tm);
    if (P->rc < 0) P->err = lsmck_last_error();  // thread-local: carried back
  };
  // While the metadata files are parsed, each context's staging slots, device
  // buffers and digest table are allocated and the pinned pages mapped: a
  // fresh process otherwise pays for them inside the stream (the first
  // Db::load of a process ran its table verify ~2 s slower than a repeat).
  struct Prewarm {
    std::vector<std::thread> t;
    ~Prewarm() {
      for (auto& x : t)
        if (x.joinable()) x.join();
    }
  } prewarm;
  auto start_prewarm = [&](size_t tables) {
    // Grow the process's descriptor table now, in one step: the verify keeps
    // up to 8192 files open, and a table grown descriptor by descriptor under
    // 16 reader threads is resized ~8 times, each resize waiting for an RCU
    // grace period (a process's first verify read its first round in 1.1 s
    // instead of 12 ms; LSMCK_TREE_TRACE).  Tables never shrink.
    prewarm.t.emplace_back([c = ctxs[0]]() {
      struct rlimit rl;
      if (getrlimit(RLIMIT_NOFILE, &rl) != 0 || rl.rlim_cur == RLIM_INFINITY) return;
      const uint32_t active = c->tree_active ? c->tree_active : kTreeActive;
      const uint64_t want = std::min<uint64_t>((uint64_t)rl.rlim_cur - 1, (uint64_t)active + 512u);
      const int fd = open("/dev/null", O_RDONLY | O_CLOEXEC);
      if (fd < 0) return;
      const int hi = fcntl(fd, F_DUPFD_CLOEXEC, (int)want);
      if (hi >= 0) close(hi);
      close(fd);
    });
    for (size_t k = 0; k < nctx; ++k)
      prewarm.t.emplace_back([c = ctxs[k], n = tables]() {
        const uint32_t active = c->tree_active ? c->tree_active : kTreeActive;
        const uint32_t slice = c->tree_slice ? c->tree_slice : kTreeSlice;
        const size_t files = std::min<size_t>(active, 2 * n);
        const size_t bytes = files * ((size_t)slice + 16) + 16;  // slices are 16-B aligned in the slot
        std::lock_guard<std::mutex> lk(c->mu);
        DevGuard g(c->dev);
        for (auto& S : c->stage) {
          if (stage_init(S) || ensure_pinned(c->pin_node, &S.h_pay, &S.cap_h_pay, bytes, true) ||
              ensure_pinned(c->pin_node, &S.h_slices, &S.cap_h_slices, files, true) ||
              ensure_dev(&S.d_pay, &S.cap_d_pay, bytes) || ensure_dev(&S.d_slices, &S.cap_d_slices, files))
            return;  // the verify reports it
          // map the pinned pages now, not on the readers' first touch
          if (madvise(S.h_pay, S.cap_h_pay, 23 /* MADV_POPULATE_WRITE */) != 0)
            for (size_t o = 0; o < S.cap_h_pay; o += 4096) ((volatile uint8_t*)S.h_pay)[o] = 0;
        }
        (void)ensure_dev(&c->tree.state, &c->tree.cap_state, 8ull * active);
        (void)ensure_dev(&c->tree.digests, &c->tree.cap_digests, 32 * 2 * n);
      });
  };
  // The top level in two parts: its first 8 x tree_overlap tables (16k by
  // default) go to the verify as soon as they are parsed, while the rest of
  // its directory is read; the rest of it follows as a second part (a top
  // level with fewer tables is one part, started once read).  Each part runs
  // verify_tables_multi on its own thread; their GPU halves take the
  // context in turn.
  const size_t early_tables = 8u * (size_t)std::max<long>(ctx->tree_overlap, 1);
  const int top = LSMCK_SSTABLE_MAX_LEVEL - 1;
  struct TopPart {
    std::vector<ListBatch*> batches;
    Part part;
    size_t first = 0, tables = 0;  // its first table's index in the top level, its tables
    std::thread th;
  };
  TopPart ta, tb;
  struct PartJoin {
    TopPart* a;
    TopPart* b;
    ~PartJoin() {
      if (a->th.joinable()) a->th.join();
      if (b->th.joinable()) b->th.join();
    }
  } part_join{&ta, &tb};
  auto start_top = [&](TopPart* P, size_t b0, size_t b1, bool prewarm_first) {
    {
      std::lock_guard<std::mutex> lk(lister.mu);
      for (size_t k = b0; k < b1; ++k) P->batches.push_back(lister.batches[k].get());
      for (size_t k = 0; k < b0; ++k) P->first += lister.batches[k]->path.size();  // (published: sizes final)
      for (ListBatch* B : P->batches) P->tables += B->path.size();
    }
    if (prewarm_first) start_prewarm(P->tables);
    P->th = std::thread([&, P, prewarm_first]() {
      {
        std::unique_lock<std::mutex> lk(lister.mu);
        lister.cv_parsed.wait(lk, [&] {
          for (ListBatch* B : P->batches)
            if (!B->done) return false;
          return true;
        });
      }
      std::vector<lsmck_host::TableMeta> m;
      std::vector<int> sv;
      for (ListBatch* B : P->batches) {
        m.insert(m.end(), B->meta.begin(), B->meta.end());
        sv.insert(sv.end(), B->st.begin(), B->st.end());
      }
      paths_of(m, sv, 0, m.size(), &P->part);
      if (prewarm_first)
        for (auto& x : prewarm.t) x.join();
      run_part(&P->part);
    });
  };
  const bool overlap = ctx->tree_overlap > 0;
  bool early = false;
  size_t ka = 0;  // top-level batches in the first part
  if ((rc = scan(top, [&](size_t nb) {
         if (overlap && !early && nb * list_batch >= early_tables) {
           early = true;
           ka = nb;
           start_top(&ta, 0, nb, true);
         }
       })))
    return rc;
  size_t top_batches = 0;
  {
    std::unique_lock<std::mutex> lk(lister.mu);
    top_batches = lister.batches.size();
    lister.cv_parsed.wait(lk, [&] { return lister.parsed >= top_batches; });
  }
  size_t n_top = 0;
  for (size_t k = 0; k < top_batches; ++k) n_top += lister.batches[k]->path.size();
  if (early) {
    if (top_batches > ka) start_top(&tb, ka, top_batches, false);
  } else if (overlap && n_top >= (size_t)ctx->tree_overlap) {
    early = true;
    ka = top_batches;
    start_top(&ta, 0, top_batches, true);
  }
  std::vector<lsmck_host::TableMeta> top_meta;
  std::vector<std::string> top_mpath;
  std::vector<int> top_st;
  for (size_t k = 0; k < top_batches; ++k) {
    ListBatch& B = *lister.batches[k];
    top_mpath.insert(top_mpath.end(), B.path.begin(), B.path.end());
    top_meta.insert(top_meta.end(), B.meta.begin(), B.meta.end());
    top_st.insert(top_st.end(), B.st.begin(), B.st.end());
  }
  Part prest;
  for (int lv = 0; lv < top; ++lv)
    if ((rc = scan(lv, {}))) return rc;
  lister.finish();
  // the listing in read_dir order: levels 0 .. top - 1, then the top level (scanned first)
  std::vector<std::string> mpath;
  std::vector<lsmck_host::TableMeta> meta;
  std::vector<int> st;
  for (size_t k = top_batches; k < lister.batches.size(); ++k) {
    ListBatch& B = *lister.batches[k];
    for (auto& x : B.path) mpath.push_back(std::move(x));
    for (auto& x : B.meta) meta.push_back(std::move(x));
    st.insert(st.end(), B.st.begin(), B.st.end());
  }
  const size_t n_low = mpath.size();
  for (size_t i = 0; i < n_top; ++i) {
    mpath.push_back(std::move(top_mpath[i]));
    meta.push_back(std::move(top_meta[i]));
    st.push_back(top_st[i]);
  }
  const size_t n = mpath.size();
  if (!early && n) start_prewarm(n);
  paths_of(meta, st, 0, early ? n_low : n, &prest);
  rep->tables = n;
  rep->list_seconds = seconds_since(t0);
  if (fn) {  // the caller's half of Db::load starts from this listing
    std::vector<lsmck_table_entry> ents(n);
    std::vector<std::string> dps(n), ips(n), cps(n);
    for (size_t i = 0; i < n; ++i) {
      lsmck_table_entry& e = ents[i];
      e.metadata_path = mpath[i].c_str();
      e.status = st[i];
      e.level = meta[i].level;
      e.id = st[i] ? "" : meta[i].id.c_str();
      if (!st[i]) {
        const std::string lvdir = lsmck_host::path_push(meta[i].base_path, "level-" + std::to_string(meta[i].level));
        dps[i] = lsmck_host::path_push(lvdir, meta[i].data_filename);
        ips[i] = lsmck_host::path_push(lvdir, meta[i].index_filename);
        cps[i] = lsmck_host::path_push(lvdir, meta[i].checksum_filename);
      }
      e.data_path = dps[i].c_str();
      e.index_path = ips[i].c_str();
      e.checksum_path = cps[i].c_str();
    }
    listed.ents.swap(ents);
    listed.dps.swap(dps);
    listed.ips.swap(ips);
    listed.cps.swap(cps);
    fn(user, listed.ents.data(), n);
  }
  if (!early)
    for (auto& x : prewarm.t) x.join();
  run_part(&prest);  // (beside the top level's verify: its host half; its GPU half waits for the context)
  for (TopPart* P : {&ta, &tb})
    if (P->th.joinable()) P->th.join();
  for (Part* P : {&prest, &ta.part, &tb.part})
    if (P->rc < 0) return lsmck_host::set_error(P->rc, P->err.c_str());
  TreeTiming tm = prest.tm;
  for (Part* P : {&ta.part, &tb.part}) {
    tm.bytes += P->tm.bytes;
    tm.rounds += P->tm.rounds;
    tm.stat += P->tm.stat;
    tm.read += P->tm.read;
    tm.wait += P->tm.wait;
    tm.compare += P->tm.compare;
    tm.fds_cached = std::max(tm.fds_cached, P->tm.fds_cached);
  }
  rep->table_bytes = tm.bytes;
  rep->rounds = tm.rounds;
  rep->stat_seconds = tm.stat;
  rep->read_seconds = tm.read;
  rep->gpu_wait_seconds = tm.wait;
  rep->compare_seconds = tm.compare;
  rep->fds_cached = tm.fds_cached;
  for (size_t j = 0; j < prest.which.size(); ++j) st[prest.which[j]] = prest.vst[j];
  for (TopPart* P : {&ta, &tb})
    for (size_t j = 0; j < P->part.which.size(); ++j) st[n_low + P->first + P->part.which[j]] = P->part.vst[j];
  rep->verify_seconds = seconds_since(t0) - rep->list_seconds;
  for (size_t i = 0; i < n; ++i) {
    if (!st[i]) continue;
    if (rep->bad_tables++ == 0) {
      rep->first_index = i;
      rep->first_status = st[i];
      snprintf(rep->first_metadata_path, sizeof rep->first_metadata_path, "%s", mpath[i].c_str());
    }
  }
  return rep->bad_tables ? 1 : 0;
}

extern "C" {

// ---------------------------------------------------------------------------
void* lsmck_dev_alloc(lsmck_ctx* ctx, size_t bytes) {
  if (!ctx) return nullptr;
  DevGuard g(ctx->dev);
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
  if (e != hipSuccess) {
    hip_error(e, "hipMalloc");
    return nullptr;
  }
  return p;
}
void lsmck_dev_free(lsmck_ctx* ctx, void* p) {
  if (!ctx || !p) return;
  DevGuard g(ctx->dev);
  (void)hipFree(p);
}
void* lsmck_host_alloc_pinned(lsmck_ctx* ctx, size_t bytes) {
  if (!ctx) return nullptr;
  DevGuard g(ctx->dev);
  void* p = nullptr;
  hipError_t e = host_malloc_near(&p, bytes ? bytes : 1, ctx->pin_node);  // (on the device's node: see stage_numa)
  if (e != hipSuccess) {
    hip_error(e, "hipHostMalloc");
    return nullptr;
  }
  return p;
}
void lsmck_host_free_pinned(lsmck_ctx* ctx, void* p) {
  if (!ctx || !p) return;
  DevGuard g(ctx->dev);
  host_free(p);
}
int lsmck_memcpy_h2d(lsmck_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream) {
  if (!ctx) return LSMCK_EINVAL;
  DevGuard g(ctx->dev);
  hipStream_t st = pick_stream(ctx, stream);
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}
int lsmck_memcpy_d2h(lsmck_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream) {
  if (!ctx) return LSMCK_EINVAL;
  DevGuard g(ctx->dev);
  hipStream_t st = pick_stream(ctx, stream);
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}
int lsmck_memset_dev(lsmck_ctx* ctx, void* dst, int value, size_t bytes, void* stream) {
  if (!ctx) return LSMCK_EINVAL;
  DevGuard g(ctx->dev);
  HIPCHK(hipMemsetAsync(dst, value, bytes, pick_stream(ctx, stream)));
  return 0;
}
int lsmck_stream_sync(lsmck_ctx* ctx, void* stream) {
  if (!ctx) return LSMCK_EINVAL;
  DevGuard g(ctx->dev);
  HIPCHK(hipStreamSynchronize(pick_stream(ctx, stream)));
  return 0;
}
int lsmck_gen_stream(lsmck_ctx* ctx, uint8_t* dst_dev, uint64_t seed, uint64_t byte_off, size_t n, void* stream) {
  if (!ctx) return LSMCK_EINVAL;
  DevGuard g(ctx->dev);
  int rc = lsmk_launch_gen_stream(dst_dev, seed, byte_off, n, pick_stream(ctx, stream));
  return rc ? launch_rc(rc, "gen_stream kernel") : 0;
}

}  // extern "C"
