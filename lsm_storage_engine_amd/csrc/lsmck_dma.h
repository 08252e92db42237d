// lsmck_dma.h -- device -> host copies on the SDMA engines, split over several.
//
// The WAL replay's records come back to the host beside the CRC pass
// (lsmck_api.cpp wal_finish).  hipMemcpyAsync moved them at ~30 GB/s on the
// pool's boxes -- one SDMA engine -- and, for the 2 GiB record array, as
// __amd_rocclr_copyBuffer, a blit kernel on the compute units that stretched
// the CRC pass beside it from 20.5 to 41-53 ms (profiles/r04/z5).  Driven
// through HSA directly, a copy dealt over four SDMA engines moves 1 GiB in
// ~20 ms (53 GB/s) and leaves a streaming kernel beside it untouched
// (tools/microbench_d2h.hip, profiles/r05/d2h).
#ifndef LSMCK_DMA_H
#define LSMCK_DMA_H
#include <stddef.h>

namespace lsmck_dma {

constexpr int kMaxChunks = 64;
constexpr int kMaxSignals = 256;  // completion signals per copier: several jobs in flight use disjoint ranges

struct Copier;  // one per context: the GPU's agent, its SDMA engines, a pool of completion signals

// nullptr when HSA or the device's SDMA engines are not usable (the caller
// then copies with hipMemcpyAsync).  dev_ptr: any allocation of the device.
Copier* create(const void* dev_ptr);
void destroy(Copier* c);
int engines(const Copier* c);  // SDMA engines usable for device -> host

// One device -> host copy of `bytes`, cut into `chunks` pieces (4 KiB
// multiples, the last one shorter) dealt round-robin over `engines` engines:
// chunk i lands after chunk i - engines (one engine runs its pieces in
// order), so the copied prefix grows about evenly.  dst must be page-locked
// (hipHostMalloc / hipHostRegister).  Issue returns at once; one job per
// copier at a time.  0 or a negative code (the copy did not start: use
// hipMemcpyAsync).  sig_base: the job's first completion signal; jobs in
// flight together take disjoint ranges [sig_base, sig_base + chunks) of the
// copier's kMaxSignals (the pipelined WAL replay reads each part back as its
// records are emitted).
struct Job {
  int n = 0;                      // chunks issued
  int base = 0;                   // its signals: [base, base + n)
  size_t off[kMaxChunks + 1] = {};  // chunk i: bytes [off[i], off[i+1])
};
int d2h(Copier* c, void* dst, const void* src, size_t bytes, int engines, int chunks, Job* j, int sig_base = 0);
// whether chunk i has landed (no wait); a failed chunk counts as landed (wait() reports it)
bool landed(Copier* c, const Job& j, int i);
// wait for chunk i (every chunk: wait_all).  0, or a negative code if the
// engine reported an error.
int wait(Copier* c, const Job& j, int i);
int wait_all(Copier* c, const Job& j);

}  // namespace lsmck_dma
#endif
