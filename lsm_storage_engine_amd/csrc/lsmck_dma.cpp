// lsmck_dma.cpp -- device -> host copies dealt over the GPU's SDMA engines
// through HSA (see lsmck_dma.h for why).  HIP runs on the same HSA runtime, so
// its allocations are HSA allocations: hsa_amd_pointer_info names their agents.
#include "lsmck_dma.h"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <cstdint>
#include <mutex>

namespace lsmck_dma {

struct Copier {
  hsa_agent_t gpu{};
  hsa_agent_t cpu{};  // the first CPU agent (a host array's own agent is used when HSA names one)
  uint32_t eng[16] = {};
  int neng = 0;
  hsa_signal_t sig[kMaxSignals] = {};
  int nsig = 0;
};

namespace {

bool hsa_up() {
  static std::once_flag once;
  static bool ok = false;
  std::call_once(once, [] { ok = hsa_init() == HSA_STATUS_SUCCESS; });
  return ok;
}

hsa_status_t first_cpu(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *(hsa_agent_t*)data = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

bool is_type(hsa_agent_t a, hsa_device_type_t want) {
  hsa_device_type_t t;
  return a.handle && hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == want;
}

// the allocation holding p: its kind, owning agent and the address agents use
bool pointer(const void* p, hsa_amd_pointer_info_t* info) {
  info->size = sizeof(*info);
  return hsa_amd_pointer_info(const_cast<void*>(p), info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS;
}

}  // namespace

Copier* create(const void* dev_ptr) {
  if (!dev_ptr || !hsa_up()) return nullptr;
  hsa_amd_pointer_info_t pi;
  if (!pointer(dev_ptr, &pi) || pi.type != HSA_EXT_POINTER_TYPE_HSA || !is_type(pi.agentOwner, HSA_DEVICE_TYPE_GPU))
    return nullptr;
  Copier* c = new Copier;
  c->gpu = pi.agentOwner;
  hsa_iterate_agents(first_cpu, &c->cpu);
  uint32_t avail = 0, pref = 0;
  if (!c->cpu.handle || hsa_amd_memory_copy_engine_status(c->cpu, c->gpu, &avail) != HSA_STATUS_SUCCESS || !avail) {
    delete c;
    return nullptr;
  }
  if (hsa_amd_memory_get_preferred_copy_engine(c->cpu, c->gpu, &pref) != HSA_STATUS_SUCCESS) pref = 0;
  // the runtime's preferred engines for this direction first, then the rest
  for (int pass = 0; pass < 2; ++pass)
    for (int b = 0; b < 16; ++b) {
      const uint32_t m = 1u << b;
      if ((avail & m) && (pass == 0) == ((pref & m) != 0)) c->eng[c->neng++] = m;
    }
  return c;
}

void destroy(Copier* c) {
  if (!c) return;
  for (int i = 0; i < c->nsig; ++i) hsa_signal_destroy(c->sig[i]);
  delete c;
}

int engines(const Copier* c) { return c ? c->neng : 0; }

int d2h(Copier* c, void* dst, const void* src, size_t bytes, int engines, int chunks, Job* j, int sig_base) {
  j->n = 0;
  j->base = sig_base;
  if (!c || !dst || !src || sig_base < 0) return -1;
  if (!bytes) return 0;
  hsa_amd_pointer_info_t pd, ps;
  if (!pointer(dst, &pd) || (pd.type != HSA_EXT_POINTER_TYPE_HSA && pd.type != HSA_EXT_POINTER_TYPE_LOCKED))
    return -2;  // pageable host memory: not for the engines
  if (!pointer(src, &ps) || ps.type != HSA_EXT_POINTER_TYPE_HSA || ps.agentOwner.handle != c->gpu.handle) return -3;
  // a locked (registered) array is addressed by the agents at its agent base
  uint8_t* d = (uint8_t*)dst;
  if (pd.type == HSA_EXT_POINTER_TYPE_LOCKED && pd.agentBaseAddress && pd.hostBaseAddress)
    d = (uint8_t*)pd.agentBaseAddress + ((uint8_t*)dst - (uint8_t*)pd.hostBaseAddress);
  const hsa_agent_t dst_agent = is_type(pd.agentOwner, HSA_DEVICE_TYPE_CPU) ? pd.agentOwner : c->cpu;
  engines = std::max(1, std::min(engines, c->neng));
  chunks = std::max(engines, std::min(chunks, kMaxChunks));
  size_t per = (bytes + (size_t)chunks - 1) / (size_t)chunks;
  per = (per + 4095) & ~(size_t)4095;
  const int n = (int)((bytes + per - 1) / per);
  if (sig_base + n > kMaxSignals) return -7;
  while (c->nsig < sig_base + n) {
    if (hsa_signal_create(1, 0, nullptr, &c->sig[c->nsig]) != HSA_STATUS_SUCCESS) return -4;
    ++c->nsig;
  }
  for (int i = 0; i < n; ++i) {
    const size_t o = per * (size_t)i, len = std::min(per, bytes - o);
    j->off[i] = o;
    j->off[i + 1] = o + len;
    hsa_signal_store_relaxed(c->sig[sig_base + i], 1);
    const hsa_status_t s = hsa_amd_memory_async_copy_on_engine(
        d + o, dst_agent, (const uint8_t*)src + o, c->gpu, len, 0, nullptr, c->sig[sig_base + i],
        (hsa_amd_sdma_engine_id_t)c->eng[i % engines], true);
    if (s != HSA_STATUS_SUCCESS) {
      // the chunks already issued must land before the caller reuses dst
      j->n = i;
      wait_all(c, *j);
      j->n = 0;
      return -5;
    }
  }
  j->n = n;
  return 0;
}

int wait(Copier* c, const Job& j, int i) {
  if (i < 0 || i >= j.n) return 0;
  hsa_signal_value_t v;
  while ((v = hsa_signal_wait_scacquire(c->sig[j.base + i], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                        HSA_WAIT_STATE_BLOCKED)) > 0) {
  }
  return v < 0 ? -6 : 0;
}

bool landed(Copier* c, const Job& j, int i) {
  if (i < 0 || i >= j.n) return true;
  return hsa_signal_load_scacquire(c->sig[j.base + i]) < 1;
}

int wait_all(Copier* c, const Job& j) {
  int rc = 0;
  for (int i = 0; i < j.n; ++i) {
    const int r = wait(c, j, i);
    if (r && !rc) rc = r;
  }
  return rc;
}

}  // namespace lsmck_dma
