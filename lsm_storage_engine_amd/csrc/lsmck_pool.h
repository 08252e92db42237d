// lsmck_pool.h -- a small persistent host thread pool (header-only, no HIP).
#pragma once
#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace lsmck_host {

// Host worker threads kept for the context's lifetime: the staging copies
// split a chunk over stage_threads threads, and spawning them per chunk cost
// ~20-40 us each (a 64 MiB chunk copies in ~1.3 ms).  run(T, f) runs f(0) on
// the caller and f(1..T-1) on the workers and returns when all are done.
class HostPool {
 public:
  HostPool() {
    // the process's mask (its main thread's, pid = tid), not the mask of
    // whichever thread builds the pool first: that one may be narrowed already
    CPU_ZERO(&orig_);
    if (sched_getaffinity(getpid(), sizeof orig_, &orig_) != 0 || CPU_COUNT(&orig_) == 0)
      for (int c = 0; c < CPU_SETSIZE; ++c) CPU_SET(c, &orig_);
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // the workers' CPUs (the device's NUMA node), for the ones running and the
  // ones to come; clear_cpus: any CPU again
  // (within the CPUs the process started with -- taskset, numactl -- when
  // the node has any of them)
  void set_cpus(const cpu_set_t& set) {
    std::lock_guard<std::mutex> one(run_mu_);
    CPU_AND(&cpus_, &set, &orig_);
    if (CPU_COUNT(&cpus_) == 0) cpus_ = set;
    pinned_ = true;
    for (auto& t : th_) (void)pthread_setaffinity_np(t.native_handle(), sizeof cpus_, &cpus_);
  }
  void clear_cpus() {
    std::lock_guard<std::mutex> one(run_mu_);
    if (!pinned_) return;
    pinned_ = false;
    cpus_ = orig_;  // the process's own mask again
    for (auto& t : th_) (void)pthread_setaffinity_np(t.native_handle(), sizeof cpus_, &cpus_);
  }
  void run(unsigned T, const std::function<void(unsigned)>& f) {
    if (T <= 1) {
      f(0);
      return;
    }
    std::lock_guard<std::mutex> one(run_mu_);  // one round at a time (callers on several threads)
    grow(T - 1);
    {
      std::lock_guard<std::mutex> lk(m_);
      f_ = &f;
      want_ = T;
      pending_ = T - 1;
      ++gen_;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return pending_ == 0; });
    f_ = nullptr;
  }

 private:
  void grow(unsigned n) {  // (before run() opens its round: the new workers take part in it)
    uint64_t g;
    {
      std::lock_guard<std::mutex> lk(m_);
      g = gen_;
    }
    while (th_.size() < n) {
      const unsigned idx = (unsigned)th_.size() + 1;
      th_.emplace_back([this, idx, g] { loop(idx, g); });
      if (pinned_) (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof cpus_, &cpus_);
    }
  }
  void loop(unsigned idx, uint64_t seen) {
    for (;;) {
      const std::function<void(unsigned)>* f;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        if (idx >= want_) continue;
        f = f_;
      }
      (*f)(idx);
      std::lock_guard<std::mutex> lk(m_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_, run_mu_;
  std::condition_variable cv_, done_;
  const std::function<void(unsigned)>* f_ = nullptr;
  unsigned want_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
  cpu_set_t cpus_{};     // (under run_mu_)
  cpu_set_t orig_{};     // the process's affinity when the pool was made
  bool pinned_ = false;
};

}  // namespace lsmck_host
