// HostPool (lsmck_pool.h) stress test: every worker index runs once per round,
// rounds from several caller threads serialise.  Built with -fsanitize=thread
// by tests/test_host_pool.py.
#include "lsmck_pool.h"
#include <atomic>
#include <cassert>
#include <cstdio>
int main() {
  for (int rep = 0; rep < 3; ++rep) {
    lsmck_host::HostPool p;
    std::atomic<long> sum{0};
    for (int round = 0; round < 2000; ++round) {
      unsigned T = 1 + (round * 7) % 12;
      std::vector<int> hit(T, 0);
      p.run(T, [&](unsigned t) { hit[t]++; sum += t; });
      for (unsigned t = 0; t < T; ++t) assert(hit[t] == 1);
    }
    // concurrent callers
    std::vector<std::thread> cs;
    for (int c = 0; c < 4; ++c) cs.emplace_back([&] { for (int r = 0; r < 300; ++r) { std::atomic<int> n{0}; p.run(6, [&](unsigned) { n++; }); assert(n == 6); } });
    for (auto& t : cs) t.join();
  }
  puts("pool ok");
}
