// Host thread fan-out shared by the exact tail and the ingest walker.
#pragma once
#include <algorithm>
#include <atomic>
#include <cstddef>
#include <thread>
#include <vector>

namespace tsg {

// fn(i) for i in [0, n) on up to `threads` threads (the caller's included),
// indices handed out one at a time.
template <typename F>
void ParallelFor(size_t n, int threads, F fn) {
  if (n == 0) return;
  if (threads <= 1 || n < 2) {
    for (size_t i = 0; i < n; i++) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (;;) {
      size_t i = next.fetch_add(1);
      if (i >= n) break;
      fn(i);
    }
  };
  int t = int(std::min<size_t>(size_t(threads), n));
  std::vector<std::thread> pool;
  for (int k = 1; k < t; k++) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}

}  // namespace tsg
