// Host thread fan-out shared by the exact tail, the allow-path pass and the
// ingest walker.  One process-wide pool of worker threads serves every
// ParallelFor, so scans in flight together (tsg_scan_submit) share the host
// cores instead of each spawning its own threads (oversubscribing a 16-core
// share measured 1.4x slower).
#pragma once
#include <pthread.h>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdlib>
#include <deque>
#include <cstdio>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace tsg {

struct PoolJob {
  const std::function<void(size_t)>* fn = nullptr;
  size_t n = 0;
  int max_helpers = 0;
  std::atomic<size_t> next{0};
  std::atomic<size_t> done{0};
  int helpers = 0;  // guarded by the pool mutex
  std::mutex mu;
  std::condition_variable cv;

  void Work() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= n) return;
      (*fn)(i);
      if (done.fetch_add(1) + 1 == n) {
        std::lock_guard<std::mutex> g(mu);
        cv.notify_all();
      }
    }
  }
};

class HostPool {
 public:
  // TSG_POOL_THREADS workers.  Default: under a cgroup CPU quota of Q CPUs,
  // Q - 4 (the callers, the GPU-driving thread and the allow-path pass run
  // beside the pool; going over the quota stalls every thread for the rest
  // of the period: on a 16-CPU box 12 workers measured 12% above 15);
  // without a quota 15 (16 cores with the calling thread).
  static HostPool& Get() {
    static HostPool* p = new HostPool();  // never destroyed: workers may be parked at exit
    return *p;
  }

  void Run(size_t n, int threads, const std::function<void(size_t)>& fn) {
    auto job = std::make_shared<PoolJob>();
    job->fn = &fn;
    job->n = n;
    job->max_helpers = int(std::min<size_t>(size_t(threads - 1), n - 1));
    if (job->max_helpers > 0 && !workers_.empty()) {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(job);
    }
    cv_.notify_all();
    job->Work();
    std::unique_lock<std::mutex> lk(job->mu);
    job->cv.wait(lk, [&] { return job->done.load() == job->n; });
  }

 private:
  HostPool() {
    const char* e = std::getenv("TSG_POOL_THREADS");
    int n = e ? std::atoi(e) : DefaultWorkers();
    if (n < 0) n = 0;
    for (int k = 0; k < n; k++) {
      workers_.emplace_back([this] {
        pthread_setname_np(pthread_self(), "tsg-pool");
        Loop();
      });
      workers_.back().detach();
    }
  }

  static int DefaultWorkers() {
    long q = 0, per = 0;
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      if (std::fscanf(f, "%ld %ld", &q, &per) != 2) q = per = 0;  // "max 100000": no quota
      std::fclose(f);
    }
    if (q > 0 && per > 0) return std::max(1, int(q / per) - 4);
    return 15;
  }

  void Loop() {
    for (;;) {
      std::shared_ptr<PoolJob> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
          while (!q_.empty() && q_.front()->next.load() >= q_.front()->n) q_.pop_front();  // all handed out
          if (!q_.empty()) break;
          cv_.wait(lk);
        }
        job = q_.front();
        if (++job->helpers >= job->max_helpers) q_.pop_front();
      }
      job->Work();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<PoolJob>> q_;
  std::vector<std::thread> workers_;
};

// fn(i) for i in [0, n) on up to `threads` threads (the caller's included),
// indices handed out one at a time; the helpers come from the shared pool.
template <typename F>
void ParallelFor(size_t n, int threads, F fn) {
  if (n == 0) return;
  if (threads <= 1 || n < 2) {
    for (size_t i = 0; i < n; i++) fn(i);
    return;
  }
  const std::function<void(size_t)> f = [&fn](size_t i) { fn(i); };
  HostPool::Get().Run(n, threads, f);
}

}  // namespace tsg
