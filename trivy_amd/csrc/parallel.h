// Host thread fan-out shared by the exact tail, the allow-path pass and the
// ingest walker.  One process-wide pool of worker threads serves every
// ParallelFor, so scans in flight together (tsg_scan_submit) share the host
// cores instead of each spawning its own threads (oversubscribing a 16-core
// share measured 1.4x slower).
#pragma once
#include <pthread.h>
#include <sched.h>
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
  bool wide = false;  // the pool's spare workers may help too
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

// Host CPUs this process may use for its pool: its affinity mask (after a
// NUMA binding, the node's CPUs), capped by the cgroup CPU quota, shared with
// the other processes of the job on this node -- LOCAL_WORLD_SIZE ranks
// (torchrun) spread over the node's CPUs, so ~LOCAL_WORLD_SIZE x mask/online
// of them share this mask, and the container's quota is split LOCAL_WORLD_SIZE
// ways -- or TSG_POOL_SHARE processes when set.  Minus the per-process
// reserve (the callers, the GPU-driving thread and the allow-path pass run
// beside the pool; going over a quota stalls every thread for the rest of the
// period: on a 16-CPU box 12 workers measured 12% above 15).
inline int PoolCpus() {
  int aff = 0, online = int(std::thread::hardware_concurrency());
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) aff = CPU_COUNT(&set);
  if (online <= 0) online = 16;
  if (aff <= 0 || aff > online) aff = online;
  double ranks = 1.0;  // processes of this job on this node
  if (const char* e = std::getenv("LOCAL_WORLD_SIZE")) ranks = std::max(1, std::atoi(e));
  double sharing = std::max(1.0, ranks * double(aff) / double(online));  // ranks on this mask
  if (const char* e = std::getenv("TSG_POOL_SHARE")) sharing = ranks = std::max(1.0, std::atof(e));
  double cpus = double(aff) / sharing;
  long q = 0, per = 0;
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    if (std::fscanf(f, "%ld %ld", &q, &per) != 2) q = per = 0;  // "max 100000": no quota
    std::fclose(f);
  }
  if (q > 0 && per > 0) cpus = std::min(cpus, double(q) / double(per) / ranks);
  return std::max(1, int(cpus));
}
inline int PoolReserve(int c) { return c >= 16 ? 4 : std::max(1, c / 4); }
inline int PoolBudget() {
  const int c = PoolCpus();
  return std::max(1, c - PoolReserve(c));
}

// Spare workers beside PoolBudget(): reserve - 1 (3 on the 16-CPU box), taken only
// by wide jobs -- the tar / FS walks (the host-bound C4 and c1fs paths, where the
// GPU-driving and allow-path threads the reserve is for are mostly idle: C4 38 -> 40
// GB/s at 15 workers, profiles/r05/r05l) and a scan's exact pass when no other scan
// is in flight (the drain at the end of a run).
inline int PoolSpare() { return std::max(0, PoolReserve(PoolCpus()) - 1); }

class HostPool {
 public:
  // TSG_POOL_THREADS workers; default PoolBudget() (12 on the 16-CPU-quota
  // one-GPU box; 12 per rank for 8 ranks sharing a 128-CPU quota; 15 with 16
  // cores and no quota) plus PoolSpare() that only wide jobs take.
  static HostPool& Get() {
    static HostPool* p = new HostPool();  // never destroyed: workers may be parked at exit
    return *p;
  }

  // wide: the job may take the spare workers too (the walks; a scan's exact pass
  // when no other scan is in flight: the end of a run, where nothing else needs the cores)
  void Run(size_t n, int threads, const std::function<void(size_t)>& fn, bool wide = false) {
    auto job = std::make_shared<PoolJob>();
    job->fn = &fn;
    job->n = n;
    job->max_helpers = int(std::min<size_t>({size_t(threads - 1), n - 1, size_t(wide ? n_workers_ : n_steady_)}));
    job->wide = wide;
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
    int n = e ? std::atoi(e) : PoolBudget();
    if (n < 0) n = 0;
    // spare workers only wide jobs use (TSG_POOL_SPARE; default PoolSpare(), none
    // when TSG_POOL_THREADS fixes the pool)
    const char* sp = std::getenv("TSG_POOL_SPARE");
    const int spare = sp ? std::max(0, std::atoi(sp)) : e ? 0 : PoolSpare();
    n_steady_ = n;
    n_workers_ = n + spare;
    n = n_workers_;
    for (int k = 0; k < n; k++) {
      const bool spare_worker = k >= n_steady_;
      workers_.emplace_back([this, spare_worker] {
        pthread_setname_np(pthread_self(), spare_worker ? "tsg-pool-spare" : "tsg-pool");
        Loop(spare_worker);
      });
      workers_.back().detach();
    }
  }

  // A spare worker takes wide jobs only, so ordinary jobs -- however many run at
  // once (pipelined scans' exact passes, allow-path passes) -- never have more
  // than n_steady_ pool threads between them besides their callers.
  void Loop(bool spare_worker) {
    for (;;) {
      std::shared_ptr<PoolJob> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
          while (!q_.empty() && q_.front()->next.load() >= q_.front()->n) q_.pop_front();  // all handed out
          auto it = q_.begin();
          while (it != q_.end()) {
            if ((*it)->next.load() >= (*it)->n) {
              it = q_.erase(it);
            } else if (spare_worker && !(*it)->wide) {
              ++it;
            } else {
              break;
            }
          }
          if (it != q_.end()) {
            job = *it;
            if (++job->helpers >= job->max_helpers) q_.erase(it);
            break;
          }
          cv_.wait(lk);
        }
      }
      job->Work();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<PoolJob>> q_;
  std::vector<std::thread> workers_;
  int n_steady_ = 0, n_workers_ = 0;  // helpers a job may take: ordinary / wide

 public:
  int steady() const { return n_steady_; }
  int workers() const { return n_workers_; }
};

// fn(i) for i in [0, n) on up to `threads` threads (the caller's included),
// indices handed out one at a time; the helpers come from the shared pool.
template <typename F>
void ParallelFor(size_t n, int threads, F fn, bool wide = false) {
  if (n == 0) return;
  if (threads <= 1 || n < 2) {
    for (size_t i = 0; i < n; i++) fn(i);
    return;
  }
  const std::function<void(size_t)> f = [&fn](size_t i) { fn(i); };
  HostPool::Get().Run(n, threads, f, wide);
}

}  // namespace tsg
