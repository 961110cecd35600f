// Shared state of the analyzer-side ingest (analyzer.cpp, fswalk.cpp): the
// analyzer's Required context and the batch collector's pinned arena.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "tsg_analyzer.h"

namespace tsg {
void SetError(const std::string& e);
}

namespace tsg {
struct TarWalkCache;  // analyzer.cpp: evaluated tar entries indexed ahead of the cursor
void FreeTarWalkCache(TarWalkCache* w);
void EndTarWalk(TarWalkCache* w);  // joins the background index of the next window
}

struct tsg_analyzer {
  const tsg_scanner* s = nullptr;
  std::string config_base;  // filepath.Base(configPath)
  // One tar walk at a time over this analyzer's collectors: the entries
  // indexed past one batch's end are the next batch's (the collectors of a
  // two-collector pipeline alternate on one layer).
  std::mutex walk_mu;
  tsg::TarWalkCache* walk = nullptr;
  // tsg_analyzer_set_walk_ahead: index the next window of a tar walk on a
  // background thread (off by default: the layer buffer must then outlive the
  // call that returned 1, the rule in tsg_analyzer.h).
  bool walk_ahead = false;
  ~tsg_analyzer() { tsg::FreeTarWalkCache(walk); }
};

struct tsg_collector {
  tsg_analyzer* a = nullptr;
  int device = -1;  // pinned arena on this device's host side; -1 plain memory
  uint8_t* arena = nullptr;
  uint64_t cap = 0, used = 0, input_bytes = 0;
  uint64_t limit = 0;  // the batch size asked for
  // GPU pre-transform mode (tsg_collector_set_gpu_transform): the arena holds
  // the bytes as read, kinds[] the transform per file (xform.h), and the batch
  // limit counts each file's largest transformed size (bound).
  bool gpu_xform = false;
  uint64_t bound = 0;
  std::vector<uint8_t> kinds;
  // gather mode (tsg_collector_set_gather): the files stay in the layer buffer
  // gbase at gsrc[f]; the arena holds nothing (offs still lay the batch out)
  bool gather = false;
  const uint8_t* gbase = nullptr;
  std::vector<uint64_t> gsrc;
  mutable std::vector<uint8_t> scratch;  // tsg_collector_file's transformed copy (GPU mode)
  int threads = 16;    // ingest threads (TSG_HOST_THREADS)
  std::vector<uint8_t> fs_scratch;  // FS walk: a window's small files, read whole by the first pass
  std::vector<uint64_t> offs{0};
  std::string path_pool;
  std::vector<uint64_t> path_off{0};
  std::vector<uint8_t> binary;
  // built at submit / file(): char* table over path_pool
  std::vector<const char*> path_ptrs;
  std::vector<uint64_t> path_lens;

  ~tsg_collector() { Release(); }
  void Release() {
    if (!arena) return;
    if (device >= 0)
      (void)hipHostFree(arena);
    else
      std::free(arena);
    arena = nullptr;
    cap = 0;
  }
  bool Reserve(uint64_t need) {  // need: arena bytes incl. the 64-B pad
    if (need <= cap) return true;
    Release();
    const uint64_t n = (need + 4095) & ~uint64_t(4095);
    void* p = nullptr;
    if (device >= 0) {
      if (hipSetDevice(device) != hipSuccess || hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) p = nullptr;
    } else if (posix_memalign(&p, 4096, n) != 0) {
      p = nullptr;
    }
    if (!p) {
      tsg::SetError("collector: cannot allocate a " + std::to_string(n) + "-byte arena");
      return false;
    }
    arena = static_cast<uint8_t*>(p);
    cap = n;
    return true;
  }
  uint32_t files() const { return uint32_t(offs.size() - 1); }
  void BuildPaths() {
    const uint32_t n = files();
    path_ptrs.resize(n);
    path_lens.resize(n);
    for (uint32_t i = 0; i < n; i++) {
      path_ptrs[i] = path_pool.data() + path_off[i];
      path_lens[i] = path_off[i + 1] - path_off[i];
    }
  }
  uint64_t acct() const { return gpu_xform ? bound : used; }  // bytes counted against the limit
  void Reset() {
    used = input_bytes = bound = 0;
    kinds.clear();
    gbase = nullptr;
    gsrc.clear();
    offs.assign(1, 0);
    path_pool.clear();
    path_off.assign(1, 0);
    binary.clear();
  }
};

