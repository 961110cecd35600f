// Global allow-path prefilter on the GPU (scanner.go:57-59, 381-386).
//
// Scan returns Secret{FilePath} for every file whose path an allow rule
// matches, so the allow-path rules run over every path of a batch -- on the
// host that was ~31 ns per path, a sixth of the host CPU of a C2 scan.  Here
// one lane per path runs a shift-and over the allow rules' required literals
// (Matcher::lits: an ASCII path holding none of a rule's lowercased literals
// cannot match it) and reports the paths that hold one, with the rules whose
// literal they hold, plus every non-ASCII path.  The host runs the exact rule
// only on those (about 10 % of C2's paths); every other path is not allowed.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <vector>

namespace tsg {

struct PathHit {        // one reported path
  uint32_t file;        // | kPathNonAscii: the host runs every rule on it
  uint32_t pad;
  uint64_t rules;       // allow rules (bit i = rule i) with a literal in the lowered path
};
constexpr uint32_t kPathNonAscii = 0x80000000u;

// Literals packed into up to four 64-bit shift-and words (a literal never
// crosses a word); the byte table is indexed by the ASCII-lowered byte.
struct PathTable {
  uint64_t B[256][4];   // positions that accept the byte
  uint64_t S[4], E[4];  // first / last position of each literal
  uint8_t rule_of[256]; // word * 64 + bit of a literal's last position -> its rule
  uint32_t words;
};

// Builds the table; false when the literals do not fit (more than 64 rules,
// a literal shorter than 2 or longer than 64 bytes, over 256 positions).
bool BuildPathTable(const std::vector<std::pair<std::string, uint32_t>>& lits, PathTable* t);

class PathFilter {
 public:
  PathFilter(int device, const PathTable& t);
  ~PathFilter();
  bool ok() const { return err_.empty(); }
  const std::string& error() const { return err_; }
  // Paths [off[i], off[i+1]) of d_paths (device), i < n: the reported ones
  // (any order).  Thread-safe: up to kSlots calls run at once, each on a
  // high-priority stream and buffers of its own (a few microseconds of GPU time
  // that should not queue behind a scan's kernels, nor behind another scan's
  // filter: one shared stream and lock serialised the first scans of a
  // pipeline, each waiting out a filter kernel queued behind a K1).
  bool Run(const uint8_t* d_paths, const uint64_t* d_off, uint32_t n, std::vector<PathHit>* out, std::string* err) {
    return RunImpl(d_paths, d_off, nullptr, nullptr, n, out, err);
  }
  // The same over paths packed in host memory (the analyzer's collectors:
  // h_off[i] .. h_off[i+1] into h_paths): staged through the slot's pinned
  // buffer and copied to HBM on the slot's stream first.
  bool RunHost(const uint8_t* h_paths, const uint64_t* h_off, uint32_t n, std::vector<PathHit>* out,
               std::string* err) {
    return RunImpl(nullptr, nullptr, h_paths, h_off, n, out, err);
  }

 private:
  bool RunImpl(const uint8_t* d_paths, const uint64_t* d_off, const uint8_t* h_paths, const uint64_t* h_off,
               uint32_t n, std::vector<PathHit>* out, std::string* err);
  struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint32_t* d_cnt = nullptr;  // two counters used in turn: each launch zeroes the next one's
    uint32_t parity = 0;
    uint32_t* h_cnt = nullptr;
    PathHit* d_out = nullptr;
    PathHit* h_out = nullptr;  // pinned: a pageable read-back stalled the engine's stream (5 ms per C2 scan)
    size_t cap = 0;
    // RunHost: the packed paths and their offsets in HBM, and their pinned staging
    uint8_t* d_paths = nullptr;
    size_t paths_cap = 0;
    uint8_t* h_stage = nullptr;
    size_t stage_cap = 0;
    bool busy = false;
  };
  static constexpr int kSlots = 4;
  std::mutex mu_;
  std::condition_variable cv_;
  Slot slots_[kSlots];
  std::atomic<uint32_t> last_k_{0};  // records of the last call: one read-back when the count repeats
  int device_ = 0;
  std::string err_;
  PathTable* d_table_ = nullptr;
};

}  // namespace tsg
