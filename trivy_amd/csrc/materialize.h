// GPU finding materialisation: toFinding / findLocation
// (pkg/fanal/secret/scanner.go:475-558) and the censored code lines
// (scanner.go:431-446, 465-473) of every finding of a batch whose arena is
// resident in HBM, run after the host's exact Go-regexp pass has found the
// locations.
//
// The host hands over, per file with findings, the surviving locations (rule,
// [s, e)) in the order the reference appends them, the file's censor spans
// (the locations merged, each with the '\n' count of the spans before it) and
// for each location an anchor (a candidate window start at or below s and the
// raw '\n' count before it, Candidate::nl_before).  One wave per location then
// computes, from the arena in HBM:
//   - StartLine / EndLine: the '\n' the censored content keeps before s (raw
//     count from the anchor minus the censored ones); EndLine == StartLine,
//     since every location is itself censored (its own '\n' are '*');
//   - the match line [ls, le) and the >100-B cut (start-30 / end+20);
//   - the code window: up to two lines above and one below (the last three
//     visible '\n' before s, the first two at or after it);
//   - each line's 100-B cut and whether the cause line shares the match text;
// and, after a prefix sum over the per-location line and text counts, writes
// the FindingOut / LineOut records and the censored text (censored bytes as
// '*') in the layout FileFindings holds, file-relative.  The host copies each
// file's three ranges into its result and sorts (scanner.go:452-457).
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>

namespace tsg {

// Findings of one file, flat (FileFindings, scanner.h): the GPU writes these
// records as the host lays them out (static_asserts below and in the .hip).
struct LineOut {
  int64_t number;
  uint32_t off, len;  // content in FileFindings::text
  bool is_cause, first_cause, last_cause;
};

struct FindingOut {
  uint32_t rule;
  int64_t start_line, end_line;
  uint32_t match_off, match_len;  // in FileFindings::text
  uint32_t line_lo, line_hi;      // into FileFindings::lines
};

static_assert(sizeof(LineOut) == 24 && offsetof(LineOut, off) == 8 && offsetof(LineOut, is_cause) == 16,
              "LineOut layout (written by the GPU)");
static_assert(sizeof(FindingOut) == 40 && offsetof(FindingOut, start_line) == 8 &&
                  offsetof(FindingOut, match_off) == 24 && offsetof(FindingOut, line_lo) == 32,
              "FindingOut layout (written by the GPU)");

struct MatFile {     // one file with findings
  uint32_t file;     // batch file index (offsets[file] .. offsets[file + 1])
  uint32_t m0, nm;   // its locations: MatMatch [m0, m0 + nm)
  uint32_t s0, ns;   // its censor spans: MatSpan [s0, s0 + ns), sorted, disjoint
  uint32_t pad;
};

struct MatMatch {    // one surviving location, in the reference's append order per file
  uint32_t rule;
  uint32_t fidx;     // its MatFile
  int64_t s, e;      // file-relative byte offsets (scanner.go Location)
  int64_t a_wlo;     // anchor: a position <= s ...
  int64_t a_nl;      // ... and the raw '\n' count in [0, a_wlo)
};

struct MatSpan {     // a merged censor span [s, e)
  int64_t s, e;
  int64_t nl_before; // '\n' inside the file's spans before this one
};

static_assert(sizeof(MatFile) == 24 && sizeof(MatMatch) == 40 && sizeof(MatSpan) == 24, "upload records");

class FindingMaterializer {
 public:
  explicit FindingMaterializer(int device);
  ~FindingMaterializer();
  bool ok() const { return err_.empty(); }
  const std::string& error() const { return err_; }

  // One call: Begin takes a free slot (blocking while all are busy) and sizes
  // its pinned upload buffers; the caller fills files() / matches() / spans();
  // Run uploads, runs the kernels over the resident arena and reads the
  // records back (blocking, the thread sleeps); the outputs stay valid until
  // End.  text_bound: an upper bound of the text bytes (sum over locations of
  // max(100, e - s + 50) + 400).
  struct Job;
  Job* Begin(uint32_t n_files, uint32_t n_match, uint32_t n_span, uint64_t text_bound, std::string* err);
  MatFile* files(Job* j);
  MatMatch* matches(Job* j);
  MatSpan* spans(Job* j);
  bool Run(Job* j, const uint8_t* d_arena, const uint64_t* d_offsets, std::string* err);
  // outputs: per location its FindingOut; LineOut / text of the whole call;
  // pref[m] = (text offset << 32) | line index of location m (exclusive, global:
  // file f's records are [pref[m0]...pref[m0 + nm]) ).
  const FindingOut* findings(Job* j) const;
  const LineOut* lines(Job* j) const;
  const char* text(Job* j) const;
  const uint64_t* pref(Job* j) const;
  void End(Job* j);

 private:
  static constexpr int kSlots = 6;  // (a depth-6 pipeline's exact passes at once)
  struct Slot;
  Slot* slots_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_;
  int device_ = 0;
  std::string err_;
};

}  // namespace tsg
