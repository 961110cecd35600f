// Host side of the drop-in Scanner (pkg/fanal/secret/scanner.go:377-558).
//
// The GPU engine returns candidate (file, rule, start-window) records; this
// module runs the exact tail that the reference runs per rule per file:
// path gates (:381, :397, :403), the exact keyword gate where the GPU bitset
// is not exact (:409), leftmost-first FindAll[Submatch]Index restricted to
// the candidate windows (:102-148), allow rules (:150-153, :214-221), exclude
// blocks (:237-275, :419-425), censoring (:431-436, :465-473), findings
// (:438-446, :475-558) and the final sort (:452-457).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <new>
#include <type_traits>
#include <vector>

#include "engine.h"
#include "materialize.h"
#include "pathfilter.h"
#include "goregex.h"
#include "rules.h"

namespace tsg {

// Regexp used as MatchString, with a required-literal prefilter.
struct Matcher {
  std::unique_ptr<Regex> re;
  std::vector<std::string> lits;  // lowercased; empty = no prefilter
  // A source that is a literal, or a few (one group of literal alternatives),
  // with optional ^ / $ (`\/vendor\/`, `\.md$`, `^usr\/(?:share|include|lib)\/`):
  // matched by byte compares, with the regex's exact result (see SimpleLiteral).
  bool simple = false, simple_begin = false, simple_end = false;
  std::vector<std::string> simple_lits;
  bool Match(const uint8_t* s, size_t n) const;
  bool MatchSimple(const uint8_t* s, size_t n) const;
};

// `src` is [^]prefix[(?:alt|alt...)]suffix[$] with plain bytes and
// backslash-escaped punctuation only (no flags, classes, repeats, other groups
// or alternation): *lits gets prefix + alt + suffix per alternative, and a
// MatchString of the regex is true iff one of them occurs (anchored as given).
bool SimpleLiteral(const std::string& src, std::vector<std::string>* lits, bool* begin, bool* end);

struct AllowRuleSpec {
  std::string id;
  std::unique_ptr<Matcher> regex, path;
};

struct RuleSpec {
  std::string id, category, title, severity, secret_group_name;
  std::string regex_src;
  bool has_regex = false;  // Rule.Regex != nil (an empty source is a regex)
  std::vector<std::string> keywords;
  std::unique_ptr<Matcher> path;
  std::vector<AllowRuleSpec> allow_rules;
  std::vector<std::unique_ptr<Regex>> exclude;
  std::vector<int> group_idx;  // capture indices named secret_group_name
  std::vector<std::string> kw_lower_host;  // for host-verified gates
  std::vector<uint8_t> kw_ascii;           // per kw_lower_host entry: all bytes ASCII
  std::vector<uint16_t> kw_rare;           // per entry: index of its least frequent letter (memchr key)
};

// Findings of one file, flat: records (LineOut, FindingOut: materialize.h)
// plus one text pool for every match and code line (three allocations per
// file, whatever the finding count).

// Bump allocator for one batch's findings: each host thread of the exact
// pass fills its own, and the batch result frees them whole -- per file the
// findings, lines and text were three heap allocations made on the pool
// threads and freed on the reaper thread (malloc arena lock traffic).
class ResultArena {
 public:
  void* Alloc(size_t n, size_t align) {
    size_t pad = (align - (reinterpret_cast<uintptr_t>(cur_) & (align - 1))) & (align - 1);
    if (n + pad > left_) {
      const size_t sz = std::max<size_t>(kBlock, n + align);
      blocks_.emplace_back(new uint8_t[sz]);
      cur_ = blocks_.back().get();
      left_ = sz;
      pad = (align - (reinterpret_cast<uintptr_t>(cur_) & (align - 1))) & (align - 1);
    }
    void* p = cur_ + pad;
    cur_ += pad + n;
    left_ -= pad + n;
    return p;
  }

 private:
  static constexpr size_t kBlock = size_t(1) << 20;
  std::vector<std::unique_ptr<uint8_t[]>> blocks_;
  uint8_t* cur_ = nullptr;
  size_t left_ = 0;
};

// Allocator over a ResultArena (deallocate is a no-op); without an arena it
// is std::allocator.
template <class T>
struct ArenaAlloc {
  using value_type = T;
  using propagate_on_container_move_assignment = std::true_type;
  using propagate_on_container_copy_assignment = std::true_type;
  using propagate_on_container_swap = std::true_type;
  ResultArena* a = nullptr;
  ArenaAlloc() = default;
  explicit ArenaAlloc(ResultArena* x) : a(x) {}
  template <class U>
  ArenaAlloc(const ArenaAlloc<U>& o) : a(o.a) {}
  T* allocate(size_t n) {
    return a ? static_cast<T*>(a->Alloc(n * sizeof(T), alignof(T))) : std::allocator<T>().allocate(n);
  }
  void deallocate(T* p, size_t n) {
    if (!a) std::allocator<T>().deallocate(p, n);
  }
  template <class U>
  bool operator==(const ArenaAlloc<U>& o) const { return a == o.a; }
  template <class U>
  bool operator!=(const ArenaAlloc<U>& o) const { return a != o.a; }
};

// a FileFindings' elements live in a ResultArena freed whole; the scratch reuse
// in HostTail move-assigns over old ones without running element destructors
static_assert(std::is_trivially_destructible<FindingOut>::value && std::is_trivially_destructible<LineOut>::value,
              "arena-held findings records must be trivially destructible");

struct FileFindings {
  explicit FileFindings(ResultArena* a = nullptr)
      : f(ArenaAlloc<FindingOut>(a)), lines(ArenaAlloc<LineOut>(a)), text(ArenaAlloc<char>(a)) {}
  std::vector<FindingOut, ArenaAlloc<FindingOut>> f;
  std::vector<LineOut, ArenaAlloc<LineOut>> lines;
  std::basic_string<char, std::char_traits<char>, ArenaAlloc<char>> text;
  bool binary = false;  // ScanArgs.Binary: findings carry Code{} (Lines nil, scanner.go:441-444)
  size_t size() const { return f.size(); }
  std::string_view Str(uint32_t off, uint32_t len) const { return std::string_view(text).substr(off, len); }
  std::string_view Match(const FindingOut& x) const { return Str(x.match_off, x.match_len); }
  uint32_t Put(std::string_view s) {
    const uint32_t at = uint32_t(text.size());
    text.append(s.data(), s.size());
    return at;
  }
};

enum FileKind : uint32_t { kNoFindings = 0, kAllowedPath = 1, kHasFindings = 2 };

struct FileResult {
  FileKind kind = kNoFindings;
  FileFindings findings;
  // GPU materialisation (materialize.h): the file's locations and censor spans
  // (with the sentinel), set by the exact pass, turned into findings after the
  // batch-wide GPU pass
  bool gpu = false;
  std::vector<MatMatch> gm;
  std::vector<MatSpan> gs;
  uint64_t text_bound = 0;
};

// Files' findings in one allocation, constructed in place by the exact pass's
// workers (moving ~50 k FileFindings into a fresh std::vector one by one -- its
// pages faulted in on the way -- was ~1-1.5 ms of serial time per C2 scan).
class FoundArray {
 public:
  FoundArray() = default;
  FoundArray(const FoundArray&) = delete;
  FoundArray& operator=(const FoundArray&) = delete;
  FoundArray(FoundArray&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr, o.n_ = 0; }
  FoundArray& operator=(FoundArray&& o) noexcept {
    if (this != &o) {
      clear();
      p_ = o.p_, n_ = o.n_;
      o.p_ = nullptr, o.n_ = 0;
    }
    return *this;
  }
  ~FoundArray() { clear(); }
  // storage for n, unconstructed: every slot must then be built with emplace(i, ...)
  void allocate(size_t n) {
    clear();
    if (n) p_ = static_cast<FileFindings*>(::operator new(n * sizeof(FileFindings), std::align_val_t(alignof(FileFindings))));
    n_ = n;
  }
  void emplace(size_t i, FileFindings&& v) { new (p_ + i) FileFindings(std::move(v)); }
  void clear() {
    for (size_t i = 0; i < n_; i++) p_[i].~FileFindings();
    if (p_) ::operator delete(p_, std::align_val_t(alignof(FileFindings)));
    p_ = nullptr;
    n_ = 0;
  }
  size_t size() const { return n_; }
  const FileFindings& operator[](size_t i) const { return p_[i]; }
  const FileFindings* begin() const { return p_; }
  const FileFindings* end() const { return p_ + n_; }

 private:
  FileFindings* p_ = nullptr;
  size_t n_ = 0;
};

// Per-batch result, sparse: a kind byte per file, findings only where present.
struct BatchResult {
  std::vector<std::unique_ptr<ResultArena>> arenas;  // the findings' storage (declared first: freed last)
  std::vector<uint8_t> kind;              // FileKind per file
  std::vector<uint32_t> found_files;      // ascending
  FoundArray found;                       // found[i]: the findings of found_files[i]
  const FileFindings* Findings(uint32_t f) const {
    auto it = std::lower_bound(found_files.begin(), found_files.end(), f);
    if (it == found_files.end() || *it != f) return nullptr;
    return &found[size_t(it - found_files.begin())];
  }
  uint64_t n_findings() const {
    uint64_t n = 0;
    for (auto& v : found) n += v.size();
    return n;
  }
};

struct BatchInput {
  uint32_t n_files = 0;
  const uint8_t* host_arena = nullptr;  // required: the exact pass reads it
  const uint64_t* host_offsets = nullptr;
  const uint8_t* dev_arena = nullptr;   // optional: resident in HBM already
  const uint64_t* dev_offsets = nullptr;
  const char* const* paths = nullptr;
  const uint64_t* path_lens = nullptr;  // optional (else strlen)
  const uint8_t* binary = nullptr;      // optional per-file Binary flag
  const uint8_t* transform = nullptr;   // optional per-file pre-transform (xform.h) run on the GPU: then
                                        // host_arena holds the bytes as read (host-resident batches only)
  // optional, per file: where the exact pass reads file f (file_data[f], file_len[f] bytes) instead of
  // host_arena + host_offsets[f] (a GPU pre-transformed batch: the gathered transformed files)
  const uint8_t* const* file_data = nullptr;
  const uint64_t* file_len = nullptr;
  const uint8_t* dev_paths = nullptr;   // optional: the paths packed in HBM (the allow-path prefilter runs
  const uint64_t* dev_path_off = nullptr;  // on the GPU, pathfilter.h); n_files + 1 offsets, device
  const uint8_t* host_paths = nullptr;      // optional: the paths packed in host memory (copied to HBM for
  const uint64_t* host_path_off = nullptr;  // the same prefilter when dev_paths is absent); n_files + 1 offsets
  // optional (with transform; host_arena NULL): file f's bytes as read are at gather_base + gather_src[f]
  // in page-locked, device-mapped memory; the engine gathers them on the GPU (GpuEngine::RunHost)
  const uint8_t* gather_base = nullptr;
  const uint64_t* gather_src = nullptr;
};

struct HostStats {
  double ms_gpu = 0, ms_allow = 0, ms_exact = 0, ms_total = 0;
  uint64_t candidates = 0, files_with_candidates = 0, findings = 0;
};

class SecretScanner {
 public:
  // device < 0: no GPU engine (test hooks only: tsg_debug_host_tail)
  SecretScanner(std::vector<RuleSpec> rules, std::vector<AllowRuleSpec> allow,
                std::vector<std::unique_ptr<Regex>> exclude, int device, std::string* err,
                const CompileOptions* opt = nullptr);
  bool ok() const {
    if (!compiled_ok_) return false;
    if (no_engine_) return true;
    if (engines_.empty()) return false;
    for (auto& e : engines_)
      if (!e->ok()) return false;
    return true;
  }
  const std::string& error() const { return err_; }

  // Thread-safe: concurrent scans report failures through *err only (no shared state).
  bool Scan(const BatchInput& in, BatchResult* out, BatchStats* gst, HostStats* hst, std::string* err);
  // The exact host tail over a given candidate list (what Scan runs after the GPU).
  // The exact host pass over the GPU's candidates.  `allowed` (per-file
  // global AllowPath results) is computed here when not supplied.
  // gpu_windows: the candidates came from the GPU engine, so the exclude-block
  // regexes (compiled as extra rules) have candidate windows too; otherwise
  // (host-only callers) each exclude regex sweeps the whole file.
  // False (with *err) only when the GPU findings pass fails.
  bool HostTail(const BatchInput& in, std::vector<Candidate>* cands, BatchResult* out, HostStats* hs,
                const std::vector<uint8_t>* allowed = nullptr, bool gpu_windows = false,
                std::string* err = nullptr) const;
  std::vector<uint8_t> AllowedPaths(const BatchInput& in) const;
  // Global.AllowPath (scanner.go:57-59)
  bool AllowPath(const uint8_t* p, size_t n) const;

  const std::vector<RuleSpec>& rules() const { return rules_; }
  const CompiledRules& compiled() const { return cr_; }
  GpuEngine* engine() { return engines_.empty() ? nullptr : engines_[0].get(); }
  size_t n_engines() const { return engines_.size(); }
  GpuEngine* engine_at(size_t i) { return engines_[i].get(); }
  int device() const { return engines_.empty() ? -1 : engines_[0]->device(); }  // -1: no GPU engine
  void set_host_threads(int n) { host_threads_ = n; }

 private:
  void ScanFile(const uint8_t* content, int64_t len, std::string_view path, bool binary,
                const Candidate* c, size_t nc, FileResult* out, bool gpu_windows) const;
  // ScanFile in two parts: the surviving locations of the rules (scanner.go:394-436)
  // into the calling thread's scratch (matched, censor), then toFinding /
  // findLocation / sort on the host (:438-457) from them
  void MatchFile(const uint8_t* content, int64_t len, std::string_view path, const Candidate* c, size_t nc,
                 bool gpu_windows) const;
  void FindingsHost(const uint8_t* content, int64_t len, std::string_view path, bool binary, const Candidate* c,
                    size_t nc, FileResult* out) const;
  // the GPU materialisation's uploads of one file (materialize.h), from the scratch of MatchFile
  void GpuFindingsInput(const uint8_t* content, const Candidate* c, size_t nc, FileResult* out) const;
  // HostTail's serial set-up buffers (the per-file counts, the grouped
  // candidates, the dispatch order), kept across calls: allocated per call,
  // their first touch (page faults on ~10 MB) was most of the set-up's time.
  struct TailScratch {
    std::vector<uint32_t> order;
    std::vector<uint64_t> key, key2;  // (file << 32 | candidate index), radix-sorted by file
    std::vector<size_t> starts;
    std::vector<double> w;
    std::vector<FileResult> tmp;      // per group
    std::vector<uint32_t> gk;         // GPU findings: the groups, their first location / span
    std::vector<uint64_t> gm0, gs0;
    std::vector<uint32_t> gord;       // GPU findings: the assembly order (heaviest files first)
  };
  // the findings of the groups HostTail marked `gpu`, made by mat_ (materialize.h)
  template <class GroupFile, class ArenaOf>
  bool GpuFindings(const BatchInput& in, TailScratch* scr, size_t nf, GroupFile group_file, ArenaOf& thread_arena,
                   bool wide, double* ms_gpu, std::string* err) const;
  std::unique_ptr<TailScratch> TakeScratch() const;
  void GiveScratch(std::unique_ptr<TailScratch> s) const;
  mutable std::mutex scratch_mu_;
  mutable std::vector<std::unique_ptr<TailScratch>> scratch_free_;
  std::vector<RuleSpec> rules_;
  std::vector<uint32_t> rule_rank_;  // RuleRanks(rules_): findings sort by RuleID as integer compares
  // Exclude-block regexes (scanner.go:237-275) are compiled after the rules as
  // extra GPU rules without keywords: their candidates bound where a block can
  // start, so the host's FindAll of each block regex runs on windows instead
  // of the whole file.  Rule index of global block regex g / rule r's k-th.
  std::vector<uint32_t> ex_global_rule_;
  std::vector<std::vector<uint32_t>> ex_rule_;
  std::vector<AllowRuleSpec> allow_;
  std::vector<std::unique_ptr<Regex>> exclude_;
  CompiledRules cr_;
  // GPU slots: each engine has its own HIP stream and per-batch device
  // buffers; consecutive batches take the slots round robin, so one batch's
  // latency-bound kernels (confirm / verify) overlap the next batch's
  // streaming filter.  One GPU phase at a time per slot.  TSG_GPU_SLOTS,
  // default 1 (2 measured slower at C2: the kernels of two batches interfere).
  std::vector<std::unique_ptr<GpuEngine>> engines_;
  std::unique_ptr<std::mutex[]> gpu_mu_;
  std::atomic<uint32_t> next_slot_{0};
  std::atomic<int> active_scans_{0};
  std::atomic<bool> host_bound_{false};  // the last scan's exact pass outlasted 1.5x its GPU phase  // Scan calls in progress: alone, the exact pass may take the pool's spare workers
  std::string err_;
  int host_threads_ = 0;
  bool compiled_ok_ = false;
  bool no_engine_ = false;
  // Global AllowPath prefilter (exact): per ASCII-lowered byte pair, the allow
  // rules that have a required literal starting with that pair; rules without
  // a literal prefilter (or with a 1-byte literal) are always evaluated.
  void BuildAllowPathFilter();
  void BuildPathFilter(int device);
  bool ap_fast_ = false;
  uint64_t ap_always_ = 0;
  std::vector<uint16_t> ap_pair_;  // 65536: 1 + index into ap_lits_, 0 = no literal starts with the pair
  uint64_t ap_first_[4] = {};      // lowercase bytes that begin some literal (checked before ap_pair_)
  std::vector<uint8_t> ap_c0_, ap_c1_;  // distinct first-two-byte pairs of the literals (SIMD prefilter)
  std::vector<std::vector<std::pair<std::string, uint32_t>>> ap_lits_;  // (literal, allow rule) per pair
  // the rules of `lit_rules` (their literal is in the ASCII path) plus the unfiltered ones, exactly
  bool AllowPathRules(const uint8_t* p, size_t n, uint64_t lit_rules) const;
  // GPU allow-path prefilter (pathfilter.h): built when every path rule has usable literals
  std::unique_ptr<PathFilter> path_filter_;
  std::unique_ptr<FindingMaterializer> mat_;  // GPU findings of HBM-resident batches
  std::atomic<int> gpu_findings_{0};

 public:
  // 1 / 0 / 2: GPU / host / auto (GPU while host-bound) findings for HBM-resident
  // batches (tests, A/B); returns the previous setting, -1 without a GPU engine
  int SetGpuFindings(int mode) { return mat_ ? gpu_findings_.exchange(std::max(0, std::min(2, mode))) : -1; }
};

// Go sort.Slice restatement (pdqsort_func) on findings, scanner.go:452-457.
// rule_rank: per rule, the rank of its ID in the sorted IDs (RuleRanks).
void SortFindings(FileFindings* f, const std::vector<uint32_t>& rule_rank);
// SortFindings' permutation, the independent pdqsort calls spread over the pool
// (not from inside a ParallelFor item)
void SortFindingsParallel(FileFindings* f, const std::vector<uint32_t>& rule_rank, int threads, bool wide);
std::vector<uint32_t> RuleRanks(const std::vector<RuleSpec>& rules);

}  // namespace tsg
