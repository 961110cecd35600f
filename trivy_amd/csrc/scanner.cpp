// Exact host tail of the drop-in Scanner (see scanner.h for the line map).
#include "scanner.h"

#include "parallel.h"

#include <pthread.h>
#include <algorithm>
#include <functional>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <condition_variable>
#include <mutex>

namespace tsg {

namespace {

double NowMs() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool AsciiContainsLower(const uint8_t* s, size_t n, const std::string& lit) {
  // case-insensitive (ASCII) substring test; lit is lowercase
  size_t m = lit.size();
  if (m == 0) return true;
  if (m > n) return false;
  const uint8_t c0 = uint8_t(lit[0]);
  const uint8_t c0u = (c0 >= 'a' && c0 <= 'z') ? uint8_t(c0 - 32) : c0;
  for (size_t i = 0; i + m <= n; i++) {
    uint8_t c = s[i];
    if (c != c0 && c != c0u) continue;
    size_t k = 1;
    for (; k < m; k++) {
      uint8_t x = s[i + k];
      if (x >= 'A' && x <= 'Z') x = uint8_t(x + 32);
      if (x != uint8_t(lit[k])) break;
    }
    if (k == m) return true;
  }
  return false;
}

struct Loc {
  int64_t s, e;
};

bool IsAsciiStr(const std::string& s) {
  for (unsigned char c : s)
    if (c >= 0x80) return false;
  return true;
}

// Index of kw's least frequent character (English letter order; non-letters
// rarest): the byte AsciiCaseContains scans for with memchr.
size_t RarestIndex(const std::string& kw) {
  static const char* kFreq = "etaoinshrdlcumwfgypbvkjxqz";
  size_t best = 0;
  int best_rank = -1;
  for (size_t i = 0; i < kw.size(); i++) {
    const char c = kw[i];
    const char* f = (c >= 'a' && c <= 'z') ? std::strchr(kFreq, c) : nullptr;
    const int rank = f ? int(f - kFreq) : 100;
    if (rank > best_rank) {
      best_rank = rank;
      best = i;
    }
  }
  return best;
}

// ---------------------------------------------------------------------------
// Go sort.Slice = pdqsort_func (sort/zsortfunc.go), restated.
// ---------------------------------------------------------------------------
struct SortData {
  FileFindings* v;
  const uint32_t* rank;  // per rule: the rank of its ID among the rules' IDs (equal IDs, equal rank)
  bool Less(int i, int j) const {
    const FindingOut& a = v->f[size_t(i)];
    const FindingOut& b = v->f[size_t(j)];
    if (rank[a.rule] != rank[b.rule]) return rank[a.rule] < rank[b.rule];  // RuleID < RuleID
    if (a.match_off == b.match_off && a.match_len == b.match_len) return false;  // one shared text: equal
    // bytes.Compare order: the first 8 bytes as a big-endian word settle most
    // pairs without a memcmp call
    const char* t = v->text.data();
    const uint32_t n = std::min(a.match_len, b.match_len);
    if (n >= 8) {
      uint64_t x, y;
      std::memcpy(&x, t + a.match_off, 8);
      std::memcpy(&y, t + b.match_off, 8);
      if (x != y) return __builtin_bswap64(x) < __builtin_bswap64(y);
    }
    const int c = std::memcmp(t + a.match_off, t + b.match_off, n);
    return c != 0 ? c < 0 : a.match_len < b.match_len;
  }
  void Swap(int i, int j) { std::swap(v->f[size_t(i)], v->f[size_t(j)]); }
};

void InsertionSort(SortData& d, int a, int b) {
  for (int i = a + 1; i < b; i++)
    for (int j = i; j > a && d.Less(j, j - 1); j--) d.Swap(j, j - 1);
}

void SiftDown(SortData& d, int lo, int hi, int first) {
  int root = lo;
  for (;;) {
    int child = 2 * root + 1;
    if (child >= hi) return;
    if (child + 1 < hi && d.Less(first + child, first + child + 1)) child++;
    if (!d.Less(first + root, first + child)) return;
    d.Swap(first + root, first + child);
    root = child;
  }
}

void HeapSort(SortData& d, int a, int b) {
  int first = a, lo = 0, hi = b - a;
  for (int i = (hi - 1) / 2; i >= 0; i--) SiftDown(d, i, hi, first);
  for (int i = hi - 1; i >= 0; i--) {
    d.Swap(first, first + i);
    SiftDown(d, lo, i, first);
  }
}

int BitsLen(unsigned x) {
  int n = 0;
  while (x) {
    n++;
    x >>= 1;
  }
  return n;
}

void BreakPatterns(SortData& d, int a, int b) {
  int length = b - a;
  if (length >= 8) {
    uint64_t r = uint64_t(length);
    unsigned modulus = 1u << BitsLen(unsigned(length));
    int idx = a + (length / 4) * 2 - 1;
    for (int i = 0; i < 3; i++) {
      r ^= r << 13;
      r ^= r >> 7;
      r ^= r << 17;
      int other = int(unsigned(r) & (modulus - 1));
      if (other >= length) other -= length;
      d.Swap(idx - 1 + i, a + other);
    }
  }
}

enum { kHintUnknown = 0, kHintIncreasing = 1, kHintDecreasing = 2 };

void Order2(SortData& d, int& a, int& b, int* swaps) {
  if (d.Less(b, a)) {
    (*swaps)++;
    std::swap(a, b);
  }
}

int Median(SortData& d, int a, int b, int c, int* swaps) {
  Order2(d, a, b, swaps);
  Order2(d, b, c, swaps);
  Order2(d, a, b, swaps);
  return b;
}

int ChoosePivot(SortData& d, int a, int b, int* hint) {
  int l = b - a, swaps = 0;
  int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
  if (l >= 8) {
    if (l >= 50) {
      i = Median(d, i - 1, i, i + 1, &swaps);
      j = Median(d, j - 1, j, j + 1, &swaps);
      k = Median(d, k - 1, k, k + 1, &swaps);
    }
    j = Median(d, i, j, k, &swaps);
  }
  *hint = swaps == 0 ? kHintIncreasing : swaps == 12 ? kHintDecreasing : kHintUnknown;
  return j;
}

void ReverseRange(SortData& d, int a, int b) {
  for (int i = a, j = b - 1; i < j; i++, j--) d.Swap(i, j);
}

bool PartialInsertionSort(SortData& d, int a, int b) {
  int i = a + 1;
  for (int step = 0; step < 5; step++) {
    while (i < b && !d.Less(i, i - 1)) i++;
    if (i == b) return true;
    if (b - a < 50) return false;
    d.Swap(i, i - 1);
    if (i - a >= 2)
      for (int j = i - 1; j >= 1; j--) {
        if (!d.Less(j, j - 1)) break;
        d.Swap(j, j - 1);
      }
    if (b - i >= 2)
      for (int j = i + 1; j < b; j++) {
        if (!d.Less(j, j - 1)) break;
        d.Swap(j, j - 1);
      }
  }
  return false;
}

int PartitionEqual(SortData& d, int a, int b, int pivot) {
  d.Swap(a, pivot);
  int i = a + 1, j = b - 1;
  for (;;) {
    while (i <= j && !d.Less(a, i)) i++;
    while (i <= j && d.Less(a, j)) j--;
    if (i > j) break;
    d.Swap(i, j);
    i++;
    j--;
  }
  return i;
}

int Partition(SortData& d, int a, int b, int pivot, bool* already) {
  d.Swap(a, pivot);
  int i = a + 1, j = b - 1;
  while (i <= j && d.Less(i, a)) i++;
  while (i <= j && !d.Less(j, a)) j--;
  if (i > j) {
    d.Swap(j, a);
    *already = true;
    return j;
  }
  d.Swap(i, j);
  i++;
  j--;
  for (;;) {
    while (i <= j && d.Less(i, a)) i++;
    while (i <= j && !d.Less(j, a)) j--;
    if (i > j) break;
    d.Swap(i, j);
    i++;
    j--;
  }
  d.Swap(j, a);
  *already = false;
  return j;
}

// A recursive call of pdqsort works on its own range and reads only the element
// before it (a pivot, or an element equal to one, that an enclosing call put in
// its final place), so the calls are independent: `spawn` (when set) takes the
// ones of at least `min_spawn` elements to run on other threads, and the moves
// each makes are the sequential sort's.
struct SortSpawn {
  virtual void Push(int a, int b, int limit) = 0;
  int min_spawn = 1 << 30;
};

void Pdqsort(SortData& d, int a, int b, int limit, SortSpawn* spawn = nullptr) {
  bool was_balanced = true, was_partitioned = true;
  for (;;) {
    int length = b - a;
    if (length <= 12) {
      InsertionSort(d, a, b);
      return;
    }
    if (limit == 0) {
      HeapSort(d, a, b);
      return;
    }
    if (!was_balanced) {
      BreakPatterns(d, a, b);
      limit--;
    }
    int hint;
    int pivot = ChoosePivot(d, a, b, &hint);
    if (hint == kHintDecreasing) {
      ReverseRange(d, a, b);
      pivot = (b - 1) - (pivot - a);
      hint = kHintIncreasing;
    }
    if (was_balanced && was_partitioned && hint == kHintIncreasing) {
      if (PartialInsertionSort(d, a, b)) return;
    }
    if (a > 0 && !d.Less(a - 1, pivot)) {
      a = PartitionEqual(d, a, b, pivot);
      continue;
    }
    bool already;
    int mid = Partition(d, a, b, pivot, &already);
    was_partitioned = already;
    int left = mid - a, right = b - mid, thr = length / 8;
    if (left < right) {
      was_balanced = left >= thr;
      if (spawn && left >= spawn->min_spawn) spawn->Push(a, mid, limit);
      else Pdqsort(d, a, mid, limit, spawn);
      a = mid + 1;
    } else {
      was_balanced = right >= thr;
      if (spawn && right >= spawn->min_spawn) spawn->Push(mid + 1, b, limit);
      else Pdqsort(d, mid + 1, b, limit, spawn);
      b = mid;
    }
  }
}

}  // namespace

std::vector<uint32_t> RuleRanks(const std::vector<RuleSpec>& rules) {
  std::vector<uint32_t> idx(rules.size()), rank(rules.size(), 0);
  for (size_t i = 0; i < idx.size(); i++) idx[i] = uint32_t(i);
  std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return rules[a].id < rules[b].id; });
  for (size_t k = 1; k < idx.size(); k++)
    rank[idx[k]] = rules[idx[k]].id == rules[idx[k - 1]].id ? rank[idx[k - 1]] : uint32_t(k);
  return rank;
}

// (A variant sorting packed keys -- RuleID rank and the match's first 12 bytes --
// measured slower on C3f: its findings' matches are censored line windows, runs
// of '*' equal well past 12 bytes, so the keys tie and the whole-match compare
// runs anyway, behind an indirection.)
void SortFindings(FileFindings* f, const std::vector<uint32_t>& rule_rank) {
  SortData d{f, rule_rank.data()};
  int n = int(f->size());
  Pdqsort(d, 0, n, BitsLen(unsigned(n)));
}

// The same permutation with the independent recursive calls (SortSpawn) spread
// over `threads` pool threads: a file with tens of thousands of findings (C3f's
// heaviest holds ~50 k) otherwise sorts on one thread for ~8 ms while the
// scan's other work has drained.  Must not run inside another ParallelFor item.
void SortFindingsParallel(FileFindings* f, const std::vector<uint32_t>& rule_rank, int threads, bool wide) {
  const int n = int(f->size());
  if (threads <= 1 || n < 4096) return SortFindings(f, rule_rank);
  struct Task {
    int a, b, limit;
  };
  struct Queue : SortSpawn {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Task> q;
    int active = 0;
    void Push(int a, int b, int limit) override {
      {
        std::lock_guard<std::mutex> g(mu);
        q.push_back(Task{a, b, limit});
      }
      cv.notify_one();
    }
  } Q;
  Q.min_spawn = std::max(1024, n / (8 * threads));
  Q.q.push_back(Task{0, n, BitsLen(unsigned(n))});
  ParallelFor(size_t(threads), threads, [&](size_t) {
    SortData d{f, rule_rank.data()};
    for (;;) {
      Task t;
      {
        std::unique_lock<std::mutex> lk(Q.mu);
        Q.cv.wait(lk, [&] { return !Q.q.empty() || Q.active == 0; });
        if (Q.q.empty()) return;  // nothing queued and nothing running: done
        t = Q.q.back();
        Q.q.pop_back();
        Q.active++;
      }
      Pdqsort(d, t.a, t.b, t.limit, &Q);
      {
        std::lock_guard<std::mutex> g(Q.mu);
        Q.active--;
      }
      Q.cv.notify_all();
    }
  }, wide);
}

bool SimpleLiteral(const std::string& src, std::vector<std::string>* lits, bool* begin, bool* end) {
  static const std::string kMeta = "\\.+*?()|[]{}^$";
  size_t i = 0, e = src.size();
  *begin = e > 0 && src[0] == '^';
  if (*begin) i = 1;
  // a trailing unescaped '$' (an even run of backslashes before it)
  *end = false;
  if (e > i && src[e - 1] == '$') {
    size_t bs = 0;
    while (e - 1 - bs > i && src[e - 2 - bs] == '\\') bs++;
    if (bs % 2 == 0) {
      *end = true;
      e--;
    }
  }
  // prefix, at most one (?:alt|alt...) group of plain literals, suffix
  std::string pre, post;
  std::vector<std::string> alts;
  int part = 0;  // 0 prefix, 1 inside the group, 2 suffix
  while (i < e) {
    const unsigned char c = static_cast<unsigned char>(src[i]);
    std::string* out = part == 0 ? &pre : part == 2 ? &post : &alts.back();
    // non-ASCII: Go's regexp matches runes (an invalid byte decodes to
    // U+FFFD, which a literal EF BF BD matches), so keep the regex for these
    if (c >= 0x80) return false;
    if (c == '\\') {
      if (i + 1 >= e) return false;
      const unsigned char d = static_cast<unsigned char>(src[i + 1]);
      if (d >= 0x80 || std::isalnum(d) || d == '_') return false;  // \d, \b, \x.. and the like
      out->push_back(char(d));
      i += 2;
    } else if (part == 0 && src.compare(i, 3, "(?:") == 0) {
      part = 1;
      alts.emplace_back();
      i += 3;
    } else if (part == 1 && c == '|') {
      alts.emplace_back();
      i++;
    } else if (part == 1 && c == ')') {
      part = 2;
      i++;
    } else {
      if (kMeta.find(char(c)) != std::string::npos) return false;
      out->push_back(char(c));
      i++;
    }
  }
  if (part == 1) return false;
  lits->clear();
  if (alts.empty()) alts.emplace_back();
  for (auto& x : alts) {
    lits->push_back(pre + x + post);
    if (lits->back().empty()) return false;  // matches everywhere: keep the regex
  }
  return true;
}

bool Matcher::MatchSimple(const uint8_t* s, size_t n) const {
  for (const std::string& lit : simple_lits) {
    const size_t k = lit.size();
    if (k > n) continue;
    const char* l = lit.data();
    if (simple_begin && simple_end ? k == n && std::memcmp(s, l, k) == 0
        : simple_begin             ? std::memcmp(s, l, k) == 0
        : simple_end               ? std::memcmp(s + n - k, l, k) == 0
                                   : memmem(s, n, l, k) != nullptr)
      return true;
  }
  return false;
}

bool Matcher::Match(const uint8_t* s, size_t n) const {
  if (!re) return false;
  if (simple) return MatchSimple(s, n);
  if (!lits.empty()) {
    bool ascii = true;
    for (size_t i = 0; i < n; i++)
      if (s[i] >= 0x80) {
        ascii = false;
        break;
      }
    if (ascii) {
      bool any = false;
      for (auto& l : lits)
        if (AsciiContainsLower(s, n, l)) {
          any = true;
          break;
        }
      if (!any) return false;
    }
  }
  return re->Match(s, int64_t(n));
}

SecretScanner::SecretScanner(std::vector<RuleSpec> rules, std::vector<AllowRuleSpec> allow,
                             std::vector<std::unique_ptr<Regex>> exclude, int device, std::string* err,
                             const CompileOptions* opt)
    : rules_(std::move(rules)), allow_(std::move(allow)), exclude_(std::move(exclude)) {
  rule_rank_ = RuleRanks(rules_);
  std::vector<RuleSrc> src;
  for (auto& r : rules_) src.push_back({r.id, r.regex_src, r.keywords, r.has_regex});
  for (size_t g = 0; g < exclude_.size(); g++) {
    ex_global_rule_.push_back(uint32_t(src.size()));
    src.push_back({"exclude-block:global:" + std::to_string(g), exclude_[g]->pattern(), {}, true});
  }
  ex_rule_.resize(rules_.size());
  for (size_t r = 0; r < rules_.size(); r++)
    for (size_t k = 0; k < rules_[r].exclude.size(); k++) {
      ex_rule_[r].push_back(uint32_t(src.size()));
      src.push_back({"exclude-block:" + rules_[r].id + ":" + std::to_string(k), rules_[r].exclude[k]->pattern(), {},
                     true});
    }
  if (!CompileRules(src, &cr_, &err_, opt)) {
    *err = err_;
    return;
  }
  compiled_ok_ = true;
  for (size_t i = 0; i < rules_.size(); i++) {
    auto& r = rules_[i];
    if (cr_.regex[i] && !r.secret_group_name.empty()) {
      const auto& names = cr_.regex[i]->cap_names();
      for (size_t k = 0; k < names.size(); k++)
        if (names[k] == r.secret_group_name) r.group_idx.push_back(int(k));
    }
    for (auto& kw : r.keywords) r.kw_lower_host.push_back(GoBytesToLower((const uint8_t*)kw.data(), kw.size()));
    for (auto& kw : r.kw_lower_host) {
      r.kw_ascii.push_back(IsAsciiStr(kw) ? 1 : 0);
      r.kw_rare.push_back(uint16_t(RarestIndex(kw)));
    }
  }
  BuildAllowPathFilter();
  BuildPathFilter(device);
  const char* ht = std::getenv("TSG_HOST_THREADS");
  host_threads_ = ht ? std::atoi(ht) : 16;
  if (host_threads_ <= 0) host_threads_ = 1;
  if (device < 0) {
    no_engine_ = true;
    return;
  }
  const char* slots_env = std::getenv("TSG_GPU_SLOTS");
  int slots = slots_env ? std::atoi(slots_env) : 1;  // 2 measured slower at C2 (kernels interfere)
  if (slots < 1) slots = 1;
  if (slots > 4) slots = 4;
  gpu_mu_.reset(new std::mutex[size_t(slots)]);
  for (int k = 0; k < slots; k++) {
    engines_.emplace_back(new GpuEngine(cr_, device));
    if (!engines_.back()->ok()) {
      err_ = engines_.back()->error();
      *err = err_;
      return;
    }
  }
  // findings of HBM-resident batches: 0 (default) on the host, 1 always on the
  // GPU, 2 on the GPU while the exact pass is the bound (TSG_GPU_FINDINGS).  The
  // host is the default because it measured faster on C3f, the finding-dense
  // case the GPU pass was built for: 536 vs 474 GB/s at depth 4, 578 vs 516 at
  // depth 6 (one box, 20 steps, profiles/r06/c3f) -- the GPU pass frees ~4 of
  // 16 host CPUs, but its round trip behind the other scans' kernels (6-8 ms)
  // and the host-side copy and sort that remain cost more latency than the
  // freed CPUs return
  const char* gf = std::getenv("TSG_GPU_FINDINGS");
  gpu_findings_.store(gf ? std::max(0, std::min(2, std::atoi(gf))) : 0);
  mat_.reset(new FindingMaterializer(device));
  if (!mat_->ok()) {
    err_ = mat_->error();
    *err = err_;
    return;
  }
}

void SecretScanner::BuildAllowPathFilter() {
  ap_fast_ = false;
  if (allow_.size() > 64) return;
  ap_pair_.assign(65536, 0);
  ap_lits_.clear();
  ap_c0_.clear();
  ap_c1_.clear();
  for (auto& w : ap_first_) w = 0;
  ap_always_ = 0;
  for (size_t i = 0; i < allow_.size(); i++) {
    const Matcher* m = allow_[i].path.get();
    if (!m || !m->re) continue;  // never matches
    bool always = m->lits.empty();
    for (auto& l : m->lits)
      if (l.size() < 2) always = true;
    if (always) {
      ap_always_ |= uint64_t(1) << i;
      continue;
    }
    for (auto& l : m->lits) {
      ap_first_[uint8_t(l[0]) >> 6] |= uint64_t(1) << (uint8_t(l[0]) & 63);
      uint16_t& slot = ap_pair_[(uint32_t(uint8_t(l[0])) << 8) | uint8_t(l[1])];
      if (!slot) {
        ap_c0_.push_back(uint8_t(l[0]));
        ap_c1_.push_back(uint8_t(l[1]));
        ap_lits_.emplace_back();
        slot = uint16_t(ap_lits_.size());
      }
      ap_lits_[slot - 1].push_back({l, uint32_t(i)});
    }
  }
  ap_fast_ = ap_lits_.size() < 65535;
}

void SecretScanner::BuildPathFilter(int device) {
  // the GPU prefilter reports every path holding one of a rule's literals
  // (and every non-ASCII path): usable when no path rule goes unfiltered
  if (!ap_fast_ || ap_always_ || device < 0 || std::getenv("TSG_GPU_ALLOW_PATH") &&
                                                    std::atoi(std::getenv("TSG_GPU_ALLOW_PATH")) == 0)
    return;
  std::vector<std::pair<std::string, uint32_t>> lits;
  for (auto& v : ap_lits_) lits.insert(lits.end(), v.begin(), v.end());
  PathTable t;
  if (!BuildPathTable(lits, &t)) return;
  std::unique_ptr<PathFilter> pf(new PathFilter(device, t));
  if (pf->ok()) path_filter_ = std::move(pf);
}

bool SecretScanner::AllowPath(const uint8_t* p, size_t n) const {
  // Matcher::Match rejects an ASCII path holding none of a rule's (lowercase)
  // literals; here the literals are located in one pass over the lowered
  // path (byte-pair table, then the whole literal), and only the rules with a
  // literal present (plus the unfiltered ones) run their regex.
  if (ap_fast_ && n <= 1024) {
    alignas(32) uint8_t low[1024 + 64];
    uint8_t high = 0;
    for (size_t i = 0; i < n; i++) {  // branch-free ASCII lowering (vectorised)
      const uint8_t b = p[i];
      high |= b;
      low[i] = uint8_t(b + ((uint8_t(b - 'A') < 26) ? 32 : 0));
    }
    std::memset(low + n, 0, 33);  // no literal holds a NUL byte
    if (!(high & 0x80)) {
      uint64_t lit_rules = 0;
      auto check_at = [&](size_t i) {
        const uint16_t slot = ap_pair_[(uint32_t(low[i]) << 8) | low[i + 1]];
        if (!slot) return;
        for (auto& lr : ap_lits_[slot - 1])
          if (!(lit_rules >> lr.second & 1) && lr.first.size() <= n - i &&
              std::memcmp(low + i, lr.first.data(), lr.first.size()) == 0)
            lit_rules |= uint64_t(1) << lr.second;
      };
      if (ap_c0_.size() <= 32) {
        // 32 positions at a time: the pairs (low[i], low[i+1]) that begin some literal
        typedef char v32 __attribute__((vector_size(32)));
        const size_t np = ap_c0_.size();
        for (size_t i = 0; i + 1 < n; i += 32) {
          v32 a, b;
          std::memcpy(&a, low + i, 32);
          std::memcpy(&b, low + i + 1, 32);
          v32 hit = {};
          for (size_t k = 0; k < np; k++) hit |= (a == char(ap_c0_[k])) & (b == char(ap_c1_[k]));
          uint32_t m = uint32_t(__builtin_ia32_pmovmskb256(hit));
          const size_t lim = n - 1 - i;  // pair starts i .. n - 2
          if (lim < 32) m &= (1u << lim) - 1;
          while (m) {
            check_at(i + size_t(__builtin_ctz(m)));
            m &= m - 1;
          }
        }
      } else {
        for (size_t i = 0; i + 1 < n; i++)
          if ((ap_first_[low[i] >> 6] >> (low[i] & 63)) & 1) check_at(i);  // L1-resident test first
      }
      return AllowPathRules(p, n, lit_rules);
    }
  }
  for (auto& a : allow_)
    if (a.path && a.path->Match(p, n)) return true;
  return false;
}

bool SecretScanner::AllowPathRules(const uint8_t* p, size_t n, uint64_t lit_rules) const {
  uint64_t mask = ap_always_ | lit_rules;
  while (mask) {
    const int i = __builtin_ctzll(mask);
    mask &= mask - 1;
    const Matcher& m = *allow_[size_t(i)].path;
    if (m.simple ? m.MatchSimple(p, n) : (lit_rules >> i & 1) ? m.re->Match(p, int64_t(n)) : m.Match(p, n))
      return true;
  }
  return false;
}

namespace {
bool HasSeq(const uint8_t* s, size_t n, const char* seq, size_t k) {  // memchr on the lead byte
  const uint8_t* p = s;
  const uint8_t* e = s + n;
  while (p + k <= e) {
    const void* q = std::memchr(p, uint8_t(seq[0]), size_t(e - p) - (k - 1));
    if (!q) return false;
    p = static_cast<const uint8_t*>(q);
    if (std::memcmp(p, seq, k) == 0) return true;
    p++;
  }
  return false;
}

// bytes.ToLower(content) contains the lowercase ASCII kw, for content holding
// U+0130 / U+212A: every kw char matches an ASCII byte of either case, and
// 'i' also C4 B0 (U+0130 lowers to 'i'), 'k' also E2 84 AA (U+212A lowers to
// 'k'); no other rune lowers into ASCII and these byte sequences always decode
// as those runes.
bool FoldCaseContains(const uint8_t* s, size_t n, const std::string& kw) {
  const size_t m = kw.size();
  if (m == 0) return true;
  for (size_t st = 0; st < n; st++) {
    size_t p = st, i = 0;
    for (; i < m && p < n; i++) {
      uint8_t c = s[p];
      if (c >= 'A' && c <= 'Z') c = uint8_t(c + 32);
      if (c == uint8_t(kw[i])) {
        p++;
        continue;
      }
      if (kw[i] == 'i' && c == 0xC4 && p + 1 < n && s[p + 1] == 0xB0) {
        p += 2;
        continue;
      }
      if (kw[i] == 'k' && c == 0xE2 && p + 2 < n && s[p + 1] == 0x84 && s[p + 2] == 0xAA) {
        p += 3;
        continue;
      }
      break;
    }
    if (i == m) return true;
  }
  return false;
}

// Is the lowercase ASCII string kw a substring of the content with ASCII letters
// case-folded?  Scans with memchr for kw's least frequent character (both cases).
bool AsciiCaseContains(const uint8_t* s, size_t n, const std::string& kw, size_t best) {
  const size_t m = kw.size();
  if (m == 0) return true;
  if (n < m) return false;
  auto eq_at = [&](const uint8_t* p) {  // p = candidate start
    for (size_t i = 0; i < m; i++) {
      uint8_t c = p[i];
      if (c >= 'A' && c <= 'Z') c = uint8_t(c + 32);
      if (c != uint8_t(kw[i])) return false;
    }
    return true;
  };
  const uint8_t c0 = uint8_t(kw[best]);
  const int passes = (c0 >= 'a' && c0 <= 'z') ? 2 : 1;
  for (int pass = 0; pass < passes; pass++) {
    const uint8_t c = pass ? uint8_t(c0 - 32) : c0;
    const uint8_t* p = s + best;
    const uint8_t* e = s + n - (m - 1 - best);  // last valid position of the scanned char + 1
    while (p < e) {
      const void* q = std::memchr(p, c, size_t(e - p));
      if (!q) break;
      const uint8_t* hitp = static_cast<const uint8_t*>(q);
      if (eq_at(hitp - best)) return true;
      p = hitp + 1;
    }
  }
  return false;
}
bool AllowRulesAllow(const std::vector<AllowRuleSpec>& rules, const uint8_t* s, size_t n) {
  for (auto& a : rules)
    if (a.regex && a.regex->Match(s, n)) return true;
  return false;
}
bool AllowRulesAllowPath(const std::vector<AllowRuleSpec>& rules, const uint8_t* s, size_t n) {
  for (auto& a : rules)
    if (a.path && a.path->Match(s, n)) return true;
  return false;
}
}  // namespace

// Host-tail phase profile (TSG_TAIL_DEBUG=1 only; otherwise the timers are inert).
const bool g_tail_debug = std::getenv("TSG_TAIL_DEBUG") != nullptr;
std::atomic<int64_t> g_prof[16];  // [8] [9] [10]: bytes memchr'd forward / backward (no hint, in a window) by the line walks
std::atomic<int64_t> g_wholefile_bytes{0}, g_wholefile_calls{0};  // TSG_TAIL_DEBUG: whole-content gate scans
constexpr uint32_t kRuleProf = 4096;
std::atomic<int64_t> g_rule_ns[kRuleProf], g_rule_calls[kRuleProf];
struct PhaseTimer {
  int k;
  std::chrono::steady_clock::time_point t0;
  explicit PhaseTimer(int kk) : k(kk) {
    if (g_tail_debug) t0 = std::chrono::steady_clock::now();
  }
  ~PhaseTimer() {
    if (g_tail_debug)
      g_prof[k] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  }
};

namespace {
// Per host thread scratch of ScanFile: cleared per file, never freed, so the
// per-file vectors cost no allocation (malloc was ~14% of the host tail).
struct ScanScratch {
  std::vector<std::pair<uint32_t, Loc>> matched;
  std::vector<Loc> censor, locs, spans, merged;
  std::vector<std::pair<int64_t, int64_t>> nla;
  std::vector<const Candidate*> hints, fhints;
  std::vector<Window> wins;
  std::vector<int64_t> m, span_nl, vnl;
  // line texts already in the file's FileFindings::text, by line number (a
  // direct-mapped cache; `gen` tags the file it belongs to)
  struct LineText {
    uint64_t gen;
    int64_t line;
    uint32_t off, len;
  };
  static constexpr size_t kLineCache = 256;
  LineText line_cache[kLineCache] = {};
  uint64_t gen = 0;
};
thread_local ScanScratch t_scan;
}  // namespace

void SecretScanner::ScanFile(const uint8_t* content, int64_t len, std::string_view path, bool binary,
                             const Candidate* c, size_t nc, FileResult* out, bool gpu_windows) const {
  PhaseTimer pt_all(7);
  MatchFile(content, len, path, c, nc, gpu_windows);
  if (t_scan.matched.empty()) {
    out->kind = kNoFindings;
    return;
  }
  FindingsHost(content, len, path, binary, c, nc, out);
}

void SecretScanner::MatchFile(const uint8_t* content, int64_t len, std::string_view path, const Candidate* c,
                              size_t nc, bool gpu_windows) const {
  const uint8_t* P = reinterpret_cast<const uint8_t*>(path.data());
  ScanScratch& S = t_scan;
  std::vector<std::pair<uint32_t, Loc>>& matched = S.matched;
  std::vector<Loc>& censor = S.censor;
  matched.clear();
  censor.clear();
  bool gblocks_done = false;
  std::vector<Loc> gblocks;
  std::string lowered;
  bool lowered_done = false;
  bool fold_done = false, fold_runes = false;

  // the candidates are sorted by rule: real rules first, then the exclude-block rules
  const uint32_t n_real = uint32_t(rules_.size());
  size_t nc_real = 0;
  while (nc_real < nc && c[nc_real].rule < n_real) nc_real++;
  auto block_windows = [&](uint32_t rule, std::vector<Window>* wins) {  // merged candidate windows of a block rule
    for (size_t k = nc_real; k < nc; k++) {
      if (c[k].rule != rule) continue;
      Window w{c[k].wlo, c[k].whi};
      if (!wins->empty() && w.lo <= wins->back().hi + 1) wins->back().hi = std::max(wins->back().hi, w.hi);
      else wins->push_back(w);
    }
  };
  auto blocks_match = [&](const std::vector<std::unique_ptr<Regex>>& rx, const std::vector<uint32_t>& rx_rule,
                          std::vector<Loc>* cache, bool* done, Loc loc) {
    if (!*done) {
      *done = true;
      for (size_t q = 0; q < rx.size(); q++) {
        std::vector<int64_t> m;
        if (gpu_windows) {  // Blocks.find (scanner.go:262-275) where a block can start
          std::vector<Window> wins;
          block_windows(rx_rule[q], &wins);
          if (wins.empty()) continue;
          rx[q]->FindAll(content, len, false, &wins, &m);
        } else {
          rx[q]->FindAll(content, len, false, nullptr, &m);
        }
        for (size_t k = 0; k + 1 < m.size(); k += 2) cache->push_back({m[k], m[k + 1]});
      }
    }
    for (auto& b : *cache)
      if (b.s <= loc.s && loc.e <= b.e) return true;
    return false;
  };

  size_t i = 0;
  while (i < nc_real) {
    uint32_t r = c[i].rule;
    size_t j = i;
    std::vector<Window>& wins = S.wins;
    wins.clear();
    uint32_t group_flags = ~0u;  // AND over the group's candidates (file-level bits agree)
    while (j < nc_real && c[j].rule == r) {
      group_flags &= c[j].flags;
      Window w{c[j].wlo, c[j].whi};
      if (!wins.empty() && w.lo <= wins.back().hi + 1) wins.back().hi = std::max(wins.back().hi, w.hi);
      else wins.push_back(w);
      j++;
    }
    i = j;
    const RuleSpec& R = rules_[r];
    const Regex* re = cr_.regex[r].get();
    if (!re) continue;
    if (R.path && !R.path->Match(P, path.size())) continue;                      // MatchPath :397
    if (AllowRulesAllowPath(R.allow_rules, P, path.size())) continue;            // AllowPath :403
    bool sub = !R.secret_group_name.empty();
    std::vector<int64_t>& m = S.m;
    m.clear();
    {
      PhaseTimer pt(0);
      const auto fa0 = g_tail_debug ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
      re->FindAll(content, len, sub, &wins, &m);
      if (g_tail_debug && r < kRuleProf) {  // per-rule FindAll time (TSG_TAIL_DEBUG)
        g_rule_ns[r] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - fa0).count();
        g_rule_calls[r] += 1;
      }
    }
    if (m.empty()) continue;
    size_t stride = sub ? size_t(2 * (re->num_cap() + 1)) : 2;
    // MatchKeywords (:409), evaluated lazily: it only matters when FindLocations
    // has matches.  A match is a run of whole runes of the content, so a
    // keyword inside its lowered bytes is inside bytes.ToLower(content) too;
    // otherwise the whole content is lowered and searched.
    if (cr_.rules[r].gate != kGateAlways) {
      PhaseTimer pt(1);
      // an open gate in the GPU's keyword bits (exact ASCII occurrences in the
      // file) settles it at once; the per-match and whole-content checks below
      // are for closed or inexact bits
      bool hit = (group_flags & kCandGateValid) && cr_.rules[r].gate == kGateKeywords &&
                 !cr_.rules[r].kw_match_implied && (group_flags & kCandGateOpen);
      for (size_t k = 0; k + stride <= m.size() && !hit; k += stride) {
        const uint8_t* ms = content + m[k];
        const size_t mn = size_t(m[k + 1] - m[k]);
        // ASCII keywords in a match without U+0130 / U+212A: the ASCII
        // case-insensitive search is exact (see the whole-content case below)
        uint8_t high = 0;  // the fold runes are multi-byte: an ASCII match holds none
        for (size_t q = 0; q < mn; q++) high |= ms[q];
        const bool fold = (high & 0x80) && (HasSeq(ms, mn, "\xC4\xB0", 2) || HasSeq(ms, mn, "\xE2\x84\xAA", 3));
        bool go = fold;
        for (size_t q = 0; q < R.kw_lower_host.size(); q++) {
          if (!R.kw_ascii[q]) go = true;
          else if (!fold && AsciiCaseContains(ms, mn, R.kw_lower_host[q], R.kw_rare[q])) {
            hit = true;
            break;
          }
        }
        if (!hit && go) {
          std::string ml = GoBytesToLower(ms, mn);
          for (auto& kw : R.kw_lower_host)
            if (ml.find(kw) != std::string::npos) {
              hit = true;
              break;
            }
        }
      }
      // GPU keyword bits (ASCII occurrences anywhere in the file) and the
      // file's U+0130/U+212A flag, when the candidates carry them
      const bool gpu_bits = (group_flags & kCandGateValid) && cr_.rules[r].gate == kGateKeywords &&
                            !cr_.rules[r].kw_match_implied;
      if (!hit && gpu_bits) {
        hit = (group_flags & kCandGateOpen) != 0;
        fold_done = true;
        fold_runes = (group_flags & kCandFoldFile) != 0;
      }
      if (!hit) {
        // ASCII keywords: an occurrence in the ASCII-lowered bytes is one in
        // bytes.ToLower(content) (ASCII bytes are whole runes); the only other
        // runes lowering into ASCII are U+0130 -> 'i' and U+212A -> 'k', so
        // without them the ASCII search is exact.  Otherwise lower as Go does.
        if (!fold_done) {
          if (g_tail_debug) {
            g_wholefile_bytes += len;
            g_wholefile_calls += 1;
          }
          fold_runes = HasSeq(content, size_t(len), "\xC4\xB0", 2) || HasSeq(content, size_t(len), "\xE2\x84\xAA", 3);
          fold_done = true;
        }
        if (g_tail_debug && !gpu_bits) {
          g_wholefile_bytes += len;
          g_wholefile_calls += 1;
        }
        if (!gpu_bits)
          for (size_t q = 0; q < R.kw_lower_host.size(); q++)
            if (R.kw_ascii[q] && AsciiCaseContains(content, size_t(len), R.kw_lower_host[q], R.kw_rare[q])) {
              hit = true;
              break;
            }
        if (!hit && fold_runes)
          for (auto& kw : R.kw_lower_host)
            if (IsAsciiStr(kw) && FoldCaseContains(content, size_t(len), kw)) {
              hit = true;
              break;
            }
        bool need_go = false;
        for (auto& kw : R.kw_lower_host)
          if (!IsAsciiStr(kw)) need_go = true;
        if (!hit && need_go) {
          PhaseTimer p6(6);
          if (!lowered_done) {
            lowered = GoBytesToLower(content, size_t(len));
            lowered_done = true;
          }
          for (auto& kw : R.kw_lower_host)
            if (lowered.find(kw) != std::string::npos) {
              hit = true;
              break;
            }
        }
      }
      if (!hit) continue;
    }
    std::vector<Loc>& locs = S.locs;
    locs.clear();
    PhaseTimer pt5(5);
    for (size_t k = 0; k + stride <= m.size(); k += stride) {
      int64_t s = m[k], e = m[k + 1];
      if (AllowRulesAllow(allow_, content + s, size_t(e - s)) ||
          AllowRulesAllow(R.allow_rules, content + s, size_t(e - s)))  // AllowLocation :150-153
        continue;
      if (sub) {
        for (int g : R.group_idx) locs.push_back({m[k + 2 * g], m[k + 2 * g + 1]});
      } else {
        locs.push_back({s, e});
      }
    }
    if (locs.empty()) continue;
    PhaseTimer pt2(2);
    bool lblocks_done = false;
    std::vector<Loc> lblocks;
    for (auto& loc : locs) {
      if (blocks_match(exclude_, ex_global_rule_, &gblocks, &gblocks_done, loc) ||
          blocks_match(R.exclude, ex_rule_[r], &lblocks, &lblocks_done, loc))
        continue;
      if (loc.s < 0) continue;  // non-participating group: the reference would panic here
      matched.push_back({r, loc});
      censor.push_back(loc);
    }
  }
}

void SecretScanner::FindingsHost(const uint8_t* content, int64_t len, std::string_view path, bool binary,
                                 const Candidate* c, size_t nc, FileResult* out) const {
  ScanScratch& S = t_scan;
  std::vector<std::pair<uint32_t, Loc>>& matched = S.matched;
  std::vector<Loc>& censor = S.censor;
  // (wlo, nl_before) anchors for line numbers
  std::vector<std::pair<int64_t, int64_t>>& nla = S.nla;
  nla.clear();
  for (size_t i = 0; i < nc; i++) nla.push_back({c[i].wlo, c[i].nl_before});
  std::sort(nla.begin(), nla.end());
  // the GPU's last-three-newlines before each window (Candidate::nl_back)
  std::vector<const Candidate*>& hints = S.hints;
  hints.clear();
  static const bool use_hints = !std::getenv("TSG_NL_HINTS") || std::atoi(std::getenv("TSG_NL_HINTS")) != 0;
  for (size_t i = 0; i < nc && use_hints; i++)
    if (c[i].nl_back[0] != kNlUnknown && c[i].nl_back[0] != 0) hints.push_back(&c[i]);  // 0: never a GPU value
  std::sort(hints.begin(), hints.end(), [](const Candidate* a, const Candidate* b) { return a->wlo < b->wlo; });
  // and the first three at or after it (Candidate::nl_fwd)
  std::vector<const Candidate*>& fhints = S.fhints;
  fhints.clear();
  for (size_t i = 0; i < nc && use_hints; i++)
    if (c[i].nl_fwd[0] != kNlUnknown) fhints.push_back(&c[i]);
  std::sort(fhints.begin(), fhints.end(), [](const Candidate* a, const Candidate* b) { return a->wlo < b->wlo; });

  // findLocation runs on the censored buffer (scanner.go:438-439): newlines
  // inside a censored span are '*' there.  Spans merged and sorted:
  std::vector<Loc>& spans = S.spans;
  spans.assign(censor.begin(), censor.end());
  std::sort(spans.begin(), spans.end(), [](const Loc& a, const Loc& b) { return a.s < b.s; });
  {
    std::vector<Loc>& m = S.merged;
    m.clear();
    for (auto& z : spans) {
      if (z.e <= z.s) continue;
      if (!m.empty() && z.s <= m.back().e) m.back().e = std::max(m.back().e, z.e);
      else m.push_back(z);
    }
    spans.swap(m);
  }
  auto first_span_after = [&](int64_t a) {  // first span with e > a (spans are disjoint and sorted)
    return size_t(std::upper_bound(spans.begin(), spans.end(), a, [](int64_t v, const Loc& z) { return v < z.e; }) -
                  spans.begin());
  };
  FileFindings& ff = out->findings;
  // content [a, b) with censored bytes as '*', into ff.text; k0: a span index at
  // or below the first span ending after a (a finding's lines ascend: one search)
  auto put_censored_from = [&](size_t k0, int64_t a, int64_t b) {
    const uint32_t at = uint32_t(ff.text.size());
    ff.text.append(reinterpret_cast<const char*>(content + a), size_t(b - a));
    size_t k = k0;
    while (k < spans.size() && spans[k].e <= a) k++;
    for (; k < spans.size() && spans[k].s < b; k++) {
      int64_t x = std::max(a, spans[k].s), y = std::min(b, spans[k].e);
      if (x < y) std::memset(&ff.text[at + size_t(x - a)], '*', size_t(y - x));
    }
    return at;
  };
  auto count_nl_raw = [&](int64_t a, int64_t b) {
    int64_t n = 0;
    const uint8_t* p = content + a;
    const uint8_t* e = content + b;
    while (p < e) {
      const void* q = std::memchr(p, '\n', size_t(e - p));
      if (!q) break;
      n++;
      p = static_cast<const uint8_t*>(q) + 1;
    }
    return n;
  };
  auto censored_nl = [&](int64_t a, int64_t b) {  // '\n' bytes hidden by censoring in [a, b)
    int64_t n = 0;
    for (size_t k = first_span_after(a); k < spans.size() && spans[k].s < b; k++) {
      int64_t x = std::max(a, spans[k].s), y = std::min(b, spans[k].e);
      if (x < y) n += count_nl_raw(x, y);
    }
    return n;
  };
  // Files with many matches for their size: an index of the '\n' the censored
  // content keeps (those outside the spans), so each finding's line number,
  // line bounds and code lines are binary searches instead of walks.
  std::vector<int64_t>& vnl = S.vnl;
  vnl.clear();
  const bool use_index = matched.size() >= 8 && uint64_t(len) <= uint64_t(matched.size()) * 8192;
  if (use_index) {
    PhaseTimer pt15(15);
    size_t k = 0;
    for (const uint8_t *p = content, *e = content + len; p < e;) {
      const void* q = std::memchr(p, '\n', size_t(e - p));
      if (!q) break;
      const int64_t at = static_cast<const uint8_t*>(q) - content;
      while (k < spans.size() && spans[k].e <= at) k++;
      if (!(k < spans.size() && spans[k].s <= at)) vnl.push_back(at);  // not censored
      p = static_cast<const uint8_t*>(q) + 1;
    }
  }
  auto vnl_below = [&](int64_t pos) {  // visible '\n' before pos
    return int64_t(std::lower_bound(vnl.begin(), vnl.end(), pos) - vnl.begin());
  };
  std::vector<int64_t>& span_nl = S.span_nl;  // '\n' in spans[0 .. i)
  span_nl.assign(spans.size() + 1, 0);
  for (size_t k = 0; k < spans.size(); k++) span_nl[k + 1] = span_nl[k] + count_nl_raw(spans[k].s, spans[k].e);
  auto censored_nl_before = [&](int64_t pos) {  // censored_nl(0, pos)
    const size_t k = first_span_after(pos);  // spans [0, k) end at or before pos
    int64_t n = span_nl[k];
    if (k < spans.size() && spans[k].s < pos) n += count_nl_raw(spans[k].s, pos);
    return n;
  };
  auto count_nl = [&](int64_t a, int64_t b) {
    if (use_index) return vnl_below(b) - vnl_below(a);
    return count_nl_raw(a, b) - censored_nl(a, b);
  };
  auto nl_before = [&](int64_t pos) {
    if (use_index) return vnl_below(pos);
    int64_t raw;
    auto it = std::upper_bound(nla.begin(), nla.end(), std::make_pair(pos, INT64_MAX));
    if (it == nla.begin()) {
      raw = count_nl_raw(0, pos);
    } else {
      --it;
      raw = it->second + count_nl_raw(it->first, pos);
    }
    return raw - censored_nl_before(pos);
  };
  auto in_span = [&](int64_t p) -> const Loc* {
    auto it = std::upper_bound(spans.begin(), spans.end(), p, [](int64_t v, const Loc& z) { return v < z.s; });
    if (it == spans.begin()) return nullptr;
    --it;
    return p < it->e ? &*it : nullptr;
  };
  auto last_nl = [&](int64_t pos) -> int64_t {  // the last '\n' in [0, pos), or -1
    if (pos <= 0) return -1;
    auto it = std::upper_bound(hints.begin(), hints.end(), pos,
                               [](int64_t v, const Candidate* h) { return v < h->wlo; });
    if (it != hints.begin()) {  // a window starting at or below pos: [wlo, pos), then its list
      const Candidate& h = **(it - 1);
      if (pos > h.wlo) {
        // the forward list names the first '\n' at or after wlo: when it ends
        // below pos, only (its last, pos) is searched, when it reaches pos or
        // the file end nothing is (a match deep in a long line: no scan back
        // over the line)
        int64_t known = -1, from = h.wlo;
        bool complete = false;
        for (int k = 0; k < 3; k++) {
          if (h.nl_fwd[k] == kNlUnknown) break;
          if (h.nl_fwd[k] == kNlNone) {
            complete = true;
            break;
          }
          const int64_t at = h.wlo + int64_t(h.nl_fwd[k]);
          if (at >= pos) {
            complete = true;
            break;
          }
          known = at;
          from = at + 1;
        }
        if (!complete && from < pos) {
          const void* q = memrchr(content + from, '\n', size_t(pos - from));
          if (g_tail_debug) g_prof[10] += q ? pos - (static_cast<const uint8_t*>(q) - content) : pos - from;
          if (q) return int64_t(static_cast<const uint8_t*>(q) - content);
        }
        if (known >= 0) return known;
      }
      return h.nl_back[0] == kNlNone ? -1 : h.wlo - int64_t(h.nl_back[0]);
    }
    if (it != hints.end()) {  // the next window above pos: its list may reach below pos
      const Candidate& h = **it;
      for (int k = 0; k < 3; k++) {
        if (h.nl_back[k] == kNlUnknown) break;
        if (h.nl_back[k] == kNlNone) return -1;  // every '\n' before wlo is listed, all >= pos
        const int64_t at = h.wlo - int64_t(h.nl_back[k]);
        if (at < pos) return at;
      }
    }
    const void* q = memrchr(content, '\n', size_t(pos));
    if (g_tail_debug) g_prof[9] += q ? pos - (static_cast<const uint8_t*>(q) - content) : pos;
    return q ? int64_t(static_cast<const uint8_t*>(q) - content) : -1;
  };
  auto line_start_of = [&](int64_t pos) {  // after the last visible '\n' before pos
    if (use_index) {
      const int64_t k = vnl_below(pos);
      return k ? vnl[size_t(k - 1)] + 1 : int64_t(0);
    }
    int64_t p = pos;  // search [0, p)
    while (p > 0) {
      const int64_t at = last_nl(p);
      if (at < 0) return int64_t(0);
      const Loc* z = in_span(at);
      if (!z) return at + 1;
      p = z->s;
    }
    return int64_t(0);
  };
  auto next_nl = [&](int64_t pos) -> int64_t {  // the first '\n' in [pos, len), or -1
    auto it = std::upper_bound(fhints.begin(), fhints.end(), pos,
                               [](int64_t v, const Candidate* h) { return v < h->wlo; });
    if (it != fhints.begin()) {  // a window starting at or below pos: its list covers [wlo, third '\n']
      const Candidate& h = **(it - 1);
      for (int k = 0; k < 3; k++) {
        if (h.nl_fwd[k] == kNlUnknown) break;
        if (h.nl_fwd[k] == kNlNone) return -1;  // every '\n' after wlo is listed, all < pos
        const int64_t at = h.wlo + int64_t(h.nl_fwd[k]);
        if (at >= pos) return at;
      }
    }
    int64_t lim = len;  // no '\n' in [pos, lim) is known; `known` is the first one at or after lim
    int64_t known = -1;
    if (it != fhints.end()) {  // the next window above pos: the '\n' around its wlo are listed
      const Candidate& h = **it;
      lim = h.wlo;
      known = h.nl_fwd[0] == kNlNone ? -1 : h.wlo + int64_t(h.nl_fwd[0]);
      if (h.nl_back[0] != kNlUnknown && h.nl_back[0] != 0) {  // the last three before wlo, nearest first
        for (int k = 0; k < 3; k++) {
          if (h.nl_back[k] == kNlUnknown) break;
          if (h.nl_back[k] == kNlNone) {  // every '\n' before wlo is listed
            lim = pos;
            break;
          }
          const int64_t at = h.wlo - int64_t(h.nl_back[k]);
          if (at < pos) {  // the listed ones at or after pos are all there are in [pos, wlo)
            lim = pos;
            break;
          }
          lim = at;  // no other '\n' in [at, wlo)
          known = at;
        }
      }
    }
    if (lim > pos) {
      const void* q = std::memchr(content + pos, '\n', size_t(lim - pos));
      if (g_tail_debug) g_prof[8] += q ? static_cast<const uint8_t*>(q) - (content + pos) : lim - pos;
      if (q) return int64_t(static_cast<const uint8_t*>(q) - content);
    }
    return known;
  };
  auto line_end_of = [&](int64_t pos) {  // first visible '\n' at or after pos, or len
    if (use_index) {
      const size_t k = size_t(vnl_below(pos));
      return k < vnl.size() ? vnl[k] : len;
    }
    int64_t p = pos;
    while (p < len) {
      const int64_t at = next_nl(p);
      if (at < 0) return len;
      const Loc* z = in_span(at);
      if (!z) return at;
      p = z->e;
    }
    return len;
  };

  out->kind = kHasFindings;
  ff.binary = binary;
  if (g_tail_debug) {
    g_prof[use_index ? 11 : 12] += int64_t(matched.size());
    g_prof[13] += int64_t(spans.size());
  }
  PhaseTimer pt3(3);
  // a line's censored text (its first 100 B, or all of it when shorter) is the
  // same for every finding whose code window holds it: stored once per file, its
  // range shared (finding-dense files repeat their neighbouring lines ~5x)
  const uint64_t gen = ++S.gen;
  auto line_text = [&](int64_t k, size_t kspan, int64_t a, int64_t b) -> uint32_t {  // line k = content [a, b)
    ScanScratch::LineText& e = S.line_cache[size_t(k) & (ScanScratch::kLineCache - 1)];
    if (e.gen == gen && e.line == k) return e.off;
    const uint32_t off = put_censored_from(kspan, a, b);
    e = ScanScratch::LineText{gen, k, off, uint32_t(b - a)};
    return off;
  };
  ff.f.reserve(matched.size());
  ff.lines.reserve(matched.size() * 5);
  ff.text.reserve(matched.size() * 320);  // match line + 4 lines of <= 100 B, typically
  // With the newline index, line L of the censored content is [line_lo(L), line_hi(L)):
  // a finding's lines are index arithmetic from the two searches for its start and
  // end (the walks below made ~12 searches per finding; C3f has 368 k findings).
  const int64_t n_vnl = int64_t(vnl.size());
  auto line_lo = [&](int64_t L) { return L > 0 ? vnl[size_t(L - 1)] + 1 : int64_t(0); };
  auto line_hi = [&](int64_t L) { return L < n_vnl ? vnl[size_t(L)] : len; };
  // A rule's matches ascend: the searches for a finding's start line and first
  // span gallop from the previous finding's answers while positions ascend.
  int64_t fg_pos = -1, fg_line = 0, fg_p = -1;
  size_t fg_span = 0;
  auto vnl_below_f = [&](int64_t pos) {  // vnl_below(pos)
    int64_t h = 0;
    if (pos >= fg_pos && fg_pos >= 0) {
      h = fg_line;  // vnl[0 .. h) < fg_pos <= pos
      int64_t step = 1;
      while (h + step <= n_vnl && vnl[size_t(h + step - 1)] < pos) {
        h += step;
        step <<= 1;
      }
      h = int64_t(std::lower_bound(vnl.begin() + h, vnl.begin() + std::min(h + step, n_vnl), pos) - vnl.begin());
    } else {
      h = vnl_below(pos);
    }
    fg_pos = pos;
    fg_line = h;
    return h;
  };
  auto first_span_after_f = [&](int64_t a) {  // first_span_after(a)
    size_t k;
    if (a >= fg_p && fg_p >= 0) {
      k = fg_span;  // spans [0, k) end at or before fg_p <= a
      size_t step = 1;
      while (k + step <= spans.size() && spans[k + step - 1].e <= a) {
        k += step;
        step <<= 1;
      }
      k = size_t(std::upper_bound(spans.begin() + k, spans.begin() + std::min(k + step, spans.size()), a,
                                  [](int64_t v, const Loc& z) { return v < z.e; }) - spans.begin());
    } else {
      k = first_span_after(a);
    }
    fg_p = a;
    fg_span = k;
    return k;
  };
  for (auto& mt : matched) {  // toFinding / findLocation :475-558
    int64_t start = mt.second.s, end = mt.second.e;
    FindingOut f;
    f.rule = mt.first;
    int64_t start_line_num, ls, le, end_line_num;
    if (use_index) {
      start_line_num = vnl_below_f(start);
      ls = line_lo(start_line_num);
      le = line_hi(start_line_num);
      end_line_num = start_line_num;  // vnl_below(end): a match spans few lines
      while (end_line_num < n_vnl && vnl[size_t(end_line_num)] < end) end_line_num++;
    } else {
      start_line_num = nl_before(start);
      ls = line_start_of(start);
      le = line_end_of(start);
      end_line_num = start_line_num + count_nl(start, end);
    }
    int64_t mls = ls, mle = le;
    if (le - ls > 100) {
      mls = (start - ls - 30 < 0) ? ls : start - 30;
      mle = (end + 20 > le) ? le : end + 20;
    }
    int64_t code_start = std::max<int64_t>(start_line_num - 2, 0);
    int64_t p = ls;
    if (use_index) p = line_lo(code_start);
    else
      for (int64_t k = start_line_num; k > code_start; k--) p = line_start_of(p - 1);
    size_t kspan = first_span_after_f(p);  // every text below starts at or after p
    // the match line: the whole line when it is <= 100 B (then the cause line's text too);
    // kspan is at or below the first span ending after ls (p <= ls)
    const uint32_t ml_off = le - ls > 100 ? put_censored_from(kspan, mls, mle)
                                          : line_text(start_line_num, kspan, ls, le);
    const uint32_t ml_len = uint32_t(mle - mls);
    bool found_first = false;
    f.line_lo = uint32_t(ff.lines.size());
    if (!binary) {
      for (int64_t k = code_start; k < end_line_num + 2; k++) {
        int64_t e = use_index ? line_hi(k) : line_end_of(p);
        bool in_cause = k >= start_line_num && k <= end_line_num;
        uint32_t off, n;
        if (e - p > 100 && in_cause) {  // the match line (shared text)
          n = ml_len;
          off = ml_off;
        } else {
          const int64_t q = e - p > 100 ? p + 100 : e;
          n = uint32_t(q - p);
          while (kspan < spans.size() && spans[kspan].e <= p) kspan++;
          off = line_text(k, kspan, p, q);
        }
        ff.lines.push_back({k + 1, off, n, in_cause, !found_first && in_cause, false});
        found_first = found_first || in_cause;
        if (e >= len) break;  // last line of bytes.Split
        p = e + 1;
      }
    }
    f.line_hi = uint32_t(ff.lines.size());
    for (uint32_t li = f.line_hi; li > f.line_lo; li--)
      if (ff.lines[li - 1].is_cause) {
        ff.lines[li - 1].last_cause = true;
        break;
      }
    f.start_line = start_line_num + 1;
    f.end_line = end_line_num + 1;
    if (binary) {
      const std::string m = "Binary file " + GoQuote(std::string(path)) + " matches a rule " + GoQuote(rules_[f.rule].title);
      f.match_off = ff.Put(m);
      f.match_len = uint32_t(m.size());
    } else {
      f.match_off = ml_off;
      f.match_len = ml_len;
    }
    ff.f.push_back(f);
  }
  if (g_tail_debug) g_prof[14] += int64_t(ff.text.size());
  PhaseTimer pt4(4);
  SortFindings(&out->findings, rule_rank_);
}

void SecretScanner::GpuFindingsInput(const uint8_t* content, const Candidate* c, size_t nc, FileResult* out) const {
  ScanScratch& S = t_scan;
  // the anchors: (wlo, raw '\n' before wlo) of every candidate window of the file
  std::vector<std::pair<int64_t, int64_t>>& nla = S.nla;
  nla.clear();
  for (size_t i = 0; i < nc; i++) nla.push_back({c[i].wlo, c[i].nl_before});
  std::sort(nla.begin(), nla.end());
  // the censor spans, merged and sorted (as FindingsHost), each with the '\n'
  // inside the spans before it, then the sentinel
  std::vector<Loc>& spans = S.spans;
  spans.assign(S.censor.begin(), S.censor.end());
  std::sort(spans.begin(), spans.end(), [](const Loc& a, const Loc& b) { return a.s < b.s; });
  out->gs.clear();
  int64_t nl = 0;
  for (auto& z : spans) {
    if (z.e <= z.s) continue;
    if (!out->gs.empty() && z.s <= out->gs.back().e) {
      MatSpan& b = out->gs.back();
      if (z.e > b.e) {  // (the '\n' of the grown part)
        for (const uint8_t *p = content + b.e, *e = content + z.e; p < e;) {
          const void* q = std::memchr(p, '\n', size_t(e - p));
          if (!q) break;
          nl++;
          p = static_cast<const uint8_t*>(q) + 1;
        }
        b.e = z.e;
      }
      continue;
    }
    out->gs.push_back({z.s, z.e, nl});
    for (const uint8_t *p = content + z.s, *e = content + z.e; p < e;) {
      const void* q = std::memchr(p, '\n', size_t(e - p));
      if (!q) break;
      nl++;
      p = static_cast<const uint8_t*>(q) + 1;
    }
  }
  out->gs.push_back({INT64_MAX, INT64_MAX, nl});
  out->gm.clear();
  uint64_t tb = 0;
  for (auto& mt : S.matched) {
    const int64_t st = mt.second.s, en = mt.second.e;
    int64_t a_wlo = 0, a_nl = 0;
    auto it = std::upper_bound(nla.begin(), nla.end(), std::make_pair(st, INT64_MAX));
    if (it != nla.begin()) {
      --it;
      a_wlo = it->first;
      a_nl = it->second;
    }
    out->gm.push_back({mt.first, 0, st, en, a_wlo, a_nl});
    tb += uint64_t(std::max<int64_t>(100, en - st + 50)) + 400;  // match text + <= 4 lines of <= 100 B
  }
  out->text_bound = tb;
  out->gpu = true;
}

bool SecretScanner::Scan(const BatchInput& in, BatchResult* out, BatchStats* gst, HostStats* hst, std::string* err) {
  double t0 = NowMs();
  struct Active {
    std::atomic<int>& n;
    explicit Active(std::atomic<int>& c) : n(c) { n.fetch_add(1); }
    ~Active() { n.fetch_sub(1); }
  } active(active_scans_);
  HostStats hs;
  std::vector<Candidate> cands;
  uint64_t n_bytes = in.n_files ? in.host_offsets[in.n_files] : 0;
  if (engines_.empty()) {
    *err = "no GPU engine bound to this scanner";
    return false;
  }
  const size_t slot = size_t(next_slot_.fetch_add(1) % engines_.size());
  GpuEngine* engine = engines_[slot].get();
  // the allow-path pass needs no GPU result: it runs on host threads while
  // this thread drives the kernels
  std::vector<uint8_t> allowed;
  double ms_allow = 0;
  std::thread allow_thread([&] {
    pthread_setname_np(pthread_self(), "tsg-allow");
    double a0 = NowMs();
    allowed = AllowedPaths(in);
    ms_allow = NowMs() - a0;
  });
  bool ok;
  std::string gpu_err;
  TailOut tail;  // GPU pre-transform: the transformed bytes of the files with candidates
  if (in.transform && in.dev_arena) {
    allow_thread.join();
    *err = "a pre-transformed batch must be host-resident";
    return false;
  }
  GpuEngine::Ticket ticket;
  if (!in.dev_arena) {  // the staging ring orders concurrent host batches; it takes the lock per chunk
    ok = engine->RunHost(in.host_arena, n_bytes, in.host_offsets, in.n_files, &cands, gst, in.transform,
                         in.transform ? &tail : nullptr, &gpu_mu_[slot], &gpu_err, in.gather_base, in.gather_src);
  } else {
    std::lock_guard<std::mutex> g(gpu_mu_[slot]);
    static const bool tickets = !std::getenv("TSG_TICKETS") || std::atoi(std::getenv("TSG_TICKETS")) != 0;
    std::string enq_err;  // a failed Enqueue (no free ticket, or a HIP error) falls back to Run
    if (tickets && engine->Enqueue(in.dev_arena, n_bytes, in.dev_offsets, in.n_files, &ticket, &enq_err))
      ok = true;  // collected below, after the lock is released
    else
      ok = engine->Run(in.dev_arena, n_bytes, in.dev_offsets, in.n_files, &cands, gst);
    if (!ok && gpu_err.empty()) gpu_err = engine->error();
  }
  if (ticket.slot >= 0) {
    bool rerun = false;
    ok = engine->Collect(&ticket, &cands, gst, &rerun, &gpu_err);
    if (ok && rerun) {  // a buffer overflowed: grow and rescan synchronously
      std::lock_guard<std::mutex> g(gpu_mu_[slot]);
      ok = engine->Run(in.dev_arena, n_bytes, in.dev_offsets, in.n_files, &cands, gst);
      if (!ok) gpu_err = engine->error();  // read under the engine's lock
    }
  }
  allow_thread.join();
  if (!ok) {
    *err = gpu_err;
    return false;
  }
  BatchInput tin = in;  // the exact pass reads the transformed bytes
  std::vector<const uint8_t*> fdata;
  std::vector<uint64_t> flen;
  if (in.transform) {  // gathered files from tail.buf, identity-transformed ones in place
    fdata.assign(in.n_files, nullptr);
    flen.assign(in.n_files, 0);
    for (const Candidate& c : cands) {
      const uint32_t f = c.file;
      if (f >= in.n_files || fdata[f]) continue;
      if (tail.raw[f]) {  // as read: in the batch arena, or where the gather took it from
        fdata[f] = in.gather_base ? in.gather_base + in.gather_src[f] : in.host_arena + in.host_offsets[f];
        flen[f] = in.host_offsets[f + 1] - in.host_offsets[f];
      } else {
        fdata[f] = tail.buf.data() + tail.off[f];
        flen[f] = tail.off[f + 1] - tail.off[f];
      }
    }
    tin.file_data = fdata.data();
    tin.file_len = flen.data();
  }
  double t1 = NowMs();
  if (const char* dump = std::getenv("TSG_DUMP_CANDS")) {  // profiling aid (tools/host_tail_bench.py)
    if (FILE* fp = std::fopen(dump, "wb")) {
      if (!cands.empty()) std::fwrite(cands.data(), sizeof(Candidate), cands.size(), fp);
      std::fclose(fp);
    }
  }
  const double t_tail = NowMs();
  if (!HostTail(tin, &cands, out, &hs, &allowed, true, err)) return false;
  if (gst && gst->ms_total > 0) host_bound_.store(hs.ms_exact > 1.5 * double(gst->ms_total));
  static const bool times = std::getenv("TSG_TAIL_TIMES") != nullptr;
  if (times)
    std::fprintf(stderr, "scan times ms: to candidates %.2f, to the tail %.2f, tail %.2f (%zu candidates)\n", t1 - t0,
                 t_tail - t1, NowMs() - t_tail, cands.size());
  hs.ms_allow = ms_allow;  // overlapped with the GPU phase
  hs.ms_gpu = t1 - t0;
  hs.ms_total = NowMs() - t0;
  if (hst) *hst = hs;
  return true;
}

std::vector<uint8_t> SecretScanner::AllowedPaths(const BatchInput& in) const {
  // Global allow path (scanner.go:381-386) for every file
  std::vector<uint8_t> allowed(in.n_files, 0);
  bool any_path_rule = false;
  for (auto& a : allow_)
    if (a.path) any_path_rule = true;
  const bool dev = in.dev_paths && in.dev_path_off, host = in.host_paths && in.host_path_off;
  if (any_path_rule && path_filter_ && (dev || host)) {
    // the GPU reports the paths that can match; every other path is not allowed
    std::vector<PathHit> hits;
    std::string perr;
    if (dev ? path_filter_->Run(in.dev_paths, in.dev_path_off, in.n_files, &hits, &perr)
            : path_filter_->RunHost(in.host_paths, in.host_path_off, in.n_files, &hits, &perr)) {
      const size_t blocks = (hits.size() + 1023) / 1024;
      ParallelFor(blocks, host_threads_, [&](size_t b) {
        const size_t lo = b * 1024, hi = std::min<size_t>(lo + 1024, hits.size());
        for (size_t k = lo; k < hi; k++) {
          const uint32_t f = hits[k].file & ~kPathNonAscii;
          if (f >= in.n_files) continue;
          const char* p = in.paths[f];
          const size_t n = in.path_lens ? size_t(in.path_lens[f]) : std::strlen(p);
          const uint8_t* P = reinterpret_cast<const uint8_t*>(p);
          const bool a = (hits[k].file & kPathNonAscii) ? AllowPath(P, n) : AllowPathRules(P, n, hits[k].rules);
          allowed[f] = a ? 1 : 0;
        }
      });
      return allowed;
    }
    // a HIP error: fall through to the host pass (the scan itself reports GPU failures)
  }
  if (any_path_rule) {
    size_t blocks = (in.n_files + 4095) / 4096;
    ParallelFor(blocks, host_threads_, [&](size_t b) {
      size_t lo = b * 4096, hi = std::min<size_t>(lo + 4096, in.n_files);
      for (size_t f = lo; f < hi; f++) {
        const char* p = in.paths[f];
        size_t n = in.path_lens ? size_t(in.path_lens[f]) : std::strlen(p);
        allowed[f] = AllowPath(reinterpret_cast<const uint8_t*>(p), n) ? 1 : 0;
      }
    });
  }
  return allowed;
}

std::unique_ptr<SecretScanner::TailScratch> SecretScanner::TakeScratch() const {
  std::lock_guard<std::mutex> g(scratch_mu_);
  if (scratch_free_.empty()) return std::unique_ptr<TailScratch>(new TailScratch());
  std::unique_ptr<TailScratch> s = std::move(scratch_free_.back());
  scratch_free_.pop_back();
  return s;
}

void SecretScanner::GiveScratch(std::unique_ptr<TailScratch> s) const {
  std::lock_guard<std::mutex> g(scratch_mu_);
  if (scratch_free_.size() < 8) scratch_free_.push_back(std::move(s));  // (as many as scans run at once)
}

bool SecretScanner::HostTail(const BatchInput& in, std::vector<Candidate>* cands_p, BatchResult* out,
                             HostStats* hs, const std::vector<uint8_t>* allowed_pre, bool gpu_windows,
                             std::string* err) const {
  std::string err_local;
  if (!err) err = &err_local;
  std::vector<Candidate>& cands = *cands_p;
  out->found_files.clear();
  out->found.clear();
  out->arenas.clear();
  double t1 = NowMs();
  std::vector<uint8_t> allowed_local;
  if (!allowed_pre) allowed_local = AllowedPaths(in);
  const std::vector<uint8_t>& allowed = allowed_pre ? *allowed_pre : allowed_local;
  // every file's kind: kAllowedPath (1) where allowed (0 / 1 per file), else
  // kNoFindings (0) -- the allowed bytes themselves (a per-file loop was 0.6 ms
  // of serial time on C2's 791 k files)
  static_assert(kNoFindings == 0 && kAllowedPath == 1, "kind bytes are the allowed bytes");
  if (allowed.size() == in.n_files) out->kind.assign(allowed.begin(), allowed.end());
  else out->kind.assign(in.n_files, uint8_t(kNoFindings));
  double t2 = NowMs();
  if (g_tail_debug) std::fprintf(stderr, "tail setup ms: allow+kind %.1f\n", t2 - t1);
  // Group candidates by file: an LSD radix sort of (file, index) keys (11-bit
  // digits: the histograms stay in L1); each group's records are gathered and
  // put in (rule, wlo) order by the worker that scans it.  (A counting sort
  // over the file ids made two random passes over a 4-byte-per-file array --
  // 3 MB for C2's 791 k files -- and then moved every 64-B record, all of it
  // serial set-up before the parallel pass.)
  std::unique_ptr<TailScratch> scr = TakeScratch();
  std::vector<size_t>& starts = scr->starts;
  std::vector<uint64_t>& key = scr->key;
  starts.clear();
  {
    const size_t nc = cands.size();
    std::vector<uint64_t>& b = scr->key2;
    key.resize(nc);
    b.resize(nc);
    uint32_t max_file = 0;
    for (size_t i = 0; i < nc; i++) {
      key[i] = uint64_t(cands[i].file) << 32 | uint32_t(i);
      max_file = std::max(max_file, cands[i].file);
    }
    constexpr int kDigit = 11;
    // passes over the file bits only (32, 43, 54: the key is 64 bits wide), and
    // only as many as max_file needs; each shift count stays below the width of
    // what it shifts (a `max_file >> 33` / `key >> 65` wraps on x86 and the extra
    // pass would sort on candidate-index bits, splitting a file's group)
    for (int shift = 32; shift < 64; shift += kDigit) {
      if (shift > 32 && (uint64_t(max_file) >> (shift - 32)) == 0) break;
      uint32_t hist[(1 << kDigit) + 1] = {};
      for (size_t i = 0; i < nc; i++) hist[((key[i] >> shift) & ((1u << kDigit) - 1)) + 1]++;
      for (int d = 0; d < (1 << kDigit); d++) hist[d + 1] += hist[d];
      for (size_t i = 0; i < nc; i++) b[hist[(key[i] >> shift) & ((1u << kDigit) - 1)]++] = key[i];
      key.swap(b);
    }
    for (size_t i = 0; i < nc; i++)
      if (i == 0 || (key[i] >> 32) != (key[i - 1] >> 32)) starts.push_back(i);
    starts.push_back(nc);
  }
  auto group_file = [&](size_t k) { return uint32_t(key[starts[k]] >> 32); };
  auto group_cand = [&](size_t q) -> const Candidate& { return cands[uint32_t(key[q])]; };
  const double t_grouped = NowMs();
  size_t nf = starts.size() - 1;
  // (capacity and elements kept across calls: each group's kind is reset by its
  // worker and its findings replaced before use, so no clear / re-construction
  // of ~50 k results in the serial set-up)
  std::vector<FileResult>& tmp = scr->tmp;
  tmp.resize(nf);
  for (auto& g : g_prof) g = 0;
  const double t_sorted = NowMs();
  if (g_tail_debug) std::fprintf(stderr, "tail setup ms: group %.1f results %.1f\n", t_grouped - t2, t_sorted - t_grouped);
  // heaviest groups (candidates x file size) first so one big file does not
  // finish last; only the top few hundred need ordering, the rest follow in
  // file order
  std::vector<uint32_t>& order = scr->order;
  order.resize(nf);
  {
    std::vector<double>& w = scr->w;
    w.resize(nf);
    constexpr size_t kWBlock = 4096;  // (random reads of the file lengths: spread over the pool)
    ParallelFor((nf + kWBlock - 1) / kWBlock, host_threads_, [&](size_t blk) {
      for (size_t k = blk * kWBlock, e = std::min(nf, k + kWBlock); k < e; k++) {
        const uint32_t f = group_file(k);
        const uint64_t flen = in.file_data ? in.file_len[f] : in.host_offsets[f + 1] - in.host_offsets[f];
        w[k] = double(starts[k + 1] - starts[k]) * double(flen + 4096);
      }
    });
    const size_t top = std::min<size_t>(nf, 1024);  // the LPT head, dispatched one group at a time below
    auto heavier = [&](uint32_t x, uint32_t y) { return w[x] > w[y] || (w[x] == w[y] && x < y); };
    if (top < nf) {
      // the top groups by weight (ties: lower index), the rest in file order: one selection
      // on a copy of the weights for the threshold, then a linear pass (no sort of the rest)
      std::vector<double> wc(w.begin(), w.end());
      std::nth_element(wc.begin(), wc.begin() + (top - 1), wc.end(), std::greater<double>());
      const double thr = wc[top - 1];
      size_t above = 0;
      for (size_t k = 0; k < nf; k++) above += w[k] > thr;
      size_t eq_take = top - above, h = 0, r = top;  // ties at the threshold: the lowest indices join the head
      for (size_t k = 0; k < nf; k++) {
        const bool head = w[k] > thr || (w[k] == thr && eq_take > 0 && (eq_take--, true));
        if (head) order[h++] = uint32_t(k);
        else order[r++] = uint32_t(k);
      }
    } else {
      for (size_t k = 0; k < nf; k++) order[k] = uint32_t(k);
    }
    std::sort(order.begin(), order.begin() + top, heavier);
  }
  const double t_ordered = NowMs();
  // The tail is bound by cold reads of the arena (the match window, the lines
  // around it, the path): past the heaviest groups, items go out in runs of
  // kRun and each one prefetches the next item's windows while it scans.
  constexpr size_t kRun = 4;
  const size_t top = std::min<size_t>(nf, 1024);
  const size_t n_items = top + (nf - top + kRun - 1) / kRun;
  auto prefetch_group = [&](size_t k) {
    const size_t a = starts[k], b = starts[k + 1];
    const uint32_t f = group_file(k);
    if (allowed[f]) return;
    __builtin_prefetch(in.paths[f]);
    const uint8_t* data = in.file_data ? in.file_data[f] : in.host_arena + in.host_offsets[f];
    const int64_t len = int64_t(in.file_data ? in.file_len[f] : in.host_offsets[f + 1] - in.host_offsets[f]);
    for (size_t q = a; q < b && q < a + 4; q++) {
      const Candidate& c = group_cand(q);
      const int64_t lo = std::max<int64_t>(0, c.wlo - 256);
      const int64_t hi = std::min<int64_t>(len, std::min(c.whi, c.wlo + 2048) + 512);
      for (int64_t x = lo & ~int64_t(63); x < hi; x += 64) __builtin_prefetch(data + x);
    }
  };
  // one findings arena per host thread of this pass (handed to the result)
  std::mutex arena_mu;
  static std::atomic<uint64_t> pass_serial{0};
  const uint64_t serial = ++pass_serial;
  auto thread_arena = [&]() -> ResultArena* {
    thread_local uint64_t t_serial = 0;
    thread_local ResultArena* t_arena = nullptr;
    if (t_serial != serial) {
      std::unique_ptr<ResultArena> a(new ResultArena());
      t_arena = a.get();
      t_serial = serial;
      std::lock_guard<std::mutex> g(arena_mu);
      out->arenas.push_back(std::move(a));
    }
    return t_arena;
  };
  // toFinding / findLocation on the GPU (materialize.h) when the arena is resident in HBM
  // (auto: when the last scan's exact pass outlasted 1.5x its GPU phase -- finding-dense batches, C3f:
  // the GPU pass costs GPU time beside the next scans' kernels, which a GPU-bound pipeline (C2) pays)
  const int gf_mode = gpu_findings_.load();
  const bool gpu_mat = mat_ && gpu_windows && (gf_mode == 1 || (gf_mode == 2 && host_bound_.load())) &&
                       in.dev_arena && in.dev_offsets && !in.file_data;
  auto scan_group = [&](size_t k) {
    const size_t a = starts[k], b = starts[k + 1];
    const uint32_t f = group_file(k);
    tmp[k].kind = kNoFindings;
    tmp[k].gpu = false;
    if (allowed[f]) {
      // no stale FileFindings from an earlier pass (its arena belongs to a result
      // that may be gone) stays behind in the reused scratch
      tmp[k].findings = FileFindings(nullptr);
      return;
    }
    tmp[k].findings = FileFindings(thread_arena());
    thread_local std::vector<Candidate> t_group;  // this group's records, gathered
    t_group.clear();
    for (size_t q = a; q < b; q++) t_group.push_back(group_cand(q));
    if (b - a > 1) {
      auto by_rule = [](const Candidate& x, const Candidate& y) {
        return x.rule != y.rule ? x.rule < y.rule : x.wlo < y.wlo;
      };
      if (!std::is_sorted(t_group.begin(), t_group.end(), by_rule)) std::sort(t_group.begin(), t_group.end(), by_rule);
    }
    const char* p = in.paths[f];
    size_t pn = in.path_lens ? size_t(in.path_lens[f]) : std::strlen(p);
    const uint8_t* data = in.file_data ? in.file_data[f] : in.host_arena + in.host_offsets[f];
    const int64_t len = int64_t(in.file_data ? in.file_len[f] : in.host_offsets[f + 1] - in.host_offsets[f]);
    const bool bin = in.binary && in.binary[f];
    if (!gpu_mat) {
      ScanFile(data, len, std::string_view(p, pn), bin, t_group.data(), t_group.size(), &tmp[k], gpu_windows);
      return;
    }
    PhaseTimer pt_all(7);
    MatchFile(data, len, std::string_view(p, pn), t_group.data(), t_group.size(), gpu_windows);
    if (t_scan.matched.empty()) return;
    if (bin) {  // (Code{}, Match from the path and title: nothing for the GPU)
      FindingsHost(data, len, std::string_view(p, pn), bin, t_group.data(), t_group.size(), &tmp[k]);
      return;
    }
    GpuFindingsInput(data, t_group.data(), t_group.size(), &tmp[k]);
  };
  // no other scan in flight (the end of a run): the pool's spare workers join in,
  // the last scan's exact pass being all that is left (TSG_DRAIN_WIDE=0: never;
  // TSG_TAIL_WIDE=1: every exact pass)
  static const bool drain_wide = !std::getenv("TSG_DRAIN_WIDE") || std::atoi(std::getenv("TSG_DRAIN_WIDE")) != 0;
  static const bool tail_wide = std::getenv("TSG_TAIL_WIDE") && std::atoi(std::getenv("TSG_TAIL_WIDE")) != 0;
  // host-bound batches (the last exact pass outlasted 1.5x its GPU phase, e.g.
  // finding-dense C3f: 40 vs 9 ms) take them too (TSG_TAIL_ADAPT=0: never)
  static const bool adapt = !std::getenv("TSG_TAIL_ADAPT") || std::atoi(std::getenv("TSG_TAIL_ADAPT")) != 0;
  const bool wide = tail_wide || (drain_wide && active_scans_.load() <= 1) || (adapt && host_bound_.load());
  ParallelFor(n_items, host_threads_, [&](size_t it) {
    if (it < top) {
      scan_group(order[it]);
      return;
    }
    const size_t kk0 = top + (it - top) * kRun, kk1 = std::min(nf, kk0 + kRun);
    prefetch_group(order[kk0]);
    for (size_t kk = kk0; kk < kk1; kk++) {
      if (kk + 1 < kk1) prefetch_group(order[kk + 1]);
      scan_group(order[kk]);
    }
  }, wide);
  const double t_par0 = NowMs();
  double ms_mat_gpu = 0;
  if (gpu_mat && !GpuFindings(in, scr.get(), nf, [&](size_t k) { return group_file(k); }, thread_arena, wide,
                              &ms_mat_gpu, err)) {
    GiveScratch(std::move(scr));
    return false;
  }
  const double t_par = NowMs();
  if (g_tail_debug)
    std::fprintf(stderr, "tail serial ms: sort+setup %.1f (order %.1f) parallel %.1f\n", t_sorted - t2,
                 t_ordered - t_sorted, t_par - t_sorted);
  if (g_tail_debug)
    std::fprintf(stderr, "tail phases ms: findall %.1f gate %.1f blocks %.1f findings %.1f sort %.1f allow-loc %.1f go %.1f "
                 "scanfile %.1f (newline index %.1f)\n",
                 g_prof[0] / 1e6, g_prof[1] / 1e6, g_prof[2] / 1e6, g_prof[3] / 1e6, g_prof[4] / 1e6,
                 g_prof[5] / 1e6, g_prof[6] / 1e6, g_prof[7] / 1e6, g_prof[15] / 1e6);
  if (g_tail_debug)
    std::fprintf(stderr, "tail findings: %lld with the newline index, %lld by walks; censor spans %lld; text %.1f MB\n",
                 (long long)g_prof[11].load(), (long long)g_prof[12].load(), (long long)g_prof[13].load(),
                 g_prof[14] / 1e6);
  if (g_tail_debug) {
    std::vector<std::pair<int64_t, uint32_t>> top;
    for (uint32_t r = 0; r < std::min<uint32_t>(kRuleProf, uint32_t(rules_.size())); r++)
      if (g_rule_ns[r]) top.push_back({g_rule_ns[r].load(), r});
    std::sort(top.rbegin(), top.rend());
    for (size_t k = 0; k < top.size() && k < 8; k++)
      std::fprintf(stderr, "tail findall by rule: %-32s %.1f ms %lld calls\n", rules_[top[k].second].id.c_str(),
                   top[k].first / 1e6, (long long)g_rule_calls[top[k].second].load());
    for (uint32_t r = 0; r < kRuleProf; r++) g_rule_ns[r] = 0, g_rule_calls[r] = 0;
  }
  if (g_tail_debug)
    std::fprintf(stderr, "tail whole-content gate scans: %lld calls, %.1f MB; line walks: %.1f MB forward, %.1f MB back"
                 " (%.1f MB inside windows)\n", (long long)g_wholefile_calls.load(), g_wholefile_bytes.load() / 1e6,
                 g_prof[8] / 1e6, (g_prof[9] + g_prof[10]) / 1e6, g_prof[10] / 1e6);
  // the files with findings, in file order: positions by one pass, then the
  // findings moved into place in parallel
  std::vector<uint32_t>& at = scr->order;  // (the dispatch order is no longer needed)
  at.resize(nf);
  size_t n_found = 0;
  for (size_t k = 0; k < nf; k++) {
    at[k] = uint32_t(n_found);
    n_found += tmp[k].kind == kHasFindings;
  }
  out->found_files.resize(n_found);
  out->found.allocate(n_found);
  constexpr size_t kMoveBlock = 2048;
  ParallelFor((nf + kMoveBlock - 1) / kMoveBlock, host_threads_, [&](size_t blk) {
    for (size_t k = blk * kMoveBlock, e = std::min(nf, k + kMoveBlock); k < e; k++) {
      if (tmp[k].kind != kHasFindings) continue;
      const uint32_t f = group_file(k);
      out->kind[f] = uint8_t(kHasFindings);
      out->found_files[at[k]] = f;
      out->found.emplace(at[k], std::move(tmp[k].findings));
    }
  }, wide);
  double t3 = NowMs();
  if (g_tail_debug) std::fprintf(stderr, "tail serial ms: collect %.1f\n", t3 - t_par);
  static const bool times = std::getenv("TSG_TAIL_TIMES") != nullptr;  // one line per pass, no per-file timers
  if (times)
    std::fprintf(stderr, "tail times ms: kind %.2f group %.2f results %.2f order %.2f parallel %.2f (gpu findings %.2f, "
                 "of which GPU %.2f) collect %.2f (files %zu, wide %d)\n", t2 - t1, t_grouped - t2, t_sorted - t_grouped,
                 t_ordered - t_sorted, t_par0 - t_ordered, t_par - t_par0, ms_mat_gpu, t3 - t_par, nf, int(wide));
  GiveScratch(std::move(scr));
  hs->ms_allow = t2 - t1;
  hs->ms_exact = t3 - t2;
  hs->candidates = cands.size();
  hs->files_with_candidates = nf;
  hs->findings = out->n_findings();
  return true;
}

template <class GroupFile, class ArenaOf>
bool SecretScanner::GpuFindings(const BatchInput& in, TailScratch* scr, size_t nf, GroupFile group_file,
                                ArenaOf& thread_arena, bool wide, double* ms_gpu, std::string* err) const {
  std::vector<FileResult>& tmp = scr->tmp;
  std::vector<uint32_t>& gk = scr->gk;  // groups whose findings the GPU makes, in file order
  gk.clear();
  for (size_t k = 0; k < nf; k++)
    if (tmp[k].gpu) gk.push_back(uint32_t(k));
  // calls of bounded size: the text offsets of one call are 32-bit
  constexpr uint64_t kTextCap = uint64_t(1) << 31, kMatchCap = uint64_t(1) << 26;
  std::vector<uint64_t>& m0 = scr->gm0;
  std::vector<uint64_t>& s0 = scr->gs0;
  size_t a = 0;
  while (a < gk.size()) {
    size_t b = a;
    uint64_t nm = 0, ns = 0, tb = 0;
    m0.clear();
    s0.clear();
    while (b < gk.size()) {
      const FileResult& R = tmp[gk[b]];
      if (b > a && (nm + R.gm.size() > kMatchCap || tb + R.text_bound > kTextCap)) break;
      m0.push_back(nm);
      s0.push_back(ns);
      nm += R.gm.size();
      ns += R.gs.size();
      tb += R.text_bound;
      b++;
    }
    if (tb > kTextCap || nm > kMatchCap) {
      *err = "GPU findings: one file's findings exceed a call's bounds";
      return false;
    }
    const double f0 = NowMs();
    FindingMaterializer::Job* job = mat_->Begin(uint32_t(b - a), uint32_t(nm), uint32_t(ns), tb, err);
    if (!job) return false;
    MatFile* F = mat_->files(job);
    MatMatch* M = mat_->matches(job);
    MatSpan* Sp = mat_->spans(job);
    constexpr size_t kBlk = 256;
    const size_t n = b - a;
    ParallelFor((n + kBlk - 1) / kBlk, host_threads_, [&](size_t blk) {
      for (size_t i = blk * kBlk, e = std::min(n, i + kBlk); i < e; i++) {
        const FileResult& R = tmp[gk[a + i]];
        F[i] = MatFile{group_file(gk[a + i]), uint32_t(m0[i]), uint32_t(R.gm.size()), uint32_t(s0[i]),
                       uint32_t(R.gs.size()), 0};
        MatMatch* mo = M + m0[i];
        for (size_t q = 0; q < R.gm.size(); q++) {
          mo[q] = R.gm[q];
          mo[q].fidx = uint32_t(i);
        }
        std::memcpy(Sp + s0[i], R.gs.data(), R.gs.size() * sizeof(MatSpan));
      }
    }, wide);
    const double g0 = NowMs();
    if (!mat_->Run(job, in.dev_arena, in.dev_offsets, err)) {
      mat_->End(job);
      return false;
    }
    const double g1 = NowMs();
    *ms_gpu += g1 - g0;
    const FindingOut* fo = mat_->findings(job);
    const LineOut* lo = mat_->lines(job);
    const char* tx = mat_->text(job);
    const uint64_t* pref = mat_->pref(job);
    // the files with the most findings first, one per item (each is a pdqsort of
    // its findings on one thread: a multi-MiB file with tens of thousands of them
    // dispatched late set the pass's length), the rest in blocks
    std::vector<uint32_t>& ord = scr->gord;
    ord.resize(n);
    for (size_t i = 0; i < n; i++) ord[i] = uint32_t(i);
    const size_t head = std::min<size_t>(n, 256);
    auto heavier = [&](uint32_t x, uint32_t y) {
      const size_t cx = tmp[gk[a + x]].gm.size(), cy = tmp[gk[a + y]].gm.size();
      return cx != cy ? cx > cy : x < y;
    };
    if (head < n) std::nth_element(ord.begin(), ord.begin() + long(head), ord.end(), heavier);
    std::sort(ord.begin(), ord.begin() + long(head), heavier);
    if (head < n) std::sort(ord.begin() + long(head), ord.end());  // the rest in file order
    // a wide pass (the pipeline's last scan: the pool is otherwise idle) sorts the
    // heaviest files first, each by all the threads (SortFindingsParallel): one of
    // ~50 k findings alone is an ~8-ms pdqsort.  Beside other scans' passes the
    // threads are taken, and that costs more than it saves (C3f at depth 6: the
    // four heavy files 13-17 ms vs 8 ms as single items beside the rest)
    size_t heavy = 0;
    static const size_t kHeavy = [] {
      const char* e = std::getenv("TSG_SORT_PAR_MIN");
      return e ? size_t(std::strtoull(e, nullptr, 10)) : size_t(16384);
    }();
    while (wide && heavy < head && heavy < 8 && tmp[gk[a + ord[heavy]]].gm.size() >= kHeavy) {
      const size_t i = ord[heavy];
      FileResult& R = tmp[gk[a + i]];
      const size_t x = m0[i], y = x + R.gm.size();
      const uint64_t p0 = pref[x], p1 = pref[y];
      FileFindings& ff = R.findings;
      ff = FileFindings(thread_arena());
      ff.f.assign(fo + x, fo + y);
      ff.lines.assign(lo + uint32_t(p0), lo + uint32_t(p1));
      ff.text.assign(tx + (p0 >> 32), tx + (p1 >> 32));
      SortFindingsParallel(&ff, rule_rank_, host_threads_, wide);
      R.kind = kHasFindings;
      heavy++;
    }
    const double h1 = NowMs();
    constexpr size_t kBlk2 = 64;
    const size_t n_items = head + (n - head + kBlk2 - 1) / kBlk2;
    static const bool times = std::getenv("TSG_TAIL_TIMES") != nullptr;
    std::atomic<uint64_t> us_copy{0}, us_sort{0}, us_max{0};  // (TSG_TAIL_TIMES)
    ParallelFor(n_items, host_threads_, [&](size_t it) {
      if (it < heavy) return;  // (sorted above)
      const size_t lo_i = it < head ? it : head + (it - head) * kBlk2;
      const size_t hi_i = it < head ? it + 1 : std::min(n, lo_i + kBlk2);
      double c_ms = 0, s_ms = 0;
      for (size_t oi = lo_i; oi < hi_i; oi++) {
        const size_t i = ord[oi];
        FileResult& R = tmp[gk[a + i]];
        const size_t x = m0[i], y = x + R.gm.size();
        const uint64_t p0 = pref[x], p1 = pref[y];
        const double t0 = times ? NowMs() : 0;
        FileFindings& ff = R.findings;
        ff = FileFindings(thread_arena());
        ff.f.assign(fo + x, fo + y);
        ff.lines.assign(lo + uint32_t(p0), lo + uint32_t(p1));
        ff.text.assign(tx + (p0 >> 32), tx + (p1 >> 32));
        const double t1 = times ? NowMs() : 0;
        SortFindings(&ff, rule_rank_);
        R.kind = kHasFindings;
        if (times) {
          const double t2 = NowMs();
          c_ms += t1 - t0;
          s_ms += t2 - t1;
        }
      }
      if (times) {
        us_copy += uint64_t(c_ms * 1e3);
        us_sort += uint64_t(s_ms * 1e3);
        const uint64_t tot = uint64_t((c_ms + s_ms) * 1e3);
        uint64_t m = us_max.load();
        while (tot > m && !us_max.compare_exchange_weak(m, tot)) {
        }
      }
    }, wide);
    mat_->End(job);
    if (times)
      std::fprintf(stderr, "gpu findings ms: slot+fill %.2f gpu %.2f assemble+sort %.2f (files %zu, findings %llu, "
                   "spans %llu; heavy files %zu in %.2f; thread-ms copy %.2f sort %.2f, longest item %.2f; lines %u "
                   "text %.1f MB)\n",
                   g0 - f0, g1 - g0, NowMs() - g1, b - a, (unsigned long long)nm, (unsigned long long)ns, heavy, h1 - g1,
                   us_copy.load() * 1e-3, us_sort.load() * 1e-3, us_max.load() * 1e-3, uint32_t(pref[nm]),
                   double(pref[nm] >> 32) * 1e-6);
    a = b;
  }
  return true;
}

}  // namespace tsg
