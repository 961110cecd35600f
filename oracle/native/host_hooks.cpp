// TEST INFRASTRUCTURE (oracle/native/tsg_oracle.h), linked with the product's
// host sources into oracle/build/libtsg_host.so -- never into libtsg.so.
//
//  * tsg_debug_host_tail[_cands]: the product's exact host tail (scanner.cpp,
//    SecretScanner::HostTail) over whole-file / given candidate windows, so the
//    CPU suite can check it against the Python oracle without a GPU;
//  * tsg_debug_scanner_host_only: a scanner without a GPU engine;
//  * tsg_cpuref_scan: the reference CPU algorithm restated in C++, the bench's
//    CPU baseline.  pkg/fanal/secret/scanner.go:377-463 per file: global
//    AllowPath (:381), then per rule MatchPath (:397), AllowPath (:403),
//    MatchKeywords (:409 -> :174-186: bytes.ToLower of the WHOLE content for
//    every rule with keywords, then bytes.Contains per lowered keyword), and
//    for the rules that pass, FindLocations over the whole file (:414 ->
//    :102-148) and the unchanged tail (allow / exclude / censor / findings /
//    sort) -- the exact tail is the product's, fed whole-file windows.
#include <cstring>
#include <memory>
#include <string>
#include <vector>
#include <thread>
#include <chrono>
#include <atomic>

#include "capi_internal.h"
#include "goregex.h"
#include "parallel.h"
#include "tsg_oracle.h"

namespace {

std::unique_ptr<tsg::SecretScanner> HostScanner(const tsg_global* g, std::string* err) {
  std::vector<tsg::RuleSpec> rules;
  std::vector<tsg::AllowRuleSpec> allow;
  std::vector<std::unique_ptr<tsg::Regex>> exclude;
  if (!tsg::MakeRules(g, &rules, err) || !tsg::MakeAllow(g->allow_rules, g->n_allow_rules, &allow, err) ||
      !tsg::MakeExclude(g->exclude_regexes, g->n_exclude_regexes, &exclude, err))
    return nullptr;
  std::unique_ptr<tsg::SecretScanner> sc(
      new tsg::SecretScanner(std::move(rules), std::move(allow), std::move(exclude), -1, err));
  if (!sc->ok()) {
    if (err->empty()) *err = sc->error();
    return nullptr;
  }
  return sc;
}

tsg::BatchInput Input(const tsg_batch* b) {
  tsg::BatchInput in;
  in.n_files = b->n_files;
  in.host_arena = b->host_arena;
  in.host_offsets = b->host_offsets;
  in.paths = b->paths;
  in.path_lens = b->path_lens;
  in.binary = b->binary;
  return in;
}

int Tail(std::unique_ptr<tsg::SecretScanner> sc, const tsg_batch* b, std::vector<tsg::Candidate>* cands,
         tsg_result** out) {
  const tsg::BatchInput in = Input(b);
  std::unique_ptr<tsg_result> r(new tsg_result());
  tsg::HostStats hs;
  // TSG_TAIL_REPS=n: the tail n times on copies of the candidates (profiling:
  // the samples then come from the tail, not from compiling the rules)
  for (int rep = std::getenv("TSG_TAIL_REPS") ? std::atoi(std::getenv("TSG_TAIL_REPS")) : 1; rep > 1; rep--) {
    std::vector<tsg::Candidate> cc(*cands);
    tsg::BatchResult tmp;
    sc->HostTail(in, &cc, &tmp, &hs);
  }
  sc->HostTail(in, cands, &r->files, &hs);
  std::memset(&r->stats, 0, sizeof(r->stats));
  r->stats.bytes = in.n_files ? in.host_offsets[in.n_files] : 0;
  r->stats.files = in.n_files;
  r->stats.findings = hs.findings;
  r->stats.candidates = hs.candidates;
  r->stats.ms_host_allow_path = hs.ms_allow;
  r->stats.ms_host_exact = hs.ms_exact;
  r->owner = sc.get();
  r->owned = std::move(sc);
  *out = r.release();
  return 0;
}

}  // namespace

extern "C" {

int tsg_debug_scanner_host_only(const tsg_global* g, tsg_scanner** out) {
  std::string err;
  auto sc = HostScanner(g, &err);
  if (!sc) {
    tsg::SetError(err);
    return -1;
  }
  std::unique_ptr<tsg_scanner> s(new tsg_scanner());
  s->s = std::move(sc);
  *out = s.release();
  return 0;
}

// Every (file, rule with a regex) with the whole file as its window: the
// tail's lazy keyword gate decides, as it does for GPU candidates.
int tsg_debug_host_tail(const tsg_global* g, const tsg_batch* b, tsg_result** out) {
  std::string err;
  auto sc = HostScanner(g, &err);
  if (!sc) {
    tsg::SetError(err);
    return -1;
  }
  std::vector<tsg::Candidate> cands;
  for (uint32_t f = 0; f < b->n_files; f++) {
    const uint64_t fs = b->host_offsets[f], fe = b->host_offsets[f + 1];
    for (uint32_t r = 0; r < sc->rules().size(); r++)
      if (sc->compiled().regex[r])
        cands.push_back(tsg::HostCandidate(f, r, 0, int64_t(fe - fs), 0, 0));
  }
  return Tail(std::move(sc), b, &cands, out);
}

int tsg_debug_host_tail_cands(const tsg_global* g, const tsg_batch* b, const void* cands, uint64_t n_cands,
                              tsg_result** out) {
  std::string err;
  auto sc = HostScanner(g, &err);
  if (!sc) {
    tsg::SetError(err);
    return -1;
  }
  std::vector<tsg::Candidate> cv(n_cands);
  if (n_cands) std::memcpy(cv.data(), cands, n_cands * sizeof(tsg::Candidate));
  for (const auto& c : cv)
    if (c.file >= b->n_files || c.rule >= sc->rules().size()) {
      tsg::SetError("candidate out of range");
      return -3;
    }
  return Tail(std::move(sc), b, &cv, out);
}

int tsg_cpuref_scan(const tsg_global* g, const tsg_batch* b, int threads, tsg_result** out) {
  std::string err;
  auto sc = HostScanner(g, &err);
  if (!sc) {
    tsg::SetError(err);
    return -1;
  }
  if (threads < 1) threads = 1;
  sc->set_host_threads(threads);
  const auto& rules = sc->rules();
  std::vector<std::vector<tsg::Candidate>> per_file(b->n_files);
  tsg::ParallelFor(b->n_files, threads, [&](size_t f) {
    const uint8_t* content = b->host_arena + b->host_offsets[f];
    const size_t len = size_t(b->host_offsets[f + 1] - b->host_offsets[f]);
    const char* p = b->paths[f];
    const size_t pn = b->path_lens ? size_t(b->path_lens[f]) : std::strlen(p);
    const uint8_t* P = reinterpret_cast<const uint8_t*>(p);
    if (sc->AllowPath(P, pn)) return;  // scanner.go:381 (the tail reports Secret{FilePath})
    for (uint32_t r = 0; r < rules.size(); r++) {
      const tsg::RuleSpec& R = rules[r];
      if (R.path && !R.path->Match(P, pn)) continue;  // MatchPath :397
      bool allowed = false;                            // AllowPath :403
      for (auto& a : R.allow_rules)
        if (a.path && a.path->Match(P, pn)) allowed = true;
      if (allowed) continue;
      if (!R.keywords.empty()) {  // MatchKeywords :174-186, lowering the whole content per rule
        const std::string lowered = tsg::GoBytesToLower(content, len);
        bool hit = false;
        for (auto& kw : R.kw_lower_host)
          if (lowered.find(kw) != std::string::npos) {
            hit = true;
            break;
          }
        if (!hit) continue;
      }
      if (!sc->compiled().regex[r]) continue;  // FindLocations: r.Regex == nil -> nil (:103)
      per_file[f].push_back(
          tsg::HostCandidate(uint32_t(f), r, 0, int64_t(len), 0, tsg::kCandGateValid | tsg::kCandGateOpen));
    }
  });
  std::vector<tsg::Candidate> cands;
  for (auto& v : per_file) cands.insert(cands.end(), v.begin(), v.end());
  return Tail(std::move(sc), b, &cands, out);
}

int tsg_debug_pool_peak(int callers, uint64_t n, int item_us, int wide, int* steady, int* workers) {
  std::atomic<int> in{0}, peak{0};
  std::vector<std::thread> ts;
  for (int k = 0; k < callers; k++)
    ts.emplace_back([&] {
      tsg::ParallelFor(size_t(n), 1 << 20, [&](size_t) {
        const int now = in.fetch_add(1) + 1;
        int p = peak.load();
        while (now > p && !peak.compare_exchange_weak(p, now)) {
        }
        std::this_thread::sleep_for(std::chrono::microseconds(item_us));
        in.fetch_sub(1);
      }, wide != 0);
    });
  for (auto& t : ts) t.join();
  *steady = tsg::HostPool::Get().steady();
  *workers = tsg::HostPool::Get().workers();
  return peak.load();
}

int tsg_debug_sort_findings(uint32_t n, const uint32_t* rule, const uint32_t* rule_rank, uint32_t n_rules,
                            const char* text, uint64_t text_len, const uint32_t* match_off, const uint32_t* match_len,
                            int threads, uint32_t* out_order) {
  tsg::FileFindings ff;
  ff.text.assign(text, size_t(text_len));
  ff.f.resize(n);
  for (uint32_t i = 0; i < n; i++) {
    ff.f[i] = tsg::FindingOut{};
    ff.f[i].rule = rule[i];
    ff.f[i].start_line = int64_t(i);  // the original position, read back as the permutation
    ff.f[i].match_off = match_off[i];
    ff.f[i].match_len = match_len[i];
  }
  const std::vector<uint32_t> rank(rule_rank, rule_rank + n_rules);
  if (threads > 0) tsg::SortFindingsParallel(&ff, rank, threads, false);
  else tsg::SortFindings(&ff, rank);
  for (uint32_t i = 0; i < n; i++) out_order[i] = uint32_t(ff.f[i].start_line);
  return 0;
}

}  // extern "C"
