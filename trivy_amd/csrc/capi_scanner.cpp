// C ABI of the drop-in scanner (include/tsg_scanner.h) and of the rule
// compiler inspection hooks (include/tsg_debug.h).
#include <pthread.h>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <memory>
#include <string>

#include "capi_internal.h"
#include "filter.h"
#include "scanner.h"
#include "tsg_debug.h"
#include "tsg_scanner.h"

struct tsg_compiled {
  tsg::CompiledRules cr;
};

namespace {
// Results are destroyed on a background thread: a batch's findings are
// thousands of small heap blocks written by the tail's worker threads, and
// freeing them would otherwise sit on the caller's critical path.
class ResultReaper {
 public:
  static ResultReaper& Get() {
    static ResultReaper r;
    return r;
  }
  void Push(tsg_result* r) {
    if (!r) return;
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(r);
    }
    cv_.notify_one();
  }
  ~ResultReaper() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_one();
    if (th_.joinable()) th_.join();
  }

 private:
  ResultReaper() : th_([this] { Run(); }) {}
  void Run() {
    pthread_setname_np(pthread_self(), "tsg-reaper");
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      while (!q_.empty()) {
        tsg_result* r = q_.front();
        q_.pop_front();
        lk.unlock();
        delete r;
        lk.lock();
      }
      if (stop_) return;
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<tsg_result*> q_;
  bool stop_ = false;
  std::thread th_;
};
}  // namespace

namespace {
std::string Str(const char* s) { return s ? std::string(s) : std::string(); }
}  // namespace

namespace tsg {

// NULL = no regex; "" is a regex that matches everywhere (Go compiles it,
// Regexp.UnmarshalYAML, scanner.go:75-87).
bool MakeMatcher(const char* src, std::unique_ptr<tsg::Matcher>* out, std::string* err) {
  if (!src) return true;
  auto re = tsg::Regex::Compile(src, err);
  if (!re) return false;
  out->reset(new tsg::Matcher());
  (*out)->lits = tsg::RequiredLiterals(*re);
  (*out)->re = std::move(re);
  tsg::Matcher& m = **out;
  m.simple = tsg::SimpleLiteral(src, &m.simple_lits, &m.simple_begin, &m.simple_end);
  return true;
}

bool MakeAllow(const tsg_allow_rule* a, uint32_t n, std::vector<tsg::AllowRuleSpec>* out, std::string* err) {
  for (uint32_t i = 0; i < n; i++) {
    tsg::AllowRuleSpec s;
    s.id = Str(a[i].id);
    if (!MakeMatcher(a[i].regex, &s.regex, err) || !MakeMatcher(a[i].path, &s.path, err)) return false;
    out->push_back(std::move(s));
  }
  return true;
}

bool MakeExclude(const char* const* rx, uint32_t n, std::vector<std::unique_ptr<tsg::Regex>>* out,
                 std::string* err) {
  for (uint32_t i = 0; i < n; i++) {
    auto re = tsg::Regex::Compile(Str(rx[i]), err);
    if (!re) return false;
    out->push_back(std::move(re));
  }
  return true;
}

bool MakeRules(const tsg_global* g, std::vector<tsg::RuleSpec>* rules, std::string* err) {
  for (uint32_t i = 0; i < g->n_rules; i++) {
    const tsg_rule& r = g->rules[i];
    tsg::RuleSpec s;
    s.id = Str(r.id);
    s.category = Str(r.category);
    s.title = Str(r.title);
    s.severity = Str(r.severity);
    s.secret_group_name = Str(r.secret_group_name);
    s.regex_src = Str(r.regex);
    s.has_regex = r.regex != nullptr;
    for (uint32_t k = 0; k < r.n_keywords; k++) s.keywords.push_back(Str(r.keywords[k]));
    if (!MakeMatcher(r.path, &s.path, err)) return false;
    if (!MakeAllow(r.allow_rules, r.n_allow_rules, &s.allow_rules, err)) return false;
    if (!MakeExclude(r.exclude_regexes, r.n_exclude_regexes, &s.exclude, err)) return false;
    rules->push_back(std::move(s));
  }
  return true;
}

}  // namespace tsg

namespace {
using tsg::MakeAllow;
using tsg::MakeExclude;
using tsg::MakeRules;

void JsonStr(std::string* o, const std::string& s) {
  static const char* hex = "0123456789abcdef";
  o->push_back('"');
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o->push_back('\\');
      o->push_back(char(c));
    } else if (c < 0x20) {
      *o += "\\u00";
      o->push_back(hex[c >> 4]);
      o->push_back(hex[c & 15]);
    } else if (c >= 0x80) {
      // raw bytes are carried as \u00XX escapes of latin-1 code points so that
      // non-UTF-8 content survives; the Python side re-encodes as latin-1.
      *o += "\\u00";
      o->push_back(hex[c >> 4]);
      o->push_back(hex[c & 15]);
    } else {
      o->push_back(char(c));
    }
  }
  o->push_back('"');
}
}  // namespace

extern "C" {

namespace {
bool CompileOpts(const tsg_compile_options* o, tsg::CompileOptions* co) {
  if (!o) return true;
  if (o->struct_size != TSG_COMPILE_OPTIONS_SIZE_V1) {
    tsg::SetError("tsg_compile_options.struct_size " + std::to_string(o->struct_size) +
                  " is not a size this library knows (v1 = " + std::to_string(TSG_COMPILE_OPTIONS_SIZE_V1) + ")");
    return false;
  }
  co->calib = o->calib;
  co->calib_n = o->calib ? o->calib_bytes : 0;
  return true;
}
}  // namespace

int tsg_scanner_new(const tsg_global* g, int device, tsg_scanner** out) {
  return tsg_scanner_new_ex(g, device, nullptr, out);
}

int tsg_scanner_new_ex(const tsg_global* g, int device, const tsg_compile_options* opt, tsg_scanner** out) {
  tsg::CompileOptions co;
  if (!CompileOpts(opt, &co)) return -1;
  std::string err;
  std::vector<tsg::RuleSpec> rules;
  std::vector<tsg::AllowRuleSpec> allow;
  std::vector<std::unique_ptr<tsg::Regex>> exclude;
  if (!MakeRules(g, &rules, &err) || !MakeAllow(g->allow_rules, g->n_allow_rules, &allow, &err) ||
      !MakeExclude(g->exclude_regexes, g->n_exclude_regexes, &exclude, &err)) {
    tsg::SetError(err);
    return -1;
  }
  std::unique_ptr<tsg_scanner> s(new tsg_scanner());
  s->s.reset(new tsg::SecretScanner(std::move(rules), std::move(allow), std::move(exclude), device, &err, &co));
  if (!s->s->ok()) {
    tsg::SetError(err.empty() ? s->s->error() : err);
    return -2;
  }
  *out = s.release();
  return 0;
}

void tsg_scanner_free(tsg_scanner* s) { delete s; }

int tsg_host_register(void* p, uint64_t bytes) {
  if (!p || !bytes) return 0;
  const hipError_t e = hipHostRegister(p, size_t(bytes), hipHostRegisterDefault);
  if (e != hipSuccess) {
    tsg::SetError(std::string("hipHostRegister: ") + hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int tsg_host_register_mapped(void* p, uint64_t bytes) {
  if (!p || !bytes) return 0;
  const hipError_t e = hipHostRegister(p, size_t(bytes), hipHostRegisterMapped);
  if (e != hipSuccess) {
    tsg::SetError(std::string("hipHostRegister (mapped): ") + hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int tsg_host_unregister(void* p) {
  if (!p) return 0;
  const hipError_t e = hipHostUnregister(p);
  if (e != hipSuccess) {
    tsg::SetError(std::string("hipHostUnregister: ") + hipGetErrorString(e));
    return -1;
  }
  return 0;
}

int tsg_scanner_allow_path(const tsg_scanner* s, const char* path, uint64_t len) {
  return s->s->AllowPath(reinterpret_cast<const uint8_t*>(path), size_t(len)) ? 1 : 0;
}

struct tsg_pending {
  std::thread th;
  tsg_result* r = nullptr;
  int rc = 0;
  std::string err;
};

namespace {

// tsg_batch_ext sizes this library reads (tsg_scanner.h): the fields past
// `base` that a caller's struct_size covers
bool CheckExtSize(const tsg_batch_ext* b) {
  if (!b) {
    tsg::SetError("tsg_scan_ext: NULL batch");
    return false;
  }
  if (b->struct_size != TSG_BATCH_EXT_SIZE_V1 && b->struct_size != TSG_BATCH_EXT_SIZE_V2) {
    tsg::SetError("tsg_scan_ext: tsg_batch_ext.struct_size " + std::to_string(b->struct_size) +
                  " is not a size this library knows (v1 = " + std::to_string(TSG_BATCH_EXT_SIZE_V1) +
                  ", v2 = " + std::to_string(TSG_BATCH_EXT_SIZE_V2) + ")");
    return false;
  }
  return true;
}

struct ExtFields {  // the fields past tsg_batch that a caller's struct_size covers
  const uint8_t* host_paths = nullptr;
  const uint64_t* host_path_off = nullptr;
  const uint8_t* gather_base = nullptr;
  const uint64_t* gather_src = nullptr;
};

ExtFields ExtOf(const tsg_batch_ext* b) {
  ExtFields e;
  e.host_paths = b->host_paths;
  e.host_path_off = b->host_path_offsets;
  if (b->struct_size >= TSG_BATCH_EXT_SIZE_V2) {
    e.gather_base = b->gather_base;
    e.gather_src = b->gather_src;
  }
  return e;
}

int ScanImpl(tsg_scanner* s, const tsg_batch* b, const ExtFields& x, tsg_result** out);

}  // namespace

int tsg_scan_submit_ext(tsg_scanner* s, const tsg_batch_ext* b, tsg_pending** out) {
  if (!CheckExtSize(b)) return -1;
  std::unique_ptr<tsg_pending> p(new tsg_pending());
  const tsg_batch bc = b->base;
  const ExtFields x = ExtOf(b);
  tsg_pending* pp = p.get();
  pp->th = std::thread([s, bc, x, pp] {
    pthread_setname_np(pthread_self(), "tsg-scan");
    pp->rc = ScanImpl(s, &bc, x, &pp->r);
    if (pp->rc != 0) pp->err = tsg_last_error();
  });
  *out = p.release();
  return 0;
}

int tsg_scan_submit(tsg_scanner* s, const tsg_batch* b, tsg_pending** out) {
  tsg_batch_ext e{};
  e.struct_size = TSG_BATCH_EXT_SIZE_V1;
  e.base = *b;  // (the frozen layout only: nothing past it is read)
  return tsg_scan_submit_ext(s, &e, out);
}

int tsg_scan_wait(tsg_pending* p, tsg_result** out) {
  if (!p) return -1;
  p->th.join();
  const int rc = p->rc;
  *out = p->r;
  if (rc != 0) tsg::SetError(p->err);
  delete p;
  return rc;
}

int tsg_scan(tsg_scanner* s, const tsg_batch* b, tsg_result** out) { return ScanImpl(s, b, ExtFields(), out); }

int tsg_scan_ext(tsg_scanner* s, const tsg_batch_ext* b, tsg_result** out) {
  if (!CheckExtSize(b)) return -1;
  return ScanImpl(s, &b->base, ExtOf(b), out);
}

namespace {

int ScanImpl(tsg_scanner* s, const tsg_batch* b, const ExtFields& x, tsg_result** out) {
  tsg::BatchInput in;
  in.n_files = b->n_files;
  in.host_arena = b->host_arena;
  in.host_offsets = b->host_offsets;
  in.dev_arena = static_cast<const uint8_t*>(b->dev_arena);
  in.dev_offsets = static_cast<const uint64_t*>(b->dev_offsets);
  in.paths = b->paths;
  in.path_lens = b->path_lens;
  in.binary = b->binary;
  in.transform = b->transform;
  in.dev_paths = static_cast<const uint8_t*>(b->dev_paths);
  in.dev_path_off = static_cast<const uint64_t*>(b->dev_path_offsets);
  in.host_paths = x.host_paths;
  in.host_path_off = x.host_path_off;
  in.gather_base = x.gather_base;
  in.gather_src = x.gather_src;
  if (in.gather_base && (!in.gather_src || !in.transform || in.dev_arena)) {
    tsg::SetError("tsg_scan: a gathered batch needs gather_src and transform, and no dev_arena");
    return -1;
  }
  std::unique_ptr<tsg_result> r(new tsg_result());
  r->owner = s->s.get();
  tsg::BatchStats gs;
  tsg::HostStats hs;
  std::string err;
  if (!s->s->Scan(in, &r->files, &gs, &hs, &err)) {
    tsg::SetError(err);
    return -1;
  }
  tsg_stats& st = r->stats;
  std::memset(&st, 0, sizeof(st));
  st.bytes = gs.bytes;
  st.files = gs.files;
  st.anchor_hits = gs.hits;
  st.candidates = gs.candidates;
  st.special_files = gs.special_files;
  st.findings = hs.findings;
  st.ms_scan_kernel = gs.ms_scan;
  st.ms_verify_kernel = gs.ms_confirm + gs.ms_verify;  // K2: confirm + NFA verify
  st.ms_fullscan_kernel = gs.ms_fullscan;
  st.ms_gpu_total = gs.ms_total;
  st.ms_host_gpu_phase = hs.ms_gpu;
  st.ms_host_allow_path = hs.ms_allow;
  st.ms_host_exact = hs.ms_exact;
  st.ms_host_total = hs.ms_total;
  st.flagged_blocks = gs.flagged_blocks;
  st.ms_careful_kernel = gs.ms_careful;
  st.follow_hits = gs.follow_hits;
  st.ms_chunkmap_kernel = gs.ms_chunkmap;
  st.ms_confirm_kernel = gs.ms_confirm;
  st.ms_nfa_kernel = gs.ms_verify;
  st.ms_finalize_kernel = gs.ms_finalize;
  st.ms_h2d_span = gs.ms_h2d_span;
  st.h2d_chunks = gs.h2d_chunks;
  st.fullscan_pairs = gs.fullscan_tasks;
  st.fold_sites = gs.fold_sites;
  st.ms_xform_kernel = gs.ms_xform;
  *out = r.release();
  return 0;
}

}  // namespace

void tsg_result_free(tsg_result* r) { ResultReaper::Get().Push(r); }

int tsg_result_file(const tsg_result* r, uint32_t file, uint32_t* kind, uint32_t* n) {
  if (file >= r->files.kind.size()) return -1;
  *kind = r->files.kind[file];
  const auto* v = r->files.Findings(file);
  *n = v ? uint32_t(v->size()) : 0;
  return 0;
}

int tsg_result_finding(const tsg_result* r, uint32_t file, uint32_t k, tsg_finding* out) {
  const auto* v = file < r->files.kind.size() ? r->files.Findings(file) : nullptr;
  if (!v || k >= v->size()) return -1;
  const auto& f = v->f[k];
  out->rule_index = f.rule;
  out->start_line = f.start_line;
  out->end_line = f.end_line;
  out->match = v->text.data() + f.match_off;
  out->match_len = f.match_len;
  out->n_lines = f.line_hi - f.line_lo;
  return 0;
}

uint64_t tsg_result_records(const tsg_result* r, tsg_record* out, uint64_t cap) {
  uint64_t n = 0;
  const auto& fs = r->files;
  for (size_t i = 0; i < fs.found_files.size(); i++) {
    const auto& v = fs.found[i];
    for (const auto& f : v.f) {
      if (n < cap) {
        uint64_t h = 0xcbf29ce484222325ull;
        auto mix = [&h](const void* p, size_t k) {
          const uint8_t* b = static_cast<const uint8_t*>(p);
          for (size_t q = 0; q < k; q++) h = (h ^ b[q]) * 0x100000001b3ull;
        };
        mix(v.text.data() + f.match_off, f.match_len);
        for (uint32_t l = f.line_lo; l < f.line_hi; l++) {
          const auto& ln = v.lines[l];
          const uint8_t fl[3] = {uint8_t(ln.is_cause), uint8_t(ln.first_cause), uint8_t(ln.last_cause)};
          mix(&ln.number, sizeof(ln.number));
          mix(fl, 3);
          mix(v.text.data() + ln.off, ln.len);
        }
        out[n] = tsg_record{fs.found_files[i], f.rule, f.start_line, f.end_line, h};
      }
      n++;
    }
  }
  return n;
}

int tsg_result_line(const tsg_result* r, uint32_t file, uint32_t k, uint32_t line, tsg_line* out) {
  const auto* v = file < r->files.kind.size() ? r->files.Findings(file) : nullptr;
  if (!v || k >= v->size()) return -1;
  const auto& f = v->f[k];
  if (line >= f.line_hi - f.line_lo) return -1;
  const auto& l = v->lines[f.line_lo + line];
  out->number = l.number;
  out->content = v->text.data() + l.off;
  out->content_len = l.len;
  out->is_cause = l.is_cause;
  out->first_cause = l.first_cause;
  out->last_cause = l.last_cause;
  return 0;
}

namespace {
void ResultJson(const tsg_result* r, uint32_t lo, uint32_t hi, std::string* out) {
  {
    const auto& rules = r->owner->rules();
    std::string& o = *out;
    o.reserve(256 + size_t(hi - lo) * 32);
    o.push_back('[');
    static const tsg::FileFindings kNone;
    for (size_t i = lo; i < hi; i++) {
      const auto* fv = r->files.Findings(uint32_t(i));
      const auto& findings = fv ? *fv : kNone;
      if (i > lo) o.push_back(',');
      o += "{\"kind\":" + std::to_string(int(r->files.kind[i])) + ",\"findings\":[";
      for (size_t k = 0; k < findings.size(); k++) {
        const auto& f = findings.f[k];
        const auto& R = rules[f.rule];
        if (k) o.push_back(',');
        o += "{\"RuleID\":";
        JsonStr(&o, R.id);
        o += ",\"Category\":";
        JsonStr(&o, R.category);
        o += ",\"Severity\":";
        JsonStr(&o, R.severity.empty() ? std::string("UNKNOWN") : R.severity);
        o += ",\"Title\":";
        JsonStr(&o, R.title);
        o += ",\"StartLine\":" + std::to_string(f.start_line) + ",\"EndLine\":" + std::to_string(f.end_line);
        // binary files: types.Code{} -> "Lines":null (scanner.go:441-444)
        o += findings.binary ? ",\"Code\":{\"Lines\":null" : ",\"Code\":{\"Lines\":[";
        for (uint32_t j = f.line_lo; j < f.line_hi; j++) {
          const auto& l = findings.lines[j];
          const std::string content(findings.Str(l.off, l.len));
          if (j > f.line_lo) o.push_back(',');
          o += "{\"Number\":" + std::to_string(l.number) + ",\"Content\":";
          JsonStr(&o, content);
          o += ",\"IsCause\":";
          o += l.is_cause ? "true" : "false";
          o += ",\"Annotation\":\"\",\"Truncated\":false,\"Highlighted\":";
          JsonStr(&o, content);
          o += ",\"FirstCause\":";
          o += l.first_cause ? "true" : "false";
          o += ",\"LastCause\":";
          o += l.last_cause ? "true" : "false";
          o.push_back('}');
        }
        o += findings.binary ? "},\"Match\":" : "]},\"Match\":";
        JsonStr(&o, std::string(findings.Match(f)));
        o.push_back('}');
      }
      o += "]}";
    }
    o.push_back(']');
  }
}
}  // namespace

int tsg_result_json(const tsg_result* rc, const char** json, uint64_t* len) {
  tsg_result* r = const_cast<tsg_result*>(rc);
  if (r->json.empty()) ResultJson(r, 0, uint32_t(r->files.kind.size()), &r->json);
  *json = r->json.data();
  *len = r->json.size();
  return 0;
}

int tsg_result_json_range(const tsg_result* rc, uint32_t lo, uint32_t hi, const char** json, uint64_t* len) {
  tsg_result* r = const_cast<tsg_result*>(rc);
  if (lo > hi || hi > r->files.kind.size()) return -1;
  // its own buffer: a range must not replace the whole-result JSON that
  // tsg_result_json builds once and returns from then on
  r->json_range.clear();
  ResultJson(r, lo, hi, &r->json_range);
  *json = r->json_range.data();
  *len = r->json_range.size();
  return 0;
}

int tsg_result_stats(const tsg_result* r, tsg_stats* out) {
  *out = r->stats;
  return 0;
}

static void FillInfo(const tsg::CompiledRules& cr, tsg_table_info* out) {
  out->n_rules = uint32_t(cr.rules.size());
  out->n_keywords = uint32_t(cr.keywords.size());
  out->n_anchors = uint32_t(cr.anchors.size());
  const tsg::FilterTables* ft = cr.filter.get();
  out->n_filter_items = ft ? uint32_t(ft->items.size()) : 0;
  out->n_filter_buckets = ft ? ft->n_buckets : 0;
  out->filter_window = ft ? ft->window : 0;
  out->filter_table_bytes =
      ft ? ft->reach.size() * 4 + ft->bucket_off.size() * 4 + ft->bucket_items.size() * 4 +
               ft->items.size() * sizeof(tsg::FilterItemGpu) + ft->item_ids.size() * 4 + ft->item_cls.size() +
               ft->classes.size() * 4 + ft->core.size() * 8 + ft->group_items.size() * 4 + ft->bucket_groups.size() * 4
         : 0;
  out->filter_est_fp = ft ? ft->est_fp : 0;
  out->n_fullscan_rules = cr.n_fullscan_rules;
  uint32_t w = 0;
  for (auto& r : cr.rules) w += r.nfa_words;
  out->nfa_words_total = w;
}

int tsg_scanner_table_info(const tsg_scanner* s, tsg_table_info* out) {
  FillInfo(s->s->compiled(), out);
  return 0;
}

const char* tsg_scanner_rule_anchor(const tsg_scanner* s, uint32_t i) {
  const auto& d = s->s->compiled().rule_anchor_desc;
  return i < d.size() ? d[i].c_str() : "";
}

// ---- tsg_debug.h: rule compiler inspection (no GPU) ------------------------

int tsg_debug_compile(const tsg_global* g, tsg_compiled** out) { return tsg_debug_compile_ex(g, nullptr, out, nullptr); }

int tsg_debug_compile_ex(const tsg_global* g, const tsg_compile_options* opt, tsg_compiled** out,
                         uint32_t* out_calibrated) {
  tsg::CompileOptions co;
  if (!CompileOpts(opt, &co)) return -1;
  std::string err;
  std::vector<tsg::RuleSrc> src;
  for (uint32_t i = 0; i < g->n_rules; i++) {
    const tsg_rule& r = g->rules[i];
    tsg::RuleSrc s{Str(r.id), Str(r.regex), {}, r.regex != nullptr};
    for (uint32_t k = 0; k < r.n_keywords; k++) s.keywords.push_back(Str(r.keywords[k]));
    src.push_back(std::move(s));
  }
  std::unique_ptr<tsg_compiled> c(new tsg_compiled());
  if (!tsg::CompileRules(src, &c->cr, &err, &co)) {
    tsg::SetError(err);
    return -1;
  }
  if (out_calibrated) *out_calibrated = c->cr.n_calibrated_anchors;
  *out = c.release();
  return 0;
}

void tsg_debug_compiled_free(tsg_compiled* c) { delete c; }

int tsg_debug_compiled_info(const tsg_compiled* c, tsg_table_info* out) {
  FillInfo(c->cr, out);
  return 0;
}


int tsg_debug_rule(const tsg_compiled* c, uint32_t i, tsg_debug_rule_info* out) {
  if (i >= c->cr.rules.size()) return -1;
  const auto& r = c->cr.rules[i];
  out->nfa_words = r.nfa_words;
  out->gate = r.gate;
  out->anchored = r.anchored;
  out->has_regex = r.has_regex;
  out->nfa = c->cr.nfa.data() + r.nfa_off;
  out->kw_ids = c->cr.rule_kw.data() + r.kw_off;
  out->n_kw = r.kw_cnt;
  return 0;
}

int tsg_debug_anchor(const tsg_compiled* c, uint32_t j, uint32_t* rule, uint32_t* lit_len, int32_t* off_lo,
                     int32_t* off_hi) {
  if (j >= c->cr.anchors.size()) return -1;
  const auto& a = c->cr.anchors[j];
  *rule = a.rule;
  *lit_len = a.lit_len;
  *off_lo = a.off_lo;
  *off_hi = a.off_hi;
  return 0;
}

int tsg_debug_filter(const tsg_compiled* c, uint32_t* shape, const uint32_t** reach, const uint32_t** bucket_off,
                     const uint32_t** bucket_items, const void** items, uint32_t* n_items, const uint8_t** item_cls,
                     const uint32_t** classes, double* est_fp) {
  const auto* f = c->cr.filter.get();
  if (!f) return -1;
  shape[0] = f->n_buckets;
  shape[1] = f->window;
  shape[2] = f->n_words;
  *reach = f->reach.data();
  *bucket_off = f->bucket_off.data();
  *bucket_items = f->bucket_items.data();
  *items = f->items.data();
  *n_items = uint32_t(f->items.size());
  *item_cls = f->item_cls.data();
  *classes = f->classes.data();
  *est_fp = f->est_fp;
  return 0;
}

int tsg_debug_filter_ids(const tsg_compiled* c, const uint32_t** ids, uint32_t* n) {
  const auto* f = c->cr.filter.get();
  if (!f) return -1;
  *ids = f->item_ids.data();
  *n = uint32_t(f->item_ids.size());
  return 0;
}

const char* tsg_debug_rule_anchor(const tsg_compiled* c, uint32_t i) {
  const auto& d = c->cr.rule_anchor_desc;
  return i < d.size() ? d[i].c_str() : nullptr;
}

const void* tsg_debug_anchor_req(const tsg_compiled* c, uint32_t j) {
  return j < c->cr.anchor_req.size() ? &c->cr.anchor_req[j] : nullptr;
}

const char* tsg_debug_keyword(const tsg_compiled* c, uint32_t k) {
  return k < c->cr.keywords.size() ? c->cr.keywords[k].c_str() : nullptr;
}

int tsg_debug_scanner_engine(tsg_scanner* s, uint64_t out[4]) {
  out[0] = out[1] = out[2] = out[3] = 0;
  if (!s || !s->s || s->s->n_engines() == 0) return -1;
  for (size_t i = 0; i < s->s->n_engines(); i++) {
    const tsg::GpuEngine::HostMemInfo m = s->s->engine_at(i)->host_mem_info();
    out[0] += m.retired_pending;
    out[1] += m.retired_freed;
    out[2] = std::max<uint64_t>(out[2], m.cand_cap);
    out[3] += m.slot_bytes;
  }
  return 0;
}

int tsg_debug_scanner_gpu_findings(tsg_scanner* s, int on) {
  if (!s || !s->s) return -1;
  return s->s->SetGpuFindings(on);
}

}  // extern "C"
