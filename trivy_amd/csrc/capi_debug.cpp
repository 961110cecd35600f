// C-ABI for host-logic inspection (include/tsg_debug.h).
#include "tsg_debug.h"

#include <atomic>
#include <cstring>
#include <string>

#include "goregex.h"
#include "parallel.h"

namespace tsg {
extern std::atomic<int> g_regex_engine;
thread_local std::string g_last_error;
void SetError(const std::string& e) { g_last_error = e; }
}  // namespace tsg

extern "C" {

const char* tsg_last_error(void) { return tsg::g_last_error.c_str(); }

int tsg_regex_find_all(const char* pattern, const uint8_t* text, uint64_t n, int submatch,
                       const int64_t* windows, uint32_t n_windows, int64_t* out, uint64_t out_cap,
                       uint64_t* out_len, int32_t* num_cap) {
  std::string err;
  auto re = tsg::Regex::Compile(pattern, &err);
  if (!re) {
    tsg::SetError(err);
    return -1;
  }
  std::vector<tsg::Window> wins;
  for (uint32_t i = 0; i < n_windows; i++) wins.push_back({windows[2 * i], windows[2 * i + 1]});
  std::vector<int64_t> res;
  re->FindAll(text, int64_t(n), submatch != 0, windows ? &wins : nullptr, &res);
  *out_len = res.size();
  *num_cap = re->num_cap();
  std::memcpy(out, res.data(), sizeof(int64_t) * (res.size() < out_cap ? res.size() : out_cap));
  return 0;
}

void tsg_debug_regex_engine(int mode) { tsg::g_regex_engine.store(mode); }

int tsg_regex_match(const char* pattern, const uint8_t* text, uint64_t n) {
  std::string err;
  auto re = tsg::Regex::Compile(pattern, &err);
  if (!re) {
    tsg::SetError(err);
    return -1;
  }
  return re->Match(text, int64_t(n)) ? 1 : 0;
}

int64_t tsg_go_bytes_to_lower(const uint8_t* s, uint64_t n, uint8_t* out, uint64_t out_cap) {
  std::string l = tsg::GoBytesToLower(s, n);
  std::memcpy(out, l.data(), l.size() < out_cap ? l.size() : out_cap);
  return int64_t(l.size());
}

int tsg_debug_pool_budget(void) { return tsg::PoolBudget(); }
}
