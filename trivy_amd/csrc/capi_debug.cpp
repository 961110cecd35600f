// C-ABI for host-logic inspection (include/tsg_debug.h).
#include "tsg_debug.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>

#include "goregex.h"
#include "parallel.h"
#include "xform.h"

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

int tsg_debug_xform(int device, const uint8_t* raw, uint64_t n_bytes, const uint64_t* offsets, uint32_t n_files,
                    const uint8_t* kinds, uint8_t* out, uint64_t out_cap, uint64_t* xoff) {
  if (offsets[0] != 0 || offsets[n_files] != n_bytes) {
    tsg::SetError("offsets must run from 0 to n_bytes");
    return -2;
  }
  void *d_raw = nullptr, *d_off = nullptr, *d_kind = nullptr, *d_xoff = nullptr, *d_out = nullptr, *d_sc = nullptr;
  hipStream_t s = nullptr;
  hipError_t e = hipSetDevice(device);
  auto ok = [&](hipError_t r) {
    if (e == hipSuccess) e = r;
    return e == hipSuccess;
  };
  const size_t sc_bytes = tsg::XformScratchBytes(n_bytes, n_files);
  if (ok(e) && ok(hipStreamCreate(&s)) && ok(hipMalloc(&d_raw, n_bytes + 64)) &&
      ok(hipMalloc(&d_off, (size_t(n_files) + 1) * 8)) && ok(hipMalloc(&d_kind, size_t(n_files) + 1)) &&
      ok(hipMalloc(&d_xoff, (size_t(n_files) + 1) * 8)) && ok(hipMalloc(&d_sc, sc_bytes)) &&
      ok(hipMemset(d_raw, 0, n_bytes + 64)) && ok(hipMemcpy(d_raw, raw, n_bytes, hipMemcpyHostToDevice)) &&
      ok(hipMemcpy(d_off, offsets, (size_t(n_files) + 1) * 8, hipMemcpyHostToDevice)) &&
      ok(hipMemcpy(d_kind, kinds, n_files, hipMemcpyHostToDevice)) && tsg::XformOnePassOn()) {
    const uint64_t cap = tsg::XformMaxOut(n_bytes, n_files) + 64;  // (the engine's bound)
    if (ok(hipMalloc(&d_out, cap)) &&
        ok(tsg::XformOnePass(static_cast<const uint8_t*>(d_raw), n_bytes, static_cast<const uint64_t*>(d_off),
                             static_cast<const uint8_t*>(d_kind), n_files, d_sc, static_cast<uint64_t*>(d_xoff),
                             static_cast<uint8_t*>(d_out), cap, s)) &&
        ok(hipMemcpyAsync(xoff, d_xoff, (size_t(n_files) + 1) * 8, hipMemcpyDeviceToHost, s)) &&
        ok(hipStreamSynchronize(s)) &&
        ok(tsg::XformErrorWord(n_bytes, n_files, d_sc, s) == 0 ? hipSuccess : hipErrorIllegalAddress))
      ok(hipMemcpy(out, d_out, std::min<uint64_t>(out_cap, xoff[n_files]), hipMemcpyDeviceToHost));
  } else if (ok(e) &&
      ok(tsg::XformPlan(static_cast<const uint8_t*>(d_raw), n_bytes, static_cast<const uint64_t*>(d_off),
                        static_cast<const uint8_t*>(d_kind), n_files, d_sc, static_cast<uint64_t*>(d_xoff), s)) &&
      ok(hipMemcpyAsync(xoff, d_xoff, (size_t(n_files) + 1) * 8, hipMemcpyDeviceToHost, s)) &&
      ok(hipStreamSynchronize(s)) && ok(hipMalloc(&d_out, xoff[n_files] + 64)) &&
      ok(tsg::XformWrite(static_cast<const uint8_t*>(d_raw), n_bytes, static_cast<const uint64_t*>(d_off),
                         static_cast<const uint8_t*>(d_kind), n_files, d_sc, static_cast<uint8_t*>(d_out),
                         xoff[n_files] + 64, s)) &&
      ok(hipStreamSynchronize(s)) &&
      ok(tsg::XformErrorWord(n_bytes, n_files, d_sc, s) == 0 ? hipSuccess : hipErrorIllegalAddress))
    ok(hipMemcpy(out, d_out, std::min<uint64_t>(out_cap, xoff[n_files]), hipMemcpyDeviceToHost));
  for (void* p : {d_raw, d_off, d_kind, d_xoff, d_out, d_sc})
    if (p) (void)hipFree(p);
  if (s) (void)hipStreamDestroy(s);
  if (e != hipSuccess) {
    tsg::SetError(std::string("tsg_debug_xform: ") + hipGetErrorString(e));
    return -1;
  }
  return 0;
}

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
