// GPU finding materialisation (materialize.h; scanner.go:438-446, 465-558).
//
// Two kernels, one wave per location, separated by a prefix sum over the
// per-location (text bytes, line count):
//   mat_locate_kernel  line number, match line, code-window line bounds, sizes
//   mat_write_kernel   FindingOut / LineOut records and the censored text
// Newline searches read the arena in 1-KiB wave windows (a 16-B block per
// lane, per-byte exact '\n' masks by SWAR), drop the '\n' inside censor spans
// (the reference runs findLocation on the censored buffer, where they are '*')
// and take the nearest ones by ballots.  Every read stays inside the file's
// 16-B-aligned blocks, which the batch arena holds (it has 64 readable bytes
// past its end).
#include "materialize.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace tsg {

namespace {

constexpr int kMatThreads = 256;  // four waves, a location each
constexpr int kMatWaves = kMatThreads / 64;
constexpr int64_t kLineCut = 100;  // scanner.go:535-541: lines over 100 B are cut

struct MatLoc {           // mat_locate_kernel -> mat_write_kernel
  int64_t line;           // '\n' the censored content keeps before s: the 0-based line of s
  int64_t mls, mle;       // the match text [mls, mle) (scanner.go:520-528)
  int64_t lb[4], le[4];   // the code lines [lb, le) from code_start on
  int64_t code_start;     // 0-based line number of lb[0]
  uint32_t nlines, cause; // line count; index of the cause line (the line of s)
};

// bit i set iff byte i of the 16 is '\n' (exact per byte: no borrow between bytes)
__device__ __forceinline__ uint32_t nl_mask16(uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t t = w[k] ^ 0x0A0A0A0Au;
    uint32_t y = (t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    y = ~(y | t | 0x7F7F7F7Fu);  // 0x80 in each byte of t that is zero
    m |= (((y >> 7) & 1u) | ((y >> 14) & 2u) | ((y >> 21) & 4u) | ((y >> 28) & 8u)) << (4 * k);
  }
  return m;
}

// '\n' mask of the 16-B block at absolute B, restricted to absolute [lo, hi);
// no load when the block is outside it
__device__ __forceinline__ uint32_t block_mask(const uint8_t* __restrict__ arena, int64_t B, int64_t lo, int64_t hi) {
  if (B + 16 <= lo || B >= hi) return 0;
  uint32_t m = nl_mask16(*reinterpret_cast<const uint4*>(arena + B));
  if (B < lo) m &= 0xFFFFu << uint32_t(lo - B);
  if (B + 16 > hi) m &= (1u << uint32_t(hi - B)) - 1u;
  return m & 0xFFFFu;
}

// clear the bits of censored bytes: spans from k (sorted, disjoint, a sentinel
// at the end) that intersect the block at file-relative b
__device__ __forceinline__ uint32_t drop_censored(uint32_t m, int64_t b, const MatSpan* __restrict__ sp, uint32_t k) {
  if (!m) return m;
  for (;; k++) {
    const int64_t ss = sp[k].s, se = sp[k].e;
    if (ss >= b + 16) break;
    if (se <= b) continue;
    const uint32_t lo = uint32_t(max(ss, b) - b), hi = uint32_t(min(se, b + 16) - b);
    m &= ~(((1u << (hi - lo)) - 1u) << lo);
  }
  return m;
}

// the first span with e > x (the sentinel's e is INT64_MAX)
__device__ __forceinline__ uint32_t span_after(const MatSpan* __restrict__ sp, uint32_t ns, int64_t x) {
  uint32_t lo = 0, hi = ns - 1;  // answer in [lo, hi]: the sentinel qualifies
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (sp[mid].e > x) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int x = 32; x >= 1; x >>= 1) v += __shfl_xor(v, x);
  return v;
}

// raw '\n' in file-relative [a, b) (4 KiB per wave step)
__device__ int64_t count_nl(const uint8_t* __restrict__ arena, int64_t fs, int64_t a, int64_t b, uint32_t lane) {
  if (b <= a) return 0;
  const int64_t lo = fs + a, hi = fs + b;
  uint32_t n = 0;
  for (int64_t W = lo & ~int64_t(15); W < hi; W += 4096) {
    uint32_t m[4];
#pragma unroll
    for (int j = 0; j < 4; j++) m[j] = block_mask(arena, W + 1024 * j + 16 * int64_t(lane), lo, hi);
#pragma unroll
    for (int j = 0; j < 4; j++) n += __popc(m[j]);
  }
  return int64_t(wave_sum(n));
}

// the last k (<= 3) visible '\n' before file-relative pos, nearest first; -1 past the file start
__device__ void back_nl(const uint8_t* __restrict__ arena, int64_t fs, int64_t pos, const MatSpan* __restrict__ sp,
                        uint32_t ns, int k, int64_t* out, uint32_t lane) {
  for (int i = 0; i < k; i++) out[i] = -1;
  int found = 0;
  int64_t top = fs + pos;  // absolute, exclusive
  while (found < k && top > fs) {
    const int64_t W = ((top - 1) & ~int64_t(15)) - 1008;  // the last of the 64 blocks holds top - 1
    const int64_t B = W + 16 * int64_t(lane);
    uint32_t m = block_mask(arena, B, fs, top);
    const int64_t wlo = max(W, fs) - fs;
    const uint32_t k0 = span_after(sp, ns, wlo);
    if (sp[k0].s < top - fs) m = drop_censored(m, B - fs, sp, k0);
    while (found < k) {
      const uint64_t bal = __ballot(m != 0);
      if (!bal) break;
      const int hl = 63 - __clzll(bal);
      const uint32_t mh = __shfl(m, hl);
      const int bit = 31 - __clz(mh);
      out[found++] = W + 16 * int64_t(hl) + bit - fs;
      if (int(lane) == hl) m &= ~(1u << bit);
    }
    top = W;
  }
}

// the first k (<= 2) visible '\n' at or after file-relative pos, nearest first; len when none
__device__ void fwd_nl(const uint8_t* __restrict__ arena, int64_t fs, int64_t len, int64_t pos,
                       const MatSpan* __restrict__ sp, uint32_t ns, int k, int64_t* out, uint32_t lane) {
  for (int i = 0; i < k; i++) out[i] = len;
  int found = 0;
  int64_t bot = fs + pos;  // absolute, inclusive
  const int64_t end = fs + len;
  while (found < k && bot < end) {
    const int64_t W = bot & ~int64_t(15);
    const int64_t B = W + 16 * int64_t(lane);
    uint32_t m = block_mask(arena, B, bot, end);
    const uint32_t k0 = span_after(sp, ns, bot - fs);
    if (sp[k0].s < W + 1024 - fs) m = drop_censored(m, B - fs, sp, k0);
    while (found < k) {
      const uint64_t bal = __ballot(m != 0);
      if (!bal) break;
      const int ll = __ffsll(static_cast<unsigned long long>(bal)) - 1;
      const uint32_t ml = __shfl(m, ll);
      const int bit = __ffs(ml) - 1;
      out[found++] = W + 16 * int64_t(ll) + bit - fs;
      if (int(lane) == ll) m &= ~(1u << bit);
    }
    bot = W + 1024;
  }
}

__global__ __launch_bounds__(kMatThreads) void mat_locate_kernel(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offsets, const MatFile* __restrict__ files,
    const MatMatch* __restrict__ mm, const MatSpan* __restrict__ spans, uint32_t nm, MatLoc* __restrict__ locs,
    uint64_t* __restrict__ cnt, uint32_t* __restrict__ err) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[nm] = 0;  // the scan's last element: the totals
  for (uint32_t m = blockIdx.x * kMatWaves + wave; m < nm; m += gridDim.x * kMatWaves) {
    const MatMatch M = mm[m];
    const MatFile F = files[M.fidx];
    const int64_t fs = int64_t(offsets[F.file]), len = int64_t(offsets[F.file + 1]) - fs;
    const MatSpan* sp = spans + F.s0;
    const uint32_t ns = F.ns;  // (with the sentinel)
    const int64_t s = M.s, e = M.e;
    // StartLine - 1 (scanner.go:496-499 on the censored content): raw '\n'
    // before s minus the censored ones
    const int64_t raw = M.a_nl + count_nl(arena, fs, M.a_wlo, s, lane);
    const uint32_t ks = span_after(sp, ns, s);
    int64_t cens = sp[ks].nl_before;
    if (sp[ks].s < s) cens += count_nl(arena, fs, sp[ks].s, s, lane);
    const int64_t line = raw - cens;
    int64_t q[3], f[2];
    back_nl(arena, fs, s, sp, ns, 3, q, lane);
    fwd_nl(arena, fs, len, s, sp, ns, 2, f, lane);
    if (lane == 0) {
      // the searches and the count agree on the visible '\n' before s
      const int nq = (q[0] >= 0) + (q[1] >= 0) + (q[2] >= 0);
      if (line < 0 || nq != int(min<int64_t>(line, 3))) atomicOr(err, 1u);
      MatLoc L;
      L.line = line;
      const int64_t ls = q[0] + 1, le = f[0];  // (q[0] == -1: line 0 starts at 0)
      int64_t mls = ls, mle = le;
      if (le - ls > kLineCut) {  // scanner.go:520-528
        mls = (s - ls - 30 < 0) ? ls : s - 30;
        mle = (e + 20 > le) ? le : e + 20;
      }
      L.mls = mls;
      L.mle = mle;
      // code lines (scanner.go:530-556): from max(line - 2, 0) to line + 1, the
      // last one that of bytes.Split (ending at len)
      const int64_t cs = line >= 2 ? line - 2 : 0;
      L.code_start = cs;
      uint32_t n = 0;
      for (int64_t t = line - cs; t >= 1; t--) {  // lines above: [q[t] + 1, q[t - 1])
        L.lb[n] = q[t] + 1;
        L.le[n] = q[t - 1];
        n++;
      }
      L.cause = n;
      L.lb[n] = ls;
      L.le[n] = le;
      n++;
      if (le < len) {  // the line below
        L.lb[n] = le + 1;
        L.le[n] = f[1];
        n++;
      }
      L.nlines = n;
      // the cause line's text is the match text: cut (> 100 B) it is the match line
      // (scanner.go:535-537), uncut the match text is the whole line (:520-528)
      uint64_t text = uint64_t(mle - mls);
      for (uint32_t i = 0; i < n; i++)
        if (i != L.cause) text += uint64_t(min(L.le[i] - L.lb[i], kLineCut));
      locs[m] = L;
      cnt[m] = (text << 32) | n;
    }
  }
}

// content [a, b) of the file, censored bytes as '*', to out
__device__ void copy_censored(const uint8_t* __restrict__ arena, int64_t fs, int64_t a, int64_t b,
                              const MatSpan* __restrict__ sp, uint32_t ns, char* __restrict__ out, uint32_t lane) {
  if (b <= a) return;
  uint32_t k = span_after(sp, ns, a);
  for (int64_t i = lane; i < b - a; i += 64) {
    const int64_t x = a + i;
    while (sp[k].e <= x) k++;
    const uint8_t c = arena[fs + x];
    out[i] = sp[k].s <= x ? '*' : char(c);
  }
}

__global__ __launch_bounds__(kMatThreads) void mat_write_kernel(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offsets, const MatFile* __restrict__ files,
    const MatMatch* __restrict__ mm, const MatSpan* __restrict__ spans, uint32_t nm, const MatLoc* __restrict__ locs,
    const uint64_t* __restrict__ pref, FindingOut* __restrict__ fout, LineOut* __restrict__ lout,
    char* __restrict__ text) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint32_t m = blockIdx.x * kMatWaves + wave; m < nm; m += gridDim.x * kMatWaves) {
    const MatMatch M = mm[m];
    const MatFile F = files[M.fidx];
    const MatLoc L = locs[m];
    const int64_t fs = int64_t(offsets[F.file]);
    const MatSpan* sp = spans + F.s0;
    const uint64_t p = pref[m], p0 = pref[F.m0];
    const uint64_t tpos = p >> 32;                                // this location's text, batch-global
    const uint32_t lpos = uint32_t(p);                            // its first line, batch-global
    const uint32_t t_rel = uint32_t(tpos - (p0 >> 32));           // ... and file-relative
    const uint32_t l_rel = lpos - uint32_t(p0);
    const uint32_t mlen = uint32_t(L.mle - L.mls);
    copy_censored(arena, fs, L.mls, L.mle, sp, F.ns, text + tpos, lane);
    uint32_t off = mlen;
    for (uint32_t i = 0; i < L.nlines; i++) {
      const int64_t ll = L.le[i] - L.lb[i];
      const bool cause = i == L.cause;
      uint32_t o = t_rel, n = mlen;  // the cause line shares the match text (its bytes, see above)
      if (!cause) {  // own text: the first 100 B (scanner.go:538-541)
        n = uint32_t(min(ll, kLineCut));
        o = t_rel + off;
        copy_censored(arena, fs, L.lb[i], L.lb[i] + n, sp, F.ns, text + tpos + off, lane);
        off += n;
      }
      if (lane == 0) {
        LineOut lo;
        lo.number = L.code_start + int64_t(i) + 1;
        lo.off = o;
        lo.len = n;
        lo.is_cause = cause;
        lo.first_cause = cause;  // one cause line: it is the first and the last
        lo.last_cause = cause;
        lout[lpos + i] = lo;
      }
    }
    if (lane == 0) {
      FindingOut fo;
      fo.rule = M.rule;
      fo.start_line = L.line + 1;  // EndLine = StartLine: the location's own '\n' are censored
      fo.end_line = L.line + 1;
      fo.match_off = t_rel;
      fo.match_len = mlen;
      fo.line_lo = l_rel;
      fo.line_hi = l_rel + L.nlines;
      fout[m] = fo;
    }
  }
}

size_t Up(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

struct FindingMaterializer::Slot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  bool busy = false;
  // uploads: files | matches | spans, one pinned buffer and its device copy
  uint8_t* h_up = nullptr;
  size_t h_up_cap = 0;
  uint8_t* d_up = nullptr;
  size_t d_up_cap = 0;
  size_t off_match = 0, off_span = 0;
  uint32_t nf = 0, nm = 0, ns = 0;
  // device work + outputs
  uint8_t* d_work = nullptr;  // locs | cnt | pref | scan temp | err
  size_t work_cap = 0;
  FindingOut* d_find = nullptr;
  size_t find_cap = 0;  // records
  LineOut* d_lines = nullptr;
  size_t lines_cap = 0;
  char* d_text = nullptr;
  size_t text_cap = 0;
  // pinned read-backs
  FindingOut* h_find = nullptr;
  size_t h_find_cap = 0;
  LineOut* h_lines = nullptr;
  size_t h_lines_cap = 0;
  char* h_text = nullptr;
  size_t h_text_cap = 0;
  uint64_t* h_pref = nullptr;
  size_t h_pref_cap = 0;
  uint64_t* h_tot = nullptr;  // [0] totals, [1] error word
  uint64_t text_bound = 0;
};

struct FindingMaterializer::Job {
  Slot* s;
};

FindingMaterializer::FindingMaterializer(int device) : device_(device) {
  slots_ = new Slot[kSlots];
  int lo = 0, hi = 0;
  if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
  bool ok = hipSetDevice(device) == hipSuccess;
  for (int i = 0; i < kSlots; i++) {
    Slot& S = slots_[i];
    ok = ok && hipStreamCreateWithPriority(&S.stream, hipStreamNonBlocking, hi) == hipSuccess &&
         hipEventCreateWithFlags(&S.done, hipEventDisableTiming) == hipSuccess &&
         hipHostMalloc(reinterpret_cast<void**>(&S.h_tot), 64, hipHostMallocDefault) == hipSuccess;
  }
  if (!ok) err_ = "FindingMaterializer: HIP setup failed";
}

FindingMaterializer::~FindingMaterializer() {
  (void)hipSetDevice(device_);
  for (int i = 0; i < kSlots; i++) {
    Slot& S = slots_[i];
    if (S.stream) (void)hipStreamSynchronize(S.stream);
    for (void* p : {static_cast<void*>(S.d_up), static_cast<void*>(S.d_work), static_cast<void*>(S.d_find),
                    static_cast<void*>(S.d_lines), static_cast<void*>(S.d_text)})
      if (p) (void)hipFree(p);
    for (void* p : {static_cast<void*>(S.h_up), static_cast<void*>(S.h_find), static_cast<void*>(S.h_lines),
                    static_cast<void*>(S.h_text), static_cast<void*>(S.h_pref), static_cast<void*>(S.h_tot)})
      if (p) (void)hipHostFree(p);
    if (S.done) (void)hipEventDestroy(S.done);
    if (S.stream) (void)hipStreamDestroy(S.stream);
  }
  delete[] slots_;
}

namespace {

// grow a device / pinned buffer to hold `need` bytes (+1/4: a buffer grows a
// few times in the first scans, then stays; freeing one waits for the device)
template <class T>
hipError_t GrowDev(T** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return hipSuccess;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  const size_t n = need + need / 4 + 4096;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), n);
  if (e == hipSuccess) *cap = n;
  return e;
}

template <class T>
hipError_t GrowHost(T** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return hipSuccess;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  const size_t n = need + need / 4 + 4096;
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(p), n, hipHostMallocDefault);
  if (e == hipSuccess) *cap = n;
  return e;
}

}  // namespace

FindingMaterializer::Job* FindingMaterializer::Begin(uint32_t n_files, uint32_t n_match, uint32_t n_span,
                                                     uint64_t text_bound, std::string* err) {
  Slot* S = nullptr;
  {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] {
      for (int i = 0; i < kSlots; i++)
        if (!slots_[i].busy) return true;
      return false;
    });
    for (int i = 0; i < kSlots; i++)
      if (!slots_[i].busy) {
        S = &slots_[i];
        break;
      }
    S->busy = true;
  }
  std::unique_ptr<Job> j(new Job{S});
  S->nf = n_files;
  S->nm = n_match;
  S->ns = n_span;
  S->text_bound = text_bound;
  S->off_match = Up(size_t(n_files) * sizeof(MatFile));
  S->off_span = S->off_match + Up(size_t(n_match) * sizeof(MatMatch));
  const size_t up = S->off_span + Up(size_t(n_span) * sizeof(MatSpan));
  hipError_t e = hipSetDevice(device_);
  if (e == hipSuccess) e = GrowHost(&S->h_up, &S->h_up_cap, up);
  if (e != hipSuccess) {
    *err = std::string("FindingMaterializer: pinned upload buffer: ") + hipGetErrorString(e);
    End(j.release());
    return nullptr;
  }
  return j.release();
}

MatFile* FindingMaterializer::files(Job* j) { return reinterpret_cast<MatFile*>(j->s->h_up); }
MatMatch* FindingMaterializer::matches(Job* j) { return reinterpret_cast<MatMatch*>(j->s->h_up + j->s->off_match); }
MatSpan* FindingMaterializer::spans(Job* j) { return reinterpret_cast<MatSpan*>(j->s->h_up + j->s->off_span); }
const FindingOut* FindingMaterializer::findings(Job* j) const { return j->s->h_find; }
const LineOut* FindingMaterializer::lines(Job* j) const { return j->s->h_lines; }
const char* FindingMaterializer::text(Job* j) const { return j->s->h_text; }
const uint64_t* FindingMaterializer::pref(Job* j) const { return j->s->h_pref; }

void FindingMaterializer::End(Job* j) {
  {
    std::lock_guard<std::mutex> g(mu_);
    j->s->busy = false;
  }
  cv_.notify_one();
  delete j;
}

bool FindingMaterializer::Run(Job* j, const uint8_t* d_arena, const uint64_t* d_offsets, std::string* err) {
  Slot& S = *j->s;
  const uint32_t nm = S.nm;
  if (nm == 0) return true;
  auto fail = [&](const char* what, hipError_t e) {
    *err = std::string("FindingMaterializer: ") + what + ": " + hipGetErrorString(e);
    return false;
  };
  // sleep-poll (as GpuEngine::WaitEvent): a spinning wait takes a core from the host pool
  auto wait = [&]() {
    hipError_t e = hipEventRecord(S.done, S.stream);
    if (e != hipSuccess) return e;
    while ((e = hipEventQuery(S.done)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(50));
    return e;
  };
  hipError_t e = hipSetDevice(device_);
  if (e != hipSuccess) return fail("hipSetDevice", e);
  size_t scan_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, static_cast<const uint64_t*>(nullptr),
                                         static_cast<uint64_t*>(nullptr), int(nm) + 1);
  const size_t o_cnt = Up(size_t(nm) * sizeof(MatLoc));
  const size_t o_pref = o_cnt + Up((size_t(nm) + 1) * 8);
  const size_t o_scan = o_pref + Up((size_t(nm) + 1) * 8);
  const size_t o_err = o_scan + Up(scan_bytes);
  const size_t work = o_err + 256;
  const size_t up = S.off_span + Up(size_t(S.ns) * sizeof(MatSpan));
  if ((e = GrowDev(&S.d_up, &S.d_up_cap, up)) != hipSuccess || (e = GrowDev(&S.d_work, &S.work_cap, work)) != hipSuccess ||
      (e = GrowDev(&S.d_find, &S.find_cap, size_t(nm) * sizeof(FindingOut))) != hipSuccess ||
      (e = GrowDev(&S.d_lines, &S.lines_cap, size_t(nm) * 4 * sizeof(LineOut))) != hipSuccess ||
      (e = GrowDev(&S.d_text, &S.text_cap, size_t(S.text_bound) + 64)) != hipSuccess ||
      (e = GrowHost(&S.h_find, &S.h_find_cap, size_t(nm) * sizeof(FindingOut))) != hipSuccess ||
      (e = GrowHost(&S.h_pref, &S.h_pref_cap, (size_t(nm) + 1) * 8)) != hipSuccess)
    return fail("buffers", e);
  MatLoc* locs = reinterpret_cast<MatLoc*>(S.d_work);
  uint64_t* cnt = reinterpret_cast<uint64_t*>(S.d_work + o_cnt);
  uint64_t* pref = reinterpret_cast<uint64_t*>(S.d_work + o_pref);
  uint32_t* derr = reinterpret_cast<uint32_t*>(S.d_work + o_err);
  const MatFile* files = reinterpret_cast<const MatFile*>(S.d_up);
  const MatMatch* mm = reinterpret_cast<const MatMatch*>(S.d_up + S.off_match);
  const MatSpan* sp = reinterpret_cast<const MatSpan*>(S.d_up + S.off_span);
  const uint32_t grid = uint32_t(std::min<uint64_t>((uint64_t(nm) + kMatWaves - 1) / kMatWaves, 16384));
  // the upload, the locate pass, the scan; the totals and the error word back
  if ((e = hipMemcpyAsync(S.d_up, S.h_up, up, hipMemcpyHostToDevice, S.stream)) != hipSuccess ||
      (e = hipMemsetAsync(derr, 0, 4, S.stream)) != hipSuccess)
    return fail("upload", e);
  mat_locate_kernel<<<grid, kMatThreads, 0, S.stream>>>(d_arena, d_offsets, files, mm, sp, nm, locs, cnt, derr);
  if ((e = hipGetLastError()) != hipSuccess) return fail("mat_locate_kernel", e);
  size_t sb = scan_bytes;
  if ((e = hipcub::DeviceScan::ExclusiveSum(S.d_work + o_scan, sb, cnt, pref, int(nm) + 1, S.stream)) != hipSuccess)
    return fail("scan", e);
  if ((e = hipMemcpyAsync(S.h_tot, pref + nm, 8, hipMemcpyDeviceToHost, S.stream)) != hipSuccess ||
      (e = hipMemcpyAsync(S.h_tot + 1, derr, 4, hipMemcpyDeviceToHost, S.stream)) != hipSuccess ||
      (e = wait()) != hipSuccess)
    return fail("totals", e);
  const uint64_t tot = S.h_tot[0];
  const uint64_t n_text = tot >> 32, n_lines = uint32_t(tot);
  if (uint32_t(S.h_tot[1]) != 0) {
    *err = "FindingMaterializer: line search and line count disagree (mat_locate_kernel)";
    return false;
  }
  if (n_text > S.text_bound || n_lines > uint64_t(nm) * 4) {
    *err = "FindingMaterializer: text / line totals past their bounds";
    return false;
  }
  if ((e = GrowHost(&S.h_lines, &S.h_lines_cap, size_t(n_lines) * sizeof(LineOut))) != hipSuccess ||
      (e = GrowHost(&S.h_text, &S.h_text_cap, size_t(n_text) + 64)) != hipSuccess)
    return fail("read-back buffers", e);
  mat_write_kernel<<<grid, kMatThreads, 0, S.stream>>>(d_arena, d_offsets, files, mm, sp, nm, locs, pref, S.d_find,
                                                       S.d_lines, S.d_text);
  if ((e = hipGetLastError()) != hipSuccess) return fail("mat_write_kernel", e);
  if ((e = hipMemcpyAsync(S.h_find, S.d_find, size_t(nm) * sizeof(FindingOut), hipMemcpyDeviceToHost, S.stream)) !=
          hipSuccess ||
      (e = hipMemcpyAsync(S.h_pref, pref, (size_t(nm) + 1) * 8, hipMemcpyDeviceToHost, S.stream)) != hipSuccess ||
      (n_lines && (e = hipMemcpyAsync(S.h_lines, S.d_lines, size_t(n_lines) * sizeof(LineOut), hipMemcpyDeviceToHost,
                                      S.stream)) != hipSuccess) ||
      (n_text && (e = hipMemcpyAsync(S.h_text, S.d_text, size_t(n_text), hipMemcpyDeviceToHost, S.stream)) !=
                     hipSuccess) ||
      (e = wait()) != hipSuccess)
    return fail("read-back", e);
  return true;
}

}  // namespace tsg
