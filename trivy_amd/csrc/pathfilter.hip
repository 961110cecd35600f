// GPU allow-path prefilter (pathfilter.h).
#include "pathfilter.h"

#include <chrono>
#include <cstring>
#include <thread>

namespace tsg {

bool BuildPathTable(const std::vector<std::pair<std::string, uint32_t>>& lits, PathTable* t) {
  std::memset(t, 0, sizeof(*t));
  uint32_t w = 0, bit = 0;
  for (auto& [lit, rule] : lits) {
    const size_t k = lit.size();
    if (k < 2 || k > 64 || rule >= 64) return false;
    if (bit + k > 64) {  // a literal never crosses a word
      w++;
      bit = 0;
    }
    if (w >= 4) return false;
    t->S[w] |= uint64_t(1) << bit;
    for (size_t j = 0; j < k; j++) {
      const uint8_t c = uint8_t(lit[j]);
      if (c >= 'A' && c <= 'Z') return false;  // the literals are lowercased (Matcher::lits)
      t->B[c][w] |= uint64_t(1) << (bit + j);
    }
    t->E[w] |= uint64_t(1) << (bit + k - 1);
    t->rule_of[w * 64 + bit + k - 1] = uint8_t(rule);
    bit += uint32_t(k);
  }
  t->words = w + 1;
  return !lits.empty();
}

namespace {

constexpr int kPathThreads = 256;

__global__ __launch_bounds__(kPathThreads) void path_filter_kernel(const uint8_t* __restrict__ paths,
                                                                   const uint64_t* __restrict__ off, uint32_t n,
                                                                   const PathTable* __restrict__ T,
                                                                   uint32_t* __restrict__ cnt,
                                                                   uint32_t* __restrict__ cnt_next,
                                                                   PathHit* __restrict__ out) {
  // the counter of this slot's next launch (stream-ordered after this one): no
  // fill kernel per call
  if (blockIdx.x == 0 && threadIdx.x == 0) *cnt_next = 0;
  __shared__ uint64_t sB[256][4];
  __shared__ uint8_t s_rule[256];
  for (uint32_t i = threadIdx.x; i < 256 * 4; i += kPathThreads) (&sB[0][0])[i] = (&T->B[0][0])[i];
  for (uint32_t i = threadIdx.x; i < 256; i += kPathThreads) s_rule[i] = T->rule_of[i];
  __syncthreads();
  uint64_t S[4], E[4];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    S[w] = T->S[w];
    E[w] = T->E[w];
  }
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t stride = gridDim.x * kPathThreads;
  // whole waves iterate together (the ballot below needs every lane)
  for (uint32_t base = blockIdx.x * kPathThreads + (threadIdx.x & ~63u); base < n; base += stride) {
    const uint32_t i = base + lane;
    uint32_t rec = 0;
    uint64_t rules = 0;
    bool emit = false;
    if (i < n) {
      uint64_t D[4] = {0, 0, 0, 0}, H[4] = {0, 0, 0, 0};
      uint32_t high = 0;
      const uint64_t e = off[i + 1];
      for (uint64_t p = off[i]; p < e; p++) {
        const uint32_t b = paths[p];
        high |= b;
        const uint32_t c = b + ((b - 'A') < 26u ? 32u : 0u);
#pragma unroll
        for (int w = 0; w < 4; w++) {
          D[w] = ((D[w] << 1) | S[w]) & sB[c][w];
          H[w] |= D[w] & E[w];
        }
      }
      if (high & 0x80u) {
        rec = i | kPathNonAscii;
        emit = true;
      } else {
#pragma unroll
        for (int w = 0; w < 4; w++)
          for (uint64_t h = H[w]; h; h &= h - 1) rules |= uint64_t(1) << s_rule[w * 64 + __builtin_ctzll(h)];
        rec = i;
        emit = rules != 0;
      }
    }
    const uint64_t m = __ballot(emit);
    if (m) {
      uint32_t at = 0;
      if (lane == 0) at = atomicAdd(cnt, uint32_t(__popcll(m)));
      at = __shfl(at, 0);
      if (emit) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
        PathHit h;
        h.file = rec;
        h.pad = 0;
        h.rules = rules;
        out[at + below] = h;
      }
    }
  }
}

}  // namespace

PathFilter::PathFilter(int device, const PathTable& t) : device_(device) {
  int lo = 0, hi = 0;
  if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
  bool ok = hipSetDevice(device) == hipSuccess &&
            hipMalloc(reinterpret_cast<void**>(&d_table_), sizeof(PathTable)) == hipSuccess &&
            hipMemcpy(d_table_, &t, sizeof(PathTable), hipMemcpyHostToDevice) == hipSuccess;
  for (Slot& S : slots_)
    ok = ok && hipStreamCreateWithPriority(&S.stream, hipStreamNonBlocking, hi) == hipSuccess &&
         hipEventCreateWithFlags(&S.done, hipEventDisableTiming) == hipSuccess &&
         hipMalloc(reinterpret_cast<void**>(&S.d_cnt), 64) == hipSuccess &&
         hipMemset(S.d_cnt, 0, 64) == hipSuccess &&
         hipHostMalloc(reinterpret_cast<void**>(&S.h_cnt), 64, hipHostMallocDefault) == hipSuccess;
  if (!ok) err_ = "PathFilter: HIP setup failed";
}

PathFilter::~PathFilter() {
  (void)hipSetDevice(device_);
  for (Slot& S : slots_) {
    if (S.d_out) (void)hipFree(S.d_out);
    if (S.h_out) (void)hipHostFree(S.h_out);
    if (S.d_paths) (void)hipFree(S.d_paths);
    if (S.h_stage) (void)hipHostFree(S.h_stage);
    if (S.d_cnt) (void)hipFree(S.d_cnt);
    if (S.h_cnt) (void)hipHostFree(S.h_cnt);
    if (S.done) (void)hipEventDestroy(S.done);
    if (S.stream) (void)hipStreamDestroy(S.stream);
  }
  if (d_table_) (void)hipFree(d_table_);
}

bool PathFilter::RunImpl(const uint8_t* d_paths, const uint64_t* d_off, const uint8_t* h_paths,
                         const uint64_t* h_off, uint32_t n, std::vector<PathHit>* out, std::string* err) {
  out->clear();
  if (n == 0) return true;
  Slot* S = nullptr;
  {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] {
      for (Slot& x : slots_)
        if (!x.busy) return true;
      return false;
    });
    for (Slot& x : slots_)
      if (!x.busy) {
        S = &x;
        break;
      }
    S->busy = true;
  }
  auto release = [&](bool ok) {
    {
      std::lock_guard<std::mutex> g(mu_);
      S->busy = false;
    }
    cv_.notify_one();
    return ok;
  };
  auto fail = [&](const char* what, hipError_t e) {
    *err = std::string("PathFilter: ") + what + ": " + hipGetErrorString(e);
    return release(false);
  };
  // sleep-poll (as GpuEngine::WaitEvent): a spinning wait takes a core from the host pool
  auto wait = [&]() {
    hipError_t e = hipEventRecord(S->done, S->stream);
    if (e != hipSuccess) return e;
    while ((e = hipEventQuery(S->done)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(100));
    return e;
  };
  hipError_t e = hipSetDevice(device_);
  if (e != hipSuccess) return fail("hipSetDevice", e);
  if (S->cap < n) {
    if (S->d_out) (void)hipFree(S->d_out);
    if (S->h_out) (void)hipHostFree(S->h_out);
    S->d_out = nullptr;
    S->h_out = nullptr;
    S->cap = 0;
    if ((e = hipMalloc(reinterpret_cast<void**>(&S->d_out), size_t(n) * sizeof(PathHit))) != hipSuccess ||
        (e = hipHostMalloc(reinterpret_cast<void**>(&S->h_out), size_t(n) * sizeof(PathHit), hipHostMallocDefault)) !=
            hipSuccess)
      return fail("hipMalloc", e);
    S->cap = n;
  }
  if (h_paths) {  // host-packed paths: offsets (rebased to 0) and bytes via pinned staging to HBM
    const uint64_t p0 = h_off[0], nb = h_off[n] - p0, ob = (uint64_t(n) + 1) * 8;
    const uint64_t need = ((ob + 15) & ~uint64_t(15)) + nb;
    if (S->paths_cap < need) {
      if (S->d_paths) (void)hipFree(S->d_paths);
      if (S->h_stage) (void)hipHostFree(S->h_stage);
      S->d_paths = nullptr;
      S->h_stage = nullptr;
      S->paths_cap = S->stage_cap = 0;
      const size_t cap = size_t(need + need / 4 + 4096);
      if ((e = hipMalloc(reinterpret_cast<void**>(&S->d_paths), cap)) != hipSuccess ||
          (e = hipHostMalloc(reinterpret_cast<void**>(&S->h_stage), cap, hipHostMallocDefault)) != hipSuccess)
        return fail("hipMalloc (paths)", e);
      S->paths_cap = S->stage_cap = cap;
    }
    // the previous call's copy out of the staging buffer is done: that call waited for its stream
    uint64_t* so = reinterpret_cast<uint64_t*>(S->h_stage);
    for (uint32_t i = 0; i <= n; i++) so[i] = h_off[i] - p0;
    const uint64_t pb = (ob + 15) & ~uint64_t(15);
    std::memcpy(S->h_stage + pb, h_paths + p0, size_t(nb));
    if ((e = hipMemcpyAsync(S->d_paths, S->h_stage, size_t(pb + nb), hipMemcpyHostToDevice, S->stream)) !=
        hipSuccess)
      return fail("hipMemcpyAsync (paths)", e);
    d_off = reinterpret_cast<const uint64_t*>(S->d_paths);
    d_paths = S->d_paths + pb;
  }
  // this launch's counter was zeroed by the slot's previous launch (or at set-up)
  uint32_t* cnt = S->d_cnt + S->parity;
  uint32_t* cnt_next = S->d_cnt + (1 - S->parity);
  S->parity ^= 1u;
  const uint32_t grid = uint32_t(std::min<uint64_t>((uint64_t(n) + kPathThreads - 1) / kPathThreads, 4096));
  path_filter_kernel<<<grid, kPathThreads, 0, S->stream>>>(d_paths, d_off, n, d_table_, cnt, cnt_next, S->d_out);
  if ((e = hipGetLastError()) != hipSuccess) {
    (void)hipStreamSynchronize(S->stream);  // (a failed launch left cnt_next as it was: clear it for the next call)
    (void)hipMemset(cnt_next, 0, 4);
    return fail("path_filter_kernel", e);
  }
  // the count and as many records as the last call had (+1/8): one round trip when the paths repeat
  const uint32_t guess = std::min<uint32_t>(n, last_k_.load() + last_k_.load() / 8 + 1024);
  if ((e = hipMemcpyAsync(S->h_cnt, cnt, 4, hipMemcpyDeviceToHost, S->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(S->h_out, S->d_out, size_t(guess) * sizeof(PathHit), hipMemcpyDeviceToHost, S->stream)) !=
          hipSuccess ||
      (e = wait()) != hipSuccess)
    return fail("read-back", e);
  const uint32_t k = *S->h_cnt;
  if (k > n) {
    *err = "PathFilter: record count out of range";
    return release(false);
  }
  if (k > guess && ((e = hipMemcpyAsync(S->h_out + guess, S->d_out + guess, size_t(k - guess) * sizeof(PathHit),
                                        hipMemcpyDeviceToHost, S->stream)) != hipSuccess ||
                    (e = wait()) != hipSuccess))
    return fail("record read-back", e);
  last_k_.store(k);
  out->assign(S->h_out, S->h_out + k);
  return release(true);
}

}  // namespace tsg
