// gfx950 kernels of the secret-scanning hot path.
//
//  K0 chunk_map   : chunk -> file index (one thread per file)
//  K1 scan        : streams every arena byte once (16-B loads), runs the
//                   case-folded Aho-Corasick DFA over keywords ∪ anchors held
//                   in LDS, sets per-file keyword bits (exact MatchKeywords,
//                   scanner.go:174-186), records anchor hits, counts '\n' per
//                   chunk and flags files holding U+0130/U+212A/U+017F.
//  K2 verify      : one lane per anchor hit; gate check, then the rule's
//                   relaxed shift-and NFA from the hit's start window;
//                   an accept emits a candidate window for the exact host pass
//                   (replaces the whole-file regexp sweeps, scanner.go:102-148).
//  K3 full-scan   : (special file x rule) and (file x unanchored rule) tasks:
//                   NFA with injection at every byte; an accept makes the
//                   whole file a candidate.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "engine.h"

namespace tsg {

namespace {

constexpr int kScanThreads = 512;
constexpr int kHitBuf = 2048;  // records per workgroup LDS staging buffer
constexpr uint32_t kKwCacheWords = 4;

#define HIP_OK(x)                                                   \
  do {                                                              \
    hipError_t e_ = (x);                                            \
    if (e_ != hipSuccess) {                                         \
      err_ = std::string(#x) + ": " + hipGetErrorString(e_);        \
      return false;                                                 \
    }                                                               \
  } while (0)

struct ScanParams {
  const uint8_t* arena;
  uint64_t n_bytes;
  const uint64_t* off;
  uint32_t n_files;
  const uint32_t* chunk_file;
  uint64_t n_chunks;
  const uint8_t* cmap;
  const uint16_t* trans;
  const uint32_t* out_off;
  const uint32_t* out_items;
  uint32_t n_states, n_classes, warm, kw_words;
  uint32_t* kwbits;
  uint32_t* flags;
  uint16_t* nl;
  uint32_t* hits;
  uint32_t hit_cap;
  uint32_t* counters;
  uint32_t* special;
  uint32_t special_cap;
};

__global__ void chunk_map_kernel(const uint64_t* __restrict__ off, uint32_t n_files,
                                 uint32_t* __restrict__ chunk_file) {
  for (uint32_t f = blockIdx.x * blockDim.x + threadIdx.x; f < n_files; f += gridDim.x * blockDim.x) {
    uint64_t s = off[f], e = off[f + 1];
    if (s >= e) continue;
    for (uint64_t c = (s + kChunk - 1) / kChunk; c * kChunk < e; c++) chunk_file[c] = f;
  }
}

struct LaneState {
  uint32_t state;
  uint32_t skip;
  uint32_t special;
  uint32_t kw_cache[kKwCacheWords];
};

__device__ __noinline__ void emit_outputs(const ScanParams& P, uint32_t st, uint32_t f, uint64_t fs,
                                          uint64_t end, LaneState& L, uint32_t* s_hits,
                                          uint32_t* s_nhits) {
  uint32_t a = P.out_off[st], b = P.out_off[st + 1];
  for (uint32_t j = a; j < b; j++) {
    uint32_t item = P.out_items[j];
    uint32_t id = item & 0x0FFFFFFFu;
    if ((item >> 28) == 0) {  // keyword
      uint32_t w = id >> 5, bit = 1u << (id & 31);
      if (P.kw_words <= kKwCacheWords) {
        uint32_t cur = w == 0 ? L.kw_cache[0] : w == 1 ? L.kw_cache[1] : w == 2 ? L.kw_cache[2] : L.kw_cache[3];
        if (!(cur & bit)) {
          if (w == 0) L.kw_cache[0] |= bit;
          else if (w == 1) L.kw_cache[1] |= bit;
          else if (w == 2) L.kw_cache[2] |= bit;
          else L.kw_cache[3] |= bit;
          atomicOr(&P.kwbits[uint64_t(f) * P.kw_words + w], bit);
        }
      } else {
        uint32_t* p = &P.kwbits[uint64_t(f) * P.kw_words + w];
        if (!(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(p, bit);
      }
    } else {  // anchor hit: (file, file-relative end, anchor id)
      uint32_t k = atomicAdd(s_nhits, 1u);
      uint32_t rel = uint32_t(end - fs);
      if (k < uint32_t(kHitBuf)) {
        s_hits[3 * k + 0] = f;
        s_hits[3 * k + 1] = rel;
        s_hits[3 * k + 2] = id;
      } else {
        uint32_t g = atomicAdd(&P.counters[0], 1u);
        if (g < P.hit_cap) {
          P.hits[3ull * g + 0] = f;
          P.hits[3ull * g + 1] = rel;
          P.hits[3ull * g + 2] = id;
        } else {
          P.counters[3] = 1;
        }
      }
    }
  }
}

// Resolve the three bytes whose multi-byte sequence can lower to / fold with ASCII.
__device__ __noinline__ uint32_t fold_special(const ScanParams& P, const uint8_t* cmap, uint32_t cls,
                                              uint64_t pos, uint64_t fe, LaneState& L) {
  const uint8_t* a = P.arena;
  if (cls == kClsFoldI) {  // C4 B0 = U+0130, bytes.ToLower -> 'i'
    if (pos + 1 < fe && a[pos + 1] == 0xB0) {
      L.skip = 1;
      L.special = 1;
      return cmap['i'];
    }
  } else if (cls == kClsFoldK) {  // E2 84 AA = U+212A, lowers to 'k'
    if (pos + 2 < fe && a[pos + 1] == 0x84 && a[pos + 2] == 0xAA) {
      L.skip = 2;
      L.special = 1;
      return cmap['k'];
    }
  } else {  // C5 BF = U+017F, folds with 's' under (?i) but lowers to itself
    if (pos + 1 < fe && a[pos + 1] == 0xBF) {
      L.skip = 1;
      L.special = 1;
      return 0;
    }
  }
  return 0;
}

template <bool kOut>
__device__ __forceinline__ void ac_step(const ScanParams& P, const uint16_t* __restrict__ T,
                                        const uint8_t* __restrict__ cmap, uint32_t b, uint64_t pos,
                                        uint32_t f, uint64_t fs, uint64_t fe, LaneState& L,
                                        uint32_t* s_hits, uint32_t* s_nhits) {
  if (L.skip) {
    L.skip--;
    return;
  }
  uint32_t cls = cmap[b];
  if (cls >= kClsFoldI) cls = fold_special(P, cmap, cls, pos, fe, L);
  uint32_t e = T[L.state * P.n_classes + cls];
  L.state = e & 0x7FFFu;
  if (kOut && (e & kAcOutFlag)) emit_outputs(P, L.state, f, fs, pos + 1 + L.skip, L, s_hits, s_nhits);
}

template <bool kLdsTable>
__global__ __launch_bounds__(kScanThreads) void scan_kernel(ScanParams P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  size_t tbytes = kLdsTable ? ((size_t(P.n_states) * P.n_classes * 2 + 15) & ~size_t(15)) : 0;
  uint16_t* s_trans = reinterpret_cast<uint16_t*>(smem);
  uint8_t* s_cmap = smem + tbytes;
  uint32_t* s_hits = reinterpret_cast<uint32_t*>(smem + tbytes + 256);
  uint32_t* s_nhits = s_hits + 3 * kHitBuf;
  uint32_t* s_base = s_nhits + 1;
  const int tid = threadIdx.x;
  if (kLdsTable) {
    const uint4* src = reinterpret_cast<const uint4*>(P.trans);
    uint4* dst = reinterpret_cast<uint4*>(s_trans);
    size_t n16 = tbytes / 16;
    for (size_t i = tid; i < n16; i += blockDim.x) dst[i] = src[i];
  }
  for (int i = tid; i < 256; i += blockDim.x) s_cmap[i] = P.cmap[i];
  if (tid == 0) *s_nhits = 0;
  __syncthreads();
  const uint16_t* T = kLdsTable ? s_trans : P.trans;

  for (uint64_t tile = blockIdx.x; tile * blockDim.x < P.n_chunks; tile += gridDim.x) {
    uint64_t c = tile * blockDim.x + tid;
    if (c < P.n_chunks) {
      uint64_t b0 = c * kChunk;
      uint64_t b1 = b0 + kChunk < P.n_bytes ? b0 + kChunk : P.n_bytes;
      uint32_t f = P.chunk_file[c];
      uint32_t nl = 0;
      LaneState L;
      while (f < P.n_files) {
        uint64_t fs = P.off[f], fe = P.off[f + 1];
        if (fs >= b1) break;
        uint64_t seg0 = fs > b0 ? fs : b0;
        uint64_t seg1 = fe < b1 ? fe : b1;
        if (seg0 < seg1) {
          L.state = 0;
          L.skip = 0;
          L.special = 0;
          L.kw_cache[0] = L.kw_cache[1] = L.kw_cache[2] = L.kw_cache[3] = 0;
          if (seg0 > fs) {
            // warm-up: the DFA state depends only on the last max_len-1 symbols
            uint64_t w = seg0 - fs > P.warm ? seg0 - P.warm : fs;
            for (uint64_t p = w; p < seg0; p++)
              ac_step<false>(P, T, s_cmap, P.arena[p], p, f, fs, fe, L, s_hits, s_nhits);
            if (L.special && w > fs) {  // folded runes shorten symbols: re-warm 3x longer
              uint64_t w3 = seg0 - fs > 3ull * P.warm ? seg0 - 3ull * P.warm : fs;
              L.state = 0;
              L.skip = 0;
              for (uint64_t p = w3; p < seg0; p++)
                ac_step<false>(P, T, s_cmap, P.arena[p], p, f, fs, fe, L, s_hits, s_nhits);
            }
            L.special = 0;
          }
          for (uint64_t p = seg0 & ~uint64_t(15); p < seg1; p += 16) {
            uint4 v = *reinterpret_cast<const uint4*>(P.arena + p);
            const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 16; k++) {
              uint64_t pos = p + k;
              uint32_t b = (wd[k >> 2] >> ((k & 3) * 8)) & 0xFFu;
              if (pos >= seg0 && pos < seg1) {
                nl += (b == '\n');
                ac_step<true>(P, T, s_cmap, b, pos, f, fs, fe, L, s_hits, s_nhits);
              }
            }
          }
          if (L.special) {
            if (atomicOr(&P.flags[f], 1u) == 0) {
              uint32_t k = atomicAdd(&P.counters[2], 1u);
              if (k < P.special_cap) P.special[k] = f;
            }
          }
        }
        if (fe > b1) break;
        f++;
      }
      P.nl[c] = uint16_t(nl);
    }
    __syncthreads();
    uint32_t nh = *s_nhits < uint32_t(kHitBuf) ? *s_nhits : uint32_t(kHitBuf);
    if (nh) {
      if (tid == 0) *s_base = atomicAdd(&P.counters[0], nh);
      __syncthreads();
      uint32_t base = *s_base;
      for (uint32_t i = tid; i < nh; i += blockDim.x) {
        uint32_t g = base + i;
        if (g < P.hit_cap) {
          P.hits[3ull * g + 0] = s_hits[3 * i + 0];
          P.hits[3ull * g + 1] = s_hits[3 * i + 1];
          P.hits[3ull * g + 2] = s_hits[3 * i + 2];
        } else {
          P.counters[3] = 1;
        }
      }
    }
    __syncthreads();
    if (tid == 0) *s_nhits = 0;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// relaxed NFA (extended shift-and)
// ---------------------------------------------------------------------------
struct NfaParams {
  const uint8_t* arena;
  const uint64_t* off;
  uint32_t n_files;
  const uint16_t* nl;
  const AnchorInfo* anchors;
  const RuleGpu* rules;
  const uint32_t* rule_kw;
  const uint32_t* kwbits;
  uint32_t kw_words;
  const uint32_t* flags;
  const uint64_t* nfa;
  const uint32_t* hits;
  uint32_t hit_cap;
  uint32_t* counters;
  Candidate* cands;
  uint32_t cand_cap;
  const uint32_t* special;
  uint32_t special_cap;
  const uint32_t* regex_rules;
  uint32_t n_regex_rules;
  const uint32_t* fullscan_rules;
  uint32_t n_fullscan_rules;
};

// Returns true at the first position whose state reaches a final position.
// Injection (a match may start here) is on for positions in [start, inj_hi].
template <int W>
__device__ bool nfa_run(const uint8_t* __restrict__ s, int64_t len, int64_t start, int64_t inj_hi,
                        const uint64_t* __restrict__ tab) {
  uint64_t O[W], Lp[W], F[W], D[W];
#pragma unroll
  for (int w = 0; w < W; w++) {
    O[w] = tab[w];
    Lp[w] = tab[W + w];
    F[w] = tab[2 * W + w];
    D[w] = 0;
  }
  const uint64_t* B = tab + 3 * W;
  for (int64_t pos = start; pos < len; pos++) {
    uint32_t b = s[pos];
    uint64_t carry = pos <= inj_hi ? 1 : 0;
    uint64_t T[W];
#pragma unroll
    for (int w = 0; w < W; w++) {
      T[w] = (D[w] << 1) | carry | (D[w] & Lp[w]);
      carry = D[w] >> 63;
    }
    uint64_t c = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      uint64_t x = T[w] & O[w];
      uint64_t s1 = O[w] + x;
      uint64_t c1 = s1 < O[w];
      uint64_t s2 = s1 + c;
      uint64_t c2 = s2 < s1;
      T[w] |= s2 ^ O[w];
      c = c1 | c2;
    }
    const uint64_t* Bb = B + size_t(b) * W;
    bool keep = (b & 0xC0u) == 0x80u;  // UTF-8 continuation: also stay
    uint64_t acc = 0, alive = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      uint64_t nd = (T[w] & Bb[w]) | (keep ? D[w] : 0);
      D[w] = nd;
      acc |= nd & F[w];
      alive |= nd;
    }
    if (acc) return true;
    if (!alive && pos >= inj_hi) return false;
  }
  return false;
}

__device__ bool nfa_dispatch(int words, const uint8_t* s, int64_t len, int64_t start, int64_t inj_hi,
                             const uint64_t* tab) {
  switch (words) {
    case 1: return nfa_run<1>(s, len, start, inj_hi, tab);
    case 2: return nfa_run<2>(s, len, start, inj_hi, tab);
    case 3: return nfa_run<3>(s, len, start, inj_hi, tab);
    default: return nfa_run<4>(s, len, start, inj_hi, tab);
  }
}

__device__ bool gate_open(const NfaParams& P, const RuleGpu& rg, uint32_t f) {
  if (rg.gate != kGateKeywords) return true;  // always / host-verified
  const uint32_t* kb = P.kwbits + uint64_t(f) * P.kw_words;
  for (uint32_t i = 0; i < rg.kw_cnt; i++) {
    uint32_t id = P.rule_kw[rg.kw_off + i];
    if (kb[id >> 5] & (1u << (id & 31))) return true;
  }
  return false;
}

__device__ int64_t count_nl(const NfaParams& P, uint64_t a, uint64_t b) {  // '\n' in arena [a, b)
  int64_t n = 0;
  uint64_t ca = (a + kChunk - 1) / kChunk, cb = b / kChunk;
  if (ca >= cb) {
    for (uint64_t p = a; p < b; p++) n += P.arena[p] == '\n';
    return n;
  }
  for (uint64_t p = a; p < ca * kChunk; p++) n += P.arena[p] == '\n';
  for (uint64_t c = ca; c < cb; c++) n += P.nl[c];
  for (uint64_t p = cb * kChunk; p < b; p++) n += P.arena[p] == '\n';
  return n;
}

__device__ void emit_candidate(const NfaParams& P, uint32_t f, uint32_t r, int64_t wlo, int64_t whi,
                               int64_t nlb) {
  uint32_t k = atomicAdd(&P.counters[1], 1u);
  if (k < P.cand_cap) {
    Candidate c;
    c.file = f;
    c.rule = r;
    c.wlo = wlo;
    c.whi = whi;
    c.nl_before = nlb;
    P.cands[k] = c;
  } else {
    P.counters[4] = 1;
  }
}

__global__ __launch_bounds__(256) void verify_kernel(NfaParams P) {
  uint32_t n = P.counters[0] < P.hit_cap ? P.counters[0] : P.hit_cap;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    uint32_t f = P.hits[3ull * i], end = P.hits[3ull * i + 1], aid = P.hits[3ull * i + 2];
    if (P.flags[f] & 1u) continue;  // special file: handled by full-scan tasks
    AnchorInfo a = P.anchors[aid];
    RuleGpu rg = P.rules[a.rule];
    if (!gate_open(P, rg, f)) continue;
    int64_t lit = int64_t(end) - int64_t(a.lit_len);
    int64_t whi = lit - a.off_lo;
    if (whi < 0) continue;
    int64_t wlo = lit - a.off_hi;
    if (wlo < 0) wlo = 0;
    uint64_t fs = P.off[f];
    int64_t len = int64_t(P.off[f + 1] - fs);
    bool acc = rg.nfa_words == 0 ||
               nfa_dispatch(rg.nfa_words, P.arena + fs, len, wlo, whi, P.nfa + rg.nfa_off);
    if (acc) emit_candidate(P, f, a.rule, wlo, whi, count_nl(P, fs, fs + uint64_t(wlo)));
  }
}

__global__ __launch_bounds__(256) void fullscan_kernel(NfaParams P) {
  uint32_t ns = P.counters[2] < P.special_cap ? P.counters[2] : P.special_cap;
  uint64_t t_special = uint64_t(ns) * P.n_regex_rules;
  uint64_t total = t_special + uint64_t(P.n_files) * P.n_fullscan_rules;
  for (uint64_t t = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; t < total;
       t += uint64_t(gridDim.x) * blockDim.x) {
    uint32_t f, r;
    if (t < t_special) {
      f = P.special[t / P.n_regex_rules];
      r = P.regex_rules[t % P.n_regex_rules];
    } else {
      uint64_t u = t - t_special;
      f = uint32_t(u / P.n_fullscan_rules);
      r = P.fullscan_rules[u % P.n_fullscan_rules];
      if (P.flags[f] & 1u) continue;  // already covered by the special tasks
    }
    RuleGpu rg = P.rules[r];
    if (!gate_open(P, rg, f)) continue;
    uint64_t fs = P.off[f];
    int64_t len = int64_t(P.off[f + 1] - fs);
    bool acc = rg.nfa_words == 0 ||
               nfa_dispatch(rg.nfa_words, P.arena + fs, len, 0, len, P.nfa + rg.nfa_off);
    if (acc) emit_candidate(P, f, r, 0, len, 0);
  }
}

template <typename T>
bool Upload(std::string* err, T** dst, const T* src, size_t n) {
  size_t bytes = std::max<size_t>(n * sizeof(T), 16);
  if (hipMalloc(dst, bytes + 16) != hipSuccess) {
    *err = "hipMalloc failed for tables";
    return false;
  }
  if (n && hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) {
    *err = "hipMemcpy failed for tables";
    return false;
  }
  return true;
}

}  // namespace

GpuEngine::GpuEngine(const CompiledRules& cr, int device) : device_(device) {
  if (hipSetDevice(device) != hipSuccess) {
    err_ = "hipSetDevice failed (no HIP device?)";
    return;
  }
  if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) {
    err_ = "hipStreamCreate failed";
    return;
  }
  for (auto& e : ev_) hipEventCreate(&e);
  n_states_ = cr.n_states;
  n_classes_ = cr.n_classes;
  max_pat_len_ = cr.max_pat_len;
  kw_words_ = std::max<uint32_t>(1, cr.kw_words());
  n_rules_ = uint32_t(cr.rules.size());
  for (uint32_t r = 0; r < n_rules_; r++) {
    if (!cr.rules[r].has_regex) continue;
    regex_rules_.push_back(r);
    if (!cr.rules[r].anchored) fullscan_rules_.push_back(r);
  }
  n_fullscan_rules_ = uint32_t(fullscan_rules_.size());
  // pad the transition table to 16 B for the vectorised LDS fill
  std::vector<uint16_t> trans = cr.trans;
  trans.resize(((trans.size() * 2 + 15) & ~size_t(15)) / 2, 0);
  if (!Upload(&err_, &d_cmap_, cr.cmap, 256) || !Upload(&err_, &d_trans_, trans.data(), trans.size()) ||
      !Upload(&err_, &d_out_off_, cr.out_off.data(), cr.out_off.size()) ||
      !Upload(&err_, &d_out_items_, cr.out_items.data(), cr.out_items.size()) ||
      !Upload(&err_, &d_anchors_, cr.anchors.data(), cr.anchors.size()) ||
      !Upload(&err_, &d_rules_, cr.rules.data(), cr.rules.size()) ||
      !Upload(&err_, &d_rule_kw_, cr.rule_kw.data(), cr.rule_kw.size()) ||
      !Upload(&err_, &d_nfa_, cr.nfa.data(), cr.nfa.size()) ||
      !Upload(&err_, &d_regex_rules_, regex_rules_.data(), regex_rules_.size()) ||
      !Upload(&err_, &d_fullscan_rules_, fullscan_rules_.data(), fullscan_rules_.size()))
    return;
  if (hipMalloc(&d_counters_, 64) != hipSuccess) {
    err_ = "hipMalloc counters";
    return;
  }
  size_t tbytes = (size_t(n_states_) * n_classes_ * 2 + 15) & ~size_t(15);
  size_t rest = 256 + size_t(3 * kHitBuf + 4) * 4;
  table_in_lds_ = tbytes + rest <= 150 * 1024;
  lds_bytes_ = (table_in_lds_ ? tbytes : 0) + rest;
  if (table_in_lds_) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&scan_kernel<true>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_bytes_));
  } else {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&scan_kernel<false>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_bytes_));
  }
}

GpuEngine::~GpuEngine() {
  hipSetDevice(device_);
  void* ps[] = {d_cmap_, d_trans_, d_out_off_, d_out_items_, d_anchors_, d_rules_, d_rule_kw_, d_nfa_,
                d_regex_rules_, d_fullscan_rules_, d_counters_, d_chunk_file_, d_nl_, d_kw_, d_flags_,
                d_hits_, d_cands_, d_special_, d_arena_stage_, d_off_stage_};
  for (void* p : ps)
    if (p) hipFree(p);
  for (auto& e : ev_)
    if (e) hipEventDestroy(e);
  if (stream_) hipStreamDestroy(stream_);
}

bool GpuEngine::Ensure(void** p, size_t* cap, size_t need) {
  if (*p && *cap >= need) return true;
  if (*p) hipFree(*p);
  *p = nullptr;
  size_t n = std::max<size_t>(need, 64);
  HIP_OK(hipMalloc(p, n));
  *cap = n;
  return true;
}

bool GpuEngine::RunHost(const uint8_t* h_arena, uint64_t n_bytes, const uint64_t* h_offsets, uint32_t n_files,
                        std::vector<Candidate>* cands, BatchStats* st) {
  HIP_OK(hipSetDevice(device_));
  if (!Ensure(&d_arena_stage_, &cap_arena_stage_, n_bytes + 64)) return false;
  if (!Ensure(&d_off_stage_, &cap_off_stage_, (size_t(n_files) + 1) * 8)) return false;
  if (n_bytes) HIP_OK(hipMemcpyAsync(d_arena_stage_, h_arena, n_bytes, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipMemsetAsync(static_cast<uint8_t*>(d_arena_stage_) + n_bytes, 0, 64, stream_));
  HIP_OK(hipMemcpyAsync(d_off_stage_, h_offsets, (size_t(n_files) + 1) * 8, hipMemcpyHostToDevice, stream_));
  return Run(static_cast<const uint8_t*>(d_arena_stage_), n_bytes, static_cast<const uint64_t*>(d_off_stage_),
             n_files, cands, st);
}

bool GpuEngine::Run(const uint8_t* d_arena, uint64_t n_bytes, const uint64_t* d_offsets, uint32_t n_files,
                    std::vector<Candidate>* cands, BatchStats* st) {
  HIP_OK(hipSetDevice(device_));
  cands->clear();
  BatchStats local;
  if (!st) st = &local;
  *st = BatchStats();
  st->bytes = n_bytes;
  st->files = n_files;
  if (n_files == 0) return true;
  uint64_t n_chunks = (n_bytes + kChunk - 1) / kChunk;
  if (n_chunks == 0) n_chunks = 1;
  if (hit_cap_ == 0) hit_cap_ = uint32_t(std::min<uint64_t>(std::max<uint64_t>(n_bytes / 64, 1 << 16), 1u << 30));
  if (cand_cap_ == 0) cand_cap_ = 1 << 16;
  for (int attempt = 0; attempt < 8; attempt++) {
    if (!Ensure(&d_chunk_file_, &cap_chunk_file_, n_chunks * 4) || !Ensure(&d_nl_, &cap_nl_, n_chunks * 2) ||
        !Ensure(&d_kw_, &cap_kw_, size_t(n_files) * kw_words_ * 4) ||
        !Ensure(&d_flags_, &cap_flags_, size_t(n_files) * 4) ||
        !Ensure(&d_special_, &cap_special_, size_t(n_files) * 4) ||
        !Ensure(&d_hits_, &cap_hits_, size_t(hit_cap_) * 12) ||
        !Ensure(&d_cands_, &cap_cands_, size_t(cand_cap_) * sizeof(Candidate)))
      return false;
    HIP_OK(hipMemsetAsync(d_kw_, 0, size_t(n_files) * kw_words_ * 4, stream_));
    HIP_OK(hipMemsetAsync(d_flags_, 0, size_t(n_files) * 4, stream_));
    HIP_OK(hipMemsetAsync(d_counters_, 0, 64, stream_));
    HIP_OK(hipMemsetAsync(d_chunk_file_, 0, n_chunks * 4, stream_));
    {
      uint32_t blocks = std::min<uint32_t>((n_files + 255) / 256, 4096);
      chunk_map_kernel<<<blocks, 256, 0, stream_>>>(d_offsets, n_files, static_cast<uint32_t*>(d_chunk_file_));
    }
    ScanParams sp;
    sp.arena = d_arena;
    sp.n_bytes = n_bytes;
    sp.off = d_offsets;
    sp.n_files = n_files;
    sp.chunk_file = static_cast<const uint32_t*>(d_chunk_file_);
    sp.n_chunks = n_chunks;
    sp.cmap = d_cmap_;
    sp.trans = d_trans_;
    sp.out_off = d_out_off_;
    sp.out_items = d_out_items_;
    sp.n_states = n_states_;
    sp.n_classes = n_classes_;
    sp.warm = max_pat_len_ > 0 ? max_pat_len_ - 1 : 0;
    sp.kw_words = kw_words_;
    sp.kwbits = static_cast<uint32_t*>(d_kw_);
    sp.flags = static_cast<uint32_t*>(d_flags_);
    sp.nl = static_cast<uint16_t*>(d_nl_);
    sp.hits = static_cast<uint32_t*>(d_hits_);
    sp.hit_cap = hit_cap_;
    sp.counters = d_counters_;
    sp.special = static_cast<uint32_t*>(d_special_);
    sp.special_cap = n_files;
    uint64_t tiles = (n_chunks + kScanThreads - 1) / kScanThreads;
    uint32_t per_cu = std::max<uint32_t>(1, uint32_t((160 * 1024) / lds_bytes_));
    uint32_t grid = uint32_t(std::min<uint64_t>(tiles, uint64_t(256) * per_cu));
    HIP_OK(hipEventRecord(ev_[0], stream_));
    if (table_in_lds_)
      scan_kernel<true><<<grid, kScanThreads, lds_bytes_, stream_>>>(sp);
    else
      scan_kernel<false><<<grid, kScanThreads, lds_bytes_, stream_>>>(sp);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev_[1], stream_));
    NfaParams np;
    np.arena = d_arena;
    np.off = d_offsets;
    np.n_files = n_files;
    np.nl = static_cast<const uint16_t*>(d_nl_);
    np.anchors = d_anchors_;
    np.rules = d_rules_;
    np.rule_kw = d_rule_kw_;
    np.kwbits = static_cast<const uint32_t*>(d_kw_);
    np.kw_words = kw_words_;
    np.flags = static_cast<const uint32_t*>(d_flags_);
    np.nfa = d_nfa_;
    np.hits = static_cast<const uint32_t*>(d_hits_);
    np.hit_cap = hit_cap_;
    np.counters = d_counters_;
    np.cands = static_cast<Candidate*>(d_cands_);
    np.cand_cap = cand_cap_;
    np.special = static_cast<const uint32_t*>(d_special_);
    np.special_cap = n_files;
    np.regex_rules = d_regex_rules_;
    np.n_regex_rules = uint32_t(regex_rules_.size());
    np.fullscan_rules = d_fullscan_rules_;
    np.n_fullscan_rules = n_fullscan_rules_;
    verify_kernel<<<2048, 256, 0, stream_>>>(np);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev_[2], stream_));
    if (np.n_regex_rules > 0) {
      fullscan_kernel<<<1024, 256, 0, stream_>>>(np);
      HIP_OK(hipGetLastError());
    }
    HIP_OK(hipEventRecord(ev_[3], stream_));
    uint32_t cnt[8];
    HIP_OK(hipMemcpyAsync(cnt, d_counters_, sizeof(cnt), hipMemcpyDeviceToHost, stream_));
    HIP_OK(hipStreamSynchronize(stream_));
    st->hits = cnt[0];
    st->special_files = cnt[2];
    st->hit_overflow = cnt[3] != 0;
    st->cand_overflow = cnt[4] != 0;
    if (st->hit_overflow) {  // grow and rescan (correctness first)
      hit_cap_ = uint32_t(std::min<uint64_t>(uint64_t(cnt[0]) + cnt[0] / 4 + 1024, 0xFFFFFFF0u));
      continue;
    }
    if (st->cand_overflow) {
      cand_cap_ = uint32_t(std::min<uint64_t>(uint64_t(cnt[1]) + cnt[1] / 4 + 1024, 0xFFFFFFF0u));
      continue;
    }
    st->candidates = cnt[1];
    cands->resize(cnt[1]);
    if (cnt[1]) {
      HIP_OK(hipMemcpyAsync(cands->data(), d_cands_, size_t(cnt[1]) * sizeof(Candidate), hipMemcpyDeviceToHost,
                            stream_));
      HIP_OK(hipStreamSynchronize(stream_));
    }
    hipEventElapsedTime(&st->ms_scan, ev_[0], ev_[1]);
    hipEventElapsedTime(&st->ms_verify, ev_[1], ev_[2]);
    hipEventElapsedTime(&st->ms_fullscan, ev_[2], ev_[3]);
    hipEventElapsedTime(&st->ms_total, ev_[0], ev_[3]);
    return true;
  }
  err_ = "candidate buffers kept overflowing";
  return false;
}

}  // namespace tsg
