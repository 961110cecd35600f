// gfx950 kernels of the secret-scanning hot path.
//
//  K0 chunk_map   : 1-KiB chunk -> file index (one thread per file)
//  K1 filter      : streams every arena byte once (64 B per lane per tile);
//                   bucketed shift-or over 15 item buckets + a newline bucket
//                   (reach table replicated 16x in LDS); records the flagged
//                   16-B blocks and counts '\n' per chunk.
//  K2 confirm     : three compacted wave phases over the flagged blocks:
//                   fires -> core-table item candidates -> exact item check
//                   with file attribution; staged anchor hits, fold-rune
//                   sites and ASCII keyword bits.
//  K2f fold       : one workgroup per fold-rune site (U+212A / U+017F / U+0130):
//                   fold-tolerant item matching in an LDS byte window.
//  K3 verify      : one lane per anchor hit: the rule's relaxed shift-and NFA
//                   from the hit's start window; an accept emits a candidate
//                   window for the exact host pass (replaces the whole-file
//                   regexp sweeps, scanner.go:102-148).
//  K4 full-scan   : (file x unanchored rule) tasks: NFA with injection at
//                   every byte; an accept makes the whole file a candidate.
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <pthread.h>

#include <thread>
#include <type_traits>

#include "engine.h"
#include "xform.h"
#include "filter.h"

namespace tsg {

namespace {

constexpr int kScanThreads = 1024;
constexpr int kScanWaves = kScanThreads / 64;

#define HIP_OK(x)                                                   \
  do {                                                              \
    hipError_t e_ = (x);                                            \
    if (e_ != hipSuccess) {                                         \
      err_ = std::string(#x) + ": " + hipGetErrorString(e_);        \
      return false;                                                 \
    }                                                               \
  } while (0)


// K0: chunk c -> the file holding byte c * kChunk (off[f] <= c * kChunk <
// off[f + 1], so never an empty file).  A thread per run of 16 chunks: a
// binary search over the offsets (L2-resident) for the first, a forward walk
// for the rest, one 64-B store.  (A thread per file left a multi-MiB file's
// thousands of stores to one thread; a search per chunk cost 20 dependent
// loads per chunk, 0.32 ms on C2.)
constexpr uint32_t kK0Run = 16;
// The per-scan clears ride on K0 (they were three hipMemsetAsync fill kernels
// per scan, 103 __amd_rocclr_fillBufferAligned launches per 18 C2 scans in
// profiles/r04final2): the per-file flags and keyword bits, the 16 counters
// and the full-scan list counters.  Every later kernel of the phase is
// stream-ordered after K0.
struct ClearParams {
  uint32_t* flags;     // n_files
  uint32_t* kw;        // n_files x kw_words
  uint64_t n_kw;       // words of kw
  uint32_t* counters;  // 16
  uint32_t* fs_ctr;    // 16, or null
};
__device__ __forceinline__ void clear_words(uint32_t* p, uint64_t n, uint64_t tid, uint64_t nthr) {
  // hipMalloc'd buffers are 256-B aligned: 16-B stores, the last n % 4 words singly
  const uint64_t n4 = n / 4;
  for (uint64_t i = tid; i < n4; i += nthr) reinterpret_cast<uint4*>(p)[i] = make_uint4(0, 0, 0, 0);
  if (tid < n % 4) p[4 * n4 + tid] = 0;
}
__global__ __launch_bounds__(256) void chunk_map_kernel(const uint64_t* __restrict__ off, uint32_t n_files,
                                                        uint64_t n_chunks, uint32_t* __restrict__ chunk_file,
                                                        ClearParams Z) {
  {
    const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x, nthr = uint64_t(gridDim.x) * blockDim.x;
    clear_words(Z.flags, n_files, tid, nthr);
    clear_words(Z.kw, Z.n_kw, tid, nthr);
    if (tid < 16) {
      Z.counters[tid] = 0;
      if (Z.fs_ctr) Z.fs_ctr[tid] = 0;
    }
  }
  const uint64_t n_runs = (n_chunks + kK0Run - 1) / kK0Run;
  for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < n_runs;
       r += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t c0 = r * kK0Run;
    uint64_t x = c0 * kChunk;
    uint32_t lo = 0, hi = n_files;  // the last f with off[f] <= x: off[lo] <= x < off[hi]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (off[mid] <= x) lo = mid;
      else hi = mid;
    }
    uint32_t v[kK0Run];
    uint64_t fe = off[lo + 1];
#pragma unroll
    for (uint32_t i = 0; i < kK0Run; i++) {
      x = (c0 + i) * kChunk;
      while (x >= fe && lo + 1 < n_files) fe = off[++lo + 1];
      v[i] = lo;
    }
    if (c0 + kK0Run <= n_chunks) {  // (the map is 64-B aligned: hipMalloc)
      uint4* d = reinterpret_cast<uint4*>(chunk_file + c0);
#pragma unroll
      for (uint32_t q = 0; q < kK0Run / 4; q++) d[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    } else {
      for (uint32_t i = 0; c0 + i < n_chunks; i++) chunk_file[c0 + i] = v[i];
    }
  }
}

__device__ __forceinline__ uint4 load16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------
// K1: streaming bucketed shift-or filter
// ---------------------------------------------------------------------------
constexpr int kFLane = 64;           // bytes per lane per tile (4 blocks of 16 B)
constexpr int kFBlocks = kFLane / 16;
constexpr int kFTile = 64 * kFLane;  // 4 KiB per wave tile
// LDS per 1024-thread workgroup: 64 KiB reach table + 12 KiB queues + 2 KiB
// newline staging = 78 KiB, so two workgroups share a CU (8 waves per SIMD at
// <= 64 VGPRs): tools/k1x.hip measured 4.98 vs 5.35 ms for one per CU (C2).
constexpr int kFFlushAt = 128;                      // flush the flagged-block queue at >= this many
constexpr int kFQueue = kFFlushAt + 64;             // per-wave queue entries (a block column appends <= 64)
constexpr int kFChunks = kFTile / 1024;             // newline chunks per tile (kChunk = 1 KiB)
#ifndef TSG_K1_NLTILES
#define TSG_K1_NLTILES 16
#endif
constexpr int kFNlTiles = TSG_K1_NLTILES;           // tiles whose newline counts a wave stages in LDS
#ifndef TSG_K1_WGS
#define TSG_K1_WGS 2
#endif
constexpr int kFWgPerCu = TSG_K1_WGS;  // 1: leaves ~80 KiB of LDS per CU to a concurrent scan's confirm kernel
#ifndef TSG_K1_GROUPQ  // flagged blocks compacted once per kFGroup tiles (0: per tile and block column)
#define TSG_K1_GROUPQ 1
#endif
constexpr uint32_t kFGroup = 8;  // tiles per compaction: 4 flag bits each, 32 per lane
#ifndef TSG_K1_READAHEAD
#define TSG_K1_READAHEAD 4
#endif
constexpr uint32_t kFReadAhead = TSG_K1_READAHEAD;  // table rows read ahead of the shift-or chain
constexpr int kFWindow = 6;          // filter window: a fire stays visible for 9 - 6 = 3 bytes
constexpr int kFWords = 4;           // 16 buckets = 4 u32 registers of 8 slots x 4 buckets
constexpr uint32_t kFireBits = 0xFFF00000u;  // slots 5..7 of a register
constexpr uint32_t kNlBits = 0x8888u;        // newline bucket (15 = register 3, lane 3), slots 0..3
static_assert(kChunk % kFLane == 0 && kChunk / kFLane <= 64, "a newline chunk must be whole lane chunks");
static_assert(kFChunks * kChunk == kFTile && kFChunks == 4, "a tile's newline counts are one u64");

struct FilterParams {
  const uint8_t* arena;
  uint64_t n_bytes;
  const uint32_t* reach;  // 256 x 4 u32 (filter.h layout)
  uint32_t diag_mode;     // TSG_DIAG_SCAN: 2 skips the filter (loads + newline count only)
  uint16_t* nl;           // '\n' per 1-KiB chunk
  uint32_t* recs;         // flagged 16-B block indices
  uint32_t rec_cap;
  uint32_t* counters;     // [7] records [8] record overflow
};

// The table row of byte b is 256 B: 16 copies of its 16-B entry, the copy
// chosen by lane & 15, so a wave's ds_read_b128s never conflict.  v_perm puts
// the byte in bits 8..15 and the lane offset in bits 0..7.
__device__ __forceinline__ uint4 reach_read(const uint8_t* sb, uint32_t w, uint32_t k, uint32_t laneoff) {
  return *reinterpret_cast<const uint4*>(sb + __builtin_amdgcn_perm(w, laneoff, 0x0C0C0000u | ((4u + k) << 8)));
}

// R = R << 4 | m, per register: one v_lshl_or_b32 each.  Written as asm so the
// compiler keeps the serial chain instead of re-associating it into shifted
// copies of the table words (which costs ~1.6x the VALU instructions).
__device__ __forceinline__ void reach_apply(const uint4& m, uint32_t* st) {
  asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(st[0]) : "v"(st[0]), "v"(m.x));
  asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(st[1]) : "v"(st[1]), "v"(m.y));
  asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(st[2]) : "v"(st[2]), "v"(m.z));
  asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(st[3]) : "v"(st[3]), "v"(m.w));
}

// '\n' bytes in a word: x = w ^ 0x0A.. is zero exactly in newline bytes; bit 7
// of ((x & 0x7F..) + 0x7F..) | w marks the nonzero ones (bit 7 of x is w's).
__device__ __forceinline__ uint32_t nl_count4(uint32_t w) {
  const uint32_t a = ((w ^ 0x0A0A0A0Au) & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return __popc(~(a | w) & 0x80808080u);
}

__device__ __forceinline__ uint32_t word_of(uint4 v, uint32_t i) {
  return i < 2 ? (i == 0 ? v.x : v.y) : (i == 2 ? v.z : v.w);
}

__device__ __forceinline__ void load_reach_lds(uint8_t* s_reach, const uint32_t* reach, uint32_t copies, int tid,
                                               int nthreads) {
  for (uint32_t i = tid; i < 256 * copies; i += nthreads) {
    const uint32_t b = i / copies;
    reinterpret_cast<uint4*>(s_reach)[i] = reinterpret_cast<const uint4*>(reach)[b];
  }
}

// K1.  A wave owns 4-KiB tiles (grid-strided); lane l streams its 64
// contiguous bytes as 4 x 16-B loads with the next tile's loads in flight.
// The 5 bytes before a lane's chunk come from lane l-1 (lane 0: an 8-B load).
// Per byte: table address by v_perm, one conflict-free ds_read_b128 (issued a
// block ahead of the chain), four v_lshl_or_b32.  Every 3 bytes the top slots
// are AND-ed into the block's accumulator; every 4 bytes the newline bucket's
// 4 slots are popcounted.  Flagged blocks go through a ballot/mbcnt-compacted
// per-wave LDS queue to the global record list (one atomic per 64 records);
// the confirm kernel (K2) checks them exactly.
// (<= 64 VGPRs in both shapes: with one workgroup per CU the other half of the
// VGPRs and LDS go to a concurrent scan's confirm kernel)
__global__ __launch_bounds__(kScanThreads, 8) void filter_kernel(FilterParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t s_reach[65536];
  __shared__ uint32_t s_queue[kScanWaves * kFQueue];
  __shared__ uint64_t s_nl[kScanWaves * kFNlTiles];  // per wave: the last tiles' 4 chunk counts
  const int tid = threadIdx.x;
  load_reach_lds(s_reach, P.reach, 16, tid, blockDim.x);
  __syncthreads();
  const uint32_t lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(uint32_t(tid) >> 6);
  const uint32_t laneoff = (lane & 15) * 16;
  uint32_t* Q = s_queue + wave * kFQueue;
  uint64_t* NL = s_nl + wave * kFNlTiles;
  uint32_t nl_slots = 0;  // wave-uniform: tiles staged in NL
  uint32_t qn = 0;  // wave-uniform
  // Each wave streams one contiguous range of tiles, so lane 0's 8-byte
  // prefix is lane 63's last 8 bytes of the wave's previous tile (carried in
  // scalar registers) -- only the range's first tile loads it.
  const uint64_t n_tiles = (P.n_bytes + kFTile - 1) / kFTile;
  const uint64_t n_waves = uint64_t(gridDim.x) * kScanWaves;
  const uint64_t wid = uint64_t(blockIdx.x) * kScanWaves + wave;
  const uint64_t per = n_tiles / n_waves, extra = n_tiles % n_waves;
  const uint64_t t_begin = wid * per + (wid < extra ? wid : extra);
  const uint64_t t_end = t_begin + per + (wid < extra ? 1 : 0);
  uint4 bufA[kFBlocks], bufB[kFBlocks];
  uint32_t pre_x = 0, pre_y = 0;  // wave-uniform: the 8 bytes before the current tile
  if (t_begin < t_end && t_begin > 0) {
    const uint2 pv = *reinterpret_cast<const uint2*>(P.arena + t_begin * kFTile - 8);
    pre_x = __builtin_amdgcn_readfirstlane(pv.x);
    pre_y = __builtin_amdgcn_readfirstlane(pv.y);
  }
  auto load_tile = [&](uint4* dst, uint64_t tt) {
    // One clamp per lane, no branch (a wave-uniform full-tile branch around
    // the loads cost 1.4 ms on C2): a lane chunk starting inside the arena is
    // readable whole (64 readable bytes past n_bytes), one past it reloads 0.
    const uint64_t b0 = tt * kFTile + uint64_t(lane) * kFLane;
    const uint8_t* lp = P.arena + (b0 < P.n_bytes ? b0 : 0);
#pragma unroll
    for (int j = 0; j < kFBlocks; j++) dst[j] = load16(lp + 16 * j);
  };
  auto flush = [&]() {  // wave-uniform
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&P.counters[7], qn);
    base = __builtin_amdgcn_readfirstlane(base);
    for (uint32_t i = lane; i < qn; i += 64) {
      if (base + i < P.rec_cap) P.recs[base + i] = Q[i];
      else P.counters[8] = 1;
    }
    qn = 0;
  };
#if TSG_K1_GROUPQ
  // Flagged blocks: each lane keeps 4 bits per tile for kFGroup consecutive
  // tiles of its range; one compaction per group appends the group's records
  // to the wave's LDS queue (a DPP wave prefix sum of the lanes' counts, each
  // lane writing its own), and the queue goes to the global list in flushes of
  // >= kFFlushAt records (one atomic each).  Against the per-tile, per-column
  // ballot appends (TSG_K1_GROUPQ=0) it measured equal to 0.2 ms faster on C2;
  // an atomic per group straight to the global list instead of the queue
  // serialised on the one counter (K1 5.5 -> 7.5 ms).  (Diagnostic builds that
  // dropped the queue let the compiler delete the filter itself -- only the
  // newline bucket's word stayed live -- so they measured nothing: DESIGN §4.1.)
  uint32_t fl_acc = 0;  // per lane: bit 4 * (tile - grp_t0) + block column
  uint32_t grp_n = 0;   // wave-uniform: tiles in the group so far
  uint64_t grp_t0 = 0;  // wave-uniform: the group's first tile
  auto compact = [&]() {  // wave-uniform; before the next tile's loads are issued (a flush's wait)
    const uint32_t cnt = __popc(fl_acc);
    // inclusive wave prefix sum by DPP: row_shr 1/2/4/8 within the 16-lane rows,
    // then row_bcast 15 / 31 carry the rows' totals (gfx9 DPP)
    uint32_t incl = cnt;
    incl += uint32_t(__builtin_amdgcn_update_dpp(0, int(incl), 0x111, 0xF, 0xF, true));
    incl += uint32_t(__builtin_amdgcn_update_dpp(0, int(incl), 0x112, 0xF, 0xF, true));
    incl += uint32_t(__builtin_amdgcn_update_dpp(0, int(incl), 0x114, 0xF, 0xF, true));
    incl += uint32_t(__builtin_amdgcn_update_dpp(0, int(incl), 0x118, 0xF, 0xF, true));
    incl += uint32_t(__builtin_amdgcn_update_dpp(0, int(incl), 0x142, 0xA, 0xF, false));
    incl += uint32_t(__builtin_amdgcn_update_dpp(0, int(incl), 0x143, 0xC, 0xF, false));
    const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
    if (total) {
      if (qn + total > kFQueue) flush();
      const uint32_t rec0 = __builtin_amdgcn_readfirstlane(uint32_t(grp_t0 * (kFTile / 16))) + lane * kFBlocks;
      uint32_t m = fl_acc;
      if (total <= kFQueue) {  // into the queue
        uint32_t at = qn + incl - cnt;
        while (m) {
          const uint32_t b = uint32_t(__builtin_ctz(m));
          m &= m - 1;
          Q[at++] = rec0 + ((b >> 2) << 8) + (b & 3u);  // tile grp_t0 + b / 4, column b % 4
        }
        qn += total;
      } else {  // a group denser than the queue: straight to the global list
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&P.counters[7], total);
        uint32_t at = __builtin_amdgcn_readfirstlane(base) + incl - cnt;
        while (m) {
          const uint32_t b = uint32_t(__builtin_ctz(m));
          m &= m - 1;
          if (at < P.rec_cap) P.recs[at] = rec0 + ((b >> 2) << 8) + (b & 3u);
          else P.counters[8] = 1;
          at++;
        }
      }
    }
    fl_acc = 0;
    grp_n = 0;
  };
#endif
  // Global stores are rare on purpose: on gfx9 a store counts in vmcnt like
  // the loads, so a store per tile would make the next tile's wait for its
  // prefetched data also wait for the store's completion.
  auto flush_nl = [&](uint64_t t_last) {  // wave-uniform; staged tiles are t_last - (nl_slots-1) .. t_last
    wave_sync();
    // the lane index through an empty asm: the compiler otherwise hoists &NL[lane]
    // out of the tile loop and, at 64 VGPRs, spills it -- and the scratch reload's
    // s_waitcnt vmcnt(0) also waited for the next tile's loads in flight
    uint32_t l = lane;
    asm volatile("" : "+v"(l));
    if (l < nl_slots) {
      const uint64_t tt = t_last - uint64_t(nl_slots - 1 - l);
      reinterpret_cast<uint64_t*>(P.nl)[tt] = NL[l];  // chunks 4tt .. 4tt+3 (buffer padded past the end)
    }
    nl_slots = 0;
  };
  // One tile: `cur` holds its 64 bytes per lane.  kTail: the arena's last,
  // partial tile (bytes past the end are zeroed); kept out of the main loop's
  // code so the full tiles carry no masking state.
  auto tile = [&](uint4* cur, uint64_t tt, auto tail_tag) {
    constexpr bool kTail = decltype(tail_tag)::value;
    if (kTail) {
      const uint64_t b0 = tt * kFTile + uint64_t(lane) * kFLane;
#pragma unroll
      for (int j = 0; j < kFBlocks; j++) {
        const uint64_t p = b0 + 16 * j;
        uint32_t wd[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint64_t wp = p + 4 * q;
          if (wp >= P.n_bytes) wd[q] = 0;
          else if (wp + 4 > P.n_bytes) wd[q] &= (1u << (8 * (P.n_bytes - wp))) - 1u;
        }
        cur[j] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
      }
    }
    // the previous 8 bytes: lane l-1's last two words by a DPP wave shift
    // (lane 0: the carried prefix, zeros at the arena start)
    const uint32_t p0 = uint32_t(__builtin_amdgcn_update_dpp(int(pre_x), int(cur[kFBlocks - 1].z), 0x138, 0xF, 0xF,
                                                             false));
    const uint32_t p1 = uint32_t(__builtin_amdgcn_update_dpp(int(pre_y), int(cur[kFBlocks - 1].w), 0x138, 0xF, 0xF,
                                                             false));
    pre_x = __builtin_amdgcn_readlane(cur[kFBlocks - 1].z, 63);
    pre_y = __builtin_amdgcn_readlane(cur[kFBlocks - 1].w, 63);
    uint32_t flagged = 0, nl = 0;
    if (P.diag_mode < 2) {
      uint32_t st[kFWords] = {~0u, ~0u, ~0u, ~0u};
      reach_apply(reach_read(s_reach, p0, 3, laneoff), st);
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) reach_apply(reach_read(s_reach, p1, k, laneoff), st);
#pragma unroll
      for (int j = 0; j < kFBlocks; j++) {
        const uint32_t wd[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
        uint32_t acc = ~0u;
        // table reads in groups of kFReadAhead ahead of the chain (independent of
        // the state): fewer live VGPRs than a whole block's 16 rows
#pragma unroll
        for (uint32_t g = 0; g < 16; g += kFReadAhead) {
          uint4 m[kFReadAhead];
#pragma unroll
          for (uint32_t q = 0; q < kFReadAhead; q++)
            m[q] = reach_read(s_reach, wd[(g + q) >> 2], (g + q) & 3, laneoff);
#pragma unroll
          for (uint32_t q = 0; q < kFReadAhead; q++) {
            const uint32_t k = g + q;
            reach_apply(m[q], st);
            if (k % 3 == 2 || k == 15) acc &= st[0] & st[1] & st[2] & st[3];
            if (k % 4 == 3) nl += __popc(~st[3] & kNlBits);
          }
        }
        flagged |= uint32_t((acc | ~kFireBits) != ~0u) << j;
      }
    } else {
#pragma unroll
      for (int j = 0; j < kFBlocks; j++)
        nl += nl_count4(cur[j].x) + nl_count4(cur[j].y) + nl_count4(cur[j].z) + nl_count4(cur[j].w);
    }
    {
    // newlines per 1-KiB chunk = per 16-lane DPP row: a row_shr 1/2/4/8 sum puts it in the row's last lane
    nl += uint32_t(__builtin_amdgcn_update_dpp(0, int(nl), 0x111, 0xF, 0xF, true));
    nl += uint32_t(__builtin_amdgcn_update_dpp(0, int(nl), 0x112, 0xF, 0xF, true));
    nl += uint32_t(__builtin_amdgcn_update_dpp(0, int(nl), 0x114, 0xF, 0xF, true));
    nl += uint32_t(__builtin_amdgcn_update_dpp(0, int(nl), 0x118, 0xF, 0xF, true));
    static_assert(kChunk / kFLane == 16, "one newline chunk per DPP row");
    static_assert(kFTile / 16 == 256, "a tile's records: 256 blocks");
    if ((lane & 15) == 15) reinterpret_cast<uint16_t*>(NL + nl_slots)[lane >> 4] = uint16_t(nl);
    if (++nl_slots == kFNlTiles) flush_nl(tt);
    }
#if TSG_K1_GROUPQ
    if (grp_n == 0) grp_t0 = tt;
    fl_acc |= flagged << (4 * grp_n);
    grp_n++;
#else
    // the flagged block columns, compacted (record = arena byte / 16)
    const uint32_t rec0 = uint32_t(tt * (kFTile / 16)) + lane * kFBlocks;
#pragma unroll
    for (int j = 0; j < kFBlocks; j++) {
      const bool fj = (flagged >> j) & 1u;
      const uint64_t m = __ballot(fj);
      if (m) {
        if (qn + 64 > kFQueue) flush();  // wave-uniform; rare (> 128 records since the last flush)
        const uint32_t below =
            __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
        if (fj) Q[qn + below] = rec0 + uint32_t(j);
        qn += uint32_t(__popcll(m));
      }
    }
#endif
  };
  // A flush's atomicAdd returns the records' base: waiting for it waits for every
  // older vector-memory op too, so it goes before the next tile's loads are issued
  // (then it only waits for the loads the coming tile needs at once anyway).
  auto flush_due = [&]() {
#if TSG_K1_GROUPQ
    if (grp_n == kFGroup) compact();
#endif
    if (qn >= kFFlushAt) flush();
  };
  using Full = std::false_type;
  // whole tiles; the arena's partial last tile (if any) is the last of its wave's range
  const uint64_t t_full = t_end < P.n_bytes / kFTile ? t_end : P.n_bytes / kFTile;
  uint64_t t = t_begin;
  // two register buffers alternate roles (no copies): tile t in A while t + 1 loads into B
  if (t < t_full) load_tile(bufA, t);
  while (t < t_full) {
    flush_due();
    load_tile(bufB, t + 1 < t_full ? t + 1 : t);  // past the range: a harmless reload
    tile(bufA, t, Full());
    t++;
    if (t >= t_full) break;
    flush_due();
    load_tile(bufA, t + 1 < t_full ? t + 1 : t);
    tile(bufB, t, Full());
    t++;
  }
  if (t < t_end) {  // the partial last tile
    flush_due();
    load_tile(bufA, t);
    tile(bufA, t, std::true_type());
    t++;
  }
#if TSG_K1_GROUPQ
  if (grp_n) compact();
#endif
  if (qn) flush();
  if (nl_slots) flush_nl(t - 1);
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
  const uint32_t* fullscan_rules;
  uint32_t n_fullscan_rules;
  uint32_t fs_chunk;       // full-scan chunk bytes per lane (min; files of > 64 chunks use larger ones)
  uint32_t kw_fold;        // kwfold_kernel ran: with no fold-site overflow the keyword bits are exact in every file
  uint32_t diag;           // TSG_DIAG_VERIFY (timing only): 1 verifies only 1-word NFAs' hits, 2 only the wider ones
};

// The keyword bits of file f may miss occurrences through U+0130 / U+212A
// (then a closed gate is not MatchKeywords == false): files holding them,
// unless kwfold_kernel covered every fold site.
__device__ __forceinline__ bool kw_bits_inexact(const NfaParams& P, uint32_t f) {
  return (P.flags[f] & 4u) && !(P.kw_fold && P.counters[10] == 0);
}



// ---------------------------------------------------------------------------
// K2: confirm flagged blocks exactly + verify the anchor hits
// ---------------------------------------------------------------------------
// Confirm-kernel shape.  The kernel is latency-bound: occupancy decides its
// time (C2, profiles/r02_confirm_variants.txt: 1 WG/CU 14.5 ms, 2 WG/CU
// 8.2 ms, 4 WG/CU 5.6 ms; 5-6 waves/SIMD by forcing <= 80 VGPRs spills and
// loses).  LDS per 256-thread workgroup: 4 KiB reach + 56 B per lane (48-B
// window + base) + queues and hit buffer (8.2 KiB) + the item tables
// (C2: 12.3 KiB) = 39 KiB: four workgroups per CU, as many as the 125 VGPRs
// allow.  The TSG_C_* macros exist for those variant builds
// (tools/build_variant.py).
#ifndef TSG_C_THREADS
#define TSG_C_THREADS 512
#endif
constexpr int kCThreads = TSG_C_THREADS;  // LDS-table variant (builtin-sized rule sets)
#ifndef TSG_C_THREADS_G
#define TSG_C_THREADS_G 256
#endif
// global-table variant (large custom sets): C3 confirm 22.5 ms at 256 threads x 4 WG/CU vs
// 32.7 ms at 512 x 2 (profiles/r02d_*)
constexpr int kCThreadsG = TSG_C_THREADS_G;
template <bool kLdsTabs>
constexpr int ConfirmThreads() { return kLdsTabs ? kCThreads : kCThreadsG; }

struct FoldSite {  // a fold rune (U+0130 / U+212A / U+017F) at arena byte x of file f
  uint64_t x;
  uint32_t f;
  uint32_t len;
};

// One slot per active lane; one atomic per call per wave (divergence-safe:
// the ballot covers exactly the lanes that call).
__device__ __forceinline__ uint32_t wave_slot(uint32_t* ctr) {
  const uint64_t m = __ballot(1);
  const uint32_t leader = uint32_t(__ffsll(static_cast<unsigned long long>(m)) - 1);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
  uint32_t base = 0;
  if (rank == 0) base = atomicAdd(ctr, uint32_t(__popcll(m)));
  base = __shfl(base, int(leader));
  return base + rank;
}

// Per-wave LDS hit buffer of the confirm kernel, flushed at >= 64 entries with
// one global atomic (emitting each hit with its own wave-aggregated atomic on
// the one hit counter cost 2.3 ms on C2: the atomics serialise at one address).
#ifndef TSG_C_HITS
#define TSG_C_HITS 96
#endif
constexpr uint32_t kCWaveHits = TSG_C_HITS;

// A hit record is 3 u32: file, the literal end in the file (low 32 bits),
// the anchor id with the end's bits 32..39 in its top byte (files of 4 GiB
// and more; anchor ids < 2^24, checked when the engine is built).
constexpr uint32_t kHitAidBits = 24;
__device__ __forceinline__ uint32_t hit_aid_word(uint32_t aid, uint64_t end) {
  return aid | (uint32_t(end >> 32) << kHitAidBits);
}
__device__ __forceinline__ void hit_unpack(const uint32_t* h, uint32_t* f, uint64_t* end, uint32_t* aid) {
  *f = h[0];
  *end = uint64_t(h[1]) | (uint64_t(h[2] >> kHitAidBits) << 32);
  *aid = h[2] & ((1u << kHitAidBits) - 1u);
}

// Appends a hit to the wave's LDS buffer (LDS atomic); a full buffer spills to
// the global list directly.
__device__ __forceinline__ void stage_hit(uint32_t* hbuf, uint32_t* hcnt, uint32_t* hits, uint32_t cap,
                                          uint32_t* counters, uint32_t f, uint64_t end, uint32_t aid) {
  const uint32_t k = atomicAdd(hcnt, 1u);
  if (k < kCWaveHits) {
    hbuf[3 * k + 0] = f;
    hbuf[3 * k + 1] = uint32_t(end);
    hbuf[3 * k + 2] = hit_aid_word(aid, end);
    return;
  }
  const uint32_t g = atomicAdd(&counters[0], 1u);
  if (g < cap) {
    hits[3ull * g + 0] = f;
    hits[3ull * g + 1] = uint32_t(end);
    hits[3ull * g + 2] = hit_aid_word(aid, end);
  } else {
    counters[3] = 1;
  }
}

// Copies the wave's staged hits to the global list with one atomic (wave-uniform call).
__device__ __forceinline__ void flush_staged(uint32_t* hbuf, uint32_t* hcnt, uint32_t* hits, uint32_t cap,
                                             uint32_t* counters, uint32_t lane) {
  wave_sync();
  const uint32_t n_all = __builtin_amdgcn_readfirstlane(*hcnt);
  const uint32_t n = n_all < kCWaveHits ? n_all : kCWaveHits;
  if (n) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&counters[0], n);
    base = __builtin_amdgcn_readfirstlane(base);
    for (uint32_t i = lane; i < n; i += 64) {
      if (base + i < cap) {
        hits[3ull * (base + i) + 0] = hbuf[3 * i + 0];
        hits[3ull * (base + i) + 1] = hbuf[3 * i + 1];
        hits[3ull * (base + i) + 2] = hbuf[3 * i + 2];
      } else {
        counters[3] = 1;
      }
    }
  }
  wave_sync();
  if (lane == 0) *hcnt = 0;
  wave_sync();
}

__device__ __forceinline__ void put_hit(uint32_t* hits, uint32_t cap, uint32_t* counters, uint32_t f, uint64_t end,
                                        uint32_t aid) {
  const uint32_t g = wave_slot(&counters[0]);
  if (g < cap) {
    hits[3ull * g + 0] = f;
    hits[3ull * g + 1] = uint32_t(end);
    hits[3ull * g + 2] = hit_aid_word(aid, end);
  } else {
    counters[3] = 1;
  }
}
// Follow requirements of an anchor hit (rules.h FollowLut), on registers.
// X[0..12] hold the 52 bytes from the literal end (little-endian words);
// avail = file bytes from there.  False only when every byte up to the last
// possible run end is ASCII and some requirement's run starts at none of its
// offsets -- then no match continues from this literal occurrence.
// Per word: nibble-table set membership of 4 bytes with v_perm (bit 4r + k
// of byte o = byte o is in run r's k-th set), runs by byte-aligned shifts
// (bit 4r of Z[o] = the run starts at o), offsets by an interval mask.
__device__ __forceinline__ bool follow_lut_pass(const FollowLut& L, const uint32_t* X, int64_t avail) {
  const uint32_t n0 = L.n[0], n1 = L.n[1];
  if (n0 == 0) return true;
  const int64_t span0 = int64_t(L.hi[0]) + n0, span1 = n1 ? int64_t(L.hi[1]) + n1 : 0;
  const int64_t lim = avail < (span0 > span1 ? span0 : span1) ? avail : (span0 > span1 ? span0 : span1);
  uint32_t nonascii = 0;
#pragma unroll
  for (int j = 0; j < 13; j++) {
    const int64_t v = lim - 4 * j;
    const uint32_t vm = v >= 4 ? ~0u : (v <= 0 ? 0u : (1u << (8 * uint32_t(v))) - 1u);
    nonascii |= X[j] & vm;
  }
  if (nonascii & 0x80808080u) return true;  // a multi-byte rune or invalid byte: offsets not fixed
  uint32_t t[4], h[2];
  __builtin_memcpy(t, L.lo_tab, 16);
  __builtin_memcpy(h, L.hi_tab, 8);
  uint32_t M[13];
#pragma unroll
  for (int j = 0; j < 13; j++) {
    const uint32_t lo = X[j] & 0x0F0F0F0Fu, hi = (X[j] >> 4) & 0x07070707u;
    const uint32_t sel = lo & 0x07070707u;
    const uint32_t a0 = __builtin_amdgcn_perm(t[1], t[0], sel), a1 = __builtin_amdgcn_perm(t[3], t[2], sel);
    const uint32_t m8 = ((lo >> 3) & 0x01010101u) * 0xFFu;
    M[j] = ((a0 & ~m8) | (a1 & m8)) & __builtin_amdgcn_perm(h[1], h[0], hi);
  }
  // valid run starts: o in [lo_r, hi_r] with the run inside the file
  auto interval = [&](int r, uint32_t n) -> uint64_t {
    int64_t a = L.lo[r], b = L.hi[r];
    if (avail - int64_t(n) < b) b = avail - int64_t(n);
    if (b < a) return 0;
    const uint64_t upto = b >= 63 ? ~uint64_t(0) : (uint64_t(1) << (b + 1)) - 1;
    return upto & ~((uint64_t(1) << a) - 1);
  };
  const uint64_t R0 = interval(0, n0), R1 = n1 ? interval(1, n1) : 0;
  uint32_t f0 = 0, f1 = 0;
#pragma unroll
  for (int j = 0; j < 12; j++) {
    const uint32_t y1 = __builtin_amdgcn_alignbyte(M[j + 1], M[j], 1);
    const uint32_t y2 = __builtin_amdgcn_alignbyte(M[j + 1], M[j], 2);
    const uint32_t y3 = __builtin_amdgcn_alignbyte(M[j + 1], M[j], 3);
    const uint32_t Z = M[j] & (y1 >> 1) & (y2 >> 2) & (y3 >> 3);
    const uint32_t s0 = ((uint32_t(R0 >> (4 * j)) & 0xFu) * 0x00204081u) & 0x01010101u;
    const uint32_t s1 = ((uint32_t(R1 >> (4 * j)) & 0xFu) * 0x00204081u) & 0x01010101u;
    f0 |= Z & s0;
    f1 |= Z & (s1 << 4);
  }
  return f0 != 0 && (n1 == 0 || f1 != 0);
}

// The 52 bytes from byte s (0..3) of the 4-B aligned pointer w as 13
// little-endian words: 14 word loads (global memory or LDS) and v_alignbyte.
// (Selecting words out of wider aligned loads by a per-lane offset made the
// compiler index a private array: 96 B of scratch per lane.)
__device__ __forceinline__ void follow_words(const uint32_t* w, uint32_t s, uint32_t* X) {
  uint32_t R[14];
#pragma unroll
  for (int j = 0; j < 14; j++) R[j] = w[j];
#pragma unroll
  for (int j = 0; j < 13; j++) X[j] = __builtin_amdgcn_alignbyte(R[j + 1], R[j], s & 3);
}

#ifndef TSG_C_WIN
#define TSG_C_WIN 48
#endif
constexpr int kCWin = TSG_C_WIN;  // per-lane LDS copy of arena bytes [base - 16, base + kCWin - 16)

struct ConfirmParams {
  const uint8_t* arena;
  uint64_t n_bytes;
  const uint64_t* off;
  const uint32_t* chunk_file;
  const uint16_t* nl;
  const uint32_t* reach;
  const void* tabs;  // bucket_off | bucket_items | items | item_ids | item_cls | classes
  uint32_t tabs_bytes, t_bucket_off, t_bucket_items, t_items, t_item_ids, t_item_cls, t_classes;
  const AnchorInfo* anchors;
  const RuleGpu* rules;
  const uint64_t* nfa;
  const uint32_t* recs;
  uint32_t rec_cap;
  uint32_t* flags;
  uint32_t* counters;  // [0] hits [2] special files [3] hit overflow [7] records [9] folds [10] fold overflow
  uint32_t* hits;      // (file, literal end in the file, anchor id)
  uint32_t hit_cap;
  FoldSite* folds;     // fold runes found (for the fold kernel)
  uint32_t fold_cap;
  uint32_t diag;       // TSG_DIAG_CONFIRM bits: 4 no item checks, 8 no attribution, 16 no emission, 32 follow first
  uint32_t* kwbits;               // per file: kw_words x u32 keyword bits
  uint32_t kw_words;
  const uint64_t* core;           // filter.h core tables (n_groups x 256)
  const uint32_t* group_items;    // n_groups x 8
  const uint32_t* bucket_groups;  // n_buckets + 1
  uint32_t* item_diag;            // TSG_DIAG_ITEMS: per item exact matches
  uint32_t t_luts;                // tabs offset of the per-anchor follow requirements (rules.h FollowLut)
  // LDS tables only: the core tables over byte classes -- class of byte b at
  // tabs[t_cmap + b], group g's column of class c at u64 [t_ccore/8 + g * n_cls + c]
  uint32_t t_cmap, t_ccore, t_gitems, t_bgroups, n_cls;
  // literal-window hash (filter.h): keys at u64 [t_hkeys/8], items at u32 [t_hitems/4], 2^hash_bits slots
  uint32_t t_hkeys, t_hitems, hash_bits, hash_buckets;
  // global-table variant: the n_classes byte classes (8 u32 each) staged in LDS (0: read from tabs)
  uint32_t n_classes_lds;
  // TSG_K2_PACK experiment: each record's 48-B window packed sequentially (64-B
  // stride) by pack_kernel, read linearly instead of gathered from the arena
  const uint8_t* wins;
};

// Shift-and NFA over arena bytes [fs + start, fs + len), read 16 B at a time
// (aligned) instead of one dependent load per byte.  Injects the start state
// at every position up to inj_hi.  Returns kNfaAccept when some position
// accepts, kNfaReject when every thread died (or the file ended), and
// kNfaUndecided after max_steps bytes with threads still alive.
constexpr int kNfaReject = 0, kNfaAccept = 1, kNfaUndecided = 2;
template <int W>
__device__ int nfa_run_abs(const uint8_t* __restrict arena, uint64_t fs, int64_t len, int64_t start, int64_t inj_hi,
                           const uint64_t* __restrict tab, int64_t max_steps) {
  uint64_t O[W], Lp[W], F[W], D[W];
#pragma unroll
  for (int w = 0; w < W; w++) {
    O[w] = tab[w];
    Lp[w] = tab[W + w];
    F[w] = tab[2 * W + w];
    D[w] = 0;
  }
  const uint64_t* B = tab + 3 * W;
  uint4 buf = make_uint4(0, 0, 0, 0);
  uint64_t buf_at = ~uint64_t(0);
  const int64_t stop = len - start > max_steps ? start + max_steps : len;
  for (int64_t pos = start; pos < stop; pos++) {
    const uint64_t abs = fs + uint64_t(pos);
    if ((abs & ~uint64_t(15)) != buf_at) {
      buf_at = abs & ~uint64_t(15);
      buf = load16(arena + buf_at);
    }
    const uint32_t b = (word_of(buf, uint32_t(abs >> 2) & 3) >> ((abs & 3) * 8)) & 0xFFu;
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
    const bool keep = (b & 0xC0u) == 0x80u;  // UTF-8 continuation: also stay
    uint64_t acc = 0, alive = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      uint64_t nd = (T[w] & Bb[w]) | (keep ? D[w] : 0);
      D[w] = nd;
      acc |= nd & F[w];
      alive |= nd;
    }
    if (acc) return kNfaAccept;
    if (!alive && pos >= inj_hi) return kNfaReject;
  }
  return stop < len ? kNfaUndecided : kNfaReject;
}

__device__ int nfa_dispatch_abs(int words, const uint8_t* arena, uint64_t fs, int64_t len, int64_t start,
                                int64_t inj_hi, const uint64_t* tab, int64_t max_steps = INT64_MAX) {
  switch (words) {
    case 1: return nfa_run_abs<1>(arena, fs, len, start, inj_hi, tab, max_steps);
    case 2: return nfa_run_abs<2>(arena, fs, len, start, inj_hi, tab, max_steps);
    case 3: return nfa_run_abs<3>(arena, fs, len, start, inj_hi, tab, max_steps);
    default: return nfa_run_abs<4>(arena, fs, len, start, inj_hi, tab, max_steps);
  }
}

// Candidate record (the host's exact pass input); nl_before < 0 and flags are
// filled by the finalize kernel once the keyword bits are final.
__device__ __forceinline__ void put_candidate(Candidate* cands, uint32_t cap, uint32_t* counters, uint32_t f,
                                              uint32_t r, int64_t wlo, int64_t whi) {
  const uint32_t k = atomicAdd(&counters[1], 1u);
  if (k < cap) {
    Candidate c;
    c.file = f;
    c.rule = r;
    c.wlo = wlo;
    c.whi = whi;
    c.nl_before = -1;
    c.flags = 0;
    c.nl_back[0] = c.nl_back[1] = c.nl_back[2] = kNlUnknown;
    c.nl_fwd[0] = c.nl_fwd[1] = c.nl_fwd[2] = kNlUnknown;
    c.pad_ = 0;
    cands[k] = c;
  } else {
    counters[4] = 1;
  }
}

// '\n' in arena [a, b) with aligned 16-B loads (bytes outside the range masked to 0)
__device__ int64_t count_nl_range(const uint8_t* arena, uint64_t a, uint64_t b) {
  int64_t n = 0;
  for (uint64_t blk = a & ~uint64_t(15); blk < b; blk += 16) {
    const uint4 v = load16(arena + blk);
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      const uint64_t wa = blk + 4 * q;
      const uint32_t lo = a > wa ? uint32_t(a - wa < 4 ? a - wa : 4) : 0u;
      const uint32_t hi = b < wa + 4 ? (b > wa ? uint32_t(b - wa) : 0u) : 4u;
      if (hi <= lo) continue;
      const uint32_t mhi = hi == 4 ? ~0u : (1u << (8 * hi)) - 1u;
      const uint32_t mlo = ~((1u << (8 * lo)) - 1u);
      n += nl_count4(word_of(v, q) & mhi & mlo);
    }
  }
  return n;
}

__device__ int64_t count_nl_abs(const uint8_t* arena, const uint16_t* nl, uint64_t a, uint64_t b) {  // arena [a, b)
  const uint64_t ca = (a + kChunk - 1) / kChunk, cb = b / kChunk;
  if (ca >= cb) return count_nl_range(arena, a, b);
  int64_t n = count_nl_range(arena, a, ca * kChunk) + count_nl_range(arena, cb * kChunk, b);
  for (uint64_t c = ca; c < cb; c++) n += nl[c];
  return n;
}

// K2.  Flagged blocks are confirmed in three wave-wide phases with LDS work
// queues between them, so every phase runs on full waves instead of diverging
// per lane:
//   A  one block per lane: its 64 arena bytes [base-16, base+48) go to the
//      lane's LDS window; the bucket fires are recomputed from the 5 bytes
//      before it; each fire position queues (lane, k, bucket mask);
//   B  one fire per lane: per fired bucket group, one AND over the 8 core-table
//      lookups of the bytes ending at k gives the items whose core matches;
//      each queues (lane, k, item);
//   C  one candidate item per lane: the item's positions outside the core are
//      checked, the start is attributed to its file (chunk map) and the anchor
//      hits (or the fold site) are staged.
#ifndef TSG_C_Q1
#define TSG_C_Q1 128
#endif
#ifndef TSG_C_Q2
#define TSG_C_Q2 96
#endif
#ifndef TSG_C_FSE
#define TSG_C_FSE 0
#endif
#ifndef TSG_C_PREFETCH
#define TSG_C_PREFETCH 1
#endif
#ifndef TSG_C_REACH_COPIES
#define TSG_C_REACH_COPIES 1
#endif
constexpr bool kCFse = TSG_C_FSE;     // cache each block's file in LDS in phase A (-0.2 ms at equal occupancy; costs 20 B/lane)
// Copies of the 4-KiB reach table in the confirm kernel's LDS, the copy chosen
// by lane & (copies - 1).  Phase A's row reads conflict (SQ_LDS_BANK_CONFLICT is
// 29 % of K2's LDS cycles, profiles/r04f), but four copies (+12 KiB per
// workgroup) measured K2 2.42 -> 3.42 ms (profiles/r04y): one copy stays.
constexpr uint32_t kCReachCopies = TSG_C_REACH_COPIES;
static_assert((kCReachCopies & (kCReachCopies - 1)) == 0, "a power of two");
constexpr uint32_t kCQ1 = TSG_C_Q1;  // fires (overflow: handled in place)
constexpr uint32_t kCQ2 = TSG_C_Q2;  // candidate items (overflow: checked in place)
constexpr size_t ConfirmFixedLds(int t) {  // LDS of a t-thread workgroup besides the staged tables
  return 4096 * kCReachCopies + size_t(t) * (kCWin + 8 + (kCFse ? 20 : 0)) + size_t(t / 64) * (kCQ1 + kCQ2) * 4 +
         size_t(t / 64) * kCWaveHits * 12 + size_t(t / 64) * 16;
}

// kLdsTabs: the item tables are staged in LDS (they fit: builtin-sized rule
// sets); otherwise they are read through the caches from global memory
// (large custom rule sets, e.g. 2,000 generated rules).
template <bool kLdsTabs>
#ifndef TSG_C_MINW
#define TSG_C_MINW 4  // <= 128 VGPRs: 4 waves per SIMD
#endif
__global__ __launch_bounds__(ConfirmThreads<kLdsTabs>(), TSG_C_MINW) void confirm_kernel(ConfirmParams P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int kCThreads = ConfirmThreads<kLdsTabs>();  // shadows the file-scope constant
  constexpr uint32_t kWaves = kCThreads / 64;
  uint8_t* s_reach = smem;                                        // 4 KiB x kCReachCopies (row b: copies x 16 B)
  uint8_t* s_win = smem + 4096 * kCReachCopies;                   // kCThreads x 64 B
  uint64_t* s_base = reinterpret_cast<uint64_t*>(s_win + kCThreads * kCWin);    // kCThreads
  uint64_t* s_fse = s_base + kCThreads;                                         // kCThreads x 2: block's file [fs, fe)
  uint32_t* s_file = reinterpret_cast<uint32_t*>(s_fse + (kCFse ? 2 * kCThreads : 0));  // kCThreads: block's file
  uint32_t* s_q1 = s_file + (kCFse ? kCThreads : 0);                            // kWaves x kCQ1
  uint32_t* s_q2 = s_q1 + kWaves * kCQ1;                                        // kWaves x kCQ2
  uint32_t* s_hbuf = s_q2 + kWaves * kCQ2;                                      // kWaves x kCWaveHits x 3
  uint32_t* s_cnt = s_hbuf + kWaves * kCWaveHits * 3;                           // kWaves x 4
  uint8_t* s_tabs = reinterpret_cast<uint8_t*>(s_cnt + kWaves * 4);
  const int tid = threadIdx.x;
  load_reach_lds(s_reach, P.reach, kCReachCopies, tid, blockDim.x);
  if (kLdsTabs) {
    const uint4* t = reinterpret_cast<const uint4*>(P.tabs);
    uint4* d = reinterpret_cast<uint4*>(s_tabs);
    for (uint32_t i = tid; i < P.tabs_bytes / 16; i += blockDim.x) d[i] = t[i];
  }
  const uint8_t* tabs = kLdsTabs ? s_tabs : static_cast<const uint8_t*>(P.tabs);
  const uint32_t lane = tid & 63, wave = tid >> 6;
  uint32_t* cnt = s_cnt + wave * 4;  // [0] staged hits [1] q1 [2] q2 [3] anchor-item matches
  if (lane < 4) cnt[lane] = 0;
  __syncthreads();
  const FilterItemGpu* items = reinterpret_cast<const FilterItemGpu*>(tabs + P.t_items);
  const uint32_t* item_ids = reinterpret_cast<const uint32_t*>(tabs + P.t_item_ids);
  const uint8_t* item_cls = tabs + P.t_item_cls;
  const uint32_t* classes = reinterpret_cast<const uint32_t*>(tabs + P.t_classes);
  if (!kLdsTabs && P.n_classes_lds) {  // large rule sets: the class words in LDS (one L2 round trip less per position)
    const uint4* c = reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(P.tabs) + P.t_classes);
    for (uint32_t i = tid; i < P.n_classes_lds * 2; i += blockDim.x) reinterpret_cast<uint4*>(s_tabs)[i] = c[i];
    __syncthreads();
    classes = reinterpret_cast<const uint32_t*>(s_tabs);
  }
  uint8_t* wwin = s_win + wave * 64 * kCWin;  // the wave's 64 windows
  uint64_t* wbase = s_base + wave * 64;      // block base per lane
  uint64_t* wfse = s_fse + wave * 128;       // the file holding the block's first byte, per lane
  uint32_t* wfile = s_file + wave * 64;
  uint32_t* q1 = s_q1 + wave * kCQ1;
  uint32_t* q2 = s_q2 + wave * kCQ2;
  uint32_t* hbuf = s_hbuf + wave * kCWaveHits * 3;
  const uint32_t n_recs = P.counters[7] < P.rec_cap ? P.counters[7] : P.rec_cap;
  uint32_t n_anchor = 0;  // anchor-item matches of this lane (stats; summed once per wave at the end)
  // phase C for one queued candidate: item `ix` whose window ends at lane l's block + k
  auto check_item = [&](uint32_t l, uint32_t k, uint32_t ix, uint32_t full) {
    const FilterItemGpu it = items[ix];
    const uint64_t base = wbase[l];
    const int64_t start = int64_t(base + k) + 1 - int64_t(it.back);
    if (start < 0 || uint64_t(start) + it.n > P.n_bytes) return;
    // [core_lo, back) verified by the core tables; a hashed candidate (full)
    // matched its case-folded window only, so every position is checked
    const uint32_t core_lo = full ? uint32_t(it.back) : (it.back > 8 ? it.back - 8u : 0u);
    // Positions [q0, q1) outside the core range, checked exactly: all of them,
    // before the follow requirements (measured on C2: checking the lookahead
    // sets only after a follow requirement passed, TSG_DIAG_CONFIRM=32, costs
    // 0.35 ms more -- the sets reject half the literal hits at a lower cost).
    const uint64_t cw0 = base >= 16 ? base - 16 : 0;  // the lane window [cw0, cw0 + kCWin)
    const uint8_t* cwin = wwin + l * kCWin;
#ifndef TSG_C_PRE
#define TSG_C_PRE 0
#endif
    // global tables: the first positions' class ids loaded up front (independent
    // loads instead of one dependent round trip per position)
    constexpr uint32_t kPre = kLdsTabs ? 0 : TSG_C_PRE;
    uint32_t pre[kPre > 0 ? kPre : 1];
#pragma unroll
    for (uint32_t q = 0; q < kPre; q++) pre[q] = q < it.n ? item_cls[it.cls_off + q] : 0u;
    auto sets_ok = [&](uint32_t q0, uint32_t q1) {
      for (uint32_t q = q0; q < q1; q++) {
        if (q >= core_lo && q < it.back) continue;
        const uint64_t pos = uint64_t(start) + q;
        const uint32_t bt = pos - cw0 < uint64_t(kCWin) ? uint32_t(cwin[pos - cw0]) : uint32_t(P.arena[pos]);
        uint32_t c = 0;
#pragma unroll
        for (uint32_t k = 0; k < kPre; k++)
          if (q == k) c = pre[k];
        if (q >= kPre) c = item_cls[it.cls_off + q];
        if (!((classes[c * 8 + (bt >> 5)] >> (bt & 31)) & 1u)) return false;
      }
      return true;
    };
    const uint32_t check_to = it.lit_end < it.n && (P.diag & 32) ? it.lit_end : it.n;  // diag 32: follow first
    if (!sets_ok(0, check_to)) return;
    if (P.diag & 16) return;
    const uint64_t s0 = uint64_t(start);
    uint32_t f = 0;
    uint64_t fs = 1, fe = 0;
    if (kCFse) {  // phase A's attribution of the block start, when the item lies in that file
      f = wfile[l];
      fs = wfse[2 * l];
      fe = wfse[2 * l + 1];
    }
    if (s0 < fs || s0 >= fe) {
      f = P.chunk_file[s0 / kChunk];
      fs = P.off[f];
      fe = P.off[f + 1];
      while (s0 >= fe) {  // s0 < n_bytes = off[n_files]
        f++;
        fs = fe;
        fe = P.off[f + 1];
      }
    }
    if (s0 < fs || s0 + it.n > fe) return;  // crosses a file boundary
    if (P.diag & 8) return;
    if (it.kind == kItemKeyword) {
      const uint32_t id = item_ids[it.ids_off];
      uint32_t* w = &P.kwbits[uint64_t(f) * P.kw_words + (id >> 5)];
      const uint32_t bit = 1u << (id & 31);
      if (!(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(w, bit);
      return;
    }
    if (it.kind == kItemFold) {
      // bit0: widen anchor offsets; bit1: U+017F; bit2: U+0130 / U+212A (lower into ASCII)
      const uint32_t fl = item_ids[it.ids_off] == 2 ? 3u : 5u;
      if (atomicOr(&P.flags[f], fl) == 0) atomicAdd(&P.counters[2], 1u);  // files with fold runes
      const uint32_t q = atomicAdd(&P.counters[9], 1u);
      if (q < P.fold_cap) P.folds[q] = FoldSite{s0, f, it.n};
      else P.counters[10] = 1;
      return;
    }
    if (P.item_diag) atomicAdd(&P.item_diag[2 * ix], 1u);
    const uint64_t lit_end = (s0 - fs) + it.lit_end;
    // The anchor's follow requirements over the 52 bytes after the literal,
    // read from the lane's LDS window when it holds them (else through the
    // caches): most hits of frequent anchor words ("aws_region", prose
    // "linear") end here instead of in the verify kernel's NFA.
    const uint64_t e = s0 + it.lit_end;
    const uint64_t w0 = wbase[l] >= 16 ? wbase[l] - 16 : 0;
    uint32_t X[13];
    bool have_x = false;
    int after = check_to < it.n ? -1 : 1;  // lookahead sets: -1 unchecked, 0 fail, 1 pass
    for (uint32_t d = 0; d < it.n_ids; d++) {
      const uint32_t aid = item_ids[it.ids_off + d];
      n_anchor++;
      const FollowLut lut = reinterpret_cast<const FollowLut*>(tabs + P.t_luts)[aid];
      if (lut.n[0] && e < P.n_bytes) {
        if (!have_x) {  // through the caches: the lane's 48-B window rarely holds the span
          follow_words(reinterpret_cast<const uint32_t*>(P.arena + (e & ~uint64_t(3))), uint32_t(e), X);
          have_x = true;
        }
        if (!follow_lut_pass(lut, X, int64_t(fe - e))) continue;
      }
      if (after < 0) after = sets_ok(check_to, it.n) ? 1 : 0;
      if (!after) return;
      stage_hit(hbuf, &cnt[0], P.hits, P.hit_cap, P.counters, f, lit_end, aid);
    }
  };
  auto run_q2 = [&]() {  // wave-uniform: phase C over the queued candidates
    wave_sync();
    const uint32_t n2 = __builtin_amdgcn_readfirstlane(cnt[2]);
    const uint32_t m2 = n2 < kCQ2 ? n2 : kCQ2;
    for (uint32_t c2 = 0; c2 < m2; c2 += 64) {
      if (c2 + lane < m2) {
        const uint32_t e = q2[c2 + lane];
        check_item(e & 63u, (e >> 6) & 15u, (e >> 10) & 0x1FFFFFu, e >> 31);
      }
      if (__builtin_amdgcn_readfirstlane(cnt[0]) >= 64) flush_staged(hbuf, &cnt[0], P.hits, P.hit_cap, P.counters, lane);
    }
    wave_sync();
    if (lane == 0) cnt[2] = 0;
    wave_sync();
  };
  // phase B for one fire entry (lane l, position k, bucket mask): queue the core-matching items
  auto do_fire = [&](uint32_t e) {
    const uint32_t l = e & 63u, k = (e >> 6) & 15u;
    uint32_t fm = e >> 10;
    const uint64_t base = wbase[l];
    uint32_t cb[8];  // the 8 bytes ending at the window end (zero before the arena, as in K1)
    const uint64_t cw0 = base >= 16 ? base - 16 : 0;  // [base + k - 7, base + k] lies in the lane window
    const uint8_t* cwin = wwin + l * kCWin;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int64_t pos = int64_t(base + k) - 7 + q;
      cb[q] = pos < 0 ? 0u : uint32_t(cwin[uint64_t(pos) - cw0]);
    }
    auto queue_item = [&](uint32_t ix, uint32_t full) {
      const uint32_t slot = atomicAdd(&cnt[2], 1u);
      if (slot < kCQ2) q2[slot] = l | (k << 6) | (ix << 10) | (full << 31);
      else check_item(l, k, ix, full);  // queue full: check in place
    };
    if (fm & P.hash_buckets) {  // literal windows: one probe with the lowercased 6 bytes
      uint64_t key = 0;
#pragma unroll
      for (int q = 0; q < 6; q++) {
        const uint32_t b = cb[2 + q];
        key |= uint64_t(b - 'A' < 26u ? b + 32 : b) << (8 * q);
      }
      const uint64_t* hk = reinterpret_cast<const uint64_t*>(tabs + P.t_hkeys);
      const uint32_t* hi = reinterpret_cast<const uint32_t*>(tabs + P.t_hitems);
      const uint32_t mask = (1u << P.hash_bits) - 1;
      const uint64_t want = key | (uint64_t(1) << 63);
      for (uint32_t slot = WindowHash(key, P.hash_bits);; slot = (slot + 1) & mask) {
        const uint64_t kk = hk[slot];
        if (!kk) break;
        if (kk == want) queue_item(hi[slot], 1u);
      }
    }
    // LDS tables: the bytes' classes once per fire, then one ds_read_b64 per
    // byte and group (the global tables cost an L2 round trip per group)
    const uint32_t* bgroups = kLdsTabs ? reinterpret_cast<const uint32_t*>(tabs + P.t_bgroups) : P.bucket_groups;
    const uint32_t* gitems = kLdsTabs ? reinterpret_cast<const uint32_t*>(tabs + P.t_gitems) : P.group_items;
    if (kLdsTabs) {
#pragma unroll
      for (int q = 0; q < 8; q++) cb[q] = tabs[P.t_cmap + cb[q]];
    }
    while (fm) {
      const uint32_t j = __builtin_ctz(fm);
      fm &= fm - 1;
      for (uint32_t g = bgroups[j]; g < bgroups[j + 1]; g++) {
        const uint64_t* ct = kLdsTabs ? reinterpret_cast<const uint64_t*>(tabs + P.t_ccore) + size_t(g) * P.n_cls
                                      : P.core + size_t(g) * 256;
        uint64_t cm = ~uint64_t(0);
#pragma unroll
        for (int q = 0; q < 8; q++) cm &= ct[cb[q]] >> (8 * q);
        uint32_t im = uint32_t(cm) & 0xFFu;
        while (im) {
          const uint32_t gi = __builtin_ctz(im);
          im &= im - 1;
          queue_item(gitems[g * 8 + gi], 0u);
        }
      }
    }
  };
  const uint32_t stride = gridDim.x * blockDim.x;
  // The records are loaded two batches ahead and their window bytes one batch
  // ahead (TSG_C_PREFETCH): the gather of the next blocks' bytes is in flight
  // while this batch's phases run, instead of one dependent global round trip
  // (record -> window bytes) at the top of every batch.
  auto load_win = [&](uint32_t r, uint32_t rec, bool valid, uint4* dst) {
    if (P.wins) {  // TSG_K2_PACK: the window packed at record r
#pragma unroll
      for (int q = 0; q < kCWin / 16; q++)
        dst[q] = valid ? load16(P.wins + uint64_t(r) * 64 + 16 * q) : make_uint4(0, 0, 0, 0);
      return;
    }
    const uint64_t base = uint64_t(rec) * 16;
    const uint64_t w0 = base >= 16 ? base - 16 : 0;
#pragma unroll
    for (int q = 0; q < kCWin / 16; q++)  // the arena holds 64 readable bytes past n_bytes
      dst[q] = valid && w0 + 16 * q + 16 <= P.n_bytes + 64 ? load16(P.arena + w0 + 16 * q) : make_uint4(0, 0, 0, 0);
  };
  const uint32_t r_first = blockIdx.x * blockDim.x + wave * 64 + lane;
  uint32_t rec_next = r_first < n_recs ? P.recs[r_first] : 0u;
#if TSG_C_PREFETCH
  uint4 dwn[kCWin / 16];
  load_win(r_first, rec_next, r_first < n_recs, dwn);
  uint32_t rec_nn = r_first + stride < n_recs ? P.recs[r_first + stride] : 0u;
#endif
  for (uint32_t r0 = blockIdx.x * blockDim.x + wave * 64; r0 < n_recs; r0 += stride) {
    // ---- A: one block per lane
    const uint32_t r = r0 + lane;
    const uint32_t rec = rec_next;
    uint4 dw[kCWin / 16];
#if TSG_C_PREFETCH
#pragma unroll
    for (int q = 0; q < kCWin / 16; q++) dw[q] = dwn[q];
    rec_next = rec_nn;
    load_win(r + stride, rec_next, r + stride < n_recs, dwn);
    rec_nn = r + 2 * stride < n_recs ? P.recs[r + 2 * stride] : 0u;
#else
    rec_next = r + stride < n_recs ? P.recs[r + stride] : 0u;
    load_win(r, rec, r < n_recs, dw);
#endif
    uint32_t fire_e[4], n_fire = 0;
    if (r < n_recs) {
      const uint64_t base = uint64_t(rec) * 16;
      const uint4 d0 = dw[0], d1 = dw[1];
      uint4* wl = reinterpret_cast<uint4*>(wwin + lane * kCWin);
#pragma unroll
      for (int q = 0; q < kCWin / 16; q++) wl[q] = dw[q];
      wbase[lane] = base;
      if (kCFse) {  // the file holding the block's first byte (check_item's attribution, usually)
        uint32_t f = P.chunk_file[base / kChunk];
        uint64_t fs = P.off[f], fe = P.off[f + 1];
        while (base >= fe) {
          f++;
          fs = fe;
          fe = P.off[f + 1];
        }
        wfile[lane] = f;
        wfse[2 * lane] = fs;
        wfse[2 * lane + 1] = fe;
      }
      const uint4 pv = base >= 16 ? d0 : make_uint4(0, 0, 0, 0);
      const uint4 v = base >= 16 ? d1 : d0;
      uint32_t st[kFWords] = {~0u, ~0u, ~0u, ~0u};
      const uint32_t rcopy = lane & (kCReachCopies - 1);
      auto rd1 = [&](uint32_t w, uint32_t k) {  // entry b, copy c at 16 * (b * copies + c)
        return *reinterpret_cast<const uint4*>(s_reach + ((((w >> (8 * k)) & 0xFFu) * kCReachCopies + rcopy) << 4));
      };
#pragma unroll
      for (uint32_t k = 11; k < 16; k++) reach_apply(rd1(word_of(pv, k >> 2), k & 3), st);
#pragma unroll
      for (uint32_t k = 0; k < 16; k++) {
        reach_apply(rd1(word_of(v, k >> 2), k & 3), st);
        // any fire at window end base + k (slot 5 = bits 20..23 of each register,
        // AND-ed over the registers); the per-bucket mask only then (rare)
        const uint32_t z = st[0] & st[1] & st[2] & st[3];
        if ((~z & 0x00F00000u) && !(P.diag & 4)) {
          uint32_t fm = 0;
#pragma unroll
          for (int w = 0; w < kFWords; w++) fm |= ((~st[w] >> 20) & 0xFu) << (4 * w);
          const uint32_t fe = lane | (k << 6) | (fm << 10);
          if (n_fire < 4) fire_e[n_fire] = fe;
          else do_fire(fe);  // more than 4 fires in one block: the 5th and later in place
          n_fire++;
        }
      }
    }
    // the fires into the wave's queue: a prefix sum over the lanes' counts
    // instead of an LDS atomic per fire
    {
      const uint32_t mine = n_fire < 4 ? n_fire : 4u;
      uint32_t incl = mine;
#pragma unroll
      for (int x = 1; x < 64; x <<= 1) {
        const uint32_t t = __shfl_up(incl, x);
        if (lane >= uint32_t(x)) incl += t;
      }
      const uint32_t at = __builtin_amdgcn_readfirstlane(cnt[1]) + incl - mine;
      for (uint32_t i = 0; i < mine; i++) {
        if (at + i < kCQ1) q1[at + i] = fire_e[i];
        else do_fire(fire_e[i]);  // queue full: handle in place
      }
      wave_sync();
      if (lane == 63) cnt[1] = at + mine < kCQ1 ? at + mine : kCQ1;
    }
    wave_sync();
    // ---- B: one fire per lane
    const uint32_t n1 = __builtin_amdgcn_readfirstlane(cnt[1]);
    const uint32_t m1 = n1 < kCQ1 ? n1 : kCQ1;
    for (uint32_t c1 = 0; c1 < m1; c1 += 64) {
      if (c1 + lane < m1) do_fire(q1[c1 + lane]);
      // ---- C: when enough candidates queued (or at the end)
      const uint32_t n2 = __builtin_amdgcn_readfirstlane(cnt[2]);
      if (n2 >= 64 || (c1 + 64 >= m1 && n2 > 0)) run_q2();
    }
    wave_sync();
    if (lane == 0) cnt[1] = 0;
    if (__builtin_amdgcn_readfirstlane(cnt[0]) >= 64) flush_staged(hbuf, &cnt[0], P.hits, P.hit_cap, P.counters, lane);
    wave_sync();
  }
  flush_staged(hbuf, &cnt[0], P.hits, P.hit_cap, P.counters, lane);
#pragma unroll
  for (int x = 32; x >= 1; x >>= 1) n_anchor += __shfl_xor(n_anchor, x);
  if (lane == 0 && n_anchor) atomicAdd(&P.counters[11], n_anchor);  // anchor-item matches (stats)
}

// TSG_K2_PACK experiment: the 48-B window of every flagged
// block record written to a sequential buffer (64-B stride), so the confirm
// kernel's phase A reads records linearly instead of gathering 128-B lines
// the filter kernel streamed long before.  Measures what the confirm kernel
// would gain if K1 streamed the windows itself.
__global__ __launch_bounds__(256) void pack_windows_kernel(const uint8_t* __restrict__ arena, uint64_t n_bytes,
                                                           const uint32_t* __restrict__ recs, uint32_t rec_cap,
                                                           const uint32_t* __restrict__ counters,
                                                           uint8_t* __restrict__ wins) {
  const uint32_t n_recs = counters[7] < rec_cap ? counters[7] : rec_cap;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n_recs; r += gridDim.x * blockDim.x) {
    const uint64_t base = uint64_t(recs[r]) * 16;
    const uint64_t w0 = base >= 16 ? base - 16 : 0;
    uint4* d = reinterpret_cast<uint4*>(wins + uint64_t(r) * 64);
#pragma unroll
    for (int q = 0; q < kCWin / 16; q++)
      d[q] = w0 + 16 * q + 16 <= n_bytes + 64 ? load16(arena + w0 + 16 * q) : make_uint4(0, 0, 0, 0);
  }
}

// Fold kernel.  Items whose bytes hold a fold rune are invisible to the byte-
// exact filter; for each fold site and each item, every item start that puts
// the rune inside the item is tried with a fold-tolerant match: a position
// also accepts U+212A (E2 84 AA) when its set holds k/K and U+017F (C5 BF)
// when it holds s/S (the only non-ASCII runes (?i) folds onto ASCII letters),
// advancing 3 / 2 bytes.  A superset of the true occurrences; hits carry the
// literal end in bytes.
//
// Work lists (per rune kind): a match holds the rune at x only if the position
// q covering byte x can take it -- its set holds k/K (U+212A) or s/S (U+017F),
// or the lead byte itself.  When no other fold rune precedes x in the window,
// every position before q spans one byte, so the start is exactly x - q: the
// "capable" list holds one task per (item, capable q).  Otherwise positions
// 0..q-1 span at least q and at most max_before(q) bytes, and the "range" list
// holds the start range [x - hi, x - lo] per item (lo = the first capable q,
// hi = max_before of the last), cut into tasks of at most kFoldTaskStarts
// starts.  Each start is tried once either way.
struct FoldPair {
  uint32_t item;
  uint16_t lo, hi;
};
constexpr int kFoldTaskStarts = 12;  // starts per range task
struct FoldParams {
  const uint8_t* arena;
  const uint64_t* off;
  const void* tabs;
  uint32_t tabs_bytes, t_items, t_item_ids, t_item_cls, t_classes, n_items;
  const FoldPair* pairs;  // [k ranges | s ranges | k capable | s capable]
  uint32_t n_pairs_k, n_pairs_s, n_cap_k, n_cap_s;
  const uint32_t* first;  // per item 8 x u32: bytes its position 0 accepts (+ E2 / C5 fold leads)
  // Capable tasks indexed by (rune kind, q, key byte): the byte at x - q (the
  // item's position 0) for q > 0, the byte after the rune (position 1) for
  // q = 0.  idx_off[(kind * kFoldIdxQ + q) * 257 + b] .. [+1] -> idx_items;
  // tasks with q >= kFoldIdxQ or a single position stay in the pair lists.
  const uint32_t* idx_off;
  const uint32_t* idx_items;
  uint32_t use_idx;
  uint32_t n_cap_k_idx, n_cap_s_idx;  // leading capable pairs covered by the index
  const FoldSite* folds;
  uint32_t fold_cap;
  uint32_t* hits;
  uint32_t hit_cap;
  uint32_t* counters;
  // global-table variant (large rule sets): the item records and the byte
  // classes staged in LDS when they fit (n_classes classes of 8 u32)
  uint32_t stage_items, n_classes;
  // global tables: test position 0 against the item's first-byte set (one more
  // dependent global load per start; without it the position loop rejects)
  uint32_t check_first;
  uint32_t diag;  // TSG_DIAG_FOLD (timing only, findings wrong): 1 skips sites with another rune before, 2 the others
};

constexpr int kFoldSpan = 3 * 48;  // an item (<= 48 positions, <= 3 bytes each) starts at most this far back
constexpr int kFoldIdxQ = 64;      // capable positions q < kFoldIdxQ go through the byte index (one lane per q)
constexpr int kFoldWin = 2 * kFoldSpan + 16;
constexpr int kFoldWaves = 4;

// One wave per fold site: the bytes [x - kFoldSpan, x + kFoldSpan) go to the
// wave's LDS window, the lanes split the tasks; a site with another fold rune
// before it (start-range tasks over every item) is handed to the whole
// workgroup (below).  With kLdsTabs the item tables and the position-0 byte
// sets are staged in LDS.
// U+0130 sites only flag the file (Go's (?i) does not fold U+0130 onto 'i').
// kWaves waves per workgroup: 16 when the items and classes are staged (~50 KB of
// LDS: three 4-wave workgroups per CU left 12 waves to hide the global loads)
#ifndef TSG_FOLD_COOP_TASKS
#define TSG_FOLD_COOP_TASKS 512  // a site with more capable tasks than this goes to the whole workgroup
#endif
#ifndef TSG_FOLD_WIDE_WPE
#define TSG_FOLD_WIDE_WPE 8  // waves per SIMD asked of the 16-wave variant: 8 = two workgroups per CU (64 VGPRs)
#endif
template <bool kLdsTabs, int kWaves = kFoldWaves>  // kLdsTabs as confirm_kernel
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(kWaves == 16 ? TSG_FOLD_WIDE_WPE : 1)))
void fold_kernel(FoldParams P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ uint8_t s_win[kWaves][kFoldWin];
  __shared__ uint32_t s_idx[kWaves][2][64];  // per wave: index lists' exclusive prefix and start, per q
  if (kLdsTabs) {
    const uint4* t = reinterpret_cast<const uint4*>(P.tabs);
    uint4* d = reinterpret_cast<uint4*>(smem);
    for (uint32_t i = threadIdx.x; i < P.tabs_bytes / 16; i += blockDim.x) d[i] = t[i];
    const uint4* f = reinterpret_cast<const uint4*>(P.first);
    uint4* df = reinterpret_cast<uint4*>(smem + P.tabs_bytes);
    for (uint32_t i = threadIdx.x; i < P.n_items * 2; i += blockDim.x) df[i] = f[i];
  } else if (P.stage_items) {
    // large rule sets: the per-start chain was item -> class id -> class word,
    // each an L2 round trip (C3: 1.9 ms of waits for 40 k sites); the items and
    // the classes in LDS leave the class-id bytes as the only global reads
    const uint4* t = reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(P.tabs) + P.t_items);
    uint4* d = reinterpret_cast<uint4*>(smem);
    for (uint32_t i = threadIdx.x; i < P.n_items; i += blockDim.x) d[i] = t[i];
    const uint4* c = reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(P.tabs) + P.t_classes);
    uint4* dc = reinterpret_cast<uint4*>(smem + 16 * size_t(P.n_items));
    for (uint32_t i = threadIdx.x; i < P.n_classes * 2; i += blockDim.x) dc[i] = c[i];
  }
  __syncthreads();
  const uint8_t* tabs = kLdsTabs ? smem : static_cast<const uint8_t*>(P.tabs);
  const uint32_t* firsts = kLdsTabs ? reinterpret_cast<const uint32_t*>(smem + P.tabs_bytes) : P.first;
  const bool staged = !kLdsTabs && P.stage_items;
  const FilterItemGpu* items =
      staged ? reinterpret_cast<const FilterItemGpu*>(smem) : reinterpret_cast<const FilterItemGpu*>(tabs + P.t_items);
  const uint32_t* item_ids = reinterpret_cast<const uint32_t*>(tabs + P.t_item_ids);
  const uint8_t* item_cls = tabs + P.t_item_cls;
  const uint32_t* classes = staged ? reinterpret_cast<const uint32_t*>(smem + 16 * size_t(P.n_items))
                                   : reinterpret_cast<const uint32_t*>(tabs + P.t_classes);
  auto in_cls = [&](uint32_t c, uint32_t b) { return (classes[c * 8 + (b >> 5)] >> (b & 31)) & 1u; };
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  struct SiteCtx {
    uint64_t x, w0, w1, fs;  // the rune, its window [w0, w1), the file start
    uint32_t f;
    const uint8_t* wb;       // the window's bytes in LDS
  };
  // one start: item `ix` beginning `back` bytes before the rune, matched fold-tolerantly
  auto try_start = [&](const SiteCtx& S, uint32_t ix, uint32_t back) {
    if (S.x < S.w0 + back) return;
    const FilterItemGpu it = items[ix];
    const uint32_t* first = firsts + 8ull * ix;
    const uint64_t st = S.x - back;
    const uint32_t b0 = S.wb[st - S.w0];
    if ((kLdsTabs || P.check_first) && !((first[b0 >> 5] >> (b0 & 31)) & 1u)) return;  // position 0 fails (superset test)
    uint64_t p = st, lit_bytes_end = 0;
    bool ok = true, covered = false;
    // the first positions' class ids up front: independent loads instead of
    // one dependent round trip per position (global tables)
    constexpr uint32_t kPre = 6;
    uint32_t pre[kPre];
#pragma unroll
    for (uint32_t q = 0; q < kPre; q++) pre[q] = q < it.n ? item_cls[it.cls_off + q] : 0u;
    for (uint32_t q = 0; q < it.n && ok; q++) {
      if (q == it.lit_end) lit_bytes_end = p;
      if (p >= S.w1) {
        ok = false;
        break;
      }
      covered = covered || p == S.x;
      uint32_t c = 0;
#pragma unroll
      for (uint32_t k = 0; k < kPre; k++)
        if (q == k) c = pre[k];
      if (q >= kPre) c = item_cls[it.cls_off + q];
      const uint32_t b = S.wb[p - S.w0];
      if (b == 0xE2 && p + 2 < S.w1 && S.wb[p + 1 - S.w0] == 0x84 && S.wb[p + 2 - S.w0] == 0xAA &&
          (in_cls(c, 'k') || in_cls(c, 'K'))) {
        p += 3;
      } else if (b == 0xC5 && p + 1 < S.w1 && S.wb[p + 1 - S.w0] == 0xBF && (in_cls(c, 's') || in_cls(c, 'S'))) {
        p += 2;
      } else if (in_cls(c, b)) {
        p += 1;
      } else {
        ok = false;
      }
    }
    if (!ok || !covered) return;
    if (it.lit_end >= it.n) lit_bytes_end = p + (it.lit_end - it.n);  // literal longer than the checked part
    for (uint32_t d = 0; d < it.n_ids; d++)
      put_hit(P.hits, P.hit_cap, P.counters, S.f, lit_bytes_end - S.fs, item_ids[it.ids_off + d]);
  };
  // A site with another fold rune before it tries every start range of every
  // item (thousands of tasks of up to 12 starts: C3 ~1.3 ms of the kernel's 1.7
  // were the few waves holding such sites, TSG_DIAG_FOLD): those sites go to
  // the whole workgroup, the others stay one per wave.  The workgroup walks its
  // sites kWaves at a time, in step, so the barriers below are uniform.
  __shared__ uint64_t s_site[kWaves][4];  // x, w0, w1, fs of a wave's cooperative site
  __shared__ uint32_t s_coop[kWaves];     // per wave: 0, or 1 | (U+212A ? 2 : 0) | (capable tasks ? 4 : 0) for a cooperative site
  __shared__ uint32_t s_coop_f[kWaves];   // its file
  __shared__ uint32_t s_total[kWaves];    // a heavy capable-task site's indexed task count (| 4 in s_coop)
  const uint32_t n_folds = P.counters[9] < P.fold_cap ? P.counters[9] : P.fold_cap;
  for (uint32_t base = blockIdx.x * kWaves; base < n_folds; base += gridDim.x * kWaves) {
    const uint32_t si = base + wave;
    uint32_t coop = 0;  // wave-uniform
    if (si < n_folds) {
      const FoldSite fsite = P.folds[si];
      SiteCtx S;
      S.x = fsite.x;
      S.f = fsite.f;
      S.fs = P.off[fsite.f];
      const uint64_t fe = P.off[fsite.f + 1];
      S.w0 = fsite.x > S.fs + kFoldSpan ? fsite.x - kFoldSpan : S.fs;
      S.w1 = fsite.x + kFoldSpan < fe ? fsite.x + kFoldSpan : fe;  // window [w0, w1)
      uint8_t* wb = s_win[wave];
      S.wb = wb;
      for (uint32_t i = lane; i < uint32_t(S.w1 - S.w0); i += 64) wb[i] = P.arena[S.w0 + i];
      wave_sync();
      const uint32_t lead = wb[S.x - S.w0];
      if (lead != 0xC4) {  // U+0130 sites only flag the file (uniform per wave)
        const bool kay = lead == 0xE2;  // U+212A, else U+017F
        bool other = false;  // another foldable rune before x (then starts are not x - q)
        for (uint64_t p = S.w0 + lane; p < S.x; p += 64) {
          const uint32_t b = wb[p - S.w0];
          if ((b == 0xE2 && p + 2 < S.w1 && wb[p + 1 - S.w0] == 0x84 && wb[p + 2 - S.w0] == 0xAA) ||
              (b == 0xC5 && p + 1 < S.w1 && wb[p + 1 - S.w0] == 0xBF))
            other = true;
        }
        other = __ballot(other) != 0;
        const bool skip = ((P.diag & 1u) && other) || ((P.diag & 2u) && !other);
        if (other && !skip) {
          coop = 1u | (kay ? 2u : 0u);
          if (lane == 0) {
            s_site[wave][0] = S.x;
            s_site[wave][1] = S.w0;
            s_site[wave][2] = S.w1;
            s_site[wave][3] = S.fs;
            s_coop_f[wave] = S.f;
          }
        } else if (!skip) {
          const FoldPair* pairs = P.pairs + P.n_pairs_k + P.n_pairs_s + (kay ? 0 : P.n_cap_k);
          const uint32_t n_pairs = kay ? P.n_cap_k : P.n_cap_s;
          uint32_t total = 0;  // indexed capable tasks
          uint32_t* ex = s_idx[wave][0];
          uint32_t* lw = s_idx[wave][1];
          if (P.use_idx) {
            // indexed capable tasks: lane q looks up its list by the key byte, a
            // wave prefix sum spreads the lists' tasks over the lanes
            const uint32_t q = lane;
            const uint32_t rl = kay ? 3u : 2u;
            uint32_t key = 256;
            if (q == 0) key = S.x + rl < S.w1 ? wb[S.x + rl - S.w0] : 256u;
            else if (S.x >= S.w0 + q) key = wb[S.x - q - S.w0];
            uint32_t lo = 0, cnt = 0;
            if (key < 256) {
              const uint32_t* o = P.idx_off + (size_t(kay ? 0 : 1) * kFoldIdxQ + q) * 257 + key;
              lo = o[0];
              cnt = o[1] - lo;
            }
            uint32_t incl = cnt;  // inclusive prefix over the lanes
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
              const uint32_t v = __shfl_up(incl, d);
              if (lane >= uint32_t(d)) incl += v;
            }
            total = __shfl(incl, 63);
            wave_sync();
            ex[lane] = incl - cnt;
            lw[lane] = lo;
            wave_sync();
          }
          // tasks outside the index (q >= kFoldIdxQ or single-position items) follow in the pair list
          const uint32_t t0 = P.use_idx ? (kay ? P.n_cap_k_idx : P.n_cap_s_idx) : 0u;
          if (total + (n_pairs > t0 ? n_pairs - t0 : 0u) > uint32_t(TSG_FOLD_COOP_TASKS)) {
            // a heavy site (many items take the rune's byte context): the workgroup's too
            coop = 1u | (kay ? 2u : 0u) | 4u;
            if (lane == 0) {
              s_site[wave][0] = S.x;
              s_site[wave][1] = S.w0;
              s_site[wave][2] = S.w1;
              s_site[wave][3] = S.fs;
              s_coop_f[wave] = S.f;
              s_total[wave] = total;
            }
          } else {
            for (uint32_t t = lane; t < total; t += 64) {
              uint32_t a = 0, b = 63;  // the lane (q) whose range holds t: the largest with ex[q] <= t
              while (a < b) {
                const uint32_t m = (a + b + 1) >> 1;
                if (ex[m] <= t) a = m;
                else b = m - 1;
              }
              try_start(S, P.idx_items[lw[a] + (t - ex[a])], a);
            }
            for (uint32_t t = t0 + lane; t < n_pairs; t += 64) {
              const FoldPair fp = pairs[t];
              for (uint32_t back = fp.lo; back <= fp.hi; back++) try_start(S, fp.item, back);
            }
          }
        }
      }
    }
    if (lane == 0) s_coop[wave] = coop;
    __syncthreads();
    // the workgroup's cooperative sites, one after another, their range tasks over every thread
    for (uint32_t w2 = 0; w2 < uint32_t(kWaves); w2++) {
      const uint32_t c = s_coop[w2];
      if (!c) continue;  // uniform: every thread reads the same word
      SiteCtx S;
      S.x = s_site[w2][0];
      S.w0 = s_site[w2][1];
      S.w1 = s_site[w2][2];
      S.fs = s_site[w2][3];
      S.f = s_coop_f[w2];
      S.wb = s_win[w2];
      const bool kay = (c & 2u) != 0;
      if (c & 4u) {  // a heavy capable-task site: its index lists (the owner wave's s_idx), then the pair list
        const uint32_t total = s_total[w2];
        const uint32_t* ex = s_idx[w2][0];
        const uint32_t* lw = s_idx[w2][1];
        for (uint32_t t = threadIdx.x; t < total; t += blockDim.x) {
          uint32_t a = 0, b = 63;
          while (a < b) {
            const uint32_t m = (a + b + 1) >> 1;
            if (ex[m] <= t) a = m;
            else b = m - 1;
          }
          try_start(S, P.idx_items[lw[a] + (t - ex[a])], a);
        }
        const FoldPair* pairs = P.pairs + P.n_pairs_k + P.n_pairs_s + (kay ? 0 : P.n_cap_k);
        const uint32_t n_pairs = kay ? P.n_cap_k : P.n_cap_s;
        const uint32_t t0 = P.use_idx ? (kay ? P.n_cap_k_idx : P.n_cap_s_idx) : 0u;
        for (uint32_t t = t0 + threadIdx.x; t < n_pairs; t += blockDim.x) {
          const FoldPair fp = pairs[t];
          for (uint32_t back = fp.lo; back <= fp.hi; back++) try_start(S, fp.item, back);
        }
        continue;
      }
      const FoldPair* pairs = P.pairs + (kay ? 0 : P.n_pairs_k);
      const uint32_t n_pairs = kay ? P.n_pairs_k : P.n_pairs_s;
      for (uint32_t t = threadIdx.x; t < n_pairs; t += blockDim.x) {
        const FoldPair fp = pairs[t];
        for (uint32_t back = fp.lo; back <= fp.hi; back++) try_start(S, fp.item, back);
      }
    }
    __syncthreads();  // the windows are refilled by the next round
  }
}

// Keyword occurrences through fold runes.  bytes.ToLower maps exactly two
// non-ASCII runes into ASCII: U+0130 (C4 B0) -> 'i' and U+212A (E2 84 AA) ->
// 'k' (SURVEY.md §8 A7), so `kw` is in bytes.ToLower(content) iff some
// occurrence matches each keyword position by an ASCII byte of either case, by
// C4 B0 where the position is 'i' or by E2 84 AA where it is 'k'.  K2 sets the
// bits of the all-ASCII occurrences; an occurrence holding a fold rune covers a
// fold site, so trying, at every U+0130 / U+212A site, each keyword that can
// take the rune at each start putting the rune inside it finds the rest.  After
// this kernel the keyword bits are MatchKeywords exactly (unless the fold-site
// list overflowed), and the full-scan and verify kernels need not open the gates
// of files holding those runes.  Work lists as the fold kernel's: "capable"
// (item, q) tasks with start x - q when no other such rune precedes x within
// the span, else start ranges.
struct KwFoldParams {
  const uint8_t* arena;
  const uint64_t* off;
  const uint8_t* tabs;  // global table blob (filter items)
  uint32_t t_items, t_item_ids, t_item_cls, t_classes;
  const FoldPair* pairs;  // [i ranges | k ranges | i capable | k capable]
  uint32_t n_rng_i, n_rng_k, n_cap_i, n_cap_k;
  const FoldSite* folds;
  uint32_t fold_cap;
  uint32_t* counters;
  uint32_t* kwbits;
  uint32_t kw_words;
};

__global__ __launch_bounds__(64 * kFoldWaves) void kwfold_kernel(KwFoldParams P) {
  __shared__ uint8_t s_win[kFoldWaves][kFoldWin];
  const FilterItemGpu* items = reinterpret_cast<const FilterItemGpu*>(P.tabs + P.t_items);
  const uint32_t* item_ids = reinterpret_cast<const uint32_t*>(P.tabs + P.t_item_ids);
  const uint8_t* item_cls = P.tabs + P.t_item_cls;
  const uint32_t* classes = reinterpret_cast<const uint32_t*>(P.tabs + P.t_classes);
  auto in_cls = [&](uint32_t c, uint32_t b) { return (classes[c * 8 + (b >> 5)] >> (b & 31)) & 1u; };
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* wb = s_win[wave];
  const uint32_t n_folds = P.counters[9] < P.fold_cap ? P.counters[9] : P.fold_cap;
  for (uint32_t si = blockIdx.x * kFoldWaves + wave; si < n_folds; si += gridDim.x * kFoldWaves) {
    const FoldSite fsite = P.folds[si];
    const uint64_t fs = P.off[fsite.f], fe = P.off[fsite.f + 1];
    const uint32_t lead = P.arena[fsite.x];
    if (lead != 0xC4 && lead != 0xE2) continue;  // U+017F: ToLower keeps it non-ASCII (wave-uniform)
    const bool kay = lead == 0xE2;
    const uint64_t w0 = fsite.x > fs + kFoldSpan ? fsite.x - kFoldSpan : fs;
    const uint64_t w1 = fsite.x + kFoldSpan < fe ? fsite.x + kFoldSpan : fe;
    wave_sync();
    for (uint32_t i = lane; i < uint32_t(w1 - w0); i += 64) wb[i] = P.arena[w0 + i];
    wave_sync();
    auto kfold = [&](uint64_t p) {
      return wb[p - w0] == 0xE2 && p + 2 < w1 && wb[p + 1 - w0] == 0x84 && wb[p + 2 - w0] == 0xAA;
    };
    auto ifold = [&](uint64_t p) { return wb[p - w0] == 0xC4 && p + 1 < w1 && wb[p + 1 - w0] == 0xB0; };
    if (!(kay ? kfold(fsite.x) : ifold(fsite.x))) continue;  // not the rune itself (wave-uniform)
    bool other = false;
    for (uint64_t p = w0 + lane; p < fsite.x; p += 64) other = other || kfold(p) || ifold(p);
    other = __ballot(other) != 0;
    const FoldPair* pairs = P.pairs + (other ? (kay ? P.n_rng_i : 0) : P.n_rng_i + P.n_rng_k + (kay ? P.n_cap_i : 0));
    const uint32_t n_pairs = other ? (kay ? P.n_rng_k : P.n_rng_i) : (kay ? P.n_cap_k : P.n_cap_i);
    for (uint32_t t = lane; t < n_pairs; t += 64) {
      const FoldPair fp = pairs[t];
      const FilterItemGpu it = items[fp.item];
      for (uint32_t back = fp.lo; back <= fp.hi; back++) {
        if (fsite.x < w0 + back) break;
        uint64_t p = fsite.x - back;
        bool ok = true, covered = false;
        for (uint32_t q = 0; q < it.n; q++) {
          if (p >= w1) {
            ok = false;
            break;
          }
          covered = covered || p == fsite.x;
          const uint32_t c = item_cls[it.cls_off + q];
          if (kfold(p) && in_cls(c, 'k')) p += 3;
          else if (ifold(p) && in_cls(c, 'i')) p += 2;
          else if (in_cls(c, wb[p - w0])) p += 1;
          else {
            ok = false;
            break;
          }
        }
        if (!ok || !covered) continue;
        for (uint32_t d = 0; d < it.n_ids; d++) {
          const uint32_t id = item_ids[it.ids_off + d];
          uint32_t* w = &P.kwbits[uint64_t(fsite.f) * P.kw_words + (id >> 5)];
          const uint32_t bit = 1u << (id & 31);
          if (!(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(w, bit);
        }
        break;  // this item is found in the file
      }
    }
  }
}

// Candidate flags for the host's lazy MatchKeywords (scanner.go:174-186).
__device__ uint32_t gate_flags(const NfaParams& P, const RuleGpu& rg, uint32_t f) {
  // kCandFoldFile: the bits may miss occurrences through U+0130 / U+212A, the
  // host re-checks the whole content (not after kwfold_kernel covered them)
  uint32_t fl = kCandGateValid | (kw_bits_inexact(P, f) ? kCandFoldFile : 0u);
  if (rg.gate == kGateKeywords && !rg.kw_match_implied) {
    const uint32_t* kb = P.kwbits + uint64_t(f) * P.kw_words;
    for (uint32_t i = 0; i < rg.kw_cnt; i++) {
      const uint32_t id = P.rule_kw[rg.kw_off + i];
      if (kb[id >> 5] & (1u << (id & 31))) {
        fl |= kCandGateOpen;
        break;
      }
    }
  }
  return fl;
}

// Verify kernel: one lane per anchor hit.  The start window comes from the
// literal position and the anchor's offsets (wider in files with fold runes,
// whose literal bytes may be up to 3x its length); the rule's relaxed NFA runs
// from wlo with injection up to whi, reading the arena 16 B at a time; an
// accept emits the candidate with the line count before wlo.
__global__ __launch_bounds__(256, 6) void verify_hits_kernel(NfaParams P) {
  const uint32_t n = P.counters[0] < P.hit_cap ? P.counters[0] : P.hit_cap;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    uint32_t f, aid;
    uint64_t end;
    hit_unpack(P.hits + 3ull * i, &f, &end, &aid);
    const AnchorInfo a = P.anchors[aid];
    const RuleGpu rg = P.rules[a.rule];  // keyword gates are evaluated lazily by the host tail
    if (((P.diag & 1u) && rg.nfa_words > 1) || ((P.diag & 2u) && rg.nfa_words <= 1)) continue;
    const uint32_t ff = P.flags[f];
    // A closed ASCII keyword gate in a file without U+0130 / U+212A is exactly
    // MatchKeywords == false (scanner.go:409): the host would drop every match
    // of the rule, so its hits need no verification.
    if (rg.gate == kGateKeywords && !rg.kw_match_implied && !kw_bits_inexact(P, f) &&
        !(gate_flags(P, rg, f) & kCandGateOpen))
      continue;
    const int64_t lit_hi = int64_t(end) - int64_t(a.lit_len);
    const int64_t lit_lo = (ff & 1u) ? int64_t(end) - 3 * int64_t(a.lit_len) : lit_hi;
    const int64_t whi = lit_hi - a.off_lo;
    if (whi < 0) continue;
    int64_t wlo = lit_lo - ((ff & 1u) ? int64_t(a.off_hi_fold) : int64_t(a.off_hi));
    if (wlo < 0) wlo = 0;
    const uint64_t fs = P.off[f];
    const int64_t len = int64_t(P.off[f + 1] - fs);

    const bool acc = rg.nfa_words == 0 ||
                     nfa_dispatch_abs(rg.nfa_words, P.arena, fs, len, wlo, whi, P.nfa + rg.nfa_off) == kNfaAccept;
    if (acc) put_candidate(P.cands, P.cand_cap, P.counters, f, a.rule, wlo, whi);
  }
}

// Unanchored rules (no literal at a bounded offset): the relaxed NFA with
// injection at every byte must find out whether any position of the file
// accepts (then the whole file is the candidate window).
//
// Work: only (file, rule) pairs whose keyword gate can be open (the GPU
// keyword bits are final here; scanner.go:409 skips the rest), one wave per
// pair.  A file is cut into <= 64 chunks, one per lane; every lane runs its
// chunk from the empty state, then the chunk entry states are iterated to the
// fixpoint: lane c re-runs its chunk from lane c-1's exit state whenever that
// state gained bits (shift-and is monotone, so exit states only grow and the
// sequential result is reached; a state that dies stops mattering at once).
// Any accept ends the pair.  More than kFsMaxRounds re-runs: the pair is
// emitted unverified (a candidate is always safe -- the host pass is exact).
constexpr int kFsMaxRounds = 6;

template <int W, typename Acc>
__device__ bool nfa_chunk(const uint8_t* __restrict arena, uint64_t a, uint64_t b, uint64_t* D,
                          const uint64_t* __restrict tab, Acc on_acc, bool inject = true) {
  // arena [a, b) from state D, a start injected at every byte (inject) or
  // none (D's paths only); on_acc(abs): an accept after byte abs, false stops
  // the chunk there
  uint64_t O[W], Lp[W], F[W];
#pragma unroll
  for (int w = 0; w < W; w++) {
    O[w] = tab[w];
    Lp[w] = tab[W + w];
    F[w] = tab[2 * W + w];
  }
  const uint64_t* B = tab + 3 * W;
  uint4 buf = make_uint4(0, 0, 0, 0);
  uint64_t buf_at = ~uint64_t(0);
  bool any = false;
  for (uint64_t abs = a; abs < b; abs++) {
    if ((abs & ~uint64_t(15)) != buf_at) {
      buf_at = abs & ~uint64_t(15);
      buf = load16(arena + buf_at);
    }
    const uint32_t byte = (word_of(buf, uint32_t(abs >> 2) & 3) >> ((abs & 3) * 8)) & 0xFFu;
    uint64_t carry = inject ? 1 : 0, T[W];
#pragma unroll
    for (int w = 0; w < W; w++) {
      T[w] = (D[w] << 1) | carry | (D[w] & Lp[w]);
      carry = D[w] >> 63;
    }
    uint64_t c = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const uint64_t x = T[w] & O[w], s1 = O[w] + x, c1 = s1 < O[w], s2 = s1 + c, c2 = s2 < s1;
      T[w] |= s2 ^ O[w];
      c = c1 | c2;
    }
    const uint64_t* Bb = B + size_t(byte) * W;
    const bool keep = (byte & 0xC0u) == 0x80u;
    uint64_t acc = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      D[w] = (T[w] & Bb[w]) | (keep ? D[w] : 0);
      acc |= D[w] & F[w];
    }
    if (acc) {
      any = true;
      if (!on_acc(abs)) return true;
    }
  }
  return any;
}

// Full scan of one (file, rule) pair by a wave: 64 lane
// chunks, exit states passed on until no chunk's entry state grows.  A rule
// with bounded match length emits candidate windows of match starts around
// its accepts (a merged run per lane, at most kFsLaneWins per lane per pass,
// then the rest of the file); unbounded rules, or a pass that does not
// settle, make the whole file the candidate (returns true).
constexpr uint32_t kFsLaneWins = 32;

template <int W>
__device__ bool fullscan_pair(const NfaParams& P, const uint8_t* arena, uint32_t f, uint32_t r, uint64_t fs,
                              uint64_t len, const uint64_t* tab, const RuleGpu& rg, uint32_t lane) {
  const uint64_t cs = (len + 63) / 64 > P.fs_chunk ? (len + 63) / 64 : uint64_t(P.fs_chunk);
  const uint64_t a = fs + uint64_t(lane) * cs, b = a + cs < fs + len ? a + cs : fs + len;
  const bool mine = a < fs + len;
  const bool win = rg.max_len != kNoMaxLen;
  int64_t wlo = 0, whi = -1;  // the lane's open window of match starts (file-relative, inclusive)
  uint32_t n_win = 0;
  auto flush = [&]() {
    if (whi >= wlo) put_candidate(P.cands, P.cand_cap, P.counters, f, r, wlo, whi);
    whi = -1;
  };
  auto on_acc = [&](uint64_t abs) -> bool {
    if (!win) return false;  // the first accept decides: the whole file
    const int64_t e = int64_t(abs + 1 - fs);  // the match ends before e
    const int64_t lo = e - int64_t(rg.max_len) > 0 ? e - int64_t(rg.max_len) : 0;
    const int64_t hi = e - int64_t(rg.min_len) < int64_t(len) ? e - int64_t(rg.min_len) : int64_t(len);
    if (whi >= wlo && lo <= whi + 1 && hi + 1 >= wlo) {  // overlaps or touches the open window
      whi = hi > whi ? hi : whi;
      wlo = lo < wlo ? lo : wlo;
      return true;
    }
    flush();
    wlo = lo;
    if (++n_win > kFsLaneWins) {  // many windows: the rest of the file from here
      whi = int64_t(len);
      return false;
    }
    whi = hi;
    return true;
  };
  uint64_t D[W] = {}, E[W] = {};  // exit state, the entry it came from
  bool acc = mine && nfa_chunk<W>(arena, a, b, D, tab, on_acc);
  if (!win && __ballot(acc)) return true;
  if (win && cs >= uint64_t(rg.max_len) + 4) {
    // Bounded matches: a match crossing into chunk c starts in the max_len
    // bytes before it, all inside chunk c-1, so lane c-1's exit state already
    // holds every such path and none of chunk c's exits depends on its entry;
    // the paths from lane c-1 only need the first max_len bytes of chunk c
    // (no start injected), and no fixpoint rounds are needed.
    uint64_t S[W];
#pragma unroll
    for (int w = 0; w < W; w++) {
      const uint32_t lo = __shfl_up(uint32_t(D[w]), 1), hi = __shfl_up(uint32_t(D[w] >> 32), 1);
      S[w] = lane == 0 ? 0 : (uint64_t(hi) << 32) | lo;
    }
    bool any_in = false;
#pragma unroll
    for (int w = 0; w < W; w++) any_in = any_in || S[w] != 0;
    if (mine && any_in) {
      flush();
      n_win = 0;
      const uint64_t e = a + uint64_t(rg.max_len) + 4 < b ? a + uint64_t(rg.max_len) + 4 : b;
      nfa_chunk<W>(arena, a, e, S, tab, on_acc, false);
    }
    flush();
    return false;
  }
  for (int round = 0; round < kFsMaxRounds; round++) {
    uint64_t in[W];
    bool grow = false;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const uint32_t lo = __shfl_up(uint32_t(D[w]), 1), hi = __shfl_up(uint32_t(D[w] >> 32), 1);
      in[w] = (uint64_t(hi) << 32) | lo;  // lane c-1's exit state
      if (lane == 0) in[w] = 0;
      grow = grow || (in[w] & ~E[w]) != 0;
    }
    if (!__ballot(grow && mine)) {  // fixpoint: no chunk's entry state changed
      flush();
      return false;
    }
    if (grow && mine) {
      uint64_t S[W];
#pragma unroll
      for (int w = 0; w < W; w++) {
        E[w] |= in[w];
        S[w] = E[w];
      }
      flush();  // a re-run finds the chunk's accepts again from its start
      n_win = 0;
      acc = nfa_chunk<W>(arena, a, b, S, tab, on_acc);
#pragma unroll
      for (int w = 0; w < W; w++) D[w] = S[w];
    }
    if (!win && __ballot(acc)) return true;
  }
  flush();
  return true;  // not settled: the whole file (always safe)
}

// Full-scan work lists (round 4).  The old shape gave each wave a slab of 64
// (file, rule) slots and ran its open pairs one after another: the pairs of a
// multi-MiB file are adjacent, so a few waves did all the work (C3f: 97 ms,
// 1,091 pairs).  Now fs_pairs_kernel compacts the open pairs into a global
// list and cuts each pair whose rule has a bounded match length into lane
// tasks of task_bytes (>= 8 x max_len): a match ending in a task's range
// [a, b) starts at or after a + 1 - max_len, so each task runs the relaxed NFA
// on its own from there (injection everywhere, accepts before a ignored) and
// needs no state from its neighbours.  fs_task_kernel spreads the tasks over
// every lane of the GPU (one list per NFA width, so the lanes of a wave run
// the same code); unbounded rules keep the wave-wide chunk fixpoint
// (fullscan_pair), one wave per pair from fs_wave_kernel.
struct FsPair {
  uint32_t f, r, task_bytes, pad;
};
struct FsTask {
  uint32_t pair, chunk;
};
struct FsLists {
  FsPair* pairs;
  uint32_t pair_cap;
  FsTask* tasks;  // list w (NFA words w + 1) at tasks + w * task_cap
  uint32_t task_cap;
  uint32_t* wave_pairs;  // pair indices run wave-wide (pair_cap entries)
  uint32_t* ctr;         // [0] pairs [1..4] tasks per NFA width [5] wave pairs
  uint32_t task_min;     // TSG_FS_TASK_BYTES
};
constexpr uint32_t kFsLaneMaxLen = 8192;  // longer bounded matches: the wave path (a lane would own >= 64 KiB)

__global__ __launch_bounds__(256) void fs_pairs_kernel(NfaParams P, FsLists Q) {
  const uint64_t total = uint64_t(P.n_files) * P.n_fullscan_rules;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += stride) {
    // one (file, rule) pair per lane: can its keyword gate be open?
    const uint32_t f = uint32_t(t / P.n_fullscan_rules);
    const uint32_t r = P.fullscan_rules[t % P.n_fullscan_rules];
    const RuleGpu rg = P.rules[r];
    bool open = rg.gate != kGateKeywords || rg.kw_match_implied || kw_bits_inexact(P, f) ||
                (gate_flags(P, rg, f) & kCandGateOpen);
    const uint64_t len = P.off[f + 1] - P.off[f];
    if (!open || len == 0) continue;
    atomicAdd(&P.counters[13], 1u);  // open pairs (stats)
    if (rg.nfa_words == 0) {  // the relaxed NFA accepts at once: the whole file
      put_candidate(P.cands, P.cand_cap, P.counters, f, r, 0, int64_t(len));
      continue;
    }
    const uint32_t p = atomicAdd(&Q.ctr[0], 1u);
    if (p >= Q.pair_cap) {
      P.counters[6] = 1;  // grow and rescan (GpuEngine::Run)
      continue;
    }
    uint32_t tb = 0;
    if (rg.max_len != kNoMaxLen && rg.max_len <= kFsLaneMaxLen) {
      tb = Q.task_min > 8 * rg.max_len ? Q.task_min : 8 * rg.max_len;
      tb = (tb + 15u) & ~15u;
      const uint32_t n = uint32_t((len + tb - 1) / tb);
      const uint32_t w = rg.nfa_words - 1u;
      const uint32_t base = atomicAdd(&Q.ctr[1 + w], n);
      for (uint32_t i = 0; i < n; i++) {
        if (base + i < Q.task_cap) Q.tasks[uint64_t(w) * Q.task_cap + base + i] = FsTask{p, i};
        else P.counters[6] = 1;
      }
    } else {
      Q.wave_pairs[atomicAdd(&Q.ctr[5], 1u)] = p;  // <= pairs <= pair_cap
    }
    Q.pairs[p] = FsPair{f, r, tb, 0};
  }
}

// The relaxed NFA of one lane over arena [s0, e) with a start injected at
// every byte; on_acc(abs) for each accept after byte abs (false stops).  The
// byte-table rows of a group of bytes are loaded before the group's chain of
// steps (they depend on the bytes only), so the chain does not wait for a
// global load per byte.
template <int W, typename Acc>
__device__ void nfa_lane(const uint8_t* __restrict arena, uint64_t s0, uint64_t e, const uint64_t* __restrict tab,
                         Acc on_acc) {
  constexpr int G = W == 1 ? 16 : (W == 2 ? 8 : 4);  // bytes per prefetched group
  uint64_t O[W], Lp[W], F[W], D[W];
#pragma unroll
  for (int w = 0; w < W; w++) {
    O[w] = tab[w];
    Lp[w] = tab[W + w];
    F[w] = tab[2 * W + w];
    D[w] = 0;
  }
  const uint64_t* B = tab + 3 * W;
  for (uint64_t g0 = s0 & ~uint64_t(15); g0 < e; g0 += 16) {
    const uint4 v = load16(arena + g0);
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int h = 0; h < 16; h += G) {
      uint64_t M[G][W];
      uint32_t by[G];
#pragma unroll
      for (int q = 0; q < G; q++) {
        by[q] = (wd[(h + q) >> 2] >> (8 * ((h + q) & 3))) & 0xFFu;
#pragma unroll
        for (int w = 0; w < W; w++) M[q][w] = B[by[q] * W + w];
      }
#pragma unroll
      for (int q = 0; q < G; q++) {
        const uint64_t abs = g0 + uint64_t(h + q);
        if (abs < s0 || abs >= e) continue;
        uint64_t carry = 1, T[W];
#pragma unroll
        for (int w = 0; w < W; w++) {
          T[w] = (D[w] << 1) | carry | (D[w] & Lp[w]);
          carry = D[w] >> 63;
        }
        uint64_t c = 0;
#pragma unroll
        for (int w = 0; w < W; w++) {
          const uint64_t x = T[w] & O[w], s1 = O[w] + x, c1 = s1 < O[w], s2 = s1 + c, c2 = s2 < s1;
          T[w] |= s2 ^ O[w];
          c = c1 | c2;
        }
        const bool keep = (by[q] & 0xC0u) == 0x80u;  // UTF-8 continuation: also stay
        uint64_t acc = 0;
#pragma unroll
        for (int w = 0; w < W; w++) {
          D[w] = (T[w] & M[q][w]) | (keep ? D[w] : 0);
          acc |= D[w] & F[w];
        }
        if (acc && !on_acc(abs)) return;
      }
    }
  }
}

// One lane task: the accepts after bytes [a, b) of the pair's file, as merged
// windows of match starts (scanner.go:409-414 candidates for the host's exact
// FindAll); more than kFsLaneWins windows: one window to the task's end.
template <int W>
__device__ void fs_lane_task(const NfaParams& P, const FsPair& pr, uint32_t chunk) {
  const RuleGpu rg = P.rules[pr.r];
  const uint64_t fs = P.off[pr.f], fe = P.off[pr.f + 1];
  const int64_t len = int64_t(fe - fs);
  const uint64_t a = fs + uint64_t(chunk) * pr.task_bytes;
  if (a >= fe) return;
  const uint64_t b = a + pr.task_bytes < fe ? a + pr.task_bytes : fe;
  const uint64_t back = rg.max_len > 0 ? rg.max_len - 1 : 0;
  const uint64_t s0 = a - fs > back ? a - back : fs;
  int64_t wlo = 0, whi = -1;
  uint32_t n_win = 0;
  auto flush = [&]() {
    if (whi >= wlo) put_candidate(P.cands, P.cand_cap, P.counters, pr.f, pr.r, wlo, whi);
    whi = -1;
  };
  nfa_lane<W>(P.arena, s0, b, P.nfa + rg.nfa_off, [&](uint64_t abs) -> bool {
    if (abs < a) return true;  // the previous task's accept
    const int64_t e = int64_t(abs + 1 - fs);  // the match ends before e
    const int64_t lo = e - int64_t(rg.max_len) > 0 ? e - int64_t(rg.max_len) : 0;
    const int64_t hi = e - int64_t(rg.min_len) < len ? e - int64_t(rg.min_len) : len;
    if (whi >= wlo && lo <= whi + 1 && hi + 1 >= wlo) {
      whi = hi > whi ? hi : whi;
      wlo = lo < wlo ? lo : wlo;
      return true;
    }
    flush();
    wlo = lo;
    if (++n_win > kFsLaneWins) {  // many windows: every start up to the task's end
      whi = int64_t(b - fs);
      return false;
    }
    whi = hi;
    return true;
  });
  flush();
}

__global__ __launch_bounds__(256) void fs_task_kernel(NfaParams P, FsLists Q) {
  uint32_t n[4], total = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    n[w] = Q.ctr[1 + w] < Q.task_cap ? Q.ctr[1 + w] : Q.task_cap;
    total += n[w];
  }
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    uint32_t w = 0, i = t;  // list w holds task t (t < total)
    if (i >= n[0]) {
      i -= n[0];
      w = 1;
      if (i >= n[1]) {
        i -= n[1];
        w = 2;
        if (i >= n[2]) {
          i -= n[2];
          w = 3;
        }
      }
    }
    const FsTask tk = Q.tasks[uint64_t(w) * Q.task_cap + i];
    const FsPair pr = Q.pairs[tk.pair];
    switch (w) {  // uniform except where a wave straddles two lists
      case 0: fs_lane_task<1>(P, pr, tk.chunk); break;
      case 1: fs_lane_task<2>(P, pr, tk.chunk); break;
      case 2: fs_lane_task<3>(P, pr, tk.chunk); break;
      default: fs_lane_task<4>(P, pr, tk.chunk); break;
    }
  }
}

// Unbounded rules (and bounds too long for a lane): one wave per pair.
__global__ __launch_bounds__(256) void fs_wave_kernel(NfaParams P, FsLists Q) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t n_waves = gridDim.x * (blockDim.x / 64);
  const uint32_t n = Q.ctr[5] < Q.pair_cap ? Q.ctr[5] : Q.pair_cap;
  for (uint32_t k = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); k < n; k += n_waves) {
    const FsPair pr = Q.pairs[Q.wave_pairs[k]];
    const RuleGpu rg = P.rules[pr.r];
    const uint64_t fs = P.off[pr.f], len = P.off[pr.f + 1] - fs;
    const uint64_t* tab = P.nfa + rg.nfa_off;
    bool acc;
    switch (rg.nfa_words) {
      case 1: acc = fullscan_pair<1>(P, P.arena, pr.f, pr.r, fs, len, tab, rg, lane); break;
      case 2: acc = fullscan_pair<2>(P, P.arena, pr.f, pr.r, fs, len, tab, rg, lane); break;
      case 3: acc = fullscan_pair<3>(P, P.arena, pr.f, pr.r, fs, len, tab, rg, lane); break;
      default: acc = fullscan_pair<4>(P, P.arena, pr.f, pr.r, fs, len, tab, rg, lane); break;
    }
    if (acc && lane == 0) put_candidate(P.cands, P.cand_cap, P.counters, pr.f, pr.r, 0, int64_t(len));
  }
}

// Finalize: per candidate, the '\n' count before its window (per-chunk counts
// from K1 + the partial chunks) and the keyword-gate flags for the host's
// lazy MatchKeywords, now that every confirm / fold block has set its bits.
// A closed ASCII gate in a file without U+0130 / U+212A is MatchKeywords ==
// false (scanner.go:409): such candidates are marked for dropping.
// One wave per candidate: the lanes sum the whole 1-KiB chunks' counts (a
// window deep in a 10-MiB file spans ~10^4 chunks), lanes 0 / 1 the partial
// chunks at either end.
__global__ __launch_bounds__(256) void finalize_kernel(NfaParams P) {
  const uint32_t n = P.counters[1] < P.cand_cap ? P.counters[1] : P.cand_cap;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t n_waves = gridDim.x * (blockDim.x / 64);
  for (uint32_t i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); i < n; i += n_waves) {
    Candidate& c = P.cands[i];
    const uint32_t file = c.file;
    const uint64_t fs = P.off[file];
    const int64_t nlb = c.nl_before;
    if (nlb < 0) {
      const uint64_t a = fs, b = fs + uint64_t(c.wlo);
      const uint64_t ca = (a + kChunk - 1) / kChunk, cb = b / kChunk;
      int64_t part = 0;
      // partial ranges (< 1 KiB each, < 2 KiB unsplit): one 16-B block per lane
      auto blocks = [&](uint64_t x, uint64_t y) {
        for (uint64_t blk = (x & ~uint64_t(15)) + 16 * lane; blk < y; blk += 16 * 64)
          part += count_nl_range(P.arena, blk > x ? blk : x, blk + 16 < y ? blk + 16 : y);
      };
      if (ca >= cb) {
        blocks(a, b);
      } else {
        blocks(a, ca * kChunk);
        blocks(cb * kChunk, b);
        for (uint64_t cc = ca + lane; cc < cb; cc += 64) part += P.nl[cc];
      }
#pragma unroll
      for (int x = 1; x < 64; x <<= 1) part += __shfl_xor(part, x);
      if (lane == 0) c.nl_before = part;
    }
    // gate flags first: a candidate the host will drop needs no newline hints
    const RuleGpu rg = P.rules[c.rule];
    uint32_t fl = gate_flags(P, rg, file);
    if (rg.gate == kGateKeywords && !rg.kw_match_implied && !kw_bits_inexact(P, file) && !(fl & kCandGateOpen))
      fl |= kCandDrop;
    // the last three '\n' before wlo: 1 KiB per step, lane 0 on the highest
    // 16-B block; a lane's newlines take ranks after those of the lanes above.
    // A 1-KiB chunk whose K1 count is 0 is skipped whole (long single lines).
    if (!(fl & kCandDrop)) {
      const uint64_t wabs = fs + uint64_t(c.wlo);
      uint64_t hi = wabs;  // [fs, hi) still unsearched
      uint32_t found = 0;
      while (found < 3 && hi > fs && wabs - hi < kNlReach) {
        const uint64_t ck = (hi - 1) / kChunk;  // wave-uniform
        if (ck * kChunk >= fs && P.nl[ck] == 0) {  // no '\n' in [ck * kChunk, hi)
          hi = ck * kChunk;
          continue;
        }
        const uint64_t blk = (((hi - 1) >> 4) - lane) << 4;  // may wrap below fs: masked out
        uint32_t mask = 0;
        if (blk + 16 > fs && blk < hi && int64_t(blk) >= 0) {
          const uint4 v = load16(P.arena + blk);
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (uint32_t q = 0; q < 4; q++)
#pragma unroll
            for (uint32_t b = 0; b < 4; b++)
              if (((w[q] >> (8 * b)) & 0xFFu) == uint32_t('\n')) mask |= 1u << (4 * q + b);
          const uint32_t lo_cut = fs > blk ? uint32_t(fs - blk) : 0u;
          const uint32_t hi_cut = hi < blk + 16 ? uint32_t(hi - blk) : 16u;
          mask &= (hi_cut >= 16 ? 0xFFFFu : ((1u << hi_cut) - 1u)) & ~((1u << lo_cut) - 1u);
        }
        const uint32_t cnt = uint32_t(__popc(mask));
        uint32_t incl = cnt;
#pragma unroll
        for (int x = 1; x < 64; x <<= 1) {
          const uint32_t t = __shfl_up(incl, x);
          if (lane >= uint32_t(x)) incl += t;
        }
        uint32_t rank = found + incl - cnt;
        for (uint32_t m = mask; m && rank < 3; rank++) {
          const uint32_t bit = 31u - uint32_t(__clz(m));
          m &= ~(1u << bit);
          c.nl_back[rank] = uint32_t(wabs - (blk + bit));
        }
        found += __shfl(incl, 63);
        const uint64_t low = ((hi - 1) >> 4) >= 63 ? ((((hi - 1) >> 4) - 63) << 4) : 0;
        hi = low;
      }
      if (hi <= fs)  // reached the file start: the remaining ranks do not exist
        for (uint32_t r = found + lane; r < 3; r += 64) c.nl_back[r] = kNlNone;
      // the first three '\n' at or after wlo, the same way forwards: lane 0 on
      // the lowest 16-B block, ranks in lane order
      const uint64_t fe = P.off[file + 1];
      uint64_t lo = wabs;  // [lo, fe) still unsearched
      found = 0;
      while (found < 3 && lo < fe && lo - wabs < kNlReach) {
        const uint64_t ck = lo / kChunk;  // wave-uniform
        if (P.nl[ck] == 0) {              // no '\n' in [lo, (ck + 1) * kChunk)
          lo = (ck + 1) * kChunk;
          continue;
        }
        const uint64_t blk = ((lo >> 4) + lane) << 4;
        uint32_t mask = 0;
        if (blk < fe) {
          const uint4 v = load16(P.arena + blk);
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (uint32_t q = 0; q < 4; q++)
#pragma unroll
            for (uint32_t b = 0; b < 4; b++)
              if (((w[q] >> (8 * b)) & 0xFFu) == uint32_t('\n')) mask |= 1u << (4 * q + b);
          const uint32_t lo_cut = lo > blk ? uint32_t(lo - blk) : 0u;
          const uint32_t hi_cut = fe < blk + 16 ? uint32_t(fe - blk) : 16u;
          mask &= (hi_cut >= 16 ? 0xFFFFu : ((1u << hi_cut) - 1u)) & ~((1u << lo_cut) - 1u);
        }
        const uint32_t cnt = uint32_t(__popc(mask));
        uint32_t incl = cnt;
#pragma unroll
        for (int x = 1; x < 64; x <<= 1) {
          const uint32_t t = __shfl_up(incl, x);
          if (lane >= uint32_t(x)) incl += t;
        }
        uint32_t rank = found + incl - cnt;
        for (uint32_t m = mask; m && rank < 3; rank++) {
          const uint32_t bit = uint32_t(__ffs(m)) - 1u;
          m &= m - 1u;
          c.nl_fwd[rank] = uint32_t(blk + bit - wabs);
        }
        found += __shfl(incl, 63);
        lo = ((lo >> 4) + 64) << 4;
      }
      if (lo >= fe)  // reached the file end: the remaining ranks do not exist
        for (uint32_t r = found + lane; r < 3; r += 64) c.nl_fwd[r] = kNlNone;
    }
    if (lane == 0) c.flags = fl;
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
  if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking) != hipSuccess) {
    err_ = "hipStreamCreate failed";
    return;
  }
  for (auto& e : ev_copied_) hipEventCreateWithFlags(&e, hipEventDisableTiming);
  for (auto& e : ev_h2d_) hipEventCreate(&e);
  for (auto& e : ev_x_) hipEventCreate(&e);
  if (const char* cm = std::getenv("TSG_INGEST_CHUNK_MB")) chunk_bytes_ = uint64_t(std::atoll(cm)) << 20;
  if (chunk_bytes_ < (uint64_t(1) << 20)) chunk_bytes_ = uint64_t(1) << 20;
  for (auto& e : ev_) hipEventCreate(&e);
  if (const char* dm = std::getenv("TSG_DIAG_SCAN")) diag_mode_ = uint32_t(std::atoi(dm));
  if (const char* dc = std::getenv("TSG_DIAG_CONFIRM")) diag_confirm_ = uint32_t(std::atoi(dc));
  if (const char* di = std::getenv("TSG_DIAG_ITEMS")) item_diag_path_ = di;
  if (const char* fc = std::getenv("TSG_FULLSCAN_CHUNK")) fs_chunk_ = uint32_t(std::atoi(fc));
  if (fs_chunk_ < 64) fs_chunk_ = 64;
  if (const char* tb = std::getenv("TSG_FS_TASK_BYTES")) fs_task_bytes_ = uint32_t(std::max(16, std::atoi(tb)));
  hipEventCreate(&ev_fs_);
  // the kernels of one scan run ~10 ms: a thread spinning on the stream for
  // that long takes a core from the host pool scanning the previous batch
  hipEventCreateWithFlags(&ev_sync_, hipEventBlockingSync | hipEventDisableTiming);
  if (const char* bs = std::getenv("TSG_BLOCKING_SYNC")) blocking_sync_ = std::atoi(bs) != 0;
  if (const char* vb = std::getenv("TSG_VERIFY_BLOCKS")) verify_blocks_ = uint32_t(std::max(1, std::atoi(vb)));
  if (const char* fb = std::getenv("TSG_FINALIZE_BLOCKS")) finalize_blocks_ = uint32_t(std::max(1, std::atoi(fb)));
  kw_words_ = std::max<uint32_t>(1, cr.kw_words());
  n_rules_ = uint32_t(cr.rules.size());
  for (uint32_t r = 0; r < n_rules_; r++)
    if (cr.rules[r].has_regex && !cr.rules[r].anchored) fullscan_rules_.push_back(r);
  n_fullscan_rules_ = uint32_t(fullscan_rules_.size());
  if (cr.anchors.size() >= (size_t(1) << kHitAidBits)) {  // hit records keep the anchor id in 24 bits
    err_ = "too many anchors for the hit records (>= 2^24)";
    return;
  }
  if (!Upload(&err_, &d_anchors_, cr.anchors.data(), cr.anchors.size()) ||
      !Upload(&err_, &d_rules_, cr.rules.data(), cr.rules.size()) ||
      !Upload(&err_, &d_rule_kw_, cr.rule_kw.data(), cr.rule_kw.size()) ||
      !Upload(&err_, &d_nfa_, cr.nfa.data(), cr.nfa.size()) ||
      !Upload(&err_, &d_fullscan_rules_, fullscan_rules_.data(), fullscan_rules_.size()))
    return;
  if (hipMalloc(&d_counters_, 64) != hipSuccess || hipMalloc(&d_fs_ctr_, 64) != hipSuccess) {
    err_ = "hipMalloc counters";
    return;
  }
  // streaming prefilter tables (filter.h)
  {
    const FilterTables* ft = cr.filter.get();
    if (!ft || ft->n_words != uint32_t(kFWords) || ft->window != uint32_t(kFWindow) || ft->nl_bucket != 15) {
      err_ = "prefilter shape not supported by the scan kernel (needs 16 buckets, window 6)";
      return;
    }
    if (!Upload(&err_, &d_reach_, ft->reach.data(), ft->reach.size()) ||
        !Upload(&err_, &d_core_, ft->core.data(), ft->core.size()) ||
        !Upload(&err_, &d_group_items_, ft->group_items.data(), ft->group_items.size()) ||
        !Upload(&err_, &d_bucket_groups_, ft->bucket_groups.data(), ft->bucket_groups.size()))
      return;
    auto pad = [](std::vector<uint8_t>& v) { v.resize((v.size() + 15) & ~size_t(15), 0); };
    std::vector<uint8_t> tb;
    auto put = [&](const void* src, size_t n) {
      size_t at = tb.size();
      tb.resize(at + n);
      if (n) std::memcpy(&tb[at], src, n);
      pad(tb);
      return uint32_t(at);
    };
    ft_bucket_off_ = put(ft->bucket_off.data(), ft->bucket_off.size() * 4);
    ft_bucket_items_ = put(ft->bucket_items.data(), ft->bucket_items.size() * 4);
    ft_items_ = put(ft->items.data(), ft->items.size() * sizeof(FilterItemGpu));
    ft_item_ids_ = put(ft->item_ids.data(), ft->item_ids.size() * 4);
    ft_item_cls_ = put(ft->item_cls.data(), ft->item_cls.size());
    ft_classes_ = put(ft->classes.data(), ft->classes.size() * 4);
    ft_luts_ = put(cr.anchor_req.data(), cr.anchor_req.size() * sizeof(FollowLut));
    if (tb.empty()) tb.assign(16, 0);
    ftabs_fold_bytes_ = uint32_t(tb.size());  // the fold kernel stages this prefix
    {  // core tables over byte classes (bytes with equal columns in every group share one)
      const size_t n_groups = ft->bucket_groups.empty() ? 0 : ft->bucket_groups.back();
      std::vector<uint8_t> cmap(256, 0);
      std::vector<uint32_t> rep;  // representative byte per class
      for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = 0;
        for (; c < rep.size(); c++) {
          bool same = true;
          for (size_t g = 0; g < n_groups && same; g++) same = ft->core[g * 256 + b] == ft->core[g * 256 + rep[c]];
          if (same) break;
        }
        if (c == rep.size()) rep.push_back(b);
        cmap[b] = uint8_t(c);
      }
      n_core_cls_ = uint32_t(rep.size());
      std::vector<uint64_t> cc(n_groups * rep.size());
      for (size_t g = 0; g < n_groups; g++)
        for (size_t c = 0; c < rep.size(); c++) cc[g * rep.size() + c] = ft->core[g * 256 + rep[c]];
      ft_cmap_ = put(cmap.data(), cmap.size());
      ft_ccore_ = put(cc.data(), cc.size() * sizeof(uint64_t));
      ft_gitems_ = put(ft->group_items.data(), ft->group_items.size() * 4);
      ft_bgroups_ = put(ft->bucket_groups.data(), ft->bucket_groups.size() * 4);
      ft_hkeys_ = put(ft->hash_keys.data(), ft->hash_keys.size() * 8);
      ft_hitems_ = put(ft->hash_items.data(), ft->hash_items.size() * 4);
      hash_bits_ = ft->hash_bits;
      hash_buckets_ = ft->hash_keys.empty() ? 0u : ft->hash_buckets;
    }
    ftabs_bytes_ = uint32_t(tb.size());
    n_fitems_ = uint32_t(ft->items.size());
    n_fclasses_ = uint32_t(ft->classes.size() / 8);
    for (auto& it : ft->items) {
      h_items_kind_.push_back(it.kind);
      h_items_id_.push_back(ft->item_ids[it.ids_off]);
    }
    uint8_t* d = nullptr;
    if (!Upload(&err_, &d, tb.data(), tb.size())) return;
    d_ftabs_ = d;
    {  // fold work list (FoldParams): (item, q) pairs per rune kind, anchor items only
      auto in_cls = [&](uint32_t c, uint32_t b) { return (ft->classes[c * 8 + (b >> 5)] >> (b & 31)) & 1u; };
      std::vector<FoldPair> pk, ps, ck, cs;  // start ranges / capable positions, per rune kind
      for (uint32_t i = 0; i < uint32_t(ft->items.size()); i++) {
        const FilterItemGpu& it = ft->items[i];
        if (it.kind != kItemAnchor) continue;
        uint32_t before = 0;  // max bytes of positions 0..q-1
        int64_t klo = -1, khi = -1, slo = -1, shi = -1;
        for (uint32_t q = 0; q < it.n; q++) {
          const uint32_t c = ft->item_cls[it.cls_off + q];
          const bool k = in_cls(c, 'k') || in_cls(c, 'K'), sf = in_cls(c, 's') || in_cls(c, 'S');
          if (k || in_cls(c, 0xE2)) {
            if (klo < 0) klo = q;
            khi = before;
            if (q <= 0xFFFF) ck.push_back({i, uint16_t(q), uint16_t(q)});
          }
          if (sf || in_cls(c, 0xC5)) {
            if (slo < 0) slo = q;
            shi = before;
            if (q <= 0xFFFF) cs.push_back({i, uint16_t(q), uint16_t(q)});
          }
          before += k ? 3 : sf ? 2 : 1;
        }
        auto add = [&](std::vector<FoldPair>& v, int64_t lo, int64_t hi) {  // split into bounded tasks
          hi = std::min<int64_t>(hi, 0xFFFF);
          for (int64_t a = lo; a <= hi; a += kFoldTaskStarts)
            v.push_back({i, uint16_t(a), uint16_t(std::min<int64_t>(a + kFoldTaskStarts - 1, hi))});
        };
        if (klo >= 0) add(pk, klo, khi);
        if (slo >= 0) add(ps, slo, shi);
      }
      std::vector<uint32_t> first(8 * std::max<size_t>(ft->items.size(), 1), ~0u);
      for (uint32_t i = 0; i < uint32_t(ft->items.size()); i++) {
        const FilterItemGpu& it = ft->items[i];
        if (it.n == 0) continue;
        const uint32_t c = ft->item_cls[it.cls_off];
        uint32_t* m = &first[8ull * i];
        for (int w = 0; w < 8; w++) m[w] = ft->classes[c * 8 + w];
        if (in_cls(c, 'k') || in_cls(c, 'K')) m[0xE2 >> 5] |= 1u << (0xE2 & 31);
        if (in_cls(c, 's') || in_cls(c, 'S')) m[0xC5 >> 5] |= 1u << (0xC5 & 31);
      }
      uint8_t* dfm = nullptr;
      if (!Upload(&err_, &dfm, reinterpret_cast<const uint8_t*>(first.data()), first.size() * sizeof(uint32_t))) return;
      d_fold_first_ = dfm;
      // byte index of the capable tasks (FoldParams idx_*): key = the byte at
      // x - q (position 0, one byte: no other fold rune precedes x) for q > 0,
      // the byte after the rune (position 1, or a fold lead when position 1
      // can be a fold rune) for q = 0.  The capable lists are reordered so the
      // indexed tasks come first; the rest stay pair-driven.
      {
        std::vector<uint32_t> off(size_t(2) * kFoldIdxQ * 257 + 1, 0);
        std::vector<std::vector<uint32_t>> lists(size_t(2) * kFoldIdxQ * 256);
        auto index_kind = [&](std::vector<FoldPair>& cap, uint32_t kind, uint32_t* n_idx) {
          std::vector<FoldPair> idx, rest;
          for (const FoldPair& fp : cap) {
            const FilterItemGpu& it = ft->items[fp.item];
            const uint32_t q = fp.lo;
            if (q >= uint32_t(kFoldIdxQ) || (q == 0 && it.n < 2)) {
              rest.push_back(fp);
              continue;
            }
            const uint32_t c = ft->item_cls[it.cls_off + (q == 0 ? 1 : 0)];
            for (uint32_t b = 0; b < 256; b++) {
              bool on = in_cls(c, b);
              if (q == 0 && b == 0xE2) on = on || in_cls(c, 'k') || in_cls(c, 'K');
              if (q == 0 && b == 0xC5) on = on || in_cls(c, 's') || in_cls(c, 'S');
              if (on) lists[(size_t(kind) * kFoldIdxQ + q) * 256 + b].push_back(fp.item);
            }
            idx.push_back(fp);
          }
          *n_idx = uint32_t(idx.size());
          idx.insert(idx.end(), rest.begin(), rest.end());
          cap.swap(idx);
        };
        index_kind(ck, 0, &n_fold_cap_k_idx_);
        index_kind(cs, 1, &n_fold_cap_s_idx_);
        std::vector<uint32_t> items_flat;
        for (size_t kq = 0; kq < size_t(2) * kFoldIdxQ; kq++)
          for (uint32_t b = 0; b < 257; b++) {
            off[kq * 257 + b] = uint32_t(items_flat.size());
            if (b < 256) {
              auto& l = lists[kq * 256 + b];
              items_flat.insert(items_flat.end(), l.begin(), l.end());
            }
          }
        if (items_flat.empty()) items_flat.push_back(0);
        uint32_t* d_off = nullptr;
        uint32_t* d_items = nullptr;
        if (!Upload(&err_, &d_off, off.data(), off.size()) || !Upload(&err_, &d_items, items_flat.data(), items_flat.size()))
          return;
        d_fold_idx_off_ = d_off;
        d_fold_idx_items_ = d_items;
        const char* fi = std::getenv("TSG_FOLD_INDEX");  // 0: pair lists only (A/B)
        fold_idx_ = !fi || std::atoi(fi) != 0;
      }
      n_fold_pairs_k_ = uint32_t(pk.size());
      n_fold_pairs_s_ = uint32_t(ps.size());
      n_fold_cap_k_ = uint32_t(ck.size());
      n_fold_cap_s_ = uint32_t(cs.size());
      pk.insert(pk.end(), ps.begin(), ps.end());
      pk.insert(pk.end(), ck.begin(), ck.end());
      pk.insert(pk.end(), cs.begin(), cs.end());
      if (pk.empty()) pk.push_back({0, 0, 0});
      uint8_t* dp = nullptr;
      if (!Upload(&err_, &dp, reinterpret_cast<const uint8_t*>(pk.data()), pk.size() * sizeof(FoldPair))) return;
      d_fold_pairs_ = dp;
    }
    {  // keyword fold work lists (kwfold_kernel): U+0130 at 'i' positions, U+212A at 'k' positions
      auto in_cls = [&](uint32_t c, uint32_t b) { return (ft->classes[c * 8 + (b >> 5)] >> (b & 31)) & 1u; };
      std::vector<FoldPair> ri, rk, ci, ck;
      kw_fold_ = true;
      for (uint32_t i = 0; i < uint32_t(ft->items.size()); i++) {
        const FilterItemGpu& it = ft->items[i];
        if (it.kind != kItemKeyword) continue;
        if (it.n > 48) kw_fold_ = false;  // beyond the kernel's window: keep those files' gates open
        uint32_t before = 0;
        int64_t ilo = -1, ihi = -1, klo = -1, khi = -1;
        for (uint32_t q = 0; q < it.n && q <= 0xFFFF; q++) {
          const uint32_t c = ft->item_cls[it.cls_off + q];
          const bool hi_ = in_cls(c, 'i'), hk = in_cls(c, 'k');
          if (hi_) {
            if (ilo < 0) ilo = q;
            ihi = before;
            ci.push_back({i, uint16_t(q), uint16_t(q)});
          }
          if (hk) {
            if (klo < 0) klo = q;
            khi = before;
            ck.push_back({i, uint16_t(q), uint16_t(q)});
          }
          before += hk ? 3 : hi_ ? 2 : 1;
        }
        auto add = [&](std::vector<FoldPair>& v, int64_t lo, int64_t hi) {
          hi = std::min<int64_t>(hi, 0xFFFF);
          for (int64_t a = lo; a <= hi; a += kFoldTaskStarts)
            v.push_back({i, uint16_t(a), uint16_t(std::min<int64_t>(a + kFoldTaskStarts - 1, hi))});
        };
        if (ilo >= 0) add(ri, ilo, ihi);
        if (klo >= 0) add(rk, klo, khi);
      }
      n_kwf_ri_ = uint32_t(ri.size());
      n_kwf_rk_ = uint32_t(rk.size());
      n_kwf_ci_ = uint32_t(ci.size());
      n_kwf_ck_ = uint32_t(ck.size());
      ri.insert(ri.end(), rk.begin(), rk.end());
      ri.insert(ri.end(), ci.begin(), ci.end());
      ri.insert(ri.end(), ck.begin(), ck.end());
      if (ri.empty()) ri.push_back({0, 0, 0});
      uint8_t* dp = nullptr;
      if (!Upload(&err_, &dp, reinterpret_cast<const uint8_t*>(ri.data()), ri.size() * sizeof(FoldPair))) return;
      d_kwfold_pairs_ = dp;
      if (const char* e = std::getenv("TSG_KWFOLD")) kw_fold_ = kw_fold_ && std::atoi(e) != 0;  // A/B knob
    }
    const size_t fixed = ConfirmFixedLds(kCThreads);
    // Tables staged in LDS only while four workgroups still fit a CU (the
    // register-bound maximum); larger ones are read from global memory
    // (L2-resident).  Measured on C2: LDS tables beat global ones by 17% at
    // equal occupancy, 4 WG/CU beats 2 by 32%; c3 (103 KB of tables): LDS at
    // 1 WG/CU 102 GB/s vs global at 4 WG/CU 164 GB/s.  TSG_LDS_TABS_MAX
    // overrides (tuning).
    size_t lds_max = 160 * 1024 * size_t(kCThreads) / 1024;  // 16 waves per CU
    if (const char* e = std::getenv("TSG_LDS_TABS_MAX")) lds_max = size_t(std::strtoull(e, nullptr, 10));
    // the fold kernel too: its dynamic tables beside its whole static LDS (windows,
    // index lists, cooperative-site state), as the compiler laid it out
    size_t fold_static = kFoldWaves * kFoldWin;
    {
      hipFuncAttributes fa{};
      if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&fold_kernel<true>)) == hipSuccess)
        fold_static = std::max(fold_static, size_t(fa.sharedSizeBytes));
    }
    lds_tabs_ = fixed + ftabs_bytes_ <= lds_max && ftabs_fold_bytes_ + 32 * size_t(n_fitems_) + fold_static <= 64 * 1024;
    if (!item_diag_path_.empty() && hipMalloc(&d_item_diag_, 8 * std::max<size_t>(n_fitems_, 1)) != hipSuccess) {
      err_ = "hipMalloc item diag";
      return;
    }
    c_lds_bytes_ = lds_tabs_ ? fixed + ftabs_bytes_ : ConfirmFixedLds(kCThreadsG);
    // global-table variant: the byte classes in LDS while four workgroups still fit a CU
    // (TSG_CONFIRM_STAGE_CLASSES=0: off)
    {
      const char* sc = std::getenv("TSG_CONFIRM_STAGE_CLASSES");
      c_stage_classes_ = !lds_tabs_ && c_lds_bytes_ + 32 * size_t(n_fclasses_) <= 40 * 1024 && (!sc || std::atoi(sc) != 0);
      if (c_stage_classes_) c_lds_bytes_ += 32 * size_t(n_fclasses_);
    }
    if (const char* e = std::getenv("TSG_CONFIRM_LDS_PAD")) c_lds_bytes_ += size_t(std::strtoull(e, nullptr, 10));  // occupancy experiments
    if (std::getenv("TSG_ENGINE_DEBUG"))
      std::fprintf(stderr, "confirm LDS: fixed %zu + tables %u (fold prefix %u) = %zu B, limit %zu, %s tables, %d threads; "
                   "fold kernel static LDS %zu B\n",
                   fixed, ftabs_bytes_, ftabs_fold_bytes_, c_lds_bytes_, lds_max, lds_tabs_ ? "LDS" : "global",
                   lds_tabs_ ? kCThreads : kCThreadsG, fold_static);
    hipFuncSetAttribute(reinterpret_cast<const void*>(lds_tabs_ ? &confirm_kernel<true> : &confirm_kernel<false>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, int(c_lds_bytes_));
    if (lds_tabs_)
      hipFuncSetAttribute(reinterpret_cast<const void*>(&fold_kernel<true>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          int(ftabs_fold_bytes_ + 32 * n_fitems_));
    // global-table fold kernel: items + classes in LDS up to 48 KiB (TSG_FOLD_STAGE=0: off)
    fold_stage_bytes_ = 16 * size_t(n_fitems_) + 32 * size_t(n_fclasses_);
    const char* fse = std::getenv("TSG_FOLD_STAGE");
    fold_stage_ = !lds_tabs_ && fold_stage_bytes_ <= 48 * 1024 && (!fse || std::atoi(fse) != 0);
    const char* ffe = std::getenv("TSG_FOLD_FIRST");
    fold_check_first_ = !ffe || std::atoi(ffe) != 0;  // r05g: without it 3.0-3.7 ms instead of 1.6-2.1
    // LDS-table fold kernel's grid: every workgroup stages the tables first (TSG_FOLD_GRID)
    if (const char* fg = std::getenv("TSG_FOLD_GRID")) fold_grid_ = uint32_t(std::max(1, std::atoi(fg)));
    const char* fwe = std::getenv("TSG_FOLD_WAVES");
    fold_wide_ = fold_stage_ && (!fwe || std::atoi(fwe) == 16);
    if (std::getenv("TSG_ENGINE_DEBUG"))
      std::fprintf(stderr, "fold: %u items, %u classes, staged %s (%zu B), first-byte test %s, %d waves per workgroup\n",
                   n_fitems_, n_fclasses_,
                   lds_tabs_ ? "(LDS tables)" : fold_stage_ ? "yes" : "no", fold_stage_bytes_,
                   lds_tabs_ || fold_check_first_ ? "on" : "off", fold_wide_ ? 16 : kFoldWaves);
    if (fold_stage_)
      hipFuncSetAttribute(fold_wide_ ? reinterpret_cast<const void*>(&fold_kernel<false, 16>)
                                     : reinterpret_cast<const void*>(&fold_kernel<false>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, int(fold_stage_bytes_));
  }
}

GpuEngine::~GpuEngine() {
  {
    std::lock_guard<std::mutex> g(ring_mu_);
    ring_stop_ = true;
  }
  ring_cv_.notify_all();
  if (copier_.joinable()) copier_.join();
  {
    std::lock_guard<std::mutex> g(reap_mu_);
    reap_stop_ = true;
  }
  reap_cv_.notify_all();
  if (reaper_.joinable()) reaper_.join();
  hipSetDevice(device_);
  void* ps[] = {d_item_diag_, d_fold_pairs_, d_kwfold_pairs_, d_fold_idx_off_, d_fold_idx_items_, d_fold_first_, d_reach_, d_core_, d_group_items_, d_bucket_groups_, d_ftabs_, d_folds_, d_recs_, d_anchors_,
                d_rules_, d_rule_kw_, d_nfa_, d_fullscan_rules_, d_counters_, d_chunk_file_, d_nl_, d_kw_,
                d_flags_, d_hits_, d_cands_, d_fs_pairs_, d_fs_tasks_, d_fs_wave_, d_fs_ctr_, d_xlen_, d_xoff_, d_xscan_,
                d_xf_, d_gfiles_, d_gdst_, d_gbuf_, d_wins_};
  for (void* p : ps)
    if (p) hipFree(p);
  for (int b = 0; b < kNStage; b++)
  {
    for (void* p : {d_stage_[b], d_stage_off_[b], d_kind_[b], d_gsrc_[b]})
      if (p) hipFree(p);
    if (h_gsrc_[b]) hipHostFree(h_gsrc_[b]);
  }
  for (auto& e : ev_)
    if (e) hipEventDestroy(e);
  for (auto& e : ev_copied_)
    if (e) hipEventDestroy(e);
  if (ev_fs_) hipEventDestroy(ev_fs_);
  if (ev_sync_) hipEventDestroy(ev_sync_);
  for (auto& S : slots_) {
    for (auto& e : S.ev)
      if (e) hipEventDestroy(e);
    if (S.ev_fs) hipEventDestroy(S.ev_fs);
    if (S.done) hipEventDestroy(S.done);
    if (S.h_cnt) hipHostFree(S.h_cnt);
    if (S.h_cands) hipHostFree(S.h_cands);
  }
  for (void* p : retired_host_) hipHostFree(p);  // (the reaper was joined first)
  for (auto& e : ev_h2d_)
    if (e) hipEventDestroy(e);
  for (auto& e : ev_x_)
    if (e) hipEventDestroy(e);
  for (auto* h : h_off_)
    if (h) hipHostFree(h);
  if (h_xoff_) hipHostFree(h_xoff_);
  for (void* h : {static_cast<void*>(h_run_cnt_), h_run_cands_, h_gup_, h_gbuf_})
    if (h) hipHostFree(h);
  if (copy_stream_) hipStreamDestroy(copy_stream_);
  if (stream_) hipStreamDestroy(stream_);
}

bool GpuEngine::Ensure(void** p, size_t* cap, size_t need) {
  if (*p && *cap >= need) return true;
  if (*p) {  // queued work (an Enqueue'd scan) may still read the old buffer
    HIP_OK(hipStreamSynchronize(stream_));
    hipFree(*p);
  }
  *p = nullptr;
  // (+1/8: a batch slightly larger than the last does not free and reallocate again --
  // hipFree synchronises the device, stalling the staging ring's copies)
  size_t n = std::max<size_t>(need + need / 8, 64);
  HIP_OK(hipMalloc(p, n));
  *cap = n;
  return true;
}

void GpuEngine::RetireHost(void* p) {
  {
    std::lock_guard<std::mutex> g(reap_mu_);
    retired_host_.push_back(p);
    retired_pending_.fetch_add(1);
    if (!reaper_.joinable()) reaper_ = std::thread([this] { ReaperLoop(); });
  }
  reap_cv_.notify_one();
}

void GpuEngine::ReaperLoop() {
  pthread_setname_np(pthread_self(), "tsg-hostfree");
  // hipHostFree waits for the device by spinning: called while scans keep the
  // GPU busy it burned a core for the whole run (3 CPU-ms per C2 step, r05a).
  // So the buffers are freed once this engine is idle -- no ticket in flight,
  // no host batch in the staging ring -- polled every few ms.
  auto idle = [&] {
    {
      std::lock_guard<std::mutex> g(slot_mu_);
      for (const auto& S : slots_)
        if (S.busy) return false;
    }
    std::lock_guard<std::mutex> g(ring_mu_);
    return ring_turn_ == ring_next_;
  };
  std::unique_lock<std::mutex> lk(reap_mu_);
  for (;;) {
    reap_cv_.wait(lk, [&] { return reap_stop_ || !retired_host_.empty(); });
    if (reap_stop_) return;  // the destructor frees what is left
    lk.unlock();
    while (!idle()) {
      lk.lock();
      const bool stop = reap_cv_.wait_for(lk, std::chrono::milliseconds(5), [&] { return reap_stop_; });
      lk.unlock();
      if (stop) return;
    }
    lk.lock();
    std::vector<void*> batch;
    batch.swap(retired_host_);
    lk.unlock();
    (void)hipSetDevice(device_);
    for (void* p : batch) {
      (void)hipHostFree(p);  // waits for the device: only this thread
      retired_pending_.fetch_sub(1);
      retired_freed_.fetch_add(1);
    }
    lk.lock();
  }
}

GpuEngine::HostMemInfo GpuEngine::host_mem_info() {
  HostMemInfo m{retired_pending_.load(), retired_freed_.load(), cand_cap_, 0};
  std::lock_guard<std::mutex> g(slot_mu_);
  for (const auto& S : slots_) m.slot_bytes += uint64_t(S.h_cap) * sizeof(Candidate);
  return m;
}

bool GpuEngine::EnsureHost(void** p, size_t* cap, size_t need) {
  if (*p && *cap >= need) return true;
  if (*p) hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  const size_t n = std::max<size_t>(need + need / 4, 4096);
  HIP_OK(hipHostMalloc(p, n, hipHostMallocDefault));
  *cap = n;
  return true;
}

// Host-resident batches (the analyzer's pinned arenas, a caller's registered
// pool): the files are cut into chunks of at most chunk_bytes_ at file
// boundaries and streamed through the staging ring (engine.h): the copier
// thread moves chunk slots into the staging buffers on copy_stream_ while the
// kernels of earlier slots run on the scan stream (which waits on the slot's
// copy event).  Pinned host memory is required for the copies to be
// asynchronous (hipHostMalloc / tsg_host_register).  The copies are issued off
// the scanning threads: on this runtime a 1-GiB hipMemcpyAsync from registered
// memory returns only once the transfer is done (profiles/r02_ingest_trace_*).
// TSG_RING_DEBUG=1: one stderr line per ring event (reserve / copy / scan), ms since the first
static void RingLog(const char* what, uint64_t slot, uint64_t extra) {
  static const bool on = std::getenv("TSG_RING_DEBUG") && std::atoi(std::getenv("TSG_RING_DEBUG")) != 0;
  if (!on) return;
  static const auto t0 = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::fprintf(stderr, "ring %10.3f %-12s slot %llu %llu\n", ms, what, (unsigned long long)slot,
               (unsigned long long)extra);
}

struct GpuEngine::HostCall {
  const uint8_t* h_arena;
  const uint64_t* h_offsets;
  const uint8_t* kinds;
  const uint8_t* gather_dev = nullptr;  // device address of the mapped gather_base (RunHost)
  const uint64_t* gather_src = nullptr;
  bool cancelled = false;  // ring_mu_: a chunk failed; the call's later slots are not copied
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // first copy issued / last chunk scanned
  bool ev0_recorded = false;
};

// One chunk slot into staging buffer slot % kNStage (copier thread).  The
// buffer is free: slot - kNStage was scanned (its kernels and copy are done).
// Errors go to *err (err_ belongs to the scanning threads).
bool GpuEngine::CopyChunk(const StageJob& j, std::string* err) {
  const int b = int(j.slot % kNStage);
  const HostCall& c = *j.call;
  const uint64_t a = c.h_offsets[j.f0], e = c.h_offsets[j.f1];
  const uint32_t nf = j.f1 - j.f0;
  auto fail = [&](const char* what, hipError_t x) {
    *err = std::string(what) + ": " + hipGetErrorString(x);
    return false;
  };
  // Growth is rare and generous: hipFree / hipHostFree synchronise the device, so
  // a buffer grown by a few bytes for each slightly larger chunk stalled the copier
  // behind every kernel in flight (20-50 ms, TSG_RING_DEBUG): the arena buffers
  // start at a whole chunk, the per-file arrays grow by half again.
  auto grow = [&](void** p, size_t* cap, size_t need, size_t floor) -> hipError_t {
    if (*p && *cap >= need) return hipSuccess;
    if (*p) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t n = std::max(need + need / 2, floor);
    const hipError_t x = hipMalloc(p, n);
    if (x == hipSuccess) *cap = n;
    return x;
  };
  hipError_t x;
  if ((x = hipEventSynchronize(ev_copied_[b])) != hipSuccess) return fail("staging event", x);  // h_off_[b] reusable
  const size_t arena_need = (e - a) + 64;
  if ((x = grow(&d_stage_[b], &cap_stage_[b], arena_need,
                std::min<size_t>(chunk_bytes_, 4 * (e - a)) + 64)) != hipSuccess ||
      (x = grow(&d_stage_off_[b], &cap_stage_off_[b], (size_t(nf) + 1) * 8, 0)) != hipSuccess ||
      (c.kinds && (x = grow(&d_kind_[b], &cap_kind_[b], size_t(nf) + 1, 0)) != hipSuccess))
    return fail("staging hipMalloc", x);
  if (cap_h_off_[b] < size_t(nf) + 1) {
    if (h_off_[b]) hipHostFree(h_off_[b]);
    h_off_[b] = nullptr;
    cap_h_off_[b] = 0;
    const size_t n = size_t(nf) + 1 + (size_t(nf) + 1) / 2;
    if ((x = hipHostMalloc(reinterpret_cast<void**>(&h_off_[b]), n * 8, hipHostMallocDefault)) != hipSuccess)
      return fail("staging hipHostMalloc", x);
    cap_h_off_[b] = n;
  }
  for (uint32_t f = j.f0; f <= j.f1; f++) h_off_[b][f - j.f0] = c.h_offsets[f] - a;
  if (!c.ev0_recorded) {
    if ((x = hipEventRecord(c.ev0, copy_stream_)) != hipSuccess) return fail("hipEventRecord", x);
    j.call->ev0_recorded = true;
  }
  uint8_t* d = static_cast<uint8_t*>(d_stage_[b]);
  if (c.gather_dev) {
    // the chunk's files gathered from the mapped host buffer by a kernel on the
    // copy stream: their source offsets and (file, piece) items staged first
    // (the pinned staging is reusable: ev_copied_[b] completed above)
    std::vector<GatherItem> items;
    items.reserve(nf);
    for (uint32_t f = 0; f < nf; f++) {
      const uint64_t len = c.h_offsets[j.f0 + f + 1] - c.h_offsets[j.f0 + f];
      for (uint32_t q = 0; uint64_t(q) * kGatherPiece < len; q++) items.push_back(GatherItem{f, q});
    }
    const size_t src_bytes = (size_t(nf) + 1) * 8, item_bytes = items.size() * sizeof(GatherItem);
    const size_t need = src_bytes + item_bytes + 16;
    if ((x = grow(&d_gsrc_[b], &cap_gsrc_[b], need, 0)) != hipSuccess) return fail("gather hipMalloc", x);
    if (cap_h_gsrc_[b] < need) {
      if (h_gsrc_[b]) hipHostFree(h_gsrc_[b]);
      h_gsrc_[b] = nullptr;
      cap_h_gsrc_[b] = 0;
      if ((x = hipHostMalloc(&h_gsrc_[b], need + need / 2, hipHostMallocDefault)) != hipSuccess)
        return fail("gather hipHostMalloc", x);
      cap_h_gsrc_[b] = need + need / 2;
    }
    uint8_t* hs = static_cast<uint8_t*>(h_gsrc_[b]);
    std::memcpy(hs, c.gather_src + j.f0, size_t(nf) * 8);
    std::memcpy(hs + src_bytes, items.data(), item_bytes);
    uint8_t* ds = static_cast<uint8_t*>(d_gsrc_[b]);
    if ((x = hipMemcpyAsync(d_stage_off_[b], h_off_[b], (size_t(nf) + 1) * 8, hipMemcpyHostToDevice, copy_stream_)) !=
            hipSuccess ||
        (x = hipMemcpyAsync(ds, hs, src_bytes + item_bytes, hipMemcpyHostToDevice, copy_stream_)) != hipSuccess ||
        (x = GatherHostFiles(c.gather_dev, reinterpret_cast<const uint64_t*>(ds),
                             static_cast<const uint64_t*>(d_stage_off_[b]),
                             reinterpret_cast<const GatherItem*>(ds + src_bytes), uint32_t(items.size()), d,
                             copy_stream_)) != hipSuccess ||
        (x = hipMemsetAsync(d + (e - a), 0, 64, copy_stream_)) != hipSuccess ||
        (c.kinds && (x = hipMemcpyAsync(d_kind_[b], c.kinds + j.f0, nf, hipMemcpyHostToDevice, copy_stream_)) !=
                        hipSuccess) ||
        (x = hipEventRecord(ev_copied_[b], copy_stream_)) != hipSuccess)
      return fail("chunk gather", x);
    return true;
  }
  // in pieces of at most 1 GiB (a lone file can make a chunk of many GiB)
  for (uint64_t p = a; p < e; p += uint64_t(1) << 30)
    if ((x = hipMemcpyAsync(d + (p - a), c.h_arena + p, std::min<uint64_t>(e - p, uint64_t(1) << 30),
                            hipMemcpyHostToDevice, copy_stream_)) != hipSuccess)
      return fail("chunk copy", x);
  if ((x = hipMemsetAsync(d + (e - a), 0, 64, copy_stream_)) != hipSuccess ||
      (x = hipMemcpyAsync(d_stage_off_[b], h_off_[b], (size_t(nf) + 1) * 8, hipMemcpyHostToDevice, copy_stream_)) !=
          hipSuccess ||
      (c.kinds && (x = hipMemcpyAsync(d_kind_[b], c.kinds + j.f0, nf, hipMemcpyHostToDevice, copy_stream_)) !=
                      hipSuccess) ||
      (x = hipEventRecord(ev_copied_[b], copy_stream_)) != hipSuccess)
    return fail("chunk copy", x);
  return true;
}

void GpuEngine::CopierLoop() {
  pthread_setname_np(pthread_self(), "tsg-copier");
  (void)hipSetDevice(device_);
  std::unique_lock<std::mutex> lk(ring_mu_);
  for (;;) {
    ring_cv_.wait(lk, [&] {
      return ring_stop_ || (!ring_jobs_.empty() && ring_jobs_.front().slot < ring_turn_ + kNStage);
    });
    if (ring_stop_) return;  // (no call in flight: the engine is being destroyed)
    const StageJob j = ring_jobs_.front();
    ring_jobs_.pop_front();
    const bool skip = j.call->cancelled;
    lk.unlock();
    std::string e;
    RingLog("copy-issue", j.slot, ring_turn_);
    RingLog("copy-src", j.slot, (reinterpret_cast<uintptr_t>(j.call->h_arena ? j.call->h_arena + j.call->h_offsets[j.f0]
                                                                               : nullptr) & 0xFFFFF) |
                                    (uint64_t(j.call->h_offsets[j.f1] - j.call->h_offsets[j.f0]) << 20));
    const bool ok = !skip && CopyChunk(j, &e);
    RingLog("copy-issued", j.slot, 0);
    lk.lock();
    const int b = int(j.slot % kNStage);
    stage_ok_[b] = ok;
    stage_err_[b] = skip ? std::string("cancelled") : e;
    ring_copied_ = j.slot + 1;
    ring_cv_.notify_all();
  }
}

bool GpuEngine::RunHost(const uint8_t* h_arena, uint64_t n_bytes, const uint64_t* h_offsets, uint32_t n_files,
                        std::vector<Candidate>* cands, BatchStats* st, const uint8_t* kinds, TailOut* tail,
                        std::mutex* dev_mu, std::string* err, const uint8_t* gather_base,
                        const uint64_t* gather_src) {
  if (!dev_mu) dev_mu = &dev_mu_;
  cands->clear();
  BatchStats local;
  if (!st) st = &local;
  *st = BatchStats();
  st->bytes = n_bytes;
  st->files = n_files;
  if (tail) {
    tail->buf.clear();
    tail->off.assign(size_t(n_files) + 1, 0);
    tail->raw.assign(n_files, 1);
    tail->xform_bytes = 0;
  }
  std::string fail;
  auto set_err = [&](const std::string& m) {  // the caller's message, not err_ (shared)
    if (err) *err = m;
    return false;
  };
  if (kinds && !tail) return set_err("RunHost: a transformed batch needs a tail output");
  if (gather_base && (!gather_src || !kinds)) return set_err("RunHost: a gathered batch needs source offsets and kinds");
  if (n_files == 0) return true;
  const uint8_t* gather_dev = nullptr;
  if (gather_base) {  // the device address of the mapped host buffer (tsg_host_register_mapped)
    void* dp = nullptr;
    if (hipSetDevice(device_) != hipSuccess ||
        hipHostGetDevicePointer(&dp, const_cast<uint8_t*>(gather_base), 0) != hipSuccess || !dp)
      return set_err("RunHost: the gather buffer is not page-locked and mapped (tsg_host_register_mapped)");
    gather_dev = static_cast<const uint8_t*>(dp);
  }
  std::vector<uint64_t> tail_len;  // per file: transformed bytes kept for the host (0: not a candidate file)
  if (kinds) tail_len.assign(n_files, 0);
  // chunk boundaries (file indices)
  std::vector<uint32_t> cut{0};
  for (uint32_t f = 0; f < n_files; f++) {
    const uint64_t c0 = h_offsets[cut.back()];
    if (f > cut.back() && h_offsets[f + 1] - c0 > chunk_bytes_) cut.push_back(f);
  }
  cut.push_back(n_files);
  const size_t n_chunks = cut.size() - 1;
  HostCall call{h_arena, h_offsets, kinds};
  call.gather_dev = gather_dev;
  call.gather_src = gather_src;
  if (hipSetDevice(device_) != hipSuccess || hipEventCreate(&call.ev0) != hipSuccess ||
      hipEventCreate(&call.ev1) != hipSuccess) {
    if (call.ev0) hipEventDestroy(call.ev0);
    return set_err("RunHost: hipEventCreate failed");
  }
  uint64_t s0;
  {
    std::lock_guard<std::mutex> g(ring_mu_);
    if (!copier_.joinable()) copier_ = std::thread(&GpuEngine::CopierLoop, this);
    s0 = ring_next_;
    ring_next_ += n_chunks;
    for (size_t k = 0; k < n_chunks; k++) ring_jobs_.push_back(StageJob{s0 + k, &call, cut[k], cut[k + 1]});
  }
  RingLog("reserve", s0, n_chunks);
  ring_cv_.notify_all();
  bool ok = true;
  std::vector<Candidate> part;
  for (size_t k = 0; k < n_chunks; k++) {
    const uint64_t slot = s0 + k;
    const int b = int(slot % kNStage);
    bool copied;
    {  // this slot's turn (slot order across calls) and its copy issued
      std::unique_lock<std::mutex> lk(ring_mu_);
      ring_cv_.wait(lk, [&] { return ring_turn_ == slot && ring_copied_ > slot; });
      copied = stage_ok_[b];
      if (ok && !copied) {
        ok = false;
        fail = "staging: " + stage_err_[b];
      }
      if (!ok) call.cancelled = true;
    }
    RingLog("turn", slot, 0);
    if (ok) {
      std::unique_lock<std::mutex> g(*dev_mu);
      RingLog("scan-start", slot, 0);
      const uint32_t f0 = cut[k], f1 = cut[k + 1];
      BatchStats cs;
      const uint8_t* scan_arena = static_cast<const uint8_t*>(d_stage_[b]);
      const uint64_t* scan_off = static_cast<const uint64_t*>(d_stage_off_[b]);
      uint64_t scan_bytes = h_offsets[f1] - h_offsets[f0];
      std::vector<uint64_t> xoff;
      float ms_x = 0;
      ok = hipSetDevice(device_) == hipSuccess && hipStreamWaitEvent(stream_, ev_copied_[b], 0) == hipSuccess &&
           (!kinds || Transform(b, f1 - f0, &scan_arena, &scan_off, &scan_bytes, &xoff, &ms_x)) &&
           Run(scan_arena, scan_bytes, scan_off, f1 - f0, &part, &cs);
      if (ok && kinds) {
        st->ms_xform += ms_x;
        cs.ms_total += ms_x;
        tail->xform_bytes += scan_bytes;
        ok = GatherTail(part, f0, f1 - f0, xoff, h_offsets + f0, kinds + f0, &tail_len, tail);
      }
      if (ok && k + 1 == n_chunks) ok = hipEventRecord(call.ev1, stream_) == hipSuccess;
      if (!ok) fail = err_.empty() ? std::string("RunHost: chunk scan failed") : err_;
      if (ok) {
        for (auto c : part) {
          c.file += f0;
          cands->push_back(c);
        }
        st->hits += cs.hits;
        st->follow_hits += cs.follow_hits;
        st->candidates += cs.candidates;
        st->special_files += cs.special_files;
        st->flagged_blocks += cs.flagged_blocks;
        st->hit_overflow = st->hit_overflow || cs.hit_overflow;
        st->cand_overflow = st->cand_overflow || cs.cand_overflow;
        st->ms_scan += cs.ms_scan;
        st->ms_confirm += cs.ms_confirm;
        st->ms_careful += cs.ms_careful;
        st->ms_verify += cs.ms_verify;
        st->ms_fullscan += cs.ms_fullscan;
        st->fullscan_tasks += cs.fullscan_tasks;
        st->fold_sites += cs.fold_sites;
        st->ms_finalize += cs.ms_finalize;
        st->ms_chunkmap += cs.ms_chunkmap;
        st->ms_total += cs.ms_total;
      }
    }
    // the staging buffer goes to slot + kNStage only once nothing reads it
    // (a scanned slot's copy and kernels are done: Run waited for them)
    if (!ok) {
      if (copied) (void)hipStreamSynchronize(copy_stream_);
      (void)hipStreamSynchronize(stream_);  // a failed chunk's kernels may still be queued
    }
    RingLog("scan-end", slot, 0);
    {
      std::lock_guard<std::mutex> g(ring_mu_);
      ring_turn_ = slot + 1;
    }
    ring_cv_.notify_all();
  }
  if (ok) {
    ok = hipEventSynchronize(call.ev1) == hipSuccess;
    hipEventElapsedTime(&st->ms_h2d_span, call.ev0, call.ev1);
    st->h2d_chunks = n_chunks;
    if (kinds)
      for (uint32_t f = 0; f < n_files; f++) tail->off[f + 1] = tail->off[f] + tail_len[f];
  }
  hipEventDestroy(call.ev0);
  hipEventDestroy(call.ev1);
  if (!ok) return set_err(fail.empty() ? std::string("RunHost failed") : fail);
  return true;
}

// Pre-transform of the chunk in staging buffer b (xform.h): lengths, their
// prefix sums (the transformed offsets, also copied back to *xoff), the
// compaction into d_xf_.  Points the scan at the transformed arena.  The
// output buffer is sized by the bound XformMaxOut, so plan and write run back
// to back and the host waits once, for the offsets and the error word together.
bool GpuEngine::Transform(int b, uint32_t nf, const uint8_t** arena, const uint64_t** offsets, uint64_t* n_bytes,
                          std::vector<uint64_t>* xoff, float* ms) {
  const uint64_t raw_bytes = *n_bytes;
  if (!Ensure(&d_xoff_, &cap_xoff_, (size_t(nf) + 1) * 8) ||
      !Ensure(&d_xscan_, &cap_xscan_, XformScratchBytes(raw_bytes, nf)) ||
      !Ensure(&d_xf_, &cap_xf_, XformMaxOut(raw_bytes, nf) + 64))
    return false;
  if (cap_h_xoff_ < size_t(nf) + 2) {  // nf + 1 offsets, then the error word
    if (h_xoff_) hipHostFree(h_xoff_);
    h_xoff_ = nullptr;
    cap_h_xoff_ = 0;
    HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&h_xoff_), (size_t(nf) + 2) * 8, hipHostMallocDefault));
    cap_h_xoff_ = size_t(nf) + 2;
  }
  const uint8_t* raw = static_cast<const uint8_t*>(d_stage_[b]);
  const uint64_t* off = static_cast<const uint64_t*>(d_stage_off_[b]);
  const uint8_t* kd = static_cast<const uint8_t*>(d_kind_[b]);
  uint64_t* xo = static_cast<uint64_t*>(d_xoff_);
  uint8_t* out = static_cast<uint8_t*>(d_xf_);
  h_xoff_[nf + 1] = 0;
  HIP_OK(hipEventRecord(ev_x_[0], stream_));
  if (XformOnePassOn()) {
    HIP_OK(XformOnePass(raw, raw_bytes, off, kd, nf, d_xscan_, xo, out, cap_xf_, stream_));
  } else {
    HIP_OK(XformPlan(raw, raw_bytes, off, kd, nf, d_xscan_, xo, stream_));
    HIP_OK(XformWrite(raw, raw_bytes, off, kd, nf, d_xscan_, out, cap_xf_, stream_));
  }
  HIP_OK(hipMemcpyAsync(h_xoff_, xo, (size_t(nf) + 1) * 8, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipMemcpyAsync(h_xoff_ + nf + 1, XformErrorPtr(raw_bytes, nf, d_xscan_), 4, hipMemcpyDeviceToHost, stream_));
  HIP_OK(hipEventRecord(ev_x_[1], stream_));
  HIP_OK(hipEventSynchronize(ev_x_[1]));
  const uint64_t total = h_xoff_[nf];
  if (const uint32_t xe = uint32_t(h_xoff_[nf + 1]); xe != 0 || total + 64 > cap_xf_) {
    err_ = "GPU pre-transform: output past its buffer (error word " + std::to_string(xe) + ", " +
           std::to_string(total) + " bytes)";
    return false;
  }
  if (XformOnePassOn()) HIP_OK(hipMemsetAsync(out + total, 0, 64, stream_));  // (XformWrite zeroes them)
  xoff->assign(h_xoff_, h_xoff_ + nf + 1);
  hipEventElapsedTime(ms, ev_x_[0], ev_x_[1]);
  *arena = out;
  *offsets = xo;
  *n_bytes = total;
  return true;
}

// The transformed bytes of the chunk's files with candidates -> tail->buf
// (appended in file order); their lengths -> (*tail_len)[f0 + f].
bool GpuEngine::GatherTail(const std::vector<Candidate>& part, uint32_t f0, uint32_t nf,
                           const std::vector<uint64_t>& xoff, const uint64_t* raw_off, const uint8_t* kinds,
                           std::vector<uint64_t>* tail_len, TailOut* tail) {
  // only the files the transform changed (a CRLF file, .pyc printable runs):
  // the others are read where they are in the host batch (TailOut::raw)
  std::vector<uint32_t> files;
  files.reserve(part.size());
  for (const auto& c : part)
    if (c.file < nf && (kinds[c.file] == 2 || xoff[c.file + 1] - xoff[c.file] != raw_off[c.file + 1] - raw_off[c.file]))
      files.push_back(c.file);
  std::sort(files.begin(), files.end());
  files.erase(std::unique(files.begin(), files.end()), files.end());
  for (uint32_t f : files) tail->raw[f0 + f] = 0;
  if (files.empty()) return true;
  std::vector<uint64_t> dst(files.size());
  uint64_t total = 0;
  for (size_t i = 0; i < files.size(); i++) {
    if (files[i] >= nf) {
      err_ = "candidate file outside its chunk";
      return false;
    }
    dst[i] = total;
    const uint64_t len = xoff[files[i] + 1] - xoff[files[i]];
    (*tail_len)[f0 + files[i]] = len;
    total += len;
  }
  if (!Ensure(&d_gfiles_, &cap_gfiles_, files.size() * 4) || !Ensure(&d_gdst_, &cap_gdst_, files.size() * 8) ||
      !Ensure(&d_gbuf_, &cap_gbuf_, total + 64))
    return false;
  // uploads and read-back through pinned staging (engine.h)
  const size_t up = files.size() * 12;
  if (!EnsureHost(&h_gup_, &cap_h_gup_, up) || !EnsureHost(&h_gbuf_, &cap_h_gbuf_, total + 1)) return false;
  uint8_t* hu = static_cast<uint8_t*>(h_gup_);
  std::memcpy(hu, dst.data(), dst.size() * 8);
  std::memcpy(hu + dst.size() * 8, files.data(), files.size() * 4);
  HIP_OK(hipMemcpyAsync(d_gdst_, hu, dst.size() * 8, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipMemcpyAsync(d_gfiles_, hu + dst.size() * 8, files.size() * 4, hipMemcpyHostToDevice, stream_));
  HIP_OK(GatherFiles(static_cast<const uint8_t*>(d_xf_), static_cast<const uint64_t*>(d_xoff_),
                     static_cast<const uint32_t*>(d_gfiles_), static_cast<const uint64_t*>(d_gdst_),
                     uint32_t(files.size()), static_cast<uint8_t*>(d_gbuf_), stream_));
  HIP_OK(hipMemcpyAsync(h_gbuf_, d_gbuf_, total, hipMemcpyDeviceToHost, stream_));
  HIP_OK(WaitStream());
  const size_t at = tail->buf.size();
  tail->buf.resize(at + total);
  std::memcpy(tail->buf.data() + at, h_gbuf_, total);
  return true;
}

// Waits for a scan's kernels sleep-poll the event (TSG_WAIT_POLL_US, default
// 200 us): even a hipEventBlockingSync wait spun in the runtime long enough to
// cost ~14 CPU-ms per C2 step, and the host side is bound by the
// box's CPU quota; 200 us of wake-up latency is hidden by the pipeline.
hipError_t GpuEngine::WaitEvent(hipEvent_t ev) {
  static const int poll_us = std::getenv("TSG_WAIT_POLL_US") ? std::atoi(std::getenv("TSG_WAIT_POLL_US")) : 200;
  if (poll_us <= 0) return hipEventSynchronize(ev);
  hipError_t e;
  while ((e = hipEventQuery(ev)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(poll_us));
  return e;
}

hipError_t GpuEngine::WaitStream() {
  if (!blocking_sync_ || !ev_sync_) return hipStreamSynchronize(stream_);
  hipError_t e = hipEventRecord(ev_sync_, stream_);
  return e != hipSuccess ? e : WaitEvent(ev_sync_);
}

void GpuEngine::InitCaps(uint64_t n_bytes) {
  if (hit_cap_ == 0) hit_cap_ = uint32_t(std::min<uint64_t>(std::max<uint64_t>(n_bytes / 512, 1 << 16), 1u << 28));
  if (cand_cap_ == 0) cand_cap_ = 1 << 16;
  if (rec_cap_ == 0) rec_cap_ = uint32_t(std::min<uint64_t>(std::max<uint64_t>(n_bytes / 128, 1 << 16), 1u << 30));
  if (fold_cap_ == 0) fold_cap_ = 1 << 16;
  if (fs_pair_cap_ == 0) fs_pair_cap_ = 1 << 14;
  if (fs_task_cap_ == 0) fs_task_cap_ = 1 << 16;
}

bool GpuEngine::Enqueue(const uint8_t* d_arena, uint64_t n_bytes, const uint64_t* d_offsets, uint32_t n_files,
                        Ticket* t, std::string* err) {
  t->slot = -1;
  if (n_files == 0 || n_bytes >= (uint64_t(1) << 36) - 64 || d_item_diag_ || diag_mode_ != 0) return false;
  int k = -1;
  {
    std::lock_guard<std::mutex> g(slot_mu_);
    for (int i = 0; i < kSlots && k < 0; i++)
      if (!slots_[i].busy) {
        slots_[i].busy = true;
        k = i;
      }
  }
  if (k < 0) return false;
  Slot& S = slots_[k];
  auto fail = [&] {
    // copies into the slot's pinned buffers may be queued: let them finish
    // before the slot (and its buffers) can be reused or freed
    (void)hipStreamSynchronize(stream_);
    *err = err_.empty() ? "Enqueue failed" : err_;
    std::lock_guard<std::mutex> g(slot_mu_);
    S.busy = false;
    return false;
  };
  if (hipSetDevice(device_) != hipSuccess) return fail();
  InitCaps(n_bytes);
  if (!S.done) {
    bool ok = hipEventCreateWithFlags(&S.done, hipEventBlockingSync | hipEventDisableTiming) == hipSuccess &&
              hipEventCreate(&S.ev_fs) == hipSuccess &&
              hipHostMalloc(reinterpret_cast<void**>(&S.h_cnt), 64, hipHostMallocDefault) == hipSuccess;
    for (auto& e : S.ev) ok = ok && hipEventCreate(&e) == hipSuccess;
    if (!ok) {
      err_ = "ticket events / pinned counters";
      return fail();
    }
  }
  const uint32_t n_copy = uint32_t(std::min<uint64_t>(cand_cap_, 2 * uint64_t(cand_recent_.load()) + 65536));
  if (S.h_cap < n_copy) {
    // Sized to the device list's capacity (not to the copy, which follows the
    // recent counts): hipHostFree waits for the whole device, so a slot regrown
    // in a running pipeline stalled its submitting thread -- holding the GPU
    // lock -- for 11-19 ms and left the GPU idle 1.7 ms per regrowth
    // (tools/drain_trace.py, profiles/r04h2).  It regrows only with cand_cap_,
    // and the old buffer goes to the reaper thread (RetireHost), which frees it
    // outside the engine's locks.
    if (S.h_cands) RetireHost(S.h_cands);
    {
      std::lock_guard<std::mutex> g(slot_mu_);
      S.h_cands = nullptr;
      S.h_cap = 0;
    }
    Candidate* hc = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&hc), size_t(cand_cap_) * sizeof(Candidate), hipHostMallocDefault) !=
        hipSuccess) {
      err_ = "hipHostMalloc failed for the candidate read-back";
      return fail();
    }
    std::lock_guard<std::mutex> g(slot_mu_);
    S.h_cands = hc;
    S.h_cap = cand_cap_;
  }
  uint64_t n_chunks = (n_bytes + kChunk - 1) / kChunk;
  if (n_chunks == 0) n_chunks = 1;
  if (!EnqueuePhase(d_arena, n_bytes, d_offsets, n_files, n_chunks, S.ev, S.ev_fs) ||
      hipMemcpyAsync(S.h_cnt, d_counters_, 64, hipMemcpyDeviceToHost, stream_) != hipSuccess ||
      hipMemcpyAsync(S.h_cands, d_cands_, size_t(n_copy) * sizeof(Candidate), hipMemcpyDeviceToHost, stream_) !=
          hipSuccess ||
      hipEventRecord(S.done, stream_) != hipSuccess) {
    if (err_.empty()) err_ = "Enqueue: HIP call failed";
    return fail();
  }
  S.n_bytes = n_bytes;
  S.n_files = n_files;
  S.has_fs = n_fullscan_rules_ > 0;
  t->slot = k;
  t->cand_copy = n_copy;
  return true;
}

bool GpuEngine::Collect(Ticket* t, std::vector<Candidate>* cands, BatchStats* st, bool* rerun, std::string* err) {
  *rerun = false;
  if (t->slot < 0 || t->slot >= kSlots) {
    *err = "Collect: no ticket";
    return false;
  }
  Slot& S = slots_[t->slot];
  auto release = [&] {
    std::lock_guard<std::mutex> g(slot_mu_);
    S.busy = false;
    t->slot = -1;
  };
  const hipError_t e = WaitEvent(S.done);
  if (e != hipSuccess) {
    *err = std::string("Collect: ") + hipGetErrorString(e);
    release();
    return false;
  }
  BatchStats local;
  if (!st) st = &local;
  *st = BatchStats();
  st->bytes = S.n_bytes;
  st->files = S.n_files;
  const uint32_t* cnt = S.h_cnt;
  for (uint32_t seen = cand_recent_.load(); cnt[1] > seen && !cand_recent_.compare_exchange_weak(seen, cnt[1]);) {
  }
  if (cnt[8] || cnt[10] || cnt[3] || cnt[4] || cnt[6] || cnt[1] > t->cand_copy) {  // an overflow: Run grows and rescans
    *rerun = true;
    release();
    return true;
  }
  st->hits = cnt[11];
  st->follow_hits = cnt[0];
  st->special_files = cnt[2];
  st->flagged_blocks = cnt[7];
  st->fullscan_tasks = cnt[13];
  st->fold_sites = cnt[9];
  cands->clear();
  cands->reserve(cnt[1]);
  for (uint32_t i = 0; i < cnt[1]; i++)  // closed keyword gates (finalize_kernel) never reach the host
    if (!(S.h_cands[i].flags & kCandDrop)) cands->push_back(S.h_cands[i]);
  st->candidates = cands->size();
  hipEventElapsedTime(&st->ms_scan, S.ev[1], S.ev[2]);
  hipEventElapsedTime(&st->ms_confirm, S.ev[2], S.ev[3]);
  hipEventElapsedTime(&st->ms_careful, S.ev[3], S.ev[4]);
  hipEventElapsedTime(&st->ms_verify, S.ev[4], S.ev[5]);
  hipEventElapsedTime(&st->ms_finalize, S.ev[5], S.ev[6]);
  if (S.has_fs) hipEventElapsedTime(&st->ms_fullscan, S.ev_fs, S.ev[5]);
  hipEventElapsedTime(&st->ms_chunkmap, S.ev[0], S.ev[1]);
  hipEventElapsedTime(&st->ms_total, S.ev[0], S.ev[6]);
  release();
  return true;
}

// The GPU phase of one scan, enqueued on stream_: clears, K0 .. finalize,
// with the phase events recorded into ev[0..6] (ev_fs before the full scan).
bool GpuEngine::EnqueuePhase(const uint8_t* d_arena, uint64_t n_bytes, const uint64_t* d_offsets, uint32_t n_files,
                             uint64_t n_chunks, hipEvent_t* ev, hipEvent_t ev_fs) {
  if (!Ensure(&d_chunk_file_, &cap_chunk_file_, n_chunks * 4) || !Ensure(&d_nl_, &cap_nl_, (n_chunks + 8) * 2) ||
      !Ensure(&d_kw_, &cap_kw_, size_t(n_files) * kw_words_ * 4) ||
      !Ensure(&d_flags_, &cap_flags_, size_t(n_files) * 4) ||
      !Ensure(&d_folds_, &cap_folds_, size_t(fold_cap_) * sizeof(FoldSite)) ||
      !Ensure(&d_recs_, &cap_recs_, size_t(rec_cap_) * 4) ||
      !Ensure(&d_hits_, &cap_hits_, size_t(hit_cap_) * 12) ||
      !Ensure(&d_cands_, &cap_cands_, size_t(cand_cap_) * sizeof(Candidate)))
    return false;
  if (n_fullscan_rules_ > 0 &&
      (!Ensure(&d_fs_pairs_, &cap_fs_pairs_, size_t(fs_pair_cap_) * sizeof(FsPair)) ||
       !Ensure(&d_fs_wave_, &cap_fs_wave_, size_t(fs_pair_cap_) * 4) ||
       !Ensure(&d_fs_tasks_, &cap_fs_tasks_, size_t(fs_task_cap_) * 4 * sizeof(FsTask))))
    return false;
  HIP_OK(hipEventRecord(ev[0], stream_));  // the GPU phase: K0 (with the clears) .. finalize
  if (d_item_diag_) HIP_OK(hipMemsetAsync(d_item_diag_, 0, 8 * std::max<size_t>(n_fitems_, 1), stream_));
  {  // every chunk below n_bytes gets its file (no clear needed)
    const uint64_t used = (n_bytes + kChunk - 1) / kChunk;
    const uint64_t runs = (used + kK0Run - 1) / kK0Run;
    const uint64_t clear_q = (uint64_t(n_files) * (1 + kw_words_) + 3) / 4;  // 16-B clear stores
    const uint64_t work = std::max(runs, clear_q);
    const uint32_t blocks = uint32_t(std::max<uint64_t>(1, std::min<uint64_t>((work + 255) / 256, 8192)));
    ClearParams z;
    z.flags = static_cast<uint32_t*>(d_flags_);
    z.kw = static_cast<uint32_t*>(d_kw_);
    z.n_kw = uint64_t(n_files) * kw_words_;
    z.counters = d_counters_;
    z.fs_ctr = n_fullscan_rules_ > 0 ? d_fs_ctr_ : nullptr;
    chunk_map_kernel<<<blocks, 256, 0, stream_>>>(d_offsets, n_files, used, static_cast<uint32_t*>(d_chunk_file_),
                                                  z);
  }
  // K1: streaming filter -> flagged block records
  FilterParams fp;
  fp.arena = d_arena;
  fp.n_bytes = n_bytes;
  fp.reach = d_reach_;
  fp.diag_mode = diag_mode_;
  fp.nl = static_cast<uint16_t*>(d_nl_);
  fp.recs = static_cast<uint32_t*>(d_recs_);
  fp.rec_cap = rec_cap_;
  fp.counters = d_counters_;
  const uint64_t f_tiles = (n_bytes + kFTile - 1) / kFTile;
  const uint32_t f_grid =
      uint32_t(std::max<uint64_t>(1, std::min<uint64_t>((f_tiles + kScanWaves - 1) / kScanWaves, 256 * kFWgPerCu)));
  HIP_OK(hipEventRecord(ev[1], stream_));
  filter_kernel<<<f_grid, kScanThreads, 0, stream_>>>(fp);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(ev[2], stream_));
  // K2: confirm + verify
  ConfirmParams cp;
  cp.arena = d_arena;
  cp.n_bytes = n_bytes;
  cp.off = d_offsets;
  cp.chunk_file = static_cast<const uint32_t*>(d_chunk_file_);
  cp.nl = static_cast<const uint16_t*>(d_nl_);
  cp.reach = d_reach_;
  cp.tabs = d_ftabs_;
  cp.tabs_bytes = ftabs_bytes_;
  cp.t_bucket_off = ft_bucket_off_;
  cp.t_bucket_items = ft_bucket_items_;
  cp.t_items = ft_items_;
  cp.t_item_ids = ft_item_ids_;
  cp.t_item_cls = ft_item_cls_;
  cp.t_classes = ft_classes_;
  cp.anchors = d_anchors_;
  cp.rules = d_rules_;
  cp.nfa = d_nfa_;
  cp.recs = static_cast<const uint32_t*>(d_recs_);
  cp.rec_cap = rec_cap_;
  cp.flags = static_cast<uint32_t*>(d_flags_);
  cp.counters = d_counters_;
  cp.hits = static_cast<uint32_t*>(d_hits_);
  cp.hit_cap = hit_cap_;
  cp.folds = static_cast<FoldSite*>(d_folds_);
  cp.fold_cap = fold_cap_;
  cp.diag = diag_confirm_;
  cp.kwbits = static_cast<uint32_t*>(d_kw_);
  cp.kw_words = kw_words_;
  cp.core = d_core_;
  cp.group_items = d_group_items_;
  cp.bucket_groups = d_bucket_groups_;
  cp.item_diag = d_item_diag_;
  cp.t_luts = ft_luts_;
  cp.t_cmap = ft_cmap_;
  cp.t_ccore = ft_ccore_;
  cp.t_gitems = ft_gitems_;
  cp.t_bgroups = ft_bgroups_;
  cp.n_cls = n_core_cls_;
  cp.t_hkeys = ft_hkeys_;
  cp.t_hitems = ft_hitems_;
  cp.hash_bits = hash_bits_;
  cp.hash_buckets = hash_buckets_;
  cp.n_classes_lds = c_stage_classes_ ? n_fclasses_ : 0u;
  cp.wins = nullptr;
  static const bool k2_pack = std::getenv("TSG_K2_PACK") && std::atoi(std::getenv("TSG_K2_PACK")) != 0;
  if (k2_pack && diag_mode_ == 0) {  // (experiment) the windows packed between K1 and K2, outside K2's events
    if (!Ensure(&d_wins_, &cap_wins_, size_t(rec_cap_) * 64)) return false;
    pack_windows_kernel<<<8192, 256, 0, stream_>>>(d_arena, n_bytes, static_cast<const uint32_t*>(d_recs_), rec_cap_,
                                                   d_counters_, static_cast<uint8_t*>(d_wins_));
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(ev[2], stream_));  // re-recorded: K1 + pack count as the scan phase, K2 alone as confirm
    cp.wins = static_cast<const uint8_t*>(d_wins_);
  }
  if (diag_mode_ == 0) {
    if (lds_tabs_)
      confirm_kernel<true><<<2048 * 256 / kCThreads, kCThreads, c_lds_bytes_, stream_>>>(cp);
    else
      confirm_kernel<false><<<2048 * 256 / kCThreadsG, kCThreadsG, c_lds_bytes_, stream_>>>(cp);
  }
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(ev[3], stream_));
  // fold runes: fold-tolerant item matching around each one
  FoldParams fo;
  fo.arena = d_arena;
  fo.off = d_offsets;
  fo.tabs = d_ftabs_;
  fo.tabs_bytes = ftabs_fold_bytes_;
  fo.t_items = ft_items_;
  fo.t_item_ids = ft_item_ids_;
  fo.t_item_cls = ft_item_cls_;
  fo.t_classes = ft_classes_;
  fo.n_items = n_fitems_;
  fo.stage_items = fold_stage_ ? 1u : 0u;
  fo.n_classes = n_fclasses_;
  fo.check_first = fold_check_first_ ? 1u : 0u;
  static const uint32_t fold_diag = std::getenv("TSG_DIAG_FOLD") ? uint32_t(std::atoi(std::getenv("TSG_DIAG_FOLD"))) : 0u;
  fo.diag = fold_diag;
  fo.pairs = static_cast<const FoldPair*>(d_fold_pairs_);
  fo.first = static_cast<const uint32_t*>(d_fold_first_);
  fo.n_pairs_k = n_fold_pairs_k_;
  fo.n_pairs_s = n_fold_pairs_s_;
  fo.n_cap_k = n_fold_cap_k_;
  fo.n_cap_s = n_fold_cap_s_;
  fo.folds = static_cast<const FoldSite*>(d_folds_);
  fo.fold_cap = fold_cap_;
  fo.idx_off = static_cast<const uint32_t*>(d_fold_idx_off_);
  fo.idx_items = static_cast<const uint32_t*>(d_fold_idx_items_);
  fo.use_idx = fold_idx_ ? 1u : 0u;
  fo.n_cap_k_idx = n_fold_cap_k_idx_;
  fo.n_cap_s_idx = n_fold_cap_s_idx_;
  fo.hits = static_cast<uint32_t*>(d_hits_);
  fo.hit_cap = hit_cap_;
  fo.counters = d_counters_;
  if (diag_mode_ == 0) {
    if (lds_tabs_)
      fold_kernel<true><<<fold_grid_, 64 * kFoldWaves, ftabs_fold_bytes_ + 32 * n_fitems_, stream_>>>(fo);
    else if (fold_wide_)
      fold_kernel<false, 16><<<2048, 64 * 16, fold_stage_bytes_, stream_>>>(fo);
    else
      fold_kernel<false><<<2048, 64 * kFoldWaves, fold_stage_ ? fold_stage_bytes_ : 0, stream_>>>(fo);
  }
  HIP_OK(hipGetLastError());
  if (diag_mode_ == 0 && kw_fold_ && n_kwf_ci_ + n_kwf_ck_ > 0) {
    KwFoldParams kf;
    kf.arena = d_arena;
    kf.off = d_offsets;
    kf.tabs = static_cast<const uint8_t*>(d_ftabs_);
    kf.t_items = ft_items_;
    kf.t_item_ids = ft_item_ids_;
    kf.t_item_cls = ft_item_cls_;
    kf.t_classes = ft_classes_;
    kf.pairs = static_cast<const FoldPair*>(d_kwfold_pairs_);
    kf.n_rng_i = n_kwf_ri_;
    kf.n_rng_k = n_kwf_rk_;
    kf.n_cap_i = n_kwf_ci_;
    kf.n_cap_k = n_kwf_ck_;
    kf.folds = static_cast<const FoldSite*>(d_folds_);
    kf.fold_cap = fold_cap_;
    kf.counters = d_counters_;
    kf.kwbits = static_cast<uint32_t*>(d_kw_);
    kf.kw_words = kw_words_;
    kwfold_kernel<<<1024, 64 * kFoldWaves, 0, stream_>>>(kf);
    HIP_OK(hipGetLastError());
  }
  HIP_OK(hipEventRecord(ev[4], stream_));
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
  static const uint32_t verify_diag = std::getenv("TSG_DIAG_VERIFY") ? uint32_t(std::atoi(std::getenv("TSG_DIAG_VERIFY"))) : 0u;
  np.diag = verify_diag;
  np.cands = static_cast<Candidate*>(d_cands_);
  np.cand_cap = cand_cap_;
  np.fullscan_rules = d_fullscan_rules_;
  np.n_fullscan_rules = n_fullscan_rules_;
  np.fs_chunk = fs_chunk_;
  np.kw_fold = kw_fold_ ? 1u : 0u;  // no keyword takes 'i' / 'k': the bits are exact without the kernel

  if (diag_mode_ == 0) verify_hits_kernel<<<verify_blocks_, 256, 0, stream_>>>(np);
  HIP_OK(hipGetLastError());
  if (np.n_fullscan_rules > 0) {
    HIP_OK(hipEventRecord(ev_fs, stream_));
    FsLists fq;
    fq.pairs = static_cast<FsPair*>(d_fs_pairs_);
    fq.pair_cap = fs_pair_cap_;
    fq.tasks = static_cast<FsTask*>(d_fs_tasks_);
    fq.task_cap = fs_task_cap_;
    fq.wave_pairs = static_cast<uint32_t*>(d_fs_wave_);
    fq.ctr = d_fs_ctr_;
    fq.task_min = fs_task_bytes_;  // (fq.ctr was cleared by K0)
    const uint64_t pairs = uint64_t(n_files) * n_fullscan_rules_;
    const uint32_t pb = uint32_t(std::min<uint64_t>(std::max<uint64_t>((pairs + 255) / 256, 1), 4096));
    fs_pairs_kernel<<<pb, 256, 0, stream_>>>(np, fq);
    HIP_OK(hipGetLastError());
    fs_task_kernel<<<2048, 256, 0, stream_>>>(np, fq);
    HIP_OK(hipGetLastError());
    fs_wave_kernel<<<1024, 256, 0, stream_>>>(np, fq);
    HIP_OK(hipGetLastError());
  }
  HIP_OK(hipEventRecord(ev[5], stream_));
  if (diag_mode_ == 0) finalize_kernel<<<finalize_blocks_, 256, 0, stream_>>>(np);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(ev[6], stream_));
  return true;
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
  if (n_bytes >= (uint64_t(1) << 36) - 64) {
    err_ = "batch arena must be < 64 GiB";
    return false;
  }
  uint64_t n_chunks = (n_bytes + kChunk - 1) / kChunk;
  if (n_chunks == 0) n_chunks = 1;
  InitCaps(n_bytes);
  for (int attempt = 0; attempt < 8; attempt++) {
    if (!EnqueuePhase(d_arena, n_bytes, d_offsets, n_files, n_chunks, ev_, ev_fs_)) return false;
    uint32_t cnt[16];
    if (!h_run_cnt_) HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&h_run_cnt_), 64, hipHostMallocDefault));
    HIP_OK(hipMemcpyAsync(h_run_cnt_, d_counters_, sizeof(cnt), hipMemcpyDeviceToHost, stream_));
    HIP_OK(WaitStream());
    std::memcpy(cnt, h_run_cnt_, sizeof(cnt));
    if (std::getenv("TSG_STATS_DEBUG"))
      std::fprintf(stderr, "counters: hits %u cands %u special %u recs %u folds %u\n", cnt[0], cnt[1], cnt[2], cnt[7],
                   cnt[9]);
    st->hits = cnt[11];  // exact anchor-item matches in the confirm kernel
    st->follow_hits = cnt[0];  // past the follow requirements (+ fold-kernel hits): the verify kernel's input
    st->special_files = cnt[2];
    st->flagged_blocks = cnt[7];
    if (cnt[8]) {  // record list overflow: grow and rescan
      rec_cap_ = uint32_t(std::min<uint64_t>(uint64_t(cnt[7]) + cnt[7] / 4 + 4096, 0xFFFFFFF0u / 4));
      continue;
    }
    st->hit_overflow = cnt[3] != 0;
    st->cand_overflow = cnt[4] != 0;
    if (cnt[6]) {  // full-scan pair / task list overflow: grow to the counts seen
      uint32_t fc[16];
      HIP_OK(hipMemcpy(fc, d_fs_ctr_, sizeof(fc), hipMemcpyDeviceToHost));
      fs_pair_cap_ = std::max<uint32_t>(fs_pair_cap_, fc[0] + fc[0] / 4 + 1024);
      const uint32_t mt = std::max(std::max(fc[1], fc[2]), std::max(fc[3], fc[4]));
      constexpr uint64_t kMaxTasks = 0x7FFFFFFFu / sizeof(FsTask) / 4;
      const uint64_t want = uint64_t(mt) + mt / 4 + 1024;
      if (want > kMaxTasks) {
        // the lists cannot grow that far: coarser lane tasks instead (any task
        // size is exact -- each lane starts max_len bytes before its range), so
        // the scan degrades instead of failing with an overflow on every attempt
        uint64_t tb = fs_task_bytes_;
        while (tb < (uint64_t(1) << 26) && want * fs_task_bytes_ / tb > kMaxTasks) tb *= 2;
        fs_task_bytes_ = uint32_t(tb);
      }
      fs_task_cap_ = uint32_t(std::min<uint64_t>(std::max<uint64_t>(fs_task_cap_, want), kMaxTasks));
      continue;
    }
    if (cnt[10]) {  // fold site list overflow
      fold_cap_ = uint32_t(std::min<uint64_t>(uint64_t(cnt[9]) + cnt[9] / 4 + 1024, 0xFFFFFFF0u / 16));
      continue;
    }
    if (st->hit_overflow) {  // grow and rescan (correctness first)
      hit_cap_ = uint32_t(std::min<uint64_t>(uint64_t(cnt[0]) + cnt[0] / 4 + 1024, 0xFFFFFFF0u / 12));
      continue;
    }
    if (st->cand_overflow) {
      cand_cap_ = uint32_t(std::min<uint64_t>(uint64_t(cnt[1]) + cnt[1] / 4 + 1024, 0xFFFFFFF0u));
      continue;
    }
    cands->resize(cnt[1]);
    if (cnt[1]) {
      const size_t nb = size_t(cnt[1]) * sizeof(Candidate);
      if (!EnsureHost(&h_run_cands_, &cap_h_run_cands_, nb)) return false;
      HIP_OK(hipMemcpyAsync(h_run_cands_, d_cands_, nb, hipMemcpyDeviceToHost, stream_));
      HIP_OK(WaitStream());
      std::memcpy(cands->data(), h_run_cands_, nb);
    }
    // closed keyword gates (finalize_kernel) never reach the host
    cands->erase(std::remove_if(cands->begin(), cands->end(), [](const Candidate& c) { return c.flags & kCandDrop; }),
                 cands->end());
    st->candidates = cands->size();
    if (d_item_diag_) DumpItemDiag();
    hipEventElapsedTime(&st->ms_scan, ev_[1], ev_[2]);
    hipEventElapsedTime(&st->ms_confirm, ev_[2], ev_[3]);
    hipEventElapsedTime(&st->ms_careful, ev_[3], ev_[4]);  // fold kernel
    hipEventElapsedTime(&st->ms_verify, ev_[4], ev_[5]);   // verify (deferred hits) + full-scan
    hipEventElapsedTime(&st->ms_finalize, ev_[5], ev_[6]);
    if (n_fullscan_rules_ > 0) hipEventElapsedTime(&st->ms_fullscan, ev_fs_, ev_[5]);
    st->fullscan_tasks = cnt[13];
    st->fold_sites = cnt[9];
    hipEventElapsedTime(&st->ms_chunkmap, ev_[0], ev_[1]);
    hipEventElapsedTime(&st->ms_total, ev_[0], ev_[6]);
    return true;
  }
  err_ = "candidate buffers kept overflowing";
  return false;
}

// TSG_DIAG_ITEMS: appends "item kind first_id exact_matches passed_on" lines
// (passed_on: anchor hits the in-place NFA did not reject).
void GpuEngine::DumpItemDiag() {
  std::vector<uint32_t> v(2 * std::max<size_t>(n_fitems_, 1));
  if (hipMemcpy(v.data(), d_item_diag_, v.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return;
  FILE* fp = std::fopen(item_diag_path_.c_str(), "a");
  if (!fp) return;
  for (uint32_t i = 0; i < n_fitems_; i++)
    std::fprintf(fp, "%u %u %u %u %u\n", i, uint32_t(h_items_kind_[i]), h_items_id_[i], v[2 * i], v[2 * i + 1]);
  std::fprintf(fp, "--\n");
  std::fclose(fp);
}

}  // namespace tsg
