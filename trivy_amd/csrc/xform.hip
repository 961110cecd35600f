// GPU pre-transform of host batches: the per-file byte
// transforms the secret analyzer applies before Scanner.Scan, run on the
// bytes as read instead of on host threads.
//   kind 0  as is
//   kind 1  every '\r' removed: bytes.ReplaceAll(content, "\r", "")
//           (pkg/fanal/analyzer/secret/secret.go:121)
//   kind 2  utils.ExtractPrintableBytes (pkg/fanal/utils/utils.go:128-160):
//           runs of more than 4 unicode.IsPrint bytes, each followed by '\n'
//           (.pyc binaries, secret.go:112-117)
// Byte-parallel (see the kernels' comment below): every output byte depends
// on at most 5 input bytes before it and 4 after it, so a lane per 16-B block
// computes its block's output with no per-file serial pass; two passes
// (count, write) around an exclusive scan of the per-KiB output counts.  A
// gather packs chosen files of the transformed arena for the host's exact
// pass (shifted 16-B block copies).
#include "xform.h"

#include <hipcub/hipcub.hpp>

#include <cstdlib>

namespace tsg {
namespace {

constexpr int kXThreads = 256;

__device__ __forceinline__ uint4 xload16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

// dst [d, d + n) = src [s, s + n) for one wave (see the file comment).  src
// has 16 readable bytes past s + n; out is 16-B aligned.
__device__ void copy_shifted(const uint8_t* __restrict__ src, uint64_t s, uint8_t* __restrict__ out, uint64_t d,
                             uint64_t n, uint32_t lane) {
  if (n == 0) return;
  const uint64_t e = d + n;
  const uint32_t k = uint32_t((s - d) & 15);  // source byte offset of every aligned destination block (uniform)
  const uint32_t q = k >> 2, r = k & 3;
  for (uint64_t y0 = (d & ~uint64_t(15)) + 16 * uint64_t(lane); y0 < e; y0 += 1024) {
    if (y0 >= d && y0 + 16 <= e) {
      const uint64_t sa = (s + (y0 - d)) & ~uint64_t(15);
      const uint4 A = xload16(src + sa), B = xload16(src + sa + 16);
      const uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
      uint32_t o[4];
      switch (q) {  // wave-uniform
        case 0:
#pragma unroll
          for (int i = 0; i < 4; i++) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], r);
          break;
        case 1:
#pragma unroll
          for (int i = 0; i < 4; i++) o[i] = __builtin_amdgcn_alignbyte(w[i + 2], w[i + 1], r);
          break;
        case 2:
#pragma unroll
          for (int i = 0; i < 4; i++) o[i] = __builtin_amdgcn_alignbyte(w[i + 3], w[i + 2], r);
          break;
        default:
#pragma unroll
          for (int i = 0; i < 4; i++) o[i] = __builtin_amdgcn_alignbyte(w[i + 4], w[i + 3], r);
          break;
      }
      *reinterpret_cast<uint4*>(out + y0) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {  // the file's first / last block: only its own bytes
      const uint64_t lo = y0 > d ? y0 : d, hi = y0 + 16 < e ? y0 + 16 : e;
      for (uint64_t y = lo; y < hi; y++) out[y] = src[s + (y - d)];
    }
  }
}

// unicode.IsPrint(rune(b)) of a byte (Latin-1): graphic or ASCII space; not U+00A0, U+00AD
__device__ __forceinline__ bool xprint(uint32_t b) { return (b >= 0x20 && b <= 0x7E) || (b >= 0xA1 && b != 0xAD); }

__device__ __forceinline__ uint32_t wave_excl(uint32_t v, uint32_t lane) {  // exclusive prefix over lanes
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= uint32_t(d)) x += y;
  }
  return x - v;
}

// ---------------------------------------------------------------------------
// Byte-parallel transform.  Every output byte is a function of a few input
// bytes around it, so the transform is a stream compaction with local rules:
//   kind 0: every byte is kept;
//   kind 1: every byte but '\r' is kept;
//   kind 2: ExtractPrintableBytes keeps a printable byte iff its run of
//     printable bytes is longer than 4, i.e. some 5 consecutive printable
//     bytes of the file cover it; a non-printable byte emits the '\n' that
//     closes the run before it iff the 5 bytes before it are printable; the
//     file's last byte emits the closing '\n' of a run reaching the file end
//     iff the last 5 bytes are printable (utils.go:128-160).
// A lane owns one 16-B block, a wave one 1-KiB tile.  Per file segment of the
// block the rule is evaluated as 16-bit masks (keep, '\n' before, '\n' after);
// pass 1 counts each tile's output bytes and records where each file starts
// inside its tile; an exclusive scan over the tiles and a per-file fix-up give
// the transformed offsets; pass 2 recomputes the masks, packs the wave's
// output in LDS at its global 16-B phase and writes aligned 16-B stores (byte
// stores only at the tile's two ragged ends, which the neighbouring tiles
// share).  Positions are 32-bit below 4 GiB per call, 64-bit above (Pos).
// ---------------------------------------------------------------------------
constexpr uint32_t kXTile = 1024;

// tile t -> the file holding byte t * kXTile: one thread per tile, binary
// search over the offsets (as engine.hip chunk_map_kernel)
__global__ __launch_bounds__(kXThreads) void xf_chunk_map_kernel(const uint64_t* __restrict__ off, uint32_t n_files,
                                                                 uint64_t n_tiles, uint32_t* __restrict__ chunk_file) {
  for (uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < n_tiles;
       t += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t x = t * kXTile;
    uint32_t lo = 0, hi = n_files;  // off[lo] <= x < off[hi]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (off[mid] <= x) lo = mid;
      else hi = mid;
    }
    chunk_file[t] = lo;
  }
}

// Positions are Pos: uint32_t for calls under 4 GiB (the common case: fewer
// registers), uint64_t for a lone file of 4 GiB or more (the reference reads
// files of any size, analyzer/secret/secret.go:110-121).
//
// A lane's 16-B block of tile t (zeros past the end).
template <typename Pos>
__device__ __forceinline__ uint4 x_block(const uint8_t* raw, Pos n_bytes, uint32_t t, uint32_t lane,
                                         uint32_t n_tiles) {
  const Pos blk = Pos(t) * kXTile + 16 * lane;
  // branch-free (a load under a branch makes the compiler's vmcnt waits after it conservative)
  const bool in = t < n_tiles && blk < n_bytes;
  // An opaque mask instead of a select on the loaded value: with the select the
  // compiler moves the load under a branch, and a memory operation under a branch
  // makes its vmcnt waits in the loop drain everything (xf_count_fast_kernel).
  uint32_t m = in ? ~0u : 0u;
  asm volatile("" : "+v"(m));
  const uint4 x = *reinterpret_cast<const uint4*>(raw + (in ? blk : Pos(0)));
  return make_uint4(x.x & m, x.y & m, x.z & m, x.w & m);
}

// The 32 bytes around a lane's block: [blk - 8, blk + 24) as 8 words (the
// neighbours' words by wave shuffles; the wave's edge lanes load theirs).
struct XWindow {
  uint32_t w[8];
  __device__ __forceinline__ uint32_t byte(uint32_t i) const {
    return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
  }
};

template <typename Pos>
__device__ __forceinline__ XWindow x_window(const uint8_t* raw, Pos n_bytes, Pos blk, uint32_t lane,
                                            const uint4& v) {
  XWindow W;
  W.w[2] = v.x;
  W.w[3] = v.y;
  W.w[4] = v.z;
  W.w[5] = v.w;
  W.w[0] = __shfl_up(v.z, 1);
  W.w[1] = __shfl_up(v.w, 1);
  W.w[6] = __shfl_down(v.x, 1);
  W.w[7] = __shfl_down(v.y, 1);
  if (lane == 0) {
    const uint2 p = blk >= 8 ? *reinterpret_cast<const uint2*>(raw + blk - 8) : make_uint2(0, 0);
    W.w[0] = p.x;
    W.w[1] = p.y;
  }
  if (lane == 63) {
    const uint2 p = blk + 16 < n_bytes ? *reinterpret_cast<const uint2*>(raw + blk + 16) : make_uint2(0, 0);
    W.w[6] = p.x;
    W.w[7] = p.y;
  }
  return W;
}

// 4-bit mask of the bytes of w equal to c (exact per byte: no carries between bytes).
__device__ __forceinline__ uint32_t eq_bytes(uint32_t w, uint32_t c4) {
  const uint32_t x = w ^ c4;
  const uint32_t t = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // bit 7 of each zero byte
  return ((t >> 7) * 0x204081u >> 21) & 0xFu;  // gather bits 0, 8, 16, 24 into bits 0..3
}

// Kind-2 masks for the file window bits [lo, hi) of the 32-byte window
// (window bit i = byte blk - 8 + i): K kept printable bytes, C bytes that emit
// the '\n' closing the run before them, Z the file's last byte when it closes
// a run reaching the file end (hi <= 24: the file ends in or before the block).
struct XMasks {
  uint32_t K, C, Z;
};
__device__ XMasks x_masks(const XWindow& W, uint32_t lo, uint32_t hi) {
  const uint32_t in = (hi >= 32 ? ~0u : (1u << hi) - 1u) & ~((1u << lo) - 1u);
  uint32_t P = 0;
#pragma unroll 4
  for (uint32_t i = 0; i < 32; i++) {
    const uint32_t b = W.byte(i);
    P |= uint32_t((b >= 0x20u && b <= 0x7Eu) || (b >= 0xA1u && b != 0xADu)) << i;
  }
  P &= in;
  const uint32_t Q = P & (P >> 1) & (P >> 2) & (P >> 3) & (P >> 4);  // bit k: bytes k .. k+4 printable
  XMasks m;
  m.K = (Q | (Q << 1) | (Q << 2) | (Q << 3) | (Q << 4)) & P;
  m.C = ~P & in & (Q << 5);
  m.Z = (hi <= 32 && hi >= 5 && ((Q >> (hi - 5)) & 1u)) ? (1u << (hi - 1)) : 0u;
  return m;
}

// The file table around a tile: offsets of files tf .. tf + 64 and kinds of
// tf .. tf + 63 staged in the wave's LDS (one coalesced load per tile, a tile
// ahead), so a lane finds the file holding its block and the files after it
// without a chain of dependent global loads; files further on (a tile of more
// than 64 tiny files) are read from global memory.
template <typename Pos>
struct XFiles {
  uint32_t tf;
  const Pos* so;
  const uint8_t* sk;
  const uint64_t* off;
  const uint8_t* kind;
  __device__ __forceinline__ Pos O(uint32_t g) const {
    const uint32_t d = g - tf;
    return d < 65u ? so[d] : Pos(off[g]);
  }
  __device__ __forceinline__ uint32_t K(uint32_t g) const {
    const uint32_t d = g - tf;
    return d < 64u ? uint32_t(sk[d]) : uint32_t(kind[g]);
  }
};

// Per lane: its slice of the file table of tile tf (loaded a tile ahead).
template <typename Pos>
struct XFileRegs {
  Pos o, o64;
  uint32_t k;
};
template <typename Pos>
__device__ __forceinline__ XFileRegs<Pos> x_file_regs(const uint64_t* off, const uint8_t* kind, uint32_t n_files,
                                                      uint32_t tf, uint32_t lane) {
  XFileRegs<Pos> r;
  const uint32_t g = tf + lane < n_files ? tf + lane : n_files;
  r.o = Pos(off[g]);
  r.o64 = Pos(off[tf + 64u < n_files ? tf + 64u : n_files]);
  const uint32_t k = kind[g < n_files ? g : 0u];  // branch-free (n_files >= 1 here)
  r.k = g < n_files ? k : 0u;
  return r;
}
template <typename Pos>
__device__ __forceinline__ void x_stage_files(Pos* so, uint8_t* sk, const XFileRegs<Pos>& r, uint32_t lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the previous tile's reads are done
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  so[lane] = r.o;
  if (lane == 0) so[64] = r.o64;
  sk[lane] = uint8_t(r.k);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// An identity tile, decided from the tile's bytes and its staged file table
// alone (no per-block segment walk): no '\r' in the tile, no kind-2 file
// starting in it or holding its first byte, at most 64 files starting in it,
// and no file starting exactly at its first byte (empty files before that one
// are named by no staged entry).  Its output is its input: the count is its
// length and a file starting in it starts at the same tile offset.
// Conservative: a tile failing the test takes the exact per-block path.
template <typename Pos>
__device__ __forceinline__ Pos x_lane0(Pos x) {  // lane 0's value (all lanes active)
  if constexpr (sizeof(Pos) == 4) {
    return Pos(__builtin_amdgcn_readfirstlane(uint32_t(x)));
  } else {
    return (Pos(__builtin_amdgcn_readfirstlane(uint32_t(uint64_t(x) >> 32))) << 32) |
           Pos(__builtin_amdgcn_readfirstlane(uint32_t(x)));
  }
}

template <typename Pos>
__device__ __forceinline__ bool x_fast_identity(const uint4& v, const XFileRegs<Pos>& fr, uint32_t tf, Pos t0,
                                                Pos tend) {
  const uint32_t cr = eq_bytes(v.x, 0x0D0D0D0Du) | eq_bytes(v.y, 0x0D0D0D0Du) | eq_bytes(v.z, 0x0D0D0D0Du) |
                      eq_bytes(v.w, 0x0D0D0D0Du);
  const bool k2 = fr.o < tend && fr.k == kXformPrintable;  // file tf + lane holds bytes of the tile
  const bool many = fr.o64 < tend;                          // file tf + 64 starts in the tile
  const bool edge = x_lane0(fr.o) == t0 && tf > 0;         // lane 0's file: the one holding byte t0
  return !__any(cr != 0u || k2) && !many && !edge;
}

// A lane's block in file order.  For each file segment [s, e) of the block:
// start(f, count so far) at a file starting inside the block (empty files
// too), then out(emit mask, nl-before mask, nl-after mask) over the block's
// 16 bytes (bit i = byte blk + i): the output is, in byte order, a '\n' for a
// bit of the second mask, the byte for a bit of the first, a '\n' for a bit of
// the third.  Returns the lane's output byte count.
template <typename Pos, typename Start, typename Out>
__device__ __forceinline__ uint32_t x_lane(Pos n_bytes, const XFiles<Pos>& T, uint32_t n_files, Pos blk,
                                           const XWindow& W, Start start, Out out) {
  // T.tf: chunk_file[] of the lane's tile, the file holding its first byte
  if (blk >= n_bytes) return 0;
  const Pos bend = blk + 16 < n_bytes ? blk + 16 : n_bytes;
  uint32_t f = T.tf;
  Pos fs = T.O(f), fe = T.O(f + 1);
  if (fs == blk)  // empty files at a tile's first byte come before the file the chunk map names
    for (uint32_t g = f; g > 0 && Pos(T.off[g - 1]) == blk;) start(--g, 0u);
  while (fe <= blk && f + 1 < n_files) {  // the file holding blk (the chunk map names the tile's first)
    f++;
    fs = fe;
    fe = T.O(f + 1);
    if (fs >= blk) start(f, 0u);  // an empty file at the block start
  }
  // the block's CR bytes (kinds 1)
  const uint32_t cr = eq_bytes(W.w[2], 0x0D0D0D0Du) | (eq_bytes(W.w[3], 0x0D0D0D0Du) << 4) |
                      (eq_bytes(W.w[4], 0x0D0D0D0Du) << 8) | (eq_bytes(W.w[5], 0x0D0D0D0Du) << 12);
  uint32_t cnt = 0;
  for (;;) {
    if (fs >= blk && fs < bend) start(f, cnt);
    const uint32_t s = fs > blk ? uint32_t(fs - blk) : 0u, e = uint32_t((fe < bend ? fe : bend) - blk);  // the segment, block bits
    if (s < e) {
      const uint32_t seg = ((1u << e) - 1u) & ~((1u << s) - 1u);
      const uint32_t k = T.K(f);
      if (k == 0) {
        out(seg, 0u, 0u);
        cnt += uint32_t(__popc(seg));
      } else if (k == 1) {
        out(seg & ~cr, 0u, 0u);
        cnt += uint32_t(__popc(seg & ~cr));
      } else {
        const uint32_t lo = fs + 8 > blk ? uint32_t(fs + 8 - blk) : 0u;  // window bits of the file
        const uint32_t hi = fe - blk + 8 < 32 ? uint32_t(fe - blk + 8) : 32u;
        const XMasks m = x_masks(W, fs + 8 >= blk ? lo : 0u, fe + 8 >= blk ? hi : 0u);
        const uint32_t K = (m.K >> 8) & seg, C = (m.C >> 8) & seg, Z = (m.Z >> 8) & seg;
        out(K, C, Z);
        cnt += uint32_t(__popc(K) + __popc(C) + __popc(Z));
      }
    }
    if (fe >= bend || f + 1 >= n_files) break;
    f++;
    fs = fe;
    fe = T.O(f + 1);
  }
  return cnt;
}

template <typename Pos>
__global__ __launch_bounds__(kXThreads) void xf_count_kernel(const uint8_t* __restrict__ raw, Pos n_bytes,
                                                             const uint64_t* __restrict__ off,
                                                             const uint8_t* __restrict__ kind, uint32_t n_files,
                                                             const uint32_t* __restrict__ chunk_file,
                                                             uint64_t* __restrict__ tile_cnt,
                                                             uint32_t* __restrict__ fstart,
                                                             const uint32_t* __restrict__ tile_fast) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t n_tiles = uint32_t((n_bytes + kXTile - 1) / kXTile);
  const uint32_t waves = gridDim.x * (kXThreads / 64);
  // The tiles xf_count_fast_kernel left (tile_fast[t] == 0: a '\r', a kind-2
  // file, an empty file at the tile start, > 64 file starts, the arena's partial
  // last tile).
  __shared__ Pos s_fo[kXThreads / 64][65];
  __shared__ uint8_t s_fk[kXThreads / 64][64];
  Pos* so = s_fo[threadIdx.x >> 6];
  uint8_t* sk = s_fk[threadIdx.x >> 6];
  // a wave's tiles are t, t + waves, ... (balanced: a CRLF file's run of tiles
  // spreads over the waves); their flags are read 64 at a time
  for (uint32_t base = blockIdx.x * (kXThreads / 64) + (threadIdx.x >> 6); base < n_tiles; base += 64 * waves) {
    const uint32_t tl = base + lane * waves;
    uint64_t left = __ballot(tl < n_tiles && tile_fast[tl] == 0u);
    while (left) {
    const uint32_t t = base + uint32_t(__builtin_ctzll(left)) * waves;
    left &= left - 1;
    const Pos blk = Pos(t) * kXTile + 16 * lane;
    const uint4 v = x_block(raw, n_bytes, t, lane, n_tiles);
    const uint32_t tf = chunk_file[t];
    const XFileRegs<Pos> fr = x_file_regs<Pos>(off, kind, n_files, tf, lane);
    x_stage_files(so, sk, fr, lane);
    const XFiles<Pos> T{tf, so, sk, off, kind};
    const XWindow W = x_window(raw, n_bytes, blk, lane, v);
    // file starts: tile-relative output offsets once the lane's prefix is known
    uint32_t sf[4], sc[4], ns = 0;
    const uint32_t c = x_lane(
        n_bytes, T, n_files, blk, W,
        [&](uint32_t f, uint32_t at) {
          if (ns < 4) {
            sf[ns] = f;
            sc[ns] = at;
          }
          ns++;
        },
        [&](uint32_t, uint32_t, uint32_t) {});
    const uint32_t ex = wave_excl(c, lane);
    if (lane == 63) tile_cnt[t] = ex + c;
    if (ns > 4) {  // many tiny files in one block: walk it again, recording all
      x_lane(n_bytes, T, n_files, blk, W, [&](uint32_t f, uint32_t at) { fstart[f] = ex + at; },
             [&](uint32_t, uint32_t, uint32_t) {});
    } else {
      for (uint32_t i = 0; i < ns; i++) fstart[sf[i]] = ex + sc[i];
    }
    }
  }
}

__global__ __launch_bounds__(kXThreads) void xf_fixup_kernel(const uint64_t* __restrict__ off, uint32_t n_files,
                                                             uint64_t n_bytes, const uint64_t* __restrict__ tile_pre,
                                                             const uint32_t* __restrict__ fstart,
                                                             const uint32_t* __restrict__ tile_fast,
                                                             uint64_t* __restrict__ xoff) {
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  for (uint32_t f = blockIdx.x * blockDim.x + threadIdx.x; f <= n_files; f += gridDim.x * blockDim.x) {
    const uint64_t s = f < n_files ? off[f] : n_bytes;
    const uint64_t t = s / kXTile;
    // an identity tile's output offsets are its input offsets (no fstart entry)
    xoff[f] = s < n_bytes ? tile_pre[t] + (tile_fast[t] ? s - t * kXTile : uint64_t(fstart[f])) : tile_pre[n_tiles];
  }
}

// The identity tiles, counted (a pass the exact count kernel then skips).  Each
// iteration issues the same loads and the same two stores whatever the tile is
// (every lane stores the tile's count and flag; no branch around a memory
// operation), so the compiler's vmcnt waits for the next tile's loads -- issued
// before this tile's stores -- need not drain the stores: on gfx9 a store counts
// in vmcnt like a load, and one branch around a load or store in the loop made
// every tile wait for all of the previous tile's memory traffic.
template <typename Pos>
__global__ __launch_bounds__(kXThreads) void xf_count_fast_kernel(const uint8_t* __restrict__ raw, Pos n_bytes,
                                                                  const uint64_t* __restrict__ off,
                                                                  const uint8_t* __restrict__ kind, uint32_t n_files,
                                                                  const uint32_t* __restrict__ chunk_file,
                                                                  uint64_t* __restrict__ tile_cnt,
                                                                  uint32_t* __restrict__ tile_fast,
                                                                  uint32_t* __restrict__ err) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t n_tiles = uint32_t((n_bytes + kXTile - 1) / kXTile);
  const uint32_t waves = gridDim.x * (kXThreads / 64);
  if (blockIdx.x == 0 && threadIdx.x < 4) {  // (instead of three memsets: each a launch)
    err[threadIdx.x] = 0;
    if (threadIdx.x == 0) tile_cnt[n_tiles] = 0;  // the exclusive scan's last input
    if (threadIdx.x == 1) tile_fast[n_tiles] = 0;
  }
  uint32_t t = __builtin_amdgcn_readfirstlane(blockIdx.x * (kXThreads / 64) + (threadIdx.x >> 6));
  if (t >= n_tiles) return;
  uint4 v = x_block(raw, n_bytes, t, lane, n_tiles);
  uint32_t tf = chunk_file[t];
  uint32_t tfn = chunk_file[t + waves < n_tiles ? t + waves : t];  // chunk map entries two tiles ahead
  XFileRegs<Pos> fr = x_file_regs<Pos>(off, kind, n_files, tf, lane);
  for (; t < n_tiles; t += waves) {
    const uint32_t t1 = t + waves < n_tiles ? t + waves : t, t2 = t + 2 * waves < n_tiles ? t + 2 * waves : t1;
    const XFileRegs<Pos> frn = x_file_regs<Pos>(off, kind, n_files, tfn, lane);
    const uint4 vn = x_block(raw, n_bytes, t1, lane, n_tiles);
    const uint32_t tfnn = chunk_file[t2];
    const Pos t0 = Pos(t) * kXTile;
    const bool fast = t0 + kXTile <= n_bytes && x_fast_identity(v, fr, tf, t0, t0 + Pos(kXTile));
    tile_cnt[t] = fast ? uint64_t(kXTile) : 0u;  // (the exact kernel counts the others)
    tile_fast[t] = fast ? 1u : 0u;
    v = vn;
    tf = tfn;
    tfn = tfnn;
    fr = frn;
  }
}

// The identity tiles, written: out[tile_pre[t] ..) = the tile's KiB (the exact
// write kernel skips them).  The same loads and stores every iteration, as
// xf_count_fast_kernel: a lane's store that must not land (a tile with edits,
// lane 0's shared first block, the ragged bytes no lane owns) goes to the
// wave's slot of `trash`; the capacity check is folded the same way.
constexpr uint32_t kXTrashWaves = 1024;  // trash: kXTrashWaves x (1 KiB + 64 B)
template <typename Pos>
__global__ __launch_bounds__(kXThreads) void xf_write_fast_kernel(const uint8_t* __restrict__ raw, Pos n_bytes,
                                                                  const uint32_t* __restrict__ tile_fast,
                                                                  const uint64_t* __restrict__ tile_pre,
                                                                  uint8_t* __restrict__ out, uint64_t out_cap,
                                                                  uint8_t* __restrict__ trash,
                                                                  uint32_t* __restrict__ err) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t n_tiles = uint32_t((n_bytes + kXTile - 1) / kXTile);
  const uint32_t waves = gridDim.x * (kXThreads / 64);
  uint32_t t = __builtin_amdgcn_readfirstlane(blockIdx.x * (kXThreads / 64) + (threadIdx.x >> 6));
  if (t >= n_tiles) return;
  if (t == 0) {  // the 64 zero bytes after the output the scan reads past its end (no tile writes there)
    const uint64_t total = tile_pre[n_tiles];
    if (total + 64 <= out_cap) out[total + lane] = 0;
  }
  uint8_t* tw = trash + size_t(t % kXTrashWaves) * (kXTile + 64);
  uint4 vn = x_block(raw, n_bytes, t, lane, n_tiles);
  uint64_t pren = tile_pre[t];
  uint32_t fn = tile_fast[t];
  bool over = false;
  for (; t < n_tiles; t += waves) {
    const uint4 v = vn;
    const uint64_t start = pren;
    const bool fast = fn != 0;
    const uint32_t t1 = t + waves < n_tiles ? t + waves : t;
    vn = x_block(raw, n_bytes, t1, lane, n_tiles);
    pren = tile_pre[t1];
    fn = tile_fast[t1];
    const uint32_t phase = uint32_t(start & 15);
    const uint32_t X[9] = {__shfl_up(v.x, 1), __shfl_up(v.y, 1), __shfl_up(v.z, 1), __shfl_up(v.w, 1),
                           v.x, v.y, v.z, v.w, 0u};  // prev ++ own
    const uint32_t sh = 16u - phase;  // output block = X bytes [sh, sh + 16)
    const uint32_t rb = sh & 3u;
    uint32_t o[4];
    switch (sh >> 2) {  // wave-uniform
#define TSG_XO(k)                                                                                \
  case k:                                                                                        \
    for (int i = 0; i < 4; i++) o[i] = __builtin_amdgcn_alignbyte(X[k + i + 1], X[k + i], rb); \
    break;
      TSG_XO(0)
      TSG_XO(1)
      TSG_XO(2)
      TSG_XO(3)
      default:
        for (int i = 0; i < 4; i++) o[i] = X[4 + i];  // phase 0
#undef TSG_XO
    }
    const uint64_t base = start - phase;
    const bool fits = base + kXTile + 16 <= out_cap;
    over = over || (fast && !fits);
    const bool live = fast && fits;
    uint8_t* blk = (live && (lane > 0 || phase == 0)) ? out + base + 16u * lane : tw + 16u * lane;
    *reinterpret_cast<uint4*>(blk) = make_uint4(o[0], o[1], o[2], o[3]);
    // the ragged ends, a byte per lane: lanes 0-15 lane 0's block, bytes [phase, 16);
    // lanes 16-31 the tile's last `phase` bytes, which spill into block 64
    const uint32_t jb = lane & 15u;
    const bool head = lane < 16;
    const uint32_t src = head ? 0u : 63u, b = head ? jb : 16u - phase + jb;
    const uint32_t a0 = __builtin_amdgcn_readlane(o[0], 0), a1 = __builtin_amdgcn_readlane(o[1], 0),
                   a2 = __builtin_amdgcn_readlane(o[2], 0), a3 = __builtin_amdgcn_readlane(o[3], 0);
    const uint32_t c0 = __builtin_amdgcn_readlane(v.x, 63), c1 = __builtin_amdgcn_readlane(v.y, 63),
                   c2 = __builtin_amdgcn_readlane(v.z, 63), c3 = __builtin_amdgcn_readlane(v.w, 63);
    const uint32_t w =
        b < 8 ? (b < 4 ? (src ? c0 : a0) : (src ? c1 : a1)) : (b < 12 ? (src ? c2 : a2) : (src ? c3 : a3));
    const bool own = live && phase != 0 && (head ? jb >= phase : (lane < 32 && jb < phase));
    uint8_t* pb = own ? out + (head ? base + jb : base + kXTile + jb) : tw + kXTile + lane;
    *pb = uint8_t(w >> (8 * (b & 3)));
  }
  if (__any(over) && lane == 0) atomicOr(err, 1u);
}

// An identity tile's output: its input moved to `start`, so each lane writes one
// aligned 16-B block composed from its own and the previous lane's bytes (a
// byte shift by the tile's output phase), no staging; the two ragged 16-B
// blocks, shared with the neighbouring tiles, a byte per lane.
__device__ __forceinline__ void x_store_identity(const uint4& v, uint64_t start, uint32_t lane, uint8_t* out,
                                                 uint64_t out_cap, uint32_t* err) {
  const uint32_t phase = uint32_t(start & 15);
  const uint32_t X[9] = {__shfl_up(v.x, 1), __shfl_up(v.y, 1), __shfl_up(v.z, 1), __shfl_up(v.w, 1),
                         v.x, v.y, v.z, v.w, 0u};  // prev ++ own
  const uint32_t sh = 16u - phase;  // output block = X bytes [sh, sh + 16)
  const uint32_t rb = sh & 3u;
  uint32_t o[4];
  switch (sh >> 2) {  // wave-uniform
#define TSG_XO(k)                                                                                \
  case k:                                                                                        \
    for (int i = 0; i < 4; i++) o[i] = __builtin_amdgcn_alignbyte(X[k + i + 1], X[k + i], rb); \
    break;
    TSG_XO(0)
    TSG_XO(1)
    TSG_XO(2)
    TSG_XO(3)
    default:
      for (int i = 0; i < 4; i++) o[i] = X[4 + i];  // phase 0
#undef TSG_XO
  }
  const uint64_t base = start - phase;
  const uint64_t g = base + 16u * lane;
  if (__any(base + kXTile + 16 > out_cap)) {  // a tile offset past the output: plan and write disagree
    if (lane == 0) atomicOr(err, 1u);
    return;
  }
  if (lane > 0 || phase == 0) *reinterpret_cast<uint4*>(out + g) = make_uint4(o[0], o[1], o[2], o[3]);
  if (phase) {  // the ragged ends, a byte per lane: the previous tile owns out[base, start)
    const uint32_t jb = lane & 15u;
    // lanes 0-15: lane 0's block, bytes [phase, 16); lanes 16-31: the tile's last
    // `phase` bytes, which spill into block 64 (lane 63's bytes [16 - phase, 16))
    const bool head = lane < 16;
    const uint32_t src = head ? 0u : 63u, b = head ? jb : 16u - phase + jb;
    const uint32_t a0 = __builtin_amdgcn_readlane(o[0], 0), a1 = __builtin_amdgcn_readlane(o[1], 0),
                   a2 = __builtin_amdgcn_readlane(o[2], 0), a3 = __builtin_amdgcn_readlane(o[3], 0);
    const uint32_t c0 = __builtin_amdgcn_readlane(v.x, 63), c1 = __builtin_amdgcn_readlane(v.y, 63),
                   c2 = __builtin_amdgcn_readlane(v.z, 63), c3 = __builtin_amdgcn_readlane(v.w, 63);
    const uint32_t w =
        b < 8 ? (b < 4 ? (src ? c0 : a0) : (src ? c1 : a1)) : (b < 12 ? (src ? c2 : a2) : (src ? c3 : a3));
    if (head ? jb >= phase : (lane < 32 && jb < phase))
      out[head ? base + jb : base + kXTile + jb] = uint8_t(w >> (8 * (b & 3)));
  }
}

// A tile with edits: the lanes' output packed in the wave's LDS stage S at its
// global 16-B phase (emit(put) replays the lanes' masks into put), then
// aligned 16-B stores, byte stores at the two ragged ends.
template <typename Emit>
__device__ __forceinline__ void x_store_staged(uint8_t* S, uint64_t start, uint32_t ex, uint32_t total,
                                               uint32_t lane, uint8_t* out, uint64_t out_cap, uint32_t* err,
                                               Emit emit, const XWindow& W) {
  const uint32_t phase = uint32_t(start & 15);  // the stage holds out[start - phase ..) at offset 0
  uint32_t at = phase + ex;
  emit([&](uint32_t K, uint32_t C, uint32_t Z) {
    for (uint32_t m = K | C | Z; m; m &= m - 1) {
      const uint32_t i = uint32_t(__ffs(m)) - 1u;
      if ((C >> i) & 1u) S[at++] = '\n';
      if ((K >> i) & 1u) S[at++] = uint8_t(W.byte(8 + i));
      if ((Z >> i) & 1u) S[at++] = '\n';
    }
  });
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint64_t base = start - phase, end = start + total;
  if (end > out_cap) {  // wave-uniform: never write past the output (the error fails the call)
    if (lane == 0) atomicOr(err, 2u);
  } else {
    for (uint32_t q = 16 * lane; base + q < end; q += 1024) {
      const uint64_t g = base + q;
      if (g >= start && g + 16 <= end) {
        *reinterpret_cast<uint4*>(out + g) = *reinterpret_cast<const uint4*>(S + q);
      } else {  // the ragged ends: only this tile's bytes
        for (uint32_t j = 0; j < 16; j++)
          if (g + j >= start && g + j < end) out[g + j] = S[q + j];
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename Pos>
__global__ __launch_bounds__(kXThreads) void xf_write_kernel(const uint8_t* __restrict__ raw, Pos n_bytes,
                                                             const uint64_t* __restrict__ off,
                                                             const uint8_t* __restrict__ kind, uint32_t n_files,
                                                             const uint32_t* __restrict__ chunk_file,
                                                             const uint64_t* __restrict__ tile_pre,
                                                             uint8_t* __restrict__ out, uint64_t out_cap,
                                                             uint32_t* __restrict__ err,
                                                             const uint32_t* __restrict__ tile_fast) {
  // the tiles xf_write_fast_kernel left; a tile emits at most 1024 + 1024 / 5 + 16
  // bytes (a '\n' per closed run of >= 5 bytes)
  constexpr uint32_t kStage = 1280 + 32;
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kXThreads / 64][kStage];
  const uint32_t lane = threadIdx.x & 63u;
  uint8_t* S = s_out[threadIdx.x >> 6];
  const uint32_t n_tiles = uint32_t((n_bytes + kXTile - 1) / kXTile);
  const uint32_t waves = gridDim.x * (kXThreads / 64);
  __shared__ Pos s_fo[kXThreads / 64][65];
  __shared__ uint8_t s_fk[kXThreads / 64][64];
  Pos* so = s_fo[threadIdx.x >> 6];
  uint8_t* sk = s_fk[threadIdx.x >> 6];
  // a wave's tiles are t, t + waves, ... (balanced: a CRLF file's run of tiles
  // spreads over the waves); their flags are read 64 at a time
  for (uint32_t base = blockIdx.x * (kXThreads / 64) + (threadIdx.x >> 6); base < n_tiles; base += 64 * waves) {
    const uint32_t tl = base + lane * waves;
    uint64_t left = __ballot(tl < n_tiles && tile_fast[tl] == 0u);
    while (left) {
    const uint32_t t = base + uint32_t(__builtin_ctzll(left)) * waves;
    left &= left - 1;
    const Pos blk = Pos(t) * kXTile + 16 * lane;
    const uint4 v = x_block(raw, n_bytes, t, lane, n_tiles);
    const uint32_t tf = chunk_file[t];
    const uint64_t start = tile_pre[t];
    const XFileRegs<Pos> fr = x_file_regs<Pos>(off, kind, n_files, tf, lane);
    // the lane's masks per segment, kept for the write below (at most a few segments per block)
    uint32_t segK[4], segC[4], segZ[4], nseg = 0, kept = 0, added = 0;
    const XFiles<Pos> T{tf, so, sk, off, kind};
    x_stage_files(so, sk, fr, lane);
    const XWindow W = x_window(raw, n_bytes, blk, lane, v);
    const uint32_t c = x_lane(n_bytes, T, n_files, blk, W, [&](uint32_t, uint32_t) {},
                              [&](uint32_t K, uint32_t C, uint32_t Z) {
                                if (nseg < 4) {
                                  segK[nseg] = K;
                                  segC[nseg] = C;
                                  segZ[nseg] = Z;
                                }
                                nseg++;
                                kept |= K;
                                added |= C | Z;
                              });
    if (__all(kept == 0xFFFFu && added == 0u && blk + 16 <= n_bytes)) {
      // an identity tile the fast test left (e.g. an empty file at its start)
      x_store_identity(v, start, lane, out, out_cap, err);
      continue;
    }
    const uint32_t ex = wave_excl(c, lane);
    x_store_staged(S, start, ex, __shfl(ex + c, 63), lane, out, out_cap, err, [&](auto put) {
      if (nseg <= 4) {
        for (uint32_t i = 0; i < nseg; i++) put(segK[i], segC[i], segZ[i]);
      } else {
        x_lane(n_bytes, T, n_files, blk, W, [&](uint32_t, uint32_t) {}, put);
      }
    }, W);
    }
  }
}

// One pass (TSG_XFORM_ONEPASS=1; the default is count, scan, fix-up, write): waves
// take tiles in ticket order, compute a tile's output length, publish it
// (status[t] = kXAgg | length), find the tile's output offset by a decoupled
// look-back over the predecessors' published lengths and prefixes (a wave
// reads 64 predecessors at a time; tile 0 and every tile done publish
// kXIncl | inclusive prefix), publish their inclusive prefix and write the
// tile and the transformed offsets of the files starting in it.  Tiles are
// claimed in order by resident waves, and a wave publishes its length before
// it waits, so every wait is for a tile that is being processed; a wait that
// still exceeds kXSpinMax rounds gives up and flags the error word (the call
// fails instead of hanging the GPU).
constexpr uint64_t kXAgg = uint64_t(1) << 62, kXIncl = uint64_t(1) << 63, kXVal = kXAgg - 1;
constexpr uint32_t kXSpinMax = 1u << 22;
#ifndef TSG_XFORM_SLEEP
#define TSG_XFORM_SLEEP 8
#endif

template <typename Pos>
__global__ __launch_bounds__(kXThreads) void xf_onepass_kernel(const uint8_t* __restrict__ raw, Pos n_bytes,
                                                               const uint64_t* __restrict__ off,
                                                               const uint8_t* __restrict__ kind, uint32_t n_files,
                                                               const uint32_t* __restrict__ chunk_file,
                                                               uint64_t* status, uint32_t* ticket,
                                                               uint64_t* __restrict__ xoff, uint8_t* __restrict__ out,
                                                               uint64_t out_cap, uint32_t* __restrict__ err) {
  constexpr uint32_t kStage = 1280 + 32;  // as xf_write_kernel
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kXThreads / 64][kStage];
  const uint32_t lane = threadIdx.x & 63u;
  uint8_t* S = s_out[threadIdx.x >> 6];
  const uint32_t n_tiles = uint32_t((n_bytes + kXTile - 1) / kXTile);
  __shared__ Pos s_fo[kXThreads / 64][65];
  __shared__ uint8_t s_fk[kXThreads / 64][64];
  Pos* so = s_fo[threadIdx.x >> 6];
  uint8_t* sk = s_fk[threadIdx.x >> 6];
  for (;;) {
    uint32_t tk = 0;
    if (lane == 0) tk = atomicAdd(ticket, 1u);
    const uint32_t t = __builtin_amdgcn_readfirstlane(tk);
    if (t >= n_tiles) break;
    const Pos t0 = Pos(t) * kXTile, tend = t0 + kXTile < n_bytes ? t0 + kXTile : n_bytes;
    const Pos blk = t0 + 16 * lane;
    const uint4 v = x_block(raw, n_bytes, t, lane, n_tiles);
    const uint32_t tf = chunk_file[t];
    const XFileRegs<Pos> fr = x_file_regs<Pos>(off, kind, n_files, tf, lane);
    const bool fast = x_fast_identity(v, fr, tf, t0, tend);
    // the tile's length and, on the exact path, the lanes' masks and file starts
    uint32_t segK[4], segC[4], segZ[4], nseg = 0, kept = 0xFFFFu, added = 0, c = 0, ex = 0;
    uint32_t sf[4], sc[4], ns = 0;
    XWindow W;
    const XFiles<Pos> T{tf, so, sk, off, kind};
    uint64_t len;
    if (fast) {
      len = uint64_t(tend - t0);
    } else {
      x_stage_files(so, sk, fr, lane);
      W = x_window(raw, n_bytes, blk, lane, v);
      kept = 0;
      c = x_lane(
          n_bytes, T, n_files, blk, W,
          [&](uint32_t f, uint32_t at) {
            if (ns < 4) {
              sf[ns] = f;
              sc[ns] = at;
            }
            ns++;
          },
          [&](uint32_t K, uint32_t C, uint32_t Z) {
            if (nseg < 4) {
              segK[nseg] = K;
              segC[nseg] = C;
              segZ[nseg] = Z;
            }
            nseg++;
            kept |= K;
            added |= C | Z;
          });
      ex = wave_excl(c, lane);
      len = __shfl(ex + c, 63);
    }
    // publish the length, then look back for the tile's output offset
    uint64_t excl = 0;
    if (t == 0) {
      if (lane == 0) __hip_atomic_store(&status[0], kXIncl | len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&status[t], kXAgg | len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t hi = t;  // predecessors [0, hi) not yet summed
      for (uint32_t spin = 0;;) {
        const int64_t p = int64_t(hi) - 1 - int64_t(lane);  // lane l reads tile hi - 1 - l
        const uint64_t st =
            p >= 0 ? __hip_atomic_load(&status[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kXIncl;
        const uint64_t incl = __ballot((st & kXIncl) != 0);
        const uint64_t ready = __ballot((st & (kXIncl | kXAgg)) != 0);
        // the nearest inclusive prefix (always within reach: tile 0 publishes one)
        const uint32_t k = incl ? uint32_t(__ffsll(static_cast<unsigned long long>(incl)) - 1) : 64u;
        const uint64_t need = k >= 63 ? ~uint64_t(0) : ((uint64_t(1) << (k + 1)) - 1);  // lanes 0..k
        if ((ready & need) == need) {
          uint64_t x = (lane <= k && p >= 0) ? (st & kXVal) : 0;
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
          excl += x;
          if (k < 64) break;
          hi -= 64;
          continue;
        }
        if (++spin > kXSpinMax) {  // never expected: fail the call rather than spin forever
          if (lane == 0) atomicOr(err, 4u);
          break;
        }
        __builtin_amdgcn_s_sleep(TSG_XFORM_SLEEP);  // (the waiting waves share the memory path with the working ones)
      }
      if (lane == 0)
        __hip_atomic_store(&status[t], kXIncl | (excl + len), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the transformed offsets of the files starting in the tile (xf_fixup_kernel's job)
    if (fast) {
      if (fr.o >= t0 && fr.o < tend) xoff[tf + lane] = excl + uint64_t(fr.o - t0);
    } else if (ns > 4) {  // many tiny files in one block: walk it again, recording all
      x_lane(n_bytes, T, n_files, blk, W, [&](uint32_t f, uint32_t at) { xoff[f] = excl + ex + at; },
             [&](uint32_t, uint32_t, uint32_t) {});
    } else {
      for (uint32_t i = 0; i < ns; i++) xoff[sf[i]] = excl + ex + sc[i];
    }
    if (t + 1 == n_tiles && lane == 0) {  // the end: files starting at n_bytes (empty) and the total
      for (uint32_t f = n_files; f > 0 && Pos(off[f - 1]) == n_bytes; f--) xoff[f - 1] = excl + len;
      xoff[n_files] = excl + len;
    }
    const bool whole = t0 + kXTile <= n_bytes;
    if (whole && (fast || __all(kept == 0xFFFFu && added == 0u))) {
      x_store_identity(v, excl, lane, out, out_cap, err);
      continue;
    }
    if (fast) {  // the arena's partial last tile, identity: its masks for the staged write
      x_stage_files(so, sk, fr, lane);
      W = x_window(raw, n_bytes, blk, lane, v);
      c = x_lane(n_bytes, T, n_files, blk, W, [&](uint32_t, uint32_t) {},
                 [&](uint32_t K, uint32_t C, uint32_t Z) {
                   if (nseg < 4) {
                     segK[nseg] = K;
                     segC[nseg] = C;
                     segZ[nseg] = Z;
                   }
                   nseg++;
                 });
      ex = wave_excl(c, lane);
    }
    x_store_staged(S, excl, ex, uint32_t(len), lane, out, out_cap, err, [&](auto put) {
      if (nseg <= 4) {
        for (uint32_t i = 0; i < nseg; i++) put(segK[i], segC[i], segZ[i]);
      } else {
        x_lane(n_bytes, T, n_files, blk, W, [&](uint32_t, uint32_t) {}, put);
      }
    }, W);
  }
}

__global__ __launch_bounds__(kXThreads) void gather_kernel(const uint8_t* __restrict__ src,
                                                           const uint64_t* __restrict__ xoff,
                                                           const uint32_t* __restrict__ files,
                                                           const uint64_t* __restrict__ dst_off, uint32_t n,
                                                           uint8_t* __restrict__ dst) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (kXThreads / 64);
  for (uint32_t i = blockIdx.x * (kXThreads / 64) + (threadIdx.x >> 6); i < n; i += waves) {
    const uint32_t f = files[i];
    const uint64_t a = xoff[f], len = xoff[f + 1] - a;
    copy_shifted(src, a, dst, dst_off[i], len, lane);
  }
}

uint32_t grid_for(uint32_t n_waves) {
  const uint32_t g = (n_waves + kXThreads / 64 - 1) / (kXThreads / 64);
  return g < 1 ? 1 : (g > 4096 ? 4096 : g);
}

}  // namespace

// Scratch of the flat transform: chunk map | tile counts | tile prefix | file starts | scan temp.
struct XformScratch {
  size_t chunk_file, tile_cnt, tile_pre, fstart, err, scan, scan_bytes, status, tile_fast, trash, total;
};

// 64-bit positions for calls of 4 GiB or more; TSG_XFORM_WIDE=1 forces them
// (tests run the wide kernels on small batches).
static bool XformWide(uint64_t n_bytes) {
  const char* e = std::getenv("TSG_XFORM_WIDE");  // read per call: tests switch it within one process
  return (e && std::atoi(e) != 0) || n_bytes >= (uint64_t(1) << 32) - 64;
}

// Workgroups of the count / write kernels (TSG_XFORM_GRID; tuning): each wave
// walks tiles grid-strided with the next tile's loads in flight.
static uint32_t XformGrid() {
  static const uint32_t g = [] {
    const char* e = std::getenv("TSG_XFORM_GRID");
    const long v = e ? std::atol(e) : 0;
    return v > 0 ? uint32_t(v) : 8192u;
  }();
  return g;
}

static XformScratch ScratchLayout(uint64_t n_bytes, uint32_t n_files) {
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  XformScratch L;
  size_t scan = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan, static_cast<const uint64_t*>(nullptr),
                                         static_cast<uint64_t*>(nullptr), int(n_tiles) + 1);
  auto up = [](size_t x) { return (x + 255) & ~size_t(255); };
  L.chunk_file = 0;
  L.tile_cnt = up(L.chunk_file + (n_tiles + 1) * 4);
  L.tile_pre = up(L.tile_cnt + (n_tiles + 1) * 8);
  L.fstart = up(L.tile_pre + (n_tiles + 1) * 8);
  L.err = up(L.fstart + (size_t(n_files) + 1) * 4);
  L.scan = up(L.err + 16);  // (the one-pass ticket lives in the error block: err[1])
  L.scan_bytes = scan;
  L.status = up(L.scan + scan + 16);
  L.tile_fast = up(L.status + (n_tiles + 1) * 8);
  L.trash = up(L.tile_fast + (n_tiles + 1) * 4);  // (u32: scalar loads by the write kernel)
  L.total = up(L.trash + size_t(kXTrashWaves) * (kXTile + 64));
  return L;
}

size_t XformScratchBytes(uint64_t n_bytes, uint32_t n_files) { return ScratchLayout(n_bytes, n_files).total; }

hipError_t XformPlan(const uint8_t* raw, uint64_t n_bytes, const uint64_t* off, const uint8_t* kind, uint32_t n_files,
                     void* scratch, uint64_t* xoff, hipStream_t s) {
  const bool wide = XformWide(n_bytes);
  const XformScratch L = ScratchLayout(n_bytes, n_files);
  uint8_t* sc = static_cast<uint8_t*>(scratch);
  uint32_t* chunk_file = reinterpret_cast<uint32_t*>(sc + L.chunk_file);
  // 64-bit counts: the scan's accumulator is the input type, and the sum of a
  // batch of 4 GiB or more does not fit 32 bits
  uint64_t* tile_cnt = reinterpret_cast<uint64_t*>(sc + L.tile_cnt);
  uint64_t* tile_pre = reinterpret_cast<uint64_t*>(sc + L.tile_pre);
  uint32_t* fstart = reinterpret_cast<uint32_t*>(sc + L.fstart);
  uint32_t* tile_fast = reinterpret_cast<uint32_t*>(sc + L.tile_fast);
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  hipError_t e;
  if (n_tiles == 0 && ((e = hipMemsetAsync(tile_cnt, 0, 8, s)) != hipSuccess ||
                       (e = hipMemsetAsync(sc + L.err, 0, 16, s)) != hipSuccess))  // (else xf_count_fast_kernel)
    return e;
  if (n_files && n_tiles) {
    const uint32_t gm = uint32_t(std::min<uint64_t>((n_tiles + kXThreads - 1) / kXThreads, 8192));
    xf_chunk_map_kernel<<<gm, kXThreads, 0, s>>>(off, n_files, n_tiles, chunk_file);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (n_tiles) {
    const uint32_t g = uint32_t(std::min<uint64_t>((n_tiles + kXThreads / 64 - 1) / (kXThreads / 64), XformGrid()));
    // identity tiles first (counted, flagged), then the exact count of the rest
    if (wide) {
      xf_count_fast_kernel<uint64_t><<<g, kXThreads, 0, s>>>(raw, n_bytes, off, kind, n_files, chunk_file, tile_cnt,
                                                             tile_fast, reinterpret_cast<uint32_t*>(sc + L.err));
      xf_count_kernel<uint64_t><<<g, kXThreads, 0, s>>>(raw, n_bytes, off, kind, n_files, chunk_file, tile_cnt, fstart,
                                                         tile_fast);
    } else {
      xf_count_fast_kernel<uint32_t><<<g, kXThreads, 0, s>>>(raw, uint32_t(n_bytes), off, kind, n_files, chunk_file,
                                                             tile_cnt, tile_fast,
                                                             reinterpret_cast<uint32_t*>(sc + L.err));
      xf_count_kernel<uint32_t><<<g, kXThreads, 0, s>>>(raw, uint32_t(n_bytes), off, kind, n_files, chunk_file,
                                                         tile_cnt, fstart, tile_fast);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  size_t sb = L.scan_bytes;
  if ((e = hipcub::DeviceScan::ExclusiveSum(sc + L.scan, sb, tile_cnt, tile_pre, int(n_tiles) + 1, s)) != hipSuccess)
    return e;
  xf_fixup_kernel<<<grid_for((n_files + 64) / 64), kXThreads, 0, s>>>(off, n_files, n_bytes, tile_pre, fstart,
                                                                      tile_fast, xoff);
  return hipGetLastError();
}

hipError_t XformWrite(const uint8_t* raw, uint64_t n_bytes, const uint64_t* off, const uint8_t* kind, uint32_t n_files,
                      const void* scratch, uint8_t* out, uint64_t out_cap, hipStream_t s) {
  const XformScratch L = ScratchLayout(n_bytes, n_files);
  const uint8_t* sc = static_cast<const uint8_t*>(scratch);
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  if (!n_tiles) return out_cap >= 64 ? hipMemsetAsync(out, 0, 64, s) : hipSuccess;  // (else xf_write_fast_kernel)
  const uint32_t g = uint32_t(std::min<uint64_t>((n_tiles + kXThreads / 64 - 1) / (kXThreads / 64), XformGrid()));
  const uint32_t* cf = reinterpret_cast<const uint32_t*>(sc + L.chunk_file);
  const uint64_t* tp = reinterpret_cast<const uint64_t*>(sc + L.tile_pre);
  uint32_t* err = reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(sc) + L.err);
  const uint32_t* tfast = reinterpret_cast<const uint32_t*>(sc + L.tile_fast);
  uint8_t* trash = const_cast<uint8_t*>(sc) + L.trash;
  if (XformWide(n_bytes)) {
    xf_write_fast_kernel<uint64_t><<<g, kXThreads, 0, s>>>(raw, n_bytes, tfast, tp, out, out_cap, trash, err);
    xf_write_kernel<uint64_t><<<g, kXThreads, 0, s>>>(raw, n_bytes, off, kind, n_files, cf, tp, out, out_cap, err,
                                                       tfast);
  } else {
    xf_write_fast_kernel<uint32_t><<<g, kXThreads, 0, s>>>(raw, uint32_t(n_bytes), tfast, tp, out, out_cap, trash,
                                                           err);
    xf_write_kernel<uint32_t><<<g, kXThreads, 0, s>>>(raw, uint32_t(n_bytes), off, kind, n_files, cf, tp, out,
                                                       out_cap, err, tfast);
  }
  return hipGetLastError();
}

// One pass (xf_onepass_kernel): xoff and out together, TSG_XFORM_ONEPASS=1 only
// (read per call: tests run both paths in one process).  Measured 3.3 ms per
// 256-MB C4 batch against 0.3 ms for the two passes, whatever the spin's sleep:
// a ticket per 1-KiB tile is 256 Ki atomics on one address, which serialise at
// ~12 ns each -- the ticket, not the look-back, sets the time.
bool XformOnePassOn() {
  const char* e = std::getenv("TSG_XFORM_ONEPASS");
  return e && std::atoi(e) != 0;
}

hipError_t XformOnePass(const uint8_t* raw, uint64_t n_bytes, const uint64_t* off, const uint8_t* kind,
                        uint32_t n_files, void* scratch, uint64_t* xoff, uint8_t* out, uint64_t out_cap,
                        hipStream_t s) {
  const XformScratch L = ScratchLayout(n_bytes, n_files);
  uint8_t* sc = static_cast<uint8_t*>(scratch);
  uint32_t* chunk_file = reinterpret_cast<uint32_t*>(sc + L.chunk_file);
  uint32_t* err = reinterpret_cast<uint32_t*>(sc + L.err);
  uint64_t* status = reinterpret_cast<uint64_t*>(sc + L.status);
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  hipError_t e;
  if ((e = hipMemsetAsync(sc + L.err, 0, 16, s)) != hipSuccess) return e;  // error word, ticket
  if (n_tiles == 0 || n_files == 0) return hipMemsetAsync(xoff, 0, (size_t(n_files) + 1) * 8, s);
  if ((e = hipMemsetAsync(status, 0, n_tiles * 8, s)) != hipSuccess) return e;
  const uint32_t gm = uint32_t(std::min<uint64_t>((n_tiles + kXThreads - 1) / kXThreads, 8192));
  xf_chunk_map_kernel<<<gm, kXThreads, 0, s>>>(off, n_files, n_tiles, chunk_file);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const uint32_t g = uint32_t(std::min<uint64_t>((n_tiles + kXThreads / 64 - 1) / (kXThreads / 64), XformGrid()));
  if (XformWide(n_bytes))
    xf_onepass_kernel<uint64_t><<<g, kXThreads, 0, s>>>(raw, n_bytes, off, kind, n_files, chunk_file, status,
                                                        err + 1, xoff, out, out_cap, err);
  else
    xf_onepass_kernel<uint32_t><<<g, kXThreads, 0, s>>>(raw, uint32_t(n_bytes), off, kind, n_files, chunk_file,
                                                        status, err + 1, xoff, out, out_cap, err);
  return hipGetLastError();
}

uint32_t XformErrorWord(uint64_t n_bytes, uint32_t n_files, const void* scratch, hipStream_t s) {
  const XformScratch L = ScratchLayout(n_bytes, n_files);
  uint32_t w = 0;
  if (hipMemcpyAsync(&w, static_cast<const uint8_t*>(scratch) + L.err, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return ~0u;
  return w;
}

const uint32_t* XformErrorPtr(uint64_t n_bytes, uint32_t n_files, const void* scratch) {
  return reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(scratch) + ScratchLayout(n_bytes, n_files).err);
}

hipError_t GatherFiles(const uint8_t* src, const uint64_t* xoff, const uint32_t* files, const uint64_t* dst_off,
                       uint32_t n, uint8_t* dst, hipStream_t s) {
  if (n == 0) return hipSuccess;
  gather_kernel<<<grid_for(n), kXThreads, 0, s>>>(src, xoff, files, dst_off, n, dst);
  return hipGetLastError();
}

}  // namespace tsg

namespace tsg {
namespace {

__device__ __forceinline__ uint32_t word_at(const uint4& a, const uint4& b, uint32_t k) {  // word k of a:b
  switch (k) {
    case 0: return a.x;
    case 1: return a.y;
    case 2: return a.z;
    case 3: return a.w;
    case 4: return b.x;
    case 5: return b.y;
    case 6: return b.z;
    default: return b.w;
  }
}

__global__ __launch_bounds__(256) void gather_host_kernel(const uint8_t* __restrict__ src,
                                                          const uint64_t* __restrict__ src_off,
                                                          const uint64_t* __restrict__ dst_off,
                                                          const GatherItem* __restrict__ items, uint32_t n_items,
                                                          uint8_t* __restrict__ dst) {
  // The source is host memory read over PCIe (~2-3 us a load): each lane issues
  // kU + 1 16-B loads before it waits, so a wave keeps ~4 KiB in flight and the
  // small grid (GatherHostFiles) ~2 MiB -- past the link's bandwidth-delay
  // product -- while it holds only a few wave slots of the CUs the scan kernels
  // of the other batches run on.
  constexpr uint32_t kU = 4;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint32_t it = blockIdx.x * 4u + wave; it < n_items; it += gridDim.x * 4u) {
    const GatherItem g = items[it];
    const uint64_t f0 = dst_off[g.file], f1 = dst_off[g.file + 1];
    const uint64_t d0 = f0 + uint64_t(g.piece) * kGatherPiece;
    const uint64_t d1 = min(f1, d0 + kGatherPiece);
    if (d0 >= d1) continue;
    const uint64_t s0 = src_off[g.file] + (d0 - f0);  // source of byte d0
    // destination blocks [align16(d0), d1): block B takes source bytes from
    // B + (s0 - d0); its aligned source block A and A + 16 (the next lane's A)
    const uint64_t b_lo = d0 & ~uint64_t(15);
    const uint64_t a_lo = (b_lo + s0 - d0) & ~uint64_t(15);  // (b_lo + s0 - d0 >= s0 - 15 >= 0 in a tar)
    const uint32_t r = uint32_t((b_lo + s0 - d0) & 15u);     // byte shift, the same for every block
    for (uint64_t k = 0; b_lo + 16 * k < d1; k += 64 * kU) {
      // the blocks of kU groups of 64, and one past the last live one (its
      // source is the last live block's next); lane 63 of the last group also
      // loads the block after the iteration's last
      uint4 a[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; u++) {
        const uint64_t j = k + 64 * u + lane;
        a[u] = make_uint4(0, 0, 0, 0);
        if (b_lo + 16 * j < d1 + 16) a[u] = *reinterpret_cast<const uint4*>(src + a_lo + 16 * j);
      }
      uint4 ex = make_uint4(0, 0, 0, 0);
      const uint64_t j_ex = k + 64 * kU;  // (lane 63 of the last group: block j_ex - 1)
      if (r && lane == 63 && b_lo + 16 * (j_ex - 1) < d1) ex = *reinterpret_cast<const uint4*>(src + a_lo + 16 * j_ex);
#pragma unroll
      for (uint32_t u = 0; u < kU; u++) {
        const uint64_t B = b_lo + 16 * (k + 64 * u + lane);
        uint4 nxt;
        nxt.x = __shfl_down(a[u].x, 1);
        nxt.y = __shfl_down(a[u].y, 1);
        nxt.z = __shfl_down(a[u].z, 1);
        nxt.w = __shfl_down(a[u].w, 1);
        if (u + 1 < kU) {  // lane 63: lane 0's block of the next group
          const uint4 n0 = make_uint4(__builtin_amdgcn_readlane(a[u + 1 < kU ? u + 1 : u].x, 0),
                                      __builtin_amdgcn_readlane(a[u + 1 < kU ? u + 1 : u].y, 0),
                                      __builtin_amdgcn_readlane(a[u + 1 < kU ? u + 1 : u].z, 0),
                                      __builtin_amdgcn_readlane(a[u + 1 < kU ? u + 1 : u].w, 0));
          if (lane == 63) nxt = n0;
        } else if (lane == 63) {
          nxt = ex;
        }
        if (B >= d1) continue;
        uint32_t o[4];
        const uint32_t q = r >> 2, sh = r & 3u;
#pragma unroll
        for (uint32_t w = 0; w < 4; w++) {
          const uint32_t lo = word_at(a[u], nxt, q + w), hi = word_at(a[u], nxt, q + w + 1 > 7 ? 7 : q + w + 1);
          o[w] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
        }
        if (B >= d0 && B + 16 <= d1) {
          *reinterpret_cast<uint4*>(dst + B) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {  // a ragged end: only the item's bytes (the neighbours belong to other files / items)
          for (uint32_t jb = 0; jb < 16; jb++) {
            const uint64_t x = B + jb;
            if (x >= d0 && x < d1) dst[x] = uint8_t(o[jb >> 2] >> (8 * (jb & 3)));
          }
        }
      }
    }
  }
}

}  // namespace

hipError_t GatherHostFiles(const uint8_t* src_dev, const uint64_t* src_off, const uint64_t* dst_off,
                           const GatherItem* items, uint32_t n_items, uint8_t* dst, hipStream_t s) {
  if (!n_items) return hipSuccess;
  // 32 workgroups (128 waves, ~640 KiB of loads in flight): enough for the link
  // (gather_host_kernel), few wave slots taken from the scan kernels of the
  // batches in flight.  C4 by grid: 16 -> 33, 24-48 -> 42-43, 64 -> 40, 128 ->
  // 37-38, 512 -> 35 GB/s (profiles/r06/c4/c4ab_r06gg*)
  static const uint64_t max_grid = [] {  // TSG_GATHER_GRID: tuning knob
    const char* e = std::getenv("TSG_GATHER_GRID");
    return e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : uint64_t(32);
  }();
  const uint32_t grid = uint32_t(std::min<uint64_t>((uint64_t(n_items) + 3) / 4, max_grid));
  gather_host_kernel<<<grid, 256, 0, s>>>(src_dev, src_off, dst_off, items, n_items, dst);
  return hipGetLastError();
}

}  // namespace tsg
