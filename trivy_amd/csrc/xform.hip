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
// A lane owns one 16-B block, a wave one 1-KiB tile.  Pass 1 counts each
// tile's output bytes and records where each file starts inside its tile;
// an exclusive scan over the tiles and a per-file fix-up give the
// transformed offsets; pass 2 recomputes the bytes, packs the wave's output
// in LDS at its global 16-B phase and writes aligned 16-B stores (byte stores
// only at the tile's two ragged ends, which the neighbouring tiles share).
// ---------------------------------------------------------------------------
constexpr uint32_t kXTile = 1024;

__global__ __launch_bounds__(kXThreads) void xf_chunk_map_kernel(const uint64_t* __restrict__ off, uint32_t n_files,
                                                                 uint32_t* __restrict__ chunk_file) {
  for (uint32_t f = blockIdx.x * blockDim.x + threadIdx.x; f < n_files; f += gridDim.x * blockDim.x) {
    const uint64_t s = off[f], e = off[f + 1];
    for (uint64_t c = (s + kXTile - 1) / kXTile; c * kXTile < e; c++) chunk_file[c] = f;
  }
}

// The 32 bytes around a lane's block: [blk - 8, blk + 24) as 8 words (the
// neighbours' words by wave shuffles; the wave's edge lanes load theirs).
struct XWindow {
  uint32_t w[8];
  __device__ __forceinline__ uint32_t byte(int i) const { return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu; }
};

__device__ __forceinline__ XWindow x_window(const uint8_t* raw, uint64_t n_bytes, uint64_t blk, uint32_t lane,
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

// Kind-2 masks over the window for the file [fs, fe): bit i of K = window
// byte i is a kept printable byte, bit i of C = window byte i closes a kept
// run (non-printable, the 5 bytes before it printable), bit i of Z = the file's
// last byte is window byte i and closes a run reaching the file end.
struct XMasks {
  uint32_t K, C, Z;
};
__device__ __forceinline__ XMasks x_masks(const XWindow& W, uint64_t blk, uint64_t fs, uint64_t fe) {
  uint32_t P = 0, in = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    const int64_t pos = int64_t(blk) - 8 + i;
    const bool inside = pos >= int64_t(fs) && pos < int64_t(fe);
    in |= uint32_t(inside) << i;
    P |= uint32_t(inside && xprint(W.byte(i))) << i;
  }
  const uint32_t Q = P & (P >> 1) & (P >> 2) & (P >> 3) & (P >> 4);  // bit k: bytes k .. k+4 printable
  XMasks m;
  m.K = (Q | (Q << 1) | (Q << 2) | (Q << 3) | (Q << 4)) & P;
  m.C = ~P & in & (Q << 5);
  const int64_t last = int64_t(fe) - 1 - (int64_t(blk) - 8);  // window index of the file's last byte
  m.Z = (last >= 4 && last < 32 && ((Q >> (last - 4)) & 1u)) ? (1u << last) : 0u;
  return m;
}

// Walks a lane's 16 bytes in file order.  emit(byte) is called per output
// byte, start(f) at each file start inside the block (before its bytes).
template <typename Emit, typename Start>
__device__ __forceinline__ void x_lane(const uint8_t* raw, uint64_t n_bytes, const uint64_t* __restrict__ off,
                                       const uint8_t* __restrict__ kind, uint32_t n_files,
                                       const uint32_t* __restrict__ chunk_file, uint64_t blk, const XWindow& W,
                                       Emit emit, Start start) {
  if (blk >= n_bytes) return;
  uint32_t f = chunk_file[blk / kXTile];
  uint64_t fs = off[f], fe = off[f + 1];
  while (fe <= blk && f + 1 < n_files) {  // files ending before the block (the chunk map names the chunk's first)
    f++;
    fs = fe;
    fe = off[f + 1];
    if (fs >= blk) start(f);  // empty files at the block start
  }
  if (fs == blk) start(f);
  uint32_t k = kind[f];
  XMasks m = {0, 0, 0};
  if (k == 2) m = x_masks(W, blk, fs, fe);
  const uint64_t end = blk + 16 < n_bytes ? blk + 16 : n_bytes;
  for (uint64_t p = blk; p < end; p++) {
    while (p >= fe && f + 1 < n_files) {
      f++;
      fs = fe;
      fe = off[f + 1];
      start(f);
      k = kind[f];
      if (k == 2) m = x_masks(W, blk, fs, fe);
    }
    const int i = int(p - blk) + 8;
    const uint32_t b = W.byte(i);
    if (k == 0) {
      emit(b);
    } else if (k == 1) {
      if (b != '\r') emit(b);
    } else {
      if ((m.C >> i) & 1u) emit('\n');
      if ((m.K >> i) & 1u) emit(b);
      if ((m.Z >> i) & 1u) emit('\n');
    }
  }
}

__global__ __launch_bounds__(kXThreads) void xf_count_kernel(const uint8_t* __restrict__ raw, uint64_t n_bytes,
                                                             const uint64_t* __restrict__ off,
                                                             const uint8_t* __restrict__ kind, uint32_t n_files,
                                                             const uint32_t* __restrict__ chunk_file,
                                                             uint32_t* __restrict__ tile_cnt,
                                                             uint32_t* __restrict__ fstart) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  const uint64_t waves = uint64_t(gridDim.x) * (kXThreads / 64);
  for (uint64_t t = uint64_t(blockIdx.x) * (kXThreads / 64) + (threadIdx.x >> 6); t < n_tiles; t += waves) {
    const uint64_t blk = t * kXTile + 16 * uint64_t(lane);
    const uint4 v = blk < n_bytes ? *reinterpret_cast<const uint4*>(raw + blk) : make_uint4(0, 0, 0, 0);
    const XWindow W = x_window(raw, n_bytes, blk, lane, v);
    uint32_t c = 0;
    bool starts = false;
    x_lane(raw, n_bytes, off, kind, n_files, chunk_file, blk, W, [&](uint32_t) { c++; },
           [&](uint32_t) { starts = true; });
    const uint32_t ex = wave_excl(c, lane);
    if (lane == 63) tile_cnt[t] = ex + c;
    if (starts) {  // the files starting in this block: their tile-relative output offsets
      uint32_t c2 = ex;
      x_lane(raw, n_bytes, off, kind, n_files, chunk_file, blk, W, [&](uint32_t) { c2++; },
             [&](uint32_t f) { fstart[f] = c2; });
    }
  }
}

__global__ __launch_bounds__(kXThreads) void xf_fixup_kernel(const uint64_t* __restrict__ off, uint32_t n_files,
                                                             uint64_t n_bytes, const uint64_t* __restrict__ tile_pre,
                                                             const uint32_t* __restrict__ fstart,
                                                             uint64_t* __restrict__ xoff) {
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  for (uint32_t f = blockIdx.x * blockDim.x + threadIdx.x; f <= n_files; f += gridDim.x * blockDim.x) {
    const uint64_t s = f < n_files ? off[f] : n_bytes;
    xoff[f] = s < n_bytes ? tile_pre[s / kXTile] + fstart[f] : tile_pre[n_tiles];
  }
}

__global__ __launch_bounds__(kXThreads) void xf_write_kernel(const uint8_t* __restrict__ raw, uint64_t n_bytes,
                                                             const uint64_t* __restrict__ off,
                                                             const uint8_t* __restrict__ kind, uint32_t n_files,
                                                             const uint32_t* __restrict__ chunk_file,
                                                             const uint64_t* __restrict__ tile_pre,
                                                             uint8_t* __restrict__ out) {
  // a tile emits at most 1024 + 1024 / 5 + 16 bytes (a '\n' per closed run of >= 5 bytes)
  constexpr uint32_t kStage = 1280 + 32;
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kXThreads / 64][kStage];
  const uint32_t lane = threadIdx.x & 63u;
  uint8_t* S = s_out[threadIdx.x >> 6];
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  const uint64_t waves = uint64_t(gridDim.x) * (kXThreads / 64);
  for (uint64_t t = uint64_t(blockIdx.x) * (kXThreads / 64) + (threadIdx.x >> 6); t < n_tiles; t += waves) {
    const uint64_t blk = t * kXTile + 16 * uint64_t(lane);
    const uint4 v = blk < n_bytes ? *reinterpret_cast<const uint4*>(raw + blk) : make_uint4(0, 0, 0, 0);
    const XWindow W = x_window(raw, n_bytes, blk, lane, v);
    uint32_t c = 0;
    x_lane(raw, n_bytes, off, kind, n_files, chunk_file, blk, W, [&](uint32_t) { c++; }, [&](uint32_t) {});
    const uint32_t ex = wave_excl(c, lane);
    const uint32_t total = __shfl(ex + c, 63);
    const uint64_t start = tile_pre[t];
    const uint32_t phase = uint32_t(start & 15);  // the stage holds out[start - phase ..) at offset 0
    uint32_t at = phase + ex;
    x_lane(raw, n_bytes, off, kind, n_files, chunk_file, blk, W, [&](uint32_t b) { S[at++] = uint8_t(b); },
           [&](uint32_t) {});
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t base = start - phase, end = start + total;
    for (uint32_t q = 16 * lane; base + q < end; q += 1024) {
      const uint64_t g = base + q;
      if (g >= start && g + 16 <= end) {
        *reinterpret_cast<uint4*>(out + g) = *reinterpret_cast<const uint4*>(S + q);
      } else {  // the ragged ends: only this tile's bytes
        for (uint32_t j = 0; j < 16; j++)
          if (g + j >= start && g + j < end) out[g + j] = S[q + j];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
  size_t chunk_file, tile_cnt, tile_pre, fstart, scan, scan_bytes, total;
};

static XformScratch ScratchLayout(uint64_t n_bytes, uint32_t n_files) {
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  XformScratch L;
  size_t scan = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan, static_cast<const uint32_t*>(nullptr),
                                         static_cast<uint64_t*>(nullptr), int(n_tiles) + 1);
  auto up = [](size_t x) { return (x + 255) & ~size_t(255); };
  L.chunk_file = 0;
  L.tile_cnt = up(L.chunk_file + (n_tiles + 1) * 4);
  L.tile_pre = up(L.tile_cnt + (n_tiles + 1) * 4);
  L.fstart = up(L.tile_pre + (n_tiles + 1) * 8);
  L.scan = up(L.fstart + (size_t(n_files) + 1) * 4);
  L.scan_bytes = scan;
  L.total = up(L.scan + scan + 16);
  return L;
}

size_t XformScratchBytes(uint64_t n_bytes, uint32_t n_files) { return ScratchLayout(n_bytes, n_files).total; }

hipError_t XformPlan(const uint8_t* raw, uint64_t n_bytes, const uint64_t* off, const uint8_t* kind, uint32_t n_files,
                     void* scratch, uint64_t* xoff, hipStream_t s) {
  const XformScratch L = ScratchLayout(n_bytes, n_files);
  uint8_t* sc = static_cast<uint8_t*>(scratch);
  uint32_t* chunk_file = reinterpret_cast<uint32_t*>(sc + L.chunk_file);
  uint32_t* tile_cnt = reinterpret_cast<uint32_t*>(sc + L.tile_cnt);
  uint64_t* tile_pre = reinterpret_cast<uint64_t*>(sc + L.tile_pre);
  uint32_t* fstart = reinterpret_cast<uint32_t*>(sc + L.fstart);
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  hipError_t e;
  if ((e = hipMemsetAsync(tile_cnt, 0, (n_tiles + 1) * 4, s)) != hipSuccess) return e;
  if (n_files) {
    xf_chunk_map_kernel<<<grid_for((n_files + 63) / 64), kXThreads, 0, s>>>(off, n_files, chunk_file);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (n_tiles) {
    const uint32_t g = uint32_t(std::min<uint64_t>((n_tiles + kXThreads / 64 - 1) / (kXThreads / 64), 8192));
    xf_count_kernel<<<g, kXThreads, 0, s>>>(raw, n_bytes, off, kind, n_files, chunk_file, tile_cnt, fstart);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  size_t sb = L.scan_bytes;
  if ((e = hipcub::DeviceScan::ExclusiveSum(sc + L.scan, sb, tile_cnt, tile_pre, int(n_tiles) + 1, s)) != hipSuccess)
    return e;
  xf_fixup_kernel<<<grid_for((n_files + 64) / 64), kXThreads, 0, s>>>(off, n_files, n_bytes, tile_pre, fstart, xoff);
  return hipGetLastError();
}

hipError_t XformWrite(const uint8_t* raw, uint64_t n_bytes, const uint64_t* off, const uint8_t* kind, uint32_t n_files,
                      const void* scratch, uint8_t* out, hipStream_t s) {
  const XformScratch L = ScratchLayout(n_bytes, n_files);
  const uint8_t* sc = static_cast<const uint8_t*>(scratch);
  const uint64_t n_tiles = (n_bytes + kXTile - 1) / kXTile;
  if (!n_tiles) return hipSuccess;
  const uint32_t g = uint32_t(std::min<uint64_t>((n_tiles + kXThreads / 64 - 1) / (kXThreads / 64), 8192));
  xf_write_kernel<<<g, kXThreads, 0, s>>>(raw, n_bytes, off, kind, n_files,
                                          reinterpret_cast<const uint32_t*>(sc + L.chunk_file),
                                          reinterpret_cast<const uint64_t*>(sc + L.tile_pre), out);
  return hipGetLastError();
}

hipError_t GatherFiles(const uint8_t* src, const uint64_t* xoff, const uint32_t* files, const uint64_t* dst_off,
                       uint32_t n, uint8_t* dst, hipStream_t s) {
  if (n == 0) return hipSuccess;
  gather_kernel<<<grid_for(n), kXThreads, 0, s>>>(src, xoff, files, dst_off, n, dst);
  return hipGetLastError();
}

}  // namespace tsg
