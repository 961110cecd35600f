// GPU pre-transform of host batches: the per-file byte
// transforms the secret analyzer applies before Scanner.Scan, run on the
// bytes as read instead of on host threads.
//   kind 0  as is
//   kind 1  every '\r' removed: bytes.ReplaceAll(content, "\r", "")
//           (pkg/fanal/analyzer/secret/secret.go:121)
//   kind 2  utils.ExtractPrintableBytes (pkg/fanal/utils/utils.go:128-160):
//           runs of more than 4 unicode.IsPrint bytes, each followed by '\n'
//           (.pyc binaries, secret.go:112-117)
// Three launches per chunk: lengths (one wave per file: SWAR '\r' counts over
// 16-B loads, or the printable-run plan), an exclusive scan of the lengths
// into the transformed offsets (hipcub), the copy (one wave per file).  Files
// that keep every byte -- all of a layer but its CRLF files and .pyc binaries
// -- are moved as 16-B-aligned destination blocks, each lane funnel-shifting
// the two aligned source blocks around its block by the file's (uniform)
// source/destination misalignment: coalesced 16-B loads and stores, byte
// stores only in a file's first and last block (shared with the neighbouring
// files' waves).  CRLF files compact 1 KiB per step (per-lane kept-byte
// counts, a wave prefix sum).  A gather packs chosen files of the transformed
// arena for the host's exact pass with the same shifted block copy.
#include "xform.h"

#include <hipcub/hipcub.hpp>

namespace tsg {
namespace {

constexpr int kXThreads = 256;

__device__ __forceinline__ uint4 xload16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

__device__ __forceinline__ uint32_t xbyte(const uint4& v, uint32_t i) {
  const uint32_t w = i < 8 ? (i < 4 ? v.x : v.y) : (i < 12 ? v.z : v.w);
  return (w >> (8 * (i & 3))) & 0xFFu;
}

// Bytes of the word at arena position wp that lie in [a, b), as a byte mask.
__device__ __forceinline__ uint32_t byte_mask(uint64_t wp, uint64_t a, uint64_t b) {
  const uint32_t lo = a > wp ? uint32_t(a - wp < 4 ? a - wp : 4) : 0u;  // bytes before a
  const uint32_t hi = b > wp ? uint32_t(b - wp < 4 ? b - wp : 4) : 0u;  // bytes before b
  const uint32_t mhi = hi >= 4 ? ~0u : (1u << (8 * hi)) - 1u;
  const uint32_t mlo = lo >= 4 ? 0u : ~((1u << (8 * lo)) - 1u);
  return mhi & mlo;
}

// '\r' bytes of w among the bytes of mask m: x = w ^ 0x0D.. is zero exactly
// in CR bytes (forced non-zero outside m); bit 7 of ((x & 0x7F..) + 0x7F..) | x
// marks the non-zero bytes.
__device__ __forceinline__ uint32_t cr_count4(uint32_t w, uint32_t m) {
  const uint32_t x = (w ^ 0x0D0D0D0Du) | ~m;
  const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
  return 4u - uint32_t(__popc(nz));
}

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

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  return v;
}

__device__ __forceinline__ uint32_t wave_excl(uint32_t v, uint32_t lane) {  // exclusive prefix over lanes
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= uint32_t(d)) x += y;
  }
  return x - v;
}

// ExtractPrintableBytes on one wave (kind 2).  The file is cut into 64 lane
// chunks.  Pass 1: each lane scans its chunk -- leading printable run (pre),
// trailing run (suf), the output of the runs strictly inside (inner), whether
// the chunk is all printable.  Lane 0 then walks the 64 chunks in order,
// joining the runs that cross chunk boundaries: it places every run's output
// and decides it kept (> 4 bytes) or not, and leaves each lane its positions.
// Pass 2 (copy kernel): each lane writes its chunk's share -- the head of a
// run that began in earlier chunks, its inner runs (the first 4 bytes of a run
// wait in registers until the run is long enough), the tail of a run that
// continues into later chunks.
struct PycPlan {
  uint64_t c0[64], c1[64];           // chunk [c0, c1) (file-relative)
  uint64_t pre[64], suf[64], inner[64];
  uint8_t full[64];
  uint64_t pos_pre[64], pos_inner[64], pos_suf[64];  // output positions (file-relative)
  uint8_t keep_pre[64], end_pre[64], keep_suf[64];   // end_pre: the run through the chunk head ends in it
  uint64_t total;
  uint64_t final_pos;  // the '\n' after a kept run that reaches the file end
  uint8_t final_keep;
};

__device__ void pyc_plan(const uint8_t* in, uint64_t n, uint32_t lane, PycPlan* P) {
  const uint64_t cs = (n + 63) / 64;
  const uint64_t c0 = lane * cs < n ? lane * cs : n, c1 = c0 + cs < n ? c0 + cs : n;
  uint64_t cur = 0, pre = 0, inner = 0;
  bool seen = false;  // a non-printable byte in the chunk
  for (uint64_t i = c0; i < c1; i++) {
    if (xprint(in[i])) {
      cur++;
      continue;
    }
    if (!seen) pre = cur;
    else if (cur > 4) inner += cur + 1;
    cur = 0;
    seen = true;
  }
  P->c0[lane] = c0;
  P->c1[lane] = c1;
  P->full[lane] = seen ? 0 : 1;
  P->pre[lane] = seen ? pre : c1 - c0;
  P->suf[lane] = seen ? cur : 0;
  P->inner[lane] = inner;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane == 0) {
    uint64_t emitted = 0, open = 0, start_pos = 0;
    int first = -1;  // first lane of the open run (-1: none); first_suf: it starts in that lane's tail
    bool first_suf = false;
    auto close = [&](int last) {  // the open run ends in lane `last` (or at the file end: last = -1)
      const bool keep = open > 4;
      for (int j = first < 0 ? 64 : first; j < 64 && (last < 0 || j <= last); j++) {
        if (j == first && first_suf) P->keep_suf[j] = keep;
        else P->keep_pre[j] = keep;
      }
      if (keep) emitted = start_pos + open + 1;
      if (last < 0) {
        P->final_keep = keep;
        P->final_pos = start_pos + open;
      }
      open = 0;
      first = -1;
    };
    P->final_keep = 0;
    for (int i = 0; i < 64; i++) {
      P->keep_pre[i] = 0;
      P->end_pre[i] = 0;
      P->keep_suf[i] = 0;
      P->pos_suf[i] = 0;
    }
    for (int i = 0; i < 64; i++) {
      const uint64_t len = P->c1[i] - P->c0[i];
      if (len == 0) continue;
      if (P->full[i]) {
        if (first < 0) {
          first = i;
          first_suf = false;
          start_pos = emitted;
        }
        P->pos_pre[i] = start_pos + open;
        open += len;
        continue;
      }
      // the run through the chunk head (possibly empty) ends here
      if (first < 0) {
        first = i;
        first_suf = false;
        start_pos = emitted;
      }
      P->pos_pre[i] = start_pos + open;
      open += P->pre[i];
      P->end_pre[i] = 1;
      close(i);
      P->pos_inner[i] = emitted;
      emitted += P->inner[i];
      if (P->suf[i] > 0) {
        first = i;
        first_suf = true;
        start_pos = emitted;
        P->pos_suf[i] = emitted;
        open = P->suf[i];
      }
    }
    if (first >= 0) close(-1);
    P->total = emitted;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Pass 2 for lane `lane` (plan from pyc_plan).
__device__ void pyc_write(const uint8_t* in, uint32_t lane, const PycPlan* P, uint8_t* out) {
  const uint64_t c0 = P->c0[lane], c1 = P->c1[lane];
  if (lane == 0 && P->final_keep) out[P->final_pos] = '\n';
  if (c1 <= c0) return;
  uint64_t i = c0;
  // head: the bytes of the run through the chunk head
  const uint64_t pre = P->pre[lane];
  if (P->keep_pre[lane])
    for (uint64_t k = 0; k < pre; k++) out[P->pos_pre[lane] + k] = in[c0 + k];
  if (P->full[lane]) return;
  if (P->end_pre[lane] && P->keep_pre[lane]) out[P->pos_pre[lane] + pre] = '\n';
  i = c0 + pre + 1;  // past the first non-printable byte
  // inner runs up to the chunk's last non-printable byte
  const uint64_t tail0 = c1 - P->suf[lane];  // the suffix run starts here
  uint64_t w = P->pos_inner[lane], run = 0;
  uint8_t held[4];
  for (; i < tail0; i++) {
    const uint8_t b = in[i];
    if (xprint(b)) {
      if (run < 4) {
        held[run] = b;
      } else {
        if (run == 4)
          for (int k = 0; k < 4; k++) out[w + k] = held[k];
        out[w + run] = b;
      }
      run++;
      continue;
    }
    if (run > 4) {
      out[w + run] = '\n';
      w += run + 1;
    }
    run = 0;
  }
  // the suffix run (its '\n' is written where it ends)
  if (P->keep_suf[lane])
    for (uint64_t k = 0; k < P->suf[lane]; k++) out[P->pos_suf[lane] + k] = in[tail0 + k];
}

__global__ __launch_bounds__(kXThreads) void xform_len_kernel(const uint8_t* __restrict__ raw,
                                                              const uint64_t* __restrict__ off,
                                                              const uint8_t* __restrict__ kind, uint32_t n_files,
                                                              uint64_t* __restrict__ len) {
  __shared__ PycPlan s_plan[kXThreads / 64];
  PycPlan* plan = &s_plan[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (kXThreads / 64);
  for (uint32_t f = blockIdx.x * (kXThreads / 64) + (threadIdx.x >> 6); f < n_files; f += waves) {
    const uint64_t a = off[f], b = off[f + 1];
    const uint32_t k = kind[f];
    uint64_t out = b - a;
    if (k == 1) {
      uint32_t cr = 0;
      for (uint64_t blk = (a & ~uint64_t(15)) + 16 * lane; blk < b; blk += 1024) {
        const uint4 v = xload16(raw + blk);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) cr += cr_count4(w[q], byte_mask(blk + 4 * q, a, b));
      }
      out -= wave_sum(cr);
    } else if (k == 2) {
      pyc_plan(raw + a, b - a, lane, plan);
      out = plan->total;
    }
    if (lane == 0) len[f] = out;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) len[n_files] = 0;
}

__global__ __launch_bounds__(kXThreads) void xform_copy_kernel(const uint8_t* __restrict__ raw,
                                                               const uint64_t* __restrict__ off,
                                                               const uint8_t* __restrict__ kind, uint32_t n_files,
                                                               const uint64_t* __restrict__ xoff,
                                                               uint8_t* __restrict__ out) {
  __shared__ PycPlan s_plan[kXThreads / 64];
  PycPlan* plan = &s_plan[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (kXThreads / 64);
  for (uint32_t f = blockIdx.x * (kXThreads / 64) + (threadIdx.x >> 6); f < n_files; f += waves) {
    const uint64_t a = off[f], b = off[f + 1];
    const uint32_t k = kind[f];
    uint8_t* dst = out + xoff[f];
    if (k == 2) {
      pyc_plan(raw + a, b - a, lane, plan);
      pyc_write(raw + a, lane, plan, dst);
      continue;
    }
    if (k != 1 || xoff[f + 1] - xoff[f] == b - a) {  // every byte kept: the shifted block copy
      copy_shifted(raw, a, out, xoff[f], b - a, lane);
      continue;
    }
    uint64_t written = 0;
    for (uint64_t t0 = a & ~uint64_t(15); t0 < b; t0 += 1024) {
      const uint64_t blk = t0 + 16 * lane;
      const uint4 v = blk < b ? xload16(raw + blk) : make_uint4(0, 0, 0, 0);
      uint32_t keep = 0;  // bit i: byte blk + i is kept
#pragma unroll
      for (uint32_t i = 0; i < 16; i++) {
        const bool in = blk + i >= a && blk + i < b;
        keep |= uint32_t(in && !(k == 1 && xbyte(v, i) == '\r')) << i;
      }
      const uint32_t c = __popc(keep);
      const uint64_t at = written + wave_excl(c, lane);
      uint32_t j = 0;
#pragma unroll
      for (uint32_t i = 0; i < 16; i++)
        if ((keep >> i) & 1u) dst[at + j++] = uint8_t(xbyte(v, i));
      written += wave_sum(c);
    }
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

hipError_t XformLengths(const uint8_t* raw, const uint64_t* off, const uint8_t* kind, uint32_t n_files, uint64_t* len,
                        hipStream_t s) {
  xform_len_kernel<<<grid_for(n_files), kXThreads, 0, s>>>(raw, off, kind, n_files, len);
  return hipGetLastError();
}

hipError_t XformScanBytes(uint32_t n_files, size_t* bytes) {
  *bytes = 0;
  return hipcub::DeviceScan::ExclusiveSum(nullptr, *bytes, static_cast<const uint64_t*>(nullptr),
                                          static_cast<uint64_t*>(nullptr), int(n_files) + 1);
}

hipError_t XformScan(void* temp, size_t temp_bytes, const uint64_t* len, uint64_t* xoff, uint32_t n_files,
                     hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, len, xoff, int(n_files) + 1, s);
}

hipError_t XformCopy(const uint8_t* raw, const uint64_t* off, const uint8_t* kind, uint32_t n_files,
                     const uint64_t* xoff, uint8_t* out, hipStream_t s) {
  xform_copy_kernel<<<grid_for(n_files), kXThreads, 0, s>>>(raw, off, kind, n_files, xoff, out);
  return hipGetLastError();
}

hipError_t GatherFiles(const uint8_t* src, const uint64_t* xoff, const uint32_t* files, const uint64_t* dst_off,
                       uint32_t n, uint8_t* dst, hipStream_t s) {
  if (n == 0) return hipSuccess;
  gather_kernel<<<grid_for(n), kXThreads, 0, s>>>(src, xoff, files, dst_off, n, dst);
  return hipGetLastError();
}

}  // namespace tsg
