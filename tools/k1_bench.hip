// K1 design microbenchmark (not product code): streaming-read patterns and the
// shift-or (FDR-layout) inner loop with an LDS-replicated mask table.
//   hipcc --offload-arch=gfx950 -O3 -o tools/k1_bench tools/k1_bench.hip
//   ./tools/k1_bench [GB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void fill_kernel(uint4* p, uint64_t n16) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull;
    uint32_t w[4];
    for (int k = 0; k < 4; k++) {
      uint32_t v = 0;
      for (int b = 0; b < 4; b++) {
        x ^= x >> 29;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 32;
        uint32_t r = uint32_t(x) % 40;
        uint32_t c = r < 6 ? ' ' : r < 7 ? '\n' : 'a' + (r - 7) % 26;
        v |= c << (8 * b);
      }
      w[k] = v;
    }
    p[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// (a) fully coalesced: consecutive lanes read consecutive 16-B pieces
__global__ __launch_bounds__(1024) void read_coalesced(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
  }
  for (; i < n16; i += stride) {
    uint4 a = p[i];
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// (b) per-lane contiguous chunks of C bytes (C multiple of 64), 64-B groups, two in flight
template <int C>
__global__ __launch_bounds__(1024) void read_lane_chunks(const uint8_t* __restrict__ a, uint64_t n, uint32_t* out) {
  const uint64_t lanes = uint64_t(gridDim.x) * blockDim.x;
  const uint64_t nch = n / C;
  uint32_t acc = 0;
  for (uint64_t c = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; c < nch; c += lanes) {
    const uint4* q = reinterpret_cast<const uint4*>(a + c * C);
#pragma unroll 2
    for (int g = 0; g < C / 16; g += 4) {
      uint4 x0 = q[g], x1 = q[g + 1], x2 = q[g + 2], x3 = q[g + 3];
      acc ^= x0.x ^ x0.y ^ x0.z ^ x0.w ^ x1.x ^ x1.y ^ x1.z ^ x1.w ^ x2.x ^ x2.y ^ x2.z ^ x2.w ^ x3.x ^ x3.y ^
             x3.z ^ x3.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__device__ __forceinline__ uint32_t nl_in_word(uint32_t w) {
  const uint32_t x = w ^ 0x0A0A0A0Au;
  const uint32_t nz = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;
  return 4u - __popc(nz & 0x80808080u);
}

// (c) shift-or over per-lane chunks: table of 256 u64 masks replicated 32x in
// LDS (row b at b*256, copy (lane&31) at +8*(lane&31)): conflict-free ds_read_b64.
template <int C, bool kNl>
__global__ __launch_bounds__(1024) void fdr_lane_chunks(const uint8_t* __restrict__ a, uint64_t n,
                                                        const uint64_t* __restrict__ tab, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint64_t s_tab[256 * 32];
  for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) s_tab[i] = tab[i >> 5];
  __syncthreads();
  const uint32_t lane8 = (threadIdx.x & 31) * 8;
  const uint8_t* sb = reinterpret_cast<const uint8_t*>(s_tab);
  const uint64_t lanes = uint64_t(gridDim.x) * blockDim.x;
  const uint64_t nch = n / C;
  uint32_t flagged = 0, nl = 0;
  for (uint64_t c = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; c < nch; c += lanes) {
    const uint4* q = reinterpret_cast<const uint4*>(a + c * C);
    uint32_t lo = ~0u, hi = ~0u;
    uint4 nx0 = q[0], nx1 = q[1];
    for (int g = 0; g < C / 16; g += 2) {
      const uint4 v0 = nx0, v1 = nx1;
      if (g + 2 < C / 16) {
        nx0 = q[g + 2];
        nx1 = q[g + 3];
      }
      const uint32_t wd[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int h = 0; h < 2; h++) {
        uint32_t acc = ~0u;
#pragma unroll
        for (int k = 0; k < 16; k++) {
          const uint32_t w = wd[h * 4 + (k >> 2)];
          const uint32_t addr = __builtin_amdgcn_perm(w, lane8, 0x0C0C0000u | ((4u + (k & 3)) << 8));
          const uint64_t m = *reinterpret_cast<const uint64_t*>(sb + addr);
          hi = __builtin_amdgcn_alignbit(hi, lo, 24) | uint32_t(m >> 32);
          lo = (lo << 8) | uint32_t(m);
          acc &= hi;
        }
        flagged += (acc >> 24) != 0xFFu;
        if (kNl) nl += nl_in_word(wd[h * 4]) + nl_in_word(wd[h * 4 + 1]) + nl_in_word(wd[h * 4 + 2]) +
                       nl_in_word(wd[h * 4 + 3]);
      }
    }
  }
  atomicAdd(out + 1, flagged);
  atomicAdd(out + 2, nl);
}


// (d) shift-or over wave tiles: lane l owns bytes [T + CL*l, T + CL*(l+1)); the 8 bytes before a lane's
// chunk come from lane l-1 (ds_bpermute) or, for lane 0, from an extra 8-B load issued with the
// prefetch of the next tile.
template <int CL>
__global__ __launch_bounds__(1024) void fdr_tiles(const uint8_t* __restrict__ a, uint64_t n,
                                                  const uint64_t* __restrict__ tab, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint64_t s_tab[256 * 32];
  for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) s_tab[i] = tab[i >> 5];
  __syncthreads();
  constexpr int NB = CL / 16;
  constexpr uint64_t TILE = uint64_t(CL) * 64;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t lane8 = (lane & 31) * 8;
  const uint8_t* sb = reinterpret_cast<const uint8_t*>(s_tab);
  const uint64_t wave = (blockIdx.x * uint64_t(blockDim.x) + threadIdx.x) >> 6;
  const uint64_t n_waves = (uint64_t(gridDim.x) * blockDim.x) >> 6;
  const uint64_t ntiles = n / TILE;
  uint32_t flagged = 0, nl = 0;
  uint4 cur[NB], nxt[NB];
  uint2 pcur = make_uint2(0, 0), pnxt = make_uint2(0, 0);
  uint64_t t = wave;
  auto load = [&](uint4* dst, uint2* pv, uint64_t tt) {
    const uint4* q = reinterpret_cast<const uint4*>(a + tt * TILE + uint64_t(lane) * CL);
#pragma unroll
    for (int j = 0; j < NB; j++) dst[j] = q[j];
    if (lane == 0 && tt > 0) *pv = *reinterpret_cast<const uint2*>(a + tt * TILE - 8);
  };
  if (t < ntiles) load(cur, &pcur, t);
  for (; t < ntiles; t += n_waves) {
    if (t + n_waves < ntiles) load(nxt, &pnxt, t + n_waves);
    uint32_t w0 = __shfl(cur[NB - 1].z, int(lane) - 1), w1 = __shfl(cur[NB - 1].w, int(lane) - 1);
    if (lane == 0) {
      w0 = pcur.x;
      w1 = pcur.y;
    }
    uint32_t lo = ~0u, hi = ~0u;
    const uint32_t pw[2] = {w0, w1};
#pragma unroll
    for (int k = 1; k < 8; k++) {
      const uint32_t addr = __builtin_amdgcn_perm(pw[k >> 2], lane8, 0x0C0C0000u | ((4u + (k & 3)) << 8));
      const uint64_t m = *reinterpret_cast<const uint64_t*>(sb + addr);
      hi = __builtin_amdgcn_alignbit(hi, lo, 24) | uint32_t(m >> 32);
      lo = (lo << 8) | uint32_t(m);
    }
#pragma unroll
    for (int j = 0; j < NB; j++) {
      const uint32_t wd[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
      uint32_t acc = ~0u;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint32_t addr = __builtin_amdgcn_perm(wd[k >> 2], lane8, 0x0C0C0000u | ((4u + (k & 3)) << 8));
        const uint64_t m = *reinterpret_cast<const uint64_t*>(sb + addr);
        hi = __builtin_amdgcn_alignbit(hi, lo, 24) | uint32_t(m >> 32);
        lo = (lo << 8) | uint32_t(m);
        acc &= hi;
      }
      flagged += (acc >> 24) != 0xFFu;
      nl += nl_in_word(wd[0]) + nl_in_word(wd[1]) + nl_in_word(wd[2]) + nl_in_word(wd[3]);
    }
#pragma unroll
    for (int j = 0; j < NB; j++) cur[j] = nxt[j];
    pcur = pnxt;
  }
  atomicAdd(out + 1, flagged);
  atomicAdd(out + 2, nl);
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  CK(hipDeviceSynchronize());
  hipEventRecord(a);
  for (int i = 0; i < reps; i++) f();
  hipEventRecord(b);
  CK(hipEventSynchronize(b));
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char** argv) {
  double gb = argc > 1 ? std::atof(argv[1]) : 8.0;
  uint64_t n = uint64_t(gb * 1e9) & ~uint64_t(4095);
  uint8_t* d;
  uint32_t* out;
  uint64_t* tab;
  CK(hipMalloc(&d, n + 4096));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&tab, 256 * 8));
  fill_kernel<<<4096, 256>>>(reinterpret_cast<uint4*>(d), n / 16);
  // table: letters allowed only at a few slots/buckets -> rare flags
  std::vector<uint64_t> h(256, ~0ull);
  const char* pats[8] = {"ghp_", "akia", "xoxb", "-----", "dapi", "sk_l", "glpa", "pypi"};
  for (int j = 0; j < 8; j++) {
    int L = 0;
    while (pats[j][L]) L++;
    for (int s = 0; s < 8; s++) {
      int k = s - (8 - L);
      for (int b = 0; b < 256; b++) {
        bool ok = k < 0 || b == pats[j][k];
        if (ok) h[b] &= ~(uint64_t(1) << (8 * s + j));
      }
    }
  }
  CK(hipMemcpy(tab, h.data(), 256 * 8, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  const int grid_c = 256 * 8;
  auto rep = [&](const char* name, float ms) {
    std::printf("%-28s %8.3f ms  %7.3f TB/s\n", name, ms, n / (ms * 1e-3) / 1e12);
  };
  rep("coalesced", timeit([&] { read_coalesced<<<grid_c, 1024>>>(reinterpret_cast<uint4*>(d), n / 16, out); }, 5));
  rep("lane_chunks<64>", timeit([&] { read_lane_chunks<64><<<256 * 2, 1024>>>(d, n, out); }, 5));
  rep("lane_chunks<256>", timeit([&] { read_lane_chunks<256><<<256 * 2, 1024>>>(d, n, out); }, 5));
  rep("lane_chunks<1024>", timeit([&] { read_lane_chunks<1024><<<256 * 2, 1024>>>(d, n, out); }, 5));
  rep("lane_chunks<4096>", timeit([&] { read_lane_chunks<4096><<<256 * 2, 1024>>>(d, n, out); }, 5));
  for (int nl = 0; nl < 2; nl++) {
    auto go = [&](auto kern, const char* name) {
      CK(hipMemset(out, 0, 64));
      float ms = timeit([&] { kern<<<256, 1024>>>(d, n, tab, out); }, 5);
      uint32_t o[3];
      CK(hipMemcpy(o, out, 12, hipMemcpyDeviceToHost));
      char buf[64];
      std::snprintf(buf, sizeof buf, "%s%s", name, nl ? "+nl" : "");
      rep(buf, ms);
      std::printf("   flagged 32-B blocks/launch %.0f  nl/launch %.0f\n", o[1] / 6.0, o[2] / 6.0);
    };
    if (nl) {
      go(fdr_lane_chunks<256, true>, "fdr<256>");
      go(fdr_lane_chunks<1024, true>, "fdr<1024>");
    } else {
      go(fdr_lane_chunks<256, false>, "fdr<256>");
      go(fdr_lane_chunks<1024, false>, "fdr<1024>");
      go(fdr_lane_chunks<4096, false>, "fdr<4096>");
    }
  }

  for (int grid : {256, 512}) {
    auto go2 = [&](auto kern, const char* name) {
      CK(hipMemset(out, 0, 64));
      float ms = timeit([&] { kern<<<grid, 1024>>>(d, n, tab, out); }, 5);
      uint32_t o[3];
      CK(hipMemcpy(o, out, 12, hipMemcpyDeviceToHost));
      char buf[64];
      std::snprintf(buf, sizeof buf, "%s g%d", name, grid);
      rep(buf, ms);
      std::printf("   flagged 16-B blocks/launch %.0f  nl/launch %.0f\n", o[1] / 6.0, o[2] / 6.0);
    };
    go2(fdr_tiles<64>, "fdr_tiles<64>");
    go2(fdr_tiles<128>, "fdr_tiles<128>");
  }
  return 0;
}
