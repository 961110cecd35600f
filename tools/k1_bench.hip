// K1 design microbenchmark (not product code): the streaming filter's hot
// loop in isolation (64-B lane chunks, 16 buckets = two u64 shift-or
// registers, LDS reach table replicated 16x), with variants that remove one
// ingredient at a time, to see which one bounds the loop.
//   hipcc --offload-arch=gfx950 -O3 -o tools/k1_bench tools/k1_bench.hip
//   ./tools/k1_bench [GB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e = (x);                                                                      \
    if (e != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(1);                                                                          \
    }                                                                                        \
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

__device__ __forceinline__ void shift_or(uint32_t& lo, uint32_t& hi, uint32_t mlo, uint32_t mhi) {
  uint32_t h;
  asm("v_alignbit_b32 %0, %1, %2, 24" : "=v"(h) : "v"(hi), "v"(lo));
  asm("v_or_b32 %0, %1, %2" : "=v"(hi) : "v"(h), "v"(mhi));
  asm("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(lo) : "v"(lo), "v"(mlo));
}

__device__ __forceinline__ uint32_t nl_count4(uint32_t w) {
  const uint32_t a = ((w ^ 0x0A0A0A0Au) & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return __popc(~(a | w) & 0x80808080u);
}

__device__ __forceinline__ uint4 rd(const uint8_t* sb, uint32_t w, uint32_t k, uint32_t laneoff) {
  return *reinterpret_cast<const uint4*>(sb + __builtin_amdgcn_perm(w, laneoff, 0x0C0C0000u | ((4u + k) << 8)));
}

// MODE 0: full (LDS reads + chain + nl); 1: no LDS (mask = data); 2: LDS reads only
// (OR-reduced, no chain); 3: loads + nl only; 4: full, no nl
template <int MODE, int LB>
__global__ __launch_bounds__(1024) void filt(const uint8_t* __restrict__ a, uint64_t n, const uint64_t* __restrict__ tab,
                                             uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t s_reach[65536];
  for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) {
    const uint32_t b = i / 16;
    reinterpret_cast<uint64_t*>(s_reach)[2 * i] = tab[2 * b];
    reinterpret_cast<uint64_t*>(s_reach)[2 * i + 1] = tab[2 * b + 1];
  }
  __syncthreads();
  constexpr int NB = LB / 16;
  constexpr uint64_t TILE = uint64_t(LB) * 64;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t laneoff = (lane & 15) * 16;
  const uint64_t wave = (blockIdx.x * uint64_t(blockDim.x) + threadIdx.x) >> 6;
  const uint64_t n_waves = (uint64_t(gridDim.x) * blockDim.x) >> 6;
  const uint64_t ntiles = n / TILE;
  uint32_t flagged = 0, nl = 0;
  uint4 cur[NB], nxt[NB];
  uint64_t t = wave;
  auto load = [&](uint4* dst, uint64_t tt) {
    const uint4* q = reinterpret_cast<const uint4*>(a + tt * TILE + uint64_t(lane) * LB);
#pragma unroll
    for (int j = 0; j < NB; j++) dst[j] = q[j];
  };
  if (t < ntiles) load(cur, t);
  for (; t < ntiles; t += n_waves) {
    if (t + n_waves < ntiles) load(nxt, t + n_waves);
    if (MODE != 3) {
      uint32_t p1 = __shfl(cur[NB - 1].w, int(lane) - 1);
      uint32_t st[4] = {~0u, ~0u, ~0u, ~0u};
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        uint4 m = rd(s_reach, p1, k, laneoff);
        shift_or(st[0], st[1], m.x, m.y);
        shift_or(st[2], st[3], m.z, m.w);
      }
#pragma unroll
      for (int j = 0; j < NB; j++) {
        const uint32_t wd[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
        uint4 m[16];
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) {
          if (MODE == 1) {
            const uint32_t x = wd[k >> 2] >> (8 * (k & 3));
            m[k] = make_uint4(x, x ^ laneoff, x + 1, x ^ 0x55);
          } else {
            m[k] = rd(s_reach, wd[k >> 2], k & 3, laneoff);
          }
        }
        uint32_t acc = ~0u;
        if (MODE == 2) {
#pragma unroll
          for (uint32_t k = 0; k < 16; k++) acc &= m[k].x | m[k].y | m[k].z | m[k].w;
        } else {
#pragma unroll
          for (uint32_t k = 0; k < 16; k++) {
            shift_or(st[0], st[1], m[k].x, m[k].y);
            shift_or(st[2], st[3], m[k].z, m[k].w);
            if (k % 3 == 2 || k == 15) acc &= st[1] & st[3];
          }
        }
        flagged += (acc | 0xFFu) != ~0u;
      }
    }
    if (MODE != 4) {
#pragma unroll
      for (int j = 0; j < NB; j++)
        nl += nl_count4(cur[j].x) + nl_count4(cur[j].y) + nl_count4(cur[j].z) + nl_count4(cur[j].w);
    }
#pragma unroll
    for (int j = 0; j < NB; j++) cur[j] = nxt[j];
  }
  atomicAdd(out + 1, flagged);
  atomicAdd(out + 2, nl);
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  double gb = argc > 1 ? std::atof(argv[1]) : 8.0;
  uint64_t n = uint64_t(gb * 1e9) & ~uint64_t(8191);
  uint8_t* d;
  uint32_t* out;
  uint64_t* tab;
  CK(hipMalloc(&d, n + 4096));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&tab, 256 * 16));
  fill_kernel<<<4096, 256>>>(reinterpret_cast<uint4*>(d), n / 16);
  std::vector<uint64_t> h(512, ~0ull);
  const char* pats[16] = {"ghp_", "akia", "xoxb", "-----", "dapi", "sk_l", "glpa", "pypi",
                          "aws_", "linea", "facebo", "twitt", "disco", "mailg", "hubsp", "asana"};
  for (int j = 0; j < 16; j++) {
    int L = 0;
    while (pats[j][L]) L++;
    for (int s = 0; s < 8; s++) {
      int k = s - (6 - L);
      for (int b = 0; b < 256; b++) {
        bool ok = s >= 6 || k < 0 || b == pats[j][k];
        if (ok) h[2 * b + j / 8] &= ~(uint64_t(1) << (8 * s + (j % 8)));
      }
    }
  }
  CK(hipMemcpy(tab, h.data(), 256 * 16, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  auto go = [&](auto kern, const char* name, int grid) {
    CK(hipMemset(out, 0, 64));
    float ms = timeit([&] { kern<<<grid, 1024>>>(d, n, tab, out); }, 5);
    uint32_t o[3];
    CK(hipMemcpy(o, out, 12, hipMemcpyDeviceToHost));
    std::printf("%-24s g%-4d %8.3f ms  %7.3f TB/s  flagged/launch %.0f\n", name, grid, ms, n / (ms * 1e-3) / 1e12,
                o[1] / 6.0);
  };
  for (int grid : {256, 512}) {
    go(filt<0, 64>, "full<64>", grid);
    go(filt<4, 64>, "full-no-nl<64>", grid);
    go(filt<1, 64>, "no-lds<64>", grid);
    go(filt<2, 64>, "lds-only<64>", grid);
    go(filt<3, 64>, "loads+nl<64>", grid);
    go(filt<0, 128>, "full<128>", grid);
  }
  return 0;
}
