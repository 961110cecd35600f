// K1 design microbenchmark (not product code): the streaming filter's hot
// loop in isolation, in the product layout (16 buckets = four u32 shift-or
// registers of 8 slots x 4 buckets, LDS reach table replicated 16x, 64 B per
// lane per tile), with compile-time variants that change one ingredient at a
// time, to see what bounds the loop.
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

__device__ __forceinline__ uint4 rd(const uint8_t* sb, uint32_t w, uint32_t k, uint32_t laneoff) {
  return *reinterpret_cast<const uint4*>(sb + __builtin_amdgcn_perm(w, laneoff, 0x0C0C0000u | ((4u + k) << 8)));
}

template <bool ASM>
__device__ __forceinline__ void apply(const uint4& m, uint32_t* st) {
  if (ASM) {
    asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(st[0]) : "v"(st[0]), "v"(m.x));
    asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(st[1]) : "v"(st[1]), "v"(m.y));
    asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(st[2]) : "v"(st[2]), "v"(m.z));
    asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(st[3]) : "v"(st[3]), "v"(m.w));
  } else {
    st[0] = (st[0] << 4) | m.x;
    st[1] = (st[1] << 4) | m.y;
    st[2] = (st[2] << 4) | m.z;
    st[3] = (st[3] << 4) | m.w;
  }
}

// Variant flags
constexpr int kNoLds = 1;     // table word = data-derived value (no LDS reads)
constexpr int kNoChain = 2;   // LDS reads OR-reduced, no shift-or chain
constexpr int kNoNl = 4;      // skip the newline popcounts
constexpr int kAsm = 8;       // chain as inline asm
constexpr int kAhead = 16;    // read block j+1's table rows before block j's chain (8 at a time)
constexpr int kHalf = 32;     // reads in two halves of 8 per block (fewer live VGPRs)
constexpr int kLoadsOnly = 64;
constexpr int kStoreNl = 128;  // per-tile u16 newline-count store (as the product kernel did)

template <int V, int LB>
__global__ __launch_bounds__(1024) void filt(const uint8_t* __restrict__ a, uint64_t n, const uint32_t* __restrict__ tab,
                                             uint32_t* out, uint16_t* nlout) {
  __shared__ __attribute__((aligned(16))) uint8_t s_reach[65536];
  for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x)
    reinterpret_cast<uint4*>(s_reach)[i] = reinterpret_cast<const uint4*>(tab)[i / 16];
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
    load(nxt, t + n_waves < ntiles ? t + n_waves : t);
    if (!(V & kLoadsOnly)) {
      uint32_t p1 = __shfl(cur[NB - 1].w, int(lane) - 1);
      uint32_t st[4] = {~0u, ~0u, ~0u, ~0u};
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) apply<(V & kAsm) != 0>(rd(s_reach, p1, k, laneoff), st);
#pragma unroll
      for (int j = 0; j < NB; j++) {
        const uint32_t wd[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
        uint32_t acc = ~0u;
        if (V & kNoChain) {
#pragma unroll
          for (uint32_t k = 0; k < 16; k++) {
            uint4 m = rd(s_reach, wd[k >> 2], k & 3, laneoff);
            acc &= m.x | m.y | m.z | m.w;
          }
        } else if (V & kHalf) {
#pragma unroll
          for (uint32_t h = 0; h < 2; h++) {
            uint4 m[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; k++) {
              const uint32_t kk = 8 * h + k;
              if (V & kNoLds) {
                const uint32_t x = wd[kk >> 2] >> (8 * (kk & 3));
                m[k] = make_uint4(x, x ^ laneoff, x + 1, x ^ 0x55);
              } else {
                m[k] = rd(s_reach, wd[kk >> 2], kk & 3, laneoff);
              }
            }
#pragma unroll
            for (uint32_t k = 0; k < 8; k++) {
              const uint32_t kk = 8 * h + k;
              apply<(V & kAsm) != 0>(m[k], st);
              if (kk % 3 == 2 || kk == 15) acc &= st[0] & st[1] & st[2] & st[3];
              if (!(V & kNoNl) && kk % 4 == 3) nl += __popc(~st[3] & 0x8888u);
            }
          }
        } else {
          uint4 m[16];
#pragma unroll
          for (uint32_t k = 0; k < 16; k++) {
            if (V & kNoLds) {
              const uint32_t x = wd[k >> 2] >> (8 * (k & 3));
              m[k] = make_uint4(x, x ^ laneoff, x + 1, x ^ 0x55);
            } else {
              m[k] = rd(s_reach, wd[k >> 2], k & 3, laneoff);
            }
          }
#pragma unroll
          for (uint32_t k = 0; k < 16; k++) {
            apply<(V & kAsm) != 0>(m[k], st);
            if (k % 3 == 2 || k == 15) acc &= st[0] & st[1] & st[2] & st[3];
            if (!(V & kNoNl) && k % 4 == 3) nl += __popc(~st[3] & 0x8888u);
          }
        }
        flagged += (acc | 0x000FFFFFu) != ~0u;
      }
      if (V & kStoreNl) {
        uint32_t c = nl;
        for (int x = 1; x < 16; x <<= 1) c += __shfl_xor(c, x);
        if ((lane & 15) == 0) nlout[t * 4 + lane / 16] = uint16_t(c);
      }
    } else {
#pragma unroll
      for (int j = 0; j < NB; j++) flagged += (cur[j].x ^ cur[j].y ^ cur[j].z ^ cur[j].w) == 0x12345678u;
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
  uint32_t* tab;
  CK(hipMalloc(&d, n + 4096));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&tab, 256 * 16));
  uint16_t* nlout;
  CK(hipMalloc(&nlout, n / 1024 * 2 + 64));
  fill_kernel<<<4096, 256>>>(reinterpret_cast<uint4*>(d), n / 16);
  // 15 item buckets of 6-byte windows + the newline bucket, filter.h layout
  std::vector<uint32_t> h(256 * 4, ~0u);
  const char* pats[15] = {"ghp_ab", "akiaxy", "xoxb-1", "------", "dapi12", "sk_liv", "glpat-", "pypi-a",
                          "aws_se", "lin_ap", "facebo", "twitte", "discor", "mailgu", "hubspo"};
  for (int j = 0; j < 16; j++)
    for (int s = 0; s < 8; s++)
      for (int b = 0; b < 256; b++) {
        bool ok;
        if (j == 15) ok = s == 0 ? b == '\n' : s < 4;
        else ok = s >= 6 || b == pats[j][s] || b == (pats[j][s] ^ 0x20);
        if (ok) h[b * 4 + j / 4] &= ~(1u << (4 * s + (j % 4)));
      }
  CK(hipMemcpy(tab, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  auto go = [&](auto kern, const char* name, int grid) {
    CK(hipMemset(out, 0, 64));
    float ms = timeit([&] { kern<<<grid, 1024>>>(d, n, tab, out, nlout); }, 5);
    uint32_t o[3];
    CK(hipMemcpy(o, out, 12, hipMemcpyDeviceToHost));
    std::printf("%-28s g%-4d %8.3f ms  %7.3f TB/s  flagged/launch %.0f nl %.0f\n", name, grid, ms,
                n / (ms * 1e-3) / 1e12, o[1] / 6.0, o[2] / 6.0);
  };
  for (int grid : {256, 512}) {
    go(filt<kAsm | kStoreNl, 64>, "asm-store-nl<64>", grid);
    go(filt<kAsm | kStoreNl, 128>, "asm-store-nl<128>", grid);
    go(filt<0, 64>, "full<64>", grid);
    go(filt<kAsm, 64>, "full-asm<64>", grid);
    go(filt<kAsm | kHalf, 64>, "asm-half<64>", grid);
    go(filt<kAsm | kNoNl, 64>, "asm-no-nl<64>", grid);
    go(filt<kAsm | kNoLds, 64>, "asm-no-lds<64>", grid);
    go(filt<kNoChain, 64>, "lds-only<64>", grid);
    go(filt<kLoadsOnly, 64>, "loads-only<64>", grid);
    go(filt<kAsm, 32>, "full-asm<32>", grid);
    go(filt<kAsm | kHalf, 32>, "asm-half<32>", grid);
    go(filt<kAsm, 128>, "full-asm<128>", grid);
  }
  return 0;
}
