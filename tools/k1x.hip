// K1 design experiments (tuning aid, not product code): the streaming
// filter's inner loop in isolation with the compiled builtin reach table and
// the real C2 corpus, one compile-time ingredient changed per variant, to find
// what bounds K1 (engine.hip filter_kernel) on gfx950.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/k1x.so tools/k1x.hip
//   python tools/k1x.py   (drives it: corpus + tables + timing table)
//
// Template knobs:
//   NREG  shift-or registers (4: 16 buckets, ds_read_b128 table replicated 16x;
//         2: 8 buckets, ds_read_b64 table replicated 32x)
//   LB    bytes per lane per tile
//   GRP   table reads issued ahead of the chain (per stream)
//   MODE  0 full, 1 LDS reads only (no chain; every word XOR-ed so the reads stay
//         b128), 2 the full loop's VALU with the row = its v_perm address (no LDS;
//         round 6: before, a multiply per word inflated the VALU), 3 loads only, 4 full with a rolling ring of GRP table rows
//         (row k + GRP read as row k is applied: GRP reads in flight at every
//         step, no group-boundary drain), 5 = 4 with sched_group_barrier
//         pinning the order (1 ds_read after every row's 4 v_lshl_or)
//   STR   independent shift-or streams per lane (2: the lane's chunk halves,
//         the second warmed up on the 5 bytes before it)
//   MINW  workgroups of 1024 per CU (__launch_bounds__ min waves per SIMD / 4)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

namespace {

__device__ __forceinline__ uint4 load16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

__device__ __forceinline__ uint32_t wsel(const uint4* buf, int i) {
  const uint4 v = buf[i >> 2];
  return (i & 3) == 0 ? v.x : (i & 3) == 1 ? v.y : (i & 3) == 2 ? v.z : v.w;
}

template <int NREG>
struct Row {
  uint32_t w[NREG];
};

template <int NREG, int MODE>
__device__ __forceinline__ Row<NREG> rd(const uint8_t* sb, uint32_t word, uint32_t k, uint32_t laneoff) {
  Row<NREG> r;
  const uint32_t a = __builtin_amdgcn_perm(word, laneoff, 0x0C0C0000u | ((4u + k) << 8));
  if (MODE == 2 || MODE == 6) {  // the row = the address itself: the full loop's VALU, no LDS
#pragma unroll
    for (int i = 0; i < NREG; i++) r.w[i] = a;
    return r;
  }
  if (NREG == 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(sb + a);
    r.w[0] = v.x;
    r.w[1] = v.y;
    if (NREG > 2) {
      r.w[NREG > 2 ? 2 : 0] = v.z;
      r.w[NREG > 3 ? 3 : 0] = v.w;
    }
  } else {
    const uint2 v = *reinterpret_cast<const uint2*>(sb + a);
    r.w[0] = v.x;
    r.w[1] = v.y;
  }
  return r;
}

template <int NREG>
__device__ __forceinline__ void apply(const Row<NREG>& m, uint32_t* st) {
#pragma unroll
  for (int i = 0; i < NREG; i++) asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(st[i]) : "v"(st[i]), "v"(m.w[i]));
}

template <int NREG>
__device__ __forceinline__ uint32_t all_and(const uint32_t* st) {
  uint32_t a = st[0];
#pragma unroll
  for (int i = 1; i < NREG; i++) a &= st[i];
  return a;
}

constexpr uint32_t kFire = 0xFFF00000u;

template <int NREG, int LB, int GRP, int MODE, int STR, int MINW>
__global__ __launch_bounds__(1024, 4 * MINW) void k1x(const uint8_t* __restrict__ arena, uint64_t n,
                                                       const uint32_t* __restrict__ reach, uint32_t* out) {
  // 16 (NREG 4) or 32 (NREG 2) replicas of the 256-entry table, row stride 256 B
  __shared__ __attribute__((aligned(16))) uint8_t s_tab[65536];
  constexpr int REP = NREG == 4 ? 16 : 32;
  for (uint32_t i = threadIdx.x; i < 256 * REP; i += blockDim.x) {
    const uint32_t b = i / REP, r = i % REP;
    uint32_t* d = reinterpret_cast<uint32_t*>(s_tab + b * 256 + r * 4 * NREG);
    if (NREG == 4) {
#pragma unroll
      for (int w = 0; w < 4; w++) d[w] = reach[b * 4 + w];
    } else {
      d[0] = reach[b * 4 + 0];
      d[1] = reach[b * 4 + 3];  // keep the newline bucket (word 3, nibble lane 3)
    }
  }
  __syncthreads();
  constexpr int NB = LB / 16;
  constexpr uint64_t TILE = uint64_t(LB) * 64;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t laneoff = (lane & (REP - 1)) * (4 * NREG);
  const uint64_t wave = (blockIdx.x * uint64_t(blockDim.x) + threadIdx.x) >> 6;
  const uint64_t n_waves = (uint64_t(gridDim.x) * blockDim.x) >> 6;
  const uint64_t ntiles = n / TILE;
  uint32_t flagged = 0, nl = 0, sink = 0;
  uint4 A[NB], B[NB];
  uint2 pa = make_uint2(0, 0), pb = make_uint2(0, 0);
  auto load = [&](uint4* dst, uint2* pv, uint64_t tt) {
    const uint8_t* q = arena + tt * TILE + uint64_t(lane) * LB;
#pragma unroll
    for (int j = 0; j < NB; j++) dst[j] = load16(q + 16 * j);
    *pv = *reinterpret_cast<const uint2*>(arena + (tt > 0 ? tt * TILE - 8 : 0));
  };
  auto tile = [&](const uint4* cur, uint2 pre, uint64_t tt) {
    if (MODE == 3) {
#pragma unroll
      for (int j = 0; j < NB; j++) sink ^= cur[j].x ^ cur[j].y ^ cur[j].z ^ cur[j].w;
      return;
    }
    const uint32_t p1 = uint32_t(__builtin_amdgcn_update_dpp(int(tt > 0 ? pre.y : 0u), int(cur[NB - 1].w), 0x138,
                                                             0xF, 0xF, false));
    const uint32_t p0 = uint32_t(__builtin_amdgcn_update_dpp(int(tt > 0 ? pre.x : 0u), int(cur[NB - 1].z), 0x138,
                                                             0xF, 0xF, false));
    if (MODE == 1) {
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < 4 * NB; i++) {
        const uint32_t wd = wsel(cur, i);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
          Row<NREG> m = rd<NREG, 0>(s_tab, wd, k, laneoff);
#pragma unroll
          for (int w = 0; w < NREG; w++) x ^= m.w[w];  // every word: the whole ds_read_b128 stays
        }
      }
      sink ^= x ^ p0 ^ p1;
      return;
    }
    if (MODE == 4 || MODE == 5) {  // rolling ring (STR 1)
      uint32_t st[NREG];
#pragma unroll
      for (int i = 0; i < NREG; i++) st[i] = ~0u;
      apply<NREG>(rd<NREG, 0>(s_tab, p0, 3, laneoff), st);
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) apply<NREG>(rd<NREG, 0>(s_tab, p1, k, laneoff), st);
      Row<NREG> ring[GRP];
#pragma unroll
      for (int q = 0; q < GRP; q++) ring[q] = rd<NREG, 0>(s_tab, wsel(cur, q >> 2), q & 3, laneoff);
      uint32_t acc = ~0u;
#pragma unroll
      for (int k = 0; k < LB; k++) {
        apply<NREG>(ring[k % GRP], st);
        if (k + GRP < LB) ring[k % GRP] = rd<NREG, 0>(s_tab, wsel(cur, (k + GRP) >> 2), (k + GRP) & 3, laneoff);
        if (k % 3 == 2 || k % 16 == 15) acc &= all_and<NREG>(st);
        if (k % 4 == 3) nl += __popc(~st[NREG - 1] & 0x8888u);
        if (k % 16 == 15) {
          flagged += (acc | ~kFire) != ~0u;
          acc = ~0u;
        }
        if (MODE == 5) {
          __builtin_amdgcn_sched_group_barrier(0x0002, NREG + 2, 0);  // the row's VALU (+ perm / and)
          __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);         // then the next row's ds_read
        }
      }
      return;
    }
    constexpr int SL = LB / STR;  // bytes per stream
    uint32_t st[STR][NREG];
#pragma unroll
    for (int s = 0; s < STR; s++)
#pragma unroll
      for (int i = 0; i < NREG; i++) st[s][i] = ~0u ^ uint32_t(MODE == 2 ? i : 0);  // (MODE 2: distinct chains)
    // warm-up: 5 bytes before each stream
    {
      Row<NREG> m0 = rd<NREG, MODE>(s_tab, p0, 3, laneoff);
      apply<NREG>(m0, st[0]);
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) apply<NREG>(rd<NREG, MODE>(s_tab, p1, k, laneoff), st[0]);
#pragma unroll
      for (int s = 1; s < STR; s++) {
#pragma unroll
        for (int q = 0; q < 5; q++) {
          const int pos = s * SL - 5 + q;
          apply<NREG>(rd<NREG, MODE>(s_tab, wsel(cur, pos >> 2), pos & 3, laneoff), st[s]);
        }
      }
    }
    uint32_t acc[STR];
#pragma unroll
    for (int s = 0; s < STR; s++) acc[s] = ~0u;
#pragma unroll
    for (int g = 0; g < SL; g += GRP) {
      Row<NREG> m[STR][GRP];
#pragma unroll
      for (int q = 0; q < GRP; q++)
#pragma unroll
        for (int s = 0; s < STR; s++) {
          const int pos = s * SL + g + q;
          m[s][q] = rd<NREG, MODE>(s_tab, wsel(cur, pos >> 2), pos & 3, laneoff);
        }
#pragma unroll
      for (int q = 0; q < GRP; q++) {
#pragma unroll
        for (int s = 0; s < STR; s++) {
          apply<NREG>(m[s][q], st[s]);
          const int k = g + q;
          if (k % 3 == 2 || k % 16 == 15) acc[s] &= all_and<NREG>(st[s]);
          if (k % 4 == 3) nl += __popc(~st[s][NREG - 1] & 0x8888u);
          if (k % 16 == 15) {
            flagged += (acc[s] | ~kFire) != ~0u;
            acc[s] = ~0u;
          }
        }
      }
    }
  };
  uint64_t t = wave;
  if (t < ntiles) load(A, &pa, t);
  while (t < ntiles) {
    load(B, &pb, t + n_waves < ntiles ? t + n_waves : t);
    tile(A, pa, t);
    t += n_waves;
    if (t >= ntiles) break;
    load(A, &pa, t + n_waves < ntiles ? t + n_waves : t);
    tile(B, pb, t);
    t += n_waves;
  }
  atomicAdd(out + 1, flagged);
  atomicAdd(out + 2, nl);
  if (sink == 0x9E3779B9u) atomicAdd(out + 3, 1u);
}

struct Variant {
  const char* name;
  void (*launch)(int grid, hipStream_t s, const uint8_t*, uint64_t, const uint32_t*, uint32_t*);
};

template <int NREG, int LB, int GRP, int MODE, int STR, int MINW>
void launch_t(int grid, hipStream_t s, const uint8_t* a, uint64_t n, const uint32_t* r, uint32_t* o) {
  hipLaunchKernelGGL((k1x<NREG, LB, GRP, MODE, STR, MINW>), dim3(grid * MINW), dim3(1024), 0, s, a, n, r, o);
}

#define V(name, ...) {name, &launch_t<__VA_ARGS__>}
const Variant kVariants[] = {
    V("r4 lb64 g16 full s1", 4, 64, 16, 0, 1, 1),   // the product shape
    V("r4 lb64 g16 lds-only", 4, 64, 16, 1, 1, 1),
    V("r4 lb64 g16 no-lds", 4, 64, 16, 2, 1, 1),
    V("r4 lb64 loads-only", 4, 64, 16, 3, 1, 1),
    V("r4 lb64 g8 full s1", 4, 64, 8, 0, 1, 1),
    V("r4 lb64 g4 full s1", 4, 64, 4, 0, 1, 1),
    V("r4 lb64 g8 full s2", 4, 64, 8, 0, 2, 1),
    V("r4 lb64 g4 full s2", 4, 64, 4, 0, 2, 1),
    V("r4 lb128 g8 full s1", 4, 128, 8, 0, 1, 1),
    V("r4 lb128 g8 full s2", 4, 128, 8, 0, 2, 1),
    V("r4 lb128 g4 full s2", 4, 128, 4, 0, 2, 1),
    V("r4 lb32 g8 full s1", 4, 32, 8, 0, 1, 1),
    V("r2 lb64 g16 full s1", 2, 64, 16, 0, 1, 1),
    V("r2 lb64 g8 full s2", 2, 64, 8, 0, 2, 1),
    V("r2 lb128 g8 full s2", 2, 128, 8, 0, 2, 1),
    V("r2 lb64 g16 lds-only", 2, 64, 16, 1, 1, 1),
    V("r4 lb32 g4 full s1 2wg", 4, 32, 4, 0, 1, 2),
    V("r4 lb64 g4 full s1 2wg", 4, 64, 4, 0, 1, 2),
    V("r2 lb32 g4 full s1 2wg", 2, 32, 4, 0, 1, 2),
    V("r4 lb64 g16 full s1 2wg", 4, 64, 16, 0, 1, 2),
    V("r4 lb64 g8 full s1 2wg", 4, 64, 8, 0, 1, 2),
    V("r4 lb128 g8 full s1 2wg", 4, 128, 8, 0, 1, 2),
    V("r4 lb64 loads-only 2wg", 4, 64, 16, 3, 1, 2),
    V("r4 lb64 g16 lds-only 2wg", 4, 64, 16, 1, 1, 2),
    V("r4 lb64 g16 no-lds 2wg", 4, 64, 16, 2, 1, 2),
    V("r2 lb64 g16 full s1 2wg", 2, 64, 16, 0, 1, 2),
    // round 6: rolling ring of table rows instead of read groups
    V("r4 lb64 ring4 s1 2wg", 4, 64, 4, 4, 1, 2),
    V("r4 lb64 ring6 s1 2wg", 4, 64, 6, 4, 1, 2),
    V("r4 lb64 ring8 s1 2wg", 4, 64, 8, 4, 1, 2),
    V("r4 lb64 ring4 sgb s1 2wg", 4, 64, 4, 5, 1, 2),
    V("r4 lb64 ring6 sgb s1 2wg", 4, 64, 6, 5, 1, 2),
    V("r4 lb64 ring8 sgb s1 2wg", 4, 64, 8, 5, 1, 2),
    V("r4 lb64 ring4 s1", 4, 64, 4, 4, 1, 1),
    V("r4 lb64 ring8 s1", 4, 64, 8, 4, 1, 1),
    V("r4 lb64 ring8 sgb s1", 4, 64, 8, 5, 1, 1),
    V("r4 lb64 ring12 sgb s1", 4, 64, 12, 5, 1, 1),
    V("r4 lb64 g8 lds-only 2wg", 4, 64, 8, 1, 1, 2),
    V("r4 lb64 g8 no-lds 2wg", 4, 64, 8, 2, 1, 2),
};
#undef V

}  // namespace

extern "C" {

int k1x_count() { return int(sizeof(kVariants) / sizeof(kVariants[0])); }
const char* k1x_name(int v) { return kVariants[v].name; }

// Times `reps` launches of variant v after one warm-up; out[1] flagged blocks,
// out[2] newlines of the last launch.  Returns 0 or a HIP error code.
int k1x_run(int v, const uint8_t* arena, uint64_t n, const uint32_t* reach, uint32_t* out, int grid, int reps,
            float* ms) {
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 1;
  kVariants[v].launch(grid, 0, arena, n, reach, out);
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return int(e);
  hipEventRecord(a, 0);
  for (int i = 0; i < reps; i++) kVariants[v].launch(grid, 0, arena, n, reach, out);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  hipEventElapsedTime(ms, a, b);
  *ms /= reps;
  hipMemsetAsync(out, 0, 16, 0);
  kVariants[v].launch(grid, 0, arena, n, reach, out);
  e = hipDeviceSynchronize();
  hipEventDestroy(a);
  hipEventDestroy(b);
  return int(e);
}
}
