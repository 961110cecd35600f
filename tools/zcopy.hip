// Zero-copy read probe (tuning aid, not product code): how fast a kernel reads
// page-locked host memory over PCIe (hipHostRegisterMapped + device pointer),
// against hipMemcpyAsync of the same bytes -- the question behind a C4 gather
// of tar-layer file data straight from the registered layer buffer.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/zcopy.so tools/zcopy.hip
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

// each lane copies 16 B per step; `unroll` independent steps per lane per iteration
template <int U>
__global__ __launch_bounds__(256) void zread(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16,
                                             uint32_t off_bytes) {
  const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  const uint8_t* s8 = reinterpret_cast<const uint8_t*>(src) + off_bytes;  // misaligned source (gather-like)
  for (uint64_t i = tid; i < n16; i += stride * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = i + stride * u;
      if (j < n16) {
        if (off_bytes) {
          const uint32_t* p = reinterpret_cast<const uint32_t*>(s8 + 16 * j);  // 4-B aligned when off % 4 == 0
          v[u] = make_uint4(p[0], p[1], p[2], p[3]);
        } else {
          v[u] = src[j];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = i + stride * u;
      if (j < n16) dst[j] = v[u];
    }
  }
}

}  // namespace

extern "C" {

// mode 0: hipMemcpyAsync; 1..: zread with unroll 1/4/8 (mode 1/2/3), off = source misalignment
int zcopy_run(void* host, uint64_t n, int mode, int grid, uint32_t off, int reps, float* ms, float* gbps) {
  void* dhost = nullptr;
  void* dev = nullptr;
  if (hipHostRegister(host, n + 64, hipHostRegisterMapped) != hipSuccess) return 1;
  if (hipHostGetDevicePointer(&dhost, host, 0) != hipSuccess) return 2;
  if (hipMalloc(&dev, n + 64) != hipSuccess) return 3;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const uint64_t n16 = n / 16;
  auto launch = [&]() {
    if (mode == 0) {
      (void)hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, 0);
    } else if (mode == 1) {
      zread<1><<<grid, 256>>>(static_cast<const uint4*>(dhost), static_cast<uint4*>(dev), n16, off);
    } else if (mode == 2) {
      zread<4><<<grid, 256>>>(static_cast<const uint4*>(dhost), static_cast<uint4*>(dev), n16, off);
    } else {
      zread<8><<<grid, 256>>>(static_cast<const uint4*>(dhost), static_cast<uint4*>(dev), n16, off);
    }
  };
  launch();
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) {
    hipEventRecord(a, 0);
    for (int r = 0; r < reps; r++) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    hipEventElapsedTime(ms, a, b);
    *ms /= reps;
    *gbps = float(double(n) / (*ms * 1e-3) / 1e9);
    e = hipDeviceSynchronize();
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipFree(dev);
  hipHostUnregister(host);
  return e == hipSuccess ? 0 : 10 + int(e);
}
}
