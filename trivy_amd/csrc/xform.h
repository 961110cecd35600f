// GPU pre-transform of host batches (xform.hip): CR strip / printable
// extraction on the bytes as read, and the gather of chosen transformed files
// for the host's exact pass.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tsg {

constexpr uint8_t kXformNone = 0, kXformStripCR = 1, kXformPrintable = 2;

// len[f] = transformed length of file f (len[n_files] = 0); raw has 16 readable bytes past off[n_files].
hipError_t XformLengths(const uint8_t* raw, const uint64_t* off, const uint8_t* kind, uint32_t n_files, uint64_t* len,
                        hipStream_t s);
// xoff = exclusive prefix sums of len (n_files + 1 entries)
hipError_t XformScanBytes(uint32_t n_files, size_t* bytes);
hipError_t XformScan(void* temp, size_t temp_bytes, const uint64_t* len, uint64_t* xoff, uint32_t n_files,
                     hipStream_t s);
// out[xoff[f] ..) = transform(kind[f], raw[off[f] .. off[f+1]))
hipError_t XformCopy(const uint8_t* raw, const uint64_t* off, const uint8_t* kind, uint32_t n_files,
                     const uint64_t* xoff, uint8_t* out, hipStream_t s);
// dst[dst_off[i] ..) = src[xoff[files[i]] .. xoff[files[i] + 1])
hipError_t GatherFiles(const uint8_t* src, const uint64_t* xoff, const uint32_t* files, const uint64_t* dst_off,
                       uint32_t n, uint8_t* dst, hipStream_t s);

}  // namespace tsg
