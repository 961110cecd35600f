// GPU pre-transform of host batches (xform.hip): CR strip / printable
// extraction on the bytes as read, and the gather of chosen transformed files
// for the host's exact pass.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tsg {

constexpr uint8_t kXformNone = 0, kXformStripCR = 1, kXformPrintable = 2;

// Flat transform of a batch (n_files + 1 offsets into raw; raw has 64
// readable bytes past n_bytes).  XformPlan writes xoff (n_files + 1 entries:
// the transformed offsets) using `scratch` (XformScratchBytes); XformWrite,
// with the same scratch, writes out[xoff[f] ..) = transform(kind[f], file f)
// and never at or past out_cap (out holds out_cap bytes): a tile whose output
// would is skipped and flagged in the scratch's error word (XformErrorWord,
// nonzero = the call failed; read after the stream's work).  XformWrite also
// zeroes the 64 bytes after the output (out_cap >= xoff[n_files] + 64).
size_t XformScratchBytes(uint64_t n_bytes, uint32_t n_files);
hipError_t XformPlan(const uint8_t* raw, uint64_t n_bytes, const uint64_t* off, const uint8_t* kind, uint32_t n_files,
                     void* scratch, uint64_t* xoff, hipStream_t s);
hipError_t XformWrite(const uint8_t* raw, uint64_t n_bytes, const uint64_t* off, const uint8_t* kind, uint32_t n_files,
                      const void* scratch, uint8_t* out, uint64_t out_cap, hipStream_t s);
// One pass (TSG_XFORM_ONEPASS=1; off by default, slower: xform.hip): XformOnePass
// writes xoff and out together (a decoupled look-back over the tiles' output
// lengths).  out_cap must hold the bound XformMaxOut -- the offsets are known
// only when the call's work is done.
bool XformOnePassOn();
hipError_t XformOnePass(const uint8_t* raw, uint64_t n_bytes, const uint64_t* off, const uint8_t* kind,
                        uint32_t n_files, void* scratch, uint64_t* xoff, uint8_t* out, uint64_t out_cap,
                        hipStream_t s);
uint32_t XformErrorWord(uint64_t n_bytes, uint32_t n_files, const void* scratch, hipStream_t s);
// The error word's device address (read it with the stream's other results).
const uint32_t* XformErrorPtr(uint64_t n_bytes, uint32_t n_files, const void* scratch);
// Upper bound of a batch's transformed size: the strip only drops bytes, the
// printable extraction replaces a byte by '\n' where it closes a run and adds one
// '\n' per file at most (a run reaching the file's end).
inline uint64_t XformMaxOut(uint64_t n_bytes, uint32_t n_files) { return n_bytes + n_files; }
// dst[dst_off[i] ..) = src[xoff[files[i]] .. xoff[files[i] + 1])
hipError_t GatherFiles(const uint8_t* src, const uint64_t* xoff, const uint32_t* files, const uint64_t* dst_off,
                       uint32_t n, uint8_t* dst, hipStream_t s);

// Gather of a host batch's files straight from page-locked, device-mapped host
// memory (a registered tar layer: each file's data where the tar holds it) into
// a staging arena: dst[dst_off[f] .. dst_off[f + 1]) = src[src_off[f] ..).  One
// wave per item of up to kGatherPiece bytes of one file (items: (file, piece),
// built by the host); 16-B aligned destination stores (byte stores at a file's
// two ragged ends), source words by aligned loads and a byte shift.  The reads
// may touch up to 16 bytes before a file's data and 32 past its end, which a tar
// holds (the 512-B header before, the 512-B block padding and the end-of-archive
// blocks after).
constexpr uint32_t kGatherPiece = 16384;
struct GatherItem {
  uint32_t file, piece;
};
hipError_t GatherHostFiles(const uint8_t* src_dev, const uint64_t* src_off, const uint64_t* dst_off,
                           const GatherItem* items, uint32_t n_items, uint8_t* dst, hipStream_t s);

}  // namespace tsg
