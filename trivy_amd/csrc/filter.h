// Streaming prefilter tables: bucketed shift-or over windows
// of the rule compiler's FilterItems.
//
// Each item is reduced to a window of at most kSlots consecutive byte sets
// (the least frequent one under a static byte-frequency prior); windows are
// clustered into n_buckets buckets (agglomerative, minimising the estimated
// false-positive rate Σ_bucket Π_slot P(union of the slot's sets)).  The
// device reach table holds, per input byte, one bit per (slot, bucket): 0 when
// the byte is allowed at that slot of that bucket.  State after byte t:
//   S_t = (S_{t-1} << 8) | reach[b_t]      (8 buckets: u64; 16: two u64)
// and bucket j fires at t when bit (8*7 + j) of S_t is 0.  The confirm pass
// then checks each of the bucket's items exactly at every position.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "rules.h"

namespace tsg {

constexpr int kFilterSlots = 8;  // maximum window length

struct FilterItemGpu {  // mirrored on the device (16 B)
  uint16_t n;        // positions (byte sets) of the item
  uint16_t back;     // item start = window-end byte + 1 - back
  uint16_t lit_end;  // anchors: literal end = item start + lit_end
  uint8_t kind;      // ItemKind
  uint8_t n_ids;     // ids of the FilterItems with this exact byte-set sequence
  uint32_t ids_off;  // into item_ids
  uint32_t cls_off;  // index of the item's first class id in item_cls
};

struct FilterTables {
  uint32_t n_buckets = 0;                // buckets
  uint32_t n_slots = 0;                  // slots per register (4 or 8)
  uint32_t window = 0;                   // window length L <= n_slots: items end at slot L-1; a fire
                                         // stays visible in slots L-1..n_slots-1, so the top slots
                                         // need checking only every n_slots - L + 1 bytes
  uint32_t n_words = 0;                  // 64-bit state registers: n_slots * n_buckets / 64
  // reach[b * n_words + w]: register w holds buckets [w*bpw, (w+1)*bpw), bpw = 64 / n_slots,
  // bit s * bpw + (j % bpw) is 0 when byte b is allowed at slot s of bucket j
  std::vector<uint64_t> reach;
  std::vector<uint32_t> bucket_off;      // n_buckets + 1 into bucket_items
  std::vector<uint32_t> bucket_items;    // item indices
  std::vector<FilterItemGpu> items;
  std::vector<uint32_t> item_ids;        // anchor / fold ids per item
  std::vector<uint8_t> item_cls;         // class id per item position (< 256)
  std::vector<uint32_t> classes;         // 8 x u32 membership words per class
  uint32_t max_after = 0;                // max positions an item extends past its window end
  double est_fp = 0;                     // estimated bucket fires per input byte
};

// Static byte-frequency prior of source/text bytes (sums to 1).
const std::vector<double>& BytePrior();

bool BuildFilter(const std::vector<FilterItem>& items, uint32_t n_slots, uint32_t window, uint32_t n_buckets,
                 FilterTables* out, std::string* err);

}  // namespace tsg
