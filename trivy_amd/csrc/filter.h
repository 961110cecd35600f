// Streaming prefilter tables: bucketed shift-or over windows
// of the rule compiler's FilterItems.
//
// Each item is reduced to a window of at most `window` consecutive byte sets
// (the least frequent one under a static byte-frequency prior); windows are
// clustered into the item buckets (agglomerative, minimising the estimated
// false-positive rate Σ_bucket Π_slot P(union of the slot's sets)).
//
// State layout: n_words u32 registers of 8 slots x 4 buckets; bucket j lives
// in register j / 4, slot s at bit 4*s + j % 4.  Per input byte b
//   R_w = (R_w << 4) | reach[b][w]          (one v_lshl_or_b32 per register)
// where a reach bit is 0 when b is allowed at that (slot, bucket).  Items end
// at slot window-1; slots past it are all-allowed, so a fire stays visible in
// slots window-1 .. 7 for 9 - window bytes and the top slots need checking
// only that often.  The last bucket counts '\n': its slot 0 allows only '\n',
// slots 1-3 carry and slots 4-7 allow nothing (it never fires), so after every
// 4th byte its slots 0-3 hold the last 4 bytes' newline bits.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "rules.h"

namespace tsg {

constexpr int kFilterSlots = 8;  // slots per register (4 bits each)

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
  uint32_t n_buckets = 0;                // buckets, including the newline bucket
  uint32_t n_words = 0;                  // u32 state registers = n_buckets / 4
  uint32_t window = 0;                   // window length (<= 8)
  uint32_t nl_bucket = 0;                // the newline-counting bucket (n_buckets - 1)
  std::vector<uint32_t> reach;           // reach[b * n_words + w]
  std::vector<uint32_t> bucket_off;      // n_buckets + 1 into bucket_items
  std::vector<uint32_t> bucket_items;    // item indices
  std::vector<FilterItemGpu> items;
  std::vector<uint32_t> item_ids;        // anchor / fold ids per item
  std::vector<uint8_t> item_cls;         // class id per item position (< 256)
  std::vector<uint32_t> classes;         // 8 x u32 membership words per class
  // Core tables for the confirm step: a bucket's items in groups of 8; per
  // group and byte b, bit 8*s + i of core[g * 256 + b] is 1 when b may stand at
  // core slot s of the group's item i -- the item positions back-8 .. back-1,
  // i.e. the 8 bytes ending at the window end (slots before the item start
  // allow every byte).  One AND over 8 independent lookups gives the items
  // whose core matches at a fire.
  std::vector<uint64_t> core;            // n_groups x 256
  std::vector<uint32_t> group_items;     // n_groups x 8 item indices (0xFFFFFFFF: none)
  std::vector<uint32_t> bucket_groups;   // n_buckets + 1 into the groups
  // Literal windows are confirmed by hashing instead: an item whose 6 window
  // sets are single ASCII characters (either case) is keyed by its window
  // lowercased (byte q at bits 8q, the window end in byte 5) in an
  // open-addressed table of 2^hash_bits slots (key | 1 << 63; 0 = empty); the
  // core groups hold the other items only.  One probe per fire replaces the
  // group scans of large literal sets.
  std::vector<uint64_t> hash_keys;
  std::vector<uint32_t> hash_items;
  uint32_t hash_bits = 0;
  uint32_t hash_buckets = 0;             // buckets holding hashed items
  uint32_t max_after = 0;                // max positions an item extends past its window end
  double est_fp = 0;                     // estimated bucket fires per input byte

};

// Key hash of the literal-window table, shared by the host build (g++) and the
// confirm kernel (hipcc compiles it for both sides).
#if defined(__HIPCC__)
#define TSG_HOST_DEVICE __host__ __device__
#else
#define TSG_HOST_DEVICE
#endif
TSG_HOST_DEVICE inline uint32_t WindowHash(uint64_t key, uint32_t bits) {
  return uint32_t((key * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}

// Static byte-frequency prior of source/text bytes (sums to 1).
const std::vector<double>& BytePrior();

// prior: byte frequencies to use instead of BytePrior() (a calibration sample's, CompileOptions)
bool BuildFilter(const std::vector<FilterItem>& items, uint32_t window, uint32_t n_buckets, FilterTables* out,
                 std::string* err, const std::vector<double>* prior = nullptr);

// The window BuildFilter keeps of an item: its least likely `window` (or fewer)
// consecutive positions under the prior, [*start, *start + *len).
void ItemWindow(const FilterItem& it, uint32_t window, size_t* start, size_t* len,
                const std::vector<double>* prior = nullptr);

}  // namespace tsg
