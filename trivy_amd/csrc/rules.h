// Rule compiler: secret rules -> GPU tables.
//
// Hooks where the reference assembles its rule list (NewScanner,
// pkg/fanal/secret/scanner.go:320-364).  For the ordered rule list it builds
//   * the keyword gate: unique strings.ToLower(keyword)s (scanner.go:174-186)
//     and, per rule, the keyword ids whose presence enables it;
//   * one anchor per rule: a set of ASCII literals every match contains, at a
//     bounded byte offset [off_lo, off_hi] from the match start;
//   * the streaming prefilter's items (byte-set sequences around each anchor
//     literal, keywords that need GPU bits, the fold runes U+0130 / U+212A /
//     U+017F), bucketed into shift-or tables by filter.cpp;
//   * a relaxed, byte-level "extended shift-and" NFA per rule whose language is
//     a superset of the rule regex (captures dropped, assertions -> ε,
//     alternations -> column unions / class runs, large repeats -> unbounded).
#pragma once
#include <cstdint>
#include <bitset>
#include <memory>
#include <string>
#include <vector>

#include "goregex.h"

namespace tsg {

constexpr int kMaxNfaWords = 4;

enum GateMode : uint8_t {
  kGateAlways = 0,    // no keywords: MatchKeywords is true
  kGateKeywords = 1,  // ASCII keywords: GPU bitset is exact
  kGateHost = 2,      // a non-ASCII keyword: GPU treats as open, host verifies
};

// Gate redundancy: a keyword every regex match contains (ASCII case-folded,
// and not through a (?i) 's' that U+017F could satisfy) makes MatchKeywords
// unable to change Scan's result -- see DESIGN.md §2.1.
bool KeywordImplied(const Regex& re, const std::string& kw_lower);
bool KeywordsImplied(const Regex& re, const std::vector<std::string>& kws_lower, bool long_s_ok);

struct RuleSrc {
  std::string id;
  std::string regex;
  std::vector<std::string> keywords;
  bool has_regex = true;  // false: Rule.Regex == nil (never matches); "" is a regex
};

struct AnchorInfo {  // mirrored on the device
  uint32_t rule;
  uint32_t lit_len;
  int32_t off_lo, off_hi;  // literal start - match start, in bytes (non-special files)
  int32_t off_hi_fold;     // the same when U+212A/U+017F/U+0130 may occur (special files)
};

// Follow requirements of an anchor (mirrored on the device): in ASCII text,
// every match continues after the anchor literal with req r's run of n[r]
// consecutive byte sets starting at a byte offset in [lo[r], hi[r]] from the
// literal end (one relaxed-NFA position per ASCII byte).  A hit whose bytes
// up to the last possible run end are ASCII and hold no such run cannot be a
// match; any byte >= 0x80 in that range leaves the hit to the NFA.  Sets are
// kept as nibble tables (slot 4r + k: run r, position k): byte b is in slot
// s's set when bit s of lo_tab[b & 15] & hi_tab[b >> 4] is set -- the
// product of the set's low- and high-nibble projections, a superset of it.
constexpr int kMaxReqs = 2, kMaxReqLen = 4, kReqSpan = 48;  // hi + n <= kReqSpan
struct FollowLut {
  uint8_t lo_tab[16];
  uint8_t hi_tab[8];       // ASCII high nibbles 0..7
  uint8_t lo[kMaxReqs], hi[kMaxReqs];
  uint8_t n[kMaxReqs];     // 0: no requirement
  uint8_t pad[2];
};
static_assert(sizeof(FollowLut) == 32, "FollowLut layout (tests/filter_model.py reads it)");

struct RuleGpu {  // mirrored on the device
  uint32_t nfa_off;     // index into nfa words (u64)
  uint8_t nfa_words;    // 0: relaxed NFA is empty -> every anchor hit is a candidate
  uint8_t gate;         // GateMode
  uint8_t anchored;     // 1: anchor-driven; 0: full-scan rule
  uint8_t has_regex;
  uint32_t kw_off, kw_cnt;  // into rule_kw
  uint32_t kw_match_implied;  // every match holds a keyword unless the file has U+017F (no GPU bits)
  // bounds of a match's length in bytes (max_len = kNoMaxLen: unbounded): a
  // full-scan accept after byte p puts the match start in [p+1-max, p+1-min]
  uint32_t min_len, max_len;
};
constexpr uint32_t kNoMaxLen = 0xFFFFFFFFu;

// Prefilter item: a fixed-width sequence of byte sets that
// every occurrence of a keyword (ASCII case-insensitive), an anchor literal
// (with the mandatory single-width classes right before and after it) or a
// fold rune (C4 B0 / E2 84 AA / C5 BF) matches byte for byte in files without
// fold runes.  The streaming filter runs bucketed shift-or over windows of
// these sequences; the confirm pass checks every position exactly.
using ByteSet = std::bitset<256>;
enum ItemKind : uint8_t { kItemKeyword = 0, kItemAnchor = 1, kItemFold = 2 };
struct FilterItem {
  uint8_t kind;
  uint32_t id;       // keyword id / anchor id / fold rune (0 U+0130, 1 U+212A, 2 U+017F)
  uint32_t lit_end;  // anchors: positions from the item start to the literal end
  std::vector<ByteSet> sets;
  // clustering group: items share buckets only within their group (1: anchors
  // a calibration sample chose, whose windows the static prior misprices)
  uint8_t group = 0;
};

struct CompiledRules {
  // keywords / anchors
  std::vector<std::string> keywords;  // unique lowercased ASCII keywords
  std::vector<AnchorInfo> anchors;
  std::vector<FollowLut> anchor_req;  // per anchor
  // rules
  std::vector<RuleGpu> rules;
  std::vector<uint32_t> rule_kw;  // keyword ids
  std::vector<uint64_t> nfa;      // per rule: O[W] L[W] F[W] B[256][W]
  std::vector<std::string> rule_anchor_desc;  // debug text
  std::vector<FilterItem> items;  // prefilter items (keywords, anchors, fold runes)
  std::shared_ptr<const struct FilterTables> filter;  // built from items (filter.h)
  std::vector<std::unique_ptr<Regex>> regex;  // exact engines (host pass)
  uint32_t n_fullscan_rules = 0;
  uint32_t n_redundant_gates = 0;
  uint32_t n_calibrated_anchors = 0;  // class-run anchors a calibration sample chose over a literal

  uint32_t kw_words() const { return (uint32_t(keywords.size()) + 31) / 32; }
};

// A set of lowercased ASCII literals (len >= 2) one of which every match of
// `re` contains, or empty if none is known.  Used as a MatchString prefilter.
std::vector<std::string> RequiredLiterals(const Regex& re);

// Optional inputs of the compiler.  calib: a sample of the bytes the scanner
// will see (e.g. its first batch).  With one, a rule that has both a literal
// anchor and a class-run anchor takes the one whose prefilter item fires less
// on the sample (K1 window fires + K2 item matches), instead of the static
// byte prior's choice -- the prior cannot know that a dictionary word such as
// `linear` (builtin-rules.go:623) is common in source trees.
struct CompileOptions {
  const uint8_t* calib = nullptr;
  uint64_t calib_n = 0;
};

// Compile; returns false with *err on a regex/limits error.
bool CompileRules(const std::vector<RuleSrc>& src, CompiledRules* out, std::string* err,
                  const CompileOptions* opt = nullptr);

}  // namespace tsg
