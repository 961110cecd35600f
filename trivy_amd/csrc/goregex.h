// Go 1.22 regexp semantics for the secret scanner's exact host pass.
//
// Re-implements what pkg/fanal/secret/scanner.go relies on from Go's
// regexp/regexp/syntax (the Perl flag set of regexp.Compile): parsing with
// scoped (?imsU) flags, simplification of counted repeats, the Thompson
// program layout (Alt priorities, (x+)? for nullable stars) and the
// leftmost-first Pike VM with submatches over UTF-8 runes (invalid byte ->
// U+FFFD width 1), and the bit-state backtracker Go uses on small inputs
// (regexp/backtrack.go; same leftmost-first result).  FindAll follows
// (*Regexp).allMatches (empty-match rules).
//
// Extension for the GPU pipeline: FindAll can be restricted to a sorted list
// of start windows (the GPU's candidate windows).  A thread is only started at
// a rune boundary inside a window; positions outside every window are jumped
// over.  Because every true match start lies in some window,
// the result equals the unrestricted search.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace tsg {

using RuneRanges = std::vector<std::pair<uint32_t, uint32_t>>;

enum EmptyOp : uint8_t {
  kEmptyBeginLine = 1,
  kEmptyEndLine = 2,
  kEmptyBeginText = 4,
  kEmptyEndText = 8,
  kEmptyWordBoundary = 16,
  kEmptyNoWordBoundary = 32,
};

enum class NodeOp : uint8_t { Empty, NoMatch, Class, Assert, Cat, Alt, Capture, Repeat };

struct Node {
  NodeOp op = NodeOp::Empty;
  uint8_t assert_op = 0;
  bool greedy = true;
  int cap = -1;
  int min = 0, max = 0;  // Repeat; max = -1 means unbounded
  RuneRanges ranges;     // Class (sorted, merged)
  std::vector<int> subs; // indices into Regex::nodes
};

struct Window {  // inclusive byte range of allowed match starts
  int64_t lo, hi;
};

enum InstOp : uint8_t { kIFail, kIAlt, kICapture, kIEmpty, kIMatch, kINop, kIRune, kIRune1, kIAny, kIAnyNotNL };

struct Inst {
  InstOp op = kIFail;
  uint8_t empty = 0;
  uint32_t out = 0, arg = 0;
  int cls = -1;      // kIRune: index into Regex::classes
  uint32_t rune = 0; // kIRune1
};

// UTF-8 decode with Go's utf8.DecodeRune contract.
struct Rune {
  int32_t r;   // -1 at end of text
  int width;
};
Rune DecodeRune(const uint8_t* s, int64_t n, int64_t pos);

class Regex {
 public:
  static std::unique_ptr<Regex> Compile(const std::string& pattern, std::string* err);

  const std::string& pattern() const { return pattern_; }
  int num_cap() const { return num_cap_; }
  const std::vector<std::string>& cap_names() const { return cap_names_; }
  const std::vector<Node>& nodes() const { return nodes_; }
  int root() const { return root_; }

  // regexp.MatchString / Match: any match anywhere.
  bool Match(const uint8_t* s, int64_t n) const;
  // FindAll[Submatch]Index(b, -1).  Appends (num_cap+1)*2 offsets per match
  // (or 2 when !submatch).  `wins` (sorted, merged) restricts match starts.
  void FindAll(const uint8_t* s, int64_t n, bool submatch, const std::vector<Window>* wins,
               std::vector<int64_t>* out) const;

 private:
  friend class Parser;
  friend class Compiler;
  friend class Machine;
  friend class Backtracker;
  bool RuneMatch(const Inst& in, int32_t c) const;
  std::string pattern_;
  std::vector<Node> nodes_;
  int root_ = -1;
  int num_cap_ = 0;
  std::vector<std::string> cap_names_;
  std::vector<Inst> prog_;
  std::vector<RuneRanges> classes_;
  std::vector<std::pair<uint64_t, uint64_t>> class_ascii_;  // ASCII membership bitmap per class
  uint32_t start_ = 0;
  bool anchored_begin_ = false;  // program begins with \A (startCond has EmptyBeginText)
  // Bytes that can begin a match (the first byte of its first rune), from the
  // program's start closure; first_all_ when a match can be empty or start
  // with any byte.  Starts at other bytes are skipped (an exact pruning).
  std::vector<uint8_t> single_pred_;  // pc entered only from one rune instruction (no visited bit needed)
  uint64_t first_[4] = {};
  bool first_all_ = true;
  // A regex that is one greedy repeat of one single-rune class, C{m,n} / C{m,}
  // with m >= 1, possibly inside capture groups (custom rules such as
  // (?i)[a-z0-9/+]{32,48}): FindAll is then a scan over class runs (FindAllRun).
  bool run_ok_ = false;
  int run_min_ = 0, run_max_ = 0;  // run_max_ < 0: unbounded
  RuneRanges run_cls_;
  uint64_t run_ascii_[2] = {};
  uint8_t run_tbl_[256] = {};  // per byte: 1 an ASCII class member, 0 an ASCII non-member, 2 a rune to decode
  void DetectRun();
  // A regex that is a concatenation of classes of one or two ASCII runes each
  // (a literal, (?i) letters folding only to their other case -- not k / s, whose
  // orbits hold U+212A / U+017F), possibly inside capture groups: Match is a
  // byte search (an ASCII class matches only the one-byte rune, never a byte
  // inside a multi-byte one).  The builtin allow rule `examples` ((?i)example)
  // runs on every match of the exact pass.
  bool lit_ok_ = false;
  std::vector<uint8_t> lit_a_, lit_b_;  // position k: byte lit_a_[k] or lit_b_[k]
  void DetectLiteral();
  bool MatchLiteral(const uint8_t* s, int64_t n) const;
  void FindAllRun(const uint8_t* s, int64_t n, bool submatch, const std::vector<Window>* wins,
                  std::vector<int64_t>* out) const;
  void ComputeFirstBytes();
  bool FirstOk(const uint8_t* s, int64_t n, int64_t pos) const {
    return first_all_ || (pos < n && ((first_[s[pos] >> 6] >> (s[pos] & 63)) & 1));
  }
};

// unicode.SimpleFold and unicode.ToLower (generated tables, Unicode 13 data).
uint32_t SimpleFold(uint32_t r);
uint32_t GoToLower(uint32_t r);
// bytes.ToLower over a whole buffer (Go semantics, invalid byte -> EF BF BD).
std::string GoBytesToLower(const uint8_t* s, size_t n);
// unicode.IsPrint and strconv.Quote (fmt %q), scanner.go:442.
bool GoIsPrint(uint32_t r);
std::string GoQuote(const std::string& s);

}  // namespace tsg
