// Go regexp semantics (see goregex.h).  Cited Go behaviour: regexp/syntax
// parse.go (flags, escapes, classes, repeat limits), simplify.go (counted
// repeats), compile.go (Alt priorities, loop/quest/star), regexp/exec.go
// (Pike VM: add/step/match), regexp/regexp.go allMatches (FindAll loop).
#include "goregex.h"

#include <algorithm>
#include <atomic>
#include <cstring>

namespace tsg {

#include "unicode_tables.inc"

namespace {
constexpr uint32_t kMaxRune = 0x10FFFF;
constexpr int kMaxRepeat = 1000;

void Clean(RuneRanges* r) {
  std::sort(r->begin(), r->end());
  RuneRanges out;
  for (auto& p : *r) {
    if (!out.empty() && p.first <= out.back().second + 1) {
      if (p.second > out.back().second) out.back().second = p.second;
    } else {
      out.push_back(p);
    }
  }
  r->swap(out);
}

RuneRanges Negate(const RuneRanges& in) {
  RuneRanges r = in;
  Clean(&r);
  RuneRanges out;
  uint32_t next = 0;
  for (auto& p : r) {
    if (p.first > next) out.push_back({next, p.first - 1});
    next = p.second + 1;
  }
  if (next <= kMaxRune) out.push_back({next, kMaxRune});
  return out;
}

bool InRanges(const RuneRanges& r, uint32_t c) {
  // binary search over sorted disjoint ranges
  size_t lo = 0, hi = r.size();
  while (lo < hi) {
    size_t m = (lo + hi) / 2;
    if (c < r[m].first) hi = m;
    else if (c > r[m].second) lo = m + 1;
    else return true;
  }
  return false;
}

bool IsWordChar(int32_t r) {
  return (r >= '0' && r <= '9') || (r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z') || r == '_';
}

uint8_t EmptyOpContext(int32_t r1, int32_t r2) {  // regexp/syntax.EmptyOpContext
  uint8_t op = kEmptyNoWordBoundary;
  int boundary = 0;
  if (IsWordChar(r1)) boundary = 1;
  else if (r1 == '\n') op |= kEmptyBeginLine;
  else if (r1 < 0) op |= kEmptyBeginText | kEmptyBeginLine;
  if (IsWordChar(r2)) boundary ^= 1;
  else if (r2 == '\n') op |= kEmptyEndLine;
  else if (r2 < 0) op |= kEmptyEndText | kEmptyEndLine;
  if (boundary) op ^= (kEmptyWordBoundary | kEmptyNoWordBoundary);
  return op;
}
}  // namespace

uint32_t SimpleFold(uint32_t r) {
  size_t n = sizeof(kFoldNext) / sizeof(kFoldNext[0]);
  size_t lo = 0, hi = n;
  while (lo < hi) {
    size_t m = (lo + hi) / 2;
    if (kFoldNext[m][0] < r) lo = m + 1;
    else hi = m;
  }
  if (lo < n && kFoldNext[lo][0] == r) return kFoldNext[lo][1];
  return r;
}

uint32_t GoToLower(uint32_t r) {
  if (r < 0x80) return (r >= 'A' && r <= 'Z') ? r + 32 : r;
  size_t n = sizeof(kLower) / sizeof(kLower[0]);
  size_t lo = 0, hi = n;
  while (lo < hi) {
    size_t m = (lo + hi) / 2;
    if (kLower[m][0] < r) lo = m + 1;
    else hi = m;
  }
  if (lo < n && kLower[lo][0] == r) return kLower[lo][1];
  return r;
}

Rune DecodeRune(const uint8_t* s, int64_t n, int64_t pos) {
  if (pos >= n) return {-1, 0};
  uint8_t b0 = s[pos];
  if (b0 < 0x80) return {b0, 1};
  auto cont = [&](int64_t i, uint8_t lo = 0x80, uint8_t hi = 0xBF) {
    return i < n && s[i] >= lo && s[i] <= hi;
  };
  if (b0 >= 0xC2 && b0 <= 0xDF) {
    if (cont(pos + 1)) return {int32_t(((b0 & 0x1F) << 6) | (s[pos + 1] & 0x3F)), 2};
    return {0xFFFD, 1};
  }
  if (b0 >= 0xE0 && b0 <= 0xEF) {
    uint8_t lo = 0x80, hi = 0xBF;
    if (b0 == 0xE0) lo = 0xA0;
    if (b0 == 0xED) hi = 0x9F;
    if (cont(pos + 1, lo, hi) && cont(pos + 2))
      return {int32_t(((b0 & 0x0F) << 12) | ((s[pos + 1] & 0x3F) << 6) | (s[pos + 2] & 0x3F)), 3};
    return {0xFFFD, 1};
  }
  if (b0 >= 0xF0 && b0 <= 0xF4) {
    uint8_t lo = 0x80, hi = 0xBF;
    if (b0 == 0xF0) lo = 0x90;
    if (b0 == 0xF4) hi = 0x8F;
    if (cont(pos + 1, lo, hi) && cont(pos + 2) && cont(pos + 3))
      return {int32_t(((b0 & 0x07) << 18) | ((s[pos + 1] & 0x3F) << 12) | ((s[pos + 2] & 0x3F) << 6) |
                      (s[pos + 3] & 0x3F)),
              4};
    return {0xFFFD, 1};
  }
  return {0xFFFD, 1};
}

bool GoIsPrint(uint32_t r) {
  if (r < 0x80) return r >= 0x20 && r < 0x7F;
  size_t n = sizeof(kPrint) / sizeof(kPrint[0]);
  size_t lo = 0, hi = n;
  while (lo < hi) {
    size_t m = (lo + hi) / 2;
    if (r < kPrint[m][0]) hi = m;
    else if (r > kPrint[m][1]) lo = m + 1;
    else return true;
  }
  return false;
}

static void AppendUtf8(std::string* out, uint32_t r);

std::string GoQuote(const std::string& s) {  // strconv.Quote
  static const char* hex = "0123456789abcdef";
  std::string o = "\"";
  const uint8_t* p = reinterpret_cast<const uint8_t*>(s.data());
  int64_t n = int64_t(s.size()), pos = 0;
  while (pos < n) {
    Rune r = DecodeRune(p, n, pos);
    if (r.r == 0xFFFD && r.width == 1) {
      o += "\\x";
      o.push_back(hex[p[pos] >> 4]);
      o.push_back(hex[p[pos] & 15]);
      pos += 1;
      continue;
    }
    uint32_t c = uint32_t(r.r);
    if (c == '"' || c == '\\') {
      o.push_back('\\');
      o.push_back(char(c));
    } else if (GoIsPrint(c)) {
      o.append(s, size_t(pos), size_t(r.width));
    } else {
      switch (c) {
        case 7: o += "\\a"; break;
        case 8: o += "\\b"; break;
        case 12: o += "\\f"; break;
        case 10: o += "\\n"; break;
        case 13: o += "\\r"; break;
        case 9: o += "\\t"; break;
        case 11: o += "\\v"; break;
        default:
          if (c < 0x20 || c == 0x7F) {
            o += "\\x";
            o.push_back(hex[c >> 4]);
            o.push_back(hex[c & 15]);
          } else if (c < 0x10000) {
            o += "\\u";
            for (int k = 12; k >= 0; k -= 4) o.push_back(hex[(c >> k) & 15]);
          } else {
            o += "\\U";
            for (int k = 28; k >= 0; k -= 4) o.push_back(hex[(c >> k) & 15]);
          }
      }
    }
    pos += r.width;
  }
  o.push_back('"');
  return o;
}

static void AppendUtf8(std::string* out, uint32_t r) {
  if (r < 0x80) {
    out->push_back(char(r));
  } else if (r < 0x800) {
    out->push_back(char(0xC0 | (r >> 6)));
    out->push_back(char(0x80 | (r & 0x3F)));
  } else if (r < 0x10000) {
    out->push_back(char(0xE0 | (r >> 12)));
    out->push_back(char(0x80 | ((r >> 6) & 0x3F)));
    out->push_back(char(0x80 | (r & 0x3F)));
  } else {
    out->push_back(char(0xF0 | (r >> 18)));
    out->push_back(char(0x80 | ((r >> 12) & 0x3F)));
    out->push_back(char(0x80 | ((r >> 6) & 0x3F)));
    out->push_back(char(0x80 | (r & 0x3F)));
  }
}

std::string GoBytesToLower(const uint8_t* s, size_t n) {
  bool ascii = true;
  for (size_t i = 0; i < n; i++)
    if (s[i] >= 0x80) { ascii = false; break; }
  std::string out;
  out.reserve(n);
  if (ascii) {
    for (size_t i = 0; i < n; i++) {
      uint8_t c = s[i];
      out.push_back(char((c >= 'A' && c <= 'Z') ? c + 32 : c));
    }
    return out;
  }
  int64_t pos = 0;
  while (pos < int64_t(n)) {
    Rune r = DecodeRune(s, n, pos);
    AppendUtf8(&out, GoToLower(uint32_t(r.r)));
    pos += r.width;
  }
  return out;
}

// ---------------------------------------------------------------------------
// Parser (regexp/syntax parse.go semantics, Perl flags)
// ---------------------------------------------------------------------------
class Parser {
 public:
  Parser(Regex* re, const std::string& s) : re_(re), s_(s) {}

  bool Parse(std::string* err) {
    re_->cap_names_.push_back("");
    int n = Alt();
    if (!err_.empty()) { *err = err_; return false; }
    if (i_ < s_.size()) {
      *err = s_[i_] == ')' ? "unexpected )" : "trailing input";
      return false;
    }
    re_->root_ = n;
    re_->num_cap_ = ncap_;
    return true;
  }

 private:
  Regex* re_;
  const std::string& s_;
  size_t i_ = 0;
  bool fi_ = false, fm_ = false, fs_ = false, fU_ = false;
  int ncap_ = 0;
  std::string err_;

  int Fail(const std::string& m) {
    if (err_.empty()) err_ = "error parsing regexp: " + m + ": `" + s_ + "`";
    return NewNode(NodeOp::NoMatch);
  }
  int NewNode(NodeOp op) {
    re_->nodes_.push_back(Node());
    re_->nodes_.back().op = op;
    return int(re_->nodes_.size()) - 1;
  }
  Node& N(int i) { return re_->nodes_[i]; }
  bool AtEnd() const { return i_ >= s_.size(); }
  int Peek(size_t k = 0) const { return i_ + k < s_.size() ? (uint8_t)s_[i_ + k] : -1; }

  // Next rune of the pattern (patterns are UTF-8 text).
  uint32_t NextRune() {
    Rune r = DecodeRune((const uint8_t*)s_.data(), s_.size(), i_);
    i_ += r.width;
    return uint32_t(r.r);
  }

  int ClassNode(RuneRanges r) {
    Clean(&r);
    int n = NewNode(NodeOp::Class);
    N(n).ranges = std::move(r);
    return n;
  }

  void AddFolded(RuneRanges* out, uint32_t lo, uint32_t hi) {
    // appendFoldedRange: add lo..hi plus every member of each rune's orbit.
    out->push_back({lo, hi});
    if (hi - lo > 0x20000) return;  // whole-plane ranges already contain their folds
    for (uint32_t c = lo; c <= hi; c++) {
      for (uint32_t f = SimpleFold(c); f != c; f = SimpleFold(f)) {
        if (f < lo || f > hi) out->push_back({f, f});
      }
    }
  }

  int Literal(uint32_t r) {
    RuneRanges rr;
    if (fi_) AddFolded(&rr, r, r);
    else rr.push_back({r, r});
    return ClassNode(rr);
  }

  int Alt() {
    std::vector<int> br;
    br.push_back(Concat());
    while (Peek() == '|') {
      i_++;
      br.push_back(Concat());
    }
    if (br.size() == 1) return br[0];
    int n = NewNode(NodeOp::Alt);
    N(n).subs = br;
    return n;
  }

  bool RepeatSpec(size_t j, int* lo, int* hi, size_t* len) {
    // {n} {n,} {n,m}
    if (j >= s_.size() || s_[j] != '{') return false;
    size_t k = j + 1;
    auto num = [&](int* v) {
      size_t st = k;
      long x = 0;
      while (k < s_.size() && s_[k] >= '0' && s_[k] <= '9') {
        x = x * 10 + (s_[k] - '0');
        if (x > 100000) x = 100000;
        k++;
      }
      *v = int(x);
      return k > st;
    };
    if (!num(lo)) return false;
    if (k < s_.size() && s_[k] == '}') {
      *hi = *lo;
      *len = k + 1 - j;
      return true;
    }
    if (k >= s_.size() || s_[k] != ',') return false;
    k++;
    if (k < s_.size() && s_[k] == '}') {
      *hi = -1;
      *len = k + 1 - j;
      return true;
    }
    if (!num(hi)) return false;
    if (k >= s_.size() || s_[k] != '}') return false;
    *len = k + 1 - j;
    return true;
  }

  int Concat() {
    std::vector<int> items;
    while (!AtEnd() && err_.empty()) {
      int c = Peek();
      if (c == '|' || c == ')') break;
      if (c == '*' || c == '+' || c == '?') return Fail("missing argument to repetition operator");
      int lo, hi;
      size_t ln;
      if (c == '{' && RepeatSpec(i_, &lo, &hi, &ln)) return Fail("missing argument to repetition operator");
      std::vector<int> atoms;
      bool is_flag = false;
      Atom(&atoms, &is_flag);
      if (is_flag) continue;
      if (atoms.empty()) continue;
      // repetition applies to the last atom only (\Q..\E yields several)
      int last = Repeats(atoms.back());
      atoms.back() = last;
      for (int a : atoms) items.push_back(a);
    }
    if (items.empty()) return NewNode(NodeOp::Empty);
    if (items.size() == 1) return items[0];
    int n = NewNode(NodeOp::Cat);
    N(n).subs = items;
    return n;
  }

  int Repeats(int atom) {
    bool had = false;
    while (!AtEnd()) {
      int c = Peek();
      int lo, hi;
      size_t ln = 1;
      if (c == '*') { lo = 0; hi = -1; }
      else if (c == '+') { lo = 1; hi = -1; }
      else if (c == '?') { lo = 0; hi = 1; }
      else if (c == '{') {
        if (!RepeatSpec(i_, &lo, &hi, &ln)) return atom;
        if (lo > kMaxRepeat || hi > kMaxRepeat || (hi >= 0 && lo > hi)) return Fail("invalid repeat count");
      } else {
        return atom;
      }
      if (had) return Fail("invalid nested repetition operator");
      i_ += ln;
      bool greedy = true;
      if (Peek() == '?') { i_++; greedy = false; }
      if (fU_) greedy = !greedy;
      int n = NewNode(NodeOp::Repeat);
      N(n).min = lo;
      N(n).max = hi;
      N(n).greedy = greedy;
      N(n).subs = {atom};
      atom = n;
      had = true;
    }
    return atom;
  }

  uint32_t EscapeRune() {  // parseEscape; i_ points after the backslash
    if (AtEnd()) { Fail("trailing backslash at end of expression"); return 0; }
    int c = Peek();
    i_++;
    if (c >= '1' && c <= '7') {
      int nx = Peek();
      if (nx < '0' || nx > '7') { Fail("invalid escape sequence"); return 0; }
      c = '0';
      i_--;
    }
    if (c == '0') {
      uint32_t v = 0;
      for (int k = 0; k < 2; k++) {
        int nx = Peek();
        if (nx >= '0' && nx <= '7') { v = v * 8 + uint32_t(nx - '0'); i_++; }
        else break;
      }
      return v;
    }
    if (c == 'x') {
      auto hexv = [](int ch) -> int {
        if (ch >= '0' && ch <= '9') return ch - '0';
        if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
        if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
        return -1;
      };
      if (Peek() == '{') {
        i_++;
        uint64_t v = 0;
        int nd = 0;
        while (!AtEnd() && Peek() != '}') {
          int h = hexv(Peek());
          if (h < 0) { Fail("invalid escape sequence"); return 0; }
          v = v * 16 + h;
          if (v > kMaxRune) { Fail("invalid escape sequence"); return 0; }
          nd++;
          i_++;
        }
        if (AtEnd() || nd == 0) { Fail("invalid escape sequence"); return 0; }
        i_++;
        return uint32_t(v);
      }
      int h1 = hexv(Peek()), h2 = hexv(Peek(1));
      if (h1 < 0 || h2 < 0) { Fail("invalid escape sequence"); return 0; }
      i_ += 2;
      return uint32_t(h1 * 16 + h2);
    }
    switch (c) {
      case 'a': return 7;
      case 'f': return 12;
      case 'n': return 10;
      case 'r': return 13;
      case 't': return 9;
      case 'v': return 11;
    }
    if (c < 0x80 && !((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')))
      return uint32_t(c);
    Fail("invalid escape sequence");
    return 0;
  }

  static RuneRanges Perl(int c) {
    switch (c) {
      case 'd': return {{'0', '9'}};
      case 's': return {{9, 10}, {12, 13}, {32, 32}};
      case 'w': return {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
    }
    return {};
  }

  static bool Posix(const std::string& name, RuneRanges* r) {
    static const struct { const char* n; RuneRanges r; } kT[] = {
        {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}},
        {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
        {"ascii", {{0, 0x7F}}},
        {"blank", {{9, 9}, {32, 32}}},
        {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}},
        {"digit", {{'0', '9'}}},
        {"graph", {{0x21, 0x7E}}},
        {"lower", {{'a', 'z'}}},
        {"print", {{0x20, 0x7E}}},
        {"punct", {{0x21, 0x2F}, {0x3A, 0x40}, {0x5B, 0x60}, {0x7B, 0x7E}}},
        {"space", {{9, 13}, {32, 32}}},
        {"upper", {{'A', 'Z'}}},
        {"word", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
        {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}},
    };
    for (auto& e : kT)
      if (name == e.n) { *r = e.r; return true; }
    return false;
  }

  void Atom(std::vector<int>* out, bool* is_flag) {
    int c = Peek();
    if (c == '(') { out->push_back(Group(is_flag)); return; }
    if (c == '[') { out->push_back(Class()); return; }
    if (c == '.') {
      i_++;
      if (fs_) out->push_back(ClassNode({{0, kMaxRune}}));
      else out->push_back(ClassNode({{0, 9}, {11, kMaxRune}}));
      return;
    }
    if (c == '^' || c == '$') {
      i_++;
      int n = NewNode(NodeOp::Assert);
      if (c == '^') N(n).assert_op = fm_ ? kEmptyBeginLine : kEmptyBeginText;
      else N(n).assert_op = fm_ ? kEmptyEndLine : kEmptyEndText;
      out->push_back(n);
      return;
    }
    if (c == '\\') {
      i_++;
      if (AtEnd()) { out->push_back(Fail("trailing backslash at end of expression")); return; }
      int e = Peek();
      if (e == 'A' || e == 'z' || e == 'b' || e == 'B') {
        i_++;
        int n = NewNode(NodeOp::Assert);
        N(n).assert_op = e == 'A' ? kEmptyBeginText : e == 'z' ? kEmptyEndText
                         : e == 'b' ? kEmptyWordBoundary : kEmptyNoWordBoundary;
        out->push_back(n);
        return;
      }
      if (e == 'd' || e == 's' || e == 'w' || e == 'D' || e == 'S' || e == 'W') {
        i_++;
        RuneRanges r = Perl(e | 0x20);
        out->push_back(ClassNode((e & 0x20) ? r : Negate(r)));
        return;
      }
      if (e == 'p' || e == 'P') { out->push_back(Fail("unicode classes unsupported")); return; }
      if (e == 'Q') {
        i_++;
        size_t end = s_.find("\\E", i_);
        size_t stop = end == std::string::npos ? s_.size() : end;
        while (i_ < stop) out->push_back(Literal(NextRune()));
        i_ = end == std::string::npos ? s_.size() : end + 2;
        return;
      }
      uint32_t r = EscapeRune();
      out->push_back(Literal(r));
      return;
    }
    out->push_back(Literal(NextRune()));
  }

  int Group(bool* is_flag) {
    // named captures (?P<name>re) / (?<name>re)
    size_t nstart = 0;
    if (s_.compare(i_, 4, "(?P<") == 0) nstart = i_ + 4;
    else if (s_.compare(i_, 3, "(?<") == 0 && s_.compare(i_, 4, "(?<=") != 0 && s_.compare(i_, 4, "(?<!") != 0)
      nstart = i_ + 3;
    if (nstart) {
      size_t end = s_.find('>', nstart);
      if (end == std::string::npos) return Fail("invalid named capture");
      std::string name = s_.substr(nstart, end - nstart);
      if (name.empty()) return Fail("invalid named capture");
      for (char ch : name)
        if (!(isalnum((unsigned char)ch) || ch == '_')) return Fail("invalid named capture");
      i_ = end + 1;
      return Capture(name);
    }
    if (s_.compare(i_, 2, "(?") == 0) {
      size_t j = i_ + 2;
      bool neg = false, seen = false;
      bool fl[4] = {fi_, fm_, fs_, fU_};
      for (;; j++) {
        if (j >= s_.size()) return Fail("missing closing )");
        char ch = s_[j];
        int k = ch == 'i' ? 0 : ch == 'm' ? 1 : ch == 's' ? 2 : ch == 'U' ? 3 : -1;
        if (k >= 0) { fl[k] = !neg; seen = true; continue; }
        if (ch == '-') {
          if (neg) return Fail("invalid or unsupported Perl syntax");
          neg = true;
          seen = false;
          continue;
        }
        if (ch == ':' || ch == ')') {
          if (neg && !seen) return Fail("invalid or unsupported Perl syntax");
          if (ch == ')' && !seen) return Fail("invalid or unsupported Perl syntax");
          break;
        }
        return Fail("invalid or unsupported Perl syntax");
      }
      if (s_[j] == ')') {
        fi_ = fl[0]; fm_ = fl[1]; fs_ = fl[2]; fU_ = fl[3];
        i_ = j + 1;
        *is_flag = true;
        return -1;
      }
      bool sv[4] = {fi_, fm_, fs_, fU_};
      fi_ = fl[0]; fm_ = fl[1]; fs_ = fl[2]; fU_ = fl[3];
      i_ = j + 1;
      int sub = Alt();
      if (Peek() != ')') return Fail("missing closing )");
      i_++;
      fi_ = sv[0]; fm_ = sv[1]; fs_ = sv[2]; fU_ = sv[3];
      return sub;
    }
    i_++;
    return Capture("");
  }

  int Capture(const std::string& name) {
    int idx = ++ncap_;
    re_->cap_names_.push_back(name);
    bool sv[4] = {fi_, fm_, fs_, fU_};
    int sub = Alt();
    if (Peek() != ')') return Fail("missing closing )");
    i_++;
    fi_ = sv[0]; fm_ = sv[1]; fs_ = sv[2]; fU_ = sv[3];
    int n = NewNode(NodeOp::Capture);
    N(n).cap = idx;
    N(n).subs = {sub};
    return n;
  }

  uint32_t ClassChar() {
    if (Peek() == '\\') {
      i_++;
      return EscapeRune();
    }
    return NextRune();
  }

  int Class() {
    i_++;
    bool negated = false;
    if (Peek() == '^') { negated = true; i_++; }
    RuneRanges rr;
    bool first = true;
    for (;;) {
      if (!err_.empty()) return NewNode(NodeOp::NoMatch);
      int c = Peek();
      if (c < 0) return Fail("missing closing ]");
      if (c == ']' && !first) { i_++; break; }
      first = false;
      if (c == '[' && Peek(1) == ':') {
        size_t end = s_.find(":]", i_ + 2);
        if (end != std::string::npos) {
          std::string name = s_.substr(i_ + 2, end - i_ - 2);
          bool neg = !name.empty() && name[0] == '^';
          if (neg) name = name.substr(1);
          RuneRanges pr;
          if (Posix(name, &pr)) {
            if (neg) pr = Negate(pr);
            if (fi_) { for (auto& p : pr) AddFolded(&rr, p.first, p.second); }
            else rr.insert(rr.end(), pr.begin(), pr.end());
            i_ = end + 2;
            continue;
          }
        }
      }
      if (c == '\\') {
        int e = Peek(1);
        if (e == 'd' || e == 's' || e == 'w' || e == 'D' || e == 'S' || e == 'W') {
          RuneRanges r = Perl(e | 0x20);
          if (!(e & 0x20)) r = Negate(r);
          rr.insert(rr.end(), r.begin(), r.end());
          i_ += 2;
          continue;
        }
        if (e == 'p' || e == 'P') return Fail("unicode classes unsupported");
      }
      uint32_t lo = ClassChar(), hi = lo;
      if (Peek() == '-' && Peek(1) >= 0 && Peek(1) != ']') {
        i_++;
        hi = ClassChar();
        if (hi < lo) return Fail("invalid character class range");
      }
      if (fi_) AddFolded(&rr, lo, hi);
      else rr.push_back({lo, hi});
    }
    Clean(&rr);
    if (negated) rr = Negate(rr);
    int n = NewNode(NodeOp::Class);
    N(n).ranges = std::move(rr);
    return n;
  }
};

// ---------------------------------------------------------------------------
// Compiler (simplify.go repeats + compile.go)
// ---------------------------------------------------------------------------
class Compiler {
 public:
  explicit Compiler(Regex* re) : re_(re) {}

  struct Frag {
    uint32_t i;
    std::vector<uint32_t> out;  // patch list: (inst << 1) | (0 = out, 1 = arg)
    bool nullable;
  };

  void Run() {
    auto& p = re_->prog_;
    p.clear();
    p.push_back(Inst());  // inst 0 = fail (Go: c.init())
    Frag f = Comp(re_->root_);
    uint32_t m = Emit(kIMatch);
    Patch(f.out, m);
    re_->start_ = f.i;
  }

 private:
  Regex* re_;

  uint32_t Emit(InstOp op) {
    re_->prog_.push_back(Inst());
    re_->prog_.back().op = op;
    return uint32_t(re_->prog_.size() - 1);
  }
  void Patch(const std::vector<uint32_t>& l, uint32_t to) {
    for (uint32_t x : l) {
      Inst& in = re_->prog_[x >> 1];
      if (x & 1) in.arg = to;
      else in.out = to;
    }
  }
  static std::vector<uint32_t> Cat(std::vector<uint32_t> a, const std::vector<uint32_t>& b) {
    a.insert(a.end(), b.begin(), b.end());
    return a;
  }

  Frag Nop() {
    uint32_t i = Emit(kINop);
    return {i, {i << 1}, true};
  }
  Frag FailFrag() { return {0, {}, false}; }

  Frag CatFrag(Frag a, Frag b) {
    if (a.i == 0 || b.i == 0) return FailFrag();
    Patch(a.out, b.i);
    return {a.i, b.out, a.nullable && b.nullable};
  }
  Frag AltFrag(Frag a, Frag b) {
    if (a.i == 0) return b;
    if (b.i == 0) return a;
    uint32_t i = Emit(kIAlt);
    re_->prog_[i].out = a.i;
    re_->prog_[i].arg = b.i;
    return {i, Cat(a.out, b.out), a.nullable || b.nullable};
  }
  Frag Quest(Frag a, bool nongreedy) {
    uint32_t i = Emit(kIAlt);
    std::vector<uint32_t> out;
    if (nongreedy) {
      re_->prog_[i].arg = a.i;
      out = {i << 1};
    } else {
      re_->prog_[i].out = a.i;
      out = {(i << 1) | 1};
    }
    return {i, Cat(out, a.out), true};
  }
  Frag Loop(Frag a, bool nongreedy) {
    uint32_t i = Emit(kIAlt);
    std::vector<uint32_t> out;
    if (nongreedy) {
      re_->prog_[i].arg = a.i;
      out = {i << 1};
    } else {
      re_->prog_[i].out = a.i;
      out = {(i << 1) | 1};
    }
    Patch(a.out, i);
    return {i, out, a.nullable};
  }
  Frag Star(Frag a, bool nongreedy) {
    if (a.nullable) return Quest(Plus(a, nongreedy), nongreedy);
    return Loop(a, nongreedy);
  }
  Frag Plus(Frag a, bool nongreedy) {
    Frag l = Loop(a, nongreedy);
    return {a.i, l.out, a.nullable};
  }

  // Simplified-repeat structure (simplify.go): returns an op tag for idempotence
  Frag Repeat(int sub, int min, int max, bool greedy) {
    bool ng = !greedy;
    const Node& s = re_->nodes_[sub];
    if (min == 0 && max == 0) return Nop();  // x{0} -> empty
    // empty-match sub: repeating it is still empty (simplify1)
    if (s.op == NodeOp::Empty) return Nop();
    if (max == -1) {
      if (min == 0) {
        if (s.op == NodeOp::Repeat && s.min == 0 && s.max == -1 && s.greedy == greedy) return Comp(sub);
        return Star(Comp(sub), ng);
      }
      if (min == 1) {
        if (s.op == NodeOp::Repeat && s.min == 1 && s.max == -1 && s.greedy == greedy) return Comp(sub);
        return Plus(Comp(sub), ng);
      }
      Frag f = Comp(sub);
      for (int k = 0; k < min - 2; k++) f = CatFrag(f, Comp(sub));
      return CatFrag(f, Plus(Comp(sub), ng));
    }
    if (min == 1 && max == 1) return Comp(sub);
    if (min == 0 && max == 1 && s.op == NodeOp::Repeat && s.min == 0 && s.max == 1 && s.greedy == greedy)
      return Comp(sub);
    // x{n,m} = n copies of x, then nested (x(x(x)?)?)?
    bool have = false;
    Frag prefix{0, {}, true};
    for (int k = 0; k < min; k++) {
      Frag c = Comp(sub);
      prefix = have ? CatFrag(prefix, c) : c;
      have = true;
    }
    if (max > min) {
      // build suffix from the innermost outwards, as Go does: suffix = x?; then (x suffix)? ...
      // compile order matters only for instruction numbering, not semantics.
      Frag suffix = Quest(Comp(sub), ng);
      for (int k = min + 1; k < max; k++) {
        Frag c = Comp(sub);
        suffix = Quest(CatFrag(c, suffix), ng);
      }
      prefix = have ? CatFrag(prefix, suffix) : suffix;
      have = true;
    }
    if (!have) return FailFrag();
    return prefix;
  }

  Frag Comp(int ni) {
    const Node n = re_->nodes_[ni];  // copy: nodes_ is not modified, but keep it simple
    switch (n.op) {
      case NodeOp::Empty: return Nop();
      case NodeOp::NoMatch: return FailFrag();
      case NodeOp::Class: {
        if (n.ranges.empty()) return FailFrag();
        if (n.ranges.size() == 1 && n.ranges[0].first == 0 && n.ranges[0].second == kMaxRune) {
          uint32_t i = Emit(kIAny);
          return {i, {i << 1}, false};
        }
        if (n.ranges.size() == 2 && n.ranges[0].first == 0 && n.ranges[0].second == 9 &&
            n.ranges[1].first == 11 && n.ranges[1].second == kMaxRune) {
          uint32_t i = Emit(kIAnyNotNL);
          return {i, {i << 1}, false};
        }
        if (n.ranges.size() == 1 && n.ranges[0].first == n.ranges[0].second) {
          uint32_t i = Emit(kIRune1);
          re_->prog_[i].rune = n.ranges[0].first;
          return {i, {i << 1}, false};
        }
        uint32_t i = Emit(kIRune);
        re_->prog_[i].cls = int(re_->classes_.size());
        re_->classes_.push_back(n.ranges);
        std::pair<uint64_t, uint64_t> a{0, 0};
        for (uint32_t c = 0; c < 128; c++)
          if (InRanges(n.ranges, c)) (c < 64 ? a.first : a.second) |= uint64_t(1) << (c & 63);
        re_->class_ascii_.push_back(a);
        return {i, {i << 1}, false};
      }
      case NodeOp::Assert: {
        uint32_t i = Emit(kIEmpty);
        re_->prog_[i].empty = n.assert_op;
        return {i, {i << 1}, true};
      }
      case NodeOp::Cat: {
        Frag f{0, {}, true};
        bool have = false;
        for (int s : n.subs) {
          Frag g = Comp(s);
          if (!have) { f = g; have = true; }
          else f = CatFrag(f, g);
        }
        return have ? f : Nop();
      }
      case NodeOp::Alt: {
        Frag f = Comp(n.subs[0]);
        for (size_t k = 1; k < n.subs.size(); k++) f = AltFrag(f, Comp(n.subs[k]));
        return f;
      }
      case NodeOp::Capture: {
        uint32_t a = Emit(kICapture);
        re_->prog_[a].arg = uint32_t(2 * n.cap);
        Frag sub = Comp(n.subs[0]);
        uint32_t b = Emit(kICapture);
        re_->prog_[b].arg = uint32_t(2 * n.cap + 1);
        Frag fa{a, {a << 1}, true};
        Frag fb{b, {b << 1}, true};
        return CatFrag(CatFrag(fa, sub), fb);
      }
      case NodeOp::Repeat: return Repeat(n.subs[0], n.min, n.max, n.greedy);
    }
    return FailFrag();
  }
};

std::unique_ptr<Regex> Regex::Compile(const std::string& pattern, std::string* err) {
  std::unique_ptr<Regex> re(new Regex());
  re->pattern_ = pattern;
  Parser p(re.get(), pattern);
  if (!p.Parse(err)) return nullptr;
  Compiler c(re.get());
  c.Run();
  // onepass-style anchoring info: does every path start with \A ?
  {
    uint32_t pc = re->start_;
    for (int guard = 0; guard < 1000; guard++) {
      const Inst& in = re->prog_[pc];
      if (in.op == kINop || in.op == kICapture) { pc = in.out; continue; }
      if (in.op == kIEmpty && (in.empty & kEmptyBeginText)) re->anchored_begin_ = true;
      break;
    }
  }
  re->ComputeFirstBytes();
  re->DetectRun();
  re->DetectLiteral();
  {  // instructions whose only predecessor is one rune instruction (Backtracker chain skip)
    std::vector<uint32_t> preds(re->prog_.size(), 0);
    std::vector<uint8_t> from_rune(re->prog_.size(), 0);
    for (const Inst& in : re->prog_) {
      switch (in.op) {
        case kIAlt: preds[in.out]++; preds[in.arg]++; break;
        case kICapture: case kIEmpty: case kINop: preds[in.out]++; break;
        case kIRune: case kIRune1: case kIAny: case kIAnyNotNL: preds[in.out]++; from_rune[in.out] = 1; break;
        default: break;
      }
    }
    preds[re->start_]++;  // the start state is entered from outside
    re->single_pred_.assign(re->prog_.size(), 0);
    for (size_t pc = 0; pc < re->prog_.size(); pc++) re->single_pred_[pc] = preds[pc] == 1 && from_rune[pc];
  }
  return re;
}

void Regex::ComputeFirstBytes() {
  uint64_t f[4] = {};
  bool all = false;
  auto add = [&](uint32_t b) { f[b >> 6] |= uint64_t(1) << (b & 63); };
  auto lead = [](uint32_t r) -> uint32_t {
    return r < 0x80 ? r : r < 0x800 ? 0xC0 | (r >> 6) : r < 0x10000 ? 0xE0 | (r >> 12) : 0xF0 | (r >> 18);
  };
  auto add_range = [&](uint32_t lo, uint32_t hi) {
    for (uint32_t b = lo; b <= hi && b < 0x80; b++) add(b);
    if (hi < 0x80) return;
    if (lo <= 0xFFFD && 0xFFFD <= hi) {  // invalid bytes decode to U+FFFD (width 1)
      for (uint32_t b = 0x80; b < 0x100; b++) add(b);
      return;
    }
    for (uint32_t b = lead(lo < 0x80 ? 0x80 : lo); b <= lead(hi); b++) add(b);
  };
  std::vector<uint32_t> stack{start_};
  std::vector<uint8_t> seen(prog_.size(), 0);
  while (!stack.empty() && !all) {
    const uint32_t pc = stack.back();
    stack.pop_back();
    if (seen[pc]) continue;
    seen[pc] = 1;
    const Inst& in = prog_[pc];
    switch (in.op) {
      case kIFail: break;
      case kIAlt: stack.push_back(in.out); stack.push_back(in.arg); break;
      case kICapture: case kIEmpty: case kINop: stack.push_back(in.out); break;  // assertions: superset
      case kIMatch: all = true; break;  // an empty match
      case kIRune1: add_range(in.rune, in.rune); break;
      case kIRune: for (auto& rg : classes_[size_t(in.cls)]) add_range(rg.first, rg.second); break;
      case kIAny: all = true; break;
      case kIAnyNotNL:
        for (uint32_t b = 0; b < 256; b++)
          if (b != '\n') add(b);
        break;
    }
  }
  first_all_ = all;
  for (int k = 0; k < 4; k++) first_[k] = f[k];
}

// ---------------------------------------------------------------------------
// Pike VM (regexp/exec.go)
// ---------------------------------------------------------------------------
class Machine {
 public:
  Machine(const Regex* re, int ncap) : re_(re), ncap_(ncap) {
    size_t n = re->prog_.size();
    for (int k = 0; k < 2; k++) {
      q_[k].sparse.assign(n, 0);
      q_[k].dense.reserve(n);
    }
    matchcap_.assign(ncap, -1);
    // Pre-size thread storage: a queue holds at most one thread per pc, so
    // 2*|prog| threads suffice; capture pointers into caps_ must stay valid.
    size_t maxt = 2 * n + 4;
    tinst_.reserve(maxt);
    caps_.reserve(maxt * size_t(ncap > 0 ? ncap : 1));
  }

  // One leftmost-first search from `pos` (m.match).  Returns true on match,
  // filling matchcap_.  `wins`: allowed start windows (nullptr = everywhere).
  bool Search(const uint8_t* s, int64_t n, int64_t pos, const std::vector<Window>* wins) {
    matched_ = false;
    std::fill(matchcap_.begin(), matchcap_.end(), -1);
    Queue* runq = &q_[0];
    Queue* nextq = &q_[1];
    Clear(runq);
    Clear(nextq);
    size_t wi = 0;
    if (wins) {
      while (wi < wins->size() && (*wins)[wi].hi < pos) wi++;
    }
    Rune r = DecodeRune(s, n, pos);
    Rune r1 = r.r >= 0 ? DecodeRune(s, n, pos + r.width) : Rune{-1, 0};
    uint8_t flag = Context(s, n, pos);
    for (;;) {
      if (runq->dense.empty()) {
        if (re_->anchored_begin_ && pos != 0) break;
        if (matched_) break;
        if (wins) {
          // jump to the next allowed start (rune-aligned)
          while (wi < wins->size() && (*wins)[wi].hi < pos) wi++;
          if (wi >= wins->size()) break;
          if ((*wins)[wi].lo > pos) {
            int64_t t = Align(s, n, (*wins)[wi].lo);
            if (t > pos) {
              pos = t;
              r = DecodeRune(s, n, pos);
              r1 = r.r >= 0 ? DecodeRune(s, n, pos + r.width) : Rune{-1, 0};
              flag = Context(s, n, pos);
            }
          }
        }
      }
      bool allowed = true;
      if (wins) {
        while (wi < wins->size() && (*wins)[wi].hi < pos) wi++;
        allowed = wi < wins->size() && (*wins)[wi].lo <= pos;
      }
      if (!matched_ && allowed && (pos == 0 || !re_->anchored_begin_)) {
        if (ncap_ > 0) matchcap_[0] = pos;
        Add(runq, re_->start_, pos, matchcap_.data(), flag, -1);
      }
      uint8_t nextflag = EmptyOpContext(r.r, r1.r);
      Step(runq, nextq, pos, pos + r.width, r.r, nextflag);
      if (r.width == 0) break;
      if (ncap_ == 0 && matched_) break;
      pos += r.width;
      r = r1;
      if (r.r >= 0) r1 = DecodeRune(s, n, pos + r.width);
      flag = nextflag;
      std::swap(runq, nextq);
    }
    Clear(nextq);
    Clear(runq);
    return matched_;
  }

  const std::vector<int64_t>& cap() const { return matchcap_; }

  // Largest Go rune-chain position <= t (see goregex.h): only a continuation
  // byte inside a valid multi-byte sequence is not a rune boundary.
  static int64_t Align(const uint8_t* s, int64_t n, int64_t t) {
    if (t >= n || t <= 0) return t;
    if ((s[t] & 0xC0) != 0x80) return t;
    for (int k = 1; k <= 3 && t - k >= 0; k++) {
      uint8_t b = s[t - k];
      if ((b & 0xC0) == 0x80) continue;
      Rune r = DecodeRune(s, n, t - k);
      if (r.width > k) return t - k;
      return t;
    }
    return t;
  }

 private:
  struct Entry {
    uint32_t pc;
    int t;  // thread index or -1
  };
  struct Queue {
    std::vector<uint32_t> sparse;
    std::vector<Entry> dense;
  };
  const Regex* re_;
  int ncap_;
  Queue q_[2];
  bool matched_ = false;
  std::vector<int64_t> matchcap_;
  std::vector<int64_t> caps_;  // thread capture storage
  std::vector<uint32_t> tinst_;
  std::vector<int> free_;

  int Alloc() {
    if (!free_.empty()) {
      int t = free_.back();
      free_.pop_back();
      return t;
    }
    int t = int(tinst_.size());
    tinst_.push_back(0);
    caps_.resize(caps_.size() + size_t(ncap_ > 0 ? ncap_ : 1));
    return t;
  }
  int64_t* Cap(int t) { return caps_.data() + size_t(t) * size_t(ncap_ > 0 ? ncap_ : 1); }

  static bool Contains(const Queue* q, uint32_t pc) {
    uint32_t j = q->sparse[pc];
    return j < q->dense.size() && q->dense[j].pc == pc;
  }
  void Clear(Queue* q) {
    for (auto& e : q->dense)
      if (e.t >= 0) free_.push_back(e.t);
    q->dense.clear();
  }

  friend class Backtracker;
  static uint8_t Context(const uint8_t* s, int64_t n, int64_t pos) {
    int32_t r1 = -1, r2 = -1;
    if (pos > 0 && pos <= n) {
      uint8_t b = s[pos - 1];
      r1 = b < 0x80 ? b : 0xFFFD;  // only ASCII word chars and '\n' matter
    }
    if (pos < n) {
      uint8_t b = s[pos];
      r2 = b < 0x80 ? b : 0xFFFD;
    }
    return EmptyOpContext(r1, r2);
  }

  // m.add: follow empty transitions; returns the (possibly unused) thread t.
  int Add(Queue* q, uint32_t pc, int64_t pos, int64_t* cap, uint8_t cond, int t) {
    if (pc == 0) return t;
    if (Contains(q, pc)) return t;
    uint32_t j = uint32_t(q->dense.size());
    q->sparse[pc] = j;
    q->dense.push_back({pc, -1});
    const Inst& in = re_->prog_[pc];
    switch (in.op) {
      case kIFail: break;
      case kIAlt:
        t = Add(q, in.out, pos, cap, cond, t);
        t = Add(q, in.arg, pos, cap, cond, t);
        break;
      case kIEmpty:
        if ((in.empty & ~cond) == 0) t = Add(q, in.out, pos, cap, cond, t);
        break;
      case kINop: t = Add(q, in.out, pos, cap, cond, t); break;
      case kICapture:
        if (int(in.arg) < ncap_) {
          int64_t opos = cap[in.arg];
          cap[in.arg] = pos;
          Add(q, in.out, pos, cap, cond, -1);
          cap[in.arg] = opos;
        } else {
          t = Add(q, in.out, pos, cap, cond, t);
        }
        break;
      default: {  // Match, Rune*, Any*
        if (t < 0) t = Alloc();
        tinst_[t] = pc;
        if (ncap_ > 0 && Cap(t) != cap) std::memcpy(Cap(t), cap, sizeof(int64_t) * size_t(ncap_));
        q->dense[j].t = t;
        t = -1;
      }
    }
    return t;
  }

  bool MatchRune(const Inst& in, int32_t c) const { return re_->RuneMatch(in, c); }

  void Step(Queue* runq, Queue* nextq, int64_t pos, int64_t nextpos, int32_t c, uint8_t nextcond) {
    for (size_t j = 0; j < runq->dense.size(); j++) {
      int t = runq->dense[j].t;
      if (t < 0) continue;
      const Inst& in = re_->prog_[tinst_[t]];
      bool add = false;
      if (in.op == kIMatch) {
        if (ncap_ > 0) {
          Cap(t)[1] = pos;
          std::memcpy(matchcap_.data(), Cap(t), sizeof(int64_t) * size_t(ncap_));
        }
        // first-match mode: cut off lower-priority threads
        for (size_t k = j + 1; k < runq->dense.size(); k++)
          if (runq->dense[k].t >= 0) free_.push_back(runq->dense[k].t);
        runq->dense.resize(j + 1);
        matched_ = true;
      } else {
        add = MatchRune(in, c);
      }
      if (add) t = Add(nextq, in.out, nextpos, ncap_ > 0 ? Cap(t) : nullptr, nextcond, t);
      if (t >= 0) free_.push_back(t);
      runq->dense[j].t = -1;
    }
    runq->dense.clear();
  }
};

bool Regex::RuneMatch(const Inst& in, int32_t c) const {
  switch (in.op) {
    case kIRune1: return c == int32_t(in.rune);
    case kIRune:
      if (c < 0) return false;
      if (c < 128) {
        const auto& a = class_ascii_[in.cls];
        return ((c < 64 ? a.first : a.second) >> (c & 63)) & 1;
      }
      return InRanges(classes_[in.cls], uint32_t(c));
    case kIAny: return c >= 0;
    case kIAnyNotNL: return c >= 0 && c != '\n';
    default: return false;
  }
}

// ---------------------------------------------------------------------------
// Bit-state backtracker (regexp/backtrack.go): depth-first in priority order
// from each allowed start position in turn, each (pc, pos) explored at most
// once per search (a state that failed from an earlier start fails again).
// The first Match reached is the leftmost-first match, as in the Pike VM.
// The visited bits are rows of |prog| bits per text position from `base_`,
// cleared lazily as the furthest position grows (paths only move forward), so
// a search costs what it touches, not the file length.  Above kMaxRows
// positions it gives up and the caller runs the Pike VM instead.
// ---------------------------------------------------------------------------
std::atomic<int> g_regex_engine{0};  // tests: 0 auto, 1 Pike VM only, 2 backtracker with an 8-row budget

class Backtracker {
 public:
  static constexpr int64_t kMaxRows = 1 << 16;
  int64_t max_rows_ = kMaxRows;

  // Same contract as Machine::Search (returns the match in cap()).  *overflow:
  // the search needed more than kMaxRows positions; the result is invalid.
  bool Search(const Regex* re, const uint8_t* s, int64_t n, int64_t pos, const std::vector<Window>* wins, int ncap,
              bool* overflow) {
    re_ = re;
    s_ = s;
    n_ = n;
    ncap_ = ncap;
    overflow_ = false;
    stride_ = (re->prog_.size() + 63) / 64;
    cap_.assign(size_t(ncap > 0 ? ncap : 1), -1);
    matchcap_.assign(size_t(ncap > 0 ? ncap : 1), -1);
    top_ = -1;  // no rows yet
    const bool anchored = re->anchored_begin_;
    size_t wi = 0;
    for (;;) {
      if (wins) {
        while (wi < wins->size() && (*wins)[wi].hi < pos) wi++;
        if (wi >= wins->size()) break;
        if ((*wins)[wi].lo > pos) {
          const int64_t t = Machine::Align(s, n, (*wins)[wi].lo);
          if (t > pos) pos = t;
        }
      }
      const bool allowed = !wins || (*wins)[wi].lo <= pos;
      if (anchored && pos != 0) break;
      if (allowed && re->FirstOk(s, n, pos)) {
        if (top_ < pos) Rebase(pos);  // states before pos are unreachable from here on
        if (ncap_ > 0) cap_[0] = pos;
        if (Try(re->start_, pos)) return true;
        if (overflow_) {
          *overflow = true;
          return false;
        }
      }
      if (pos >= n) break;
      pos += DecodeRune(s, n, pos).width;
    }
    return false;
  }
  const std::vector<int64_t>& cap() const { return matchcap_; }

 private:
  struct Job {
    uint32_t pc;
    bool arg;
    int64_t pos;  // capture-restore jobs: the saved capture value
  };
  const Regex* re_ = nullptr;
  const uint8_t* s_ = nullptr;
  int64_t n_ = 0;
  int ncap_ = 0;
  bool overflow_ = false;
  size_t stride_ = 1;  // u64 words per position row
  int64_t base_ = 0, top_ = -1;  // rows [base_, top_] are cleared / in use
  std::vector<uint64_t> visited_;
  std::vector<Job> jobs_;
  std::vector<int64_t> cap_, matchcap_;

  void Rebase(int64_t pos) {
    base_ = pos;
    top_ = pos - 1;
  }
  bool ShouldVisit(uint32_t pc, int64_t pos) {
    if (pos > top_) {
      if (pos - base_ >= max_rows_) {
        overflow_ = true;
        return false;
      }
      const size_t need = size_t(pos - base_ + 1) * stride_;
      if (visited_.size() < need) visited_.resize(std::max(need, visited_.size() * 2));
      std::fill(visited_.begin() + ptrdiff_t(size_t(top_ + 1 - base_) * stride_), visited_.begin() + ptrdiff_t(need),
                uint64_t(0));
      top_ = pos;
    }
    uint64_t& w = visited_[size_t(pos - base_) * stride_ + (pc >> 6)];
    const uint64_t bit = uint64_t(1) << (pc & 63);
    if (w & bit) return false;
    w |= bit;
    return true;
  }
  void Push(uint32_t pc, int64_t pos, bool arg) {
    if (re_->prog_[pc].op != kIFail && (arg || ShouldVisit(pc, pos))) jobs_.push_back({pc, arg, pos});
  }
  bool Try(uint32_t pc0, int64_t pos0) {
    const std::vector<Inst>& prog = re_->prog_;
    jobs_.clear();
    Push(pc0, pos0, false);
    while (!jobs_.empty()) {
      if (overflow_) return false;
      const Job j = jobs_.back();
      jobs_.pop_back();
      uint32_t pc = j.pc;
      int64_t pos = j.pos;
      bool arg = j.arg;
      goto skip;
    check:
      if (!ShouldVisit(pc, pos)) continue;
    skip : {
      const Inst& in = prog[pc];
      switch (in.op) {
        case kIFail: continue;
        case kIAlt:
          if (arg) {  // finished in.out; try in.arg
            arg = false;
            pc = in.arg;
          } else {
            Push(pc, pos, true);
            pc = in.out;
          }
          goto check;
        case kIRune:
        case kIRune1:
        case kIAny:
        case kIAnyNotNL: {
          // ASCII bytes inline (the classes' ASCII bitmaps); other runes decoded
          if (pos < n_ && s_[pos] < 0x80) {
            const uint32_t c = s_[pos];
            bool ok;
            if (in.op == kIRune) {
              const auto& a = re_->class_ascii_[size_t(in.cls)];
              ok = ((c < 64 ? a.first : a.second) >> (c & 63)) & 1;
            } else {
              ok = in.op == kIRune1 ? c == in.rune : (in.op == kIAny || c != '\n');
            }
            if (!ok) continue;
            pos += 1;
          } else {
            const Rune r = DecodeRune(s_, n_, pos);
            if (!re_->RuneMatch(in, r.r)) continue;
            pos += r.width;
          }
          pc = in.out;
          // a successor reached from this instruction only: (pc, pos) cannot have
          // been visited, since its one predecessor state is visited once
          if (re_->single_pred_[pc]) goto skip;
          goto check;
        }
        case kICapture:
          if (arg) {  // restore the saved value
            cap_[in.arg] = pos;
            continue;
          }
          if (int(in.arg) < ncap_) {
            jobs_.push_back({pc, true, cap_[in.arg]});
            cap_[in.arg] = pos;
          }
          pc = in.out;
          goto check;
        case kIEmpty:
          if ((in.empty & ~Machine::Context(s_, n_, pos)) != 0) continue;
          pc = in.out;
          goto check;
        case kINop:
          pc = in.out;
          goto check;
        case kIMatch:
          if (ncap_ > 1) cap_[1] = pos;
          matchcap_ = cap_;
          return true;
      }
    }
    }
    return false;
  }
};

namespace {
thread_local Backtracker t_bt;  // per host thread: its visited rows and job stack are reused
}

// MatchString: any match at all.  The bit-state backtracker answers it without
// allocating (a Pike VM per call cost 15% of the host tail, mostly in the
// allow-path regexes); the Pike VM only past its row budget.
bool Regex::Match(const uint8_t* s, int64_t n) const {
  const int mode = g_regex_engine.load(std::memory_order_relaxed);
  if (lit_ok_ && mode == 0) return MatchLiteral(s, n);
  Backtracker& bt = t_bt;
  if (mode != 1) {
    bt.max_rows_ = mode == 2 ? 8 : Backtracker::kMaxRows;
    bool overflow = false;
    if (bt.Search(this, s, n, 0, nullptr, 0, &overflow)) return true;
    if (!overflow) return false;
  }
  Machine m(this, 0);
  return m.Search(s, n, 0, nullptr);
}

void Regex::DetectLiteral() {
  if (anchored_begin_) return;
  int x = root_;
  while (nodes_[size_t(x)].op == NodeOp::Capture) x = nodes_[size_t(x)].subs[0];
  std::vector<int> parts;
  const Node& top = nodes_[size_t(x)];
  if (top.op == NodeOp::Cat) {
    for (int sub : top.subs) {
      int y = sub;
      while (nodes_[size_t(y)].op == NodeOp::Capture) y = nodes_[size_t(y)].subs[0];
      if (nodes_[size_t(y)].op == NodeOp::Empty) continue;
      parts.push_back(y);
    }
  } else {
    parts.push_back(x);
  }
  if (parts.empty() || parts.size() > 64) return;
  std::vector<uint8_t> a, b;
  for (int y : parts) {
    const Node& nd = nodes_[size_t(y)];
    if (nd.op != NodeOp::Class) return;
    uint32_t runes[2], k = 0;
    for (const auto& rg : nd.ranges)
      for (uint32_t r = rg.first; r <= rg.second; r++) {
        if (r >= 0x80 || k == 2) return;
        runes[k++] = r;
      }
    if (k == 0) return;
    a.push_back(uint8_t(runes[0]));
    b.push_back(uint8_t(runes[k - 1]));
  }
  lit_a_ = std::move(a);
  lit_b_ = std::move(b);
  lit_ok_ = true;
}

bool Regex::MatchLiteral(const uint8_t* s, int64_t n) const {
  const int64_t L = int64_t(lit_a_.size());
  const uint8_t a0 = lit_a_[0], b0 = lit_b_[0];
  for (int64_t p = 0; p + L <= n; p++) {
    if (s[p] != a0 && s[p] != b0) continue;
    int64_t j = 1;
    while (j < L && (s[p + j] == lit_a_[size_t(j)] || s[p + j] == lit_b_[size_t(j)])) j++;
    if (j == L) return true;
  }
  return false;
}

void Regex::DetectRun() {
  int x = root_, caps = 0;
  for (;;) {  // through capture groups and single-element concatenations
    const Node& nd = nodes_[size_t(x)];
    if (nd.op == NodeOp::Capture) {
      caps++;
      x = nd.subs[0];
      continue;
    }
    if (nd.op == NodeOp::Cat) {
      int only = -1, cnt = 0;
      for (int sub : nd.subs)
        if (nodes_[size_t(sub)].op != NodeOp::Empty) {
          only = sub;
          cnt++;
        }
      if (cnt != 1) return;
      x = only;
      continue;
    }
    break;
  }
  const Node& r = nodes_[size_t(x)];
  if (r.op != NodeOp::Repeat || !r.greedy || r.min < 1 || caps != num_cap_) return;
  const Node& c = nodes_[size_t(r.subs[0])];
  if (c.op != NodeOp::Class) return;
  run_cls_ = c.ranges;
  run_ascii_[0] = run_ascii_[1] = 0;
  for (uint32_t b = 0; b < 128; b++)
    if (InRanges(run_cls_, b)) run_ascii_[b >> 6] |= uint64_t(1) << (b & 63);
  for (uint32_t b = 0; b < 256; b++) run_tbl_[b] = b >= 0x80 ? 2 : uint8_t((run_ascii_[b >> 6] >> (b & 63)) & 1);
  run_min_ = r.min;
  run_max_ = r.max;
  run_ok_ = true;
}

// FindAll of C{m,n} (greedy, m >= 1), leftmost-first as the backtracker finds
// it: at a start, the match is the longest run of class runes there, cut at n;
// with fewer than m class runes at a start, no start up to the rune that ended
// the run can match either (their runs are shorter), so the search resumes
// after it.  Windows restrict the starts as in Backtracker::Search.
void Regex::FindAllRun(const uint8_t* s, int64_t n, bool submatch, const std::vector<Window>* wins,
                       std::vector<int64_t>* out) const {
  const int groups = submatch ? num_cap_ + 1 : 1;
  const int64_t lim = run_max_ < 0 ? INT64_MAX : int64_t(run_max_);
  int64_t pos = 0;
  size_t wi = 0;
  while (pos < n) {
    if (wins) {
      while (wi < wins->size() && (*wins)[wi].hi < pos) wi++;
      if (wi >= wins->size()) break;
      if ((*wins)[wi].lo > pos) {
        const int64_t t = Machine::Align(s, n, (*wins)[wi].lo);
        if (t > pos) pos = t;
      }
      if (pos >= n) break;
      if ((*wins)[wi].lo > pos) {  // not a start the windows allow: the next rune
        pos += DecodeRune(s, n, pos).width;
        continue;
      }
    }
    int64_t q = pos, k = 0;
    int w = 1;
    while (q < n && k < lim) {
      const uint8_t t = run_tbl_[s[q]];
      if (t == 1) {  // an ASCII member: the common case
        q++;
        k++;
        continue;
      }
      bool in;
      if (t == 0) {
        w = 1;
        in = false;
      } else {
        const Rune r = DecodeRune(s, n, q);
        w = r.width;
        in = InRanges(run_cls_, uint32_t(r.r));
      }
      if (!in) break;
      q += w;
      k++;
    }
    if (k >= run_min_) {
      for (int g = 0; g < groups; g++) {
        out->push_back(pos);
        out->push_back(q);
      }
      pos = q;
      continue;
    }
    pos = q < n ? q + w : n;  // q: the rune that ended the run (w: its width)
  }
}

void Regex::FindAll(const uint8_t* s, int64_t n, bool submatch, const std::vector<Window>* wins,
                    std::vector<int64_t>* out) const {
  int ncap = submatch ? 2 * (num_cap_ + 1) : 2;
  Backtracker& bt = t_bt;
  const int mode = g_regex_engine.load(std::memory_order_relaxed);
  if (run_ok_ && mode == 0) {  // modes 1-3: the general engines (tests compare them)
    FindAllRun(s, n, submatch, wins, out);
    return;
  }
  bt.max_rows_ = mode == 2 ? 8 : Backtracker::kMaxRows;
  std::unique_ptr<Machine> m;  // only when the backtracker's row budget runs out
  if (mode == 1) m.reset(new Machine(this, ncap));
  int64_t pos = 0, prev_end = -1;
  while (pos <= n) {
    bool overflow = false;
    const std::vector<int64_t>* cp;
    if (!m && bt.Search(this, s, n, pos, wins, ncap, &overflow)) {
      cp = &bt.cap();
    } else {
      if (!overflow && !m) break;
      if (!m) m.reset(new Machine(this, ncap));
      if (!m->Search(s, n, pos, wins)) break;
      cp = &m->cap();
    }
    const auto& c = *cp;
    bool accept = true;
    if (c[1] == pos) {  // empty match
      if (c[0] == prev_end) accept = false;
      Rune r = DecodeRune(s, n, pos);
      pos += r.width > 0 ? r.width : 1;
    } else {
      pos = c[1];
    }
    prev_end = c[1];
    if (accept) out->insert(out->end(), c.begin(), c.end());
  }
}

}  // namespace tsg
