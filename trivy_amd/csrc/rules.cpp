// Rule compiler (see rules.h).  Superset arguments are in DESIGN.md §2-3.
#include "rules.h"

#include <cstdio>
#include <cstdlib>

#include "filter.h"

#include <algorithm>
#include <array>
#include <bitset>
#include <deque>
#include <functional>
#include <map>
#include <set>

namespace tsg {

namespace {
constexpr int64_t kInf = int64_t(1) << 40;
constexpr size_t kMaxAnchorLit = 32;

bool IsFoldOnlyRune(uint32_t r) { return r == 0x212A || r == 0x17F || r == 0x130; }

int Utf8Len(uint32_t r) { return r < 0x80 ? 1 : r < 0x800 ? 2 : r < 0x10000 ? 3 : 4; }

bool ClassHas(const RuneRanges& rr, uint32_t c) {
  for (auto& p : rr)
    if (c >= p.first && c <= p.second) return true;
  return false;
}

// Byte-length range of one rune matched by the class, over the runes that can
// appear in a non-special file (U+212A/U+017F/U+0130 only occur in files the
// GPU routes to full-scan mode).
void ClassBytes(const RuneRanges& rr, int64_t* mn, int64_t* mx, bool fold_runes) {
  int lo = 5, hi = 0;
  bool any = false;
  for (auto& p : rr) {
    uint32_t a = p.first, b = p.second;
    // split across utf8 length boundaries
    const uint32_t bounds[4][2] = {{0, 0x7F}, {0x80, 0x7FF}, {0x800, 0xFFFF}, {0x10000, 0x10FFFF}};
    for (int k = 0; k < 4; k++) {
      uint32_t x = std::max(a, bounds[k][0]), y = std::min(b, bounds[k][1]);
      if (x > y) continue;
      // skip the fold-only runes if they are the only members in this part
      bool only_special = !fold_runes;
      for (uint32_t c = x; c <= y && only_special; c++) {
        if (!IsFoldOnlyRune(c)) only_special = false;
        if (c - x > 4) only_special = false;
      }
      if (only_special) continue;
      any = true;
      lo = std::min(lo, k + 1);
      hi = std::max(hi, k + 1);
    }
  }
  if (ClassHas(rr, 0xFFFD)) { lo = 1; hi = std::max(hi, 1); any = true; }
  if (!any) { lo = 1; hi = 1; }
  *mn = lo;
  *mx = hi;
}

// A class that is one ASCII character, possibly case-folded (incl. its
// U+212A/U+017F orbit members).  Returns the lowercased char or -1.
int LitChar(const Node& n) {
  if (n.op != NodeOp::Class) return -1;
  std::vector<uint32_t> asc, uni;
  uint64_t total = 0;
  for (auto& p : n.ranges) {
    total += uint64_t(p.second - p.first) + 1;
    if (total > 4) return -1;
    for (uint32_t c = p.first; c <= p.second; c++) (c < 0x80 ? asc : uni).push_back(c);
  }
  if (asc.empty() || asc.size() > 2) return -1;
  uint32_t c = asc[0];
  if (asc.size() == 2) {
    uint32_t a = asc[0], b = asc[1];
    if (!(a >= 'A' && a <= 'Z' && b == a + 32)) return -1;
    c = b;
  }
  uint32_t lc = (c >= 'A' && c <= 'Z') ? c + 32 : c;
  for (uint32_t u : uni) {
    if (!((u == 0x212A && lc == 'k') || (u == 0x17F && lc == 's'))) return -1;
  }
  return int(lc);
}

struct Analyzer {
  const std::vector<Node>& nodes;
  bool fold;
  std::map<int, std::pair<int64_t, int64_t>> memo;

  Analyzer(const std::vector<Node>& n, bool f) : nodes(n), fold(f) {}

  std::pair<int64_t, int64_t> Bytes(int i) {
    auto it = memo.find(i);
    if (it != memo.end()) return it->second;
    const Node& n = nodes[i];
    std::pair<int64_t, int64_t> r{0, 0};
    switch (n.op) {
      case NodeOp::Empty:
      case NodeOp::NoMatch:
      case NodeOp::Assert: break;
      case NodeOp::Class: ClassBytes(n.ranges, &r.first, &r.second, fold); break;
      case NodeOp::Cat:
        for (int s : n.subs) {
          auto b = Bytes(s);
          r.first += b.first;
          r.second = (r.second >= kInf || b.second >= kInf) ? kInf : r.second + b.second;
        }
        break;
      case NodeOp::Alt: {
        r.first = kInf;
        for (int s : n.subs) {
          auto b = Bytes(s);
          r.first = std::min(r.first, b.first);
          r.second = std::max(r.second, b.second);
        }
        break;
      }
      case NodeOp::Capture: r = Bytes(n.subs[0]); break;
      case NodeOp::Repeat: {
        auto b = Bytes(n.subs[0]);
        r.first = b.first * n.min;
        if (n.max < 0 || b.second >= kInf) r.second = b.second == 0 ? 0 : kInf;
        else r.second = b.second * n.max;
        if (r.second > kInf) r.second = kInf;
        break;
      }
    }
    memo[i] = r;
    return r;
  }

  void Flatten(int i, std::vector<int>* out) {
    const Node& n = nodes[i];
    if (n.op == NodeOp::Cat) {
      for (int s : n.subs) Flatten(s, out);
    } else if (n.op == NodeOp::Capture) {
      Flatten(n.subs[0], out);
    } else if (n.op == NodeOp::Empty || n.op == NodeOp::Assert) {
      // zero-width: contributes no bytes, literal runs continue across it
    } else {
      out->push_back(i);
    }
  }

  // Nodes of the leading literal run of a node's flattened sequence.
  std::vector<int> LeadNodes(int i) {
    std::vector<int> items, run;
    Flatten(i, &items);
    for (int it : items) {
      if (LitChar(nodes[it]) < 0 || run.size() >= kMaxAnchorLit) break;
      run.push_back(it);
    }
    return run;
  }

  // Leading literal run of a node's flattened sequence ("" if none).
  std::string LeadLiteral(int i) {
    std::vector<int> items;
    Flatten(i, &items);
    std::string s;
    for (int it : items) {
      int c = LitChar(nodes[it]);
      if (c < 0 || s.size() >= kMaxAnchorLit) break;
      s.push_back(char(c));
    }
    return s;
  }
};

struct Cand {
  std::vector<std::string> lits;
  int64_t olo, ohi;
  int64_t ohi_fold = 0;
  std::vector<std::vector<int>> follow;  // per literal: flattened items after it
  std::vector<std::vector<int>> lit_nodes;  // per literal: the class nodes of its chars
  size_t pre_k = 0;                          // top-level flattened items before the literal(s)
  std::vector<std::pair<std::string, std::vector<int>>> variants;  // every branch literal before dedupe
  bool class_run = false;  // ExtractClassRun: a run of one-byte classes, not a literal
  size_t minlen() const {
    size_t m = SIZE_MAX;
    for (auto& l : lits) m = std::min(m, l.size());
    return m;
  }
};

bool ExtractAnchor(const Regex& re, Cand* best, bool need_offset = true) {
  Analyzer an(re.nodes(), false), anf(re.nodes(), true);
  std::vector<int> items;
  an.Flatten(re.root(), &items);
  std::vector<Cand> cands;
  int64_t olo = 0, ohi = 0, ohf = 0;
  auto tail = [&](size_t from) { return std::vector<int>(items.begin() + long(from), items.end()); };
  for (size_t k = 0; k < items.size();) {
    const Node& n = re.nodes()[items[k]];
    int c = LitChar(n);
    if (c >= 0) {
      std::string s;
      size_t j = k;
      while (j < items.size()) {
        int cj = LitChar(re.nodes()[items[j]]);
        if (cj < 0) break;
        s.push_back(char(cj));
        j++;
      }
      if (ohi < kInf || !need_offset) {
        // an anchor literal is at most kMaxAnchorLit chars: the rest of a
        // longer run stays in the follow sequence (the prefilter item and
        // the fold kernel's window assume short items)
        const size_t jl = std::min(j, k + kMaxAnchorLit);
        Cand cd{{s.substr(0, jl - k)}, olo, ohi};
        cd.ohi_fold = ohf;
        cd.follow.push_back(tail(jl));
        cd.lit_nodes.push_back(std::vector<int>(items.begin() + long(k), items.begin() + long(jl)));
        cd.pre_k = k;
        cands.push_back(cd);
      }
      // the literal chars themselves are 1 byte each normally, up to 3 when folded
      int64_t fb = 0;
      for (size_t q = k; q < j; q++) fb += anf.Bytes(items[q]).second;
      olo += int64_t(s.size());
      if (ohi < kInf) ohi += int64_t(s.size());
      if (ohf < kInf) ohf += fb;
      k = j;
      continue;
    }
    int alt = -1;
    if (n.op == NodeOp::Alt) alt = items[k];
    if (n.op == NodeOp::Repeat && n.min >= 1) {
      int sub = n.subs[0];
      while (re.nodes()[sub].op == NodeOp::Capture) sub = re.nodes()[sub].subs[0];
      if (re.nodes()[sub].op == NodeOp::Alt) alt = -2 - sub;  // alternation inside a repeat: no lookahead
      else {
        std::string s = an.LeadLiteral(sub);
        if (!s.empty() && (ohi < kInf || !need_offset)) {
          Cand cd{{s}, olo, ohi};
          cd.ohi_fold = ohf;
          cd.follow.push_back({});
          cd.lit_nodes.push_back(an.LeadNodes(sub));
          cd.pre_k = k;
          cands.push_back(cd);
        }
      }
    }
    if (alt != -1 && (ohi < kInf || !need_offset)) {
      bool in_repeat = alt <= -2;
      int an_node = in_repeat ? -2 - alt : alt;
      Cand cd{{}, olo, ohi};
      cd.ohi_fold = ohf;
      cd.pre_k = k;
      bool ok = true;
      for (int b : re.nodes()[an_node].subs) {
        std::string s = an.LeadLiteral(b);
        if (s.empty()) { ok = false; break; }
        cd.lits.push_back(s);
        cd.lit_nodes.push_back(an.LeadNodes(b));
        std::vector<int> bi;
        an.Flatten(b, &bi);
        std::vector<int> fol;
        if (!in_repeat) {
          fol.assign(bi.begin() + long(s.size()), bi.end());
          auto t = tail(k + 1);
          fol.insert(fol.end(), t.begin(), t.end());
        }
        cd.follow.push_back(fol);
      }
      if (ok) cands.push_back(cd);
    }
    auto b = an.Bytes(items[k]);
    auto bf = anf.Bytes(items[k]);
    olo += b.first;
    ohi = (ohi >= kInf || b.second >= kInf) ? kInf : ohi + b.second;
    ohf = (ohf >= kInf || bf.second >= kInf) ? kInf : ohf + bf.second;
    k++;
  }
  bool have = false;
  for (auto& cd : cands) {
    // dedupe literals (keep the first follow list of each)
    std::vector<std::string> L;
    std::vector<std::vector<int>> F, N;
    for (size_t i = 0; i < cd.lits.size(); i++) {
      cd.variants.push_back({cd.lits[i], cd.lit_nodes[i]});
      auto it = std::find(L.begin(), L.end(), cd.lits[i]);
      if (it != L.end()) {  // same case-folded literal in two branches: keep no lookahead
        size_t at = size_t(it - L.begin());
        if (F[at] != cd.follow[i]) F[at].clear();
        continue;
      }
      L.push_back(cd.lits[i]);
      F.push_back(cd.follow[i]);
      N.push_back(cd.lit_nodes[i]);
    }
    cd.lits = L;
    cd.follow = F;
    cd.lit_nodes = N;
    if (!have || cd.minlen() > best->minlen() ||
        (cd.minlen() == best->minlen() && cd.lits.size() < best->lits.size())) {
      *best = cd;
      have = true;
    }
  }
  return have && best->minlen() >= 2;
}

bool ExactSet(const Node& n, ByteSet* out);

// Anchor for a rule with no required literal (else it would run in full-scan
// mode over every file with an open gate): the rarest run of fixed one-byte
// positions -- classes with an exact byte set (ASCII members, fold-only runes
// left to the fold kernel) and fixed repeats of them -- at a bounded offset,
// e.g. [g-z]{3}[0-9]{3}[._-] in `\b[g-z]{3}[0-9]{3}[._-][a-z0-9]{16}\b`.  Every
// match holds the run at [olo, ohi], exactly as for a literal anchor (the
// prefilter items are byte sets either way).  Taken only when its least
// likely 6-position window is below kClassRunMaxProb (printable-uniform prior);
// a commoner run would cost more than the gated full scans.
constexpr double kClassRunMaxProb = 1e-5;
// with a calibration sample (CompileOptions) a rule with a literal anchor also
// considers class runs up to this prior probability: the sample decides
constexpr double kClassRunCalibProb = 1e-3;
// every_run (calibration): each run under max_prob that is not simply a literal
// (a run of literal characters is the literal anchor's business), by prior
bool ExtractClassRun(const Regex& re, Cand* best, double max_prob = kClassRunMaxProb,
                     std::vector<std::pair<double, Cand>>* every_run = nullptr) {
  const std::vector<Node>& nodes = re.nodes();
  Analyzer an(nodes, false), anf(nodes, true);
  std::vector<int> items;
  an.Flatten(re.root(), &items);
  auto prob = [](const ByteSet& b) {
    int n = 0;
    for (int c = 0x20; c < 0x7F; c++) n += b.test(size_t(c));
    n += b.test('\n') + b.test('\t');
    return double(n) / 97.0;
  };
  int64_t olo = 0, ohi = 0, ohf = 0;
  double best_p = max_prob;
  bool have = false;
  for (size_t k = 0; k < items.size() && ohi < kInf; k++) {
    std::vector<int> pos;
    std::vector<double> ps;
    size_t j = k;
    while (j < items.size() && pos.size() < kMaxAnchorLit) {
      const Node& n = nodes[items[j]];
      ByteSet b;
      if (n.op == NodeOp::Class && ExactSet(n, &b)) {
        pos.push_back(items[j]);
        ps.push_back(prob(b));
        j++;
        continue;
      }
      if (n.op == NodeOp::Repeat && n.min >= 1 && n.max == n.min) {
        int sub = n.subs[0];
        while (nodes[sub].op == NodeOp::Capture) sub = nodes[sub].subs[0];
        if (nodes[sub].op == NodeOp::Class && ExactSet(nodes[sub], &b) &&
            pos.size() + size_t(n.min) <= kMaxAnchorLit) {
          for (int m = 0; m < n.min; m++) {
            pos.push_back(sub);
            ps.push_back(prob(b));
          }
          j++;
          continue;
        }
      }
      break;
    }
    if (pos.size() >= 3) {
      double p_run = 1.0;  // the least likely window of <= 6 positions (what the prefilter keeps)
      const size_t wl = std::min<size_t>(pos.size(), 6);
      for (size_t a = 0; a + wl <= pos.size(); a++) {
        double pw = 1.0;
        for (size_t q = a; q < a + wl; q++) pw *= ps[q];
        p_run = a == 0 ? pw : std::min(p_run, pw);
      }
      auto make = [&]() {
        Cand cd{{std::string(pos.size(), '\x01')}, olo, ohi};
        cd.ohi_fold = ohf;
        cd.follow.push_back(std::vector<int>(items.begin() + long(j), items.end()));
        cd.lit_nodes.push_back(pos);
        cd.pre_k = k;
        cd.variants.push_back({cd.lits[0], pos});
        cd.class_run = true;
        return cd;
      };
      if (every_run && p_run < max_prob) {
        bool literal = true;
        for (size_t q = k; q < j && literal; q++) literal = LitChar(nodes[items[q]]) >= 0;
        if (!literal) every_run->push_back({p_run, make()});
      }
      if (p_run < best_p) {
        best_p = p_run;
        *best = make();
        have = true;
      }
    }
    auto b = an.Bytes(items[k]);
    auto bf = anf.Bytes(items[k]);
    olo += b.first;
    ohi = (ohi >= kInf || b.second >= kInf) ? kInf : ohi + b.second;
    ohf = (ohf >= kInf || bf.second >= kInf) ? kInf : ohf + bf.second;
  }
  return have;
}

// ---------------------------------------------------------------------------
// relaxed class-sequence NFA
// ---------------------------------------------------------------------------
using Reach = std::bitset<256>;

Reach ByteReach(const RuneRanges& rr) {
  Reach r;
  for (uint32_t b = 0; b < 0x80; b++)
    if (ClassHas(rr, b)) r.set(b);
  bool fffd = ClassHas(rr, 0xFFFD);
  auto any_in = [&](uint32_t lo, uint32_t hi) {
    for (auto& p : rr)
      if (p.first <= hi && p.second >= lo) return true;
    return false;
  };
  for (uint32_t b = 0x80; b < 0x100; b++) {
    bool on = fffd;  // invalid byte -> U+FFFD
    if (b >= 0xC2 && b <= 0xDF) on = on || any_in((b & 0x1F) << 6, ((b & 0x1F) << 6) | 0x3F);
    else if (b >= 0xE0 && b <= 0xEF) on = on || any_in((b & 0x0F) << 12, ((b & 0x0F) << 12) | 0xFFF);
    else if (b >= 0xF0 && b <= 0xF4) on = on || any_in((b & 0x07) << 18, ((b & 0x07) << 18) | 0x3FFFF);
    if (on) r.set(b);
  }
  return r;
}

struct Elem {
  Reach reach;
  int64_t min, max;  // max < 0: unbounded
};

int64_t SeqMin(const std::vector<Elem>& s) {
  int64_t m = 0;
  for (auto& e : s) m += e.min;
  return m;
}
int64_t SeqMax(const std::vector<Elem>& s) {
  int64_t m = 0;
  for (auto& e : s) {
    if (e.max < 0) return -1;
    m += e.max;
  }
  return m;
}
Reach SeqUnion(const std::vector<Elem>& s) {
  Reach r;
  for (auto& e : s) r |= e.reach;
  return r;
}

std::vector<Elem> Relax(const std::vector<Node>& nodes, int i) {
  const Node& n = nodes[i];
  switch (n.op) {
    case NodeOp::Empty:
    case NodeOp::NoMatch:
    case NodeOp::Assert: return {};
    case NodeOp::Class: return {{ByteReach(n.ranges), 1, 1}};
    case NodeOp::Capture: return Relax(nodes, n.subs[0]);
    case NodeOp::Cat: {
      std::vector<Elem> out;
      for (int s : n.subs) {
        auto r = Relax(nodes, s);
        out.insert(out.end(), r.begin(), r.end());
      }
      return out;
    }
    case NodeOp::Alt: {
      std::vector<std::vector<Elem>> br;
      for (int s : n.subs) br.push_back(Relax(nodes, s));
      bool columns = true;
      for (auto& b : br) {
        if (b.size() != br[0].size()) columns = false;
        for (auto& e : b)
          if (e.min != 1 || e.max != 1) columns = false;
      }
      if (columns && !br[0].empty()) {
        std::vector<Elem> out = br[0];
        for (size_t k = 1; k < br.size(); k++)
          for (size_t j = 0; j < out.size(); j++) out[j].reach |= br[k][j].reach;
        return out;
      }
      Elem e{Reach(), kInf, 0};
      for (auto& b : br) {
        e.reach |= SeqUnion(b);
        e.min = std::min(e.min, SeqMin(b));
        int64_t mx = SeqMax(b);
        if (mx < 0 || e.max < 0) e.max = -1;
        else e.max = std::max(e.max, mx);
      }
      if (e.max == 0) return {};
      return {e};
    }
    case NodeOp::Repeat: {
      auto s = Relax(nodes, n.subs[0]);
      if (s.empty()) return {};
      if (s.size() == 1) {
        Elem e = s[0];
        e.min = e.min * n.min;
        e.max = (n.max < 0 || e.max < 0) ? -1 : e.max * n.max;
        if (e.max == 0) return {};
        return {e};
      }
      if (n.max == 0) return {};
      std::vector<Elem> out;
      if (n.min >= 1) out = s;
      Elem rest{SeqUnion(s), SeqMin(s) * std::max(0, n.min - 1), -1};
      int64_t smax = SeqMax(s);
      if (n.max >= 0 && smax >= 0) rest.max = smax * (n.min >= 1 ? n.max - 1 : n.max);
      if (n.min == 0) rest.min = 0;
      if (rest.max != 0) out.push_back(rest);
      return out;
    }
  }
  return {};
}

int64_t Positions(const Elem& e) { return e.max >= 0 ? e.max : std::max<int64_t>(e.min, 1); }

// Shrinks a relaxed sequence to at most `budget` NFA positions, keeping it a
// superset: the largest element is relaxed first (X{m,n} -> X{m,}, then
// X{m,} -> X{m/2,}); once every element is a single position, the last two
// elements merge into one [X|Y]{0,} (X{a,b}Y{c,d} is inside it), so every
// round strictly lowers the element count or the position total.
void FitPositions(std::vector<Elem>* seq_p, int64_t budget) {
  std::vector<Elem>& seq = *seq_p;
  for (;;) {
    int64_t tot = 0;
    for (auto& e : seq) tot += Positions(e);
    if (tot <= budget || seq.empty()) break;
    size_t big = 0;
    for (size_t k = 1; k < seq.size(); k++)
      if (Positions(seq[k]) > Positions(seq[big])) big = k;
    Elem& e = seq[big];
    if (Positions(e) > 1) {
      if (e.max >= 0 && e.max > e.min) e.max = -1;
      else { e.min = e.min / 2; e.max = -1; }
      continue;
    }
    Elem m{seq[seq.size() - 2].reach | seq.back().reach, 0, -1};
    seq.pop_back();
    seq.back() = m;
  }
}

void BuildNfa(std::vector<Elem> seq, std::vector<uint64_t>* nfa, RuleGpu* rg) {
  // A relaxed language holding the empty string: the kernels only accept after
  // a byte, so such a rule makes every (anchor hit / file) a candidate instead
  // (Go reports empty matches too; the exact pass finds them).
  const bool nullable = SeqMin(seq) == 0;
  FitPositions(&seq, 64 * kMaxNfaWords);  // fit into kMaxNfaWords * 64 positions
  int64_t P = 0;
  for (auto& e : seq) P += Positions(e);
  rg->nfa_off = uint32_t(nfa->size());
  if (P == 0 || nullable) {
    rg->nfa_words = 0;
    return;
  }
  int W = int((P + 63) / 64);
  rg->nfa_words = uint8_t(W);
  std::vector<uint64_t> O(W, 0), L(W, 0), F(W, 0), B(256 * W, 0);
  auto setb = [&](std::vector<uint64_t>& v, int64_t p) { v[p >> 6] |= uint64_t(1) << (p & 63); };
  int64_t p = 0;
  std::vector<bool> opt(P, false);
  for (auto& e : seq) {
    int64_t np = Positions(e);
    for (int64_t j = 0; j < np; j++, p++) {
      for (int b = 0; b < 256; b++)
        if (e.reach.test(b)) B[size_t(b) * W + (p >> 6)] |= uint64_t(1) << (p & 63);
      if (e.max >= 0) {
        if (j >= e.min) { setb(O, p); opt[p] = true; }
      } else {
        if (j == np - 1) setb(L, p);
        if (e.min == 0) { setb(O, p); opt[p] = true; }
      }
    }
  }
  setb(F, P - 1);
  for (int64_t q = P - 1; q >= 1 && opt[q]; q--) setb(F, q - 1);
  nfa->insert(nfa->end(), O.begin(), O.end());
  nfa->insert(nfa->end(), L.begin(), L.end());
  nfa->insert(nfa->end(), F.begin(), F.end());
  nfa->insert(nfa->end(), B.begin(), B.end());
}

std::string AsciiLower(const std::string& s) {
  std::string o = s;
  for (auto& c : o)
    if (c >= 'A' && c <= 'Z') c = char(c + 32);
  return o;
}

bool IsAscii(const std::string& s) {
  for (unsigned char c : s)
    if (c >= 0x80) return false;
  return true;
}

// ---------------------------------------------------------------------------
// prefilter items
// ---------------------------------------------------------------------------
// Byte set of a single-rune class as it can match in a file without fold
// runes: its ASCII members.  False when the class has another non-ASCII member
// (then the position's byte width is not fixed).
bool ExactSet(const Node& n, ByteSet* out) {
  if (n.op != NodeOp::Class) return false;
  ByteSet s;
  for (auto& p : n.ranges) {
    for (uint32_t c = p.first; c <= p.second && c < 0x80; c++) s.set(c);
    if (p.second >= 0x80) {
      uint32_t a = std::max<uint32_t>(p.first, 0x80);
      if (p.second - a > 0x10000) return false;
      for (uint32_t c = a; c <= p.second; c++)
        if (!IsFoldOnlyRune(c)) return false;
    }
  }
  if (s.none()) return false;
  *out = s;
  return true;
}

// The fixed-width byte-set sequence of a node, if it has one (classes, fixed
// repeats of them, concatenations, and alternations whose branches are such
// sequences of one length -- the position-wise union).  `cap` bounds its length.
bool FixedSets(const std::vector<Node>& nodes, int i, std::vector<ByteSet>* out, size_t cap) {
  const Node& n = nodes[i];
  switch (n.op) {
    case NodeOp::Empty:
    case NodeOp::Assert: return true;
    case NodeOp::Class: {
      ByteSet b;
      if (!ExactSet(n, &b) || out->size() >= cap) return false;
      out->push_back(b);
      return true;
    }
    case NodeOp::Capture: return FixedSets(nodes, n.subs[0], out, cap);
    case NodeOp::Cat:
      for (int s : n.subs)
        if (!FixedSets(nodes, s, out, cap)) return false;
      return true;
    case NodeOp::Repeat: {
      if (n.max != n.min || n.min < 0) return false;
      for (int r = 0; r < n.min; r++)
        if (!FixedSets(nodes, n.subs[0], out, cap)) return false;
      return true;
    }
    case NodeOp::Alt: {
      std::vector<ByteSet> u;
      bool first = true;
      for (int s : n.subs) {
        std::vector<ByteSet> b;
        if (!FixedSets(nodes, s, &b, cap)) return false;
        if (first) u = b;
        else if (b.size() != u.size()) return false;
        else
          for (size_t k = 0; k < u.size(); k++) u[k] |= b[k];
        first = false;
      }
      if (out->size() + u.size() > cap) return false;
      out->insert(out->end(), u.begin(), u.end());
      return true;
    }
    default: return false;
  }
}

// Byte sets at the first offsets after a literal, for any match: first the
// exact (ASCII) sets of whole fixed-width items, then "continuation sets" from
// the relaxed NFA of the remaining items -- offset i's set is the union of the
// byte reaches of the positions the NFA can be in after i bytes.  A continuation
// byte (0x80-0xBF) keeps the state (as in the NFA) and once the match may have
// ended the offset is unconstrained, so every match satisfies every set: a
// superset filter.  Trailing all-byte sets are dropped.
std::vector<ByteSet> AfterSets(const std::vector<Node>& nodes, const std::vector<int>& fol, size_t cap) {
  std::vector<ByteSet> out;
  size_t k = 0;
  for (; k < fol.size() && out.size() < cap; k++) {
    std::vector<ByteSet> b;
    if (!FixedSets(nodes, fol[k], &b, cap - out.size())) break;
    out.insert(out.end(), b.begin(), b.end());
  }
  if (out.size() < cap && k < fol.size()) {
    // expand the relaxed sequence into NFA positions (as BuildNfa): a run
    // {min,max} gives min mandatory + (max-min) optional positions; an
    // unbounded one max(min,1) positions, the last looping
    struct P {
      Reach r;
      bool opt, loop;
    };
    std::vector<P> pos;
    const size_t kMaxPos = 4 * cap + 8;  // enough to reach `cap` offsets; beyond: unconstrained
    bool truncated = false;
    for (size_t q = k; q < fol.size() && !truncated; q++)
      for (const Elem& e : Relax(nodes, fol[q])) {
        const int64_t np = Positions(e);
        for (int64_t j = 0; j < np; j++) {
          if (pos.size() >= kMaxPos) {
            truncated = true;
            break;
          }
          P x{e.reach, false, false};
          if (e.max >= 0) x.opt = j >= e.min;
          else {
            x.opt = e.min == 0;
            x.loop = j == np - 1;
          }
          pos.push_back(x);
        }
        if (truncated) break;
      }
    const size_t n = pos.size();  // index n = end of the (possibly truncated) sequence
    std::vector<bool> act(n + 1, false);
    auto activate = [&](std::vector<bool>& a, size_t i) {  // i and the optional positions after it
      while (i <= n) {
        a[i] = true;
        if (i == n || !pos[i].opt) break;
        i++;
      }
    };
    activate(act, 0);
    Reach cont;
    for (int c = 0x80; c < 0xC0; c++) cont.set(size_t(c));
    while (out.size() < cap) {
      if (act[n]) break;  // the match may end here: nothing after is constrained
      Reach set;
      for (size_t i = 0; i < n; i++)
        if (act[i]) set |= pos[i].r;
      if (set.all() || set.none()) break;
      out.push_back(set);
      std::vector<bool> nx(n + 1, false);
      const bool keep = (set & cont).any();
      for (size_t i = 0; i < n; i++) {
        if (!act[i]) continue;
        if (keep) nx[i] = true;
        if (pos[i].loop) nx[i] = true;
        activate(nx, i + 1);
      }
      act.swap(nx);
    }
  }
  while (!out.empty() && out.back().all()) out.pop_back();
  if (out.size() > cap) out.resize(cap);
  return out;
}

// Byte sets at the first offsets after a literal, from a Glushkov position
// automaton of the items after it (Alt branches and optional groups kept
// apart, repeats unrolled up to the offsets asked for), so offset i's set is
// the union of the reaches of the positions some path can be in after i bytes
// -- e.g. after "aws" in aws_?(sec(ret)?)?_?(access)?_?key offset 1 allows
// _ s a k e c, where the relaxed sequence of AfterSets allows every letter of
// the optional words at each offset.  Still a superset filter: assertions are
// ε, positions are exact ASCII sets (fold-only runes left to the fold kernel,
// as ExactSet) or byte reaches, the sets stop after an offset that admits a
// byte >= 0x80 (a multi-byte rune's continuation bytes would follow) or once
// the match may have ended.  Empty when the expansion grows past its budget.
std::vector<ByteSet> AfterSetsExact(const std::vector<Node>& nodes, const std::vector<int>& fol, size_t cap) {
  struct Pos {
    ByteSet reach;
    std::vector<int> next;
  };
  std::vector<Pos> pos;
  struct Frag {
    std::vector<int> first, last;
    bool nullable;
  };
  constexpr size_t kBudget = 4096;
  const int kCopies = int(cap) + 1;  // repeats beyond this many copies only shape offsets >= cap
  bool over = false;
  auto link = [&](const std::vector<int>& from, const std::vector<int>& to) {
    for (int a : from)
      for (int b : to) pos[size_t(a)].next.push_back(b);
  };
  auto cat = [&](Frag a, const Frag& b) {
    link(a.last, b.first);
    Frag r;
    r.first = a.first;
    if (a.nullable) r.first.insert(r.first.end(), b.first.begin(), b.first.end());
    r.last = b.last;
    if (b.nullable) r.last.insert(r.last.end(), a.last.begin(), a.last.end());
    r.nullable = a.nullable && b.nullable;
    return r;
  };
  std::function<Frag(int)> build = [&](int i) -> Frag {
    const Node& n = nodes[size_t(i)];
    if (over) return Frag{{}, {}, true};
    switch (n.op) {
      case NodeOp::Empty:
      case NodeOp::Assert: return Frag{{}, {}, true};
      case NodeOp::NoMatch: return Frag{{}, {}, false};
      case NodeOp::Class: {
        if (pos.size() >= kBudget) {
          over = true;
          return Frag{{}, {}, true};
        }
        ByteSet b;
        if (!ExactSet(n, &b)) b = ByteReach(n.ranges);
        pos.push_back(Pos{b, {}});
        const int p = int(pos.size()) - 1;
        return Frag{{p}, {p}, false};
      }
      case NodeOp::Capture: return build(n.subs[0]);
      case NodeOp::Cat: {
        Frag r{{}, {}, true};
        for (int s : n.subs) r = cat(r, build(s));
        return r;
      }
      case NodeOp::Alt: {
        Frag r{{}, {}, false};
        for (int s : n.subs) {
          Frag b = build(s);
          r.first.insert(r.first.end(), b.first.begin(), b.first.end());
          r.last.insert(r.last.end(), b.last.begin(), b.last.end());
          r.nullable = r.nullable || b.nullable;
        }
        return r;
      }
      case NodeOp::Repeat: {
        const int mn = std::min(n.min, kCopies);
        const bool star = n.max < 0 || n.max - n.min > kCopies;
        const int opt = star ? 0 : n.max - n.min;
        Frag r{{}, {}, true};
        for (int k = 0; k < mn; k++) r = cat(r, build(n.subs[0]));
        for (int k = 0; k < opt; k++) {
          Frag o = build(n.subs[0]);
          o.nullable = true;
          r = cat(r, o);
        }
        if (star) {
          Frag o = build(n.subs[0]);
          link(o.last, o.first);
          o.nullable = true;
          r = cat(r, o);
        }
        return r;
      }
    }
    return Frag{{}, {}, true};
  };
  Frag seq{{}, {}, true};
  for (int it : fol) seq = cat(seq, build(it));
  std::vector<ByteSet> out;
  if (over) return out;
  std::vector<char> is_last(pos.size(), 0);
  for (int p : seq.last) is_last[size_t(p)] = 1;
  std::vector<char> act(pos.size(), 0);
  for (int p : seq.first) act[size_t(p)] = 1;
  bool ended = seq.nullable;  // the match may end at this offset
  while (out.size() < cap && !ended) {
    ByteSet set;
    bool any = false;
    for (size_t p = 0; p < pos.size(); p++)
      if (act[p]) {
        set |= pos[p].reach;
        any = true;
      }
    if (!any || set.all() || set.none()) break;
    out.push_back(set);
    bool high = false;
    for (int b = 0x80; b < 0x100 && !high; b++) high = set.test(size_t(b));
    if (high) break;
    std::vector<char> nx(pos.size(), 0);
    for (size_t p = 0; p < pos.size(); p++) {
      if (!act[p]) continue;
      if (is_last[p]) ended = true;
      for (int q : pos[p].next) nx[size_t(q)] = 1;
    }
    act.swap(nx);
  }
  while (!out.empty() && out.back().all()) out.pop_back();
  return out;
}

// Mandatory fixed-width sets right before top-level item `k` (up to `cap`).
std::vector<ByteSet> BeforeSets(const std::vector<Node>& nodes, const std::vector<int>& items, size_t k, size_t cap) {
  std::vector<ByteSet> out;  // reversed
  for (size_t q = k; q-- > 0;) {
    std::vector<ByteSet> b;
    if (!FixedSets(nodes, items[q], &b, 64)) break;
    for (size_t r = b.size(); r-- > 0 && out.size() < cap;) out.push_back(b[r]);
    if (out.size() >= cap) break;
  }
  std::reverse(out.begin(), out.end());
  return out;
}

// Follow requirements (rules.h AnchorReq) from the relaxed element sequence of
// the items after an anchor literal.  A candidate run starts at a mandatory
// element j (min >= 1) whose preceding elements have a bounded total length;
// it holds j's mandatory positions and continues into the next elements while
// they are fixed-length.  The (at most two, disjoint) runs with the fewest
// expected chance occurrences over their offset range (static byte prior)
// are kept.
FollowLut FollowReqs(const std::vector<Node>& nodes, const std::vector<int>& fol) {
  FollowLut rq{};
  for (int s = 0; s < 8; s++) {  // unused slots accept every ASCII byte
    for (auto& x : rq.lo_tab) x |= uint8_t(1u << s);
    for (auto& x : rq.hi_tab) x |= uint8_t(1u << s);
  }
  std::vector<Elem> seq;
  for (int it : fol) {
    auto r = Relax(nodes, it);
    seq.insert(seq.end(), r.begin(), r.end());
  }
  const auto& prior = BytePrior();
  struct Run {
    int64_t lo, hi;
    size_t j0, j1;  // elements covered [j0, j1)
    std::vector<Reach> sets;
    double score;
  };
  std::vector<Run> runs;
  int64_t lo = 0, hi = 0;
  for (size_t j = 0; j < seq.size() && hi < kInf; j++) {
    if (seq[j].min >= 1 && hi <= 48) {
      Run r{lo, hi, j, j, {}, 0};
      for (size_t k = j; k < seq.size() && r.sets.size() < size_t(kMaxReqLen); k++) {
        const Elem& e = seq[k];
        if (e.min < 1) break;
        for (int64_t c = 0; c < e.min && r.sets.size() < size_t(kMaxReqLen); c++) r.sets.push_back(e.reach);
        r.j1 = k + 1;
        if (e.max != e.min) break;  // the next element's offset is no longer fixed
      }
      double p = 1.0;
      for (auto& s : r.sets) {
        double q = 0;
        for (int b = 0; b < 0x80; b++)
          if (s.test(size_t(b))) q += prior[size_t(b)];
        p *= q;
      }
      r.score = double(hi - lo + 1) * p;
      if (r.score < 1.0 && hi + int64_t(r.sets.size()) <= kReqSpan) runs.push_back(r);
    }
    lo += seq[j].min;
    hi = (seq[j].max < 0 || hi >= kInf) ? kInf : hi + seq[j].max;
  }
  std::sort(runs.begin(), runs.end(), [](const Run& a, const Run& b) { return a.score < b.score; });
  int nr = 0;
  std::vector<std::pair<size_t, size_t>> used;
  for (auto& r : runs) {
    bool overlap = false;
    for (auto& u : used)
      if (r.j0 < u.second && u.first < r.j1) overlap = true;
    if (overlap) continue;
    used.push_back({r.j0, r.j1});
    rq.lo[nr] = uint8_t(r.lo);
    rq.hi[nr] = uint8_t(r.hi);
    rq.n[nr] = uint8_t(r.sets.size());
    for (size_t k = 0; k < r.sets.size(); k++) {
      const uint8_t bit = uint8_t(1u << (4 * nr + int(k)));
      for (auto& x : rq.lo_tab) x &= uint8_t(~bit);
      for (auto& x : rq.hi_tab) x &= uint8_t(~bit);
      for (int b = 0; b < 0x80; b++)
        if (r.sets[k].test(size_t(b))) {
          rq.lo_tab[b & 15] |= bit;
          rq.hi_tab[b >> 4] |= bit;
        }
    }
    if (++nr == kMaxReqs) break;
  }
  return rq;
}

}  // namespace

// Every match contains one of `kws` (lowercased ASCII), case-folded: found in
// a required literal run, or in every branch of a required alternation (or
// small class) together with the literal runs around it.  With long_s_ok a
// (?i) 's' may be matched by U+017F (files holding it are checked exactly);
// otherwise such positions do not count (bytes.ToLower keeps U+017F).
bool KeywordsImplied(const Regex& re, const std::vector<std::string>& kws, bool long_s_ok) {
  for (auto& kw : kws)
    if (kw.empty()) return true;
  Analyzer an(re.nodes(), false);
  const auto& nodes = re.nodes();
  struct Ch {
    char c;
    bool hz;  // U+017F in the class
  };
  auto ch_of = [&](int it) { return Ch{char(LitChar(nodes[it])), ClassHas(nodes[it].ranges, 0x17F)}; };
  auto contains = [&](const std::vector<Ch>& s) {
    for (auto& kw : kws)
      for (size_t o = 0; o + kw.size() <= s.size(); o++) {
        bool ok = true;
        for (size_t i = 0; i < kw.size() && ok; i++)
          if (s[o + i].c != kw[i] || (kw[i] == 's' && s[o + i].hz && !long_s_ok)) ok = false;
        if (ok) return true;
      }
    return false;
  };
  // branch alternatives as char sequences: the lead literal run, and whether it is the whole branch
  auto lead = [&](int node, bool* whole) {
    std::vector<int> items;
    an.Flatten(node, &items);
    std::vector<Ch> run;
    size_t i = 0;
    for (; i < items.size() && LitChar(nodes[items[i]]) >= 0; i++) run.push_back(ch_of(items[i]));
    *whole = i == items.size();
    return run;
  };
  std::vector<int> items;
  an.Flatten(re.root(), &items);
  auto lit_run = [&](size_t from, size_t to) {  // literal chars items[from, to)
    std::vector<Ch> r;
    for (size_t q = from; q < to; q++) r.push_back(ch_of(items[q]));
    return r;
  };
  for (size_t k = 0; k < items.size(); k++) {
    if (LitChar(nodes[items[k]]) >= 0) {
      size_t e = k;
      while (e < items.size() && LitChar(nodes[items[e]]) >= 0) e++;
      if (contains(lit_run(k, e))) return true;
      k = e - 1;
      continue;
    }
    // the literal runs right before and after items[k]
    size_t pb = k;
    while (pb > 0 && LitChar(nodes[items[pb - 1]]) >= 0) pb--;
    size_t ne = k + 1;
    while (ne < items.size() && LitChar(nodes[items[ne]]) >= 0) ne++;
    const std::vector<Ch> before = lit_run(pb, k), after = lit_run(k + 1, ne);
    std::vector<std::vector<Ch>> alts;  // per alternative: its chars; `after` appended when whole
    const Node& n = nodes[items[k]];
    int alt = -1;
    if (n.op == NodeOp::Alt) alt = items[k];
    if (n.op == NodeOp::Repeat && n.min >= 1) {
      int sub = n.subs[0];
      while (nodes[sub].op == NodeOp::Capture) sub = nodes[sub].subs[0];
      if (nodes[sub].op == NodeOp::Alt) alt = sub;
      else {
        bool whole;
        std::vector<Ch> r = lead(sub, &whole);
        if (contains(r)) return true;
      }
    }
    if (alt >= 0) {
      for (int b : nodes[alt].subs) {
        bool whole;
        std::vector<Ch> r = before;
        std::vector<Ch> l = lead(b, &whole);
        r.insert(r.end(), l.begin(), l.end());
        if (whole && n.op == NodeOp::Alt) r.insert(r.end(), after.begin(), after.end());
        alts.push_back(r);
      }
    } else if (n.op == NodeOp::Class) {  // a small class: one alternative per case-folded char
      std::vector<char> cs;
      uint64_t total = 0;
      for (auto& p : n.ranges) {
        total += uint64_t(p.second - p.first) + 1;
        if (total > 16) break;
        for (uint32_t c = p.first; c <= p.second && c < 0x80; c++) {
          char lc = char((c >= 'A' && c <= 'Z') ? c + 32 : c);
          if (std::find(cs.begin(), cs.end(), lc) == cs.end()) cs.push_back(lc);
        }
      }
      if (total <= 16 && !cs.empty()) {
        bool nonascii = false;
        for (auto& p : n.ranges)
          if (p.second >= 0x80) nonascii = true;
        if (!nonascii)
          for (char c : cs) {
            std::vector<Ch> r = before;
            r.push_back(Ch{c, false});
            r.insert(r.end(), after.begin(), after.end());
            alts.push_back(r);
          }
      }
    }
    if (!alts.empty()) {
      bool all = true;
      for (auto& r : alts)
        if (!contains(r)) {
          all = false;
          break;
        }
      if (all) return true;
    }
  }
  return false;
}

bool KeywordImplied(const Regex& re, const std::string& kw) { return KeywordsImplied(re, {kw}, false); }

std::vector<std::string> RequiredLiterals(const Regex& re) {
  Cand best{{}, 0, 0};
  if (!ExtractAnchor(re, &best, false)) return {};
  return best.lits;
}

namespace {

// The prefilter item of anchor literal li of `best`: the sets before it, the
// literal's sets (the union over same-folded variants), the lookahead sets.
FilterItem AnchorItem(const Regex& re, const Cand& best, size_t li, uint32_t aid) {
  const std::string& l = best.lits[li];
  FilterItem fi;
  fi.kind = kItemAnchor;
  fi.id = aid;
  std::vector<int> top;
  Analyzer(re.nodes(), false).Flatten(re.root(), &top);
  fi.sets = BeforeSets(re.nodes(), top, best.pre_k, 16);
  std::vector<ByteSet> lit(l.size());
  for (auto& v : best.variants) {
    if (v.first != l) continue;
    for (size_t q = 0; q < l.size() && q < v.second.size(); q++) {
      ByteSet b;
      if (ExactSet(re.nodes()[v.second[q]], &b)) lit[q] |= b;
      else lit[q].set();
    }
  }
  for (auto& b : lit)
    if (b.none()) b.set();
  fi.sets.insert(fi.sets.end(), lit.begin(), lit.end());
  fi.lit_end = uint32_t(fi.sets.size());
  // the tighter of the two lookahead computations, position by position
  // (both are supersets of every match's bytes; the exact one stops
  // early on non-ASCII sets, the relaxed one on ended fixed items)
  auto after = AfterSets(re.nodes(), best.follow[li], 16);
  const auto exact = AfterSetsExact(re.nodes(), best.follow[li], 16);
  for (size_t q = 0; q < exact.size(); q++) {
    if (q < after.size()) after[q] &= exact[q];
    else after.push_back(exact[q]);
  }
  fi.sets.insert(fi.sets.end(), after.begin(), after.end());
  return fi;
}

uint32_t FilterWindow() {
  const char* e = std::getenv("TSG_FILTER_WINDOW");  // model experiments
  return e ? uint32_t(std::atoi(e)) : 6u;
}

// What an item costs on a calibration sample: the positions where its
// prefilter window matches (K1 fires, each a flagged block for K2) plus those
// where the whole item does (K2's exact anchor-item matches).
uint64_t SampleCost(const FilterItem& it, const uint8_t* a, uint64_t n, const std::vector<double>* prior) {
  const size_t m = it.sets.size();
  if (m == 0 || n < m) return 0;
  size_t ws = 0, wl = 0;
  ItemWindow(it, FilterWindow(), &ws, &wl, prior);
  std::vector<std::array<uint8_t, 256>> T(m);
  for (size_t q = 0; q < m; q++)
    for (int b = 0; b < 256; b++) T[q][size_t(b)] = it.sets[q].test(size_t(b)) ? 1 : 0;
  size_t piv = ws;  // the window's narrowest position first
  for (size_t q = ws; q < ws + wl; q++)
    if (it.sets[q].count() < it.sets[piv].count()) piv = q;
  uint64_t win = 0, item = 0;
  for (uint64_t p = 0; p + m <= n; p++) {
    if (!T[piv][a[p + piv]]) continue;
    bool ok = true;
    for (size_t q = ws; q < ws + wl && ok; q++) ok = T[q][a[p + q]] != 0;
    if (!ok) continue;
    win++;
    for (size_t q = 0; q < m && ok; q++) ok = T[q][a[p + q]] != 0;
    item += ok;
  }
  return win + item;
}

}  // namespace

bool CompileRules(const std::vector<RuleSrc>& src, CompiledRules* out, std::string* err, const CompileOptions* opt) {
  // TSG_CALIB_PRIOR=1 (experiment, off by default): a calibration sample's byte
  // frequencies replace the static prior of the prefilter's window choice and
  // clustering.  Unstable: independent bytes misprice runs (hex, base64), and on
  // the C2 corpus a 16-MB sample's prior flagged 3.3 % of the blocks, a 4-MB
  // one's 1.4 %, the static prior 1.4 % (with the calibrated anchor choice).
  std::vector<double> cal_prior;
  const std::vector<double>* cal_prior_p = nullptr;
  const char* cp_env = std::getenv("TSG_CALIB_PRIOR");
  if (opt && opt->calib && opt->calib_n && cp_env && std::atoi(cp_env) != 0) {
    std::vector<uint64_t> h(256, 0);
    for (uint64_t i = 0; i < opt->calib_n; i++) h[opt->calib[i]]++;
    cal_prior.resize(256);
    for (int b = 0; b < 256; b++) cal_prior[size_t(b)] = (double(h[size_t(b)]) + 0.5) / (double(opt->calib_n) + 128.0);
    cal_prior_p = &cal_prior;
  }
  std::map<std::string, uint32_t> kw_ids;
  out->rules.clear();
  out->regex.clear();
  for (size_t ri = 0; ri < src.size(); ri++) {
    const RuleSrc& r = src[ri];
    RuleGpu rg{};
    rg.max_len = kNoMaxLen;
    std::unique_ptr<Regex> re;
    if (r.has_regex) {
      re = Regex::Compile(r.regex, err);
      if (!re) return false;
      rg.has_regex = 1;
    }
    // keyword gate (strings.ToLower of each keyword); redundant when some
    // keyword is implied by every match of the regex
    rg.kw_off = uint32_t(out->rule_kw.size());
    bool host_gate = false;
    bool redundant = false;
    bool ascii_implied = false;  // in files without U+017F every match holds a keyword
    if (re) {
      std::vector<std::string> lows;
      bool all_ascii = true;
      for (auto& kw : r.keywords) {
        if (!IsAscii(kw)) all_ascii = false;
        lows.push_back(AsciiLower(kw));
      }
      if (all_ascii && !lows.empty()) {
        redundant = KeywordsImplied(*re, lows, false);
        ascii_implied = redundant || KeywordsImplied(*re, lows, true);
      }
    }
    if (redundant) out->n_redundant_gates++;
    for (auto& kw : r.keywords) {
      if (redundant) break;
      if (!IsAscii(kw)) {
        host_gate = true;
        continue;
      }
      std::string l = AsciiLower(kw);
      auto it = kw_ids.find(l);
      uint32_t id;
      if (it == kw_ids.end()) {
        id = uint32_t(out->keywords.size());
        kw_ids[l] = id;
        out->keywords.push_back(l);

      } else {
        id = it->second;
      }
      out->rule_kw.push_back(id);
    }
    rg.kw_cnt = uint32_t(out->rule_kw.size()) - rg.kw_off;
    rg.kw_match_implied = ascii_implied ? 1 : 0;
    if (!redundant && !host_gate && !ascii_implied && rg.kw_cnt) {  // GPU keyword bits (file-level, ASCII)
      for (uint32_t q = rg.kw_off; q < rg.kw_off + rg.kw_cnt; q++) {
        const uint32_t id = out->rule_kw[q];
        bool have = false;
        for (auto& it : out->items)
          if (it.kind == kItemKeyword && it.id == id) have = true;
        if (have) continue;
        FilterItem fi;
        fi.kind = kItemKeyword;
        fi.id = id;
        for (unsigned char ch : out->keywords[id]) {
          ByteSet b;
          b.set(ch);
          if (ch >= 'a' && ch <= 'z') b.set(size_t(ch - 32));
          fi.sets.push_back(b);
        }
        fi.lit_end = uint32_t(fi.sets.size());
        if (!fi.sets.empty()) out->items.push_back(std::move(fi));
      }
    }
    bool empty_kw = false;
    for (auto& kw : r.keywords)
      if (kw.empty()) empty_kw = true;
    if (r.keywords.empty() || empty_kw || redundant) rg.gate = kGateAlways;  // "" is a substring of anything
    else rg.gate = host_gate ? kGateHost : kGateKeywords;
    // anchor + relaxed NFA
    std::string desc = "-";
    if (re) {
      Cand best{{}, 0, 0};
      const char* cr_env = std::getenv("TSG_CLASS_RUNS");  // 0: literal anchors only (full-scan tests)
      const bool class_runs = !cr_env || std::atoi(cr_env) != 0;
      bool have = ExtractAnchor(*re, &best);
      bool calibrated = false;
      if (!have) {
        have = class_runs && ExtractClassRun(*re, &best);
      } else if (class_runs && opt && opt->calib && opt->calib_n) {
        // both kinds of anchor: the calibration sample decides (the class run
        // when it costs under half the literal's, and the literal is not rare)
        Cand run{{}, 0, 0};
        std::vector<std::pair<double, Cand>> runs;
        ExtractClassRun(*re, &run, kClassRunCalibProb, &runs);
        if (!runs.empty()) {
          uint64_t c_lit = 0;
          for (size_t li = 0; li < best.lits.size(); li++)
            c_lit += SampleCost(AnchorItem(*re, best, li, 0), opt->calib, opt->calib_n, cal_prior_p);
          // only a literal that fires often enough to matter (>= 1e-4 per sample byte) is moved:
          // the moved items' windows take buckets of their own (FilterItem::group)
          const uint64_t kCalibMinCost = std::max<uint64_t>(16, opt->calib_n / 10000);
          std::sort(runs.begin(), runs.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
          if (runs.size() > 4) runs.resize(4);  // the likeliest candidates by the prior
          for (auto& cr : runs) {
            if (c_lit < kCalibMinCost) break;  // a rare literal stays
            const uint64_t c_run = SampleCost(AnchorItem(*re, cr.second, 0, 0), opt->calib, opt->calib_n, cal_prior_p);
            if (std::getenv("TSG_CALIB_DEBUG"))
              std::fprintf(stderr, "calib %s: literal %llu, class run of %zu at [%lld,%lld] %llu\n", r.id.c_str(),
                           (unsigned long long)c_lit, cr.second.lits[0].size(), (long long)cr.second.olo,
                           (long long)cr.second.ohi, (unsigned long long)c_run);
            if (2 * c_run < c_lit) {
              best = cr.second;
              c_lit = c_run;
              calibrated = true;
            }
          }
          if (calibrated) out->n_calibrated_anchors++;
        }
      }
      if (have) {
        rg.anchored = 1;
        desc = "[" + std::to_string(best.olo) + "," + std::to_string(best.ohi) + "]";
        if (calibrated) desc += " (calibrated)";
        for (size_t li = 0; li < best.lits.size(); li++) {
          const std::string& l = best.lits[li];
          uint32_t aid = uint32_t(out->anchors.size());
          AnchorInfo ai{};
          ai.rule = uint32_t(ri);
          ai.lit_len = uint32_t(l.size());
          ai.off_lo = int32_t(best.olo);
          ai.off_hi = int32_t(best.ohi);
          ai.off_hi_fold = int32_t(std::min<int64_t>(best.ohi_fold, 1 << 30));
          out->anchors.push_back(ai);
          out->anchor_req.push_back(FollowReqs(re->nodes(), best.follow[li]));
          out->items.push_back(AnchorItem(*re, best, li, aid));  // prefilter item
          if (calibrated) out->items.back().group = 1;
          desc += best.class_run ? " <" + std::to_string(l.size()) + " classes>" : " " + l;
        }
      } else {
        rg.anchored = 0;
        out->n_fullscan_rules++;
      }
      {  // match length bounds: the fold runes widen the max, the min ignores them
        const int64_t mx = Analyzer(re->nodes(), true).Bytes(re->root()).second;
        const int64_t mn = Analyzer(re->nodes(), false).Bytes(re->root()).first;
        rg.min_len = uint32_t(std::min<int64_t>(std::max<int64_t>(mn, 0), 1 << 30));
        rg.max_len = mx >= (int64_t(1) << 20) ? kNoMaxLen : uint32_t(mx);
      }
      BuildNfa(Relax(re->nodes(), re->root()), &out->nfa, &rg);
    }
    out->rule_anchor_desc.push_back(desc);
    out->rules.push_back(rg);
    out->regex.push_back(std::move(re));
  }
  {  // fold runes: files holding them take the careful path
    const char* seqs[3] = {"\xC4\xB0", "\xE2\x84\xAA", "\xC5\xBF"};
    for (uint32_t k = 0; k < 3; k++) {
      FilterItem fi;
      fi.kind = kItemFold;
      fi.id = k;
      for (const char* p = seqs[k]; *p; p++) {
        ByteSet b;
        b.set(uint8_t(*p));
        fi.sets.push_back(b);
      }
      fi.lit_end = uint32_t(fi.sets.size());
      out->items.push_back(std::move(fi));
    }
  }
  {
    uint32_t nb = 16, nw = FilterWindow();
    if (const char* e = std::getenv("TSG_FILTER_BUCKETS")) nb = uint32_t(std::atoi(e));
    auto ft = std::make_shared<FilterTables>();
    if (!BuildFilter(out->items, nw, nb, ft.get(), err, cal_prior_p)) return false;
    out->filter = ft;
  }
  return true;
}

}  // namespace tsg
