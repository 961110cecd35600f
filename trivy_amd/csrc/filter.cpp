// Streaming prefilter tables (see filter.h).
#include "filter.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <cstdlib>
#include <map>

namespace tsg {

const std::vector<double>& BytePrior() {
  static const std::vector<double> prior = [] {
    std::vector<double> f(256, 1e-6);
    static const double en[26] = {8.2, 1.5, 2.8, 4.3, 12.7, 2.2, 2.0, 6.1, 7.0, 0.15, 0.8, 4.0, 2.4,
                                  6.7, 7.5, 1.9, 0.1, 6.0, 6.3, 9.1, 2.8, 1.0, 2.4, 0.15, 2.0, 0.07};
    double tot = 0;
    for (double x : en) tot += x;
    for (int i = 0; i < 26; i++) {
      f['a' + i] = 0.50 * en[i] / tot;
      f['A' + i] = 0.06 * en[i] / tot;
    }
    for (int d = '0'; d <= '9'; d++) f[d] = 0.006;
    for (int c = 0x21; c < 0x7F; c++)
      if (f[c] < 1e-4) f[c] = 0.001;
    f[' '] = 0.14;
    f['\n'] = 0.025;
    f['\t'] = 0.005;
    const std::pair<char, double> punct[] = {{'_', 0.015}, {'.', 0.012}, {',', 0.008}, {'"', 0.01}, {'\'', 0.006},
                                             {'(', 0.008}, {')', 0.008}, {'=', 0.008}, {':', 0.006}, {'-', 0.006},
                                             {'/', 0.005}, {';', 0.004}, {'{', 0.003}, {'}', 0.003}, {'[', 0.002},
                                             {']', 0.002}};
    for (auto& p : punct) f[uint8_t(p.first)] = p.second;
    for (int b = 0x80; b < 0x100; b++) f[b] = 1e-4;
    double s = 0;
    for (double x : f) s += x;
    for (double& x : f) x /= s;
    return f;
  }();
  return prior;
}

namespace {

// 256-bit byte set as four words (the clustering's working type).
struct B256 {
  uint64_t w[4];
  void set_all() { w[0] = w[1] = w[2] = w[3] = ~uint64_t(0); }
  bool test(int b) const { return (w[b >> 6] >> (b & 63)) & 1; }
  bool all() const { return (w[0] & w[1] & w[2] & w[3]) == ~uint64_t(0); }
};
B256 ToB256(const ByteSet& s) {
  B256 r{};
  for (int b = 0; b < 256; b++)
    if (s.test(size_t(b))) r.w[b >> 6] |= uint64_t(1) << (b & 63);
  return r;
}

// T[g * 256 + m] = prior mass of mask m over bytes 8g..8g+7
std::vector<double> PriorTable(const std::vector<double>& f) {
  std::vector<double> t(32 * 256, 0.0);
  for (int g = 0; g < 32; g++)
    for (int m = 0; m < 256; m++)
      for (int k = 0; k < 8; k++)
        if ((m >> k) & 1) t[size_t(g) * 256 + size_t(m)] += f[size_t(8 * g + k)];
  return t;
}

// The prior of the BuildFilter / ItemWindow call running on this thread: the
// static one, or a calibration sample's byte frequencies (CompileOptions).
thread_local const std::vector<double>* t_prior_table = nullptr;

struct PriorScope {
  std::vector<double> table;
  const std::vector<double>* saved;
  explicit PriorScope(const std::vector<double>* prior) : saved(t_prior_table) {
    if (prior) {
      table = PriorTable(*prior);
      t_prior_table = &table;
    }
  }
  ~PriorScope() { t_prior_table = saved; }
};

// P(byte in s) under the prior: 32 lookups of 8-byte groups.
double SetProb(const B256& s) {
  static const std::vector<double> T_static = PriorTable(BytePrior());
  const std::vector<double>& T = t_prior_table ? *t_prior_table : T_static;
  if (s.all()) return 1.0;
  double p = 0;
  for (int g = 0; g < 32; g++) p += T[size_t(g) * 256 + ((s.w[g >> 3] >> (8 * (g & 7))) & 0xFF)];
  return std::min(p, 1.0);
}

struct Cluster {
  B256 u[kFilterSlots];
  std::vector<uint32_t> members;
  double cost = 0;
};

// Window probability under the prior, with runs of one repeated non-letter
// byte rated as runs: text repeats punctuation and digits ("-----", "=====",
// "0000"), so each further copy of the same single byte counts as at least
// kRepeatProb instead of the independent byte's probability.
constexpr double kRepeatProb = 0.3;
bool SameSingleNonLetter(const B256& a, const B256& b) {
  int n = 0, x = -1;
  for (int k = 0; k < 4; k++) {
    if (a.w[k] != b.w[k]) return false;
    n += __builtin_popcountll(a.w[k]);
    if (a.w[k]) x = 64 * k + __builtin_ctzll(a.w[k]);
  }
  return n == 1 && !((x | 0x20) >= 'a' && (x | 0x20) <= 'z');
}
double WindowProb(const B256* u, int n) {
  double c = 1.0;
  for (int s = 0; s < n; s++) {
    double p = SetProb(u[s]);
    if (s > 0 && SameSingleNonLetter(u[s], u[s - 1])) p = std::max(p, kRepeatProb);
    c *= p;
  }
  return c;
}

double Cost(const B256* u) { return WindowProb(u, kFilterSlots); }  // unused slots stay "any" (P = 1)

}  // namespace

void ItemWindow(const FilterItem& it, uint32_t window, size_t* start, size_t* len, const std::vector<double>* prior) {
  PriorScope scope(prior);
  const size_t m = it.sets.size();
  size_t w = 0, wl = std::min<size_t>(m, window);
  double best = std::numeric_limits<double>::infinity();
  for (size_t s = 0; s + wl <= m; s++) {
    B256 win[kFilterSlots];
    for (size_t q = s; q < s + wl; q++) win[q - s] = ToB256(it.sets[q]);
    const double c = WindowProb(win, int(wl));
    if (c < best) {
      best = c;
      w = s;
    }
  }
  *start = w;
  *len = wl;
}

bool BuildFilter(const std::vector<FilterItem>& items, uint32_t window, uint32_t n_buckets, FilterTables* out,
                 std::string* err, const std::vector<double>* prior) {
  PriorScope scope(prior);
  if ((n_buckets != 8 && n_buckets != 16) || window < 2 || window > uint32_t(kFilterSlots)) {
    *err = "unsupported prefilter shape";
    return false;
  }
  *out = FilterTables();
  out->n_buckets = n_buckets;
  out->n_words = n_buckets / 4;
  out->window = window;
  out->nl_bucket = n_buckets - 1;
  const uint32_t n_item_buckets = n_buckets - 1;
  const uint32_t S = window;
  // identical byte-set sequences (rules sharing an anchor) become one item
  std::vector<FilterItem> uniq;
  std::vector<std::vector<uint32_t>> ids;
  {
    std::map<std::string, size_t> seen;
    for (auto& it : items) {
      std::string key(1, char(it.kind));
      key += char('0' + it.group);
      key += std::to_string(it.lit_end) + ":";
      for (auto& b : it.sets) key += b.to_string();
      auto f = seen.find(key);
      if (f != seen.end() && ids[f->second].size() < 255) {
        ids[f->second].push_back(it.id);
        continue;
      }
      seen[key] = uniq.size();
      uniq.push_back(it);
      ids.push_back({it.id});
    }
  }
  const size_t n = uniq.size();
  // classes (deduplicated byte sets) and per-item windows
  std::map<std::string, uint32_t> cls_ids;
  std::vector<ByteSet> classes;
  std::vector<Cluster> cl(n);
  for (size_t i = 0; i < n; i++) {
    const FilterItem& it = uniq[i];
    if (it.sets.empty() || it.sets.size() > 0xFFFF) {
      *err = "prefilter item with no (or too many) positions";
      return false;
    }
    const size_t m = it.sets.size();
    // least frequent window of <= kFilterSlots positions
    size_t w = 0, wl = 0;
    ItemWindow(it, S, &w, &wl, nullptr);  // (under this call's prior)
    for (int s = 0; s < kFilterSlots; s++) cl[i].u[s].set_all();
    for (size_t q = 0; q < wl; q++) cl[i].u[S - wl + q] = ToB256(it.sets[w + q]);
    cl[i].members = {uint32_t(i)};
    cl[i].cost = Cost(cl[i].u);
    FilterItemGpu g{};
    g.n = uint16_t(m);
    g.back = uint16_t(w + wl);
    g.lit_end = uint16_t(it.lit_end);
    g.kind = it.kind;
    g.n_ids = uint8_t(ids[i].size());
    g.ids_off = uint32_t(out->item_ids.size());
    out->item_ids.insert(out->item_ids.end(), ids[i].begin(), ids[i].end());
    g.cls_off = uint32_t(out->item_cls.size());
    out->max_after = std::max<uint32_t>(out->max_after, uint32_t(m - (w + wl)));
    for (auto& b : it.sets) {
      std::string key = b.to_string();
      auto f = cls_ids.find(key);
      uint32_t id;
      if (f == cls_ids.end()) {
        id = uint32_t(classes.size());
        if (id >= 256) {
          *err = "prefilter needs more than 256 distinct byte classes";
          return false;
        }
        cls_ids[key] = id;
        classes.push_back(b);
      } else {
        id = f->second;
      }
      out->item_cls.push_back(uint8_t(id));
    }
    out->items.push_back(g);
  }
  // agglomerative clustering down to n_buckets: always merge the pair whose
  // union adds the least estimated fire rate.  Each row caches its best
  // partner; after a merge only rows whose partner died are rescanned
  // (O(n^2) in practice instead of a full O(n^2) scan per merge).
  std::vector<bool> alive(n, true);
  size_t n_alive = n;
  auto merged = [&](const Cluster& a, const Cluster& b, B256* u) {
    for (int s = 0; s < kFilterSlots; s++)
      for (int k = 0; k < 4; k++) u[s].w[k] = a.u[s].w[k] | b.u[s].w[k];
    return Cost(u);
  };
  std::vector<bool> solo(n, false);
  if (const char* e = std::getenv("TSG_FILTER_SOLO")) {  // experiment: items kept in buckets of their own
    for (const char* q = e; *q;) {
      char* end = nullptr;
      const unsigned long v = std::strtoul(q, &end, 10);
      if (end == q) break;
      if (v < n) solo[v] = true;
      q = *end ? end + 1 : end;
    }
  }
  auto delta_of = [&](size_t i, size_t j) {
    if (solo[i] || solo[j] || uniq[i].group != uniq[j].group) return std::numeric_limits<double>::infinity();
    B256 u[kFilterSlots];
    return merged(cl[i], cl[j], u) - cl[i].cost - cl[j].cost;
  };
  std::vector<double> delta(n > 1 ? n * n : 1, 0.0);  // symmetric, rows of n
  for (size_t i = 0; i < n; i++)
    for (size_t j = i + 1; j < n; j++) delta[i * n + j] = delta[j * n + i] = delta_of(i, j);
  const double kInf = std::numeric_limits<double>::infinity();
  std::vector<size_t> best(n, 0);
  std::vector<double> best_d(n, kInf);
  auto rescan = [&](size_t i) {
    best_d[i] = kInf;
    for (size_t j = 0; j < n; j++)
      if (j != i && alive[j] && delta[i * n + j] < best_d[i]) {
        best_d[i] = delta[i * n + j];
        best[i] = j;
      }
  };
  for (size_t i = 0; i < n; i++) rescan(i);
  while (n_alive > n_item_buckets) {
    size_t bi = 0, bj = 0;
    double bd = kInf;
    for (size_t i = 0; i < n; i++)
      if (alive[i] && best_d[i] < bd) {
        bd = best_d[i];
        bi = i;
        bj = best[i];
      }
    if (bd == kInf) {  // (more solo items / groups than buckets)
      *err = "prefilter: no bucket merge left (solo items or groups exceed the buckets)";
      return false;
    }
    if (bj < bi) std::swap(bi, bj);
    B256 u[kFilterSlots];
    double c = merged(cl[bi], cl[bj], u);
    for (int s = 0; s < kFilterSlots; s++) cl[bi].u[s] = u[s];
    cl[bi].cost = c;
    cl[bi].members.insert(cl[bi].members.end(), cl[bj].members.begin(), cl[bj].members.end());
    alive[bj] = false;
    n_alive--;
    for (size_t k = 0; k < n; k++) {
      if (!alive[k] || k == bi) continue;
      const double d = delta_of(bi, k);
      delta[k * n + bi] = delta[bi * n + k] = d;
    }
    rescan(bi);
    for (size_t k = 0; k < n; k++) {
      if (!alive[k] || k == bi) continue;
      if (best[k] == bi || best[k] == bj) {
        rescan(k);  // its partner changed or died
      } else if (delta[k * n + bi] < best_d[k]) {
        best_d[k] = delta[k * n + bi];
        best[k] = bi;
      }
    }
  }
  // reach table
  const uint32_t W = out->n_words;
  out->reach.assign(256 * W, ~0u);
  auto allow = [&](uint32_t b, uint32_t j, uint32_t slot) { out->reach[size_t(b) * W + j / 4] &= ~(1u << (4 * slot + j % 4)); };
  out->bucket_off.push_back(0);
  uint32_t j = 0;
  for (size_t i = 0; i < n; i++) {
    if (!alive[i]) continue;
    out->est_fp += cl[i].cost;
    for (uint32_t sl = 0; sl < uint32_t(kFilterSlots); sl++)  // slots >= window: all bytes allowed (carry the fire)
      for (int b = 0; b < 256; b++)
        if (sl >= S || cl[i].u[sl].test(b)) allow(uint32_t(b), j, sl);
    for (uint32_t m : cl[i].members) out->bucket_items.push_back(m);
    out->bucket_off.push_back(uint32_t(out->bucket_items.size()));
    j++;
  }
  for (; j < n_buckets; j++) {  // empty item buckets never fire; the newline bucket allows '\n' at slot 0
    if (j == out->nl_bucket) {  // slot 0: '\n' only; slots 1-3 carry; slots 4-7 never allow (no fires)
      allow('\n', j, 0);
      for (uint32_t sl = 1; sl < 4; sl++)
        for (int b = 0; b < 256; b++) allow(uint32_t(b), j, sl);
    }
    out->bucket_off.push_back(uint32_t(out->bucket_items.size()));
  }
  // literal windows -> hash table (filter.h); the rest -> core groups
  std::vector<uint8_t> hashed(n, 0);
  std::vector<std::pair<uint64_t, uint32_t>> hkeys;
  const char* hash_env = std::getenv("TSG_WINDOW_HASH");  // 0: core groups only (A/B)
  // Large rule sets only: builtin-sized buckets hold 1-2 groups, whose LDS core
  // lookups beat a probe plus the full position check (C2 confirm 5.08 vs 5.35
  // ms with hashing; C3, 2,108 items: 25.0 -> 4.0 ms, profiles/r02_wl/wl_r02h_*)
  const bool use_hash = hash_env ? std::atoi(hash_env) != 0 && S == 6 : (S == 6 && n > 256);
  for (size_t i = 0; i < n && use_hash; i++) {
    const FilterItemGpu& g = out->items[i];
    if (g.back < 6) continue;
    uint64_t key = 0;
    bool ok = true;
    for (int q = 0; q < 6 && ok; q++) {
      const ByteSet& b = uniq[i].sets[size_t(g.back - 6 + q)];
      const size_t pc = b.count();
      int c = -1;
      for (int x = 0; x < 128 && pc <= 2; x++)
        if (b.test(size_t(x))) {
          c = x;
          break;
        }
      if (c < 0 || pc > 2) {
        ok = false;
        break;
      }
      for (int x = 128; x < 256; x++)
        if (b.test(size_t(x))) ok = false;
      if (pc == 2) ok = ok && c >= 'A' && c <= 'Z' && b.test(size_t(c + 32));
      const int lc = (c >= 'A' && c <= 'Z') ? c + 32 : c;
      key |= uint64_t(lc) << (8 * q);
    }
    if (!ok) continue;
    hashed[i] = 1;
    hkeys.push_back({key, uint32_t(i)});
  }
  if (!hkeys.empty()) {
    uint32_t bits = 4;
    while ((size_t(1) << bits) < 2 * hkeys.size()) bits++;
    out->hash_bits = bits;
    out->hash_keys.assign(size_t(1) << bits, 0);
    out->hash_items.assign(size_t(1) << bits, 0);
    for (auto& kv : hkeys) {
      uint32_t slot = WindowHash(kv.first, bits);
      while (out->hash_keys[slot]) slot = (slot + 1) & ((1u << bits) - 1);
      out->hash_keys[slot] = kv.first | (uint64_t(1) << 63);
      out->hash_items[slot] = kv.second;
    }
    for (uint32_t b = 0; b < n_buckets; b++)
      for (uint32_t k = out->bucket_off[b]; k < out->bucket_off[b + 1]; k++)
        if (hashed[out->bucket_items[k]]) out->hash_buckets |= 1u << b;
  }
  // core tables (filter.h), over the items not hashed
  out->bucket_groups.push_back(0);
  uint32_t n_groups = 0;
  for (uint32_t b = 0; b < n_buckets; b++) {
    std::vector<uint32_t> grp;
    for (uint32_t k = out->bucket_off[b]; k < out->bucket_off[b + 1]; k++)
      if (!hashed[out->bucket_items[k]]) grp.push_back(out->bucket_items[k]);
    const uint32_t lo = 0, hi = uint32_t(grp.size());
    for (uint32_t g0 = lo; g0 < hi; g0 += 8) {
      std::vector<uint64_t> tab(256, 0);
      for (uint32_t i = 0; i < 8; i++) {
        if (g0 + i >= hi) {
          out->group_items.push_back(0xFFFFFFFFu);
          continue;
        }
        const uint32_t item = grp[g0 + i];
        out->group_items.push_back(item);
        const FilterItem& it = uniq[item];
        const int back = out->items[item].back;
        for (int sl = 0; sl < 8; sl++) {
          const int q = back - 8 + sl;
          for (int x = 0; x < 256; x++)
            if (q < 0 || it.sets[size_t(q)].test(size_t(x))) tab[size_t(x)] |= uint64_t(1) << (8 * sl + i);
        }
      }
      out->core.insert(out->core.end(), tab.begin(), tab.end());
      n_groups++;
    }
    out->bucket_groups.push_back(n_groups);
  }
  for (auto& b : classes) {
    uint32_t w[8] = {};
    for (int x = 0; x < 256; x++)
      if (b.test(x)) w[x >> 5] |= 1u << (x & 31);
    out->classes.insert(out->classes.end(), w, w + 8);
  }
  return true;
}

}  // namespace tsg
