// Deterministic synthetic corpus for the bench and the large-size tests
// (include/tsg_corpus.h; spec: SURVEY.md §8(d)).  Not part of the scan path.
//
// Per file: SplitMix64(seed ^ index) drives a log-normal size (median 8 KiB,
// sigma 1.5, clipped [10 B, 10 MiB]) and a content class: 70 % source-like
// text with keyword collisions, 20 % prose/markdown, 8 % base64/hex/JSON
// blobs, 2 % UTF-8 (incl. U+0130, U+212A, U+017F and invalid bytes).  Lines
// are geometric (mean ~40 B) with 1 % > 100 B and 0.1 % > 10 KiB.  Secrets
// from a sampled pool are planted at 1 per 256 KiB (Poisson).  Contents are
// generated CR-free; tsg_corpus_crlf turns a share of the files into CRLF
// text afterwards (5 % of C1/C2 files; the analyzer strips the
// CRs before Scan).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "tsg_corpus.h"

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t Next() {  // SplitMix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double U() { return double(Next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t Below(uint32_t n) { return uint32_t((Next() >> 32) * uint64_t(n) >> 32); }
  double Normal() {
    double u1 = U(), u2 = U();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
  uint32_t Geometric(double mean) {
    double u = U();
    if (u < 1e-12) u = 1e-12;
    return uint32_t(-std::log(u) * mean);
  }
};

const char* kCode[] = {
    "key", "value", "task", "ask", "desk", "risk", "global", "blob", "return", "func", "def", "class", "import",
    "from", "self", "this", "config", "token", "secret", "password", "user", "name", "index", "buffer", "data",
    "api_key", "access_key", "aws_region", "skip", "mask", "disk", "public", "private", "live_", "pk.",
    "msg.", "err", "nil", "None", "true", "false", "if", "else", "for", "while", "let", "const", "var", "int",
    "string", "map", "list", "dict", "result", "request", "response", "handler", "context", "logger", "debug",
    "key_id", "keys", "monkey", "they", "eyes", "test", "testing", "-----", "=>", ":=", "==", "!=", "+=", "->",
    "::", "&&", "||", "0x1f", "42", "1024", "3.14", "i", "j", "n", "err", "ok", "len", "size", "count", "path",
    "file", "open", "close", "read", "write", "append", "print", "format", "value", "item", "node", "next",
};
// vendor / rule words: realistic but rare collisions (0.5 % of tokens)
const char* kVendor[] = {
    "github", "slack", "stripe", "heroku", "twitter", "facebook", "discord", "linear", "lobby", "mailgun",
    "hf_hub", "sk", "sg.", "dapi", "pul-", "npm_", "asana", "twitch", "adobe", "intercom", "typeform",
    "shippo", "finicity", "fastly", "beamer", "aws_secret", "AKIA", "ghp_", "xoxb-", "eyJ", "pk_live_",
};
const char* kProse[] = {
    "the", "of", "and", "to", "a", "in", "is", "it", "you", "that", "he", "was", "for", "on", "are", "with",
    "as", "I", "his", "they", "be", "at", "one", "have", "this", "from", "or", "had", "by", "word", "but",
    "what", "some", "we", "can", "out", "other", "were", "all", "there", "when", "up", "use", "your", "how",
    "said", "an", "each", "she", "which", "do", "their", "time", "if", "will", "way", "about", "many", "then",
    "them", "write", "would", "like", "so", "these", "her", "long", "make", "thing", "see", "him", "two",
    "has", "look", "more", "day", "could", "go", "come", "did", "number", "sound", "no", "most", "people",
    "key", "keys", "global", "task", "asked", "risky", "example", "linear", "public", "service", "account",
};
const char* kUtf8[] = {"\xC3\xA9", "\xC3\xBC", "\xE6\x97\xA5\xE6\x9C\xAC", "\xF0\x9F\x98\x80", "\xE2\x80\x94",
                       "\xE2\x80\x99", "\xD0\x96", "\xCE\xBB", "\xC3\xB1"};
const char* kSpecial[] = {"\xC4\xB0", "\xE2\x84\xAA", "\xC5\xBF", "\xFF", "\xC3", "\x80"};
const char* kExt[] = {".go", ".py", ".js", ".ts", ".java", ".c", ".txt", ".yaml", ".json", ".sh", ".conf",
                      ".rb", ".rs", ".xml", ".env", ".ini"};

constexpr int kNCode = sizeof(kCode) / sizeof(kCode[0]);
constexpr int kNProse = sizeof(kProse) / sizeof(kProse[0]);

struct Out {
  uint8_t* p;
  uint64_t n, cap;
  bool Full() const { return n >= cap; }
  void Put(const char* s, size_t k) {
    if (n + k > cap) k = size_t(cap - n);
    std::memcpy(p + n, s, k);
    n += k;
  }
  void Put(const char* s) { Put(s, std::strlen(s)); }
  void C(char c) {
    if (n < cap) p[n++] = uint8_t(c);
  }
};

const char kAlnum[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
const char kHex[] = "0123456789abcdef";

void RandomRun(Out& o, Rng& r, const char* alpha, uint32_t na, uint32_t len) {
  for (uint32_t i = 0; i < len && !o.Full(); i++) o.C(alpha[r.Below(na)]);
}

uint32_t LineTarget(Rng& r) {
  double u = r.U();
  if (u < 0.001) return 10240 + r.Below(40000);  // minified
  if (u < 0.011) return 100 + r.Below(900);      // long
  return 1 + r.Geometric(40.0);
}

void SourceLine(Out& o, Rng& r, uint32_t target) {
  uint64_t start = o.n;
  uint32_t ind = r.Below(4) * 2;
  for (uint32_t i = 0; i < ind; i++) o.C(' ');
  while (o.n - start < target && !o.Full()) {
    uint32_t t = r.Below(100);
    if (t < 70) {
      if (r.Below(200) == 0) o.Put(kVendor[r.Below(sizeof(kVendor) / sizeof(kVendor[0]))]);
      else o.Put(kCode[r.Below(kNCode)]);
    } else if (t < 80) {
      o.C('"');
      RandomRun(o, r, kAlnum, 62, 1 + r.Below(24));
      o.C('"');
    } else if (t < 85) {
      RandomRun(o, r, kHex, 16, 4 + r.Below(36));
    } else {
      static const char* p = "(){}[];,.:=+-*/<>";
      o.C(p[r.Below(17)]);
    }
    o.C(r.Below(4) == 0 ? '_' : ' ');
  }
  o.C('\n');
}

void ProseLine(Out& o, Rng& r, uint32_t target, bool utf8) {
  uint64_t start = o.n;
  if (r.Below(30) == 0) o.Put("## ");
  if (r.Below(60) == 0) {
    o.Put("-----\n");
    return;
  }
  while (o.n - start < target && !o.Full()) {
    o.Put(kProse[r.Below(kNProse)]);
    if (utf8 && r.Below(6) == 0) o.Put(kUtf8[r.Below(sizeof(kUtf8) / sizeof(kUtf8[0]))]);
    if (utf8 && r.Below(400) == 0) o.Put(kSpecial[r.Below(sizeof(kSpecial) / sizeof(kSpecial[0]))]);
    o.C(r.Below(12) == 0 ? ',' : ' ');
  }
  o.C('\n');
}

void BlobLine(Out& o, Rng& r, uint32_t kind) {
  if (kind == 0) {
    RandomRun(o, r, kB64, 64, 76);
  } else if (kind == 1) {
    RandomRun(o, r, kHex, 16, 64);
  } else {
    o.Put("  \"");
    o.Put(kCode[r.Below(kNCode)]);
    o.Put("\": \"");
    RandomRun(o, r, kAlnum, 62, 4 + r.Below(40));
    o.Put("\",");
  }
  o.C('\n');
}

uint64_t FileSize(uint64_t seed, uint64_t i) {
  Rng r(seed ^ (i * 0xD1B54A32D192ED03ull));
  double z = r.Normal();
  double s = 8192.0 * std::exp(1.5 * z);
  if (s < 10) s = 10;
  if (s > 10485760.0) s = 10485760.0;
  return uint64_t(s);
}

// One file's content (the class draw, planted secrets, lines) into o.
void FillContent(Rng& r, Out& o, const char* pool, const uint64_t* pool_off, uint32_t n_pool,
                 double secrets_per_byte) {
  const uint64_t fs = 0, fe = o.cap;
  uint32_t cls = r.Below(100);
  // planted secrets: Poisson(size * rate) positions
  double lam = double(fe - fs) * secrets_per_byte;
  std::vector<uint64_t> plant;
  {
    double l = std::exp(-lam), p = 1.0;
    int k = 0;
    if (lam > 30) k = int(lam + std::sqrt(lam) * r.Normal());
    else
      for (;;) {
        p *= r.U();
        if (p < l) break;
        k++;
      }
    for (int j = 0; j < k && n_pool; j++) plant.push_back(r.Next() % (fe - fs));
    std::sort(plant.begin(), plant.end());
  }
  size_t pi = 0;
  while (!o.Full()) {
    while (pi < plant.size() && plant[pi] <= o.n) {
      uint32_t s = r.Below(n_pool);
      static const char* pre[] = {" ", "export TOKEN=", "key: \"", "\t", "= '", "", "(\""};
      o.Put(pre[r.Below(7)]);
      o.Put(pool + pool_off[s], size_t(pool_off[s + 1] - pool_off[s]));
      o.C(r.Below(2) ? '\n' : ' ');
      pi++;
    }
    uint32_t t = LineTarget(r);
    if (cls < 70) SourceLine(o, r, t);
    else if (cls < 90) ProseLine(o, r, t, false);
    else if (cls < 98) BlobLine(o, r, cls % 3);
    else ProseLine(o, r, t, true);
  }
}


// ---- C4: an uncompressed image layer (ustar) of many small files ----------
struct LayerEntry {
  uint64_t hdr;   // header offset in the archive
  uint64_t size;  // data bytes
  uint8_t kind;   // 0 text, 1 CRLF text, 2 ELF-like binary, 3 .pyc-like, 4 dir, 5 symlink, 6 whiteout
  std::string path;
};

const char* kPkgs[] = {"openssl", "curl", "bash", "coreutils", "nginx", "python3", "zlib", "libssl", "apt",
                       "dpkg", "tzdata", "ca-certificates", "perl", "git", "node", "redis", "postgres", "sed"};
const char* kAppDirs[] = {"opt/app/src", "srv/api/handlers", "home/app/project", "var/www/html", "app/services",
                          "etc", "root", "opt/tools/scripts", "workspace/lib", "srv/config"};

// Layer plan: per file SplitMix64(seed ^ i): size log-normal (median 1.5 KiB,
// sigma 1.2, clipped [10 B, 10 MiB]) and a path mimicking a distro tree.
std::vector<LayerEntry> PlanLayer(uint64_t seed, uint64_t target_file_bytes) {
  std::vector<LayerEntry> v;
  uint64_t total = 0, off = 0;
  std::string last_dir;
  Rng g(seed ^ 0xC4C4C4C4ull);  // directory groups: a new one every ~24 files
  uint64_t group = 0;
  for (uint64_t i = 0; total < target_file_bytes; i++) {
    Rng r(seed ^ (i * 0xA24BAED4963EE407ull) ^ 0xC4C4C4C4ull);
    if (g.Below(24) == 0) group++;
    Rng gr(seed ^ (group * 0x9FB21C651E98DF25ull));
    double z = r.Normal();
    double sz = 1536.0 * std::exp(1.2 * z);
    sz = std::min(std::max(sz, 10.0), 10485760.0);
    uint64_t size = uint64_t(sz);
    const uint32_t pk = gr.Below(1000);
    const char* pkg = kPkgs[gr.Below(sizeof(kPkgs) / sizeof(kPkgs[0]))];
    const char* ad = kAppDirs[gr.Below(sizeof(kAppDirs) / sizeof(kAppDirs[0]))];
    const unsigned sub = unsigned(gr.Below(1000));
    char buf[128];
    uint8_t kind = 0;
    std::string dir;
    if (pk < 300) {  // allow-listed system dirs (Required skips them by path)
      static const char* sys[] = {"usr/share/doc/", "usr/lib/x86_64-linux-gnu/", "usr/include/", "usr/share/zoneinfo/"};
      dir = std::string(sys[pk % 4]) + pkg + "/d" + std::to_string(sub);
      snprintf(buf, sizeof buf, "%s/f%llu.txt", dir.c_str(), (unsigned long long)i);
    } else if (pk < 360) {  // executables
      dir = std::string(pk < 330 ? "usr/bin" : "usr/sbin");
      snprintf(buf, sizeof buf, "%s/%s-%llu", dir.c_str(), pkg, (unsigned long long)i);
      kind = 2;
    } else if (pk < 380) {  // compiled python (binary, scanned via printable runs)
      dir = std::string("opt/app/venv/") + pkg + std::to_string(sub) + "/__pycache__";
      snprintf(buf, sizeof buf, "%s/m%llu.cpython-311.pyc", dir.c_str(), (unsigned long long)i);
      kind = 3;
    } else if (pk < 410) {  // skipped extensions
      dir = std::string("usr/local/share/") + pkg + "/img" + std::to_string(sub);
      snprintf(buf, sizeof buf, "%s/i%llu%s", dir.c_str(), (unsigned long long)i, pk < 395 ? ".png" : ".gz");
      kind = 2;
    } else {
      dir = std::string(ad) + "/" + pkg + "/m" + std::to_string(sub);
      snprintf(buf, sizeof buf, "%s/file%llu%s", dir.c_str(), (unsigned long long)i,
               kExt[r.Below(sizeof(kExt) / sizeof(kExt[0]))]);
      kind = r.Below(100) < 5 ? 1 : 0;
    }
    if (dir != last_dir) {  // a directory entry when the walk changes directory
      v.push_back({off, 0, 4, dir + "/"});
      off += 512;
      last_dir = dir;
    }
    if (r.Below(500) == 0) {  // whiteout / symlink entries
      v.push_back({off, 0, uint8_t(r.Below(2) ? 5 : 6), dir + (r.Below(2) ? "/.wh.old" : "/link")});
      off += 512;
    }
    if (total + size > target_file_bytes) size = target_file_bytes - total;
    if (size == 0) break;
    v.push_back({off, size, kind, std::string(buf)});
    off += 512 + ((size + 511) & ~uint64_t(511));
    total += size;
  }
  return v;
}

void Octal(char* dst, int width, uint64_t v) {  // width-1 octal digits + NUL
  for (int k = width - 2; k >= 0; k--) {
    dst[k] = char('0' + (v & 7));
    v >>= 3;
  }
  dst[width - 1] = 0;
}

void WriteHeader(uint8_t* h, const LayerEntry& e) {
  std::memset(h, 0, 512);
  std::string name = e.path, prefix;
  if (name.size() > 100) {  // ustar prefix split at a '/'
    size_t k = name.rfind('/', 154);
    prefix = name.substr(0, k);
    name = name.substr(k + 1);
  }
  std::memcpy(h, name.data(), std::min<size_t>(name.size(), 100));
  Octal(reinterpret_cast<char*>(h + 100), 8, e.kind == 4 ? 0755 : 0644);
  Octal(reinterpret_cast<char*>(h + 108), 8, 0);
  Octal(reinterpret_cast<char*>(h + 116), 8, 0);
  Octal(reinterpret_cast<char*>(h + 124), 12, e.size);
  Octal(reinterpret_cast<char*>(h + 136), 12, 1700000000);
  h[156] = e.kind == 4 ? '5' : e.kind == 5 ? '2' : '0';
  if (e.kind == 5) std::memcpy(h + 157, "../target", 9);
  std::memcpy(h + 257, "ustar\0" "00", 8);
  std::memcpy(h + 345, prefix.data(), std::min<size_t>(prefix.size(), 155));
  std::memset(h + 148, ' ', 8);
  uint32_t sum = 0;
  for (int k = 0; k < 512; k++) sum += h[k];
  Octal(reinterpret_cast<char*>(h + 148), 7, sum);
  h[155] = ' ';
}
}  // namespace

extern "C" {

int64_t tsg_corpus_plan(uint64_t seed, uint64_t target_bytes, uint64_t* offsets, uint64_t cap) {
  uint64_t total = 0, n = 0;
  if (offsets && cap) offsets[0] = 0;
  while (total < target_bytes) {
    uint64_t s = FileSize(seed, n);
    if (total + s > target_bytes) s = target_bytes - total;
    total += s;
    n++;
    if (offsets && n < cap) offsets[n] = total;
  }
  return int64_t(n);
}

int tsg_corpus_fill(uint64_t seed, const uint64_t* offsets, uint64_t n_files, const char* pool,
                    const uint64_t* pool_off, uint32_t n_pool, double secrets_per_byte, uint8_t* arena,
                    char* paths, uint32_t path_stride, int threads) {
  if (threads <= 0) threads = 1;
  std::atomic<uint64_t> next{0};
  auto work = [&]() {
    for (;;) {
      uint64_t lo = next.fetch_add(256);
      if (lo >= n_files) break;
      uint64_t hi = std::min<uint64_t>(lo + 256, n_files);
      for (uint64_t i = lo; i < hi; i++) {
        Rng r(seed ^ (i * 0x9E3779B97F4A7C15ull) ^ 0xA5A5A5A5ull);
        uint64_t fs = offsets[i], fe = offsets[i + 1];
        Out o{arena + fs, 0, fe - fs};
        FillContent(r, o, pool, pool_off, n_pool, secrets_per_byte);
        if (paths) {
          char* P = paths + i * path_stride;
          uint32_t pk = r.Below(100);
          const char* dir = pk < 3 ? "test/" : pk < 5 ? "vendor/" : pk < 7 ? "docs/" : "";
          const char* ext = pk >= 95 ? ".md" : kExt[r.Below(sizeof(kExt) / sizeof(kExt[0]))];
          snprintf(P, path_stride, "repo%u/pkg%u/%sfile%llu%s", unsigned(i % 97), unsigned(r.Below(50)), dir,
                   (unsigned long long)i, ext);
        }
      }
    }
  };
  std::vector<std::thread> pool_t;
  for (int t = 1; t < threads; t++) pool_t.emplace_back(work);
  work();
  for (auto& th : pool_t) th.join();
  return 0;
}

int64_t tsg_corpus_crlf(uint64_t seed, const uint64_t* offsets, uint64_t n_files, uint8_t* arena, double share,
                        uint8_t* is_crlf, int threads) {
  if (threads <= 0) threads = 1;
  std::atomic<uint64_t> next{0}, count{0};
  auto work = [&]() {
    std::vector<uint8_t> tmp;
    for (;;) {
      const uint64_t lo = next.fetch_add(256);
      if (lo >= n_files) break;
      const uint64_t hi = std::min<uint64_t>(lo + 256, n_files);
      for (uint64_t i = lo; i < hi; i++) {
        Rng r(seed ^ (i * 0xD1B54A32D192ED03ull) ^ 0xC3C3C3C3ull);
        const bool on = double(r.Below(1u << 20)) < share * double(1u << 20);
        if (is_crlf) is_crlf[i] = on ? 1 : 0;
        if (!on) continue;
        count++;
        // LF -> CR LF, cut at the file's size (the lines past it are dropped)
        uint8_t* d = arena + offsets[i];
        const uint64_t n = offsets[i + 1] - offsets[i];
        tmp.assign(d, d + n);
        uint64_t w = 0;
        for (uint64_t k = 0; k < n && w < n; k++) {
          if (tmp[k] == '\n') {
            d[w++] = '\r';
            if (w >= n) break;
          }
          d[w++] = tmp[k];
        }
      }
    }
  };
  std::vector<std::thread> pool_t;
  for (int t = 1; t < threads; t++) pool_t.emplace_back(work);
  work();
  for (auto& th : pool_t) th.join();
  return int64_t(count.load());
}

int tsg_corpus_strip(const uint64_t* offsets, uint64_t n_files, const uint8_t* in, uint8_t* out, uint64_t* out_offsets,
                     int threads) {
  if (threads <= 0) threads = 1;
  std::vector<uint64_t> cr(n_files + 1, 0);
  auto par = [&](auto fn) {
    std::atomic<uint64_t> next{0};
    auto work = [&]() {
      for (;;) {
        const uint64_t lo = next.fetch_add(512);
        if (lo >= n_files) break;
        for (uint64_t i = lo; i < std::min<uint64_t>(lo + 512, n_files); i++) fn(i);
      }
    };
    std::vector<std::thread> ts;
    for (int t = 1; t < threads; t++) ts.emplace_back(work);
    work();
    for (auto& th : ts) th.join();
  };
  par([&](uint64_t i) {
    const uint8_t* p = in + offsets[i];
    const uint8_t* e = in + offsets[i + 1];
    uint64_t c = 0;
    while (p < e && (p = static_cast<const uint8_t*>(std::memchr(p, '\r', size_t(e - p))))) {
      c++;
      p++;
    }
    cr[i] = c;
  });
  out_offsets[0] = 0;
  for (uint64_t i = 0; i < n_files; i++) out_offsets[i + 1] = out_offsets[i] + (offsets[i + 1] - offsets[i]) - cr[i];
  par([&](uint64_t i) {
    const uint8_t* p = in + offsets[i];
    const uint8_t* e = in + offsets[i + 1];
    uint8_t* d = out + out_offsets[i];
    if (!cr[i]) {
      std::memcpy(d, p, size_t(e - p));
      return;
    }
    while (p < e) {
      const uint8_t* q = static_cast<const uint8_t*>(std::memchr(p, '\r', size_t(e - p)));
      const uint8_t* stop = q ? q : e;
      std::memcpy(d, p, size_t(stop - p));
      d += stop - p;
      p = q ? q + 1 : e;
    }
  });
  return 0;
}

int64_t tsg_corpus_layer(uint64_t seed, uint64_t target_file_bytes, const char* pool, const uint64_t* pool_off,
                         uint32_t n_pool, double secrets_per_byte, uint8_t* out, uint64_t cap, int threads,
                         uint64_t* n_entries) {
  const std::vector<LayerEntry> plan = PlanLayer(seed, target_file_bytes);
  const uint64_t end = plan.empty() ? 0 : plan.back().hdr + 512 + ((plan.back().size + 511) & ~uint64_t(511));
  const uint64_t total = end + 1024;  // two zero blocks
  if (n_entries) *n_entries = plan.size();
  if (!out) return int64_t(total);
  if (cap < total) return -1;
  if (threads <= 0) threads = 1;
  std::atomic<uint64_t> next{0};
  auto work = [&]() {
    std::vector<uint8_t> tmp;
    for (;;) {
      const uint64_t lo = next.fetch_add(512);
      if (lo >= plan.size()) break;
      const uint64_t hi = std::min<uint64_t>(lo + 512, plan.size());
      for (uint64_t i = lo; i < hi; i++) {
        const LayerEntry& e = plan[i];
        uint8_t* h = out + e.hdr;
        WriteHeader(h, e);
        uint8_t* d = h + 512;
        const uint64_t padded = (e.size + 511) & ~uint64_t(511);
        std::memset(d + e.size, 0, size_t(padded - e.size));
        if (!e.size) continue;
        Rng r(seed ^ (i * 0x9E3779B97F4A7C15ull) ^ 0x5A5A5A5Aull);
        if (e.kind == 0 || e.kind == 3) {
          Out o{d, 0, e.size};
          FillContent(r, o, pool, pool_off, n_pool, secrets_per_byte);
          if (e.kind == 3) {  // .pyc-like: a binary header and NULs between text runs
            static const uint8_t magic[8] = {0xA7, 0x0D, 0x0D, 0x0A, 0, 0, 0, 0};
            std::memcpy(d, magic, std::min<uint64_t>(8, e.size));
            for (uint64_t k = 8; k < e.size; k += 16 + r.Below(48)) d[k] = 0;
          }
        } else if (e.kind == 1) {  // CRLF text: generate, then expand '\n' -> "\r\n" up to the size
          tmp.assign(size_t(e.size), 0);
          Out o{tmp.data(), 0, e.size};
          FillContent(r, o, pool, pool_off, n_pool, secrets_per_byte);
          uint64_t w = 0;
          for (uint64_t k = 0; k < e.size && w < e.size; k++) {
            if (tmp[k] == '\n') {
              d[w++] = '\r';
              if (w >= e.size) break;
            }
            d[w++] = tmp[k];
          }
        } else {  // ELF-like binary
          static const uint8_t elf[8] = {0x7F, 'E', 'L', 'F', 2, 1, 1, 0};
          for (uint64_t k = 0; k < e.size; k++) d[k] = uint8_t(r.Next());
          std::memcpy(d, elf, std::min<uint64_t>(8, e.size));
        }
      }
    }
  };
  std::vector<std::thread> pool_t;
  for (int t = 1; t < threads; t++) pool_t.emplace_back(work);
  work();
  for (auto& th : pool_t) th.join();
  std::memset(out + end, 0, 1024);
  return int64_t(total);
}

}  // extern "C"
