// The secret analyzer's ingest side (include/tsg_analyzer.h): the per-file
// work pkg/fanal/analyzer/secret/secret.go does before Scanner.Scan, the
// analyzer group's Required gate, and an uncompressed-tar layer walker
// (pkg/fanal/walker/tar.go), all packing straight into one batch arena.
#include <atomic>
#include <chrono>
#include <cstdio>
#include "tsg_analyzer.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>
#include <memory>
#include <pthread.h>
#include <thread>
#include <string>
#include <string_view>
#include <vector>

#include "capi_internal.h"
#include "parallel.h"

namespace tsg {
void SetError(const std::string& e);

// utils.IsBinary (utils.go:85-103): the head is min(size, 300) bytes.
bool IsBinaryHead(const uint8_t* p, uint64_t size) {
  const uint64_t n = size < 300 ? size : 300;
  uint64_t i = 0;
  // 32 bytes at a time: a byte below 0x20 is looked up by its low nibble in
  // the table of its half (0x00-0x0F / 0x10-0x1F); 0x7F compared directly
  const __m256i lo_tab = _mm256_setr_epi8(1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 1, 0, 0, 1, 1,  //
                                          1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 1, 0, 0, 1, 1);
  const __m256i hi_tab = _mm256_setr_epi8(1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 1, 1, 1, 1,  //
                                          1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 1, 1, 1, 1);
  for (; i + 32 <= n; i += 32) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p + i));
    const __m256i nib = _mm256_and_si256(v, _mm256_set1_epi8(0x0F));
    const __m256i lt16 = _mm256_cmpeq_epi8(_mm256_min_epu8(v, _mm256_set1_epi8(0x0F)), v);
    const __m256i lt32 = _mm256_cmpeq_epi8(_mm256_min_epu8(v, _mm256_set1_epi8(0x1F)), v);
    const __m256i t = _mm256_blendv_epi8(_mm256_shuffle_epi8(hi_tab, nib), _mm256_shuffle_epi8(lo_tab, nib), lt16);
    const __m256i bad = _mm256_or_si256(_mm256_and_si256(lt32, _mm256_cmpgt_epi8(t, _mm256_setzero_si256())),
                                        _mm256_cmpeq_epi8(v, _mm256_set1_epi8(0x7F)));
    if (_mm256_movemask_epi8(bad)) return true;
  }
  for (; i < n; i++) {
    const uint8_t b = p[i];
    if (b < 7 || b == 11 || (13 < b && b < 27) || (27 < b && b < 0x20) || b == 0x7f) return true;
  }
  return false;
}

// memcpy into a batch arena with non-temporal stores for the 32-B aligned
// middle: the arena is only read again by the DMA engine, so its lines need
// not be fetched for ownership (a plain copy of small files reads them) nor
// kept in the caches.  The caller fences (_mm_sfence) before the arena is
// handed on.
void CopyToArena(uint8_t* dst, const uint8_t* src, uint64_t n) {
  if (n < 256) {
    std::memcpy(dst, src, n);
    return;
  }
  const uint64_t head = (32 - (reinterpret_cast<uintptr_t>(dst) & 31)) & 31;
  std::memcpy(dst, src, head);
  uint64_t i = head;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
    const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), d);
  }
  for (; i + 32 <= n; i += 32)
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i),
                        _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i)));
  std::memcpy(dst + i, src + i, n - i);
}

// unicode.IsPrint(rune(b)) for a byte (Latin-1 code points): graphic
// characters and the ASCII space; U+00A0 and the soft hyphen U+00AD are not.
inline bool IsPrintByte(uint8_t b) { return (b >= 0x20 && b <= 0x7E) || (b >= 0xA1 && b != 0xAD); }

// utils.ExtractPrintableBytes (utils.go:128-160): minLength = 4, a run is kept
// when longer than that, each kept run is followed by '\n'.
uint64_t ExtractPrintable(const uint8_t* in, uint64_t n, uint8_t* out) {
  uint64_t w = 0, run = 0;  // the current run is in[i - run, i)
  for (uint64_t i = 0; i <= n; i++) {
    if (i < n && IsPrintByte(in[i])) {
      run++;
      continue;
    }
    if (run > 4) {
      std::memmove(out + w, in + i - run, run);
      w += run;
      out[w++] = '\n';
    }
    run = 0;
  }
  return w;
}

// Output length of ExtractPrintable without writing.
uint64_t PrintableLen(const uint8_t* in, uint64_t n) {
  uint64_t w = 0, run = 0;
  for (uint64_t i = 0; i <= n; i++) {
    if (i < n && IsPrintByte(in[i])) {
      run++;
      continue;
    }
    if (run > 4) w += run + 1;
    run = 0;
  }
  return w;
}

uint64_t CountCR(const uint8_t* in, uint64_t n) {
  uint64_t k = 0;
  for (const uint8_t* p = in; (p = static_cast<const uint8_t*>(std::memchr(p, '\r', size_t(in + n - p)))); p++) k++;
  return k;
}

// bytes.ReplaceAll(content, "\r", "") (secret.go:121), memchr-driven.
uint64_t StripCR(const uint8_t* in, uint64_t n, uint8_t* out) {
  uint64_t r = 0, w = 0;
  while (r < n) {
    const void* q = std::memchr(in + r, '\r', size_t(n - r));
    const uint64_t e = q ? uint64_t(static_cast<const uint8_t*>(q) - in) : n;
    if (out + w != in + r) std::memmove(out + w, in + r, size_t(e - r));
    w += e - r;
    r = e + (q ? 1 : 0);
  }
  return w;
}

// True when path.Clean(p) == p: no empty, "." or ".." element, no trailing
// slash (other than the root itself).  Most archive names already are clean.
inline bool GoPathIsClean(const char* p, size_t n) {
  if (n == 0) return false;
  if (n == 1) return p[0] != '.';
  if (p[n - 1] == '/') return false;
  size_t s = 0;  // element start
  for (size_t i = 0; i <= n; i++) {
    if (i < n && p[i] != '/') continue;
    const size_t len = i - s;
    if (len == 0 && i != 0) return false;                      // "//" (a leading '/' is the root)
    if (len == 1 && p[s] == '.') return false;                 // "."
    if (len == 2 && p[s] == '.' && p[s + 1] == '.') return false;  // ".."
    s = i + 1;
  }
  return true;
}

// path.Clean (Go, slash-separated).
std::string GoPathClean(const std::string& path) {
  if (path.empty()) return ".";
  if (GoPathIsClean(path.data(), path.size())) return path;
  const bool rooted = path[0] == '/';
  const size_t n = path.size();
  std::string out;
  out.reserve(n + 1);
  size_t r = 0, dotdot = 0;
  if (rooted) {
    out.push_back('/');
    r = dotdot = 1;
  }
  while (r < n) {
    if (path[r] == '/') {
      r++;
    } else if (path[r] == '.' && (r + 1 == n || path[r + 1] == '/')) {
      r++;
    } else if (path[r] == '.' && path[r + 1] == '.' && (r + 2 == n || path[r + 2] == '/')) {
      r += 2;
      if (out.size() > dotdot) {  // back to the last '/' at or after dotdot (Go: w--, then while out[w] != '/')
        size_t w = out.size() - 1;
        while (w > dotdot && out[w] != '/') w--;
        out.resize(w);
      } else if (!rooted) {
        if (!out.empty()) out.push_back('/');
        out += "..";
        dotdot = out.size();
      }
    } else {
      if ((rooted && out.size() != 1) || (!rooted && !out.empty())) out.push_back('/');
      for (; r < n && path[r] != '/'; r++) out.push_back(path[r]);
    }
  }
  if (out.empty()) return ".";
  return out;
}

// filepath.Ext / filepath.Base (Unix).
std::string GoExt(const std::string& p) {
  for (size_t i = p.size(); i-- > 0 && p[i] != '/';)
    if (p[i] == '.') return p.substr(i);
  return "";
}
std::string GoBase(std::string p) {
  if (p.empty()) return ".";
  while (!p.empty() && p.back() == '/') p.pop_back();
  if (p.empty()) return "/";
  const size_t k = p.rfind('/');
  return k == std::string::npos ? p : p.substr(k + 1);
}

// secret.go:28-62 (skipFiles, skipDirs, skipExts): inlined in Required below
}  // namespace tsg

#include "collector.h"

namespace tsg {
bool RequiredPath(const tsg_analyzer* a, const char* path, uint64_t len, int64_t size);
}
namespace {
bool Required(const tsg_analyzer* a, const char* path, uint64_t len, int64_t size) {  // secret.go:152-190
  if (size < 10) return false;
  const std::string_view fp(path, size_t(len));
  const size_t slash = fp.rfind('/');
  const std::string_view dir = slash == std::string_view::npos ? std::string_view() : fp.substr(0, slash + 1);
  const std::string_view name = slash == std::string_view::npos ? fp : fp.substr(slash + 1);
  // strings.Split(dir, "/") holds a skip dir: dir (which ends in '/') starts
  // with "<skip>/" or contains "/<skip>/"
  constexpr std::string_view kGit = "/.git/", kNode = "/node_modules/";
  if (dir.substr(0, kGit.size() - 1) == kGit.substr(1) || dir.substr(0, kNode.size() - 1) == kNode.substr(1))
    return false;
  for (size_t q = dir.find('/'); q != std::string_view::npos; q = dir.find('/', q + 1)) {
    const std::string_view rest = dir.substr(q);
    if (rest.substr(0, kGit.size()) == kGit || rest.substr(0, kNode.size()) == kNode) return false;
  }
  static constexpr std::string_view kFiles[] = {"go.mod", "go.sum", "package-lock.json", "yarn.lock",
                                                "pnpm-lock.yaml", "Pipfile.lock", "Gemfile.lock"};
  for (const std::string_view f : kFiles)
    if (name == f) return false;
  if (a->config_base == fp) return false;
  const size_t dot = name.rfind('.');  // filepath.Ext
  if (dot != std::string_view::npos && name.size() - dot <= 7) {
    static constexpr std::string_view kExts[] = {".jpg", ".png", ".gif", ".doc", ".pdf", ".bin", ".svg",
                                                 ".socket", ".deb", ".rpm", ".zip", ".gz", ".gzip", ".tar"};
    const std::string_view ext = name.substr(dot);
    for (const std::string_view x : kExts)
      if (ext == x) return false;
  }
  if (a->s->s->AllowPath(reinterpret_cast<const uint8_t*>(path), size_t(len))) return false;
  return true;
}
}  // namespace
namespace tsg {
bool RequiredPath(const tsg_analyzer* a, const char* path, uint64_t len, int64_t size) {
  return Required(a, path, len, size);
}
}  // namespace tsg
namespace {

// Analyze up to the Scan call (secret.go:103-136).
int64_t Add(tsg_collector* c, const char* path, uint64_t plen, bool image, const uint8_t* content, uint64_t size) {
  const bool bin = tsg::IsBinaryHead(content, size);
  if (bin && tsg::GoExt(std::string(path, size_t(plen))) != ".pyc") return TSG_SKIPPED;
  const uint64_t need = bin ? size + size / 5 + 1 : size;
  if (c->files() > 0 && c->acct() + need > c->limit) return TSG_FULL;
  if (c->used + need + 64 > c->cap) {  // only a lone file larger than the batch gets here
    if (c->files() > 0) return TSG_FULL;
    if (!c->Reserve(need + 64)) return -3;
  }
  uint8_t* dst = c->arena + c->used;
  uint64_t len;
  if (c->gpu_xform) {  // as read; the GPU transforms it
    std::memcpy(dst, content, size);
    len = size;
    c->bound += need;
    c->kinds.push_back(bin ? 2 : 1);
  } else {
    len = bin ? tsg::ExtractPrintable(content, size, dst) : tsg::StripCR(content, size, dst);
  }
  c->used += len;
  std::memset(c->arena + c->used, 0, 64);  // the engine reads up to 64 B past the end
  c->offs.push_back(c->used);
  if (image) c->path_pool.push_back('/');  // files extracted from an image (secret.go:130-135)
  c->path_pool.append(path, size_t(plen));
  c->path_off.push_back(c->path_pool.size());
  c->binary.push_back(bin ? 1 : 0);
  c->input_bytes += size;
  return int64_t(c->files() - 1);
}

// ---- archive/tar header reading (Go 1.22 archive/tar/reader.go semantics) ----
bool AllZero(const uint8_t* b) {
  uint64_t acc;
  std::memcpy(&acc, b, 8);  // a header starts with its name: almost always decided here
  if (acc) return false;
  for (int i = 0; i < 64; i++) {
    uint64_t w;
    std::memcpy(&w, b + 8 * i, 8);
    acc |= w;
  }
  return acc == 0;
}
std::string CStr(const uint8_t* b, size_t n) {  // parseString: up to the first NUL
  size_t k = 0;
  while (k < n && b[k]) k++;
  return std::string(reinterpret_cast<const char*>(b), k);
}
bool ParseNumeric(const uint8_t* b, size_t n, int64_t* out) {  // parseNumeric
  if (n > 0 && (b[0] & 0x80)) {  // base-256 (two's complement, big-endian)
    const bool neg = b[0] & 0x40;
    uint64_t v = 0;
    for (size_t i = 0; i < n; i++) {
      uint8_t c = i == 0 ? (b[0] & 0x7F) : b[i];
      if (neg) c ^= 0xFF;
      if (i == 0 && neg) c &= 0x7F;
      if (v >> 56) return false;
      v = (v << 8) | c;
    }
    if (v >> 63) return false;
    *out = neg ? -int64_t(v) - 1 : int64_t(v);
    return true;
  }
  // parseOctal: trim spaces and NULs at both ends
  size_t lo = 0, hi = n;
  while (lo < hi && (b[lo] == ' ' || b[lo] == 0)) lo++;
  while (hi > lo && (b[hi - 1] == ' ' || b[hi - 1] == 0)) hi--;
  int64_t v = 0;
  for (size_t i = lo; i < hi; i++) {
    if (b[i] < '0' || b[i] > '7') return false;
    if (v >> 60) return false;
    v = v * 8 + (b[i] - '0');
  }
  *out = v;
  return true;
}
bool ChecksumOK(const uint8_t* b) {
  int64_t want = 0;
  if (!ParseNumeric(b + 148, 8, &want)) return false;
  // the unsigned byte sum with the checksum field read as spaces, else the
  // signed one (old writers); plain loops, vectorised by the compiler
  __m256i acc = _mm256_setzero_si256();  // unsigned sum: psadbw against zero, 32 B a step
  for (int i = 0; i < 512; i += 32)
    acc = _mm256_add_epi64(acc, _mm256_sad_epu8(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(b + i)),
                                                 _mm256_setzero_si256()));
  int32_t u = int32_t(_mm256_extract_epi64(acc, 0) + _mm256_extract_epi64(acc, 1) + _mm256_extract_epi64(acc, 2) +
                      _mm256_extract_epi64(acc, 3));
  for (int i = 148; i < 156; i++) u += ' ' - b[i];
  if (want == u) return true;
  int32_t s = 0;
  for (int i = 0; i < 512; i++) s += int8_t(b[i]);
  for (int i = 148; i < 156; i++) s += ' ' - int8_t(b[i]);
  return want == s;
}
// PAX records "%d %s=%s\n" (parsePAX): path, size and linkpath matter here.
bool ParsePax(const uint8_t* d, uint64_t n, std::string* path, int64_t* size, bool* has_path, bool* has_size) {
  uint64_t p = 0;
  while (p < n) {
    uint64_t sp = p;
    while (sp < n && d[sp] != ' ') sp++;
    if (sp >= n) return false;
    uint64_t len = 0;
    for (uint64_t i = p; i < sp; i++) {
      if (d[i] < '0' || d[i] > '9') return false;
      len = len * 10 + (d[i] - '0');
    }
    if (len < sp - p + 2 || p + len > n || d[p + len - 1] != '\n') return false;
    const std::string rec(reinterpret_cast<const char*>(d + sp + 1), size_t(len - (sp + 1 - p) - 1));
    const size_t eq = rec.find('=');
    if (eq == std::string::npos) return false;
    const std::string k = rec.substr(0, eq), v = rec.substr(eq + 1);
    if (k == "path") {
      *path = v;
      *has_path = true;
    } else if (k == "size") {
      char* e = nullptr;
      *size = std::strtoll(v.c_str(), &e, 10);
      if (v.empty() || *e) return false;
      *has_size = true;
    }
    p += len;
  }
  return true;
}
bool HeaderOnly(char t) { return t == '1' || t == '2' || t == '3' || t == '4' || t == '5' || t == '6'; }
}  // namespace

extern "C" {

int tsg_is_binary(const uint8_t* content, uint64_t size) { return tsg::IsBinaryHead(content, size) ? 1 : 0; }
uint64_t tsg_extract_printable(const uint8_t* in, uint64_t n, uint8_t* out) { return tsg::ExtractPrintable(in, n, out); }
uint64_t tsg_strip_cr(const uint8_t* in, uint64_t n, uint8_t* out) { return tsg::StripCR(in, n, out); }

int tsg_analyzer_new(const tsg_scanner* s, const char* config_path, tsg_analyzer** out) {
  if (!s || !out) {
    tsg::SetError("tsg_analyzer_new: null argument");
    return -1;
  }
  auto* a = new tsg_analyzer();
  a->s = s;
  a->config_base = tsg::GoBase(config_path ? config_path : "");
  *out = a;
  return 0;
}
void tsg_analyzer_free(tsg_analyzer* a) { delete a; }

int tsg_analyzer_required(const tsg_analyzer* a, const char* path, uint64_t path_len, int64_t size) {
  return Required(a, path, path_len, size) ? 1 : 0;
}

int tsg_collector_new(tsg_analyzer* a, uint64_t arena_bytes, tsg_collector** out) {
  if (!a || !out) {
    tsg::SetError("tsg_collector_new: null analyzer or out");
    return -1;
  }
  auto* c = new tsg_collector();
  c->a = a;
  c->device = a->s->s->device();
  c->limit = arena_bytes ? arena_bytes : (uint64_t(256) << 20);
  if (const char* e = std::getenv("TSG_HOST_THREADS")) c->threads = std::max(1, std::atoi(e));
  if (!c->Reserve(c->limit + 64)) {
    delete c;
    return -1;
  }
  *out = c;
  return 0;
}
void tsg_collector_free(tsg_collector* c) { delete c; }

int64_t tsg_collector_add(tsg_collector* c, const char* path, uint64_t path_len, const char* dir,
                          const uint8_t* content, uint64_t size) {
  if (c->gather) {
    tsg::SetError("tsg_collector_add: the collector gathers from tar layers (tsg_collector_set_gather)");
    return -3;
  }
  return Add(c, path, path_len, !dir || !*dir, content, size);
}

}  // extern "C"

namespace tsg {
// One archive entry as the walk sees it (header chain resolved).
struct TarEntry {
  uint64_t start, next;  // header chain start, next entry
  uint64_t hdr;          // the entry's own header
  uint64_t data, size;   // content
  uint64_t long_off, long_len;  // GNU 'L' long name data (long_len == ~0: none)
  uint8_t what;          // 0 other, 1 whiteout, 2 opaque dir, 3 regular file
  uint8_t has_pax_path;
  uint8_t bad;           // the entry header's checksum is wrong (checked on the threads)
  // The cleaned path (walker/tar.go:46-48): a view of the header's name field
  // in the archive itself when that is already the answer (a ustar name with
  // no prefix, clean), else an owned string (PAX / GNU long names, prefixes,
  // names that Clean changes) -- no allocation per entry on the common path.
  std::unique_ptr<std::string> fp_own;  // set: the path is *fp_own
  uint64_t fp_off = 0;
  uint32_t fp_len = 0;
  std::string_view path(const uint8_t* tar) const {
    return fp_own ? std::string_view(*fp_own) : std::string_view(reinterpret_cast<const char*>(tar + fp_off), fp_len);
  }
  void own(std::string v) { fp_own.reset(new std::string(std::move(v))); }
  // filled by the parallel pass
  uint8_t state;         // 0 not required, 1 binary skipped, 2 add
  uint8_t bin;
  uint64_t out_len, out_off;
};

}  // namespace tsg

namespace {
using tsg::TarEntry;

// Sequential step of the walk: hop over the header chain starting at p using
// only what decides the next entry's position (zero block, typeflag, size,
// PAX size).  Extended headers are checked here (rare); the entry header's
// checksum and name are resolved later on the ingest threads (Resolve).
// 0 = entry read, 1 = end of archive, <0 = malformed.
int ChainEntry(const uint8_t* tar, uint64_t n, uint64_t p, TarEntry* e) {
  e->start = p;
  e->long_len = ~uint64_t(0);
  e->has_pax_path = 0;
  std::string pax_path;
  bool has_pax_path = false, has_pax_size = false;
  int64_t pax_size = 0, size = 0;
  const uint8_t* h = nullptr;
  char type = 0;
  for (;;) {
    if (p + 512 > n) {
      if (p >= n) return 1;  // io.EOF without the zero blocks
      tsg::SetError("tar: truncated header");
      return -1;
    }
    h = tar + p;
    if (AllZero(h)) return 1;  // end-of-archive marker
    type = char(h[156]);
    if (!ParseNumeric(h + 124, 12, &size) || size < 0) {
      tsg::SetError("tar: invalid size field");
      return -1;
    }
    const uint64_t dsz = HeaderOnly(type) ? 0 : uint64_t(size);
    const uint64_t data = p + 512;
    if (data + dsz > n) {
      tsg::SetError("tar: truncated entry data");
      return -1;
    }
    if (type != 'x' && type != 'L' && type != 'K') break;
    if (!ChecksumOK(h)) {
      tsg::SetError("tar: invalid header checksum at offset " + std::to_string(p));
      return -1;
    }
    if (type == 'x' && !ParsePax(tar + data, dsz, &pax_path, &pax_size, &has_pax_path, &has_pax_size)) {
      tsg::SetError("tar: invalid PAX record");
      return -1;
    }
    if (type == 'L') {
      e->long_off = data;
      e->long_len = dsz;
    }
    p = data + ((dsz + 511) & ~uint64_t(511));
  }
  e->hdr = p;
  if (has_pax_size) size = pax_size;
  if (type == '\0') {  // TypeRegA: a directory when the name ends in '/' (resolved name: Resolve)
    type = '0';
  }
  const uint64_t dsz = HeaderOnly(type) ? 0 : uint64_t(size);
  e->data = p + 512;
  if (e->data + dsz > n) {
    tsg::SetError("tar: truncated entry data");
    return -1;
  }
  e->size = dsz;
  e->next = e->data + ((dsz + 511) & ~uint64_t(511));
  e->what = type == '0' ? 3 : 0;
  if (has_pax_path) {
    e->own(std::move(pax_path));
    e->has_pax_path = 1;
  }
  return 0;
}

void Classify(const uint8_t* tar, TarEntry* e);

// Everything the walk decides about one entry, on the thread that indexed it
// (its header and path are still in that core's cache): the name (Classify),
// AnalyzeFile's Required, Analyze's binary gate and the transformed length.
std::atomic<int64_t> g_eval_ns[3];
struct EvalCtx {  // what Evaluate needs of the collector (copied: a background index outlives the call)
  const tsg_analyzer* a;
  bool gpu_xform;
};
void Evaluate(const EvalCtx* c, const uint8_t* tar, TarEntry* e) {
  static const bool dbg = std::getenv("TSG_WALK_DEBUG") && std::atoi(std::getenv("TSG_WALK_DEBUG")) >= 2;  // per-entry timers: level 2
  auto t0 = dbg ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
  Classify(tar, e);
  e->state = 0;
  if (dbg) {
    auto t1 = std::chrono::steady_clock::now();
    g_eval_ns[0] += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    const std::string_view fp = e->path(tar);
    const bool req = e->what == 3 && Required(c->a, fp.data(), fp.size(), int64_t(e->size));
    g_eval_ns[1] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t1).count();
    if (!req) return;
  } else if (e->what != 3 || !Required(c->a, e->path(tar).data(), e->path(tar).size(), int64_t(e->size))) {
    return;
  }
  const uint8_t* d = tar + e->data;
  e->bin = tsg::IsBinaryHead(d, e->size) ? 1 : 0;
  if (e->bin && tsg::GoExt(std::string(e->path(tar))) != ".pyc") {
    e->state = 1;
    return;
  }
  e->state = 2;
  if (c->gpu_xform)  // the largest transformed size: the batch limit counts it, the GPU transforms
    e->out_len = e->bin ? e->size + e->size / 5 + 1 : e->size;
  else
    e->out_len = e->bin ? tsg::PrintableLen(d, e->size) : e->size - tsg::CountCR(d, e->size);
}

// Entries of [p, ...) as the sequential walk reads them, the index found in
// parallel: the window [p, p + window) is cut into segments; each segment's
// thread starts at its first block that parses as a header (segment 0: at p)
// and follows the header chain while it stays in the segment.  The merge then
// takes a segment's entries from the one starting where the true chain
// arrives (chains that meet coincide from there: ChainEntry depends on the
// start position only); when no speculative entry starts there (a segment
// start inside file data that looked like a header, or a header chain cut in
// two) that segment is walked sequentially from the true position.  Stops
// after `max_regular` bytes of regular files (at least one entry), at the end
// of the archive (*at_end) or on a malformed header (-1).
int IndexEntries(const EvalCtx* c, const uint8_t* tar, uint64_t n, uint64_t p, uint64_t window,
                 uint64_t max_regular, int threads, std::vector<std::vector<TarEntry>>& spec,
                 std::vector<std::vector<TarEntry>>& fallback, std::vector<TarEntry*>* out, uint64_t* next,
                 bool* at_end) {
  // *out points into spec / fallback, which hold the entries until the next call
  out->clear();
  fallback.clear();
  fallback.reserve(size_t(std::max(1, threads) * 4) + 8);
  *at_end = false;
  const uint64_t end = std::min<uint64_t>(n, p + window);
  const size_t n_seg = size_t(std::max(1, threads) * 4);
  const uint64_t seg = std::max<uint64_t>(((end - p) / n_seg + 511) & ~uint64_t(511), 1 << 16);
  const size_t segs = size_t(std::max<uint64_t>(1, (end - p + seg - 1) / seg));
  // per-segment vectors kept across windows (their pages stay mapped)
  if (spec.size() < segs) spec.resize(segs);
  for (auto& v : spec) v.clear();
  static const bool dbg = std::getenv("TSG_WALK_DEBUG") != nullptr;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t0 = dbg ? now() : 0;
  tsg::ParallelFor(segs, threads, [&](size_t s) {
    const uint64_t a = p + s * seg, b = std::min(end, a + seg);
    spec[s].reserve(size_t(seg / 2048) + 8);
    uint64_t q = a;
    if (s > 0) {  // first block that parses as a header (512-aligned from p)
      while (q + 512 <= b && (AllZero(tar + q) || !ChecksumOK(tar + q))) q += 512;
    }
    while (q < b) {
      TarEntry e;
      if (ChainEntry(tar, n, q, &e) != 0) break;  // end marker or garbage: the merge decides
      q = e.next;
      // the next header (all 8 lines: its checksum reads them) and this
      // entry's content head (IsBinaryHead) are on their way while this
      // entry is evaluated: the chain is a walk through cold memory
      if (q + 512 <= n)
        for (int l = 0; l < 512; l += 64) __builtin_prefetch(tar + q + l);
      if (e.size) {
        __builtin_prefetch(tar + e.data);
        __builtin_prefetch(tar + e.data + 64);
      }
      Evaluate(c, tar, &e);
      spec[s].push_back(std::move(e));
    }
  }, true);
  // The merge plans ranges of the speculative vectors (and of the rare
  // sequential fallbacks) first, reading only positions and sizes; *out then
  // gets pointers to the entries, filled in parallel.
  struct Range {
    std::vector<TarEntry>* v;
    size_t lo, hi;
  };
  const double t1 = dbg ? now() : 0;
  size_t n_fallback = 0;
  std::vector<Range> plan;
  uint64_t cur = p, regular = 0;
  bool ended = false;
  for (size_t s = 0; s < segs && !ended; s++) {
    const uint64_t b = std::min(end, p + (s + 1) * seg);
    if (cur >= b) continue;
    auto& v = spec[s];
    auto it = std::lower_bound(v.begin(), v.end(), cur, [](const TarEntry& e, uint64_t x) { return e.start < x; });
    if (it != v.end() && it->start == cur) {
      const size_t lo = size_t(it - v.begin());
      size_t i = lo;
      for (; i < v.size();) {
        cur = v[i].next;
        if (v[i].what == 3) regular += v[i].size + 512;
        i++;
        if (regular > max_regular) break;
      }
      plan.push_back({&v, lo, i});
    }
    if (cur < b && regular <= max_regular) {  // sequential from the true position
      fallback.emplace_back();
      auto& fb = fallback.back();
      while (cur < b && regular <= max_regular) {
        TarEntry e;
        const int r = ChainEntry(tar, n, cur, &e);
        if (r < 0) return -1;
        if (r == 1) {
          *at_end = true;
          ended = true;
          break;
        }
        cur = e.next;
        Evaluate(c, tar, &e);
        if (e.what == 3) regular += e.size + 512;
        fb.push_back(std::move(e));
        n_fallback++;
      }
      plan.push_back({&fb, 0, fb.size()});
    }
    if (regular > max_regular) break;
  }
  {
    std::vector<size_t> at(plan.size() + 1, 0);
    for (size_t k = 0; k < plan.size(); k++) at[k + 1] = at[k] + (plan[k].hi - plan[k].lo);
    out->resize(at.back());
    tsg::ParallelFor(plan.size(), threads, [&](size_t k) {
      for (size_t i = plan[k].lo; i < plan[k].hi; i++) (*out)[at[k] + (i - plan[k].lo)] = &(*plan[k].v)[i];
    }, true);
  }
  if (dbg) {
    size_t n_spec = 0;
    for (auto& v : spec) n_spec += v.size();
    std::fprintf(stderr, "index: segs %zu spec %.3f s (%zu entries) merge+move %.3f s (kept %zu, fallback %zu)\n", segs,
                 t1 - t0, n_spec, now() - t1, out->size(), n_fallback);
  }
  if (ended) {
    *next = cur;
    return 0;
  }
  if (out->empty() || (cur >= n && !*at_end)) {  // nothing in the window (a huge entry) or the tail
    fallback.emplace_back();
    auto& fb = fallback.back();
    while (out->empty() && fb.empty()) {
      TarEntry e;
      const int r = ChainEntry(tar, n, cur, &e);
      if (r < 0) return -1;
      if (r == 1) {
        *at_end = true;
        break;
      }
      cur = e.next;
      Evaluate(c, tar, &e);
      fb.push_back(std::move(e));
    }
    for (auto& e : fb) out->push_back(&e);
  }
  if (!*at_end && cur >= n) *at_end = true;  // io.EOF without the zero blocks
  if (!*at_end && regular <= max_regular && cur < n && end >= n) {
    // window reached the archive's end region: check for the end marker at cur
    TarEntry e;
    const int r = ChainEntry(tar, n, cur, &e);
    if (r < 0) return -1;
    if (r == 1) *at_end = true;
  }
  *next = cur;
  return 0;
}

}  // namespace

namespace tsg {
// Entries indexed and evaluated ahead of the walk's cursor (see tsg_collector_add_tar).
struct TarWindow {  // a window of entries indexed from `start`
  std::vector<TarEntry*> ents;              // the window's entries in archive order
  std::vector<std::vector<TarEntry>> spec;  // their storage: IndexEntries' per-segment vectors
  std::vector<std::vector<TarEntry>> fallback;  // and its sequential fallbacks
  uint64_t start = 0;
  uint64_t next = 0;     // the position after the last indexed entry
  bool at_end = false;   // the archive ends at `next`
};
struct TarWalkCache {
  const uint8_t* tar = nullptr;
  uint64_t n = 0;
  bool gpu_xform = false;
  TarWindow w;
  size_t pos = 0;        // the next entry of w to accept
  // The window after w, indexed on a background thread while the batches of w
  // are accepted and scanned (tsg_collector_add_tar); it reads the archive
  // after the call that started it returned -- the buffer-lifetime rule of
  // tsg_analyzer.h.
  TarWindow ahead;
  const uint8_t* ahead_tar = nullptr;
  uint64_t ahead_n = 0;
  bool ahead_xform = false, ahead_ok = false;
  std::thread bg;
  void Join() {
    if (bg.joinable()) bg.join();
  }
  ~TarWalkCache() { Join(); }
};
void FreeTarWalkCache(TarWalkCache* w) { delete w; }
void EndTarWalk(TarWalkCache* w) {
  if (!w) return;
  w->Join();
  // nothing of the ended walk may be reused: a later layer buffer at the same
  // address must not hit the cached window of this one
  w->ahead_ok = false;
  w->ahead_tar = nullptr;
  w->ahead = TarWindow();
  w->tar = nullptr;
  w->n = 0;
  w->w = TarWindow();
  w->pos = 0;
}
}  // namespace tsg

namespace {
// The entry's name (ustar prefix, GNU long name, PAX path) and header checksum.
void Resolve(const uint8_t* tar, TarEntry* e) {
  const uint8_t* h = tar + e->hdr;
  e->bad = ChecksumOK(h) ? 0 : 1;
  if (e->has_pax_path) return;
  if (e->long_len != ~uint64_t(0)) {
    e->own(CStr(tar + e->long_off, size_t(e->long_len)));
  } else {
    auto clen = [](const uint8_t* b, size_t n) {
      const void* z = std::memchr(b, 0, n);
      return z ? size_t(static_cast<const uint8_t*>(z) - b) : n;
    };
    const size_t nl = clen(h, 100);
    size_t pl = 0;
    if (std::memcmp(h + 257, "ustar\0", 6) == 0 && std::memcmp(h + 263, "00", 2) == 0) pl = clen(h + 345, 155);
    if (pl) {
      std::string v;
      v.reserve(pl + 1 + nl);
      v.append(reinterpret_cast<const char*>(h + 345), pl);
      v.push_back('/');
      v.append(reinterpret_cast<const char*>(h), nl);
      e->own(std::move(v));
    } else {
      e->fp_own.reset();
      e->fp_off = e->hdr;
      e->fp_len = uint32_t(nl);
    }
  }
}

// LayerTar.Walk's per-entry path logic (walker/tar.go:41-84): clean the name,
// classify whiteout / opaque markers.
void Classify(const uint8_t* tar, TarEntry* e) {
  Resolve(tar, e);
  std::string_view fp = e->path(tar);
  if (tar[e->hdr + 156] == '\0' && !fp.empty() && fp.back() == '/') e->what = 0;  // TypeRegA dir
  if (!tsg::GoPathIsClean(fp.data(), fp.size())) {
    e->own(tsg::GoPathClean(std::string(fp)));
    fp = *e->fp_own;
  }
  size_t t = 0;
  while (t < fp.size() && fp[t] == '/') t++;
  if (t) {
    if (e->fp_own) {
      e->fp_own->erase(0, t);
    } else {
      e->fp_off += t;
      e->fp_len -= uint32_t(t);
    }
    fp = e->path(tar);
  }
  const size_t slash = fp.rfind('/');
  const std::string_view file_name = fp.substr(slash == std::string_view::npos ? 0 : slash + 1);
  if (file_name == ".wh..wh..opq") e->what = 2;
  else if (file_name.substr(0, 4) == ".wh.") e->what = 1;
}
}  // namespace

namespace {
// The bulk part of the walk's accept step: the longest run of whole
// kAcceptBlock-entry blocks from k0 that fits the batch (limit and arena) and
// holds no bad header, appended to the collector exactly as the entry-by-entry
// loop would (same offsets, paths, kinds, flags, stats).  Returns the number
// of entries taken.
constexpr size_t kAcceptBlock = 4096;
size_t AcceptBlocks(tsg_collector* c, const uint8_t* tar, std::vector<TarEntry*>& ents, size_t k0, tsg_tar_stats* st) {
  const size_t nb = (ents.size() - k0) / kAcceptBlock;
  if (nb == 0) return 0;
  struct Sum {
    uint64_t files = 0, used = 0, acct = 0, pbytes = 0, input = 0;
    uint64_t entries = 0, whiteouts = 0, opaque = 0, regular = 0, required = 0, skipped = 0;
    bool bad = false;
  };
  std::vector<Sum> sum(nb);
  tsg::ParallelFor(nb, c->threads, [&](size_t b) {
    Sum& q = sum[b];
    for (size_t i = k0 + b * kAcceptBlock; i < k0 + (b + 1) * kAcceptBlock; i++) {
      const TarEntry& e = *ents[i];
      q.bad = q.bad || e.bad;
      if (e.state == 2) {
        q.files++;
        q.used += c->gpu_xform ? e.size : e.out_len;
        q.acct += e.out_len;
        q.pbytes += 1 + e.path(tar).size();
        q.input += e.size;
      }
      q.whiteouts += e.what == 1;
      q.opaque += e.what == 2;
      q.regular += e.what == 3;
      q.required += e.state != 0;
      q.skipped += e.state == 1;
    }
    q.entries = kAcceptBlock;
  }, true);
  // the blocks that fit, and each one's starting row
  std::vector<Sum> at(1);
  uint64_t acct = c->acct(), used = c->used;
  size_t m = 0;
  for (; m < nb; m++) {
    const Sum& q = sum[m];
    if (q.bad || acct + q.acct > c->limit || used + q.used + 64 > c->cap) break;
    acct += q.acct;
    used += q.used;
    Sum n = at.back();
    n.files += q.files;
    n.used += q.used;
    n.pbytes += q.pbytes;
    at.push_back(n);
  }
  if (m == 0) return 0;
  const size_t f0 = c->files(), p0 = c->path_pool.size();
  const uint64_t u0 = c->used;
  const Sum& tot = at[m];
  c->offs.resize(f0 + 1 + tot.files);
  c->path_off.resize(f0 + 1 + tot.files);
  c->path_pool.resize(p0 + tot.pbytes);
  c->binary.resize(f0 + tot.files);
  if (c->gpu_xform) c->kinds.resize(f0 + tot.files);
  if (c->gather) c->gsrc.resize(f0 + tot.files);
  tsg::ParallelFor(m, c->threads, [&](size_t b) {
    size_t f = f0 + at[b].files, pp = p0 + at[b].pbytes;
    uint64_t u = u0 + at[b].used;
    for (size_t i = k0 + b * kAcceptBlock; i < k0 + (b + 1) * kAcceptBlock; i++) {
      TarEntry& e = *ents[i];
      if (e.state != 2) continue;
      e.out_off = u;
      u += c->gpu_xform ? e.size : e.out_len;
      if (c->gpu_xform) c->kinds[f] = e.bin ? 2 : 1;
      if (c->gather) c->gsrc[f] = e.data;
      c->binary[f] = e.bin;
      c->offs[f + 1] = u;
      const std::string_view fp = e.path(tar);
      c->path_pool[pp] = '/';  // Dir "" (image files, secret.go:130-135)
      std::memcpy(&c->path_pool[pp + 1], fp.data(), fp.size());
      pp += 1 + fp.size();
      c->path_off[f + 1] = pp;
      f++;
    }
  }, true);
  for (size_t b = 0; b < m; b++) {
    const Sum& q = sum[b];
    c->used += q.used;
    if (c->gpu_xform) c->bound += q.acct;
    c->input_bytes += q.input;
    st->added += q.files;
    st->input_bytes += q.input;
    st->entries += q.entries;
    st->whiteouts += q.whiteouts;
    st->opaque_dirs += q.opaque;
    st->regular += q.regular;
    st->required += q.required;
    st->skipped_binary += q.skipped;
  }
  return m * kAcceptBlock;
}

}  // namespace

extern "C" {

// The walk runs in rounds: index a window of entries ahead of the cursor in
// parallel (each evaluated on the thread that found it: name, Required,
// binary gate, transformed length), accept the longest prefix that fits the
// batch, copy the accepted contents on the threads.  The window is several
// batches long and its entries past this batch stay in the analyzer's walk
// cache, so the next call (on this or the other collector of a pipeline)
// starts accepting at once: one parallel index pass per window instead of a
// shrinking series of them per batch.
int tsg_collector_add_tar(tsg_collector* c, const uint8_t* tar, uint64_t n, uint64_t* cursor, tsg_tar_stats* st) {
  tsg_tar_stats local{};
  if (!st) st = &local;
  if (c->gather) {  // a gathered batch holds one layer's files (one gather_base)
    if (c->files() > 0 && c->gbase != tar) return 1;
    c->gbase = tar;
  }
  std::lock_guard<std::mutex> walk_lock(c->a->walk_mu);
  if (!c->a->walk) c->a->walk = new tsg::TarWalkCache();
  tsg::TarWalkCache& W = *c->a->walk;
  uint64_t p = *cursor;
  static const bool dbg = std::getenv("TSG_WALK_DEBUG") != nullptr;
  static const uint64_t ahead = std::getenv("TSG_WALK_AHEAD") ? uint64_t(std::atoi(std::getenv("TSG_WALK_AHEAD"))) : 8;
  static double t_phase[4];
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const EvalCtx ectx{c->a, c->gpu_xform};
  // the next window on a background thread only when the caller opted in
  // (tsg_analyzer_set_walk_ahead; TSG_WALK_BG=0 turns it off everywhere)
  static const bool bg_env = !std::getenv("TSG_WALK_BG") || std::atoi(std::getenv("TSG_WALK_BG")) != 0;
  const bool bg_index = bg_env && c->a->walk_ahead;
  for (;;) {
    // 1. the cached entries from p on, else the window indexed ahead in the
    // background (when it starts at p), else index a window starting at p
    double t0 = dbg ? now() : 0;
    const bool hit = W.tar == tar && W.n == n && W.gpu_xform == c->gpu_xform &&
                     ((W.pos < W.w.ents.size() && W.w.ents[W.pos]->start == p) ||
                      (W.pos == W.w.ents.size() && W.w.next == p && W.w.at_end));
    if (!hit) {
      const uint64_t room = std::max<uint64_t>(c->limit, 1 << 20);
      const uint64_t window = ahead * room + (1 << 20);
      W.Join();  // the background window (if any) is complete, or this walk moved elsewhere
      const bool take = W.ahead_ok && W.ahead_tar == tar && W.ahead_n == n && W.ahead_xform == c->gpu_xform &&
                        W.ahead.start == p;
      W.ahead_ok = false;
      W.tar = tar;
      W.n = n;
      W.gpu_xform = c->gpu_xform;
      W.pos = 0;
      if (take) {
        std::swap(W.w, W.ahead);
      } else {
        W.w.start = p;
        W.w.at_end = false;
        // every entry indexed in the window is kept (no re-indexing past a cut)
        if (IndexEntries(&ectx, tar, n, p, window, ~uint64_t(0) >> 1, c->threads, W.w.spec, W.w.fallback, &W.w.ents,
                         &W.w.next, &W.w.at_end) < 0) {
          W.tar = nullptr;
          W.Join();
          return -1;
        }
      }
      if (bg_index && !W.w.at_end && W.w.next < n) {
        // the next window on a background thread (a malformed header there
        // is found again, with its error, when the walk gets to it)
        W.ahead_tar = tar;
        W.ahead_n = n;
        W.ahead_xform = c->gpu_xform;
        W.ahead.start = W.w.next;
        W.ahead.at_end = false;
        const int threads = c->threads;
        W.bg = std::thread([&W, ectx, tar, n, window, threads] {
          pthread_setname_np(pthread_self(), "tsg-walk-bg");
          W.ahead_ok = IndexEntries(&ectx, tar, n, W.ahead.start, window, ~uint64_t(0) >> 1, threads, W.ahead.spec,
                                    W.ahead.fallback, &W.ahead.ents, &W.ahead.next, &W.ahead.at_end) == 0;
        });
      }
    }
    double t1 = dbg ? now() : 0;
    double t2 = dbg ? now() : 0;
    const size_t kBlock = 64;
    // 2. accept in order: whole blocks of entries that fit the batch in bulk
    // (per-block sums, then the blocks' rows written in parallel), the block
    // where the batch fills entry by entry
    const size_t k0 = W.pos;
    size_t k = k0 + AcceptBlocks(c, tar, W.w.ents, k0, st);
    bool full = false;
    for (; k < W.w.ents.size(); k++) {
      TarEntry& e = *W.w.ents[k];
      if (e.bad) {
        tsg::SetError("tar: invalid header checksum at offset " + std::to_string(e.hdr));
        W.tar = nullptr;
        W.Join();  // a walk that fails ends here: the background index must not outlive it
        return -1;
      }
      if (e.state == 2) {
        if (c->files() > 0 && c->acct() + e.out_len > c->limit) {
          full = true;
          break;
        }
        if (c->used + e.out_len + 64 > c->cap && !c->Reserve(e.out_len + 64)) {  // a lone large file
          W.Join();
          return -1;
        }
        e.out_off = c->used;
        if (c->gpu_xform) {
          c->used += e.size;
          c->bound += e.out_len;
          c->kinds.push_back(e.bin ? 2 : 1);
        } else {
          c->used += e.out_len;
        }
        c->offs.push_back(c->used);
        if (c->gather) c->gsrc.push_back(e.data);
        c->path_pool.push_back('/');  // Dir "" (image files, secret.go:130-135)
        const std::string_view fp = e.path(tar);
      c->path_pool.append(fp.data(), fp.size());
        c->path_off.push_back(c->path_pool.size());
        c->binary.push_back(e.bin);
        c->input_bytes += e.size;
        st->added++;
        st->input_bytes += e.size;
      }
      st->entries++;
      st->whiteouts += e.what == 1;
      st->opaque_dirs += e.what == 2;
      st->regular += e.what == 3;
      st->required += e.state != 0;
      st->skipped_binary += e.state == 1;
    }
    W.pos = k;
    double t3 = dbg ? now() : 0;
    // 3. copy / transform the accepted contents (gather mode: nothing to copy,
    // the GPU reads them in the layer buffer)
    if (!c->gather) tsg::ParallelFor((k - k0 + kBlock - 1) / kBlock, c->threads, [&](size_t b) {
      for (size_t i = k0 + b * kBlock; i < std::min(k, k0 + (b + 1) * kBlock); i++) {
        const TarEntry& e = *W.w.ents[i];
        if (e.state != 2) continue;
        uint8_t* dst = c->arena + e.out_off;
        if (c->gpu_xform) tsg::CopyToArena(dst, tar + e.data, e.size);
        else if (e.bin) tsg::ExtractPrintable(tar + e.data, e.size, dst);
        else tsg::StripCR(tar + e.data, e.size, dst);
      }
      _mm_sfence();
    }, true);
    if (!c->gather) std::memset(c->arena + c->used, 0, 64);  // the engine reads up to 64 B past the end
    if (dbg) {
      const double t4 = now();
      t_phase[0] += t1 - t0;
      t_phase[1] += t2 - t1;
      t_phase[2] += t3 - t2;
      t_phase[3] += t4 - t3;
      std::fprintf(stderr, "walk phases (cumulative s): index+evaluate %.3f (classify %.3f) accept %.3f copy %.3f"
                   " | thread-s: classify %.3f required %.3f\n", t_phase[0], t_phase[1], t_phase[2], t_phase[3],
                   g_eval_ns[0] / 1e9, g_eval_ns[1] / 1e9);
    }
    if (full) {
      *cursor = W.w.ents[k]->start;
      return 1;
    }
    p = W.w.next;
    *cursor = p;
    if (W.w.at_end) return 0;
  }
}

int tsg_analyzer_walk_end(tsg_analyzer* a) {
  std::lock_guard<std::mutex> g(a->walk_mu);
  tsg::EndTarWalk(a->walk);
  return 0;
}

int tsg_analyzer_set_walk_ahead(tsg_analyzer* a, int on) {
  if (!a) {
    tsg::SetError("tsg_analyzer_set_walk_ahead: null analyzer");
    return -1;
  }
  std::lock_guard<std::mutex> g(a->walk_mu);
  if (!on) tsg::EndTarWalk(a->walk);  // no background index outlives the switch
  a->walk_ahead = on != 0;
  return 0;
}

uint32_t tsg_collector_files(const tsg_collector* c) { return c->files(); }
uint64_t tsg_collector_bytes(const tsg_collector* c) { return c->used; }
uint64_t tsg_collector_input_bytes(const tsg_collector* c) { return c->input_bytes; }

int tsg_collector_file(const tsg_collector* c, uint32_t i, const char** path, uint64_t* path_len,
                       const uint8_t** content, uint64_t* len, int* binary) {
  if (i >= c->files()) return -1;
  *path = c->path_pool.data() + c->path_off[i];
  *path_len = c->path_off[i + 1] - c->path_off[i];
  *content = c->gather ? c->gbase + c->gsrc[i] : c->arena + c->offs[i];
  *len = c->offs[i + 1] - c->offs[i];
  *binary = c->binary[i];
  if (c->gpu_xform) {  // as it will be scanned: transformed here (tests / host-language mirror only)
    const uint64_t n = *len;
    c->scratch.resize(size_t(n + n / 5 + 2));
    *len = c->kinds[i] == 2 ? tsg::ExtractPrintable(*content, n, c->scratch.data())
                            : tsg::StripCR(*content, n, c->scratch.data());
    *content = c->scratch.data();
  }
  return 0;
}

int tsg_collector_set_gather(tsg_collector* c, int on) {
  if (c->files() > 0) {
    tsg::SetError("tsg_collector_set_gather: the batch is not empty");
    return -1;
  }
  if (on && !c->gpu_xform) {
    tsg::SetError("tsg_collector_set_gather: gather mode needs the GPU pre-transform (tsg_collector_set_gpu_transform)");
    return -1;
  }
  c->gather = on != 0;
  return 0;
}

int tsg_collector_set_gpu_transform(tsg_collector* c, int on) {
  if (c->files() > 0) {
    tsg::SetError("tsg_collector_set_gpu_transform: the batch is not empty");
    return -1;
  }
  if (!on && c->gather) {
    tsg::SetError("tsg_collector_set_gpu_transform: gather mode needs the GPU pre-transform (tsg_collector_set_gather 0 first)");
    return -1;
  }
  c->gpu_xform = on != 0;
  return 0;
}

int tsg_collector_submit(tsg_collector* c, tsg_pending** out) {
  c->BuildPaths();
  tsg_batch_ext b{};
  b.struct_size = TSG_BATCH_EXT_SIZE;
  b.base.n_files = c->files();
  b.base.host_arena = c->arena;
  b.base.host_offsets = c->offs.data();
  b.base.paths = c->path_ptrs.data();
  b.base.path_lens = c->path_lens.data();
  b.base.binary = c->binary.data();
  b.base.transform = c->gpu_xform ? c->kinds.data() : nullptr;
  // the paths are packed already: the global allow-path rules are prefiltered on the GPU
  b.host_paths = reinterpret_cast<const uint8_t*>(c->path_pool.data());
  b.host_path_offsets = c->path_off.data();
  if (c->gather) {  // the GPU reads the files in the layer buffer
    b.base.host_arena = nullptr;
    b.gather_base = c->gbase;
    b.gather_src = c->gsrc.data();
  }
  return tsg_scan_submit_ext(const_cast<tsg_scanner*>(c->a->s), &b, out);
}

void tsg_collector_reset(tsg_collector* c) { c->Reset(); }

}  // extern "C"
