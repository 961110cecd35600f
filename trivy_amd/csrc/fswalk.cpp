// Filesystem walker feeding the batch collectors (include/tsg_analyzer.h
// tsg_fs_walk_*): FS.Walk (pkg/fanal/walker/fs.go:25-78) -- filepath.WalkDir
// order, SkipDirs / SkipFiles as doublestar patterns (utils.SkipPath,
// pkg/fanal/utils/utils.go:105-126; defaultSkipDirs walk.go:11-16), regular
// files only, permission errors ignored (fs.go:80-95) -- then AnalyzeFile's
// Required gate and Analyze up to Scan (analyzer/secret/secret.go:103-190),
// with the file contents read straight into the pinned batch arena.
//
// The tree is listed level by level on the host pool (each directory's
// entries sorted by name, as os.ReadDir returns them) and flattened into
// WalkDir's depth-first lexical order, so file ids and results are those of
// the sequential walk.  Reads go to the arena at the offsets the accept step
// assigned, on the pool threads.  A file larger than the batch gets a batch of
// its own (the collector grows its arena; the reference's cachedFile temp-file
// spill at 100 MiB, walker/cached_file.go:36-66, is a tar-walker detail the
// fs opener does not have: fs.go:106-111 opens the file directly).
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>
#include <atomic>
#include <cerrno>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

#include "collector.h"
#include "parallel.h"

namespace tsg {
void SetError(const std::string& e);
bool IsBinaryHead(const uint8_t* p, uint64_t size);
uint64_t ExtractPrintable(const uint8_t* in, uint64_t n, uint8_t* out);
uint64_t StripCR(const uint8_t* in, uint64_t n, uint8_t* out);
std::string GoExt(const std::string& p);
bool RequiredPath(const tsg_analyzer* a, const char* path, uint64_t len, int64_t size);

namespace {

// One UTF-8 rune of s at i (invalid byte: itself, width 1).
uint32_t RuneAt(std::string_view s, size_t i, size_t* w) {
  const uint8_t b = uint8_t(s[i]);
  auto cont = [&](size_t k) { return i + k < s.size() && (uint8_t(s[i + k]) & 0xC0) == 0x80; };
  if (b < 0x80) {
    *w = 1;
    return b;
  }
  if ((b & 0xE0) == 0xC0 && cont(1)) {
    *w = 2;
    return ((b & 0x1Fu) << 6) | (uint8_t(s[i + 1]) & 0x3Fu);
  }
  if ((b & 0xF0) == 0xE0 && cont(1) && cont(2)) {
    *w = 3;
    return ((b & 0x0Fu) << 12) | ((uint8_t(s[i + 1]) & 0x3Fu) << 6) | (uint8_t(s[i + 2]) & 0x3Fu);
  }
  if ((b & 0xF8) == 0xF0 && cont(1) && cont(2) && cont(3)) {
    *w = 4;
    return ((b & 0x07u) << 18) | ((uint8_t(s[i + 1]) & 0x3Fu) << 12) | ((uint8_t(s[i + 2]) & 0x3Fu) << 6) |
           (uint8_t(s[i + 3]) & 0x3Fu);
  }
  *w = 1;
  return b;
}

}  // namespace

// doublestar.Match (github.com/bmatcuk/doublestar/v4, the matcher behind
// utils.SkipPath): '*' any run of non-'/' characters, '?' one non-'/'
// character, '[...]' a class ('!' or '^' negates, a-z ranges, '\' escapes),
// '{a,b}' alternatives, '\' escapes, and '**' as a whole path component zero
// or more directories ("a/**" also matches "a").  Returns -1 for a malformed
// pattern (ErrBadPattern: SkipPath then stops and reports false).
int DoubleStarMatch(std::string_view p, std::string_view s) {
  size_t i = 0;
  while (i < p.size()) {
    const char c = p[i];
    const bool comp_start = i == 0 || p[i - 1] == '/';
    if (c == '*' && comp_start && i + 1 < p.size() && p[i + 1] == '*' && (i + 2 == p.size() || p[i + 2] == '/')) {
      if (i + 2 == p.size()) return 1;  // trailing "**": everything below
      const std::string_view rest = p.substr(i + 3);
      for (size_t k = 0;;) {  // zero or more leading components of s
        const int r = DoubleStarMatch(rest, s.substr(k));
        if (r != 0) return r;
        const size_t sl = s.find('/', k);
        if (sl == std::string_view::npos) return 0;
        k = sl + 1;
      }
    }
    if (c == '/' && s.empty() && p.substr(i) == "/**") return 1;  // "a/**" matches "a"
    if (c == '*') {  // a run of '*' that is not a whole "**" component is one '*'
      size_t j = i;
      while (j < p.size() && p[j] == '*') j++;
      const std::string_view rest = p.substr(j);
      for (;;) {
        const int r = DoubleStarMatch(rest, s);
        if (r != 0) return r;
        if (s.empty() || s[0] == '/') return 0;
        size_t w;
        RuneAt(s, 0, &w);
        s.remove_prefix(w);
      }
    }
    if (c == '{') {  // alternatives up to the matching '}' (nesting allowed)
      size_t depth = 0, j = i, start = i + 1;
      std::vector<std::string_view> alts;
      for (; j < p.size(); j++) {
        if (p[j] == '\\') {
          j++;
          continue;
        }
        if (p[j] == '{') {
          depth++;
        } else if (p[j] == '}' && --depth == 0) {
          break;
        } else if (p[j] == ',' && depth == 1) {
          alts.push_back(p.substr(start, j - start));
          start = j + 1;
        }
      }
      if (j >= p.size()) return -1;
      alts.push_back(p.substr(start, j - start));
      const std::string_view rest = p.substr(j + 1);
      int bad = 0;
      for (auto a : alts) {
        std::string q(p.substr(0, 0));
        q.append(a.data(), a.size());
        q.append(rest.data(), rest.size());
        const int r = DoubleStarMatch(q, s);
        if (r == 1) return 1;
        if (r < 0) bad = -1;
      }
      return bad;
    }
    if (s.empty()) {
      if (c == '[' && p.find(']', i + 1) == std::string_view::npos) return -1;
      if (c == '\\' && i + 1 >= p.size()) return -1;
      return 0;
    }
    size_t w;
    const uint32_t r = RuneAt(s, 0, &w);
    if (c == '?') {
      if (r == '/') return 0;
      i++;
      s.remove_prefix(w);
      continue;
    }
    if (c == '[') {
      size_t j = i + 1;
      bool neg = false;
      if (j < p.size() && (p[j] == '!' || p[j] == '^')) {
        neg = true;
        j++;
      }
      bool hit = false, first = true;
      for (;;) {
        if (j >= p.size()) return -1;
        if (p[j] == ']' && !first) break;
        first = false;
        size_t cw;
        uint32_t lo;
        if (p[j] == '\\') {
          if (j + 1 >= p.size()) return -1;
          lo = RuneAt(p, j + 1, &cw);
          j += 1 + cw;
        } else {
          lo = RuneAt(p, j, &cw);
          j += cw;
        }
        uint32_t hi = lo;
        if (j + 1 < p.size() && p[j] == '-' && p[j + 1] != ']') {
          size_t hw;
          if (p[j + 1] == '\\') {
            if (j + 2 >= p.size()) return -1;
            hi = RuneAt(p, j + 2, &hw);
            j += 2 + hw;
          } else {
            hi = RuneAt(p, j + 1, &hw);
            j += 1 + hw;
          }
        }
        if (lo <= r && r <= hi) hit = true;
      }
      if (r == '/' || hit == neg) return 0;
      i = j + 1;
      s.remove_prefix(w);
      continue;
    }
    uint32_t want;
    size_t pw;
    if (c == '\\') {
      if (i + 1 >= p.size()) return -1;
      want = RuneAt(p, i + 1, &pw);
      pw += 1;
    } else {
      want = RuneAt(p, i, &pw);
    }
    if (want != r) return 0;
    i += pw;
    s.remove_prefix(w);
  }
  return s.empty() ? 1 : 0;
}

// doublestar.ValidatePattern: brackets and braces closed, no trailing '\'.
bool DoubleStarValid(std::string_view p) {
  int brace = 0;
  for (size_t i = 0; i < p.size(); i++) {
    if (p[i] == '\\') {
      if (++i >= p.size()) return false;
    } else if (p[i] == '[') {
      size_t j = i + 1;
      if (j < p.size() && (p[j] == '!' || p[j] == '^')) j++;
      if (j < p.size() && p[j] == ']') j++;  // a leading ']' is a member
      while (j < p.size() && p[j] != ']') j += p[j] == '\\' ? 2 : 1;
      if (j >= p.size()) return false;
      i = j;
    } else if (p[i] == '{') {
      brace++;
    } else if (p[i] == '}' && brace > 0) {
      brace--;
    }
  }
  return brace == 0;
}

// doublestar.Match: on a mismatch the pattern is validated (ErrBadPattern -> -1).
int DoubleStarMatchChecked(std::string_view p, std::string_view s) {
  const int r = DoubleStarMatch(p, s);
  return r == 0 && !DoubleStarValid(p) ? -1 : r;
}

// utils.SkipPath (utils.go:112-126).
bool SkipPath(std::string_view path, const std::vector<std::string>& pats) {
  while (!path.empty() && path[0] == '/') path.remove_prefix(1);
  for (const auto& p : pats) {
    const int m = DoubleStarMatchChecked(p, path);
    if (m < 0) return false;  // a bad pattern ends the check
    if (m == 1) return true;
  }
  return false;
}

}  // namespace tsg

struct tsg_fs_walk {
  std::string root;
  std::vector<std::string> skip_dirs, skip_files;
  struct File {
    std::string rel;  // slash-separated path relative to the root (the FilePath)
    uint64_t size;
  };
  std::vector<File> files;  // every regular, unskipped file in WalkDir order
  size_t next = 0;
  bool listed = false;
  bool root_is_file = false;
  // a bare file name as the root: path.Split gives Dir "" and Analyze reports
  // "/" + name (artifact/local/fs.go:90-93, analyzer/secret/secret.go:130-135)
  bool slash_prefix = false;
  uint64_t dirs = 0, skipped_dirs = 0, nonregular = 0, skipped_files = 0, perm_errors = 0;
};

namespace {

struct DirNode {
  std::string rel;  // "." for the root
  struct Child {
    std::string name;
    int kind;  // 0 file, 1 dir, 2 other
    uint64_t size;
    int64_t node;  // dir: its DirNode index (-1 skipped)
  };
  std::vector<Child> kids;
  int err = 0;
};

std::string JoinRel(const std::string& dir_rel, const std::string& name) {
  return dir_rel == "." ? name : dir_rel + "/" + name;
}

// Lists the tree level by level (directories of one level in parallel) and
// flattens it in WalkDir order.
bool ListTree(tsg_fs_walk* w, int threads) {
  struct stat rs;
  if (lstat(w->root.c_str(), &rs) != 0) {
    tsg::SetError("walk dir error: lstat " + w->root + ": " + std::strerror(errno));
    return false;
  }
  if (!S_ISDIR(rs.st_mode)) {  // a file root: fs.go walks "." (artifact/local/fs.go:90-93 splits the path)
    if (S_ISREG(rs.st_mode) && !tsg::SkipPath(".", w->skip_files)) {
      const size_t sl = w->root.find_last_of('/');
      w->files.push_back({sl == std::string::npos ? w->root : w->root.substr(sl + 1), uint64_t(rs.st_size)});
      w->root_is_file = true;
      w->slash_prefix = sl == std::string::npos;
    }
    return true;
  }
  // WalkDir visits the root first with relPath ".": a SkipDirs pattern
  // matching "." skips the whole tree (walker/fs.go:51-55)
  if (tsg::SkipPath(".", w->skip_dirs)) {
    w->skipped_dirs++;
    return true;
  }
  std::vector<DirNode> nodes(1);
  nodes[0].rel = ".";
  std::vector<size_t> level{0};
  std::atomic<bool> fail{false};
  std::string fail_msg;
  std::mutex fail_mu;
  while (!level.empty()) {
    std::vector<std::vector<DirNode::Child>> got(level.size());
    tsg::ParallelFor(level.size(), threads, [&](size_t k) {
      DirNode& d = nodes[level[k]];
      const std::string abs = d.rel == "." ? w->root : w->root + "/" + d.rel;
      const int fd = open(abs.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
      if (fd < 0) {
        d.err = errno;
        return;
      }
      DIR* dp = fdopendir(fd);
      if (!dp) {
        d.err = errno;
        close(fd);
        return;
      }
      std::vector<DirNode::Child>& out = got[k];
      while (struct dirent* e = readdir(dp)) {
        const char* nm = e->d_name;
        if (nm[0] == '.' && (nm[1] == 0 || (nm[1] == '.' && nm[2] == 0))) continue;
        DirNode::Child ch{nm, 2, 0, -1};
        unsigned char t = e->d_type;
        struct stat st;
        bool have_st = false;
        if (t == DT_UNKNOWN || t == DT_REG) {  // regular files need their size (d.Info(), fs.go:69)
          if (fstatat(fd, nm, &st, AT_SYMLINK_NOFOLLOW) != 0) {
            if (errno == ENOENT) continue;  // removed meanwhile
            if (errno == EACCES || errno == EPERM) continue;
            std::lock_guard<std::mutex> g(fail_mu);
            fail_msg = "file info error: " + abs + "/" + nm + ": " + std::strerror(errno);
            fail = true;
            continue;
          }
          have_st = true;
          t = S_ISREG(st.st_mode) ? DT_REG : S_ISDIR(st.st_mode) ? DT_DIR : DT_LNK;
        }
        if (t == DT_DIR) ch.kind = 1;
        else if (t == DT_REG) {
          ch.kind = 0;
          ch.size = have_st ? uint64_t(st.st_size) : 0;
        }
        out.push_back(std::move(ch));
      }
      closedir(dp);
      // os.ReadDir: sorted by filename (byte order)
      std::sort(out.begin(), out.end(), [](const DirNode::Child& a, const DirNode::Child& b) { return a.name < b.name; });
    }, true);
    if (fail) {
      tsg::SetError(fail_msg);
      return false;
    }
    std::vector<size_t> nxt;
    for (size_t k = 0; k < level.size(); k++) {
      const size_t di = level[k];
      const int err = nodes[di].err;
      if (err) {
        if (err == EACCES || err == EPERM) {  // onError: permission errors are ignored (fs.go:86-88)
          w->perm_errors++;
          continue;
        }
        tsg::SetError("walk dir error: " + w->root + "/" + nodes[di].rel + ": " + std::strerror(err));
        return false;
      }
      for (auto& ch : got[k]) {
        if (ch.kind == 1) {
          const std::string rel = JoinRel(nodes[di].rel, ch.name);
          if (tsg::SkipPath(rel, w->skip_dirs)) {  // filepath.SkipDir
            w->skipped_dirs++;
          } else {
            ch.node = int64_t(nodes.size());
            nodes.push_back(DirNode{rel, {}, 0});
            nxt.push_back(size_t(ch.node));
            w->dirs++;
          }
        }
      }
      nodes[di].kids = std::move(got[k]);
    }
    level.swap(nxt);
  }
  // WalkDir order: a directory's entries in name order, each subdirectory walked where it sorts
  std::vector<std::pair<size_t, size_t>> stack{{0, 0}};
  while (!stack.empty()) {
    auto& top = stack.back();
    DirNode& d = nodes[top.first];
    if (top.second >= d.kids.size()) {
      stack.pop_back();
      continue;
    }
    const DirNode::Child& ch = d.kids[top.second++];
    if (ch.kind == 1) {
      if (ch.node >= 0) stack.push_back({size_t(ch.node), 0});
      continue;
    }
    if (ch.kind != 0) {  // !d.Type().IsRegular()
      w->nonregular++;
      continue;
    }
    std::string rel = JoinRel(d.rel, ch.name);
    if (tsg::SkipPath(rel, w->skip_files)) {
      w->skipped_files++;
      continue;
    }
    w->files.push_back({std::move(rel), ch.size});
  }
  return true;
}

// Reads up to n bytes of path into dst; returns the bytes read or -1.
int64_t ReadInto(const std::string& path, uint8_t* dst, uint64_t n) {
  const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  uint64_t got = 0;
  while (got < n) {
    const ssize_t r = pread(fd, dst + got, size_t(n - got), off_t(got));
    if (r < 0) {
      if (errno == EINTR) continue;
      close(fd);
      return -1;
    }
    if (r == 0) break;
    got += uint64_t(r);
  }
  close(fd);
  return int64_t(got);
}

}  // namespace

extern "C" {

int tsg_fs_walk_new(const char* root, const char* const* skip_dirs, uint32_t n_skip_dirs,
                    const char* const* skip_files, uint32_t n_skip_files, tsg_fs_walk** out) {
  auto w = new tsg_fs_walk();
  w->root = root ? root : ".";
  while (w->root.size() > 1 && w->root.back() == '/') w->root.pop_back();
  for (uint32_t i = 0; i < n_skip_dirs; i++) w->skip_dirs.push_back(skip_dirs[i]);
  for (const char* d : {"**/.git", "proc", "sys", "dev"}) w->skip_dirs.push_back(d);  // defaultSkipDirs
  for (uint32_t i = 0; i < n_skip_files; i++) w->skip_files.push_back(skip_files[i]);
  *out = w;
  return 0;
}

void tsg_fs_walk_free(tsg_fs_walk* w) { delete w; }

int tsg_doublestar_match(const char* pattern, const char* path) { return tsg::DoubleStarMatchChecked(pattern, path); }

int tsg_fs_walk_stats(const tsg_fs_walk* w, tsg_fs_stats* st) {
  st->files = w->files.size();
  st->dirs = w->dirs;
  st->skipped_dirs = w->skipped_dirs;
  st->skipped_files = w->skipped_files;
  st->nonregular = w->nonregular;
  st->perm_errors = w->perm_errors;
  return 0;
}

int tsg_collector_add_fs(tsg_collector* c, tsg_fs_walk* w, tsg_fs_add_stats* st) {
  if (c->gather) {
    tsg::SetError("tsg_collector_add_fs: the collector gathers from tar layers (tsg_collector_set_gather)");
    return -1;
  }
  tsg_fs_add_stats local{};
  if (!st) st = &local;
  if (!w->listed) {
    if (!ListTree(w, c->threads)) return -1;
    w->listed = true;
  }
  const std::string base = w->root_is_file ? std::string() : w->root + "/";
  // per file of a window: Required, the 300-byte head (IsBinary), the arena
  // size it needs; then accept in order, then read the accepted ones.  A small
  // required file is read whole by the first pass (into the window's scratch):
  // one open / read / close instead of two, the second pass copies it
  struct Cand {
    int state;  // 0 not required, 1 binary skipped, 2 added, 3 vanished
    bool bin;
    uint64_t size, out_len, out_off;
    uint64_t scr_off;  // small files: offset in the scratch (kNoScratch: read in the second pass)
    int64_t scr_len;   // bytes read into the scratch
  };
  // (the scratch holds at most a window's small files: <= 1.5x the batch size)
  constexpr uint64_t kSmall = 64 << 10, kNoScratch = ~uint64_t(0);
  for (;;) {
    if (w->next >= w->files.size()) return 0;
    const uint64_t room = c->limit > c->acct() ? c->limit - c->acct() : 0;
    // a window of the next files worth ~1.5x the room (at least one)
    size_t hi = w->next;
    uint64_t want = 0;
    while (hi < w->files.size() && (hi == w->next || want < room + room / 2)) want += w->files[hi++].size;
    const size_t lo = w->next, n = hi - lo;
    std::vector<Cand> cd(n);
    std::vector<uint8_t> req(n);
    tsg::ParallelFor((n + 255) / 256, c->threads, [&](size_t b) {
      for (size_t i = b * 256; i < std::min(n, b * 256 + 256); i++) {
        const auto& f = w->files[lo + i];
        req[i] = tsg::RequiredPath(c->a, f.rel.data(), f.rel.size(), int64_t(f.size)) ? 1 : 0;
      }
    }, true);
    uint64_t scr_total = 0;
    for (size_t i = 0; i < n; i++) {
      const uint64_t sz = w->files[lo + i].size;
      cd[i] = Cand{0, false, sz, 0, 0, kNoScratch, 0};
      if (req[i] && sz <= kSmall) {
        cd[i].scr_off = scr_total;
        scr_total += sz;
      }
    }
    if (c->fs_scratch.size() < scr_total) c->fs_scratch.resize(scr_total + scr_total / 4);
    uint8_t* scr = c->fs_scratch.data();
    tsg::ParallelFor((n + 31) / 32, c->threads, [&](size_t b) {
      for (size_t i = b * 32; i < std::min(n, b * 32 + 32); i++) {
        const auto& f = w->files[lo + i];
        Cand& x = cd[i];
        if (!req[i]) continue;
        uint8_t head_buf[300];
        const uint8_t* head = head_buf;
        int64_t h;
        if (x.scr_off != kNoScratch) {  // small: the whole file now
          x.scr_len = ReadInto(w->root_is_file ? w->root : base + f.rel, scr + x.scr_off, f.size);
          h = x.scr_len < 0 ? -1 : std::min<int64_t>(300, x.scr_len);
          head = scr + x.scr_off;
        } else {
          h = ReadInto(w->root_is_file ? w->root : base + f.rel, head_buf, std::min<uint64_t>(300, f.size));
        }
        if (h < 0) {
          x.state = 3;
          continue;
        }
        x.bin = tsg::IsBinaryHead(head, uint64_t(h));
        if (x.bin && tsg::GoExt(f.rel) != ".pyc") {
          x.state = 1;
          continue;
        }
        x.state = 2;
        x.out_len = x.bin ? f.size + f.size / 5 + 1 : f.size;  // the largest transformed size
      }
    }, true);
    size_t k = 0;
    bool full = false;
    std::vector<size_t> added;
    for (; k < n; k++) {
      Cand& x = cd[k];
      const auto& f = w->files[lo + k];
      if (x.state == 2) {
        const uint64_t acct_need = c->gpu_xform ? x.out_len : x.size;
        if (c->files() > 0 && c->acct() + acct_need > c->limit) {
          full = true;
          break;
        }
        const uint64_t need = c->gpu_xform ? x.size : x.out_len;  // arena bytes (host mode: transformed in place)
        if (c->used + need + 64 > c->cap) {
          if (c->files() > 0) {
            full = true;
            break;
          }
          if (!c->Reserve(need + 64)) return -1;  // a lone file larger than the batch
        }
        x.out_off = c->used;
        c->used += need;  // final length fixed after the read (host mode)
        added.push_back(k);
        c->offs.push_back(c->used);
        if (w->slash_prefix) c->path_pool.push_back('/');
        c->path_pool.append(f.rel);  // Dir = root: FilePath as walked (secret.go:130-135 adds no '/')
        c->path_off.push_back(c->path_pool.size());
        c->binary.push_back(x.bin);
        if (c->gpu_xform) {
          c->bound += x.out_len;
          c->kinds.push_back(x.bin ? 2 : 1);
        }
      }
      st->walked++;
      st->required += x.state >= 2 || x.state == 1;
      st->skipped_binary += x.state == 1;
    }
    // read the accepted files into the arena (host mode: transformed in place)
    std::vector<int64_t> final_len(added.size());
    std::atomic<int> read_err{0};
    tsg::ParallelFor(added.size(), c->threads, [&](size_t j) {
      const Cand& x = cd[added[j]];
      const auto& f = w->files[lo + added[j]];
      uint8_t* dst = c->arena + x.out_off;
      int64_t r;
      if (x.scr_off != kNoScratch) {  // read whole by the first pass
        r = x.scr_len;
        std::memcpy(dst, scr + x.scr_off, size_t(r));
      } else {
        r = ReadInto(w->root_is_file ? w->root : base + f.rel, dst, x.size);
      }
      if (r < 0) {
        read_err = errno ? errno : EIO;
        final_len[j] = 0;
        return;
      }
      if (c->gpu_xform) {
        final_len[j] = r;
      } else if (x.bin) {
        // ExtractPrintable writes at most the input length: in place
        final_len[j] = int64_t(tsg::ExtractPrintable(dst, uint64_t(r), dst));
      } else {
        final_len[j] = int64_t(tsg::StripCR(dst, uint64_t(r), dst));
      }
    }, true);
    if (read_err && read_err != EACCES && read_err != ENOENT) {
      tsg::SetError(std::string("fs walk: read error: ") + std::strerror(read_err));
      return -1;
    }
    // offsets: the files were placed at their largest length; compact to the
    // lengths read / transformed (a file that shrank since the listing, or
    // host-mode transforms) with memmove in order
    if (!added.empty()) {
      const uint32_t f0 = c->files() - uint32_t(added.size());
      uint64_t at = c->offs[f0];
      for (size_t j = 0; j < added.size(); j++) {
        const Cand& x = cd[added[j]];
        if (at != x.out_off) std::memmove(c->arena + at, c->arena + x.out_off, size_t(final_len[j]));
        at += uint64_t(final_len[j]);
        c->offs[f0 + 1 + j] = at;
        c->input_bytes += x.size;
        st->added++;
        st->input_bytes += x.size;
      }
      c->used = at;
      std::memset(c->arena + c->used, 0, 64);  // the engine reads up to 64 B past the end
    }
    w->next = lo + k;
    if (full) return 1;
  }
}

}  // extern "C"
