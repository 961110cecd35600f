/* libtsg.so -- the secret analyzer's ingest side, C ABI (cgo / ctypes bindable).
 *
 * Replaces the per-file half of pkg/fanal/analyzer/secret (undistro/trivy @
 * 2024-12-20) that runs before Scanner.Scan, and the analyzer group's
 * goroutine-per-file fan-out for this analyzer, with a batch collector that
 * packs transformed contents straight into one (pinned) arena for tsg_scan:
 *
 * Entry point                  replaces (reference)
 *   tsg_is_binary              utils.IsBinary                      pkg/fanal/utils/utils.go:85-103
 *   tsg_extract_printable      utils.ExtractPrintableBytes         pkg/fanal/utils/utils.go:128-160
 *   tsg_strip_cr               bytes.ReplaceAll(content, "\r", "") pkg/fanal/analyzer/secret/secret.go:121
 *   tsg_analyzer_new           NewSecretAnalyzer + Init            secret.go:79-101
 *   tsg_analyzer_required      (*SecretAnalyzer).Required          secret.go:152-190
 *   tsg_collector_add          (*SecretAnalyzer).Analyze up to the secret.go:103-136
 *                              Scan call (binary gate, transform,
 *                              "/" prefix for image files)
 *   tsg_collector_submit       the Scan calls of a batch           secret.go:137-141 -> scanner.go:377
 *   tsg_collector_add_tar      LayerTar.Walk + AnalyzeFile's       pkg/fanal/walker/tar.go:35-103,
 *                              Required gate for this analyzer     pkg/fanal/analyzer/analyzer.go:403-455
 *
 * Results: tsg_scan_wait gives a tsg_result whose file i is the collector's
 * i-th added file; Analyze returns nil unless that file's kind is 2 (findings),
 * secret.go:143-149.  Conventions as in tsg_scanner.h (0 = OK, <0 = error,
 * text via tsg_last_error()).
 */
#ifndef TSG_ANALYZER_H
#define TSG_ANALYZER_H
#include <stdint.h>

#include "tsg_scanner.h"
#ifdef __cplusplus
extern "C" {
#endif

/* utils.IsBinary over the first min(size, 300) bytes of content: 1 = binary. */
int tsg_is_binary(const uint8_t* content, uint64_t size);
/* utils.ExtractPrintableBytes: runs of unicode.IsPrint bytes longer than 4, each
 * followed by '\n'.  out must hold n + n / 5 + 1 bytes; returns the length. */
uint64_t tsg_extract_printable(const uint8_t* in, uint64_t n, uint8_t* out);
/* every '\r' removed; out must hold n bytes (may equal in); returns the length. */
uint64_t tsg_strip_cr(const uint8_t* in, uint64_t n, uint8_t* out);

typedef struct tsg_analyzer tsg_analyzer;
/* The scanner is borrowed for the analyzer's lifetime; config_path is the
 * SecretScannerOption.ConfigPath given to Init ("" = builtin rules). */
int tsg_analyzer_new(const tsg_scanner* s, const char* config_path, tsg_analyzer** out);
void tsg_analyzer_free(tsg_analyzer* a);
/* Required(filePath, fi) with fi.Size() = size: 1 = analyze, 0 = skip. */
int tsg_analyzer_required(const tsg_analyzer* a, const char* path, uint64_t path_len, int64_t size);

typedef struct tsg_collector tsg_collector;
/* A batch of at most arena_bytes transformed bytes (a single larger file is
 * accepted alone); the arena is pinned host memory when the scanner has a GPU. */
int tsg_collector_new(tsg_analyzer* a, uint64_t arena_bytes, tsg_collector** out);
void tsg_collector_free(tsg_collector* c);

#define TSG_SKIPPED (-1) /* binary and not .pyc: Analyze returns nil without scanning */
#define TSG_FULL (-2)    /* the batch is full: submit (or reset) and add again */
/* Analyze's pre-scan half for one file (dir = AnalysisInput.Dir; "" means a
 * file extracted from an image, whose path gets the "/" prefix).  Returns the
 * file's index in the batch (>= 0), TSG_SKIPPED or TSG_FULL; -3 (error set)
 * when the arena cannot grow or the collector gathers (tsg_collector_set_gather). */
int64_t tsg_collector_add(tsg_collector* c, const char* path, uint64_t path_len, const char* dir,
                          const uint8_t* content, uint64_t size);

typedef struct tsg_tar_stats {
  uint64_t entries, regular, required, added, skipped_binary, whiteouts, opaque_dirs, input_bytes;
} tsg_tar_stats;
/* Walk an uncompressed tar layer held in memory from *cursor (a header
 * offset; 0 to start): every regular file that Required accepts is added as
 * an image file (Dir "").  Returns 0 at the end of the archive, 1 when the
 * batch filled up (*cursor = the entry to resume from), <0 on a malformed
 * archive.  Whiteout (.wh.) and opaque-dir entries are counted, not added. */
int tsg_collector_add_tar(tsg_collector* c, const uint8_t* tar, uint64_t n, uint64_t* cursor, tsg_tar_stats* st);
/* Walk-ahead (opt-in, off by default): with tsg_analyzer_set_walk_ahead(a, 1)
 * the analyzer indexes the next window of entries on a background thread after
 * tsg_collector_add_tar returns 1.  Buffer lifetime in that mode: `tar` must
 * stay valid and unchanged until the walk ends -- add_tar returned 0 (end of
 * the archive) or < 0 -- or until tsg_analyzer_walk_end / tsg_analyzer_free /
 * tsg_analyzer_set_walk_ahead(a, 0) returns (call one before freeing the
 * buffer of a walk abandoned midway).  With walk-ahead off, nothing reads
 * `tar` after add_tar returns.  tsg_analyzer_walk_end also drops the walk's
 * cached window, so a later buffer at the same address starts afresh. */
int tsg_analyzer_set_walk_ahead(tsg_analyzer* a, int on);
int tsg_analyzer_walk_end(tsg_analyzer* a);

/* GPU pre-transform mode (empty collector only): files go into the arena as
 * read, and the CR strip / printable extraction runs on the GPU at scan time
 * (tsg_batch.transform).  The batch limit then counts each file's largest
 * transformed size. */
int tsg_collector_set_gpu_transform(tsg_collector* c, int on);
/* Gather mode (round 6; GPU-transform collectors, tar walks only): the walk no
 * longer copies a file's bytes into the arena -- the batch records where the
 * layer holds them, and the GPU gathers them from the layer buffer itself
 * (tsg_batch_ext v2 gather_base / gather_src).  The layer buffer must be
 * page-locked and device-mapped (tsg_host_register_mapped) for the whole walk
 * and until the batch's tsg_scan_wait.  A batch holds one layer's files: a
 * tsg_collector_add_tar on another buffer returns 1 (full) while the batch is
 * not empty.  tsg_collector_add / _add_fs fail in this mode. */
int tsg_collector_set_gather(tsg_collector* c, int on);

/* FS.Walk (pkg/fanal/walker/fs.go:25-78) feeding a collector: the tree under
 * root in filepath.WalkDir order, skip_dirs / skip_files as utils.SkipPath
 * doublestar patterns relative to root (the caller applies BuildSkipPaths,
 * fs.go:102-155; defaultSkipDirs are added here), regular files only,
 * permission errors ignored; per file AnalyzeFile's Required and Analyze up
 * to Scan (binary gate, contents read into the batch arena; FilePath = the
 * path relative to root, Dir = root).  tsg_collector_add_fs returns 1 when the
 * collector is full (submit, reset, call again), 0 when the walk is done,
 * <0 on error (tsg_last_error). */
typedef struct tsg_fs_walk tsg_fs_walk;
typedef struct tsg_fs_stats {
  uint64_t files, dirs, skipped_dirs, skipped_files, nonregular, perm_errors;
} tsg_fs_stats;
typedef struct tsg_fs_add_stats {
  uint64_t walked, required, skipped_binary, added, input_bytes;
} tsg_fs_add_stats;
int tsg_fs_walk_new(const char* root, const char* const* skip_dirs, uint32_t n_skip_dirs,
                    const char* const* skip_files, uint32_t n_skip_files, tsg_fs_walk** out);
int tsg_collector_add_fs(tsg_collector* c, tsg_fs_walk* w, tsg_fs_add_stats* st);
int tsg_fs_walk_stats(const tsg_fs_walk* w, tsg_fs_stats* st);
void tsg_fs_walk_free(tsg_fs_walk* w);
/* utils.SkipPath's doublestar.Match: 1 match, 0 no match, -1 malformed pattern. */
int tsg_doublestar_match(const char* pattern, const char* path);
uint32_t tsg_collector_files(const tsg_collector* c);
uint64_t tsg_collector_bytes(const tsg_collector* c);       /* arena bytes (transformed; as read in GPU mode) */
uint64_t tsg_collector_input_bytes(const tsg_collector* c); /* bytes as read, added files only */
/* The ScanArgs of file i as they will be scanned (tests / host-language mirror). */
int tsg_collector_file(const tsg_collector* c, uint32_t i, const char** path, uint64_t* path_len,
                       const uint8_t** content, uint64_t* len, int* binary);
/* Scan the batch (tsg_scan_submit); the arena stays borrowed until tsg_scan_wait.
 * Reset the collector after the wait to reuse it. */
int tsg_collector_submit(tsg_collector* c, tsg_pending** out);
void tsg_collector_reset(tsg_collector* c);

#ifdef __cplusplus
}
#endif
#endif
