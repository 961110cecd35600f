/* libtsg.so -- MI355X secret-scanning engine, C ABI (cgo / ctypes bindable).
 *
 * Drop-in boundary for pkg/fanal/secret (undistro/trivy @ 2024-12-20).  The
 * host language keeps ParseConfig / NewScanner's rule-set assembly
 * (pkg/fanal/secret/scanner.go:277-364) and hands the resulting *Global* to
 * tsg_scanner_new; Scan(ScanArgs) (scanner.go:377-463) becomes a batched
 * tsg_scan over a contiguous arena of CR-stripped file contents
 * (pkg/fanal/analyzer/secret/secret.go:117-141 does the stripping).
 *
 * Entry point                 replaces (reference)
 *   tsg_scanner_new           secret.NewScanner(config)            scanner.go:320-364
 *   tsg_scanner_allow_path    (Global).AllowPath(path)             scanner.go:57-59
 *   tsg_scan                  (*Scanner).Scan(ScanArgs), per file  scanner.go:377-463
 *   tsg_result_*              types.Secret / SecretFinding / Code  pkg/fanal/types/secret.go:5-20,
 *                                                                 misconf.go:48-61
 * Conventions: all pointers are borrowed for the duration of the call;
 * results are owned by the library until tsg_result_free.  Status: 0 = OK,
 * <0 = error, text via tsg_last_error() (tsg_debug.h).  Thread-safety: scans on
 * one scanner may overlap (tsg_scan_submit); their GPU phases are serialized
 * on the scanner's HIP stream, the exact host passes run concurrently.
 */
#ifndef TSG_SCANNER_H
#define TSG_SCANNER_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct tsg_allow_rule {  /* AllowRule, scanner.go:196-201 */
  const char* id;
  const char* regex;             /* NULL = none; "" = matches everything (Go compiles "") */
  const char* path;              /* NULL = none; "" = matches everything */
} tsg_allow_rule;

typedef struct tsg_rule {        /* Rule, scanner.go:89-100 */
  const char* id;
  const char* category;
  const char* title;
  const char* severity;          /* already normalised by ParseConfig */
  const char* regex;             /* NULL = rule without regex (never matches); "" = empty regex */
  const char* path;              /* NULL = any path; "" = empty regex (matches every path) */
  const char* secret_group_name; /* "" = whole match */
  const char* const* keywords;
  uint32_t n_keywords;
  const tsg_allow_rule* allow_rules;
  uint32_t n_allow_rules;
  const char* const* exclude_regexes; /* ExcludeBlock.Regexes */
  uint32_t n_exclude_regexes;
} tsg_rule;

typedef struct tsg_global {      /* Global, scanner.go:45-49 (the assembled rule set) */
  const tsg_rule* rules;
  uint32_t n_rules;
  const tsg_allow_rule* allow_rules;
  uint32_t n_allow_rules;
  const char* const* exclude_regexes;
  uint32_t n_exclude_regexes;
} tsg_global;

typedef struct tsg_scanner tsg_scanner;
typedef struct tsg_result tsg_result;

/* Compile the rule set (keyword/anchor automaton + relaxed NFAs) and bind a HIP device. */
int tsg_scanner_new(const tsg_global* g, int device, tsg_scanner** out);

/* Compiler options (versioned like tsg_batch_ext: struct_size first, unknown
 * sizes refused).  v1: calib / calib_bytes, an optional sample of the bytes
 * the scanner will see (e.g. the first batch of a scan job): a rule with both
 * a literal and a class-run anchor then takes the one that fires less on it
 * (trivy_amd/csrc/rules.h CompileOptions).  Findings never depend on it --
 * only which prefilter item finds the candidates. */
typedef struct tsg_compile_options {
  uint32_t struct_size;
  uint32_t reserved;
  const uint8_t* calib;
  uint64_t calib_bytes;
} tsg_compile_options;
#define TSG_COMPILE_OPTIONS_SIZE_V1 ((uint32_t)(offsetof(tsg_compile_options, calib_bytes) + sizeof(uint64_t)))
int tsg_scanner_new_ex(const tsg_global* g, int device, const tsg_compile_options* opt, tsg_scanner** out);
void tsg_scanner_free(tsg_scanner* s);
/* 1 if path is globally allowed (Global.AllowPath), else 0. */
int tsg_scanner_allow_path(const tsg_scanner* s, const char* path, uint64_t len);

typedef struct tsg_batch {
  uint32_t n_files;
  const uint8_t* host_arena;     /* concatenated contents, required (exact pass) */
  const uint64_t* host_offsets;  /* n_files + 1 */
  const void* dev_arena;         /* optional: same bytes already in HBM (16-B aligned, 64 readable
                                    bytes past the end) */
  const void* dev_offsets;       /* optional: device copy of host_offsets */
  const char* const* paths;      /* ScanArgs.FilePath per file */
  const uint64_t* path_lens;     /* optional */
  const uint8_t* binary;         /* optional ScanArgs.Binary per file */
  /* optional, per file: the analyzer's pre-scan transform, run on the GPU
   * (then host_arena / host_offsets hold the bytes as read, and dev_arena
   * must be NULL): 0 as is, 1 every '\r' removed (secret.go:121), 2
   * utils.ExtractPrintableBytes (.pyc, secret.go:112-117, utils.go:128-160) */
  const uint8_t* transform;
  /* optional: the FilePath bytes packed in HBM (dev_path_offsets: n_files + 1
   * u64, device) -- the global allow-path rules (scanner.go:381-386) are then
   * prefiltered on the GPU and the host runs them only on the paths that hold
   * one of their literals (trivy_amd/csrc/pathfilter.h).  `paths` is still
   * required (the exact rule and the results use it). */
  const void* dev_paths;
  const void* dev_path_offsets;
} tsg_batch;  /* frozen: the layout of round 4; later fields go to tsg_batch_ext */

/* Versioned batch.  struct_size is sizeof(tsg_batch_ext) as the caller was
 * built: the library reads only the fields that size covers, and refuses a
 * size it does not know (status <0, tsg_last_error names the sizes it knows),
 * so a caller built against an older or newer header never has fields read
 * past the end of its struct.  Known sizes: TSG_BATCH_EXT_SIZE_V1 (112 on
 * the 64-bit ABI), TSG_BATCH_EXT_SIZE_V2 (128).  The plain tsg_batch entry points read the frozen fields
 * only (a caller built against the round-4 header passes exactly those). */
typedef struct tsg_batch_ext {
  uint32_t struct_size;
  tsg_batch base;
  /* v1: the FilePath bytes packed in host memory (host_path_offsets: n_files
   * + 1 u64 into host_paths), as the analyzer's collectors hold them; without
   * base.dev_paths the engine copies them to HBM for the same GPU allow-path
   * prefilter (NULL: the host runs the rules over every path). */
  const uint8_t* host_paths;
  const uint64_t* host_path_offsets;
  /* v2 (round 6): gather_base / gather_src, with base.transform set and
   * base.host_arena NULL -- file f's bytes as read are gather_base +
   * gather_src[f] .. + (host_offsets[f + 1] - host_offsets[f]) in page-locked,
   * device-mapped host memory (tsg_host_register_mapped; a tar layer as the
   * analyzer's collectors hold it): the GPU gathers them itself, no host copy.
   * host_offsets still lay out the batch (the files back to back).  The GPU
   * reads aligned 16-B blocks: the 16 bytes before each file's data and the 32
   * after its end must lie in the mapped region too (a tar's 512-B headers and
   * padding provide them). */
  const uint8_t* gather_base;
  const uint64_t* gather_src;
} tsg_batch_ext;
#define TSG_BATCH_EXT_SIZE_V1 ((uint32_t)(offsetof(tsg_batch_ext, host_path_offsets) + sizeof(const uint64_t*)))
#define TSG_BATCH_EXT_SIZE_V2 ((uint32_t)(offsetof(tsg_batch_ext, gather_src) + sizeof(const uint64_t*)))
#define TSG_BATCH_EXT_SIZE TSG_BATCH_EXT_SIZE_V2  /* what this header's callers set */

int tsg_scan(tsg_scanner* s, const tsg_batch* batch, tsg_result** out);
int tsg_scan_ext(tsg_scanner* s, const tsg_batch_ext* batch, tsg_result** out);
/* Pipelined scanning: tsg_scan on a background thread.  The GPU phases of
 * the scans in flight on one scanner run one after another (one HIP stream);
 * a batch's exact host pass overlaps the next batch's kernels.  The batch's
 * buffers stay borrowed until tsg_scan_wait returns. */
typedef struct tsg_pending tsg_pending;
int tsg_scan_submit(tsg_scanner* s, const tsg_batch* batch, tsg_pending** out);
int tsg_scan_submit_ext(tsg_scanner* s, const tsg_batch_ext* batch, tsg_pending** out);
int tsg_scan_wait(tsg_pending* p, tsg_result** out); /* frees p */
void tsg_result_free(tsg_result* r);

/* kind: 0 = types.Secret{} (no findings), 1 = Secret{FilePath} (allowed path), 2 = findings */
int tsg_result_file(const tsg_result* r, uint32_t file, uint32_t* kind, uint32_t* n_findings);

typedef struct tsg_finding {
  uint32_t rule_index;           /* into tsg_global.rules */
  int64_t start_line, end_line;
  const char* match;
  uint64_t match_len;
  uint32_t n_lines;
} tsg_finding;
int tsg_result_finding(const tsg_result* r, uint32_t file, uint32_t k, tsg_finding* out);

typedef struct tsg_line {
  int64_t number;
  const char* content;
  uint64_t content_len;
  uint8_t is_cause, first_cause, last_cause;
} tsg_line;
int tsg_result_line(const tsg_result* r, uint32_t file, uint32_t k, uint32_t line, tsg_line* out);

/* Compact record of every finding, in file then finding order: the unit a
 * multi-process (one rank per GPU) job gathers to its merging rank, where
 * the findings are put in AnalysisResult.Sort order (pkg/fanal/analyzer/
 * analyzer.go:225-234) by the file paths the caller holds.  digest is a
 * 64-bit FNV-1a over the finding's Match and its Code lines (number, flags,
 * content), so the merged set can be compared without the text.  Returns the
 * record count; writes up to cap of them. */
typedef struct tsg_record {
  uint32_t file, rule_index;
  int64_t start_line, end_line;
  uint64_t digest;
} tsg_record;
uint64_t tsg_result_records(const tsg_result* r, tsg_record* out, uint64_t cap);

/* Whole batch as JSON ([{"kind":..,"findings":[..]}...], Go field names). */
int tsg_result_json(const tsg_result* r, const char** json, uint64_t* len);
/* Files [lo, hi) only (same format; the text stays valid until the next range call on r; the
   whole-result text of tsg_result_json is kept apart). */
int tsg_result_json_range(const tsg_result* r, uint32_t lo, uint32_t hi, const char** json, uint64_t* len);

/* Timings / counters of the batch (GPU ms from HIP events on the engine stream). */
typedef struct tsg_stats {
  uint64_t bytes, files, anchor_hits, candidates, special_files, findings;
  double ms_scan_kernel, ms_verify_kernel, ms_fullscan_kernel, ms_gpu_total;
  double ms_host_gpu_phase, ms_host_allow_path, ms_host_exact, ms_host_total;
  uint64_t flagged_blocks;   /* 16-B blocks the streaming filter sent to its exact confirm step */
  double ms_careful_kernel;  /* fold-rune files' careful pass (part of ms_gpu_total) */
  /* per-kernel split of ms_gpu_total (HIP events on the engine stream) */
  uint64_t follow_hits;      /* anchor_hits (exact anchor-item matches) past the follow requirements */
  double ms_chunkmap_kernel, ms_confirm_kernel, ms_nfa_kernel, ms_finalize_kernel;
  /* host-resident batches: copies + kernels from the first H2D to the last chunk (chunks streamed) */
  double ms_h2d_span;
  uint64_t h2d_chunks;
  uint64_t fullscan_pairs;   /* (file, unanchored rule) pairs with an open keyword gate, NFA-scanned */
  uint64_t fold_sites;       /* U+212A / U+017F / U+0130 occurrences the fold kernel examined */
  double ms_xform_kernel;    /* GPU pre-transform (batch.transform; part of ms_gpu_total) */
} tsg_stats;
int tsg_result_stats(const tsg_result* r, tsg_stats* out);

/* Page-lock a caller's host buffer (hipHostRegister) so batches in it stream
 * to the GPU asynchronously (the engine's staging ring: copies of this and of
 * the next submitted batches overlap the kernels): the Go caller's pinned arena
 * pool.  Unregister before freeing it. */
int tsg_host_register(void* p, uint64_t bytes);
/* The same, also mapped into the device's address space, so kernels read it
 * directly (tsg_batch_ext.gather_base: a tar layer the GPU gathers from). */
int tsg_host_register_mapped(void* p, uint64_t bytes);
int tsg_host_unregister(void* p);

/* Compiled-table facts (for reports/tests). */
typedef struct tsg_table_info {
  uint32_t n_rules, n_keywords, n_anchors, n_filter_items, n_filter_buckets, filter_window;
  uint32_t n_fullscan_rules, nfa_words_total;
  uint64_t filter_table_bytes;  /* reach + item + class + core tables */
  double filter_est_fp;         /* estimated bucket fires per input byte (static byte prior) */
} tsg_table_info;
int tsg_scanner_table_info(const tsg_scanner* s, tsg_table_info* out);
/* Anchor description of rule i ("[lo,hi] lit lit..." or "-"). */
const char* tsg_scanner_rule_anchor(const tsg_scanner* s, uint32_t i);

#ifdef __cplusplus
}
#endif
#endif
