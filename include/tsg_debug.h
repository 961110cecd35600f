/* Host-logic inspection entry points of libtsg.so (no GPU needed).
 *
 * These expose the exact host pass's Go-regexp engine so the CPU test-suite can
 * check it against the oracle.  They replace nothing in the reference: they are
 * the C-ABI view of Go's regexp calls made by pkg/fanal/secret/scanner.go:112
 * (FindAllIndex), :130 (FindAllSubmatchIndex) and :171/:207/:216 (MatchString).
 * Status codes: 0 = OK, <0 = error (text via tsg_last_error()).
 */
#ifndef TSG_DEBUG_H
#define TSG_DEBUG_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* FindAll[Submatch]Index(text, -1).  windows: optional (lo,hi) inclusive pairs
 * restricting match starts (sorted); pass NULL/0 for an unrestricted search.
 * Writes up to out_cap int64 offsets; *out_len receives the full count and
 * *num_cap the number of capture groups. */
int tsg_regex_find_all(const char* pattern, const uint8_t* text, uint64_t n, int submatch,
                       const int64_t* windows, uint32_t n_windows, int64_t* out, uint64_t out_cap,
                       uint64_t* out_len, int32_t* num_cap);

/* Engine selection for the exact pass's FindAll (tests only; process-wide):
 * 0 auto (bit-state backtracker, Pike VM past its row budget), 1 Pike VM only,
 * 2 backtracker with an 8-position budget (exercises the fallback). */
void tsg_debug_regex_engine(int mode);
/* The GPU pre-transform (trivy_amd/csrc/xform.hip) on a host batch, on HIP
 * device `device`: out receives the transformed arena (up to out_cap bytes),
 * xoff the n_files + 1 transformed offsets.  kinds per file: 0 as is, 1 CR
 * strip (secret.go:121), 2 ExtractPrintableBytes (utils.go:128-160).  Tests
 * compare it with the oracle's transforms byte for byte. */
int tsg_debug_xform(int device, const uint8_t* raw, uint64_t n_bytes, const uint64_t* offsets, uint32_t n_files,
                    const uint8_t* kinds, uint8_t* out, uint64_t out_cap, uint64_t* xoff);
/* regexp.MatchString: 1 = match, 0 = no match, <0 = compile error. */
int tsg_regex_match(const char* pattern, const uint8_t* text, uint64_t n);

/* bytes.ToLower (Go semantics).  Writes up to out_cap bytes, returns the full length. */
int64_t tsg_go_bytes_to_lower(const uint8_t* s, uint64_t n, uint8_t* out, uint64_t out_cap);

/* ---- rule compiler inspection (tables the GPU kernels consume) ---- */
struct tsg_global;
typedef struct tsg_compiled tsg_compiled;
struct tsg_table_info;
typedef struct tsg_debug_rule_info {
  uint32_t nfa_words;     /* 0: relaxed NFA empty */
  uint32_t gate;          /* 0 always, 1 keyword bitset, 2 host-verified */
  uint32_t anchored;      /* 1 anchor-driven, 0 full-scan */
  uint32_t has_regex;
  const uint64_t* nfa;    /* O[W] L[W] F[W] B[256][W] */
  const uint32_t* kw_ids;
  uint32_t n_kw;
} tsg_debug_rule_info;
int tsg_debug_compile(const struct tsg_global* g, tsg_compiled** out);
/* The same with compiler options (tsg_scanner.h tsg_compile_options); out_calibrated (optional):
 * the anchors the calibration sample moved to a class run. */
struct tsg_compile_options;
int tsg_debug_compile_ex(const struct tsg_global* g, const struct tsg_compile_options* opt, tsg_compiled** out,
                         uint32_t* out_calibrated);
void tsg_debug_compiled_free(tsg_compiled* c);
int tsg_debug_compiled_info(const tsg_compiled* c, struct tsg_table_info* out);
int tsg_debug_rule(const tsg_compiled* c, uint32_t i, tsg_debug_rule_info* out);
int tsg_debug_anchor(const tsg_compiled* c, uint32_t j, uint32_t* rule, uint32_t* lit_len,
                     int32_t* off_lo, int32_t* off_hi);
const char* tsg_debug_keyword(const tsg_compiled* c, uint32_t k);
/* Anchor j's follow requirements (trivy_amd/csrc/rules.h FollowLut, 32 B), or NULL. */
const void* tsg_debug_anchor_req(const tsg_compiled* c, uint32_t j);
/* The streaming prefilter's tables (trivy_amd/csrc/filter.h): shape = {buckets, window, words},
 * reach[256 * words] (u32; bucket j in word j/4, slot s at bit 4s + j%4; the last bucket counts
 * newlines), bucket_off[buckets+1] -> bucket_items, items (16-B records), item_cls, classes
 * (8 u32 each). */
int tsg_debug_filter(const tsg_compiled* c, uint32_t* shape, const uint32_t** reach, const uint32_t** bucket_off,
                     const uint32_t** bucket_items, const void** items, uint32_t* n_items, const uint8_t** item_cls,
                     const uint32_t** classes, double* est_fp);
/* The anchor / fold ids of the prefilter items (items[k] owns ids[ids_off .. ids_off + n_ids)). */
int tsg_debug_filter_ids(const tsg_compiled* c, const uint32_t** ids, uint32_t* n);
/* Rule i's anchor summary: "[off_lo,off_hi] lit[*][+la] ..." or "-" (no anchor). */
const char* tsg_debug_rule_anchor(const tsg_compiled* c, uint32_t i);

/* The CPU-only test hooks (host tail with whole-file windows, host-only
 * scanners) and the CPU reference scan are NOT in libtsg.so: they live in the
 * oracle's library (oracle/native/tsg_oracle.h, oracle/build/libtsg_host.so). */

/* Host workers the process-wide pool would start now (TSG_POOL_THREADS unset):
 * the affinity mask, capped by the cgroup quota, shared by LOCAL_WORLD_SIZE
 * ranks (or TSG_POOL_SHARE processes), minus the per-process reserve. */
int tsg_debug_pool_budget(void);

/* A scanner's GPU engines' host-memory bookkeeping, summed over its engines:
 * out[0] retired pinned read-back buffers not yet freed, out[1] retired buffers
 * freed (by the engine's reaper thread), out[2] the largest candidate capacity,
 * out[3] pinned read-back bytes held by the ticket slots.  Returns -1 for a
 * scanner without a GPU engine.  (Bookkeeping for tests; call it between scans.) */
struct tsg_scanner;
int tsg_debug_scanner_engine(struct tsg_scanner* s, uint64_t out[4]);

/* Where a scanner makes the findings of HBM-resident batches (tsg_batch.dev_arena):
 * mode 1 the GPU (trivy_amd/csrc/materialize.h), 0 the host, 2 (the default;
 * TSG_GPU_FINDINGS at scanner creation) the GPU while the exact host pass is
 * the bound (the last scan's outlasted 1.5x its GPU phase).  Returns the
 * previous mode, -1 for a scanner without a GPU engine.  (A/B and parity tests.) */
int tsg_debug_scanner_gpu_findings(struct tsg_scanner* s, int mode);

/* Thread-local text of the last error. */
const char* tsg_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
