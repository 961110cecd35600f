/* oracle/build/libtsg_host.so -- TEST INFRASTRUCTURE, not the product.
 *
 * Built from the product's host sources plus oracle/native/*.cpp by
 * oracle/build_native.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it.  It exports the whole libtsg.so C-ABI (its own
 * copy, loaded RTLD_LOCAL) plus:
 *
 *   tsg_debug_host_tail / _cands   the exact host tail over whole-file / given
 *                                  candidate windows (no GPU): checks the tail
 *                                  against the oracle on CPU
 *   tsg_debug_scanner_host_only    a scanner without a GPU engine (analyzer
 *                                  host logic on CPU)
 *   tsg_cpuref_scan                the reference CPU algorithm restated in C++
 *                                  (pkg/fanal/secret/scanner.go:377-463: per file
 *                                  and rule, bytes.ToLower + Contains keyword
 *                                  gate, then whole-file regexp FindAll, then
 *                                  the same exact tail) -- bench.py's CPU
 *                                  baseline ("port", restated reference)
 */
#ifndef TSG_ORACLE_H
#define TSG_ORACLE_H
#include <stdint.h>

#include "tsg_scanner.h"
#ifdef __cplusplus
extern "C" {
#endif

int tsg_debug_host_tail(const tsg_global* g, const tsg_batch* b, tsg_result** out);
/* candidates: 64-B records (trivy_amd/csrc/engine.h Candidate), e.g. dumped by TSG_DUMP_CANDS */
int tsg_debug_host_tail_cands(const tsg_global* g, const tsg_batch* b, const void* cands, uint64_t n_cands,
                              tsg_result** out);
int tsg_debug_scanner_host_only(const tsg_global* g, tsg_scanner** out);

/* The reference algorithm on `threads` host threads (files in parallel, like
 * the analyzer's --parallel goroutines).  Result: as tsg_scan. */
int tsg_cpuref_scan(const tsg_global* g, const tsg_batch* b, int threads, tsg_result** out);

/* The host pool (trivy_amd/csrc/parallel.h) under `callers` concurrent
 * ParallelFor jobs of n items each (each item sleeps `item_us`), all wide or
 * all ordinary: returns the peak number of threads inside the jobs' bodies at
 * once, and the pool's steady / total worker counts. */
int tsg_debug_pool_peak(int callers, uint64_t n, int item_us, int wide, int* steady, int* workers);

/* The findings sort (scanner.go:452-457, pdqsort): n findings with rule ids,
 * RuleID ranks and match texts; threads 0 = SortFindings, > 0 =
 * SortFindingsParallel on that many pool threads.  out_order[i] = the original
 * index of the finding sorted to position i. */
int tsg_debug_sort_findings(uint32_t n, const uint32_t* rule, const uint32_t* rule_rank, uint32_t n_rules,
                            const char* text, uint64_t text_len, const uint32_t* match_off, const uint32_t* match_len,
                            int threads, uint32_t* out_order);

#ifdef __cplusplus
}
#endif
#endif
