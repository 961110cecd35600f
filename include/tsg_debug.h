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

/* regexp.MatchString: 1 = match, 0 = no match, <0 = compile error. */
int tsg_regex_match(const char* pattern, const uint8_t* text, uint64_t n);

/* bytes.ToLower (Go semantics).  Writes up to out_cap bytes, returns the full length. */
int64_t tsg_go_bytes_to_lower(const uint8_t* s, uint64_t n, uint8_t* out, uint64_t out_cap);

/* Thread-local text of the last error. */
const char* tsg_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
