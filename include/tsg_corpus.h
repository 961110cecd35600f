/* Synthetic corpus generator (bench / large-size tests only; not the scan path).
 * Deterministic: SplitMix64(seed ^ f(file index)); spec in SURVEY.md §8(d). */
#ifndef TSG_CORPUS_H
#define TSG_CORPUS_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* File sizes for target_bytes total; returns the file count and, when offsets
 * is non-NULL, writes offsets[0..min(n, cap-1)]. */
int64_t tsg_corpus_plan(uint64_t seed, uint64_t target_bytes, uint64_t* offsets, uint64_t cap);
/* Fill arena (offsets[n_files] bytes) and paths (n_files * path_stride,
 * NUL-terminated) using `threads` host threads.  Planted secrets are drawn
 * from pool (concatenated strings, pool_off[n_pool+1]). */
int tsg_corpus_fill(uint64_t seed, const uint64_t* offsets, uint64_t n_files, const char* pool,
                    const uint64_t* pool_off, uint32_t n_pool, double secrets_per_byte, uint8_t* arena,
                    char* paths, uint32_t path_stride, int threads);
/* Turns a deterministic `share` of the files CRLF in place ('\n' -> "\r\n",
 * cut at each file's size); is_crlf (optional, n_files) marks them.  Returns
 * the number of CRLF files. */
int64_t tsg_corpus_crlf(uint64_t seed, const uint64_t* offsets, uint64_t n_files, uint8_t* arena, double share,
                        uint8_t* is_crlf, int threads);
/* bytes.ReplaceAll(content, "\r", "") per file (secret.go:121), the packing
 * step of the HBM-resident C2 bench: out gets the stripped files back to back,
 * out_offsets their n_files + 1 offsets. */
int tsg_corpus_strip(const uint64_t* offsets, uint64_t n_files, const uint8_t* in, uint8_t* out, uint64_t* out_offsets,
                     int threads);
/* BASELINE configs[3] (C4): an uncompressed ustar image layer of many small
 * files (log-normal sizes, median 1.5 KiB, sigma 1.2) with distro-like paths
 * (allow-listed system dirs, executables, .pyc files, skipped extensions, app
 * files with 5 % CRLF), directory / symlink / whiteout entries.  Returns the
 * archive size (out == NULL: the size needed), -1 if cap is too small. */
int64_t tsg_corpus_layer(uint64_t seed, uint64_t target_file_bytes, const char* pool, const uint64_t* pool_off,
                         uint32_t n_pool, double secrets_per_byte, uint8_t* out, uint64_t cap, int threads,
                         uint64_t* n_entries);
#ifdef __cplusplus
}
#endif
#endif
