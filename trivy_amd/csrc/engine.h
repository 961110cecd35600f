// GPU candidate engine: one instance per HIP device.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "rules.h"

namespace tsg {

constexpr uint32_t kChunk = 1024;  // bytes per chunk of the per-chunk '\n' counts and chunk -> file map

constexpr uint32_t kCandGateOpen = 1;   // a keyword of the rule occurs in the file (ASCII, GPU bits)
constexpr uint32_t kCandFoldFile = 2;   // keyword bits may miss occurrences through U+0130 / U+212A in this file
constexpr uint32_t kCandGateValid = 4;  // the two bits above were computed (GPU candidates)
constexpr uint32_t kCandDrop = 8;       // MatchKeywords is false for the rule in this file (never reaches the host)

struct Candidate {      // produced by the verify / full-scan kernels
  uint32_t file;
  uint32_t rule;
  int64_t wlo, whi;     // allowed match-start window, file-relative, inclusive
  int64_t nl_before;    // '\n' count in [file start, wlo)
  uint32_t flags;       // kCand*
  // wlo minus the positions of the last three '\n' before wlo, nearest first
  // (finalize kernel): the host's code-context walk reads these instead of
  // scanning back over long lines.  kNlNone: fewer newlines precede wlo;
  // kNlUnknown: not computed (host candidates, or farther than kNlReach).
  uint32_t nl_back[3];
  // The first three '\n' at or after wlo, as distances from wlo, nearest
  // first (finalize kernel): the line ends of the match line and the code
  // lines after it, which the host otherwise finds by memchr over long lines.
  // kNlNone: fewer newlines follow before the file end; kNlUnknown: not
  // computed (host candidates, or farther than kNlReach).
  uint32_t nl_fwd[3];
  uint32_t pad_;
};
static_assert(sizeof(Candidate) == 64, "Candidate is a 64-B record (tsg_oracle.h, tests/test_host_tail.py)");
constexpr uint32_t kNlNone = 0xFFFFFFFEu, kNlUnknown = 0xFFFFFFFFu;
// A candidate made on the host (no newline hints).
inline Candidate HostCandidate(uint32_t file, uint32_t rule, int64_t wlo, int64_t whi, int64_t nl_before,
                               uint32_t flags) {
  return Candidate{file, rule, wlo, whi, nl_before, flags, {kNlUnknown, kNlUnknown, kNlUnknown},
                   {kNlUnknown, kNlUnknown, kNlUnknown}, 0};
}
constexpr uint64_t kNlReach = uint64_t(1) << 20;

// The transformed bytes of chosen files of a host batch whose transform ran
// on the GPU (RunHost with kinds): buf holds them in file order, off is a
// full n_files+1 offset table into buf (files not chosen are empty).
// Files whose transform is the identity (kind 0, or kind 1 without a '\r')
// are not gathered: raw[f] = 1 and the exact pass reads them in the host
// batch as given.
struct TailOut {
  std::vector<uint8_t> buf;
  std::vector<uint64_t> off;
  std::vector<uint8_t> raw;
  uint64_t xform_bytes = 0;  // transformed arena bytes of the whole batch
};

struct BatchStats {
  uint64_t bytes = 0, files = 0, hits = 0, candidates = 0, special_files = 0, fullscan_tasks = 0, fold_sites = 0;
  uint64_t flagged_blocks = 0;
  uint64_t follow_hits = 0;     // anchor hits past the follow requirements + fold-kernel hits (the NFA runs on these)
  float ms_scan = 0, ms_confirm = 0, ms_careful = 0, ms_verify = 0, ms_fullscan = 0, ms_total = 0;
  float ms_finalize = 0, ms_chunkmap = 0;
  float ms_h2d_span = 0;  // RunHost: first copy issued -> last chunk done (the ingest-inclusive GPU time)
  float ms_xform = 0;     // RunHost with kinds: pre-transform kernels (part of ms_total)
  uint64_t h2d_chunks = 0;
  bool hit_overflow = false, cand_overflow = false;
};

class GpuEngine {
 public:
  GpuEngine(const CompiledRules& cr, int device);
  ~GpuEngine();
  bool ok() const { return err_.empty(); }
  const std::string& error() const { return err_; }
  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }

  // Run the kernels over a device-resident arena.  Offsets: n_files+1 u64
  // (device); the arena must have 64 readable bytes past n_bytes.  The
  // candidates are copied back into `cands`.
  bool Run(const uint8_t* d_arena, uint64_t n_bytes, const uint64_t* d_offsets, uint32_t n_files,
           std::vector<Candidate>* cands, BatchStats* st);

  // Host-resident batch (PCIe-inclusive path): streamed in chunks through the
  // engine's staging ring (below), copies overlapping the kernels of earlier
  // chunks -- of this call and of the calls before it.  With kinds (per file,
  // xform.h), h_arena holds the bytes as read: each chunk is transformed on the
  // GPU before the scan, and the transformed bytes of the files that got
  // candidates come back in *tail.  Concurrent calls are allowed; the caller
  // must NOT hold the engine's device lock: RunHost takes `dev_mu` (the lock
  // the caller's other scans on this engine use) around each chunk's GPU work;
  // a null dev_mu means the engine's own device lock (dev_mu_), which then
  // must be the only lock guarding this engine's Run / Enqueue calls.  A
  // failure's text comes back in *err (err_ is shared with the other users of
  // the engine, so it is not the channel for a call that runs beside them).
  // gather_base / gather_src (optional, with kinds): the files are not in
  // h_arena (NULL then) but at gather_base + gather_src[f] in page-locked,
  // device-mapped host memory (a registered tar layer); each chunk is gathered
  // from there into its staging buffer by a kernel (xform.h GatherHostFiles)
  // instead of one DMA copy -- no host copy of the file bytes.
  bool RunHost(const uint8_t* h_arena, uint64_t n_bytes, const uint64_t* h_offsets, uint32_t n_files,
               std::vector<Candidate>* cands, BatchStats* st, const uint8_t* kinds, TailOut* tail,
               std::mutex* dev_mu, std::string* err, const uint8_t* gather_base = nullptr,
               const uint64_t* gather_src = nullptr);

  // Split form of Run for pipelined callers: Enqueue (with the engine's lock
  // held) puts the whole GPU phase and the copies of the counters and of the
  // full candidate buffer into pinned host memory on the stream and returns;
  // Collect (no lock) waits for that ticket.  The next scan's kernels queue
  // right behind the copies, so the GPU does not idle while a caller wakes
  // up, reads back and releases the lock.  Enqueue returns false when no
  // ticket is free or a diagnostic mode is on (then call Run); Collect sets
  // *rerun when a buffer overflowed (then call Run under the lock: it grows
  // the buffers and rescans).
  // The candidate read-back copies min(cand_cap, 2 x the largest count of
  // the last collected scans + 64 Ki) records: a one-off spike that grew the
  // device buffer does not make every later scan copy all of it; a count
  // above the copied part reruns the scan (as an overflow does).  Errors of
  // Enqueue / Collect are returned in *err (Collect runs without the engine's
  // lock, so it must not write err_).
  struct Ticket {
    int slot = -1;
    uint32_t cand_copy = 0;  // candidates copied back
  };
  bool Enqueue(const uint8_t* d_arena, uint64_t n_bytes, const uint64_t* d_offsets, uint32_t n_files, Ticket* t,
               std::string* err);
  bool Collect(Ticket* t, std::vector<Candidate>* cands, BatchStats* st, bool* rerun, std::string* err);

  // Device buffers of the last run (for tests / bench).
  hipEvent_t ev_scan0() const { return ev_[1]; }
  hipEvent_t ev_scan1() const { return ev_[2]; }

 private:
  bool Ensure(void** p, size_t* cap, size_t need);
  bool EnqueuePhase(const uint8_t* d_arena, uint64_t n_bytes, const uint64_t* d_offsets, uint32_t n_files,
                    uint64_t n_chunks, hipEvent_t* ev, hipEvent_t ev_fs);
  void InitCaps(uint64_t n_bytes);
  struct Slot {  // one in-flight Enqueue: its phase events and pinned read-back buffers
    hipEvent_t ev[7] = {};
    hipEvent_t ev_fs = nullptr, done = nullptr;
    uint32_t* h_cnt = nullptr;
    Candidate* h_cands = nullptr;
    size_t h_cap = 0;
    bool busy = false, has_fs = false;
    uint64_t n_bytes = 0;
    uint32_t n_files = 0;
  };
  static constexpr int kSlots = 4;
  std::atomic<uint32_t> cand_recent_{0};  // largest candidate count of the recently collected scans
  Slot slots_[kSlots];
  std::mutex slot_mu_;
  std::mutex dev_mu_;  // RunHost's device lock when the caller passes none
  // Outgrown pinned read-back buffers.  hipHostFree waits for the whole
  // device, so they are not freed by the thread that regrows a slot (it holds
  // the GPU lock); a reaper thread frees them outside every engine lock, so
  // only that thread waits for the device.  Nothing references a retired
  // buffer: a slot is regrown only after Collect released its last ticket.
  void RetireHost(void* p);
  void ReaperLoop();
  std::mutex reap_mu_;
  std::condition_variable reap_cv_;
  std::vector<void*> retired_host_;  // (reap_mu_)
  bool reap_stop_ = false;           // (reap_mu_)
  std::thread reaper_;               // started with the first retirement
  std::atomic<uint64_t> retired_pending_{0}, retired_freed_{0};

 public:
  // Host memory bookkeeping (tests, tsg_debug_scanner_engine): retired
  // buffers not yet freed, retired buffers freed, the candidate capacity and
  // the pinned read-back bytes the ticket slots hold.
  struct HostMemInfo {
    uint64_t retired_pending, retired_freed, cand_cap, slot_bytes;
  };
  HostMemInfo host_mem_info();

 private:
  bool Transform(int b, uint32_t nf, const uint8_t** arena, const uint64_t** offsets, uint64_t* n_bytes,
                 std::vector<uint64_t>* xoff, float* ms);
  bool GatherTail(const std::vector<Candidate>& part, uint32_t f0, uint32_t nf, const std::vector<uint64_t>& xoff,
                  const uint64_t* raw_off, const uint8_t* kinds, std::vector<uint64_t>* tail_len, TailOut* tail);
  void DumpItemDiag();
  std::vector<uint8_t> h_items_kind_;
  std::vector<uint32_t> h_items_id_;
  std::string err_;
  int device_ = 0;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_[7] = {};  // K0 | K1 | confirm | fold | verify+fullscan | finalize
  // tables
  uint32_t diag_mode_ = 0, diag_confirm_ = 0;
  AnchorInfo* d_anchors_ = nullptr;
  RuleGpu* d_rules_ = nullptr;
  uint32_t* d_rule_kw_ = nullptr;
  uint64_t* d_nfa_ = nullptr;
  uint32_t* d_fullscan_rules_ = nullptr;
  uint32_t kw_words_ = 0, n_rules_ = 0, n_fullscan_rules_ = 0;
  std::vector<uint32_t> fullscan_rules_;
  // streaming prefilter (filter.h)
  uint32_t* d_reach_ = nullptr;
  uint64_t* d_core_ = nullptr;
  uint32_t* d_group_items_ = nullptr;
  uint32_t* d_bucket_groups_ = nullptr;
  void* d_ftabs_ = nullptr;
  void* d_fold_pairs_ = nullptr;  // fold kernel work list
  void* d_fold_first_ = nullptr;  // per item: bytes that can start it (fold kernel prefilter)
  uint32_t n_fold_pairs_k_ = 0, n_fold_pairs_s_ = 0, n_fold_cap_k_ = 0, n_fold_cap_s_ = 0;
  void* d_fold_idx_off_ = nullptr;   // fold kernel: capable tasks by (rune kind, q, key byte)
  void* d_fold_idx_items_ = nullptr;
  uint32_t n_fold_cap_k_idx_ = 0, n_fold_cap_s_idx_ = 0;
  bool fold_idx_ = true;
  void* d_kwfold_pairs_ = nullptr;  // kwfold kernel work list (keyword items through U+0130 / U+212A)
  uint32_t n_kwf_ri_ = 0, n_kwf_rk_ = 0, n_kwf_ci_ = 0, n_kwf_ck_ = 0;
  bool kw_fold_ = false;
  uint32_t ftabs_bytes_ = 0, ft_bucket_off_ = 0, ft_bucket_items_ = 0, ft_items_ = 0;
  uint32_t ft_item_ids_ = 0, ft_item_cls_ = 0, ft_classes_ = 0, ft_luts_ = 0;
  // confirm-only part of the table blob (after the fold kernel's prefix): the
  // core tables over byte classes (filter.h core, columns deduplicated)
  uint32_t ftabs_fold_bytes_ = 0, ft_cmap_ = 0, ft_ccore_ = 0, ft_gitems_ = 0, ft_bgroups_ = 0, n_core_cls_ = 0;
  uint32_t ft_hkeys_ = 0, ft_hitems_ = 0, hash_bits_ = 0, hash_buckets_ = 0;  // literal-window hash
  size_t c_lds_bytes_ = 0;
  bool lds_tabs_ = true;  // confirm/fold kernels stage the item tables in LDS
  bool fold_stage_ = false;        // global-table fold kernel: items + classes staged in LDS
  uint32_t fold_grid_ = 2048;      // workgroups of the LDS-table fold kernel (TSG_FOLD_GRID)
  bool fold_wide_ = false;         // staged global-table fold kernel: 16-wave workgroups (TSG_FOLD_WAVES=4: 4)
  bool fold_check_first_ = true;   // global-table fold kernel: first-byte set test per start (TSG_FOLD_FIRST=0: off)
  bool c_stage_classes_ = false;   // global-table confirm kernel: classes staged in LDS
  size_t fold_stage_bytes_ = 0;
  uint32_t n_fclasses_ = 0;
  void* d_recs_ = nullptr; size_t cap_recs_ = 0;
  uint32_t rec_cap_ = 0, fold_cap_ = 0, n_fitems_ = 0;
  // per-batch buffers
  void* d_chunk_file_ = nullptr; size_t cap_chunk_file_ = 0;
  void* d_nl_ = nullptr; size_t cap_nl_ = 0;
  void* d_kw_ = nullptr; size_t cap_kw_ = 0;
  void* d_flags_ = nullptr; size_t cap_flags_ = 0;
  void* d_hits_ = nullptr; size_t cap_hits_ = 0;
  void* d_cands_ = nullptr; size_t cap_cands_ = 0;
  void* d_folds_ = nullptr; size_t cap_folds_ = 0;
  void* d_wins_ = nullptr; size_t cap_wins_ = 0;  // TSG_K2_PACK experiment: packed confirm windows
  uint32_t* d_counters_ = nullptr;  // [0] hits [1] cands [2] special files [3] hit overflow [4] cand overflow
                                    // [7] flagged-block records [8] record overflow
                                    // [9] fold sites [10] fold-site overflow
                                    // [6] full-scan list overflow [11] anchor-item matches [13] open pairs
  // host-batch streaming (RunHost): a ring of staging buffers, a copy stream
  hipStream_t copy_stream_ = nullptr;
  static constexpr int kNStage = 4;  // staging buffers: the copier runs up to three chunks ahead
  // The staging ring.  RunHost reserves one slot per chunk, numbered in call
  // arrival order across calls; slot s uses staging buffer s % kNStage.  One
  // copier thread (CopierLoop) copies the slots in order, slot s as soon as
  // slot s - kNStage has been scanned; chunks are scanned in slot order
  // (ring_turn_).  So the copy engine moves the next call's first chunks while
  // this call's last chunk is transformed, scanned and read back, and several
  // small host batches in flight (the analyzer's collectors) overlap their
  // copies with each other's kernels.
  struct HostCall;
  struct StageJob {
    uint64_t slot;
    HostCall* call;
    uint32_t f0, f1;  // the chunk's files
  };
  bool CopyChunk(const StageJob& j, std::string* err);
  void CopierLoop();
  std::mutex ring_mu_;
  std::condition_variable ring_cv_;
  std::deque<StageJob> ring_jobs_;                     // reserved, not yet copied (slot order)
  uint64_t ring_next_ = 0, ring_turn_ = 0, ring_copied_ = 0;  // next slot to reserve / to scan / copied below
  bool stage_ok_[kNStage] = {};                        // the copy of the buffer's current slot was issued
  std::string stage_err_[kNStage];
  bool ring_stop_ = false;
  std::thread copier_;
  hipEvent_t ev_copied_[kNStage] = {}, ev_h2d_[2] = {};
  void* d_stage_[kNStage] = {}; size_t cap_stage_[kNStage] = {};
  void* d_stage_off_[kNStage] = {}; size_t cap_stage_off_[kNStage] = {};
  uint64_t* h_off_[kNStage] = {}; size_t cap_h_off_[kNStage] = {};  // pinned, rebased chunk offsets
  uint64_t* h_xoff_ = nullptr; size_t cap_h_xoff_ = 0;  // pinned: transformed offsets + the error word
  // Pinned staging of Run's counter / candidate read-back and GatherTail's
  // uploads and read-back: a pageable hipMemcpy goes through the runtime's own
  // staging and held up the copier's H2D of later chunks (blocking 20-80 ms
  // copies at fixed chunks of the C2 ingest leg, TSG_RING_DEBUG).
  uint32_t* h_run_cnt_ = nullptr;
  void* h_run_cands_ = nullptr; size_t cap_h_run_cands_ = 0;
  void* h_gup_ = nullptr; size_t cap_h_gup_ = 0;
  void* h_gbuf_ = nullptr; size_t cap_h_gbuf_ = 0;
  bool EnsureHost(void** p, size_t* cap, size_t need);
  // GPU pre-transform (xform.h): per-chunk kinds, lengths, transformed offsets and bytes, the gather
  void* d_kind_[kNStage] = {}; size_t cap_kind_[kNStage] = {};
  // host-memory gather (RunHost gather_base): per staging buffer the chunk's source
  // offsets + work items (device) and their pinned staging
  void* d_gsrc_[kNStage] = {}; size_t cap_gsrc_[kNStage] = {};
  void* h_gsrc_[kNStage] = {}; size_t cap_h_gsrc_[kNStage] = {};
  void* d_xlen_ = nullptr; size_t cap_xlen_ = 0;
  void* d_xoff_ = nullptr; size_t cap_xoff_ = 0;
  void* d_xscan_ = nullptr; size_t cap_xscan_ = 0;
  void* d_xf_ = nullptr; size_t cap_xf_ = 0;
  void* d_gfiles_ = nullptr; size_t cap_gfiles_ = 0;
  void* d_gdst_ = nullptr; size_t cap_gdst_ = 0;
  void* d_gbuf_ = nullptr; size_t cap_gbuf_ = 0;
  hipEvent_t ev_x_[2] = {};
  uint64_t chunk_bytes_ = uint64_t(1) << 30;             // TSG_INGEST_CHUNK_MB
  uint32_t hit_cap_ = 0, cand_cap_ = 0;
  uint32_t fs_chunk_ = 65536;         // TSG_FULLSCAN_CHUNK: full-scan bytes per lane (min, wave-wide pairs)
  uint32_t fs_task_bytes_ = 4096;     // TSG_FS_TASK_BYTES: full-scan lane task size (min; >= 8 x max_len)
  uint32_t fs_pair_cap_ = 0, fs_task_cap_ = 0;
  void* d_fs_pairs_ = nullptr; size_t cap_fs_pairs_ = 0;  // FsPair list
  void* d_fs_tasks_ = nullptr; size_t cap_fs_tasks_ = 0;  // 4 x FsTask lists (by NFA width)
  void* d_fs_wave_ = nullptr; size_t cap_fs_wave_ = 0;    // pairs run wave-wide
  uint32_t* d_fs_ctr_ = nullptr;                          // [0] pairs [1..4] tasks [5] wave pairs
  hipEvent_t ev_fs_ = nullptr;
  hipEvent_t ev_sync_ = nullptr;  // blocking-sync: the host waits asleep, not spinning
  bool blocking_sync_ = true;
  uint32_t verify_blocks_ = 4096;  // a lane per deferred hit (0.59 -> 0.51 ms vs 2048 on C2)
  uint32_t finalize_blocks_ = 16384;  // a wave per candidate, latency-bound: ~1 candidate per wave (0.42 -> 0.25 ms vs 1024)
  hipError_t WaitStream();
  hipError_t WaitEvent(hipEvent_t ev);
  uint32_t* d_item_diag_ = nullptr;   // TSG_DIAG_ITEMS=<file>: per-item counters dumped after each run
  std::string item_diag_path_;
};

}  // namespace tsg
