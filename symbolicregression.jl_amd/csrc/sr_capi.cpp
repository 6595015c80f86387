// sr_capi.cpp — the C ABI (include/sr_amd.h) over the HIP interpreter.
//
// Call path of one batched scoring call (sr_eval_loss_batch):
//   host: compile the trees (sr_compile.cpp) -> upload programs -> interpreter kernel (partials per
//   row block) -> fixed-order reduce kernel -> copy per-tree {Σloss, flags} back -> rare exact-sum
//   check for trees whose checked values came close to overflowing -> loss = Σ / denominator.
// Mirrors reference src/LossFunctions.jl:90-117 (`_eval_loss`) for each tree of the batch.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <limits.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/sr_amd.h"
#include "sr_compile.h"
#include "sr_eval.h"
#include "sr_fold.h"
#include "sr_fold_dev.h"

namespace {

thread_local std::string g_last_error;
struct SrComm;  // the sharded calls' transport (multi-GPU section below)

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define SR_HIP_CHECK(expr)                                                                          \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess)                                                                           \
      return set_error(SR_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));              \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      hipError_t e = hipFree(p);
      if (e != hipSuccess) return e;
      p = nullptr;
      cap = 0;
    }
    size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <typename U>
  U* as() const {
    return static_cast<U*>(p);
  }
};

// Pinned host staging (programs, offsets, launch order): hipMemcpyAsync from it is a true async DMA,
// so the host compiles the next chunk while the device runs the previous one.
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  unsigned flags = hipHostMallocDefault;
  hipError_t ensure(size_t bytes, hipStream_t s, hipStream_t s2) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      hipError_t e = hipStreamSynchronize(s);  // no DMA may still read the old buffer
      if (e == hipSuccess && s2) e = hipStreamSynchronize(s2);  // (a context's second stream is created lazily)
      if (e == hipSuccess) e = hipHostFree(p);
      if (e != hipSuccess) return e;
      p = nullptr;
      cap = 0;
    }
    size_t want = bytes < 65536 ? 65536 : bytes + bytes / 4;
    hipError_t e = hipHostMalloc(&p, want, flags);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <typename U>
  U* as() const {
    return static_cast<U*>(p);
  }
};

constexpr int kMaxChunks = 4;
constexpr int kLossCodeBase = 256;

// Parameter-free losses (and HuberLoss with its default delta = 1) may be passed by kind.
inline bool loss_direct_ok(int kind) {
  switch (kind) {
    case SR_LOSS_LP: case SR_LOSS_L1_EPS_INS: case SR_LOSS_L2_EPS_INS: case SR_LOSS_PERIODIC:
    case SR_LOSS_QUANTILE: case SR_LOSS_SMOOTH_L1_HINGE: case SR_LOSS_DWD_MARGIN:
      return false;
    default:
      return kind >= 0 && kind < SR_LOSS_COUNT;
  }
}

}  // namespace

// the thread-local error message, for the other translation units of the library (sr_search.cpp)
int sr_set_error(int code, const std::string& msg) { return set_error(code, msg); }

struct sr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // second stream of the chunked pipeline (odd chunks), created on the first chunked call: a HIP
  // stream takes one of the process's GPU_MAX_HW_QUEUES (4) hardware queues round-robin at creation, so
  // an idle second stream per context left the search's four scoring lanes sharing two queues
  hipStream_t stream2 = nullptr;
  hipError_t need_stream2() {
    return stream2 ? hipSuccess : hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking);
  }
  hipEvent_t ev_join = nullptr;
  hipEvent_t ev_start = nullptr, ev_k0 = nullptr, ev_k1 = nullptr, ev_end = nullptr;
  hipEvent_t ev_c0[kMaxChunks] = {}, ev_c1[kMaxChunks] = {};  // per-chunk interpreter launches
  hipEvent_t ev_d0 = nullptr, ev_d1 = nullptr;                 // the derived-column launch
  // the last gradient call's tangent-kernel launches, per tangent bucket (1, 2, 4, 8, 16): HIP events,
  // algorithmic flops (sr_last_grad_info), work items, rows per lane
  static constexpr int kGradBuckets = 5;
  hipEvent_t ev_g0[kGradBuckets] = {}, ev_g1[kGradBuckets] = {};
  // the in-order loss fold's device phases (sr_last_fold_ms): PRED pass, segment sums, composed steps,
  // chain; events around each, accumulated over the call's fold batches (the fold is rare: always timed)
  hipEvent_t ev_f[5] = {};
  double fold_ms[4] = {0, 0, 0, 0};
  bool grad_timed[kGradBuckets] = {};
  double grad_flops[kGradBuckets] = {};
  int64_t grad_items[kGradBuckets] = {};
  int grad_rows[kGradBuckets] = {};
  int n_chunks_last = 0;
  bool derived_last = false;  // the last run_batch launched derived columns (timed by ev_d0/ev_d1)
  int n_derived_last = 0;
  int64_t n_exact_last = 0;  // trees of the last eval_loss call sent through the exact-sum pass
  int64_t n_fold_last = 0;   // trees of the last eval_loss call whose loss fold was computed in order (sr_fold.h)
  int64_t fold_slow_last = 0;  // ... their segments folded row by row (the rest: composed steps)
  int64_t fold_seg_last = 0;   // ... and the segment length used
  int64_t fold_seg = -1;       // SR_AMD_FOLD_SEG / sr_set_tuning "fold_seg": -1 automatic, 0 one scan per tree
  double exact_kernel_ms = 0.0;  // device time of that pass (its interpreter + combine launches)
  // programs + per-tree metadata of the last run_batch: ONE device allocation and ONE pinned staging
  // buffer with the same layout (code | offsets | static_bad | launch order), so a single-chunk call
  // uploads with one DMA; per-tree {Σ loss, flags} likewise share one allocation (one DMA back)
  HostBuf h_prog, h_outs, h_grad;  // (h_grad: the gradient call's staging image, then its results)
  // Small calls with several row blocks (round 5, SR_AMD_HOST_REDUCE / "host_reduce"): the
  // interpreter writes its per-(row block, tree) partials straight into pinned host memory (h_part)
  // and the host reduces them after the one stream synchronisation, in the reduce kernel's own order
  // (sr_reduce_positions: lane l folds row blocks l, l + 64, ...; a shfl_xor butterfly over the 64
  // lanes), so the bits are the reduce launch's; a C3 scoring call loses that launch and its gap.
  // The bound is on the call's partials (trees x row blocks): a C3 / C5 scoring call has ~1,600; a
  // 1,250-tree x 256-row-block call (320k partials) wrote 3.8 MB over PCIe and spent ~1 ms reducing on
  // the host (tools/share_probe.py: 2.47 ms per call against 1.1 with the reduce launch).
  int64_t host_reduce = 8192;
  HostBuf h_part;
  struct HostReduction {
    int64_t p0, np;
    int n_rb;
  };
  std::vector<HostReduction> host_reductions;  // this call's launches whose partials await the host
  std::vector<double> host_acc;                // (their per-(position, lane) accumulators)
  std::vector<uint32_t> host_fl;
  int64_t host_red_rb = 0;                     // their partial buffer's row-block stride (n_rb)
  const uint8_t* h_bad_last = nullptr;         // the last run_batch's staged static flags and launch order
  const uint32_t* h_perm_last = nullptr;
  void* d_code = nullptr;
  uint32_t* d_off = nullptr;
  uint8_t* d_bad = nullptr;
  uint32_t* d_perm = nullptr;
  uint32_t* d_end = nullptr;  // [nt] end of each tree's program (code is staged in launch order)
  double* d_out_sum = nullptr;
  uint32_t* d_out_flag = nullptr;
  size_t outs_flag_off = 0;
  // Small single-chunk LOSS calls (the search's regime: tens of trees, ~100 rows) are latency-bound:
  // SR_AMD_HOST_IO = 1 (default) lets the kernel write the per-tree results straight into pinned
  // host memory (no copy back); 0 copies them.  (Round 5's 2 — programs read from the pinned staging
  // buffer — was measured without payoff and removed in round 6.)
  int host_io = 1;
  bool want_host_out = false;  // set by eval_loss_impl around its run_batch
  bool outs_on_host = false;   // the last run_batch wrote {Σ, flags} to h_outs
  uint32_t hint_epoch = 0;  // dead-tree hint epoch of the current call
  int debug_hint_regrow = 0;       // tests (sr_set_tuning "debug_hint_regrow"): grow the hint array in place
  void* hint_reserve = nullptr;    // its fixed-address reservation
  int exact_g = 0;          // SR_AMD_EXACT_G (tuning): listed trees per workgroup of the EXACT pass
  int exact_w = 4;          // SR_AMD_EXACT_W / sr_set_tuning "exact_w": waves per EXACT workgroup (4, or 1)
  int par_stage = 1;        // SR_AMD_PAR_STAGE: large chunks' programs copied to the staging buffer in parallel
  // SR_AMD_DERIVED (default 1): nodes unary(feature) shared by several trees of a large LOSS call
  // are evaluated once per call into derived columns (LOAD_DERIVED); 0 disables
  int derived = 1;
  std::mutex mu;
  std::vector<SrOpset> opsets;
  std::vector<int> tiers;
  std::vector<std::pair<int, double>> losses;  // registered (kind, param); code = kLossCodeBase + index
  DevBuf prog, outs, part_sum, part_flag, pred, row_idx, tree_list,
      range_lo, range_hi, range_sums, packed, hint, jsum_prog, jsum_scratch, probe_sum, probe_flag, g_code, g_offsets, g_consts, g_const_off, g_items, g_part, g_out,
      derived_cols, probe_derived, fold_io;
  // The exact-sum pass's small transfers (round 5): the leaf ranges and the Julia-sum level program
  // depend only on the view's row count, so they stay on the device between calls (host mirrors below;
  // a buffer that grows loses them); the tree list goes up and the verdicts come back through pinned
  // memory.  Pageable copies cost ~15 us each, and a one-tree pass made five of them.
  HostBuf h_exact;
  std::vector<int64_t> exact_lo_dev, exact_hi_dev;  // what range_lo / range_hi hold
  int64_t jsum_n_dev = -1;                          // the row count jsum_prog was built for
  // SR_AMD_EXACT_LIST_HOST (default 1): the pass reads its tree list from the pinned staging buffer
  // (no upload ahead of the kernel); 0 copies it to the device first
  int exact_list_host = 1;
#ifdef SR_STAMPS
  DevBuf stamps;  // latency-analysis builds: the last main launch's per-wave stamps (sr_debug_stamps)
  int64_t n_stamps = 0;
#endif
  int stress_probe = 1;  // SR_AMD_STRESS_PROBE: the probe runs the dataset's stress rows (below)
  int code_cache = 1;    // SR_AMD_CODE_CACHE: LDS program cache of the register-stack launches (0: off)
  // SR_AMD_FUSED_REDUCE: multi-row-block LOSS launches reduce their partials in the launch (the last
  // workgroup of a tree group) when the group holds at most this many partials; 0 (default): a reduce
  // launch — measured faster: every workgroup's drained stores + barrier + counter add cost more than
  // the launch they save (C3 search 14.4 vs 13.3 iterations/s, C2's dead trees 0.52 vs 0.71 ms;
  // profiles/r04_ab_fused_reduce.txt)
  int64_t fused_reduce = 0;
  int vstk_rows = 0;        // SR_AMD_VSTK_ROWS / "vstk_rows": rows per lane of the register-stack kernel (0: default)
  int grad_rows_force = 0;  // SR_AMD_GRAD_ROWS / "grad_rows": the gradient kernel's rows per lane (0: chosen per call)
  int grad_sort = 1;        // SR_AMD_GRAD_SORT / "grad_sort": gradient work items ordered by program cost
  DevBuf group_cnt;      // its per-group counters (zeroed at allocation; each launch leaves them zero)
  int first_chunk = 6;   // SR_AMD_FIRST_CHUNK: the two-chunk pipeline's first chunk is 1/first_chunk
  int64_t chunk_min = 1024;  // SR_AMD_CHUNK_MIN: the two-chunk pipeline runs when its first chunk holds this many trees
  // data-path transport of the sharded calls: the library's own RCCL over xGMI on its own HIP runtime
  // (sr_comm_init; torch's bundled runtime cannot share the GPU with this one in a process), or the
  // caller's host collectives (sr_comm_init_host)
  std::unique_ptr<SrComm> xport;
  int comm_ranks = 0;
  int comm_rank = 0;
  uint64_t comm_gen = 0;  // process-unique id of the current communicator (shard layouts are cached per id)
  // buffers of the sharded calls' collectives only (their growth is identical on every rank: Prep):
  // shard layout / exact-pass folds / loss-fold chain / tree results, the packed partials, the agree word
  DevBuf coll_buf, coll_packed, ctl;
  HostBuf h_coll;        // pinned staging of the tree-sharded results
  int inject_fail = 0;   // tests (sr_set_tuning "inject_failure"): the next k collective-buffer growths fail
  int inject_post = 0;         // tests ("inject_failure_post"): a HIP failure right after the sharded all-reduce
  int inject_post_exact = 0;   // tests ("inject_failure_post_exact"): ... after the exact-sum all-gather
  int inject_post_gather = 0;  // tests ("inject_failure_post_gather" k): this rank's copy of the k-th fold gather fails
  double last_eval_ms = 0.0, last_total_ms = 0.0;
  double last_busy_ms = 0.0;  // union of the last call's interpreter launch intervals (sr_last_phase_ms out[8])
  // the two above are read from the last call's events lazily, when asked for (sr_last_kernel_ms /
  // sr_last_phase_ms): a small call (the search's) does not pay the event queries it never reads
  bool timing_pending = false;
  int timing = 1;           // 0: no timing events at all (sr_set_tuning "timing"; the search engine's calls)
  bool timed_last = false;  // the last run_batch recorded its events
  // host-side phases of the last eval_loss call (ms): compile, upload+launch, wait, exact pass,
  // finalize (sr_last_phase_ms)
  double phase_ms[5] = {0, 0, 0, 0, 0};
  std::chrono::steady_clock::time_point phase_t;
  void start_phases(std::chrono::steady_clock::time_point t) {
    phase_t = t;
    for (double& v : phase_ms) v = 0.0;
  }
  bool internal_pass = false;  // the fold's PRED passes: run_batch leaves the call's phase clock alone
  void mark_phase(int i) {
    if (internal_pass) return;
    const auto now = std::chrono::steady_clock::now();
    phase_ms[i] = std::chrono::duration<double, std::milli>(now - phase_t).count();
    phase_t = now;
  }
  int cu_count = 256;
  int rows_override = 0;    // SR_AMD_ROWS_PER_LANE (tuning): 4 selects the f32 BASIC 4-rows/lane kernel
  int tree_group = 0;       // SR_AMD_TREES_PER_BLOCK override (0 = heuristic)
  int rows_last = 0;        // rows per lane of the last interpreter call (sr_last_phase_ms out[7])
  int waves_override = 0;   // SR_AMD_WAVES (tuning): 8 selects the 8-wave f32 BASIC L2 loss kernel
  bool cost_order = true;   // launch trees in decreasing estimated cost (SR_AMD_NO_SORT=1 disables)
  bool balance_groups = true;  // deal the cost order round-robin over tree groups (SR_AMD_BALANCE=0: contiguous)
  bool dead_hints = true;   // share dead-tree hints across row blocks (SR_AMD_NO_HINT=1 disables)
  // SR_AMD_MAX_ROW_BLOCKS (tuning): upper bound on row blocks per tree.  512 since round 5 (A/B, three
  // alternating passes on one box, profiles/r05_ab_row_blocks.txt): C2 4.47 vs 4.51 ms per step, C4
  // 1,520 vs 1,533 ms, the tree-sharding share (1,250 trees) 1.03 vs 1.09 ms: a small population keeps
  // 128 trees per workgroup instead of halving it to fill the GPU.  Results do not depend on it only
  // up to the f64 summation order of the partials (row blocks are a function of the rows alone).
  int max_row_blocks = 512;
  int chunks = 2;           // SR_AMD_CHUNKS: pipeline compile/launch over this many tree chunks (1 = off)
  int probe = 2;            // dead-tree probe launch (SR_AMD_PROBE): 0 off, 1 before every chunk,
                            // 2 (default) only before the chunks after the first, whose probe
                            // overlaps the first chunk's kernel (profiles/r01_ab_probe_modes.txt)
  std::vector<uint32_t> perm_host;
  // The reference's in-order loss fold for EVERY complete tree (round 6; sr_fold_dev.h, sr_aux.hip): a
  // complete tree's loss is LossFunctions' left-to-right fold in T of its elementwise losses
  // (src/LossFunctions.jl:38-58), divided in T, not the device's f64 sum.  SR_AMD_REF_FOLD / "ref_fold":
  // 1 (default) single-GPU loss calls with weights >= 0; 0 the f64 sums (rounds 1-5).  Small calls
  // (every tree's losses fit fold_store_mb) keep the loss launch's losses; larger Float32 calls run the
  // complete trees again in FOLD mode (slow segments' losses in up to fold_slot_mb of slots); larger
  // Float64 calls, and calls whose row blocks pass fold_seg_max rows (C4: 2^26 rows per GPU), keep the f64
  // sum (Float64: within ~1e-13 of the fold, north_star's f64 bar is 1e-10).
  int ref_fold = 1;
  int64_t fold_store_mb = 512;
  int64_t fold_slot_mb = 24576;  // (allocated as needed: ~24 slots per tree; C4's 2^26 rows take ~21 GB)
  // the plan's window: the fold within 2^-8 of the f64 prefix, else the tree fails (C2's trees: the fold is
  // within 2.1e-3 of the f64 sum at 2^20 rows; 2^-6 kept twice the slow segments)
  int fold_delta_log2 = 8;
  int64_t fold_seg_max = 16384;  // SR_AMD_FOLD_SEG_MAX: calls whose row blocks are longer keep the f64 sum
  int64_t fold_rows_max = int64_t(1) << 24;  // SR_AMD_FOLD_ROWS_MAX: longer folds keep the f64 sum
  int fold_debug_fail = 0;   // (tests: "fold_debug_fail")
  int fold_reduce = 1;
  int fold_pre_start = 1;    // SR_AMD_FOLD_PRE_START: stored-loss folds start in the pair kernel (0: in the walk)       // SR_AMD_FOLD_REDUCE: stored-loss folds reduce in the pair kernel (0: a reduce launch)
  int fold_walk_dbg = 0;     // SR_AMD_FOLD_WALK_DBG (analysis): 2 no O(1) slow blocks, 4 no serial start
  int fold_stats = 0;        // SR_AMD_FOLD_STATS=1: per-tree walk statistics to stderr after each call (analysis)
  DevBuf fold_dbg;
  bool want_fold = false;    // set by eval_loss_submit around its run_batch
  int fold_path_last = 0;    // 0 none, 1 stored losses, 2 FOLD mode
  DevBuf fold_code, fold_tab, fold_store, fold_ctl, fold_io2, fold_sq, fold_tab2;
  std::shared_ptr<void> fold_job;  // a row-sharded call's FoldJob<T>, until its ranks agree on the verdicts
  int inject_post_wsum = 0;        // tests ("inject_failure_post_wsum"): this rank's copy of the weights' sum gather fails
  size_t outs_fval_off = 0, outs_fst_off = 0, outs_bytes_all = 0;
  hipEvent_t ev_fc0[kMaxChunks] = {}, ev_fc1[kMaxChunks] = {};  // each chunk's fold launches
  bool fold_timed_last = false;
  int64_t n_ref_ok_last = 0, n_ref_fail_last = 0;  // trees whose loss is the walk's fold / that fell back
  double fold_kernel_ms_last = 0.0;
};

// For the search engine (sr_search.cpp, not in the public header): set the context's "timing" knob
// and return its previous value, under the context's lock (a caller's setting is restored after the
// engine's calls).
int sr_ctx_swap_timing(sr_ctx* ctx, int value) {
  std::lock_guard<std::mutex> g(ctx->mu);
  const int old = ctx->timing;
  ctx->timing = value != 0 ? 1 : 0;
  return old;
}

struct sr_dataset {
  sr_ctx* ctx = nullptr;
  int dtype = SR_DTYPE_F32;
  int64_t nf = 0, n = 0, ld = 0;
  void* X = nullptr;  // [nf][ld]
  void* y = nullptr;  // [ld] or NULL
  void* w = nullptr;  // [ld] or NULL
  std::vector<double> w_host;  // weights (for Σw of SubDataset views)
  double wsum = 0.0;
  double w_min = 0.0;      // smallest weight (the loss-fold overflow rule needs w >= 0: sr_fold.h)
  double max_abs_x = 0.0;  // max |X| over the data (NaN / Inf if any value is non-finite)
  mutable double wsum_jl_f32 = NAN, wsum_jl_f64 = NAN;  // Base.sum(w) in Float32 / Float64 (cached on first use)
  // dead-tree probe rows (large datasets): the "stress rows" — per feature the K largest, K smallest
  // and K smallest-magnitude values, where exp overflows, logs and divisions blow up — then rows 0, 1,
  // ... up to kProbeRows; int64 row indices on the device (NULL for small datasets)
  void* probe_rows = nullptr;
  int64_t n_probe = 0;
  // row-sharded calls (sr_eval_loss_sharded): every shard's rows, Σw and max|X|, exchanged once per
  // communicator (shard_gen = its sr_ctx::comm_gen; rank r holds global rows [offs[r], offs[r + 1]))
  mutable uint64_t shard_gen = 0;
  mutable std::vector<int64_t> shard_offs;
  mutable double shard_wsum = 0.0, shard_max_abs_x = 0.0;
  mutable double shard_w_min = 0.0;  // smallest weight over every shard
  mutable int64_t shard_min_rows = 0;
};

namespace {

constexpr int64_t kRowAlign = 2048;  // a multiple of every kernel's row tile (64 lanes x R rows)
constexpr int64_t kProbeRows = 2048;
constexpr int kProbeTiles = 4;  // row tiles of a dead-tree probe launch
// dynamic LDS a register-stack workgroup may use with its program cache: with the 5 KiB of static
// libm tables, 4 workgroups still fit a CU's 160 KiB
constexpr size_t kCodeCacheLds = 34 * 1024;

// Work decomposition: row tiles of 64*R rows (one LDS image each), `tiles` per block; trees grouped G
// per block (the block's 4 waves share the G trees of a tile).
struct Grid {
  int G = 32, tiles = 1, n_row_blocks = 1, n_groups = 1, R = 8, W = 4;
  int64_t n_blocks = 1;
  size_t lds = 0;
};
constexpr size_t kLdsMax = 160 * 1024;
template <typename T>
Grid make_grid(int64_t n_rows, int64_t n_trees, int R, int W, int nf, int depth, int max_checks, bool weighted,
               int g_override = 0, int max_row_blocks = 256) {
  const int64_t rows_per_tile = 64 * int64_t(R);
  Grid g;
  g.R = R;
  g.W = W;
  const int64_t n_tiles = (n_rows + rows_per_tile - 1) / rows_per_tile;
  int64_t tiles = (n_tiles + max_row_blocks - 1) / max_row_blocks;  // keep <= max row blocks per tree
  if (tiles < 1) tiles = 1;
  g.tiles = int(tiles);
  g.n_row_blocks = int((n_tiles + tiles - 1) / tiles);
  if (g.n_row_blocks < 1) g.n_row_blocks = 1;
  // more trees per tile amortise the tile's LDS staging and barriers (G 16 -> 128: -29% kernel time
  // on the C2 population); shrink only to keep >= 4096 workgroups for small populations
  int G = 128;
  while (G > 4 && int64_t(g.n_row_blocks) * ((n_trees + G - 1) / G) < 4096) G /= 2;
  if (g_override > 0) G = g_override;
  if (G < W) G = W;  // at least one tree per wave
  if (n_trees > 0 && G > n_trees) G = int(n_trees);
  if (G < 1) G = 1;
  g.G = G;
  g.n_groups = int((n_trees + G - 1) / G);
  g.n_blocks = int64_t(g.n_row_blocks) * g.n_groups;
  g.lds = sr_tile_lds_bytes(int(sizeof(T)), nf, R, depth, G, max_checks, W, weighted);
  return g;
}

template <typename T>
double t_max() {
  return double(SrM<T>::big);
}

struct Lock {
  std::lock_guard<std::mutex> g;
  explicit Lock(sr_ctx* c) : g(c->mu) {}
};

int check_ctx(sr_ctx* ctx) {
  if (!ctx) return set_error(SR_ERR_INVALID_ARG, "NULL context");
  return SR_OK;
}

int validate_common(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!ds || ds->ctx != ctx)
    return set_error(SR_ERR_INVALID_ARG, "dataset is NULL or belongs to another context");
  if (opset_id < 0 || opset_id >= int(ctx->opsets.size()))
    return set_error(SR_ERR_INVALID_ARG, "unknown opset id " + std::to_string(opset_id));
  if (!trees) return set_error(SR_ERR_INVALID_ARG, "NULL tree batch");
  if (trees->n_trees < 0) return set_error(SR_ERR_INVALID_ARG, "negative tree count");
  if (trees->n_trees > (int64_t(1) << 30)) return set_error(SR_ERR_INVALID_ARG, "too many trees in one batch");
  return SR_OK;
}

// loss_kind as passed to the eval calls -> (SrLossKind, parameter).
int decode_loss(sr_ctx* ctx, int code, int* kind, double* param) {
  if (code >= kLossCodeBase) {
    const size_t i = size_t(code - kLossCodeBase);
    if (i >= ctx->losses.size()) return set_error(SR_ERR_INVALID_ARG, "unknown registered loss code " + std::to_string(code));
    *kind = ctx->losses[i].first;
    *param = ctx->losses[i].second;
    return SR_OK;
  }
  if (!loss_direct_ok(code))
    return set_error(SR_ERR_INVALID_ARG, "loss kind " + std::to_string(code) +
                                             " is unknown or needs a parameter: register it with sr_register_loss");
  *kind = code;
  *param = code == SR_LOSS_HUBER ? 1.0 : 0.0;
  return SR_OK;
}

// Shared engine: compile + upload + interpreter(+reduce).  Leaves per-tree {sum, flag} in
// ctx->d_out_sum / ctx->d_out_flag (device).  n_eval rows (full dataset or row_idx view).
//
// Large LOSS batches are pipelined in up to kMaxChunks tree chunks: the host compiles chunk c+1
// while the device runs chunk c (programs staged through pinned memory, async DMA).  Every chunk is
// an independent launch over its own slice of the per-tree device arrays; `prog` receives the merged
// per-tree summary (offsets into the device code buffer, static_bad, max_depth, max_checks) that
// the exact-sum pass and the callers use — its `code` stays empty.
// Derived columns of a LOSS call: the unary(feature) nodes of the batch's transcendental operators
// (exp / cos / sin / safe_log / safe_sqrt) that at least kDerivedMinUses trees of a sample share,
// most used first, at most SR_MAX_DERIVED.  dmap: [SR_U_COUNT][nf] -> column or -1.
constexpr int64_t kDerivedMinRows = 16384;  // below this the per-call column pass does not pay
constexpr int kDerivedMinUses = 4;
constexpr double kDerivedMinWork = 33554432.0;  // trees x rows (2^25) below which the column pass does not pay
constexpr int64_t kDerivedSample = 1024;    // trees scanned
void choose_derived(const sr_tree_batch& trees, const SrOpset& ops, int64_t nf, SrDerivedSpec* spec,
                    std::vector<int16_t>* dmap) {
  spec->n = 0;
  dmap->assign(size_t(SR_U_COUNT) * size_t(nf), int16_t(-1));
  auto eligible = [](uint32_t u) {
    return u == SR_U_EXP || u == SR_U_COS || u == SR_U_SIN || u == SR_U_LOG || u == SR_U_SQRT;
  };
  std::vector<int32_t> uses(size_t(SR_U_COUNT) * size_t(nf), 0);
  const int64_t ns = trees.n_trees < kDerivedSample ? trees.n_trees : kDerivedSample;
  for (int64_t k = 0; k < ns; ++k) {
    const int64_t b = trees.offsets[k], e = trees.offsets[k + 1];
    // pre-order: node i (degree 1) has its child at i + 1
    for (int64_t i = b; i + 1 < e; ++i) {
      if (trees.degree[i] != 1 || trees.degree[i + 1] != 0 || trees.constant[i + 1]) continue;
      const int oi = int(trees.op[i]) - 1;
      const int f = int(trees.feature[i + 1]) - 1;
      if (oi < 0 || oi >= int(ops.unary.size()) || f < 0 || f >= nf) continue;
      const uint32_t u = ops.unary[size_t(oi)];
      if (eligible(u)) ++uses[size_t(u) * size_t(nf) + size_t(f)];
    }
  }
  std::vector<std::pair<int32_t, size_t>> cand;
  for (size_t q = 0; q < uses.size(); ++q)
    if (uses[q] >= kDerivedMinUses) cand.push_back({uses[q], q});
  std::stable_sort(cand.begin(), cand.end(), [](const auto& x, const auto& y) { return x.first > y.first; });
  for (const auto& c : cand) {
    if (spec->n >= SR_MAX_DERIVED) break;
    const int k = spec->n++;
    spec->op[k] = uint8_t(c.second / size_t(nf));
    spec->feat[k] = uint16_t(c.second % size_t(nf));
    (*dmap)[c.second] = int16_t(k);
  }
}

// Row-sharded calls decide data-dependent launch choices from the statistics of ALL shards, so every
// rank compiles identical programs (same derived columns: the exact path numbers checked arrays the
// same on every rank): max|X| over every shard and the smallest shard's row count.
struct ShardCtl {
  double max_abs_x;
  int64_t min_rows;
};

// Several row views in one LOSS call (sr_eval_loss_batch_views): tree t is scored on the rows
// view_rows[tree_view[t] * view_len ...] (the caller's row_idx array holds n_views views of view_len rows).
struct ViewSpec {
  const int32_t* tree_view;
  int n_views;
  int64_t view_len;
};

// Rows of the reference's loss fold for the overflow rule (sr_fold.h), or 0 when the rule does not
// apply (negative weights: the fold is not monotone).
inline int64_t fold_terms(const sr_dataset* ds, int64_t n_rows) { return (ds->w && ds->w_min < 0.0) ? 0 : n_rows; }

// ---------------------------------------------------------------- every complete tree's in-order fold
// One loss launch of a call whose trees the in-order fold covers (sr_ctx::ref_fold): its arguments (the
// FOLD pass re-launches them), launch positions [pos0, pos0 + np) of the call (chunk t0: perm values and
// per-tree arrays are chunk-local), grid and kernel build.
template <typename T>
struct FoldRegion {
  SrEvalArgs<T> a;
  int64_t t0, pos0, np, n_blocks;
  int Rc;
  bool vstk;
  Grid g;
};
// A call's fold: its regions and the launch facts every fold kernel needs (kept by a row-sharded call's
// run_batch until the ranks have agreed on the verdicts: FoldJob::deferred).
template <typename T>
struct FoldJob {
  std::vector<FoldRegion<T>> regions;
  int path = 0;  // 1 stored losses, 2 FOLD pass
  int tier = 0;
  bool gather = false;
  int64_t n_eval = 0, n_rb = 0, slot_rows = 0, n_terms = 0;
  int slot_cap = 0;
  double delta = 0.0;
  bool fuse_reduce = false;  // (stored losses, one GPU: the pair kernel does the call's reduce)
};

// a region's plan arrays at partial-buffer offset off
template <typename T>
SrFoldTabs fold_tabs(sr_ctx* ctx, size_t off) {
  using Pair = typename SrFoldTab<T>::Pair;
  return SrFoldTabs{ctx->fold_code.as<int32_t>() + off, ctx->fold_tab.as<char>() + off * sizeof(Pair),
                    ctx->fold_sq.as<int32_t>() + off, ctx->fold_tab2.as<char>() + off * sizeof(Pair)};
}
// A stored-loss call of one row block of at most 256 rows that starts the fold (C1's 100-row calls): the
// walk's serial start folds every row and takes eligibility from the call's flags itself, so the pair
// kernel's launch is skipped (round 6: ~5 us of a ~45 us call)
template <typename T>
bool fold_tiny(const FoldJob<T>& job, const FoldRegion<T>& fr, const SrFoldWho& who) {
  return job.path == 1 && fr.g.n_row_blocks == 1 && job.n_eval <= 256 && who.first && who.elig == nullptr &&
         who.est == nullptr;
}
// A region's steps: the stored-loss tables (path 1) or the plan and the FOLD pass (path 2).  who: the
// call's whole-batch arrays (sums / flags / elig / est at the caller's tree index; this function adds
// the region's chunk offset).
template <typename T>
int fold_steps(sr_ctx* ctx, const FoldJob<T>& job, const FoldRegion<T>& fr, SrFoldWho who, hipStream_t cs) {
  const int nrb = fr.g.n_row_blocks;
  const int64_t rb_rows = int64_t(fr.g.tiles) * 64 * fr.Rc;
  const size_t off = size_t(job.n_rb) * size_t(fr.pos0);  // (the region's offset in the partial buffers)
  const SrFoldTabs ft = fold_tabs<T>(ctx, off);
  const double* part = nrb > 1 ? fr.a.part_sum : nullptr;
  const int np = int(fr.np);
  if (who.sums) who.sums += fr.t0;
  if (who.flags) who.flags += fr.t0;
  if (who.elig) who.elig += fr.t0;
  if (who.est) who.est += fr.t0;
  if (job.path == 1) {
    if (fold_tiny(job, fr, who)) return SR_OK;  // (the walk's serial start is the whole fold: no pairs)
    const bool fr_red = job.fuse_reduce && nrb > 1;
    SR_HIP_CHECK(sr_launch_fold_stab<T>(part, np, nrb, rb_rows, job.n_eval, fr.a.perm, who, job.delta, fr.a.fold_loss,
                                        ft, fr_red ? fr.a.part_flag : nullptr, fr_red ? ctx->d_bad + fr.t0 : nullptr,
                                        fr_red ? ctx->d_out_sum + fr.t0 : nullptr,
                                        fr_red ? ctx->d_out_flag + fr.t0 : nullptr, cs));
    return SR_OK;
  }
  SR_HIP_CHECK(sr_launch_fold_plan<T>(part, np, nrb, fr.a.perm, who, job.delta, ft, ctx->fold_ctl.as<int>(),
                                      job.slot_cap, cs));
  SrEvalArgs<T> fa = fr.a;
  fa.hint = nullptr;
  fa.out_sum = nullptr;
  fa.out_flag = nullptr;
  fa.group_cnt = nullptr;
  fa.stamps = nullptr;
  fa.fold_code = ft.code;
  fa.fold_tab = ft.tab;
  fa.fold_sq = ft.sq;
  fa.fold_tab2 = ft.tab2;
  fa.fold_loss = ctx->fold_store.as<T>();
  fa.fold_slot_rows = job.slot_rows;
  fa.fold_pos_stride = 0;
  SR_HIP_CHECK(sr_launch_eval<T>(fa, SR_MODE_FOLD, job.gather, job.tier, fr.Rc, fr.g.W, fr.vstk, int(fr.n_blocks), cs));
  return SR_OK;
}
// A region's walk: the folds' values and status at the caller's tree index (out arrays and carry are
// whole-batch, tree-indexed).
template <typename T>
int fold_walk(sr_ctx* ctx, const FoldJob<T>& job, const FoldRegion<T>& fr, SrFoldWho who, const T* carry, T* out_val,
              int32_t* out_st, hipStream_t cs) {
  const int nrb = fr.g.n_row_blocks;
  const int tiny = carry == nullptr && fold_tiny(job, fr, who) ? 16 : 0;
  // (stored losses, the pair kernel launched, the fold starting here: it did the serial start)
  const int pre = job.path == 1 && !tiny && carry == nullptr && who.first && ctx->fold_pre_start ? 32 : 0;
  if (who.sums) who.sums += fr.t0;
  if (who.flags) who.flags += fr.t0;
  if (who.elig) who.elig += fr.t0;
  if (who.est) who.est += fr.t0;
  if (who.msum) who.msum += fr.t0;
  if (who.mflag) who.mflag += fr.t0;
  const int64_t rb_rows = int64_t(fr.g.tiles) * 64 * fr.Rc;
  const size_t off = size_t(job.n_rb) * size_t(fr.pos0);
  const SrFoldTabs ft = fold_tabs<T>(ctx, off);
  const T* losses = job.path == 1 ? fr.a.fold_loss : ctx->fold_store.as<T>();
  const int64_t slot_rows = job.path == 1 ? rb_rows : job.slot_rows;
  int4* dbg = ctx->fold_stats ? ctx->fold_dbg.as<int4>() + fr.t0 : nullptr;  // (SR_AMD_FOLD_STATS)
  SR_HIP_CHECK(sr_launch_fold_walk<T>(ft, who, int(fr.np), nrb, rb_rows, job.n_eval, losses, slot_rows, fr.a.perm,
                                      carry ? carry + fr.t0 : nullptr, out_val + fr.t0, out_st + fr.t0, dbg,
                                      int(job.path == 1) | tiny | pre | ctx->fold_walk_dbg, cs));
  if (ctx->fold_stats == 2)  // (analysis: the same walk again, its loads now warm: the statistics are the second's)
    SR_HIP_CHECK(sr_launch_fold_walk<T>(ft, who, int(fr.np), nrb, rb_rows, job.n_eval, losses, slot_rows, fr.a.perm,
                                        carry ? carry + fr.t0 : nullptr, out_val + fr.t0, out_st + fr.t0, dbg,
                                        int(job.path == 1) | tiny | pre | ctx->fold_walk_dbg, cs));
  return SR_OK;
}

template <typename T>
int run_batch(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees, const int64_t* row_idx,
              int64_t n_idx, int64_t n_total, int loss_kind, int mode, SrProgramBatch<T>* prog, Grid* grid_out,
              bool allow_derived = false, const ShardCtl* shard = nullptr, const ViewSpec* views = nullptr) {
  const bool gather = row_idx != nullptr && n_idx > 0;
  // PRED passes (the fold's few band trees) write no partials: more row blocks fill the GPU (C4's 14 trees
  // x 2^26 rows ran 1,024 workgroups at 256)
  int mrb = mode == SR_MODE_PRED ? std::max(ctx->max_row_blocks, 4096) : ctx->max_row_blocks;
  const int64_t n_eval = gather ? n_idx : ds->n;
  if (n_eval <= 0) return set_error(SR_ERR_INVALID_ARG, "no rows to evaluate");
  // under the in-order fold, row blocks of at most fold_seg_max rows on the largest shard (every rank
  // the same count): a slow block's rows are kept whole (C4's 2^26 rows per GPU: 4,096 blocks of 16k)
  if (mode == SR_MODE_LOSS && ctx->want_fold && ctx->ref_fold && sizeof(T) == 4 && ctx->fold_seg_max > 0 &&
      (shard ? n_total : n_eval) <= ctx->fold_rows_max) {
    int64_t max_rows = n_eval;
    if (shard)
      for (size_t r = 0; r + 1 < ds->shard_offs.size(); ++r) max_rows = std::max(max_rows, ds->shard_offs[r + 1] - ds->shard_offs[r]);
    const int64_t need = (max_rows + ctx->fold_seg_max - 1) / ctx->fold_seg_max;
    if (need > mrb) mrb = int(std::min<int64_t>(need, 16384));
  }
  // several views: one launch, its tree groups view-pure (SrSegment); rows uploaded for every view
  const bool multi = views != nullptr && gather && mode == SR_MODE_LOSS;
  const int64_t n_rows_up = multi ? int64_t(views->n_views) * n_idx : n_idx;
  if (multi) allow_derived = false;
  int lkind = 0;
  double lparam = 0.0;
  if (decode_loss(ctx, loss_kind, &lkind, &lparam) != SR_OK) return SR_ERR_INVALID_ARG;
  const int64_t nt = trees->n_trees;
  if (nt < 0) return set_error(SR_ERR_INVALID_ARG, "negative tree count");
  if (nt > 0 && !trees->offsets) return set_error(SR_ERR_INVALID_ARG, "sr_tree_batch has NULL arrays");
  const int64_t total_nodes = nt > 0 ? trees->offsets[nt] - trees->offsets[0] : 0;
  if (total_nodes < 0 || total_nodes > int64_t(0xffffffffu) / 2)
    return set_error(SR_ERR_INVALID_ARG, "tree batch node count out of range");
  // (SR_TRACK_LITE: the deferred-check kernels bound untracked values by L x max|x| for trees of up to
  //  L nodes; data at or above tbig / L — huge or non-finite values, never seen in practice — runs the
  //  per-node-check kernels instead, whose checks hold for any data)
  int tier = ctx->tiers[opset_id];
#ifdef SR_TRACK_LITE
  if (tier == SR_TIER_BASIC && mode == SR_MODE_LOSS && nt > 0) {
    int64_t lmax = 1;
    for (int64_t t = 0; t < nt; ++t) lmax = std::max<int64_t>(lmax, trees->offsets[t + 1] - trees->offsets[t]);
    const double mx = shard ? shard->max_abs_x : ds->max_abs_x;
    if (!(mx < double(T(t_max<T>() / (2.0 * double(n_total > 0 ? n_total : 1)))) / double(lmax))) tier = SR_TIER_FULL;
  }
#endif
  const int R = sr_rows_per_lane<T>(mode, tier, ctx->rows_override);
  const int W = sr_waves_per_block(int(sizeof(T)), mode, tier, R, ctx->waves_override);
  // register-stack kernel (f32 BASIC loss over the full dataset): Rv rows per lane, used for every
  // chunk whose programs need <= 2 operand-stack slots (all trees of <= 30 nodes); other chunks run
  // the LDS-stack kernel at R rows per lane
  int Rv = (mode == SR_MODE_LOSS && tier == SR_TIER_BASIC && !gather)
               ? sr_vstk_rows(int(sizeof(T)), n_eval, ctx->vstk_rows ? ctx->vstk_rows : ctx->rows_override)
               : 0;
  // a wide dataset whose register-stack tile (its rows per lane are twice the classic kernel's) would
  // not fit the LDS runs the classic kernel instead (Float64 with ~40-75 features)
  if (Rv > 0 && make_grid<T>(n_eval, nt > 0 ? nt : 1, Rv, W, int(ds->nf), 0, 0, ds->w != nullptr, ctx->tree_group,
                             mrb).lds > kLdsMax)
    Rv = 0;
  ctx->rows_last = Rv > 0 ? Rv : R;  // (every C2-like tree fits the register stack)
  hipStream_t s = ctx->stream;
  // error exits while chunks are in flight: no DMA may still read the staging buffers
  auto sync_both = [&] {
    (void)hipStreamSynchronize(s);
    if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
  };

  // chunking (SR_AMD_CHUNKS, default 2; LOSS mode only — PRED writes rows by caller tree index).
  // Default: a first chunk of 1/6 of the trees runs while the host compiles the rest (exposed compile
  // 0.72 -> 0.27 ms on C2, every test population's step faster).  k > 2 equal chunks (>= 2048 trees
  // each) alternate over the two streams; they cost kernel time on complete-heavy populations.
  constexpr int64_t kChunkTrees = 2048;
  int n_chunks = 1;
  if (multi) {
    // (one chunk: the segments cover the whole launch)
  } else if (mode == SR_MODE_LOSS && ctx->chunks == 2) {
    n_chunks = nt / ctx->first_chunk >= ctx->chunk_min ? 2 : 1;  // the small first chunk holds >= chunk_min trees
  } else if (mode == SR_MODE_LOSS && ctx->chunks > 2) {
    const int64_t k = nt / kChunkTrees;
    const int64_t cap = ctx->chunks < kMaxChunks ? ctx->chunks : kMaxChunks;
    n_chunks = int(k < 1 ? 1 : (k > cap ? cap : k));
  }

  // device + pinned buffers sized for the whole batch up front (a chunk's kernel may still run while
  // the next one is staged): a program has at most one instruction per node
  Grid g0 = make_grid<T>(n_eval, nt > 0 ? nt : 1, R, W, int(ds->nf), 1, 0, ds->w != nullptr, ctx->tree_group,
                         mrb);
  int n_rb = g0.n_row_blocks;  // row blocks the partial buffers hold per tree (the most any kernel uses)
  if (Rv > 0)
    n_rb = std::max(n_rb, make_grid<T>(n_eval, nt > 0 ? nt : 1, Rv, W, int(ds->nf), 0, 0, ds->w != nullptr,
                                       ctx->tree_group, mrb).n_row_blocks);
  const size_t code_cap = size_t(total_nodes) + 16;
  auto align256 = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t o_off = align256(code_cap * sizeof(SrIns<T>));
  const size_t o_bad = align256(o_off + (size_t(nt) + 1) * sizeof(uint32_t));
  const size_t o_perm = align256(o_bad + size_t(nt) + 16);
  const size_t o_end = align256(o_perm + (size_t(nt) + 1) * sizeof(uint32_t));
  const size_t o_seg = align256(o_end + (size_t(nt) + 1) * sizeof(uint32_t));
  const size_t n_seg_cap = multi ? size_t(views->n_views) : 0;
  const size_t prog_bytes = o_seg + n_seg_cap * sizeof(SrSegment);
  SR_HIP_CHECK(ctx->prog.ensure(prog_bytes));
  SR_HIP_CHECK(ctx->h_prog.ensure(prog_bytes, s, ctx->stream2));
  char* const dprog = ctx->prog.as<char>();
  ctx->d_code = dprog;
  ctx->d_off = reinterpret_cast<uint32_t*>(dprog + o_off);
  ctx->d_bad = reinterpret_cast<uint8_t*>(dprog + o_bad);
  ctx->d_perm = reinterpret_cast<uint32_t*>(dprog + o_perm);
  ctx->d_end = reinterpret_cast<uint32_t*>(dprog + o_end);
  const size_t n_part = size_t(nt) * size_t(n_rb);
  SR_HIP_CHECK(ctx->part_sum.ensure(n_part * sizeof(double) + 8));
  SR_HIP_CHECK(ctx->part_flag.ensure(n_part * sizeof(uint32_t) + 4));
  if (mode == SR_MODE_LOSS && ctx->fused_reduce > 0 && size_t(nt) * sizeof(uint32_t) + 4 > ctx->group_cnt.cap) {
    SR_HIP_CHECK(hipStreamSynchronize(s));  // (the second stream runs only inside a call)
    SR_HIP_CHECK(ctx->group_cnt.ensure(size_t(nt) * sizeof(uint32_t) + 4));
    SR_HIP_CHECK(hipMemset(ctx->group_cnt.p, 0, ctx->group_cnt.cap));
  }
  // the reference's in-order loss fold of every complete tree (sr_ctx::ref_fold): 1 = the loss launch
  // stores every tree's losses (they fit fold_store_mb), 2 = the FOLD-mode pass over the complete trees
  // (a row-sharded call: the global rows and every shard's weights; its ranks fold or not together —
  //  the choice below depends on the largest shard's rows, known to every rank)
  const int64_t fold_n_terms = shard ? ((ds->w && ds->shard_w_min < 0.0) ? 0 : n_total) : fold_terms(ds, n_eval);
  int fold_path = 0;
  int64_t fold_slot_rows = 0;
  if (shard) ctx->fold_job.reset();
  if (ctx->want_fold && ctx->ref_fold && mode == SR_MODE_LOSS && nt > 0 && fold_n_terms > 0) {
    // rows a position's store covers under either kernel's grid (row blocks x rows: >= the view)
    auto cover = [&](int Rc, int depth_c, int64_t* rb_rows) {
      const Grid gg = make_grid<T>(n_eval, nt, Rc, W, int(ds->nf), depth_c, 0, ds->w != nullptr, ctx->tree_group, mrb);
      *rb_rows = int64_t(gg.tiles) * 64 * Rc;
      return int64_t(gg.n_row_blocks) * *rb_rows;
    };
    int64_t rbr = 0, rbv = 0;
    int64_t pos_rows = cover(R, 1, &rbr);
    if (Rv > 0) pos_rows = std::max(pos_rows, cover(Rv, 0, &rbv));
    fold_slot_rows = std::max(rbr, rbv);
    const bool fold_mode_builds = tier == SR_TIER_BASIC ? (R == 8 && (Rv == 0 || Rv == 16)) : R == 4;
    int64_t max_shard = n_eval;
    if (shard)
      for (size_t r = 0; r + 1 < ds->shard_offs.size(); ++r) max_shard = std::max(max_shard, ds->shard_offs[r + 1] - ds->shard_offs[r]);
    // Float64: only with stored losses (no FOLD build), decided on the largest shard so every rank agrees
    const bool f64_off = sizeof(T) == 8 && double(nt) * double(pos_rows) * double(max_shard) / double(n_eval) *
                                               double(sizeof(T)) > double(ctx->fold_store_mb) * 1048576.0;
    // segments (row blocks) past fold_seg_max rows on the largest shard: no fold (a slow segment's rows
    // are kept whole).  The launch above already takes enough row blocks for fold_seg_max (up to 16,384
    // blocks); decided on that grid whatever max_row_blocks says, so the knob never changes a result.
    int64_t rb_big = 0;
    {
      const Grid gb = make_grid<T>(max_shard, nt, R, W, int(ds->nf), 1, 0, ds->w != nullptr, ctx->tree_group,
                                   std::max<int64_t>(512, (max_shard + ctx->fold_seg_max - 1) / std::max<int64_t>(1, ctx->fold_seg_max)));
      rb_big = int64_t(gb.tiles) * 64 * R;
    }
    // folds longer than fold_rows_max (2^24) keep the f64 sum: past ~2^23 rows the reference's Float32
    // fold stalls (a loss below half an ulp of the running sum adds nothing; C4's 2^26 rows: up to 50 %
    // below the exact mean) and drifts out of every window the f64 prefix gives the plan, so the walks
    // fail and the fallback's prediction pass takes the call (C4 folded: 26.6k trees, 37.7 s a step)
    const int64_t fold_len = shard ? n_total : n_eval;
    if (f64_off || rb_big > ctx->fold_seg_max || fold_len > ctx->fold_rows_max) {
    } else if (double(nt) * double(pos_rows) * double(sizeof(T)) <= double(ctx->fold_store_mb) * 1048576.0) {
      fold_path = 1;
      SR_HIP_CHECK(ctx->fold_store.ensure(size_t(nt) * size_t(pos_rows) * sizeof(T)));
    } else if (sizeof(T) == 4 && fold_mode_builds) {
      fold_path = 2;
      // (slots for ~24 slow segments per tree — C2 averages 10 — up to fold_slot_mb)
      const int64_t slots = std::max<int64_t>(1, std::min<int64_t>(int64_t(nt) * 24, ctx->fold_slot_mb * 1048576 /
                                                                                     (fold_slot_rows * int64_t(sizeof(T)))));
      SR_HIP_CHECK(ctx->fold_store.ensure(size_t(slots) * size_t(fold_slot_rows) * sizeof(T)));
      SR_HIP_CHECK(ctx->fold_ctl.ensure(64));
      SR_HIP_CHECK(hipMemsetAsync(ctx->fold_ctl.p, 0, sizeof(int), s));  // the call's slot counter
    }
    if (fold_path && ctx->fold_stats) {
      SR_HIP_CHECK(ctx->fold_dbg.ensure(size_t(nt) * sizeof(int4) + 16));
      SR_HIP_CHECK(hipMemsetAsync(ctx->fold_dbg.p, 0, size_t(nt) * sizeof(int4), s));
    }
    if (fold_path) {
      SR_HIP_CHECK(ctx->fold_code.ensure(n_part * sizeof(int32_t) + 4));
      SR_HIP_CHECK(ctx->fold_tab.ensure(n_part * sizeof(typename SrFoldTab<T>::Pair) + 16));
      SR_HIP_CHECK(ctx->fold_sq.ensure(n_part * sizeof(int32_t) + 4));
      SR_HIP_CHECK(ctx->fold_tab2.ensure(n_part * sizeof(typename SrFoldTab<T>::Pair) + 16));
    }
  }
  if (!ctx->internal_pass) {  // (the fallback's prediction passes leave the call's record alone)
    ctx->fold_path_last = fold_path;
    ctx->fold_timed_last = false;
  }
  // {Σ loss | flags | the fold's values | their status}, one allocation (one DMA back)
  ctx->outs_flag_off = align256(size_t(nt) * sizeof(double) + 8);
  ctx->outs_fval_off = align256(ctx->outs_flag_off + size_t(nt) * sizeof(uint32_t) + 4);
  ctx->outs_fst_off = align256(ctx->outs_fval_off + size_t(nt) * sizeof(T) + 8);
  const size_t outs_bytes = ctx->outs_fst_off + size_t(nt) * sizeof(int32_t) + 4;
  ctx->outs_bytes_all = outs_bytes;
  SR_HIP_CHECK(ctx->outs.ensure(outs_bytes));
  // latency path (see host_io): results written to pinned host memory, programs read from it
  const bool small_call = n_chunks == 1 && mode == SR_MODE_LOSS;
  // (under the in-order fold the plan reads the call's flags and partials on the device; a stored-loss
  // fold of one row block of <= 256 rows — fold_tiny, the walk alone — reads and writes pinned memory)
  const bool fold_small = fold_path == 1 && n_rb == 1 && n_eval <= 256;
  const bool host_out = small_call && ctx->host_io >= 1 && ctx->want_host_out && (fold_path == 0 || fold_small);
  // (other stored-loss folds of a small call: Σ and flags stay on the device for the pair kernel, and the
  //  walk copies them to pinned memory beside the fold's values — no copy back, SrFoldWho::msum)
  const bool fold_mirror = small_call && ctx->host_io >= 1 && ctx->want_host_out && fold_path == 1 && !fold_small &&
                           !shard;
  if (host_out || fold_mirror) SR_HIP_CHECK(ctx->h_outs.ensure(outs_bytes, s, ctx->stream2));
  ctx->outs_on_host = host_out || fold_mirror;
  const bool host_red = host_out && ctx->host_reduce > 0 && !multi && n_rb > 1 && int64_t(n_part) <= ctx->host_reduce;
  ctx->host_reductions.clear();
  ctx->host_red_rb = n_rb;
  if (host_red) SR_HIP_CHECK(ctx->h_part.ensure(n_part * (sizeof(double) + sizeof(uint32_t)) + 16, s, ctx->stream2));
  ctx->d_out_sum = reinterpret_cast<double*>(host_out ? ctx->h_outs.as<char>() : ctx->outs.as<char>());
  ctx->d_out_flag = reinterpret_cast<uint32_t*>((host_out ? ctx->h_outs.as<char>() : ctx->outs.as<char>()) +
                                                ctx->outs_flag_off);
  if (mode == SR_MODE_PRED) SR_HIP_CHECK(ctx->pred.ensure(size_t(nt) * size_t(n_eval) * sizeof(T) + 16));
  const bool use_hint = ctx->dead_hints && mode == SR_MODE_LOSS && n_rb > 1;  // (hints are per position)
  if (use_hint) {
    // epoch-tagged hints: each call marks dead positions with its own epoch, so the array needs a
    // reset only when (re)allocated or when the epoch counter wraps
    // (a reallocation is detected by the capacity, not the address: the allocator may hand back the
    // freed address for the larger buffer, whose new part then holds stale words — possibly equal to
    // this call's epoch, which would mark live trees dead)
    const size_t cap_before = ctx->hint.cap;
    const size_t hint_bytes = size_t(nt) * sizeof(uint32_t) + 4;
    if (ctx->debug_hint_regrow && hint_bytes > ctx->hint.cap) {
      // (tests: sr_set_tuning "debug_hint_regrow") the array grows IN PLACE, at the same address, its
      // new words holding the epoch the next call would use without a reset — the conditions of the
      // round-3 stale-hint bug (a reallocation that got the freed address back); only the capacity
      // check below catches it
      constexpr size_t kReserve = size_t(64) << 20;
      if (hint_bytes + hint_bytes / 4 > kReserve) return set_error(SR_ERR_INVALID_ARG, "debug_hint_regrow: batch too large");
      if (ctx->hint_reserve == nullptr) SR_HIP_CHECK(hipMalloc(&ctx->hint_reserve, kReserve));
      if (ctx->hint.p != ctx->hint_reserve) {
        ctx->hint.release();
        ctx->hint.p = ctx->hint_reserve;
      }
      // (word-aligned: an earlier ordinary allocation may have left an odd capacity)
      const size_t from = (cap_before + 3) & ~size_t(3);
      const size_t want = (hint_bytes + hint_bytes / 4 + 255) & ~size_t(255);
      SR_HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(static_cast<char*>(ctx->hint.p) + from),
                                     int(ctx->hint_epoch + 1), (want - from) / 4, s));
      ctx->hint.cap = want;
    } else {
      if (ctx->hint.p == ctx->hint_reserve && ctx->hint_reserve != nullptr) {  // (leaving the debug mode)
        ctx->hint.p = nullptr;
        ctx->hint.cap = 0;
      }
      SR_HIP_CHECK(ctx->hint.ensure(hint_bytes));
    }
    if (ctx->hint.cap != cap_before || ctx->hint_epoch == 0xffffffffu) {
      SR_HIP_CHECK(hipMemsetAsync(ctx->hint.p, 0, ctx->hint.cap, s));
      ctx->hint_epoch = 0;
    }
    ++ctx->hint_epoch;
  }
  // dead-tree probe: the first kProbeTiles row tiles of the view, hints only (scratch partials)
  const bool use_probe = use_hint && ctx->probe && n_rb >= 16 && !multi;  // (per chunk: its grid has >= 16 row blocks)
  if (use_probe) {
    SR_HIP_CHECK(ctx->probe_sum.ensure(size_t(nt) * kProbeTiles * sizeof(double) + 8));
    SR_HIP_CHECK(ctx->probe_flag.ensure(size_t(nt) * kProbeTiles * sizeof(uint32_t) + 4));
  }
  if (gather) {
    for (int64_t i = 0; i < n_rows_up; ++i)
      if (row_idx[i] < 0 || row_idx[i] >= ds->n)
        return set_error(SR_ERR_INVALID_ARG, "row index " + std::to_string(row_idx[i]) + " out of range");
    SR_HIP_CHECK(ctx->row_idx.ensure(size_t(n_rows_up) * sizeof(int64_t)));
  }
  if (multi)
    for (int64_t t = 0; t < nt; ++t)
      if (views->tree_view[t] < 0 || views->tree_view[t] >= views->n_views)
        return set_error(SR_ERR_INVALID_ARG, "tree " + std::to_string(t) + ": view index out of range");

  prog->code.clear();
  prog->offsets.assign(size_t(nt) + 1, 0);
  prog->static_bad.assign(size_t(nt), 0);
  prog->n_checks.assign(size_t(nt), 0);
  prog->max_depth = 0;
  prog->tier = tier;
  prog->max_checks = 0;
  prog->total_nodes = 0;
  prog->total_ops = 0;
  char* const hprog = ctx->h_prog.as<char>();
  SrIns<T>* h_code = reinterpret_cast<SrIns<T>*>(hprog);
  uint32_t* h_off = reinterpret_cast<uint32_t*>(hprog + o_off);
  uint8_t* h_bad = reinterpret_cast<uint8_t*>(hprog + o_bad);
  uint32_t* h_perm = reinterpret_cast<uint32_t*>(hprog + o_perm);
  ctx->h_bad_last = h_bad;
  ctx->h_perm_last = h_perm;
  uint32_t* h_end = reinterpret_cast<uint32_t*>(hprog + o_end);
  ctx->n_chunks_last = 0;
  ctx->derived_last = false;
  ctx->n_derived_last = 0;
  ctx->timed_last = ctx->timing != 0;
  if (ctx->timed_last) SR_HIP_CHECK(hipEventRecord(ctx->ev_start, s));
  if (gather)
    SR_HIP_CHECK(hipMemcpyAsync(ctx->row_idx.p, row_idx, size_t(n_rows_up) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  // derived columns (LOAD_DERIVED): for the BASIC-tier deferred-check loss kernels over many rows,
  // every unary(feature) node of a transcendental shared by several trees is evaluated once for the
  // call.  Chosen from a sample of the batch; not when the data itself needs tracked feature loads.
  std::vector<int16_t> dmap;
  SrDerivedSpec spec{};
  const int64_t dld = (n_eval + kRowAlign - 1) / kRowAlign * kRowAlign;
  // (row-sharded calls pass `shard`: the choice then depends only on the trees and on statistics of
  // every shard, so all ranks compile the same programs and number their checked arrays alike)
  const double max_abs_x = shard ? shard->max_abs_x : ds->max_abs_x;
  const int64_t derived_rows = shard ? shard->min_rows : n_eval;
  // (and only for calls with enough work: the column pass is one more launch, which a search's small
  // calls — tens of trees x 1e5 rows — would pay in latency for nothing)
  if (allow_derived && ctx->derived && mode == SR_MODE_LOSS && tier == SR_TIER_BASIC && derived_rows >= kDerivedMinRows &&
      nt >= 64 && double(nt) * double(derived_rows) >= kDerivedMinWork &&
      max_abs_x < double(T(t_max<T>() / (2.0 * double(n_total > 0 ? n_total : 1))))) {  // (track_x off)
    choose_derived(*trees, ctx->opsets[opset_id], ds->nf, &spec, &dmap);
    if (spec.n > 0) {
      SR_HIP_CHECK(ctx->derived_cols.ensure(size_t(spec.n) * size_t(dld) * sizeof(T)));
      if (ctx->timed_last) SR_HIP_CHECK(hipEventRecord(ctx->ev_d0, s));
      SR_HIP_CHECK(sr_launch_derived<T>(static_cast<const T*>(ds->X), ds->ld, gather ? ctx->row_idx.as<int64_t>() : nullptr,
                                        n_eval, dld, spec, ctx->derived_cols.as<T>(), dld, s));
      if (ctx->timed_last) SR_HIP_CHECK(hipEventRecord(ctx->ev_d1, s));
      ctx->derived_last = true;
      ctx->n_derived_last = spec.n;
    } else {
      dmap.clear();
    }
  }
  // the probe over the dataset's stress rows (full views only: a gathered view's rows are its own);
  // its LOAD_DERIVED nodes read columns computed over those rows
  const bool stress_probe = use_probe && !gather && ds->probe_rows != nullptr && ctx->stress_probe;
  if (stress_probe && !dmap.empty()) {
    SR_HIP_CHECK(ctx->probe_derived.ensure(size_t(spec.n) * size_t(kProbeRows) * sizeof(T)));
    SR_HIP_CHECK(sr_launch_derived<T>(static_cast<const T*>(ds->X), ds->ld, static_cast<const int64_t*>(ds->probe_rows),
                                      ds->n_probe, kProbeRows, spec, ctx->probe_derived.as<T>(), kProbeRows, s));
  }
  if (n_chunks > 1) {  // odd chunks run on the second stream, after the shared setup above
    SR_HIP_CHECK(ctx->need_stream2());
    SR_HIP_CHECK(hipEventRecord(ctx->ev_join, s));
    SR_HIP_CHECK(hipStreamWaitEvent(ctx->stream2, ctx->ev_join, 0));
  }

  // the fold's launches per chunk: every launch of the chunk, then its plan / tables / FOLD pass / walk
  FoldJob<T> fjob;  // (the regions of the chunk being launched; a row-sharded call's: all of them, kept)
  fjob.path = fold_path;
  fjob.tier = tier;
  fjob.gather = gather;
  fjob.n_eval = n_eval;
  fjob.n_rb = n_rb;
  fjob.slot_rows = fold_slot_rows;
  fjob.n_terms = fold_n_terms;
  fjob.delta = std::ldexp(1.0, -ctx->fold_delta_log2);
  // stored losses on one GPU: the pair kernel reduces the partials itself (one launch fewer a call;
  // SR_AMD_FOLD_REDUCE=0: the reduce launch)
  fjob.fuse_reduce = fold_path == 1 && !shard && mode == SR_MODE_LOSS && ctx->fold_reduce;
  fjob.slot_cap = fold_path == 2 ? int(std::min<int64_t>(INT_MAX / 2, int64_t(ctx->fold_store.cap /
                                                                             (size_t(fold_slot_rows) * sizeof(T)))))
                                 : 0;
  size_t fold_store_at = 0;  // (stored losses: the regions one after another, [position][n_rb x rb rows])
  char* const outs_base = (host_out || fold_mirror) ? ctx->h_outs.as<char>() : ctx->outs.as<char>();
  T* const d_fval = reinterpret_cast<T*>(outs_base + ctx->outs_fval_off);
  int32_t* const d_fst = reinterpret_cast<int32_t*>(outs_base + ctx->outs_fst_off);
  uint32_t code_base = 0;
  static const bool phase_debug = std::getenv("SR_AMD_PHASE_DEBUG") != nullptr;  // (latency analysis)
  const auto t_pre = std::chrono::steady_clock::now();
  Grid glast = g0;
  std::string err;
  for (int c = 0; c < n_chunks && nt > 0; ++c) {
    // two chunks: a small first one (1/6) runs while the host compiles the rest, so the exposed
    // compile time is the small chunk's; more chunks: equal pieces
    auto bound = [&](int k) -> int64_t {
      if (k <= 0) return 0;
      if (k >= n_chunks) return nt;
      return n_chunks == 2 ? nt / ctx->first_chunk : nt * k / n_chunks;
    };
    const int64_t t0 = bound(c), t1 = bound(c + 1), nc = t1 - t0;
    uint32_t max_nodes = 1;  // the chunk's largest tree (bounds the untracked values: SR_TRACK_LITE)
    for (int64_t t = t0; t < t1; ++t)
      max_nodes = std::max<uint32_t>(max_nodes, uint32_t(trees->offsets[t + 1] - trees->offsets[t]));
    // chunks alternate between two streams: chunk c+1's workgroups fill the GPU while chunk c drains
    const hipStream_t cs = (c & 1) ? ctx->stream2 : s;
    sr_tree_batch sub = *trees;
    sub.n_trees = nc;
    sub.offsets = trees->offsets + t0;  // node arrays stay indexed by absolute offsets
    SrProgramBatch<T> pc;
    pc.keep_pieces = true;  // (staged below straight from the compile workers' buffers)
    int rc = sr_compile_batch<T>(sub, ctx->opsets[opset_id], n_total, ds->nf, false, &pc, &err,
                                 dmap.empty() ? nullptr : dmap.data());
    if (rc != SR_OK) {
      sync_both();  // earlier chunks may still read the staging buffers
      if (rc == SR_ERR_BAD_TREE || rc == SR_ERR_INVALID_ARG) {
        // report the tree index of the whole batch
        const size_t at = err.find("tree ");
        if (at == 0) {
          const int64_t k = std::atoll(err.c_str() + 5);
          err = "tree " + std::to_string(k + t0) + err.substr(err.find(':'));
        }
      }
      return set_error(rc, err);
    }
    if (c == 0) {
      if (phase_debug) {
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[sr phase] trees %lld chunks %d: setup %.3f ms, compile of chunk 0 (%lld trees) %.3f ms\n",
                     (long long)nt, n_chunks, std::chrono::duration<double, std::milli>(t_pre - ctx->phase_t).count(),
                     (long long)nc, std::chrono::duration<double, std::milli>(now - t_pre).count());
      }
      ctx->mark_phase(0);
    }
    const int depth = pc.max_depth > 0 ? pc.max_depth : 1;
    // Trees whose programs fit the register stack (<= 2 slots: every tree of < 23 nodes, most of the
    // rest) run on the register-stack kernel; the few deeper ones follow in a second launch of the
    // LDS-stack kernel over the tail of the launch order.
    int64_t n_vs = 0;  // launch positions [0, n_vs) -> register-stack kernel
    if (Rv > 0)
      for (int64_t i = 0; i < nc; ++i) n_vs += pc.depth[size_t(i)] <= SR_VSTK_SLOTS ? 1 : 0;
    // stage: code at code_base, offsets made absolute, static_bad, launch order (chunk-local)
    const size_t ncode = pc.n_code;
    if (code_base + ncode > code_cap) {
      sync_both();
      return set_error(SR_ERR_INVALID_ARG, "program longer than its node count");
    }
    std::memcpy(h_bad + t0, pc.static_bad.data(), size_t(nc));
    {
      // launch order: register-stack trees first, each class in decreasing estimated cost so every
      // block's waves get similar work (counting sort: costs are small integers; ties keep order)
      const std::vector<uint32_t>& cost = pc.cost;
      const bool sort = ctx->cost_order && nc > 1;
      uint32_t cmax = 0;
      if (sort)
        for (uint32_t v : cost) cmax = v > cmax ? v : cmax;
      const size_t nkey = size_t(cmax) + 1;
      // several views: the view first (each view's trees contiguous: its own segment of tree groups)
      const size_t n_cls = multi ? size_t(views->n_views) : 2;
      std::vector<uint32_t> start(n_cls * nkey + 1, 0);
      auto key = [&](int64_t i) -> size_t {
        const size_t cls = multi ? size_t(views->tree_view[t0 + i])
                                 : ((Rv > 0 && pc.depth[size_t(i)] > SR_VSTK_SLOTS) ? 1 : 0);
        return cls * nkey + (sort ? size_t(cmax - cost[size_t(i)]) : 0);
      };
      for (int64_t i = 0; i < nc; ++i) ++start[key(i) + 1];
      for (size_t k = 1; k < start.size(); ++k) start[k] += start[k - 1];
      for (int64_t i = 0; i < nc; ++i) h_perm[t0 + start[key(i)]++] = uint32_t(i);
      // Deal the cost-ordered trees of each class round-robin over that launch's tree groups (group
      // g takes ranks g, g + n_groups, ...; each group's positions stay in decreasing cost, so its
      // waves still get equal work).  Contiguous cost ranks made the first groups' workgroups several
      // times longer than the last groups' and the launch ended on a tail of heavy workgroups (C2's
      // complete trees: 4.36 ms with contiguous groups of 128, 3.32 unsorted).
      if (sort && ctx->balance_groups && !multi) {
        auto deal = [&](int64_t p0, int64_t np, int Rc, int depth_c) {
          if (np <= 1) return;
          const Grid gc = make_grid<T>(n_eval, np, Rc, W, int(ds->nf), depth_c, 0, ds->w != nullptr, ctx->tree_group,
                                       mrb);
          const int64_t G = gc.G, ng = gc.n_groups;
          if (ng <= 1) return;
          std::vector<uint32_t> ranked(h_perm + t0 + p0, h_perm + t0 + p0 + np);
          int64_t k = 0;
          for (int64_t j = 0; j < G; ++j)
            for (int64_t gi = 0; gi < ng; ++gi) {
              const int64_t size = gi + 1 < ng ? G : np - (ng - 1) * G;
              if (j < size) h_perm[t0 + p0 + gi * G + j] = ranked[size_t(k++)];
            }
        };
        if (n_vs > 0) deal(0, n_vs, Rv, 0);
        if (n_vs < nc) deal(n_vs, nc - n_vs, R, depth);
      }
    }
    {
      // programs in launch order: a tree group's code is one contiguous span (the kernel's LDS program
      // cache copies it in one pass); offsets / ends stay indexed by tree
      uint32_t at = code_base;
      for (int64_t p = 0; p < nc; ++p) {  // destinations: a prefix over the launch order
        const uint32_t i = h_perm[t0 + p];
        const uint32_t len = pc.offsets[size_t(i) + 1] - pc.offsets[size_t(i)];
        h_off[t0 + i] = at;
        h_end[t0 + i] = at + len;
        at += len;
      }
      // the copies into the pinned staging buffer: a large chunk's ~2 MB on the compile workers
      // (single-threaded they sat on the host path between the first chunk's launch and the second's)
      auto copy = [&](int64_t p0, int64_t p1) {
        for (int64_t p = p0; p < p1; ++p) {
          const uint32_t i = h_perm[t0 + p];
          const uint32_t len = h_end[t0 + i] - h_off[t0 + i];
          if (len) std::memcpy(h_code + h_off[t0 + i], pc.tree_code(i), size_t(len) * sizeof(SrIns<T>));
        }
      };
      constexpr int64_t kCopyPiece = 512;
      if (ctx->par_stage && nc >= 4 * kCopyPiece) {
        sr_parallel_for(int((nc + kCopyPiece - 1) / kCopyPiece), [&](int w) {
          const int64_t p0 = int64_t(w) * kCopyPiece;
          copy(p0, std::min<int64_t>(nc, p0 + kCopyPiece));
        });
      } else {
        copy(0, nc);
      }
    }
    // several views: one segment per view present (launch positions in view order), tree groups of the
    // launch's G, blocks in segment order
    int n_seg = 0;
    int64_t seg_blocks = 0;
    if (multi && nc > 0) {
      const Grid gm = make_grid<T>(n_eval, nc, R, W, int(ds->nf), depth, 0, ds->w != nullptr, ctx->tree_group,
                                   mrb);
      SrSegment* hs = reinterpret_cast<SrSegment*>(hprog + o_seg);
      for (int64_t p = 0; p < nc;) {
        const int v = views->tree_view[t0 + h_perm[t0 + p]];
        int64_t q = p;
        while (q < nc && views->tree_view[t0 + h_perm[t0 + q]] == v) ++q;
        SrSegment sg{};
        sg.block0 = int(seg_blocks);
        sg.pos0 = int(p);
        sg.n_pos = int(q - p);
        sg.groups = int((q - p + gm.G - 1) / gm.G);
        sg.row_off = int64_t(v) * n_idx;
        hs[n_seg++] = sg;
        seg_blocks += int64_t(sg.groups) * gm.n_row_blocks;
        p = q;
      }
    }
    if (n_chunks == 1) {  // the whole staging image (code, offsets, static_bad, order): one DMA
      const size_t img = multi ? o_seg + size_t(n_seg) * sizeof(SrSegment) : o_end + size_t(nc) * sizeof(uint32_t);
      SR_HIP_CHECK(hipMemcpyAsync(dprog, hprog, img, hipMemcpyHostToDevice, cs));
    } else {
      if (ncode)
        SR_HIP_CHECK(hipMemcpyAsync(static_cast<SrIns<T>*>(ctx->d_code) + code_base, h_code + code_base,
                                    ncode * sizeof(SrIns<T>), hipMemcpyHostToDevice, cs));
      SR_HIP_CHECK(hipMemcpyAsync(ctx->d_off + t0, h_off + t0, size_t(nc) * sizeof(uint32_t), hipMemcpyHostToDevice, cs));
      SR_HIP_CHECK(hipMemcpyAsync(ctx->d_end + t0, h_end + t0, size_t(nc) * sizeof(uint32_t), hipMemcpyHostToDevice, cs));
      SR_HIP_CHECK(hipMemcpyAsync(ctx->d_bad + t0, h_bad + t0, size_t(nc), hipMemcpyHostToDevice, cs));
      SR_HIP_CHECK(hipMemcpyAsync(ctx->d_perm + t0, h_perm + t0, size_t(nc) * sizeof(uint32_t), hipMemcpyHostToDevice, cs));
    }
    // merged summary
    for (int64_t i = 0; i < nc; ++i) prog->offsets[size_t(t0 + i)] = h_off[t0 + i];  // (starts; ends: h_end)
    std::memcpy(prog->static_bad.data() + t0, pc.static_bad.data(), size_t(nc));
    std::copy(pc.n_checks.begin(), pc.n_checks.end(), prog->n_checks.begin() + t0);
    if (pc.max_depth > prog->max_depth) prog->max_depth = pc.max_depth;
    if (pc.max_checks > prog->max_checks) prog->max_checks = pc.max_checks;
    prog->total_nodes += pc.total_nodes;
    prog->total_ops += pc.total_ops;

    if (ctx->timed_last) SR_HIP_CHECK(hipEventRecord(ctx->ev_c0[c], cs));  // the chunk's kernel time includes its probe
    // one launch over launch positions [p0, p0 + np) of the chunk; its partials occupy
    // [n_rb][np] words from p0 * n_rb (the chunk's region holds n_rb rows for every position)
    auto launch = [&](int64_t p0, int64_t np, bool vstk) -> int {
      const int Rc = vstk ? Rv : R;
      Grid g = make_grid<T>(n_eval, np, Rc, W, int(ds->nf), vstk ? 0 : depth, 0, ds->w != nullptr, ctx->tree_group,
                           mrb);
      if (g.lds > kLdsMax)
        return set_error(SR_ERR_TOO_DEEP, "the row tile (" + std::to_string(ds->nf) + " features, " +
                                              std::to_string(depth) + " stack slots) needs " + std::to_string(g.lds) +
                                              " bytes of LDS; the limit is 160 KiB");
      if (g.n_blocks > 0x7fffffff || g.n_row_blocks > n_rb) return set_error(SR_ERR_INVALID_ARG, "grid too large");
      glast = g;
      SrEvalArgs<T> a{};
      a.code = static_cast<const SrIns<T>*>(ctx->d_code);
      a.offsets = ctx->d_off + t0;
      a.ends = ctx->d_end + t0;
      a.perm = ctx->d_perm + t0 + p0;
      a.hint = use_hint ? ctx->hint.as<uint32_t>() + t0 + p0 : nullptr;
      a.hint_epoch = ctx->hint_epoch;
      a.n_trees = int(np);
      a.trees_per_block = g.G;
      a.X = static_cast<const T*>(ds->X);
      a.y = static_cast<const T*>(ds->y);
      a.w = static_cast<const T*>(ds->w);
      a.row_idx = gather ? ctx->row_idx.as<int64_t>() : nullptr;
      a.ld = ds->ld;
      a.derived = dmap.empty() ? nullptr : ctx->derived_cols.as<T>();
      a.dld = dld;
      a.n_rows = n_eval;
      a.nf = int(ds->nf);
      a.tiles_per_block = g.tiles;
      a.n_row_blocks = g.n_row_blocks;
      a.n_groups = g.n_groups;
      a.stack_depth = vstk ? std::min(depth, SR_VSTK_SLOTS) : depth;  // (the register-stack trees need <= SR_VSTK_SLOTS)
      // Σ over n_total rows of values below tbig cannot overflow T, even with rounding slack.
      a.tbig = T(t_max<T>() / (2.0 * double(n_total > 0 ? n_total : 1)));
      {  // the view's padded rows over every shard: n_total + at most one 2048-row tile of padding per shard
        const double padded = double(n_total > 0 ? n_total : 1) + 2048.0 * double(shard ? ctx->comm_ranks : 1);
        a.big_budget = 64.0 * (t_max<T>() / (1.01 * padded));  // (f64: 64 x DBL_MAX alone is +Inf)
      }
      a.track_x = !(max_abs_x < double(a.tbig)) ? 1 : 0;
#ifdef SR_TRACK_LITE
      if (mode == SR_MODE_LOSS && tier == SR_TIER_BASIC) {
        // (the deferred-check kernels leave +, - of stack values / features and cos, sin, neg, abs,
        //  sqrt untracked: such a value is at most L x max(tracked max, max|x|, 1) for a tree of L
        //  nodes, so with tbig / L as the tracked threshold every value stays below tbig, and a tile
        //  within budget / L - 64 (max|x| + 1) keeps every array's sum within the original budget;
        //  max|x| < tbig / L here: larger data took the per-node-check tier above)
        const double L = double(std::max<uint32_t>(1u, max_nodes));
        a.tbig = T(double(a.tbig) / L);
        a.big_budget = a.big_budget / L - 64.0 * (max_abs_x + 1.0);
        a.track_x = 0;
      }
#endif
      a.loss_kind = lkind;
      a.loss_param = T(lparam);
      a.part_sum = (host_red ? ctx->h_part.as<double>() : ctx->part_sum.as<double>()) + size_t(n_rb) * size_t(t0 + p0);
      a.part_flag = (host_red ? reinterpret_cast<uint32_t*>(ctx->h_part.as<double>() + n_part)
                              : ctx->part_flag.as<uint32_t>()) + size_t(n_rb) * size_t(t0 + p0);
      a.pred = ctx->pred.as<T>();
      a.pred_ld = n_eval;
      if (fold_path == 1) {  // (small calls under the in-order fold: every live tree's losses, [position][rows])
        a.fold_pos_stride = int64_t(g.n_row_blocks) * int64_t(g.tiles) * 64 * Rc;
        a.fold_loss = ctx->fold_store.as<T>() + fold_store_at;
        fold_store_at += size_t(np) * size_t(a.fold_pos_stride);
      }
      // LDS program cache (register-stack launches: 4 workgroups per CU leave ~36 KiB of dynamic LDS
      // each): sized for the longest group span of this launch, capped by that budget (groups longer
      // than the cap stream their windows from global memory)
      a.code_lds = 0;
      // (round 4's cache in the classic launches too — code_cache 2 — was measured without payoff and
      //  removed in round 6)
      const size_t code_budget = vstk ? kCodeCacheLds : 0;
      if (mode == SR_MODE_LOSS && ctx->code_cache && size_t(g.lds) < code_budget) {
        int64_t maxspan = 0;
        for (int64_t q = 0; q < g.n_groups; ++q) {
          const int64_t pf = p0 + q * g.G, pl = std::min<int64_t>(p0 + np, pf + g.G) - 1;
          const int64_t sp = int64_t(h_end[t0 + h_perm[t0 + pl]]) - int64_t(h_off[t0 + h_perm[t0 + pf]]);
          maxspan = std::max(maxspan, sp);
        }
        const int64_t cap = int64_t((code_budget - size_t(g.lds)) / 16);
        a.code_lds = int(std::min(maxspan, cap));
        if (a.code_lds < 64) a.code_lds = 0;
      }
      int64_t n_blocks = g.n_blocks;
      if (multi) {  // (one launch over the whole chunk: the segments computed above)
        a.segs = reinterpret_cast<const SrSegment*>(dprog + o_seg);
        a.n_segs = n_seg;
        n_blocks = seg_blocks;
        if (n_blocks > 0x7fffffff) return set_error(SR_ERR_INVALID_ARG, "grid too large");
      }
      const bool direct = mode == SR_MODE_LOSS && g.n_row_blocks == 1;
      if (direct) {  // the interpreter writes the final per-tree values; no reduce launch
        a.out_sum = ctx->d_out_sum + t0;
        a.out_flag = ctx->d_out_flag + t0;
        a.static_bad = ctx->d_bad + t0;
      }
      // several row blocks: the last workgroup of each tree group reduces it (no reduce launch)
      const bool fused = !direct && !host_red && mode == SR_MODE_LOSS && ctx->fused_reduce > 0 &&
                         int64_t(g.G) * int64_t(g.n_row_blocks) <= ctx->fused_reduce;
      if (fused) {
        a.group_cnt = ctx->group_cnt.as<uint32_t>() + t0 + p0;
        a.fused_sum = ctx->d_out_sum + t0;
        a.fused_flag = ctx->d_out_flag + t0;
        a.static_bad = ctx->d_bad + t0;
      }
      // mode 2 (default): every chunk after the first (its probe overlaps the first chunk's kernel),
      // and a single-chunk call when it is large (>= 512 trees x 2^18 rows: the tree-sharding share,
      // 1,250 trees x 1M rows, 1.09 -> 1.01 ms; the search's small calls pay the probe's launch and
      // keep none: profiles/r05_ab_probe.txt)
      // (round 5, later: also the first of two chunks when it is that large — C4's 8M-row shard
      //  216.9 -> 214.4 ms per call, C2 unchanged; tools/c4_shard_probe.py, profiles/r05_ab_c4_shard.txt)
      const bool probe_first = nc >= 512 && n_eval >= (int64_t(1) << 18);
      if (use_probe && p0 == 0 && g.n_row_blocks >= 16 && (ctx->probe != 2 || c > 0 || probe_first)) {
        // Trees that are non-finite on the first rows are flagged before the main launch, so its
        // workgroups skip them from their first tile (without the probe, the ~16 row blocks that
        // start together evaluate every such tree in full before a hint exists).  Only hints come
        // out of it: a tree non-finite on some rows of the view is incomplete on the whole view.
        // a wide, short grid: 16 trees x 1 tile per workgroup, kProbeTiles row blocks; always the
        // classic kernel at R rows per lane (a register-stack launch's 2x longer tiles would double the
        // probe's work for the same verdicts: C2's dead trees 0.88 -> 0.6x ms)
        SrEvalArgs<T> pa = a;
        pa.fold_loss = nullptr;  // (its rows are the stress rows; the main launch stores the view's)
        pa.stack_depth = depth;
        pa.out_sum = nullptr;
        pa.out_flag = nullptr;
        pa.code_lds = 0;  // (its groups differ from the main launch's)
        pa.group_cnt = nullptr;
        pa.stamps = nullptr;
        pa.trees_per_block = std::max(16, g.W);
        pa.n_groups = int((np + pa.trees_per_block - 1) / pa.trees_per_block);
        pa.tiles_per_block = 1;
        pa.n_row_blocks = kProbeTiles;
        pa.n_rows = std::min<int64_t>(n_eval, int64_t(kProbeTiles) * 64 * R);
        pa.part_sum = ctx->probe_sum.as<double>();
        pa.part_flag = ctx->probe_flag.as<uint32_t>();
        if (stress_probe) {  // the stress rows first (sr_dataset::probe_rows), through the gather build
          pa.row_idx = static_cast<const int64_t*>(ds->probe_rows);
          pa.n_rows = std::min<int64_t>(ds->n_probe, int64_t(kProbeTiles) * 64 * R);
          if (!dmap.empty()) {
            pa.derived = ctx->probe_derived.as<T>();
            pa.dld = kProbeRows;
          }
        }
        SR_HIP_CHECK(sr_launch_eval<T>(pa, mode, gather || stress_probe, tier, R, W, false, pa.n_groups * kProbeTiles, cs));
      }
#ifdef SR_STAMPS
      ctx->n_stamps = g.n_blocks * g.W * SR_NSTAMPS;
      SR_HIP_CHECK(ctx->stamps.ensure(size_t(ctx->n_stamps) * sizeof(uint64_t)));
      SR_HIP_CHECK(hipMemsetAsync(ctx->stamps.p, 0, size_t(ctx->n_stamps) * sizeof(uint64_t), cs));
      a.stamps = ctx->stamps.as<uint64_t>();
#endif
      SR_HIP_CHECK(sr_launch_eval<T>(a, mode, gather, tier, Rc, g.W, vstk, int(n_blocks), cs));
      if (fold_path) fjob.regions.push_back({a, t0, t0 + p0, np, n_blocks, Rc, vstk, g});
      if (!direct && !fused && host_red)
        ctx->host_reductions.push_back({t0 + p0, np, g.n_row_blocks});
      else if (!direct && !fused && !fjob.fuse_reduce)
        SR_HIP_CHECK(sr_launch_reduce(a.part_sum, a.part_flag, int(np), g.n_row_blocks, a.perm,
                                    ctx->d_bad + t0, ctx->d_out_sum + t0, ctx->d_out_flag + t0, cs));
      return SR_OK;
    };
    int lrc = SR_OK;
    if (n_vs > 0) lrc = launch(0, n_vs, true);
    if (lrc == SR_OK && n_vs < nc) lrc = launch(n_vs, nc - n_vs, false);
    if (lrc != SR_OK) {
      sync_both();
      return lrc;
    }
    if (ctx->timed_last) SR_HIP_CHECK(hipEventRecord(ctx->ev_c1[c], cs));
    if (fold_path && !shard && !fjob.regions.empty()) {
      // the in-order fold of this chunk's complete trees (sr_aux.hip): the launches' partials and flags
      // are final here (reduce / direct write / in-launch reduction ran on this stream)
      if (ctx->timed_last) SR_HIP_CHECK(hipEventRecord(ctx->ev_fc0[c], cs));
      SrFoldWho who{ctx->d_out_sum, ctx->d_out_flag, fold_n_terms, nullptr, nullptr, 1};
      if (fold_mirror) {
        who.msum = ctx->h_outs.as<double>();
        who.mflag = reinterpret_cast<uint32_t*>(ctx->h_outs.as<char>() + ctx->outs_flag_off);
      }
      for (const FoldRegion<T>& fr : fjob.regions) {
        int frc = fold_steps<T>(ctx, fjob, fr, who, cs);
        if (frc == SR_OK) frc = fold_walk<T>(ctx, fjob, fr, who, nullptr, d_fval, d_fst, cs);
        if (frc != SR_OK) {
          sync_both();
          return frc;
        }
      }
      fjob.regions.clear();
      if (ctx->timed_last) {
        SR_HIP_CHECK(hipEventRecord(ctx->ev_fc1[c], cs));
        ctx->fold_timed_last = true;
      }
    }
    ctx->n_chunks_last = c + 1;
    code_base += uint32_t(ncode);
  }
  if (n_chunks > 1) {  // the caller continues on the first stream: join the second
    SR_HIP_CHECK(hipEventRecord(ctx->ev_join, ctx->stream2));
    SR_HIP_CHECK(hipStreamWaitEvent(s, ctx->ev_join, 0));
  }
  if (nt == 0) ctx->mark_phase(0);
  *grid_out = glast;
  if (fold_path && shard) ctx->fold_job = std::make_shared<FoldJob<T>>(std::move(fjob));  // (eval_sharded_impl)
  ctx->mark_phase(1);
  return SR_OK;
}

// Interpreter time of the last run_batch (ms): Σ of its launches' durations (as a kernel trace sums
// them; chunks on the two streams may overlap, so this can exceed the wall time they span).
inline double chunk_kernel_ms(sr_ctx* ctx) {
  double ms = 0.0;
  if (!ctx->timed_last) return 0.0;
  for (int c = 0; c < ctx->n_chunks_last; ++c) {
    float m = 0.f;
    if (hipEventElapsedTime(&m, ctx->ev_c0[c], ctx->ev_c1[c]) == hipSuccess) ms += double(m);
  }
  if (ctx->derived_last) {  // the derived columns are part of the call's interpreter work
    float m = 0.f;
    if (hipEventElapsedTime(&m, ctx->ev_d0, ctx->ev_d1) == hipSuccess) ms += double(m);
  }
  return ms;
}

// The same launches' device-busy time: the UNION of their [start, end] intervals (chunks on the two
// streams overlap, so the sum above can exceed the wall time they span; this cannot).
inline double chunk_busy_ms(sr_ctx* ctx) {
  std::vector<std::pair<double, double>> iv;
  if (!ctx->timed_last) return 0.0;
  auto add = [&](hipEvent_t a, hipEvent_t b) {
    float t0 = 0.f, t1 = 0.f;
    if (hipEventElapsedTime(&t0, ctx->ev_start, a) == hipSuccess && hipEventElapsedTime(&t1, ctx->ev_start, b) == hipSuccess)
      iv.push_back({double(t0), double(t1)});
  };
  for (int c = 0; c < ctx->n_chunks_last; ++c) add(ctx->ev_c0[c], ctx->ev_c1[c]);
  if (ctx->derived_last) add(ctx->ev_d0, ctx->ev_d1);
  if (ctx->fold_timed_last)  // (the in-order fold's launches: device work of the call too)
    for (int c = 0; c < ctx->n_chunks_last; ++c) add(ctx->ev_fc0[c], ctx->ev_fc1[c]);
  std::sort(iv.begin(), iv.end());
  double busy = 0.0, lo = 0.0, hi = -1.0;
  for (const auto& [a, b] : iv) {
    if (a > hi) {
      if (hi > lo) busy += hi - lo;
      lo = a;
      hi = b;
    } else {
      hi = std::max(hi, b);
    }
  }
  if (hi > lo) busy += hi - lo;
  return busy;
}

// ---------------------------------------------------------------- Julia's pairwise `sum`
// DynamicExpressions decides a checked array with isfinite(sum(x)); Base's `sum` over an Array runs
// Base.mapreduce_impl: [lo, hi] splits at lo + (hi - lo) >> 1 until hi - lo < 1024
// (pairwise_blocksize), each leaf block is folded sequentially (v = a[lo]; v = v + a[i]) in T, and
// the halves are added back in the same recursion (arrays of < 16 elements: one sequential fold,
// which is the same thing).  The kernel's EXACT mode computes the leaf folds over row ranges; the
// host adds them in recursion order.  Row sharding: the global leaves are intersected with each
// shard; a leaf that starts in an earlier shard is carried by its first shard's prefix fold and
// continued, row by row, with this shard's values ("head" ranges of one row each).
struct JlRange {
  int64_t lo, hi;  // local rows of this view / shard (inclusive)
  int64_t leaf;    // global leaf index
  bool head;       // a single row continuing a leaf that starts in an earlier shard
};

std::vector<std::pair<int64_t, int64_t>> jl_leaves(int64_t n) {
  std::vector<std::pair<int64_t, int64_t>> out, st;
  if (n <= 0) return out;
  st.push_back({0, n - 1});
  while (!st.empty()) {
    const auto [lo, hi] = st.back();
    st.pop_back();
    if (hi - lo < 1024) {
      out.push_back({lo, hi});
    } else {
      const int64_t mid = lo + ((hi - lo) >> 1);
      st.push_back({mid + 1, hi});
      st.push_back({lo, mid});
    }
  }
  return out;
}

// The ranges a shard holding global rows [off, off + n) of n_total sums (in this order).
std::vector<JlRange> jl_ranges(int64_t off, int64_t n, int64_t n_total) {
  std::vector<JlRange> out;
  const auto leaves = jl_leaves(n_total);
  const int64_t last = off + n - 1;
  for (size_t k = 0; k < leaves.size(); ++k) {
    const auto [L, H] = leaves[k];
    if (H < off || L > last) continue;
    const int64_t h = H < last ? H : last;
    if (L >= off) {
      out.push_back({L - off, h - off, int64_t(k), false});
    } else {
      for (int64_t r = off; r <= h; ++r) out.push_back({r - off, r - off, int64_t(k), true});
    }
  }
  return out;
}

template <typename T>
T jl_reduce(const std::vector<T>& leafval, int64_t lo, int64_t hi, size_t* idx) {
  if (hi - lo < 1024) return leafval[(*idx)++];
  const int64_t mid = lo + ((hi - lo) >> 1);
  const T a = jl_reduce<T>(leafval, lo, mid, idx);
  const T b = jl_reduce<T>(leafval, mid + 1, hi, idx);
  return a + b;
}

// isfinite(Julia sum) of n_arrays arrays of n_total rows from every shard's range folds:
// rank_vals[r] = [n_arrays][ranges of shard r] (T), shards r = [offs[r], offs[r + 1]).
template <typename T>
void jl_finite(int64_t n_total, int n_ranks, const int64_t* offs, const T* const* rank_vals, int64_t n_arrays,
               uint8_t* out_finite) {
  const size_t n_leaves = jl_leaves(n_total).size();
  std::vector<std::vector<JlRange>> ranges(static_cast<size_t>(n_ranks));
  for (int r = 0; r < n_ranks; ++r) ranges[size_t(r)] = jl_ranges(offs[r], offs[r + 1] - offs[r], n_total);
  std::vector<T> leafval(n_leaves);
  for (int64_t a = 0; a < n_arrays; ++a) {
    for (int r = 0; r < n_ranks; ++r) {
      const std::vector<JlRange>& rg = ranges[size_t(r)];
      const T* v = rank_vals[r] + size_t(a) * rg.size();
      for (size_t i = 0; i < rg.size(); ++i) {
        T& dst = leafval[size_t(rg[i].leaf)];
        dst = rg[i].head ? T(dst + v[i]) : v[i];
      }
    }
    size_t idx = 0;
    const T sum = n_total > 0 ? jl_reduce<T>(leafval, 0, n_total - 1, &idx) : T(0);
    out_finite[a] = std::isfinite(sum) ? 1 : 0;
  }
}

// Base.mapreduce_impl's combine of one view's leaf folds as a level-ordered node list: internal
// node m = (left, right) with c >= 0 = leaf c (leaves numbered in row order) and c < 0 = internal
// node -c-1; nodes are grouped by height (level_off), so every node's children lie in earlier levels.
struct JlLevels {
  std::vector<int32_t> nodes;      // 2 per internal node
  std::vector<int32_t> level_off;  // n_levels + 1
};
JlLevels jl_levels(int64_t n) {
  struct Tmp {
    int64_t l, r;  // >= 0 leaf, < 0 temporary internal id -x-1
    int h;
  };
  std::vector<Tmp> tmp;
  int64_t n_leaf = 0;
  // returns (code, height)
  std::function<std::pair<int64_t, int>(int64_t, int64_t)> rec = [&](int64_t lo, int64_t hi) -> std::pair<int64_t, int> {
    if (hi - lo < 1024) return {n_leaf++, 0};
    const int64_t mid = lo + ((hi - lo) >> 1);
    const auto L = rec(lo, mid);
    const auto R = rec(mid + 1, hi);
    const int h = 1 + std::max(L.second, R.second);
    tmp.push_back(Tmp{L.first, R.first, h});
    return {-int64_t(tmp.size()), h};
  };
  JlLevels out;
  if (n > 0) rec(0, n - 1);
  int max_h = 0;
  for (const Tmp& t : tmp) max_h = std::max(max_h, t.h);
  std::vector<int64_t> final_id(tmp.size());
  out.level_off.assign(size_t(max_h) + 1, 0);
  for (const Tmp& t : tmp) out.level_off[size_t(t.h)]++;  // counts at heights 1..max_h
  for (int h = 1; h <= max_h; ++h) out.level_off[size_t(h)] += out.level_off[size_t(h - 1)];
  std::vector<int64_t> fill(out.level_off.begin(), out.level_off.end() - 1);  // level h-1 starts at level_off[h-1]
  for (size_t i = 0; i < tmp.size(); ++i) final_id[i] = fill[size_t(tmp[i].h - 1)]++;
  out.nodes.resize(2 * tmp.size());
  auto code = [&](int64_t c) -> int32_t { return c >= 0 ? int32_t(c) : int32_t(-final_id[size_t(-c - 1)] - 1); };
  for (size_t i = 0; i < tmp.size(); ++i) {
    out.nodes[2 * size_t(final_id[i])] = code(tmp[i].l);
    out.nodes[2 * size_t(final_id[i]) + 1] = code(tmp[i].r);
  }
  return out;
}

// One view's leaves and combine program depend only on its row count: built once per thread and
// count (every call of a search or a step sees the same n; ~2k recursive calls for 1M rows).
const std::vector<JlRange>& jl_ranges_cached(int64_t n) {
  thread_local int64_t cn = -1;
  thread_local std::vector<JlRange> c;
  if (cn != n) {
    c = jl_ranges(0, n, n);
    cn = n;
  }
  return c;
}
const JlLevels& jl_levels_cached(int64_t n) {
  thread_local int64_t cn = -1;
  thread_local JlLevels c;
  if (cn != n) {
    c = jl_levels(n);
    cn = n;
  }
  return c;
}

// EXACT pass: the Julia-order fold of every checked array of the listed trees over `ranges` of this
// view -> host_vals[n_list][max_checks][ranges] (T; a tree's unused check slots hold 0).  With
// host_finite (single view: the ranges are the view's leaves in order) the leaves are combined on
// the device in recursion order and only isfinite(sum) per array comes back: host_finite[n_list][max_checks].
// Speculative use (stream `st`, sync = false; host_finite required, one batch): the launches are
// only enqueued — after a synchronisation of `st` the verdicts are at h_exact + *fin_off
// ([n_list][max_checks]) and ev_k0 / ev_k1 bracket the pass.
template <typename T>
int run_exact(sr_ctx* ctx, const sr_dataset* ds, const SrProgramBatch<T>& prog, const int64_t* row_idx,
              int64_t n_idx, const int64_t* list, int64_t n_list, int max_checks, const std::vector<JlRange>& ranges,
              T* host_vals, uint8_t* host_finite = nullptr, int64_t dev_row_off = 0, hipStream_t st = nullptr,
              bool sync = true, size_t* fin_off = nullptr) {
  if (n_list == 0 || max_checks == 0 || ranges.empty()) return SR_OK;
  if (!sync && (!host_finite || !fin_off)) return set_error(SR_ERR_INVALID_ARG, "speculative exact pass: no verdict buffer");
  const bool gather = row_idx != nullptr && n_idx > 0;
  const int64_t n_eval = gather ? n_idx : ds->n;
  hipStream_t s = st ? st : ctx->stream;
  const int depth = prog.max_depth > 0 ? prog.max_depth : 1;
  const int R = sr_rows_per_lane<T>(SR_MODE_EXACT, SR_TIER_FULL, 0);
  const int64_t rows = 64 * int64_t(R);
  // (BASIC operator sets: the BASIC-tier build of the pass, same rows and LDS plan, a smaller
  //  dispatch; SR_AMD_EXACT_TIER=full keeps the FULL-tier build for A/B runs)
  static const bool exact_full = [] {
    const char* v = std::getenv("SR_AMD_EXACT_TIER");
    return v && std::strcmp(v, "full") == 0;
  }();
  const int etier = (prog.tier == SR_TIER_BASIC && !exact_full) ? SR_TIER_BASIC : SR_TIER_FULL;
  const int64_t n_ranges = int64_t(ranges.size());
  int64_t max_len = 1;
  std::vector<int64_t> lo(static_cast<size_t>(n_ranges)), hi(static_cast<size_t>(n_ranges));
  for (int64_t i = 0; i < n_ranges; ++i) {
    lo[size_t(i)] = ranges[size_t(i)].lo;
    hi[size_t(i)] = ranges[size_t(i)].hi;
    if (hi[size_t(i)] < lo[size_t(i)] || hi[size_t(i)] >= n_eval) return set_error(SR_ERR_INVALID_ARG, "bad row range");
    max_len = std::max(max_len, hi[size_t(i)] - lo[size_t(i)] + 1);
  }
  // listed trees in batches whose range folds fit a bounded scratch buffer
  const size_t per_tree = size_t(max_checks) * size_t(n_ranges) * sizeof(T);
  const int64_t batch = std::max<int64_t>(1, int64_t((size_t(256) << 20) / per_tree));
  // pinned staging: [leaf ranges lo | hi | Julia-sum level program | tree list | verdicts]
  static const JlLevels kNoLevels{};
  const JlLevels& lv = host_finite ? jl_levels_cached(n_eval) : kNoLevels;
  const size_t n_lvp = lv.nodes.size() + lv.level_off.size();
  const size_t o_hi = size_t(n_ranges) * sizeof(int64_t), o_lvp = 2 * o_hi;
  const size_t o_list = (o_lvp + n_lvp * sizeof(int32_t) + 15) & ~size_t(15);
  const size_t o_fin = (o_list + size_t(std::min(batch, n_list)) * sizeof(uint32_t) + 15) & ~size_t(15);
  const size_t n_fin = host_finite ? size_t(std::min(batch, n_list)) * size_t(max_checks) : 0;
  SR_HIP_CHECK(ctx->h_exact.ensure(o_fin + n_fin + 16, s, ctx->stream2));
  char* const hx = ctx->h_exact.as<char>();
  {
    const size_t cap_lo = ctx->range_lo.cap, cap_hi = ctx->range_hi.cap;
    SR_HIP_CHECK(ctx->range_lo.ensure(size_t(n_ranges) * sizeof(int64_t)));
    SR_HIP_CHECK(ctx->range_hi.ensure(size_t(n_ranges) * sizeof(int64_t)));
    if (ctx->range_lo.cap != cap_lo || ctx->range_hi.cap != cap_hi || ctx->exact_lo_dev != lo || ctx->exact_hi_dev != hi) {
      ctx->exact_lo_dev.clear();  // (re-set only once the copies are queued)
      std::memcpy(hx, lo.data(), o_hi);
      std::memcpy(hx + o_hi, hi.data(), o_hi);
      SR_HIP_CHECK(hipMemcpyAsync(ctx->range_lo.p, hx, o_hi, hipMemcpyHostToDevice, s));
      SR_HIP_CHECK(hipMemcpyAsync(ctx->range_hi.p, hx + o_hi, o_hi, hipMemcpyHostToDevice, s));
      ctx->exact_lo_dev = lo;
      ctx->exact_hi_dev = hi;
    }
  }
  int n_internal = 0, n_levels = 0;
  if (host_finite) {
    n_internal = int(lv.nodes.size() / 2);
    n_levels = int(lv.level_off.size()) - 1;
    if (n_internal != n_ranges - 1 && !(n_ranges == 1 && n_internal == 0))
      return set_error(SR_ERR_INVALID_ARG, "bad leaf structure");
    // nodes then level offsets, one upload (kept for the next call over as many rows)
    const size_t cap = ctx->jsum_prog.cap;
    SR_HIP_CHECK(ctx->jsum_prog.ensure(n_lvp * sizeof(int32_t)));
    if (ctx->jsum_prog.cap != cap || ctx->jsum_n_dev != n_eval) {
      ctx->jsum_n_dev = -1;
      int32_t* b = reinterpret_cast<int32_t*>(hx + o_lvp);
      std::copy(lv.nodes.begin(), lv.nodes.end(), b);
      std::copy(lv.level_off.begin(), lv.level_off.end(), b + lv.nodes.size());
      SR_HIP_CHECK(hipMemcpyAsync(ctx->jsum_prog.p, b, n_lvp * sizeof(int32_t), hipMemcpyHostToDevice, s));
      ctx->jsum_n_dev = n_eval;
    }
  }
  if (!sync && batch < n_list) return set_error(SR_ERR_INVALID_ARG, "speculative exact pass: list too long");
  for (int64_t b0 = 0; b0 < n_list; b0 += batch) {
    const int64_t nb = std::min(batch, n_list - b0);
    // one wave per workgroup, G listed trees per workgroup (LDS: X tile + one wave's checked
    // values [max_checks][rows] + running sums [G][max_checks]): G amortises the tile staging over
    // trees, small G spreads few trees over more waves; aim at >= 1024 waves (one per SIMD), G <= 16
    // (C2's 8 listed trees x 1024 leaf ranges: G 1 -> 8, exact pass 0.28 -> 0.21 ms;
    // profiles/r02_ab_exact_g.txt)
    const int64_t g_fill = (nb * n_ranges + 1023) / 1024;
    int G = int(std::min<int64_t>(nb, ctx->exact_g > 0 ? ctx->exact_g : std::max<int64_t>(1, std::min<int64_t>(16, g_fill))));
    // four waves per workgroup share the staged rows, each folding its own trees: one wave per
    // workgroup left ~1 wave per SIMD for C2's 8 listed trees x 1024 leaves (latency-bound)
    int W = (ctx->exact_w == 4 && G >= 4) ? 4 : 1;
    size_t lds = 0;
    for (;;) {
      lds = sr_tile_lds_bytes(int(sizeof(T)), int(ds->nf), R, depth, G, max_checks, W, false);
      if (lds <= kLdsMax || G == 1) break;
      G /= 2;
      if (G < W) W = 1;
    }
    if (lds > kLdsMax) return set_error(SR_ERR_TOO_DEEP, "exact-sum pass needs more LDS than 160 KiB");
    uint32_t* list32 = reinterpret_cast<uint32_t*>(hx + o_list);  // (the previous batch's pass has completed)
    for (int64_t i = 0; i < nb; ++i) list32[i] = uint32_t(list[b0 + i]);
    if (!ctx->exact_list_host) {
      SR_HIP_CHECK(ctx->tree_list.ensure(size_t(nb) * sizeof(uint32_t)));
      SR_HIP_CHECK(hipMemcpyAsync(ctx->tree_list.p, list32, size_t(nb) * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    }
    SR_HIP_CHECK(ctx->range_sums.ensure(size_t(nb) * per_tree));
    SrEvalArgs<T> a{};
    a.code = static_cast<const SrIns<T>*>(ctx->d_code);
    a.offsets = ctx->d_off;
    a.ends = ctx->d_end;
    a.perm = ctx->exact_list_host ? list32 : ctx->tree_list.as<uint32_t>();
    a.n_trees = int(nb);
    a.trees_per_block = G;
    a.X = static_cast<const T*>(ds->X);
    a.row_idx = gather ? ctx->row_idx.as<int64_t>() + dev_row_off : nullptr;  // (this view's rows on the device)
    a.ld = ds->ld;
    a.n_rows = n_eval;
    a.nf = int(ds->nf);
    a.tiles_per_block = int((max_len + rows - 1) / rows);
    a.n_row_blocks = int(n_ranges);
    a.n_groups = int((nb + G - 1) / G);
    a.stack_depth = depth;
    a.tbig = T(0);
    a.max_checks = max_checks;
    a.range_lo = ctx->range_lo.as<int64_t>();
    a.range_hi = ctx->range_hi.as<int64_t>();
    a.range_sums = ctx->range_sums.p;
    const int64_t blocks = int64_t(a.n_groups) * n_ranges;
    if (blocks > 0x7fffffff) return set_error(SR_ERR_INVALID_ARG, "grid too large");
    SR_HIP_CHECK(hipEventRecord(ctx->ev_k0, s));
    SR_HIP_CHECK(sr_launch_eval<T>(a, SR_MODE_EXACT, gather, etier, R, W, false, int(blocks), s));
    if (host_finite) {
      const int64_t n_arrays = nb * max_checks;
      SR_HIP_CHECK(ctx->jsum_scratch.ensure(size_t(std::max<int64_t>(1, n_arrays * n_internal)) * sizeof(T)));
      const int32_t* lvp = ctx->jsum_prog.as<int32_t>();
      // (the verdicts go straight into the pinned staging buffer: no copy back)
      uint8_t* fin = reinterpret_cast<uint8_t*>(hx + o_fin);
      SR_HIP_CHECK(sr_launch_jsum_levels<T>(static_cast<const T*>(ctx->range_sums.p), n_arrays, int(n_ranges),
                                            reinterpret_cast<const int2*>(lvp), n_internal, lvp + 2 * n_internal,
                                            n_levels, ctx->jsum_scratch.as<T>(), fin, s));
    } else {
      SR_HIP_CHECK(hipMemcpyAsync(host_vals + size_t(b0) * max_checks * size_t(n_ranges), ctx->range_sums.p,
                                  size_t(nb) * per_tree, hipMemcpyDeviceToHost, s));
    }
    SR_HIP_CHECK(hipEventRecord(ctx->ev_k1, s));
    if (!sync) {
      *fin_off = o_fin;
      return SR_OK;
    }
    SR_HIP_CHECK(hipStreamSynchronize(s));
    if (host_finite)
      std::memcpy(host_finite + size_t(b0) * max_checks, hx + o_fin, size_t(nb) * size_t(max_checks));
    float km = 0.f;
    if (hipEventElapsedTime(&km, ctx->ev_k0, ctx->ev_k1) == hipSuccess) ctx->exact_kernel_ms += double(km);
  }
  return SR_OK;
}

// EXACT pass over the whole view on this GPU -> list_ok[i] = every checked array of tree list[i]
// passes isfinite(Julia sum).
template <typename T>
int exact_list_ok(sr_ctx* ctx, const sr_dataset* ds, const SrProgramBatch<T>& prog, const int64_t* row_idx,
                  int64_t n_idx, const std::vector<int64_t>& list, std::vector<uint8_t>* list_ok,
                  int64_t dev_row_off = 0) {
  list_ok->assign(list.size(), 1);
  if (list.empty() || prog.max_checks == 0) return SR_OK;
  const bool gather = row_idx != nullptr && n_idx > 0;
  const int64_t n_eval = gather ? n_idx : ds->n;
  const std::vector<JlRange>& ranges = jl_ranges_cached(n_eval);
  // check slots: the most any LISTED tree has (the LDS image and the fold buffers scale with it)
  int mc = 0;
  for (int64_t t : list) mc = std::max(mc, int(prog.n_checks[size_t(t)]));
  if (mc == 0) return SR_OK;
  // leaf folds combined in recursion order on the device: only the verdicts come back
  std::vector<uint8_t> fin(list.size() * size_t(mc));
  int rc = run_exact<T>(ctx, ds, prog, row_idx, n_idx, list.data(), int64_t(list.size()), mc, ranges, nullptr,
                        fin.data(), dev_row_off);
  if (rc != SR_OK) return rc;
  for (size_t i = 0; i < list.size(); ++i)
    for (int k = 0; k < mc; ++k) (*list_ok)[i] &= fin[i * size_t(mc) + size_t(k)];
  return SR_OK;
}

// Finalize one tree: complete unless flagged; BIG-only trees take their exact verdict (list_ok).  A
// complete tree's loss is Σ / denom, or +Inf where the reference's T-precision fold of the losses
// overflows (sr_fold.h; n_terms = rows of the fold, 0: only SR_FLAG_ELEMINF is applied).  Trees the
// bounds cannot decide are appended to *fold_list (when given) for the exact in-order fold.
// fold (may be NULL): every complete tree's in-order fold from the call's walk (values, SR_FST_* status,
// and the T denominators: T(count), or Base.sum(w) in T, per tree); a tree the walk folded takes
// fold / denominator in T (the reference's own arithmetic), one whose walk failed joins *fold_list.
template <typename T>
struct FoldResults {
  const T* val;
  const int32_t* st;
  std::function<T(int64_t)> den;
  int64_t n_ok = 0, n_fail = 0;
  int debug_fail = 0;  // (tests, "fold_debug_fail" k: trees t % k == 0 take the fallback as if their walk failed)
};
template <typename T>
void finalize(int64_t nt, const double* sums, const uint32_t* flags, double denom, const int64_t* list,
              int64_t n_list, const uint8_t* list_ok, T* out_loss, uint8_t* out_complete, int64_t n_terms = 0,
              std::vector<int64_t>* fold_list = nullptr, const double* denoms = nullptr, FoldResults<T>* fold = nullptr) {
  std::vector<int64_t> pos;
  if (n_list > 0) {
    pos.assign(size_t(nt), -1);
    for (int64_t i = 0; i < n_list; ++i) pos[size_t(list[i])] = i;
  }
  for (int64_t t = 0; t < nt; ++t) {
    bool ok = (flags[t] & (SR_FLAG_NONFINITE | SR_FLAG_STATIC)) == 0;
    if (ok && (flags[t] & SR_FLAG_BIG)) {
      const int64_t p = pos.empty() ? -1 : pos[size_t(t)];
      if (p >= 0 && list_ok && !list_ok[p]) ok = false;
    }
    out_complete[t] = ok ? 1 : 0;
    out_loss[t] = ok ? T(sums[t] / (denoms ? denoms[t] : denom)) : T(INFINITY);
    if (!ok) continue;
    const bool elem_inf = (flags[t] & SR_FLAG_ELEMINF) != 0;
    const int cls = n_terms > 0 ? sr_fold_class<T>(sums[t], elem_inf, n_terms) : (elem_inf ? SR_FOLD_INF : SR_FOLD_FINITE);
    if (cls == SR_FOLD_INF) {
      out_loss[t] = T(INFINITY);
    } else if (cls == SR_FOLD_EXACT && fold_list) {
      fold_list->push_back(t);
    } else if (cls == SR_FOLD_FINITE && fold) {
      if (fold->st[t] == SR_FST_OK && !(fold->debug_fail > 0 && t % fold->debug_fail == 0)) {
        out_loss[t] = T(fold->val[t] / fold->den(t));
        ++fold->n_ok;
      } else if (fold->st[t] != SR_FST_NONE && fold_list) {
        fold_list->push_back(t);
        ++fold->n_fail;
      }
    }
  }
}

// The trees `idx` of a batch as a batch of their own (node arrays copied: a tree is a contiguous range).
template <typename T>
struct SubBatch {
  std::vector<int64_t> offs;
  std::vector<uint8_t> deg, op, con;
  std::vector<uint16_t> feat;
  std::vector<T> val;
  sr_tree_batch b{};
  SubBatch(const sr_tree_batch& trees, const int64_t* idx, size_t n) {
    offs.assign(n + 1, 0);
    for (size_t i = 0; i < n; ++i) offs[i + 1] = offs[i] + (trees.offsets[idx[i] + 1] - trees.offsets[idx[i]]);
    const size_t nn = size_t(offs.back());
    deg.resize(nn);
    op.resize(nn);
    con.resize(nn);
    feat.resize(nn);
    val.resize(nn);
    const T* vals = static_cast<const T*>(trees.val);
    for (size_t i = 0; i < n; ++i) {
      const int64_t b0 = trees.offsets[idx[i]], len = offs[i + 1] - offs[i], o = offs[i];
      std::memcpy(deg.data() + o, trees.degree + b0, size_t(len));
      std::memcpy(op.data() + o, trees.op + b0, size_t(len));
      std::memcpy(con.data() + o, trees.constant + b0, size_t(len));
      std::memcpy(feat.data() + o, trees.feature + b0, size_t(len) * sizeof(uint16_t));
      std::memcpy(val.data() + o, vals + b0, size_t(len) * sizeof(T));
    }
    b = sr_tree_batch{int64_t(n), offs.data(), deg.data(), op.data(), feat.data(), con.data(), val.data()};
  }
};

// Rows per segment of the fold's segmented chain (sr_aux.hip): ctx->fold_seg < 0 chooses (<= 1024
// segments of 8k-64k rows), 0 folds the whole view with one workgroup scan per tree (rounds 3-4).
inline int64_t fold_seg_len(const sr_ctx* ctx, int64_t n) {
  if (ctx->fold_seg >= 0) return ctx->fold_seg;
  const int64_t L = ((n / 512 + 8191) / 8192) * 8192;
  return std::min<int64_t>(std::max<int64_t>(L, 8192), 65536);
}

// The prediction buffer of the fold's PRED passes is kept up to 1/32 of the device memory (9 GB on a
// 288 GB MI355X: C4's 14 band trees x 2^26 rows are 3.6 GB, and a re-allocation cost the step ~35 ms);
// anything larger is released after the call.
inline void release_large_pred(sr_ctx* ctx) {
  size_t free_b = 0, total_b = 0;
  const size_t keep = hipMemGetInfo(&free_b, &total_b) == hipSuccess ? std::max(total_b / 32, size_t(2) << 30)
                                                                       : (size_t(2) << 30);
  if (ctx->pred.cap > keep) ctx->pred.release();
}

// Device scratch of one fold batch of nb trees and n_seg segments (ctx->fold_io): segment sums,
// binades and composed steps, carries, estimates, results and slow-segment counts.
template <typename T>
struct FoldDev {
  double* segsum = nullptr;
  int2* tq = nullptr;
  int64_t* tab = nullptr;
  double* carry_est = nullptr;
  T* carry = nullptr;
  T* out = nullptr;
  int* slow = nullptr;
  static size_t al(size_t b) { return (b + 255) & ~size_t(255); }
  static size_t bytes(size_t nb, int64_t n_seg) {
    const size_t ns = nb * size_t(n_seg > 0 ? n_seg : 1);
    return al(ns * 8) + al(ns * 8) + al(ns * 32) + al(nb * 8) + 2 * al(nb * sizeof(T)) + al(nb * 4);
  }
  void bind(void* base, size_t nb, int64_t n_seg) {
    const size_t ns = nb * size_t(n_seg > 0 ? n_seg : 1);
    char* c = static_cast<char*>(base);
    segsum = reinterpret_cast<double*>(c);
    c += al(ns * 8);
    tq = reinterpret_cast<int2*>(c);
    c += al(ns * 8);
    tab = reinterpret_cast<int64_t*>(c);
    c += al(ns * 32);
    carry_est = reinterpret_cast<double*>(c);
    c += al(nb * 8);
    carry = reinterpret_cast<T*>(c);
    c += al(nb * sizeof(T));
    out = reinterpret_cast<T*>(c);
    c += al(nb * sizeof(T));
    slow = reinterpret_cast<int*>(c);
  }
};

// The fold's PRED passes are internal: the call's interpreter timing (its chunk events) and the kernel
// it reports (rows per lane, derived columns) stay those of the call's own loss launches.
struct KeepCallInfo {
  sr_ctx* c;
  int timing, n_chunks, n_derived, rows;
  bool timed, derived;
  explicit KeepCallInfo(sr_ctx* x)
      : c(x), timing(x->timing), n_chunks(x->n_chunks_last), n_derived(x->n_derived_last), rows(x->rows_last),
        timed(x->timed_last), derived(x->derived_last) {
    x->timing = 0;
    x->internal_pass = true;
  }
  ~KeepCallInfo() {
    c->internal_pass = false;
    c->timing = timing;
    c->n_chunks_last = n_chunks;
    c->n_derived_last = n_derived;
    c->rows_last = rows;
    c->timed_last = timed;
    c->derived_last = derived;
  }
};

// Trees per PRED pass of the fold: predictions of at most `budget` bytes (and half the free device
// memory when `use_free`; the row-sharded call uses a fixed budget so that every rank cuts the list
// alike).
inline int64_t fold_batch_trees(int64_t n_eval, size_t elem, bool use_free) {
  size_t budget = size_t(8) << 30, free_b = 0, total_b = 0;
  if (use_free && hipMemGetInfo(&free_b, &total_b) == hipSuccess) budget = std::min(budget, free_b / 2);
  return std::max<int64_t>(1, int64_t(budget / (size_t(std::max<int64_t>(n_eval, 1)) * elem)));
}

// One batch of listed trees, first half: the PRED interpreter over this view (or shard) into ctx->pred,
// the device scratch bound, and (segmented) the segment sums.
template <typename T>
int fold_prepare(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees, const int64_t* row_idx,
                 int64_t n_idx, int64_t n_total, int loss_kind, const int64_t* list, size_t nb, int64_t seg_len,
                 FoldDev<T>* fd) {
  int lkind = 0;
  double lparam = 0.0;
  if (decode_loss(ctx, loss_kind, &lkind, &lparam) != SR_OK) return SR_ERR_INVALID_ARG;
  const bool gather = row_idx != nullptr && n_idx > 0;
  const int64_t n_eval = gather ? n_idx : ds->n;
  SubBatch<T> sub(*trees, list, nb);
  SrProgramBatch<T> prog;
  Grid g;
  SR_HIP_CHECK(hipEventRecord(ctx->ev_f[0], ctx->stream));
  int rc = run_batch<T>(ctx, ds, opset_id, &sub.b, row_idx, n_idx, n_total, loss_kind, SR_MODE_PRED, &prog, &g);
  if (rc != SR_OK) return rc;
  SR_HIP_CHECK(hipEventRecord(ctx->ev_f[1], ctx->stream));
  const int64_t n_seg = seg_len > 0 ? (n_eval + seg_len - 1) / seg_len : 0;
  SR_HIP_CHECK(ctx->fold_io.ensure(FoldDev<T>::bytes(nb, n_seg)));
  fd->bind(ctx->fold_io.p, nb, n_seg);
  if (seg_len > 0)
    SR_HIP_CHECK(sr_launch_fold_segsum<T>(ctx->pred.as<T>(), n_eval, int(nb), static_cast<const T*>(ds->y),
                                          static_cast<const T*>(ds->w), gather ? ctx->row_idx.as<int64_t>() : nullptr,
                                          n_eval, lkind, T(lparam), seg_len, fd->segsum, ctx->stream));
  SR_HIP_CHECK(hipEventRecord(ctx->ev_f[2], ctx->stream));
  return SR_OK;
}

// Second half: the segments' composed steps (carry_est: device, per tree, or NULL) and the chain
// (carry: device, per tree, or NULL); the folds into out (host) after one synchronisation.
template <typename T>
int fold_finish(sr_ctx* ctx, const sr_dataset* ds, const int64_t* row_idx, int64_t n_idx, int loss_kind, size_t nb,
                int64_t seg_len, const FoldDev<T>& fd, bool with_carry_est, bool with_carry, T* out) {
  int lkind = 0;
  double lparam = 0.0;
  if (decode_loss(ctx, loss_kind, &lkind, &lparam) != SR_OK) return SR_ERR_INVALID_ARG;
  const bool gather = row_idx != nullptr && n_idx > 0;
  const int64_t n_eval = gather ? n_idx : ds->n;
  hipStream_t s = ctx->stream;
  const T* y = static_cast<const T*>(ds->y);
  const T* w = static_cast<const T*>(ds->w);
  const int64_t* ri = gather ? ctx->row_idx.as<int64_t>() : nullptr;
  if (seg_len > 0)
    SR_HIP_CHECK(sr_launch_fold_segtab<T>(ctx->pred.as<T>(), n_eval, int(nb), y, w, ri, n_eval, lkind, T(lparam),
                                          seg_len, fd.segsum, with_carry_est ? fd.carry_est : nullptr, fd.tq, fd.tab, s));
  SR_HIP_CHECK(hipEventRecord(ctx->ev_f[3], s));
  SR_HIP_CHECK(sr_launch_fold<T>(ctx->pred.as<T>(), n_eval, int(nb), y, w, ri, n_eval, lkind, T(lparam), seg_len, fd.tq,
                                 fd.tab, with_carry ? fd.carry : nullptr, fd.out, fd.slow, s));
  SR_HIP_CHECK(hipEventRecord(ctx->ev_f[4], s));
  std::vector<int> slow(nb, 0);
  SR_HIP_CHECK(hipMemcpyAsync(out, fd.out, nb * sizeof(T), hipMemcpyDeviceToHost, s));
  SR_HIP_CHECK(hipMemcpyAsync(slow.data(), fd.slow, nb * sizeof(int), hipMemcpyDeviceToHost, s));
  SR_HIP_CHECK(hipStreamSynchronize(s));
  for (int v : slow) ctx->fold_slow_last += v;
  for (int i = 0; i < 4; ++i) {  // (events 0-2 were recorded by fold_prepare on the same stream)
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, ctx->ev_f[i], ctx->ev_f[i + 1]) == hipSuccess) ctx->fold_ms[i] += double(ms);
  }
  ctx->fold_seg_last = seg_len;
  return SR_OK;
}

// The reference's fold of the listed trees' losses over this view, exactly and in row order
// (sr_fold.h; sr_aux.hip): their predictions from the PRED interpreter (the values the LOSS kernels
// saw), then the segmented fold.  out: the folds (T; +Inf where the fold overflows).  Runs after the
// call's other passes (it reuses the context's program buffers).
template <typename T>
int fold_exact(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees, const int64_t* row_idx,
               int64_t n_idx, int64_t n_total, int loss_kind, const std::vector<int64_t>& list, std::vector<T>* out) {
  out->assign(list.size(), T(0));
  if (list.empty()) return SR_OK;
  const bool gather = row_idx != nullptr && n_idx > 0;
  const int64_t n_eval = gather ? n_idx : ds->n;
  const int64_t seg_len = fold_seg_len(ctx, n_eval);
  KeepCallInfo keep(ctx);
  const int64_t per = fold_batch_trees(n_eval, sizeof(T), true);
  for (size_t b0 = 0; b0 < list.size(); b0 += size_t(per)) {
    const size_t nb = std::min(list.size() - b0, size_t(per));
    FoldDev<T> fd;
    int rc = fold_prepare<T>(ctx, ds, opset_id, trees, row_idx, n_idx, n_total, loss_kind, list.data() + b0, nb, seg_len,
                             &fd);
    if (rc != SR_OK) return rc;
    rc = fold_finish<T>(ctx, ds, row_idx, n_idx, loss_kind, nb, seg_len, fd, false, false, out->data() + b0);
    if (rc != SR_OK) return rc;
  }
  release_large_pred(ctx);
  return SR_OK;
}

// Base.sum in T of v[idx[i]] (or v[i]), i < n: Base.mapreduce_impl's pairwise recursion (blocks of
// < 1024 folded sequentially) — the reference's sum(w) (LossFunctions' normalize = true).
template <typename T>
T jl_sum_T(const double* v, const int64_t* idx, int64_t lo, int64_t hi) {  // inclusive [lo, hi]
  auto at = [&](int64_t i) { return T(v[idx ? idx[i] : i]); };
  if (lo == hi) return at(lo);
  if (hi - lo < 1024) {
    T a = at(lo) + at(lo + 1);
    for (int64_t i = lo + 2; i <= hi; ++i) a = a + at(i);
    return a;
  }
  const int64_t mid = lo + ((hi - lo) >> 1);
  const T x = jl_sum_T<T>(v, idx, lo, mid);
  const T y = jl_sum_T<T>(v, idx, mid + 1, hi);
  return x + y;
}

// The partials of the call's launches (ctx->host_reductions) reduced on the host into {Σ, flags}, in
// sr_reduce_positions' order: lane l sums row blocks l, l + 64, ... from 0.0, then for off = 32 .. 1 every
// lane adds its partner l ^ off (IEEE addition commutes, so both partners hold the same bits), lane 0's
// value is the result; flags ORed; the static flags from the staging image.
void host_reduce_partials(sr_ctx* ctx, int64_t nt) {
  const size_t n_part = size_t(nt) * size_t(ctx->host_red_rb);
  const double* ps = ctx->h_part.as<double>();
  const uint32_t* pf = reinterpret_cast<const uint32_t*>(ps + n_part);
  double* out_sum = ctx->h_outs.as<double>();
  uint32_t* out_flag = reinterpret_cast<uint32_t*>(ctx->h_outs.as<char>() + ctx->outs_flag_off);
  const uint32_t* perm = ctx->h_perm_last;
  const uint8_t* bad = ctx->h_bad_last;
  // (the partials are read once, in memory order — row block by row block, each a contiguous run of
  //  positions — into per-(position, lane) accumulators; lane l still adds its row blocks l, l + 64,
  //  ... in increasing order, so the sums are the reduce kernel's bit for bit.  Round 5: the column
  //  walk it replaces touched a new cache line per partial, ~6k device-written lines per C3 call)
  std::vector<double>& acc = ctx->host_acc;
  std::vector<uint32_t>& fls = ctx->host_fl;
  for (const sr_ctx::HostReduction& hr : ctx->host_reductions) {
    const double* s0 = ps + size_t(ctx->host_red_rb) * size_t(hr.p0);
    const uint32_t* f0 = pf + size_t(ctx->host_red_rb) * size_t(hr.p0);
    const size_t np = size_t(hr.np);
    acc.assign(np * 64, 0.0);
    fls.assign(np, 0u);
    for (int i = 0; i < hr.n_rb; ++i) {
      double* a = acc.data() + size_t(i & 63);
      const double* srow = s0 + size_t(i) * np;
      const uint32_t* frow = f0 + size_t(i) * np;
      for (size_t pos = 0; pos < np; ++pos) {
        a[pos * 64] += srow[pos];
        fls[pos] |= frow[pos];
      }
    }
    for (size_t pos = 0; pos < np; ++pos) {
      double v[64];
      std::memcpy(v, acc.data() + pos * 64, sizeof(v));
      for (int off = 32; off >= 1; off >>= 1) {
        double nv[64];
        for (int l = 0; l < 64; ++l) nv[l] = v[l] + v[l ^ off];
        std::memcpy(v, nv, sizeof(v));
      }
      uint32_t fl = fls[pos];
      const uint32_t tree = perm[hr.p0 + pos];
      if (bad[tree]) fl |= SR_FLAG_STATIC | SR_FLAG_NONFINITE;
      out_sum[tree] = v[0];
      out_flag[tree] = fl;
    }
  }
  ctx->host_reductions.clear();
}

// Base.sum(w) in T over a view (the reference's normalize = true denominator); the full view's is cached
// per dataset and type.
template <typename T>
T jl_wsum_view(const sr_dataset* ds, const int64_t* row_idx, int64_t n) {
  if (n <= 0) return T(0);
  if (row_idx) return jl_sum_T<T>(ds->w_host.data(), row_idx, 0, n - 1);
  double& c = sizeof(T) == 4 ? ds->wsum_jl_f32 : ds->wsum_jl_f64;
  if (!(c == c)) c = double(jl_sum_T<T>(ds->w_host.data(), nullptr, 0, n - 1));
  return T(c);
}

template <typename T>
double view_denominator(const sr_dataset* ds, const int64_t* row_idx, int64_t n_idx) {
  const bool gather = row_idx != nullptr && n_idx > 0;
  if (!ds->w) return double(gather ? n_idx : ds->n);
  if (!gather) return ds->wsum;
  double s = 0.0;
  for (int64_t i = 0; i < n_idx; ++i) s += ds->w_host[size_t(row_idx[i])];
  return s;
}


// views (may be NULL): several row views in one call (sr_eval_loss_batch_views); row_idx then holds
// views->n_views views of n_idx rows each.
// The second half of an eval_loss call: what finishing it needs once its device work is enqueued.
template <typename T>
struct LossCall {
  const sr_dataset* ds = nullptr;
  int opset_id = 0, loss_kind = 0;
  sr_tree_batch trees{};
  const int64_t* row_idx = nullptr;
  int64_t n_idx = 0;
  void* out_loss = nullptr;
  uint8_t* out_complete = nullptr;
  bool has_views = false;
  ViewSpec views{};
  SrProgramBatch<T> prog;
  std::chrono::steady_clock::time_point t0;
};
template <typename T>
int eval_loss_finish(sr_ctx* ctx, LossCall<T>& c);

// First half: compile, stage, launch, and the copy of {Σ, flags} (or the kernel's own writes into
// pinned memory); *c holds what eval_loss_finish needs.
template <typename T>
int eval_loss_submit(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                     const int64_t* row_idx, int64_t n_idx, int loss_kind, void* out_loss, uint8_t* out_complete,
                     const ViewSpec* views, LossCall<T>* c) {
  const int64_t nt = trees->n_trees;
  if (nt > 0 && (!out_loss || !out_complete)) return set_error(SR_ERR_INVALID_ARG, "NULL output buffers");
  const bool gather = row_idx != nullptr && n_idx > 0;
  const int64_t n_eval = gather ? n_idx : ds->n;
  auto t0 = std::chrono::steady_clock::now();
  ctx->start_phases(t0);
  c->ds = ds;
  c->opset_id = opset_id;
  c->loss_kind = loss_kind;
  c->trees = *trees;
  c->row_idx = row_idx;
  c->n_idx = n_idx;
  c->out_loss = out_loss;
  c->out_complete = out_complete;
  c->has_views = views != nullptr;
  if (views) c->views = *views;
  c->t0 = t0;
  SrProgramBatch<T>& prog = c->prog;
  Grid g;
  ctx->want_host_out = true;
  ctx->want_fold = true;
  int rc = run_batch<T>(ctx, ds, opset_id, trees, row_idx, n_idx, n_eval, loss_kind, SR_MODE_LOSS, &prog, &g, true,
                        nullptr, views);
  ctx->want_host_out = false;
  ctx->want_fold = false;
  if (rc != SR_OK) return rc;
  if (nt == 0) return SR_OK;
  hipStream_t s = ctx->stream;
  // {Σ loss, flags} of every tree: already in pinned memory (host_io), or one DMA there
  if (!ctx->outs_on_host) {
    const size_t out_bytes = ctx->fold_path_last ? ctx->outs_bytes_all : ctx->outs_flag_off + size_t(nt) * sizeof(uint32_t);
    SR_HIP_CHECK(ctx->h_outs.ensure(out_bytes, s, ctx->stream2));
    SR_HIP_CHECK(hipMemcpyAsync(ctx->h_outs.p, ctx->outs.p, out_bytes, hipMemcpyDeviceToHost, s));
  }
  return SR_OK;
}

template <typename T>
int eval_loss_finish(sr_ctx* ctx, LossCall<T>& c) {
  const sr_dataset* ds = c.ds;
  const int opset_id = c.opset_id;
  const sr_tree_batch* trees = &c.trees;
  const int64_t* row_idx = c.row_idx;
  const int64_t n_idx = c.n_idx;
  const int loss_kind = c.loss_kind;
  void* out_loss = c.out_loss;
  uint8_t* out_complete = c.out_complete;
  const ViewSpec* views = c.has_views ? &c.views : nullptr;
  SrProgramBatch<T>& prog = c.prog;
  const auto t0 = c.t0;
  const int64_t nt = trees->n_trees;
  if (nt == 0) return SR_OK;
  const bool gather = row_idx != nullptr && n_idx > 0;
  const int64_t n_eval = gather ? n_idx : ds->n;
  const int n_views = views ? views->n_views : 1;
  auto view_of = [&](int64_t t) -> int { return views ? int(views->tree_view[t]) : 0; };
  auto rows_of = [&](int v) -> const int64_t* { return gather ? row_idx + int64_t(v) * n_idx : nullptr; };
  hipStream_t s = ctx->stream;
  int rc = SR_OK;

  SR_HIP_CHECK(hipStreamSynchronize(s));
  if (!ctx->host_reductions.empty()) host_reduce_partials(ctx, nt);
  const double* hs = ctx->h_outs.as<double>();
  const uint32_t* hf = reinterpret_cast<const uint32_t*>(ctx->h_outs.as<char>() + ctx->outs_flag_off);
  std::vector<double> sums(hs, hs + nt);
  std::vector<uint32_t> flags(hf, hf + nt);
  ctx->timing_pending = true;
  ctx->mark_phase(2);
  std::vector<int64_t> list;
  for (int64_t t = 0; t < nt; ++t)
    if ((flags[t] & (SR_FLAG_NONFINITE | SR_FLAG_STATIC)) == 0 && (flags[t] & SR_FLAG_BIG)) list.push_back(t);
  std::vector<uint8_t> list_ok(list.size(), 1);
  ctx->n_exact_last = int64_t(list.size());
  ctx->exact_kernel_ms = 0.0;
  for (int v = 0; v < n_views && !list.empty(); ++v) {  // (each view's listed trees over its own rows)
    std::vector<int64_t> lv;
    std::vector<size_t> at;
    for (size_t i = 0; i < list.size(); ++i)
      if (view_of(list[i]) == v) {
        lv.push_back(list[i]);
        at.push_back(i);
      }
    if (lv.empty()) continue;
    std::vector<uint8_t> ok;
    rc = exact_list_ok<T>(ctx, ds, prog, rows_of(v), n_idx, lv, &ok, int64_t(v) * n_idx);
    if (rc != SR_OK) return rc;
    for (size_t i = 0; i < lv.size(); ++i) list_ok[at[i]] = ok[i];
  }
  ctx->mark_phase(3);
  std::vector<double> vden(static_cast<size_t>(n_views)), denoms;
  for (int v = 0; v < n_views; ++v) vden[size_t(v)] = view_denominator<T>(ds, rows_of(v), n_idx);
  if (views) {
    denoms.resize(size_t(nt));
    for (int64_t t = 0; t < nt; ++t) denoms[size_t(t)] = vden[size_t(view_of(t))];
  }
  std::vector<int64_t> fold_list;
  // the in-order fold's results (sr_ctx::ref_fold) and the reference's T denominators per view
  std::vector<T> tden(static_cast<size_t>(n_views));
  FoldResults<T> fres;
  const bool have_fold = ctx->fold_path_last != 0;
  if (have_fold) {
    for (int v = 0; v < n_views; ++v)
      tden[size_t(v)] = (ds->w && n_eval > 0) ? jl_wsum_view<T>(ds, rows_of(v), n_eval) : T(double(n_eval));
    fres.val = reinterpret_cast<const T*>(ctx->h_outs.as<char>() + ctx->outs_fval_off);
    fres.st = reinterpret_cast<const int32_t*>(ctx->h_outs.as<char>() + ctx->outs_fst_off);
    fres.den = [&](int64_t t) { return tden[size_t(view_of(t))]; };
    fres.debug_fail = ctx->fold_debug_fail;
  }
  finalize<T>(nt, sums.data(), flags.data(), vden[0], list.data(), int64_t(list.size()), list_ok.data(),
              static_cast<T*>(out_loss), out_complete, fold_terms(ds, n_eval), &fold_list,
              views ? denoms.data() : nullptr, have_fold ? &fres : nullptr);
  ctx->n_ref_ok_last = fres.n_ok;
  ctx->n_ref_fail_last = fres.n_fail;
  if (have_fold && ctx->fold_stats) {  // (analysis: slow segments, rounds, runs and walk time per folded tree)
    std::vector<int4> st(static_cast<size_t>(nt));
    if (hipMemcpy(st.data(), ctx->fold_dbg.p, st.size() * sizeof(int4), hipMemcpyDeviceToHost) == hipSuccess) {
      int64_t m = 0;
      double a[4] = {0, 0, 0, 0};
      int mx[4] = {0, 0, 0, 0};
      int64_t n_skip = 0;
      for (size_t i = 0; i < st.size(); ++i) {
        int4 v = st[i];
        if (v.x == 0 && v.y == 0 && v.z == 0) continue;
        n_skip += v.x % 1000;  // (x: slow segments x 1000 + those advanced by their steps)
        v.x /= 1000;
        ++m;
        if (v.z < 0)
          std::fprintf(stderr, "[sr fold] tree %zu failed: site %d after %d slow segments, %d rounds, %d us\n", i, -v.z,
                       v.x, v.y, v.w);
        const int w[4] = {v.x, v.y, v.z < 0 ? 0 : v.z, v.w};
        for (int i = 0; i < 4; ++i) {
          a[i] += w[i];
          mx[i] = std::max(mx[i], w[i]);
        }
      }
      std::fprintf(stderr, "[sr fold] path %d: %lld walks, mean/max slow segments %.1f/%d, rounds %.1f/%d, slow-segment us %.1f/%d, walk us %.1f/%d; folded %lld fallback %lld\n",
                   ctx->fold_path_last, (long long)m, m ? a[0] / m : 0.0, mx[0], m ? a[1] / m : 0.0, mx[1],
                   m ? a[2] / m : 0.0, mx[2], m ? a[3] / m : 0.0, mx[3], (long long)fres.n_ok, (long long)fres.n_fail);
      std::fprintf(stderr, "[sr fold] slow segments advanced by their steps (no rows read): %lld\n", (long long)n_skip);
    }
  }
  ctx->n_fold_last = int64_t(fold_list.size());
  ctx->fold_slow_last = ctx->fold_seg_last = 0;
  for (double& v : ctx->fold_ms) v = 0.0;
  for (int v = 0; v < n_views && !fold_list.empty(); ++v) {  // rare: the reference's own fold, in row order (sr_fold.h)
    std::vector<int64_t> fv;
    for (int64_t t : fold_list)
      if (view_of(t) == v) fv.push_back(t);
    if (fv.empty()) continue;
    std::vector<T> fold;
    rc = fold_exact<T>(ctx, ds, opset_id, trees, rows_of(v), n_idx, n_eval, loss_kind, fv, &fold);
    if (rc != SR_OK) return rc;
    // mean: total / count, in T; weighted: total / sum(w), the reference's pairwise Base.sum in T
    const T den = (ds->w && n_eval > 0) ? jl_wsum_view<T>(ds, rows_of(v), n_eval) : T(vden[size_t(v)]);
    for (size_t i = 0; i < fv.size(); ++i) static_cast<T*>(out_loss)[fv[i]] = T(fold[i] / den);
  }
  ctx->mark_phase(4);
  auto t1 = std::chrono::steady_clock::now();
  ctx->last_total_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  (void)n_eval;
  return SR_OK;
}

// The whole call (sr_eval_loss_batch / _views): submit, then finish.
template <typename T>
int eval_loss_impl(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                   const int64_t* row_idx, int64_t n_idx, int loss_kind, void* out_loss, uint8_t* out_complete,
                   const ViewSpec* views = nullptr) {
  LossCall<T> c;
  const int rc = eval_loss_submit<T>(ctx, ds, opset_id, trees, row_idx, n_idx, loss_kind, out_loss, out_complete, views,
                                     &c);
  if (rc != SR_OK) return rc;
  return eval_loss_finish<T>(ctx, c);
}

template <typename T>
int eval_pred_impl(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                   const int64_t* row_idx, int64_t n_idx, void* out_pred, uint8_t* out_complete) {
  const int64_t nt = trees->n_trees;
  if (nt > 0 && (!out_pred || !out_complete)) return set_error(SR_ERR_INVALID_ARG, "NULL output buffers");
  const bool gather = row_idx != nullptr && n_idx > 0;
  const int64_t n_eval = gather ? n_idx : ds->n;
  SrProgramBatch<T> prog;
  Grid g;
  int rc = run_batch<T>(ctx, ds, opset_id, trees, row_idx, n_idx, n_eval, SR_LOSS_L2DIST, SR_MODE_PRED, &prog, &g);
  if (rc != SR_OK) return rc;
  if (nt == 0) return SR_OK;
  hipStream_t s = ctx->stream;
  std::vector<double> sums(static_cast<size_t>(nt));
  std::vector<uint32_t> flags(static_cast<size_t>(nt));
  SR_HIP_CHECK(hipMemcpyAsync(out_pred, ctx->pred.p, size_t(nt) * size_t(n_eval) * sizeof(T), hipMemcpyDeviceToHost, s));
  SR_HIP_CHECK(hipMemcpyAsync(flags.data(), ctx->d_out_flag, size_t(nt) * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  SR_HIP_CHECK(hipStreamSynchronize(s));
  std::vector<int64_t> list;
  for (int64_t t = 0; t < nt; ++t)
    if ((flags[t] & (SR_FLAG_NONFINITE | SR_FLAG_STATIC)) == 0 && (flags[t] & SR_FLAG_BIG)) list.push_back(t);
  std::vector<uint8_t> list_ok;
  rc = exact_list_ok<T>(ctx, ds, prog, row_idx, n_idx, list, &list_ok);
  if (rc != SR_OK) return rc;
  std::vector<T> dummy(static_cast<size_t>(nt));
  finalize<T>(nt, sums.data(), flags.data(), 1.0, list.data(), int64_t(list.size()), list_ok.data(), dummy.data(),
              out_complete);
  // statically incomplete trees have no program: fill their rows with NaN
  T* p = static_cast<T*>(out_pred);
  for (int64_t t = 0; t < nt; ++t)
    if (prog.static_bad[size_t(t)])
      for (int64_t i = 0; i < n_eval; ++i) p[size_t(t) * size_t(n_eval) + size_t(i)] = T(NAN);
  return SR_OK;
}

// The dead-tree probe's rows (sr_dataset::probe_rows): a tree that is non-finite on some row of the
// data is incomplete, and random trees go non-finite first on extreme inputs (exp of the largest
// values, division by and log of the values nearest zero), so those rows lead the probe.  X is
// Julia's column-major [nf, n] on the host.
template <typename T>
std::vector<int64_t> stress_rows(const T* X, int64_t nf, int64_t n) {
  const int64_t K = std::max<int64_t>(1, std::min<int64_t>(100, (kProbeRows * 3 / 4) / (3 * std::max<int64_t>(nf, 1))));
  std::vector<int64_t> pick;
  std::vector<int64_t> idx(static_cast<size_t>(n));
  for (int64_t f = 0; f < nf; ++f) {
    auto val = [&](int64_t i) { return double(X[size_t(i) * size_t(nf) + size_t(f)]); };
    auto mag = [&](int64_t i) { return std::fabs(val(i)); };
    auto take = [&](auto less) {
      for (int64_t i = 0; i < n; ++i) idx[size_t(i)] = i;
      std::nth_element(idx.begin(), idx.begin() + K, idx.end(), less);
      pick.insert(pick.end(), idx.begin(), idx.begin() + K);
    };
    // (NaN values order arbitrarily here; any row is a valid probe row)
    take([&](int64_t a, int64_t b) { return val(a) > val(b); });
    take([&](int64_t a, int64_t b) { return val(a) < val(b); });
    take([&](int64_t a, int64_t b) { return mag(a) < mag(b); });
  }
  std::sort(pick.begin(), pick.end());
  pick.erase(std::unique(pick.begin(), pick.end()), pick.end());
  if (int64_t(pick.size()) > kProbeRows) pick.resize(size_t(kProbeRows));
  for (int64_t i = 0; int64_t(pick.size()) < kProbeRows && i < n; ++i) pick.push_back(i);
  return pick;
}

template <typename T>
int upload_impl(sr_ctx* ctx, const void* X, int64_t nf, int64_t n, const void* y, const void* w, sr_dataset** out) {
  auto* ds = new sr_dataset();
  ds->ctx = ctx;
  ds->dtype = sizeof(T) == 4 ? SR_DTYPE_F32 : SR_DTYPE_F64;
  ds->nf = nf;
  ds->n = n;
  ds->ld = ((n + kRowAlign - 1) / kRowAlign) * kRowAlign;
  hipStream_t s = ctx->stream;
  auto fail = [&](hipError_t e, const char* what) {
    if (ds->X) (void)hipFree(ds->X);
    if (ds->y) (void)hipFree(ds->y);
    if (ds->w) (void)hipFree(ds->w);
    if (ds->probe_rows) (void)hipFree(ds->probe_rows);
    delete ds;
    return set_error(SR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  };
  {
    const T* xh = static_cast<const T*>(X);
    double m = 0.0;
    bool bad = false;
    for (int64_t i = 0; i < nf * n; ++i) {
      const double v = std::fabs(double(xh[i]));
      bad |= !std::isfinite(v);
      m = v > m ? v : m;
    }
    ds->max_abs_x = bad ? double(INFINITY) : m;
  }
  hipError_t e;
  if ((e = hipMalloc(&ds->X, size_t(nf) * size_t(ds->ld) * sizeof(T))) != hipSuccess) return fail(e, "hipMalloc X");
  void* tmp = nullptr;
  if ((e = hipMalloc(&tmp, size_t(nf) * size_t(n) * sizeof(T))) != hipSuccess) return fail(e, "hipMalloc staging");
  if ((e = hipMemcpyAsync(tmp, X, size_t(nf) * size_t(n) * sizeof(T), hipMemcpyHostToDevice, s)) != hipSuccess) {
    (void)hipFree(tmp);
    return fail(e, "copy X");
  }
  if ((e = sr_launch_transpose<T>(static_cast<const T*>(tmp), nf, n, ds->ld, static_cast<T*>(ds->X), s)) != hipSuccess) {
    (void)hipFree(tmp);
    return fail(e, "transpose X");
  }
  if ((e = hipStreamSynchronize(s)) != hipSuccess) {
    (void)hipFree(tmp);
    return fail(e, "sync");
  }
  (void)hipFree(tmp);
  if (y) {
    if ((e = hipMalloc(&ds->y, size_t(ds->ld) * sizeof(T))) != hipSuccess) return fail(e, "hipMalloc y");
    if ((e = hipMemcpyAsync(ds->y, y, size_t(n) * sizeof(T), hipMemcpyHostToDevice, s)) != hipSuccess) return fail(e, "copy y");
    if ((e = sr_launch_pad<T>(static_cast<T*>(ds->y), n, ds->ld, T(0), 1, s)) != hipSuccess) return fail(e, "pad y");
  }
  if (w) {
    const T* wh = static_cast<const T*>(w);
    ds->w_host.resize(size_t(n));
    double sum = 0.0, wmin = INFINITY;
    for (int64_t i = 0; i < n; ++i) {
      ds->w_host[size_t(i)] = double(wh[i]);
      sum += double(wh[i]);
      wmin = std::min(wmin, double(wh[i]));
    }
    ds->wsum = sum;
    ds->w_min = wmin;
    if ((e = hipMalloc(&ds->w, size_t(ds->ld) * sizeof(T))) != hipSuccess) return fail(e, "hipMalloc w");
    if ((e = hipMemcpyAsync(ds->w, w, size_t(n) * sizeof(T), hipMemcpyHostToDevice, s)) != hipSuccess) return fail(e, "copy w");
    if ((e = sr_launch_pad<T>(static_cast<T*>(ds->w), n, ds->ld, T(0), 0, s)) != hipSuccess) return fail(e, "pad w");
  }
  if (n >= 4 * kProbeRows) {
    const std::vector<int64_t> rows = stress_rows<T>(static_cast<const T*>(X), nf, n);
    if ((e = hipMalloc(&ds->probe_rows, rows.size() * sizeof(int64_t))) != hipSuccess) return fail(e, "hipMalloc probe rows");
    if ((e = hipMemcpy(ds->probe_rows, rows.data(), rows.size() * sizeof(int64_t), hipMemcpyHostToDevice)) != hipSuccess)
      return fail(e, "copy probe rows");
    ds->n_probe = int64_t(rows.size());
  }
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail(e, "sync");
  *out = ds;
  return SR_OK;
}

// Batched forward-mode gradient (sr_eval_grad_batch): exact loss + complete flags from the loss
// kernel, then d loss / d constants of every complete tree from the tangent kernel.
// views (may be NULL): several row views in one call (sr_eval_grad_batch_views), as eval_loss_impl.
template <typename T>
int eval_grad_impl(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                   const int64_t* row_idx, int64_t n_idx, int loss_kind, void* out_loss, void* out_grad,
                   uint8_t* out_complete, const ViewSpec* views = nullptr) {
  const SrOpset& ops = ctx->opsets[opset_id];
  for (uint32_t u : ops.unary)
    if (!sr_unary_grad_supported(u)) return set_error(SR_ERR_UNSUPPORTED_OP, "operator without a gradient rule");
  for (uint32_t b : ops.binary)
    if (!sr_binary_grad_supported(b)) return set_error(SR_ERR_UNSUPPORTED_OP, "operator without a gradient rule");
  int lkind = 0;
  double lparam = 0.0;
  if (decode_loss(ctx, loss_kind, &lkind, &lparam) != SR_OK) return SR_ERR_INVALID_ARG;
  int rc = eval_loss_impl<T>(ctx, ds, opset_id, trees, row_idx, n_idx, loss_kind, out_loss, out_complete, views);
  if (rc != SR_OK) return rc;
  const int64_t nt = trees->n_trees;
  if (nt == 0) return SR_OK;
  const bool gather = row_idx != nullptr && n_idx > 0;
  const int64_t n_eval = gather ? n_idx : ds->n;
  const int n_views = (views && gather) ? views->n_views : 1;
  auto view_of = [&](int64_t t) -> int { return n_views > 1 ? int(views->tree_view[t]) : 0; };
  SrProgramBatch<T> prog;
  std::string err;
  rc = sr_compile_batch<T>(*trees, ops, n_eval, ds->nf, true, &prog, &err);
  if (rc != SR_OK) return set_error(rc, err);
  // pre-order constants of every tree (get_scalar_constants order)
  const T* vals = static_cast<const T*>(trees->val);
  std::vector<T> consts;
  consts.reserve(size_t(prog.const_off[size_t(nt)]));
  for (int64_t t = 0; t < nt; ++t)
    for (int64_t i = trees->offsets[t]; i < trees->offsets[t + 1]; ++i)
      if (trees->degree[i] == 0 && trees->constant[i]) consts.push_back(vals[i]);
  T* g = static_cast<T*>(out_grad);
  std::fill(g, g + consts.size(), T(0));
  // work items per tangent width: (tree, first constant)
  // tangent buckets: a tree runs with the narrowest width that holds its constants (1, 2, 4, 8; more
  // than 8: passes of 16), so a one-constant tree carries one tangent, not four
  constexpr int kNB = 5;
  std::vector<uint32_t> items[kNB], k0s[kNB];
  const int kts[kNB] = {1, 2, 4, 8, 16};
  for (int64_t t = 0; t < nt; ++t) {
    const uint32_t nc = prog.n_consts[size_t(t)];
    if (nc == 0 || !out_complete[t]) continue;
    if (nc > 128) return set_error(SR_ERR_TOO_DEEP, "more than 128 constants in one tree");
    const int b = nc <= 1 ? 0 : (nc <= 2 ? 1 : (nc <= 4 ? 2 : (nc <= 8 ? 3 : 4)));
    for (uint32_t k0 = 0; k0 < nc; k0 += uint32_t(kts[b])) {
      items[b].push_back(uint32_t(t));
      k0s[b].push_back(k0);
    }
  }
  // each bucket's items by estimated program cost, longest first (stable): the kWaves waves of a
  // workgroup share every row tile and wait for each other at its barrier, so items of similar cost go
  // together (an item's gradient does not depend on its position: bit-identical either way)
  if (ctx->grad_sort) {
    std::vector<double> tcost(size_t(nt), 0.0);
    for (int64_t t = 0; t < nt; ++t) {
      double c = 0.0;
      for (uint32_t i = prog.offsets[size_t(t)]; i < prog.offsets[size_t(t) + 1]; ++i) {
        const uint32_t opc = prog.code[i].op & SR_OP_MASK;
        const uint32_t u = opc >= SR_OP_UNARY_INF0 ? opc - SR_OP_UNARY_INF0 : opc - SR_OP_UNARY0;
        const bool transc = opc >= SR_OP_UNARY0 && opc < SR_OP_LOAD_DERIVED &&
                            (u == SR_U_EXP || u == SR_U_LOG || u == SR_U_COS || u == SR_U_SIN);
        c += transc ? 5.0 : 1.0;
      }
      tcost[size_t(t)] = c;
    }
    for (int b = 0; b < kNB; ++b) {
      std::vector<size_t> ord(items[b].size());
      for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
      std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return tcost[items[b][x]] > tcost[items[b][y]]; });
      std::vector<uint32_t> it2(ord.size()), k2(ord.size());
      for (size_t i = 0; i < ord.size(); ++i) {
        it2[i] = items[b][ord[i]];
        k2[i] = k0s[b][ord[i]];
      }
      items[b].swap(it2);
      k0s[b].swap(k2);
    }
  }
  hipStream_t s = ctx->stream;
  // the loss pass's in-order folds re-upload their own view's rows: put every view's rows back
  if (gather && ctx->n_fold_last > 0) {
    SR_HIP_CHECK(ctx->row_idx.ensure(size_t(n_views) * size_t(n_idx) * sizeof(int64_t)));
    SR_HIP_CHECK(hipMemcpyAsync(ctx->row_idx.p, row_idx, size_t(n_views) * size_t(n_idx) * sizeof(int64_t),
                                hipMemcpyHostToDevice, s));
  }
  // several views: each bucket's work items ordered by view (stable), one segment per view; the
  // segments' tree groups (kWaves items each) and blocks are laid out below
  constexpr int kWaves = 4;
  std::vector<SrSegment> segs[kNB];
  if (n_views > 1)
    for (int b = 0; b < kNB; ++b) {
      std::vector<size_t> ord(items[b].size());
      for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
      std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return view_of(items[b][x]) < view_of(items[b][y]); });
      std::vector<uint32_t> it2(ord.size()), k2(ord.size());
      for (size_t i = 0; i < ord.size(); ++i) {
        it2[i] = items[b][ord[i]];
        k2[i] = k0s[b][ord[i]];
      }
      items[b].swap(it2);
      k0s[b].swap(k2);
      for (size_t p = 0; p < items[b].size();) {
        const int v = view_of(items[b][p]);
        size_t q = p;
        while (q < items[b].size() && view_of(items[b][q]) == v) ++q;
        SrSegment sg{};
        sg.pos0 = int(p);
        sg.n_pos = int(q - p);
        sg.groups = int((q - p + kWaves - 1) / kWaves);
        sg.row_off = int64_t(v) * n_idx;
        segs[b].push_back(sg);
        p = q;
      }
    }
  // one pinned staging image (programs, offsets, constants, constant offsets, every bucket's work
  // items and segments) -> ONE upload; every bucket's kernel and reduce go out back to back, their
  // results come back in ONE copy, and the host waits once (round 3: four uploads, then per bucket an
  // upload, a copy back and a wait)
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t o_code = 0;
  const size_t o_offs = al(o_code + prog.code.size() * sizeof(SrIns<T>));
  const size_t o_cons = al(o_offs + prog.offsets.size() * sizeof(uint32_t));
  const size_t o_coff = al(o_cons + consts.size() * sizeof(T));
  size_t o_items[kNB], o_vals[kNB], o_segs[kNB];
  size_t at = al(o_coff + prog.const_off.size() * sizeof(uint32_t)), n_vals_all = 0;
  for (int b = 0; b < kNB; ++b) {
    o_items[b] = at;
    at = al(at + 2 * items[b].size() * sizeof(uint32_t));
    o_segs[b] = at;
    at = al(at + segs[b].size() * sizeof(SrSegment));
    o_vals[b] = n_vals_all;
    n_vals_all += items[b].size() * size_t(kts[b]);
  }
  const size_t stage_bytes = at;
  SR_HIP_CHECK(ctx->g_code.ensure(stage_bytes + 16));
  SR_HIP_CHECK(ctx->h_grad.ensure(std::max(stage_bytes, n_vals_all * sizeof(double)) + 16, s, ctx->stream2));
  char* hs = ctx->h_grad.as<char>();
  if (!prog.code.empty()) std::memcpy(hs + o_code, prog.code.data(), prog.code.size() * sizeof(SrIns<T>));
  std::memcpy(hs + o_offs, prog.offsets.data(), prog.offsets.size() * sizeof(uint32_t));
  if (!consts.empty()) std::memcpy(hs + o_cons, consts.data(), consts.size() * sizeof(T));
  std::memcpy(hs + o_coff, prog.const_off.data(), prog.const_off.size() * sizeof(uint32_t));
  for (int b = 0; b < kNB; ++b) {
    uint32_t* d = reinterpret_cast<uint32_t*>(hs + o_items[b]);
    std::copy(items[b].begin(), items[b].end(), d);
    std::copy(k0s[b].begin(), k0s[b].end(), d + items[b].size());
  }
  char* ds_ = ctx->g_code.as<char>();
  SR_HIP_CHECK(ctx->g_out.ensure(n_vals_all * sizeof(double) + 16));
  std::vector<double> vden(static_cast<size_t>(n_views));
  for (int v = 0; v < n_views; ++v) vden[size_t(v)] = view_denominator<T>(ds, gather ? row_idx + int64_t(v) * n_idx : nullptr, n_idx);
  size_t part_need = 0;
  struct Launch { int64_t n_rb, tiles_per_block, n_groups; int rows, depth; };
  Launch lc[kNB] = {};
  for (int b = 0; b < kNB; ++b) {
    const int64_t ni = int64_t(items[b].size());
    if (ni == 0) continue;
    const int kt = kts[b];
    // the bucket's own deepest program sizes its LDS operand stacks; rows per lane drop to 1 when the
    // default's tile + stacks would not fit (many features, Float64, deep trees: ADVICE r3)
    int bdepth = 1;
    for (uint32_t t : items[b]) bdepth = std::max(bdepth, int(prog.depth[t]));
    const int rows = sr_grad_launch_rows(int(sizeof(T)), kt, int(ds->nf), ds->w != nullptr, bdepth, kWaves, kLdsMax,
                                         ctx->grad_rows_force);
    if (rows == 0) return set_error(SR_ERR_TOO_DEEP, "gradient tile needs more than 160 KiB of LDS");
    int64_t n_groups = (ni + kWaves - 1) / kWaves;
    if (!segs[b].empty()) {  // (view-pure groups: a few more than ni / kWaves)
      n_groups = 0;
      for (const SrSegment& sg : segs[b]) n_groups += sg.groups;
    }
    // row blocks in units of 512 rows (64 lanes x the largest rows per lane): they cover the same rows
    // whatever the rows per lane, and a lane accumulates its rows (lane mod 64) in row order inside a
    // block either way, so the gradients are bit-identical for every rows-per-lane choice
    constexpr int64_t kUnit = 512;
    const int64_t n_units = (n_eval + kUnit - 1) / kUnit;
    int64_t n_rb = (4096 + n_groups - 1) / n_groups;
    if (n_rb > n_units) n_rb = n_units;
    if (n_rb < 1) n_rb = 1;
    const int64_t units_per_block = (n_units + n_rb - 1) / n_rb;
    n_rb = (n_units + units_per_block - 1) / units_per_block;
    const int64_t tiles_per_block = units_per_block * (kUnit / int64_t(sr_grad_tile_rows(rows)));
    if (n_rb * n_groups > 0x7fffffff) return set_error(SR_ERR_INVALID_ARG, "grid too large");
    int64_t blk = 0;  // segments' first blocks
    for (SrSegment& sg : segs[b]) {
      sg.block0 = int(blk);
      blk += int64_t(sg.groups) * n_rb;
    }
    if (!segs[b].empty()) std::memcpy(hs + o_segs[b], segs[b].data(), segs[b].size() * sizeof(SrSegment));
    lc[b] = Launch{n_rb, tiles_per_block, n_groups, rows, bdepth};
    part_need = std::max(part_need, size_t(n_rb) * size_t(ni) * size_t(kt));
  }
  SR_HIP_CHECK(hipMemcpyAsync(ds_, hs, stage_bytes, hipMemcpyHostToDevice, s));
  // (buckets run one after another on the stream, so they share the partials buffer)
  SR_HIP_CHECK(ctx->g_part.ensure(part_need * sizeof(double) + 16));
  // algorithmic flops of each bucket's tangent kernel (bench.py's gradient roofline), per row of an
  // item (tree, first tangent) of KT tangents: each unary node 1 (value, transcendentals count 1) +
  // 1 (its derivative) + KT (tangents scaled), each binary node 1 + 2 (partials) + 2 KT (the
  // tangents' product and fused add), and the loss epilogue 3 (d loss / d pred, weight) + KT
  // accumulations; loads move data only
  static_assert(kNB == sr_ctx::kGradBuckets, "gradient buckets");
  for (int b = 0; b < kNB; ++b) {
    ctx->grad_timed[b] = false;
    ctx->grad_items[b] = int64_t(items[b].size());
    ctx->grad_rows[b] = lc[b].rows;
    double per_row = 0.0;
    const double kt = kts[b];
    for (uint32_t t : items[b]) {
      per_row += 3.0 + kt;
      for (uint32_t i = prog.offsets[t]; i < prog.offsets[t + 1]; ++i) {
        const uint32_t opc = prog.code[i].op & SR_OP_MASK;
        if (opc >= SR_OP_BINARY0) per_row += 3.0 + 2.0 * kt;
        else if (opc >= SR_OP_UNARY0 && opc < SR_OP_LOAD_DERIVED) per_row += 2.0 + kt;
      }
    }
    ctx->grad_flops[b] = per_row * double(n_eval);
  }
  for (int b = 0; b < kNB; ++b) {
    const int64_t ni = int64_t(items[b].size());
    if (ni == 0) continue;
    const int kt = kts[b];
    SrGradArgs<T> a{};
    a.code = reinterpret_cast<const SrIns<T>*>(ds_ + o_code);
    a.offsets = reinterpret_cast<const uint32_t*>(ds_ + o_offs);
    a.consts = reinterpret_cast<const T*>(ds_ + o_cons);
    a.const_off = reinterpret_cast<const uint32_t*>(ds_ + o_coff);
    a.item_tree = reinterpret_cast<const uint32_t*>(ds_ + o_items[b]);
    a.item_k0 = a.item_tree + ni;
    a.n_items = int(ni);
    a.X = static_cast<const T*>(ds->X);
    a.y = static_cast<const T*>(ds->y);
    a.w = static_cast<const T*>(ds->w);
    a.row_idx = gather ? ctx->row_idx.as<int64_t>() : nullptr;
    a.ld = ds->ld;
    a.n_rows = n_eval;
    a.nf = int(ds->nf);
    a.tiles_per_block = int(lc[b].tiles_per_block);
    a.n_row_blocks = int(lc[b].n_rb);
    a.n_groups = int(lc[b].n_groups);
    a.stack_depth = lc[b].depth;
    a.loss_kind = lkind;
    a.loss_param = T(lparam);
    a.part = ctx->g_part.as<double>();
    if (!segs[b].empty()) {
      a.segs = reinterpret_cast<const SrSegment*>(ds_ + o_segs[b]);
      a.n_segs = int(segs[b].size());
    }
    if (ctx->timing) SR_HIP_CHECK(hipEventRecord(ctx->ev_g0[b], s));
    SR_HIP_CHECK(sr_launch_grad_any<T>(a, kt, gather, lc[b].rows, int(lc[b].n_rb * lc[b].n_groups), s));
    if (ctx->timing) {
      SR_HIP_CHECK(hipEventRecord(ctx->ev_g1[b], s));
      ctx->grad_timed[b] = true;
    }
    SR_HIP_CHECK(sr_launch_grad_reduce(a.part, int(lc[b].n_rb), int(size_t(ni) * kt), ctx->g_out.as<double>() + o_vals[b], s));
  }
  double* out = ctx->h_grad.as<double>();  // (the staging image is no longer needed: the upload is done)
  SR_HIP_CHECK(hipMemcpyAsync(out, ctx->g_out.p, n_vals_all * sizeof(double), hipMemcpyDeviceToHost, s));
  SR_HIP_CHECK(hipStreamSynchronize(s));
  for (int b = 0; b < kNB; ++b) {
    const int kt = kts[b];
    for (size_t i = 0; i < items[b].size(); ++i) {
      const uint32_t t = items[b][i], k0 = k0s[b][i];
      const uint32_t nc = prog.n_consts[t];
      for (int q = 0; q < kt && k0 + uint32_t(q) < nc; ++q)
        g[prog.const_off[t] + k0 + uint32_t(q)] = T(out[o_vals[b] + i * size_t(kt) + size_t(q)] / vden[size_t(view_of(t))]);
    }
  }
  return SR_OK;
}

int tier_of(const SrOpset& o) {
  auto basic_u = [](uint32_t u) {
    return u == SR_U_NEG || u == SR_U_SQUARE || u == SR_U_CUBE || u == SR_U_EXP || u == SR_U_COS ||
           u == SR_U_SIN || u == SR_U_LOG || u == SR_U_SQRT || u == SR_U_ABS;
  };
  auto basic_b = [](uint32_t b) { return b == SR_B_ADD || b == SR_B_SUB || b == SR_B_MUL || b == SR_B_DIV; };
  for (uint32_t u : o.unary)
    if (!basic_u(u)) return SR_TIER_FULL;
  for (uint32_t b : o.binary)
    if (!basic_b(b)) return SR_TIER_FULL;
  return SR_TIER_BASIC;
}

// ---------------------------------------------------------------- multi-GPU
std::atomic<uint64_t> g_comm_gen{0};

#define SR_NCCL_CHECK(expr)                                                                         \
  do {                                                                                              \
    const ncclResult_t _r = (expr);                                                                 \
    if (_r != ncclSuccess) return set_error(SR_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

// The file a symbol was loaded from (dladdr), with symlinks resolved.
std::string so_path(const void* sym) {
  Dl_info info{};
  if (!dladdr(sym, &info) || !info.dli_fname) return "?";
  char buf[PATH_MAX];
  return realpath(info.dli_fname, buf) ? std::string(buf) : std::string(info.dli_fname);
}
std::string dir_of(const std::string& p) {
  const size_t k = p.rfind('/');
  return k == std::string::npos ? std::string() : p.substr(0, k);
}
// The HIP runtime and the RCCL this library's calls bind to.  The dynamic loader reuses an already
// loaded soname, so when a process loaded torch's bundled ROCm first, the library runs on torch's
// HIP and RCCL, otherwise on /opt/rocm's: either way the two must come from ONE tree, because RCCL
// is handed this library's streams and device buffers.
std::string runtime_paths() {
  return "hip=" + so_path(reinterpret_cast<const void*>(&hipStreamSynchronize)) +
         ";rccl=" + so_path(reinterpret_cast<const void*>(&ncclAllReduce));
}
int check_runtime_pair() {
  const std::string hip = so_path(reinterpret_cast<const void*>(&hipStreamSynchronize));
  const std::string rccl = so_path(reinterpret_cast<const void*>(&ncclAllReduce));
  if (dir_of(hip) != dir_of(rccl))
    return set_error(SR_ERR_HIP, "the HIP runtime (" + hip + ") and RCCL (" + rccl +
                                     ") come from different ROCm trees: RCCL would run this library's streams "
                                     "on another runtime; load libsr_amd before anything else that loads HIP");
  return SR_OK;
}

// The sharded calls' data-path transport: the library's own RCCL communicator over xGMI
// (sr_comm_init), or collectives the caller registers (sr_comm_init_host: host callbacks such as a gloo
// group — several ranks can then share one GPU, and they run this same code).  Buffers are device
// memory on the library's stream; a call returns once its result is usable on that stream.
struct SrComm {
  int nranks = 1, rank = 0;
  virtual ~SrComm() = default;
  virtual const char* kind() const = 0;
  virtual int allreduce_sum(double* d, size_t n, hipStream_t s) = 0;                     // in place
  virtual int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;  // recv[nranks][bytes]
};

struct SrRcclComm final : SrComm {
  ncclComm_t comm = nullptr;
  ~SrRcclComm() override {
    if (comm) (void)ncclCommDestroy(comm);
  }
  const char* kind() const override { return "rccl"; }
  int allreduce_sum(double* d, size_t n, hipStream_t s) override {
    SR_NCCL_CHECK(ncclAllReduce(d, d, n, ncclDouble, ncclSum, comm, s));
    return SR_OK;
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    SR_NCCL_CHECK(ncclAllGather(send, recv, bytes, ncclChar, comm, s));
    return SR_OK;
  }
};

// Host callbacks: the buffers are staged through host memory.  A failed staging copy still calls the
// callback, with this rank's contribution poisoned (NaN bytes): every caller appends an error word to
// its payload, which then reads non-zero on every rank.  A rank never skips a collective its peers
// enter.
struct SrHostComm final : SrComm {
  sr_host_allreduce_fn ar = nullptr;
  sr_host_allgather_fn ag = nullptr;
  void* user = nullptr;
  std::vector<char> h_send, h_recv;
  const char* kind() const override { return "host"; }
  int allreduce_sum(double* d, size_t n, hipStream_t s) override {
    h_send.resize(n * sizeof(double));
    const bool staged = hipMemcpyAsync(h_send.data(), d, h_send.size(), hipMemcpyDeviceToHost, s) == hipSuccess &&
                        hipStreamSynchronize(s) == hipSuccess;
    if (!staged) std::memset(h_send.data(), 0xff, h_send.size());
    if (ar(user, reinterpret_cast<double*>(h_send.data()), int64_t(n)) != 0)
      return set_error(SR_ERR_HIP, "the host all-reduce callback failed");
    SR_HIP_CHECK(hipMemcpyAsync(d, h_send.data(), h_send.size(), hipMemcpyHostToDevice, s));
    SR_HIP_CHECK(hipStreamSynchronize(s));
    return staged ? SR_OK : set_error(SR_ERR_HIP, "staging the all-reduce buffer failed");
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    h_send.resize(bytes);
    h_recv.resize(bytes * size_t(nranks));
    const bool staged = hipMemcpyAsync(h_send.data(), send, bytes, hipMemcpyDeviceToHost, s) == hipSuccess &&
                        hipStreamSynchronize(s) == hipSuccess;
    if (!staged) std::memset(h_send.data(), 0xff, bytes);
    if (ag(user, h_send.data(), h_recv.data(), int64_t(bytes)) != 0)
      return set_error(SR_ERR_HIP, "the host all-gather callback failed");
    SR_HIP_CHECK(hipMemcpyAsync(recv, h_recv.data(), h_recv.size(), hipMemcpyHostToDevice, s));
    SR_HIP_CHECK(hipStreamSynchronize(s));
    return staged ? SR_OK : set_error(SR_ERR_HIP, "staging the all-gather buffer failed");
  }
};

// A buffer of a sharded call's collectives, grown before the collective.  Growth happens on every rank
// at the same call (the sizes depend only on the batch and the number of ranks, and the collective
// buffers serve the collective calls alone), so whether a call grows a buffer is the same on every
// rank; a call that grows one first agrees on the outcome (agree below).  ctx->inject_fail (tests,
// sr_set_tuning "inject_failure") makes the next growths fail on this rank.
struct Prep {
  sr_ctx* ctx;
  bool grew = false;
  int rc = SR_OK;
  std::vector<DevBuf*> touched;
  std::vector<HostBuf*> touched_host;
  bool inject() {
    if (ctx->inject_fail <= 0) return false;
    --ctx->inject_fail;
    return true;
  }
  void fail(hipError_t e) {
    if (e != hipSuccess && rc == SR_OK) rc = set_error(SR_ERR_HIP, std::string("collective buffer: ") + hipGetErrorString(e));
  }
  void need(DevBuf& b, size_t bytes) {
    if (bytes <= b.cap) return;
    grew = true;
    touched.push_back(&b);
    if (rc != SR_OK) return;
    if (inject()) {
      b.release();
      fail(hipErrorOutOfMemory);
    } else {
      fail(b.ensure(bytes));
    }
  }
  void need(HostBuf& b, size_t bytes) {  // (pinned staging of a collective's results)
    if (bytes <= b.cap) return;
    grew = true;
    touched_host.push_back(&b);
    if (rc != SR_OK) return;
    if (inject()) {
      b.release();
      fail(hipErrorOutOfMemory);
    } else {
      fail(b.ensure(bytes, ctx->stream, ctx->stream2));
    }
  }
};

// Every rank's readiness before a collective: one Σ of error words (a rank whose preparation failed
// still enters it), so either every rank proceeds or every rank returns an error.
int agree(sr_ctx* ctx, int local, const char* what = "failed to prepare its collective buffers") {
  hipStream_t s = ctx->stream;
  double* d = ctx->ctl.as<double>();
  double e = local != SR_OK ? 1.0 : 0.0;
  double sum = 0.0;
  bool set = hipMemcpyAsync(d, &e, sizeof(double), hipMemcpyHostToDevice, s) == hipSuccess;
  if (!set) {  // the word must not be stale: poison it synchronously, so every peer sees a non-zero sum
    e = 1.0;
    (void)hipMemcpy(d, &e, sizeof(double), hipMemcpyHostToDevice);
  }
  int rc = ctx->xport->allreduce_sum(d, 1, s);
  bool got = false;
  if (rc == SR_OK) got = hipMemcpyAsync(&sum, d, sizeof(double), hipMemcpyDeviceToHost, s) == hipSuccess &&
                         hipStreamSynchronize(s) == hipSuccess;
  if (local != SR_OK) return local;
  if (!set) return set_error(SR_ERR_HIP, "error word upload failed");
  if (rc != SR_OK) return rc;
  if (!got) return set_error(SR_ERR_HIP, "agreement: copy of the error sum failed");
  if (sum != 0.0) return set_error(SR_ERR_HIP, std::string("a peer rank ") + what);
  return SR_OK;
}
// Grown buffers are agreed on; after a failure every rank releases them, so the next call grows them
// on every rank again (the ranks' buffer states stay identical).
int agree_prep(sr_ctx* ctx, Prep& p) {
  if (!p.grew) return SR_OK;
  const int rc = agree(ctx, p.rc);
  if (rc != SR_OK) {
    for (DevBuf* b : p.touched) b->release();
    for (HostBuf* b : p.touched_host) b->release();
  }
  return rc;
}

constexpr int kLayoutWords = 6;
// Every shard's rows, Σw, max|X| and smallest weight (one all-gather per dataset and communicator; its buffer is
// prepared and agreed on by the caller).  Collective: a local failure still enters the all-gather,
// with its error word set.
int shard_layout(sr_ctx* ctx, const sr_dataset* ds) {
  constexpr int K = kLayoutWords;
  const int nr = ctx->comm_ranks;
  hipStream_t s = ctx->stream;
  // n, Σw, max|X|, weighted, min w, error word
  double mine[K] = {double(ds->n), ds->w ? ds->wsum : 0.0, ds->max_abs_x, ds->w ? 1.0 : 0.0, ds->w ? ds->w_min : 0.0, 0.0};
  double* d = ctx->coll_buf.as<double>();
  if (hipMemcpyAsync(d, mine, sizeof(mine), hipMemcpyHostToDevice, s) != hipSuccess) {
    mine[K - 1] = 1.0;
    (void)hipMemcpy(d, mine, sizeof(mine), hipMemcpyHostToDevice);
  }
  int rc = ctx->xport->allgather(d, d + K, K * sizeof(double), s);
  if (rc != SR_OK) return rc;
  std::vector<double> all(size_t(K) * size_t(nr));
  SR_HIP_CHECK(hipMemcpyAsync(all.data(), d + K, all.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  SR_HIP_CHECK(hipStreamSynchronize(s));
  std::vector<int64_t> offs(size_t(nr) + 1, 0);
  double wsum = 0.0, mx = 0.0, wmin = INFINITY;
  int64_t mn = INT64_MAX;
  int weighted = 0;
  for (int r = 0; r < nr; ++r) {
    const double* a = all.data() + size_t(K) * size_t(r);
    if (a[K - 1] != 0.0) return set_error(SR_ERR_HIP, "the shard layout exchange failed on rank " + std::to_string(r));
    const int64_t n = int64_t(a[0]);
    offs[size_t(r) + 1] = offs[size_t(r)] + n;
    wsum += a[1];
    mx = (a[2] > mx || a[2] != a[2]) ? a[2] : mx;  // NaN / Inf (non-finite data) propagate
    mn = std::min(mn, n);
    weighted += a[3] != 0.0 ? 1 : 0;
    wmin = std::min(wmin, a[4]);
  }
  if (weighted != 0 && weighted != nr) return set_error(SR_ERR_INVALID_ARG, "some shards have weights and some do not");
  if (int64_t(all[size_t(K) * size_t(ctx->comm_rank)]) != ds->n) return set_error(SR_ERR_INVALID_ARG, "shard layout exchange failed");
  ds->shard_offs = offs;
  ds->shard_wsum = wsum;
  ds->shard_w_min = weighted ? wmin : 0.0;
  ds->shard_max_abs_x = (mx != mx) ? double(INFINITY) : mx;
  ds->shard_min_rows = mn;
  ds->shard_gen = ctx->comm_gen;
  return SR_OK;
}

// EXACT verdicts of the listed (BIG-only) trees over the GLOBAL rows of a row-sharded call: each rank
// folds the Julia leaf blocks it holds (sr_jsum_partials' ranges), the folds are all-gathered, and
// every rank adds them in Base.mapreduce_impl's recursion order.  Collective (the list is the same on
// every rank: it comes from the all-reduced flags); a local failure travels in the error word.
template <typename T>
int exact_sharded(sr_ctx* ctx, const sr_dataset* ds, const SrProgramBatch<T>& prog, const std::vector<int64_t>& list,
                  std::vector<uint8_t>* list_ok) {
  list_ok->assign(list.size(), 1);
  int mc = 0;
  for (int64_t t : list) mc = std::max(mc, int(prog.n_checks[size_t(t)]));
  if (list.empty() || mc == 0) return SR_OK;
  const int nr = ctx->comm_ranks, me = ctx->comm_rank;
  const std::vector<int64_t>& offs = ds->shard_offs;
  const int64_t n_total = offs[size_t(nr)];
  if (nr == 1) return exact_list_ok<T>(ctx, ds, prog, nullptr, 0, list, list_ok);  // one shard = the whole view
  std::vector<std::vector<JlRange>> ranges(static_cast<size_t>(nr));
  size_t max_r = 0;
  for (int r = 0; r < nr; ++r) {
    ranges[size_t(r)] = jl_ranges(offs[size_t(r)], offs[size_t(r) + 1] - offs[size_t(r)], n_total);
    max_r = std::max(max_r, ranges[size_t(r)].size());
  }
  const size_t n_arrays = list.size() * size_t(mc);
  // per rank: [n_arrays][its own range count] folds, then an error word (bytes of one double)
  const size_t payload = n_arrays * max_r * sizeof(T);
  const size_t slot = (payload + sizeof(double) + 255) & ~size_t(255);
  std::vector<char> mine(slot, 0);
  int local = run_exact<T>(ctx, ds, prog, nullptr, 0, list.data(), int64_t(list.size()), mc, ranges[size_t(me)],
                           reinterpret_cast<T*>(mine.data()));
  if (local != SR_OK) std::fill(mine.begin(), mine.end(), 0);
  const double err = local != SR_OK ? 1.0 : 0.0;
  std::memcpy(mine.data() + payload, &err, sizeof(double));
  hipStream_t s = ctx->stream;
  Prep prep{ctx};
  prep.need(ctx->coll_buf, slot * size_t(nr + 1));
  int rc = agree_prep(ctx, prep);
  if (rc != SR_OK) return local != SR_OK ? local : rc;
  char* d = ctx->coll_buf.as<char>();
  if (hipMemcpyAsync(d, mine.data(), slot, hipMemcpyHostToDevice, s) != hipSuccess) {
    std::memset(mine.data() + payload, 0xff, sizeof(double));  // (poisoned error word)
    (void)hipMemcpy(d, mine.data(), slot, hipMemcpyHostToDevice);
  }
  rc = ctx->xport->allgather(d, d + slot, slot, s);
  if (rc != SR_OK) return rc;
  std::vector<char> every(slot * size_t(nr));
  // a copy failure here must not leave this rank out of the fold collectives its peers may enter next
  // (the fold list depends on these verdicts): the ranks agree on it first
  int post = SR_OK;
  if (hipMemcpyAsync(every.data(), d + slot, every.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    post = set_error(SR_ERR_HIP, "the exact-sum pass: copy of the gathered folds failed");
  if (ctx->inject_post_exact > 0) {  // tests
    --ctx->inject_post_exact;
    if (post == SR_OK) post = set_error(SR_ERR_HIP, "injected failure after the exact-sum all-gather");
  }
  rc = agree(ctx, post, "failed after the exact-sum all-gather");
  if (rc != SR_OK) return local != SR_OK ? local : rc;
  for (int r = 0; r < nr; ++r) {
    double e = 0.0;
    std::memcpy(&e, every.data() + slot * size_t(r) + payload, sizeof(double));
    if (e != 0.0) return local != SR_OK ? local : set_error(SR_ERR_HIP, "the exact-sum pass failed on rank " + std::to_string(r));
  }
  std::vector<const T*> rank_vals(static_cast<size_t>(nr));
  for (int r = 0; r < nr; ++r) rank_vals[size_t(r)] = reinterpret_cast<const T*>(every.data() + slot * size_t(r));
  std::vector<uint8_t> fin(n_arrays);
  jl_finite<T>(n_total, nr, offs.data(), rank_vals.data(), int64_t(n_arrays), fin.data());
  for (size_t i = 0; i < list.size(); ++i)
    for (int k = 0; k < mc; ++k) (*list_ok)[i] &= fin[i * size_t(mc) + size_t(k)];
  return SR_OK;
}

// One all-gather of `payload` bytes per rank plus an error word (every rank enters it, also after a
// local failure: its payload zeroed, its error word set); every[r] = rank r's payload.  Returns the
// local error, or an error when any rank's word is set.
int gather_checked(sr_ctx* ctx, const void* payload, size_t bytes, int local, std::vector<char>* every, size_t* slot_out,
                   const char* what, int* pending) {
  // a failure of this rank's copy of the gathered payloads is not returned here (its peers have theirs
  // and go on to the next collective): it goes to *pending, which the caller sends in the next
  // collective's error word (or agrees on after the last one)
  if (*pending != SR_OK && local == SR_OK) local = *pending;
  const int nr = ctx->comm_ranks;
  const size_t slot = (bytes + sizeof(double) + 255) & ~size_t(255);
  *slot_out = slot;
  std::vector<char> mine(slot, 0);
  if (local == SR_OK && bytes) std::memcpy(mine.data(), payload, bytes);
  const double err = local != SR_OK ? 1.0 : 0.0;
  std::memcpy(mine.data() + bytes, &err, sizeof(double));
  hipStream_t s = ctx->stream;
  char* d = ctx->coll_buf.as<char>();
  if (hipMemcpyAsync(d, mine.data(), slot, hipMemcpyHostToDevice, s) != hipSuccess) {
    std::memset(mine.data() + bytes, 0xff, sizeof(double));  // (poisoned error word)
    (void)hipMemcpy(d, mine.data(), slot, hipMemcpyHostToDevice);
  }
  int rc = ctx->xport->allgather(d, d + slot, slot, s);
  if (rc != SR_OK) return local != SR_OK ? local : rc;
  every->assign(slot * size_t(nr), 0);
  bool copied = hipMemcpyAsync(every->data(), d + slot, every->size(), hipMemcpyDeviceToHost, s) == hipSuccess;
  copied = hipStreamSynchronize(s) == hipSuccess && copied;
  if (local != SR_OK) return local;
  if (ctx->inject_post_gather > 0 && --ctx->inject_post_gather == 0) copied = false;  // tests: the k-th gather's copy
  if (!copied) {
    *pending = set_error(SR_ERR_HIP, std::string(what) + ": copy of the gathered payloads failed");
    return SR_OK;
  }
  for (int r = 0; r < nr; ++r) {
    double e = 0.0;
    std::memcpy(&e, every->data() + slot * size_t(r) + bytes, sizeof(double));
    if (e != 0.0) return set_error(SR_ERR_HIP, std::string(what) + " failed on rank " + std::to_string(r));
  }
  return SR_OK;
}

// The reference's loss fold of the listed trees over the GLOBAL rows, in row order.  Per batch of trees:
// every rank runs its shard's PRED pass and segment sums in parallel; one all-gather of the shards'
// f64 totals gives each rank the estimate of the fold's value at its first row, and every rank
// tabulates its segments' composed steps in parallel; then the chain runs rank after rank, each
// continuing from the previous shard's fold (one all-gather per rank; a rank's chain is O(1) per
// segment but for the segments where the fold crosses a binade).  Collective; out = the folds (T).
template <typename T>
int fold_sharded(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees, int loss_kind,
                 const std::vector<int64_t>& list, std::vector<T>* out) {
  out->assign(list.size(), T(0));
  if (list.empty()) return SR_OK;
  const int nr = ctx->comm_ranks, me = ctx->comm_rank;
  const std::vector<int64_t>& offs = ds->shard_offs;
  const int64_t n_total = offs[size_t(nr)];
  if (nr == 1) return fold_exact<T>(ctx, ds, opset_id, trees, nullptr, 0, n_total, loss_kind, list, out);
  int64_t max_rows = 0;
  for (int r = 0; r < nr; ++r) max_rows = std::max(max_rows, offs[size_t(r) + 1] - offs[size_t(r)]);
  const int64_t per = fold_batch_trees(max_rows, sizeof(T), false);  // the same cut on every rank
  const size_t max_nb = std::min(list.size(), size_t(per));
  Prep prep{ctx};
  prep.need(ctx->coll_buf, ((max_nb * sizeof(double) + sizeof(double) + 255) & ~size_t(255)) * size_t(nr + 1));
  int rc = agree_prep(ctx, prep);
  if (rc != SR_OK) return rc;
  const int64_t seg_len = fold_seg_len(ctx, ds->n);
  const int64_t n_seg = seg_len > 0 ? (ds->n + seg_len - 1) / seg_len : 0;
  hipStream_t s = ctx->stream;
  KeepCallInfo keep(ctx);
  std::vector<char> every;
  size_t slot = 0;
  int pending = SR_OK;  // a local failure after a gather: sent in the next one's error word
  for (size_t b0 = 0; b0 < list.size(); b0 += size_t(per)) {
    const size_t nb = std::min(list.size() - b0, size_t(per));
    // 1. this shard's predictions and segment sums; its per-tree total
    FoldDev<T> fd;
    int local = fold_prepare<T>(ctx, ds, opset_id, trees, nullptr, 0, n_total, loss_kind, list.data() + b0, nb, seg_len,
                                &fd);
    std::vector<double> tot(nb, 0.0);
    if (local == SR_OK && seg_len > 0) {
      std::vector<double> ss(nb * size_t(n_seg));
      if (hipMemcpyAsync(ss.data(), fd.segsum, ss.size() * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess) {
        local = set_error(SR_ERR_HIP, "fold: segment sums copy failed");
      } else {
        for (size_t b = 0; b < nb; ++b)
          for (int64_t j = 0; j < n_seg; ++j) tot[b] += ss[b * size_t(n_seg) + size_t(j)];
      }
    }
    // 2. every shard's totals -> the f64 sum of the rows before this shard; the composed steps
    rc = gather_checked(ctx, tot.data(), nb * sizeof(double), local, &every, &slot, "the loss fold's shard totals",
                        &pending);
    if (rc != SR_OK) return rc;
    std::vector<double> est(nb, 0.0);
    for (int r = 0; r < me; ++r) {
      const double* v = reinterpret_cast<const double*>(every.data() + slot * size_t(r));
      for (size_t b = 0; b < nb; ++b) est[b] += v[b];
    }
    if (seg_len > 0 && hipMemcpyAsync(fd.carry_est, est.data(), nb * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess)
      local = set_error(SR_ERR_HIP, "fold: estimate upload failed");
    // 3. the chain, shard after shard
    std::vector<T> carry(nb, T(0)), vals(nb, T(0));
    for (int r = 0; r < nr; ++r) {
      if (me == r && local == SR_OK && pending == SR_OK) {
        if (r > 0 && hipMemcpyAsync(fd.carry, carry.data(), nb * sizeof(T), hipMemcpyHostToDevice, s) != hipSuccess)
          local = set_error(SR_ERR_HIP, "fold: carry upload failed");
        if (local == SR_OK) local = fold_finish<T>(ctx, ds, nullptr, 0, loss_kind, nb, seg_len, fd, true, r > 0, vals.data());
      }
      rc = gather_checked(ctx, vals.data(), nb * sizeof(T), me == r ? local : SR_OK, &every, &slot, "the loss fold",
                          &pending);
      if (rc != SR_OK) return local != SR_OK ? local : rc;
      std::memcpy(carry.data(), every.data() + slot * size_t(r), nb * sizeof(T));
    }
    std::copy(carry.begin(), carry.end(), out->begin() + ptrdiff_t(b0));
  }
  release_large_pred(ctx);
  // a failure after the last gather: the ranks agree on it (the weights' sum gather may follow)
  return agree(ctx, pending, "failed in the loss fold");
}

// Every complete tree's in-order loss fold across the shards (sr_ctx::ref_fold; round 6).  The verdicts
// the ranks agreed on after the all-reduce and the exact pass choose the trees (the same bytes on every
// rank); one all-gather of the shards' per-tree f64 totals gives each rank the fold's estimated value at
// its first row; every rank's steps (stored-loss tables, or the plan and the FOLD pass) run in parallel;
// the walks run rank after rank, each from the previous shard's fold values (one all-gather per rank).
// folds / ok: the trees every walk took; *fallback: those some walk failed (the caller folds them
// through the prediction pass).  Collective (every rank enters every gather, also after a failure).
template <typename T>
int fold_all_sharded(sr_ctx* ctx, int64_t nt, const uint8_t* out_complete, const T* out_loss, std::vector<T>* folds,
                     std::vector<uint8_t>* ok, std::vector<int64_t>* fallback) {
  folds->assign(size_t(nt), T(0));
  ok->assign(size_t(nt), 0);
  std::shared_ptr<FoldJob<T>> job = std::static_pointer_cast<FoldJob<T>>(ctx->fold_job);
  ctx->fold_job.reset();
  if (!job || nt == 0) return SR_OK;  // (the ranks decide to fold or not alike: run_batch)
  const int nr = ctx->comm_ranks, me = ctx->comm_rank;
  hipStream_t s = ctx->stream;
  std::vector<uint8_t> elig(static_cast<size_t>(nt));
  bool any = false;
  for (int64_t t = 0; t < nt; ++t) {
    elig[size_t(t)] = ((out_complete[t] & 1) && !(out_complete[t] & SR_COMP_FOLD) && std::isfinite(double(out_loss[t]))) ? 1 : 0;
    any = any || elig[size_t(t)];
  }
  if (!any) return SR_OK;
  const size_t pay = size_t(nt) * (sizeof(T) + sizeof(int32_t));
  Prep prep{ctx};
  prep.need(ctx->coll_buf, ((std::max(size_t(nt) * sizeof(double), pay) + sizeof(double) + 255) & ~size_t(255)) * size_t(nr + 1));
  const size_t o_est = (size_t(nt) + 255) & ~size_t(255), o_car = o_est + ((size_t(nt) * 8 + 255) & ~size_t(255));
  prep.need(ctx->fold_io2, o_car + size_t(nt) * sizeof(T) + 64);
  int rc = agree_prep(ctx, prep);
  if (rc != SR_OK) return rc;
  int local = SR_OK, pending = SR_OK;
  auto hip_local = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && local == SR_OK) local = set_error(SR_ERR_HIP, std::string("fold: ") + what + ": " + hipGetErrorString(e));
  };
  std::vector<double> tot(static_cast<size_t>(nt), 0.0);
  hip_local(hipMemcpyAsync(tot.data(), ctx->d_out_sum, size_t(nt) * sizeof(double), hipMemcpyDeviceToHost, s), "totals copy");
  hip_local(hipStreamSynchronize(s), "totals copy");
  std::vector<char> every;
  size_t slot = 0;
  rc = gather_checked(ctx, tot.data(), size_t(nt) * sizeof(double), local, &every, &slot, "the loss fold's shard totals",
                      &pending);
  if (rc != SR_OK) return rc;
  std::vector<double> est(static_cast<size_t>(nt), 0.0);
  for (int r = 0; r < me; ++r) {
    const double* v = reinterpret_cast<const double*>(every.data() + slot * size_t(r));
    for (int64_t t = 0; t < nt; ++t) est[size_t(t)] += v[t];
  }
  char* io = ctx->fold_io2.as<char>();
  uint8_t* d_elig = reinterpret_cast<uint8_t*>(io);
  double* d_est = reinterpret_cast<double*>(io + o_est);
  T* d_carry = reinterpret_cast<T*>(io + o_car);
  T* d_fval = reinterpret_cast<T*>(ctx->outs.as<char>() + ctx->outs_fval_off);
  int32_t* d_fst = reinterpret_cast<int32_t*>(ctx->outs.as<char>() + ctx->outs_fst_off);
  int step = SR_OK;  // (a failure from here on rides in the next gather's error word)
  auto hip_step = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && step == SR_OK) step = set_error(SR_ERR_HIP, std::string("fold: ") + what + ": " + hipGetErrorString(e));
  };
  hip_step(hipMemcpyAsync(d_elig, elig.data(), size_t(nt), hipMemcpyHostToDevice, s), "verdicts upload");
  hip_step(hipMemcpyAsync(d_est, est.data(), size_t(nt) * sizeof(double), hipMemcpyHostToDevice, s), "estimates upload");
  const SrFoldWho who{ctx->d_out_sum, ctx->d_out_flag, job->n_terms, d_elig, d_est, me == 0 ? 1 : 0};
  if (step == SR_OK && pending == SR_OK)
    for (const FoldRegion<T>& fr : job->regions)
      if (step == SR_OK) step = fold_steps<T>(ctx, *job, fr, who, s);
  std::vector<T> carry(static_cast<size_t>(nt), T(0));
  std::vector<uint8_t> failed(static_cast<size_t>(nt), 0);
  std::vector<char> payload(pay, 0);
  for (int r = 0; r < nr; ++r) {
    if (me == r && step == SR_OK && pending == SR_OK) {
      if (r > 0) hip_step(hipMemcpyAsync(d_carry, carry.data(), size_t(nt) * sizeof(T), hipMemcpyHostToDevice, s), "carry upload");
      for (const FoldRegion<T>& fr : job->regions)
        if (step == SR_OK) step = fold_walk<T>(ctx, *job, fr, who, r > 0 ? d_carry : nullptr, d_fval, d_fst, s);
      hip_step(hipMemcpyAsync(payload.data(), d_fval, size_t(nt) * sizeof(T), hipMemcpyDeviceToHost, s), "walk copy");
      hip_step(hipMemcpyAsync(payload.data() + size_t(nt) * sizeof(T), d_fst, size_t(nt) * sizeof(int32_t),
                              hipMemcpyDeviceToHost, s), "walk copy");
      hip_step(hipStreamSynchronize(s), "walk");
    }
    rc = gather_checked(ctx, payload.data(), pay, me == r ? step : SR_OK, &every, &slot, "the loss fold's walk", &pending);
    if (rc != SR_OK) return rc;
    const char* got = every.data() + slot * size_t(r);
    std::memcpy(carry.data(), got, size_t(nt) * sizeof(T));
    const int32_t* st = reinterpret_cast<const int32_t*>(got + size_t(nt) * sizeof(T));
    for (int64_t t = 0; t < nt; ++t)
      if (elig[size_t(t)] && st[t] != SR_FST_OK) failed[size_t(t)] = 1;
  }
  for (int64_t t = 0; t < nt; ++t) {
    if (!elig[size_t(t)]) continue;
    if (failed[size_t(t)]) {
      fallback->push_back(t);
    } else {
      (*folds)[size_t(t)] = carry[size_t(t)];
      (*ok)[size_t(t)] = 1;
    }
  }
  return agree(ctx, pending, "failed in the loss fold");
}

// Base.sum(w) in T over the GLOBAL rows of a row-sharded dataset: each shard folds its Julia leaf
// blocks (one-row heads continue a block begun on an earlier shard), one all-gather, and every rank
// combines them in Base.mapreduce_impl's recursion order.  Collective.
template <typename T>
int jl_wsum_sharded(sr_ctx* ctx, const sr_dataset* ds, T* out) {
  const int nr = ctx->comm_ranks, me = ctx->comm_rank;
  const std::vector<int64_t>& offs = ds->shard_offs;
  const int64_t n_total = offs[size_t(nr)];
  std::vector<std::vector<JlRange>> ranges(static_cast<size_t>(nr));
  size_t max_r = 0;
  for (int r = 0; r < nr; ++r) {
    ranges[size_t(r)] = jl_ranges(offs[size_t(r)], offs[size_t(r) + 1] - offs[size_t(r)], n_total);
    max_r = std::max(max_r, ranges[size_t(r)].size());
  }
  std::vector<T> mine(max_r, T(0));
  for (size_t i = 0; i < ranges[size_t(me)].size(); ++i) {
    const JlRange& g = ranges[size_t(me)][i];
    T a = T(ds->w_host[size_t(g.lo)]);
    for (int64_t k = g.lo + 1; k <= g.hi; ++k) a = a + T(ds->w_host[size_t(k)]);
    mine[i] = a;
  }
  Prep prep{ctx};
  prep.need(ctx->coll_buf, ((max_r * sizeof(T) + sizeof(double) + 255) & ~size_t(255)) * size_t(nr + 1));
  int rc = agree_prep(ctx, prep);
  if (rc != SR_OK) return rc;
  std::vector<char> every;
  size_t slot = 0;
  int pending = SR_OK;
  rc = gather_checked(ctx, mine.data(), max_r * sizeof(T), SR_OK, &every, &slot, "the weights' sum", &pending);
  if (rc != SR_OK) return rc;
  if (ctx->inject_post_wsum > 0 && --ctx->inject_post_wsum == 0 && pending == SR_OK)  // (tests)
    pending = set_error(SR_ERR_HIP, "injected failure after the weights' sum gather");
  // a local failure after the gather (this rank's copy of it): every rank learns of it and fails
  // together, as after the fold's gathers (a lone failing rank left its peers to enter the
  // next step's all-reduce without it)
  rc = agree(ctx, pending, "failed in the weights' sum");
  if (rc != SR_OK) return rc;
  std::vector<const T*> rank_vals(static_cast<size_t>(nr));
  for (int r = 0; r < nr; ++r) rank_vals[size_t(r)] = reinterpret_cast<const T*>(every.data() + slot * size_t(r));
  std::vector<T> leafval(jl_leaves(n_total).size());
  for (int r = 0; r < nr; ++r) {
    const std::vector<JlRange>& rg = ranges[size_t(r)];
    for (size_t i = 0; i < rg.size(); ++i) {
      T& dst = leafval[size_t(rg[i].leaf)];
      dst = rg[i].head ? T(dst + rank_vals[size_t(r)][i]) : rank_vals[size_t(r)][i];
    }
  }
  size_t idx = 0;
  *out = n_total > 0 ? jl_reduce<T>(leafval, 0, n_total - 1, &idx) : T(0);
  return SR_OK;
}

// The row-sharded step (sr_eval_loss_sharded): this rank's shard through the same launch pipeline as
// a single-GPU call (derived columns, dead-tree probe, two-chunk compile/launch overlap), the packed
// [5, n_trees] partials plus an error word summed by ONE in-place all-reduce on the device, losses
// finalized on the device (Σ / global denominator), the rare BIG-only trees decided by the exact pass
// over the global rows, and the rarer trees whose loss fold the bounds cannot decide folded in row
// order across the shards.  Every rank enters every collective, also after a local failure (its
// partials zeroed, its error word set), and then every rank returns an error.
template <typename T>
int eval_sharded_impl(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees, int loss_kind,
                      T* out_loss, uint8_t* out_complete) {
  const int64_t nt = trees->n_trees;
  const int nr = ctx->comm_ranks;
  const size_t n5 = size_t(5) * size_t(nt);
  // [5][nt] partials | error word, then the finalized losses (T) and complete codes
  const size_t o_loss = ((n5 + 1) * sizeof(double) + 255) & ~size_t(255);
  const size_t o_comp = o_loss + ((size_t(nt) * sizeof(T) + 255) & ~size_t(255));
  // 1. every buffer this call's collectives use, grown (and agreed on) before the first of them
  const bool need_layout = !(ds->shard_gen == ctx->comm_gen && !ds->shard_offs.empty());
  Prep prep{ctx};
  if (need_layout) prep.need(ctx->coll_buf, sizeof(double) * kLayoutWords * size_t(nr + 1));
  prep.need(ctx->coll_packed, o_comp + size_t(nt) + 16);
  int rc = agree_prep(ctx, prep);
  if (rc != SR_OK) return rc;
  // 2. the shards' layout (first call per dataset and communicator)
  if (need_layout) {
    rc = shard_layout(ctx, ds);
    if (rc != SR_OK) return rc;
  }
  const int64_t n_total = ds->shard_offs[size_t(nr)];
  const ShardCtl sc{ds->shard_max_abs_x, ds->shard_min_rows};
  auto t0 = std::chrono::steady_clock::now();
  ctx->start_phases(t0);
  // 3. this shard
  SrProgramBatch<T> prog;
  Grid g;
  ctx->want_fold = true;  // (the in-order fold's steps and walks follow the ranks' agreement, step 6)
  int local = nt > 0 ? run_batch<T>(ctx, ds, opset_id, trees, nullptr, 0, n_total, loss_kind, SR_MODE_LOSS, &prog, &g,
                                    true, &sc)
                     : SR_OK;
  ctx->want_fold = false;
  hipStream_t s = ctx->stream;
  char* base = ctx->coll_packed.as<char>();
  double* dst = reinterpret_cast<double*>(base);
  if (local == SR_OK && nt > 0) {
    const hipError_t e = sr_launch_pack_partials(ctx->d_out_sum, ctx->d_out_flag, int(nt), dst, s);
    if (e != hipSuccess) local = set_error(SR_ERR_HIP, std::string("pack partials: ") + hipGetErrorString(e));
  }
  double err_word = local != SR_OK ? 1.0 : 0.0;
  if (local != SR_OK && hipMemsetAsync(dst, 0, n5 * sizeof(double), s) != hipSuccess) err_word = NAN;
  if (hipMemcpyAsync(dst + n5, &err_word, sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess && local == SR_OK)
    local = set_error(SR_ERR_HIP, "error word upload failed");
  ctx->mark_phase(1);
  // 4. the path's one exchange step: every rank's partials (and error words), summed in place
  rc = ctx->xport->allreduce_sum(dst, n5 + 1, s);
  if (rc != SR_OK) return local != SR_OK ? local : rc;
  const double denom = ds->w ? ds->shard_wsum : double(n_total);
  T* d_loss = reinterpret_cast<T*>(base + o_loss);
  uint8_t* d_comp = reinterpret_cast<uint8_t*>(base + o_comp);
  double err_sum = 0.0;
  // After the all-reduce a local HIP failure must not return on this rank alone: its peers would
  // enter the exact / fold collectives below without it.  The failure rides in `post`, and the ranks
  // agree on it (one Σ of error words) before any further collective.
  int post = SR_OK;
  auto hip_post = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && post == SR_OK) post = set_error(SR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  };
  hip_post(hipMemcpyAsync(&err_sum, dst + n5, sizeof(double), hipMemcpyDeviceToHost, s), "error sum copy");
  const int64_t n_terms = (ds->w && ds->shard_w_min < 0.0) ? 0 : n_total;
  if (post == SR_OK) hip_post(sr_launch_finalize_packed<T>(dst, int(nt), denom, n_terms, d_loss, d_comp, s), "finalize");
  if (nt > 0 && post == SR_OK) {
    hip_post(hipMemcpyAsync(out_loss, d_loss, size_t(nt) * sizeof(T), hipMemcpyDeviceToHost, s), "loss copy");
    hip_post(hipMemcpyAsync(out_complete, d_comp, size_t(nt), hipMemcpyDeviceToHost, s), "flag copy");
  }
  hip_post(hipStreamSynchronize(s), "stream synchronize");
  if (ctx->inject_post > 0) {  // tests: a local failure between the all-reduce and the exact / fold passes
    --ctx->inject_post;
    if (post == SR_OK) post = set_error(SR_ERR_HIP, "injected failure after the all-reduce");
  }
  ctx->timing_pending = local == SR_OK && post == SR_OK && nt > 0;
  if (!ctx->timing_pending) ctx->last_eval_ms = ctx->last_busy_ms = 0.0;
  ctx->mark_phase(2);
  if (nr > 1) {
    rc = agree(ctx, local != SR_OK ? local : post, "failed after the all-reduce");
    if (rc != SR_OK) return local != SR_OK ? local : rc;
  } else if (post != SR_OK) {
    return local != SR_OK ? local : post;
  }
  if (err_sum != 0.0) return local != SR_OK ? local : set_error(SR_ERR_HIP, "the row-sharded step failed on a peer rank");
  // 5. rare: BIG-only trees, DynamicExpressions' exact check over the global rows
  std::vector<int64_t> list;
  for (int64_t t = 0; t < nt; ++t)
    if (out_complete[t] & 2) list.push_back(t);
  std::vector<uint8_t> list_ok;
  ctx->n_exact_last = int64_t(list.size());
  ctx->exact_kernel_ms = 0.0;
  rc = exact_sharded<T>(ctx, ds, prog, list, &list_ok);
  if (rc != SR_OK) return rc;
  for (size_t i = 0; i < list.size(); ++i) {
    const int64_t t = list[i];
    out_complete[t] = uint8_t((out_complete[t] & ~3) | (list_ok[i] ? 1 : 0));
    if (!list_ok[i]) out_loss[t] = T(INFINITY);
  }
  ctx->mark_phase(3);
  // 6. every complete tree's in-order fold across the shards (sr_ctx::ref_fold), and — rarer — the trees
  //    whose fold the overflow band or a failed walk leaves to the prediction pass (sr_fold.h)
  std::vector<int64_t> fold_list;
  std::vector<T> rfold;
  std::vector<uint8_t> rok;
  rc = fold_all_sharded<T>(ctx, nt, out_complete, out_loss, &rfold, &rok, &fold_list);
  if (rc != SR_OK) return rc;
  ctx->n_ref_fail_last = int64_t(fold_list.size());
  ctx->n_ref_ok_last = 0;
  for (uint8_t v : rok) ctx->n_ref_ok_last += v;
  for (int64_t t = 0; t < nt; ++t)
    if ((out_complete[t] & 1) && (out_complete[t] & SR_COMP_FOLD)) fold_list.push_back(t);
  std::sort(fold_list.begin(), fold_list.end());
  ctx->n_fold_last = int64_t(fold_list.size());
  ctx->fold_slow_last = ctx->fold_seg_last = 0;
  for (double& v : ctx->fold_ms) v = 0.0;
  std::vector<T> fold;
  rc = fold_sharded<T>(ctx, ds, opset_id, trees, loss_kind, fold_list, &fold);
  if (rc != SR_OK) return rc;
  // mean: total / count, in T; weighted: total / sum(w), the reference's pairwise Base.sum in T
  T fden = T(denom);
  if (ds->w && (!fold_list.empty() || ctx->n_ref_ok_last > 0)) {  // (the same on every rank)
    rc = nr > 1 ? jl_wsum_sharded<T>(ctx, ds, &fden) : (fden = jl_wsum_view<T>(ds, nullptr, ds->n), SR_OK);
    if (rc != SR_OK) return rc;
  }
  for (size_t i = 0; i < fold_list.size(); ++i) out_loss[fold_list[i]] = T(fold[i] / fden);
  for (int64_t t = 0; t < nt; ++t)
    if (rok[size_t(t)]) out_loss[t] = T(rfold[size_t(t)] / fden);
  for (int64_t t = 0; t < nt; ++t) out_complete[t] &= 1;
  ctx->mark_phase(4);
  ctx->last_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return SR_OK;
}

// Owner rank of every tree for tree sharding: sorted by node count (largest first, stable), dealt in
// snake order 0..N-1, N-1..0, ... (sr_amd.distributed.tree_owners is the same rule).
std::vector<int> tree_owners(const sr_tree_batch* trees, int nr) {
  const int64_t nt = trees->n_trees;
  std::vector<int64_t> order(static_cast<size_t>(nt));
  for (int64_t t = 0; t < nt; ++t) order[size_t(t)] = t;
  auto size_of = [&](int64_t t) { return trees->offsets[t + 1] - trees->offsets[t]; };
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return size_of(a) > size_of(b); });
  std::vector<int> owner(static_cast<size_t>(nt));
  for (int64_t k = 0; k < nt; ++k) {
    const int64_t round = k / nr, pos = k % nr;
    owner[size_t(order[size_t(k)])] = int((round & 1) ? (nr - 1 - pos) : pos);
  }
  return owner;
}

// Tree-sharded scoring (sr_eval_loss_tree_sharded): the dataset is replicated, the trees are split over
// the ranks by estimated cost (tree_owners), each rank scores its own trees with the single-GPU call,
// and ONE all-gather of every rank's results ([loss (T) | complete] of its trees, in tree order, and
// an error word) hands every rank every result.
template <typename T>
int eval_tree_sharded_impl(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees, int loss_kind,
                           T* out_loss, uint8_t* out_complete) {
  const int64_t nt = trees->n_trees;
  const int nr = ctx->comm_ranks, me = ctx->comm_rank;
  const std::vector<int> owner = nr > 1 ? tree_owners(trees, nr) : std::vector<int>(size_t(nt), 0);
  std::vector<std::vector<int64_t>> of(static_cast<size_t>(nr));
  for (int64_t t = 0; t < nt; ++t) of[size_t(owner[size_t(t)])].push_back(t);
  size_t max_cnt = 0;
  for (const auto& v : of) max_cnt = std::max(max_cnt, v.size());
  const size_t o_comp = max_cnt * sizeof(T);
  const size_t o_err = (o_comp + max_cnt + 7) & ~size_t(7);
  const size_t slot = (o_err + sizeof(double) + 255) & ~size_t(255);
  Prep prep{ctx};
  prep.need(ctx->h_coll, slot * size_t(nr + 1));
  prep.need(ctx->coll_buf, slot * size_t(nr + 1));
  int rc = agree_prep(ctx, prep);
  if (rc != SR_OK) return rc;
  const std::vector<int64_t>& mine = of[size_t(me)];
  char* hm = ctx->h_coll.as<char>();  // pinned: this rank's slot, then every rank's
  std::memset(hm, 0, slot);
  int local = SR_OK;
  if (!mine.empty()) {
    T* l = reinterpret_cast<T*>(hm);
    uint8_t* c = reinterpret_cast<uint8_t*>(hm + o_comp);
    if (nr == 1) {  // (one rank owns every tree, in order: no sub-batch)
      local = eval_loss_impl<T>(ctx, ds, opset_id, trees, nullptr, 0, loss_kind, l, c);
    } else {
      SubBatch<T> sub(*trees, mine.data(), mine.size());
      local = eval_loss_impl<T>(ctx, ds, opset_id, &sub.b, nullptr, 0, loss_kind, l, c);
    }
  }
  const double err = local != SR_OK ? 1.0 : 0.0;
  if (local != SR_OK) std::memset(hm, 0, slot);
  std::memcpy(hm + o_err, &err, sizeof(double));
  hipStream_t s = ctx->stream;
  char* d = ctx->coll_buf.as<char>();
  if (hipMemcpyAsync(d, hm, slot, hipMemcpyHostToDevice, s) != hipSuccess) {
    std::memset(hm + o_err, 0xff, sizeof(double));
    (void)hipMemcpy(d, hm, slot, hipMemcpyHostToDevice);
  }
  rc = ctx->xport->allgather(d, d + slot, slot, s);
  if (rc != SR_OK) return local != SR_OK ? local : rc;
  char* every = hm + slot;
  SR_HIP_CHECK(hipMemcpyAsync(every, d + slot, slot * size_t(nr), hipMemcpyDeviceToHost, s));
  SR_HIP_CHECK(hipStreamSynchronize(s));
  for (int r = 0; r < nr; ++r) {
    double e = 0.0;
    std::memcpy(&e, every + slot * size_t(r) + o_err, sizeof(double));
    if (e != 0.0) return local != SR_OK ? local : set_error(SR_ERR_HIP, "tree-sharded scoring failed on rank " + std::to_string(r));
  }
  for (int r = 0; r < nr; ++r) {
    const T* l = reinterpret_cast<const T*>(every + slot * size_t(r));
    const uint8_t* c = reinterpret_cast<const uint8_t*>(every + slot * size_t(r) + o_comp);
    const std::vector<int64_t>& v = of[size_t(r)];
    for (size_t i = 0; i < v.size(); ++i) {
      out_loss[v[i]] = l[i];
      out_complete[v[i]] = c[i] ? 1 : 0;
    }
  }
  return SR_OK;
}

}  // namespace

// ====================================================================== C ABI
extern "C" {

const char* sr_last_error(void) { return g_last_error.c_str(); }
int sr_version(void) { return SR_AMD_VERSION; }

int sr_device_count(int* count) {
  if (!count) return set_error(SR_ERR_INVALID_ARG, "NULL count");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *count = 0;
    return set_error(SR_ERR_NO_DEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *count = c;
  return SR_OK;
}

int sr_init(int device, sr_ctx** out) {
  if (!out) return set_error(SR_ERR_INVALID_ARG, "NULL output");
  *out = nullptr;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess || c <= 0) return set_error(SR_ERR_NO_DEVICE, "no HIP device visible");
  if (device < 0 || device >= c) return set_error(SR_ERR_INVALID_ARG, "device index out of range");
  SR_HIP_CHECK(hipSetDevice(device));
  // SR_AMD_SCHED (A/B only): how the host waits for the device — spin / yield / block
  if (const char* v = std::getenv("SR_AMD_SCHED")) {
    const unsigned f = std::strcmp(v, "spin") == 0    ? hipDeviceScheduleSpin
                       : std::strcmp(v, "yield") == 0 ? hipDeviceScheduleYield
                       : std::strcmp(v, "block") == 0 ? hipDeviceScheduleBlockingSync
                                                      : hipDeviceScheduleAuto;
    const hipError_t e = hipSetDeviceFlags(f);
    if (e != hipSuccess) std::fprintf(stderr, "[sr] hipSetDeviceFlags(%s): %s\n", v, hipGetErrorString(e));
  }
  auto* ctx = new sr_ctx();
  ctx->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->cu_count = prop.multiProcessorCount;
  if (const char* v = std::getenv("SR_AMD_ROWS_PER_LANE")) ctx->rows_override = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_TREES_PER_BLOCK")) ctx->tree_group = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_WAVES")) ctx->waves_override = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_NO_SORT")) ctx->cost_order = std::atoi(v) == 0;
  if (const char* v = std::getenv("SR_AMD_BALANCE")) ctx->balance_groups = std::atoi(v) != 0;
  if (const char* v = std::getenv("SR_AMD_NO_HINT")) ctx->dead_hints = std::atoi(v) == 0;
  // (A/B: the program staging buffer allocated non-coherent, so that kernels reading programs from it
  //  — SR_AMD_HOST_IO=2 — may cache them in L2; the dispatch's acquire makes each call's writes visible)
  if (const char* v = std::getenv("SR_AMD_CHUNKS")) ctx->chunks = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_PROBE")) ctx->probe = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_FOLD_SEG")) ctx->fold_seg = std::atoll(v);
  if (const char* v = std::getenv("SR_AMD_HOST_REDUCE")) ctx->host_reduce = std::atoll(v);
  if (const char* v = std::getenv("SR_AMD_STRESS_PROBE")) ctx->stress_probe = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_CODE_CACHE")) ctx->code_cache = std::atoi(v) != 0 ? 1 : 0;
  if (const char* v = std::getenv("SR_AMD_FUSED_REDUCE")) ctx->fused_reduce = std::atoll(v);
  if (const char* v = std::getenv("SR_AMD_GRAD_ROWS")) ctx->grad_rows_force = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_GRAD_SORT")) ctx->grad_sort = std::atoi(v) != 0 ? 1 : 0;
  if (const char* v = std::getenv("SR_AMD_VSTK_ROWS")) ctx->vstk_rows = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_FIRST_CHUNK")) ctx->first_chunk = std::max(2, std::atoi(v));
  if (const char* v = std::getenv("SR_AMD_CHUNK_MIN")) ctx->chunk_min = std::max<int64_t>(1, std::atoll(v));
  if (const char* v = std::getenv("SR_AMD_HOST_IO")) ctx->host_io = std::atoi(v) != 0 ? 1 : 0;
  if (const char* v = std::getenv("SR_AMD_EXACT_G")) ctx->exact_g = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_EXACT_W")) ctx->exact_w = std::atoi(v) == 1 ? 1 : 4;
  if (const char* v = std::getenv("SR_AMD_EXACT_LIST_HOST")) ctx->exact_list_host = std::atoi(v) != 0 ? 1 : 0;
  if (const char* v = std::getenv("SR_AMD_PAR_STAGE")) ctx->par_stage = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_DERIVED")) ctx->derived = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_MAX_ROW_BLOCKS")) ctx->max_row_blocks = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("SR_AMD_REF_FOLD")) ctx->ref_fold = std::atoi(v) != 0 ? 1 : 0;
  if (const char* v = std::getenv("SR_AMD_FOLD_STORE_MB")) ctx->fold_store_mb = std::max<int64_t>(0, std::atoll(v));
  if (const char* v = std::getenv("SR_AMD_FOLD_SLOT_MB")) ctx->fold_slot_mb = std::max<int64_t>(1, std::atoll(v));
  if (const char* v = std::getenv("SR_AMD_FOLD_STATS")) ctx->fold_stats = std::atoi(v);
  if (const char* v = std::getenv("SR_AMD_FOLD_DELTA_LOG2")) ctx->fold_delta_log2 = std::max(1, std::min(40, std::atoi(v)));
  if (const char* v = std::getenv("SR_AMD_FOLD_SEG_MAX")) ctx->fold_seg_max = std::max<int64_t>(0, std::atoll(v));
  if (const char* v = std::getenv("SR_AMD_FOLD_ROWS_MAX")) ctx->fold_rows_max = std::max<int64_t>(0, std::atoll(v));
  if (const char* v = std::getenv("SR_AMD_FOLD_WALK_DBG")) ctx->fold_walk_dbg = std::atoi(v) & 6;
  if (const char* v = std::getenv("SR_AMD_FOLD_REDUCE")) ctx->fold_reduce = std::atoi(v) != 0 ? 1 : 0;
  if (const char* v = std::getenv("SR_AMD_FOLD_PRE_START")) ctx->fold_pre_start = std::atoi(v) != 0 ? 1 : 0;
  hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e == hipSuccess && std::getenv("SR_AMD_EAGER_STREAM2")) e = ctx->need_stream2();  // (A/B: the round-4 layout)
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreate(&ctx->ev_start);
  if (e == hipSuccess) e = hipEventCreate(&ctx->ev_k0);
  if (e == hipSuccess) e = hipEventCreate(&ctx->ev_k1);
  if (e == hipSuccess) e = hipEventCreate(&ctx->ev_end);
  if (e == hipSuccess) e = hipEventCreate(&ctx->ev_d0);
  if (e == hipSuccess) e = hipEventCreate(&ctx->ev_d1);
  for (int c = 0; c < kMaxChunks; ++c) {
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev_c0[c]);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev_c1[c]);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev_fc0[c]);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev_fc1[c]);
  }
  for (int b = 0; b < sr_ctx::kGradBuckets; ++b) {
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev_g0[b]);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev_g1[b]);
  }
  for (hipEvent_t& ev : ctx->ev_f)
    if (e == hipSuccess) e = hipEventCreate(&ev);
  if (e != hipSuccess) {
    delete ctx;
    return set_error(SR_ERR_HIP, std::string("stream/event creation: ") + hipGetErrorString(e));
  }
  *out = ctx;
  return SR_OK;
}

int sr_shutdown(sr_ctx* ctx) {
  if (!ctx) return SR_OK;
  {
    Lock l(ctx);
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    ctx->xport.reset();
    if (ctx->hint.p == ctx->hint_reserve) {
      ctx->hint.p = nullptr;
      ctx->hint.cap = 0;
    }
    if (ctx->hint_reserve) (void)hipFree(ctx->hint_reserve);
    ctx->hint_reserve = nullptr;
    for (DevBuf* b : {&ctx->prog, &ctx->outs, &ctx->part_sum, &ctx->part_flag, &ctx->pred, &ctx->row_idx, &ctx->tree_list, &ctx->range_lo, &ctx->range_hi, &ctx->range_sums, &ctx->packed,
                      &ctx->hint, &ctx->jsum_prog, &ctx->jsum_scratch, &ctx->probe_sum, &ctx->probe_flag, &ctx->g_code, &ctx->g_offsets, &ctx->g_consts, &ctx->g_const_off,
                      &ctx->g_items, &ctx->g_part, &ctx->g_out, &ctx->derived_cols, &ctx->probe_derived, &ctx->coll_buf, &ctx->coll_packed, &ctx->ctl, &ctx->fold_io, &ctx->group_cnt,
                      &ctx->fold_code, &ctx->fold_tab, &ctx->fold_store, &ctx->fold_ctl, &ctx->fold_io2, &ctx->fold_sq,
                      &ctx->fold_tab2})
      b->release();
    for (HostBuf* b : {&ctx->h_prog, &ctx->h_outs, &ctx->h_grad, &ctx->h_coll, &ctx->h_part, &ctx->h_exact})
      b->release();
    for (int c = 0; c < kMaxChunks; ++c) {
      (void)hipEventDestroy(ctx->ev_c0[c]);
      (void)hipEventDestroy(ctx->ev_c1[c]);
      (void)hipEventDestroy(ctx->ev_fc0[c]);
      (void)hipEventDestroy(ctx->ev_fc1[c]);
    }
    for (int b = 0; b < sr_ctx::kGradBuckets; ++b) {
      (void)hipEventDestroy(ctx->ev_g0[b]);
      (void)hipEventDestroy(ctx->ev_g1[b]);
    }
    for (hipEvent_t ev : ctx->ev_f) (void)hipEventDestroy(ev);
    if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
    (void)hipEventDestroy(ctx->ev_join);
    if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
    (void)hipEventDestroy(ctx->ev_start);
    (void)hipEventDestroy(ctx->ev_k0);
    (void)hipEventDestroy(ctx->ev_k1);
    (void)hipEventDestroy(ctx->ev_end);
    (void)hipEventDestroy(ctx->ev_d0);
    (void)hipEventDestroy(ctx->ev_d1);
    (void)hipStreamDestroy(ctx->stream);
  }
  delete ctx;
  return SR_OK;
}

int sr_register_opset(sr_ctx* ctx, int n_unary, const char* const* unary_names, int n_binary,
                      const char* const* binary_names, int* opset_id) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!opset_id || n_unary < 0 || n_binary < 0 || (n_unary > 0 && !unary_names) || (n_binary > 0 && !binary_names))
    return set_error(SR_ERR_INVALID_ARG, "bad operator name arrays");
  if (n_unary > 255 || n_binary > 255) return set_error(SR_ERR_INVALID_ARG, "more than 255 operators of one degree");
  SrOpset o;
  for (int i = 0; i < n_unary; ++i) {
    const uint32_t id = unary_names[i] ? sr_unary_id(unary_names[i]) : 0;
    if (!id) return set_error(SR_ERR_UNSUPPORTED_OP, std::string("unsupported unary operator: ") +
                                                         (unary_names[i] ? unary_names[i] : "(null)"));
    o.unary.push_back(id);
  }
  for (int i = 0; i < n_binary; ++i) {
    const uint32_t id = binary_names[i] ? sr_binary_id(binary_names[i]) : 0;
    if (!id) return set_error(SR_ERR_UNSUPPORTED_OP, std::string("unsupported binary operator: ") +
                                                         (binary_names[i] ? binary_names[i] : "(null)"));
    o.binary.push_back(id);
  }
  Lock l(ctx);
  ctx->opsets.push_back(o);
  ctx->tiers.push_back(tier_of(o));
  *opset_id = int(ctx->opsets.size()) - 1;
  return SR_OK;
}

int sr_register_loss(sr_ctx* ctx, int kind, double param, int* loss_code) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!loss_code || kind < 0 || kind >= SR_LOSS_COUNT) return set_error(SR_ERR_INVALID_ARG, "unknown loss kind");
  if (!std::isfinite(param)) return set_error(SR_ERR_INVALID_ARG, "loss parameter must be finite");
  Lock l(ctx);
  for (size_t i = 0; i < ctx->losses.size(); ++i)
    if (ctx->losses[i].first == kind && ctx->losses[i].second == param) {
      *loss_code = kLossCodeBase + int(i);
      return SR_OK;
    }
  ctx->losses.emplace_back(kind, param);
  *loss_code = kLossCodeBase + int(ctx->losses.size()) - 1;
  return SR_OK;
}

int sr_dataset_upload(sr_ctx* ctx, int dtype, const void* X, int64_t nfeatures, int64_t n, const void* y,
                      const void* weights, sr_dataset** out) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!out || !X || nfeatures <= 0 || n <= 0) return set_error(SR_ERR_INVALID_ARG, "bad dataset arguments");
  if (nfeatures > 65535) return set_error(SR_ERR_INVALID_ARG, "nfeatures exceeds Node.feature (UInt16)");
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  if (dtype == SR_DTYPE_F32) return upload_impl<float>(ctx, X, nfeatures, n, y, weights, out);
  if (dtype == SR_DTYPE_F64) return upload_impl<double>(ctx, X, nfeatures, n, y, weights, out);
  return set_error(SR_ERR_INVALID_ARG, "unknown dtype");
}

int sr_dataset_free(sr_dataset* ds) {
  if (!ds) return SR_OK;
  if (ds->ctx) {
    Lock l(ds->ctx);
    (void)hipSetDevice(ds->ctx->device);
    (void)hipStreamSynchronize(ds->ctx->stream);
    if (ds->X) (void)hipFree(ds->X);
    if (ds->y) (void)hipFree(ds->y);
    if (ds->w) (void)hipFree(ds->w);
    if (ds->probe_rows) (void)hipFree(ds->probe_rows);
  }
  delete ds;
  return SR_OK;
}

int sr_dataset_info(const sr_dataset* ds, int* dtype, int64_t* nfeatures, int64_t* n) {
  if (!ds) return set_error(SR_ERR_INVALID_ARG, "NULL dataset");
  if (dtype) *dtype = ds->dtype;
  if (nfeatures) *nfeatures = ds->nf;
  if (n) *n = ds->n;
  return SR_OK;
}

int sr_dataset_denominator(const sr_dataset* ds, double* denom) {
  if (!ds || !denom) return set_error(SR_ERR_INVALID_ARG, "NULL argument");
  *denom = ds->w ? ds->wsum : double(ds->n);
  return SR_OK;
}

int sr_eval_loss_batch(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                       const int64_t* row_idx, int64_t n_idx, int loss_kind, void* out_loss, uint8_t* out_complete) {
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  if (ds->dtype == SR_DTYPE_F32)
    return eval_loss_impl<float>(ctx, ds, opset_id, trees, row_idx, n_idx, loss_kind, out_loss, out_complete);
  return eval_loss_impl<double>(ctx, ds, opset_id, trees, row_idx, n_idx, loss_kind, out_loss, out_complete);
}

// several row views in one call (per-island minibatches): validated here, ViewSpec below the ABI
static int check_views(const sr_tree_batch* trees, const int32_t* tree_view, int n_views, const int64_t* view_rows,
                       int64_t view_len) {
  if (n_views < 1 || view_len < 1 || !view_rows || (trees->n_trees > 0 && !tree_view))
    return set_error(SR_ERR_INVALID_ARG, "bad row views");
  return SR_OK;
}

int sr_eval_loss_batch_views(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                             const int32_t* tree_view, int n_views, const int64_t* view_rows, int64_t view_len,
                             int loss_kind, void* out_loss, uint8_t* out_complete) {
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  if ((rc = check_views(trees, tree_view, n_views, view_rows, view_len)) != SR_OK) return rc;
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  const ViewSpec vs{tree_view, n_views, view_len};
  const ViewSpec* v = n_views > 1 ? &vs : nullptr;  // (one view: the plain gather path)
  if (ds->dtype == SR_DTYPE_F32)
    return eval_loss_impl<float>(ctx, ds, opset_id, trees, view_rows, view_len, loss_kind, out_loss, out_complete, v);
  return eval_loss_impl<double>(ctx, ds, opset_id, trees, view_rows, view_len, loss_kind, out_loss, out_complete, v);
}

int sr_eval_grad_batch_views(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                             const int32_t* tree_view, int n_views, const int64_t* view_rows, int64_t view_len,
                             int loss_kind, void* out_loss, void* out_grad, uint8_t* out_complete) {
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  if ((rc = check_views(trees, tree_view, n_views, view_rows, view_len)) != SR_OK) return rc;
  if (trees->n_trees > 0 && (!out_loss || !out_grad || !out_complete))
    return set_error(SR_ERR_INVALID_ARG, "NULL output buffers");
  if (!ds->y) return set_error(SR_ERR_INVALID_ARG, "dataset has no y");
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  const ViewSpec vs{tree_view, n_views, view_len};
  const ViewSpec* v = n_views > 1 ? &vs : nullptr;
  if (ds->dtype == SR_DTYPE_F32)
    return eval_grad_impl<float>(ctx, ds, opset_id, trees, view_rows, view_len, loss_kind, out_loss, out_grad,
                                 out_complete, v);
  return eval_grad_impl<double>(ctx, ds, opset_id, trees, view_rows, view_len, loss_kind, out_loss, out_grad,
                                out_complete, v);
}

int sr_eval_tree_array(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                       const int64_t* row_idx, int64_t n_idx, void* out_pred, uint8_t* out_complete) {
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  if (ds->dtype == SR_DTYPE_F32)
    return eval_pred_impl<float>(ctx, ds, opset_id, trees, row_idx, n_idx, out_pred, out_complete);
  return eval_pred_impl<double>(ctx, ds, opset_id, trees, row_idx, n_idx, out_pred, out_complete);
}

int sr_eval_loss_partials(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                          int64_t n_total, int loss_kind, double* out_sum, uint32_t* out_flags, int out_on_device) {
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  const int64_t nt = trees->n_trees;
  if (nt > 0 && (!out_sum || !out_flags)) return set_error(SR_ERR_INVALID_ARG, "NULL output buffers");
  if (n_total < ds->n) return set_error(SR_ERR_INVALID_ARG, "n_total smaller than this shard");
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  Grid g;
  auto t0 = std::chrono::steady_clock::now();
  if (ds->dtype == SR_DTYPE_F32) {
    SrProgramBatch<float> prog;
    rc = run_batch<float>(ctx, ds, opset_id, trees, nullptr, 0, n_total, loss_kind, SR_MODE_LOSS, &prog, &g);
  } else {
    SrProgramBatch<double> prog;
    rc = run_batch<double>(ctx, ds, opset_id, trees, nullptr, 0, n_total, loss_kind, SR_MODE_LOSS, &prog, &g);
  }
  if (rc != SR_OK || nt == 0) return rc;
  hipStream_t s = ctx->stream;
  const hipMemcpyKind kind = out_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  SR_HIP_CHECK(hipMemcpyAsync(out_sum, ctx->d_out_sum, size_t(nt) * sizeof(double), kind, s));
  SR_HIP_CHECK(hipMemcpyAsync(out_flags, ctx->d_out_flag, size_t(nt) * sizeof(uint32_t), kind, s));
  SR_HIP_CHECK(hipStreamSynchronize(s));
  ctx->timing_pending = true;
  ctx->last_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return SR_OK;
}

int sr_eval_loss_partials_packed(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                                 int64_t n_total, int loss_kind, double* out, int out_on_device) {
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  const int64_t nt = trees->n_trees;
  if (nt > 0 && !out) return set_error(SR_ERR_INVALID_ARG, "NULL output buffer");
  if (n_total < ds->n) return set_error(SR_ERR_INVALID_ARG, "n_total smaller than this shard");
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  Grid g;
  auto t0 = std::chrono::steady_clock::now();
  if (ds->dtype == SR_DTYPE_F32) {
    SrProgramBatch<float> prog;
    rc = run_batch<float>(ctx, ds, opset_id, trees, nullptr, 0, n_total, loss_kind, SR_MODE_LOSS, &prog, &g);
  } else {
    SrProgramBatch<double> prog;
    rc = run_batch<double>(ctx, ds, opset_id, trees, nullptr, 0, n_total, loss_kind, SR_MODE_LOSS, &prog, &g);
  }
  if (rc != SR_OK || nt == 0) return rc;
  hipStream_t s = ctx->stream;
  const size_t bytes = size_t(5) * size_t(nt) * sizeof(double);
  double* dst = out;
  if (!out_on_device) {
    SR_HIP_CHECK(ctx->packed.ensure(bytes));
    dst = ctx->packed.as<double>();
  }
  SR_HIP_CHECK(sr_launch_pack_partials(ctx->d_out_sum, ctx->d_out_flag, int(nt), dst, s));
  if (!out_on_device) SR_HIP_CHECK(hipMemcpyAsync(out, dst, bytes, hipMemcpyDeviceToHost, s));
  SR_HIP_CHECK(hipStreamSynchronize(s));
  ctx->timing_pending = true;
  ctx->last_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return SR_OK;
}

int sr_comm_unique_id(void* out_id) {
  if (!out_id) return set_error(SR_ERR_INVALID_ARG, "NULL output");
  if (check_runtime_pair() != SR_OK) return SR_ERR_HIP;
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return set_error(SR_ERR_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  static_assert(sizeof(id) == SR_COMM_ID_BYTES, "RCCL unique id size");
  std::memcpy(out_id, &id, sizeof(id));
  return SR_OK;
}

// A fresh transport: the collective buffers restart empty (every rank of the new group alike), shard
// layouts are re-exchanged (new generation).
static int install_comm(sr_ctx* ctx, std::unique_ptr<SrComm> x, int nranks, int rank) {
  for (DevBuf* b : {&ctx->coll_buf, &ctx->coll_packed}) b->release();
  ctx->h_coll.release();
  SR_HIP_CHECK(ctx->ctl.ensure(256));
  x->nranks = nranks;
  x->rank = rank;
  ctx->xport = std::move(x);
  ctx->comm_ranks = nranks;
  ctx->comm_rank = rank;
  ctx->comm_gen = ++g_comm_gen;
  return SR_OK;
}

int sr_comm_init(sr_ctx* ctx, int nranks, int rank, const void* id_bytes) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!id_bytes || nranks < 1 || rank < 0 || rank >= nranks) return set_error(SR_ERR_INVALID_ARG, "bad communicator arguments");
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  ctx->xport.reset();
  ctx->comm_ranks = 0;
  if (check_runtime_pair() != SR_OK) return SR_ERR_HIP;
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, sizeof(id));
  auto x = std::make_unique<SrRcclComm>();
  const ncclResult_t r = ncclCommInitRank(&x->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    x->comm = nullptr;
    return set_error(SR_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  return install_comm(ctx, std::move(x), nranks, rank);
}

int sr_comm_init_host(sr_ctx* ctx, int nranks, int rank, sr_host_allreduce_fn allreduce, sr_host_allgather_fn allgather,
                      void* user) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!allreduce || !allgather || nranks < 1 || rank < 0 || rank >= nranks)
    return set_error(SR_ERR_INVALID_ARG, "bad host communicator arguments");
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  ctx->xport.reset();
  ctx->comm_ranks = 0;
  auto x = std::make_unique<SrHostComm>();
  x->ar = allreduce;
  x->ag = allgather;
  x->user = user;
  return install_comm(ctx, std::move(x), nranks, rank);
}

int sr_comm_destroy(sr_ctx* ctx) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  Lock l(ctx);
  ctx->xport.reset();
  ctx->comm_ranks = 0;
  return SR_OK;
}

// Row-sharded step with the exchange on the device: this shard's packed [5, n_trees] partials
// (sr_eval_loss_partials_packed) summed over every rank by ONE in-place all-reduce on the library's
// stream, then copied to out_host (every rank gets the global sums and flag counts).
int sr_eval_loss_partials_allreduce(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                                    int64_t n_total, int loss_kind, double* out_host) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!ctx->xport) return set_error(SR_ERR_INVALID_ARG, "no communicator: call sr_comm_init first");
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  const int64_t nt = trees->n_trees;
  if (nt > 0 && !out_host) return set_error(SR_ERR_INVALID_ARG, "NULL output buffer");
  if (n_total < ds->n) return set_error(SR_ERR_INVALID_ARG, "n_total smaller than this shard");
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  const size_t n = size_t(5) * size_t(nt > 0 ? nt : 0);
  Prep prep{ctx};
  prep.need(ctx->coll_packed, (n + 1) * sizeof(double));
  rc = agree_prep(ctx, prep);
  if (rc != SR_OK) return rc;
  Grid g;
  auto t0 = std::chrono::steady_clock::now();
  if (ds->dtype == SR_DTYPE_F32) {
    SrProgramBatch<float> prog;
    rc = run_batch<float>(ctx, ds, opset_id, trees, nullptr, 0, n_total, loss_kind, SR_MODE_LOSS, &prog, &g);
  } else {
    SrProgramBatch<double> prog;
    rc = run_batch<double>(ctx, ds, opset_id, trees, nullptr, 0, n_total, loss_kind, SR_MODE_LOSS, &prog, &g);
  }
  int local = rc;
  hipStream_t s = ctx->stream;
  double* dst = ctx->coll_packed.as<double>();
  if (local == SR_OK && nt > 0 && sr_launch_pack_partials(ctx->d_out_sum, ctx->d_out_flag, int(nt), dst, s) != hipSuccess)
    local = set_error(SR_ERR_HIP, "pack partials failed");
  // every rank enters the collective, also with an empty batch (the counts agree: same trees) and
  // after a local failure (partials zeroed, the error word after them set): then every rank fails
  double err_word = local != SR_OK ? 1.0 : 0.0;
  if (local != SR_OK && hipMemsetAsync(dst, 0, n * sizeof(double), s) != hipSuccess) err_word = NAN;
  (void)hipMemcpyAsync(dst + n, &err_word, sizeof(double), hipMemcpyHostToDevice, s);
  rc = ctx->xport->allreduce_sum(dst, n + 1, s);
  if (rc != SR_OK) return local != SR_OK ? local : rc;
  double err_sum = 0.0;
  SR_HIP_CHECK(hipMemcpyAsync(&err_sum, dst + n, sizeof(double), hipMemcpyDeviceToHost, s));
  if (nt > 0) SR_HIP_CHECK(hipMemcpyAsync(out_host, dst, n * sizeof(double), hipMemcpyDeviceToHost, s));
  SR_HIP_CHECK(hipStreamSynchronize(s));
  if (err_sum != 0.0) return local != SR_OK ? local : set_error(SR_ERR_HIP, "the row-sharded step failed on a peer rank");
  ctx->timing_pending = true;
  ctx->last_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return SR_OK;
}

int sr_eval_loss_sharded(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees, int loss_kind,
                         void* out_loss, uint8_t* out_complete) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!ctx->xport) return set_error(SR_ERR_INVALID_ARG, "no communicator: call sr_comm_init first");
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  if (trees->n_trees > 0 && (!out_loss || !out_complete)) return set_error(SR_ERR_INVALID_ARG, "NULL output buffers");
  if (!ds->y) return set_error(SR_ERR_INVALID_ARG, "dataset has no y");
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  if (ds->dtype == SR_DTYPE_F32)
    return eval_sharded_impl<float>(ctx, ds, opset_id, trees, loss_kind, static_cast<float*>(out_loss), out_complete);
  return eval_sharded_impl<double>(ctx, ds, opset_id, trees, loss_kind, static_cast<double*>(out_loss), out_complete);
}

int sr_eval_loss_tree_sharded(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                              int loss_kind, void* out_loss, uint8_t* out_complete) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!ctx->xport) return set_error(SR_ERR_INVALID_ARG, "no communicator: call sr_comm_init first");
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  if (trees->n_trees > 0 && (!out_loss || !out_complete)) return set_error(SR_ERR_INVALID_ARG, "NULL output buffers");
  if (trees->n_trees > 0 && !trees->offsets) return set_error(SR_ERR_INVALID_ARG, "sr_tree_batch has NULL arrays");
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  if (ds->dtype == SR_DTYPE_F32)
    return eval_tree_sharded_impl<float>(ctx, ds, opset_id, trees, loss_kind, static_cast<float*>(out_loss), out_complete);
  return eval_tree_sharded_impl<double>(ctx, ds, opset_id, trees, loss_kind, static_cast<double*>(out_loss), out_complete);
}

int sr_comm_info(sr_ctx* ctx, int* nranks, int* rank, char* paths, int64_t capacity) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  Lock l(ctx);
  if (nranks || rank) {
    if (!ctx->xport) return set_error(SR_ERR_INVALID_ARG, "no communicator: call sr_comm_init first");
    int c = ctx->comm_ranks, r = ctx->comm_rank;
    if (auto* rc = dynamic_cast<SrRcclComm*>(ctx->xport.get())) {  // as RCCL itself reports them
      SR_NCCL_CHECK(ncclCommCount(rc->comm, &c));
      SR_NCCL_CHECK(ncclCommUserRank(rc->comm, &r));
    }
    if (nranks) *nranks = c;
    if (rank) *rank = r;
  }
  if (paths && capacity > 0 && ctx->xport) {  // "transport=rccl|host;hip=...;rccl=..."
    const std::string p = std::string("transport=") + ctx->xport->kind() + ";" + runtime_paths();
    const size_t n = std::min(p.size(), size_t(capacity - 1));
    std::memcpy(paths, p.data(), n);
    paths[n] = '\0';
    return SR_OK;
  }
  return sr_runtime_info(paths, capacity);
}

int sr_runtime_info(char* paths, int64_t capacity) {
  if (!paths || capacity <= 0) return SR_OK;
  const std::string p = runtime_paths();
  const size_t n = std::min(p.size(), size_t(capacity - 1));
  std::memcpy(paths, p.data(), n);
  paths[n] = '\0';
  return SR_OK;
}

int sr_max_checks(sr_ctx* ctx, int dtype, int opset_id, const sr_tree_batch* trees, int* max_checks) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!trees || !max_checks || opset_id < 0 || opset_id >= int(ctx->opsets.size()) ||
      (dtype != SR_DTYPE_F32 && dtype != SR_DTYPE_F64))
    return set_error(SR_ERR_INVALID_ARG, "bad arguments");
  // compiled in the batch's own element type (`val` holds T): the same programs the eval calls build
  std::string err;
  auto go = [&](auto tag) -> int {
    using T = decltype(tag);
    SrProgramBatch<T> prog;
    const int rc = sr_compile_batch<T>(*trees, ctx->opsets[opset_id], 1, 65535, false, &prog, &err);
    if (rc != SR_OK) return set_error(rc, err);
    *max_checks = prog.max_checks;
    return SR_OK;
  };
  return dtype == SR_DTYPE_F32 ? go(0.0f) : go(0.0);
}

int sr_jsum_range_count(int64_t row_offset, int64_t n_local, int64_t n_total, int64_t* out_n_ranges) {
  if (!out_n_ranges || row_offset < 0 || n_local < 1 || row_offset + n_local > n_total)
    return set_error(SR_ERR_INVALID_ARG, "bad shard bounds");
  *out_n_ranges = int64_t(jl_ranges(row_offset, n_local, n_total).size());
  return SR_OK;
}

int sr_jsum_ranges(int64_t row_offset, int64_t n_local, int64_t n_total, int64_t* lo, int64_t* hi, int64_t* leaf,
                   uint8_t* head) {
  if (row_offset < 0 || n_local < 1 || row_offset + n_local > n_total) return set_error(SR_ERR_INVALID_ARG, "bad shard bounds");
  const std::vector<JlRange> r = jl_ranges(row_offset, n_local, n_total);
  for (size_t i = 0; i < r.size(); ++i) {
    if (lo) lo[i] = r[i].lo;
    if (hi) hi[i] = r[i].hi;
    if (leaf) leaf[i] = r[i].leaf;
    if (head) head[i] = r[i].head ? 1 : 0;
  }
  return SR_OK;
}

int sr_jsum_partials(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                     const int64_t* tree_list, int64_t n_list, int max_checks, int64_t row_offset, int64_t n_total,
                     void* out_vals) {
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  if (n_list < 0 || (n_list > 0 && (!tree_list || !out_vals)) || max_checks < 0)
    return set_error(SR_ERR_INVALID_ARG, "bad tree list");
  if (row_offset < 0 || row_offset + ds->n > n_total) return set_error(SR_ERR_INVALID_ARG, "bad shard bounds");
  for (int64_t i = 0; i < n_list; ++i)
    if (tree_list[i] < 0 || tree_list[i] >= trees->n_trees) return set_error(SR_ERR_INVALID_ARG, "tree index out of range");
  if (n_list == 0 || max_checks == 0) return SR_OK;
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  Grid g;
  const std::vector<JlRange> ranges = jl_ranges(row_offset, ds->n, n_total);
  auto go = [&](auto tag) -> int {
    using T = decltype(tag);
    SrProgramBatch<T> prog;
    int r = run_batch<T>(ctx, ds, opset_id, trees, nullptr, 0, n_total, SR_LOSS_L2DIST, SR_MODE_LOSS, &prog, &g);
    if (r != SR_OK) return r;
    SR_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (prog.max_checks > max_checks) return set_error(SR_ERR_INVALID_ARG, "max_checks too small");
    return run_exact<T>(ctx, ds, prog, nullptr, 0, tree_list, n_list, max_checks, ranges, static_cast<T*>(out_vals));
  };
  return ds->dtype == SR_DTYPE_F32 ? go(float{}) : go(double{});
}

int sr_jsum_finite(int dtype, int64_t n_total, int n_ranks, const int64_t* row_offsets, const void* const* rank_vals,
                   int64_t n_arrays, uint8_t* out_finite) {
  if (n_total < 1 || n_ranks < 1 || !row_offsets || !rank_vals || n_arrays < 0 || (n_arrays > 0 && !out_finite))
    return set_error(SR_ERR_INVALID_ARG, "bad arguments");
  if (row_offsets[0] != 0 || row_offsets[n_ranks] != n_total) return set_error(SR_ERR_INVALID_ARG, "shards must cover [0, n_total)");
  for (int r = 0; r < n_ranks; ++r)
    if (row_offsets[r + 1] <= row_offsets[r] || !rank_vals[r]) return set_error(SR_ERR_INVALID_ARG, "bad shard bounds");
  if (dtype == SR_DTYPE_F32)
    jl_finite<float>(n_total, n_ranks, row_offsets, reinterpret_cast<const float* const*>(rank_vals), n_arrays, out_finite);
  else if (dtype == SR_DTYPE_F64)
    jl_finite<double>(n_total, n_ranks, row_offsets, reinterpret_cast<const double* const*>(rank_vals), n_arrays,
                      out_finite);
  else
    return set_error(SR_ERR_INVALID_ARG, "unknown dtype");
  return SR_OK;
}

int sr_finalize_losses(int dtype, int64_t n_trees, const double* sums, const uint32_t* flags, double denom,
                       const int64_t* tree_list, int64_t n_list, const uint8_t* list_ok, void* out_loss,
                       uint8_t* out_complete) {
  if (n_trees < 0 || (n_trees > 0 && (!sums || !flags || !out_loss || !out_complete)))
    return set_error(SR_ERR_INVALID_ARG, "bad arguments");
  if (n_list > 0 && (!tree_list || !list_ok)) return set_error(SR_ERR_INVALID_ARG, "NULL tree list");
  for (int64_t i = 0; i < n_list; ++i)
    if (tree_list[i] < 0 || tree_list[i] >= n_trees) return set_error(SR_ERR_INVALID_ARG, "tree index out of range");
  if (dtype == SR_DTYPE_F32)
    finalize<float>(n_trees, sums, flags, denom, tree_list, n_list, list_ok, static_cast<float*>(out_loss), out_complete);
  else if (dtype == SR_DTYPE_F64)
    finalize<double>(n_trees, sums, flags, denom, tree_list, n_list, list_ok, static_cast<double*>(out_loss),
                     out_complete);
  else
    return set_error(SR_ERR_INVALID_ARG, "unknown dtype");
  return SR_OK;
}

int sr_eval_grad_batch(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                       const int64_t* row_idx, int64_t n_idx, int loss_kind, void* out_loss, void* out_grad,
                       uint8_t* out_complete) {
  int rc = validate_common(ctx, ds, opset_id, trees);
  if (rc != SR_OK) return rc;
  if (trees->n_trees > 0 && (!out_loss || !out_grad || !out_complete))
    return set_error(SR_ERR_INVALID_ARG, "NULL output buffers");
  if (!ds->y) return set_error(SR_ERR_INVALID_ARG, "dataset has no y");
  Lock l(ctx);
  SR_HIP_CHECK(hipSetDevice(ctx->device));
  if (ds->dtype == SR_DTYPE_F32)
    return eval_grad_impl<float>(ctx, ds, opset_id, trees, row_idx, n_idx, loss_kind, out_loss, out_grad, out_complete);
  return eval_grad_impl<double>(ctx, ds, opset_id, trees, row_idx, n_idx, loss_kind, out_loss, out_grad, out_complete);
}

int sr_compile_info(int dtype, int n_unary, const char* const* unary_names, int n_binary,
                    const char* const* binary_names, const sr_tree_batch* trees, int64_t n_rows,
                    int64_t nfeatures, int32_t* out_len, uint8_t* out_static_bad, int32_t* out_max_depth,
                    void* out_code, int64_t code_capacity) {
  if (!trees || n_unary < 0 || n_binary < 0 || (n_unary > 0 && !unary_names) || (n_binary > 0 && !binary_names))
    return set_error(SR_ERR_INVALID_ARG, "bad arguments");
  SrOpset o;
  for (int i = 0; i < n_unary; ++i) {
    const uint32_t id = unary_names[i] ? sr_unary_id(unary_names[i]) : 0;
    if (!id) return set_error(SR_ERR_UNSUPPORTED_OP, std::string("unsupported unary operator: ") +
                                                         (unary_names[i] ? unary_names[i] : "(null)"));
    o.unary.push_back(id);
  }
  for (int i = 0; i < n_binary; ++i) {
    const uint32_t id = binary_names[i] ? sr_binary_id(binary_names[i]) : 0;
    if (!id) return set_error(SR_ERR_UNSUPPORTED_OP, std::string("unsupported binary operator: ") +
                                                         (binary_names[i] ? binary_names[i] : "(null)"));
    o.binary.push_back(id);
  }
  std::string err;
  auto report = [&](auto& prog) -> int {
    const int64_t nt = trees->n_trees;
    for (int64_t t = 0; t < nt; ++t) {
      if (out_len) out_len[t] = int32_t(prog.offsets[size_t(t) + 1] - prog.offsets[size_t(t)]);
      if (out_static_bad) out_static_bad[t] = prog.static_bad[size_t(t)];
    }
    if (out_max_depth) *out_max_depth = prog.max_depth;
    if (out_code) {
      const int64_t n = int64_t(prog.code.size()) < code_capacity ? int64_t(prog.code.size()) : code_capacity;
      std::memcpy(out_code, prog.code.data(), size_t(n) * 16);
    }
    return SR_OK;
  };
  if (dtype == SR_DTYPE_F32) {
    SrProgramBatch<float> prog;
    int rc = sr_compile_batch<float>(*trees, o, n_rows, nfeatures, false, &prog, &err);
    if (rc != SR_OK) return set_error(rc, err);
    return report(prog);
  }
  if (dtype == SR_DTYPE_F64) {
    SrProgramBatch<double> prog;
    int rc = sr_compile_batch<double>(*trees, o, n_rows, nfeatures, false, &prog, &err);
    if (rc != SR_OK) return set_error(rc, err);
    return report(prog);
  }
  return set_error(SR_ERR_INVALID_ARG, "unknown dtype");
}

int sr_host_unary(int dtype, const char* name, int64_t n, const void* x, void* out) {
  const uint32_t id = name ? sr_unary_id(name) : 0;
  if (!id) return set_error(SR_ERR_UNSUPPORTED_OP, std::string("unsupported unary operator: ") + (name ? name : "(null)"));
  if (n < 0 || (n > 0 && (!x || !out))) return set_error(SR_ERR_INVALID_ARG, "bad arguments");
  if (dtype == SR_DTYPE_F32) {
    for (int64_t i = 0; i < n; ++i) static_cast<float*>(out)[i] = sr_unary<float>(id, static_cast<const float*>(x)[i]);
  } else if (dtype == SR_DTYPE_F64) {
    for (int64_t i = 0; i < n; ++i) static_cast<double*>(out)[i] = sr_unary<double>(id, static_cast<const double*>(x)[i]);
  } else {
    return set_error(SR_ERR_INVALID_ARG, "unknown dtype");
  }
  return SR_OK;
}

// the last call's kernel / busy times from its events (computed on first request)
static void settle_timing(sr_ctx* ctx) {
  if (!ctx->timing_pending) return;
  ctx->timing_pending = false;
  ctx->last_eval_ms = chunk_kernel_ms(ctx);
  ctx->last_busy_ms = chunk_busy_ms(ctx);
  ctx->fold_kernel_ms_last = 0.0;
  if (ctx->fold_timed_last)
    for (int c = 0; c < ctx->n_chunks_last; ++c) {
      float m = 0.f;
      if (hipEventElapsedTime(&m, ctx->ev_fc0[c], ctx->ev_fc1[c]) == hipSuccess) ctx->fold_kernel_ms_last += double(m);
    }
}

int sr_last_phase_ms(sr_ctx* ctx, double* out, int n) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  Lock l(ctx);
  if (n > 8) settle_timing(ctx);
  for (int i = 0; i < n && i < 5; ++i) out[i] = ctx->phase_ms[i];
  if (n > 5) out[5] = double(ctx->n_chunks_last);
  if (n > 6) out[6] = ctx->exact_kernel_ms;
  if (n > 7) out[7] = double(ctx->rows_last);
  if (n > 8) out[8] = ctx->last_busy_ms;
  if (n > 9) out[9] = double(ctx->n_fold_last);
  if (n > 10) out[10] = double(ctx->fold_slow_last);
  if (n > 11) out[11] = double(ctx->fold_seg_last);
  for (int i = 0; i < 4; ++i)
    if (n > 12 + i) out[12 + i] = ctx->fold_ms[i];
  return SR_OK;
}

int sr_set_tuning(sr_ctx* ctx, const char* name, int64_t value) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (!name) return set_error(SR_ERR_INVALID_ARG, "tuning knob name is NULL");
  Lock l(ctx);
  if (std::strcmp(name, "derived") == 0) {
    ctx->derived = value != 0 ? 1 : 0;
    return SR_OK;
  }
  if (std::strcmp(name, "grad_sort") == 0) {  // gradient work items ordered by program cost (SR_AMD_GRAD_SORT)
    ctx->grad_sort = value != 0 ? 1 : 0;
    return SR_OK;
  }
  if (std::strcmp(name, "chunk_min") == 0) {  // the two-chunk pipeline's smallest first chunk (SR_AMD_CHUNK_MIN)
    ctx->chunk_min = std::max<int64_t>(1, value);
    return SR_OK;
  }
  if (std::strcmp(name, "first_chunk") == 0) {  // the two-chunk pipeline's first chunk is 1/value (SR_AMD_FIRST_CHUNK)
    ctx->first_chunk = int(std::max<int64_t>(2, std::min<int64_t>(64, value)));
    return SR_OK;
  }
  if (std::strcmp(name, "max_row_blocks") == 0) {  // row blocks per tree of a LOSS launch (SR_AMD_MAX_ROW_BLOCKS)
    ctx->max_row_blocks = int(std::max<int64_t>(1, std::min<int64_t>(value, 1 << 16)));
    return SR_OK;
  }
  if (std::strcmp(name, "probe") == 0) {  // dead-tree probe mode (SR_AMD_PROBE)
    ctx->probe = int(value);
    return SR_OK;
  }
  if (std::strcmp(name, "host_io") == 0) {  // small-call results written to pinned memory (SR_AMD_HOST_IO: 0, 1)
    if (value < 0 || value > 1) return set_error(SR_ERR_INVALID_ARG, "host_io must be 0 or 1");
    ctx->host_io = int(value);
    return SR_OK;
  }
  if (std::strcmp(name, "vstk_rows") == 0) {  // register-stack rows per lane (SR_AMD_VSTK_ROWS; 0: default)
    ctx->vstk_rows = int(value);
    return SR_OK;
  }
  if (std::strcmp(name, "grad_rows") == 0) {  // gradient kernel rows per lane (SR_AMD_GRAD_ROWS; 0: automatic)
    ctx->grad_rows_force = int(value);
    return SR_OK;
  }
  if (std::strcmp(name, "host_reduce") == 0) {  // largest call (trees x row blocks) reduced on the host (SR_AMD_HOST_REDUCE)
    ctx->host_reduce = value < 0 ? 0 : value;
    return SR_OK;
  }
  if (std::strcmp(name, "fused_reduce") == 0) {  // in-launch partial reduction bound (SR_AMD_FUSED_REDUCE)
    ctx->fused_reduce = value;
    return SR_OK;
  }
  if (std::strcmp(name, "ref_fold") == 0) {  // every complete tree's loss = the in-order fold (SR_AMD_REF_FOLD)
    ctx->ref_fold = value != 0 ? 1 : 0;
    return SR_OK;
  }
  if (std::strcmp(name, "fold_store_mb") == 0) {  // small calls: stored losses up to this size (SR_AMD_FOLD_STORE_MB)
    ctx->fold_store_mb = value < 0 ? 0 : value;
    return SR_OK;
  }
  if (std::strcmp(name, "fold_slot_mb") == 0) {  // FOLD mode: slow-segment slots (SR_AMD_FOLD_SLOT_MB)
    ctx->fold_slot_mb = value < 1 ? 1 : value;
    return SR_OK;
  }
  if (std::strcmp(name, "fold_debug_fail") == 0) {  // tests: trees t % value == 0 take the fold's fallback
    ctx->fold_debug_fail = int(value < 0 ? 0 : value);
    return SR_OK;
  }
  if (std::strcmp(name, "fold_delta_log2") == 0) {  // the plan's window 2^-value around the f64 prefix
    ctx->fold_delta_log2 = int(value < 1 ? 1 : (value > 40 ? 40 : value));
    return SR_OK;
  }
  if (std::strcmp(name, "fold_seg_max") == 0) {  // longest row block folded (SR_AMD_FOLD_SEG_MAX)
    ctx->fold_seg_max = value < 0 ? 0 : value;
    return SR_OK;
  }
  if (std::strcmp(name, "fold_rows_max") == 0) {  // longest fold (SR_AMD_FOLD_ROWS_MAX)
    ctx->fold_rows_max = value < 0 ? 0 : value;
    return SR_OK;
  }
  if (std::strcmp(name, "fold_seg") == 0) {  // rows per segment of the in-order loss fold (SR_AMD_FOLD_SEG)
    ctx->fold_seg = value < 0 ? -1 : value;
    return SR_OK;
  }
  if (std::strcmp(name, "exact_w") == 0) {  // waves per workgroup of the EXACT pass (SR_AMD_EXACT_W)
    ctx->exact_w = value == 1 ? 1 : 4;
    return SR_OK;
  }
  if (std::strcmp(name, "exact_g") == 0) {  // listed trees per EXACT workgroup, 0 = heuristic (SR_AMD_EXACT_G)
    ctx->exact_g = int(value < 0 ? 0 : (value > 64 ? 64 : value));
    return SR_OK;
  }
  if (std::strcmp(name, "code_cache") == 0) {  // LDS program cache (SR_AMD_CODE_CACHE)
    ctx->code_cache = value != 0 ? 1 : 0;
    return SR_OK;
  }
  if (std::strcmp(name, "timing") == 0) {  // 0: record no timing events (kernel times read as 0)
    ctx->timing = value != 0 ? 1 : 0;
    return SR_OK;
  }
  if (std::strcmp(name, "stress_probe") == 0) {  // the probe over the stress rows (SR_AMD_STRESS_PROBE)
    ctx->stress_probe = value != 0 ? 1 : 0;
    return SR_OK;
  }
  if (std::strcmp(name, "rows_per_lane") == 0) {  // kernel build per call (SR_AMD_ROWS_PER_LANE; 0 = default)
    ctx->rows_override = int(value);
    return SR_OK;
  }
  if (std::strcmp(name, "balance") == 0) {  // launch order dealt over tree groups (SR_AMD_BALANCE)
    ctx->balance_groups = value != 0;
    return SR_OK;
  }
  if (std::strcmp(name, "debug_hint_regrow") == 0) {  // tests: hint-array growth in place, stale epochs in it
    ctx->debug_hint_regrow = value != 0 ? 1 : 0;
    return SR_OK;
  }
  if (std::strcmp(name, "inject_failure_post") == 0) {
    ctx->inject_post = int(value);
    return SR_OK;
  }
  if (std::strcmp(name, "inject_failure_post_exact") == 0) {
    ctx->inject_post_exact = int(value);
    return SR_OK;
  }
  if (std::strcmp(name, "inject_failure_post_wsum") == 0) {  // tests: this rank's copy of the k-th Σw gather fails
    ctx->inject_post_wsum = int(value);
    return SR_OK;
  }
  if (std::strcmp(name, "inject_failure_post_gather") == 0) {
    ctx->inject_post_gather = int(value);
    return SR_OK;
  }
  if (std::strcmp(name, "inject_failure") == 0) {  // tests: the next `value` collective-buffer growths fail
    ctx->inject_fail = int(value);
    return SR_OK;
  }
  return set_error(SR_ERR_INVALID_ARG, std::string("unknown tuning knob '") + name + "'");
}

int sr_last_grad_info(sr_ctx* ctx, int n, double* kernel_ms, double* flops, int64_t* items, int* rows_per_lane) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  Lock l(ctx);
  for (int b = 0; b < n && b < sr_ctx::kGradBuckets; ++b) {
    float m = 0.f;
    if (kernel_ms)
      kernel_ms[b] = (ctx->grad_timed[b] && hipEventElapsedTime(&m, ctx->ev_g0[b], ctx->ev_g1[b]) == hipSuccess) ? double(m) : 0.0;
    if (flops) flops[b] = ctx->grad_flops[b];
    if (items) items[b] = ctx->grad_items[b];
    if (rows_per_lane) rows_per_lane[b] = ctx->grad_rows[b];
  }
  return SR_OK;
}

int sr_tuning_info(sr_ctx* ctx, int* used_derived_columns, int64_t* exact_trees) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  if (used_derived_columns) *used_derived_columns = ctx->n_derived_last;
  if (exact_trees) *exact_trees = ctx->n_exact_last;
  return SR_OK;
}

int sr_ref_fold_info(sr_ctx* ctx, int* path, int64_t* n_folded, int64_t* n_fallback, double* fold_kernel_ms) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  Lock l(ctx);
  settle_timing(ctx);
  if (path) *path = ctx->fold_path_last;
  if (n_folded) *n_folded = ctx->n_ref_ok_last;
  if (n_fallback) *n_fallback = ctx->n_ref_fail_last;
  if (fold_kernel_ms) *fold_kernel_ms = ctx->fold_kernel_ms_last;
  return SR_OK;
}

#ifdef SR_STAMPS
// latency-analysis builds only (not in include/sr_amd.h): the last main launch's stamps
// [block][wave][SR_NSTAMPS] (wall clock, 100 MHz) and their count
int sr_debug_stamps(sr_ctx* ctx, uint64_t* out, int64_t cap, int64_t* n) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  Lock lk(ctx);
  *n = ctx->n_stamps;
  if (ctx->n_stamps > 0 && out && cap >= ctx->n_stamps) {
    SR_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    SR_HIP_CHECK(hipMemcpy(out, ctx->stamps.p, size_t(ctx->n_stamps) * sizeof(uint64_t), hipMemcpyDeviceToHost));
  }
  return SR_OK;
}
#endif

int sr_last_kernel_ms(sr_ctx* ctx, double* eval_ms, double* total_ms) {
  if (check_ctx(ctx) != SR_OK) return SR_ERR_INVALID_ARG;
  Lock l(ctx);
  settle_timing(ctx);
  if (eval_ms) *eval_ms = ctx->last_eval_ms;
  if (total_ms) *total_ms = ctx->last_total_ms;
  return SR_OK;
}

}  // extern "C"
