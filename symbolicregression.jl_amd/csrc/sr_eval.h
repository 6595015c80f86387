// sr_eval.h — kernel argument block and launchers shared by the kernels and the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "sr_ops.h"
#include "../../include/sr_amd.h"

// SR_MODE_FOLD (round 6): the loss programs of complete trees again, composing each row tile's steps of
// the reference's in-order loss fold for the binades of the call's fold plan (sr_fold_dev.h), no checks
enum { SR_MODE_LOSS = 0, SR_MODE_PRED = 1, SR_MODE_EXACT = 2, SR_MODE_FOLD = 3 };
// operand-stack slots the register-stack kernels hold in VGPRs (1: trees needing a second slot —
// 6 % of C2's — run on the LDS-stack kernel instead)
// The deferred checks leave bounded outputs untracked (sr_tile_impl.h sr_untracked_u / _b; round 5:
// C2 kernel -4 %, arithmetic-only -9 %, profiles/r05_ab_track_lite.txt); -DSR_TRACK_FULL tracks all.
#ifndef SR_TRACK_FULL
#define SR_TRACK_LITE 1
#endif
#ifndef SR_VSTK_SLOTS
#define SR_VSTK_SLOTS 2
#endif
enum { SR_TIER_BASIC = 0, SR_TIER_FULL = 1 };

// One row view's launch positions in a several-view launch (sr_eval_loss_batch_views): positions
// [pos0, pos0 + n_pos) in tree groups of trees_per_block, blocks [block0, block0 + groups x row blocks),
// rows row_idx[row_off .. row_off + n_rows).
struct SrSegment {
  int block0, pos0, n_pos, groups;
  int64_t row_off;
};

// Per-tree reduction of [row block][position] partials, one wave per tree: lane l folds row blocks
// l, l + 64, ... in order, then a fixed shfl_xor butterfly adds the 64 lane sums; lane 0 writes the
// tree's Σ and OR of flags (static_bad ORed in) at perm[position].  The SAME arithmetic serves the
// reduce launch and the in-launch reduction (bit-identical results).  The wave handles `count`
// positions pos0, pos0 + step, ...; K of them at a time, so their loads are in flight together.
// SC1: the partials were written by other workgroups in this launch (write-through `sc1` stores):
// read them with `sc1` loads, which bypass this CU's L1.
template <int K, bool SC1>
__device__ inline void sr_reduce_positions(const double* part_sum, const uint32_t* part_flag, int n_trees,
                                           int n_row_blocks, int pos0, int step, int count,
                                           const uint32_t* perm, const uint8_t* static_bad, double* out_sum,
                                           uint32_t* out_flag, int lane) {
  for (int j0 = 0; j0 < count; j0 += K) {
    double s[K];
    uint32_t f[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      s[k] = 0.0;
      f[k] = 0u;
    }
    for (int i = lane; i < n_row_blocks; i += 64) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (j0 + k < count) {
          const size_t o = size_t(i) * size_t(n_trees) + size_t(pos0 + (j0 + k) * step);
          if (SC1) {
            s[k] += __longlong_as_double(static_cast<long long>(__hip_atomic_load(
                reinterpret_cast<unsigned long long*>(const_cast<double*>(part_sum + o)), __ATOMIC_RELAXED,
                __HIP_MEMORY_SCOPE_AGENT)));
            f[k] |= __hip_atomic_load(const_cast<uint32_t*>(part_flag + o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            s[k] += part_sum[o];
            f[k] |= part_flag[o];
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        s[k] += __shfl_xor(s[k], off, 64);
        f[k] |= __shfl_xor(f[k], off, 64);
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (j0 + k < count) {
          const int pos = pos0 + (j0 + k) * step;
          const int tree = perm ? int(perm[pos]) : pos;
          uint32_t fl = f[k];
          if (static_bad && static_bad[tree]) fl |= SR_FLAG_STATIC | SR_FLAG_NONFINITE;
          out_sum[tree] = s[k];
          out_flag[tree] = fl;
        }
      }
    }
  }
}

template <typename T>
struct SrEvalArgs {
  // programs
  const SrIns<T>* code;
  const uint32_t* offsets;     // [n_trees + 1], indexed by the caller's tree index
  const uint32_t* ends;        // [n_trees] end of each tree's program (NULL: offsets[t + 1]); programs are
                               // staged in launch order, so a tree group's code is one contiguous span
  const uint32_t* perm;        // launch position -> caller's tree index (NULL: identity); EXACT: tree list
  uint32_t* hint;              // [n_trees] per position: dead-tree hints across row blocks (LOSS; may be NULL)
  uint32_t hint_epoch;         // a position is dead when its hint equals this call's epoch (no reset pass)
  int n_trees;                 // trees (or listed trees in EXACT mode)
  int trees_per_block;         // G
  // data (per-feature rows, leading dimension ld; padded rows replicate row 0)
  const T* X;
  const T* y;                  // may be NULL (prediction only)
  const T* w;                  // NULL -> unweighted
  const int64_t* row_idx;      // GATHER mode: rows of the SubDataset
  int64_t ld;
  const T* derived;            // LOAD_DERIVED columns [k][dld] over the rows of the view (NULL: none)
  int64_t dld;
  int64_t n_rows;              // rows evaluated
  int nf;
  int tiles_per_block;
  int n_row_blocks;
  int n_groups;                // tree groups (blockIdx = row_block * n_groups + group)
  int stack_depth;             // LDS operand-stack slots per wave (>= 1)
  int code_lds;                // LOSS: instructions of LDS program cache per workgroup (0: windows
                               // stream from global memory); a group whose span exceeds it streams too
  T tbig;                      // |v| >= tbig may overflow the array-sum check
  double big_budget;           // a tile holding |v| >= tbig is BIG only when its lanes' Σ max|v| passes this
                               // (64 x floatmax / (1.01 x the view's padded rows, every shard)): below it,
                               // no checked array's Julia-order sum can reach floatmax (sr_tile_impl.h)
  int track_x;                 // the data holds |x| >= tbig or non-finite values: checked feature
                               // loads join the deferred checks (FAST path)
  int loss_kind;               // SrLossKind
  T loss_param;                // its parameter (HuberLoss delta, QuantileLoss tau, ...)
  // outputs
  double* part_sum;            // [n_row_blocks][n_trees], per launch position
  uint32_t* part_flag;         // [n_row_blocks][n_trees], per launch position
  // single row block (n_row_blocks == 1): the per-tree results go straight to out_sum / out_flag
  // (tree order, static_bad ORed in) and no reduce launch follows; NULL otherwise
  double* out_sum;
  uint32_t* out_flag;
  const uint8_t* static_bad;
  // several row blocks, reduced in the launch (LOSS; NULL: a reduce launch follows): the last row
  // block of a tree group to finish reduces the group's partials into fused_sum / fused_flag (tree
  // order, static_bad ORed in), in sr_reduce_partials_kernel's order; group_cnt[first position of
  // the group] counts the group's finished blocks (zero between launches: the last one resets it)
  uint32_t* group_cnt;
  double* fused_sum;
  uint32_t* fused_flag;
  T* pred;                   // PRED: [n_trees][pred_ld]
  int64_t pred_ld;
  // EXACT mode (perm = listed trees): row block rb = row range [range_lo[rb], range_hi[rb]] of the
  // view; range_sums[list position][check][rb] (T) = Julia-order sum of the checked array over it
  int max_checks;
  const int64_t* range_lo;
  const int64_t* range_hi;
  void* range_sums;
  // several row views in one launch (GATHER LOSS; NULL: one view, blockIdx = row_block * n_groups + group)
  const SrSegment* segs;
  int n_segs;
  // the reference's in-order loss fold (round 6, sr_fold_dev.h).  LOSS: fold_loss non-NULL stores every
  // evaluated tree's elementwise losses at fold_loss[position * fold_pos_stride + row] (small calls: the
  // fold's tables are composed from them).  FOLD: fold_code [n_row_blocks][n_trees] per position (the
  // plan), fold_tab the same shape of composed-step pairs (SrFoldTab<T>::Pair, written for steps
  // segments), fold_loss the slow segments' losses, slot (code - SR_FCODE_SLOT0) x fold_slot_rows.
  // fold_sq / fold_tab2 (same shape): a slow segment's lower window binade, and the composed steps of
  // its rows under that binade (in fold_tab) and the next (fold_tab2), so that the walk advances a slow
  // segment the running value does not actually leave a binade in without reading its rows
  T* fold_loss;
  int64_t fold_pos_stride;
  const int32_t* fold_code;
  void* fold_tab;
  int64_t fold_slot_rows;
  const int32_t* fold_sq;
  void* fold_tab2;
  // -DSR_STAMPS builds only (latency analysis, tools/stamps.py): per wave, SR_NSTAMPS wall-clock
  // stamps at fixed points of the kernel, [block][wave][SR_NSTAMPS]; NULL otherwise
  uint64_t* stamps;
};
constexpr int SR_NSTAMPS = 8;

template <typename T, int R, int MODE, bool GATHER, int TIER, int W = 4, int LK = -1, bool VSTK = false>
hipError_t sr_launch_tile(const SrEvalArgs<T>& a, int n_blocks, hipStream_t s);
// LDS bytes one workgroup (W waves) of the tile kernel needs.
size_t sr_tile_lds_bytes(int elem_size, int nf, int rows_per_lane, int stack_depth, int trees_per_block,
                         int max_checks, int waves, bool weighted, int code_lds = 0);
// Waves per workgroup the dispatcher uses for (mode, tier, rows per lane); `requested` overrides.
int sr_waves_per_block(int elem_size, int mode, int tier, int rows_per_lane, int requested);
// Rows per lane the dispatcher uses for (mode, tier); `requested` 4 selects the f32 BASIC tuning kernel.
template <typename T>
int sr_rows_per_lane(int mode, int tier, int requested);
// Rows per lane of the register-stack f32 BASIC loss kernel for n rows (0: use the LDS-stack kernel).
int sr_vstk_rows(int elem_size, int64_t n_rows, int requested);
// Runtime dispatch over the instantiated kernels: R rows per lane (sr_rows_per_lane, or
// sr_vstk_rows with vstk = true: operand stack in VGPRs, programs of <= 2 stack slots).
template <typename T>
hipError_t sr_launch_eval(const SrEvalArgs<T>& a, int mode, bool gather, int tier, int R, int waves, bool vstk,
                          int n_blocks, hipStream_t s);
// Derived columns of a call (LOAD_DERIVED): column k = op[k](X[feat[k]]) over the view's rows.
constexpr int SR_MAX_DERIVED = 32;
struct SrDerivedSpec {
  int n;
  uint8_t op[SR_MAX_DERIVED];
  uint16_t feat[SR_MAX_DERIVED];  // 0-based feature
};
template <typename T>
hipError_t sr_launch_derived(const T* X, int64_t ld, const int64_t* row_idx, int64_t n_view, int64_t n_pad,
                             const SrDerivedSpec& spec, T* out, int64_t dld, hipStream_t s);

hipError_t sr_launch_reduce(const double* part_sum, const uint32_t* part_flag, int n_trees, int n_row_blocks,
                            const uint32_t* perm, const uint8_t* static_bad, double* out_sum, uint32_t* out_flag,
                            hipStream_t s);
// isfinite(Julia pairwise sum) of n_arrays arrays from their leaf folds [n_arrays][n_leaves] (T),
// combined by the post-order program `prog` (leaf index: push; -1: add the top two).
template <typename T>
hipError_t sr_launch_jsum_levels(const T* leaf_sums, int64_t n_arrays, int n_leaves, const int2* nodes, int n_internal,
                                 const int32_t* level_off, int n_levels, T* scratch, uint8_t* out, hipStream_t s);
hipError_t sr_launch_pack_partials(const double* sum, const uint32_t* flag, int n, double* out, hipStream_t s);
// comp codes of the row-sharded finalize: 0 incomplete, 1 complete, 2 BIG only (exact check pending),
// | SR_COMP_FOLD: the loss fold is computed in order (sr_fold.h)
constexpr int SR_COMP_FOLD = 4;
template <typename T>
hipError_t sr_launch_finalize_packed(const double* packed, int n, double denom, int64_t n_terms, T* loss, uint8_t* comp,
                                     hipStream_t s);
template <typename T>
hipError_t sr_launch_transpose(const T* Xh_dev, int64_t nf, int64_t n, int64_t ld, T* Xd, hipStream_t s);
template <typename T>
hipError_t sr_launch_pad(T* v, int64_t n, int64_t ld, T pad_value, int replicate_first, hipStream_t s);

// Arguments of the forward-mode constant-gradient kernel (csrc/sr_grad_impl.h).
template <typename T>
struct SrGradArgs {
  const SrIns<T>* code;
  const uint32_t* offsets;   // [n_trees + 1]
  const T* consts;           // pre-order constants of every tree
  const uint32_t* const_off; // [n_trees + 1]
  const uint32_t* item_tree; // work item -> tree
  const uint32_t* item_k0;   // work item -> first tangent (constant index)
  int n_items;
  const T* X;
  const T* y;
  const T* w;
  const int64_t* row_idx;    // GATHER: rows of the SubDataset
  int64_t ld;
  int64_t n_rows;
  int nf;
  int tiles_per_block;
  int n_row_blocks;
  int n_groups;
  int stack_depth;
  int loss_kind;
  T loss_param;
  double* part;              // [n_row_blocks][n_items][KT]
  const SrSegment* segs;     // several row views (GATHER; positions = work items); NULL: one view
  int n_segs;
};

// rows: rows per lane, sr_grad_rows_per_lane(kt) or 1 (sr_grad_launch_rows)
template <typename T>
hipError_t sr_launch_grad_any(const SrGradArgs<T>& a, int kt, bool gather, int rows, int n_blocks, hipStream_t s);
// Largest rows per lane of the gradient kernel for KT tangents (a staged tile is 64 x that many rows);
// kernels exist for it, its halves down to 2, and 1.
constexpr int sr_grad_rows_per_lane(int kt) { return kt <= 2 ? 8 : (kt <= 4 ? 4 : (kt <= 8 ? 2 : 1)); }
// Rows of a staged gradient tile at `rows` rows per lane: 256, or one program pass when that is longer
// (a divisor of the host's 512-row units)
constexpr int sr_grad_tile_rows(int rows) { return 64 * rows > 256 ? 64 * rows : 256; }
// LDS of one gradient workgroup (W waves): the X / y / w tile and the waves' operand stacks (value +
// KT tangents per row, stack_depth slots)
inline size_t sr_grad_lds_bytes(int elem_size, int kt, int rows, int nf, bool weighted, int stack_depth, int waves) {
  return (size_t(nf) + 1 + (weighted ? 1 : 0)) * size_t(sr_grad_tile_rows(rows)) * size_t(elem_size) +
         size_t(waves) * size_t(stack_depth) * size_t(1 + kt) * size_t(rows) * 64 * size_t(elem_size);
}
// Rows per lane a bucket of KT tangents runs with (results do not depend on it): `force` when it is
// one the kernels exist for and fits; otherwise the preferred count (Float32: the largest; Float64:
// half of it — the f64 value and tangents of 8 rows need ~190 VGPRs, two waves per SIMD), halved
// while the workgroup's LDS (tile + operand stacks, which grow with the bucket's deepest program)
// passes lds_max / 2, so that two workgroups share a CU; 0 when even one row per lane does not fit.
inline int sr_grad_launch_rows(int elem_size, int kt, int nf, bool weighted, int stack_depth, int waves, size_t lds_max,
                               int force = 0) {
  const int rmax = sr_grad_rows_per_lane(kt);
  auto fits = [&](int r, size_t cap) { return sr_grad_lds_bytes(elem_size, kt, r, nf, weighted, stack_depth, waves) <= cap; };
  auto valid = [&](int r) { return r == 1 || (r <= rmax && r >= 2 && (r & (r - 1)) == 0); };
  if (force > 0 && valid(force) && fits(force, lds_max)) return force;
  int r = elem_size == 8 && rmax > 1 ? rmax / 2 : rmax;
  while (r > 1 && !fits(r, lds_max / 2)) r /= 2;
  if (fits(r, lds_max)) return r;
  return fits(1, lds_max) ? 1 : 0;
}
hipError_t sr_launch_grad_reduce(const double* part, int n_row_blocks, int n_vals, double* out, hipStream_t s);
// The reference's loss fold in row order for listed trees (sr_fold.h; sr_aux.hip): predictions
// pred[b][pred_ld] of n rows, losses against y (and w) at row_idx (or the row itself).
// sr_launch_fold_segsum: per segment of seg_len rows, segsum[b][seg] = the f64 sum of its losses;
// sr_launch_fold_segtab: the segment's composed steps tq / tab for the binades around the f64 prefix
// (carry_est[b]: the f64 sum of the rows before this shard, or NULL).
template <typename T>
hipError_t sr_launch_fold_segsum(const T* pred, int64_t pred_ld, int n_trees, const T* y, const T* w,
                                 const int64_t* row_idx, int64_t n, int loss_kind, T loss_param, int64_t seg_len,
                                 double* segsum, hipStream_t s);
template <typename T>
hipError_t sr_launch_fold_segtab(const T* pred, int64_t pred_ld, int n_trees, const T* y, const T* w,
                                 const int64_t* row_idx, int64_t n, int loss_kind, T loss_param, int64_t seg_len,
                                 const double* segsum, const double* carry_est, int2* tq, int64_t* tab, hipStream_t s);
// Every complete tree's fold (round 6; sr_aux.hip): the plan of a large call (codes per (row block,
// position), slots for the FOLD mode's slow segments), the stored-loss tables of a small call, and the
// walk (per position: the fold's value and status at the caller's tree index perm[position]).
struct SrFoldWho;  // (sr_fold_dev.h)
// a region's plan arrays, [row block][position] each: codes, composed-step pairs (steps segments; a slow
// segment's under its lower window binade sq), sq (slow segments; SR_FCODE_SKIP: none), and a slow
// segment's pair under sq + 1
struct SrFoldTabs {
  int32_t* code;
  void* tab;
  int32_t* sq;
  void* tab2;
};
template <typename T>
hipError_t sr_launch_fold_plan(const double* part, int np, int n_rb, const uint32_t* perm, const SrFoldWho& who,
                               double delta, SrFoldTabs ft, int* slot_next, int slot_cap, hipStream_t s);
template <typename T>
hipError_t sr_launch_fold_stab(const double* part, int np, int n_rb, int64_t rb_rows, int64_t n, const uint32_t* perm,
                               const SrFoldWho& who, double delta, const T* losses, SrFoldTabs ft,
                               const uint32_t* part_flag, const uint8_t* static_bad, double* red_sum,
                               uint32_t* red_flag, hipStream_t s);
template <typename T>
hipError_t sr_launch_fold_walk(SrFoldTabs ft, const SrFoldWho& who, int np, int n_rb, int64_t rb_rows, int64_t n,
                               const T* losses, int64_t slot_rows, const uint32_t* perm, const T* carry, T* out_val,
                               int32_t* out_st, void* dbg, int all_rows, hipStream_t s);
template <typename T>
hipError_t sr_launch_fold(const T* pred, int64_t pred_ld, int n_trees, const T* y, const T* w, const int64_t* row_idx,
                          int64_t n, int loss_kind, T loss_param, int64_t seg_len, const int2* tq, const int64_t* tab,
                          const T* carry, T* out, int* n_slow, hipStream_t s);
