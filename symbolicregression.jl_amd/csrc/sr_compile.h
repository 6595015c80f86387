// sr_compile.h — host-side program compiler: DynamicExpressions Node trees -> device programs.
//
// The compiler restates, per tree and at compile time, every decision DynamicExpressions 2.4's
// recursive `_eval_tree_array` makes from the tree SHAPE alone:
//   * maximal constant subtrees are folded to a scalar with a validity check after every op
//     (DE's "speed hack for constant trees");
//   * which node outputs get the `isfinite(sum(array))` early-exit check (children of general
//     unary/binary nodes, the root);
//   * which unary nodes are the fused `deg1_l2_ll0_lr0` / `deg1_l1_ll0` kernels (non-finite inner
//     value -> +Inf output);
//   * scalar checks of constant leaves inside fused `deg2_*` kernels.
// Data-dependent checks are encoded as CHECK bits for the kernel.  Evaluation order is chosen by
// Sethi–Ullman numbering (deeper child first) so the operand stack stays tiny; this is legal because
// the `complete` flag is the AND of all check predicates, independent of order.
#pragma once
#include <stdint.h>
#include <functional>
#include <string>
#include <vector>
#include "sr_ops.h"
#include "../../include/sr_amd.h"

struct SrOpset {
  std::vector<uint32_t> unary;   // options.operators.ops[1][i] -> SrUnaryOp
  std::vector<uint32_t> binary;  // options.operators.ops[2][i] -> SrBinaryOp
};

// Returns SrUnaryOp / SrBinaryOp id for an operator name, 0 if unsupported.
uint32_t sr_unary_id(const char* name);
uint32_t sr_binary_id(const char* name);

template <typename T>
struct SrProgramBatch {
  std::vector<SrIns<T>> code;       // all trees, concatenated
  std::vector<uint32_t> offsets;    // [n_trees + 1] into code
  std::vector<uint8_t> static_bad;  // 1: tree incomplete regardless of X
  std::vector<uint32_t> n_checks;   // CHECK instructions per tree
  std::vector<uint32_t> n_consts;   // constants per tree (pre-order, for gradients)
  std::vector<uint32_t> const_off;  // [n_trees + 1] prefix sum of n_consts
  std::vector<uint32_t> cost;       // estimated device cost per tree (launch ordering / balancing)
  std::vector<uint8_t> depth;       // operand-stack slots each tree needs
  int max_depth = 0;                // operand-stack slots needed (below top-of-stack)
  int tier = 1;                     // operator tier the programs ran under (SR_TIER_*; set by run_batch):
                                    // the exact-sum pass runs the same tier's kernel
  int max_checks = 0;
  int64_t total_nodes = 0;          // Σ count_nodes (metric unit)
  int64_t total_ops = 0;            // Σ operator nodes
  // Lazy form (the caller sets keep_pieces before compiling): `code` stays empty and tree k's
  // offsets[k + 1] - offsets[k] instructions sit at pieces[piece[k]][begin[k]...] (the compile
  // workers' own buffers), so a caller that re-stages the programs anyway (run_batch, in launch
  // order) copies them once instead of twice.  n_code counts the instructions in either form.
  bool keep_pieces = false;
  std::vector<std::vector<SrIns<T>>> pieces;
  std::vector<uint32_t> piece, begin;
  size_t n_code = 0;
  const SrIns<T>* tree_code(size_t k) const {
    return keep_pieces ? pieces[piece[k]].data() + begin[k] : code.data() + offsets[k];
  }
};

// Compile a batch.  n_rows: rows the programs will be evaluated on (static overflow checks of
// constant arrays).  nfeatures: columns of X.  with_const_index: emit constant-slot indices in
// `arg` of CONST loads (gradient kernels).  Returns SR_OK or an error code with *err set.
// fn(0) .. fn(n - 1) on the compile workers and the caller (the persistent pool sr_compile_batch uses).
void sr_parallel_for(int n, const std::function<void(int)>& fn);

// Estimated cost of one program instruction on the device, in VALU-instruction-like units per row
// step (dispatch overhead included): used only to order trees for load balance.
uint32_t sr_instruction_cost(uint32_t opcode);

// derived: optional [SR_U_COUNT][nfeatures] map (-1 = none) of the call's derived columns; nodes
// unary(feature) with a column become one LOAD_DERIVED (BASIC-tier LOSS programs only; ignored with
// with_const_index).
template <typename T>
int sr_compile_batch(const sr_tree_batch& trees, const SrOpset& ops, int64_t n_rows, int64_t nfeatures,
                     bool with_const_index, SrProgramBatch<T>* out, std::string* err,
                     const int16_t* derived = nullptr);
