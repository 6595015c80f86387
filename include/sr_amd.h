/*
 * sr_amd.h — C ABI of the MI355X fitness-evaluation library (libsr_amd.so).
 *
 * Drop-in boundary for SymbolicRegression.jl's scoring hot path:
 *   eval_cost -> eval_loss -> _eval_loss -> eval_tree_dispatch -> DE.eval_tree_array
 *   (reference src/LossFunctions.jl:64-117,139-159,193-209; src/InterfaceDynamicExpressions.jl:58-88).
 * A Julia `ccall` binding flattens DynamicExpressions `Node{T,2}` trees into the
 * pre-order struct-of-arrays `sr_tree_batch` below and calls these entry points.  Every function
 * returns an `int` status (SR_OK = 0, negative = error); `sr_last_error()` gives a thread-local
 * message.  Non-finite evaluations are NOT errors: they come back as complete = 0, loss = +Inf,
 * exactly like `_eval_loss` returning `L(Inf)` (src/LossFunctions.jl:97-99).
 *
 * Ownership: the caller owns every host buffer (borrowed for the duration of the call); the
 * library owns device memory behind the opaque handles.  All calls are synchronous.
 */
#ifndef SR_AMD_H
#define SR_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SR_AMD_VERSION 2

/* status codes */
#define SR_OK 0
#define SR_ERR_INVALID_ARG (-1)
#define SR_ERR_HIP (-2)
#define SR_ERR_UNSUPPORTED_OP (-3)   /* operator outside the device catalog: caller keeps its CPU path */
#define SR_ERR_BAD_TREE (-4)         /* malformed pre-order arrays, feature out of range */
#define SR_ERR_TOO_DEEP (-5)         /* tree needs more stack slots than the kernel holds */
#define SR_ERR_NO_DEVICE (-6)

/* element types (Dataset{T}): Float32 / Float64 */
#define SR_DTYPE_F32 0
#define SR_DTYPE_F64 1

/* elementwise losses (Options.elementwise_loss; the LossFunctions.jl catalog of src/Options.jl:301-328).
 * The parameter-free ones are passed as `loss_kind` directly; a parametric one (and HuberLoss with
 * delta != 1) is registered with sr_register_loss, which returns the code to pass instead. */
#define SR_LOSS_L2DIST 0            /* L2DistLoss() — the default (src/Options.jl:772) */
#define SR_LOSS_L1DIST 1            /* L1DistLoss() */
#define SR_LOSS_LPDIST 2            /* LPDistLoss{P}()          param P */
#define SR_LOSS_LOGITDIST 3         /* LogitDistLoss() */
#define SR_LOSS_HUBERLOSS 4         /* HuberLoss(d)             param d (direct code: d = 1) */
#define SR_LOSS_L1EPSINS 5          /* L1EpsilonInsLoss(eps)    param eps */
#define SR_LOSS_L2EPSINS 6          /* L2EpsilonInsLoss(eps)    param eps */
#define SR_LOSS_PERIODICLOSS 7      /* PeriodicLoss(circ)       param circ */
#define SR_LOSS_QUANTILELOSS 8      /* QuantileLoss(tau)        param tau */
#define SR_LOSS_ZEROONE 9           /* ZeroOneLoss() */
#define SR_LOSS_PERCEPTRONLOSS 10   /* PerceptronLoss() */
#define SR_LOSS_L1HINGE 11          /* L1HingeLoss() */
#define SR_LOSS_L2HINGE 12          /* L2HingeLoss() */
#define SR_LOSS_SMOOTHEDL1HINGE 13  /* SmoothedL1HingeLoss(gamma) param gamma */
#define SR_LOSS_MODIFIEDHUBER 14    /* ModifiedHuberLoss() */
#define SR_LOSS_L2MARGIN 15         /* L2MarginLoss() */
#define SR_LOSS_EXPLOSS 16          /* ExpLoss() */
#define SR_LOSS_SIGMOIDLOSS 17      /* SigmoidLoss() */
#define SR_LOSS_DWDMARGIN 18        /* DWDMarginLoss(q)         param q */

/* per-tree partial flag bits (sr_eval_loss_partials) */
#define SR_FLAG_NONFINITE 1u /* some checked intermediate array holds NaN/Inf: complete = false */
#define SR_FLAG_BIG 2u       /* some checked value is so large its array sum may overflow: exact check needed */
#define SR_FLAG_STATIC 4u    /* tree is incomplete independent of X (constant checks, constant folding) */
#define SR_FLAG_ELEMINF 8u   /* an elementwise loss, or the T sum of two, is +Inf: the reference's loss fold
                                (LossFunctions' sequential sum in T, src/LossFunctions.jl:38-58) is +Inf */

typedef struct sr_ctx sr_ctx;
typedef struct sr_dataset sr_dataset;

/*
 * A batch of expression trees in DynamicExpressions' own node fields, pre-order (depth-first,
 * parent before children, left before right — the order of `get_scalar_constants`,
 * test/integration/ad/zygote/test_derivatives.jl:127-155).  Tree t occupies node positions
 * [offsets[t], offsets[t+1]).
 */
typedef struct sr_tree_batch {
  int64_t n_trees;
  const int64_t* offsets;   /* [n_trees + 1] */
  const uint8_t* degree;    /* Node.degree: 0 leaf, 1 unary, 2 binary */
  const uint8_t* op;        /* Node.op: 1-based index into options.operators.ops[degree] */
  const uint16_t* feature;  /* Node.feature: 1-based column of X (leaf, !constant) */
  const uint8_t* constant;  /* Node.constant (leaf) */
  const void* val;          /* Node.val (leaf, constant): Float32 or Float64 = dataset dtype */
} sr_tree_batch;

/* ------------------------------------------------------------------ library / device */
const char* sr_last_error(void);
int sr_version(void);
int sr_device_count(int* count);
/* Open a context on HIP device `device` (one process per GPU: pass LOCAL_RANK). */
int sr_init(int device, sr_ctx** out);
int sr_shutdown(sr_ctx* ctx);

/*
 * Register an operator set: the printed names of options.operators.ops[1] (unary) and
 * ops[2] (binary), in order, e.g. {"cos","exp","log"} and {"+","-","*","/"}.  Names follow
 * DynamicExpressions' printing ("log" = safe_log, "^" = safe_pow, ...; src/Operators.jl:126-185)
 * and the function names themselves ("safe_log", "plus", ...) are accepted too.
 * Returns SR_ERR_UNSUPPORTED_OP if any operator is outside the device catalog.
 */
int sr_register_opset(sr_ctx* ctx, int n_unary, const char* const* unary_names, int n_binary,
                      const char* const* binary_names, int* opset_id);

/*
 * Register an elementwise loss with its parameter (Options.elementwise_loss, e.g. HuberLoss(1.5) =
 * {SR_LOSS_HUBERLOSS, 1.5}); *loss_code is what the eval calls take as `loss_kind`.
 */
int sr_register_loss(sr_ctx* ctx, int kind, double param, int* loss_code);

/*
 * Upload a dataset (src/Dataset.jl:131-246).  X is Julia's column-major [nfeatures, n] matrix
 * (address f + nfeatures*i); the device copy is transposed to per-feature contiguous rows.
 * y has n entries; weights may be NULL (unweighted).  dtype is SR_DTYPE_F32 / SR_DTYPE_F64.
 */
int sr_dataset_upload(sr_ctx* ctx, int dtype, const void* X, int64_t nfeatures, int64_t n,
                      const void* y, const void* weights, sr_dataset** out);
int sr_dataset_free(sr_dataset* ds);
int sr_dataset_info(const sr_dataset* ds, int* dtype, int64_t* nfeatures, int64_t* n);

/*
 * Batched eval_loss (src/LossFunctions.jl:90-117 applied to every tree).
 * row_idx (0-based, may repeat) selects a SubDataset view (src/Dataset.jl:90-112,300-308);
 * pass NULL / 0 for the full dataset.  out_loss[n_trees] has the dataset dtype (L == T);
 * out_complete[n_trees] is the `complete` flag of eval_tree_array.
 */
int sr_eval_loss_batch(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                       const int64_t* row_idx, int64_t n_idx, int loss_kind, void* out_loss,
                       uint8_t* out_complete);

/*
 * The same for trees on different row views in ONE call: tree t is scored on the n_views x view_len
 * row array's view tree_view[t] (rows view_rows[tree_view[t] * view_len + i], 0-based, may repeat).  This
 * is SymbolicRegression's batching with one minibatch per island (src/SingleIteration.jl:40, 77;
 * src/Dataset.jl:303-304): the children of every island in one launch, each on its own island's rows.
 * Results equal sr_eval_loss_batch per view.
 */
int sr_eval_loss_batch_views(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                             const int32_t* tree_view, int n_views, const int64_t* view_rows, int64_t view_len,
                             int loss_kind, void* out_loss, uint8_t* out_complete);


/*
 * Batched eval_tree_array (src/InterfaceDynamicExpressions.jl:58-88): predictions
 * out_pred[n_trees][n_rows] (dataset dtype, row-major per tree) and complete flags.
 */
int sr_eval_tree_array(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                       const int64_t* row_idx, int64_t n_idx, void* out_pred, uint8_t* out_complete);

/*
 * Row-sharded form for multi-GPU scoring.  The dataset on this rank holds one shard of the
 * rows; n_total is the number of rows over ALL shards (it sets the overflow-check threshold).
 * Writes per-tree partial Σ w·loss (f64) and flag bits (SR_FLAG_*).  With out_on_device = 1 the
 * two output pointers are device pointers (e.g. a torch tensor to all-reduce with RCCL).
 * Combine across ranks: sums add, flags OR; trees whose combined flags == SR_FLAG_BIG get the exact
 * verdict from sr_jsum_partials + sr_jsum_finite; then sr_finalize_losses.
 */
int sr_eval_loss_partials(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                          int64_t n_total, int loss_kind, double* out_sum, uint32_t* out_flags,
                          int out_on_device);
/*
 * The same partials packed for ONE all-reduce (SUM): out[5][n_trees] f64 = Σ w·loss, then the
 * SR_FLAG_NONFINITE, SR_FLAG_BIG, SR_FLAG_STATIC and SR_FLAG_ELEMINF bits as 0/1 (summed over ranks:
 * > 0 means set).
 * out_on_device = 1: `out` is a device pointer on this context's GPU (no host round trip).
 */
int sr_eval_loss_partials_packed(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                                 int64_t n_total, int loss_kind, double* out, int out_on_device);
/* RCCL for the row-sharded path, on the library's own HIP runtime: rank 0 calls
 * sr_comm_unique_id, the caller broadcasts the SR_COMM_ID_BYTES bytes (any CPU channel: MPI, a TCP
 * store, torch.distributed's gloo group), every rank calls sr_comm_init with them.
 * sr_eval_loss_partials_allreduce = sr_eval_loss_partials_packed on this shard, then ONE in-place
 * all-reduce (sum) of the [5, n_trees] f64 buffer on the device over xGMI, then the global
 * partials to out_host (what sr_finalize_losses / the exact path take).  Every rank must call it
 * with the same trees.  (Replaces the Julia-side Distributed reduction of the reference's
 * per-worker losses for one batched call.) */
#define SR_COMM_ID_BYTES 128
int sr_comm_unique_id(void* out_id);
int sr_comm_init(sr_ctx* ctx, int nranks, int rank, const void* id_bytes);
/* The same sharded calls over collectives the caller provides instead of RCCL (any transport: a gloo /
 * MPI group on the host, a test harness; several ranks may then share one GPU).  Both callbacks are
 * collective and return 0 on success: allreduce sums buf[n] over the ranks in place; allgather writes
 * every rank's `bytes` send bytes into recv[nranks][bytes] in rank order.  The library calls them with
 * host buffers, on the calling thread, in the same order on every rank. */
typedef int (*sr_host_allreduce_fn)(void* user, double* buf, int64_t n);
typedef int (*sr_host_allgather_fn)(void* user, const void* send, void* recv, int64_t bytes);
int sr_comm_init_host(sr_ctx* ctx, int nranks, int rank, sr_host_allreduce_fn allreduce, sr_host_allgather_fn allgather,
                      void* user);
int sr_comm_destroy(sr_ctx* ctx);
int sr_eval_loss_partials_allreduce(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                                    int64_t n_total, int loss_kind, double* out_host);
/*
 * The whole row-sharded step of batched eval_loss (SURVEY §8(e) row sharding, config C4) in one call:
 * rank r's `ds` holds global rows [Σ_{q<r} n_q, Σ_{q<=r} n_q) (shards in rank order; their sizes, Σw
 * and max|X| are exchanged over the communicator at the first call per dataset).  This shard runs
 * the single-GPU launch pipeline, the packed [5, n_trees] partials are summed by ONE in-place RCCL
 * all-reduce over xGMI, losses are finalized on the device (Σ / global n or Σw), trees flagged BIG
 * get DynamicExpressions' exact isfinite(sum) verdict over the GLOBAL rows (leaf folds all-gathered),
 * and the rare trees whose T-precision loss fold may overflow are folded in row order across the shards.
 * out_loss / out_complete as sr_eval_loss_batch over the union of the shards, on every rank.
 * Collective: every rank calls it with the same trees.  A failure on one rank (HIP error, bad tree)
 * still enters the collectives with its error word set, and every rank then returns an error.
 * (Replaces SymbolicRegression's per-worker scoring over a distributed dataset for one batched call.)
 */
int sr_eval_loss_sharded(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees, int loss_kind,
                         void* out_loss, uint8_t* out_complete);
/*
 * Tree-sharded batched eval_loss (SURVEY §8(e) tree sharding): `ds` is the whole dataset on every
 * rank; the trees are dealt over the ranks by size (snake order over the sorted batch), each rank
 * scores its share with sr_eval_loss_batch, and ONE all-reduce hands every rank every (loss, complete).
 * Serves the member-parallel scoring sites (src/Population.jl:49-60, src/SingleIteration.jl:79-92).
 * Collective, same trees on every rank, same error rule as sr_eval_loss_sharded.
 */
int sr_eval_loss_tree_sharded(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                              int loss_kind, void* out_loss, uint8_t* out_complete);
/* The communicator's size and this rank (as RCCL reports them: ncclCommCount / ncclCommUserRank; may be
 * NULL), and "transport=rccl|host;hip=<file>;rccl=<file>": the transport and the HIP runtime and RCCL
 * this library's calls bind to (`paths` may be NULL).  sr_comm_unique_id / sr_comm_init fail if the two come from different ROCm
 * trees (RCCL would then run this library's streams on another HIP runtime). */
int sr_comm_info(sr_ctx* ctx, int* nranks, int* rank, char* paths, int64_t capacity);
/* The same "hip=...;rccl=..." string without a context (no device needed). */
int sr_runtime_info(char* paths, int64_t capacity);
/* Maximum number of checked nodes per tree for `trees` (element type dtype; sizes the
 * sr_jsum_partials output). */
int sr_max_checks(sr_ctx* ctx, int dtype, int opset_id, const sr_tree_batch* trees, int* max_checks);
/*
 * Exact validity check, DynamicExpressions' isfinite(sum(x)) on every checked node with Base's
 * pairwise `sum` in T (Base.mapreduce_impl: halves split at lo + (hi-lo)>>1 down to blocks of < 1024
 * elements folded sequentially).  This dataset holds global rows [row_offset, row_offset + n) of
 * n_total.  sr_jsum_range_count gives the number of row ranges this shard folds (the global leaf
 * blocks it holds, and one-row ranges continuing a block that starts in an earlier shard);
 * sr_jsum_partials writes, for the listed trees, out_vals[n_list][max_checks][n_ranges] (T: the
 * fold of each checked array over each range).  sr_jsum_finite combines every shard's values
 * (row_offsets[n_ranks + 1] bounds the shards, rank_vals[r] = shard r's out_vals) into
 * out_finite[n_arrays] (n_arrays = n_list * max_checks): a tree is complete iff all its arrays are.
 */
int sr_jsum_range_count(int64_t row_offset, int64_t n_local, int64_t n_total, int64_t* out_n_ranges);
/* The ranges themselves (each output may be NULL): local rows [lo, hi], global leaf index, and
 * head = 1 for a one-row range continuing a leaf that starts in an earlier shard. */
int sr_jsum_ranges(int64_t row_offset, int64_t n_local, int64_t n_total, int64_t* lo, int64_t* hi, int64_t* leaf,
                   uint8_t* head);
int sr_jsum_partials(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                     const int64_t* tree_list, int64_t n_list, int max_checks, int64_t row_offset, int64_t n_total,
                     void* out_vals);
int sr_jsum_finite(int dtype, int64_t n_total, int n_ranks, const int64_t* row_offsets, const void* const* rank_vals,
                   int64_t n_arrays, uint8_t* out_finite);
/*
 * Host-side combine: loss = sum / denom (denom = n_total, or Σweights), +Inf when incomplete.
 * Trees flagged SR_FLAG_BIG alone are listed in tree_list with their exact verdict list_ok
 * (1 = every checked array's Julia sum is finite); list may be empty (NULL, 0).
 */
int sr_finalize_losses(int dtype, int64_t n_trees, const double* sums, const uint32_t* flags, double denom,
                       const int64_t* tree_list, int64_t n_list, const uint8_t* list_ok, void* out_loss,
                       uint8_t* out_complete);
/* Σ weights of this shard (f64), or the row count when unweighted. */
int sr_dataset_denominator(const sr_dataset* ds, double* denom);

/*
 * Forward-mode gradient of the loss with respect to every constant of every tree (the batched
 * BFGS objective+gradient of src/ConstantOptimization.jl:77-167).  Constants are ordered
 * pre-order per tree (get_scalar_constants); out_grad is laid out per tree at the running sum of
 * constant counts.  out_loss / out_complete as in sr_eval_loss_batch.
 */
int sr_eval_grad_batch(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                       const int64_t* row_idx, int64_t n_idx, int loss_kind, void* out_loss,
                       void* out_grad, uint8_t* out_complete);

/* sr_eval_grad_batch over several row views (as sr_eval_loss_batch_views): the constant optimisation of
 * every island's members in one lock-step pass, each on its island's minibatch. */
int sr_eval_grad_batch_views(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                             const int32_t* tree_view, int n_views, const int64_t* view_rows, int64_t view_len,
                             int loss_kind, void* out_loss, void* out_grad, uint8_t* out_complete);

/*
 * Host-only dry run of the tree compiler (no device needed): compile `trees` for an operator set
 * and report, per tree, the program length in instructions (out_len), whether the tree is
 * incomplete independent of X (out_static_bad), and the operand-stack depth it needs
 * (*out_max_depth).  With out_code != NULL the raw 16-byte instructions (Σ out_len of them, the
 * layout of SrIns in csrc/sr_ops.h) are copied there, up to code_capacity instructions.
 */
int sr_compile_info(int dtype, int n_unary, const char* const* unary_names, int n_binary,
                    const char* const* binary_names, const sr_tree_batch* trees, int64_t n_rows,
                    int64_t nfeatures, int32_t* out_len, uint8_t* out_static_bad, int32_t* out_max_depth,
                    void* out_code, int64_t code_capacity);

/*
 * Host-side evaluation of one unary operator (the code constant folding uses; the device runs the
 * same functions): out[i] = op(x[i]) for n values of dtype.  For testing host/device agreement.
 */
int sr_host_unary(int dtype, const char* name, int64_t n, const void* x, void* out);

/* ------------------------------------------------------------------ native search engine
 * equation_search's inner loop (s_r_cycle, optimize_and_simplify_population, the head's per-island
 * bookkeeping: src/SingleIteration.jl, src/RegularizedEvolution.jl, src/Mutate.jl,
 * src/MutationFunctions.jl, src/Population.jl, src/SymbolicRegression.jl:1040-1140) in C++, with
 * every island's children of a regularised-evolution round scored by ONE sr_eval_loss_batch call.
 * Islands shard over ranks (island i on rank i % world_size); per iteration a rank runs
 * sr_search_iterate on its islands, the ranks exchange sr_search_export buffers (all-gather) and
 * sr_search_import them, and every rank runs sr_search_head (identical bookkeeping, migration into
 * an island by its owner).  Single process: start, then (iterate, head) per iteration.
 */
typedef struct sr_search sr_search;

/* mutation kinds, the order of sr_search_options.mutation_weights (src/MutationWeights.jl) */
#define SR_MUT_MUTATE_CONSTANT 0
#define SR_MUT_MUTATE_OPERATOR 1
#define SR_MUT_MUTATE_FEATURE 2
#define SR_MUT_SWAP_OPERANDS 3
#define SR_MUT_ROTATE_TREE 4
#define SR_MUT_ADD_NODE 5
#define SR_MUT_INSERT_NODE 6
#define SR_MUT_DELETE_NODE 7
#define SR_MUT_SIMPLIFY 8
#define SR_MUT_RANDOMIZE 9
#define SR_MUT_DO_NOTHING 10
#define SR_MUT_OPTIMIZE 11
#define SR_N_MUTATIONS 12

/* member sets of sr_search_member_count / sr_search_members (>= 0: that island) */
#define SR_SEARCH_HALL_OF_FAME (-1)
#define SR_SEARCH_PARETO (-2)

/* Options fields the search reads (src/OptionsStruct.jl types: Float32 fields are float) */
typedef struct sr_search_options {
  int populations, population_size, ncycles_per_iteration, tournament_selection_n;
  float tournament_selection_p;
  int maxsize, maxdepth;
  float parsimony;
  float crossover_probability;
  int annealing;
  float alpha, perturbation_factor, probability_negate_constant;
  int use_frequency, use_frequency_in_tournament;
  double adaptive_parsimony_scaling;
  float fraction_replaced, fraction_replaced_hof;
  int topn, migration, hof_migration, skip_mutation_failures, should_simplify;
  int should_optimize_constants;
  float optimizer_probability;
  int optimizer_iterations, optimizer_nrestarts;
  int batching;
  int64_t batch_size;
  float warmup_maxsize_by;
  double mutation_weights[SR_N_MUTATIONS];
  int64_t optimizer_f_calls_limit; /* Optim.Options f_calls_limit (the reference's default 10_000; 0: none) */
} sr_search_options;

typedef struct sr_search_info {
  int64_t iterations, s_r_cycles, device_calls;
  double num_evals;
  double device_ms; /* wall time inside the scoring calls (device launches + their host sides) */
  double host_ms;   /* selection, mutation and acceptance */
  double baseline_loss;
  int use_baseline;
  double kernel_ms; /* device-busy time of the scoring calls' interpreter launches (loss calls) */
} sr_search_info;

/* CPU scorers for tests (the library's own device path when not set): sr_eval_loss_batch /
 * sr_eval_grad_batch semantics over the search's dataset; return SR_OK or an error code. */
typedef int (*sr_loss_fn)(void* user, const sr_tree_batch* trees, const int64_t* row_idx, int64_t n_idx,
                          void* out_loss, uint8_t* out_complete);
typedef int (*sr_grad_fn)(void* user, const sr_tree_batch* trees, const int64_t* row_idx, int64_t n_idx,
                          void* out_loss, void* out_grad, uint8_t* out_complete);

int sr_search_create(int dtype, int64_t nfeatures, int64_t n_rows, int n_unary, const char* const* unary_names,
                     int n_binary, const char* const* binary_names, const sr_search_options* opts, uint64_t seed,
                     int rank, int world_size, sr_search** out);
int sr_search_free(sr_search* s);
/* score on the device: `ds` must match the search's dtype / features / rows */
int sr_search_use_device(sr_search* s, sr_ctx* ctx, const sr_dataset* ds, int opset_id, int loss_code);
/* an extra scoring lane (before sr_search_start): its own context and dataset copy on the same or
 * another GPU.  sr_search_iterate then splits this rank's islands over the lanes, one host thread
 * per lane, so one lane's device round trips overlap the others' work.  Results do not depend on
 * the number of lanes (every draw comes from the islands' own streams); num_evals is summed per
 * lane, so its last bits can differ. */
int sr_search_add_device(sr_search* s, sr_ctx* ctx, const sr_dataset* ds, int opset_id, int loss_code);
int sr_search_use_callbacks(sr_search* s, sr_loss_fn loss, sr_grad_fn grad, void* user);
/* update_baseline_loss! and the initial populations of this rank's islands */
int sr_search_start(sr_search* s, int niterations);
int sr_search_iterate(sr_search* s);
int sr_search_head(sr_search* s);
/* this rank's islands (members + best-seen) as bytes: call with buf = NULL for the size */
int sr_search_export(sr_search* s, void* buf, int64_t capacity, int64_t* size);
int sr_search_import(sr_search* s, const void* buf, int64_t size);
int sr_search_get_info(sr_search* s, sr_search_info* out);
int sr_search_member_count(sr_search* s, int which, int64_t* n_members, int64_t* n_nodes);
/* members as pre-order node arrays (offsets[n_members + 1]) + cost / loss (dtype) and bookkeeping */
int sr_search_members(sr_search* s, int which, int64_t* offsets, uint8_t* degree, uint8_t* op, uint16_t* feature,
                      uint8_t* constant, void* val, void* cost, void* loss, int64_t* birth, int64_t* ref,
                      int64_t* parent, int32_t* complexity);

/*
 * A population of n_trees random trees from gen_random_tree_fixed_size (src/MutationFunctions.jl:441-471;
 * the engine's generator and draws) with node_count ~ U{1..max_size}, one xoshiro256** stream keyed by
 * `seed` (Population init at scale, and the benchmark populations).  Pre-order node arrays of at most
 * `capacity` nodes (n_trees * max_size always suffices); offsets[n_trees + 1]; val has the dtype.
 */
int sr_gen_random_population(int dtype, int64_t n_trees, int64_t nfeatures, int n_unary, int n_binary, int max_size,
                              uint64_t seed, int64_t capacity, int64_t* offsets, uint8_t* degree, uint8_t* op,
                              uint16_t* feature, uint8_t* constant, void* val);

/*
 * Batched constant optimisation (optimize_constants, src/ConstantOptimization.jl:29-116) of every
 * tree: BFGS with BackTracking (Newton for one constant, its curvature from the device gradient)
 * from the tree's constants and from `nrestarts` starts x0 .* (1 + eps/2), eps ~ randn(T) from the
 * stream `seed`; each round of line-search trials is one batched loss call, each gradient one
 * sr_eval_grad_batch call; `iterations` and `f_calls_limit` are Optim.Options' (Options.jl:988-997:
 * optimizer_iterations, optimizer_f_calls_limit; 0 = no call limit): a start stops after the iteration
 * at whose end its objective calls reach the limit.  Out: the constants (pre-order per tree, concatenated; unchanged where
 * not improved), the loss at them, improved = the minimum beat the start, and the objective
 * evaluations per tree (num_evals = (f_calls + improved) x dataset fraction).
 */
int sr_optimize_constants_batch(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                                const int64_t* row_idx, int64_t n_idx, int loss_kind, int iterations,
                                int64_t f_calls_limit, int nrestarts, uint64_t seed, void* out_consts, void* out_loss,
                                uint8_t* out_improved, int64_t* out_f_calls);

/* The same optimiser with the scoring calls answered by CPU callbacks (sr_loss_fn / sr_grad_fn, as
 * sr_search_use_callbacks): a test seam and the host-port baseline.  dtype = the trees' element type. */
int sr_optimize_constants_callbacks(int dtype, const sr_tree_batch* trees, const int64_t* row_idx, int64_t n_idx,
                                    int iterations, int64_t f_calls_limit, int nrestarts, uint64_t seed, sr_loss_fn loss,
                                    sr_grad_fn grad, void* user, void* out_consts, void* out_loss,
                                    uint8_t* out_improved, int64_t* out_f_calls);

/* Timing of the last device call on this context (ms): kernel-only, via HIP events. */
int sr_last_kernel_ms(sr_ctx* ctx, double* eval_ms, double* total_ms);

/* Host-side phases of the last sr_eval_loss_batch / sr_eval_loss_sharded call (ms, wall clock), up to
 * n of: compile, upload + launch, wait for the interpreter + reduction (sharded: + the all-reduce),
 * exact-sum pass, finalize (with the in-order loss fold of sr_fold.h, when any); out[5] (n >= 6)
 * = the number of interpreter launches of the call (the batch is compiled and launched in chunks),
 * out[6] (n >= 7) = device time of the exact-sum pass (ms), out[7] (n >= 8) = rows per lane of its
 * interpreter kernel, out[8] (n >= 9) = the device-busy time of those launches: the UNION of their
 * intervals (launches on the two pipeline streams overlap, so their summed durations can exceed it),
 * out[9] (n >= 10) = the number of trees whose loss fold was computed in row order (the overflow rule of
 * the reference's T-precision fold: csrc/sr_fold.h), out[10] (n >= 11) = the segments of those folds
 * folded row by row (the rest advanced by their composed steps), out[11] (n >= 12) = the fold's
 * segment length in rows (0: one scan over every row), out[12..15] (n >= 16) = the fold's device time
 * (ms, HIP events, summed over its batches) in its PRED pass, segment sums, composed steps and chain.  sr_last_kernel_ms's eval_ms is the sum of
 * those launches' durations. */
int sr_last_phase_ms(sr_ctx* ctx, double* out, int n);

/* Run-time tuning of a context (the SR_AMD_* environment variables are read once at sr_init):
 * "derived" (0 / 1: derived columns for unary(feature) nodes of large LOSS calls), "probe" (dead-tree
 * probe: 0 off, 1 before every chunk, 2 before the chunks after the first), "stress_probe" (0 / 1: the
 * probe runs the dataset's stress rows — per feature the extreme and nearest-zero values — instead of
 * its first rows), "code_cache" (0 / 1: register-stack launches copy each tree group's programs into
 * LDS once instead of streaming them per tile from global memory), "timing" (0 / 1: record the HIP
 * events behind sr_last_kernel_ms / sr_last_phase_ms), "rows_per_lane" (0: the default kernel per
 * call; Float32 16 / 32 force the register-stack kernel and 4 / 8 the LDS-stack one, Float64 8 / 4
 * likewise), "balance" (0 / 1: deal the cost-ordered trees round-robin over tree groups),
 * "fused_reduce" (the largest tree group, in trees x row blocks, whose partials the interpreter launch
 * reduces itself — its last workgroup per group; 0: always a separate reduce launch), "exact_w" (4 / 1:
 * waves per workgroup of the exact-sum pass), "exact_g" (listed trees per exact-sum workgroup; 0: the
 * heuristic), "fold_seg" (rows per segment of the in-order loss fold: -1 automatic, 0 one workgroup
 * scan over every row per tree, as rounds 3-4), "ref_fold" (1, the default: every complete tree's loss
 * is the reference's in-order fold in T of its elementwise losses (src/LossFunctions.jl:38-58), divided
 * in T; 0: the f64 sum of rounds 1-5, whose last bits — ~5e-4 relative at 2^20 rows in Float32 —
 * differ), "fold_store_mb" / "fold_slot_mb" (the fold's stored-loss and slow-segment budgets),
 * "fold_delta_log2" (the fold plan's window), "fold_seg_max" (the longest row block folded: a folding
 * call takes enough row blocks for it), "fold_rows_max" (the longest fold, 2^24 rows: a longer call —
 * C4's 2^26 rows — keeps the f64 sum, as "ref_fold" 0).  Results do not depend on any knob but these
 * three ("ref_fold", "fold_seg_max", "fold_rows_max": whether a call folds) and — without the fold only
 * — "max_row_blocks", which sets how many f64 partials a tree's sum adds (the last bit of a loss may
 * differ).  SR_ERR_INVALID_ARG for an unknown name.  sr_tuning_info (optional outputs)
 * reports how many derived columns the last sr_eval_loss_batch used and how many of its trees went
 * through the exact-sum pass (flagged BIG). */
int sr_set_tuning(sr_ctx* ctx, const char* name, int64_t value);
/* The last sr_eval_grad_batch(_views) call's tangent kernels, per tangent bucket b = 0..4 (1, 2, 4, 8,
 * 16 tangents; up to n of each output, each may be NULL): device time (ms, HIP events; 0 when the
 * context's "timing" is off or the bucket was empty), algorithmic flops (per row of a (tree, first
 * tangent) work item: each unary node 2 + KT, each binary node 3 + 2 KT, the loss epilogue 3 + KT),
 * work items and rows per lane. */
int sr_last_grad_info(sr_ctx* ctx, int n, double* kernel_ms, double* flops, int64_t* items, int* rows_per_lane);
int sr_tuning_info(sr_ctx* ctx, int* used_derived_columns, int64_t* exact_trees);
/* The last sr_eval_loss_batch(_views)'s in-order loss fold (tuning "ref_fold"; each output may be NULL):
 * the path (0 none — "ref_fold" 0, negative weights, a fold past "fold_rows_max", or a Float64 call
 * too large to keep its losses; 1 the loss launch kept every tree's losses; 2 the FOLD-mode pass re-ran the
 * complete trees), the trees whose loss is the walk's exact fold, those whose walk left the plan's
 * window and were folded through the prediction pass instead, and the fold launches' device time (ms,
 * HIP events; 0 with "timing" off). */
int sr_ref_fold_info(sr_ctx* ctx, int* path, int64_t* n_folded, int64_t* n_fallback, double* fold_kernel_ms);

#ifdef __cplusplus
}
#endif
#endif /* SR_AMD_H */
