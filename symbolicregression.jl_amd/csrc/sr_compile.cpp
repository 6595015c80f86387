// sr_compile.cpp — see sr_compile.h.  Reference semantics restated here:
//   DynamicExpressions 2.4 `_eval_tree_array` / `dispatch_deg1_eval` / `dispatch_deg2_eval` /
//   `dispatch_constant_tree` (not vendored; SymbolicRegression calls it from
//   src/InterfaceDynamicExpressions.jl:81 and src/LossFunctions.jl:68,79), the fused-kernel list
//   pinned by test/unit/evaluation/test_evaluation.jl:15-51 and the flag known answers of
//   test/integration/ext/loopvectorization/test_nan_detection.jl:17-51.
#include "sr_compile.h"

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>

namespace {

// Persistent compile workers: spawning threads per batch cost more than compiling 10k trees.
// run(n, fn) calls fn(0..n-1) on the caller and whichever workers wake in time; one batch at a time.
// The caller never waits for a worker to wake up: it takes jobs itself from the start and waits only
// for jobs a worker has already taken (a search's small batches finish before a sleeping worker is
// scheduled: waiting for every worker to check in cost ~40 us per call).  Jobs are handed out by
// tickets (generation << 32 | index), so a worker that wakes late never runs a finished batch's job.
// A forked child (no threads of its own) gets a fresh pool.
class WorkerPool {
 public:
  static WorkerPool& get() {
    static std::mutex m;
    static WorkerPool* pool = nullptr;
    std::lock_guard<std::mutex> g(m);
    if (!pool || pool->pid_ != getpid()) pool = new WorkerPool();  // (a pre-fork pool is leaked)
    return *pool;
  }
  int size() const { return int(threads_.size()) + 1; }
  void run(int n, const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> batch(batch_mu_);
    uint64_t g;
    {
      std::lock_guard<std::mutex> lk(mu_);
      g = ++gen_;
      job_ = &fn;
      n_jobs_ = n;
      done_.store(0);
      ticket_.store(g << 32);
      gen_pub_.store(g, std::memory_order_release);
    }
    if (n > 1 && !threads_.empty()) cv_.notify_all();
    drain(g, &fn, n);
    while (done_.load(std::memory_order_acquire) < n) std::this_thread::yield();  // (jobs already taken)
  }

 private:
  WorkerPool() : pid_(getpid()) {
    unsigned hc = std::thread::hardware_concurrency();
    int n = int(hc == 0 ? 4 : (hc > 16 ? 16 : hc));
    if (const char* v = std::getenv("SR_AMD_COMPILE_THREADS")) n = std::atoi(v) > 0 ? std::atoi(v) : 1;
    if (const char* v = std::getenv("SR_AMD_COMPILE_SPIN_US")) spin_us_ = std::max(0, std::atoi(v));
    --n;  // the caller is a worker too
    for (int i = 0; i < n; ++i) threads_.emplace_back([this] { loop(); });
    for (auto& t : threads_) t.detach();  // lives for the process
  }
  // take jobs of generation g until none is left (a ticket of another generation ends the loop)
  void drain(uint64_t g, const std::function<void(int)>* job, int n) {
    uint64_t t = ticket_.load();
    for (;;) {
      if ((t >> 32) != g || int(t & 0xffffffffu) >= n) return;
      if (!ticket_.compare_exchange_weak(t, t + 1)) continue;  // (t reloaded)
      (*job)(int(t & 0xffffffffu));
      done_.fetch_add(1, std::memory_order_release);
      t = ticket_.load();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      uint64_t g;
      const std::function<void(int)>* job;
      int n;
      // optional spin before sleeping (SR_AMD_COMPILE_SPIN_US; off by default: on the box the spinning
      // workers cost the calling thread more than their wake-ups — C2 4.07-4.16 ms per step without,
      // 4.16-4.24 with 300 us, 4.22 with 2 ms; profiles/r05_ab_exact_compile.txt)
      const auto t0 = std::chrono::steady_clock::now();
      while (gen_pub_.load(std::memory_order_acquire) == seen &&
             std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(spin_us_))
        std::this_thread::yield();
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = g = gen_;
        job = job_;
        n = n_jobs_;
      }
      drain(g, job, n);
    }
  }
  pid_t pid_;
  std::vector<std::thread> threads_;
  std::mutex batch_mu_, mu_;
  std::condition_variable cv_;
  const std::function<void(int)>* job_ = nullptr;
  int n_jobs_ = 0;
  std::atomic<uint64_t> ticket_{0};
  std::atomic<int> done_{0};
  uint64_t gen_ = 0;
  std::atomic<uint64_t> gen_pub_{0};  // gen_, readable without the mutex (the spin above)
  int spin_us_ = 0;                   // SR_AMD_COMPILE_SPIN_US
};

struct NameId {
  const char* name;
  uint32_t id;
};

// Names as DynamicExpressions prints them (get_op_name, src/Operators.jl:126-160) plus the
// Julia function names SymbolicRegression maps them to (OP_MAP, src/Options.jl:182-202).
const NameId kUnary[] = {
    {"neg", SR_U_NEG},       {"-", SR_U_NEG},          {"square", SR_U_SQUARE},  {"cube", SR_U_CUBE},
    {"exp", SR_U_EXP},       {"cos", SR_U_COS},        {"sin", SR_U_SIN},        {"tan", SR_U_TAN},
    {"log", SR_U_LOG},       {"safe_log", SR_U_LOG},   {"log2", SR_U_LOG2},      {"safe_log2", SR_U_LOG2},
    {"log10", SR_U_LOG10},   {"safe_log10", SR_U_LOG10}, {"log1p", SR_U_LOG1P}, {"safe_log1p", SR_U_LOG1P},
    {"sqrt", SR_U_SQRT},     {"safe_sqrt", SR_U_SQRT}, {"abs", SR_U_ABS},        {"sign", SR_U_SIGN},
    {"tanh", SR_U_TANH},     {"sinh", SR_U_SINH},      {"cosh", SR_U_COSH},      {"atan", SR_U_ATAN},
    {"asin", SR_U_ASIN},     {"safe_asin", SR_U_ASIN}, {"acos", SR_U_ACOS},      {"safe_acos", SR_U_ACOS},
    {"acosh", SR_U_ACOSH},   {"safe_acosh", SR_U_ACOSH}, {"atanh", SR_U_ATANH}, {"safe_atanh", SR_U_ATANH},
    {"asinh", SR_U_ASINH},   {"relu", SR_U_RELU},      {"inv", SR_U_INV},        {"erf", SR_U_ERF},
    {"erfc", SR_U_ERFC},     {"gamma", SR_U_GAMMA},    {"round", SR_U_ROUND},    {"floor", SR_U_FLOOR},
    {"ceil", SR_U_CEIL},     {"exp2", SR_U_EXP2},      {"expm1", SR_U_EXPM1},
};
const NameId kBinary[] = {
    {"+", SR_B_ADD},          {"plus", SR_B_ADD},           {"-", SR_B_SUB},       {"sub", SR_B_SUB},
    {"*", SR_B_MUL},          {"mult", SR_B_MUL},           {"/", SR_B_DIV},       {"div", SR_B_DIV},
    {"^", SR_B_POW},          {"safe_pow", SR_B_POW},       {"pow", SR_B_POW},     {"max", SR_B_MAX},
    {"min", SR_B_MIN},        {"mod", SR_B_MOD},            {">", SR_B_GREATER},   {"greater", SR_B_GREATER},
    {"<", SR_B_LESS},         {"less", SR_B_LESS},          {">=", SR_B_GREATER_EQUAL},
    {"greater_equal", SR_B_GREATER_EQUAL},                  {"<=", SR_B_LESS_EQUAL},
    {"less_equal", SR_B_LESS_EQUAL},                        {"cond", SR_B_COND},
    {"logical_or", SR_B_LOGICAL_OR},                        {"logical_and", SR_B_LOGICAL_AND},
    {"atan2", SR_B_ATAN2},    {"atan", SR_B_ATAN2},
};

template <typename T>
struct Tree {
  // per node (pre-order position within the tree)
  std::vector<int32_t> l, r;
  const uint8_t* degree;
  const uint8_t* op;
  const uint16_t* feature;
  const uint8_t* constant;
  const T* val;
  int64_t n;
};

// v[0..n) = x, growing v only when it is too short (the compiler's per-tree arrays keep their
// capacity from tree to tree: an out-of-line vector::assign per array was ~10 % of a small batch)
template <typename V, typename X>
inline void reset_n(V& v, int64_t n, X x) {
  if (int64_t(v.size()) < n) v.resize(size_t(n));
  std::fill(v.begin(), v.begin() + n, x);
}

template <typename T>
struct TreeCompiler {
  const SrOpset& ops;
  int64_t n_rows;
  int64_t nfeatures;
  bool with_const_index;
  Tree<T> t;
  std::vector<uint8_t> is_const, folded, arr_check, infsub;
  std::vector<T> fold_val;
  std::vector<int32_t> const_slot;  // pre-order constant index of constant leaves
  std::vector<int32_t> need;
  std::vector<SrIns<T>> code;
  std::vector<int32_t> sz;  // parse(): subtree sizes (kept across trees: no per-tree allocation)
  bool bad = false;
  int err = SR_OK;
  std::string msg;
  int depth = 0, max_depth = 0;
  uint32_t n_checks = 0;
  uint32_t n_consts = 0;
  int64_t n_ops = 0;

  const int16_t* derived = nullptr;  // [SR_U_COUNT][nfeatures]: derived column of unary(feature), -1 none
  // constant-operand binaries fused as PBC fields (SR_AMD_PBC=0 turns it off: A/B runs)
  const bool fuse_pbc = [] {
    static const bool on = [] {
      const char* v = std::getenv("SR_AMD_PBC");
      return !(v && v[0] == '0');
    }();
    return on;
  }();

  TreeCompiler(const SrOpset& o, int64_t nr, int64_t nf, bool wci, const int16_t* dm = nullptr)
      : ops(o), n_rows(nr), nfeatures(nf), with_const_index(wci), derived(dm) {}

  // The derived column holding node i = unary(feature leaf) for the whole view, or -1.  (Such a node
  // is a general deg1 node: its child is an unfused leaf, never constant here.)
  int derived_col(int i) {
    if (!derived || t.degree[i] != 1) return -1;
    const int c = t.l[i];
    if (t.degree[c] != 0 || t.constant[c]) return -1;
    const uint32_t u = unary_id(i);
    if (u == SR_U_NONE || u >= SR_U_COUNT) return -1;
    return derived[size_t(u) * size_t(nfeatures) + size_t(t.feature[c] - 1)];
  }

  bool leaf(int i) const { return t.degree[i] == 0; }
  bool effleaf(int i) const { return t.degree[i] == 0 || folded[i]; }

  uint32_t unary_id(int i) {
    const int k = int(t.op[i]) - 1;
    if (k < 0 || k >= int(ops.unary.size())) {
      fail(SR_ERR_BAD_TREE, "unary op index out of range");
      return SR_U_NONE;
    }
    return ops.unary[k];
  }
  uint32_t binary_id(int i) {
    const int k = int(t.op[i]) - 1;
    if (k < 0 || k >= int(ops.binary.size())) {
      fail(SR_ERR_BAD_TREE, "binary op index out of range");
      return SR_B_NONE;
    }
    return ops.binary[k];
  }
  void fail(int code, const char* m) {
    if (err == SR_OK) {
      err = code;
      msg = m;
    }
  }

  // Parse pre-order arrays into child links, in ONE reverse scan (round 5: the explicit-stack descent
  // plus separate constant-numbering and constant-marking passes were ~40 % of a small batch): a
  // node's children come after it, so subtree sizes are known when it is reached — left child i + 1,
  // right child i + 1 + size(left) — and so is whether its subtree is all constants (`is_const`,
  // DE's constant-tree test).  The root's subtree must cover every node.
  bool parse() {
    const int64_t n = t.n;
    if (n <= 0) {
      fail(SR_ERR_BAD_TREE, "empty tree");
      return false;
    }
    reset_n(t.l, n, -1);
    reset_n(t.r, n, -1);
    if (int64_t(sz.size()) < n) sz.resize(size_t(n));
    if (int64_t(is_const.size()) < n) is_const.resize(size_t(n));
    for (int64_t i = n - 1; i >= 0; --i) {
      const int d = t.degree[i];
      if (d == 0) {
        sz[i] = 1;
        if (t.constant[i]) {
          is_const[i] = 1;
        } else {
          is_const[i] = 0;
          const int f = int(t.feature[i]);
          if (f < 1 || f > nfeatures) {
            fail(SR_ERR_BAD_TREE, "feature index out of range");
            return false;
          }
        }
        continue;
      }
      if (d > 2) {
        fail(SR_ERR_BAD_TREE, "degree > 2");
        return false;
      }
      const int64_t a = i + 1;
      if (a >= n) {
        fail(SR_ERR_BAD_TREE, "pre-order arrays end inside a subtree");
        return false;
      }
      t.l[i] = int32_t(a);
      if (d == 1) {
        sz[i] = 1 + sz[a];
        is_const[i] = is_const[a];
      } else {
        const int64_t b = a + sz[a];
        if (b >= n) {
          fail(SR_ERR_BAD_TREE, "pre-order arrays end inside a subtree");
          return false;
        }
        t.r[i] = int32_t(b);
        sz[i] = 1 + sz[a] + sz[b];
        is_const[i] = is_const[a] & is_const[b];
      }
    }
    if (sz[0] != n) {
      fail(SR_ERR_BAD_TREE, "extra nodes after the root subtree");
      return false;
    }
    return true;
  }

  // dispatch_constant_tree: scalar fold with is_valid after every op.  Leaf constants are
  // validated too (unpinned choice — a non-finite leaf constant makes the subtree
  // invalid, which also keeps Julia's cos(Inf) DomainError unreachable).
  bool fold(int i, T* out) {
    const int d = t.degree[i];
    if (d == 0) {
      *out = t.val[i];
      return sr_isfinite(*out);
    }
    if (d == 1) {
      T x;
      if (!fold(t.l[i], &x)) return false;
      const uint32_t id = unary_id(i);
      *out = sr_unary<T>(id, x);
      return sr_isfinite(*out);
    }
    T a, b;
    if (!fold(t.l[i], &a)) return false;
    if (!fold(t.r[i], &b)) return false;
    const uint32_t id = binary_id(i);
    *out = sr_binary<T>(id, a, b);
    return sr_isfinite(*out);
  }

  // Scalar check of a constant leaf (DE @return_on_nonfinite_val in fused deg2 kernels).
  void scalar_check(int i) {
    if (leaf(i) && t.constant[i] && !sr_isfinite(t.val[i])) bad = true;
  }

  // Mirror of _eval_tree_array's control flow: decides fold / checks / fused kernels.
  void evalmark(int i) {
    const int d = t.degree[i];
    if (d == 0) return;  // deg0_eval: copy / fill, no check here
    if (is_const[i]) {   // constant-tree fast path
      T v;
      if (!fold(i, &v)) bad = true;
      folded[i] = 1;
      fold_val[i] = v;
      return;
    }
    if (d == 1) {
      const int c = t.l[i];
      const int cd = t.degree[c];
      if (cd == 2 && leaf(t.l[c]) && leaf(t.r[c])) {  // deg1_l2_ll0_lr0
        infsub[i] = 1;
        scalar_check(t.l[c]);
        scalar_check(t.r[c]);
      } else if (cd == 1 && leaf(t.l[c])) {            // deg1_l1_ll0
        infsub[i] = 1;
        scalar_check(t.l[c]);
      } else {                                         // general deg1: child array checked
        evalmark(c);
        arr_check[c] = 1;
      }
      return;
    }
    const int a = t.l[i], b = t.r[i];
    if (leaf(a) && leaf(b)) {          // deg2_l0_r0
      scalar_check(a);
      scalar_check(b);
    } else if (leaf(b)) {              // deg2_r0: left evaluated + checked
      evalmark(a);
      arr_check[a] = 1;
      scalar_check(b);
    } else if (leaf(a)) {              // deg2_l0: right evaluated + checked
      evalmark(b);
      arr_check[b] = 1;
      scalar_check(a);
    } else {                           // general deg2: both checked
      evalmark(a);
      arr_check[a] = 1;
      evalmark(b);
      arr_check[b] = 1;
    }
  }

  // Static form of isfinite(sum(fill(c, n))) for constant arrays that are checked.
  void static_array_check(T c) {
    if (!sr_isfinite(c)) {
      bad = true;
      return;
    }
    const double s = std::fabs(double(c)) * double(n_rows);
    if (!(s <= double(SrM<T>::big))) bad = true;
  }

  int compute_need(int i) {
    if (effleaf(i)) return need[i] = 0;
    if (t.degree[i] == 1) return need[i] = compute_need(t.l[i]);
    const int a = t.l[i], b = t.r[i];
    const int na = compute_need(a), nb = compute_need(b);
    if (effleaf(a)) return need[i] = nb;
    if (effleaf(b)) return need[i] = na;
    return need[i] = (na == nb) ? na + 1 : (na > nb ? na : nb);
  }

  // Leaf as a LOAD (push = false; PUSH is patched in later) or as a binary operand.
  // is_operand: binary opcode base (variant FL/FR/CL/CR chosen from the leaf kind + side).
  static constexpr uint32_t kNoSlot = SR_M_INDEX;

  SrIns<T> leaf_ins(int i) {
    SrIns<T> in{};
    // a constant's index: its slot in gradient programs, else 0 (the interpreter reads the X row
    // named by every instruction's index before dispatching on the opcode)
    in.meta = with_const_index ? kNoSlot : 0u;
    if (folded[i]) {
      in.op = SR_OP_LOAD_CONST;
      in.set_value(fold_val[i]);
    } else if (t.constant[i]) {
      in.op = SR_OP_LOAD_CONST;
      in.set_value(t.val[i]);
      if (with_const_index) in.meta = uint32_t(const_slot[i]);
    } else {
      in.op = SR_OP_LOAD_FEAT;
      in.meta = uint32_t(t.feature[i]) - 1u;
    }
    return in;
  }
  static bool commutes(uint32_t bop) { return bop == SR_B_ADD || bop == SR_B_MUL; }
  SrIns<T> operand_ins(int i, uint32_t bop, bool left) {
    SrIns<T> in = leaf_ins(i);
    const bool is_const = in.op == SR_OP_LOAD_CONST;
    if (commutes(bop)) left = false;  // IEEE + and * commute: one variant per operand kind
    const uint32_t v = is_const ? (left ? SR_V_CL : SR_V_CR) : (left ? SR_V_FL : SR_V_FR);
    in.op = SR_BIN_OPC(bop, v);
    return in;
  }
  SrIns<T> stack_ins(uint32_t bop, bool left, int slot) {
    SrIns<T> in{};
    if (commutes(bop)) left = false;
    in.op = SR_BIN_OPC(bop, left ? SR_V_SL : SR_V_SR);
    in.meta = uint32_t(slot);
    return in;
  }

  void emit_check(int i) {
    if (!arr_check[i]) return;
    if (effleaf(i) && (folded[i] || t.constant[i])) {
      static_array_check(folded[i] ? fold_val[i] : t.val[i]);
      return;
    }
    code.back().meta |= SR_M_CHECK;
    ++n_checks;
  }

  // The first instruction of every subtree's code is a leaf LOAD or a PAIR: it first stores the
  // old top of stack to `slot`.
  void mark_push(SrIns<T>& in, int slot) {
    if (slot >= int(SR_MAX_STACK_SLOTS)) {
      fail(SR_ERR_TOO_DEEP, "tree needs more operand-stack slots than the encoding holds");
      return;
    }
    const uint32_t base = in.op & SR_OP_MASK;  // (a fused POST unary sits above the opcode)
    if (base >= SR_OP_PAIR0) in.op += SR_P_PUSH;                     // PAIR v -> PAIR v + PUSH
    else if (base == SR_OP_LOAD_DERIVED) in.op += SR_OP_LOAD_DERIVED_PUSH - SR_OP_LOAD_DERIVED;
    else in.op += SR_OP_LOAD_FEAT_PUSH - SR_OP_LOAD_FEAT;             // LOAD_x -> LOAD_x_PUSH
    in.meta |= uint32_t(slot + 1) << SR_M_PUSH_SHIFT;
  }

  // A binary node whose children are both leaves (DE deg2_l0_r0: no array check on either leaf)
  // as one PAIR instruction.  Gradient programs keep the plain form (the gradient kernel reads
  // constants by slot).  Returns false when the pair form does not apply.
  bool emit_pair(int i, uint32_t bop) {
    const int a = t.l[i], b = t.r[i];
    if (with_const_index || !effleaf(a) || !effleaf(b)) return false;
    SrIns<T> la = leaf_ins(a), lb = leaf_ins(b);
    const bool ca = la.op == SR_OP_LOAD_CONST, cb = lb.op == SR_OP_LOAD_CONST;
    if (ca && cb) return false;  // (only when folding is off)
    for (const int c : {a, b})   // a checked feature array needs its own LOAD (its CHECK bit)
      if (arr_check[c] && !(folded[c] || t.constant[c])) return false;
    for (const int c : {a, b})   // a checked constant array: the static check emit_check makes
      if (arr_check[c]) static_array_check(folded[c] ? fold_val[c] : t.val[c]);
    SrIns<T> in{};
    if (!ca && !cb) {
      in.op = SR_PAIR_OPC(bop, SR_P_FF);
      in.meta = la.meta;
      in.c0 = lb.meta;  // second feature
    } else if (!ca) {
      in.op = SR_PAIR_OPC(bop, SR_P_FC);
      in.meta = la.meta;
      in.c0 = lb.c0;
      in.c1 = lb.c1;
    } else if (commutes(bop)) {  // c op x == x op c (IEEE + and *)
      in.op = SR_PAIR_OPC(bop, SR_P_FC);
      in.meta = lb.meta;
      in.c0 = la.c0;
      in.c1 = la.c1;
    } else {
      in.op = SR_PAIR_OPC(bop, SR_P_CF);
      in.meta = lb.meta;
      in.c0 = la.c0;
      in.c1 = la.c1;
    }
    code.push_back(in);
    return true;
  }

  // A folded constant subtree DE evaluates as an array (a general deg2 child) is checked statically,
  // as in emit_pair (round 5: the operand forms CR / CL had skipped it — (x1 + x2) * (1e30 * 1e8) over
  // 4,000 rows scored complete where DE's isfinite(sum) of that child array fails)
  void const_operand_check(int leaf) {
    if (arr_check[leaf] && (folded[leaf] || t.constant[leaf])) static_array_check(folded[leaf] ? fold_val[leaf] : t.val[leaf]);
  }

  // A binary node op(tos, c) / op(c, tos) whose constant operand `leaf` (a constant or folded subtree) rides on
  // the instruction that computed tos as its PBC field (sr_ops.h), when that instruction holds no
  // constant of its own and no PBC yet; its own check becomes PBC_CHECK.  Gradient programs keep the
  // plain form.  Returns false when the fused form does not apply.
  bool fuse_const_operand(int i, int leaf, uint32_t bop, bool left) {
    if (with_const_index || code.empty() || !fuse_pbc) return false;
    SrIns<T> lf = leaf_ins(leaf);
    if (lf.op != SR_OP_LOAD_CONST) return false;
    SrIns<T>& last = code.back();
    if ((last.op >> SR_OP_PBC_SHIFT) != 0u) return false;
    const uint32_t base = last.op & SR_OP_MASK;
    const bool free_c = base == SR_OP_LOAD_FEAT || base == SR_OP_LOAD_FEAT_PUSH ||
                        (base >= SR_OP_UNARY0 && base < SR_OP_LOAD_DERIVED) ||
                        (base >= SR_OP_BINARY0 && base < SR_OP_PAIR0 && (base - SR_OP_BINARY0) % 6u < SR_V_CL);
    if (!free_c) return false;
    uint32_t v = 0;
    switch (bop) {
      case SR_B_ADD: v = SR_PBC_ADD; break;
      case SR_B_SUB: v = left ? SR_PBC_SUB_L : SR_PBC_SUB_R; break;
      case SR_B_MUL: v = SR_PBC_MUL; break;
      case SR_B_DIV: v = left ? SR_PBC_DIV_L : SR_PBC_DIV_R; break;
      default: return false;
    }
    const_operand_check(leaf);
    last.op |= v << SR_OP_PBC_SHIFT;
    last.c0 = lf.c0;
    last.c1 = lf.c1;
    if (arr_check[i]) {
      last.op |= SR_OP_PBC_CHECK;
      ++n_checks;
    }
    return true;
  }

  void emit(int i) {
    if (effleaf(i)) {
      code.push_back(leaf_ins(i));
      emit_check(i);
      return;
    }
    const int d = t.degree[i];
    ++n_ops;
    if (d == 1) {
      const int dc = infsub[i] ? -1 : derived_col(i);
      if (dc >= 0) {  // the whole node from the call's derived column
        SrIns<T> in{};
        in.op = SR_OP_LOAD_DERIVED;
        in.meta = uint32_t(dc);
        // (op, feature) for kernels that recompute the node in place (the exact-sum pass)
        in.c0 = (unary_id(i) << 16) | uint32_t(t.feature[t.l[i]] - 1);
        code.push_back(in);
        emit_check(i);
        return;
      }
      emit(t.l[i]);
      // the child's code ends with the instruction computing it: the unary rides on it as its POST
      // operator (one dispatch for both), unless that instruction carries one already; gradient
      // programs keep the plain form (their kernel has no post operators)
      if (!with_const_index && !code.empty() && (code.back().op >> SR_OP_POST_SHIFT) == 0u) {  // (no POST, no PBC)
        code.back().op |= (unary_id(i) << SR_OP_POST_SHIFT) | (infsub[i] ? SR_OP_POST_INF : 0u);
        if (arr_check[i]) {
          code.back().op |= SR_OP_POST_CHECK;
          ++n_checks;
        }
        return;
      }
      SrIns<T> in{};
      // fused unary: non-finite input -> +Inf
      in.op = (infsub[i] ? SR_OP_UNARY_INF0 : SR_OP_UNARY0) + unary_id(i);
      code.push_back(in);
      emit_check(i);
      return;
    }
    const int a = t.l[i], b = t.r[i];
    const uint32_t bop = binary_id(i);
    if (err != SR_OK) return;
    if (emit_pair(i, bop)) {
      // both operands in one instruction
    } else if (effleaf(b)) {  // op(tos = left, operand = right leaf)
      emit(a);
      if (fuse_const_operand(i, b, bop, false)) return;
      const_operand_check(b);
      code.push_back(operand_ins(b, bop, false));
    } else if (effleaf(a)) {  // op(operand = left leaf, tos = right)
      emit(b);
      if (fuse_const_operand(i, a, bop, true)) return;
      const_operand_check(a);
      code.push_back(operand_ins(a, bop, true));
    } else {  // the operand needing more slots first, pushed to slot `depth`; the other in tos
      const bool left_first = need[a] >= need[b];
      emit(left_first ? a : b);
      const size_t start = code.size();
      const int slot = depth;
      ++depth;
      if (depth > max_depth) max_depth = depth;
      emit(left_first ? b : a);
      mark_push(code[start], slot);
      --depth;
      code.push_back(stack_ins(bop, left_first, slot));
    }
    emit_check(i);
  }

  // Pre-order constant numbering (get_scalar_constants order).
  void number_constants() {
    reset_n(const_slot, t.n, -1);
    uint32_t k = 0;
    for (int64_t i = 0; i < t.n; ++i)
      if (t.degree[i] == 0 && t.constant[i]) const_slot[i] = int32_t(k++);
    n_consts = k;
  }

  // Compile tree `tree` (the vectors keep their capacity from the previous tree).
  bool run(const Tree<T>& tree) {
    t.degree = tree.degree;
    t.op = tree.op;
    t.feature = tree.feature;
    t.constant = tree.constant;
    t.val = tree.val;
    t.n = tree.n;
    code.clear();
    bad = false;
    err = SR_OK;
    msg.clear();
    depth = max_depth = 0;
    n_checks = n_consts = 0;
    n_ops = 0;
    if (!parse()) return false;
    const int64_t n = t.n;
    reset_n(folded, n, 0);
    reset_n(arr_check, n, 0);
    reset_n(infsub, n, 0);
    reset_n(fold_val, n, T(0));
    reset_n(need, n, 0);
    number_constants();
    // (is_const from parse(); gradient programs keep every constant leaf live: no folding)
    if (with_const_index) reset_n(is_const, n, 0);
    evalmark(0);
    arr_check[0] = 1;  // final is_bad_array check on the output
    if (err != SR_OK) return false;
    if (bad) {
      code.clear();
      return true;
    }
    compute_need(0);
    emit(0);
    if (err != SR_OK) return false;
    if (bad) code.clear();
    return true;
  }
};

}  // namespace

static uint32_t sr_unary_cost(uint32_t u) {
  switch (u) {
    case SR_U_NEG: case SR_U_SQUARE: case SR_U_CUBE: case SR_U_ABS: return 2;
    case SR_U_EXP: return 9;
    case SR_U_LOG: return 16;
    case SR_U_SQRT: return 8;
    case SR_U_COS: case SR_U_SIN: return 32;
    default: return 30;
  }
}

static uint32_t sr_instruction_cost_slow(uint32_t code) {
  const uint32_t post = (code >> SR_OP_POST_SHIFT) & 0x3fu;
  const uint32_t pbc = (code >> SR_OP_PBC_SHIFT) & 7u;
  uint32_t c = 6;  // dispatch + operand fetch + validity tracking
  if (post) c += 2 + sr_unary_cost(post) + ((code & SR_OP_POST_INF) ? 2u : 0u);
  if (pbc) c += 3 + ((pbc == SR_PBC_DIV_R || pbc == SR_PBC_DIV_L) ? 6u : 1u);
  code &= SR_OP_MASK;
  if (code == SR_OP_LOAD_FEAT_PUSH || code == SR_OP_LOAD_CONST_PUSH || code == SR_OP_LOAD_DERIVED_PUSH) c += 2;
  if (code == SR_OP_LOAD_DERIVED || code == SR_OP_LOAD_DERIVED_PUSH) return c + 3;
  if (code >= SR_OP_PAIR0) {
    c += ((code - SR_OP_PAIR0) % 6u >= SR_P_PUSH) ? 3 : 1;  // second operand (+ push)
    code = SR_OP_BINARY0 + (code - SR_OP_PAIR0) / 6u * 6u;  // priced as its binary operator
  }
  if (code >= SR_OP_BINARY0) {
    const uint32_t b = (code - SR_OP_BINARY0) / 6u + 1u;
    if (b == SR_B_DIV) c += 6;
    else if (b == SR_B_ADD || b == SR_B_SUB || b == SR_B_MUL) c += 1;
    else c += 20;
  } else if (code > SR_OP_UNARY0) {
    const uint32_t u = code >= SR_OP_UNARY_INF0 ? code - SR_OP_UNARY_INF0 : code - SR_OP_UNARY0;
    if (code >= SR_OP_UNARY_INF0) c += 2;
    c += sr_unary_cost(u);
  } else {
    c += 1;
  }
  return c;
}

// The same, from tables: the opcode's own cost (512 entries) plus the POST unary's (64) and the PBC
// binary's (8) — called per compiled instruction, a switch per call was ~10 % of a small batch
uint32_t sr_instruction_cost(uint32_t code) {
  struct Tabs {
    uint16_t op[SR_OP_MASK + 1], post[64], pbc[8];
    Tabs() {
      for (uint32_t c = 0; c <= SR_OP_MASK; ++c) op[c] = uint16_t(sr_instruction_cost_slow(c));
      for (uint32_t u = 0; u < 64; ++u) post[u] = uint16_t(u ? sr_instruction_cost_slow(u << SR_OP_POST_SHIFT) - op[0] : 0);
      for (uint32_t b = 0; b < 8; ++b) pbc[b] = uint16_t(b ? sr_instruction_cost_slow(b << SR_OP_PBC_SHIFT) - op[0] : 0);
    }
  };
  static const Tabs t;
  return t.op[code & SR_OP_MASK] + t.post[(code >> SR_OP_POST_SHIFT) & 0x3fu] + ((code & SR_OP_POST_INF) ? 2u : 0u) +
         t.pbc[(code >> SR_OP_PBC_SHIFT) & 7u];
}

uint32_t sr_unary_id(const char* name) {
  for (const auto& e : kUnary)
    if (std::strcmp(e.name, name) == 0) return e.id;
  return 0;
}
uint32_t sr_binary_id(const char* name) {
  for (const auto& e : kBinary)
    if (std::strcmp(e.name, name) == 0) return e.id;
  return 0;
}

void sr_parallel_for(int n, const std::function<void(int)>& fn) {
  if (n <= 1) {
    if (n == 1) fn(0);
    return;
  }
  WorkerPool::get().run(n, fn);
}

template <typename T>
int sr_compile_batch(const sr_tree_batch& trees, const SrOpset& ops, int64_t n_rows, int64_t nfeatures,
                     bool with_const_index, SrProgramBatch<T>* out, std::string* err, const int16_t* derived) {
  const int64_t nt = trees.n_trees;
  if (nt < 0 || (nt > 0 && (!trees.offsets || !trees.degree || !trees.op || !trees.feature ||
                            !trees.constant || !trees.val))) {
    *err = "sr_tree_batch has NULL arrays";
    return SR_ERR_INVALID_ARG;
  }
  // per tree: where its code sits in its thread's buffer, and its summary
  struct PerTree {
    int thread;
    uint32_t begin, len;
    uint8_t bad;
    uint32_t checks, consts, cost;
    int depth;
    int64_t nodes, ops;
  };
  std::vector<PerTree> per(size_t(nt > 0 ? nt : 0));
  std::vector<int> errs(size_t(nt > 0 ? nt : 0), SR_OK);
  const T* vals = static_cast<const T*>(trees.val);
  // work split: pieces of 32..256 trees, about four per persistent worker (round 5: 128 at least
  // left a 1,250-tree batch in 10 pieces, the caller and the first workers awake doing most of them:
  // the tree-sharding share's compile phase 0.13-0.14 -> 0.10-0.12 ms, profiles/r05_ab_exact_compile.txt);
  // batches of up to 128 trees compile on the caller alone (waking the pool costs more: 40 trees
  // 13-25 us through it against ~7 inline on the box, profiles/r04_latency_ab.txt)
  const int64_t pool = nt > 128 ? WorkerPool::get().size() : 1;
  static const int64_t min_piece = [] {
    const char* v = std::getenv("SR_AMD_COMPILE_PIECE");  // (A/B: the smallest piece)
    return v ? std::max<int64_t>(1, std::atoll(v)) : int64_t(32);
  }();
  const int64_t kPiece = std::max<int64_t>(min_piece, std::min<int64_t>(256, (nt + 4 * pool - 1) / (4 * pool)));
  const int n_pieces = int(nt <= kPiece ? 1 : (nt + kPiece - 1) / kPiece);
  const int nthreads = n_pieces;  // one code buffer per piece
  std::vector<std::vector<SrIns<T>>> bufs(static_cast<size_t>(nthreads));

  auto work = [&](int w, int64_t lo, int64_t hi) {
    TreeCompiler<T> tc(ops, n_rows, nfeatures, with_const_index, with_const_index ? nullptr : derived);
    std::vector<SrIns<T>>& buf = bufs[size_t(w)];
    buf.reserve(size_t(trees.offsets[hi] - trees.offsets[lo]));
    for (int64_t k = lo; k < hi; ++k) {
      const int64_t b = trees.offsets[k], e = trees.offsets[k + 1];
      if (e < b) {
        errs[k] = SR_ERR_BAD_TREE;
        continue;
      }
      Tree<T> tree;
      tree.degree = trees.degree + b;
      tree.op = trees.op + b;
      tree.feature = trees.feature + b;
      tree.constant = trees.constant + b;
      tree.val = vals + b;
      tree.n = e - b;
      tc.run(tree);
      if (tc.err != SR_OK) {
        errs[k] = tc.err;
        continue;
      }
      uint32_t cost = 0;
      for (const auto& in : tc.code) cost += sr_instruction_cost(in.op);
      PerTree& p = per[k];
      p.thread = w;
      p.begin = uint32_t(buf.size());
      p.len = uint32_t(tc.code.size());
      buf.insert(buf.end(), tc.code.begin(), tc.code.end());
      p.cost = cost;
      p.bad = (tc.bad || tc.code.empty()) ? 1 : 0;
      p.checks = tc.n_checks;
      p.consts = tc.n_consts;
      p.depth = tc.max_depth;
      p.nodes = e - b;
      p.ops = 0;
      for (int64_t i = b; i < e; ++i) p.ops += trees.degree[i] > 0 ? 1 : 0;
    }
  };
  if (n_pieces <= 1) {
    work(0, 0, nt);
  } else {
    WorkerPool::get().run(n_pieces, [&](int w) {
      const int64_t lo = int64_t(w) * kPiece, hi = (lo + kPiece < nt) ? lo + kPiece : nt;
      if (lo < hi) work(w, lo, hi);
    });
  }
  for (int64_t k = 0; k < nt; ++k)
    if (errs[k] != SR_OK) {
      *err = "tree " + std::to_string(k) + ": malformed tree or operator index";
      return errs[k];
    }
  out->code.clear();
  out->offsets.assign(size_t(nt + 1), 0);
  out->static_bad.assign(size_t(nt), 0);
  out->n_checks.assign(size_t(nt), 0);
  out->n_consts.assign(size_t(nt), 0);
  out->const_off.assign(size_t(nt + 1), 0);
  out->cost.assign(size_t(nt), 0);
  out->depth.assign(size_t(nt), 0);
  out->max_depth = 0;
  out->max_checks = 0;
  out->total_nodes = 0;
  out->total_ops = 0;
  size_t total = 0;
  for (int64_t k = 0; k < nt; ++k) total += per[k].len;
  out->n_code = total;
  const bool lazy = out->keep_pieces;
  if (lazy) {
    out->piece.resize(size_t(nt));
    out->begin.resize(size_t(nt));
  } else {
    out->code.resize(total);
  }
  size_t at = 0;
  for (int64_t k = 0; k < nt; ++k) {
    const PerTree& p = per[k];
    out->offsets[k] = uint32_t(at);
    if (lazy) {
      out->piece[size_t(k)] = uint32_t(p.thread);
      out->begin[size_t(k)] = p.begin;
    } else if (p.len) {
      std::memcpy(out->code.data() + at, bufs[size_t(p.thread)].data() + p.begin, size_t(p.len) * sizeof(SrIns<T>));
    }
    at += p.len;
    out->static_bad[k] = p.bad;
    out->cost[k] = p.bad ? 0u : p.cost;
    out->depth[k] = uint8_t(p.bad ? 0 : (p.depth > 255 ? 255 : p.depth));
    out->n_checks[k] = p.checks;
    out->n_consts[k] = p.consts;
    out->const_off[k + 1] = out->const_off[k] + p.consts;
    if (p.depth > out->max_depth) out->max_depth = p.depth;
    if (int(p.checks) > out->max_checks) out->max_checks = int(p.checks);
    out->total_nodes += p.nodes;
    out->total_ops += p.ops;
  }
  out->offsets[nt] = uint32_t(total);
  if (lazy) out->pieces = std::move(bufs);
  return SR_OK;
}

template int sr_compile_batch<float>(const sr_tree_batch&, const SrOpset&, int64_t, int64_t, bool,
                                     SrProgramBatch<float>*, std::string*, const int16_t*);
template int sr_compile_batch<double>(const sr_tree_batch&, const SrOpset&, int64_t, int64_t, bool,
                                      SrProgramBatch<double>*, std::string*, const int16_t*);
