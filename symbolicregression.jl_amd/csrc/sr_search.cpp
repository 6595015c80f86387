// sr_search.cpp — native equation_search engine: lock-step islands scored by batched device calls.
//
// Restates the reference's search around the scoring path:
//   * s_r_cycle (src/SingleIteration.jl:19-66): ncycles_per_iteration annealing temperatures
//     LinRange(1, 0), one reg_evol_cycle each, best-seen members per complexity;
//   * reg_evol_cycle (src/RegularizedEvolution.jl:12-160): ceil(n / tournament_selection_n) rounds of
//     tournament selection (best_of_sample, src/Population.jl:109-159 with argmin_fast / bottomk_fast,
//     src/Utils.jl:96-147), next_generation (src/Mutate.jl:174-356) or crossover_generation
//     (:661-733), replacing the oldest member(s);
//   * optimize_and_simplify_population (src/SingleIteration.jl:68-139) and finalize_costs
//     (src/Population.jl:182-196); _dispatch_s_r_cycle's best-seen re-scoring under batching
//     (src/SymbolicRegression.jl:1253-1296);
//   * the head node's per-island bookkeeping of _main_search_loop! (src/SymbolicRegression.jl:
//     1040-1140): running statistics (src/AdaptiveParsimony.jl), hall of fame (update_hall_of_fame!,
//     src/SearchUtils.jl:717-736; calculate_pareto_frontier, src/HallOfFame.jl:96-124), migration
//     (migrate!, src/Migration.jl:15-37 with poisson_sample, src/Utils.jl:149-157), get_cur_maxsize
//     (src/SearchUtils.jl:656-671).
//
// MI355X-first change: the islands advance in LOCK-STEP.  At every regularised-evolution round each
// owned island selects and mutates on the host, and the children of ALL islands are scored by ONE
// batched device call; each island's serial semantics (its next round sees its own replacements)
// are kept.  Constant optimisation runs batched over every island's selected members.  Islands shard
// across ranks (island i on rank i % world): a rank runs its islands' cycles, the ranks exchange
// islands (sr_search_export / sr_search_import over torch.distributed) and every rank replays the
// head's island-by-island bookkeeping identically; migration into an island is done by its owner
// with the island's own stream.  Random streams and birth counters are per island (sr_rng.h), so a
// sharded search equals the single-process one.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <memory>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/sr_amd.h"
#include "sr_compile.h"
#include "sr_constopt.h"
#include "sr_libm.h"
#include "sr_search_tree.h"

int sr_set_error(int code, const std::string& msg);  // sr_capi.cpp
int sr_ctx_swap_timing(sr_ctx* ctx, int value);        // sr_capi.cpp: set "timing", return the old value

namespace {

using Clock = std::chrono::steady_clock;
inline double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

template <typename T>
struct Member {
  SrTree<T> tree;
  T cost = T(0), loss = T(0);  // L == T
  int64_t birth = 0, ref = 0, parent = -1;
  int complexity = 0;
};

template <typename T>
struct Hof {
  std::vector<Member<T>> m;
  std::vector<uint8_t> exists;
  void reset(int maxsize) {
    m.assign(size_t(maxsize), Member<T>());
    exists.assign(size_t(maxsize), 0);
  }
};

// Julia isless on floats: NaN sorts last
template <typename T>
inline bool jl_isless(T a, T b) {
  if (a != a) return false;
  if (b != b) return true;
  return a < b;
}

struct Flat {
  std::vector<int64_t> offsets;
  std::vector<uint8_t> degree, op, constant;
  std::vector<uint16_t> feature;
  std::vector<double> vd;
  std::vector<float> vf;
  void clear() {
    offsets.assign(1, 0);
    degree.clear();
    op.clear();
    constant.clear();
    feature.clear();
    vd.clear();
    vf.clear();
  }
  template <typename T>
  void add(const SrTree<T>& t, const std::vector<double>* consts = nullptr) {
    size_t k = 0;
    for (const auto& n : t) {
      degree.push_back(n.degree);
      op.push_back(n.op);
      constant.push_back(n.constant);
      feature.push_back(n.feature);
      T v = n.val;
      if (consts && n.degree == 0 && n.constant) v = T((*consts)[k++]);
      if constexpr (sizeof(T) == 4)
        vf.push_back(v);
      else
        vd.push_back(v);
    }
    offsets.push_back(offsets.back() + int64_t(t.size()));
  }
  // the trees ks of this batch as a batch of their own (CPU scorers over several row views)
  Flat take(const std::vector<size_t>& ks) const {
    Flat f;
    f.clear();
    for (size_t k : ks) {
      const int64_t b = offsets[k], e = offsets[k + 1];
      f.degree.insert(f.degree.end(), degree.begin() + b, degree.begin() + e);
      f.op.insert(f.op.end(), op.begin() + b, op.begin() + e);
      f.constant.insert(f.constant.end(), constant.begin() + b, constant.begin() + e);
      f.feature.insert(f.feature.end(), feature.begin() + b, feature.begin() + e);
      if (!vf.empty()) f.vf.insert(f.vf.end(), vf.begin() + b, vf.begin() + e);
      if (!vd.empty()) f.vd.insert(f.vd.end(), vd.begin() + b, vd.begin() + e);
      f.offsets.push_back(f.offsets.back() + (e - b));
    }
    return f;
  }
  template <typename T>
  sr_tree_batch batch() const {
    sr_tree_batch b{};
    b.n_trees = int64_t(offsets.size()) - 1;
    b.offsets = offsets.data();
    b.degree = degree.data();
    b.op = op.data();
    b.feature = feature.data();
    b.constant = constant.data();
    if constexpr (sizeof(T) == 4)
      b.val = vf.data();
    else
      b.val = vd.data();
    return b;
  }
};

// ---------------------------------------------------------------- byte stream (island exchange)
struct Writer {
  std::vector<uint8_t> buf;
  template <typename V>
  void put(const V& v) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
    buf.insert(buf.end(), p, p + sizeof(V));
  }
};
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  template <typename V>
  V get() {
    V v{};
    if (p + sizeof(V) > end) {
      ok = false;
      return v;
    }
    memcpy(&v, p, sizeof(V));
    p += sizeof(V);
    return v;
  }
};

// The scoring calls of the search: the library's own device path, or CPU callbacks (tests).
template <typename T>
struct Scorer {
  sr_ctx* ctx = nullptr;
  const sr_dataset* ds = nullptr;
  int opset_id = -1, loss_code = 0;
  sr_loss_fn loss_cb = nullptr;
  sr_grad_fn grad_cb = nullptr;
  void* cb_user = nullptr;
  int64_t calls = 0;
  double ms = 0.0;  // wall time inside the calls
  double kernel_ms = 0.0;  // device-busy time of the loss calls' interpreter launches
  // (SR_AMD_SEARCH_KERNEL_TIMES=1: reading it costs every call its event queries, so off by default)
  bool time_kernels = [] {
    const char* v = std::getenv("SR_AMD_SEARCH_KERNEL_TIMES");
    return v && std::atoi(v) != 0;
  }();
  bool ready() const { return ctx != nullptr || loss_cb != nullptr; }
  bool has_grad() const { return ctx != nullptr || grad_cb != nullptr; }
  // Rows per tree (per-island minibatches): tree k on *rows[k] (all of one length); empty: every tree
  // on the full dataset.  -> the distinct views (tree_view, their rows concatenated); false when the
  // trees share one view (*one = it).
  using TreeRows = std::vector<const std::vector<int64_t>*>;
  static bool make_views(const TreeRows& tr, std::vector<int32_t>* tv, std::vector<int64_t>* cat, int* nv,
                         int64_t* len, const std::vector<int64_t>** one) {
    std::vector<const std::vector<int64_t>*> uniq;
    tv->resize(tr.size());
    for (size_t k = 0; k < tr.size(); ++k) {
      size_t u = 0;
      while (u < uniq.size() && uniq[u] != tr[k]) ++u;
      if (u == uniq.size()) uniq.push_back(tr[k]);
      (*tv)[k] = int32_t(u);
    }
    *one = uniq.empty() ? nullptr : uniq[0];
    if (uniq.size() <= 1) return false;
    *nv = int(uniq.size());
    *len = int64_t(uniq[0]->size());
    cat->clear();
    for (auto* r : uniq) cat->insert(cat->end(), r->begin(), r->end());
    return true;
  }
  int loss(const Flat& flat, const TreeRows& tr, std::vector<T>* out) {
    static const std::vector<int64_t> kAll;
    std::vector<int32_t> tv;
    std::vector<int64_t> cat;
    int nv = 1;
    int64_t len = 0;
    const std::vector<int64_t>* one = nullptr;
    if (tr.empty() || !make_views(tr, &tv, &cat, &nv, &len, &one)) return loss(flat, one ? *one : kAll, out);
    const int64_t nt = int64_t(flat.offsets.size()) - 1;
    out->assign(size_t(nt), T(0));
    const auto t0 = Clock::now();
    int rc = SR_OK;
    if (loss_cb) {  // CPU scorers: one callback per view over that view's trees
      for (int v = 0; v < nv && rc == SR_OK; ++v) {
        std::vector<size_t> ks;
        for (int64_t k = 0; k < nt; ++k)
          if (tv[size_t(k)] == v) ks.push_back(size_t(k));
        const Flat sub = flat.take(ks);
        const sr_tree_batch b = sub.batch<T>();
        std::vector<T> l(ks.size());
        std::vector<uint8_t> c(ks.size());
        rc = loss_cb(cb_user, &b, cat.data() + int64_t(v) * len, len, l.data(), c.data());
        for (size_t j = 0; j < ks.size(); ++j) (*out)[ks[j]] = c[j] ? l[j] : T(INFINITY);
      }
    } else {  // the device: every view in ONE call
      const sr_tree_batch b = flat.batch<T>();
      std::vector<uint8_t> comp(static_cast<size_t>(nt));
      const int timing_was = !time_kernels ? sr_ctx_swap_timing(ctx, 0) : -1;
      rc = sr_eval_loss_batch_views(ctx, ds, opset_id, &b, tv.data(), nv, cat.data(), len, loss_code, out->data(),
                                    comp.data());
      if (timing_was >= 0) sr_ctx_swap_timing(ctx, timing_was);
      for (int64_t k = 0; k < nt; ++k)
        if (!comp[size_t(k)]) (*out)[size_t(k)] = T(INFINITY);
    }
    ms += ms_since(t0);
    ++calls;
    return rc;
  }
  int grad(const Flat& flat, const TreeRows& tr, size_t n_consts, std::vector<T>* out, std::vector<T>* g,
           std::vector<uint8_t>* comp) {
    static const std::vector<int64_t> kAll;
    std::vector<int32_t> tv;
    std::vector<int64_t> cat;
    int nv = 1;
    int64_t len = 0;
    const std::vector<int64_t>* one = nullptr;
    if (tr.empty() || !make_views(tr, &tv, &cat, &nv, &len, &one)) return grad(flat, one ? *one : kAll, n_consts, out, g, comp);
    const sr_tree_batch b = flat.batch<T>();
    const int64_t nt = b.n_trees;
    out->assign(size_t(nt), T(0));
    g->assign(n_consts + 1, T(0));
    comp->assign(size_t(nt), 0);
    const auto t0 = Clock::now();
    int rc = SR_OK;
    if (grad_cb) {  // CPU scorers: one callback per view; the gradient slots scattered back per tree
      std::vector<size_t> coff(size_t(nt) + 1, 0);
      for (int64_t k = 0; k < nt; ++k) {
        size_t c = 0;
        for (int64_t i = b.offsets[k]; i < b.offsets[k + 1]; ++i) c += (b.degree[i] == 0 && b.constant[i]) ? 1 : 0;
        coff[size_t(k) + 1] = coff[size_t(k)] + c;
      }
      for (int v = 0; v < nv && rc == SR_OK; ++v) {
        std::vector<size_t> ks;
        size_t nc = 0;
        for (int64_t k = 0; k < nt; ++k)
          if (tv[size_t(k)] == v) {
            ks.push_back(size_t(k));
            nc += coff[size_t(k) + 1] - coff[size_t(k)];
          }
        const Flat sub = flat.take(ks);
        const sr_tree_batch sb = sub.batch<T>();
        std::vector<T> l(ks.size()), gg(nc + 1);
        std::vector<uint8_t> c(ks.size());
        rc = grad_cb(cb_user, &sb, cat.data() + int64_t(v) * len, len, l.data(), gg.data(), c.data());
        size_t at = 0;
        for (size_t j = 0; j < ks.size(); ++j) {
          (*out)[ks[j]] = l[j];
          (*comp)[ks[j]] = c[j];
          for (size_t q = coff[ks[j]]; q < coff[ks[j] + 1]; ++q) (*g)[q] = gg[at++];
        }
      }
    } else {
      const int timing_was = !time_kernels ? sr_ctx_swap_timing(ctx, 0) : -1;
      rc = sr_eval_grad_batch_views(ctx, ds, opset_id, &b, tv.data(), nv, cat.data(), len, loss_code, out->data(),
                                    g->data(), comp->data());
      if (timing_was >= 0) sr_ctx_swap_timing(ctx, timing_was);
    }
    ms += ms_since(t0);
    ++calls;
    return rc;
  }
  // A round's scoring call in two halves (round_submit / round_finish): the call runs whole at submit
  // (round 5's asynchronous device call and two-half lane pipeline were measured without payoff and
  // removed in round 6: profiles/r05_ab_search_pipeline.txt); loss_wait is then a no-op.
  struct AsyncLoss {
    std::vector<T>* out = nullptr;
  };
  int loss_submit(const Flat& flat, const TreeRows& tr, std::vector<T>* out, AsyncLoss* a) {
    a->out = out;
    return loss(flat, tr, out);
  }
  int loss_wait(AsyncLoss*) { return SR_OK; }
  // losses of `flat`'s trees (+Inf where incomplete)
  int loss(const Flat& flat, const std::vector<int64_t>& rows, std::vector<T>* out) {
    const sr_tree_batch b = flat.batch<T>();
    const int64_t nt = b.n_trees;
    out->assign(size_t(nt), T(0));
    if (nt == 0) return SR_OK;
    std::vector<uint8_t> comp(static_cast<size_t>(nt));
    const int64_t* r = rows.empty() ? nullptr : rows.data();
    const auto t0 = Clock::now();
    // (no timing events on the search's small calls unless their kernel times are wanted; the
    // context's own setting is restored afterwards)
    const int timing_was = (!loss_cb && !time_kernels) ? sr_ctx_swap_timing(ctx, 0) : -1;
    const int rc = loss_cb ? loss_cb(cb_user, &b, r, int64_t(rows.size()), out->data(), comp.data())
                           : sr_eval_loss_batch(ctx, ds, opset_id, &b, r, int64_t(rows.size()), loss_code, out->data(),
                                                comp.data());
    if (timing_was >= 0) sr_ctx_swap_timing(ctx, timing_was);
    ms += ms_since(t0);
    ++calls;
    if (rc != SR_OK) return rc;
    if (!loss_cb && time_kernels) {  // the interpreter launches' device-busy time of this call
      double ph[9] = {0};
      if (sr_last_phase_ms(ctx, ph, 9) == SR_OK) kernel_ms += ph[8];
    }
    for (int64_t k = 0; k < nt; ++k)
      if (!comp[size_t(k)]) (*out)[size_t(k)] = T(INFINITY);
    return SR_OK;
  }
  // losses and d loss / d constants (pre-order per tree, concatenated)
  int grad(const Flat& flat, const std::vector<int64_t>& rows, size_t n_consts, std::vector<T>* out,
           std::vector<T>* g, std::vector<uint8_t>* comp) {
    const sr_tree_batch b = flat.batch<T>();
    out->assign(size_t(b.n_trees), T(0));
    g->assign(n_consts + 1, T(0));
    comp->assign(size_t(b.n_trees), 0);
    if (b.n_trees == 0) return SR_OK;
    const int64_t* r = rows.empty() ? nullptr : rows.data();
    const auto t0 = Clock::now();
    const int timing_was = (!grad_cb && !time_kernels) ? sr_ctx_swap_timing(ctx, 0) : -1;
    const int rc = grad_cb ? grad_cb(cb_user, &b, r, int64_t(rows.size()), out->data(), g->data(), comp->data())
                           : sr_eval_grad_batch(ctx, ds, opset_id, &b, r, int64_t(rows.size()), loss_code, out->data(),
                                                g->data(), comp->data());
    if (timing_was >= 0) sr_ctx_swap_timing(ctx, timing_was);
    ms += ms_since(t0);
    ++calls;
    return rc;
  }
};

// The BFGS objective over a batch of trees: f / grad f of item k = tree k with constants xs[k]
// (rounded to T), one batched device call per evaluation round.
template <typename T>
struct TreeObjective : SrObjective {
  using TreeRows = typename Scorer<T>::TreeRows;
  Scorer<T>* sc;
  Flat* flat;
  const std::vector<const SrTree<T>*>* trees;
  const TreeRows* rows;  // per tree (its island's minibatch), or empty: the full dataset
  std::vector<int64_t> f_calls;
  TreeRows rows_of(const std::vector<int>& items) const {
    TreeRows r;
    if (!rows->empty())
      for (int k : items) r.push_back((*rows)[size_t(k)]);
    return r;
  }
  int f(const std::vector<int>& items, const std::vector<std::vector<double>>& xs, std::vector<double>* out) override {
    flat->clear();
    for (size_t j = 0; j < items.size(); ++j) {
      flat->add(*(*trees)[size_t(items[j])], &xs[j]);
      if (counting) ++f_calls[size_t(items[j])];
    }
    std::vector<T> loss;
    const int rc = sc->loss(*flat, rows_of(items), &loss);
    if (rc) return rc;
    out->resize(loss.size());
    for (size_t j = 0; j < loss.size(); ++j) (*out)[j] = double(loss[j]);
    return SR_OK;
  }
  int fg(const std::vector<int>& items, const std::vector<std::vector<double>>& xs, std::vector<double>* out,
         std::vector<std::vector<double>>* grads) override {
    flat->clear();
    size_t nc = 0;
    for (size_t j = 0; j < items.size(); ++j) {
      flat->add(*(*trees)[size_t(items[j])], &xs[j]);
      if (counting) ++f_calls[size_t(items[j])];
      nc += xs[j].size();
    }
    std::vector<T> loss, g;
    std::vector<uint8_t> comp;
    const int rc = sc->grad(*flat, rows_of(items), nc, &loss, &g, &comp);
    if (rc != SR_OK) return rc;
    out->resize(items.size());
    grads->resize(items.size());
    size_t at = 0;
    for (size_t j = 0; j < items.size(); ++j) {
      (*out)[j] = comp[j] ? double(loss[j]) : INFINITY;
      (*grads)[j].assign(xs[j].size(), 0.0);
      for (size_t q = 0; q < xs[j].size(); ++q) (*grads)[j][q] = double(g[at + q]);
      at += xs[j].size();
    }
    return SR_OK;
  }
};

// optimize_constants (src/ConstantOptimization.jl:29-116) for a batch of trees with the perturbed
// restart points already drawn: best constants per tree, whether the minimum beat the start, the
// loss at the adopted constants (one more batched call, f(result.minimizer)) and f_calls per tree.
template <typename T>
int optimize_trees(Scorer<T>& sc, Flat& flat, const std::vector<const SrTree<T>*>& trees,
                   const std::vector<std::vector<double>>& x0,
                   const std::vector<std::vector<std::vector<double>>>& restarts, int iterations,
                   const typename Scorer<T>::TreeRows& rows, std::vector<std::vector<double>>* best_x,
                   std::vector<uint8_t>* improved, std::vector<T>* adopted_loss, std::vector<int64_t>* f_calls,
                   int64_t f_calls_limit) {
  const size_t n = trees.size();
  TreeObjective<T> obj;
  obj.sc = &sc;
  obj.flat = &flat;
  obj.trees = &trees;
  obj.rows = &rows;
  obj.f_calls.assign(n, 0);
  std::vector<double> bf, base;
  int rc = sr_optimize_batch(obj, x0, restarts, iterations, best_x, &bf, &base, f_calls_limit);
  if (rc) return rc;
  improved->assign(n, 0);
  adopted_loss->assign(n, T(0));
  std::vector<size_t> better;
  for (size_t k = 0; k < n; ++k)
    if (bf[k] < base[k]) {
      (*improved)[k] = 1;
      better.push_back(k);
    } else {
      (*adopted_loss)[k] = T(base[k]);
    }
  if (!better.empty()) {
    flat.clear();
    typename Scorer<T>::TreeRows br;
    for (size_t k : better) {
      flat.add(*trees[k], &(*best_x)[k]);
      if (!rows.empty()) br.push_back(rows[k]);
    }
    std::vector<T> loss;
    if ((rc = sc.loss(flat, br, &loss))) return rc;
    for (size_t j = 0; j < better.size(); ++j) (*adopted_loss)[better[j]] = loss[j];
  }
  *f_calls = obj.f_calls;
  return SR_OK;
}

// one restart point x0 .* (1 + eps/2), eps ~ randn(T), in T (src/ConstantOptimization.jl:95-97)
template <typename T>
void draw_restart(SrRng& rng, const std::vector<double>& x0, std::vector<double>* xt) {
  xt->resize(x0.size());
  for (size_t q = 0; q < x0.size(); ++q) {
    const T eps = T(rng.normal());
    (*xt)[q] = double(T(x0[q]) * (T(1) + T(0.5) * eps));
  }
}

}  // namespace

struct sr_search_base {
  virtual ~sr_search_base() = default;
  int dtype = SR_DTYPE_F32;
};

namespace {

template <typename T>
struct Engine : sr_search_base {
  sr_search_options o{};
  SrTreeSpec sp;
  int64_t n_rows = 0;
  uint64_t seed = 0;
  int rank = 0, world = 1;
  std::vector<int> owned;
  Scorer<T> sc;
  // dataset-level state (update_baseline_loss!)
  T baseline = T(1);
  bool use_baseline = false;
  // islands
  std::vector<std::vector<Member<T>>> pops;
  std::vector<SrRng> rngs;
  std::vector<int64_t> births, refs;
  std::vector<Hof<T>> best_seen;
  std::vector<std::vector<Member<T>>> best_sub;
  std::vector<std::vector<double>> snap;  // normalized frequencies handed to each island's next cycle
  std::vector<int> cur_maxsize;           // maxsize handed to each island's next cycle
  // head
  std::vector<double> freq;
  Hof<T> hof;
  int64_t total_cycles = 1, cycles_remaining = 1;
  int head_maxsize = 1;  // state.cur_maxsizes[j]
  int iteration = 0;
  // accounting
  double num_evals = 0.0;
  const bool profile_lanes = [] {
    const char* v = std::getenv("SR_AMD_SEARCH_PROFILE");
    return v && std::atoi(v) != 0;
  }();
  int64_t s_r_cycles = 0;
  double host_ms = 0.0;
  Flat flat;
  // Scoring lanes: lane 0 is (sc, flat, num_evals, host_ms); further lanes (sr_search_add_device:
  // their own context and dataset copy) each run a share of the owned islands' iteration on their
  // own host thread, so one lane's device round trip overlaps the others' host work and calls.
  struct Lane {
    Scorer<T>* sc;
    Flat* flat;
    double* num_evals;
    double* host_ms;
  };
  struct ExtraLane {
    Scorer<T> sc;
    Flat flat;
    double num_evals = 0.0, host_ms = 0.0;
  };
  std::vector<std::unique_ptr<ExtraLane>> extra;
  Lane lane0() { return Lane{&sc, &flat, &num_evals, &host_ms}; }
  double total_num_evals() const {
    double v = num_evals;
    for (const auto& x : extra) v += x->num_evals;
    return v;
  }

  bool owns(int i) const { return i % world == rank; }
  int64_t new_birth(int i) { return ++births[size_t(i)]; }
  int64_t new_ref(int i) { return (int64_t(i + 1) << 40) | ++refs[size_t(i)]; }

  // ------------------------------------------------------------ scoring
  // loss_to_cost (src/LossFunctions.jl:169-190) in L
  T cost_of(T loss, int complexity) const {
    const T norm = (baseline >= T(0.01) && use_baseline) ? baseline : T(0.01);
    T v = loss / norm;
    v = v + T(float(complexity) * o.parsimony);
    return v;
  }
  using TreeRows = typename Scorer<T>::TreeRows;
  // each tree's rows: its island's minibatch (batching), or none (the full dataset)
  TreeRows rows_for(const std::vector<int>& island, const std::vector<std::vector<int64_t>>& by_island) const {
    TreeRows r;
    if (o.batching)
      for (int i : island) r.push_back(&by_island[size_t(i)]);
    return r;
  }
  int score_trees(Lane L, const std::vector<const SrTree<T>*>& trees, const TreeRows& rows,
                  std::vector<T>* loss, std::vector<T>* cost) {
    L.flat->clear();
    for (auto* t : trees) L.flat->add(*t);
    int rc = L.sc->loss(*L.flat, rows, loss);
    if (rc) return rc;
    cost->resize(loss->size());
    for (size_t k = 0; k < loss->size(); ++k) (*cost)[k] = cost_of((*loss)[k], int(trees[k]->size()));
    return SR_OK;
  }
  double fraction(const TreeRows& rows) const {
    return rows.empty() ? 1.0 : double(rows[0]->size()) / double(n_rows);
  }

  // ------------------------------------------------------------ constant optimisation
  // optimize_constants over members (pointers); perturbation draws come from each member's island
  // stream, in member order (deterministic whatever the batch composition)
  int optimize_members(Lane L, const std::vector<Member<T>*>& ms, const std::vector<int>& island,
                       const std::vector<std::vector<int64_t>>& rows_by_island, std::vector<uint8_t>* improved_out) {
    const TreeRows rows = rows_for(island, rows_by_island);
    const size_t n = ms.size();
    improved_out->assign(n, 0);
    if (n == 0) return SR_OK;
    if (!L.sc->has_grad()) return sr_set_error(SR_ERR_INVALID_ARG, "constant optimisation needs a gradient scorer");
    std::vector<const SrTree<T>*> trees(n);
    std::vector<std::vector<double>> x0(n);
    for (size_t k = 0; k < n; ++k) {
      trees[k] = &ms[k]->tree;
      for (const auto& nd : ms[k]->tree)
        if (nd.degree == 0 && nd.constant) x0[k].push_back(double(nd.val));
    }
    std::vector<std::vector<std::vector<double>>> restarts(size_t(o.optimizer_nrestarts),
                                                           std::vector<std::vector<double>>(n));
    for (size_t k = 0; k < n; ++k)
      for (int r = 0; r < o.optimizer_nrestarts; ++r) draw_restart<T>(rngs[size_t(island[k])], x0[k], &restarts[size_t(r)][k]);
    std::vector<std::vector<double>> bx;
    std::vector<uint8_t> imp;
    std::vector<T> loss;
    std::vector<int64_t> f_calls;
    const int rc = optimize_trees<T>(*L.sc, *L.flat, trees, x0, restarts, o.optimizer_iterations, rows, &bx, &imp, &loss, &f_calls,
                                    o.optimizer_f_calls_limit);
    if (rc) return rc;
    const double frac = fraction(rows);
    for (size_t k = 0; k < n; ++k) {
      *L.num_evals += double(f_calls[k]) * frac;
      if (!imp[k]) continue;
      // adopt: constants, the loss at the minimiser, cost, birth
      Member<T>& m = *ms[k];
      size_t q = 0;
      for (auto& nd : m.tree)
        if (nd.degree == 0 && nd.constant) nd.val = T(bx[k][q++]);
      m.loss = loss[k];
      m.cost = cost_of(m.loss, m.complexity);
      m.birth = new_birth(island[k]);
      *L.num_evals += frac;
      (*improved_out)[k] = 1;
    }
    return SR_OK;
  }

  // ------------------------------------------------------------ selection
  std::vector<float> tweights;
  void make_tournament_weights() {
    const float p = o.tournament_selection_p;
    tweights.resize(size_t(o.tournament_selection_n));
    for (int k = 0; k < o.tournament_selection_n; ++k) tweights[size_t(k)] = p * float(pow(double(1.0f - p), k));
  }
  // StatsBase.sample(Weights): first index whose running Float32 sum reaches rand() * sum
  int draw_place(SrRng& rng) {
    float total = 0.0f;
    for (float w : tweights) total += w;
    const double t = rng.uniform() * double(total);
    size_t i = 0;
    float cw = tweights[0];
    while (double(cw) < t && i + 1 < tweights.size()) {
      ++i;
      cw += tweights[i];
    }
    return int(i);
  }
  // best_of_sample (a copy of the winner)
  Member<T> best_of_sample(int i) {
    SrRng& rng = rngs[size_t(i)];
    const auto& pop = pops[size_t(i)];
    const int64_t np = int64_t(pop.size());
    const int64_t n = std::min<int64_t>(o.tournament_selection_n, np);
    std::vector<int64_t> idx(static_cast<size_t>(np));
    for (int64_t k = 0; k < np; ++k) idx[size_t(k)] = k;
    for (int64_t k = 0; k < n; ++k) std::swap(idx[size_t(k)], idx[size_t(k + rng.below(np - k))]);
    std::vector<T> adj(static_cast<size_t>(n));
    const std::vector<double>& nf = snap[size_t(i)];
    for (int64_t k = 0; k < n; ++k) {
      const Member<T>& m = pop[size_t(idx[size_t(k)])];
      if (o.use_frequency_in_tournament) {
        const T scaling = T(o.adaptive_parsimony_scaling);
        const T f = (m.complexity > 0 && m.complexity <= o.maxsize) ? T(nf[size_t(m.complexity - 1)]) : T(0);
        T e;
        if constexpr (sizeof(T) == 4)
          e = sr_expf(scaling * f);
        else
          e = exp(scaling * f);
        adj[size_t(k)] = m.cost * e;
      } else {
        adj[size_t(k)] = m.cost;
      }
    }
    const int place = o.tournament_selection_p == 1.0f ? 0 : draw_place(rng);
    // bottomk_fast / argmin_fast: strict <, values must beat typemax (Inf), the initial index 1
    // stays when fewer than place + 1 values qualify
    const int K = place + 1;
    std::vector<T> mv(static_cast<size_t>(K), T(INFINITY));
    std::vector<int64_t> mi(static_cast<size_t>(K), 0);
    for (int64_t k = 0; k < n; ++k) {
      if (adj[size_t(k)] < mv[size_t(K - 1)]) {
        mv[size_t(K - 1)] = adj[size_t(k)];
        mi[size_t(K - 1)] = k;
        for (int q = K - 1; q > 0; --q)
          if (mv[size_t(q)] < mv[size_t(q - 1)]) {
            std::swap(mv[size_t(q)], mv[size_t(q - 1)]);
            std::swap(mi[size_t(q)], mi[size_t(q - 1)]);
          }
      }
    }
    return pop[size_t(idx[size_t(mi[size_t(K - 1)])])];
  }

  // ------------------------------------------------------------ mutation choice
  void condition_weights(const Member<T>& m, int curmax, double* w) const {
    const SrTree<T>& t = m.tree;
    if (t[0].degree == 0) {
      w[SR_MUT_MUTATE_OPERATOR] = w[SR_MUT_SWAP_OPERANDS] = w[SR_MUT_DELETE_NODE] = w[SR_MUT_SIMPLIFY] = 0.0;
      if (!t[0].constant) {
        w[SR_MUT_OPTIMIZE] = 0.0;
        w[SR_MUT_MUTATE_CONSTANT] = 0.0;
      } else {
        w[SR_MUT_MUTATE_FEATURE] = 0.0;
      }
      return;
    }
    bool bin = false;
    for (const auto& n : t) bin |= n.degree == 2;
    if (!bin) w[SR_MUT_SWAP_OPERANDS] = 0.0;
    w[SR_MUT_MUTATE_CONSTANT] *= double(std::min(8, sr_count_constants(t))) / 8.0;
    if (sp.nfeatures <= 1) w[SR_MUT_MUTATE_FEATURE] = 0.0;
    if (m.complexity >= curmax) w[SR_MUT_ADD_NODE] = w[SR_MUT_INSERT_NODE] = 0.0;
    if (!o.should_simplify) w[SR_MUT_SIMPLIFY] = 0.0;
  }
  // sample_mutation: one draw proportional to the conditioned weights
  int sample_mutation(const double* w, SrRng& rng) const {
    double total = 0.0;
    for (int k = 0; k < SR_N_MUTATIONS; ++k) total += w[k];
    const double r = rng.uniform() * total;
    double acc = 0.0;
    for (int k = 0; k < SR_N_MUTATIONS; ++k) {
      acc += w[k];
      if (r < acc) return k;
    }
    for (int k = SR_N_MUTATIONS - 1; k >= 0; --k)
      if (w[k] > 0) return k;
    return SR_MUT_DO_NOTHING;
  }
  void apply_mutation(int choice, SrTree<T>& t, double temperature, int curmax, SrRng& rng) const {
    switch (choice) {
      case SR_MUT_MUTATE_CONSTANT: sr_mutate_constant(t, sp, temperature, rng); break;
      case SR_MUT_MUTATE_OPERATOR: sr_mutate_operator(t, sp, rng); break;
      case SR_MUT_MUTATE_FEATURE: sr_mutate_feature(t, sp, rng); break;
      case SR_MUT_SWAP_OPERANDS: sr_swap_operands(t, rng); break;
      case SR_MUT_ROTATE_TREE: sr_rotate_tree(t, rng); break;
      case SR_MUT_ADD_NODE:
        if (rng.uniform() < 0.5)
          sr_append_random_op(t, sp, rng);
        else
          sr_prepend_random_op(t, sp, rng);
        break;
      case SR_MUT_INSERT_NODE: sr_insert_random_op(t, sp, rng); break;
      case SR_MUT_DELETE_NODE: sr_delete_random_op(t, rng); break;
      case SR_MUT_RANDOMIZE: t = sr_gen_random_tree_fixed_size<T>(int(1 + rng.below(curmax)), sp, rng); break;
      default: break;
    }
  }

  // replace the oldest member (argmin_fast over births: first minimum)
  void replace_oldest(int i, Member<T>&& b) {
    auto& pop = pops[size_t(i)];
    size_t k = 0;
    for (size_t j = 1; j < pop.size(); ++j)
      if (pop[j].birth < pop[k].birth) k = j;
    pop[k] = std::move(b);
  }
  void replace_two_oldest(int i, Member<T>&& b1, Member<T>&& b2) {
    auto& pop = pops[size_t(i)];
    size_t k1 = 0;
    for (size_t j = 1; j < pop.size(); ++j)
      if (pop[j].birth < pop[k1].birth) k1 = j;
    size_t k2 = k1 == 0 ? 1 : 0;
    for (size_t j = 0; j < pop.size(); ++j)
      if (j != k1 && pop[j].birth < pop[k2].birth) k2 = j;
    pop[k1] = std::move(b1);
    pop[k2] = std::move(b2);
  }

  // ------------------------------------------------------------ one lock-step round
  enum Kind { K_MUT, K_CROSS, K_KEEP, K_REJECT, K_CROSS_FAIL, K_OPT, K_SIMPLIFIED };
  struct Plan {
    Kind kind;
    int island;
    Member<T> parent, parent2;
    SrTree<T> tree, tree2;
    size_t slot = 0;
  };

  // One regularised-evolution round of a set of islands, in two halves: round_submit selects and mutates
  // (host) and scores every island's children with ONE call; round_finish replaces members.
  struct RoundState {
    std::vector<Plan> plans;
    std::vector<const SrTree<T>*> pending;
    std::vector<int> pend_island;
    TreeRows rows;
    std::vector<T> loss, cost;
    typename Scorer<T>::AsyncLoss async;
    double temperature = 1.0;
  };
  int round(Lane L, const std::vector<int>& islands, double temperature,
            const std::vector<std::vector<int64_t>>& rows_by_island) {
    RoundState st;
    int rc = round_submit(L, islands, temperature, rows_by_island, &st);
    if (rc) return rc;
    return round_finish(L, rows_by_island, &st);
  }
  int round_submit(Lane L, const std::vector<int>& islands, double temperature,
                   const std::vector<std::vector<int64_t>>& rows_by_island, RoundState* st) {
    st->temperature = temperature;
    std::vector<Plan>& plans = st->plans;
    plans.clear();
    plans.reserve(islands.size());
    std::vector<const SrTree<T>*>& pending = st->pending;
    pending.clear();
    auto tp = Clock::now();
    for (int i : islands) {
      SrRng& rng = rngs[size_t(i)];
      const int curmax = cur_maxsize[size_t(i)];
      Plan pl;
      pl.island = i;
      if (rng.uniform() > double(o.crossover_probability)) {
        pl.parent = best_of_sample(i);
        double w[SR_N_MUTATIONS];
        for (int k = 0; k < SR_N_MUTATIONS; ++k) w[k] = o.mutation_weights[k];
        condition_weights(pl.parent, curmax, w);
        const int choice = sample_mutation(w, rng);
        if (choice == SR_MUT_DO_NOTHING) {
          pl.kind = K_KEEP;
        } else if (choice == SR_MUT_SIMPLIFY) {
          pl.kind = K_SIMPLIFIED;
          pl.tree = pl.parent.tree;
          sr_simplify_tree(pl.tree, sp);
        } else if (choice == SR_MUT_OPTIMIZE) {
          pl.kind = K_OPT;
        } else {
          bool ok = false;
          for (int attempt = 0; attempt < 10 && !ok; ++attempt) {
            pl.tree = pl.parent.tree;
            apply_mutation(choice, pl.tree, temperature, curmax, rng);
            ok = sr_check_constraints(pl.tree, sp, curmax);
          }
          pl.kind = ok ? K_MUT : K_REJECT;
        }
      } else {
        pl.parent = best_of_sample(i);
        pl.parent2 = best_of_sample(i);
        bool ok = false;
        for (int tries = 1; tries <= 11 && !ok; ++tries) {
          sr_crossover_trees(pl.parent.tree, pl.parent2.tree, rng, &pl.tree, &pl.tree2);
          ok = sr_check_constraints(pl.tree, sp, curmax) && sr_check_constraints(pl.tree2, sp, curmax);
        }
        pl.kind = ok ? K_CROSS : K_CROSS_FAIL;
      }
      plans.push_back(std::move(pl));
    }
    std::vector<int>& pend_island = st->pend_island;
    pend_island.clear();
    for (auto& pl : plans) {
      if (pl.kind == K_MUT || pl.kind == K_CROSS) {
        pl.slot = pending.size();
        pending.push_back(&pl.tree);
        pend_island.push_back(pl.island);
        if (pl.kind == K_CROSS) {
          pending.push_back(&pl.tree2);
          pend_island.push_back(pl.island);
        }
      }
    }
    // device: ONE batched eval_cost for every island's children (each on its island's minibatch)
    st->rows = rows_for(pend_island, rows_by_island);
    L.flat->clear();
    for (auto* t : pending) L.flat->add(*t);
    *L.host_ms += ms_since(tp);
    return L.sc->loss_submit(*L.flat, st->rows, &st->loss, &st->async);
  }
  int round_finish(Lane L, const std::vector<std::vector<int64_t>>& rows_by_island, RoundState* st) {
    int rc = L.sc->loss_wait(&st->async);
    if (rc) return rc;
    std::vector<Plan>& plans = st->plans;
    const std::vector<T>& loss = st->loss;
    std::vector<T>& cost = st->cost;
    cost.resize(loss.size());
    for (size_t k = 0; k < loss.size(); ++k) cost[k] = cost_of(loss[k], int(st->pending[k]->size()));
    const double temperature = st->temperature;
    const double frac = fraction(st->rows);
    *L.num_evals += double(st->pending.size()) * frac;
    // batched optimize mutations (rare: weight 0 by default)
    {
      std::vector<Member<T>*> om;
      std::vector<int> oi;
      for (auto& pl : plans)
        if (pl.kind == K_OPT && sr_count_constants(pl.parent.tree) > 0) {
          om.push_back(&pl.parent);
          oi.push_back(pl.island);
        }
      std::vector<uint8_t> imp;
      if ((rc = optimize_members(L, om, oi, rows_by_island, &imp))) return rc;
    }
    const auto tp = Clock::now();
    for (auto& pl : plans) {
      const int i = pl.island;
      SrRng& rng = rngs[size_t(i)];
      switch (pl.kind) {
        case K_KEEP: {  // do_nothing: a new member with the parent's tree, cost and loss
          Member<T> b = pl.parent;
          b.parent = pl.parent.ref;
          b.ref = new_ref(i);
          b.birth = new_birth(i);
          replace_oldest(i, std::move(b));
          break;
        }
        case K_SIMPLIFIED: {
          Member<T> b = pl.parent;
          b.tree = std::move(pl.tree);
          b.complexity = int(b.tree.size());
          b.parent = pl.parent.ref;
          b.ref = new_ref(i);
          b.birth = new_birth(i);
          replace_oldest(i, std::move(b));
          break;
        }
        case K_OPT:  // optimize: the (possibly re-fitted) copy replaces the oldest as it is
          replace_oldest(i, std::move(pl.parent));
          break;
        case K_REJECT: {
          if (o.skip_mutation_failures) break;
          Member<T> b = pl.parent;
          b.parent = pl.parent.ref;
          b.ref = new_ref(i);
          b.birth = new_birth(i);
          replace_oldest(i, std::move(b));
          break;
        }
        case K_CROSS_FAIL:  // the two sampled copies themselves (same births)
          if (!o.skip_mutation_failures) replace_two_oldest(i, std::move(pl.parent), std::move(pl.parent2));
          break;
        case K_CROSS: {
          Member<T> b1, b2;
          b1.tree = std::move(pl.tree);
          b1.complexity = int(b1.tree.size());
          b1.loss = loss[pl.slot];
          b1.cost = cost[pl.slot];
          b1.parent = pl.parent.ref;
          b1.ref = new_ref(i);
          b1.birth = new_birth(i);
          b2.tree = std::move(pl.tree2);
          b2.complexity = int(b2.tree.size());
          b2.loss = loss[pl.slot + 1];
          b2.cost = cost[pl.slot + 1];
          b2.parent = pl.parent2.ref;
          b2.ref = new_ref(i);
          b2.birth = new_birth(i);
          replace_two_oldest(i, std::move(b1), std::move(b2));
          break;
        }
        case K_MUT: {
          const T after = cost[pl.slot];
          bool accept = !(after != after);  // NaN cost: rejected
          if (accept) {
            double prob = 1.0;
            if (o.annealing) {
              const T delta = after - pl.parent.cost;
              prob *= exp(-double(delta) / (temperature * double(o.alpha)));
            }
            const int new_size = int(pl.tree.size());
            if (o.use_frequency) {
              const std::vector<double>& nf = snap[size_t(i)];
              const int old_size = pl.parent.complexity;
              const double of = (old_size > 0 && old_size <= o.maxsize) ? nf[size_t(old_size - 1)] : 1e-6;
              const double nw = (new_size > 0 && new_size <= o.maxsize) ? nf[size_t(new_size - 1)] : 1e-6;
              prob *= of / nw;
            }
            accept = !(prob < rng.uniform());
          }
          if (accept) {
            Member<T> b;
            b.tree = std::move(pl.tree);
            b.complexity = int(b.tree.size());
            b.loss = loss[pl.slot];
            b.cost = after;
            b.parent = pl.parent.ref;
            b.ref = new_ref(i);
            b.birth = new_birth(i);
            replace_oldest(i, std::move(b));
          } else if (!o.skip_mutation_failures) {
            Member<T> b = pl.parent;
            b.parent = pl.parent.ref;
            b.ref = new_ref(i);
            b.birth = new_birth(i);
            replace_oldest(i, std::move(b));
          }
          break;
        }
      }
    }
    *L.host_ms += ms_since(tp);
    return SR_OK;
  }

  // ------------------------------------------------------------ minibatches
  // batch(dataset, batch_size): rows drawn with replacement (src/Dataset.jl:303-304), one minibatch
  // per island per iteration for its s_r_cycle (salt 0, src/SingleIteration.jl:40) and one for its
  // constant optimisation (salt 1, :77), each from its own stream keyed by (seed, iteration, island):
  // independent of the island's other draws, of lanes and of which rank owns the island.  The device
  // scores every island's trees on their own rows in one launch (sr_eval_loss_batch_views).
  std::vector<int64_t> draw_batch(int island, uint64_t salt) const {
    std::vector<int64_t> rows;
    if (!o.batching) return rows;
    SrRng r;
    r.seed(seed ^ 0x6261746368ull, (uint64_t(iteration) * uint64_t(o.populations) + uint64_t(island)) * 2 + salt);
    rows.resize(size_t(o.batch_size));
    for (auto& v : rows) v = r.below(n_rows);
    return rows;
  }

  // ------------------------------------------------------------ public steps
  int start(int niterations) {
    const int np = o.populations;
    pops.assign(size_t(np), {});
    rngs.assign(size_t(np), SrRng());
    births.assign(size_t(np), 0);
    refs.assign(size_t(np), 0);
    best_seen.assign(size_t(np), Hof<T>());
    for (auto& h : best_seen) h.reset(o.maxsize);
    best_sub.assign(size_t(np), {});
    owned.clear();
    for (int i = 0; i < np; ++i) {
      rngs[size_t(i)].seed(seed, uint64_t(i));
      if (owns(i)) owned.push_back(i);
    }
    freq.assign(size_t(o.maxsize), 1.0);
    hof.reset(o.maxsize);
    total_cycles = int64_t(niterations) * np;
    if (total_cycles < 1) total_cycles = 1;
    cycles_remaining = total_cycles;
    iteration = 0;
    snap.assign(size_t(np), normalized());
    head_maxsize = get_cur_maxsize();
    cur_maxsize.assign(size_t(np), head_maxsize);
    make_tournament_weights();
    // update_baseline_loss!: the constant init_value(T) = 0 tree
    {
      SrTree<T> zero(1);
      zero[0].constant = 1;
      std::vector<T> l, c;
      const std::vector<const SrTree<T>*> one{&zero};
      int rc = score_trees(lane0(), one, {}, &l, &c);
      if (rc) return rc;
      if (std::isfinite(double(l[0]))) {
        baseline = l[0];
        use_baseline = true;
      } else {
        baseline = T(1);
        use_baseline = false;
      }
    }
    // Population(dataset; population_size, nlength = 3): gen_random_tree(3) per member, one launch
    std::vector<SrTree<T>> init;
    std::vector<int> who;
    for (int i : owned)
      for (int k = 0; k < o.population_size; ++k) {
        init.push_back(sr_gen_random_tree<T>(3, sp, rngs[size_t(i)]));
        who.push_back(i);
      }
    std::vector<const SrTree<T>*> ptr;
    for (auto& t : init) ptr.push_back(&t);
    std::vector<T> l, c;
    int rc = score_trees(lane0(), ptr, {}, &l, &c);
    if (rc) return rc;
    num_evals += double(init.size());
    for (size_t k = 0; k < init.size(); ++k) {
      const int i = who[k];
      Member<T> m;
      m.tree = std::move(init[k]);
      m.complexity = int(m.tree.size());
      m.loss = l[k];
      m.cost = c[k];
      m.birth = new_birth(i);
      m.ref = new_ref(i);
      pops[size_t(i)].push_back(std::move(m));
    }
    for (int i : owned) best_sub[size_t(i)] = best_sub_pop(pops[size_t(i)]);
    return SR_OK;
  }

  std::vector<double> normalized() const {
    double s = 0.0;
    for (double f : freq) s += f;
    std::vector<double> out(freq.size());
    for (size_t k = 0; k < freq.size(); ++k) out[k] = freq[k] / s;
    return out;
  }
  int get_cur_maxsize() const {
    const int64_t elapsed = total_cycles - cycles_remaining;
    const float frac = float(elapsed) / float(total_cycles);
    if (o.warmup_maxsize_by > 0.0f && frac <= o.warmup_maxsize_by)
      return 3 + int(floorf(float(o.maxsize - 3) * frac / o.warmup_maxsize_by));
    return o.maxsize;
  }
  std::vector<Member<T>> best_sub_pop(const std::vector<Member<T>>& pop) const {
    std::vector<size_t> idx(pop.size());
    for (size_t k = 0; k < idx.size(); ++k) idx[k] = k;
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return jl_isless(pop[a].cost, pop[b].cost); });
    std::vector<Member<T>> out;
    for (size_t k = 0; k < idx.size() && int(k) < o.topn; ++k) out.push_back(pop[idx[k]]);
    return out;
  }

  // s_r_cycle + optimize_and_simplify_population (+ finalize_costs) of a set of islands, scored on
  // one lane (every draw comes from the islands' own streams: the result does not depend on how the
  // owned islands are split over lanes)
  int iterate_islands(Lane L, const std::vector<int>& islands, const std::vector<std::vector<int64_t>>& rows,
                      const std::vector<std::vector<int64_t>>& orows) {
    const auto t_start = Clock::now();
    const int64_t calls0 = L.sc->calls;
    const int ncyc = o.ncycles_per_iteration;
    const int n_evol = (o.population_size + o.tournament_selection_n - 1) / o.tournament_selection_n;
    auto temp_of = [&](int c) {  // LinRange(1, 0, ncyc)
      return ncyc > 1 ? (o.annealing ? 1.0 - double(c) / double(ncyc - 1) : 1.0) : 1.0;
    };
    auto cycle_end = [&](const std::vector<int>& isl) {  // best-seen members per complexity
      for (int i : isl)
        for (const auto& m : pops[size_t(i)]) {
          const int s = m.complexity;
          auto& h = best_seen[size_t(i)];
          if (s > 0 && s <= o.maxsize && (!h.exists[size_t(s - 1)] || m.cost < h.m[size_t(s - 1)].cost)) {
            h.exists[size_t(s - 1)] = 1;
            h.m[size_t(s - 1)] = m;
          }
        }
    };
    for (int c = 0; c < ncyc; ++c) {
      for (int r = 0; r < n_evol; ++r) {
        int rc = round(L, islands, temp_of(c), rows);
        if (rc) return rc;
      }
      cycle_end(islands);
    }
    // optimize_and_simplify_population: the simplification of every member, then one batched
    // constant optimisation over every island's selected members
    std::vector<Member<T>*> sel;
    std::vector<int> sel_island;
    for (int i : islands) {
      auto& pop = pops[size_t(i)];
      std::vector<uint8_t> doopt(pop.size());
      for (size_t j = 0; j < pop.size(); ++j) doopt[j] = rngs[size_t(i)].uniform() < double(o.optimizer_probability);
      for (size_t j = 0; j < pop.size(); ++j) {
        if (o.should_simplify) {  // cost and loss kept; setting the tree resets the cached complexity
          sr_simplify_tree(pop[j].tree, sp);
          pop[j].complexity = int(pop[j].tree.size());
        }
        if (o.should_optimize_constants && doopt[j] && sr_count_constants(pop[j].tree) > 0) {
          sel.push_back(&pop[j]);
          sel_island.push_back(i);
        }
      }
    }
    const double cyc_ms = ms_since(t_start);
    const int64_t calls1 = L.sc->calls;
    std::vector<uint8_t> imp;
    int rc = optimize_members(L, sel, sel_island, orows, &imp);
    if (rc) return rc;
    if (profile_lanes)  // SR_AMD_SEARCH_PROFILE=1: per lane and iteration, to stderr
      std::fprintf(stderr, "[sr_search] iteration %d lane islands %zu: cycles %.2f ms (%lld calls), optimise %.2f ms (%lld calls, %zu members)\n",
                   iteration, islands.size(), cyc_ms, (long long)(calls1 - calls0), ms_since(t_start) - cyc_ms,
                   (long long)(L.sc->calls - calls1), sel.size());
    if (o.batching) {  // finalize_costs + best-seen re-scoring on the full data
      std::vector<Member<T>*> ms;
      for (int i : islands) {
        for (auto& m : pops[size_t(i)]) ms.push_back(&m);
        auto& h = best_seen[size_t(i)];
        for (size_t s = 0; s < h.m.size(); ++s)
          if (h.exists[s]) ms.push_back(&h.m[s]);
      }
      std::vector<const SrTree<T>*> tr;
      for (auto* m : ms) tr.push_back(&m->tree);
      std::vector<T> l, c;
      if ((rc = score_trees(L, tr, {}, &l, &c))) return rc;
      for (size_t k = 0; k < ms.size(); ++k) {
        ms[k]->loss = l[k];
        ms[k]->cost = cost_of(l[k], ms[k]->complexity);
      }
      *L.num_evals += double(ms.size());
    }
    for (int i : islands)
      for (auto& m : pops[size_t(i)]) {
        m.parent = m.ref;
        m.ref = new_ref(i);
      }
    return SR_OK;
  }

  int iterate() {
    std::vector<std::vector<int64_t>> rows(size_t(o.populations)), orows(size_t(o.populations));
    for (int i : owned) {
      rows[size_t(i)] = draw_batch(i, 0);
      orows[size_t(i)] = draw_batch(i, 1);
    }
    for (int i : owned) best_seen[size_t(i)].reset(o.maxsize);
    const size_t nl = std::min(owned.size(), extra.size() + 1);
    if (nl <= 1) {
      const int rc = iterate_islands(lane0(), owned, rows, orows);
      if (rc) return rc;
    } else {
      // contiguous shares of the owned islands, one host thread per extra lane
      std::vector<std::vector<int>> share(nl);
      for (size_t k = 0; k < owned.size(); ++k) share[k * nl / owned.size()].push_back(owned[k]);
      std::vector<int> rcs(nl, SR_OK);
      std::vector<std::string> msgs(nl);
      std::vector<std::thread> th;
      for (size_t q = 1; q < nl; ++q)
        th.emplace_back([&, q] {
          ExtraLane& x = *extra[q - 1];
          rcs[q] = iterate_islands(Lane{&x.sc, &x.flat, &x.num_evals, &x.host_ms}, share[q], rows, orows);
          if (rcs[q]) msgs[q] = sr_last_error();
        });
      rcs[0] = iterate_islands(lane0(), share[0], rows, orows);
      if (rcs[0]) msgs[0] = sr_last_error();
      for (auto& t : th) t.join();
      for (size_t q = 0; q < nl; ++q)
        if (rcs[q]) return sr_set_error(rcs[q], msgs[q]);
    }
    s_r_cycles += int64_t(owned.size());
    return SR_OK;
  }

  void hof_update(const Member<T>& m) {
    const int s = m.complexity;
    if (!(s > 0 && s <= o.maxsize)) return;
    if (!sr_check_constraints(m.tree, sp, o.maxsize)) return;
    if (!hof.exists[size_t(s - 1)] || m.cost < hof.m[size_t(s - 1)].cost) {
      hof.m[size_t(s - 1)] = m;
      hof.exists[size_t(s - 1)] = 1;
    }
  }
  std::vector<const Member<T>*> pareto() const {
    std::vector<const Member<T>*> out;
    for (size_t s = 0; s < hof.m.size(); ++s) {
      if (!hof.exists[s]) continue;
      bool better = true;
      for (size_t q = 0; q < s && better; ++q)
        if (hof.exists[q] && hof.m[s].loss >= hof.m[q].loss) better = false;  // (a NaN loss stays 'better')
      if (better) out.push_back(&hof.m[s]);
    }
    return out;
  }
  void migrate(const std::vector<const Member<T>*>& cands, int i, float frac) {
    auto& pop = pops[size_t(i)];
    SrRng& rng = rngs[size_t(i)];
    const int64_t n = int64_t(pop.size());
    const float lam = float(n) * frac;
    int64_t k = 0;
    if (lam != 0.0f) {  // poisson_sample in Float32
      const float L = sr_expf(-lam);
      float p = 1.0f;
      while (p > L) {
        ++k;
        p *= rng.uniform_f32();
      }
      --k;
    }
    k = std::min<int64_t>(k, int64_t(cands.size()));
    k = std::min<int64_t>(k, n);
    if (k <= 0) return;
    std::vector<int64_t> loc(static_cast<size_t>(k)), mig(static_cast<size_t>(k));
    for (auto& v : loc) v = rng.below(n);
    for (auto& v : mig) v = rng.below(int64_t(cands.size()));
    for (int64_t q = 0; q < k; ++q) {
      pop[size_t(loc[size_t(q)])] = *cands[size_t(mig[size_t(q)])];
      pop[size_t(loc[size_t(q)])].birth = new_birth(i);
    }
  }
  // the head's island-by-island bookkeeping (every rank, identically)
  int head() {
    for (int i = 0; i < o.populations; ++i) {
      // the island's next cycle gets the maxsize current when its output arrives
      cur_maxsize[size_t(i)] = head_maxsize;
      best_sub[size_t(i)] = best_sub_pop(pops[size_t(i)]);
      for (const auto& m : pops[size_t(i)])
        if (m.complexity > 0 && m.complexity <= int(freq.size())) freq[size_t(m.complexity - 1)] += 1.0;
      for (const auto& m : pops[size_t(i)]) hof_update(m);
      const auto& bs = best_seen[size_t(i)];
      for (size_t s = 0; s < bs.m.size(); ++s)
        if (bs.exists[s]) hof_update(bs.m[s]);
      const std::vector<const Member<T>*> dom = pareto();
      if (owns(i)) {
        if (o.migration) {
          std::vector<const Member<T>*> c;
          for (const auto& p : best_sub)
            for (const auto& m : p) c.push_back(&m);
          migrate(c, i, o.fraction_replaced);
        }
        if (o.hof_migration && !dom.empty()) migrate(dom, i, o.fraction_replaced_hof);
      }
      --cycles_remaining;
      snap[size_t(i)] = normalized();  // the copy the island's next s_r_cycle gets
      head_maxsize = get_cur_maxsize();
      move_window();
    }
    ++iteration;
    return SR_OK;
  }
  void move_window() {
    const double window = 100000.0, smallest = 1.0;
    double s = 0.0;
    for (double f : freq) s += f;
    if (s <= window) return;
    double diff = s - window;
    int loops = 0;
    while (diff > 0) {
      std::vector<size_t> idx;
      double mn = INFINITY;
      for (size_t k = 0; k < freq.size(); ++k)
        if (freq[k] > smallest) {
          idx.push_back(k);
          mn = std::min(mn, freq[k]);
        }
      if (idx.empty()) break;
      const double amount = std::min(diff / double(idx.size()), mn - smallest);
      for (size_t k : idx) freq[k] -= amount;
      const double total = amount * double(idx.size());
      diff -= total;
      ++loops;
      if (loops > 1000 || total < 1e-6) break;
    }
  }

  // ------------------------------------------------------------ exchange / export
  static void put_member(Writer& w, const Member<T>& m) {
    w.put(double(m.cost));
    w.put(double(m.loss));
    w.put(m.birth);
    w.put(m.ref);
    w.put(m.parent);
    w.put(int32_t(m.complexity));
    w.put(int32_t(m.tree.size()));
    for (const auto& n : m.tree) {
      w.put(n.degree);
      w.put(n.op);
      w.put(n.constant);
      w.put(n.feature);
      w.put(n.val);
    }
  }
  static bool get_member(Reader& r, Member<T>* m) {
    m->cost = T(r.get<double>());
    m->loss = T(r.get<double>());
    m->birth = r.get<int64_t>();
    m->ref = r.get<int64_t>();
    m->parent = r.get<int64_t>();
    m->complexity = r.get<int32_t>();
    const int32_t nn = r.get<int32_t>();
    if (!r.ok || nn < 1 || nn > (1 << 20)) return false;
    m->tree.resize(size_t(nn));
    for (auto& n : m->tree) {
      n.degree = r.get<uint8_t>();
      n.op = r.get<uint8_t>();
      n.constant = r.get<uint8_t>();
      n.feature = r.get<uint16_t>();
      n.val = r.get<T>();
    }
    return r.ok;
  }
  std::vector<uint8_t> export_owned() const {
    Writer w;
    w.put(int32_t(owned.size()));
    for (int i : owned) {
      w.put(int32_t(i));
      w.put(int32_t(pops[size_t(i)].size()));
      for (const auto& m : pops[size_t(i)]) put_member(w, m);
      const auto& h = best_seen[size_t(i)];
      w.put(int32_t(h.m.size()));
      for (size_t s = 0; s < h.m.size(); ++s) {
        w.put(h.exists[s]);
        if (h.exists[s]) put_member(w, h.m[s]);
      }
    }
    return w.buf;
  }
  int import_islands(const uint8_t* p, int64_t n) {
    Reader r{p, p + n};
    const int32_t k = r.get<int32_t>();
    for (int32_t q = 0; q < k && r.ok; ++q) {
      const int32_t i = r.get<int32_t>();
      if (i < 0 || i >= o.populations) return sr_set_error(SR_ERR_INVALID_ARG, "island index out of range");
      const int32_t nm = r.get<int32_t>();
      std::vector<Member<T>> pop(static_cast<size_t>(std::max(nm, 0)));
      for (auto& m : pop)
        if (!get_member(r, &m)) return sr_set_error(SR_ERR_INVALID_ARG, "truncated island buffer");
      Hof<T> h;
      const int32_t ns = r.get<int32_t>();
      h.reset(ns);
      for (int32_t s = 0; s < ns && r.ok; ++s) {
        h.exists[size_t(s)] = r.get<uint8_t>();
        if (h.exists[size_t(s)] && !get_member(r, &h.m[size_t(s)]))
          return sr_set_error(SR_ERR_INVALID_ARG, "truncated island buffer");
      }
      if (!r.ok) return sr_set_error(SR_ERR_INVALID_ARG, "truncated island buffer");
      if (owns(i)) continue;  // this rank's own islands are authoritative here
      pops[size_t(i)] = std::move(pop);
      best_seen[size_t(i)] = std::move(h);
    }
    return r.ok ? SR_OK : sr_set_error(SR_ERR_INVALID_ARG, "truncated island buffer");
  }
  std::vector<const Member<T>*> members_of(int which) const {
    std::vector<const Member<T>*> out;
    if (which >= 0) {
      for (const auto& m : pops[size_t(which)]) out.push_back(&m);
    } else if (which == SR_SEARCH_HALL_OF_FAME) {
      for (size_t s = 0; s < hof.m.size(); ++s)
        if (hof.exists[s]) out.push_back(&hof.m[s]);
    } else if (which == SR_SEARCH_PARETO) {
      out = pareto();
    }
    return out;
  }
};

template <typename T>
Engine<T>* as_engine(sr_search* s) {
  return static_cast<Engine<T>*>(reinterpret_cast<sr_search_base*>(s));
}

template <typename R, typename F>
int dispatch(sr_search* s, F f) {
  if (!s) return sr_set_error(SR_ERR_INVALID_ARG, "NULL search handle");
  auto* b = reinterpret_cast<sr_search_base*>(s);
  if (b->dtype == SR_DTYPE_F32) return f(as_engine<float>(s));
  return f(as_engine<double>(s));
}

// The batched constant optimiser over `trees` with a ready scorer (device or CPU callbacks): the
// reference's optimize_constants per tree (src/ConstantOptimization.jl:29-116), all trees in lock-step.
template <typename T>
int optimize_common(Scorer<T>& sc, const sr_tree_batch* trees, const int64_t* row_idx, int64_t n_idx, int iterations,
                    int64_t f_calls_limit, int nrestarts, uint64_t seed, void* out_consts, void* out_loss,
                    uint8_t* out_improved, int64_t* out_f_calls) {
  if (iterations < 0 || nrestarts < 0 || f_calls_limit < 0)
    return sr_set_error(SR_ERR_INVALID_ARG, "negative iterations / f_calls_limit / restarts");
  const int64_t nt = trees->n_trees;
  if (nt < 0) return sr_set_error(SR_ERR_INVALID_ARG, "negative tree count");
  if (nt == 0) return SR_OK;
  if (!trees->offsets || !trees->degree || !trees->op || !trees->feature || !trees->constant || !trees->val ||
      !out_consts || !out_loss || !out_improved || !out_f_calls)
    return sr_set_error(SR_ERR_INVALID_ARG, "NULL arrays");
  std::vector<SrTree<T>> tv(static_cast<size_t>(nt));
  std::vector<std::vector<double>> x0(static_cast<size_t>(nt));
  const T* vals = static_cast<const T*>(trees->val);
  for (int64_t t = 0; t < nt; ++t)
    for (int64_t i = trees->offsets[t]; i < trees->offsets[t + 1]; ++i) {
      SrNode<T> nd;
      nd.degree = trees->degree[i];
      nd.op = trees->op[i];
      nd.feature = trees->feature[i];
      nd.constant = trees->constant[i];
      nd.val = vals[i];
      tv[size_t(t)].push_back(nd);
      if (nd.degree == 0 && nd.constant) x0[size_t(t)].push_back(double(nd.val));
    }
  SrRng rng;
  rng.seed(seed, 0x6f7074696d697a65ull);
  std::vector<std::vector<std::vector<double>>> restarts(static_cast<size_t>(nrestarts),
                                                         std::vector<std::vector<double>>(static_cast<size_t>(nt)));
  for (int64_t t = 0; t < nt; ++t)
    for (int r = 0; r < nrestarts; ++r) draw_restart<T>(rng, x0[size_t(t)], &restarts[size_t(r)][size_t(t)]);
  std::vector<const SrTree<T>*> ptr;
  for (auto& t : tv) ptr.push_back(&t);
  Flat flat;
  const std::vector<int64_t> view(row_idx && n_idx > 0 ? row_idx : nullptr, row_idx && n_idx > 0 ? row_idx + n_idx : nullptr);
  typename Scorer<T>::TreeRows rows;  // (one view for every tree, or the full dataset)
  if (!view.empty()) rows.assign(size_t(nt), &view);
  std::vector<std::vector<double>> bx;
  std::vector<uint8_t> imp;
  std::vector<T> loss;
  std::vector<int64_t> f_calls;
  const int e = optimize_trees<T>(sc, flat, ptr, x0, restarts, iterations, rows, &bx, &imp, &loss, &f_calls, f_calls_limit);
  if (e) return e;
  size_t at = 0;
  for (int64_t t = 0; t < nt; ++t) {
    for (size_t q = 0; q < x0[size_t(t)].size(); ++q)
      static_cast<T*>(out_consts)[at++] = imp[size_t(t)] ? T(bx[size_t(t)][q]) : T(x0[size_t(t)][q]);
    static_cast<T*>(out_loss)[t] = loss[size_t(t)];
    out_improved[t] = imp[size_t(t)];
    out_f_calls[t] = f_calls[size_t(t)];
  }
  return SR_OK;
}

}  // namespace

extern "C" {

int sr_search_create(int dtype, int64_t nfeatures, int64_t n_rows, int n_unary, const char* const* unary_names,
                     int n_binary, const char* const* binary_names, const sr_search_options* opts, uint64_t seed,
                     int rank, int world_size, sr_search** out) {
  if (!opts || !out) return sr_set_error(SR_ERR_INVALID_ARG, "NULL options or output handle");
  if (dtype != SR_DTYPE_F32 && dtype != SR_DTYPE_F64) return sr_set_error(SR_ERR_INVALID_ARG, "unknown dtype");
  if (nfeatures < 1 || nfeatures > 65535 || n_rows < 1) return sr_set_error(SR_ERR_INVALID_ARG, "bad dataset shape");
  if (world_size < 1 || rank < 0 || rank >= world_size) return sr_set_error(SR_ERR_INVALID_ARG, "bad rank / world size");
  const sr_search_options& o = *opts;
  // (tournament_selection_n > population_size samples the whole island: min(n, pop) as Population.jl)
  if (o.populations < 1 || o.population_size < 2 || o.tournament_selection_n < 1 || o.maxsize < 1 || o.ncycles_per_iteration < 1 ||
      o.optimizer_nrestarts < 0 || o.optimizer_iterations < 0 || o.optimizer_f_calls_limit < 0 || (o.batching && o.batch_size < 1))
    return sr_set_error(SR_ERR_INVALID_ARG, "invalid search options");
  if (n_unary < 0 || n_binary < 0 || n_unary + n_binary == 0 || n_unary > 255 || n_binary > 255)
    return sr_set_error(SR_ERR_INVALID_ARG, "bad operator counts");
  SrTreeSpec sp;
  sp.nfeatures = int(nfeatures);
  sp.nops[0] = n_unary;
  sp.nops[1] = n_binary;
  for (int k = 0; k < n_unary; ++k) {
    const uint32_t id = unary_names && unary_names[k] ? sr_unary_id(unary_names[k]) : 0;
    if (!id) return sr_set_error(SR_ERR_UNSUPPORTED_OP, "unsupported unary operator");
    sp.unary_ids.push_back(id);
  }
  for (int k = 0; k < n_binary; ++k) {
    const uint32_t id = binary_names && binary_names[k] ? sr_binary_id(binary_names[k]) : 0;
    if (!id) return sr_set_error(SR_ERR_UNSUPPORTED_OP, "unsupported binary operator");
    sp.binary_ids.push_back(id);
  }
  sp.maxdepth = o.maxdepth > 0 ? o.maxdepth : o.maxsize;
  sp.perturbation_factor = double(o.perturbation_factor);
  sp.probability_negate_constant = double(o.probability_negate_constant);
  auto make = [&](auto* e) {
    e->dtype = dtype;
    e->o = o;
    e->sp = sp;
    e->n_rows = n_rows;
    e->seed = seed;
    e->rank = rank;
    e->world = world_size;
    *out = reinterpret_cast<sr_search*>(static_cast<sr_search_base*>(e));
    return SR_OK;
  };
  if (dtype == SR_DTYPE_F32) return make(new Engine<float>());
  return make(new Engine<double>());
}

int sr_gen_random_population(int dtype, int64_t n_trees, int64_t nfeatures, int n_unary, int n_binary, int max_size,
                              uint64_t seed, int64_t capacity, int64_t* offsets, uint8_t* degree, uint8_t* op,
                              uint16_t* feature, uint8_t* constant, void* val) {
  if (dtype != SR_DTYPE_F32 && dtype != SR_DTYPE_F64) return sr_set_error(SR_ERR_INVALID_ARG, "unknown dtype");
  if (n_trees < 0 || nfeatures < 1 || nfeatures > 65535 || max_size < 1 || n_unary < 0 || n_binary < 0 ||
      n_unary > 255 || n_binary > 255 || !offsets || !degree || !op || !feature || !constant || !val)
    return sr_set_error(SR_ERR_INVALID_ARG, "bad arguments");
  SrTreeSpec sp;
  sp.nfeatures = int(nfeatures);
  sp.nops[0] = n_unary;
  sp.nops[1] = n_binary;
  SrRng rng;
  rng.seed(seed, 0x9e11ull);
  auto go = [&](auto tag) -> int {
    using T = decltype(tag);
    T* v = static_cast<T*>(val);
    int64_t at = 0;
    offsets[0] = 0;
    for (int64_t k = 0; k < n_trees; ++k) {
      const int size = int(1 + rng.below(max_size));
      const SrTree<T> t = sr_gen_random_tree_fixed_size<T>(size, sp, rng);
      if (at + int64_t(t.size()) > capacity) return sr_set_error(SR_ERR_INVALID_ARG, "node capacity too small");
      for (const SrNode<T>& nd : t) {
        degree[at] = nd.degree;
        op[at] = nd.op;
        feature[at] = nd.feature;
        constant[at] = nd.constant;
        v[at] = nd.val;
        ++at;
      }
      offsets[k + 1] = at;
    }
    return SR_OK;
  };
  return dtype == SR_DTYPE_F32 ? go(0.0f) : go(0.0);
}

int sr_search_free(sr_search* s) {
  if (s) delete reinterpret_cast<sr_search_base*>(s);
  return SR_OK;
}

int sr_search_use_device(sr_search* s, sr_ctx* ctx, const sr_dataset* ds, int opset_id, int loss_code) {
  return dispatch<int>(s, [&](auto* e) {
    if (!ctx || !ds) return sr_set_error(SR_ERR_INVALID_ARG, "NULL context or dataset");
    int dt = 0;
    int64_t nf = 0, n = 0;
    int rc = sr_dataset_info(ds, &dt, &nf, &n);
    if (rc) return rc;
    if (dt != e->dtype || nf != e->sp.nfeatures || n != e->n_rows)
      return sr_set_error(SR_ERR_INVALID_ARG, "dataset does not match the search (dtype, features, rows)");
    e->sc.ctx = ctx;
    e->sc.ds = ds;
    e->sc.opset_id = opset_id;
    e->sc.loss_code = loss_code;
    e->sc.loss_cb = nullptr;
    e->sc.grad_cb = nullptr;
    return SR_OK;
  });
}

int sr_search_add_device(sr_search* s, sr_ctx* ctx, const sr_dataset* ds, int opset_id, int loss_code) {
  return dispatch<int>(s, [&](auto* e) {
    if (!ctx || !ds) return sr_set_error(SR_ERR_INVALID_ARG, "NULL context or dataset");
    if (!e->sc.ctx) return sr_set_error(SR_ERR_INVALID_ARG, "sr_search_use_device first (lane 0)");
    if (!e->pops.empty()) return sr_set_error(SR_ERR_INVALID_ARG, "lanes must be added before sr_search_start");
    int dt = 0;
    int64_t nf = 0, n = 0;
    int rc = sr_dataset_info(ds, &dt, &nf, &n);
    if (rc) return rc;
    if (dt != e->dtype || nf != e->sp.nfeatures || n != e->n_rows)
      return sr_set_error(SR_ERR_INVALID_ARG, "dataset does not match the search (dtype, features, rows)");
    using E = std::remove_reference_t<decltype(*e)>;
    auto x = std::make_unique<typename E::ExtraLane>();
    x->sc.ctx = ctx;
    x->sc.ds = ds;
    x->sc.opset_id = opset_id;
    x->sc.loss_code = loss_code;
    e->extra.push_back(std::move(x));
    return SR_OK;
  });
}

int sr_search_use_callbacks(sr_search* s, sr_loss_fn loss, sr_grad_fn grad, void* user) {
  return dispatch<int>(s, [&](auto* e) {
    if (!loss) return sr_set_error(SR_ERR_INVALID_ARG, "NULL loss callback");
    e->sc.loss_cb = loss;
    e->sc.grad_cb = grad;
    e->sc.cb_user = user;
    e->sc.ctx = nullptr;
    e->sc.ds = nullptr;
    e->extra.clear();
    return SR_OK;
  });
}

int sr_search_start(sr_search* s, int niterations) {
  return dispatch<int>(s, [&](auto* e) {
    if (!e->sc.ready()) return sr_set_error(SR_ERR_INVALID_ARG, "no scorer: call sr_search_use_device first");
    if (niterations < 0) return sr_set_error(SR_ERR_INVALID_ARG, "negative iteration count");
    return e->start(niterations);
  });
}

int sr_search_iterate(sr_search* s) {
  return dispatch<int>(s, [&](auto* e) {
    if (e->pops.empty()) return sr_set_error(SR_ERR_INVALID_ARG, "search not started");
    return e->iterate();
  });
}

int sr_search_head(sr_search* s) {
  return dispatch<int>(s, [&](auto* e) {
    if (e->pops.empty()) return sr_set_error(SR_ERR_INVALID_ARG, "search not started");
    for (int i = 0; i < e->o.populations; ++i)
      if (e->pops[size_t(i)].empty()) return sr_set_error(SR_ERR_INVALID_ARG, "island missing: import every rank's islands first");
    return e->head();
  });
}

int sr_search_export(sr_search* s, void* buf, int64_t capacity, int64_t* size) {
  return dispatch<int>(s, [&](auto* e) {
    if (!size) return sr_set_error(SR_ERR_INVALID_ARG, "NULL size");
    const std::vector<uint8_t> b = e->export_owned();
    *size = int64_t(b.size());
    if (buf && capacity >= int64_t(b.size())) memcpy(buf, b.data(), b.size());
    return SR_OK;
  });
}

int sr_search_import(sr_search* s, const void* buf, int64_t size) {
  return dispatch<int>(s, [&](auto* e) {
    if (!buf || size < 4) return sr_set_error(SR_ERR_INVALID_ARG, "empty island buffer");
    return e->import_islands(static_cast<const uint8_t*>(buf), size);
  });
}

int sr_search_get_info(sr_search* s, sr_search_info* out) {
  return dispatch<int>(s, [&](auto* e) {
    if (!out) return sr_set_error(SR_ERR_INVALID_ARG, "NULL output");
    out->iterations = e->iteration;
    out->s_r_cycles = e->s_r_cycles;
    out->num_evals = e->total_num_evals();
    out->device_calls = e->sc.calls;
    out->device_ms = e->sc.ms;
    out->kernel_ms = e->sc.kernel_ms;
    out->host_ms = e->host_ms;
    for (const auto& x : e->extra) {  // (summed over lanes: lanes run concurrently)
      out->device_calls += x->sc.calls;
      out->device_ms += x->sc.ms;
      out->kernel_ms += x->sc.kernel_ms;
      out->host_ms += x->host_ms;
    }
    out->baseline_loss = double(e->baseline);
    out->use_baseline = e->use_baseline ? 1 : 0;
    return SR_OK;
  });
}

int sr_search_member_count(sr_search* s, int which, int64_t* n_members, int64_t* n_nodes) {
  return dispatch<int>(s, [&](auto* e) {
    if (!n_members || !n_nodes) return sr_set_error(SR_ERR_INVALID_ARG, "NULL output");
    if (which >= e->o.populations || which < SR_SEARCH_PARETO || (which >= 0 && e->pops.empty()))
      return sr_set_error(SR_ERR_INVALID_ARG, "bad member set");
    const auto ms = e->members_of(which);
    *n_members = int64_t(ms.size());
    int64_t nn = 0;
    for (auto* m : ms) nn += int64_t(m->tree.size());
    *n_nodes = nn;
    return SR_OK;
  });
}

int sr_search_members(sr_search* s, int which, int64_t* offsets, uint8_t* degree, uint8_t* op, uint16_t* feature,
                      uint8_t* constant, void* val, void* cost, void* loss, int64_t* birth, int64_t* ref,
                      int64_t* parent, int32_t* complexity) {
  return dispatch<int>(s, [&](auto* e) {
    using T = std::remove_reference_t<decltype(e->baseline)>;
    if (which >= e->o.populations || which < SR_SEARCH_PARETO || (which >= 0 && e->pops.empty()))
      return sr_set_error(SR_ERR_INVALID_ARG, "bad member set");
    if (!offsets || !degree || !op || !feature || !constant || !val || !cost || !loss || !birth || !ref || !parent ||
        !complexity)
      return sr_set_error(SR_ERR_INVALID_ARG, "NULL output array");
    const auto ms = e->members_of(which);
    int64_t at = 0;
    offsets[0] = 0;
    for (size_t k = 0; k < ms.size(); ++k) {
      const auto* m = ms[k];
      for (const auto& n : m->tree) {
        degree[at] = n.degree;
        op[at] = n.op;
        feature[at] = n.feature;
        constant[at] = n.constant;
        static_cast<T*>(val)[at] = n.val;
        ++at;
      }
      offsets[k + 1] = at;
      static_cast<T*>(cost)[k] = m->cost;
      static_cast<T*>(loss)[k] = m->loss;
      birth[k] = m->birth;
      ref[k] = m->ref;
      parent[k] = m->parent;
      complexity[k] = m->complexity;
    }
    return SR_OK;
  });
}

int sr_optimize_constants_batch(sr_ctx* ctx, const sr_dataset* ds, int opset_id, const sr_tree_batch* trees,
                                const int64_t* row_idx, int64_t n_idx, int loss_kind, int iterations,
                                int64_t f_calls_limit, int nrestarts, uint64_t seed, void* out_consts, void* out_loss,
                                uint8_t* out_improved, int64_t* out_f_calls) {
  if (!ctx || !ds || !trees) return sr_set_error(SR_ERR_INVALID_ARG, "NULL context, dataset or trees");
  int dt = 0;
  int64_t nf = 0, n = 0;
  int rc = sr_dataset_info(ds, &dt, &nf, &n);
  if (rc) return rc;
  auto run = [&](auto zero) -> int {
    using T = decltype(zero);
    Scorer<T> sc;
    sc.ctx = ctx;
    sc.ds = ds;
    sc.opset_id = opset_id;
    sc.loss_code = loss_kind;
    return optimize_common<T>(sc, trees, row_idx, n_idx, iterations, f_calls_limit, nrestarts, seed, out_consts,
                              out_loss, out_improved, out_f_calls);
  };
  return dt == SR_DTYPE_F32 ? run(0.0f) : run(0.0);
}

int sr_optimize_constants_callbacks(int dtype, const sr_tree_batch* trees, const int64_t* row_idx, int64_t n_idx,
                                    int iterations, int64_t f_calls_limit, int nrestarts, uint64_t seed, sr_loss_fn loss,
                                    sr_grad_fn grad, void* user, void* out_consts, void* out_loss,
                                    uint8_t* out_improved, int64_t* out_f_calls) {
  if (!trees || !loss || !grad) return sr_set_error(SR_ERR_INVALID_ARG, "NULL trees or scorer callbacks");
  if (dtype != SR_DTYPE_F32 && dtype != SR_DTYPE_F64) return sr_set_error(SR_ERR_INVALID_ARG, "unknown dtype");
  auto run = [&](auto zero) -> int {
    using T = decltype(zero);
    Scorer<T> sc;
    sc.loss_cb = loss;
    sc.grad_cb = grad;
    sc.cb_user = user;
    return optimize_common<T>(sc, trees, row_idx, n_idx, iterations, f_calls_limit, nrestarts, seed, out_consts,
                              out_loss, out_improved, out_f_calls);
  };
  return dtype == SR_DTYPE_F32 ? run(0.0f) : run(0.0);
}

}  // extern "C"
