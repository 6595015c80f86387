// sr_search_tree.h — expression trees of the native search and the reference's mutation functions.
//
// A tree is its pre-order node array (DynamicExpressions Node{T,2} fields, parent before children,
// left before right — the sr_tree_batch layout, so a population flattens into a device batch by
// concatenation).  Subtrees are contiguous ranges; mutations splice ranges.  Every function restates
// the reference function it names, drawing its random numbers in the reference's order (sr_rng.h):
//   src/MutationFunctions.jl   swap_operands :83-96, mutate_operator :107-117, mutate_constant /
//     mutate_factor :128-158, mutate_feature :173-183, append_random_op :199-222,
//     insert_random_op :238-265, prepend_random_op :281-309, make_random_leaf :311-333,
//     delete_random_op! :342-357, randomize_tree :372-381, gen_random_tree :384-397,
//     _arity_picker / gen_random_tree_fixed_size :423-471, crossover_trees :489-517,
//     randomly_rotate_tree! :578-611 (form/break_connection are 0-weight for plain Node trees)
//   src/CheckConstraints.jl:75-92 (size and depth; no per-operator constraints)
//   DynamicExpressions simplify_tree! / combine_operators (not vendored under /root/reference:
//     restated from DE's published algorithm, parity unpinned — see DESIGN.md §9).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "sr_ops.h"
#include "sr_rng.h"

template <typename T>
struct SrNode {
  uint8_t degree = 0, op = 0, constant = 0;
  uint16_t feature = 0;
  T val = T(0);
};
template <typename T>
using SrTree = std::vector<SrNode<T>>;

// What the mutation functions read from Options.
struct SrTreeSpec {
  int nfeatures = 1;
  int nops[2] = {0, 0};             // options.nops: unary, binary
  std::vector<uint32_t> unary_ids;  // SrUnaryOp per op index (simplification folds constants)
  std::vector<uint32_t> binary_ids;
  int maxdepth = 30;
  double perturbation_factor = 0.129, probability_negate_constant = 0.00743;
};

// end (exclusive) of the subtree rooted at i
template <typename T>
inline size_t sr_subtree_end(const SrTree<T>& t, size_t i) {
  int64_t need = 1;
  size_t j = i;
  while (need > 0) {
    need += int64_t(t[j].degree) - 1;
    ++j;
  }
  return j;
}

template <typename T>
inline int sr_count_depth(const SrTree<T>& t) {
  // pre-order with a stack of remaining-children counts
  int depth = 0;
  std::vector<int> open;  // children still to visit at each level
  open.reserve(32);
  for (const auto& n : t) {
    const int d = int(open.size()) + 1;
    depth = std::max(depth, d);
    if (!open.empty()) --open.back();
    if (n.degree > 0)
      open.push_back(n.degree);
    else
      while (!open.empty() && open.back() == 0) open.pop_back();
  }
  return depth;
}

template <typename T>
inline int sr_count_constants(const SrTree<T>& t) {
  int c = 0;
  for (const auto& n : t) c += (n.degree == 0 && n.constant) ? 1 : 0;
  return c;
}

// check_constraints with the complexity = node count (default complexities)
template <typename T>
inline bool sr_check_constraints(const SrTree<T>& t, const SrTreeSpec& sp, int maxsize) {
  if (int(t.size()) > maxsize) return false;
  return sr_count_depth(t) <= sp.maxdepth;
}

// uniform choice among the pre-order positions satisfying `keep` (DE NodeSampler); -1 if none
template <typename T, typename F>
inline int64_t sr_sample_node(const SrTree<T>& t, SrRng& rng, F keep) {
  int64_t n = 0;
  for (size_t i = 0; i < t.size(); ++i) n += keep(t[i]) ? 1 : 0;
  if (n == 0) return -1;
  int64_t k = rng.below(n);
  for (size_t i = 0; i < t.size(); ++i)
    if (keep(t[i]) && k-- == 0) return int64_t(i);
  return -1;
}

// replace the subtree at i by `sub`
template <typename T>
inline void sr_splice(SrTree<T>& t, size_t i, const SrNode<T>* sub, size_t n) {
  const size_t e = sr_subtree_end(t, i);
  SrTree<T> out;
  out.reserve(t.size() - (e - i) + n);
  out.insert(out.end(), t.begin(), t.begin() + i);
  out.insert(out.end(), sub, sub + n);
  out.insert(out.end(), t.begin() + e, t.end());
  t.swap(out);
}

template <typename T>
inline SrNode<T> sr_make_random_leaf(const SrTreeSpec& sp, SrRng& rng) {
  SrNode<T> n;
  if (rng.coin()) {
    n.constant = 1;
    n.val = T(rng.normal());  // sample_value = randn(T)
  } else {
    n.feature = uint16_t(1 + rng.below(sp.nfeatures));
  }
  return n;
}

// arity chosen by scaled_rand = rand() * (n_unary + n_binary) as append/insert/prepend do
inline int sr_scaled_arity(const SrTreeSpec& sp, SrRng& rng) {
  const double c1 = double(sp.nops[0]), c2 = c1 + double(sp.nops[1]);
  const double x = rng.uniform() * c2;
  return (x > 0.0 && x <= c1) ? 1 : 2;
}

// ---------------------------------------------------------------- mutations
template <typename T>
inline T sr_mutate_factor(const SrTreeSpec& sp, double temperature, SrRng& rng) {
  const double max_change = sp.perturbation_factor * temperature + 1.0 + 0.1;
  T factor = T(pow(max_change, double(rng.uniform_t<T>())));
  const bool bigger = rng.coin();
  factor = bigger ? factor : T(1) / factor;
  if (rng.uniform() > sp.probability_negate_constant) factor = factor * T(-1);
  return factor;
}

template <typename T>
inline void sr_mutate_constant(SrTree<T>& t, const SrTreeSpec& sp, double temperature, SrRng& rng) {
  const int64_t i = sr_sample_node(t, rng, [](const SrNode<T>& n) { return n.degree == 0 && n.constant; });
  if (i < 0) return;
  t[size_t(i)].val = t[size_t(i)].val * sr_mutate_factor<T>(sp, temperature, rng);
}

template <typename T>
inline void sr_mutate_operator(SrTree<T>& t, const SrTreeSpec& sp, SrRng& rng) {
  const int64_t i = sr_sample_node(t, rng, [](const SrNode<T>& n) { return n.degree != 0; });
  if (i < 0) return;
  auto& n = t[size_t(i)];
  n.op = uint8_t(1 + rng.below(sp.nops[n.degree - 1]));
}

template <typename T>
inline void sr_mutate_feature(SrTree<T>& t, const SrTreeSpec& sp, SrRng& rng) {
  if (sp.nfeatures <= 1) return;
  const int64_t i = sr_sample_node(t, rng, [](const SrNode<T>& n) { return n.degree == 0 && !n.constant; });
  if (i < 0) return;
  auto& n = t[size_t(i)];
  const int64_t k = rng.below(sp.nfeatures - 1);  // among 1:nfeatures without the current one
  n.feature = uint16_t(k + 1 < n.feature ? k + 1 : k + 2);
}

template <typename T>
inline void sr_swap_operands(SrTree<T>& t, SrRng& rng) {
  const int64_t i = sr_sample_node(t, rng, [](const SrNode<T>& n) { return n.degree > 1; });
  if (i < 0) return;
  (void)rng.below(2);  // i1 = rand(1:2); i2 = the other child
  const size_t a = size_t(i) + 1, b = sr_subtree_end(t, a), e = sr_subtree_end(t, b);
  std::rotate(t.begin() + a, t.begin() + b, t.begin() + e);
}

// new operator node of `arity`: op first, then its leaves (DE constructor keyword order)
template <typename T>
inline void sr_make_node(int arity, const SrTreeSpec& sp, SrRng& rng, SrTree<T>* out) {
  SrNode<T> h;
  h.degree = uint8_t(arity);
  h.op = uint8_t(1 + rng.below(sp.nops[arity - 1]));
  out->push_back(h);
  for (int j = 0; j < arity; ++j) out->push_back(sr_make_random_leaf<T>(sp, rng));
}

template <typename T>
inline void sr_append_random_op(SrTree<T>& t, const SrTreeSpec& sp, SrRng& rng) {
  const int64_t leaf = sr_sample_node(t, rng, [](const SrNode<T>& n) { return n.degree == 0; });
  const int arity = sr_scaled_arity(sp, rng);
  SrTree<T> nn;
  sr_make_node<T>(arity, sp, rng, &nn);
  sr_splice(t, size_t(leaf), nn.data(), nn.size());
}

// insert_random_op / prepend_random_op: the carried subtree's slot, the other leaves, then the op
template <typename T>
inline void sr_wrap_node(int arity, const SrNode<T>* carry, size_t carry_n, const SrTreeSpec& sp, SrRng& rng,
                         SrTree<T>* out) {
  const int64_t slot = rng.below(arity);
  SrNode<T> leaves[2];
  for (int j = 0; j < arity; ++j)
    if (j != slot) leaves[j] = sr_make_random_leaf<T>(sp, rng);
  SrNode<T> h;
  h.degree = uint8_t(arity);
  h.op = uint8_t(1 + rng.below(sp.nops[arity - 1]));
  out->push_back(h);
  for (int j = 0; j < arity; ++j) {
    if (j == slot)
      out->insert(out->end(), carry, carry + carry_n);
    else
      out->push_back(leaves[j]);
  }
}

template <typename T>
inline void sr_insert_random_op(SrTree<T>& t, const SrTreeSpec& sp, SrRng& rng) {
  const int64_t i = rng.below(int64_t(t.size()));
  const int arity = sr_scaled_arity(sp, rng);
  const size_t e = sr_subtree_end(t, size_t(i));
  SrTree<T> nn;
  sr_wrap_node<T>(arity, t.data() + i, e - size_t(i), sp, rng, &nn);
  sr_splice(t, size_t(i), nn.data(), nn.size());
}

template <typename T>
inline void sr_prepend_random_op(SrTree<T>& t, const SrTreeSpec& sp, SrRng& rng) {
  const int arity = sr_scaled_arity(sp, rng);
  SrTree<T> nn;
  sr_wrap_node<T>(arity, t.data(), t.size(), sp, rng, &nn);
  t.swap(nn);
}

template <typename T>
inline void sr_delete_random_op(SrTree<T>& t, SrRng& rng) {
  if (t[0].degree == 0) return;
  const int64_t i = sr_sample_node(t, rng, [](const SrNode<T>& n) { return n.degree > 0; });
  const int64_t c = rng.below(t[size_t(i)].degree);
  size_t a = size_t(i) + 1;
  if (c == 1) a = sr_subtree_end(t, a);
  const size_t e = sr_subtree_end(t, a);
  SrTree<T> carry(t.begin() + a, t.begin() + e);
  sr_splice(t, size_t(i), carry.data(), carry.size());
}

template <typename T>
inline SrTree<T> sr_gen_random_tree_fixed_size(int node_count, const SrTreeSpec& sp, SrRng& rng) {
  SrTree<T> t{sr_make_random_leaf<T>(sp, rng)};
  int cur = 1;
  while (true) {
    const int remaining = node_count - cur;
    if (remaining == 0) break;
    // _arity_picker
    const int limit = std::min(2, remaining);
    int total = 0;
    for (int k = 0; k < limit; ++k) total += sp.nops[k];
    if (total == 0) break;
    const int64_t thresh = 1 + rng.below(total);
    int arity = limit, acc = 0;
    for (int k = 1; k < limit; ++k) {
      acc += sp.nops[k - 1];
      if (thresh <= acc) {
        arity = k;
        break;
      }
    }
    const int64_t leaf = sr_sample_node(t, rng, [](const SrNode<T>& n) { return n.degree == 0; });
    SrTree<T> nn;
    sr_make_node<T>(arity, sp, rng, &nn);
    sr_splice(t, size_t(leaf), nn.data(), nn.size());
    cur += arity;
  }
  return t;
}

// gen_random_tree(length): `length` append_random_op on the placeholder constant init_value(T) = 0
template <typename T>
inline SrTree<T> sr_gen_random_tree(int length, const SrTreeSpec& sp, SrRng& rng) {
  SrNode<T> z;
  z.constant = 1;
  SrTree<T> t{z};
  for (int i = 0; i < length; ++i) sr_append_random_op(t, sp, rng);
  return t;
}

// randomly_rotate_tree!
template <typename T>
inline void sr_rotate_tree(SrTree<T>& t, SrRng& rng) {
  const size_t n = t.size();
  std::vector<size_t> ends(n);
  for (size_t i = 0; i < n; ++i) ends[i] = sr_subtree_end(t, i);
  auto child = [&](size_t i, int c) { return c == 0 ? i + 1 : ends[i + 1]; };
  auto valid = [&](size_t i) {
    if (t[i].degree == 0) return false;
    for (int c = 0; c < t[i].degree; ++c)
      if (t[child(i, c)].degree > 0) return true;
    return false;
  };
  int64_t nvalid = 0;
  for (size_t i = 0; i < n; ++i) nvalid += valid(i) ? 1 : 0;
  if (nvalid == 0) return;
  const bool at_root = rng.uniform() < 1.0 / double(nvalid);
  size_t root = 0;
  if (!at_root) {
    int64_t cnt = 0;
    for (size_t i = 1; i < n; ++i) cnt += valid(i) ? 1 : 0;
    int64_t k = rng.below(cnt);
    for (size_t i = 1; i < n; ++i)
      if (valid(i) && k-- == 0) {
        root = i;
        break;
      }
  }
  int cand[2], nc = 0;
  for (int c = 0; c < t[root].degree; ++c)
    if (t[child(root, c)].degree > 0) cand[nc++] = c;
  const int pivot_c = cand[rng.below(nc)];
  const size_t pivot = child(root, pivot_c);
  const int gc_c = int(rng.below(t[pivot].degree));
  const size_t grand = child(pivot, gc_c);
  // root' = root with child pivot_c := grand; new subtree = pivot with child gc_c := root'
  SrTree<T> root2;
  root2.push_back(t[root]);
  for (int c = 0; c < t[root].degree; ++c) {
    const size_t a = c == pivot_c ? grand : child(root, c);
    root2.insert(root2.end(), t.begin() + a, t.begin() + ends[a]);
  }
  SrTree<T> sub;
  sub.push_back(t[pivot]);
  for (int c = 0; c < t[pivot].degree; ++c) {
    if (c == gc_c) {
      sub.insert(sub.end(), root2.begin(), root2.end());
    } else {
      const size_t a = child(pivot, c);
      sub.insert(sub.end(), t.begin() + a, t.begin() + ends[a]);
    }
  }
  sr_splice(t, root, sub.data(), sub.size());
}

// crossover_trees: a uniformly chosen subtree of each copy swapped (t1's node drawn first)
template <typename T>
inline void sr_crossover_trees(const SrTree<T>& a, const SrTree<T>& b, SrRng& rng, SrTree<T>* out1, SrTree<T>* out2) {
  const size_t i1 = size_t(rng.below(int64_t(a.size())));
  const size_t i2 = size_t(rng.below(int64_t(b.size())));
  const size_t e1 = sr_subtree_end(a, i1), e2 = sr_subtree_end(b, i2);
  *out1 = a;
  sr_splice(*out1, i1, b.data() + i2, e2 - i2);
  *out2 = b;
  sr_splice(*out2, i2, a.data() + i1, e1 - i1);
}

// ---------------------------------------------------------------- simplification
// simplify_tree! (fold every operator whose children are all finite constants, bottom-up, when the
// result is finite) then combine_operators (merge constants through + / * chains and - pairs).
// The arena form (child indices) makes DE's pointer rewrites direct.
template <typename T>
struct SrArena {
  struct N {
    SrNode<T> v;
    int l = -1, r = -1;
  };
  std::vector<N> a;
  int build(const SrTree<T>& t, size_t* pos) {
    const int id = int(a.size());
    a.push_back(N{t[*pos], -1, -1});
    ++*pos;
    if (a[id].v.degree >= 1) {
      const int l = build(t, pos);
      a[id].l = l;
    }
    if (a[id].v.degree == 2) {
      const int r = build(t, pos);
      a[id].r = r;
    }
    return id;
  }
  void emit(int id, SrTree<T>* out) const {
    out->push_back(a[id].v);
    if (a[id].v.degree >= 1) emit(a[id].l, out);
    if (a[id].v.degree == 2) emit(a[id].r, out);
  }
  bool is_const(int id) const { return a[id].v.degree == 0 && a[id].v.constant; }
};

template <typename T>
inline bool sr_is_valid(T x) {
  return sr_isfinite(x);
}

template <typename T>
inline void sr_fold_constants(SrArena<T>& A, int id, const SrTreeSpec& sp) {
  auto& n = A.a[id];
  if (n.v.degree == 0) return;
  sr_fold_constants(A, n.l, sp);
  if (n.v.degree == 2) sr_fold_constants(A, A.a[id].r, sp);
  auto& m = A.a[id];
  if (!A.is_const(m.l) || (m.v.degree == 2 && !A.is_const(m.r))) return;
  const T x = A.a[m.l].v.val;
  if (!sr_is_valid(x)) return;
  T out;
  if (m.v.degree == 1) {
    out = sr_unary<T>(sp.unary_ids[m.v.op - 1], x);
  } else {
    const T y = A.a[m.r].v.val;
    if (!sr_is_valid(y)) return;
    out = sr_binary<T>(sp.binary_ids[m.v.op - 1], x, y);
  }
  if (!sr_is_valid(out)) return;
  SrNode<T> c;
  c.constant = 1;
  c.val = out;
  m.v = c;
  m.l = m.r = -1;
}

template <typename T>
inline int sr_combine_operators(SrArena<T>& A, int id, const SrTreeSpec& sp) {
  {
    auto& n = A.a[id];
    if (n.v.degree == 0) return id;
    const int l = sr_combine_operators(A, n.l, sp);
    A.a[id].l = l;
    if (A.a[id].v.degree == 2) {
      const int r = sr_combine_operators(A, A.a[id].r, sp);
      A.a[id].r = r;
    }
  }
  auto bid = [&](int i) { return sp.binary_ids[A.a[i].v.op - 1]; };
  auto node = [&](int i) -> typename SrArena<T>::N& { return A.a[i]; };
  const bool top_const = node(id).v.degree == 2 && (A.is_const(node(id).l) || A.is_const(node(id).r));
  if (top_const && (bid(id) == SR_B_MUL || bid(id) == SR_B_ADD)) {
    const uint8_t op = node(id).v.op;
    const uint32_t b = bid(id);
    if (A.is_const(node(id).l)) std::swap(node(id).l, node(id).r);  // constant on the right
    const T top = node(node(id).r).v.val;
    const int below = node(id).l;
    if (node(below).v.degree == 2 && node(below).v.op == op) {
      if (A.is_const(node(below).l)) {
        id = below;
        node(node(id).l).v.val = sr_binary<T>(b, node(node(id).l).v.val, top);
      } else if (A.is_const(node(below).r)) {
        id = below;
        node(node(id).r).v.val = sr_binary<T>(b, node(node(id).r).v.val, top);
      }
    }
  }
  if (node(id).v.degree == 2 && bid(id) == SR_B_SUB &&
      (A.is_const(node(id).l) || A.is_const(node(id).r))) {
    if (A.is_const(node(id).l)) {
      const int r = node(id).r;
      if (node(r).v.degree == 2 && bid(r) == SR_B_SUB) {
        const int l = node(id).l;
        if (A.is_const(node(r).l)) {
          // (c1 - (c2 - x)) => (x - (-(c1 - c2)))
          const T c = -(node(l).v.val - node(node(r).l).v.val);
          node(id).l = node(r).r;
          node(id).r = l;
          node(l).v.val = c;
        } else if (A.is_const(node(r).r)) {
          // (c1 - (x - c2)) => ((c1 + c2) - x)
          const T c = node(l).v.val + node(node(r).r).v.val;
          node(id).r = node(r).l;
          node(l).v.val = c;
        }
      }
    } else {
      const int l = node(id).l;
      if (node(l).v.degree == 2 && bid(l) == SR_B_SUB) {
        const int r = node(id).r;
        if (A.is_const(node(l).l)) {
          // ((c1 - x) - c2) => ((c1 - c2) - x)
          const T c = node(node(l).l).v.val - node(r).v.val;
          node(id).r = node(l).r;
          node(id).l = r;
          node(r).v.val = c;
        } else if (A.is_const(node(l).r)) {
          // ((x - c1) - c2) => (x - (c1 + c2))
          const T c = node(r).v.val + node(node(l).r).v.val;
          node(id).l = node(l).l;
          node(r).v.val = c;
        }
      }
    }
  }
  return id;
}

template <typename T>
inline void sr_simplify_tree(SrTree<T>& t, const SrTreeSpec& sp) {
  SrArena<T> A;
  A.a.reserve(t.size());
  size_t pos = 0;
  const int root = A.build(t, &pos);
  sr_fold_constants(A, root, sp);
  const int r2 = sr_combine_operators(A, root, sp);
  SrTree<T> out;
  out.reserve(t.size());
  A.emit(r2, &out);
  t.swap(out);
}
