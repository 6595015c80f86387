/*
 * de_eval_impl.h — TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline).  Included twice by
 * de_eval.c with T = float / double.  Nothing in the product path links this code.
 *
 * Restatement of DynamicExpressions 2.4's CPU evaluator as SymbolicRegression calls it
 * (src/InterfaceDynamicExpressions.jl:58-88 -> DE.eval_tree_array(tree, X, operators;
 * eval_options=EvalOptions(turbo=false, bumper=false))).  DE is not vendored in the reference; the
 * control flow below is restated from its published algorithm and pinned by the reference tests
 * listed in DESIGN.md §3 (test_evaluation.jl fused shapes, test_nan_detection.jl flags):
 *   _eval_tree_array(tree):
 *     degree 0                -> deg0_eval: constant -> fill(val), feature -> copy of X[f, :]
 *     is_constant(tree)       -> dispatch_constant_tree: scalar fold, is_valid after each op
 *     degree 1                -> fused deg1_l2_ll0_lr0 / deg1_l1_ll0 (x = is_valid(x_l) ? op(x_l) : Inf)
 *                                else child evaluated, early exit if !is_valid_array(child)
 *     degree 2                -> deg2_l0_r0 (scalar-checked constants), deg2_l0 / deg2_r0 (the non-leaf
 *                                child evaluated + checked), general (both evaluated + checked)
 *   eval_tree_array: complete = result.ok && is_valid_array(result)
 *   is_valid(x) = isfinite(x); is_valid_array(a) = isfinite(sum(a)) with Julia's pairwise `sum`
 *   (Base.mapreduce_impl, block size 1024).
 * Loss (src/LossFunctions.jl:38-58 via LossFunctions.jl): L2DistLoss abs2(ŷ - y) / L1DistLoss
 * abs(ŷ - y); mean = sequential T fold / n ("ref" accumulation) or an f64 fold ("f64").
 */

#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)
#define FN(name) CAT(name, SFX)

typedef struct {
  int64_t n;
  const uint8_t* degree;
  const uint8_t* op;
  const uint16_t* feature;
  const uint8_t* constant;
  const T* val;
  int32_t* left;  /* child positions (filled by parse) */
  int32_t* right;
  uint8_t* is_const;
  const int32_t* un_ids;
  const int32_t* bin_ids;
  int n_un, n_bin;
  int perturb; /* 0, or +-1: scale every libm result by (1 + perturb * eps) (conditioning probe) */
} FN(otree);

/* ---------------------------------------------------------------- operators (src/Operators.jl) */
static T FN(o_nan)(void) { return (T)NAN; }

static T FN(o_unary)(int id, T x) {
  switch (id) {
    case O_NEG: return -x;
    case O_SQUARE: return x * x;                           /* Operators.jl:81 */
    case O_CUBE: return x * x * x;                         /* Operators.jl:82 */
    case O_EXP: return x > MAX_EXP ? (T)INFINITY : M_EXP(x); /* Julia exp overflow threshold */
    case O_COS: return M_COS(x);
    case O_SIN: return M_SIN(x);
    case O_TAN: return M_TAN(x);
    case O_LOG: return x > (T)0 ? M_LOG(x) : FN(o_nan)();          /* safe_log :50-52 */
    case O_LOG2: return x > (T)0 ? M_LOG2(x) : FN(o_nan)();        /* safe_log2 */
    case O_LOG10: return x > (T)0 ? M_LOG10(x) : FN(o_nan)();      /* safe_log10 */
    case O_LOG1P: return x > (T)-1 ? M_LOG1P(x) : FN(o_nan)();     /* safe_log1p */
    case O_SQRT: return x >= (T)0 ? M_SQRT(x) : FN(o_nan)();       /* safe_sqrt :74-76 */
    case O_ABS: return M_FABS(x);
    case O_SIGN: return x < (T)0 ? (T)-1 : (x > (T)0 ? (T)1 : x);
    case O_TANH: return M_TANH(x);
    case O_SINH: return M_SINH(x);
    case O_COSH: return M_COSH(x);
    case O_ATAN: return M_ATAN(x);
    case O_ASIN: return (x >= (T)-1 && x <= (T)1) ? M_ASIN(x) : FN(o_nan)();
    case O_ACOS: return (x >= (T)-1 && x <= (T)1) ? M_ACOS(x) : FN(o_nan)();
    case O_ACOSH: return x >= (T)1 ? M_ACOSH(x) : FN(o_nan)();
    case O_ATANH: return (x >= (T)-1 && x <= (T)1) ? M_ATANH(x) : FN(o_nan)();
    case O_ASINH: return M_ASINH(x);
    case O_RELU: return x > (T)0 ? x : M_COPYSIGN((T)0, x);      /* (x > 0) * x, Bool strong zero */
    case O_INV: return (T)1 / x;
    case O_ERF: return M_ERF(x);
    case O_ERFC: return M_ERFC(x);
    case O_GAMMA: { T g = M_TGAMMA(x); return isinf(g) ? FN(o_nan)() : g; }
    case O_ROUND: return M_RINT(x);
    case O_FLOOR: return M_FLOOR(x);
    case O_CEIL: return M_CEIL(x);
    case O_EXP2: return M_EXP2(x);
    case O_EXPM1: return M_EXPM1(x);
  }
  return FN(o_nan)();
}

static T FN(o_binary)(int id, T x, T y) {
  switch (id) {
    case O_ADD: return x + y;
    case O_SUB: return x - y;
    case O_MUL: return x * y;
    case O_DIV: return x / y;
    case O_POW: { /* safe_pow, Operators.jl:35-49 */
      const int isint = (y - M_TRUNC(y)) == (T)0;
      if (isint) {
        if (y < (T)0 && x == (T)0) return FN(o_nan)();
      } else {
        if (y > (T)0 && x < (T)0) return FN(o_nan)();
        if (y < (T)0 && x <= (T)0) return FN(o_nan)();
      }
      return M_POW(x, y);
    }
    case O_MAX:
      if (isnan(x)) return x;
      if (isnan(y)) return y;
      return (y > x || (x == y && signbit(x) && !signbit(y))) ? y : x;
    case O_MIN:
      if (isnan(x)) return x;
      if (isnan(y)) return y;
      return (y < x || (x == y && signbit(y) && !signbit(x))) ? y : x;
    case O_MOD: {
      T r = M_FMOD(x, y);
      if (r == (T)0) return M_COPYSIGN(r, y);
      if ((r > (T)0) != (y > (T)0)) return r + y;
      return r;
    }
    case O_GREATER: return x > y ? (T)1 : (T)0;
    case O_LESS: return x < y ? (T)1 : (T)0;
    case O_GREATER_EQUAL: return x >= y ? (T)1 : (T)0;
    case O_LESS_EQUAL: return x <= y ? (T)1 : (T)0;
    case O_COND: return x > (T)0 ? y : M_COPYSIGN((T)0, y);
    case O_LOGICAL_OR: return (x > (T)0 || y > (T)0) ? (T)1 : (T)0;
    case O_LOGICAL_AND: return (x > (T)0 && y > (T)0) ? (T)1 : (T)0;
    case O_ATAN2: return M_ATAN2(x, y);
  }
  return FN(o_nan)();
}

/* Conditioning probe: a libm whose results differ by +-1 ulp with a pseudo-random sign per
 * (node, row) — independent last-bit differences, as between two correctly rounded libms.
 * Seed p != 0 selects the sign pattern; exact IEEE ops (and sqrt) are left alone. */
static int FN(psign)(int node, int64_t row, int p) {
  uint32_t h = (uint32_t)node * 0x9E3779B1u ^ (uint32_t)row * 0x85EBCA77u ^ (uint32_t)p * 0xC2B2AE3Du;
  h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
  return (h & 1u) ? 1 : -1;
}
/* p = seed | (op << 8): a non-zero op (unary id, or 64 + binary id) restricts the probe to that one
 * operator (bench.py's parity.held_trees names the operator a tree's loss is most sensitive to). */
static T FN(perturb_unary)(int id, T v, int p, int node, int64_t row) {
  if (!p) return v;
  if ((p >> 8) && (p >> 8) != id) return v;
  p &= 0xff;
  switch (id) {
    case O_NEG: case O_SQUARE: case O_CUBE: case O_ABS: case O_SIGN: case O_RELU: case O_INV:
    case O_ROUND: case O_FLOOR: case O_CEIL: case O_SQRT:
      return v;
  }
  return v * ((T)1 + (T)FN(psign)(node, row, p) * PERTURB_EPS);
}
static T FN(perturb_binary)(int id, T v, int p, int node, int64_t row) {
  if (!p || id != O_POW) return v;
  if ((p >> 8) && (p >> 8) != 64 + id) return v;
  p &= 0xff;
  return v * ((T)1 + (T)FN(psign)(node, row, p) * PERTURB_EPS);
}

/* ---------------------------------------------------------------- Julia sum (pairwise) */
static T FN(jl_sum_range)(const T* a, int64_t lo, int64_t hi) { /* inclusive [lo, hi] */
  if (lo == hi) return a[lo];
  if (hi - lo < 1024) {
    T v = a[lo] + a[lo + 1];
    for (int64_t i = lo + 2; i <= hi; ++i) v = v + a[i];
    return v;
  }
  const int64_t mid = lo + ((hi - lo) >> 1);
  const T v1 = FN(jl_sum_range)(a, lo, mid);
  const T v2 = FN(jl_sum_range)(a, mid + 1, hi);
  return v1 + v2;
}
static int FN(is_valid_array)(const T* a, int64_t n) {
  if (n == 0) return 1;
  const T s = FN(jl_sum_range)(a, 0, n - 1);
  return isfinite(s) ? 1 : 0;
}

/* ---------------------------------------------------------------- tree structure */
static int FN(parse)(FN(otree) * t) {
  int64_t pos = 0;
  int32_t* stack_parent = (int32_t*)malloc(sizeof(int32_t) * (size_t)(2 * t->n + 2));
  int8_t* stack_which = (int8_t*)malloc((size_t)(2 * t->n + 2));
  int64_t sp = 0;
  stack_parent[sp] = -1;
  stack_which[sp] = 0;
  ++sp;
  int ok = 1;
  while (sp > 0) {
    --sp;
    const int32_t parent = stack_parent[sp];
    const int which = stack_which[sp];
    if (pos >= t->n) { ok = 0; break; }
    const int32_t i = (int32_t)pos++;
    if (parent >= 0) {
      if (which == 0) t->left[parent] = i; else t->right[parent] = i;
    }
    t->left[i] = t->right[i] = -1;
    const int d = t->degree[i];
    if (d == 2) {
      stack_parent[sp] = i; stack_which[sp] = 1; ++sp;
      stack_parent[sp] = i; stack_which[sp] = 0; ++sp;
    } else if (d == 1) {
      stack_parent[sp] = i; stack_which[sp] = 0; ++sp;
    } else if (d != 0) { ok = 0; break; }
  }
  if (pos != t->n) ok = 0;
  free(stack_parent);
  free(stack_which);
  if (!ok) return 0;
  for (int64_t i = t->n - 1; i >= 0; --i) {
    const int d = t->degree[i];
    if (d == 0) t->is_const[i] = t->constant[i] ? 1 : 0;
    else if (d == 1) t->is_const[i] = t->is_const[t->left[i]];
    else t->is_const[i] = t->is_const[t->left[i]] && t->is_const[t->right[i]];
  }
  return 1;
}

static int FN(uid)(const FN(otree) * t, int i) { return t->un_ids[t->op[i] - 1]; }
static int FN(bid)(const FN(otree) * t, int i) { return t->bin_ids[t->op[i] - 1]; }

/* dispatch_constant_tree: scalar with validity (leaf constants validated too: DESIGN.md §3) */
static int FN(const_tree)(const FN(otree) * t, int i, T* out) {
  const int d = t->degree[i];
  if (d == 0) {
    *out = t->val[i];
    return isfinite(*out) ? 1 : 0;
  }
  if (d == 1) {
    T x;
    if (!FN(const_tree)(t, t->left[i], &x)) return 0;
    *out = FN(perturb_unary)(FN(uid)(t, i), FN(o_unary)(FN(uid)(t, i), x), t->perturb, i, 0);
    return isfinite(*out) ? 1 : 0;
  }
  T a, b;
  if (!FN(const_tree)(t, t->left[i], &a)) return 0;
  if (!FN(const_tree)(t, t->right[i], &b)) return 0;
  *out = FN(perturb_binary)(FN(bid)(t, i), FN(o_binary)(FN(bid)(t, i), a, b), t->perturb, i, 0);
  return isfinite(*out) ? 1 : 0;
}

/* X is Julia column-major [nf, n]: X[f, j] at f + nf*j (f 0-based here). */
typedef struct {
  const T* X;
  int64_t nf, n;
} FN(oview);

static T FN(xat)(const FN(oview) * v, int f, int64_t j) { return v->X[(int64_t)f + v->nf * j]; }

/* _eval_tree_array: returns a malloc'd array (n) in *out; result ok flag. */
static int FN(eval_rec)(const FN(otree) * t, int i, const FN(oview) * v, T** out);

static T* FN(alloc)(int64_t n) { return (T*)malloc(sizeof(T) * (size_t)(n > 0 ? n : 1)); }

static int FN(eval_rec)(const FN(otree) * t, int i, const FN(oview) * v, T** out) {
  const int64_t n = v->n;
  T* r = FN(alloc)(n);
  *out = r;
  const int d = t->degree[i];
  if (d == 0) { /* deg0_eval */
    if (t->constant[i]) {
      for (int64_t j = 0; j < n; ++j) r[j] = t->val[i];
    } else {
      const int f = t->feature[i] - 1;
      for (int64_t j = 0; j < n; ++j) r[j] = FN(xat)(v, f, j);
    }
    return 1;
  }
  if (t->is_const[i]) { /* speed hack for constant trees */
    T c;
    if (!FN(const_tree)(t, i, &c)) return 0;
    for (int64_t j = 0; j < n; ++j) r[j] = c;
    return 1;
  }
  if (d == 1) {
    const int op = FN(uid)(t, i);
    const int l = t->left[i];
    if (t->degree[l] == 2 && t->degree[t->left[l]] == 0 && t->degree[t->right[l]] == 0) {
      /* deg1_l2_ll0_lr0_eval */
      const int ll = t->left[l], lr = t->right[l];
      const int op_l = FN(bid)(t, l);
      if (t->constant[ll] && !isfinite(t->val[ll])) return 0;
      if (t->constant[lr] && !isfinite(t->val[lr])) return 0;
      for (int64_t j = 0; j < n; ++j) {
        const T a = t->constant[ll] ? t->val[ll] : FN(xat)(v, t->feature[ll] - 1, j);
        const T b = t->constant[lr] ? t->val[lr] : FN(xat)(v, t->feature[lr] - 1, j);
        const T x_l = FN(perturb_binary)(op_l, FN(o_binary)(op_l, a, b), t->perturb, l, j);
        r[j] = isfinite(x_l) ? FN(perturb_unary)(op, FN(o_unary)(op, x_l), t->perturb, i, j) : (T)INFINITY;
      }
      return 1;
    }
    if (t->degree[l] == 1 && t->degree[t->left[l]] == 0) {
      /* deg1_l1_ll0_eval */
      const int ll = t->left[l];
      const int op_l = FN(uid)(t, l);
      if (t->constant[ll] && !isfinite(t->val[ll])) return 0;
      for (int64_t j = 0; j < n; ++j) {
        const T a = t->constant[ll] ? t->val[ll] : FN(xat)(v, t->feature[ll] - 1, j);
        const T x_l = FN(perturb_unary)(op_l, FN(o_unary)(op_l, a), t->perturb, l, j);
        r[j] = isfinite(x_l) ? FN(perturb_unary)(op, FN(o_unary)(op, x_l), t->perturb, i, j) : (T)INFINITY;
      }
      return 1;
    }
    /* general deg1: evaluate child, early exit on non-finite array */
    T* c = NULL;
    const int ok = FN(eval_rec)(t, l, v, &c);
    if (!ok || !FN(is_valid_array)(c, n)) {
      free(c);
      return 0;
    }
    for (int64_t j = 0; j < n; ++j) r[j] = FN(perturb_unary)(op, FN(o_unary)(op, c[j]), t->perturb, i, j);
    free(c);
    return 1;
  }
  /* degree 2 */
  const int op = FN(bid)(t, i);
  const int l = t->left[i], rr = t->right[i];
  const int l0 = t->degree[l] == 0, r0 = t->degree[rr] == 0;
  if (l0 && r0) { /* deg2_l0_r0_eval */
    if (t->constant[l] && !isfinite(t->val[l])) return 0;
    if (t->constant[rr] && !isfinite(t->val[rr])) return 0;
    for (int64_t j = 0; j < n; ++j) {
      const T a = t->constant[l] ? t->val[l] : FN(xat)(v, t->feature[l] - 1, j);
      const T b = t->constant[rr] ? t->val[rr] : FN(xat)(v, t->feature[rr] - 1, j);
      r[j] = FN(perturb_binary)(op, FN(o_binary)(op, a, b), t->perturb, i, j);
    }
    return 1;
  }
  if (r0) { /* deg2_r0_eval: left evaluated + checked, right leaf */
    T* c = NULL;
    const int ok = FN(eval_rec)(t, l, v, &c);
    if (!ok || !FN(is_valid_array)(c, n)) { free(c); return 0; }
    if (t->constant[rr] && !isfinite(t->val[rr])) { free(c); return 0; }
    for (int64_t j = 0; j < n; ++j) {
      const T b = t->constant[rr] ? t->val[rr] : FN(xat)(v, t->feature[rr] - 1, j);
      r[j] = FN(perturb_binary)(op, FN(o_binary)(op, c[j], b), t->perturb, i, j);
    }
    free(c);
    return 1;
  }
  if (l0) { /* deg2_l0_eval: right evaluated + checked, left leaf */
    T* c = NULL;
    const int ok = FN(eval_rec)(t, rr, v, &c);
    if (!ok || !FN(is_valid_array)(c, n)) { free(c); return 0; }
    if (t->constant[l] && !isfinite(t->val[l])) { free(c); return 0; }
    for (int64_t j = 0; j < n; ++j) {
      const T a = t->constant[l] ? t->val[l] : FN(xat)(v, t->feature[l] - 1, j);
      r[j] = FN(perturb_binary)(op, FN(o_binary)(op, a, c[j]), t->perturb, i, j);
    }
    free(c);
    return 1;
  }
  /* general deg2 */
  T* a = NULL;
  int ok = FN(eval_rec)(t, l, v, &a);
  if (!ok || !FN(is_valid_array)(a, n)) { free(a); return 0; }
  T* b = NULL;
  ok = FN(eval_rec)(t, rr, v, &b);
  if (!ok || !FN(is_valid_array)(b, n)) { free(a); free(b); return 0; }
  for (int64_t j = 0; j < n; ++j) r[j] = FN(perturb_binary)(op, FN(o_binary)(op, a[j], b[j]), t->perturb, i, j);
  free(a);
  free(b);
  return 1;
}

/* eval_tree_array(tree, X, operators) -> out[n], complete. Returns 0 on malformed input. */
int FN(oracle_eval_tree)(int64_t n_nodes, const uint8_t* degree, const uint8_t* op, const uint16_t* feature,
                         const uint8_t* constant, const T* val, const int32_t* un_ids, int n_un,
                         const int32_t* bin_ids, int n_bin, const T* X, int64_t nf, int64_t n, T* out,
                         int* complete, int perturb) {
  FN(otree) t;
  t.perturb = perturb;
  t.n = n_nodes; t.degree = degree; t.op = op; t.feature = feature; t.constant = constant; t.val = val;
  t.un_ids = un_ids; t.bin_ids = bin_ids; t.n_un = n_un; t.n_bin = n_bin;
  t.left = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_nodes);
  t.right = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_nodes);
  t.is_const = (uint8_t*)malloc((size_t)n_nodes);
  if (!FN(parse)(&t)) {
    free(t.left); free(t.right); free(t.is_const);
    return 0;
  }
  for (int64_t i = 0; i < n_nodes; ++i) {
    if (degree[i] == 0 && !constant[i] && (feature[i] < 1 || feature[i] > nf)) {
      free(t.left); free(t.right); free(t.is_const);
      return 0;
    }
    if (degree[i] == 1 && (op[i] < 1 || op[i] > n_un)) { free(t.left); free(t.right); free(t.is_const); return 0; }
    if (degree[i] == 2 && (op[i] < 1 || op[i] > n_bin)) { free(t.left); free(t.right); free(t.is_const); return 0; }
  }
  FN(oview) v;
  v.X = X; v.nf = nf; v.n = n;
  T* r = NULL;
  int ok = FN(eval_rec)(&t, 0, &v, &r);
  ok = ok && FN(is_valid_array)(r, n);
  if (out) memcpy(out, r, sizeof(T) * (size_t)n);
  free(r);
  *complete = ok;
  free(t.left); free(t.right); free(t.is_const);
  return 1;
}

/* LossFunctions.jl 0.11 SupervisedLoss values (not vendored; published definitions restated):
 * d = output - target, a = target * output, p = the loss's parameter.  Julia's max(0, x) propagates
 * NaN.  Kinds as SrLossKind (csrc/sr_ops.h). */
static inline T FN(pos)(T x) { return (x != x) ? x : (x > (T)0 ? x : (T)0); }
static inline T FN(elem_loss)(int kind, double pd, T pred, T target) {
  const T p = (T)pd, d = pred - target, ad = M_FABS(d), a = target * pred;
  T e;
  switch (kind) {
    case 1: return ad;                                                     /* L1DistLoss */
    case 2: return M_POW(ad, p);                                           /* LPDistLoss{P} */
    case 3: return -M_LOG((T)4) - d + (T)2 * M_LOG((T)1 + M_EXP(d));       /* LogitDistLoss */
    case 4: return ad <= p ? d * d / (T)2 : p * (ad - p / (T)2);           /* HuberLoss(d) */
    case 5: return FN(pos)(ad - p);                                        /* L1EpsilonInsLoss */
    case 6: e = FN(pos)(ad - p); return e * e;                             /* L2EpsilonInsLoss */
    case 7: return (T)1 - M_COS(d * ((T)2 * (T)3.14159265358979323846 / p)); /* PeriodicLoss(circ) */
    case 8: return d * ((d > (T)0 ? (T)1 : (T)0) - p);                     /* QuantileLoss(tau) */
    case 9: return a < (T)0 ? (T)1 : (T)0;                                 /* ZeroOneLoss */
    case 10: return FN(pos)(-a);                                           /* PerceptronLoss */
    case 11: return FN(pos)((T)1 - a);                                     /* L1HingeLoss */
    case 12: e = FN(pos)((T)1 - a); return e * e;                          /* L2HingeLoss */
    case 13:                                                               /* SmoothedL1HingeLoss(g) */
      if (a >= (T)1 - p) { e = FN(pos)((T)1 - a); return e * e / ((T)2 * p); }
      return (T)1 - p / (T)2 - a;
    case 14:                                                               /* ModifiedHuberLoss */
      if (a >= (T)-1) { e = FN(pos)((T)1 - a); return e * e; }
      return (T)-4 * a;
    case 15: e = (T)1 - a; return e * e;                                   /* L2MarginLoss */
    case 16: return M_EXP(-a);                                             /* ExpLoss */
    case 17: return (T)1 - M_TANH(a);                                      /* SigmoidLoss */
    case 18:                                                               /* DWDMarginLoss(q) */
      if (a <= p / (p + (T)1)) return (T)1 - a;
      return (M_POW(p, p) / M_POW(p + (T)1, p + (T)1)) / M_POW(a, p);
    default: return d * d;                                                 /* L2DistLoss */
  }
}

/* _eval_loss: L(Inf) if incomplete; accum 0 = sequential T fold ("ref"), 1 = f64 fold. */
int FN(oracle_eval_loss)(int64_t n_nodes, const uint8_t* degree, const uint8_t* op, const uint16_t* feature,
                         const uint8_t* constant, const T* val, const int32_t* un_ids, int n_un,
                         const int32_t* bin_ids, int n_bin, const T* X, int64_t nf, int64_t n, const T* y,
                         const T* w, int loss_kind, double loss_param, int accum, T* loss, int* complete,
                         int perturb) {
  T* pred = FN(alloc)(n);
  if (!FN(oracle_eval_tree)(n_nodes, degree, op, feature, constant, val, un_ids, n_un, bin_ids, n_bin, X, nf, n,
                            pred, complete, perturb)) {
    free(pred);
    return 0;
  }
  if (!*complete) {
    *loss = (T)INFINITY;
    free(pred);
    return 1;
  }
  if (accum == 0) {
    /* LossFunctions 0.11: mean(loss, x, y) = the left fold of the losses / n; the weighted
     * sum(loss, x, y, w; normalize=true) = the left fold of w_i * l_i / sum(w), where sum(w) is Base's
     * pairwise sum of the weight vector in T (jl_sum_range; ADVICE r4: not a sequential fold) */
    T s = (T)0;
    for (int64_t j = 0; j < n; ++j) {
      T l = FN(elem_loss)(loss_kind, loss_param, pred[j], y[j]);
      if (w) l = w[j] * l;
      s = j == 0 ? l : s + l;
    }
    const T ws = (w && n > 0) ? FN(jl_sum_range)(w, 0, n - 1) : (T)0;
    *loss = w ? s / ws : s / (T)n;
  } else {
    /* the value from an f64 accumulation (the device's arithmetic), the overflow verdict from the
     * reference's own T fold (src/LossFunctions.jl:38-58: a fold that passes floatmax(T) is +Inf) */
    double s = 0.0, ws = 0.0;
    T st = (T)0;
    for (int64_t j = 0; j < n; ++j) {
      T l = FN(elem_loss)(loss_kind, loss_param, pred[j], y[j]);
      if (w) { l = w[j] * l; ws += (double)w[j]; }
      s += (double)l;
      st = j == 0 ? l : st + l;
    }
    *loss = (T)(w ? s / ws : s / (double)n);
    if (st == (T)INFINITY) *loss = (T)INFINITY;
  }
  free(pred);
  return 1;
}

/* Batched loss over many trees (the CPU baseline: OpenMP over trees, each tree single-threaded,
 * as SymbolicRegression parallelises scoring across islands/members). */
int FN(oracle_eval_loss_batch)(int64_t n_trees, const int64_t* offsets, const uint8_t* degree, const uint8_t* op,
                               const uint16_t* feature, const uint8_t* constant, const T* val,
                               const int32_t* un_ids, int n_un, const int32_t* bin_ids, int n_bin, const T* X,
                               int64_t nf, int64_t n, const T* y, const T* w, int loss_kind, double loss_param,
                               int accum, int n_threads, T* loss, int* complete, int perturb) {
  int bad = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads) reduction(| : bad)
  for (int64_t k = 0; k < n_trees; ++k) {
    const int64_t b = offsets[k], e = offsets[k + 1];
    int c = 0;
    if (!FN(oracle_eval_loss)(e - b, degree + b, op + b, feature + b, constant + b, val + b, un_ids, n_un, bin_ids,
                              n_bin, X, nf, n, y, w, loss_kind, loss_param, accum, loss + k, &c, perturb))
      bad |= 1;
    complete[k] = c;
  }
  return bad ? 0 : 1;
}

/* The search engine's CPU scorers (sr_search_use_callbacks): the same engine, seeds and draws as a
 * device-scored search, with every batched scoring call answered by this port on the host cores —
 * the "port" CPU baseline of the search-throughput metric (bench.py).  The loss folds sequentially in
 * T (the reference's order).  The gradient is what the reference's Optim BFGS uses by default
 * (src/ConstantOptimization.jl:77-116, autodiff_backend = nothing): central finite differences of
 * that loss, step cbrt(eps(T)) * max(1, |c|) per constant (FiniteDiff.jl's central rule). */
typedef struct {
  const void* X;  /* Julia layout [n][nf] (row j's features contiguous) */
  int64_t nf, n;
  const void* y;
  const void* w;  /* NULL: unweighted */
  const int32_t* un;
  int n_un;
  const int32_t* bi;
  int n_bi;
  int loss_kind;
  double loss_param;
  int n_threads;
} FN(oscorer);

static int FN(view_gather)(const FN(oscorer) * sc, const int64_t* row_idx, int64_t n_idx, T** Xv, T** yv, T** wv) {
  *Xv = NULL; *yv = NULL; *wv = NULL;
  if (!row_idx || n_idx <= 0) return 0;
  *Xv = FN(alloc)(n_idx * sc->nf);
  *yv = FN(alloc)(n_idx);
  if (sc->w) *wv = FN(alloc)(n_idx);
  for (int64_t i = 0; i < n_idx; ++i) {
    const int64_t r = row_idx[i];
    memcpy(*Xv + i * sc->nf, (const T*)sc->X + r * sc->nf, sizeof(T) * (size_t)sc->nf);
    (*yv)[i] = ((const T*)sc->y)[r];
    if (sc->w) (*wv)[i] = ((const T*)sc->w)[r];
  }
  return 1;
}

int FN(oracle_search_loss)(void* user, const oracle_tree_batch* tb, const int64_t* row_idx, int64_t n_idx,
                           void* out_loss, uint8_t* out_complete) {
  const FN(oscorer)* sc = (const FN(oscorer)*)user;
  T *Xv, *yv, *wv;
  const int g = FN(view_gather)(sc, row_idx, n_idx, &Xv, &yv, &wv);
  const int64_t n = g ? n_idx : sc->n;
  int* comp = (int*)malloc(sizeof(int) * (size_t)(tb->n_trees > 0 ? tb->n_trees : 1));
  const int ok = FN(oracle_eval_loss_batch)(tb->n_trees, tb->offsets, tb->degree, tb->op, tb->feature, tb->constant,
                                            (const T*)tb->val, sc->un, sc->n_un, sc->bi, sc->n_bi,
                                            g ? Xv : (const T*)sc->X, sc->nf, n, g ? yv : (const T*)sc->y,
                                            g ? wv : (const T*)sc->w, sc->loss_kind, sc->loss_param, 0,
                                            sc->n_threads, (T*)out_loss, comp, 0);
  for (int64_t k = 0; k < tb->n_trees; ++k) out_complete[k] = comp[k] ? 1 : 0;
  free(comp); free(Xv); free(yv); free(wv);
  return ok ? 0 : -4;
}

int FN(oracle_search_grad)(void* user, const oracle_tree_batch* tb, const int64_t* row_idx, int64_t n_idx,
                           void* out_loss, void* out_grad, uint8_t* out_complete) {
  const FN(oscorer)* sc = (const FN(oscorer)*)user;
  T *Xv, *yv, *wv;
  const int g = FN(view_gather)(sc, row_idx, n_idx, &Xv, &yv, &wv);
  const int64_t n = g ? n_idx : sc->n;
  const T* X = g ? Xv : (const T*)sc->X;
  const T* y = g ? yv : (const T*)sc->y;
  const T* w = g ? wv : (const T*)sc->w;
  const T* val = (const T*)tb->val;
  /* first gradient slot of each tree (constants in pre-order, trees concatenated) */
  int64_t* goff = (int64_t*)malloc(sizeof(int64_t) * (size_t)(tb->n_trees + 1));
  goff[0] = 0;
  for (int64_t k = 0; k < tb->n_trees; ++k) {
    int64_t c = 0;
    for (int64_t i = tb->offsets[k]; i < tb->offsets[k + 1]; ++i) c += (tb->degree[i] == 0 && tb->constant[i]) ? 1 : 0;
    goff[k + 1] = goff[k] + c;
  }
  int bad = 0;
  const T h0 = (T)(sizeof(T) == 4 ? 4.921566601151848e-03 : 6.055454452393343e-06); /* cbrt(eps(T)) */
#pragma omp parallel for schedule(dynamic, 1) num_threads(sc->n_threads) reduction(| : bad)
  for (int64_t k = 0; k < tb->n_trees; ++k) {
    const int64_t b = tb->offsets[k], e = tb->offsets[k + 1];
    T* v = FN(alloc)(e - b);
    memcpy(v, val + b, sizeof(T) * (size_t)(e - b));
    int c = 0;
    T l0;
    if (!FN(oracle_eval_loss)(e - b, tb->degree + b, tb->op + b, tb->feature + b, tb->constant + b, v, sc->un,
                              sc->n_un, sc->bi, sc->n_bi, X, sc->nf, n, y, w, sc->loss_kind, sc->loss_param, 0, &l0,
                              &c, 0))
      bad |= 1;
    ((T*)out_loss)[k] = l0;
    out_complete[k] = c ? 1 : 0;
    int64_t slot = goff[k];
    for (int64_t i = 0; i < e - b; ++i) {
      if (!(tb->degree[b + i] == 0 && tb->constant[b + i])) continue;
      T gi = (T)0;
      if (c) {
        const T x0 = v[i];
        const T h = h0 * (M_FABS(x0) > (T)1 ? M_FABS(x0) : (T)1);
        T lp, lm;
        int cp = 0, cm = 0;
        v[i] = x0 + h;
        bad |= !FN(oracle_eval_loss)(e - b, tb->degree + b, tb->op + b, tb->feature + b, tb->constant + b, v, sc->un,
                                     sc->n_un, sc->bi, sc->n_bi, X, sc->nf, n, y, w, sc->loss_kind, sc->loss_param,
                                     0, &lp, &cp, 0);
        v[i] = x0 - h;
        bad |= !FN(oracle_eval_loss)(e - b, tb->degree + b, tb->op + b, tb->feature + b, tb->constant + b, v, sc->un,
                                     sc->n_un, sc->bi, sc->n_bi, X, sc->nf, n, y, w, sc->loss_kind, sc->loss_param,
                                     0, &lm, &cm, 0);
        v[i] = x0;
        gi = (lp - lm) / ((x0 + h) - (x0 - h));
      }
      ((T*)out_grad)[slot++] = gi;
    }
    free(v);
  }
  free(goff); free(Xv); free(yv); free(wv);
  return bad ? -4 : 0;
}

#undef FN
