// sr_constopt.h — batched constant optimisation (reference src/ConstantOptimization.jl:29-116).
//
// The reference optimises one member at a time: Optim.optimize with BFGS(linesearch=BackTracking())
// (Newton for a single constant) from the member's constants and from optimizer_nrestarts perturbed
// starts x0 .* (1 + eps/2), keeps the best, and adopts it only when it beats the starting loss.
// Here every member of a batch runs the same algorithm in lock-step: each round of line-search
// trials is ONE batched objective call and each gradient ONE batched gradient call over all members
// still iterating.  The optimiser restates Optim.jl's BFGS (inverse-Hessian update from the
// identity, g_abstol 1e-8, `iterations` = optimizer_iterations) and LineSearches.jl's BackTracking
// (order 3, c1 = 1e-4, rho_hi = 0.5, rho_lo = 0.1, initial step 1, halving until finite first);
// Newton for one constant takes its curvature from a central difference of the device gradient.
// Arithmetic is Float64 (Optim runs in T): the trajectory is not Optim's bit for bit, the objective
// and gradient values it consumes are the device's.
#pragma once
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

// Batched objective over (item, x) pairs: f -> losses, fg -> losses + gradients.  Items index the
// batch being optimised; calls return an SR_* status.
struct SrObjective {
  // false around evaluations the reference's Optim does not count in f_calls (Newton's curvature
  // probes: there the Hessian comes from its own differencing, not from objective calls)
  bool counting = true;
  virtual ~SrObjective() = default;
  virtual int f(const std::vector<int>& items, const std::vector<std::vector<double>>& xs, std::vector<double>* out) = 0;
  virtual int fg(const std::vector<int>& items, const std::vector<std::vector<double>>& xs, std::vector<double>* out,
                 std::vector<std::vector<double>>* grads) = 0;
};

namespace srco {

inline double dot(const std::vector<double>& a, const std::vector<double>& b) {
  double s = 0.0;
  for (size_t i = 0; i < a.size(); ++i) s += a[i] * b[i];
  return s;
}
inline double max_abs(const std::vector<double>& a) {
  double m = 0.0;
  for (double v : a) m = std::max(m, fabs(v));
  return m;
}
inline std::vector<double> axpy(const std::vector<double>& x, double a, const std::vector<double>& d) {
  std::vector<double> o(x.size());
  for (size_t i = 0; i < x.size(); ++i) o[i] = x[i] + a * d[i];
  return o;
}

// one BackTracking interpolation step (quadratic on the first iteration, cubic after)
inline double backtrack_step(double phi0, double dphi0, double a1, double a2, double phix0, double phix1, int it) {
  double a_tmp;
  if (it == 1) {
    const double den = 2.0 * (phix1 - phi0 - dphi0 * a2);
    a_tmp = den != 0.0 ? -(dphi0 * a2 * a2) / den : a2 * 0.5;
  } else {
    const double div = a2 != a1 ? 1.0 / (a1 * a1 * a2 * a2 * (a2 - a1)) : INFINITY;
    const double r1 = phix1 - phi0 - dphi0 * a2;
    const double r0 = phix0 - phi0 - dphi0 * a1;
    const double a = (a1 * a1 * r1 - a2 * a2 * r0) * div;
    const double b = (-a1 * a1 * a1 * r1 + a2 * a2 * a2 * r0) * div;
    if (!isfinite(a) || !isfinite(b)) {
      a_tmp = a2 * 0.5;
    } else if (fabs(a) <= 2.220446049250313e-16) {
      a_tmp = b != 0.0 ? dphi0 / (2.0 * b) : a2 * 0.5;
    } else {
      const double d = std::max(b * b - 3.0 * a * dphi0, 0.0);
      a_tmp = (-b + sqrt(d)) / (3.0 * a);
    }
  }
  if (!isfinite(a_tmp)) a_tmp = a2 * 0.5;
  a_tmp = std::min(a_tmp, a2 * 0.5);  // rho_hi
  return std::max(a_tmp, a2 * 0.1);   // rho_lo
}

// lock-step BackTracking for the members `idx` (positions into the caller's arrays)
inline int line_search(SrObjective& obj, const std::vector<int>& items, const std::vector<std::vector<double>>& xs,
                       const std::vector<double>& fs, const std::vector<std::vector<double>>& gs,
                       const std::vector<std::vector<double>>& dirs, std::vector<double>* alpha,
                       std::vector<double>* fnew, std::vector<uint8_t>* ok, std::vector<int>* trials) {
  const size_t n = items.size();
  const double c1 = 1e-4;
  std::vector<double> phi0(fs), dphi0(n), a1(n, 1.0), a2(n, 1.0), phix0(fs), phix1;
  for (size_t k = 0; k < n; ++k) dphi0[k] = dot(gs[k], dirs[k]);
  std::vector<std::vector<double>> trial(n);
  for (size_t k = 0; k < n; ++k) trial[k] = axpy(xs[k], 1.0, dirs[k]);
  int rc = obj.f(items, trial, &phix1);
  if (rc) return rc;
  std::vector<int> it(n, 0);
  std::vector<uint8_t> done(n, 0);
  trials->assign(n, 1);  // objective calls per item (the first trial above)
  for (int round = 0; round < 40; ++round) {
    std::vector<int> todo;
    for (size_t k = 0; k < n; ++k) {
      if (done[k]) continue;
      if (!isfinite(phix1[k])) {  // halve until the value is finite
        ++it[k];
        a1[k] = a2[k];
        a2[k] = a2[k] * 0.5;
        todo.push_back(int(k));
      } else if (phix1[k] > phi0[k] + c1 * a2[k] * dphi0[k]) {
        ++it[k];
        const double nw = backtrack_step(phi0[k], dphi0[k], a1[k], a2[k], phix0[k], phix1[k], it[k]);
        a1[k] = a2[k];
        a2[k] = nw;
        phix0[k] = phix1[k];
        todo.push_back(int(k));
      } else {
        done[k] = 1;
      }
    }
    if (todo.empty()) break;
    std::vector<int> sub;
    std::vector<std::vector<double>> tx;
    for (int k : todo) {
      sub.push_back(items[size_t(k)]);
      tx.push_back(axpy(xs[size_t(k)], a2[size_t(k)], dirs[size_t(k)]));
    }
    std::vector<double> vals;
    rc = obj.f(sub, tx, &vals);
    if (rc) return rc;
    for (size_t j = 0; j < todo.size(); ++j) {
      phix1[size_t(todo[j])] = vals[j];
      ++(*trials)[size_t(todo[j])];
    }
  }
  alpha->assign(a2.begin(), a2.end());
  *fnew = phix1;
  ok->assign(n, 0);
  for (size_t k = 0; k < n; ++k) (*ok)[k] = done[k] && isfinite(phix1[k]);
  return 0;
}

// batched BFGS (newton[k] = 0: n >= 2 constants) or 1-D Newton (newton[k] = 1: one constant) from
// x0s; minimisers and minima out.  Every item runs its own algorithm on its own values: the batch only
// decides which items share a call (each item's k-th line-search trial is in round k whatever the
// others do), so the restarts and both groups of a batch run in one lock-step pass.
// f_calls_limit > 0: Optim.Options' f_calls_limit — an item stops after the iteration at whose end its
// own objective calls (as Optim counts them: the curvature probes excluded) reach the limit.
inline int minimize(SrObjective& obj, const std::vector<int>& items, std::vector<std::vector<double>> xs,
                    int iterations, const std::vector<uint8_t>& newton, std::vector<std::vector<double>>* x_out,
                    std::vector<double>* f_out, int64_t f_calls_limit = 0) {
  const double g_tol = 1e-8;
  const size_t n = items.size();
  std::vector<double> fs;
  std::vector<std::vector<double>> gs;
  std::vector<int64_t> calls(n, 1);  // per item (start): the first value + gradient
  int rc = obj.fg(items, xs, &fs, &gs);
  if (rc) return rc;
  std::vector<std::vector<double>> invH(n);
  for (size_t k = 0; k < n; ++k)
    if (!newton[k]) {
      const size_t d = xs[k].size();
      invH[k].assign(d * d, 0.0);
      for (size_t i = 0; i < d; ++i) invH[k][i * d + i] = 1.0;
    }
  std::vector<uint8_t> active(n);
  for (size_t k = 0; k < n; ++k) active[k] = isfinite(fs[k]) && max_abs(gs[k]) > g_tol;
  for (int iter = 0; iter < iterations; ++iter) {
    std::vector<int> act;
    for (size_t k = 0; k < n; ++k)
      if (active[k]) act.push_back(int(k));
    if (act.empty()) break;
    std::vector<int> sub;
    std::vector<std::vector<double>> sx, sg, dirs;
    std::vector<double> sf;
    for (int k : act) sub.push_back(items[size_t(k)]);
    // Newton items: curvature from a central difference of the gradient, both probes of every such
    // item in ONE gradient call (x + h then x - h)
    std::vector<int> nsub;
    std::vector<std::vector<double>> probes, xm;
    std::vector<double> h;
    for (int k : act)
      if (newton[size_t(k)]) {
        const double hk = 1e-4 * std::max(1.0, fabs(xs[size_t(k)][0]));
        h.push_back(hk);
        nsub.push_back(items[size_t(k)]);
        probes.push_back({xs[size_t(k)][0] + hk});
        xm.push_back({xs[size_t(k)][0] - hk});
      }
    const size_t nn = nsub.size();
    std::vector<std::vector<double>> gpm;
    if (nn > 0) {
      for (size_t j = 0; j < nn; ++j) nsub.push_back(nsub[j]);
      probes.insert(probes.end(), xm.begin(), xm.end());
      std::vector<double> fpm;
      obj.counting = false;  // (num_evals follows Optim's f_calls: the curvature probes are not in it)
      rc = obj.fg(nsub, probes, &fpm, &gpm);
      obj.counting = true;
      if (rc) return rc;
    }
    size_t q = 0;
    for (int k : act) {
      if (newton[size_t(k)]) {
        double H = (gpm[q][0] - gpm[nn + q][0]) / (2.0 * h[q]);
        H = isfinite(H) ? (H > 1e-12 ? H : std::max(fabs(H), 1.0)) : 1.0;
        dirs.push_back({-gs[size_t(k)][0] / H});
        ++q;
        continue;
      }
      const size_t d = xs[size_t(k)].size();
      std::vector<double> dd(d, 0.0);
      for (size_t i = 0; i < d; ++i) {
        double s = 0.0;
        for (size_t j = 0; j < d; ++j) s += invH[size_t(k)][i * d + j] * gs[size_t(k)][j];
        dd[i] = -s;
      }
      dirs.push_back(dd);
    }
    for (int k : act) {
      sx.push_back(xs[size_t(k)]);
      sf.push_back(fs[size_t(k)]);
      sg.push_back(gs[size_t(k)]);
    }
    std::vector<double> alpha, fnew;
    std::vector<uint8_t> ok;
    std::vector<int> trials;
    if ((rc = line_search(obj, sub, sx, sf, sg, dirs, &alpha, &fnew, &ok, &trials))) return rc;
    for (size_t j = 0; j < act.size(); ++j) calls[size_t(act[j])] += trials[j];
    std::vector<int> moved;
    for (size_t j = 0; j < act.size(); ++j) {
      if (ok[j])
        moved.push_back(int(j));
      else
        active[size_t(act[j])] = 0;  // line search failed: Optim stops
    }
    if (moved.empty()) break;
    std::vector<int> msub;
    std::vector<std::vector<double>> xnew;
    for (int j : moved) {
      msub.push_back(sub[size_t(j)]);
      xnew.push_back(axpy(xs[size_t(act[size_t(j)])], alpha[size_t(j)], dirs[size_t(j)]));
    }
    std::vector<double> f2;
    std::vector<std::vector<double>> g2;
    if ((rc = obj.fg(msub, xnew, &f2, &g2))) return rc;
    for (size_t m = 0; m < moved.size(); ++m) {
      const size_t k = size_t(act[size_t(moved[m])]);
      ++calls[k];
      const size_t d = xs[k].size();
      std::vector<double> dx(d), dg(d);
      for (size_t i = 0; i < d; ++i) {
        dx[i] = xnew[m][i] - xs[k][i];
        dg[i] = g2[m][i] - gs[k][i];
      }
      xs[k] = xnew[m];
      fs[k] = f2[m];
      gs[k] = g2[m];
      if (newton[k]) {
        if (!isfinite(fs[k]) || fabs(gs[k][0]) <= g_tol) active[k] = 0;
        continue;
      }
      const double dx_dg = dot(dx, dg);
      if (!isfinite(fs[k]) || dx_dg == 0.0) {
        active[k] = 0;
        continue;
      }
      std::vector<double> u(d, 0.0);
      for (size_t i = 0; i < d; ++i)
        for (size_t j = 0; j < d; ++j) u[i] += invH[k][i * d + j] * dg[j];
      const double c1 = (dx_dg + dot(dg, u)) / (dx_dg * dx_dg);
      const double c2 = 1.0 / dx_dg;
      for (size_t i = 0; i < d; ++i)
        for (size_t j = 0; j < d; ++j)
          invH[k][i * d + j] += c1 * dx[i] * dx[j] - c2 * (u[i] * dx[j] + dx[i] * u[j]);
      if (max_abs(gs[k]) <= g_tol) active[k] = 0;
    }
    if (f_calls_limit > 0)
      for (int k : act)
        if (calls[size_t(k)] >= f_calls_limit) active[size_t(k)] = 0;  // (Optim: f_calls >= f_calls_limit)
  }
  *x_out = xs;
  *f_out = fs;
  return 0;
}

}  // namespace srco

// Optimise items [0, n) whose starting constants are x0[k] (restarts: starts[r][k] for r = 1..R, the
// perturbed x0 .* (1 + eps/2) drawn by the caller).  Out: best constants, best minimum, baseline
// f(x0); a member improves iff best < baseline.
inline int sr_optimize_batch(SrObjective& obj, const std::vector<std::vector<double>>& x0,
                             const std::vector<std::vector<std::vector<double>>>& restarts, int iterations,
                             std::vector<std::vector<double>>* best_x, std::vector<double>* best_f,
                             std::vector<double>* baseline, int64_t f_calls_limit = 0) {
  const size_t n = x0.size();
  std::vector<int> all(n);
  for (size_t k = 0; k < n; ++k) all[k] = int(k);
  int rc = obj.f(all, x0, baseline);
  if (rc) return rc;
  *best_x = x0;
  best_f->assign(n, INFINITY);
  // every (start, member) pair with constants, in the reference's order (the member's own constants
  // first, then each restart; per start BFGS members before Newton ones): one lock-step pass
  std::vector<int> items;
  std::vector<std::vector<double>> starts;
  std::vector<uint8_t> newton;
  for (size_t r = 0; r <= restarts.size(); ++r)
    for (int g = 0; g < 2; ++g)
      for (size_t k = 0; k < n; ++k) {
        if (x0[k].empty() || (x0[k].size() > 1) != (g == 0)) continue;  // (no constants: nothing to do)
        items.push_back(int(k));
        starts.push_back(r == 0 ? x0[k] : restarts[r - 1][k]);
        newton.push_back(g == 1 ? 1 : 0);
      }
  if (items.empty()) return 0;
  std::vector<std::vector<double>> xs;
  std::vector<double> fs;
  if ((rc = srco::minimize(obj, items, starts, iterations, newton, &xs, &fs, f_calls_limit))) return rc;
  for (size_t j = 0; j < items.size(); ++j) {  // the best over starts, earlier starts winning ties
    const size_t k = size_t(items[j]);
    if (fs[j] < (*best_f)[k]) {
      (*best_f)[k] = fs[j];
      (*best_x)[k] = xs[j];
    }
  }
  return 0;
}
