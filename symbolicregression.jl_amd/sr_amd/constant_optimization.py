"""Batched constant optimisation (reference src/ConstantOptimization.jl), driven by the device's
batched objective / forward-mode gradient.

The reference optimises one member at a time: ``optimize_constants`` (:29-59) runs
``Optim.optimize`` with ``BFGS(linesearch=BackTracking())`` (Newton for a single constant) from the
current constants and from ``optimizer_nrestarts`` perturbed starts ``x0 .* (1 + eps/2)``
(:77-116), keeps the best, and adopts it only if it beats the starting loss.  Here every member
of a batch runs the same algorithm in lock-step: each round of line-search trials is ONE
``sr_eval_loss_batch`` call and each gradient ONE ``sr_eval_grad_batch`` call for all members
still iterating, so a whole population's constant optimisation costs a few dozen device launches.

The optimiser restates Optim.jl's BFGS (inverse-Hessian update, identity start, g_abstol 1e-8,
``iterations`` = options.optimizer_iterations) and LineSearches.jl's ``BackTracking`` (order 3,
c1 = 1e-4, rho_hi = 0.5, rho_lo = 0.1, initial step 1, finite-value backtracking first).  Newton
for one constant uses the device gradient and a central difference of it for the curvature.
Optim's exact floating-point trajectory is not reproduced bit for bit (Julia is not available to
pin it); the objective and gradient values it consumes are the device's.
"""
from __future__ import annotations

import numpy as np

from .loss import eval_grad_batch, eval_loss_batch
from .node import TreeBatch


class _Objective:
    """Batched f / grad f over (tree, constant vector) pairs of one TreeBatch."""

    def __init__(self, tb: TreeBatch, dataset, options):
        self.tb = tb
        self.dataset = dataset
        self.options = options
        self.co = tb.constant_offsets()
        self.nc = np.diff(self.co)
        self.f_calls = np.zeros(tb.n_trees, dtype=np.int64)
        self.g_calls = np.zeros(tb.n_trees, dtype=np.int64)

    def _batch(self, idx, xs):
        sub = self.tb.subset(idx)
        consts = np.concatenate([np.asarray(x, dtype=sub.val.dtype) for x in xs]) if len(xs) else np.zeros(0)
        return sub.with_constants(consts)

    def f(self, idx, xs):
        idx = np.asarray(idx, dtype=np.int64)
        if len(idx) == 0:
            return np.zeros(0)
        loss, _ = eval_loss_batch(self._batch(idx, xs), self.dataset, self.options)
        self.f_calls[idx] += 1
        return loss.astype(np.float64)

    def fg(self, idx, xs):
        idx = np.asarray(idx, dtype=np.int64)
        if len(idx) == 0:
            return np.zeros(0), []
        sub = self._batch(idx, xs)
        loss, g, _ = eval_grad_batch(sub, self.dataset, self.options)
        co = sub.constant_offsets()
        self.f_calls[idx] += 1
        self.g_calls[idx] += 1
        return loss.astype(np.float64), [g[co[k]:co[k + 1]].astype(np.float64) for k in range(len(idx))]


def _backtracking_step(phi0, dphi0, a1, a2, phix0, phix1, iteration):
    """One LineSearches.BackTracking (order 3) interpolation: the next trial step."""
    with np.errstate(all="ignore"):
        return _backtracking_step_impl(phi0, dphi0, a1, a2, phix0, phix1, iteration)


def _backtracking_step_impl(phi0, dphi0, a1, a2, phix0, phix1, iteration):
    if iteration == 1:  # quadratic interpolation
        den = 2.0 * (phix1 - phi0 - dphi0 * a2)
        a_tmp = -(dphi0 * a2 * a2) / den if den != 0 else a2 * 0.5
    else:  # cubic interpolation
        div = 1.0 / (a1 * a1 * a2 * a2 * (a2 - a1)) if a2 != a1 else np.inf
        r1 = phix1 - phi0 - dphi0 * a2
        r0 = phix0 - phi0 - dphi0 * a1
        a = (a1 * a1 * r1 - a2 * a2 * r0) * div
        b = (-a1 ** 3 * r1 + a2 ** 3 * r0) * div
        if not np.isfinite(a) or not np.isfinite(b):
            a_tmp = a2 * 0.5
        elif abs(a) <= np.finfo(float).eps:
            a_tmp = dphi0 / (2.0 * b) if b != 0 else a2 * 0.5
        else:
            d = max(b * b - 3.0 * a * dphi0, 0.0)
            a_tmp = (-b + np.sqrt(d)) / (3.0 * a)
    if not np.isfinite(a_tmp):
        a_tmp = a2 * 0.5
    a_tmp = min(a_tmp, a2 * 0.5)   # rho_hi: avoid too small reductions
    return max(a_tmp, a2 * 0.1)    # rho_lo: avoid too big reductions


def _line_search(obj, idx, xs, fs, gs, dirs, c1=1e-4, max_iter=40):
    """Lock-step BackTracking for every member in idx; returns (alpha, f(x + alpha d))."""
    n = len(idx)
    phi0 = np.array(fs, dtype=np.float64)
    dphi0 = np.array([float(np.dot(g, d)) for g, d in zip(gs, dirs)])
    a1 = np.ones(n)
    a2 = np.ones(n)
    phix0 = phi0.copy()
    phix1 = obj.f(idx, [x + d for x, d in zip(xs, dirs)])
    it = np.zeros(n, dtype=np.int64)
    done = np.zeros(n, dtype=bool)
    for _ in range(max_iter):
        todo = []
        for k in range(n):
            if done[k]:
                continue
            if not np.isfinite(phix1[k]):  # hard-coded halving until the value is finite
                it[k] += 1
                a1[k], a2[k] = a2[k], a2[k] * 0.5
                todo.append(k)
            elif phix1[k] > phi0[k] + c1 * a2[k] * dphi0[k]:
                it[k] += 1
                new = _backtracking_step(phi0[k], dphi0[k], a1[k], a2[k], phix0[k], phix1[k], it[k])
                a1[k], a2[k] = a2[k], new
                phix0[k] = phix1[k]
                todo.append(k)
            else:
                done[k] = True
        if not todo:
            break
        vals = obj.f(idx[todo], [xs[k] + a2[k] * dirs[k] for k in todo])
        for j, k in enumerate(todo):
            phix1[k] = vals[j]
    ok = done & np.isfinite(phix1)
    return a2, phix1, ok


def _bfgs(obj, idx, x0s, iterations, g_tol=1e-8):
    """Batched BFGS (Optim.jl) from x0s; returns (minimizers, minima)."""
    idx = np.asarray(idx, dtype=np.int64)
    n = len(idx)
    xs = [np.array(x, dtype=np.float64) for x in x0s]
    fs, gs = obj.fg(idx, xs)
    fs = np.array(fs)
    invH = [np.eye(len(x)) for x in xs]
    active = np.array([np.isfinite(fs[k]) and np.max(np.abs(gs[k]), initial=0.0) > g_tol for k in range(n)])
    for _ in range(iterations):
        act = np.nonzero(active)[0]
        if len(act) == 0:
            break
        dirs = [-(invH[k] @ gs[k]) for k in act]
        alpha, fnew, ok = _line_search(obj, idx[act], [xs[k] for k in act], fs[act], [gs[k] for k in act], dirs)
        moved = [j for j in range(len(act)) if ok[j]]
        for j in range(len(act)):
            if not ok[j]:
                active[act[j]] = False  # line search failed: Optim stops
        if not moved:
            break
        ks = act[moved]
        x_new = [xs[k] + alpha[j] * dirs[j] for j, k in zip(moved, ks)]
        f_new, g_new = obj.fg(idx[ks], x_new)
        for m, k in enumerate(ks):
            dx = x_new[m] - xs[k]
            dg = g_new[m] - gs[k]
            xs[k], fs[k], gs[k] = x_new[m], f_new[m], g_new[m]
            dx_dg = float(np.dot(dx, dg))
            if not np.isfinite(fs[k]) or dx_dg == 0.0:
                active[k] = False
                continue
            u = invH[k] @ dg
            c1 = (dx_dg + float(np.dot(dg, u))) / (dx_dg * dx_dg)
            c2 = 1.0 / dx_dg
            invH[k] = invH[k] + c1 * np.outer(dx, dx) - c2 * (np.outer(u, dx) + np.outer(dx, u))
            if np.max(np.abs(gs[k]), initial=0.0) <= g_tol:
                active[k] = False
    return xs, fs


def _newton1(obj, idx, x0s, iterations, g_tol=1e-8):
    """Batched 1-D Newton with BackTracking (Optim.Newton for a single constant)."""
    idx = np.asarray(idx, dtype=np.int64)
    n = len(idx)
    xs = [np.array(x, dtype=np.float64) for x in x0s]
    fs, gs = obj.fg(idx, xs)
    fs = np.array(fs)
    active = np.array([np.isfinite(fs[k]) and abs(gs[k][0]) > g_tol for k in range(n)])
    for _ in range(iterations):
        act = np.nonzero(active)[0]
        if len(act) == 0:
            break
        h = np.array([1e-4 * max(1.0, abs(xs[k][0])) for k in act])
        _, gp = obj.fg(idx[act], [xs[k] + h[j] for j, k in enumerate(act)])
        _, gm = obj.fg(idx[act], [xs[k] - h[j] for j, k in enumerate(act)])
        dirs = []
        for j, k in enumerate(act):
            H = (gp[j][0] - gm[j][0]) / (2 * h[j])
            H = H if np.isfinite(H) and H > 1e-12 else max(abs(H), 1.0) if np.isfinite(H) else 1.0
            dirs.append(np.array([-gs[k][0] / H]))
        alpha, fnew, ok = _line_search(obj, idx[act], [xs[k] for k in act], fs[act], [gs[k] for k in act], dirs)
        moved = [j for j in range(len(act)) if ok[j]]
        for j in range(len(act)):
            if not ok[j]:
                active[act[j]] = False
        if not moved:
            break
        ks = act[moved]
        x_new = [xs[k] + alpha[j] * dirs[j] for j, k in zip(moved, ks)]
        f_new, g_new = obj.fg(idx[ks], x_new)
        for m, k in enumerate(ks):
            xs[k], fs[k], gs[k] = x_new[m], f_new[m], g_new[m]
            if not np.isfinite(fs[k]) or abs(gs[k][0]) <= g_tol:
                active[k] = False
    return xs, fs


def optimize_constants_batch(trees, dataset, options, rng=None, *, iterations=None, nrestarts=None):
    """Optimise the constants of every tree of ``trees`` (TreeBatch or Nodes) on ``dataset``.

    Returns ``(new_batch, losses, improved, num_evals)``: the batch with adopted constants, the
    loss of each tree after optimisation (unchanged when not improved), which trees improved
    (``result.minimum < baseline``), and the reference's ``num_evals`` accounting
    (f calls x dataset fraction, src/ConstantOptimization.jl:92-109).
    """
    from .loss import _as_batch

    rng = rng if rng is not None else np.random.default_rng()
    iterations = iterations if iterations is not None else getattr(options, "optimizer_iterations", 8)
    nrestarts = nrestarts if nrestarts is not None else getattr(options, "optimizer_nrestarts", 2)
    tb = _as_batch(trees, dataset.full.dtype)
    obj = _Objective(tb, dataset, options)
    nt = tb.n_trees
    consts = tb.get_constants().astype(np.float64)
    co = obj.co
    x0 = [consts[co[k]:co[k + 1]] for k in range(nt)]
    baseline = obj.f(np.arange(nt), x0)
    best_x = [x.copy() for x in x0]
    best_f = np.full(nt, np.inf)
    multi = np.nonzero(obj.nc > 1)[0]
    single = np.nonzero(obj.nc == 1)[0]
    T = dataset.full.dtype.type
    for r in range(1 + nrestarts):
        for group, algo in ((multi, _bfgs), (single, _newton1)):
            if len(group) == 0:
                continue
            if r == 0:
                starts = [x0[k] for k in group]
            else:  # xt = x0 .* (1 + eps/2), eps ~ randn(T)
                starts = [x0[k] * (1.0 + 0.5 * rng.standard_normal(len(x0[k])).astype(T)) for k in group]
            xs, fs = algo(obj, group, starts, iterations)
            for j, k in enumerate(group):
                if fs[j] < best_f[k]:
                    best_f[k], best_x[k] = fs[j], xs[j]
    improved = best_f < baseline
    new_consts = consts.copy()
    losses = baseline.copy()
    for k in np.nonzero(improved)[0]:
        new_consts[co[k]:co[k + 1]] = best_x[k]
    new_tb = tb.with_constants(new_consts)
    if improved.any():
        idx = np.nonzero(improved)[0]
        losses[idx], _ = eval_loss_batch(new_tb.subset(idx), dataset, options)
    frac = dataset.dataset_fraction()
    num_evals = (obj.f_calls + improved.astype(np.int64)) * frac
    return new_tb, losses, improved, num_evals
