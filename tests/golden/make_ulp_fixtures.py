"""Generate tests/golden/libm_ulp.json — correctly rounded reference values for the device libm.

TEST INFRASTRUCTURE (fixture generator; runs in the build container, needs mpmath).

The reference evaluates `exp`, `log` (safe_log), `cos`, `sin` and `sqrt` with Julia's Base.Math
(SURVEY.md §8(c) lists "bitwise exp/cos/log" as parity unpinned: no Julia runtime here).  Julia's
Float32/Float64 kernels are accurate to < 1 ulp; the bar the device libm is held to is therefore
the correctly rounded value itself: |device - exact| <= 1 ulp of T on every point, so the device is
never further from Julia than the two libms' own error budgets allow.

Each entry is [x, hi, lo]: x is exactly representable in T; exact = mpmath(f(x)) at 400 bits;
hi = exact rounded to the nearest float64 and lo = (exact - hi) rounded to float64, so a test can
form (device - hi) - lo without cancellation.  hi = +-inf marks a result beyond T's finite range.

Inputs: seeded random points over each function's domain plus the hard spots — exp's overflow and
underflow thresholds (Julia: 88.72284f0 / 709.782712893384), log near 1 and at subnormals, cos/sin
at the floating-point numbers nearest to multiples of pi/2 (worst cases of argument reduction) and
at huge arguments.

Run:  python tests/golden/make_ulp_fixtures.py   (deterministic; rewrites the JSON)
"""
import json
import os

import mpmath
import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libm_ulp.json")
mpmath.mp.prec = 400
FLT_MAX = float(np.finfo(np.float32).max)


def _near_multiples_pi2(dtype, rng, n, kmax):
    """Floats of `dtype` nearest to k*pi/2 (and their neighbours): the hardest reductions."""
    ks = np.unique(np.concatenate([np.arange(1, 64), rng.integers(1, kmax, n)]))
    out = []
    for k in ks:
        v = mpmath.mpf(int(k)) * mpmath.pi / 2
        f = dtype(float(v))
        for d in (-1, 0, 1):
            out.append(float(np.nextafter(f, dtype(np.inf) if d > 0 else dtype(-np.inf))) if d else float(f))
    return out


def _logu(rng, lo, hi, n):
    return np.exp(rng.uniform(np.log(lo), np.log(hi), n))


def inputs(fn, dtype, rng):
    f32 = dtype == np.float32
    n = 700
    if fn == "exp":
        top = 88.72284 if f32 else 709.782712893384
        bot = -103.0 if f32 else -745.0
        xs = np.concatenate([rng.uniform(-5, 5, n), rng.uniform(bot, top, n // 2), rng.uniform(-1e-3, 1e-3, 40)])
        edge = [top, -87.33654, -87.3365478515625, 0.0, -0.0, 1.0, -1.0, 88.0, 88.72283, 88.7228, 709.78, 709.0]
        xs = np.concatenate([xs, edge])
        xs = xs.astype(dtype)
        step = [np.nextafter(dtype(top), dtype(-np.inf)), dtype(top), np.nextafter(dtype(top), dtype(np.inf))]
        xs = np.concatenate([xs, np.array(step, dtype=dtype)])
    elif fn == "log":
        tiny = float(np.finfo(dtype).tiny)
        big = float(np.finfo(dtype).max)
        ones = [1.0 + k * float(np.finfo(dtype).eps) for k in range(-8, 9)]
        xs = np.concatenate([_logu(rng, tiny, big, n), rng.uniform(0.5, 2.0, n // 2), ones,
                             [tiny, tiny / 4, tiny / 1024, big, 1.0, 2.0, 0.5, 10.0]])
        xs = xs.astype(dtype)
        xs = xs[xs > 0]
    elif fn in ("cos", "sin"):
        big = float(np.finfo(dtype).max)
        xs = np.concatenate([rng.uniform(-10, 10, n), rng.uniform(-1e4, 1e4, n // 3),
                             _logu(rng, 1e-8, big, n // 2) * rng.choice([-1, 1], n // 2),
                             [0.0, -0.0, 1e-30, 1.5707964, 3.1415927, 1e5, 1e10, 1e20, big]])
        xs = np.concatenate([xs.astype(dtype),
                             np.array(_near_multiples_pi2(dtype, rng, 150, 1 << 22), dtype=dtype)])
    elif fn == "sqrt":
        tiny = float(np.finfo(dtype).tiny)
        xs = np.concatenate([_logu(rng, tiny / 1024, float(np.finfo(dtype).max), n),
                             np.arange(0, 64, dtype=np.float64), [2.0, 3.0, 0.25]]).astype(dtype)
    else:
        raise ValueError(fn)
    xs = xs[np.isfinite(xs)]
    return np.unique(xs)


def exact(fn, x):
    v = mpmath.mpf(float(x))
    return {"exp": mpmath.exp, "log": mpmath.log, "cos": mpmath.cos, "sin": mpmath.sin, "sqrt": mpmath.sqrt}[fn](v)


def entry(fn, x, dtype):
    e = exact(fn, x)
    limit = FLT_MAX if dtype == np.float32 else float(np.finfo(np.float64).max)
    if dtype == np.float32:
        # beyond FLT_MAX + half an ulp the result rounds to Inf
        half = mpmath.mpf(2) ** (127 - 24)
        if abs(e) >= mpmath.mpf(limit) + half:
            return [float(x), float("inf") if e > 0 else float("-inf"), 0.0]
    elif abs(e) > mpmath.mpf(limit):
        return [float(x), float("inf") if e > 0 else float("-inf"), 0.0]
    hi = float(e)
    lo = float(e - mpmath.mpf(hi))
    return [float(x), hi, lo]


def main():
    rng = np.random.default_rng(20261016)
    out = {
        "generator": "tests/golden/make_ulp_fixtures.py (mpmath %s, 400-bit)" % mpmath.__version__,
        "note": "entries [x, hi, lo]: exact f(x) = hi + lo (double-double); bar: |device - exact| <= 1 ulp of T",
    }
    for dtype, name in ((np.float32, "float32"), (np.float64, "float64")):
        out[name] = {}
        for fn in ("exp", "log", "cos", "sin", "sqrt"):
            xs = inputs(fn, dtype, rng)
            out[name][fn] = [entry(fn, x, dtype) for x in xs]
    with open(OUT, "w") as f:
        json.dump(out, f, separators=(",", ":"))
        f.write("\n")
    print(OUT, {k: {f: len(v) for f, v in out[k].items()} for k in ("float32", "float64")})


if __name__ == "__main__":
    main()
