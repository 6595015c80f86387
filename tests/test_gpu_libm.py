"""Device libm vs correctly rounded values (tests/golden/libm_ulp.json, mpmath 400-bit).

The reference evaluates exp / safe_log / cos / sin / safe_sqrt with Julia's Base.Math, whose
Float32/Float64 kernels are accurate to < 1 ulp.  No Julia runtime exists here (SURVEY.md §8(c):
bitwise libm parity is unpinned), so the device is held to the correctly rounded value itself:
<= 1 ulp of T on every fixture point (including the reduction worst cases near multiples of pi/2,
huge arguments, exp's overflow threshold and log near 1), and sqrt exactly rounded (IEEE, as Julia).
The CPU test pins the fixture: glibc's float64 libm (numpy) sits within 1 ulp of it.
"""
import json
import os

import numpy as np
import pytest

from sr_amd import Options, eval_tree_array, parse_expression

HERE = os.path.dirname(os.path.abspath(__file__))
FNS = ("exp", "log", "cos", "sin", "sqrt")


@pytest.fixture(scope="module")
def ulp_fixture():
    with open(os.path.join(HERE, "golden", "libm_ulp.json")) as f:
        return json.load(f)


def ulp_errors(dtype, xs_out, entries):
    """|device - exact| in ulps of dtype (exact = hi + lo); inf entries must match exactly."""
    e = np.array(entries, dtype=np.float64)
    hi, lo = e[:, 1], e[:, 2]
    dev = np.asarray(xs_out, dtype=np.float64)
    inf = np.isinf(hi)
    assert np.array_equal(dev[inf], hi[inf]), "overflowing results must be +-Inf"
    fin = ~inf
    ulp = np.spacing(np.abs(hi[fin]).astype(dtype)).astype(np.float64)
    # the spacing below a power of two is half the one above: use the smaller (stricter) one
    ulp = np.minimum(ulp, np.spacing(np.nextafter(np.abs(hi[fin]).astype(dtype), dtype(0))).astype(np.float64))
    ulp = np.maximum(ulp, float(np.finfo(dtype).smallest_subnormal))
    with np.errstate(invalid="ignore"):
        err = np.abs((dev[fin] - hi[fin]) - lo[fin]) / ulp
    return err


def test_fixture_pinned_by_glibc_f64(ulp_fixture):
    """CPU: glibc (numpy float64) exp/log/cos/sin/sqrt are within 1 ulp of the fixture."""
    g = ulp_fixture["float64"]
    for fn in FNS:
        e = np.array(g[fn], dtype=np.float64)
        with np.errstate(over="ignore"):
            out = getattr(np, fn)(e[:, 0])
        err = ulp_errors(np.float64, out, g[fn])
        assert np.all(err <= 1.0), (fn, float(np.max(err)))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype_name", ["float32", "float64"])
@pytest.mark.parametrize("fn", FNS)
def test_device_libm_within_one_ulp(ulp_fixture, dtype_name, fn):
    dtype = np.float32 if dtype_name == "float32" else np.float64
    opts = Options(binary_operators=["+"], unary_operators=[fn])
    tree = parse_expression(f"{fn}(x1)", opts)
    everything = ulp_fixture[dtype_name][fn]
    # DE's validity check is isfinite(sum(array)): a non-finite value, or values so large that their
    # sum overflows, make the whole tree incomplete (and its array is not returned).  Points whose
    # value could do that are evaluated one by one; overflowing ones must come back incomplete.
    big = float(np.finfo(dtype).max) / (4 * len(everything))
    small = [abs(e[1]) <= big and abs(e[0]) <= big for e in everything]  # (the input array is checked too)
    single = [e for e, ok in zip(everything, small) if not ok]
    entries = [e for e, ok in zip(everything, small) if ok]
    outs = []
    for e in single:
        o, complete = eval_tree_array(tree, np.array([[e[0]]], dtype=dtype), opts)
        assert complete is bool(np.isfinite(e[1])), (fn, e[0])
        if complete:
            entries.append(e)
            outs.append(float(o[0]))
    xs = np.array([e[0] for e in entries[:len(entries) - len(outs)]], dtype=dtype)
    out, complete = eval_tree_array(tree, xs[None, :], opts)
    assert complete, fn
    out = np.concatenate([np.asarray(out, dtype=np.float64), np.array(outs, dtype=np.float64)])
    err = ulp_errors(dtype, out, entries)
    worst = int(np.argmax(err))
    fin = entries
    print(f"{dtype_name} {fn}: n={len(entries)} max_ulp={float(err.max()):.3f} "
          f"correctly_rounded={float(np.mean(err <= 0.5)):.4f}")
    assert float(err.max()) <= (0.5 if fn == "sqrt" else 1.0), (fn, fin[worst][0], float(out[worst]), float(err.max()))


def host_unary(dtype, fn, xs):
    import ctypes

    from sr_amd import _lib

    xs = np.ascontiguousarray(xs, dtype=dtype)
    out = np.empty_like(xs)
    _lib.check(_lib.lib.sr_host_unary(_lib.SR_DTYPE_F32 if dtype == np.float32 else _lib.SR_DTYPE_F64, fn.encode(),
                                      xs.size, xs.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p)))
    return out


# Float32 bars of the library's own functions (sr_libm.h): exp is correctly rounded but for values
# within 2^-38 of a midpoint; cos / sin (256-entry (sin, cos)(k pi/128) table, degree-3/2 polynomials)
# are within 0.5223 ulp over EVERY Float32 |x| < 2^20 and log (degree-4 log1p) within 0.5101 over every
# positive normal Float32 (tools/libm_exhaustive.cpp, profiles/r03_libm_exhaustive.txt).
F32_BAR = {"exp": 0.5 + 2 ** -16, "log": 0.5101, "cos": 0.5224, "sin": 0.5224}


@pytest.mark.parametrize("fn", ["exp", "log", "cos", "sin"])
def test_host_libm_f32_within_half_ulp_plus(ulp_fixture, fn):
    """CPU: the library's Float32 exp/log/cos/sin (sr_libm.h; the device runs the same code) are
    within their bar (F32_BAR) of the exact value on every fixture point."""
    entries = ulp_fixture["float32"][fn]
    xs = np.array([e[0] for e in entries], dtype=np.float32)
    with np.errstate(all="ignore"):
        out = host_unary(np.float32, fn, xs)
    hi = np.array([e[1] for e in entries])
    fin = np.isfinite(hi)
    if fn == "exp":
        assert np.all(np.isinf(out[~fin]))
    err = ulp_errors(np.float32, out[fin], [e for e, f in zip(entries, fin) if f])
    assert float(err.max()) <= F32_BAR[fn], (fn, float(err.max()))


@pytest.mark.parametrize("fn", ["exp", "log", "cos", "sin"])
def test_host_libm_f32_random_vs_glibc(fn):
    """CPU, 400k random Float32 points per function: within F32_BAR of glibc's float64 result; exp
    equal to it rounded to Float32 except where that value sits within 2^-30 of a rounding midpoint
    (then <= 1 ulp apart)."""
    rng = np.random.default_rng(7)
    if fn == "exp":
        xs = rng.uniform(-103, 88.7, 400_000)
    elif fn == "log":
        xs = np.exp(rng.uniform(-87, 88, 400_000))
    else:
        xs = np.concatenate([rng.uniform(-20, 20, 200_000), np.exp(rng.uniform(0, 88, 200_000)) * rng.choice([-1, 1], 200_000)])
    xs = xs.astype(np.float32)
    with np.errstate(all="ignore"):
        out = host_unary(np.float32, fn, xs).astype(np.float64)
        ref64 = getattr(np, fn)(xs.astype(np.float64))
    ref = ref64.astype(np.float32).astype(np.float64)
    diff = out != ref
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    # glibc double results are within 1 double ulp: a Float32 rounding of it can only differ from the
    # correctly rounded value when the exact value is that close to a midpoint
    mid = np.abs(np.abs(ref64 - ref) - ulp / 2) <= np.abs(ref64) * 2.0 ** -30
    assert np.all(np.abs(out - ref)[diff] <= ulp[diff]), fn
    # error in ulps of the result's binade (the smaller spacing at a power of two)
    u = np.minimum(ulp, np.spacing(np.nextafter(np.abs(ref).astype(np.float32), np.float32(0))).astype(np.float64))
    fin = np.isfinite(ref64) & (u > 0)
    assert float(np.max(np.abs(out - ref64)[fin] / u[fin])) <= F32_BAR[fn] + 2 ** -20, fn
    if fn == "exp":
        assert np.all(mid[diff]), (fn, int(diff.sum()), xs[diff & ~mid][:5])
