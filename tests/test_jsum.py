"""The exact validity check in Julia's summation order (CPU: host half of the C ABI).

DynamicExpressions decides a checked array with isfinite(sum(x)); Base's `sum` over an Array is
Base.mapreduce_impl (halves split at lo + (hi - lo) >> 1 down to blocks of < 1024 elements, each
folded sequentially in T) — restated below in numpy float32 as the test's own reference, pinned to
the oracle (whose root check is the same predicate).  The library's side: `sr_jsum_ranges` (the
row ranges a shard folds) and `sr_jsum_finite` (adds the folds of every shard in recursion order).
The cases are the ones where an exact (f64) sum and the T-precision Julia sum disagree: mixed-sign
values whose partial sums overflow, totals within half an ulp of FLT_MAX, Inf/NaN mixes.
"""
import numpy as np
import pytest

from oracle import Oracle
from sr_amd import Options, flatten_trees, parse_expression
from sr_amd.distributed import jsum_finite, jsum_ranges

F32 = np.float32
FMAX = float(np.finfo(np.float32).max)


def jl_sum(a, lo=0, hi=None):
    """Base.mapreduce_impl(+, a, lo, hi) in T (the test's restatement)."""
    hi = len(a) - 1 if hi is None else hi
    if hi - lo < 1024:
        v = a[lo]
        with np.errstate(over="ignore", invalid="ignore"):
            for i in range(lo + 1, hi + 1):
                v = v + a[i]
        return v
    mid = lo + ((hi - lo) >> 1)
    with np.errstate(over="ignore", invalid="ignore"):
        return jl_sum(a, lo, mid) + jl_sum(a, mid + 1, hi)


def shard_folds(a, offs):
    """Every shard's range folds of `a` (what sr_jsum_partials computes on the GPU)."""
    out = []
    for r in range(len(offs) - 1):
        lo, hi, _, _ = jsum_ranges(offs[r], offs[r + 1] - offs[r], len(a))
        loc = a[offs[r]:offs[r + 1]]
        out.append(np.array([[jl_sum(loc, int(l), int(h)) for l, h in zip(lo, hi)]], dtype=a.dtype))
    return out


def cases():
    rng = np.random.default_rng(3)
    big = np.full(5000, 2e35, dtype=F32)
    big[2500:] = -2e35  # the first half's leaf folds overflow; the exact total is 0
    alt = np.tile(np.array([3e38, 3e38, -3e38, -3e38], dtype=F32), 600)
    near = np.zeros(3000, dtype=F32)
    near[0] = FMAX
    near[1700] = F32(2.0 ** 103)  # FLT_MAX + half an ulp: rounds to Inf (ties to even)
    under = near.copy()
    under[1700] = F32(2.0 ** 102)  # rounds back to FLT_MAX: finite
    return {
        "mixed_overflow_small": np.array([3e38, 3e38, -3e38, -3e38], dtype=F32),
        "mixed_overflow_pairwise": big,
        "alternating": alt,
        "fmax_plus_half_ulp": near,
        "fmax_plus_quarter_ulp": under,
        "inf_nan": np.array([1.0, np.inf, np.nan, -np.inf], dtype=F32),
        "inf_minus_inf": np.concatenate([np.full(1500, 1.0, F32), [np.inf], np.full(1500, 1.0, F32), [-np.inf]]),
        "random_large": (rng.standard_normal(70_000) * 1e33).astype(F32),
        "one": np.array([FMAX], dtype=F32),
        "fifteen": np.full(15, FMAX / 16, dtype=F32),
    }


@pytest.mark.parametrize("name", list(cases()))
def test_julia_sum_restatement_matches_oracle(name):
    """The numpy restatement's verdict == the oracle's root check on the tree `x1`."""
    a = cases()[name]
    opts = Options(binary_operators=["+"], unary_operators=[])
    _, complete = Oracle.from_options(opts).eval_tree_array(flatten_trees([parse_expression("x1", opts)], F32), 0,
                                                           a[None, :])
    assert bool(complete) == bool(np.isfinite(jl_sum(a))), name


@pytest.mark.parametrize("name", list(cases()))
@pytest.mark.parametrize("split", [None, 2, 3, "tiny"])
def test_jsum_finite_over_shards(name, split):
    """Folds of 1, 2 or 3 row shards (boundaries inside leaf blocks included) combine to Julia's
    verdict, identical whatever the sharding."""
    a = cases()[name]
    n = len(a)
    if split is None:
        offs = [0, n]
    elif split == "tiny":  # shards shorter than a leaf block: blocks span several shards
        if n < 40:
            pytest.skip("too short")
        offs = [0, 7, 19, n]
    else:
        if n < 1000:
            pytest.skip("too short")
        offs = [n * k // split for k in range(split + 1)]
        offs[1] = max(1, offs[1] - 333)  # not on a block boundary
    fin = jsum_finite(np.float32, n, offs, shard_folds(a, offs))
    assert bool(fin[0]) == bool(np.isfinite(jl_sum(a))), (name, split)


def test_expected_verdicts():
    """Where the exact f64 sum says 'finite' but T-precision Julia overflows (and vice versa)."""
    c = cases()
    verdict = {k: bool(np.isfinite(jl_sum(v))) for k, v in c.items()}
    assert np.isfinite(np.sum(c["mixed_overflow_small"].astype(np.float64)))
    assert verdict["mixed_overflow_small"] is False
    assert verdict["mixed_overflow_pairwise"] is False
    assert verdict["alternating"] is False
    assert verdict["fmax_plus_half_ulp"] is False
    assert verdict["fmax_plus_quarter_ulp"] is True
    assert verdict["inf_nan"] is False and verdict["inf_minus_inf"] is False
    assert verdict["one"] is True and verdict["fifteen"] is True


def test_ranges_cover_every_row_once():
    for n_total, offs in ((5000, [0, 1234, 5000]), (70_000, [0, 9000, 30_001, 70_000]), (3, [0, 1, 3])):
        seen = np.zeros(n_total, dtype=int)
        for r in range(len(offs) - 1):
            lo, hi, leaf, head = jsum_ranges(offs[r], offs[r + 1] - offs[r], n_total)
            for l, h in zip(lo, hi):
                seen[offs[r] + l: offs[r] + h + 1] += 1
            assert np.all(np.diff(leaf) >= 0)
            assert np.all(hi[head] == lo[head])
        assert np.all(seen == 1)
