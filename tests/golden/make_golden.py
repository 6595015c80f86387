"""Generate tests/golden/reference_known_answers.json — the reference's own known answers for the
scoring path, re-expressed with explicit data.

The reference's tests draw their data from Julia's MersenneTwister, which cannot be reproduced
here (no Julia runtime); every case below keeps the reference's tree, operators, element type,
expected outcome and tolerance, with the input data drawn from numpy (seeded) and stored in the
fixture.  Expected values are the reference's closed forms evaluated in float64 by numpy/math.

Sources (all under /root/reference, read as text):
  test/unit/evaluation/test_evaluation.jl:1-76            fused-kernel shapes vs closed form
  test/integration/ext/loopvectorization/test_nan_detection.jl:1-55   non-finite flags
  test/unit/dataset/test_batched_dataset.jl:90-130         exact MSE on a 1x3 dataset / batches
  test/unit/misc/test_losses.jl:1-34                       L1 mean / weighted mean
  test/integration/ext/loopvectorization/test_operators.jl:1-77   safe-operator domains
  test/integration/ad/forwarddiff/test_tree_construction.jl:23-122  loss ~ 0, cost relations

Run:  python tests/golden/make_golden.py   (deterministic; rewrites the JSON)
"""
import json
import math
import os

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_known_answers.json")


def f32list(a):
    return [float(np.float32(v)) for v in np.asarray(a).ravel()]


def flist(a):
    return [float(v) for v in np.asarray(a).ravel()]


def fused_shapes():
    rng = np.random.default_rng(0)
    X = rng.standard_normal((3, 100)).astype(np.float32)
    x1, x2, x3 = (X[i].astype(np.float64) for i in range(3))
    c = np.cos
    s = np.sin
    cases = [
        # deg2_l0_r0_eval
        ("x1 * x2", x1 * x2),
        ("x1 * 3.0", x1 * 3.0),
        ("3.0 * x2", 3.0 * x2),
        ("3.0 * 6.0", np.full(100, 18.0)),
        # deg2_l0_eval
        ("x1 * sin(x2)", x1 * s(x2)),
        ("3.0 * sin(x2)", 3.0 * s(x2)),
        # deg2_r0_eval
        ("sin(x1) * x2", s(x1) * x2),
        ("sin(x1) * 3.0", s(x1) * 3.0),
        # deg1_l2_ll0_lr0_eval
        ("cos(x1 * x2)", c(x1 * x2)),
        ("cos(x1 * 3.0)", c(x1 * 3.0)),
        ("cos(3.0 * x2)", c(3.0 * x2)),
        ("cos(3.0 * -0.5)", np.full(100, math.cos(-1.5))),
        # deg1_l1_ll0_eval
        ("cos(sin(x1))", c(s(x1))),
        ("cos(sin(3.0))", np.full(100, math.cos(math.sin(3.0)))),
        # everything else
        ("(sin(cos(sin(cos(x1) * x3) * 3.0) * -0.5) + 2.0) * 5.0",
         (s(c(s(c(x1) * x3) * 3.0) * -0.5) + 2.0) * 5.0),
    ]
    return {
        "source": "test/unit/evaluation/test_evaluation.jl:1-76",
        "binary_operators": ["+", "*", "/", "-"],
        "unary_operators": ["cos", "sin"],
        "dtype": "float32",
        "X": [f32list(X[i]) for i in range(3)],
        "tolerance_abs_over_N": 1e-6,
        "cases": [{"expr": e, "expected": flist(v)} for e, v in cases],
    }


def nan_detection():
    cases = []
    for dtype in ("float32", "float64"):
        cases += [
            {"dtype": dtype, "expr": "exp(exp(exp(exp(x1 + 1.0))))", "X": [[100.0] * 10]},
            {"dtype": dtype, "expr": "cos(x1 / 0.0)", "X": [[100.0] * 10]},
            {"dtype": dtype, "expr": "sqrt(x1 - 1.0)", "X": [[0.0] * 10]},
            {"dtype": dtype, "expr": "(x1 - 1.0) ^ 0.5", "X": [[0.0] * 10]},
            {"dtype": dtype, "expr": "cos(x1 + inf)", "X": [[0.0] * 10]},
            {"dtype": dtype, "expr": "cos(x1 + nan)", "X": [[0.0] * 10]},
        ]
    return {
        "source": "test/integration/ext/loopvectorization/test_nan_detection.jl:6-52",
        "binary_operators": ["+", "*", "/", "-", "^"],
        "unary_operators": ["cos", "sin", "exp", "sqrt"],
        "expected_complete": False,
        "cases": cases,
    }


def batched_mse():
    return {
        "source": "test/unit/dataset/test_batched_dataset.jl:90-130",
        "binary_operators": ["+", "*", "-", "/"],
        "unary_operators": [],
        "dtype": "float64",
        "X": [[1.0, 2.0, 3.0]],
        "y": [2.0, 6.0, 12.0],
        "expr": "x1 * 1.0",
        "cases": [
            {"indices": None, "loss": (1.0 ** 2 + 4.0 ** 2 + 9.0 ** 2) / 3},
            {"indices": [0], "loss": 1.0},
            {"indices": [1], "loss": 16.0},
            {"indices": [2], "loss": 81.0},
            {"indices": [0, 2], "loss": (1.0 + 81.0) / 2},
        ],
    }


def losses():
    rng = np.random.default_rng(0)
    x = rng.standard_normal(100).astype(np.float32)
    y = np.random.default_rng(1).standard_normal(100).astype(np.float32)
    w = np.abs(np.random.default_rng(2).standard_normal(100)).astype(np.float32)
    d = np.abs(x.astype(np.float64) - y.astype(np.float64))
    return {
        "source": "test/unit/misc/test_losses.jl:15-33",
        "dtype": "float32",
        "x": f32list(x), "y": f32list(y), "w": f32list(w),
        "L1DistLoss": {"mean": float(d.sum() / 100), "weighted": float((d * w).sum() / w.astype(np.float64).sum())},
        "L2DistLoss": {"mean": float((d * d).sum() / 100), "weighted": float((d * d * w).sum() / w.astype(np.float64).sum())},
        "tolerance": 1e-6,
    }


def safe_operators():
    val, val2 = 0.5, 3.2
    nan = "nan"
    unary = [
        ("log", val, math.log(val)), ("log", -val, nan), ("log2", val, math.log2(val)), ("log2", -val, nan),
        ("log10", val, math.log10(val)), ("log10", -val, nan), ("log1p", val, math.log1p(val)),
        ("acosh", val2, math.acosh(val2)), ("acosh", -val2, nan), ("asin", val, math.asin(val)),
        ("asin", val2, nan), ("acos", val, math.acos(val)), ("acos", val2, nan), ("atanh", val, math.atanh(val)),
        ("atanh", val2, nan), ("neg", -val, val), ("sqrt", val, math.sqrt(val)), ("sqrt", -val, nan),
        ("square", val, val * val), ("cube", val, val * val * val), ("log", 0.0, nan), ("log2", 0.0, nan),
        ("log10", 0.0, nan), ("log1p", -2.0, nan), ("relu", -val, 0.0), ("relu", val, val),
    ]
    binary = [
        ("*", val, val2, val * val2), ("+", val, val2, val + val2), ("-", val, val2, val - val2),
        ("^", 0.0, -1.0, nan), ("^", -val, val2, nan), ("^", -val, -val2, nan), ("^", 0.0, -val2, nan),
        ("^", val, val2, val ** val2), ("^", val, -val2, val ** (-val2)), ("^", -1.0, 2.0, 1.0),
        ("^", -1.0, 2.1, nan), ("greater", val, val2, 0.0), ("greater", val2, val, 1.0),
        ("logical_or", val, val2, 1.0), ("logical_or", 0.0, val2, 1.0), ("logical_and", 0.0, val2, 0.0),
        ("cond", val, val2, val2), ("cond", -val, val2, 0.0),
    ]
    return {
        "source": "test/integration/ext/loopvectorization/test_operators.jl:26-76",
        "tolerance": 1e-6,
        "unary": [{"op": o, "x": x, "expected": e} for o, x, e in unary],
        "binary": [{"op": o, "x": x, "y": y, "expected": e} for o, x, y, e in binary],
    }


def tree_construction():
    def gamma(x):
        return np.vectorize(math.gamma)(x)

    unaops = {
        "cos": np.cos, "exp": np.exp, "log": np.log, "log2": np.log2, "log10": np.log10, "sqrt": np.sqrt,
        "relu": lambda x: np.where(x > 0, x, 0.0), "gamma": gamma, "acosh": np.arccosh,
    }
    cases = []
    for k, (name, f) in enumerate(unaops.items()):
        for dtype in ("float32", "float64"):
            rng = np.random.default_rng(100 + k)
            if name in ("log", "log2", "log10", "acosh", "sqrt"):
                X = rng.random((5, 100)) / 3
            else:
                X = rng.standard_normal((5, 100)) / 3
            X = X.astype(dtype)
            X = X + np.sign(X) * np.asarray(0.1, dtype=dtype)
            if name == "acosh":
                X = X + np.asarray(1.0, dtype=dtype)
            X = X.astype(dtype)
            x1 = X[0].astype(np.float64)
            y = (np.abs(3.0 * f(x1)) ** 2.0) - (-1.2)
            cases.append({
                "unaop": name, "dtype": dtype, "X": [flist(r) for r in X], "y": flist(np.asarray(y, dtype=dtype)),
                "tolerance": 3e-2 if name == "gamma" else 1e-6,
            })
    return {
        "source": "test/integration/ad/forwarddiff/test_tree_construction.jl:23-122",
        "binary_operators": ["+", "*", "^", "/", "-"],
        "unary_operators_template": ["UNAOP", "abs"],
        "good_expr": "(abs(3.0 * UNAOP(x1)) ^ 2.0) - -1.2",
        "bad_expr": "(abs(3.0 * UNAOP(x1)) ^ 2.1) - -1.3",
        "count_nodes": 9,
        "parsimony_default": 0.0001,
        "cases": cases,
    }


def main():
    doc = {
        "generator": "tests/golden/make_golden.py",
        "note": "reference known answers re-expressed with explicit numpy data (Julia RNG streams are not reproducible here)",
        "fused_shapes": fused_shapes(),
        "nan_detection": nan_detection(),
        "batched_mse": batched_mse(),
        "losses": losses(),
        "safe_operators": safe_operators(),
        "tree_construction": tree_construction(),
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1, allow_nan=False)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes)")


if __name__ == "__main__":
    main()
