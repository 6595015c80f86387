"""CPU: pin the oracle (oracle/de_eval.c) against the reference's own known answers.

Every fixture in tests/golden/reference_known_answers.json comes from a reference test file (cited
in the fixture's "source"); see tests/golden/make_golden.py.  If the oracle passes these, it is the
checker the GPU parity tests (`-m gpu`) compare libsr_amd against.
"""
import math

import numpy as np
import pytest

from oracle import Oracle
from sr_amd import Options, flatten_trees, loss_to_cost, parse_expression


def _dt(name):
    return np.float32 if name == "float32" else np.float64


def test_fused_shapes(golden):
    g = golden["fused_shapes"]
    opts = Options(binary_operators=g["binary_operators"], unary_operators=g["unary_operators"])
    orc = Oracle.from_options(opts)
    X = np.array(g["X"], dtype=np.float32)
    N = X.shape[1]
    for case in g["cases"]:
        tb = flatten_trees([parse_expression(case["expr"], opts)], dtype=np.float32)
        out, complete = orc.eval_tree_array(tb, 0, X)
        assert complete, case["expr"]
        err = np.abs(out.astype(np.float64) - np.array(case["expected"])) / N
        assert np.all(err < g["tolerance_abs_over_N"]), (case["expr"], err.max())


def test_nan_detection_flags(golden):
    g = golden["nan_detection"]
    opts = Options(binary_operators=g["binary_operators"], unary_operators=g["unary_operators"])
    orc = Oracle.from_options(opts)
    for case in g["cases"]:
        dt = _dt(case["dtype"])
        tb = flatten_trees([parse_expression(case["expr"], opts)], dtype=dt)
        _, complete = orc.eval_tree_array(tb, 0, np.array(case["X"], dtype=dt))
        assert complete == g["expected_complete"], case


def test_batched_dataset_mse(golden):
    g = golden["batched_mse"]
    opts = Options(binary_operators=g["binary_operators"], unary_operators=g["unary_operators"])
    orc = Oracle.from_options(opts)
    X = np.array(g["X"], dtype=np.float64)
    y = np.array(g["y"], dtype=np.float64)
    tb = flatten_trees([parse_expression(g["expr"], opts)], dtype=np.float64)
    for case in g["cases"]:
        idx = case["indices"]
        Xv = X if idx is None else X[:, idx]
        yv = y if idx is None else y[idx]
        loss, comp = orc.eval_loss_batch(tb, Xv, yv)
        assert comp[0]
        assert loss[0] == pytest.approx(case["loss"], rel=1e-12)


@pytest.mark.parametrize("kind,name", [(1, "L1DistLoss"), (0, "L2DistLoss")])
def test_losses_mean_and_weighted(golden, kind, name):
    g = golden["losses"]
    opts = Options(binary_operators=["+"], unary_operators=[])
    orc = Oracle.from_options(opts)
    x = np.array(g["x"], dtype=np.float32)
    y = np.array(g["y"], dtype=np.float32)
    w = np.array(g["w"], dtype=np.float32)
    tb = flatten_trees([parse_expression("x1", opts)], dtype=np.float32)
    for accum in ("ref", "f64"):
        loss, _ = orc.eval_loss_batch(tb, x[None, :], y, loss_kind=kind, accum=accum)
        assert abs(float(loss[0]) - g[name]["mean"]) < g["tolerance"]
        lw, _ = orc.eval_loss_batch(tb, x[None, :], y, w=w, loss_kind=kind, accum=accum)
        assert abs(float(lw[0]) - g[name]["weighted"]) < g["tolerance"]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_safe_operators(golden, dtype):
    g = golden["safe_operators"]
    for case in g["unary"]:
        opts = Options(binary_operators=["+"], unary_operators=[case["op"]])
        orc = Oracle.from_options(opts)
        tb = flatten_trees([parse_expression(f"{case['op']}(x1)", opts)], dtype=dtype)
        out, _ = orc.eval_tree_array(tb, 0, np.array([[case["x"]]], dtype=dtype))
        if case["expected"] == "nan":
            assert math.isnan(out[0]), case
        else:
            assert abs(float(out[0]) - case["expected"]) < g["tolerance"], case
    for case in g["binary"]:
        opts = Options(binary_operators=[case["op"]], unary_operators=[])
        orc = Oracle.from_options(opts)
        op = case["op"]
        from sr_amd import Node

        tree = Node(op=1, l=Node(feature=1), r=Node(feature=2))
        tb = flatten_trees([tree], dtype=dtype)
        out, _ = orc.eval_tree_array(tb, 0, np.array([[case["x"]], [case["y"]]], dtype=dtype))
        if case["expected"] == "nan":
            assert math.isnan(out[0]), (op, case)
        else:
            assert abs(float(out[0]) - case["expected"]) < g["tolerance"], (op, case)


def test_tree_construction_loss_and_cost(golden):
    g = golden["tree_construction"]
    for case in g["cases"]:
        dt = _dt(case["dtype"])
        una = case["unaop"]
        opts = Options(binary_operators=g["binary_operators"], unary_operators=[una, "abs"],
                       parsimony=g["parsimony_default"])
        orc = Oracle.from_options(opts)
        good = parse_expression(g["good_expr"].replace("UNAOP", una), opts)
        bad = parse_expression(g["bad_expr"].replace("UNAOP", una), opts)
        assert good.count_nodes() == g["count_nodes"]
        X = np.array(case["X"], dtype=dt)
        y = np.array(case["y"], dtype=dt)
        tb = flatten_trees([good, bad], dtype=dt)
        loss, comp = orc.eval_loss_batch(tb, X, y)
        assert comp[0], case["unaop"]
        assert abs(float(loss[0])) < case["tolerance"], (una, case["dtype"], float(loss[0]))
        # cost relations (src/LossFunctions.jl:170-190): baseline 1 (fresh Dataset)
        one = dt(1)
        c0 = loss_to_cost(loss[0], True, one, good, Options(g["binary_operators"], [una, "abs"], parsimony=0.0))
        c1 = loss_to_cost(loss[0], True, one, good, Options(g["binary_operators"], [una, "abs"], parsimony=1.0))
        assert abs(float(c0)) < case["tolerance"]
        assert float(c1) > 1.0
        cg = loss_to_cost(loss[0], True, one, good, opts)
        cb = loss_to_cost(loss[1], True, one, bad, opts)
        assert float(cg) < float(cb)
        cb10 = loss_to_cost(loss[1], True, dt(10), bad, opts)
        assert float(cb10) < float(cb)


def test_loss_catalog_known_answers():
    """The oracle's LossFunctions restatement at hand-computed points (d = output - target,
    a = target * output).  Constant trees over a dataset with y = target."""
    import math

    from oracle import Oracle
    from sr_amd import Node, Options, flatten_trees

    pts = [(0.5, 0.0), (3.0, 0.0), (-2.0, 0.0), (0.25, 1.0), (-0.5, 1.0), (2.0, -1.0)]  # (output, target)
    k = 2 * math.pi / 6.0

    def hinge(x):
        return max(0.0, x)

    spec = {  # elementwise_loss -> f(output, target)
        "L2DistLoss()": lambda o, t: (o - t) ** 2,
        "L1DistLoss()": lambda o, t: abs(o - t),
        "LPDistLoss{3}()": lambda o, t: abs(o - t) ** 3,
        "LogitDistLoss()": lambda o, t: -math.log(4 * math.exp(o - t) / (1 + math.exp(o - t)) ** 2),
        "HuberLoss(1.0)": lambda o, t: 0.5 * (o - t) ** 2 if abs(o - t) <= 1 else abs(o - t) - 0.5,
        "L1EpsilonInsLoss(0.3)": lambda o, t: hinge(abs(o - t) - 0.3),
        "L2EpsilonInsLoss(0.3)": lambda o, t: hinge(abs(o - t) - 0.3) ** 2,
        "PeriodicLoss(6.0)": lambda o, t: 1 - math.cos((o - t) * k),
        "QuantileLoss(0.3)": lambda o, t: (o - t) * ((1.0 if o - t > 0 else 0.0) - 0.3),
        "ZeroOneLoss()": lambda o, t: 1.0 if t * o < 0 else 0.0,
        "PerceptronLoss()": lambda o, t: hinge(-t * o),
        "L1HingeLoss()": lambda o, t: hinge(1 - t * o),
        "L2HingeLoss()": lambda o, t: hinge(1 - t * o) ** 2,
        "SmoothedL1HingeLoss(0.5)": lambda o, t: (hinge(1 - t * o) ** 2 / 1.0 if t * o >= 0.5 else 0.75 - t * o),
        "ModifiedHuberLoss()": lambda o, t: hinge(1 - t * o) ** 2 if t * o >= -1 else -4 * t * o,
        "L2MarginLoss()": lambda o, t: (1 - t * o) ** 2,
        "ExpLoss()": lambda o, t: math.exp(-t * o),
        "SigmoidLoss()": lambda o, t: 1 - math.tanh(t * o),
        "DWDMarginLoss(2)": lambda o, t: 1 - t * o if t * o <= 2 / 3 else (4 / 27) / (t * o) ** 2,
    }
    X = np.zeros((1, 4))
    for name, f in spec.items():
        opts = Options(binary_operators=["+"], elementwise_loss=name)
        orc = Oracle.from_options(opts)
        for o, t in pts:
            tb = flatten_trees([Node(val=np.float64(o))], np.float64)
            loss, comp = orc.eval_loss_batch(tb, X, np.full(4, t), loss_kind=opts.loss_kind,
                                             loss_param=opts.loss_param)
            assert comp[0]
            assert loss[0] == pytest.approx(f(o, t), rel=1e-12, abs=1e-15), (name, o, t)
