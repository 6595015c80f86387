"""CPU: host-side mirror of the reference API (no device calls)."""
import numpy as np
import pytest

import sr_amd
from sr_amd import (Dataset, Node, Options, batch, extend_operators, flatten_trees, gen_random_tree_fixed_size,
                    get_scalar_constants, loss_to_cost, parse_expression, set_scalar_constants, string_tree)
from sr_amd.mutation import _arity_picker


def test_op_map_matches_reference():
    # src/Options.jl:182-202 OP_MAP: log -> safe_log, ^ -> safe_pow, sqrt -> safe_sqrt, / stays /
    o = Options(binary_operators=["+", "-", "*", "/", "^"], unary_operators=["log", "sqrt", "cos", "acosh"])
    assert o.operators.binops == ("+", "-", "*", "/", "safe_pow")
    assert o.operators.unaops == ("safe_log", "safe_sqrt", "cos", "safe_acosh")
    assert o.operators.nops == (4, 5)
    assert isinstance(o.parsimony, np.float32)


def test_unsupported_operator_raises():
    with pytest.raises(ValueError):
        Options(binary_operators=["+"], unary_operators=["my_custom_op"])
    with pytest.raises(ValueError):
        Options(elementwise_loss="CrossEntropyLoss()")  # not in the device catalog
    with pytest.raises(ValueError):
        Options(elementwise_loss="QuantileLoss")  # needs its parameter


def test_loss_catalog_parsing():
    """The LossFunctions catalog of src/Options.jl:301-328, as the device's (kind, parameter)."""
    cases = {"L2DistLoss()": (0, 0.0), "L1DistLoss": (1, 0.0), "LPDistLoss{3}()": (2, 3.0), "LPDistLoss(1.5)": (2, 1.5),
             "LogitDistLoss()": (3, 0.0), "HuberLoss()": (4, 1.0), "HuberLoss(2.5)": (4, 2.5),
             "L1EpsilonInsLoss(0.1)": (5, 0.1), "L2EpsilonInsLoss(0.2)": (6, 0.2), "PeriodicLoss(6.0)": (7, 6.0),
             "QuantileLoss(0.3)": (8, 0.3), "ZeroOneLoss()": (9, 0.0), "PerceptronLoss()": (10, 0.0),
             "L1HingeLoss()": (11, 0.0), "L2HingeLoss()": (12, 0.0), "SmoothedL1HingeLoss(0.5)": (13, 0.5),
             "ModifiedHuberLoss()": (14, 0.0), "L2MarginLoss()": (15, 0.0), "ExpLoss()": (16, 0.0),
             "SigmoidLoss()": (17, 0.0), "DWDMarginLoss(2)": (18, 2.0)}
    for spec, want in cases.items():
        o = Options(elementwise_loss=spec)
        assert (o.loss_kind, o.loss_param) == want, spec


def test_parse_print_roundtrip_and_preorder():
    o = Options(binary_operators=["+", "*", "/", "-"], unary_operators=["cos", "exp", "log"])
    t = parse_expression("cos(x1 * 3.0) + exp(x2) / 2.5", o)
    assert t.count_nodes() == 9
    assert string_tree(t, o.operators) == "(cos((x1 * 3.0)) + (exp(x2) / 2.5))"
    tb = flatten_trees([t, parse_expression("x3", o)])
    assert tb.n_trees == 2
    assert list(tb.degree[:9]) == [2, 1, 2, 0, 0, 2, 1, 0, 0]
    assert list(tb.constant[:9]) == [0, 0, 0, 0, 1, 0, 0, 0, 1]
    back = tb.tree(0)
    assert string_tree(back, o.operators) == string_tree(t, o.operators)
    assert list(get_scalar_constants(t)) == [3.0, 2.5]  # pre-order (get_scalar_constants)
    set_scalar_constants(t, [1.0, 2.0])
    assert list(get_scalar_constants(t)) == [1.0, 2.0]


def test_node_arithmetic_with_extend_operators():
    o = Options(binary_operators=["+", "*", "-", "/"], unary_operators=["cos"])
    extend_operators(o)
    x1, x2 = Node("x1"), Node("x2")
    t = sr_amd.apply_unary("cos", x1 * 2.0) - x2 / 3.0
    assert string_tree(t, o.operators) == "(cos((x1 * 2.0)) - (x2 / 3.0))"


@pytest.mark.parametrize("size", [1, 2, 5, 17, 30])
def test_gen_random_tree_fixed_size(size):
    # src/MutationFunctions.jl:441-471: exactly node_count nodes when both arities exist
    o = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])
    rng = np.random.default_rng(size)
    for _ in range(50):
        t = gen_random_tree_fixed_size(size, o, 5, np.float32, rng)
        assert t.count_nodes() == size
        for n in t.preorder():
            if n.degree == 0 and not n.constant:
                assert 1 <= n.feature <= 5


def test_arity_picker_distribution():
    rng = np.random.default_rng(0)
    picks = [_arity_picker(rng, 10, (3, 4)) for _ in range(20000)]
    frac_unary = picks.count(1) / len(picks)
    assert abs(frac_unary - 3 / 7) < 0.02
    assert all(_arity_picker(rng, 1, (3, 4)) == 1 for _ in range(100))
    assert _arity_picker(rng, 1, (0, 4)) == 0


def test_loss_to_cost():
    o = Options(parsimony=0.5)
    t = parse_expression("x1 + 1.0", o)
    f = np.float32
    # normalization floor 0.01 (src/LossFunctions.jl:179-183)
    assert loss_to_cost(f(2.0), True, f(0.001), t, o) == f(2.0) / f(0.01) + f(3 * 0.5)
    assert loss_to_cost(f(2.0), True, f(4.0), t, o) == f(0.5) + f(1.5)
    assert loss_to_cost(f(2.0), False, f(4.0), t, o, complexity=10) == f(200.0) + f(5.0)


def test_dataset_layout_and_batch():
    X = np.arange(12, dtype=np.float32).reshape(3, 4)
    y = np.arange(4, dtype=np.float32)
    d = Dataset(X, y, weights=np.ones(4, dtype=np.float32))
    assert (d.nfeatures, d.n) == (3, 4)
    sub = batch(d, [0, 2, 2])
    assert sub.n == 3
    assert sub.X.shape == (3, 3)
    assert list(sub.y) == [0.0, 2.0, 2.0]
    assert sub.dataset_fraction() == pytest.approx(0.75)
    assert sub.baseline_loss == d.baseline_loss
    s2 = batch(d, 16, np.random.default_rng(0))
    assert s2.n == 16 and s2.indices.max() < 4
    with pytest.raises(TypeError):
        Dataset(X, y.astype(np.float64))
