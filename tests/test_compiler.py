"""CPU: the tree compiler (csrc/sr_compile.cpp, via the host-only sr_compile_info entry point).

The compiled programs are executed by tests/bytecode_vm.py (numpy restatement of the kernel's
instruction semantics) and compared with the oracle: this pins constant folding, DE check placement,
fused-unary detection and Sethi–Ullman ordering without a GPU.
"""
import numpy as np
import pytest

import bytecode_vm as vm
from parity_util import assert_losses_within, loss_tolerance
from oracle import Oracle
from sr_amd import Options, flatten_trees, gen_random_population, parse_expression

OPTS = dict(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp", "log"])


def _data(n, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((5, n)).astype(np.float32)
    y = (2 * np.cos(X[3]) + X[0] ** 2 - 2).astype(np.float32)
    return X, y


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_compiled_programs_match_oracle(seed):
    opts = Options(**OPTS)
    X, y = _data(257, seed)
    tb = flatten_trees(gen_random_population(1500, opts, 5, seed=seed), np.float32)
    loss, comp = vm.eval_loss_batch(opts, tb, X, y)
    tol, ol, oc, n_wide = loss_tolerance(Oracle.from_options(opts), tb, X, y)
    mism = np.nonzero(comp != oc)[0]
    assert len(mism) == 0, mism[:10]
    assert n_wide < 0.15 * oc.sum()  # most complete trees are well-conditioned
    assert_losses_within(loss, ol, comp, tol)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_post_binary_constant_fusion(dtype):
    """A binary node with a constant operand rides on the instruction computing its other operand (the
    PBC field, csrc/sr_ops.h): one instruction fewer, every variant (+, - and / on both sides, *), the
    fused node's own array check (PBC_CHECK) and a folded constant operand's static check."""
    opts = Options(binary_operators=["+", "-", "*", "/"], unary_operators=["cos", "exp"])
    cases = {  # expression: (instructions, PBC variant of the last instruction)
        "(x1 + x2) * 3.0": (2, 0),                         # PAIR computes tos: no free constant word
        "cos(x1 + x2) * 3.0": (2, 0),                      # PAIR + POST cos: the constant stays separate
        "(x1 + cos(x2)) + 3.0": (2, 1),                    # LOAD+cos, FR add, then PBC +c
        "(x1 + cos(x2)) - 3.0": (2, 2),
        "3.0 - (x1 + cos(x2))": (2, 3),
        "(x1 + cos(x2)) * 3.0": (2, 4),
        "(x1 + cos(x2)) / 3.0": (2, 5),
        "3.0 / (x1 + cos(x2))": (2, 6),
        "cos(x1) * 1.0e30": (1, 4),                        # LOAD + POST cos + PBC
        "(x1 * cos(x2)) * (1.0e30 * 1.0e3)": (2, 4),      # folded operand: checked statically,
        "(x1 * cos(x2)) * (BIG * 1.0e8)": (0, 0),         # ... its 4000-row sum overflows: static_bad
        "(x1 + x2) * (BIG * 1.0e8)": (0, 0),              # (the unfused operand form checks it too)
        "exp(x1 * cos(x2)) - 1.0e38": (2, 2),
    }
    big = "1.0e30" if dtype == np.float32 else "1.0e300"
    trees = [parse_expression(e.replace("BIG", big), opts) for e in cases]
    tb = flatten_trees(trees, dtype)
    code, offs, bad, _ = vm.compile_info(opts, tb, 4000, 5, dtype)
    got = [(int(offs[k + 1] - offs[k]), (int(code["op"][offs[k + 1] - 1]) >> 24 & 7) if offs[k + 1] > offs[k] else 0)
           for k in range(len(cases))]
    assert got == list(cases.values()), list(zip(cases, got))
    rng = np.random.default_rng(3)
    X = rng.standard_normal((5, 4000)).astype(dtype)
    X[0] = np.abs(X[0]) + 50.0  # exp(x1 cos(x2)) reaches Inf on some rows: the PBC node's input check
    y = rng.standard_normal(4000).astype(dtype)
    loss, comp = vm.eval_loss_batch(opts, tb, X, y, dtype)
    tol, ol, oc, _ = loss_tolerance(Oracle.from_options(opts), tb, X, y)
    assert np.array_equal(comp, oc), [(e, c, o) for e, c, o in zip(cases, comp, oc) if c != o]
    assert_losses_within(loss, ol, comp, tol)


def test_stack_depth_bound_for_maxsize_30():
    # Sethi-Ullman: a tree needing d stack slots has >= 1 + 2*m(d-1) nodes, m(0)=2 -> d <= 3 at 30 nodes
    opts = Options(**OPTS)
    tb = flatten_trees(gen_random_population(3000, opts, 5, seed=9), np.float32)
    _, _, _, depth = vm.compile_info(opts, tb, 100, 5, np.float32)
    assert depth <= 3


def test_program_shapes():
    opts = Options(**OPTS)
    cases = {
        "x1": 1,                          # LOAD
        "x1 * 3.0": 1,                    # PAIR MUL FC
        "cos(3.0 * 2.0)": 1,              # folded constant tree
        "cos(x1) + cos(x2)": 3,           # LOAD+cos, LOAD+PUSH+cos, ADD stack (unaries fused as POST)
        "(x1 * 2.0) * (3.0 * 4.0)": 2,    # PAIR, then the folded right child as constant operand
    }
    trees = [parse_expression(e, opts) for e in cases]
    tb = flatten_trees(trees, np.float32)
    code, offs, bad, depth = vm.compile_info(opts, tb, 100, 5, np.float32)
    assert list(np.diff(offs)) == list(cases.values())
    assert not bad.any()
    # CHECK bit placement: cos(x1) is a general unary -> x1's array is checked; root always checked
    k = list(cases).index("cos(x1) + cos(x2)")
    ops = [int(v) for v in code["op"][offs[k]:offs[k + 1]]]
    meta = [int(v) for v in code["meta"][offs[k]:offs[k + 1]]]
    assert [vm.is_check(m) for m in meta] == [1, 1, 1]
    # LOAD x1 + POST cos, LOAD_PUSH x2 (cos(x1) to slot 0) + POST cos, ADD with slot 0 (commuted: R
    # variant); each cos output is checked (child of a general binary): POST_CHECK
    post_cos = (5 << vm.POST_SHIFT) | vm.POST_CHECK
    assert ops == [0 | post_cos, 2 | post_cos, 80 + 1]
    assert [vm.push_slot(m) for m in meta] == [-1, 0, -1]
    assert vm.operand(meta[2]) == 0 and vm.operand(meta[1]) == 1
    # fused unary: cos(x1 * 2.0) -> PAIR MUL FC with POST INF-cos (the root: POST_CHECK); no CHECK on
    # the inner product
    tb2 = flatten_trees([parse_expression("cos(x1 * 2.0)", opts)], np.float32)
    code2, offs2, _, depth2 = vm.compile_info(opts, tb2, 100, 5, np.float32)
    ops2 = [int(v) for v in code2["op"][:offs2[1]]]
    meta2 = [int(v) for v in code2["meta"][:offs2[1]]]
    assert ops2 == [(256 + 6 * 2 + 1) | (5 << vm.POST_SHIFT) | vm.POST_INF | vm.POST_CHECK]
    assert [vm.is_check(m) for m in meta2] == [0]
    # a unary of a unary: the inner one rides on the LOAD, the outer one is its own instruction
    tb5 = flatten_trees([parse_expression("exp(cos(x1))", opts)], np.float32)
    code5, offs5, _, _ = vm.compile_info(opts, tb5, 100, 5, np.float32)
    assert [int(v) & vm.OP_MASK for v in code5["op"][:offs5[1]]] == [0, 40 + 4]  # (DE fused form: INF-exp)
    assert (int(code5["op"][0]) >> vm.POST_SHIFT) & 0x3F == 5
    assert depth2 == 0  # the fused unary needs no stack slot
    # non-commutative stack operand keeps its side: (x1 - cos(x2)) - exp(x3) style trees
    tb3 = flatten_trees([parse_expression("cos(x1) - exp(x2)", opts)], np.float32)
    code3, offs3, _, _ = vm.compile_info(opts, tb3, 100, 5, np.float32)
    assert int(code3["op"][offs3[1] - 1]) == 80 + 6 * 1 + 0  # SUB, SL: op(slot, tos)
    # PAIR instructions: leaf-leaf binaries in one instruction (FF / FC / CF, + 3 with a push)
    exprs = ["x1 * 3.0", "3.0 - x2", "x1 / x3", "3.0 * x2", "(x1 - x2) * (x3 + 2.0)"]
    tb4 = flatten_trees([parse_expression(e, opts) for e in exprs], np.float32)
    code4, offs4, _, _ = vm.compile_info(opts, tb4, 100, 5, np.float32)
    prog = [[int(v) for v in code4["op"][offs4[k]:offs4[k + 1]]] for k in range(len(exprs))]
    assert prog[0] == [256 + 6 * 2 + 1]
    assert prog[1] == [256 + 6 * 1 + 2]
    assert prog[2] == [256 + 6 * 3 + 0] and int(code4["c1"][offs4[2]]) == 0
    assert int(code4["val"][offs4[2]].view(np.uint32)) == 2  # second feature (x3)
    assert prog[3] == [256 + 6 * 2 + 1]  # commuted to FC
    assert prog[4] == [256 + 6 * 1 + 0, 256 + 0 + 1 + 3, 80 + 6 * 2 + 1]
    assert vm.push_slot(int(code4["meta"][offs4[4] + 1])) == 0


def test_static_incomplete():
    opts = Options(**OPTS)
    exprs = ["x1 + inf", "cos(inf)", "exp(1000.0)", "x1 * nan", "1e36 * 1.0", "x1 + 1.0"]
    tb = flatten_trees([parse_expression(e, opts) for e in exprs], np.float32)
    _, _, bad, _ = vm.compile_info(opts, tb, 1000, 5, np.float32)
    # constant 1e36 filled over 1000 rows: its array sum overflows Float32 -> statically incomplete
    assert list(bad) == [True, True, True, True, True, False]
    _, _, bad1, _ = vm.compile_info(opts, tb, 1, 5, np.float32)
    assert list(bad1) == [True, True, True, True, False, False]


def test_bad_trees_rejected():
    from sr_amd import Node, SRError

    opts = Options(**OPTS)
    with pytest.raises(SRError):
        vm.compile_info(opts, flatten_trees([Node(feature=6)]), 10, 5, np.float32)
    with pytest.raises(SRError):
        vm.compile_info(opts, flatten_trees([Node(op=9, l=Node(feature=1))]), 10, 5, np.float32)
