"""Expression trees with DynamicExpressions' ``Node{T,2}`` fields, and their pre-order flattening.

Fields follow DE 2.x: ``degree`` (0 leaf / 1 unary / 2 binary), ``constant``, ``val``, ``feature``
(1-based), ``op`` (1-based index into ``options.operators.ops[degree]``), children ``l``/``r``.
``flatten_trees`` produces the struct-of-arrays ``sr_tree_batch`` the C ABI takes (pre-order =
``get_scalar_constants`` order, test/integration/ad/zygote/test_derivatives.jl:127-155).
"""
from __future__ import annotations

import ast
import ctypes
from typing import Iterable, List, Optional, Sequence

import numpy as np

from . import _lib
from .operators import OperatorEnum, canonical_binary, canonical_unary, print_name


class Node:
    __slots__ = ("degree", "constant", "val", "feature", "op", "l", "r")

    def __init__(self, *args, val=None, feature=None, op=None, l=None, r=None, children=None):
        # Node("x3") / Node(feature=3) / Node(val=1.5) / Node(op=1, l=..) / Node(op=2, l=.., r=..)
        self.degree = 0
        self.constant = False
        self.val = 0.0
        self.feature = 0
        self.op = 0
        self.l = None
        self.r = None
        if args:
            if len(args) == 1 and isinstance(args[0], str):
                s = args[0]
                if not s.startswith("x"):
                    raise ValueError(f"variable names must look like 'x1', got {s!r}")
                feature = int(s[1:])
            elif isinstance(args[0], int) and len(args) in (2, 3):
                op = args[0]
                children = args[1:]
            else:
                raise ValueError(f"unsupported Node constructor arguments {args!r}")
        if children is not None:
            children = tuple(children)
            if len(children) == 1:
                l = children[0]
            elif len(children) == 2:
                l, r = children
        if op is not None:
            if l is None:
                raise ValueError("operator node needs children")
            self.op = int(op)
            self.l = l
            self.r = r
            self.degree = 2 if r is not None else 1
        elif feature is not None:
            self.feature = int(feature)
        elif val is not None:
            self.constant = True
            self.val = val
        else:
            raise ValueError("Node needs val=, feature= or op=")

    # ------------------------------------------------------------------ DE-style utilities
    def copy(self) -> "Node":
        n = Node.__new__(Node)
        n.degree, n.constant, n.val, n.feature, n.op = self.degree, self.constant, self.val, self.feature, self.op
        n.l = self.l.copy() if self.l is not None else None
        n.r = self.r.copy() if self.r is not None else None
        return n

    def set_node(self, other: "Node") -> None:
        """DE ``set_node!``: overwrite this node's contents with ``other``'s."""
        self.degree, self.constant, self.val, self.feature, self.op = (
            other.degree, other.constant, other.val, other.feature, other.op)
        self.l, self.r = other.l, other.r

    def preorder(self) -> List["Node"]:
        out, stack = [], [self]
        push, pop, emit = stack.append, stack.pop, out.append  # hot in the host search loop
        while stack:
            n = pop()
            emit(n)
            d = n.degree
            if d:
                if d == 2:
                    push(n.r)
                push(n.l)
        return out

    def count_nodes(self) -> int:
        return len(self.preorder())

    def count_constants(self) -> int:
        return sum(1 for n in self.preorder() if n.degree == 0 and n.constant)

    def count_depth(self) -> int:
        if self.degree == 0:
            return 1
        if self.degree == 1:
            return 1 + self.l.count_depth()
        return 1 + max(self.l.count_depth(), self.r.count_depth())

    def is_constant(self) -> bool:
        return all(n.constant for n in self.preorder() if n.degree == 0)

    def __repr__(self):
        return f"Node({string_tree(self)})"

    # arithmetic sugar, resolved against the operators activated by `extend_operators`
    def _bin(self, name, other, swap=False):
        ops = _active_operators()
        o = other if isinstance(other, Node) else Node(val=other)
        a, b = (o, self) if swap else (self, o)
        return Node(op=ops.binary_index(name), l=a, r=b)

    def __add__(self, o): return self._bin("+", o)
    def __radd__(self, o): return self._bin("+", o, True)
    def __sub__(self, o): return self._bin("-", o)
    def __rsub__(self, o): return self._bin("-", o, True)
    def __mul__(self, o): return self._bin("*", o)
    def __rmul__(self, o): return self._bin("*", o, True)
    def __truediv__(self, o): return self._bin("/", o)
    def __rtruediv__(self, o): return self._bin("/", o, True)
    def __pow__(self, o): return self._bin("^", o)
    def __rpow__(self, o): return self._bin("^", o, True)
    def __neg__(self): return apply_unary("neg", self)


def get_scalar_constants(tree: Node) -> np.ndarray:
    return np.array([n.val for n in tree.preorder() if n.degree == 0 and n.constant])


def set_scalar_constants(tree: Node, values: Sequence[float]) -> None:
    k = 0
    for n in tree.preorder():
        if n.degree == 0 and n.constant:
            n.val = values[k]
            k += 1


# ------------------------------------------------------------------ operator context (@extend_operators)
_ACTIVE: List[OperatorEnum] = []


def extend_operators(options_or_ops) -> None:
    """Make Node arithmetic and ``apply_unary`` resolve operator indices against these operators
    (the role of DynamicExpressions' ``@extend_operators``)."""
    ops = getattr(options_or_ops, "operators", options_or_ops)
    _ACTIVE[:] = [ops]


def _active_operators() -> OperatorEnum:
    if not _ACTIVE:
        raise RuntimeError("call extend_operators(options) before building trees with operators")
    return _ACTIVE[0]


def apply_unary(name, child, operators: Optional[OperatorEnum] = None) -> Node:
    ops = operators or _active_operators()
    c = child if isinstance(child, Node) else Node(val=child)
    return Node(op=ops.unary_index(name), l=c)


def apply_binary(name, a, b, operators: Optional[OperatorEnum] = None) -> Node:
    ops = operators or _active_operators()
    a = a if isinstance(a, Node) else Node(val=a)
    b = b if isinstance(b, Node) else Node(val=b)
    return Node(op=ops.binary_index(name), l=a, r=b)


# ------------------------------------------------------------------ printing / parsing
def string_tree(tree: Node, operators: Optional[OperatorEnum] = None) -> str:
    ops = operators or (_ACTIVE[0] if _ACTIVE else None)

    def name(deg, op):
        if ops is None:
            return f"op{deg}_{op}"
        return print_name(ops.ops[deg][op - 1])

    def rec(n: Node) -> str:
        if n.degree == 0:
            return repr(n.val) if n.constant else f"x{n.feature}"
        if n.degree == 1:
            return f"{name(1, n.op)}({rec(n.l)})"
        nm = name(2, n.op)
        if nm in ("+", "-", "*", "/", "^", ">", "<", ">=", "<="):
            return f"({rec(n.l)} {nm} {rec(n.r)})"
        return f"{nm}({rec(n.l)}, {rec(n.r)})"

    return rec(tree)


_PY_BINOPS = {ast.Add: "+", ast.Sub: "-", ast.Mult: "*", ast.Div: "/", ast.Pow: "^"}
_PY_CMP = {ast.Gt: ">", ast.Lt: "<", ast.GtE: ">=", ast.LtE: "<="}


def parse_expression(expr: str, operators) -> Node:
    """Parse e.g. ``"cos(x1 * 3.0) + x2 ^ 2"`` into a Node using ``operators`` (or Options)."""
    ops = getattr(operators, "operators", operators)
    expr = expr.replace("^", "**")

    def rec(e):
        if isinstance(e, ast.Expression):
            return rec(e.body)
        if isinstance(e, ast.Constant):
            return Node(val=float(e.value))
        if isinstance(e, ast.Name):
            if e.id in ("inf", "Inf"):
                return Node(val=float("inf"))
            if e.id in ("nan", "NaN"):
                return Node(val=float("nan"))
            return Node(e.id)
        if isinstance(e, ast.UnaryOp) and isinstance(e.op, ast.USub):
            if isinstance(e.operand, ast.Constant):
                return Node(val=-float(e.operand.value))
            if "neg" in ops.unaops:
                return Node(op=ops.unary_index("neg"), l=rec(e.operand))
            return Node(op=ops.binary_index("*"), l=Node(val=-1.0), r=rec(e.operand))
        if isinstance(e, ast.BinOp):
            return Node(op=ops.binary_index(_PY_BINOPS[type(e.op)]), l=rec(e.left), r=rec(e.right))
        if isinstance(e, ast.Compare) and len(e.ops) == 1:
            return Node(op=ops.binary_index(_PY_CMP[type(e.ops[0])]), l=rec(e.left), r=rec(e.comparators[0]))
        if isinstance(e, ast.Call):
            fname = e.func.id
            args = [rec(a) for a in e.args]
            if len(args) == 1:
                return Node(op=ops.unary_index(fname), l=args[0])
            if len(args) == 2:
                return Node(op=ops.binary_index(fname), l=args[0], r=args[1])
        raise ValueError(f"cannot parse {ast.dump(e)}")

    return rec(ast.parse(expr, mode="eval"))


# ------------------------------------------------------------------ flattening for the C ABI
class TreeBatch:
    """Pre-order struct-of-arrays of many trees, kept alive while the C call runs."""

    def __init__(self, offsets, degree, op, feature, constant, val):
        self.offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self.degree = np.ascontiguousarray(degree, dtype=np.uint8)
        self.op = np.ascontiguousarray(op, dtype=np.uint8)
        self.feature = np.ascontiguousarray(feature, dtype=np.uint16)
        self.constant = np.ascontiguousarray(constant, dtype=np.uint8)
        self.val = np.ascontiguousarray(val)
        self.n_trees = len(self.offsets) - 1

    @property
    def n_nodes(self) -> int:
        return int(self.offsets[-1])

    @property
    def n_operator_nodes(self) -> int:
        return int(np.count_nonzero(self.degree))

    def astype(self, dtype) -> "TreeBatch":
        return TreeBatch(self.offsets, self.degree, self.op, self.feature, self.constant, self.val.astype(dtype))

    def tree_sizes(self) -> np.ndarray:
        return np.diff(self.offsets)

    def take(self, idx) -> "TreeBatch":
        """The batch of trees idx (in that order): the node arrays of each, concatenated."""
        idx = np.asarray(idx, dtype=np.int64)
        b, e = self.offsets[idx], self.offsets[idx + 1]
        nodes = np.concatenate([np.arange(x, y) for x, y in zip(b, e)]) if idx.size else np.zeros(0, np.int64)
        offs = np.concatenate([[0], np.cumsum(e - b)])
        return TreeBatch(offs, self.degree[nodes], self.op[nodes], self.feature[nodes], self.constant[nodes],
                         self.val[nodes])

    def to_struct(self) -> _lib.SrTreeBatch:
        def ptr(a, t):
            return a.ctypes.data_as(ctypes.POINTER(t))

        s = _lib.SrTreeBatch()
        s.n_trees = self.n_trees
        s.offsets = ptr(self.offsets, ctypes.c_int64)
        s.degree = ptr(self.degree, ctypes.c_uint8)
        s.op = ptr(self.op, ctypes.c_uint8)
        s.feature = ptr(self.feature, ctypes.c_uint16)
        s.constant = ptr(self.constant, ctypes.c_uint8)
        s.val = self.val.ctypes.data_as(ctypes.c_void_p)
        return s

    def constant_mask(self) -> np.ndarray:
        return (self.degree == 0) & (self.constant != 0)

    def constant_offsets(self) -> np.ndarray:
        """[n_trees + 1] prefix sum of per-tree constant counts (pre-order, get_scalar_constants)."""
        m = self.constant_mask().astype(np.int64)
        c = np.concatenate([[0], np.cumsum(m)])
        return c[self.offsets]

    def get_constants(self) -> np.ndarray:
        """All trees' constants, pre-order per tree, concatenated (see constant_offsets)."""
        return self.val[self.constant_mask()].copy()

    def with_constants(self, consts) -> "TreeBatch":
        """Same trees with their constants replaced (set_scalar_constants! for the whole batch)."""
        val = self.val.copy()
        val[self.constant_mask()] = np.asarray(consts, dtype=val.dtype)
        return TreeBatch(self.offsets, self.degree, self.op, self.feature, self.constant, val)

    def subset(self, idx) -> "TreeBatch":
        idx = np.asarray(idx, dtype=np.int64)
        starts, ends = self.offsets[idx], self.offsets[idx + 1]
        sel = np.concatenate([np.arange(s, e) for s, e in zip(starts, ends)]) if len(idx) else np.zeros(0, np.int64)
        offs = np.concatenate([[0], np.cumsum(ends - starts)])
        return TreeBatch(offs, self.degree[sel], self.op[sel], self.feature[sel], self.constant[sel], self.val[sel])

    def tree(self, k: int) -> Node:
        b, e = int(self.offsets[k]), int(self.offsets[k + 1])
        pos = [b]

        def rec():
            i = pos[0]
            pos[0] += 1
            d = int(self.degree[i])
            if d == 0:
                if self.constant[i]:
                    return Node(val=self.val[i].item())
                return Node(feature=int(self.feature[i]))
            l = rec()
            r = rec() if d == 2 else None
            return Node(op=int(self.op[i]), l=l, r=r)

        t = rec()
        assert pos[0] == e
        return t


def flatten_trees(trees: Iterable[Node], dtype=np.float32) -> TreeBatch:
    nodes, offsets = [], [0]
    for t in trees:
        t = getattr(t, "tree", t)  # PopMember / Expression wrappers
        nodes.extend(t.preorder())
        offsets.append(len(nodes))
    degree = [n.degree for n in nodes]
    op = [n.op for n in nodes]
    feature = [n.feature for n in nodes]
    constant = [1 if (n.degree == 0 and n.constant) else 0 for n in nodes]
    val = [n.val if n.constant else 0.0 for n in nodes]
    return TreeBatch(offsets, degree, op, feature, constant, np.array(val, dtype=dtype))
