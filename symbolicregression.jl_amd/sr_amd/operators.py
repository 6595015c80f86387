"""Operator catalog of the device evaluator, keyed the way SymbolicRegression names operators.

``Options`` maps what the user passes (``log``, ``^``, ``sqrt``, ...) through the reference's
``OP_MAP`` (src/Options.jl:182-202) to the safe versions (src/Operators.jl:35-124); the resulting
names are what ``sr_register_opset`` receives.
"""
from __future__ import annotations

import operator as _op

# user-facing name / alias -> canonical (post OP_MAP) name
BINARY_ALIASES = {
    "+": "+", "plus": "+", "add": "+",
    "-": "-", "sub": "-",
    "*": "*", "mult": "*", "mul": "*",
    "/": "/", "div": "/", "truediv": "/",
    "^": "safe_pow", "pow": "safe_pow", "safe_pow": "safe_pow", "**": "safe_pow",
    "max": "max", "min": "min", "mod": "mod",
    ">": "greater", "greater": "greater",
    "<": "less", "less": "less",
    ">=": "greater_equal", "greater_equal": "greater_equal",
    "<=": "less_equal", "less_equal": "less_equal",
    "cond": "cond", "logical_or": "logical_or", "logical_and": "logical_and",
    "atan2": "atan2",
}
UNARY_ALIASES = {
    "neg": "neg", "square": "square", "cube": "cube", "exp": "exp", "cos": "cos", "sin": "sin",
    "tan": "tan", "log": "safe_log", "safe_log": "safe_log", "log2": "safe_log2",
    "safe_log2": "safe_log2", "log10": "safe_log10", "safe_log10": "safe_log10",
    "log1p": "safe_log1p", "safe_log1p": "safe_log1p", "sqrt": "safe_sqrt",
    "safe_sqrt": "safe_sqrt", "abs": "abs", "sign": "sign", "tanh": "tanh", "sinh": "sinh",
    "cosh": "cosh", "atan": "atan", "asin": "safe_asin", "safe_asin": "safe_asin",
    "acos": "safe_acos", "safe_acos": "safe_acos", "acosh": "safe_acosh",
    "safe_acosh": "safe_acosh", "atanh": "safe_atanh", "safe_atanh": "safe_atanh",
    "asinh": "asinh", "relu": "relu", "inv": "inv", "erf": "erf", "erfc": "erfc",
    "gamma": "gamma", "round": "round", "floor": "floor", "ceil": "ceil", "exp2": "exp2",
    "expm1": "expm1",
}
# How DynamicExpressions prints each canonical operator (get_op_name, src/Operators.jl:126-160).
PRINT_NAME = {
    "safe_pow": "^", "safe_log": "log", "safe_log2": "log2", "safe_log10": "log10",
    "safe_log1p": "log1p", "safe_sqrt": "sqrt", "safe_asin": "asin", "safe_acos": "acos",
    "safe_acosh": "acosh", "safe_atanh": "atanh", "greater": ">", "less": "<",
    "greater_equal": ">=", "less_equal": "<=",
}
_PY_FUNCS = {
    _op.add: "+", _op.sub: "-", _op.mul: "*", _op.truediv: "/", _op.pow: "^", _op.neg: "neg",
    max: "max", min: "min", abs: "abs",
}


def canonical_binary(op) -> str:
    name = _PY_FUNCS.get(op, op) if not isinstance(op, str) else op
    if not isinstance(name, str):
        name = getattr(op, "__name__", repr(op))
    if name not in BINARY_ALIASES:
        raise ValueError(f"binary operator {name!r} is not in the device catalog")
    return BINARY_ALIASES[name]


def canonical_unary(op) -> str:
    name = _PY_FUNCS.get(op, op) if not isinstance(op, str) else op
    if not isinstance(name, str):
        name = getattr(op, "__name__", repr(op))
    if name not in UNARY_ALIASES:
        raise ValueError(f"unary operator {name!r} is not in the device catalog")
    return UNARY_ALIASES[name]


def print_name(canonical: str) -> str:
    return PRINT_NAME.get(canonical, canonical)


class OperatorEnum:
    """``options.operators``: ops[1] = unary, ops[2] = binary (canonical names, in order)."""

    def __init__(self, unaops, binops):
        self.unaops = tuple(canonical_unary(o) for o in unaops)
        self.binops = tuple(canonical_binary(o) for o in binops)

    @property
    def ops(self):
        return {1: self.unaops, 2: self.binops}

    @property
    def nops(self):
        return (len(self.unaops), len(self.binops))

    def unary_index(self, name) -> int:
        c = canonical_unary(name)
        return self.unaops.index(c) + 1

    def binary_index(self, name) -> int:
        c = canonical_binary(name)
        return self.binops.index(c) + 1

    def key(self):
        return (self.unaops, self.binops)

    def __repr__(self):
        return f"OperatorEnum(unaops={self.unaops}, binops={self.binops})"
