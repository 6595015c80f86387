"""``Options`` — the subset of SymbolicRegression's options that the scoring path reads.

Reference: src/Options.jl:502-1214 (constructor + defaults), src/OptionsStruct.jl:177-259 (struct).
The scoring path uses: the operator enum (after OP_MAP), ``elementwise_loss`` (default
``L2DistLoss()``, src/Options.jl:772), ``parsimony`` (stored as Float32, src/OptionsStruct.jl:198),
``loss_function``/``loss_function_expression`` (custom objectives stay on the caller's CPU path) and
the new ``device`` switch that selects this evaluator (it rides next to ``turbo``/``bumper``,
src/OptionsStruct.jl:186-187).
"""
from __future__ import annotations

import re

import numpy as np

from .operators import OperatorEnum

# Elementwise losses the device evaluates: the LossFunctions.jl catalog src/Options.jl:301-328 lists,
# as (SrLossKind, parameter name or None).  Kinds match include/sr_amd.h SR_LOSS_*.
LOSS_KINDS = {
    "L2DistLoss": (0, None), "L1DistLoss": (1, None), "LPDistLoss": (2, "P"), "LogitDistLoss": (3, None),
    "HuberLoss": (4, "d"), "L1EpsilonInsLoss": (5, "eps"), "L2EpsilonInsLoss": (6, "eps"),
    "PeriodicLoss": (7, "circ"), "QuantileLoss": (8, "tau"), "ZeroOneLoss": (9, None),
    "PerceptronLoss": (10, None), "L1HingeLoss": (11, None), "L2HingeLoss": (12, None),
    "SmoothedL1HingeLoss": (13, "gamma"), "ModifiedHuberLoss": (14, None), "L2MarginLoss": (15, None),
    "ExpLoss": (16, None), "SigmoidLoss": (17, None), "DWDMarginLoss": (18, "q"),
}
LOSS_DEFAULTS = {"HuberLoss": 1.0}  # LossFunctions' HuberLoss() default delta
LOSSES = {"l2": 0, "l1": 1}  # short aliases


def parse_loss(spec):
    """'HuberLoss(1.5)', 'LPDistLoss{3}()', 'QuantileLoss(0.3)', 'L2DistLoss()', ... -> (kind, param)."""
    if isinstance(spec, str) and spec in LOSSES:
        return LOSSES[spec], 0.0
    if not isinstance(spec, str):
        raise ValueError(f"elementwise_loss {spec!r} is not supported by the device path")
    m = re.fullmatch(r"\s*([A-Za-z0-9]+)\s*(?:\{\s*([^}]*)\s*\})?\s*(?:\(\s*([^)]*)\s*\))?\s*", spec)
    if not m or m.group(1) not in LOSS_KINDS:
        raise ValueError(f"elementwise_loss {spec!r} is not supported by the device path")
    name, curly, paren = m.group(1), m.group(2), m.group(3)
    kind, pname = LOSS_KINDS[name]
    arg = (curly or "").strip() or (paren or "").strip()
    if pname is None:
        if arg:
            raise ValueError(f"{name} takes no parameter")
        return kind, 0.0
    if not arg:
        if name not in LOSS_DEFAULTS:
            raise ValueError(f"{name} needs its parameter {pname}, e.g. {name}(1.0)")
        return kind, LOSS_DEFAULTS[name]
    return kind, float(arg)


class Options:
    def __init__(
        self,
        binary_operators=("+", "-", "/", "*"),
        unary_operators=(),
        *,
        operators: OperatorEnum | None = None,
        elementwise_loss="L2DistLoss",
        loss_function=None,
        loss_function_expression=None,
        parsimony: float = 0.0,
        maxsize: int = 30,
        maxdepth: int | None = None,
        populations: int = 31,
        population_size: int = 27,
        ncycles_per_iteration: int = 380,
        tournament_selection_n: int = 15,
        tournament_selection_p: float = 0.982,
        batching: bool = False,
        batch_size: int = 50,
        should_optimize_constants: bool = True,
        optimizer_probability: float = 0.14,
        optimizer_nrestarts: int = 2,
        optimizer_iterations: int | None = None,
        optimizer_f_calls_limit: int | None = None,
        optimizer_algorithm: str = "BFGS",
        turbo: bool = False,
        bumper: bool = False,
        device: str = "mi355x",
        deterministic: bool = False,
        seed=None,
    ):
        self.operators = operators if operators is not None else OperatorEnum(unary_operators, binary_operators)
        if callable(elementwise_loss) and not isinstance(elementwise_loss, str):
            raise ValueError("custom elementwise loss functions stay on the reference CPU path")
        self.elementwise_loss = elementwise_loss
        self.loss_kind, self.loss_param = parse_loss(elementwise_loss)
        self.loss_function = loss_function
        self.loss_function_expression = loss_function_expression
        self.parsimony = np.float32(parsimony)
        self.maxsize = int(maxsize)
        self.maxdepth = int(maxdepth) if maxdepth is not None else int(maxsize)
        self.populations = populations
        self.population_size = population_size
        self.ncycles_per_iteration = ncycles_per_iteration
        self.tournament_selection_n = tournament_selection_n
        self.tournament_selection_p = tournament_selection_p
        self.batching = batching
        self.batch_size = batch_size
        # constant optimisation (src/Options.jl:613-619, 988-997)
        self.should_optimize_constants = should_optimize_constants
        self.optimizer_probability = optimizer_probability
        self.optimizer_nrestarts = optimizer_nrestarts
        self.optimizer_iterations = 8 if optimizer_iterations is None else int(optimizer_iterations)
        self.optimizer_f_calls_limit = 10_000 if optimizer_f_calls_limit is None else int(optimizer_f_calls_limit)
        # the device optimiser is Optim's BFGS with BackTracking (Newton for one constant, as the
        # reference chooses); any other algorithm (the reference accepts "NelderMead",
        # src/Options.jl:738-746) stays on the reference's CPU optimize_constants
        if str(optimizer_algorithm) not in ("BFGS", "NelderMead"):
            raise ValueError(f"unknown optimizer_algorithm {optimizer_algorithm!r}")
        self.optimizer_algorithm = str(optimizer_algorithm)
        self.turbo = turbo
        self.bumper = bumper
        if device not in ("mi355x", "gpu", "hip"):
            raise ValueError("this package implements only the MI355X device path (device='mi355x')")
        self.device = "mi355x"
        self.deterministic = deterministic
        self.seed = seed

    @property
    def nops(self):
        return self.operators.nops

    def __repr__(self):
        return f"Options(operators={self.operators!r}, elementwise_loss={self.elementwise_loss}, parsimony={self.parsimony})"
