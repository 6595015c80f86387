"""``Dataset`` / ``SubDataset`` / ``batch`` (reference src/Dataset.jl:53-112, 131-246, 300-308).

``X`` is ``[nfeatures, n]`` exactly as in Julia.  The device copy is uploaded once per context
(transposed to per-feature contiguous rows on the GPU) and stays resident; minibatches
(``SubDataset``) only send their row indices.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .device import get_context


class Dataset:
    def __init__(self, X, y=None, *, weights=None, variable_names=None, loss_type=None):
        X = np.asarray(X)
        if X.ndim != 2:
            raise ValueError("X must be a [nfeatures, n] matrix")
        if X.dtype not in (np.float32, np.float64):
            X = X.astype(np.float64)
        self.X = X
        self.nfeatures, self.n = X.shape
        self.dtype = X.dtype
        if y is not None:
            y = np.asarray(y)
            if y.dtype != X.dtype:
                # `_loss` refuses mismatched element types (src/LossFunctions.jl:22-36)
                raise TypeError(
                    f"Element type of `x` is {X.dtype} is different from element type of `y` which is {y.dtype}."
                )
            if y.shape != (self.n,):
                raise ValueError("y must have n entries")
        self.y = y
        if weights is not None:
            weights = np.asarray(weights)
            if weights.dtype != X.dtype:
                raise TypeError("All element types must be the same.")
            if weights.shape != (self.n,):
                raise ValueError("weights must have n entries")
        self.weights = weights
        self.index = 1
        self.avg_y = None if y is None else (
            float(np.sum(y * weights) / np.sum(weights)) if weights is not None else float(np.mean(y)))
        self.use_baseline = True
        self.baseline_loss = X.dtype.type(1.0)
        self.variable_names = variable_names or [f"x{i + 1}" for i in range(self.nfeatures)]
        self._device = {}

    # ---------------------------------------------------------------- device residency
    def device_handle(self, ctx=None):
        ctx = ctx or get_context()
        key = ctx.handle.value  # one copy per context (a search's scoring lanes each hold one)
        h = self._device.get(key)
        if h is None:
            Xj = np.ascontiguousarray(self.X.T)  # Julia column-major [nf, n]: address f + nf*i
            y = None if self.y is None else np.ascontiguousarray(self.y)
            w = None if self.weights is None else np.ascontiguousarray(self.weights)
            out = ctypes.c_void_p()
            _lib.check(
                _lib.lib.sr_dataset_upload(
                    ctx.handle,
                    _lib.SR_DTYPE_F32 if self.dtype == np.float32 else _lib.SR_DTYPE_F64,
                    Xj.ctypes.data_as(ctypes.c_void_p),
                    self.nfeatures,
                    self.n,
                    None if y is None else y.ctypes.data_as(ctypes.c_void_p),
                    None if w is None else w.ctypes.data_as(ctypes.c_void_p),
                    ctypes.byref(out),
                )
            )
            h = out
            self._device[key] = h
        return h

    def free_device(self):
        for h in self._device.values():
            _lib.lib.sr_dataset_free(h)
        self._device.clear()

    def __del__(self):
        try:
            self.free_device()
        except Exception:
            pass

    # ---------------------------------------------------------------- SubDataset protocol
    @property
    def full(self) -> "Dataset":
        return self

    @property
    def indices(self):
        return None

    def is_weighted(self) -> bool:
        return self.weights is not None

    def dataset_fraction(self) -> float:
        return 1.0


class SubDataset:
    """Index view of a BasicDataset (src/Dataset.jl:90-112); indices are 0-based here."""

    def __init__(self, dataset: Dataset, indices):
        self._dataset = dataset
        self._indices = np.ascontiguousarray(np.asarray(indices, dtype=np.int64))
        if self._indices.size and (self._indices.min() < 0 or self._indices.max() >= dataset.n):
            raise IndexError("SubDataset index out of range")

    @property
    def full(self) -> Dataset:
        return self._dataset

    @property
    def indices(self) -> np.ndarray:
        return self._indices

    @property
    def X(self):
        return self._dataset.X[:, self._indices]

    @property
    def y(self):
        return None if self._dataset.y is None else self._dataset.y[self._indices]

    @property
    def weights(self):
        return None if self._dataset.weights is None else self._dataset.weights[self._indices]

    @property
    def n(self) -> int:
        return int(self._indices.size)

    def is_weighted(self) -> bool:
        return self._dataset.weights is not None

    def dataset_fraction(self) -> float:
        return self.n / self._dataset.n

    def __getattr__(self, name):
        # forward everything else (baseline_loss, nfeatures, dtype, ...) like getproperty
        return getattr(self._dataset, name)


def batch(dataset: Dataset, indices_or_size, rng: np.random.Generator | None = None) -> SubDataset:
    """``batch(dataset, indices)`` or ``batch(dataset, batch_size, rng)`` — rows drawn with
    replacement, as ``rand(rng, 1:n, batch_size)`` (src/Dataset.jl:300-308)."""
    if np.isscalar(indices_or_size):
        rng = rng or np.random.default_rng()
        return SubDataset(dataset, rng.integers(0, dataset.n, size=int(indices_or_size)))
    return SubDataset(dataset, indices_or_size)
