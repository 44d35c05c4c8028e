"""Streaming metrics (state kept on device; read back only when a value is asked for)."""
from __future__ import annotations

import torch


class Metric:
    def __init__(self, name=None):
        self.name = name or type(self).__name__.lower()
        self.reset_state()

    def reset_state(self):
        # zero in place once allocated: a captured (hipGraph) step keeps accumulating into these
        if getattr(self, "_total", None) is not None:
            self._total.zero_()
            self._count.zero_()
        else:
            self._total = None
            self._count = None

    def _acc(self, total, count):
        if self._total is None:
            self._total = total.detach().float().clone()
            self._count = count.detach().float().clone() if isinstance(count, torch.Tensor) else torch.tensor(
                float(count), device=total.device)
        else:
            self._total += total.detach().float()
            self._count += count.detach().float() if isinstance(count, torch.Tensor) else float(count)

    def update_state(self, *args, **kw):
        raise NotImplementedError

    def result(self):
        if self._total is None or float(self._count) == 0.0:
            return 0.0
        return float(self._total / self._count.clamp_min(1e-12))

    def merge_state(self, other):
        if other._total is not None:
            self._acc(other._total, other._count)


class Mean(Metric):
    def update_state(self, value, sample_weight=None):
        v = torch.as_tensor(value).float()
        self._acc(v.sum(), v.numel())


class SparseCategoricalAccuracy(Metric):
    def __init__(self, name="sparse_categorical_accuracy"):
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
        pred = y_pred.argmax(-1)
        t = y_true.reshape(pred.shape).to(pred.dtype)
        self._acc((pred == t).float().sum(), pred.numel())


class Accuracy(Metric):
    def update_state(self, y_true, y_pred, sample_weight=None):
        self._acc((y_true.reshape(y_pred.shape) == y_pred).float().sum(), y_pred.numel())


class BinaryAccuracy(Metric):
    def __init__(self, name="binary_accuracy", threshold=0.5):
        self.threshold = threshold
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
        p = (y_pred.float() > self.threshold).float()
        self._acc((p == y_true.float().reshape(p.shape)).float().sum(), p.numel())


class MeanSquaredError(Metric):
    def __init__(self, name="mean_squared_error"):
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
        d = y_pred.float() - y_true.float().reshape(y_pred.shape)
        self._acc((d * d).sum(), d.numel())


class TopKCategoricalAccuracy(Metric):
    def __init__(self, k=5, name="top_k_categorical_accuracy"):
        self.k = k
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
        topk = y_pred.topk(self.k, -1).indices
        t = y_true.reshape(-1, 1).to(topk.dtype)
        self._acc((topk == t).any(-1).float().sum(), t.shape[0])


_ALIASES = {"accuracy": SparseCategoricalAccuracy, "sparse_categorical_accuracy": SparseCategoricalAccuracy,
            "mse": MeanSquaredError, "mean_squared_error": MeanSquaredError,
            "top_k_categorical_accuracy": TopKCategoricalAccuracy, "binary_accuracy": BinaryAccuracy}


def get(identifier):
    if isinstance(identifier, Metric):
        return identifier
    m = _ALIASES[str(identifier).lower()]()
    m.name = str(identifier)  # Keras reports a metric under the string it was requested with
    return m
