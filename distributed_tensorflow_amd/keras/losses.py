"""Keras losses (reduction: sum_over_batch_size by default, as tf.keras).

The reference's loss is ``reduce_sum(square(Y - X*w - b))`` (reference
trainer/task.py:69) — ``MeanSquaredError(reduction="sum")`` here.
The cross-entropy losses run the fused softmax-CE HIP kernel on GPU.
"""
from __future__ import annotations

import torch

from .. import ops


class Loss:
    def __init__(self, reduction="sum_over_batch_size", name=None):
        self.reduction = reduction
        self.name = name or type(self).__name__

    def per_example(self, y_true, y_pred):
        raise NotImplementedError

    def __call__(self, y_true, y_pred, sample_weight=None):
        l = self.per_example(y_true, y_pred).float()
        if sample_weight is not None:
            l = l * sample_weight
        if self.reduction == "none":
            return l
        if self.reduction == "sum":
            return l.sum()
        return l.mean()


class MeanSquaredError(Loss):
    def per_example(self, y_true, y_pred):
        d = y_pred.float() - y_true.float().reshape(y_pred.shape)
        return (d * d).reshape(d.shape[0], -1).mean(-1) if d.dim() > 1 else d * d


class SumSquaredError(Loss):
    """Reference loss: sum over everything of (y - y_hat)^2."""

    def __init__(self, name=None):
        super().__init__("sum", name)

    def per_example(self, y_true, y_pred):
        d = y_pred.float() - y_true.float().reshape(y_pred.shape)
        return (d * d).reshape(-1)


class MeanAbsoluteError(Loss):
    def per_example(self, y_true, y_pred):
        d = (y_pred.float() - y_true.float().reshape(y_pred.shape)).abs()
        return d.reshape(d.shape[0], -1).mean(-1) if d.dim() > 1 else d


class SparseCategoricalCrossentropy(Loss):
    def __init__(self, from_logits=False, ignore_class=None, label_smoothing=0.0, **kw):
        super().__init__(**kw)
        self.from_logits, self.ignore_class, self.smooth = from_logits, ignore_class, label_smoothing

    def per_example(self, y_true, y_pred):
        labels = y_true.reshape(y_pred.shape[:-1]).long()
        if self.ignore_class is not None:
            labels = torch.where(labels == self.ignore_class, torch.full_like(labels, -100), labels)
        if self.from_logits:
            return ops.sparse_softmax_cross_entropy(y_pred, labels, self.smooth)
        p = y_pred.float().clamp_min(1e-7)
        return torch.nn.functional.nll_loss(p.log().reshape(-1, p.shape[-1]), labels.reshape(-1),
                                            reduction="none").reshape(labels.shape)

    def __call__(self, y_true, y_pred, sample_weight=None):
        l = self.per_example(y_true, y_pred).float()
        if sample_weight is not None:
            l = l * sample_weight
        if self.reduction == "none":
            return l
        if self.reduction == "sum":
            return l.sum()
        if self.ignore_class is not None:
            valid = (y_true.reshape(l.shape) != self.ignore_class).float()
            return l.sum() / valid.sum().clamp_min(1.0)
        return l.mean()


class CategoricalCrossentropy(Loss):
    def __init__(self, from_logits=False, label_smoothing=0.0, **kw):
        super().__init__(**kw)
        self.from_logits, self.smooth = from_logits, label_smoothing

    def per_example(self, y_true, y_pred):
        t = y_true.float()
        if self.smooth:
            t = t * (1 - self.smooth) + self.smooth / t.shape[-1]
        logp = torch.log_softmax(y_pred.float(), -1) if self.from_logits else y_pred.float().clamp_min(1e-7).log()
        return -(t * logp).sum(-1)


class BinaryCrossentropy(Loss):
    def __init__(self, from_logits=False, **kw):
        super().__init__(**kw)
        self.from_logits = from_logits

    def per_example(self, y_true, y_pred):
        t = y_true.float().reshape(y_pred.shape)
        if self.from_logits:
            l = torch.nn.functional.binary_cross_entropy_with_logits(y_pred.float(), t, reduction="none")
        else:
            l = torch.nn.functional.binary_cross_entropy(y_pred.float().clamp(1e-7, 1 - 1e-7), t, reduction="none")
        return l.reshape(l.shape[0], -1).mean(-1) if l.dim() > 1 else l


_ALIASES = {
    "mse": MeanSquaredError, "mean_squared_error": MeanSquaredError, "mae": MeanAbsoluteError,
    "sum_squared_error": SumSquaredError,
    "sparse_categorical_crossentropy": SparseCategoricalCrossentropy,
    "categorical_crossentropy": CategoricalCrossentropy, "binary_crossentropy": BinaryCrossentropy,
}


def get(identifier):
    if identifier is None or isinstance(identifier, Loss) or callable(identifier):
        return identifier
    return _ALIASES[str(identifier).lower()]()
