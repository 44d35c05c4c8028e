"""The reference's model: scalar linear regression y = X*w + b with instance keys passthrough.

Reference trainer/task.py:62-75 (standalone) and :130-142 (distributed): placeholders
``keys:int32[None,1]``, ``X,Y:f32[None,1]``; variables ``weight``, ``bias`` (f32, init 0.0) and
the untrainable ``global_step``; loss ``reduce_sum(square(Y - X*w - b))``; ``predict = X*w + b``;
serving signature inputs ``keys``/``features`` -> outputs ``keys``/``prediction``
(trainer/task.py:164-173).
"""
from __future__ import annotations

import torch

from ..keras import losses
from ..keras.models import Model


class LinearRegression(Model):
    def __init__(self, name="linear", **kw):
        super().__init__(name=name, **kw)
        self.built = True
        self.weight = self._scalar("weight")
        self.bias = self._scalar("bias")

    def _scalar(self, nm):
        from .. import context
        from ..variables import Variable
        v = Variable(0.0, trainable=True, name=nm, device=context.current_device())
        self._own_weights.append(v)
        return v

    def call(self, X, training=None):
        X = X.reshape(-1, 1).to(self.weight.dtype)
        return X * self.weight + self.bias

    def serve(self, keys, features):
        """serving_default: {keys:int32[None,1], features:f32[None,1]} -> {keys, prediction}."""
        with torch.no_grad():
            return {"keys": keys, "prediction": self(features.float()).reshape(-1, 1)}

    @staticmethod
    def reference_loss():
        return losses.SumSquaredError()

    def serving_signature(self):
        return {
            "inputs": {"keys": ("int32", [-1, 1]), "features": ("float32", [-1, 1])},
            "outputs": {"keys": ("int32", [-1, 1]), "prediction": ("float32", [-1, 1])},
            "method_name": "tensorflow/serving/predict",
            "fn": "serve",
        }

    def get_config(self):
        return {"name": self.name}
