"""The reference's model: scalar linear regression y = X*w + b with instance keys passthrough.

Reference trainer/task.py:62-75 (standalone) and :130-142 (distributed): placeholders
``keys:int32[None,1]``, ``X,Y:f32[None,1]``; variables ``weight``, ``bias`` (f32, init 0.0) and
the untrainable ``global_step``; loss ``reduce_sum(square(Y - X*w - b))``; ``predict = X*w + b``;
serving signature inputs ``keys``/``features`` -> outputs ``keys``/``prediction``
(trainer/task.py:164-173).
"""
from __future__ import annotations

import numpy as np
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

    # TF1 optimizer ops and their extra inputs after (var, slots...): (op, [slot names], scalar hyper inputs)
    _TF_APPLY = {
        "sgd": ("ApplyGradientDescent", [], ["lr"]),
        "momentum": ("ApplyMomentum", ["Momentum"], ["lr", "grad", "momentum"]),
        "adam": ("ApplyAdam", ["Adam", "Adam_1"], ["beta1_power", "beta2_power", "lr", "beta1", "beta2", "epsilon"]),
        "adagrad": ("ApplyAdagrad", ["Adagrad"], ["lr"]),
        "adadelta": ("ApplyAdadelta", ["Adadelta", "Adadelta_1"], ["lr", "rho", "epsilon"]),
        "ftrl": ("ApplyFtrl", ["Ftrl", "Ftrl_1"], ["grad", "lr", "l1", "l2", "lr_power"]),
        "rmsprop": ("ApplyRMSProp", ["RMSProp", "RMSProp_1"], ["lr", "rho", "momentum", "epsilon"]),
    }

    def tf_graph(self, g, reads, training=False, optimizer=None):
        """This model as a TF1 graph in `g` (graph_def.GraphBuilder) — the graph the reference builds at
        trainer/task.py:130-142 (placeholders, Mul/Add prediction, keys passthrough) and, with `training`, its
        loss, gradients, optimizer apply ops on the variables and the global_step increment (what
        optimizer.minimize adds). Returns (signature tensor names, train op name or None)."""
        from ..saved_model import graph_def as GD
        keys = g.placeholder("keys", "int32", [-1, 1])
        features = g.placeholder("features", "float32", [-1, 1])
        keys_out = g.identity("keys_identity", keys, "int32")
        pred = g.binary("Add", "prediction", g.binary("Mul", "mul", features, reads["weight"]), reads["bias"])
        names = {"inputs": {"keys": f"{keys}:0", "features": f"{features}:0"},
                 "outputs": {"keys": f"{keys_out}:0", "prediction": f"{pred}:0"}}
        if not training:
            return names, None
        labels = g.placeholder("labels", "float32", [-1, 1])
        gstep = "global_step"
        if not any(v[0] == gstep for v in g.variables):
            g.variable(gstep, np.int32(0), "int32", trainable=False)
        diff = g.binary("Sub", "sub", labels, pred)
        loss = g.reduce_sum("loss", g.unary("Square", "Square", diff), 2)
        # d loss / d prediction = -2 (labels - prediction); reduced over the batch for the scalar variables
        gpred = g.binary("Mul", "gradients/prediction_grad", diff, g.const("gradients/mul/y", -2.0, "float32"))
        grads = {"weight": g.reduce_sum("gradients/weight_grad", g.binary("Mul", "gradients/mul_grad", gpred,
                                                                               features), 2),
                 "bias": g.reduce_sum("gradients/bias_grad", gpred, 2)}
        kind = getattr(optimizer, "kind", "sgd")
        op, slots, extra = self._TF_APPLY.get(kind, self._TF_APPLY["sgd"])
        hyper = dict(getattr(optimizer, "hyper", {}) or {})
        lr_v = float(optimizer._lr_value(0)) if optimizer is not None else 0.01
        scope = getattr(optimizer, "name", None) or "GradientDescent"
        consts = {"lr": lr_v, "beta1": hyper.get("beta_1", 0.9), "beta2": hyper.get("beta_2", 0.999),
                  "epsilon": hyper.get("epsilon", 1e-8), "rho": hyper.get("rho", 0.95 if kind == "adadelta" else 0.9),
                  "momentum": hyper.get("momentum", 0.0), "l1": hyper.get("l1_regularization_strength", 0.0),
                  "l2": hyper.get("l2_regularization_strength", 0.0), "lr_power": -0.5}
        if kind == "adam":  # non-slot accumulators, colocated with the first variable (TF1 Adam)
            for nm, b in (("beta1_power", consts["beta1"]), ("beta2_power", consts["beta2"])):
                consts[nm] = g.variable(nm, np.float32(b), "float32", trainable=False)
        applies = []
        for v in ("weight", "bias"):
            slot_reads = []
            for sn in slots:
                init = 0.1 if sn in ("Adagrad", "Ftrl") else 1.0 if sn == "RMSProp" else 0.0
                g.variable(f"{v}/{sn}", np.float32(init), "float32", trainable=False)
                slot_reads.append(f"{v}/{sn}")
            ins = [v] + slot_reads
            for e in extra:
                if e == "grad":
                    ins.append(grads[v])
                elif isinstance(consts.get(e), str):
                    ins.append(consts[e])
                else:
                    ins.append(g.const(f"{scope}/{e}", float(consts[e]), "float32"))
            if "grad" not in extra:
                ins.append(grads[v])
            applies.append(g.node(f"{scope}/update_{v}/{op}", op, ins,
                                  {"T": GD.attr_type("float32"), "use_locking": GD.attr_bool(False)}))
        inc = g.node(f"{scope}/update", "AssignAdd", [gstep, g.const(f"{scope}/value", 1, "int32")],
                     {"T": GD.attr_type("int32"), "use_locking": GD.attr_bool(False)})
        train_op = g.node(scope, "NoOp", [f"^{a}" for a in applies] + [f"^{inc}"])
        g.node("summaries/loss", "ScalarSummary", [g.const("summaries/loss/tags", "loss", "string"), loss],
               {"T": GD.attr_type("float32")})
        return names, train_op
