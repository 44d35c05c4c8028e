"""Keras-style layers on the framework's ops.

Conventions (MI355X-first): images are channels-last NHWC (the layout the
implicit-GEMM conv kernel and FusedBatchNorm kernels want); Dense kernels are
stored ``[units, in]`` and Conv2D kernels ``[filters, kh, kw, in]`` (KRSC) as
f32 master variables — the layouts the MFMA kernels read without a transpose.
``mixed_bfloat16`` is the GPU compute policy: variables f32, activations bf16.
"""
from __future__ import annotations

import math
import re

import torch

from .. import context, ops
from ..variables import Variable, unique_name
from . import initializers

_policy = {"name": "mixed_bfloat16"}


def set_global_policy(name):
    _policy["name"] = str(name)


def global_policy():
    return _policy["name"]


def _snake(name):
    s = re.sub(r"(.)([A-Z][a-z]+)", r"\1_\2", name)
    return re.sub(r"([a-z0-9])([A-Z])", r"\1_\2", s).lower()


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class Layer:
    """Base layer: weight creation, sublayer tracking, lazy build on first call."""

    def __new__(cls, *args, **kwargs):
        obj = super().__new__(cls)
        object.__setattr__(obj, "_init_args", (args, dict(kwargs)))  # for SavedModel re-construction
        return obj

    def __init__(self, name=None, trainable=True, dtype=None, **kwargs):
        object.__setattr__(self, "_layers", [])
        object.__setattr__(self, "_own_weights", [])
        self._name = name or unique_name(_snake(type(self).__name__))
        self._trainable = trainable
        self.built = False
        self._dtype = dtype
        self.input_spec = None

    # ---- tracking
    def __setattr__(self, key, value):
        if isinstance(value, Layer) and not key.startswith("_"):
            if value not in self._layers:
                self._layers.append(value)
        elif isinstance(value, (list, tuple)) and value and all(isinstance(v, Layer) for v in value):
            for v in value:
                if v not in self._layers:
                    self._layers.append(v)
        object.__setattr__(self, key, value)

    @property
    def name(self):
        return self._name

    @property
    def trainable(self):
        return self._trainable

    @trainable.setter
    def trainable(self, v):
        self._trainable = bool(v)
        for l in self._layers:
            l.trainable = v

    @property
    def layers(self):
        return list(self._layers)

    def add_weight(self, name, shape, initializer="glorot_uniform", trainable=True, dtype=torch.float32):
        init = initializers.get(initializer)
        value = init(tuple(shape), dtype) if not isinstance(init, (int, float)) else torch.full(shape, init)
        v = Variable(value, trainable=trainable, name=f"{self.name}/{name}", device=context.current_device())
        self._own_weights.append(v)
        return v

    def _all_weights(self):
        out, seen = [], set()
        for w in self._own_weights:
            if id(w) not in seen:
                seen.add(id(w))
                out.append(w)
        for l in self._layers:
            for w in l._all_weights():
                if id(w) not in seen:
                    seen.add(id(w))
                    out.append(w)
        return out

    @property
    def weights(self):
        return self.trainable_weights + self.non_trainable_weights

    @property
    def variables(self):
        return self.weights

    def _collect(self, trainable_ctx=True):
        """(weight, effectively_trainable) pairs, depth-first, de-duplicated by identity."""
        out, seen = [], set()

        def rec(layer, ctx):
            ctx = ctx and layer._trainable
            for w in layer._own_weights:
                if id(w) not in seen:
                    seen.add(id(w))
                    out.append((w, ctx and w.trainable))
            for l in layer._layers:
                rec(l, ctx)
        rec(self, trainable_ctx)
        return out

    @property
    def trainable_weights(self):
        return [w for w, t in self._collect() if t]

    trainable_variables = trainable_weights

    @property
    def non_trainable_weights(self):
        return [w for w, t in self._collect() if not t]

    non_trainable_variables = non_trainable_weights

    def count_params(self):
        return sum(w.numel() for w in self.weights)

    # ---- execution
    def build(self, input_shape):
        self.built = True

    def call(self, inputs, *args, **kwargs):
        return inputs

    def __call__(self, inputs, *args, **kwargs):
        if _has_symbolic(inputs):
            return _symbolic_call(self, inputs, args, kwargs)
        if not self.built:
            shape = tuple(inputs.shape) if isinstance(inputs, torch.Tensor) else (
                [tuple(i.shape) for i in inputs] if isinstance(inputs, (list, tuple)) else None)
            with context.device(context.current_device()):
                self.build(shape)
            self.built = True
            object.__setattr__(self, "_build_input_shape", shape)
        return self.call(inputs, *args, **kwargs)

    def get_config(self):
        return {"name": self.name, "trainable": self._trainable}

    def get_weights(self):
        return [w.detach().cpu().numpy() for w in self.weights]

    def set_weights(self, values):
        for w, v in zip(self.weights, values):
            w.assign(torch.as_tensor(v))


def _compute_dtype(x):
    if x.is_cuda and global_policy() == "mixed_bfloat16":
        return torch.bfloat16
    return torch.float32


class InputLayer(Layer):
    def __init__(self, input_shape=None, name=None, **kw):
        super().__init__(name=name, **kw)
        self.input_shape = input_shape


class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", **kw):
        super().__init__(**kw)
        self.units = int(units)
        self.activation = activation
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer

    def build(self, input_shape):
        fan_in = input_shape[-1]
        self.kernel = self.add_weight("kernel", (self.units, fan_in), self.kernel_initializer)
        self.bias = self.add_weight("bias", (self.units,), self.bias_initializer) if self.use_bias else None
        self.built = True

    def call(self, x, training=None):
        fused = self.activation if self.activation in (None, "linear", "relu", "gelu") else None
        y = ops.dense(x, self.kernel, self.bias, act=fused)
        if fused is None and self.activation is not None:
            y = activations_get(self.activation)(y)
        return y

    def get_config(self):
        return {**super().get_config(), "units": self.units, "activation": self.activation,
                "use_bias": self.use_bias}


class Conv2D(Layer):
    """NHWC convolution; padding 'valid'|'same' (TF semantics)."""

    def __init__(self, filters, kernel_size, strides=1, padding="valid", dilation_rate=1, activation=None,
                 use_bias=True, kernel_initializer="glorot_uniform", bias_initializer="zeros", **kw):
        super().__init__(**kw)
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding.lower()
        self.dilation_rate = _pair(dilation_rate)
        self.activation = activation
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer

    def _pads(self, H, W):
        if self.padding == "valid":
            return (0, 0), (0, 0)
        (pt, th) = ops.same_pads(H, self.kernel_size[0], self.strides[0], self.dilation_rate[0])
        (pl, tw) = ops.same_pads(W, self.kernel_size[1], self.strides[1], self.dilation_rate[1])
        return (pt, pl), (th - pt, tw - pl)

    def build(self, input_shape):
        cin = input_shape[-1]
        kh, kw = self.kernel_size
        self.kernel = self.add_weight("kernel", (self.filters, kh, kw, cin), self.kernel_initializer)
        self.bias = self.add_weight("bias", (self.filters,), self.bias_initializer) if self.use_bias else None
        self.built = True

    def call(self, x, training=None):
        N, H, W, C = x.shape
        (pt, pl), (pb, pr) = self._pads(H, W)
        if pb != pt or pr != pl:  # asymmetric SAME padding: pad the extra row/col explicitly
            x = torch.nn.functional.pad(x, (0, 0, 0, pr - pl, 0, pb - pt))
        act = 1 if self.activation == "relu" else 0
        y = ops.conv2d(x, self.kernel, self.bias, self.strides, (pt, pl), self.dilation_rate, act=act)
        if self.activation not in (None, "linear", "relu"):
            y = activations_get(self.activation)(y)
        return y

    def get_config(self):
        return {**super().get_config(), "filters": self.filters, "kernel_size": self.kernel_size,
                "strides": self.strides, "padding": self.padding}


class BatchNormalization(Layer):
    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True, **kw):
        super().__init__(**kw)
        if axis not in (-1, 3):
            raise ValueError("only channels-last BatchNormalization (axis=-1) is supported")
        self.momentum, self.epsilon, self.center, self.scale = momentum, epsilon, center, scale

    def build(self, input_shape):
        c = input_shape[-1]
        self.gamma = self.add_weight("gamma", (c,), "ones") if self.scale else None
        self.beta = self.add_weight("beta", (c,), "zeros") if self.center else None
        self.moving_mean = self.add_weight("moving_mean", (c,), "zeros", trainable=False)
        self.moving_variance = self.add_weight("moving_variance", (c,), "ones", trainable=False)
        self.built = True

    def call(self, x, training=None):
        return ops.batch_norm(x, self.gamma, self.beta, self.moving_mean, self.moving_variance,
                              training=bool(training), momentum=self.momentum, eps=self.epsilon)


class ConvBN(Layer):
    """Fused Conv2D(no bias) -> BatchNormalization -> [+residual] -> [ReLU] (one autograd node).

    On GPU the BN batch statistics come from the conv epilogue and the
    normalize/residual/ReLU is a single pass (ops.conv_bn)."""

    def __init__(self, filters, kernel_size, strides=1, padding="same", relu=True, momentum=0.9, epsilon=1e-5,
                 kernel_initializer="he_normal", gamma_initializer="ones", **kw):
        super().__init__(**kw)
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding
        self.relu = relu
        self.momentum, self.epsilon = momentum, epsilon
        self.kernel_initializer = kernel_initializer
        self.gamma_initializer = gamma_initializer

    def build(self, input_shape):
        cin = input_shape[-1]
        kh, kw = self.kernel_size
        self.kernel = self.add_weight("kernel", (self.filters, kh, kw, cin), self.kernel_initializer)
        self.gamma = self.add_weight("bn/gamma", (self.filters,), self.gamma_initializer)
        self.beta = self.add_weight("bn/beta", (self.filters,), "zeros")
        self.moving_mean = self.add_weight("bn/moving_mean", (self.filters,), "zeros", trainable=False)
        self.moving_variance = self.add_weight("bn/moving_variance", (self.filters,), "ones", trainable=False)
        self.built = True

    def call(self, x, residual=None, training=None, link=None, role=None, pool=None, s2d=False):
        """link/role: residual-gradient join of a block (ops.conv.ResidualGradLink). pool: a MaxPooling2D
        applied to the (ReLU) output, fused with the BatchNorm (ops.conv_bn_maxpool); s2d: x is the
        space-to-depth image of a 7x7/2 conv's input (ops.image_to_s2d_bf16; the layer must be built)."""
        if self.padding == "same":
            pad = ((self.kernel_size[0] - 1) // 2, (self.kernel_size[1] - 1) // 2)
        else:
            pad = (0, 0)
        if pool is not None:
            if not (self.relu and residual is None and link is None):
                return pool(self.call(x, residual, training, link, role))
            return ops.conv_bn_maxpool(x, self.kernel, self.gamma, self.beta, self.moving_mean,
                                       self.moving_variance, stride=self.strides, pad=pad, momentum=self.momentum,
                                       eps=self.epsilon, training=bool(training), pool_size=pool.pool_size,
                                       pool_strides=pool.strides, pool_pad=pool.pads(), s2d=s2d)
        return ops.conv_bn(x, self.kernel, self.gamma, self.beta, self.moving_mean, self.moving_variance,
                           stride=self.strides, pad=pad, relu=self.relu, residual=residual, momentum=self.momentum,
                           eps=self.epsilon, training=bool(training), link=link, role=role)


class MaxPooling2D(Layer):
    def __init__(self, pool_size=2, strides=None, padding="valid", **kw):
        super().__init__(**kw)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides if strides is not None else pool_size)
        self.padding = padding

    def pads(self):
        if self.padding == "same":
            return ((self.pool_size[0] - 1) // 2, (self.pool_size[1] - 1) // 2)
        return (0, 0)

    def call(self, x, training=None):
        return ops.max_pool2d(x, self.pool_size, self.strides, self.pads())


class GlobalAveragePooling2D(Layer):
    def call(self, x, training=None):
        return ops.global_avg_pool(x)


class Flatten(Layer):
    def call(self, x, training=None):
        return x.reshape(x.shape[0], -1)


class Reshape(Layer):
    def __init__(self, target_shape, **kw):
        super().__init__(**kw)
        self.target_shape = tuple(target_shape)

    def call(self, x, training=None):
        return x.reshape(x.shape[0], *self.target_shape)


def _softmax_act(x):
    return torch.softmax(x.float(), -1)


_ACTIVATIONS = {
    None: lambda x: x, "linear": lambda x: x, "relu": ops.relu, "gelu": ops.gelu,
    "sigmoid": lambda x: torch.sigmoid(x), "tanh": lambda x: torch.tanh(x), "softmax": _softmax_act,
}


def activations_get(a):
    if callable(a):
        return a
    return _ACTIVATIONS[a]


class Activation(Layer):
    def __init__(self, activation, **kw):
        super().__init__(**kw)
        self.activation = activation

    def call(self, x, training=None):
        return activations_get(self.activation)(x)


class ReLU(Activation):
    def __init__(self, **kw):
        super().__init__("relu", **kw)


class Softmax(Layer):
    def call(self, x, training=None):
        return _softmax_act(x)


class Dropout(Layer):
    def __init__(self, rate, seed=None, **kw):
        super().__init__(**kw)
        self.rate, self.seed = float(rate), seed

    def call(self, x, training=None):
        return ops.dropout(x, self.rate, training=bool(training))


class Add(Layer):
    def call(self, inputs, training=None):
        out = inputs[0]
        for t in inputs[1:]:
            out = ops.add(out, t)
        return out


class LayerNormalization(Layer):
    def __init__(self, axis=-1, epsilon=1e-3, **kw):
        super().__init__(**kw)
        self.epsilon = epsilon

    def build(self, input_shape):
        d = input_shape[-1]
        self.gamma = self.add_weight("gamma", (d,), "ones")
        self.beta = self.add_weight("beta", (d,), "zeros")
        self.built = True

    def call(self, x, training=None, link=None):
        return ops.layer_norm(x, self.gamma, self.beta, self.epsilon, link=link)


class Embedding(Layer):
    def __init__(self, input_dim, output_dim, embeddings_initializer="random_uniform", **kw):
        super().__init__(**kw)
        self.input_dim, self.output_dim = int(input_dim), int(output_dim)
        self.embeddings_initializer = embeddings_initializer

    def build(self, input_shape):
        self.embeddings = self.add_weight("embeddings", (self.input_dim, self.output_dim),
                                          self.embeddings_initializer)
        self.built = True

    def call(self, ids, training=None):
        return ops.embedding(ids, self.embeddings)


class Lambda(Layer):
    def __init__(self, fn, **kw):
        super().__init__(**kw)
        self.fn = fn

    def call(self, x, training=None):
        return self.fn(x)


# ---------------------------------------------------------------------------------------------------------------
# Functional API: keras.Input returns a symbolic KerasTensor; calling a layer on symbolic inputs records a node
# (layer, symbolic inputs, call arguments) and returns symbolic outputs, which Model(inputs=..., outputs=...) turns
# into a graph that it evaluates in topological order. The reference builds its model as a graph of ops
# (reference trainer/task.py:62-71: placeholders X, keys -> Mul/Add prediction, keys passthrough); this is the Keras
# form of that construction. Layers are built (their weights created) when the node is recorded, by running the
# layer once on a batch-1 example of each symbolic input under no_grad.
_DTYPES = {None: torch.float32, "float32": torch.float32, "float": torch.float32, "float16": torch.float16,
           "bfloat16": torch.bfloat16, "int32": torch.int32, "int64": torch.int64, "bool": torch.bool}


class _Node:
    """One recorded layer call: the layer, its (nested) symbolic inputs and the extra call arguments."""
    __slots__ = ("layer", "inputs", "args", "kwargs")

    def __init__(self, layer, inputs, args, kwargs):
        self.layer, self.inputs, self.args, self.kwargs = layer, inputs, tuple(args), dict(kwargs)


class KerasTensor:
    """Symbolic tensor of a functional model: shape (batch dimension None), dtype and the node that produces it
    (``node is None``: a model input)."""

    def __init__(self, shape, dtype=torch.float32, node=None, index=None, name=None):
        self.shape = tuple(shape)
        self.dtype = dtype
        self.node = node
        self.index = index  # path of this output in the layer's (nested) outputs, None for a single output
        self.name = name or (unique_name("input") if node is None else f"{node.layer.name}/out")

    @property
    def layer(self):
        return self.node.layer if self.node is not None else None

    @property
    def inputs(self):
        return self.node.inputs if self.node is not None else None

    @property
    def input_shape(self):  # Sequential([Input(...), ...]) compatibility: the per-sample shape
        return self.shape[1:]

    def example(self):
        """A zero batch-1 tensor of this spec on the current device (used to build layers)."""
        shape = tuple(1 if d is None else d for d in self.shape)
        return torch.zeros(shape, dtype=self.dtype, device=context.current_device())

    def __repr__(self):
        src = "input" if self.layer is None else self.layer.name
        return f"<KerasTensor shape={self.shape} dtype={self.dtype} from={src}>"


def _flatten(struct):
    if isinstance(struct, dict):
        return [v for k in sorted(struct) for v in _flatten(struct[k])]
    if isinstance(struct, (list, tuple)):
        return [v for x in struct for v in _flatten(x)]
    return [struct]


def _map_structure(fn, struct):
    if isinstance(struct, dict):
        return {k: _map_structure(fn, v) for k, v in struct.items()}
    if isinstance(struct, (list, tuple)):
        return type(struct)(_map_structure(fn, v) for v in struct)
    return fn(struct)


def _has_symbolic(struct):
    return any(isinstance(t, KerasTensor) for t in _flatten(struct))


def _symbolic_call(layer, inputs, args, kwargs):
    """Record `layer(inputs, *args, **kwargs)` on symbolic inputs; returns symbolic outputs of the same structure
    as the layer's concrete outputs."""
    example = _map_structure(lambda t: t.example() if isinstance(t, KerasTensor) else t, inputs)
    kw = {k: v for k, v in kwargs.items() if k != "training"}
    with torch.no_grad():
        out = layer(example, *args, training=False, **kw) if _takes_training(layer) else layer(example, *args, **kw)
    node = _Node(layer, inputs, args, kw)

    def wrap(o, path):
        if isinstance(o, dict):
            return {k: wrap(v, path + (k,)) for k, v in o.items()}
        if isinstance(o, (list, tuple)):
            return type(o)(wrap(v, path + (i,)) for i, v in enumerate(o))
        return KerasTensor((None,) + tuple(o.shape[1:]), o.dtype, node, index=path or None)

    return wrap(out, ())


def _takes_training(layer):
    import inspect
    try:
        return "training" in inspect.signature(layer.call).parameters
    except (TypeError, ValueError):
        return False


def Input(shape=None, batch_size=None, dtype=None, name=None):
    """A symbolic model input (shape excludes the batch dimension): feed it to layers to build a functional
    Model(inputs=..., outputs=...), or list it first in a Sequential to declare the input shape."""
    dt = _DTYPES.get(dtype, dtype) if not isinstance(dtype, torch.dtype) else dtype
    return KerasTensor((batch_size,) + tuple(shape or ()), dt, name=name)


__all__ = [n for n in dir() if not n.startswith("_")]
del math
