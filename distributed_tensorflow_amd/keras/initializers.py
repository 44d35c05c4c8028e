"""Keras weight initializers (deterministic under dtf.random.set_seed)."""
from __future__ import annotations

import math

import torch

_gen = torch.Generator()
_gen.manual_seed(1234)


def set_seed(seed):
    _gen.manual_seed(int(seed))
    torch.manual_seed(int(seed))


def _fans(shape, layout):
    shape = tuple(shape)
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        if layout == "out_in":  # [out, in] (our Dense kernel layout)
            return shape[1], shape[0]
        return shape[0], shape[1]
    # conv KRSC: [out, kh, kw, in]
    rf = 1
    for d in shape[1:-1]:
        rf *= d
    return shape[-1] * rf, shape[0] * rf


class Initializer:
    layout = "out_in"

    def __call__(self, shape, dtype=torch.float32):
        raise NotImplementedError

    def get_config(self):
        return {"class_name": type(self).__name__}


class Zeros(Initializer):
    def __call__(self, shape, dtype=torch.float32):
        return torch.zeros(shape, dtype=dtype)


class Ones(Initializer):
    def __call__(self, shape, dtype=torch.float32):
        return torch.ones(shape, dtype=dtype)


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def __call__(self, shape, dtype=torch.float32):
        return torch.full(shape, float(self.value), dtype=dtype)


class RandomNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05):
        self.mean, self.std = mean, stddev

    def __call__(self, shape, dtype=torch.float32):
        return torch.randn(shape, generator=_gen, dtype=torch.float32).mul_(self.std).add_(self.mean).to(dtype)


class TruncatedNormal(RandomNormal):
    def __call__(self, shape, dtype=torch.float32):
        t = torch.randn(shape, generator=_gen)
        t = torch.fmod(t, 2.0)
        return t.mul_(self.std).add_(self.mean).to(dtype)


class RandomUniform(Initializer):
    def __init__(self, minval=-0.05, maxval=0.05):
        self.lo, self.hi = minval, maxval

    def __call__(self, shape, dtype=torch.float32):
        return (torch.rand(shape, generator=_gen) * (self.hi - self.lo) + self.lo).to(dtype)


class VarianceScaling(Initializer):
    def __init__(self, scale=1.0, mode="fan_in", distribution="truncated_normal"):
        self.scale, self.mode, self.dist = scale, mode, distribution

    def __call__(self, shape, dtype=torch.float32):
        fi, fo = _fans(shape, self.layout)
        n = {"fan_in": fi, "fan_out": fo, "fan_avg": (fi + fo) / 2}[self.mode]
        s = self.scale / max(1.0, n)
        if self.dist == "uniform":
            lim = math.sqrt(3 * s)
            return RandomUniform(-lim, lim)(shape, dtype)
        if self.dist == "untruncated_normal":
            return RandomNormal(0, math.sqrt(s))(shape, dtype)
        return TruncatedNormal(0, math.sqrt(s) / 0.87962566103423978)(shape, dtype)


class GlorotUniform(VarianceScaling):
    def __init__(self):
        super().__init__(1.0, "fan_avg", "uniform")


class GlorotNormal(VarianceScaling):
    def __init__(self):
        super().__init__(1.0, "fan_avg", "truncated_normal")


class HeNormal(VarianceScaling):
    def __init__(self):
        super().__init__(2.0, "fan_in", "truncated_normal")


class HeUniform(VarianceScaling):
    def __init__(self):
        super().__init__(2.0, "fan_in", "uniform")


_ALIASES = {
    "zeros": Zeros, "ones": Ones, "glorot_uniform": GlorotUniform, "glorot_normal": GlorotNormal,
    "he_normal": HeNormal, "he_uniform": HeUniform, "random_normal": RandomNormal, "random_uniform": RandomUniform,
    "truncated_normal": TruncatedNormal,
}


def get(identifier):
    if identifier is None:
        return None
    if isinstance(identifier, Initializer) or callable(identifier) and not isinstance(identifier, str):
        return identifier
    return _ALIASES[str(identifier).lower()]()
