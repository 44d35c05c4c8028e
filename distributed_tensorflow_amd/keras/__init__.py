"""Keras-style high-level API (tf.keras surface used by the reference and its successors)."""
from . import callbacks, initializers, layers, losses, metrics, optimizers
from .layers import Input
from .models import Model, Sequential

__all__ = ["Model", "Sequential", "Input", "layers", "losses", "metrics", "optimizers", "callbacks",
           "initializers"]
