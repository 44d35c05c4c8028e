"""MNIST 2-layer MLP (BASELINE.json config 1: MirroredStrategy on CPU:0,CPU:1 plumbing)."""
from __future__ import annotations

from ..keras import layers as KL
from ..keras.models import Sequential


def MnistMLP(hidden=128, num_classes=10, dropout=0.0):
    layers = [KL.Flatten(), KL.Dense(hidden, activation="relu")]
    if dropout:
        layers.append(KL.Dropout(dropout))
    layers.append(KL.Dense(num_classes))
    return Sequential(layers, name="mnist_mlp")


def synthetic_mnist(n=2048, seed=0):
    """Synthetic MNIST-shaped data (no dataset download): class-conditional blobs in 28x28."""
    import numpy as np
    rng = np.random.RandomState(seed)
    y = rng.randint(0, 10, size=n)
    centers = rng.randn(10, 28 * 28).astype(np.float32)
    x = centers[y] + 0.5 * rng.randn(n, 28 * 28).astype(np.float32)
    return x.reshape(n, 28, 28), y.astype(np.int64)
