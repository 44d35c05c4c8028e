"""Keras functional API: keras.Input -> layer calls -> Model(inputs=..., outputs=...).

The reference builds its model as a graph of ops (reference trainer/task.py:62-71: placeholders X, Y, keys; the
Mul/Add prediction; the keys Identity passthrough of the serving signature, :164-173). These tests build that graph
functionally and train it with the reference's setup (SGD lr 0.01, batch 1, samples in order) against the TF1
numpy oracle of SURVEY §4.3, and check graph evaluation (branches, shared layers, nested models, dict I/O)."""
import numpy as np
import pytest
import torch

from distributed_tensorflow_amd import keras
from distributed_tensorflow_amd.keras import layers as KL


def _reference_graph():
    keys = keras.Input(shape=(1,), dtype="int32", name="keys")
    features = keras.Input(shape=(1,), name="features")
    pred = KL.Dense(1, kernel_initializer="zeros", bias_initializer="zeros", name="linear")(features)
    return keys, features, pred


def test_reference_linear_graph_trains_to_tf1_oracle():
    from distributed_tensorflow_amd.data import reference_linear_data
    keys, features, pred = _reference_graph()
    model = keras.Model(inputs=features, outputs=pred)
    assert [w.name for w in model.trainable_weights] == ["linear/kernel", "linear/bias"]
    model.compile(optimizer=keras.optimizers.SGD(0.01), loss="mse")
    x, y = reference_linear_data(0)
    model.fit(x.reshape(-1, 1).astype(np.float32), y.reshape(-1, 1).astype(np.float32), batch_size=1, epochs=10,
              shuffle=False, verbose=0)
    lin = model.get_layer("linear")
    w, b = float(lin.kernel.detach().reshape(())), float(lin.bias.detach().reshape(()))
    # sgd, 10 epochs -> w 2.031, b 10.021 (batch 1: mean squared error == the reference's sum)
    assert abs(w - 2.031) < 5e-3 and abs(b - 10.021) < 5e-3, (w, b)


def test_dict_inputs_and_keys_passthrough():
    keys, features, pred = _reference_graph()
    model = keras.Model(inputs={"keys": keys, "features": features}, outputs={"keys": keys, "prediction": pred})
    layer = model.layers[0]
    layer.kernel.assign(torch.full((1, 1), 2.0))
    layer.bias.assign(torch.full((1,), 10.0))
    out = model({"keys": torch.tensor([[11], [2]], dtype=torch.int32),
                 "features": torch.tensor([[1.0], [2.0]])})
    assert set(out) == {"keys", "prediction"}
    assert out["keys"].tolist() == [[11], [2]]
    assert torch.allclose(out["prediction"], torch.tensor([[12.0], [14.0]]))


def test_branches_shared_layer_and_nested_model():
    torch.manual_seed(0)
    inp = keras.Input(shape=(8,))
    shared = KL.Dense(8, activation="relu", name="shared")
    a = shared(inp)
    b = shared(a)  # the same layer (and weights) twice
    c = KL.Dense(8, name="side")(inp)
    out = KL.Add()([b, c])
    inner = keras.Model(inp, out)
    assert len(inner.trainable_weights) == 4  # shared counted once
    x = torch.randn(5, 8)
    sh, side = inner.layers[0], inner.layers[1]
    ref = torch.relu(torch.relu(x @ sh.kernel.t() + sh.bias) @ sh.kernel.t() + sh.bias) + (x @ side.kernel.t()
                                                                                           + side.bias)
    assert torch.allclose(inner(x), ref, atol=1e-5)
    # a functional model is itself a layer of another functional model
    inp2 = keras.Input(shape=(8,))
    head = KL.Dense(3, name="head")(inner(inp2))
    outer = keras.Model(inputs=[inp2], outputs=[head])
    y = outer([x])
    assert isinstance(y, list) and y[0].shape == (5, 3)
    hd = outer.layers[1]
    assert torch.allclose(y[0], ref @ hd.kernel.t() + hd.bias, atol=1e-5)
    # gradients flow to every weight of the nested graph
    y[0].sum().backward()
    assert all(w.grad is not None for w in outer.trainable_weights)


def test_functional_errors():
    inp = keras.Input(shape=(4,))
    other = keras.Input(shape=(4,))
    out = KL.Dense(2)(other)
    with pytest.raises(ValueError):
        keras.Model(inputs=inp, outputs=out)  # output not reachable from the declared inputs
    with pytest.raises(ValueError):
        keras.Model(inputs=inp, outputs=None)


def test_sequential_still_accepts_input():
    m = keras.Sequential([keras.Input(shape=(3,)), KL.Dense(2)])
    m.build()
    assert m(torch.zeros(4, 3)).shape == (4, 2)
