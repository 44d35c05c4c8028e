"""tf.data-style input pipelines.

``Dataset`` supports the combinators the training loops need (from_tensor_slices,
map, batch, shuffle, repeat, take, prefetch, shard) plus on-device synthetic
datasets for benchmarks (``synthetic_imagenet``, ``synthetic_tokens``) and the
reference's synthetic regression data (reference trainer/task.py:36-37:
x = linspace(-1, 1, 100), y = 2x + 10 + 0.33*N(0,1)).

Batches are moved to the compute device by a background prefetch thread
(pinned host memory + non-blocking copies on a side stream) when
``prefetch_to_device`` is used.
"""
from __future__ import annotations

import queue
import threading

import numpy as np
import torch


def _to_tensor(x):
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x))


def _map_struct(fn, x):
    if isinstance(x, dict):
        return {k: _map_struct(fn, v) for k, v in x.items()}
    if isinstance(x, (tuple, list)):
        return type(x)(_map_struct(fn, v) for v in x)
    return fn(x)


def _first(x):
    if isinstance(x, dict):
        return _first(next(iter(x.values())))
    if isinstance(x, (tuple, list)):
        return _first(x[0])
    return x


class Dataset:
    def __init__(self, gen_fn, length=None):
        self._gen_fn = gen_fn
        self._length = length

    def __iter__(self):
        return iter(self._gen_fn())

    def __len__(self):
        if self._length is None:
            raise TypeError("dataset length is unknown")
        return self._length

    def cardinality(self):
        return -1 if self._length is None else self._length

    # ------------------------------------------------------------ sources
    @staticmethod
    def from_tensor_slices(tensors):
        t = _map_struct(_to_tensor, tensors)
        n = _first(t).shape[0]

        def gen():
            for i in range(n):
                yield _map_struct(lambda a: a[i], t)
        ds = Dataset(gen, n)
        ds._slices = t
        return ds

    @staticmethod
    def from_generator(fn, length=None):
        return Dataset(fn, length)

    @staticmethod
    def range(*args):
        r = range(*args)
        return Dataset(lambda: (torch.tensor(i) for i in r), len(r))

    # ------------------------------------------------------------ transforms
    def map(self, fn):
        src = self

        def gen():
            for e in src:
                yield fn(*e) if isinstance(e, tuple) else fn(e)
        return Dataset(gen, self._length)

    def batch(self, batch_size, drop_remainder=False):
        src = self
        slices = getattr(self, "_slices", None)
        n = self._length

        if slices is not None and n is not None:  # vectorized batching of in-memory slices
            def gen():
                stop = n - (n % batch_size) if drop_remainder else n
                for s in range(0, stop, batch_size):
                    yield _map_struct(lambda a: a[s:s + batch_size], slices)
            ln = n // batch_size if drop_remainder else (n + batch_size - 1) // batch_size
            return Dataset(gen, ln)

        def gen():
            buf = []
            for e in src:
                buf.append(e)
                if len(buf) == batch_size:
                    yield _stack(buf)
                    buf = []
            if buf and not drop_remainder:
                yield _stack(buf)
        ln = None if n is None else (n // batch_size if drop_remainder else (n + batch_size - 1) // batch_size)
        return Dataset(gen, ln)

    def shuffle(self, buffer_size, seed=None, reshuffle_each_iteration=True):
        src = self
        slices = getattr(self, "_slices", None)
        rng = np.random.default_rng(seed)
        if slices is not None:
            n = self._length

            def gen():
                perm = torch.as_tensor(rng.permutation(n))
                for i in perm:
                    yield _map_struct(lambda a: a[int(i)], slices)
            ds = Dataset(gen, n)
            return ds

        def gen():
            buf = []
            for e in src:
                buf.append(e)
                if len(buf) >= buffer_size:
                    j = int(rng.integers(len(buf)))
                    buf[j], buf[-1] = buf[-1], buf[j]
                    yield buf.pop()
            rng.shuffle(buf)
            yield from buf
        return Dataset(gen, self._length)

    def repeat(self, count=None):
        src = self

        def gen():
            i = 0
            while count is None or i < count:
                yield from src
                i += 1
        return Dataset(gen, None if count is None or self._length is None else self._length * count)

    def take(self, n):
        src = self

        def gen():
            for i, e in enumerate(src):
                if i >= n:
                    return
                yield e
        return Dataset(gen, n if self._length is None else min(n, self._length))

    def skip(self, n):
        src = self

        def gen():
            for i, e in enumerate(src):
                if i >= n:
                    yield e
        return Dataset(gen, None if self._length is None else max(0, self._length - n))

    def shard(self, num_shards, index):
        """Every num_shards-th element starting at index (tf.data shard semantics)."""
        src = self

        def gen():
            for i, e in enumerate(src):
                if i % num_shards == index:
                    yield e
        ln = None if self._length is None else (self._length - index + num_shards - 1) // num_shards
        return Dataset(gen, ln)

    def prefetch(self, buffer_size=2):
        return self.prefetch_to_device(None, buffer_size)

    def prefetch_to_device(self, device, buffer_size=2):
        src = self

        def gen():
            q = queue.Queue(maxsize=max(1, buffer_size))
            stop = object()
            dev = torch.device(device) if device is not None else None
            stream = torch.cuda.Stream(device=dev) if dev is not None and dev.type == "cuda" else None

            def worker():
                try:
                    for e in src:
                        if dev is not None:
                            def mv(a):
                                a = a.pin_memory() if dev.type == "cuda" and not a.is_cuda else a
                                return a.to(dev, non_blocking=True)
                            if stream is not None:
                                with torch.cuda.stream(stream):
                                    e = _map_struct(mv, e)
                                    ev = torch.cuda.Event()
                                    ev.record(stream)
                                q.put((e, ev))
                            else:
                                q.put((_map_struct(mv, e), None))
                        else:
                            q.put((e, None))
                finally:
                    q.put((stop, None))

            th = threading.Thread(target=worker, daemon=True)
            th.start()
            while True:
                e, ev = q.get()
                if e is stop:
                    break
                if ev is not None:
                    torch.cuda.current_stream().wait_event(ev)
                yield e
        return Dataset(gen, self._length)

    def as_numpy_iterator(self):
        for e in self:
            yield _map_struct(lambda a: a.cpu().numpy(), e)


def _stack(items):
    f = items[0]
    if isinstance(f, dict):
        return {k: _stack([i[k] for i in items]) for k in f}
    if isinstance(f, (tuple, list)):
        return type(f)(_stack([i[j] for i in items]) for j in range(len(f)))
    return torch.stack([_to_tensor(i) for i in items])


# ---------------------------------------------------------------- synthetic data
def reference_linear_data(seed=None, n=100):
    """The reference's regression data: x = linspace(-1,1,100), y = 2x + 10 + 0.33 N(0,1)."""
    rng = np.random.RandomState(seed) if seed is not None else np.random
    x = np.linspace(-1, 1, n)
    y = 2 * x + rng.randn(*x.shape) * 0.33 + 10
    return x.astype(np.float32), y.astype(np.float32)


def synthetic_imagenet(batch_size, device, image_size=224, num_classes=1000, channels_last=False, seed=0,
                       dtype=torch.float32):
    """One fixed random batch resident on the device, yielded forever (tf_cnn_benchmarks-style synthetic data)."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    shape = (batch_size, image_size, image_size, 3) if channels_last else (batch_size, 3, image_size, image_size)
    x = torch.randn(shape, generator=g).to(dtype).to(device)
    y = torch.randint(0, num_classes, (batch_size,), generator=g).to(device)

    def gen():
        while True:
            yield x, y
    return Dataset(gen, None)


def synthetic_tokens(batch_size, seq_len, vocab_size, device, seed=0, mlm=False):
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    ids = torch.randint(0, vocab_size, (batch_size, seq_len), generator=g).to(device)
    labels = torch.randint(0, vocab_size, (batch_size, seq_len), generator=g).to(device)

    def gen():
        while True:
            yield ids, labels
    return Dataset(gen, None)
