"""MonitoredTrainingSession + hooks (the reference's dead MTS path, trainer/task.py:178-213, made real),
and the profiler's CPU-safe pieces (roctx ranges are no-ops without a profiler attached)."""
import os

import torch

from distributed_tensorflow_amd import profiler, train
from distributed_tensorflow_amd.summary import read_events
from distributed_tensorflow_amd.variables import Variable


def _linear_step(w, b, x, y, lr=0.05):
    pred = x * w + b
    loss = ((y - pred) ** 2).sum()
    gw, gb = torch.autograd.grad(loss, [w, b])
    with torch.no_grad():
        w -= lr * gw
        b -= lr * gb
    return {"loss": float(loss)}


def test_monitored_session_stop_checkpoint_resume(tmp_path):
    d = str(tmp_path / "ckpt")
    w = Variable(0.0, name="weight")
    b = Variable(0.0, name="bias")
    gs = Variable(0, trainable=False, name="global_step", dtype=torch.int64)
    xs = torch.linspace(-1, 1, 20)
    ys = 2 * xs + 10
    hook = train.LoggingTensorHook({"loss": "loss"}, every_n_iter=10)
    with train.MonitoredTrainingSession(True, d, variables={"weight": w, "bias": b, "global_step": gs},
                                        hooks=[train.StopAtStepHook(last_step=30), hook],
                                        save_checkpoint_steps=10, log_step_count_steps=5) as sess:
        i = 0
        while not sess.should_stop():
            sess.run(_linear_step, w, b, xs[i % 20], ys[i % 20])
            i += 1
    assert i == 30 and int(gs.item()) == 30 and len(hook.lines) == 3
    assert train.latest_checkpoint(d).endswith("model.ckpt-30")
    ev = [e for f in os.listdir(d) if f.startswith("events") for e in read_events(os.path.join(d, f))]
    assert any("global_step/sec" in str(e) for e in ev)
    w2 = Variable(0.0, name="weight")
    b2 = Variable(0.0, name="bias")
    gs2 = Variable(0, trainable=False, name="global_step", dtype=torch.int64)
    with train.MonitoredTrainingSession(True, d, variables={"weight": w2, "bias": b2, "global_step": gs2},
                                        hooks=[train.StopAtStepHook(num_steps=5)]) as sess:
        assert sess.restored_from is not None and sess.global_step == 30
        assert float(w2) == float(w)
        while not sess.should_stop():
            sess.run(_linear_step, w2, b2, xs[0], ys[0])
    assert sess.global_step == 35


def test_nan_hook_and_profiler_cpu():
    import pytest
    h = train.NanTensorHook()
    with train.MonitoredTrainingSession(hooks=[h]) as sess:
        with pytest.raises(FloatingPointError):
            sess.run(lambda: {"loss": float("nan")})
    with profiler.range("fwd"):
        profiler.mark("hello")
    st = profiler.StepStats(items_per_step=256, unit="images/sec", every=2)
    for _ in range(5):
        st.step(0)
    assert len(st.history) == 2 and st.history[0]["images/sec"] > 0
