"""Reference-parity trainer: ``python -m distributed_tensorflow_amd.cli.train [--flags]``.

The equivalent of ``python -m trainer.task`` (reference trainer/task.py + auto_stop_ps/task.py):
same flags and defaults, TF_CONFIG decides the mode:
  * empty/absent TF_CONFIG -> standalone per-sample training of y = w*x + b (batch 1, max_epochs x 100
    steps), ``Epoch: i, loss: ...`` every ``checkpoint_period`` epochs, summaries ``loss`` and
    ``training/hptuning/metric``, final ``w``/``b`` print;
  * ``ps`` task -> parameter-server daemon that exits once every trainer reported done
    (auto_stop_ps behaviour; ``--ps_join_forever`` keeps the plain ``server.join()`` behaviour);
  * ``worker`` / ``master`` (or ``chief``) -> asynchronous PS training with Supervisor-style chief
    init/restore + timed checkpoints (``--save_model_secs``, 60), chief-only summaries, and the chief
    exporting ``saved_model_path/model_version`` BEFORE signalling done.
Differences from the reference, on purpose: seeded data (``--seed``), errors
exit non-zero, and the chief's export cannot race the PS shutdown.
"""
from __future__ import annotations

import datetime
import os
import sys

import numpy as np
import torch

from ..utils import flags

flags.DEFINE_integer("max_epochs", 10, "Number of epochs (of 100 per-sample steps) to run.")
flags.DEFINE_string("checkpoint_path", "./checkpoint/", "The checkpoint directory")
flags.DEFINE_string("output_path", "./tensorboard/", "indicates training output")
flags.DEFINE_integer("checkpoint_period", 1, "Number of epochs between eval/summary points.")
flags.DEFINE_string("model_path", "./model/", "The model directory")
flags.DEFINE_float("learning_rate", 0.01, "Initial learning rate.")
flags.DEFINE_string("optimizer", "sgd", "Optimizer to train")
flags.DEFINE_string("saved_model_path", "./saved_model/", "The path of the saved model")
flags.DEFINE_integer("model_version", 1, "The version of the model")
flags.DEFINE_integer("seed", -1, "Data seed (-1: unseeded like the reference)")
flags.DEFINE_string("device", "cpu", "Compute device for the linear model (cpu, cuda:0, /GPU:0; auto = the task's "
                                     "GPU when one is visible, else the CPU)")
flags.DEFINE_integer("save_model_secs", 60, "Chief checkpoint interval in seconds")
flags.DEFINE_boolean("export_standalone", False, "Also export a SavedModel in standalone mode")
flags.DEFINE_boolean("ps_join_forever", False, "PS never exits (trainer/task.py server.join())")
flags.DEFINE_string("partitioner", "round_robin", "PS variable placement: round_robin | balanced")
FLAGS = flags.FLAGS


def _data():
    from ..data import reference_linear_data
    return reference_linear_data(None if FLAGS.seed < 0 else FLAGS.seed)


def _optimizer():
    from ..keras import optimizers
    print("Use the optimizer: {}".format(FLAGS.optimizer))
    try:
        return optimizers.get(FLAGS.optimizer, FLAGS.learning_rate, tf1=True)
    except ValueError:
        print("Unknow optimizer: {}, exit now".format(FLAGS.optimizer))
        sys.exit(1)


def _export(model):
    from .. import saved_model
    path = os.path.join(FLAGS.saved_model_path, str(FLAGS.model_version))
    saved_model.save(model, path)
    print("Exported SavedModel to {}".format(path))
    return path


def _step(model, loss_fn, x, y):
    pred = model(x)
    loss = loss_fn(y, pred)
    loss.backward()
    return loss


def _device():
    from .. import context
    return context.default_device() if FLAGS.device == "auto" else context.parse_device(FLAGS.device)


def _graph_def(model, opt):
    """The training GraphDef (reference FileWriter(output_path, sess.graph), trainer/task.py:80,228)."""
    from ..saved_model.graph_def import model_graph
    return model_graph(model, training=True, optimizer=opt)[0].graph_def()


def _meta_graph(model, opt):
    """model.ckpt-N.meta next to every checkpoint (the Supervisor's Saver writes it in TF)."""
    from ..saved_model.graph_def import training_meta_graph
    return training_meta_graph(model, optimizer=opt)


def run_standalone():
    from .. import context, summary
    from ..models.linear import LinearRegression
    train_X, train_Y = _data()
    start = datetime.datetime.now()
    opt = _optimizer()
    dev = _device()
    with context.device(dev):
        model = LinearRegression()
    loss_fn = LinearRegression.reference_loss()
    arena = opt.arena_for(model.trainable_variables)
    print("Save tensorboard files into: {}".format(FLAGS.output_path))
    writer = summary.FileWriter(FLAGS.output_path, graph=_graph_def(model, opt))
    X = torch.as_tensor(train_X, device=dev).reshape(-1, 1, 1)
    Y = torch.as_tensor(train_Y, device=dev).reshape(-1, 1, 1)
    print("Run training with epoch number: {}".format(FLAGS.max_epochs))
    for i in range(FLAGS.max_epochs):
        for j in range(X.shape[0]):
            _step(model, loss_fn, X[j], Y[j])
            opt.apply_arena(arena, zero_grad=True)
        if i % FLAGS.checkpoint_period == 0:
            with torch.no_grad():
                loss = float(loss_fn(Y[0], model(X[0])))
            step = opt.host_iterations()
            writer.add_summary({"loss": loss, "training/hptuning/metric": loss}, step)
            print("Epoch: {}, loss: {}".format(i, loss))
    writer.close()
    end = datetime.datetime.now()
    print("[{}] End of standalone training.".format(end - start))
    print("Get the model, w: {}, b: {}".format(float(model.weight), float(model.bias)))
    if FLAGS.export_standalone:
        _export(model)
    return model


def run_distributed(resolver):
    from .. import context, summary
    from ..models.linear import LinearRegression
    from ..parallel.fault import injector
    from ..parallel.parameter_server import ParameterServerStrategy
    from ..train.checkpoint import Saver
    from ..train.supervisor import ManagedTraining
    from ..variables import Variable
    train_X, train_Y = _data()
    start = datetime.datetime.now()
    opt = _optimizer()
    dev = _device()
    strategy = ParameterServerStrategy(resolver, variable_partitioner=FLAGS.partitioner, device=dev)
    print("PS data plane: {}".format(strategy.transport), flush=True)
    is_chief = strategy.is_chief
    with strategy.scope():
        model = LinearRegression()
    loss_fn = LinearRegression.reference_loss()
    arena = opt.arena_for(strategy.order_variables(model.trainable_variables))
    global_step = Variable(0, trainable=False, name="global_step", dtype=torch.int64)

    def before_save():  # checkpoint the PS state (the Saver runs on the PS shards in TF)
        strategy.pull()
        global_step.assign(strategy.global_step())

    saver = Saver({"weight": model.weight, "bias": model.bias, "global_step": global_step},
                  meta_graph_def=lambda: _meta_graph(model, opt))
    mt = ManagedTraining(is_chief, FLAGS.checkpoint_path, saver, global_step=lambda: strategy.global_step(),
                         save_model_secs=FLAGS.save_model_secs, before_save=before_save)
    with mt:
        if is_chief and mt.restored_from:
            strategy.kv.add("global_step", int(global_step.item()) - strategy.global_step())
            print("Restored from {} at global_step {}".format(mt.restored_from, int(global_step.item())))
        strategy.setup_model(model, arena, opt)
        print("Save tensorboard files into: {}".format(FLAGS.output_path))
        writer = summary.FileWriter(FLAGS.output_path, graph=_graph_def(model, opt)) if is_chief else None
        X = torch.as_tensor(train_X, device=dev).reshape(-1, 1, 1)
        Y = torch.as_tensor(train_Y, device=dev).reshape(-1, 1, 1)
        print("Run training with epoch number: {}".format(FLAGS.max_epochs))
        faults = injector()
        for i in range(FLAGS.max_epochs):
            for j in range(X.shape[0]):
                _step(model, loss_fn, X[j], Y[j])
                strategy.apply_gradients(opt, arena)
                faults.on_step(i * X.shape[0] + j + 1)
            if i % FLAGS.checkpoint_period == 0:
                with torch.no_grad():
                    loss = float(loss_fn(Y[0], model(X[0])))
                step = strategy.global_step()
                print("Epoch: {}, loss: {}".format(i, loss))
                if writer is not None:
                    writer.add_summary({"loss": loss}, step)
        if writer is not None:
            writer.close()
        end = datetime.datetime.now()
        print("[{}] End of distributed training.".format(end - start))
        strategy.pull()
        global_step.assign(strategy.global_step())
        if is_chief:
            _export(model)  # export first, then report done (no PS-shutdown race)
    strategy.shutdown()
    print("Get the model, w: {}, b: {}".format(float(model.weight), float(model.bias)))
    return model


def main(argv=None):
    FLAGS(argv if argv is not None else sys.argv[1:], known_only=True)
    from ..parallel.cluster_resolver import TFConfigClusterResolver
    if os.environ.get("TF_CONFIG", "") == "":
        run_standalone()
        return 0
    r = TFConfigClusterResolver()
    if r.is_ps:
        from ..parallel.parameter_server import ParameterServer
        ps = ParameterServer(r, device=_device())
        print("PS data plane: {}".format(ps.transport), flush=True)
        ps.serve(forever=bool(FLAGS.ps_join_forever))  # forever: plain server.join() (no auto-stop)
        print("PS applied {} updates".format(ps.applies))
        print("PS exits after all workers done")
        return 0
    if r.task_type in ("worker", "master", "chief"):
        run_distributed(r)
        return 0
    print("Unknown task type: {}".format(r.task_type))
    return 1


if __name__ == "__main__":
    sys.exit(main())
