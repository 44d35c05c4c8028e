"""Keras callbacks.

Covers the reference's lifecycle hooks: the periodic eval/summary every
``checkpoint_period`` epochs (reference trainer/task.py:89-96), the chief's
timed checkpoints + restore (Supervisor, :215-223 -> ``ModelCheckpoint`` /
``BackupAndRestore``) and ``StopAtStepHook`` (:178, -> ``StopAtStep``).
"""
from __future__ import annotations

import math
import os
import time


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_model(self, model):
        self.model = model

    def set_params(self, params):
        self.params = params

    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass
    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_train_batch_begin(self, batch, logs=None): pass
    def on_train_batch_end(self, batch, logs=None): pass
    def on_test_begin(self, logs=None): pass
    def on_test_end(self, logs=None): pass
    def on_test_batch_end(self, batch, logs=None): pass
    def on_predict_batch_end(self, batch, logs=None): pass


class CallbackList(Callback):
    def __init__(self, callbacks=None, model=None, params=None):
        super().__init__()
        self.callbacks = list(callbacks or [])
        for c in self.callbacks:
            if model is not None:
                c.set_model(model)
            if params is not None:
                c.set_params(params)

    def __getattribute__(self, name):
        if name.startswith("on_"):
            cbs = object.__getattribute__(self, "callbacks")

            def fan(*a, **k):
                for c in cbs:
                    getattr(c, name)(*a, **k)
            return fan
        return object.__getattribute__(self, name)


class History(Callback):
    def __init__(self):
        super().__init__()
        self.history = {}
        self.epoch = []

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


class ProgbarLogger(Callback):
    def __init__(self, verbose=1, rank_prefix=""):
        super().__init__()
        self.verbose, self.prefix = verbose, rank_prefix
        self._t0 = None

    def on_epoch_begin(self, epoch, logs=None):
        self._t0 = time.time()

    def on_epoch_end(self, epoch, logs=None):
        if self.verbose:
            items = " - ".join(f"{k}: {v:.4f}" for k, v in (logs or {}).items() if isinstance(v, float))
            print(f"{self.prefix}Epoch {epoch + 1}/{self.params.get('epochs', '?')} - "
                  f"{time.time() - self._t0:.2f}s - {items}", flush=True)


class LambdaCallback(Callback):
    def __init__(self, **fns):
        super().__init__()
        for k, f in fns.items():
            setattr(self, k, f)


class StopAtStep(Callback):
    """StopAtStepHook analogue: stop once the optimizer's iteration count reaches last_step."""

    def __init__(self, last_step):
        super().__init__()
        self.last_step = int(last_step)

    def on_train_batch_end(self, batch, logs=None):
        if self.model.optimizer.host_iterations() >= self.last_step:
            self.model.stop_training = True


class TerminateOnNaN(Callback):
    def on_train_batch_end(self, batch, logs=None):
        l = (logs or {}).get("loss")
        if l is not None and (math.isnan(l) or math.isinf(l)):
            print(f"Batch {batch}: invalid loss, terminating training")
            self.model.stop_training = True


class EarlyStopping(Callback):
    def __init__(self, monitor="val_loss", min_delta=0.0, patience=0, mode="auto", restore_best_weights=False):
        super().__init__()
        self.monitor, self.min_delta, self.patience = monitor, abs(min_delta), patience
        self.mode = "max" if (mode == "max" or (mode == "auto" and "acc" in monitor)) else "min"
        self.restore = restore_best_weights
        self.best, self.wait, self.best_weights = None, 0, None

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None:
            return
        better = self.best is None or (cur < self.best - self.min_delta if self.mode == "min"
                                       else cur > self.best + self.min_delta)
        if better:
            self.best, self.wait = cur, 0
            if self.restore:
                self.best_weights = self.model.get_weights()
        else:
            self.wait += 1
            if self.wait > self.patience:
                self.model.stop_training = True
                if self.restore and self.best_weights is not None:
                    self.model.set_weights(self.best_weights)


class LearningRateScheduler(Callback):
    def __init__(self, schedule, verbose=0):
        super().__init__()
        self.schedule, self.verbose = schedule, verbose

    def on_epoch_begin(self, epoch, logs=None):
        opt = self.model.optimizer
        lr = self.schedule(epoch, opt._lr_value())
        opt.learning_rate = float(lr)


def _sync_sharded_state(model):
    """Sharded (ZeRO-1) optimizer slots are current only on their owner: gather them before a save."""
    s = getattr(model, "distribute_strategy", None)
    if s is not None and hasattr(s, "sync_optimizer_state") and getattr(model, "optimizer", None) is not None:
        s.sync_optimizer_state(model.optimizer)


def _agree(model, flag, every=None):
    """A wall-clock save trigger must fire on every replica together when the save is collective. every=1 forces
    the exchange (epoch / training end: a pending time-based save is never skipped between exchange points)."""
    s = getattr(model, "distribute_strategy", None)
    if s is None or not hasattr(s, "agree"):
        return flag
    return s.agree(flag) if every is None else s.agree(flag, every=every)


class ModelCheckpoint(Callback):
    """Save a tensor-bundle checkpoint every epoch, or every `save_freq` batches, or every `save_secs`
    seconds (the Supervisor's save_model_secs=60 of reference trainer/task.py:223)."""

    def __init__(self, filepath, save_freq="epoch", save_secs=None, save_weights_only=True, max_to_keep=5,
                 verbose=0, agree_every=16):
        """agree_every: under ZeRO-1 the save_secs trigger is exchanged between replicas every `agree_every` batches
        (strategy.agree) and always at epoch and training end."""
        super().__init__()
        self.filepath, self.save_freq, self.save_secs, self.verbose = filepath, save_freq, save_secs, verbose
        self.agree_every = agree_every
        self.max_to_keep = max_to_keep
        self._last = time.time()
        self._mgr = None

    def _manager(self):
        if self._mgr is None:
            from ..train.checkpoint import Checkpoint, CheckpointManager
            ck = Checkpoint(model=self.model, optimizer=self.model.optimizer)
            d = self.filepath if os.path.splitext(self.filepath)[1] == "" else os.path.dirname(self.filepath)
            self._mgr = CheckpointManager(ck, d or ".", max_to_keep=self.max_to_keep)
        return self._mgr

    def _save(self):
        _sync_sharded_state(self.model)  # collective under ZeRO-1: every replica reaches it
        if not getattr(self.model, "_is_chief", True):
            return
        p = self._manager().save(checkpoint_number=self.model.optimizer.host_iterations())
        if self.verbose:
            print(f"saved checkpoint {p}")
        self._last = time.time()

    def on_train_batch_end(self, batch, logs=None):
        if self.save_secs is not None and _agree(self.model, time.time() - self._last >= self.save_secs,
                                                 self.agree_every):
            self._save()
        elif isinstance(self.save_freq, int) and (batch + 1) % self.save_freq == 0:
            self._save()

    def on_epoch_end(self, epoch, logs=None):
        if self.save_freq == "epoch" and self.save_secs is None:
            self._save()
        elif self.save_secs is not None and _agree(self.model, time.time() - self._last >= self.save_secs, 1):
            self._save()

    def on_train_end(self, logs=None):
        if self.save_secs is not None and _agree(self.model, time.time() - self._last >= self.save_secs, 1):
            self._save()


class BackupAndRestore(Callback):
    """Fault tolerance: restore model+optimizer+epoch from backup_dir on train begin, back up every epoch.
    Unlike the reference (which restarts its epoch loop at 0 after a restore, Appendix A.5), the epoch
    counter is restored too."""

    def __init__(self, backup_dir, save_freq="epoch", delete_checkpoint=True):
        super().__init__()
        self.backup_dir, self.save_freq, self.delete = backup_dir, save_freq, delete_checkpoint
        self._mgr = None

    def _manager(self):
        if self._mgr is None:
            from ..train.checkpoint import Checkpoint, CheckpointManager
            from ..variables import Variable
            import torch
            if not hasattr(self.model, "_ckpt_epoch"):
                self.model._ckpt_epoch = Variable(0, trainable=False, name="_ckpt_epoch", dtype=torch.int64)
            ck = Checkpoint(model=self.model, optimizer=self.model.optimizer, epoch=self.model._ckpt_epoch)
            self._mgr = CheckpointManager(ck, self.backup_dir, max_to_keep=1)
        return self._mgr

    def on_train_begin(self, logs=None):
        m = self._manager()
        if m.latest_checkpoint:
            m.checkpoint.restore(m.latest_checkpoint)
            self.model._initial_epoch = int(self.model._ckpt_epoch.item())

    def on_epoch_end(self, epoch, logs=None):
        self.model._ckpt_epoch.assign(epoch + 1)
        _sync_sharded_state(self.model)
        if getattr(self.model, "_is_chief", True):
            self._manager().save(checkpoint_number=epoch + 1)

    def on_train_end(self, logs=None):
        if self.delete and getattr(self.model, "_is_chief", True) and not getattr(self.model, "stop_training", False):
            import shutil
            shutil.rmtree(self.backup_dir, ignore_errors=True)


class TensorBoard(Callback):
    """Writes scalar summaries to a TF event file (TFRecord framing, masked CRC32C; C++ writer)."""

    def __init__(self, log_dir="./logs", update_freq="epoch", write_graph=False):
        super().__init__()
        self.log_dir, self.update_freq = log_dir, update_freq
        self._w = None

    def _writer(self):
        if self._w is None:
            from ..summary import create_file_writer
            self._w = create_file_writer(os.path.join(self.log_dir, "train"))
        return self._w

    def on_train_batch_end(self, batch, logs=None):
        if isinstance(self.update_freq, int) and (batch + 1) % self.update_freq == 0:
            step = self.model.optimizer.host_iterations()
            for k, v in (logs or {}).items():
                if isinstance(v, float):
                    self._writer().scalar(f"batch_{k}", v, step)

    def on_epoch_end(self, epoch, logs=None):
        if not getattr(self.model, "_is_chief", True):
            return
        for k, v in (logs or {}).items():
            if isinstance(v, float):
                self._writer().scalar(f"epoch_{k}", v, epoch)
        self._writer().flush()

    def on_train_end(self, logs=None):
        if self._w is not None:
            self._w.close()
