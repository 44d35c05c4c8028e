"""tf.train surface: checkpoints, Saver, ManagedTraining (Supervisor), ClusterSpec/Server, TF1 optimizers."""
from .checkpoint import (Saver, Checkpoint, CheckpointManager, latest_checkpoint, get_checkpoint_state,  # noqa
                         list_variables, load_variable, save_tensors, load_tensors)
from ..keras.optimizers import (GradientDescentOptimizer, AdadeltaOptimizer, AdagradOptimizer, AdamOptimizer,  # noqa
                                FtrlOptimizer, RMSPropOptimizer, MomentumOptimizer)
from ..parallel.cluster_resolver import ClusterSpec  # noqa
from .supervisor import ManagedTraining  # noqa
from .monitored import (MonitoredTrainingSession, SessionRunHook, StopAtStepHook, CheckpointSaverHook,  # noqa
                        StepCounterHook, SummarySaverHook, LoggingTensorHook, NanTensorHook)
