"""distributed_tensorflow_amd — an MI355X-native distributed training framework.

A re-design (not a port) of the capabilities of yaokeepmoving/distributed_tensorflow
(TF1 parameter-server training of a linear model, Supervisor checkpointing,
SavedModel export, REST serving, PS auto-shutdown) plus the tf.distribute /
Keras surface named in BASELINE.json, built on PyTorch-ROCm tensors,
hand-written gfx950 HIP kernels and RCCL over xGMI.
"""
__version__ = "0.1.0"

from .variables import Variable, ParamArena  # noqa: F401
