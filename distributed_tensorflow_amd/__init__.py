"""distributed_tensorflow_amd — an MI355X-native distributed training framework.

A re-design (not a port) of the capabilities of yaokeepmoving/distributed_tensorflow
(TF1 parameter-server training of a linear model, Supervisor checkpointing,
SavedModel export, REST serving, PS auto-shutdown) plus the tf.distribute /
Keras surface named in BASELINE.json, built on PyTorch-ROCm tensors,
hand-written gfx950 HIP kernels and RCCL over xGMI.
"""
__version__ = "0.1.0"

# Streams per process: main (data-gradient chain), the weight-gradient side stream (which also issues the bucket
# collectives), RCCL's internal stream (+ the per-bucket update stream of DTF_OVERLAP_UPDATE, the PS push copy
# stream on the parameter-server path): within HIP's default of 4 hardware queues per process, with the side stream
# created before RCCL's (ops._util.reserve_streams). GPU_MAX_HW_QUEUES is left to the user / the box default.

from .variables import Variable, ParamArena  # noqa: F401
