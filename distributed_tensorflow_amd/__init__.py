"""distributed_tensorflow_amd — an MI355X-native distributed training framework.

A re-design (not a port) of the capabilities of yaokeepmoving/distributed_tensorflow
(TF1 parameter-server training of a linear model, Supervisor checkpointing,
SavedModel export, REST serving, PS auto-shutdown) plus the tf.distribute /
Keras surface named in BASELINE.json, built on PyTorch-ROCm tensors,
hand-written gfx950 HIP kernels and RCCL over xGMI.
"""
__version__ = "0.1.0"

import os as _os

# One process drives up to five HIP streams per GPU (main / data-gradient chain, weight-gradient side stream,
# gradient-bucket communication stream, RCCL's internal stream, per-bucket update stream). With HIP's default of 4
# hardware queues per process two of them share an in-order AQL queue, and a cross-stream wait on one blocks the
# other: measured on MI355X (ResNet-50 b256, single rank on the forced collective path) the side stream landed on
# the main stream's queue and the step went from 22.8 to 25.7 ms (profiles/r3_hw_queues.txt). 8 queues keep every
# stream on its own queue; set before the HIP runtime initialises (importing torch does not), a user's own setting
# wins.
_os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

from .variables import Variable, ParamArena  # noqa: F401
