"""Op layer: every hot op dispatches to a hand-written gfx950 HIP kernel for GPU
tensors and to an explicit f32 torch reference for CPU tensors."""
from .linalg import gemm, dense, bmm, matmul, colsum  # noqa: F401
from .conv import conv2d, conv_bn, conv_bn_maxpool, image_to_nhwc_bf16, image_to_s2d_bf16, same_pads, out_size  # noqa: F401
from .norm import batch_norm, layer_norm  # noqa: F401
from .nn import (max_pool2d, global_avg_pool, relu, gelu, dropout, add, add_dropout, embedding,  # noqa: F401
                 sparse_softmax_cross_entropy, softmax, gather_rows, sort_keys)
from .optim import optim_apply  # noqa: F401
from .mha import attention, attention_packed  # noqa: F401
