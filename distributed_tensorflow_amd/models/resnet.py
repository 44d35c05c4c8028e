"""ResNet-50 v1.5 (the headline benchmark model of BASELINE.json), channels-last.

Every conv is a fused ``ConvBN`` (conv -> training BatchNorm with statistics
from the conv epilogue -> [+residual] -> [ReLU]) so each bottleneck block is
three implicit-GEMM launches plus three single-pass normalisation launches.
v1.5: the stride of a down-sampling bottleneck sits on its 3x3 conv.

Input: f32 NCHW images (the usual host/dataset layout); the first op moves them
to bf16 NHWC with the 3 colour channels zero-padded to 8 (the implicit-GEMM
gather reads 16-B channel chunks). conv1's filter therefore has 8 input
channels; the 5 padded channels see only zeros (their weights receive zero
gradient and never influence the output).
"""
from __future__ import annotations


import torch

from .. import ops
from ..keras import layers as KL
from ..keras.models import Model

from ..ops.conv import ResidualGradLink

RES_LINK = True
FUSE_STEM = True  # stem BN + ReLU + MaxPool as one pass
S2D_STEM = True  # stem conv over the 2x2 space-to-depth image
STAGES = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3), 26: (2, 2, 2, 2)}


class Bottleneck(KL.Layer):
    def __init__(self, width, stride=1, project=False, bn_momentum=0.9, **kw):
        super().__init__(**kw)
        m = dict(momentum=bn_momentum, epsilon=1e-5)
        self.c1 = KL.ConvBN(width, 1, 1, relu=True, **m)
        self.c2 = KL.ConvBN(width, 3, stride, relu=True, **m)
        self.c3 = KL.ConvBN(width * 4, 1, 1, relu=True, **m)
        self.proj = KL.ConvBN(width * 4, 1, stride, relu=False, **m) if project else None

    def call(self, x, training=None):
        # The projection runs after c1 so that its backward runs before c1's: the shortcut gradient is then
        # parked in `link` and c1's dgrad epilogue adds into it (no separate add of the two gradients of x).
        link = ResidualGradLink() if (training and RES_LINK and torch.is_grad_enabled()) else None
        y = self.c1(x, training=training, link=link, role="acc")
        if self.proj is not None:
            sc = self.proj(x, training=training, link=link, role="proj")
            y = self.c2(y, training=training)
            return self.c3(y, residual=sc, training=training)
        y = self.c2(y, training=training)
        return self.c3(y, residual=x, training=training, link=link, role="res")


class ResNet(Model):
    def __init__(self, depth=50, num_classes=1000, width=64, bn_momentum=0.9, in_pad=8, **kw):
        super().__init__(name=kw.pop("name", f"resnet{depth}"), **kw)
        self.in_pad = in_pad
        self.num_classes = num_classes
        self.stem = KL.ConvBN(width, 7, 2, relu=True, momentum=bn_momentum)
        self.pool = KL.MaxPooling2D(3, 2, padding="same")
        blocks = []
        for si, n in enumerate(STAGES[depth]):
            w = width * (2 ** si)
            for bi in range(n):
                stride = 2 if (bi == 0 and si > 0) else 1
                blocks.append(Bottleneck(w, stride, project=(bi == 0), bn_momentum=bn_momentum))
        self.blocks = blocks
        self.gap = KL.GlobalAveragePooling2D()
        self.fc = KL.Dense(num_classes, kernel_initializer="glorot_uniform")

    def call(self, images, training=None):
        nchw = images.dim() == 4 and images.shape[1] in (1, 3) and images.shape[-1] not in (1, 3, self.in_pad)
        if nchw and FUSE_STEM and S2D_STEM and images.is_cuda and images.shape[2] % 2 == 0 \
                and images.shape[3] % 2 == 0:
            # 7x7/2 stem as a 4x4/1 conv over the 2x2 space-to-depth image, BN + ReLU + MaxPool fused
            N, _, H, W = images.shape
            if not self.stem.built:  # the 7x7 filter keeps its [64, 7, 7, in_pad] shape (checkpoints)
                self.stem.build((N, H, W, self.in_pad))
                self.stem.built = True
            xs = ops.image_to_s2d_bf16(images if images.is_floating_point() else images.float())
            x = self.stem(xs, training=training, pool=self.pool, s2d=True)
        else:
            if nchw:
                x = ops.image_to_nhwc_bf16(images.float() if not images.is_floating_point() else images,
                                           self.in_pad)
            else:
                x = images
            if FUSE_STEM:  # BN + ReLU + MaxPool in one pass (ops.conv_bn_maxpool)
                x = self.stem(x, training=training, pool=self.pool)
            else:
                x = self.stem(x, training=training)
                x = self.pool(x)
        for b in self.blocks:
            x = b(x, training=training)
        x = self.gap(x)
        return self.fc(x)


def ResNet50(num_classes=1000, **kw):
    return ResNet(50, num_classes, **kw)


def ResNet101(num_classes=1000, **kw):
    return ResNet(101, num_classes, **kw)


def ResNet152(num_classes=1000, **kw):
    return ResNet(152, num_classes, **kw)
