"""ResNet-50/101/152 backbone with keras-resnet semantics (the reference's
models/resnet.py:78-112 wraps keras_resnet.models.ResNet{50,101,152}(inputs,
include_top=False, freeze_bn=True) and feeds ``outputs[1:]`` = C3, C4, C5 to
retinanet.retinanet).

keras-resnet (third-party, not vendored in the reference; semantics restated):
  stem: ZeroPadding2D(3) -> Conv2D(64, 7x7, stride 2, no bias) -> frozen BN
        (eps 1e-5) -> ReLU -> MaxPooling2D(3x3, stride 2, 'same')
  bottleneck_2d(filters, stage, block): stride = 2 on block 0 of stages 1..3,
        applied on the FIRST 1x1 conv (2a) and the 1x1 projection shortcut;
        2a 1x1 -> BN -> ReLU -> ZeroPadding2D(1) -> 2b 3x3 -> BN -> ReLU ->
        2c 1x1 (4x filters) -> BN; shortcut = 1x1 conv + BN on block 0 else x;
        y = ReLU(2c + shortcut).
  Every BN is frozen (inference mode, non-trainable) and folded into the conv
  (scale into the compute-weight copy, shift into the epilogue bias).
"""
from torch import nn

import fpnmt
from fpnmt import ops
from fpnmt.layers import Conv2D

BLOCKS = {"resnet50": [3, 4, 6, 3], "resnet101": [3, 4, 23, 3], "resnet152": [3, 8, 36, 3]}


def _conv(cin, cout, k, stride=1, padding="valid", activation=None, init=None, name=None):
    return Conv2D(cin, cout, k, strides=stride, padding=padding, activation=activation, use_bias=False,
                  kernel_initializer="he_normal", frozen_bn=True, init=init, name=name)


class Bottleneck2D(nn.Module):
    def __init__(self, cin, filters, stage, block, init=None):
        super().__init__()
        stride = 1 if (block != 0 or stage == 0) else 2
        self.block = block
        self.conv2a = _conv(cin, filters, 1, stride, activation="relu", init=init)
        self.conv2b = _conv(filters, filters, 3, 1, padding=(1, 1, 1, 1), activation="relu", init=init)
        self.conv2c = _conv(filters, filters * 4, 1, 1, activation="relu", init=init)  # relu after + shortcut
        self.shortcut = _conv(cin, filters * 4, 1, stride, init=init) if block == 0 else None

    def forward(self, x):
        if self.shortcut is None and fpnmt.config.fuse_bottleneck:
            y = ops.bottleneck_fused(self, x)  # inference: one launch, intermediates on chip
            if y is not None:
                return y
        if self.shortcut is not None:
            ops.expect_consumers(x, 2)  # 2a and the shortcut: dx summed in their bwd-data launches
        sc = self.shortcut(x) if self.shortcut is not None else x
        if fpnmt.config.fuse_conv_chains:  # 2a/2b outputs feed only the next conv
            return ops.conv_chain([self.conv2a, self.conv2b, self.conv2c], x, residual=sc)
        y = self.conv2b(self.conv2a(x))
        return self.conv2c(y, residual=sc)


class ResNetBackbone(nn.Module):
    """Returns [C2, C3, C4, C5] like keras_resnet.models.ResNet(include_top=False)."""

    def __init__(self, backbone="resnet50", init=None):
        super().__init__()
        if backbone not in BLOCKS:
            raise ValueError("Backbone ('{}') not in allowed backbones ({}).".format(backbone, list(BLOCKS)))
        self.backbone = backbone
        self.conv1 = _conv(3, 64, 7, 2, padding=(3, 3, 3, 3), activation="relu", init=init, name="conv1")
        stages = []
        cin, features = 64, 64
        for stage_id, iterations in enumerate(BLOCKS[backbone]):
            blocks = []
            for block_id in range(iterations):
                blocks.append(Bottleneck2D(cin, features, stage_id, block_id, init=init))
                cin = features * 4
            stages.append(nn.Sequential(*blocks))
            features *= 2
        self.stages = nn.ModuleList(stages)
        self.out_channels = [256, 512, 1024, 2048]

    def forward(self, x):
        x = self.conv1(x)
        x = ops.max_pool2d_same(x, 3, 2)
        outs = []
        for st in self.stages:
            x = st(x)
            outs.append(x)
        return outs

    def segments(self):
        """[(fn, parameter-name prefixes)] for x -> C3, C3 -> C4, C4 -> C5: the
        data-parallel engine runs the backward one segment at a time and
        all-reduces each segment's gradients while the next one computes."""
        def c3(x):
            x = ops.max_pool2d_same(self.conv1(x), 3, 2)
            return self.stages[1](self.stages[0](x))
        return [(c3, ["conv1.", "stages.0.", "stages.1."]), (self.stages[2], ["stages.2."]),
                (self.stages[3], ["stages.3."])]


def ResNet50(inputs=None, include_top=False, freeze_bn=True, init=None):
    return ResNetBackbone("resnet50", init=init)


def ResNet101(inputs=None, include_top=False, freeze_bn=True, init=None):
    return ResNetBackbone("resnet101", init=init)


def ResNet152(inputs=None, include_top=False, freeze_bn=True, init=None):
    return ResNetBackbone("resnet152", init=init)


def resnet_retinanet(num_classes, backbone="resnet50", inputs=None, modifier=None, **kwargs):
    """Reference models/resnet.py:78-112: a RetinaNet over the ResNet's C3..C5."""
    from . import retinanet
    if backbone not in BLOCKS:
        raise ValueError("Backbone ('{}') is invalid.".format(backbone))
    init = kwargs.pop("init", None)  # backbone, FPN and submodels draw from one generator
    resnet = ResNetBackbone(backbone, init=init)
    if modifier:
        resnet = modifier(resnet)
    return retinanet.retinanet(inputs=inputs, backbone_layers=resnet, num_classes=num_classes, init=init, **kwargs)


def resnet50_retinanet(num_classes, inputs=None, **kwargs):
    return resnet_retinanet(num_classes=num_classes, backbone="resnet50", inputs=inputs, **kwargs)


def resnet101_retinanet(num_classes, inputs=None, **kwargs):
    return resnet_retinanet(num_classes=num_classes, backbone="resnet101", inputs=inputs, **kwargs)


def resnet152_retinanet(num_classes, inputs=None, **kwargs):
    return resnet_retinanet(num_classes=num_classes, backbone="resnet152", inputs=inputs, **kwargs)
