"""MobileNetV2 backbone — the reference FeatureExtractor's default
(models/retinanet.py:274 builds mobilenet.mobilenet_retinanet(80,
'mobilenet224_1.0'); models/mobilenet.py:43-72 wraps
keras.applications.mobilenet_v2.MobileNetV2(input_tensor=Input((None, None,
3)), alpha, include_top=False, weights=None) and taps 'block_5_add',
'block_12_add', 'out_relu' as C3, C4, C5 for retinanet.retinanet).

keras-applications MobileNetV2 (third-party, unpinned; restated):
  Conv1: ZeroPadding2D(correct_pad) -> Conv2D(32, 3, stride 2, valid, no
         bias) -> BN -> ReLU6
  _inverted_res_block(expansion t, filters f, stride s) x 17
         (block 0: no expand); expand 1x1 (t * in) -> BN -> ReLU6;
         [ZeroPadding2D(correct_pad) if s == 2] DepthwiseConv2D(3, s,
         'same' if s == 1 else 'valid') -> BN -> ReLU6; project 1x1 (f) -> BN;
         + input when in == f and s == 1
  Conv_1 1x1 (1280) -> BN -> ReLU6 ('out_relu')
  Every BN: epsilon 1e-3, momentum 0.999, TRAINABLE (training mode in the
  train step: batch statistics; the moving averages at inference).
correct_pad on an Input((None, None, 3)) tensor (unknown size) pads
(top 0, bottom 1, left 0, right 1) for every stride-2 3x3.

Weights: glorot_uniform conv / depthwise kernels (weights=None), BN gamma 1,
beta 0, moving mean 0, variance 1.
"""
from torch import nn

from fpnmt.layers import BatchNormalization, Conv2D, DepthwiseConv2D

# (expansion, filters, stride) of block_0 .. block_16 (alpha = 1.0)
BLOCKS = [(1, 16, 1), (6, 24, 2), (6, 24, 1), (6, 32, 2), (6, 32, 1), (6, 32, 1), (6, 64, 2), (6, 64, 1), (6, 64, 1),
          (6, 64, 1), (6, 96, 1), (6, 96, 1), (6, 96, 1), (6, 160, 2), (6, 160, 1), (6, 160, 1), (6, 320, 1)]
STRIDE2_PADS = (0, 1, 0, 1)
TAPS = (5, 12)  # block_5_add, block_12_add
ALLOWED = ["mobilenet128", "mobilenet160", "mobilenet192", "mobilenet224"]


def _make_divisible(v, divisor=8, min_value=None):
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def _bn(c):
    return BatchNormalization(c, epsilon=1e-3, momentum=0.999)


class InvertedResBlock(nn.Module):
    def __init__(self, cin, expansion, filters, stride, alpha=1.0, block_id=0, init=None):
        super().__init__()
        pw = _make_divisible(int(filters * alpha), 8)
        self.stride = stride
        self.has_expand = block_id != 0
        mid = expansion * cin
        if self.has_expand:
            self.expand = Conv2D(cin, mid, 1, padding="same", use_bias=False, init=init)
            self.expand_bn = _bn(mid)
        else:
            mid = cin
        self.depthwise = DepthwiseConv2D(mid, 3, stride, STRIDE2_PADS if stride == 2 else (1, 1, 1, 1), init=init)
        self.depthwise_bn = _bn(mid)
        self.project = Conv2D(mid, pw, 1, padding="same", use_bias=False, init=init)
        self.project_bn = _bn(pw)
        self.add = cin == pw and stride == 1
        self.out_channels = pw

    def forward(self, x, training):
        inp = x
        if self.has_expand:
            x = self.expand_bn(self.expand(x), training, "relu6")
        x = self.depthwise_bn(self.depthwise(x), training, "relu6")
        return self.project_bn(self.project(x), training, None, residual=inp if self.add else None)


class MobileNetV2Backbone(nn.Module):
    """Returns [None, C3, C4, C5] (block_5_add, block_12_add, out_relu) like
    the reference's tapped keras Model; ``bn_training`` selects the BN mode
    (set by FeatureExtractor from the call's training flag)."""

    def __init__(self, alpha=1.0, init=None):
        super().__init__()
        first = _make_divisible(32 * alpha, 8)
        self.conv1 = Conv2D(3, first, 3, strides=2, padding=STRIDE2_PADS, use_bias=False, init=init, name="Conv1")
        self.bn_conv1 = _bn(first)
        blocks, cin = [], first
        for bi, (t, f, s) in enumerate(BLOCKS):
            b = InvertedResBlock(cin, t, f, s, alpha, bi, init=init)
            blocks.append(b)
            cin = b.out_channels
        self.blocks = nn.ModuleList(blocks)
        last = _make_divisible(1280 * alpha, 8) if alpha > 1.0 else 1280
        self.conv_1 = Conv2D(cin, last, 1, padding="same", use_bias=False, init=init, name="Conv_1")
        self.conv_1_bn = _bn(last)
        self.out_channels = [0, blocks[TAPS[0]].out_channels, blocks[TAPS[1]].out_channels, last]
        self.bn_training = True

    def forward(self, x):
        tr = self.bn_training
        x = self.bn_conv1(self.conv1(x), tr, "relu6")
        taps = []
        for bi, b in enumerate(self.blocks):
            x = b(x, tr)
            if bi in TAPS:
                taps.append(x)
        x = self.conv_1_bn(self.conv_1(x), tr, "relu6")
        return [None, taps[0], taps[1], x]

    def segments(self):
        """[(fn, parameter-name prefixes)] for x -> C3, C3 -> C4, C4 -> C5 (see
        ResNetBackbone.segments)."""
        def run(lo, hi, x):
            for b in self.blocks[lo:hi]:
                x = b(x, self.bn_training)
            return x

        def c3(x):
            return run(0, TAPS[0] + 1, self.bn_conv1(self.conv1(x), self.bn_training, "relu6"))

        def c5(x):
            return self.conv_1_bn(self.conv_1(run(TAPS[1] + 1, len(self.blocks), x)), self.bn_training, "relu6")
        return [(c3, ["conv1.", "bn_conv1."] + [f"blocks.{i}." for i in range(TAPS[0] + 1)]),
                (lambda x: run(TAPS[0] + 1, TAPS[1] + 1, x), [f"blocks.{i}." for i in range(TAPS[0] + 1, TAPS[1] + 1)]),
                (c5, [f"blocks.{i}." for i in range(TAPS[1] + 1, len(self.blocks))] + ["conv_1.", "conv_1_bn."])]


def validate(backbone):
    name, _, alpha = backbone.partition("_")
    if name not in ALLOWED:
        raise ValueError("Backbone ('{}') not in allowed backbones ({}).".format(backbone, ALLOWED))
    return float(alpha or 1.0)


def mobilenet_retinanet(num_classes, backbone="mobilenet224_1.0", inputs=None, modifier=None, **kwargs):
    """models/mobilenet.py:43-72: a RetinaNet over MobileNetV2's taps."""
    from . import retinanet
    alpha = validate(backbone)
    init = kwargs.pop("init", None)  # backbone, FPN and submodels draw from one generator
    net = MobileNetV2Backbone(alpha, init=init)
    if modifier:
        net = modifier(net)
    return retinanet.retinanet(inputs=inputs, backbone_layers=net, num_classes=num_classes, init=init, **kwargs)
