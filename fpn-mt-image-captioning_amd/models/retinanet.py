"""RetinaNet FPN feature extractor (reference: models/retinanet.py).

Same call surface as the reference module, as torch Modules over NHWC tensors:
default_classification_model / default_regression_model (:25-102),
__create_pyramid_features (:105-141), default_submodels (:144-159),
retinanet (:217-263) and FeatureExtractor (:266-307).

Every convolution is the fpnmt implicit-GEMM MFMA kernel; the FPN top-down
upsample + add pair is ONE fused sweep (fpnmt_fpn_topdown_fwd/bwd).
"""
import torch
from torch import nn

from common.common_definitions import (ACTIVATION, BACKBONE, KERNEL_INITIALIZER, LEAKY_ALPHA, N_CONV_SUBMODULE,
                                       NUM_OF_ANCHORS, NUM_OF_CLASSES, NUM_OF_RETINANET_FILTERS, d_model)
import fpnmt
from fpnmt import ops
from fpnmt.layers import Conv2D
from .coattention import CoAttention_CNN


class _Submodel(nn.Module):
    """Two 3x3 'same' ReLU convs, N(0, 0.01) kernels, zero bias (retinanet.py:54-62 / 94-100)."""

    def __init__(self, pyramid_feature_size, feature_size, prefix, init=None):
        super().__init__()
        self.convs = nn.ModuleList([
            Conv2D(pyramid_feature_size if i == 0 else feature_size, feature_size, 3, padding="same",
                   activation="relu", kernel_initializer="normal", std=0.01, init=init,
                   name="{}_{}".format(prefix, i))
            for i in range(2)])

    def forward(self, x):
        for c in self.convs:
            x = c(x)
        return x


def default_classification_model(num_classes, num_anchors, pyramid_feature_size=256, prior_probability=0.01,
                                 classification_feature_size=256, name="classification_submodel", init=None):
    return _Submodel(pyramid_feature_size, classification_feature_size, "pyramid_classification", init=init)


def default_regression_model(num_values, num_anchors, pyramid_feature_size=256, regression_feature_size=256,
                             name="regression_submodel", init=None):
    return _Submodel(pyramid_feature_size, regression_feature_size, "pyramid_regression", init=init)


class PyramidFeatures(nn.Module):
    """FPN of retinanet.py:105-141 (P6/P7 by 3x3 ReLU conv + 2x2 max pool, as
    the reference does, not the paper's stride-2 convs)."""

    def __init__(self, c3, c4, c5, feature_size=256, init=None):
        super().__init__()
        f = feature_size
        self.C5_reduced = Conv2D(c5, f, 1, padding="same", init=init, name="C5_reduced")
        self.P5 = Conv2D(f, f, 3, padding="same", activation="relu", init=init, name="P5")
        self.C4_reduced = Conv2D(c4, f, 1, padding="same", init=init, name="C4_reduced")
        self.P4 = Conv2D(f, f, 3, padding="same", activation="relu", init=init, name="P4")
        self.C3_reduced = Conv2D(c3, f, 1, padding="same", init=init, name="C3_reduced")
        self.P3 = Conv2D(f, f, 3, padding="same", activation="relu", init=init, name="P3")
        self.P6_conv = Conv2D(f, f, 3, padding="same", activation="relu", init=init, name="P6_conv")
        self.P7_conv = Conv2D(f, f, 3, padding="same", activation="relu", init=init, name="P7_conv")

    def forward(self, C3, C4, C5):
        ps = self.to_p6(C3, C4, C5)
        return ps + [self.p7(ps[3])]

    def to_p6(self, C3, C4, C5):
        """[P3, P4, P5, P6] (retinanet.py:105-136)."""
        # C3 / C4 also feed the next backbone stage's projection block, p5f
        # feeds P5, the top-down sweep and P6: their gradients are summed in
        # the consumers' bwd-data launches (ops.expect_consumers)
        ops.expect_consumers(C3, 1)
        ops.expect_consumers(C4, 1)
        p5f = self.C5_reduced(C5)
        ops.expect_consumers(p5f, 3)
        P5 = self.P5(p5f)
        lat4 = self.C4_reduced(C4)
        lat3 = self.C3_reduced(C3)
        # P4_merged = lat4 + up(P5f); P3_merged = lat3 + up(P4_merged) — one kernel
        p4m, p3m = ops.FpnTopDownFn.apply(p5f, lat4, lat3)
        P4 = self.P4(p4m)
        P3 = self.P3(p3m)
        P6 = ops.max_pool2d_valid(self.P6_conv(p5f))
        return [P3, P4, P5, P6]

    def p7(self, P6):
        """P7 from P6 (retinanet.py:137-139); P6 is also a pyramid output, read
        by the heads: P7_conv's gradient joins theirs in the bwd-data launches."""
        ops.expect_consumers(P6, 1)
        return ops.max_pool2d_valid(self.P7_conv(P6))


def __create_pyramid_features(C3, C4, C5, feature_size=256):
    """Functional form of the reference builder: creates fresh FPN layers (as
    Keras does at graph build time) and applies them."""
    m = PyramidFeatures(C3.shape[-1], C4.shape[-1], C5.shape[-1], feature_size).to(C3.device)
    return m(C3, C4, C5)


def default_submodels(num_classes, num_anchors, init=None):
    return [("regression", default_regression_model(4, num_anchors, init=init)),
            ("classification", default_classification_model(num_classes, num_anchors, init=init))]


class RetinaNet(nn.Module):
    """retinanet(): backbone -> FPN -> per-level submodels. forward returns, per
    submodel, the list of per-level outputs (the reference concatenates them
    along axis 1, which only type-checks for equal widths and is never
    evaluated on the captioning path)."""

    def __init__(self, backbone, num_classes, num_anchors=None, submodels=None, init=None):
        super().__init__()
        self.backbone = backbone
        ch = backbone.out_channels
        self.fpn = PyramidFeatures(ch[1], ch[2], ch[3], init=init)
        subs = submodels if submodels is not None else default_submodels(num_classes, num_anchors or NUM_OF_ANCHORS,
                                                                          init=init)
        self.submodel_names = [n for n, _ in subs]
        self.submodels = nn.ModuleList([m for _, m in subs])

    def pyramid(self, x):
        C2, C3, C4, C5 = self.backbone(x)
        return self.fpn(C3, C4, C5)

    def forward(self, x):
        feats = self.pyramid(ops.cast(x, fpnmt.compute_dtype()))
        return [[m(f) for f in feats] for m in self.submodels]


def retinanet(inputs=None, backbone_layers=None, num_classes=NUM_OF_CLASSES, num_anchors=None,
              create_pyramid_features=None, submodels=None, name="retinanet", init=None):
    if num_anchors is None:
        num_anchors = NUM_OF_ANCHORS
    return RetinaNet(backbone_layers, num_classes, num_anchors, submodels, init=init)


def _make_backbone_retinanet(backbone, init=None):
    if backbone.startswith("resnet"):
        from . import resnet
        return resnet.resnet_retinanet(NUM_OF_CLASSES, backbone=backbone, init=init)
    if backbone.startswith("mobilenet"):  # the reference default (retinanet.py:274)
        from . import mobilenet
        return mobilenet.mobilenet_retinanet(NUM_OF_CLASSES, backbone=backbone, init=init)
    raise ValueError("Backbone ('{}') is not supported by this build (resnet50, resnet101, resnet152, "
                     "mobilenet{{128,160,192,224}}_<alpha>).".format(backbone))


class FeatureExtractor(nn.Module):
    """Feature extractor feeding the multi-view transformer (retinanet.py:266-307).
    backbone: 'resnet50' | 'resnet101' | 'resnet152' (frozen BN, the
    BASELINE configurations) or 'mobilenet224_1.0' (the reference default).

    Per pyramid level (ONE shared weight set for all five, :297-301):
    regression/classification submodels (2 ReLU convs each, tapped at
    layers[N_CONV_SUBMODULE]), heads conv3x3->1 and conv3x3->256 (linear,
    he_normal, :287-288), CoAttention_CNN (:291), conv3x3 256 leaky (:292),
    MaxPooling2D (:293), conv3x3 d_model leaky (:294).
    Returns 5 NHWC tensors (B, h/2, w/2, d_model) for P3..P7.
    """

    def __init__(self, retinanet_weight_path=None, backbone=None, init=None):
        super().__init__()
        backbone = backbone or BACKBONE
        self.retinanet_model = _make_backbone_retinanet(backbone, init=init)
        if retinanet_weight_path is not None:
            raise NotImplementedError("Keras h5 retinanet weights cannot be read in this build; restore an fpnmt "
                                      "safetensors checkpoint with fpnmt.checkpoint.Checkpoint(...).restore(path)")
        assert N_CONV_SUBMODULE == 2
        F = NUM_OF_RETINANET_FILTERS
        self.regression = Conv2D(F, 1, 3, padding="same", kernel_initializer=KERNEL_INITIALIZER, init=init,
                                 name="regression_head")
        self.classification = Conv2D(F, F, 3, padding="same", kernel_initializer=KERNEL_INITIALIZER, init=init,
                                     name="classification_head")
        self.coattention = CoAttention_CNN()
        self.post_conv = Conv2D(F, F, 3, padding="same", activation=ACTIVATION, act_alpha=LEAKY_ALPHA,
                                kernel_initializer=KERNEL_INITIALIZER, init=init, name="coatt_conv")
        self.out_conv = Conv2D(F, d_model, 3, padding="same", activation=ACTIVATION, act_alpha=LEAKY_ALPHA,
                               kernel_initializer=KERNEL_INITIALIZER, init=init, name="coatt_out")

    def _heads(self, features):
        """regression(reg_sub(f)), classification(cls_sub(f)): the submodels'
        ReLU convs only feed the next conv, so each head is one conv chain."""
        reg_sub, cls_sub = self.retinanet_model.submodels[0], self.retinanet_model.submodels[1]
        for f in (features if isinstance(features, (list, tuple)) else [features]):
            ops.expect_consumers(f, 2)  # both head chains read every level
        if fpnmt.config.fuse_conv_chains:
            return (ops.conv_chain(list(reg_sub.convs) + [self.regression], features),
                    ops.conv_chain(list(cls_sub.convs) + [self.classification], features))
        return self.regression(reg_sub(features)), self.classification(cls_sub(features))

    def level(self, feature):
        regression, classification = self._heads(feature)
        out = self.coattention(regression, classification)
        out = self.post_conv(out)
        out = ops.max_pool2d_valid(out)
        return self.out_conv(out)

    def levels(self, features):
        """level() over every pyramid level at once: each shared conv is one
        grouped launch for all levels (fpnmt_conv2d_*_grouped)."""
        regression, classification = self._heads(list(features))
        out = [self.coattention(r, c) for r, c in zip(regression, classification)]
        out = self.post_conv(out)
        out = [ops.max_pool2d_valid(o) for o in out]
        return self.out_conv(out)

    # P7_conv runs in the heads' stage (staged(): P7 from P6's leaf)
    HEAD_PREFIXES = ["regression.", "classification.", "post_conv.", "out_conv.", "retinanet_model.submodels.",
                     "retinanet_model.fpn.P7_conv."]

    def stage_prefixes(self):
        """Parameter-name prefixes of the staged backward (see staged()), in
        backward order: heads, FPN, backbone C4->C5, C3->C4, input->C3."""
        bb = "retinanet_model.backbone."
        segs = self.retinanet_model.backbone.segments()
        return [self.HEAD_PREFIXES, ["retinanet_model.fpn."]] + [[bb + p for p in segs[i][1]]
                                                                  for i in reversed(range(len(segs)))]

    def set_training(self, training=None):
        bb = self.retinanet_model.backbone
        if hasattr(bb, "bn_training"):
            bb.bn_training = self.training if training is None else bool(training)

    def staged(self, inp, training=None):
        """forward() cut at the backbone taps and the pyramid: returns
        (outputs, stages), stages in BACKWARD order as (outputs, leaves,
        parameter prefixes): the stage's output tensors, the detached leaves
        that the next stage consumed in their place (whose .grad is the
        stage's incoming gradient; None for the heads, whose outputs the
        caller detaches), and its parameters. Each stage's backward is then a
        separate step whose parameters' gradients are final when it ends (the
        data-parallel engine all-reduces them while the next stage computes)."""
        self.set_training(training)
        x = ops.cast(inp, fpnmt.compute_dtype())
        rm = self.retinanet_model
        segs = rm.backbone.segments()
        leaf = lambda t: t.detach().requires_grad_(t.requires_grad)  # noqa: E731
        seg_out, cs = [], []
        cur = x
        for fn, _ in segs:
            y = fn(cur)
            seg_out.append(y)
            cur = leaf(y)
            cs.append(cur)
        ps = rm.fpn.to_p6(*cs)
        pl = [leaf(t) for t in ps]
        # P7 from P6's leaf, in the heads' stage: P6's gradient (heads + P7_conv)
        # is complete when the FPN stage starts, with no autograd sum
        outs = self.levels(pl + [rm.fpn.p7(pl[3])])
        pref = self.stage_prefixes()
        stages = [(list(outs), None, pref[0]), (list(ps), pl, pref[1])]
        for j, i in enumerate(reversed(range(len(segs)))):
            stages.append(([seg_out[i]], [cs[i]], pref[2 + j]))
        return outs, stages

    def forward(self, inp, training=None):
        """training: BatchNormalization mode of a trainable-BN backbone
        (MobileNetV2; Keras propagates the train step's training=True to the
        backbone, predict() runs it with False). None: the module's mode."""
        self.set_training(training)
        x = ops.cast(inp, fpnmt.compute_dtype())
        features = self.retinanet_model.pyramid(x)
        return self.levels(features)

    call = forward
