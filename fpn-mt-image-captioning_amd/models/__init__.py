"""Model modules mirroring the reference's models/ package (retinanet,
transformer, coattention, resnet). Backbone selection replaces the
reference's Keras Backbone registry (models/__init__.py:5-63)."""

BACKBONES = ("resnet50", "resnet101", "resnet152", "mobilenet128", "mobilenet160", "mobilenet192", "mobilenet224")


def backbone(backbone_name):
    if backbone_name.split("_")[0] not in BACKBONES:
        raise NotImplementedError("Backbone class for  '{}' not implemented.".format(backbone_name))
    return backbone_name
