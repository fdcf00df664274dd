"""Layer-type selection for the compression callers (reference: util/pytorch/quantization.py:8-129,
161-180: the ``*_LAYERS`` tables, ``LAYERS_TYPES``, ``DEFAULT_LAYER_TYPES``,
``is_valid_layer_type``). Kept in its own module here; ``quantization`` re-exports it."""

from torch import nn

SEQUENTIAL_LAYERS = [nn.Sequential, nn.ModuleList]
DICT_LAYERS = [nn.ModuleDict]
CONV_LAYERS = [nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.ConvTranspose1d, nn.ConvTranspose2d,
               nn.ConvTranspose3d, nn.Unfold, nn.Fold]
POOL_LAYERS = [nn.MaxPool1d, nn.MaxPool2d, nn.MaxPool3d, nn.MaxUnpool1d, nn.MaxUnpool2d,
               nn.MaxUnpool3d, nn.AvgPool1d, nn.AvgPool2d, nn.AvgPool3d, nn.FractionalMaxPool2d,
               nn.LPPool1d, nn.LPPool2d, nn.AdaptiveMaxPool1d, nn.AdaptiveMaxPool2d,
               nn.AdaptiveAvgPool2d, nn.AdaptiveAvgPool1d, nn.AdaptiveMaxPool3d,
               nn.AdaptiveAvgPool3d]
PAD_LAYERS = [nn.ReflectionPad1d, nn.ReflectionPad2d, nn.ReplicationPad1d, nn.ReplicationPad2d,
              nn.ZeroPad2d, nn.ConstantPad1d, nn.ConstantPad2d, nn.ConstantPad3d]
ACTIVATION_LAYERS = [nn.ELU, nn.Hardshrink, nn.Hardtanh, nn.LeakyReLU, nn.LogSigmoid, nn.PReLU,
                     nn.ReLU, nn.ReLU6, nn.RReLU, nn.SELU, nn.Sigmoid, nn.Softplus, nn.Softshrink,
                     nn.Softsign, nn.Tanh, nn.Tanhshrink, nn.Threshold, nn.Softmin, nn.Softmax,
                     nn.Softmax2d, nn.LogSoftmax]
NORM_LAYERS = [nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d, nn.GroupNorm, nn.InstanceNorm1d,
               nn.InstanceNorm2d, nn.InstanceNorm3d, nn.LayerNorm, nn.LocalResponseNorm]
LINEAR_LAYERS = [nn.Linear, nn.Bilinear]
DROPOUT_LAYERS = [nn.Dropout, nn.Dropout2d, nn.Dropout3d, nn.AlphaDropout]
LOSS_LAYERS = [nn.L1Loss, nn.MSELoss, nn.CrossEntropyLoss, nn.NLLLoss, nn.PoissonNLLLoss,
               nn.KLDivLoss, nn.BCELoss, nn.BCEWithLogitsLoss, nn.MarginRankingLoss,
               nn.HingeEmbeddingLoss, nn.MultiLabelMarginLoss, nn.SmoothL1Loss,
               nn.SoftMarginLoss, nn.MultiLabelSoftMarginLoss, nn.MultiMarginLoss,
               nn.TripletMarginLoss]

LAYERS_TYPES = {
    "conv": CONV_LAYERS,
    "linear": LINEAR_LAYERS,
    "pool": POOL_LAYERS,
    "pad": PAD_LAYERS,
    "activation": ACTIVATION_LAYERS,
    "normalization": NORM_LAYERS,
    "dropout": DROPOUT_LAYERS,
    "loss": LOSS_LAYERS,
}

DEFAULT_LAYER_TYPES = ["conv", "linear", "pool", "normalization"]

# module paths whose classes always count (the reference's own model zoo, containers, activations)
_ALWAYS_VALID_PATHS = ("smart_compress.models.pytorch.", "torch.nn.modules.container.",
                       "torch.nn.modules.activation.")


def is_valid_layer_type(module, layer_types=DEFAULT_LAYER_TYPES) -> bool:
    """quantization.py:164-180: the module's exact type is in the selected tables, or its class
    lives in one of the always-valid module paths."""
    selected = []
    for layer_type in layer_types:
        assert layer_type in LAYERS_TYPES, layer_type
        selected += LAYERS_TYPES[layer_type]
    module_type = type(module)
    if module_type in selected:
        return True
    type_name = str(module_type)
    return any(p in type_name for p in _ALWAYS_VALID_PATHS)
