"""Process-wide forward hooks and the optimizer wrapper (reference: smart_compress/util/pytorch/
hooks.py:15-53).

``register_global_hooks(compress_fn, hparams, layer_types)`` installs (when
``hparams.compress_forward``) one global module forward hook that replaces the tensor output of
every selected layer by ``compress_fn(output, tag="forward_hook")`` and returns the handles.
``wrap_optimizer`` is implemented in ``optimizer`` (it builds the fused ``OptimLP``) and is
re-exported here under the reference's module path.
"""

from typing import List

import torch
import torch.nn as nn
from torch.nn.modules.module import register_module_forward_hook
from torch.utils.hooks import RemovableHandle

from .layers import DEFAULT_LAYER_TYPES, is_valid_layer_type
from .optimizer import wrap_optimizer

__all__ = ["register_global_hooks", "wrap_optimizer"]

HOOK_TAG = "forward_hook"


def _output_compressor(compress_fn, layer_types):
    def hook(module: nn.Module, inputs, output):
        # only plain tensor outputs of the selected layer types are replaced (hooks.py:40-44)
        if type(output) is torch.Tensor and is_valid_layer_type(module, layer_types=layer_types):
            return compress_fn(output, tag=HOOK_TAG)
        return None

    return hook


def register_global_hooks(compress_fn, hparams,
                          layer_types=DEFAULT_LAYER_TYPES) -> List[RemovableHandle]:
    if not hparams.compress_forward:
        return []
    return [register_module_forward_hook(_output_compressor(compress_fn, layer_types))]
