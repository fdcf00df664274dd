"""Activation / gradient-map compression through autograd (reference:
smart_compress/util/pytorch/autograd.py:12-77).

Same contract as the reference: ``Compressor(compress_fn, forward, backward)`` is a module whose
forward runs ``compress_fn(x, ..., tag="forward_autograd")`` (a trailing
``{"batch_norm_stats": (weight, bias)}`` argument becomes keyword arguments of the codec), and whose
backward runs ``compress_fn(grad_output, tag="backward_autograd")``; either direction can be
switched off. ``register_autograd_module`` puts one shared ``Compressor`` behind the output of
every layer ``is_valid_layer_type`` selects.

Implementation note: one module-level autograd Function carries a small spec object (codec +
direction flags) instead of a Function class built per Compressor. With this package's codecs
each call is one or two launches on the caller's stream and no host synchronisation (unless
compression-ratio logging is on). When ``compress_fn`` is a ``SmartFP`` codec (the reference's
train.py:198-213 passes the codec instance itself), the forward call and a C++ autograd node whose
backward compresses the grad-map are created in one C call (csrc/torchfast.cpp,
``SmartFP._autograd_fast``): an eager step that compresses every layer is bound by the host time
of these calls, and the Python Function costs as much as the codec call in each direction. The
calls, their order and their values are the same as through the Python Function.
"""

from argparse import Namespace
from typing import Any, Callable, List, Tuple

import torch
import torch.nn as nn
from torch.autograd import Function

from .layers import is_valid_layer_type

__all__ = ["Compressor", "process_input", "register_autograd_module"]

FORWARD_TAG = "forward_autograd"
BACKWARD_TAG = "backward_autograd"


def process_input(args: List[Any]) -> Tuple[List[Any], dict]:
    """autograd.py:12-15: a trailing dict holding ``batch_norm_stats`` becomes keyword args."""
    if args and type(args[-1]) == dict and "batch_norm_stats" in args[-1]:
        return args[:-1], args[-1]
    return args, {}


class _Spec:
    __slots__ = ("codec", "forward", "backward")

    def __init__(self, codec: Callable, forward: bool, backward: bool):
        self.codec, self.forward, self.backward = codec, forward, backward


class _CodecFunction(Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, spec: _Spec, *args):
        ctx.spec = spec
        ctx.n_inputs = 2 + len(args)
        if not spec.forward:
            return x
        rest, extra = process_input(list(args))
        return spec.codec(x, *rest, **extra, tag=FORWARD_TAG)

    @staticmethod
    def backward(ctx, grad_output):
        nones = (None,) * (ctx.n_inputs - 1)
        if not ctx.spec.backward:
            return (grad_output,) + nones
        if not ctx.needs_input_grad[0]:
            return (None,) + nones
        return (ctx.spec.codec(grad_output, tag=BACKWARD_TAG),) + nones


class Compressor(nn.Module):
    def __init__(self, compress_fn, forward=True, backward=True):
        super().__init__()
        self._spec = _Spec(compress_fn, bool(forward), bool(backward))
        # the codec's C autograd path (SmartFP._autograd_fast), for the forward-compressing case
        self._fast = getattr(compress_fn, "_autograd_fast", None) if forward else None

    def compress_fn(self, x: torch.Tensor, *args):
        return _CodecFunction.apply(x, self._spec, *args)

    def forward(self, x: torch.Tensor, *args):
        fast = self._fast
        if fast is not None and not args:
            y = fast(x, self._spec.backward)
            if y is not None:
                return y
        return self.compress_fn(x, *args)


def register_autograd_module(model: nn.Module, compress_fn, hparams: Namespace):
    """autograd.py:50-77. BatchNorm2d layers hand their (weight, bias) to the codec when
    ``hparams.use_batch_norm`` is set (smart.py's BN variant)."""
    compressor = Compressor(compress_fn, forward=hparams.compress_forward,
                            backward=hparams.compress_backward)
    use_bn = bool(getattr(hparams, "use_batch_norm", False))
    from .saved import replayable

    def wrap(module: nn.Module):
        if not is_valid_layer_type(module):
            return
        inner = module.forward
        bn = use_bn and type(module) == nn.BatchNorm2d
        # PackedActivations: an in-place activation on a codec output is noted before it runs, so
        # the value it leaves is saved as that output's stream with the activation replayed
        note = getattr(compress_fn, "note_inplace", None)
        if note is not None and not replayable(module):
            note = None

        def forward(*args, **kwargs):
            if note is not None and args:
                note(module, args[0])
            y = inner(*args, **kwargs)
            if bn:
                return compressor(y, {"batch_norm_stats": (module.weight.detach(),
                                                           module.bias.detach())})
            return compressor(y)

        module.forward = forward

    return model.apply(wrap)
