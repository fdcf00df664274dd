"""qtorch-style float quantisation on MI355X: drop-in for
smart_compress/util/pytorch/quantization.py:131-204 (``float_quantize``, ``_get_max_value``,
``add_float_quantize_args``, ``TORCH_FLOAT_MAX`` / ``TORCH_FLOAT_EPS``).

The reference calls the un-vendored qtorch 0.2.0 ``float_quantize(x, exp, man, rounding)`` and then
turns elements equal to the format's largest finite value into +inf (``check_inf``,
quantization.py:195-199). Here both are one ``smq_float_quant_f32`` launch (8 B/elem, random word
from the counter-based RNG in registers instead of a materialised ``randint_like`` tensor).
"""

from argparse import ArgumentParser

import torch

from ... import _native as N
from .layers import (ACTIVATION_LAYERS, CONV_LAYERS, DEFAULT_LAYER_TYPES, DICT_LAYERS,  # noqa: F401
                     DROPOUT_LAYERS, LAYERS_TYPES, LINEAR_LAYERS, LOSS_LAYERS, NORM_LAYERS,
                     PAD_LAYERS, POOL_LAYERS, SEQUENTIAL_LAYERS, is_valid_layer_type)

TORCH_FLOAT_MAX = torch.tensor(torch.finfo(torch.float32).max, dtype=torch.float32)
TORCH_FLOAT_EPS = torch.tensor(torch.finfo(torch.float32).eps, dtype=torch.float32)

MAX_VALUES = dict()

_rng = None


def quant_rng() -> N.RngState:
    """Process-wide RNG stream of float_quantize (qtorch draws from torch's generator)."""
    global _rng
    if _rng is None:
        _rng = N.RngState()
    return _rng


def _get_max_value(exp: int, man: int) -> torch.Tensor:
    """Nearest-quantised FLT_MAX of the (exp, man) format, cached (quantization.py:138-150)."""
    key = (exp, man)
    if key not in MAX_VALUES:
        MAX_VALUES[key] = torch.tensor(N.lib().smq_float_quant_max_value(exp, man),
                                       dtype=torch.float32)
    return MAX_VALUES[key]


def add_float_quantize_args(parent_parser: ArgumentParser) -> ArgumentParser:
    parser = ArgumentParser(parents=[parent_parser], add_help=False)
    parser.add_argument(
        "--no_float_quantize_check_inf", action="store_false", dest="float_quantize_check_inf"
    )
    return parser


def float_quantize(x: torch.Tensor, exp: int, man: int, hparams) -> torch.Tensor:
    """Stochastic (exp, man) round trip of ``x`` (quantization.py:187-204)."""
    half_io = hparams.precision == 16
    src = x.float() if half_io else x
    N.require_device_f32(src, "float_quantize")
    src = src.contiguous()
    out = torch.empty_like(src)
    seed, offset = quant_rng().take(src.numel())
    N.check(
        N.lib().smq_float_quant_f32(
            src.data_ptr(), out.data_ptr(), src.numel(), exp, man, N.SMQ_ROUND_STOCHASTIC,
            1 if hparams.float_quantize_check_inf else 0, None, seed, offset,
            N.stream_ptr(src.device),
        ),
        "smq_float_quant_f32",
    )
    return out.half() if half_io else out
