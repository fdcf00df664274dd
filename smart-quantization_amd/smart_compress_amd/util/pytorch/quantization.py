"""qtorch-style float quantisation on MI355X: drop-in for
smart_compress/util/pytorch/quantization.py:131-204 (``float_quantize``, ``_get_max_value``,
``add_float_quantize_args``, ``TORCH_FLOAT_MAX`` / ``TORCH_FLOAT_EPS``).

The reference calls the un-vendored qtorch 0.2.0 ``float_quantize(x, exp, man, rounding)`` and then
turns elements equal to the format's largest finite value into +inf (``check_inf``,
quantization.py:195-199). Here both are one ``smq_float_quant`` launch (8 B/elem for fp32, random
word from the counter-based RNG in registers instead of a materialised ``randint_like`` tensor). At
precision 16 the reference's ``x.float()`` and ``.half()`` passes are fused into that launch (the
kernel reads fp16 / bf16 and writes fp16: 4 B/elem instead of five passes).

``graph_safe(True, device)`` moves the stream position of ``float_quantize`` and S2FP8 (the
process-wide ``quant_rng()``) to a device counter so that captured hipGraphs draw fresh streams.
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
_graph_safe = False


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


def graph_safe(enable: bool = True, device=None) -> None:
    """Process-wide switch for the float codecs' random stream (``quant_rng()``): device-counter
    positions (hipGraph-capturable) when enabled; back to host offsets, continuing from the device
    position, when disabled. Create the counter before capture (``device=`` or one eager call)."""
    global _graph_safe
    _graph_safe = bool(enable)
    if enable and device is not None:
        quant_rng().counter(device)
    if not enable:
        quant_rng().release_counters()


def rng_stream(n: int, device):
    """(seed, offset, offset_counter pointer or None) for a call drawing ``n`` words."""
    r = quant_rng()
    if _graph_safe:
        return r.seed, 0, r.counter(device).data_ptr()
    seed, offset = r.take(n)
    return seed, offset, None


def float_quantize(x: torch.Tensor, exp: int, man: int, hparams) -> torch.Tensor:
    """Stochastic (exp, man) round trip of ``x`` (quantization.py:187-204). Precision 16: ``x``
    (fp32 / fp16 / bf16 / fp64) is quantised as ``x.float()`` and returned as fp16. Precision 32:
    fp32 in, fp32 out; fp64 in, fp64 out (the quantised fp32 rounding of each element: qtorch
    0.2.0's kernel reads ``data_ptr<float>()`` and raises on fp64, so this is its dtype-generic
    extension, include/smq.h SMQ_DTYPE_F64)."""
    half_io = hparams.precision == 16
    N.require_supported(x, "float_quantize")
    f64 = x.dtype == torch.float64
    if half_io:
        if x.dtype not in N.DTYPE_CODES and not f64:
            raise NotImplementedError(f"float_quantize: dtype {x.dtype} is not supported")
    elif x.dtype != torch.float32 and not f64:
        raise NotImplementedError(
            f"float_quantize: dtype {x.dtype} at precision 32 is not supported (float32/float64)")
    src = x.contiguous()
    out_dt = torch.float16 if half_io else (torch.float64 if f64 else torch.float32)
    out = torch.empty_like(src, dtype=out_dt)
    code_in = N.SMQ_DTYPE_F64 if f64 else N.DTYPE_CODES[src.dtype]
    code_out = {torch.float16: N.SMQ_DTYPE_F16, torch.float32: N.SMQ_DTYPE_F32,
                torch.float64: N.SMQ_DTYPE_F64}[out_dt]
    n = src.numel()
    if n == 0:
        return out
    if N.on_cpu(src):  # the library's host path, host RNG offsets
        seed, offset = quant_rng().take(n)
        N.check(N.lib().smq_cpu_float_quant(
            src.data_ptr(), code_in, out.data_ptr(), code_out, n, exp, man, N.SMQ_ROUND_STOCHASTIC,
            1 if hparams.float_quantize_check_inf else 0, None, seed, offset, N.cpu_threads()),
            "smq_cpu_float_quant")
        return out
    global _fq
    if _fq is None:
        _fq = N.lib().smq_float_quant
    seed, offset, ctr = rng_stream(n, src.device)
    rc = _fq(src.data_ptr(), code_in, out.data_ptr(), code_out, n, exp, man, N.SMQ_ROUND_STOCHASTIC,
             1 if hparams.float_quantize_check_inf else 0, None, seed, offset, ctr,
             N.stream_ptr(src.device))
    if rc:
        N.check(rc, "smq_float_quant")
    return out


_fq = None  # the bound C entry point, resolved on first use
