"""S2FP8 codec: drop-in for smart_compress/compress/s2fp8.py:11-48.

Reference algorithm (per tensor): L = log2|x| with zeros as 0; mu = mean(L), m = max(L);
alpha = 15 / (m - mu), beta = -alpha * mu; Y = |x|^alpha * 2^beta; T = E5M2 stochastic
float_quantize(Y) (+ check_inf); y = (T * 2^-beta)^(1/alpha) * sign(x). Logged as 8 bits per element
plus 64 bits of per-tensor overhead (s2fp8.py:29).

On MI355X this is ``smq_s2fp8_roundtrip``. fp32 tensors up to 4M elements run as ONE launch: every
workgroup holds its chunk in registers, publishes the chunk's log2-domain (sum, max) partial,
gathers all partials, reduces them in a fixed order, derives alpha, beta, evaluates the 131
possible inverse powers into an LDS table, and transforms, quantises and inverts its registers.
Larger tensors (and precision 16) take a statistics launch (one partial per workgroup) and an
apply launch that does the same reduce / derive / table per workgroup; both shapes give the same
bytes.

Precision 16 (quantization.py:187-204's half branch) keeps the reference's dtypes: fp16 / bf16
inputs run the statistics and the forward transform in their own type, float_quantize returns half,
the inverse power runs in half; the result is fp16 for fp16 inputs and fp32 for fp32 / bf16 inputs
(torch's promotion of ``... * signs``).
"""

from argparse import ArgumentParser

import torch

from .. import _native as N
from ..util.pytorch import quantization as _q
from ..util.pytorch.quantization import add_float_quantize_args
from .base import CompressionAlgorithmBase


class S2FP8(CompressionAlgorithmBase):
    @staticmethod
    def add_argparse_args(parent_parser: ArgumentParser) -> ArgumentParser:
        return ArgumentParser(
            parents=[add_float_quantize_args(CompressionAlgorithmBase.add_argparse_args(parent_parser))],
            add_help=False,
        )

    def graph_safe(self, enable: bool = True, device=None):
        """hipGraph-capturable random stream (process-wide, see quantization.graph_safe)."""
        _q.graph_safe(enable, device)
        return self

    _fn = None  # the bound C entry point and its workspace size, resolved on first use
    _ws_bytes = 0

    def __call__(self, tensor: torch.Tensor, tag: str = None, **_):
        hp = self.hparams
        if hp.measure_compression_ratio:  # (log_size returns at once otherwise)
            self.log_ratio(tag, tensor.numel(), 32, 8, overhead=64)
        if tensor.is_cuda and tensor.dtype is torch.float32 and hp.precision != 16:
            # no autograd op runs on this path (a fresh output the library writes), so no
            # grad-mode switch: torch.no_grad costs ~1.5 us of the ~13 us eager call at C4
            return self._call_device_f32(tensor)
        return self._call(tensor)

    @torch.no_grad()
    def _call(self, tensor: torch.Tensor) -> torch.Tensor:
        """Everything but the fp32 device hot path, under torch.no_grad as s2fp8.py:27."""
        hp = self.hparams
        precision = 16 if hp.precision == 16 else 32
        N.require_supported(tensor, "S2FP8")
        if tensor.dtype == torch.float64:
            return self._call_f64(tensor, precision)
        if precision == 32:
            if tensor.dtype != torch.float32:
                raise NotImplementedError(
                    f"S2FP8: dtype {tensor.dtype} at precision 32 is not supported "
                    "(float32/float64)")
            out_dtype = torch.float32
        else:
            if tensor.dtype not in (torch.float32, torch.float16, torch.bfloat16):
                raise NotImplementedError(f"S2FP8: dtype {tensor.dtype} is not supported")
            out_dtype = torch.float16 if tensor.dtype == torch.float16 else torch.float32
        x = tensor.contiguous()
        y = torch.empty_like(x, dtype=out_dtype)
        n = x.numel()
        if n == 0:
            return y
        if N.on_cpu(x):  # the library's host path, host RNG offsets
            seed, offset = _q.quant_rng().take(n)
            N.check(N.lib().smq_cpu_s2fp8_roundtrip(
                x.data_ptr(), N.DTYPE_CODES[x.dtype], y.data_ptr(), n, precision,
                1 if hp.float_quantize_check_inf else 0, None, seed, offset, None, None, 0, 0,
                N.cpu_threads()), "smq_cpu_s2fp8_roundtrip")
            return y
        fn = S2FP8._fn
        if fn is None:
            lib = N.lib()
            S2FP8._ws_bytes = lib.smq_s2fp8_workspace_bytes(1)  # the same for every n
            fn = S2FP8._fn = lib.smq_s2fp8_roundtrip
        dev = x.device
        st = N.stream_ptr(dev)
        ws = N.workspace("s2fp8", dev, S2FP8._ws_bytes, st)
        seed, offset, ctr = _q.rng_stream(n, dev)
        rc = fn(x.data_ptr(), N.DTYPE_CODES[x.dtype], y.data_ptr(), n, precision,
                1 if hp.float_quantize_check_inf else 0, None, seed, offset, ctr, None,
                ws.data_ptr(), ws.numel(), st)
        if rc:
            N.check(rc, "smq_s2fp8_roundtrip")
        return y


    _ws_get = None

    def _call_device_f32(self, tensor: torch.Tensor) -> torch.Tensor:
        """The eager hot path (an fp32 device tensor at precision 32): at BERT-hidden size (C4) the
        host enqueue is as long as the launch. Host offsets: one C call on the tensor
        (csrc/torchfast.cpp: allocation, stream, workspace, stream position, launch); graph-safe
        streams or no binding: the same call with its per-call Python trimmed — a C-level stream
        query, one lookup in the bounded per-(device, stream) workspace table
        (_native.workspace), the fast-call binding."""
        T = N._torch_fast if N._torch_fast_tried else N.torch_fast()
        if T is not None and not _q._graph_safe:
            get = S2FP8._ws_get
            if get is None:
                get = S2FP8._ws_get = N.ws_getter("s2fp8")
            y = T.s2fp8(tensor, self.hparams.float_quantize_check_inf, _q.quant_rng().__dict__, get)
            if y is not None:
                return y
        x = tensor if tensor.is_contiguous() else tensor.detach().contiguous()
        y = torch.empty_like(x, requires_grad=False)
        n = x.numel()
        if n == 0:
            return y
        fn = S2FP8._fn
        if fn is None:
            lib = N.lib()
            S2FP8._ws_bytes = lib.smq_s2fp8_workspace_bytes(1)  # the same for every n
            fn = S2FP8._fn = lib.smq_s2fp8_roundtrip
        dev = x.get_device()
        st = N.raw_stream(dev)
        ws = N._ws.get(("s2fp8", dev, st))  # the bounded workspace table's hit path, inlined
        if ws is None:
            ws = N.workspace("s2fp8", x.device, S2FP8._ws_bytes, st)
        seed, offset, ctr = _q.rng_stream(n, x.device)
        fast = N._fast if N._fast_tried else N.fast()
        if fast is not None:  # the fast-call binding: no ctypes argument conversion (~4 us)
            rc = fast.s2fp8_roundtrip(x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, 32,
                                      1 if self.hparams.float_quantize_check_inf else 0, seed,
                                      offset, ctr, ws.data_ptr(), ws.numel(), st)
        else:
            rc = fn(x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, 32,
                    1 if self.hparams.float_quantize_check_inf else 0, None, seed, offset, ctr,
                    None, ws.data_ptr(), ws.numel(), st)
        if rc:
            N.check(rc, "smq_s2fp8_roundtrip")
        return y

    def _call_f64(self, tensor: torch.Tensor, precision: int) -> torch.Tensor:
        """float64 data: s2fp8.py:27-48 in fp64 (smq_s2fp8_roundtrip_f64 / its host twin), output
        float64 (the fp64 signs promote the precision-16 half inverse back to fp64)."""
        hp = self.hparams
        x = tensor.contiguous()
        y = torch.empty_like(x, dtype=torch.float64)
        n = x.numel()
        if n == 0:
            return y
        lib = N.lib()
        inf = 1 if hp.float_quantize_check_inf else 0
        if N.on_cpu(x):
            seed, offset = _q.quant_rng().take(n)
            ws = N.cpu_workspace("s2fp8", lib.smq_s2fp8_workspace_bytes(n))
            N.check(lib.smq_cpu_s2fp8_roundtrip_f64(
                x.data_ptr(), y.data_ptr(), n, precision, inf, None, seed, offset, None,
                ws.data_ptr(), ws.numel(), 0, N.cpu_threads()), "smq_cpu_s2fp8_roundtrip_f64")
            return y
        dev = x.device
        st = N.stream_ptr(dev)
        ws = N.workspace("s2fp8", dev, lib.smq_s2fp8_workspace_bytes(n), st)
        seed, offset, ctr = _q.rng_stream(n, dev)
        N.check(lib.smq_s2fp8_roundtrip_f64(
            x.data_ptr(), y.data_ptr(), n, precision, inf, None, seed, offset, ctr, None,
            ws.data_ptr(), ws.numel(), 0, st), "smq_s2fp8_roundtrip_f64")
        return y
