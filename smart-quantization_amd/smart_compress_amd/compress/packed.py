"""Packed SmaQ: the codes of smart.py stored for real.

The reference's ``SmartFP`` (smart.py:110-190) only *simulates* SmaQ: it quantises and immediately
de-quantises in fp32, and reports the size the codes would take (smart.py:184-188). The paper's
memory saving (README.md:25-28: ``[outlier flag][sign][N-2 magnitude bits]``, 6 bits per main
element and 8 per outlier by default) needs the codes to be kept. ``SmartFPPacked`` keeps them in
the container of include/smq.h ("Packed SmaQ container"):

* ``compress(x)`` -> ``SmaqPacked``: device bytes (header, block directory, per block a fixed
  section — outlier mask and a plane of num_bits_main - 1 bits per element — and a variable
  section — the outliers' remaining code bits and the escape list for codes outside the budget),
  built by ``smq_smaq_compress`` (statistics + three packing launches);
* ``decompress(p)`` -> fp32 tensor, bit-identical to what ``SmartFP`` returns for the same input,
  flags and random stream (``smq_smaq_decompress_ex``, one launch);
* float64 tensors: the fp64 chain's codes (smart.py on a float64 tensor, as ``SmartFP`` runs it) in a
  float64 stream (flag SMQ_PACK_FLAG_F64: 3-word escapes, fp64 statistics; ``smq_smaq_compress_f64``
  / ``smq_cpu_smaq_compress_f64``), decoded to float64 — again bit-identical to ``SmartFP``;
* ``__call__`` = decompress(compress(x)), a drop-in SmaQ codec whose ``new_size`` log is the real
  stream size.

Same flags as ``SmartFP`` (it is a subclass), incl. the BatchNorm variant (smart.py:136-149,
174-179: the stream carries the compress-time gamma / beta, so ``decompress`` needs no arguments)
and any threshold (``main_std_dev_threshold < 0``: an element above -T and below T at once is the
third state smart.py:157-161 gives it).

No call synchronises the host: ``compress`` writes into a buffer of the worst-case size
(``smq_smaq_pack_bound``) whose real stream size stays on the device (header ``total_bytes``);
``SmaqPacked.nbytes`` reads it when asked (one synchronisation, cached), and ``compact()`` returns a
right-sized copy for a caller that keeps the stream (the memory saving). ``__call__`` and a
``compress`` + ``decompress`` pair therefore run inside a captured hipGraph.
"""

import ctypes
from typing import Optional, Tuple

import numpy as np
import torch

from .. import _native as N
from ..util.globals import profile
from .smart import SmartFP

__all__ = ["SmaqPacked", "SmartFPPacked"]

_HDR_BYTES = ctypes.sizeof(N.SmqPackedHeader)
_TOTAL_OFF = N.SmqPackedHeader.total_bytes.offset


class SmaqPacked:
    """A packed SmaQ tensor: ``data`` (uint8, on the device; the stream, possibly followed by unused
    capacity) plus the original shape. ``raw``: a tensor below ``min_size``, kept as its original
    fp32 bytes (smart.py:123-128)."""

    def __init__(self, data: torch.Tensor, shape: torch.Size, n: int, raw: bool = False,
                 widths=None, total: Optional[int] = None, dtype: torch.dtype = torch.float32):
        self.data = data
        self.shape = torch.Size(shape)
        self.n = int(n)
        self.raw = raw
        self.dtype = dtype    # of the decoded values (float64: a float64 stream; raw: as kept)
        self.widths = widths  # (num_bits_main, num_bits_outlier) the stream was written with
        # the stream size when known on the host (raw data: all of it)
        self._total = int(data.numel()) if raw else total

    @property
    def nbytes(self) -> int:
        """The stream size in bytes (header ``total_bytes``: one host synchronisation the first
        time it is asked for)."""
        if self._total is None:
            self._total = int(self.data[_TOTAL_OFF:_TOTAL_OFF + 8].cpu().numpy().view(np.uint64)[0])
        return self._total

    def compact(self) -> "SmaqPacked":
        """A right-sized copy of the stream (the memory a kept stream should take)."""
        total = self.nbytes
        if total == self.data.numel():
            return self
        return SmaqPacked(self.data[:total].clone(), self.shape, self.n, widths=self.widths,
                          total=total, dtype=self.dtype)

    @property
    def bits_per_element(self) -> float:
        return 8.0 * self.nbytes / max(1, self.n)

    def compression_ratio(self, orig_bits: int = 32) -> float:
        return orig_bits * self.n / (8.0 * self.nbytes)

    def header(self) -> dict:
        """The stream header as a dict (reads 128 bytes from the device)."""
        if self.raw:
            return {"raw": True, "n": self.n}
        raw = bytes(self.data[:_HDR_BYTES].cpu().numpy())
        h = N.SmqPackedHeader.from_buffer_copy(raw)
        return {k: getattr(h, k) for k, _ in N.SmqPackedHeader._fields_ if k != "reserved"}


class SmartFPPacked(SmartFP):
    def compress(self, data: torch.Tensor, all_positive: bool = False,
                 batch_norm_stats: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                 out: Optional[torch.Tensor] = None) -> SmaqPacked:
        """The stream of ``data`` (smart.py:110-190's codes). A ROCm tensor: ``smq_smaq_compress``
        on the caller's stream, no host synchronisation, into a buffer of the worst-case size
        (``smq_smaq_pack_bound``: several times the tensor; ``SmaqPacked.compact()`` or
        ``nbytes`` trim / read the real size) — ``out``, a caller's uint8 device buffer of at least
        that size (reused across calls: the returned stream then lives in it), or a new one. A CPU
        tensor: ``smq_cpu_smaq_compress``, the same bytes, right-sized at once (the call is
        synchronous)."""
        hp = self.hparams
        numel = data.numel()
        if numel < hp.min_size:  # smart.py:123-128: kept as is
            kdt = torch.float64 if data.dtype == torch.float64 else torch.float32
            raw = data.detach().to(kdt).contiguous().reshape(-1).view(torch.uint8)
            return SmaqPacked(raw.clone(), data.shape, numel, raw=True, dtype=kdt)
        if hp.main_std_dev_threshold != hp.main_std_dev_threshold:
            raise NotImplementedError("SmartFPPacked: main_std_dev_threshold is NaN")
        N.require_supported(data, "SmartFPPacked")
        if data.dtype == torch.float64:
            return self._compress_f64(data, all_positive, batch_norm_stats, out)
        code = N.DTYPE_CODES.get(data.dtype)
        if code is None:
            raise NotImplementedError(
                f"SmartFPPacked: dtype {data.dtype} is not supported "
                "(float32/float16/bfloat16/float64)")
        if data.dtype == torch.float16 and hp.precision != 16:
            raise RuntimeError("value cannot be converted to type c10::Half without overflow")
        x = data.contiguous()
        lib = N.lib()
        cpu = N.on_cpu(x)
        p = self._params(numel, all_positive, x.dtype, None if cpu else x.device)
        keep = None
        if hp.use_batch_norm and batch_norm_stats is not None:
            keep = self._bind_batch_norm(p, x, batch_norm_stats)
        bound = lib.smq_smaq_pack_bound_bn(numel, hp.num_bits_main, hp.num_bits_outlier,
                                           p.bn_channels if keep is not None else 0)
        widths = (hp.num_bits_main, hp.num_bits_outlier)
        sampled = p.stats_source == N.SMQ_STATS_SAMPLED_DEVICE
        if cpu:
            out = torch.empty(bound, dtype=torch.uint8)
            ws = N.cpu_workspace("smaq", self.workspace_bytes(numel))
            N.check(lib.smq_cpu_smaq_compress(x.data_ptr(), code, numel, p, out.data_ptr(),
                                              out.numel(), ws.data_ptr(), ws.numel(),
                                              N.cpu_threads()), "smq_cpu_smaq_compress")
            del keep
            total = int(out[_TOTAL_OFF:_TOTAL_OFF + 8].numpy().view(np.uint64)[0])
            return SmaqPacked(out[:total].clone(), data.shape, numel, widths=widths, total=total)
        if out is None:
            out = torch.empty(bound, dtype=torch.uint8, device=x.device)
        elif out.dtype != torch.uint8 or out.device != x.device or out.numel() < bound:
            raise ValueError(f"SmartFPPacked.compress: out must be a uint8 buffer of >= {bound} "
                             f"bytes on {x.device}")
        nws = (lib.smq_smaq_pack_workspace_bytes_sampled(numel, p.num_samples) if sampled
               else lib.smq_smaq_pack_workspace_bytes(numel))
        ws = N.workspace("smaq_pack", x.device, nws)
        N.check(lib.smq_smaq_compress(x.data_ptr(), code, numel, p, out.data_ptr(), out.numel(),
                                      ws.data_ptr(), ws.numel(), N.stream_ptr(x.device)),
                "smq_smaq_compress")
        del keep
        # the stream size stays on the device (SmaqPacked.nbytes / compact read it when asked)
        return SmaqPacked(out, data.shape, numel, widths=widths)

    def roundtrip_compress(self, data: torch.Tensor, all_positive: bool = False,
                           batch_norm_stats: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                           capacity: Optional[int] = None, pack_stream=None,
                           workspace: Optional[torch.Tensor] = None
                           ) -> Tuple[torch.Tensor, SmaqPacked]:
        """``(y, p)``: ``y`` what ``SmartFP`` returns for ``data`` (smart.py:110-190) and ``p`` its
        stream — ``decompress(p) == y`` bit for bit — from one statistics pass
        (``smq_smaq_roundtrip_compress``: the round trip, then the packing launches on its
        statistics; no decode to get ``y``). ``capacity``: bytes of the stream buffer (default
        ``smq_smaq_pack_bound``); a smaller one holds the stream when it fits, which
        ``p.nbytes <= capacity`` tells (a stream that did not fit must not be decoded).
        ``pack_stream``: a torch stream for the packing launches (they wait for the statistics
        on the current stream, then overlap what follows it; ``smq_smaq_roundtrip_compress_ex``) —
        the caller then orders readers of the stream after it and passes a ``workspace`` (uint8,
        ``smq_smaq_pack_workspace_bytes``) no other call uses until ``pack_stream`` has passed.
        CPU and float64 tensors: ``compress`` then ``decompress`` (the same values)."""
        hp = self.hparams
        if pack_stream is not None and workspace is None:
            # the shared per-(device, stream) workspace would be cleared and rewritten by the next
            # call on the current stream while pack_stream may still read it
            raise ValueError("roundtrip_compress: pack_stream needs a private workspace "
                             "(smq_smaq_pack_workspace_bytes) that no other call uses until "
                             "pack_stream has passed")
        numel = data.numel()
        if (numel < hp.min_size or N.on_cpu(data) or data.dtype == torch.float64
                or hp.main_std_dev_threshold != hp.main_std_dev_threshold):
            p = self.compress(data, all_positive, batch_norm_stats)
            return self.decompress(p), p
        N.require_supported(data, "SmartFPPacked")
        code = N.DTYPE_CODES.get(data.dtype)
        if code is None:
            raise NotImplementedError(
                f"SmartFPPacked: dtype {data.dtype} is not supported "
                "(float32/float16/bfloat16/float64)")
        if data.dtype == torch.float16 and hp.precision != 16:
            raise RuntimeError("value cannot be converted to type c10::Half without overflow")
        x = data.contiguous()
        lib = N.lib()
        p = self._params(numel, all_positive, x.dtype, x.device)
        keep = None
        if hp.use_batch_norm and batch_norm_stats is not None:
            keep = self._bind_batch_norm(p, x, batch_norm_stats)
        if capacity is None:
            capacity = lib.smq_smaq_pack_bound_bn(numel, hp.num_bits_main, hp.num_bits_outlier,
                                                  p.bn_channels if keep is not None else 0)
        out = torch.empty(int(capacity), dtype=torch.uint8, device=x.device)
        y = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        sampled = p.stats_source == N.SMQ_STATS_SAMPLED_DEVICE
        nws = (lib.smq_smaq_pack_workspace_bytes_sampled(numel, p.num_samples) if sampled
               else lib.smq_smaq_pack_workspace_bytes(numel))
        ws = N.workspace("smaq_pack", x.device, nws) if workspace is None else workspace
        N.check(lib.smq_smaq_roundtrip_compress_ex(
            x.data_ptr(), code, y.data_ptr(), numel, p, out.data_ptr(), out.numel(),
            ws.data_ptr(), ws.numel(), N.stream_ptr(x.device),
            None if pack_stream is None else pack_stream.cuda_stream),
            "smq_smaq_roundtrip_compress_ex")
        if pack_stream is not None:  # read there: not reused before pack_stream has passed
            for t in (x, out) + (tuple(keep) if keep is not None else ()):
                t.record_stream(pack_stream)
        del keep
        return y, SmaqPacked(out, data.shape, numel,
                             widths=(hp.num_bits_main, hp.num_bits_outlier))

    def _compress_f64(self, data, all_positive, batch_norm_stats, out):
        """float64 data: the fp64 chain (SmartFP._call_f64's) in a float64 stream."""
        hp = self.hparams
        numel = data.numel()
        x = data.contiguous()
        lib = N.lib()
        cpu = N.on_cpu(x)
        p = self._params(numel, all_positive, torch.float64, None if cpu else x.device)
        keep = None
        if hp.use_batch_norm and batch_norm_stats is not None:
            keep = self._bind_batch_norm(p, x, batch_norm_stats)  # fp64 parameters
        bound = lib.smq_smaq_pack_bound_f64(numel, hp.num_bits_main, hp.num_bits_outlier,
                                            p.bn_channels if keep is not None else 0)
        widths = (hp.num_bits_main, hp.num_bits_outlier)
        if cpu:
            buf = torch.empty(bound, dtype=torch.uint8)
            ws = N.cpu_workspace("smaq", self.workspace_bytes(numel))
            N.check(lib.smq_cpu_smaq_compress_f64(x.data_ptr(), numel, p, buf.data_ptr(),
                                                  buf.numel(), ws.data_ptr(), ws.numel(),
                                                  N.cpu_threads()), "smq_cpu_smaq_compress_f64")
            del keep
            total = int(buf[_TOTAL_OFF:_TOTAL_OFF + 8].numpy().view(np.uint64)[0])
            return SmaqPacked(buf[:total].clone(), data.shape, numel, widths=widths, total=total,
                              dtype=torch.float64)
        if out is None:
            out = torch.empty(bound, dtype=torch.uint8, device=x.device)
        elif out.dtype != torch.uint8 or out.device != x.device or out.numel() < bound:
            raise ValueError(f"SmartFPPacked.compress: out must be a uint8 buffer of >= {bound} "
                             f"bytes on {x.device}")
        k = p.num_samples if p.stats_source == N.SMQ_STATS_SAMPLED_DEVICE else 0
        ws = N.workspace("smaq_pack_f64", x.device, lib.smq_smaq_pack_workspace_bytes_f64(numel, k))
        N.check(lib.smq_smaq_compress_f64(x.data_ptr(), numel, p, out.data_ptr(), out.numel(),
                                          ws.data_ptr(), ws.numel(), N.stream_ptr(x.device)),
                "smq_smaq_compress_f64")
        del keep
        return SmaqPacked(out, data.shape, numel, widths=widths, dtype=torch.float64)

    def decompress(self, packed: SmaqPacked) -> torch.Tensor:
        """fp32 values, bit-identical to ``SmartFP`` on the compressed tensor (same flags and random
        stream), on the device the stream is on (a CPU stream: ``smq_cpu_smaq_decompress``)."""
        if packed.raw:
            return packed.data.view(packed.dtype).reshape(packed.shape).clone()
        N.require_supported(packed.data, "SmartFPPacked.decompress")
        lib = N.lib()
        if packed.dtype == torch.float64:
            y = torch.empty(packed.shape, dtype=torch.float64, device=packed.data.device)
            if N.on_cpu(packed.data):
                N.check(lib.smq_cpu_smaq_decompress_f64(packed.data.data_ptr(), y.data_ptr(),
                                                        packed.n, N.cpu_threads()),
                        "smq_cpu_smaq_decompress_f64")
            else:
                bm, bo = packed.widths if packed.widths is not None else (
                    packed.header()["num_bits_main"], packed.header()["num_bits_outlier"])
                N.check(lib.smq_smaq_decompress_f64(packed.data.data_ptr(), y.data_ptr(), packed.n,
                                                    bm, bo, N.stream_ptr(y.device)),
                        "smq_smaq_decompress_f64")
            return y
        y = torch.empty(packed.shape, dtype=torch.float32, device=packed.data.device)
        if N.on_cpu(packed.data):
            N.check(lib.smq_cpu_smaq_decompress(packed.data.data_ptr(), y.data_ptr(), packed.n,
                                                N.cpu_threads()), "smq_cpu_smaq_decompress")
            return y
        st = N.stream_ptr(y.device)
        if packed.widths is not None:
            # the widths the stream was written with: the decoder locates its sections without
            # waiting for the header
            bm, bo = packed.widths
            N.check(lib.smq_smaq_decompress_ex(packed.data.data_ptr(), y.data_ptr(), packed.n, bm,
                                               bo, st), "smq_smaq_decompress_ex")
        else:  # a stream from elsewhere: the widths its header records
            N.check(lib.smq_smaq_decompress(packed.data.data_ptr(), y.data_ptr(), packed.n, st),
                    "smq_smaq_decompress")
        return y

    def __call__(self, data: torch.Tensor, tag: str = None, all_positive=False,
                 batch_norm_stats: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, **_):
        with profile("smaq"):
            numel = data.numel()
            if numel < self.hparams.min_size:
                self.log_ratio(tag, numel * 32, 32, 32)  # smart.py:125
                return data
            packed = self.compress(data, all_positive, batch_norm_stats)
            y = self.decompress(packed)
            # the real stream size, read (one synchronisation) only if the ratio is measured
            self.log_size(tag, numel * 32, lambda: packed.nbytes * 8)
            return y

    # __call__ returns SmartFP's values for the same flags and random stream; only its log_size
    # differs (the real stream size), and the C hot path declines calls that log: SmartFP's C path
    # (the single launch, its autograd node) serves this codec as well
    _smartfp_call = __call__
