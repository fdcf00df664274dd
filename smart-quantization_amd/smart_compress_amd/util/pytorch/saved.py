"""SmaQ-packed activations for backward: the memory saving the reference only reports.

The reference compresses each layer output through autograd (smart_compress/util/pytorch/
autograd.py:18-77: ``y = compress_fn(x)``, smart.py:110-190) but keeps ``y`` as an fp32 tensor, so
the tensors autograd saves for backward take their full size; the memory saving the paper claims
("reduce the memory usage during training by up to 6.7x", README.md:25) exists only as the size
``log_size`` reports (smart.py:184-188).

``PackedActivations`` makes it real with identical numerics. Used as the ``compress_fn`` of
``register_autograd_module``, each forward call computes ``P = SmartFPPacked.compress(x)`` and
returns ``y = decompress(P)`` — bit for bit what ``SmartFP`` returns for the same input, flags and
random stream (include/smq.h "Packed SmaQ container"). Inside ``with activations:`` a
``torch.autograd.graph.saved_tensors_hooks`` pair replaces every saved tensor that IS such a ``y``
(same storage, shape, strides, and not modified in place since) by ``P``, and the backward decodes
it again: the gradients equal those of the unpacked SmaQ run bit for bit, while a saved activation
takes ~7.4 bits per element (6/8-bit codes on N(0,1)-like data) instead of 32.

The packer writes into a buffer of the worst-case size and leaves the stream size on the device
(no host synchronisation per call); saved streams are trimmed to their size in batches: when the
untrimmed ones exceed ``trim_bytes`` and when the context exits (one host synchronisation per
batch, every stream's size read in one copy). Backward-direction calls (grad-maps, never saved)
and calls outside the context run as the plain codec call.
"""

import weakref
from typing import Dict, List, Optional

import torch

from ...compress.packed import SmaqPacked, SmartFPPacked, _TOTAL_OFF

__all__ = ["PackedActivations"]

FORWARD_TAG = "forward_autograd"


class _Saved:
    """What autograd holds instead of a saved activation: the packed stream and the decoder."""

    __slots__ = ("packed", "codec")

    def __init__(self, packed: SmaqPacked, codec: SmartFPPacked):
        self.packed, self.codec = packed, codec


class _Entry:
    __slots__ = ("ref", "packed", "version", "shape", "stride", "dtype")


class PackedActivations:
    def __init__(self, codec: SmartFPPacked, trim_bytes: int = 256 << 20):
        if not isinstance(codec, SmartFPPacked):
            raise TypeError("PackedActivations needs a SmartFPPacked codec")
        self.codec = codec
        self.trim_bytes = int(trim_bytes)
        self._live: Dict[int, _Entry] = {}  # data_ptr of a forward output -> its stream
        self._untrimmed: List[SmaqPacked] = []
        self._untrimmed_bytes = 0
        self._hooks = None
        self.saved_packed = 0    # saved tensors held as streams (since construction)
        self.saved_bytes = 0     # the distinct streams' trimmed bytes
        self.saved_elements = 0  # and elements

    # -- the compress_fn of register_autograd_module ---------------------------------------------
    def __call__(self, x: torch.Tensor, tag: str = None, all_positive=False,
                 batch_norm_stats=None, **kw):
        codec = self.codec
        if (self._hooks is None or tag != FORWARD_TAG or x.numel() < codec.hparams.min_size
                or not x.is_cuda):
            return codec(x, tag=tag, all_positive=all_positive, batch_norm_stats=batch_norm_stats,
                         **kw)
        packed = codec.compress(x, all_positive, batch_norm_stats)
        y = codec.decompress(packed)
        codec.log_size(tag, x.numel() * 32, lambda: packed.nbytes * 8)
        e = _Entry()
        key = y.data_ptr()
        e.ref = weakref.ref(y, lambda _r, k=key, d=self._live: d.pop(k, None))
        e.packed, e.version = packed, y._version
        e.shape, e.stride, e.dtype = y.shape, y.stride(), y.dtype
        self._live[key] = e
        return y

    # -- saved_tensors_hooks ------------------------------------------------------------------------
    def _pack(self, t: torch.Tensor):
        e = self._live.get(t.data_ptr()) if t.is_cuda else None
        if (e is None or e.ref() is None or t._version != e.version or t.shape != e.shape
                or t.stride() != e.stride or t.dtype != e.dtype):
            return t  # not a forward output of this codec, or modified in place since
        p = e.packed
        if p._total is None and not any(q is p for q in self._untrimmed):
            self._untrimmed.append(p)
            self._untrimmed_bytes += p.data.numel()
            if self._untrimmed_bytes > self.trim_bytes:
                self.trim()
        self.saved_packed += 1
        return _Saved(p, self.codec)

    @staticmethod
    def _unpack(h):
        if isinstance(h, _Saved):
            return h.codec.decompress(h.packed)
        return h

    def trim(self) -> None:
        """Cut every untrimmed saved stream to its size: one host synchronisation (every header's
        stream size in one copy), then right-sized device copies."""
        ps = self._untrimmed
        if not ps:
            return
        sizes = torch.cat([p.data[_TOTAL_OFF:_TOTAL_OFF + 8] for p in ps]).cpu()
        for p, total in zip(ps, sizes.view(torch.int64).tolist()):
            p._total = int(total)
            if p.data.numel() > total:
                p.data = p.data[:total].clone()
            self.saved_bytes += int(total)
            self.saved_elements += p.n
        self._untrimmed = []
        self._untrimmed_bytes = 0

    def __enter__(self):
        self._hooks = torch.autograd.graph.saved_tensors_hooks(self._pack, self._unpack)
        self._hooks.__enter__()
        return self

    def __exit__(self, *exc):
        hooks, self._hooks = self._hooks, None
        try:
            self.trim()
        finally:
            self._live.clear()
            hooks.__exit__(*exc)
        return False

    def stats(self) -> Dict[str, Optional[float]]:
        """Saved tensors held as streams, and the bytes / bits per element of the distinct streams
        trimmed so far."""
        return {"saved_packed": self.saved_packed, "saved_elements": self.saved_elements,
                "saved_stream_bytes": self.saved_bytes,
                "bits_per_element": (8.0 * self.saved_bytes / self.saved_elements
                                     if self.saved_elements else None)}
