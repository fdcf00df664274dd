"""Codec plugin base class with the reference's public surface.

Reference: smart_compress/compress/base.py:25-106 (CompressionAlgorithmBase) and 8-22 (the sum
reduction used for `*size*` metrics). What callers rely on, and what is kept:

* class attributes ``log`` / ``log_custom`` — injected by util/train.py:203-210;
* ``add_argparse_args(parent)`` adding ``--measure_compression_ratio`` (base.py:29-37);
* ``log_ratio`` / ``log_size`` emitting ``compression_ratio[_tag]``, ``new_size[_tag]`` and
  ``orig_size[_tag]`` (base.py:60-102); sizes may be callables evaluated lazily, only when
  measuring; tags starting with ``optimizer_`` go to ``log_custom`` (base.py:101);
* ``__call__(tensor, tag=None, **kwargs)`` (base.py:104-106).
"""

from abc import abstractmethod
from argparse import ArgumentParser, Namespace
from typing import Callable, Dict, List, Optional, Union

import torch

SizeLike = Union[float, int, Callable[[], float]]


@torch.no_grad()
def _reduce_fx(values: Union[torch.Tensor, List]):
    """Sum the per-step values of a `*size*` metric (tensors or plain numbers)."""
    if not isinstance(values, list):
        return torch.sum(values)
    if len(values) == 0:
        return 0
    return torch.stack(values).sum() if torch.is_tensor(values[0]) else sum(values)


def _resolve(v: SizeLike) -> float:
    return v() if callable(v) else v


class CompressionAlgorithmBase:
    log = None
    log_custom = None

    @staticmethod
    def add_argparse_args(parent_parser: ArgumentParser) -> ArgumentParser:
        parser = ArgumentParser(parents=[parent_parser], add_help=False)
        parser.add_argument(
            "--measure_compression_ratio", action="store_true", dest="measure_compression_ratio"
        )
        return parser

    def __init__(self, hparams: Namespace):
        super().__init__()
        self.hparams = hparams

    def update_hparams(self, hparams: Namespace):
        self.hparams = hparams

    # -- metrics -------------------------------------------------------------------------------
    def _emit(self, metrics: Dict[str, float], custom: bool) -> None:
        if custom and self.log_custom is not None:
            self.log_custom(metrics)
            return
        for key, value in metrics.items():
            extra = {}
            if "size" in key:
                extra = {"reduce_fx": _reduce_fx, "tbptt_reduce_fx": _reduce_fx}
            self.log(key, value, **extra)

    def log_ratio(self, tag: Optional[str], size: int, orig_bitcount: float,
                  new_bitcount: float, overhead=0):
        return self.log_size(tag, size * orig_bitcount, size * new_bitcount, overhead=overhead)

    def log_size(self, tag: Optional[str], orig_size: SizeLike, new_size: SizeLike, overhead=0):
        if not self.hparams.measure_compression_ratio:
            return
        assert hasattr(self, "log")
        orig = _resolve(orig_size)
        new = _resolve(new_size) + overhead
        ratio = orig / new
        metrics = {}
        for name, value in (("compression_ratio", ratio), ("new_size", new), ("orig_size", orig)):
            metrics[name] = float(value)
            metrics[f"{name}_{tag}"] = float(value)
        self._emit(metrics, custom=tag.startswith("optimizer_"))

    @abstractmethod
    def __call__(self, tensor: torch.Tensor, tag: str = None, **_):
        raise Exception("Not implemented")
