"""Codec plugins (reference: smart_compress/compress/*)."""

from .base import CompressionAlgorithmBase
from .bf16 import BF16
from .fp8 import FP8, FP8E4M3
from .fp16 import FP16
from .fp32 import FP32
from .s2fp8 import S2FP8
from .packed import SmaqPacked, SmartFPPacked
from .smart import SmartFP

__all__ = ["CompressionAlgorithmBase", "SmartFP", "SmartFPPacked", "SmaqPacked", "FP8", "FP8E4M3", "S2FP8", "FP16", "BF16", "FP32"]
