"""FP16 codec: drop-in for smart_compress/compress/fp16.py:11-31 (qtorch (exp=5, man=10))."""

from .._float_formats import FP16_FORMAT
from ._float_codec import FloatFormatCodec


class FP16(FloatFormatCodec):
    EXP_BITS, MAN_BITS = FP16_FORMAT
    STORED_BITS = 16
