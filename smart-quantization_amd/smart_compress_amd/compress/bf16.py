"""BF16 codec: drop-in for smart_compress/compress/bf16.py:11-31 (qtorch (exp=8, man=7))."""

from .._float_formats import BF16_FORMAT
from ._float_codec import FloatFormatCodec


class BF16(FloatFormatCodec):
    EXP_BITS, MAN_BITS = BF16_FORMAT
    STORED_BITS = 16
