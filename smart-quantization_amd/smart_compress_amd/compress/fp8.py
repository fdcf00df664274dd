"""FP8 codec: drop-in for smart_compress/compress/fp8.py:11-31.

NB the reference's FP8 is **E5M2** (``float_quantize(tensor, exp=5, man=2)``, fp8.py:31), stochastic
rounding, with check_inf; BASELINE.json's "E4M3" label is wrong. ``FP8E4M3`` is an
opt-in extra with the same qtorch semantics at (exp=4, man=3).
"""

from .._float_formats import E4M3, E5M2
from ._float_codec import FloatFormatCodec


class FP8(FloatFormatCodec):
    EXP_BITS, MAN_BITS = E5M2
    STORED_BITS = 8


class FP8E4M3(FloatFormatCodec):
    EXP_BITS, MAN_BITS = E4M3
    STORED_BITS = 8
