"""smart_compress_amd — MI355X-native SmaQ / FP8 / S2FP8 codecs behind the reference plugin API.

Drop-in for the codec layer of nimashoghi/smart-quantization (``smart_compress.compress``): same
classes, flags and call signatures; the arithmetic runs in libsmq.so (HIP, gfx950) through the
C-ABI in include/smq.h. Only ROCm device tensors are accepted; there is no CPU fallback.
"""

__version__ = "0.1.0"
