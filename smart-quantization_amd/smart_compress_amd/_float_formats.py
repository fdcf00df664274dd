"""(exp_bits, man_bits) of the qtorch float formats used by the reference codecs."""

E5M2 = (5, 2)         # compress/fp8.py:31
E4M3 = (4, 3)         # opt-in extra (BASELINE.json config 3 label)
FP16_FORMAT = (5, 10)  # compress/fp16.py:31
BF16_FORMAT = (8, 7)   # compress/bf16.py:31
