"""ORACLE — CPU restatement of the reference's hot path. TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and
only as the checker (or as the timed CPU baseline). The product path (smart-quantization_amd/)
never imports it; it runs libsmq.so or raises.

Modules (each function cites the reference file:line it restates):
  rng.py          the counter-based RNG of libsmq (smq_common.h), bit-exact, vectorised numpy
  smaq.py         smart_compress/compress/smart.py:86-190 op for op in numpy float32
  qtorch_float.py qtorch 0.2.0 float_quantize (un-vendored third-party dependency, pinned in the
                  reference's poetry.lock:773-781) + quantization.py:131-204 (check_inf, max value)
  s2fp8.py        smart_compress/compress/s2fp8.py:27-48

Pinning:
  * smaq.py is pinned bit-for-bit against golden vectors produced by importing the reference's own
    smart.py in the build container (tests/golden/make_golden.py, fixtures tests/golden/*.npz).
  * qtorch_float.py: qtorch is absent from the container (no network), so the quantiser itself is
    "parity unpinned" — restated from qtorch's published algorithm and checked by known-answer
    tests; the reference's own wrapper code around it (float_quantize/check_inf, quantization.py)
    and the S2FP8 transform (s2fp8.py) ARE pinned by golden vectors produced by running the
    reference code with this quantiser substituted for qtorch.
"""
