"""Measurement aid for C4 (S2FP8 [32,128,768], 48 rotating buffers): device time per call of
  full      smq_s2fp8_roundtrip (the single launch for fp32 up to 8M elements)
  split     the same forced to two launches (SMQ_S2FP8_SPLIT: partials + apply)
  injected  the same with (mu, m) given: a 1-thread derive launch + the apply without the reduce
  fp8       smq_float_quant E5M2 (one read+write launch over the same bytes: the pass floor)
  copy      torch copy_ of the same bytes
Events around 48-call loops; interleaved rounds; medians in microseconds per call."""

import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from smart_compress_amd import _native as N  # noqa: E402


def main():
    lib = N.lib()
    nbuf = int(os.environ.get("S2B_NBUF", "48"))
    shape = (int(os.environ.get("S2B_N", str(32 * 128 * 768))),)
    n = int(np.prod(shape))
    xs = [torch.randn(shape, device="cuda") for _ in range(nbuf)]
    ys = [torch.empty_like(x) for x in xs]
    ws = torch.zeros(lib.smq_s2fp8_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    s = N.SmqS2fp8Stats()
    s.mu, s.m, s.n_used = -1.5, 2.2, n
    raw = np.frombuffer(ctypes.string_at(ctypes.addressof(s), 64), dtype=np.uint8).copy()
    st_in = torch.from_numpy(raw).cuda()
    flags = int(os.environ.get("S2B_FLAGS", "0"))

    def full(i):
        N.check(lib.smq_s2fp8_roundtrip_ex(xs[i].data_ptr(), 0, ys[i].data_ptr(), n, 32, 1, None,
                                           1, i * n, None, None, ws.data_ptr(), ws.numel(), flags,
                                           st), "s2")

    def split(i):
        N.check(lib.smq_s2fp8_roundtrip_ex(xs[i].data_ptr(), 0, ys[i].data_ptr(), n, 32, 1, None,
                                           1, i * n, None, None, ws.data_ptr(), ws.numel(),
                                           flags | N.SMQ_S2FP8_SPLIT, st), "s2s")

    def injected(i):
        N.check(lib.smq_s2fp8_roundtrip_ex(xs[i].data_ptr(), 0, ys[i].data_ptr(), n, 32, 1, None,
                                           1, i * n, None, st_in.data_ptr(), ws.data_ptr(),
                                           ws.numel(), flags, st), "s2i")

    def fp8(i):
        N.check(lib.smq_float_quant_f32(xs[i].data_ptr(), ys[i].data_ptr(), n, 5, 2, 1, 1, None,
                                        1, i * n, st), "fq")

    def copy(i):
        ys[i].copy_(xs[i])

    variants = dict(full=full, split=split, injected=injected, fp8=fp8, copy=copy)
    res = {k: [] for k in variants}
    for _ in range(3):
        for fn in variants.values():
            for i in range(nbuf):
                fn(i)
    torch.cuda.synchronize()
    for _ in range(7):
        for k, fn in variants.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(nbuf):
                fn(i)
            b.record()
            b.synchronize()
            res[k].append(a.elapsed_time(b) * 1e3 / nbuf)
    print(json.dumps({k: round(float(np.median(v)), 3) for k, v in res.items()}))


if __name__ == "__main__":
    main()
