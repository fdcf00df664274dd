"""Host cost of one S2FP8 call and its pieces (eager mode), microseconds per call (GPU box).

python tools/host_cost_s2.py"""

import os
import sys
import time
from argparse import ArgumentParser

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd")]

import torch  # noqa: E402

from smart_compress_amd import _native as N  # noqa: E402
from smart_compress_amd.compress.s2fp8 import S2FP8  # noqa: E402
from smart_compress_amd.util.pytorch import quantization as _q  # noqa: E402


def per_call(fn, reps=3000):
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    return dt / reps * 1e6


def main():
    n = int(os.environ.get("HC_N", "65536"))
    x = torch.randn(n, device="cuda")
    hp = S2FP8.add_argparse_args(ArgumentParser()).parse_args([])
    hp.precision = 32
    c = S2FP8(hp)
    c(x)
    lib = N.lib()
    y = torch.empty_like(x)
    st = N.stream_ptr(x.device)
    ws = N.workspace("s2fp8", x.device, S2FP8._ws_bytes, st)
    fn = lib.smq_s2fp8_roundtrip
    out = {
        "s2fp8_call": per_call(lambda: c(x)),
        "empty_like": per_call(lambda: torch.empty_like(x)),
        "contiguous": per_call(lambda: x.contiguous()),
        "stream_ptr": per_call(lambda: N.stream_ptr(x.device)),
        "ws_lookup": per_call(lambda: N.workspace("s2fp8", x.device, S2FP8._ws_bytes, st)),
        "rng_stream": per_call(lambda: _q.rng_stream(n, x.device)),
        "on_cpu": per_call(lambda: N.on_cpu(x)),
        "ctypes_call": per_call(lambda: fn(x.data_ptr(), 0, y.data_ptr(), n, 32, 1, None, 1, 0,
                                           None, None, ws.data_ptr(), ws.numel(), st)),
        "data_ptr": per_call(lambda: x.data_ptr()),
    }
    print({k: round(v, 2) for k, v in out.items()}, flush=True)


if __name__ == "__main__":
    main()
