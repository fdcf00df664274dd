"""Where does the bench's per-step time go? Times K steps of the 256M SmaQ round trip in several
variants in ONE process, interleaved: the bench path (SmartFP + per-kernel events), SmartFP without
events, SmartFP with events around the whole step only, and the raw C-ABI round trip."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd")]
import json  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from smart_compress_amd import _native as N  # noqa: E402
from smart_compress_amd.compress.smart import SmartFP  # noqa: E402


def main():
    n = 1 << 28
    steps = 20
    xs = [torch.randn(n, device="cuda") for _ in range(2)]
    codec = SmartFP(bench.smaq_hparams())
    lib = N.lib()
    ws = torch.zeros(lib.smq_smaq_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    yfix = torch.empty_like(xs[0])
    p = codec._params(n, False)
    st = torch.cuda.current_stream().cuda_stream
    state = {"i": 0}

    def v_bench():
        codec._trace = bench.EventTrace()
        state["y"] = codec(xs[state["i"] & 1])
        state["i"] += 1

    def v_noevents():
        codec._trace = None
        state["y"] = codec(xs[state["i"] & 1])
        state["i"] += 1

    def v_stepevents():
        codec._trace = None
        a = torch.cuda.Event(enable_timing=True)
        a.record()
        state["y"] = codec(xs[state["i"] & 1])
        b = torch.cuda.Event(enable_timing=True)
        b.record()
        state["i"] += 1

    def v_capi():
        x = xs[state["i"] & 1]
        N.check(lib.smq_smaq_roundtrip_f32(x.data_ptr(), yfix.data_ptr(), n, p, None, ws.data_ptr(),
                                           ws.numel(), st), "rt")
        state["i"] += 1

    def v_capi_samex():
        N.check(lib.smq_smaq_roundtrip_f32(xs[0].data_ptr(), yfix.data_ptr(), n, p, None,
                                           ws.data_ptr(), ws.numel(), st), "rt")

    variants = dict(bench=v_bench, noevents=v_noevents, stepevents=v_stepevents, capi=v_capi,
                    capi_samex=v_capi_samex)
    res = {k: [] for k in variants}
    for _ in range(5):
        for k, f in variants.items():
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                f()
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / steps * 1e3)
    print(json.dumps({k: dict(ms=float(np.median(v)), GBps=12 * n / (np.median(v) * 1e-3) / 1e9)
                      for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
