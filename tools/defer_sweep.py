"""Per-call time of smq_smaq_roundtrip against tensor size, back to back on one stream over 8
rotating input buffers (activation-like: written just before, MALL-warm).

python tools/defer_sweep.py  ->  one line per size: n, us per call. DS_FLAGS: smq_smaq_roundtrip_ex
flags (0: the product's choice — the single launch up to 8,388,611 elements; 1: SMQ_SMAQ_SPLIT, the
deferred two-launch path; 2: SMQ_SMAQ_NO_DEFER). tools/fused_exp.sh interleaves them.
"""

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd import _native as N  # noqa: E402
from smart_compress_amd.compress.smart import SmartFP  # noqa: E402

SIZES = [int(s) for s in os.environ.get(
    "DS_SIZES", "65536,262144,1048576,2097152,4194304,8388608,16777216,33554432").split(",")]
CALLS = int(os.environ.get("DS_CALLS", "200"))
GRAPH = os.environ.get("DS_GRAPH") == "1"
FLAGS = int(os.environ.get("DS_FLAGS", "0"))


def main():
    lib = N.lib()
    codec = SmartFP(smaq_hparams())
    for n in SIZES:
        xs = [torch.randn(n, device="cuda") for _ in range(8)]
        ys = [torch.empty(n, device="cuda") for _ in range(8)]
        ws = torch.zeros(lib.smq_smaq_workspace_bytes(n), dtype=torch.uint8, device="cuda")
        p = codec._params(n, False)
        if os.environ.get("DS_CTR") == "1":  # graph-safe stream position in a device counter
            ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
            p.offset_counter = ctr.data_ptr()

        def call(i):
            st = torch.cuda.current_stream().cuda_stream
            N.check(lib.smq_smaq_roundtrip_ex(xs[i % 8].data_ptr(), N.SMQ_DTYPE_F32,
                                              ys[i % 8].data_ptr(), n, p, None, ws.data_ptr(),
                                              ws.numel(), FLAGS, st), "roundtrip")

        for i in range(20):
            call(i)
        run = lambda: [call(i) for i in range(CALLS)]  # noqa: E731
        if GRAPH:  # the same calls captured into one hipGraph, replayed
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                for i in range(CALLS):
                    call(i)
            run = gr.replay
            gr.replay()
            torch.cuda.synchronize()
        best = []
        for r in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run()
            b.record()
            b.synchronize()
            best.append(a.elapsed_time(b) * 1e3 / CALLS)
        print(f"flags={FLAGS} n={n} us_per_call={min(best):.2f} runs={' '.join(f'{t:.2f}' for t in best)}",
              flush=True)


if __name__ == "__main__":
    main()
