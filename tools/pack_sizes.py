"""Per-call device time of PackedActivations' forward call at activation sizes (measurement script,
not product): smq_smaq_roundtrip_compress (y and the stream; the single launch's PACK variant
where it applies) against SmartFP's round trip alone and against the separate compress, for
N(0,1) data and for an activation-like tensor (per-channel means and scales, ReLU), each timed
with events over back-to-back calls.

python tools/pack_sizes.py [reps]"""

import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd.compress import SmartFP, SmartFPPacked  # noqa: E402
from smart_compress_amd.util.pytorch.saved import stream_capacity  # noqa: E402


def timed(fn, reps):
    """Device time per call: the calls are enqueued behind a ~50 ms spin kernel, so the host
    (Python, ~10-20 us per call) runs ahead and the events see only the device's back-to-back
    execution."""
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(100_000_000)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps  # us per call


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    pk, ref = SmartFPPacked(smaq_hparams()), SmartFP(smaq_hparams())
    out = []
    for shape in ((128, 512, 4, 4), (128, 256, 8, 8), (128, 128, 16, 16), (128, 64, 16, 16),
                  (128, 64, 32, 32), (64, 64, 32, 32)):
        n = 1
        for s in shape:
            n *= s
        for kind in ("normal", "activation"):
            x = torch.randn(shape, generator=g, device=dev)
            if kind == "activation":
                c = shape[1]
                mu = torch.randn(1, c, 1, 1, generator=g, device=dev) * 2.0
                sc = torch.rand(1, c, 1, 1, generator=g, device=dev) * 2.0 + 0.2
                x = torch.relu(x * sc + mu)
            cap = stream_capacity(n, 6, 8)
            r = {"shape": shape, "n": n, "kind": kind,
                 "roundtrip_compress_us": round(timed(lambda: pk.roundtrip_compress(x, capacity=cap), reps), 2),
                 "smartfp_us": round(timed(lambda: ref(x), reps), 2),
                 "compress_us": round(timed(lambda: pk.compress(x), reps), 2)}
            out.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
