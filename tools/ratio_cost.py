"""Device and host cost of ratio logging per SmartFP call (measurement script, not product):
SmartFP with and without --measure_compression_ratio (the counted call, smq_smaq_roundtrip_counted,
logging 0-dim device values into a bounded sink) at activation sizes — device time per call behind a
~50 ms spin kernel (the host runs ahead, the events see the device's back-to-back execution) and
host time per call with the device kept busy.

python tools/ratio_cost.py [reps]"""

import collections
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd.compress import SmartFP  # noqa: E402


def device_us(fn, reps):
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
    return a.elapsed_time(b) * 1e3 / reps


def host_us(fn, reps):
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    dt = time.perf_counter() - t0
    torch.cuda.synchronize()
    return dt * 1e6 / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    plain = SmartFP(smaq_hparams())
    counted = SmartFP(smaq_hparams(measure_compression_ratio=True))
    sink = collections.deque(maxlen=1 << 14)
    counted.log = lambda k, v, _s=sink, **kw: _s.append((k, v))
    for n in (262_144, 524_288, 1 << 20, 2 << 20, 8 << 20):
        x = torch.randn(n, generator=g, device=dev)
        r = {"n": n,
             "device_us_plain": round(device_us(lambda: plain(x), reps), 2),
             "device_us_counted": round(device_us(lambda: counted(x, tag="forward_autograd"), reps), 2),
             "host_us_plain": round(host_us(lambda: plain(x), reps), 2),
             "host_us_counted": round(host_us(lambda: counted(x, tag="forward_autograd"), reps), 2)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
