"""Per-kernel timing of libsmq launches through the C-ABI (hipEvents on the launch stream).

python tools/kbench.py [--n N] [--reps R]  ->  one JSON object with ms and GB/s per variant.
"""

import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from smart_compress_amd import _native as N  # noqa: E402


PRE = [None]  # optional untimed action before every timed launch (cache flush)


def timed(fn, reps):
    ts = []
    for r in range(reps + 3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if PRE[0] is not None:
            PRE[0]()
        a.record()
        fn()
        b.record()
        b.synchronize()
        if r >= 3:
            ts.append(a.elapsed_time(b))
    return float(np.median(ts))


class Interleaved:
    """Variants timed in interleaved rounds in one process (methodology rule: A/B deltas only
    from interleaved runs); reports the median over all rounds."""

    def __init__(self):
        self.fns, self.ts = {}, {}

    def add(self, name, fn, bytes_):
        self.fns[name] = (fn, bytes_)
        self.ts[name] = []

    def run(self, rounds, reps):
        for _ in range(rounds):
            for name, (fn, _) in self.fns.items():
                self.ts[name].append(timed(fn, reps))
        return {k: dict(ms=float(np.median(v)), GBps=self.fns[k][1] / float(np.median(v)) / 1e6)
                for k, v in self.ts.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 28)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--quick", action="store_true", help="SmaQ variants only")
    ap.add_argument("--cold", action="store_true",
                    help="read an unrelated 1 GiB buffer (untimed) before every timed launch so "
                         "no input is served from the 256 MB Infinity Cache")
    args = ap.parse_args()
    n = args.n
    lib = N.lib()
    x = torch.randn(n, device="cuda")
    y = torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.zeros(lib.smq_smaq_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    out = {"n": n, "SMQ_APPLY_TILE": os.environ.get("SMQ_APPLY_TILE", "default"), "cold": args.cold}
    if args.cold:
        scratch = torch.ones(1 << 28, device="cuda")
        sink = torch.zeros(1, device="cuda")
        PRE[0] = lambda: sink.add_(scratch.sum())

    def params(**kw):
        p = N.SmqSmaqParams()
        lib.smq_smaq_params_init(p)
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    p = params()
    iv = Interleaved()
    iv.add("stats", lambda: N.check(lib.smq_smaq_stats_f32(x.data_ptr(), n, p, ws.data_ptr(),
                                                           ws.numel(), st), "s"), 4 * n)
    for name, pp in (("apply_sr", params()), ("apply_trunc", params(stochastic_rounding=0)),
                     ("apply_sr_allpos", params(all_positive=1)),
                     ("apply_sr_count", params(count_outliers=1))):
        iv.add(name, lambda pp=pp: N.check(lib.smq_smaq_apply_f32(
            x.data_ptr(), y.data_ptr(), n, pp, None, None, ws.data_ptr(), ws.numel(), st), "a"), 8 * n)
    ps = params(stats_source=N.SMQ_STATS_SAMPLED)
    lib.smq_smaq_draw_samples(ps, n, 16)
    iv.add("apply_sampled", lambda: N.check(lib.smq_smaq_apply_f32(
        x.data_ptr(), y.data_ptr(), n, ps, None, None, ws.data_ptr(), ws.numel(), st), "a"), 8 * n)
    iv.add("roundtrip", lambda: N.check(lib.smq_smaq_roundtrip_f32(
        x.data_ptr(), y.data_ptr(), n, p, None, ws.data_ptr(), ws.numel(), st), "r"), 12 * n)
    iv.add("copylike_fq_8_22_nearest", lambda: N.check(lib.smq_float_quant_f32(
        x.data_ptr(), y.data_ptr(), n, 8, 22, 0, 0, None, 1, 0, st), "c"), 8 * n)
    out.update(iv.run(args.rounds, args.reps))
    if args.quick:
        print(json.dumps(out, indent=1))
        return
    for e, m in ((5, 2), (5, 10), (8, 7)):
        f = lambda e=e, m=m: N.check(lib.smq_float_quant_f32(x.data_ptr(), y.data_ptr(), n, e, m, 1, 1,
                                                             None, 1, 0, st), "f")
        ms = timed(f, args.reps)
        out[f"float_quant_{e}_{m}"] = dict(ms=ms, GBps=8 * n / ms / 1e6)
    ws2 = torch.zeros(lib.smq_s2fp8_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    f = lambda: N.check(lib.smq_s2fp8_roundtrip_f32(x.data_ptr(), y.data_ptr(), n, 1, None, 1, 0, None,
                                                    ws2.data_ptr(), ws2.numel(), st), "s2")
    ms = timed(f, args.reps)
    out["s2fp8_roundtrip"] = dict(ms=ms, GBps=12 * n / ms / 1e6)
    torch.cuda.synchronize()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
