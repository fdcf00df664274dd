"""Host cost of one SmartFP call, its pieces, and the autograd wrapper around it (eager mode),
microseconds per call on the GPU box — the ResNet-34 autograd step is host-bound at ~20 us per
call (bench.py --config autograd_resnet34, smaq_eager).

python tools/host_cost_smaq.py"""

import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd import _native as N  # noqa: E402
from smart_compress_amd.compress.smart import SmartFP  # noqa: E402
from smart_compress_amd.util.pytorch.autograd import Compressor  # noqa: E402


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
    hp = smaq_hparams()
    c = SmartFP(hp)
    c(x)
    comp = Compressor(c)
    xg = torch.randn(n, device="cuda", requires_grad=True)
    lib = N.lib()
    y = torch.empty_like(x)
    st = N.stream_ptr(x.device)
    ws = N.workspace("smaq", x.device, c.workspace_bytes(n), st)
    p = c._params(n, False, x.dtype, x.device)
    fn = lib.smq_smaq_roundtrip

    def fwd_bwd():
        comp(xg).sum().backward()

    slow = SmartFP(hp)
    object.__setattr__(slow, "_hot", False)  # the Python hot path (no C state)
    slow(x)
    comp_py = Compressor(lambda v, tag=None, **kw: c(v, tag=tag, **kw))  # the Python Function

    def fwd_bwd_py():
        comp_py(xg).sum().backward()

    # a chain of 16 compressors: the backward of one call is the next call's input, so the
    # per-call backward cost is not hidden behind one engine start per backward()
    chain, chain_py = [Compressor(c) for _ in range(16)], [comp_py] * 16

    def chain_fn(cs):
        def f():
            v = xg
            for cc in cs:
                v = cc(v)
            v.sum().backward()
        return f

    # --measure_compression_ratio (the reference scripts' setting): the counted C path, logging
    # into a bounded sink
    import collections
    sink = collections.deque(maxlen=4096)
    cr = SmartFP(smaq_hparams(measure_compression_ratio=True))
    cr.log = lambda k, v, **kw: sink.append((k, v))
    cr(x, tag="t")
    comp_r = Compressor(cr)
    chain_r = [Compressor(cr) for _ in range(16)]
    out = {
        "smartfp_call_counted": per_call(lambda: cr(x, tag="t")),
        "autograd_fwd_counted": per_call(lambda: comp_r(xg)),
        "autograd_chain16_fwd_bwd_counted": per_call(chain_fn(chain_r), 300),
        "smartfp_call": per_call(lambda: c(x)),
        "smartfp_call_python_path": per_call(lambda: slow(x)),
        "autograd_fwd": per_call(lambda: comp(xg)),
        "autograd_fwd_python_function": per_call(lambda: comp_py(xg)),
        "autograd_chain16_fwd_bwd": per_call(chain_fn(chain), 300),
        "autograd_chain16_fwd_bwd_python_function": per_call(chain_fn(chain_py), 300),
        "autograd_fwd_bwd": per_call(fwd_bwd, 1000),
        "autograd_fwd_bwd_python_function": per_call(fwd_bwd_py, 1000),
        "plain_fwd_bwd": per_call(lambda: (xg * 1.0).sum().backward(), 1000),
        "params": per_call(lambda: c._params(n, False, x.dtype, x.device)),
        "empty": per_call(lambda: torch.empty(x.shape, dtype=torch.float32, device=x.device)),
        "contiguous": per_call(lambda: x.contiguous()),
        "stream_ptr": per_call(lambda: N.stream_ptr(x.device)),
        "ws_lookup": per_call(lambda: N.workspace("smaq", x.device, c.workspace_bytes(n), st)),
        "require_supported": per_call(lambda: N.require_supported(x, "SmartFP")),
        "on_cpu": per_call(lambda: N.on_cpu(x)),
        "ctypes_call": per_call(lambda: fn(x.data_ptr(), 0, y.data_ptr(), n, p, None,
                                           ws.data_ptr(), ws.numel(), st)),
    }
    print({k: round(v, 2) for k, v in out.items()}, flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(2000):
        c(x)
        cr(x, tag="t")
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(14)


if __name__ == "__main__":
    main()
