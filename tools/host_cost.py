"""Host cost of one SmartFP call and its pieces (eager mode), microseconds per call.

python tools/host_cost.py   (GPU box: the launches are real; the tensor is small so the host
path, not the device, sets the pace)"""

import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd import _native as N  # noqa: E402
from smart_compress_amd.compress.smart import SmartFP  # noqa: E402


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
    c = SmartFP(smaq_hparams())
    lib = N.lib()
    y = torch.empty_like(x)
    p = c._params(n, False)
    st = N.stream_ptr(x.device)
    ws = N.workspace("smaq", x.device, lib.smq_smaq_workspace_bytes(n), st)
    out = {
        "smartfp_call": per_call(lambda: c(x)),
        "params": per_call(lambda: c._params(n, False)),
        "empty": per_call(lambda: torch.empty(x.shape, dtype=torch.float32, device=x.device)),
        "stream_ptr": per_call(lambda: N.stream_ptr(x.device)),
        "ws_lookup": per_call(lambda: N.workspace("smaq", x.device,
                                                  lib.smq_smaq_workspace_bytes(n), st)),
        "ctypes_roundtrip": per_call(lambda: lib.smq_smaq_roundtrip(
            x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, p, None, ws.data_ptr(), ws.numel(),
            st)),
        "require_supported": per_call(lambda: N.require_supported(x, "SmartFP")),
    }
    print({k: round(v, 2) for k, v in out.items()}, flush=True)


if __name__ == "__main__":
    main()
