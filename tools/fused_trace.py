"""Per-workgroup timeline of the single-launch SmaQ round trip (csrc/smaq_fused.hip), from an
experiment build with -DSMQ_FUSED_TRACE=1 (tools/build_variant.py fused_trace -DSMQ_FUSED_TRACE=1;
run with SMQ_LIB=exp/fused_trace/libsmq.so). Back-to-back calls, each on its own workspace (the
stamps live past its end); medians over the calls of: loads + partial published, every partial
gathered, statistics final, transform issued, stores drained (us from the call's first workgroup
start; max: the slowest workgroup's), the arrival words' hand-off after the transform, the
slowest workgroup's end, and the gap to the next call's first start."""

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd import _native as N  # noqa: E402
from smart_compress_amd.compress.smart import SmartFP  # noqa: E402

SIZES = [int(s) for s in os.environ.get("FT_SIZES", "1048576,4194304,8388608").split(",")]
CALLS = 24


def main():
    lib = N.lib()
    codec = SmartFP(smaq_hparams())
    for n in SIZES:
        xs = [torch.randn(n, device="cuda") for _ in range(8)]
        ys = [torch.empty(n, device="cuda") for _ in range(8)]
        nb = lib.smq_smaq_workspace_bytes(n) + 16 * 8 * 256
        wss = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(CALLS)]
        p = codec._params(n, False)
        st = torch.cuda.current_stream().cuda_stream
        for rep in range(2):  # the second pass is measured (first: warm-up)
            for i in range(CALLS):
                N.check(lib.smq_smaq_roundtrip(xs[i % 8].data_ptr(), N.SMQ_DTYPE_F32,
                                               ys[i % 8].data_ptr(), n, p, None, wss[i].data_ptr(),
                                               nb, st), "roundtrip")
            torch.cuda.synchronize()
        off = lib.smq_smaq_workspace_bytes(n)
        tr = [w[off:off + 16 * 8 * 256].cpu().numpy().view(np.uint64).reshape(256, 16) for w in wss]
        G = int(np.count_nonzero(tr[0][:, 0]))
        rows = []
        for i in range(CALLS - 1):
            t = tr[i][:G].astype(np.int64)
            t0 = t[:, 0].min()
            rel = (t - t0) / 100.0  # 100 MHz -> us
            end = max(t[:, 5].max(), t[:, 7].max())
            gap = (tr[i + 1][:G, 0].astype(np.int64).min() - end) / 100.0
            rows.append([np.median(rel[:, k]) for k in range(6)] + [
                (end - t0) / 100.0, gap, rel[:, 0].max(), rel[:, 1].max(), rel[:, 2].max(),
                np.median(rel[:, 7]), np.median(rel[:, 10]), np.median(rel[:, 8]),
                np.median(rel[:, 9])])
        m = np.median(np.array(rows), axis=0)
        print(f"n={n} G={G} start_spread={m[8]:.2f} published={m[1]:.2f} (max {m[9]:.2f}) "
              f"gathered={m[2]:.2f} (max {m[10]:.2f}) [summed {m[12]:.2f} reduced {m[13]:.2f} "
              f"finalised {m[14]:.2f}] final={m[3]:.2f} transformed={m[4]:.2f} "
              f"drained={m[5]:.2f} arrived={m[11]:.2f} last={m[6]:.2f} gap_to_next={m[7]:.2f} "
              f"(us, medians over {len(rows)} calls)", flush=True)


if __name__ == "__main__":
    main()
