"""Per-workgroup timeline of the single-launch S2FP8 (measurement aid, SMQ_S2_TRACE=1): C4
[32,128,768] with 48 rotating buffers, each call its own workspace with trace room; stamps
(s_memrealtime, 10 ns) per workgroup: start, loaded + summed, published, gathered, table built,
end (stores drained); word 6 = partials computed for missing workgroups."""

import json
import os
import sys

os.environ["SMQ_S2_TRACE"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from smart_compress_amd import _native as N  # noqa: E402


def main():
    lib = N.lib()
    nbuf = 48
    n = 32 * 128 * 768
    xs = [torch.randn(n, device="cuda") for _ in range(nbuf)]
    ys = [torch.empty_like(x) for x in xs]
    wb = lib.smq_s2fp8_workspace_bytes(n)
    wss = [torch.zeros(wb + 128 * 256, dtype=torch.uint8, device="cuda") for _ in range(nbuf)]
    if os.environ.get("S2T_SHARED") == "1":  # one workspace for every call, like the codec's
        wss = [wss[0]] * nbuf
    st = torch.cuda.current_stream().cuda_stream
    flags = int(os.environ.get("S2B_FLAGS", "0"))
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda") if os.environ.get("S2T_CTR") == "1" else None

    def call(i):
        nonlocal st
        N.check(lib.smq_s2fp8_roundtrip_ex(xs[i].data_ptr(), 0, ys[i].data_ptr(), n, 32, 1, None,
                                           1, i * n, ctr.data_ptr() if ctr is not None else None,
                                           None, wss[i].data_ptr(), wss[i].numel(),
                                           flags, st), "s2")

    for _ in range(20):
        for i in range(nbuf):
            call(i)
    torch.cuda.synchronize()
    graph = os.environ.get("S2T_GRAPH") == "1"
    if graph:  # the same 48 calls captured once, replayed
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            st = torch.cuda.current_stream().cuda_stream
            for i in range(nbuf):
                call(i)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    if graph:
        g.replay()
    else:
        for i in range(nbuf):
            call(i)
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) * 1e3 / nbuf
    rows = []
    for i in range(nbuf):
        t = wss[i][wb:wb + 128 * 256].cpu().numpy().view(np.uint64).reshape(256, 16).astype(np.int64)
        t0 = t[:, 0].min()
        rel = (t - t0) / 100.0  # us (columns 0-5, 8-11 are stamps)
        rows.append(dict(
            start_spread=rel[:, 0].max(), loaded_med=float(np.median(rel[:, 1])),
            loaded_max=rel[:, 1].max(), published_med=float(np.median(rel[:, 2])),
            published_max=rel[:, 2].max(), gathered_min=rel[:, 3].min(),
            gathered_max=rel[:, 3].max(), table_max=rel[:, 4].max(), end_med=float(np.median(rel[:, 5])),
            epochs=len(set((t[:, 12] & 0xffffffff).tolist())), end_max=rel[:, 5].max(), first_poll_back_med=float(np.median(rel[:, 11] - rel[:, 2])),
            reduced_minus_gathered_med=float(np.median(rel[:, 8] - rel[:, 3])),
            derive_med=float(np.median(rel[:, 9] - rel[:, 8])),
            lut_med=float(np.median(rel[:, 10] - rel[:, 9])),
            barrier_after_lut_med=float(np.median(rel[:, 4] - rel[:, 10])), stolen=int((t[:, 6] & 0xffffffff).sum()),
            xcc=len(set((t[:, 7] & 0xff).tolist())),
            cus=len(set(((t[:, 7] >> 32) & 0xffff0f00).tolist()))))
    keys = rows[0].keys()
    med = {k: round(float(np.median([r[k] for r in rows])), 2) for k in keys}
    mx = {k: round(float(np.max([r[k] for r in rows])), 2) for k in keys}
    gaps = []
    for i in range(1, nbuf):
        p = wss[i - 1][wb:wb + 128 * 256].cpu().numpy().view(np.uint64).reshape(256, 16)
        c = wss[i][wb:wb + 128 * 256].cpu().numpy().view(np.uint64).reshape(256, 16)
        gaps.append((int(c[:, 0].min()) - int(p[:, 5].max())) / 100.0)
    print(json.dumps(dict(us_per_call=round(us, 2), median=med, max=mx,
                          gap_prev_end_to_start_med=round(float(np.median(gaps)), 2),
                          gap_min=round(float(np.min(gaps)), 2))))


if __name__ == "__main__":
    main()
