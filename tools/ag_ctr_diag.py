"""Arrival-counter diagnosis for the autograd graph variant: capture one VGG training step with
SmaQ on every activation / grad-map (as bench.py --config autograd), replay it, and print the
workspace's 64 tagged counter words (tag, count) after each replay, plus whether the host saw
the codec's stream as capturing. Run with SMQ_DEFER_MAX_N=0 to force the counter path."""

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd")]

from argparse import Namespace  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import bench  # noqa: E402
from smart_compress_amd import _native as N  # noqa: E402
from smart_compress_amd.compress.smart import SmartFP  # noqa: E402
from smart_compress_amd.util.pytorch.autograd import register_autograd_module  # noqa: E402


def words(ws):
    off = N.SMQ_WS_SAMPLES_OFFSET + 8 * N.SMQ_MAX_DEVICE_SAMPLES
    w = ws[off: off + 512].cpu().numpy().view(np.uint64)
    return [(int(v) >> 32, int(v) & 0xFFFFFFFF) for v in w]


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    x = torch.randn(128, 3, 32, 32, device=dev)
    t = torch.randint(0, 10, (128,), device=dev)
    net = bench._vgg_cifar().to(dev)
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
    codec = SmartFP(bench.smaq_hparams())
    seen = []

    def fn(v, tag=None, **kw):
        st = torch.cuda.current_stream()
        seen.append((v.numel(), st.cuda_stream, torch.cuda.is_current_stream_capturing()))
        return codec(v, tag=tag, **kw)

    register_autograd_module(net, fn, Namespace(compress_forward=True, compress_backward=True,
                                                use_batch_norm=False))

    def step():
        opt.zero_grad(set_to_none=False)
        F.cross_entropy(net(x), t).backward()
        opt.step()

    codec.graph_safe(device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    seen.clear()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    print("captured calls:", len(seen), "streams:", sorted({s_ for _, s_, _ in seen}),
          "capturing flags:", sorted({c for _, _, c in seen}))
    wss = [(k, v.data_ptr()) for k, v in N._ws.items() if k[0] == "smaq"]
    print("smaq workspaces:", wss)
    for r in range(3):
        g.replay()
        torch.cuda.synchronize()
        for k, v in N._ws.items():
            if k[0] == "smaq":
                w = words(v)
                print(f"replay {r} ws stream {k[2]}: nonzero words",
                      [(i, tg, c) for i, (tg, c) in enumerate(w) if tg or c][:70])


if __name__ == "__main__":
    main()
