"""Where the time of a ResNet-34 / CIFAR b128 step with PackedActivations goes (bench.py --config
autograd_resnet34, variant smaq_eager_packed_saved): forward / verify / backward wall time with
synchronisation between phases, then a cProfile of three steps (host functions by own time).

python tools/saved_profile.py"""

import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from argparse import Namespace  # noqa: E402

import bench  # noqa: E402
from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd.compress.packed import SmartFPPacked  # noqa: E402
from smart_compress_amd.util.pytorch.autograd import register_autograd_module  # noqa: E402
from smart_compress_amd.util.pytorch.saved import PackedActivations  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = bench._ResNet().to(dev)
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
    acts = PackedActivations(SmartFPPacked(smaq_hparams()))
    register_autograd_module(net, acts, Namespace(compress_forward=True, compress_backward=True,
                                                  use_batch_norm=False))
    x = torch.randn(128, 3, 32, 32, device=dev)
    t = torch.randint(0, 10, (128,), device=dev)

    def step(phases=None):
        opt.zero_grad(set_to_none=False)
        t0 = time.perf_counter()
        with acts:
            loss = F.cross_entropy(net(x), t)
            if phases is not None:
                torch.cuda.synchronize()
                phases["forward"] += time.perf_counter() - t0
        t1 = time.perf_counter()
        if phases is not None:
            phases["exit_verify"] += t1 - t0 - phases["_f"] if False else 0.0
        loss.backward()
        opt.step()
        if phases is not None:
            torch.cuda.synchronize()
            phases["backward_step"] += time.perf_counter() - t1

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ph = {"forward": 0.0, "exit_verify": 0.0, "backward_step": 0.0, "_f": 0.0}
    for _ in range(5):
        step(ph)
    print({k: round(v / 5 * 1e3, 3) for k, v in ph.items() if not k.startswith("_")}, flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    print(acts.stats())


if __name__ == "__main__":
    main()
