"""Where a ResNet-34 / CIFAR b128 step with PackedActivations spends its time (measurement script,
not product): ms/step of SmartFP eager and of PackedActivations (default: one stream, the C
forward call) and with its packing launches overlapped on a side stream, each
interleaved over rounds; then the host time of one forward without the GPU waiting (the forward
enqueued behind 100 large GEMMs, synchronised afterwards) and a cProfile of the packed steps.

python tools/saved_ab.py [rounds] [kinds: comma list of smartfp, smartfp_ratio, packed,
packed_overlap, packed_event (sizes by batch requests and events instead of notify words),
packed_noskip (every forward output packed, also those never saved as streams),
packed_noreplay (in-place activations of codec outputs saved as fp32, not replayed),
packed_v<MiB> (verify_bytes), packed_b<MiB> (the event path's batch)]
Also prints each kind's step peak above the memory resident before it."""

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
from smart_compress_amd.compress.smart import SmartFP  # noqa: E402
from smart_compress_amd.util.pytorch.autograd import register_autograd_module  # noqa: E402
from smart_compress_amd.util.pytorch.saved import PackedActivations  # noqa: E402

dev = torch.device("cuda", 0)
flags = Namespace(compress_forward=True, compress_backward=True, use_batch_norm=False)


def build(kind):
    torch.manual_seed(0)
    net = bench._ResNet().to(dev)
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
    acts = None
    if kind in ("smartfp", "smartfp_ratio"):
        # smartfp_ratio: --measure_compression_ratio (every reference script's setting), logged
        # into a bounded in-memory sink (bench.py autograd smaq_eager_ratio)
        codec = SmartFP(smaq_hparams(measure_compression_ratio=kind == "smartfp_ratio"))
        if kind == "smartfp_ratio":
            import collections
            sink = collections.deque(maxlen=1 << 14)
            codec.log = lambda k, v, _s=sink, **kw: _s.append((k, v))
        register_autograd_module(net, codec, flags)
    else:
        # packed_v<MiB>: PackedActivations with verify_bytes = <MiB> MiB (default: 256 for the
        # notified calls, 32 for the event path)
        vb = int(kind[len("packed_v"):]) << 20 if kind.startswith("packed_v") else None
        # packed_b<MiB>: verify_batch = <MiB> MiB for the event path (default verify_bytes); b0:
        # one batch per budget (round 6's first form: the host waited for the call it had enqueued)
        vbat = None
        if kind.startswith("packed_b"):
            vbat = int(kind[len("packed_b"):]) << 20 or None
        codec = SmartFPPacked(smaq_hparams())
        acts = PackedActivations(codec, verify_bytes=vb, overlap=kind == "packed_overlap",
                                 verify_batch=vbat)
        if kind == "packed_event":  # round 6's first form: sizes by batch requests + events
            acts._arm = lambda: (None, None)
        if kind == "packed_noskip":  # every forward output packed (no call-site skipping)
            acts._REPROBE = 1
        if kind == "packed_noreplay":  # in-place ReLUs of codec outputs saved as fp32 (round 6)
            acts.replay_inplace = False
        register_autograd_module(net, acts, flags)
    return net, opt, acts


x = torch.randn(128, 3, 32, 32, device=dev)
t = torch.randint(0, 10, (128,), device=dev)


def make_step(net, opt, acts):
    def fwd():
        if acts is None:
            return F.cross_entropy(net(x), t)
        with acts:
            return F.cross_entropy(net(x), t)

    def step():
        opt.zero_grad(set_to_none=False)
        loss = fwd()
        loss.backward()
        opt.step()
    return step, fwd


STEPS_PER_ROUND = 20


def timed(step, k=STEPS_PER_ROUND):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    kinds = (sys.argv[2] if len(sys.argv) > 2 else "smartfp,packed,packed_overlap").split(",")
    global busy
    busy = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    built = {k: build(k) for k in kinds}
    steps = {k: make_step(*built[k]) for k in kinds}
    for k in kinds:
        for _ in range(3):
            steps[k][0]()
    res = {k: [] for k in kinds}
    w0 = {k: (built[k][2].size_waits, built[k][2].size_wait_s) for k in kinds
          if built[k][2] is not None}
    for _ in range(rounds):
        for k in kinds:
            res[k].append(round(timed(steps[k][0]), 3))
    print("ms/step", res, flush=True)
    nsteps = rounds * STEPS_PER_ROUND
    print("host waits for sizes per step (count, ms)",
          {k: (round((built[k][2].size_waits - w[0]) / nsteps, 2),
               round((built[k][2].size_wait_s - w[1]) * 1e3 / nsteps, 3)) for k, w in w0.items()},
          flush=True)
    mem = {}
    for k in kinds:  # one step's peak above the memory resident before it (bench.py's measure)
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated(dev)
        torch.cuda.reset_peak_memory_stats(dev)
        steps[k][0]()
        torch.cuda.synchronize()
        mem[k] = round((torch.cuda.max_memory_allocated(dev) - base) / 2**20, 1)
    print("step peak above resident MiB", mem, flush=True)
    # host time of one forward with the device busy: the enqueue cost alone (until the context's
    # exit; a verify inside the forward would wait for the busy device, so the budget is lifted)
    for k in kinds:
        step, fwd = steps[k]
        hs = []
        for _ in range(5):
            torch.cuda.synchronize()
            for _ in range(100):  # tens of ms of device busy time ahead of the forward
                busy @ busy
            acts = built[k][2]
            if acts is not None:
                budgets = acts.verify_bytes, acts.notify_bytes
                acts.verify_bytes = acts.notify_bytes = 1 << 40
                acts.__enter__()
            t0 = time.perf_counter()
            loss = F.cross_entropy(built[k][0](x), t)
            hs.append((time.perf_counter() - t0) * 1e3)  # before the context's exit verify
            if acts is not None:
                acts.__exit__(None, None, None)
                acts.verify_bytes, acts.notify_bytes = budgets
            torch.cuda.synchronize()
            loss.backward()
            torch.cuda.synchronize()
        print(f"host forward ms ({k}, device busy):", [round(v, 3) for v in hs], flush=True)
    if "packed" not in built:
        return
    acts = built["packed"][2]
    print("packed stats", acts.stats(), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        steps["packed"][0]()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(22)


if __name__ == "__main__":
    main()
