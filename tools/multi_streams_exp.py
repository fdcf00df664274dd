"""C5 (the fused multi-tensor SmaQ step, bench.py run_multi) as ONE SmaqMulti call against the same
148 tensors split into two calls: on one stream (the split's own cost), and on two streams (the
second call on a side stream, forked from and joined back to the current one), so that one call's
launch ramps, tails and boundaries overlap the other's work. Measurement script, not product:
µs per step over 200 steps, interleaved rounds.

python tools/multi_streams_exp.py [rounds]"""

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

import bench  # noqa: E402
from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd.util.pytorch.multi import SmaqMulti  # noqa: E402

dev = torch.device("cuda", 0)
tensors = bench.resnet34_c5_tensors(dev, 0)
outs = [torch.empty_like(t) for t in tensors]
one = SmaqMulti(smaq_hparams(), seed=1).bind(tensors, outs)
order = sorted(range(len(tensors)), key=lambda i: -tensors[i].numel())
halves = [sorted(order[0::2]), sorted(order[1::2])]
parts = [SmaqMulti(smaq_hparams(), seed=2 + j).bind([tensors[i] for i in h], [outs[i] for i in h])
         for j, h in enumerate(halves)]
side = torch.cuda.Stream(dev)


def step_one():
    one()


def step_split():
    parts[0]()
    parts[1]()


def step_two():
    cur = torch.cuda.current_stream(dev)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        parts[1]()
    parts[0]()
    cur.wait_stream(side)


kinds = {"one": step_one, "split_one_stream": step_split, "two_streams": step_two}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
res = {k: [] for k in kinds}
for f in kinds.values():
    for _ in range(50):
        f()
torch.cuda.synchronize()
for _ in range(rounds):
    for k, f in kinds.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(200):
            f()
        b.record()
        torch.cuda.synchronize()
        res[k].append(round(a.elapsed_time(b) / 200 * 1e3, 2))
print("us/step", res)
print("medians", {k: sorted(v)[len(v) // 2] for k, v in res.items()})
