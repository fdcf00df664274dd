"""ResNet-34 / CIFAR b128 steps with PackedActivations (verification at context exit) for a
rocprofv3 kernel trace (measurement script, not product): which launches the packed-saved step's
device time goes to. python tools/saved_trace.py [steps]"""

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tools")]

import torch  # noqa: E402

import saved_ab  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    kind = sys.argv[2] if len(sys.argv) > 2 else "packed"
    net, opt, acts = saved_ab.build(kind)
    step, _ = saved_ab.make_step(net, opt, acts)
    for _ in range(3 + steps):
        step()
    torch.cuda.synchronize()
    print(kind, "steps", steps, "stats", acts.stats() if acts else None, flush=True)


if __name__ == "__main__":
    main()
