"""Debug aid (not product): every codec call of the CNN of
tests/test_gpu_optim.py::test_register_autograd_module_every_call_bitexact through SmartFPPacked,
each compared with SmartFP on the same input and stream position; prints the first mismatches."""
import os
import sys
from argparse import Namespace

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd.compress import SmartFP, SmartFPPacked  # noqa: E402
from smart_compress_amd.util.pytorch.autograd import register_autograd_module  # noqa: E402


def _cnn():
    def block(cin, cout):
        return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout),
                             nn.ReLU())
    return nn.Sequential(block(3, 16), block(16, 16), nn.MaxPool2d(2), block(16, 32),
                         block(32, 32), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10))


hp = smaq_hparams()
pk, ref = SmartFPPacked(hp), SmartFP(hp)
pk.rng.seed = ref.rng.seed = 99
bad = 0
FAIL = None


def compress(x, tag=None, **kw):
    global bad
    off = pk.rng.offset
    ref.rng.offset = off
    y_ref = ref(x.detach().clone(), tag=tag)
    p = pk.compress(x)
    y = pk.decompress(p)
    torch.cuda.synchronize()
    same = torch.equal(y.view(torch.int32), y_ref.view(torch.int32))
    h = p.header()
    print(tag, tuple(x.shape), x.stride(), x.data_ptr() % 16, x.is_contiguous(), x.numel(),
          "blocks", h["n_blocks"], "data_words", h["data_words"], "same", same, flush=True)
    if not same and bad < 3:
        global FAIL
        FAIL = x.detach().clone()
        bad += 1
        # the same call again, same stream position: which side is not repeatable?
        end = pk.rng.offset
        pk.rng.offset = off
        p2 = pk.compress(x)
        y2 = pk.decompress(p2)
        ref.rng.offset = off
        y_ref2 = ref(x.detach().clone())
        pk.rng.offset = end
        torch.cuda.synchronize()
        t1, t2 = p.nbytes, p2.nbytes
        print("  stream repeat equal:", t1 == t2 and torch.equal(p.data[:t1], p2.data[:t2]),
              "decode repeat == first:", torch.equal(y2.view(torch.int32), y.view(torch.int32)),
              "SmartFP repeat == first:", torch.equal(y_ref2.view(torch.int32), y_ref.view(torch.int32)),
              "decode repeat == SmartFP repeat:", torch.equal(y2.view(torch.int32), y_ref2.view(torch.int32)),
              flush=True)
        d = (y.view(torch.int32) != y_ref.view(torch.int32)).flatten().nonzero().flatten()
        print("  first diffs at", d[:8].tolist(), "of", d.numel(), "blocks",
              sorted(set((d // 4096).tolist()))[:20], flush=True)
    return y


torch.manual_seed(3)
net = _cnn().cuda()
register_autograd_module(net, compress, Namespace(compress_forward=True, compress_backward=True,
                                                  use_batch_norm=False))
x = torch.randn(32, 3, 32, 32, device="cuda", requires_grad=True)
loss = torch.nn.functional.cross_entropy(net(x), torch.arange(32, device="cuda") % 10)
loss.backward()
print("done, mismatching calls:", bad)
