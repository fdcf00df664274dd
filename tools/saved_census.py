"""What the packed-saved ResNet-34 step holds for backward (measurement script, not product): every
tensor autograd saves during the forward inside PackedActivations, classified —
  packed   a codec output held as its SmaQ stream (util/pytorch/saved.py _Saved),
  kept     a codec output whose stream did not fit its capacity (the fp32 activation kept),
  raw      anything else, by what produced it: a parameter (resident anyway), a codec output
           modified in place after the codec (e.g. BasicBlock's `out += identity`, an in-place
           ReLU: its stream no longer describes it), or a tensor no codec produced (the input
           batch, pooling / ReLU / BN outputs of unwrapped modules, BN's saved statistics);
with bytes counted once per storage. Also the step's memory: allocated before the forward, held
after it (before backward), peak — for the packed step, the SmartFP step and the uncompressed one.

python tools/saved_census.py [out.json]"""

import collections
import json
import os
import sys
from argparse import Namespace

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import bench  # noqa: E402
from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd.compress.packed import SmartFPPacked  # noqa: E402
from smart_compress_amd.compress.smart import SmartFP  # noqa: E402
from smart_compress_amd.util.pytorch.autograd import register_autograd_module  # noqa: E402
from smart_compress_amd.util.pytorch import saved as S  # noqa: E402

dev = torch.device("cuda", 0)
flags = Namespace(compress_forward=True, compress_backward=True, use_batch_norm=False)
MiB = 1 << 20


def _meta(v):
    """A saved tensor's storage key, bytes, shape and dtype (no reference to it: the census must
    not keep saved tensors alive)."""
    st = v.untyped_storage()
    return st.data_ptr(), st.nbytes(), list(v.shape), str(v.dtype)


def run(kind):
    torch.manual_seed(0)
    net = bench._ResNet().to(dev)
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
    acts = None
    if kind == "smartfp":
        register_autograd_module(net, SmartFP(smaq_hparams()), flags)
    elif kind == "packed":
        acts = S.PackedActivations(SmartFPPacked(smaq_hparams()))
        register_autograd_module(net, acts, flags)
    x = torch.randn(128, 3, 32, 32, device=dev)
    t = torch.randint(0, 10, (128,), device=dev)
    params = {p.untyped_storage().data_ptr() for p in net.parameters()}

    def step(census=None):
        opt.zero_grad(set_to_none=False)
        if acts is None:
            hooks = None
            if census is not None:
                def pack(v):
                    census.append(("raw", _meta(v), None))
                    return v
                hooks = torch.autograd.graph.saved_tensors_hooks(pack, lambda v: v)
                hooks.__enter__()
            loss = F.cross_entropy(net(x), t)
            if hooks is not None:
                hooks.__exit__(None, None, None)
        else:
            if census is not None:
                inner = acts._pack

                def pack(v):
                    codec_out = v.is_cuda and v.data_ptr() in acts._live
                    h = inner(v)
                    census.append(("packed" if isinstance(h, S._Saved) else
                                   ("raw:codec output (changed in place / a view)" if codec_out
                                    else "raw"), _meta(v), h))
                    return h
                acts._pack = pack
            with acts:
                loss = F.cross_entropy(net(x), t)
            if census is not None:
                acts._pack = inner
        torch.cuda.synchronize()
        held = torch.cuda.memory_allocated(dev)
        loss.backward()
        opt.step()
        torch.cuda.synchronize()
        return held

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    census = []
    base = torch.cuda.memory_allocated(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    held = step(census)
    peak = torch.cuda.max_memory_allocated(dev)
    seen, cls = set(), collections.OrderedDict()
    for kind_, (key, nbytes, shape, dtype), h in census:
        if kind_ == "packed":
            if h.y is not None:  # kept: the stream did not fit
                kind_ = "kept"
            else:
                key = ("stream", h.packed.data.data_ptr())
                nbytes = h.packed.data.numel()
        else:
            if key in params:
                kind_ = "raw:parameter"
            elif kind_ == "raw":
                kind_ = "raw:activation / statistics"
        if key in seen:
            continue
        seen.add(key)
        c = cls.setdefault(kind_, {"tensors": 0, "mib": 0.0, "largest": []})
        c["tensors"] += 1
        c["mib"] += nbytes / MiB
        c["largest"].append((round(nbytes / MiB, 2), shape, dtype))
    for c in cls.values():
        c["mib"] = round(c["mib"], 1)
        c["largest"] = sorted(c["largest"], reverse=True)[:6]
    return {"kind": kind, "resident_mib": round(base / MiB, 1),
            "held_for_backward_mib": round((held - base) / MiB, 1),
            "step_peak_above_resident_mib": round((peak - base) / MiB, 1),
            "saved_by_class": cls}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    res = [run(k) for k in ("uncompressed", "smartfp", "packed")]
    for r in res:
        print(json.dumps(r), flush=True)
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
