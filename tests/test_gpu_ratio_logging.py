"""--measure_compression_ratio on the fast path (csrc/torchfast.cpp + smq_smaq_roundtrip_counted /
smq_smaq_multi_size_metrics) against the host path it replaces.

Every reference script trains with the flag (scripts/train.ps1:7-13, .vscode/launch.json:39): per
SmartFP call the reference logs compression_ratio / new_size / orig_size (smart.py:184-188,
base.py:72-102), converting each to a Python float — a device->host synchronisation per call. The
fast path leaves the values on the device (0-dim fp64 tensors the logger converts when it consumes
them). The logged keys, their order and their values must equal the host path's for every call:
eager calls of every size class (single launch, two launches, below min_size), half inputs,
the autograd wrapper's forward / backward tags, and the optimizer_* tags of the fused OptimLP."""

from argparse import Namespace

import pytest
import torch
import torch.nn as nn

from helpers import smaq_hparams

pytestmark = pytest.mark.gpu


def _python_path(codec):
    object.__setattr__(codec, "_hot", False)
    return codec


def _pair(hp, seed=11, offset=5):
    from smart_compress_amd.compress.smart import SmartFP

    a, b = SmartFP(hp), _python_path(SmartFP(hp))
    for c in (a, b):
        c.rng.seed, c.rng.offset = seed, offset
    logs = ([], [])
    a.log = lambda k, v, **kw: logs[0].append((k, v, kw))
    b.log = lambda k, v, **kw: logs[1].append((k, v, kw))
    return a, b, logs


def _same_logs(fast, slow, device_values=True):
    """Same keys, order, reduce_fx and values; the fast path's counted values are device tensors."""
    assert [k for k, _, _ in fast] == [k for k, _, _ in slow]
    n_dev = 0
    for (k, v, kw), (k2, v2, kw2) in zip(fast, slow):
        assert sorted(kw) == sorted(kw2), k
        if torch.is_tensor(v):
            assert v.is_cuda and v.dim() == 0 and v.dtype == torch.float64, k
            n_dev += 1
            v = v.item()
        assert not torch.is_tensor(v2)
        assert float(v) == float(v2), (k, float(v), float(v2))
    if device_values:
        assert n_dev > 0
    return n_dev


def _eq(a, b):
    return torch.equal(a.view(torch.int32), b.view(torch.int32))


@pytest.mark.parametrize("dtype,precision", [(torch.float32, 32), (torch.bfloat16, 32),
                                             (torch.float16, 16)])
def test_counted_calls_equal_host_path(dtype, precision):
    from smart_compress_amd import _native as N

    assert N.torch_fast() is not None
    hp = smaq_hparams(measure_compression_ratio=True, precision=precision)
    fast, slow, logs = _pair(hp)
    g = torch.Generator(device="cuda").manual_seed(3)
    # single launch (70K, 4099, 1M, 3M), two launches (9M), below min_size (5), ReLU-like data
    for i, n in enumerate((70_000, 4099, 1 << 20, 5, 3_000_001, 9_000_000)):
        x = (torch.randn(n, generator=g, device="cuda") * (1 + i) + 0.2 * i).to(dtype)
        for ap in (False, True):
            xi = x.relu() if ap else x
            y1 = fast(xi, tag=f"t{i}", all_positive=ap)
            y2 = slow(xi, tag=f"t{i}", all_positive=ap)
            if n < hp.min_size:
                assert y1 is xi and y2 is xi
            else:
                assert _eq(y1, y2)
    assert fast.rng.offset == slow.rng.offset
    assert fast._hot not in (None, False)  # the C path served them
    n_dev = _same_logs(*logs)
    assert n_dev == 6 * 10  # 6 device values (3 metrics, with and without the tag) per counted call
    # the values are what the host path computes from the reference's formula
    for k, v, kw in logs[0]:
        if k.startswith("new_size") or k.startswith("orig_size"):
            assert "reduce_fx" in kw


def test_counted_autograd_forward_and_backward_tags():
    """Compressor with a SmartFP codec (the C autograd node): the forward_autograd and
    backward_autograd calls log what the Python Function path logs, in the same order."""
    from smart_compress_amd.util.pytorch.autograd import register_autograd_module

    hp = smaq_hparams(measure_compression_ratio=True)
    outs = []
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    for fast_path in (True, False):
        from smart_compress_amd.compress.smart import SmartFP

        codec = SmartFP(hp)
        if not fast_path:
            _python_path(codec)
        codec.rng.seed, codec.rng.offset = 4, 0
        logged = []
        codec.log = lambda k, v, _l=logged, **kw: _l.append((k, v, kw))
        torch.manual_seed(0)
        net = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1), nn.BatchNorm2d(16), nn.ReLU(),
                            nn.Conv2d(16, 16, 3, padding=1), nn.AdaptiveAvgPool2d(1),
                            nn.Flatten(), nn.Linear(16, 10)).cuda()
        register_autograd_module(net, codec, Namespace(compress_forward=True, compress_backward=True,
                                                       use_batch_norm=False))
        x = torch.randn(32, 3, 32, 32, device="cuda", generator=torch.Generator(
            device="cuda").manual_seed(1))
        loss = nn.functional.cross_entropy(net(x), torch.arange(32, device="cuda") % 10)
        loss.backward()
        outs.append((logged, loss.detach(), [p.grad.clone() for p in net.parameters()]))
        if fast_path:
            assert codec._hot not in (None, False)
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    (lf, l1, g1), (ls, l2, g2) = outs
    assert _eq(l1, l2) and all(_eq(a, b) for a, b in zip(g1, g2))
    tags = {k for k, _, _ in lf if k.startswith("compression_ratio_")}
    assert tags == {"compression_ratio_forward_autograd", "compression_ratio_backward_autograd"}
    _same_logs(lf, ls)


def test_counted_optimizer_tags_device_metrics():
    """The fused OptimLP (one SmaqMulti call per quantiser loop): the optimizer_* metrics go to
    log_custom with the same values as the host read of the counts, without reading them."""
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.optimizer import OptimLP, wrap_optimizer

    flags = Namespace(compress_weights=True, compress_gradients=True,
                      compress_momentum_vectors=True)
    res = []
    for device_metrics in (True, False):
        torch.manual_seed(0)
        model = nn.Sequential(nn.Linear(64, 256), nn.ReLU(), nn.Linear(256, 10)).cuda()
        codec = SmartFP(smaq_hparams(measure_compression_ratio=True))
        codec.rng.seed, codec.rng.offset = 9, 0
        logs = []
        codec.log_custom = lambda d, _l=logs: _l.append(d)
        opt = wrap_optimizer(torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9), codec,
                             flags)
        prev = OptimLP.device_metrics
        OptimLP.device_metrics = device_metrics
        try:
            for step in range(2):
                x = torch.randn(128, 64, device="cuda",
                                generator=torch.Generator(device="cuda").manual_seed(step))
                opt.zero_grad()
                nn.functional.cross_entropy(model(x), torch.arange(128, device="cuda") % 10
                                            ).backward()
                opt.step()
        finally:
            OptimLP.device_metrics = prev
        res.append((logs, [p.detach().clone() for p in model.parameters()]))
    (ld, pd), (lh, ph) = res
    assert all(_eq(a, b) for a, b in zip(pd, ph))
    assert len(ld) == len(lh) > 0
    n_dev = 0
    for a, b in zip(ld, lh):
        assert list(a) == list(b)
        for k in a:
            v = a[k]
            if torch.is_tensor(v):
                assert v.is_cuda
                n_dev += 1
                v = v.item()
            assert float(v) == float(b[k]), k
    assert n_dev > 0
    tags = {k for d in ld for k in d if k.startswith("compression_ratio_")}
    assert tags == {"compression_ratio_optimizer_grad", "compression_ratio_optimizer_weight",
                    "compression_ratio_optimizer_momentum"}


def test_counted_call_refuses_graph_capture():
    """Ratio logging cannot run inside a graph capture (the logged values would be the capture's):
    the C path declines and the host path raises, as before."""
    from smart_compress_amd.compress.smart import SmartFP

    codec = SmartFP(smaq_hparams(measure_compression_ratio=True))
    codec.log = lambda *a, **k: None
    x = torch.randn(1 << 16, device="cuda")
    codec(x, tag="warm")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with pytest.raises(RuntimeError, match="graph capture"):
            with torch.cuda.graph(g, stream=s):
                codec(x, tag="captured")
    torch.cuda.synchronize()
