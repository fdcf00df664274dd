"""Fused OptimLP (optimizer.py:37-180 surface) and the autograd activation path on the GPU."""

import copy
from argparse import Namespace

import numpy as np
import pytest
import torch
import torch.nn as nn

from helpers import smaq_hparams

pytestmark = pytest.mark.gpu


def _model(seed=0):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Conv2d(3, 16, 3), nn.BatchNorm2d(16), nn.ReLU(), nn.Flatten(),
                         nn.Linear(16 * 6 * 6, 10)).cuda()


def _groups(model):
    bn, other = [], []
    for m in model.modules():
        (bn if isinstance(m, nn.BatchNorm2d) else other).extend(m.parameters(recurse=False))
    return [dict(params=bn, no_weight_compression=True), dict(params=other)]


def _train(model, opt, steps=3, seed=1):
    g = torch.Generator(device="cuda").manual_seed(seed)
    for _ in range(steps):
        x = torch.randn(8, 3, 8, 8, generator=g, device="cuda")
        y = torch.randint(0, 10, (8,), generator=g, device="cuda")

        def closure():
            opt.zero_grad()
            loss = nn.functional.cross_entropy(model(x), y)
            loss.backward()
            return loss

        opt.step(closure)


def _flags(**kw):
    d = dict(compress_weights=True, compress_gradients=True, compress_momentum_vectors=True)
    d.update(kw)
    return Namespace(**d)


@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
@pytest.mark.parametrize("sr", [False, True])
def test_fused_equals_per_tensor(opt_name, sr):
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.optimizer import OptimLP, TaggedQuant, wrap_optimizer

    results = []
    for fused in (True, False):
        model = _model()
        base = (torch.optim.SGD(_groups(model), lr=0.1, momentum=0.9) if opt_name == "sgd"
                else torch.optim.Adam(_groups(model), lr=1e-2))
        codec = SmartFP(smaq_hparams(stochastic_rounding=sr, smq_seed=7))
        if fused:
            opt = wrap_optimizer(base, codec, _flags())
            assert isinstance(opt, OptimLP) and isinstance(opt.grad_quant, TaggedQuant)
        else:  # opaque callables -> the reference's per-tensor calls
            opt = OptimLP(base,
                          weight_quant=lambda t, **kw: codec(t, tag="optimizer_weight", **kw),
                          grad_quant=lambda t, **kw: codec(t, tag="optimizer_grad", **kw),
                          momentum_quant=lambda t, **kw: codec(t, tag="optimizer_momentum", **kw))
        _train(model, opt)
        results.append([p.detach().cpu().numpy() for p in model.parameters()])
        if opt_name == "adam":
            for st in base.state.values():
                assert (st["exp_avg_sq"] >= 0).all()
    same = total = 0
    for a, b in zip(*results):
        same += int((a == b).sum())
        total += a.size
        assert np.allclose(a, b, atol=0.05, rtol=0.05)
    assert same / total > 0.97, same / total  # identical RNG streams and arithmetic per tensor


def test_bn_weights_untouched_and_logging():
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.optimizer import wrap_optimizer

    model = _model()
    base = torch.optim.SGD(_groups(model), lr=0.0, momentum=0.0)
    codec = SmartFP(smaq_hparams(measure_compression_ratio=True))
    logs = []
    codec.log_custom = lambda d: logs.append(d)
    bn_before = [p.detach().clone() for p in model[1].parameters()]
    opt = wrap_optimizer(base, codec, _flags())
    _train(model, opt, steps=1)
    for a, b in zip(bn_before, model[1].parameters()):
        assert torch.equal(a, b)  # lr 0 and no_weight_compression: BN weights exactly unchanged
    tags = {k for d in logs for k in d if k.startswith("compression_ratio_")}
    assert tags == {"compression_ratio_optimizer_grad", "compression_ratio_optimizer_weight"}
    n_params = sum(1 for _ in model.parameters())
    # grads twice (pre + post closure) for every parameter, weights for the non-BN parameters
    assert len(logs) == 2 * n_params + (n_params - 2)


def test_autograd_compressor_path():
    """The reference's Compressor (autograd.py:18-47) pattern: compress activations forward and
    grad-maps backward through the codec; training signals stay close to uncompressed."""
    from smart_compress_amd.compress.smart import SmartFP

    codec = SmartFP(smaq_hparams())

    class Fn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return codec(x, tag="forward_autograd")

        @staticmethod
        def backward(ctx, g):
            return codec(g, tag="backward_autograd")

    torch.manual_seed(0)
    net = nn.Sequential(nn.Conv2d(3, 8, 3), nn.ReLU(), nn.Conv2d(8, 4, 3)).cuda()
    x = torch.randn(4, 3, 16, 16, device="cuda", requires_grad=True)
    ref = net(x).square().mean()
    ref.backward()
    gref = x.grad.clone()
    x.grad = None
    h = Fn.apply(net[0](x))
    out = Fn.apply(net[2](net[1](h))).square().mean()
    out.backward()
    assert abs(out.item() - ref.item()) / ref.item() < 0.05
    cos = torch.nn.functional.cosine_similarity(x.grad.flatten(), gref.flatten(), dim=0).item()
    assert cos > 0.95
