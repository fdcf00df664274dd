"""Fused OptimLP (optimizer.py:37-180 surface) and the autograd activation path on the GPU."""

import copy
from argparse import Namespace

import numpy as np
import pytest
import torch
import torch.nn as nn

from helpers import n_diff_f32, same_f32, smaq_hparams

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
    # the fused multi-tensor call computes each tensor's statistics in the single-tensor
    # partition and reduction order (csrc/smaq_multi.hip), at the same stream offsets: every
    # parameter after training is bit-identical
    for a, b in zip(*results):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


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


def _cnn():
    def block(cin, cout):
        return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout),
                             nn.ReLU())

    return nn.Sequential(block(3, 16), block(16, 16), nn.MaxPool2d(2), block(16, 32),
                         block(32, 32), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10))


def test_register_autograd_module_every_call_bitexact():
    """autograd.py:50-77 at model scale: a CNN's forward activations and backward grad-maps all go
    through SmartFP (BN variant on); every recorded call equals the oracle bit for bit (device
    statistics, counter RNG); the packed codec gives the identical training step."""
    from argparse import Namespace

    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress import SmartFP, SmartFPPacked
    from smart_compress_amd.util.pytorch.autograd import register_autograd_module

    flags = Namespace(compress_forward=True, compress_backward=True, use_batch_norm=True)
    hp = smaq_hparams(use_batch_norm=True)

    def run(cls, record):
        torch.manual_seed(3)
        net = _cnn().cuda()
        codec = cls(hp)
        codec.rng.seed, codec.rng.offset = 99, 0
        calls = []

        def compress(x, tag=None, **kw):
            seed, off = codec.rng.seed, codec.rng.offset
            y = codec(x, tag=tag, **kw)
            if record and y is not x:
                ws = N._ws[("smaq", 0, N.stream_ptr(x.device))]  # this stream's workspace
                calls.append((x.detach().clone(), y.detach().clone(), seed, off,
                              SmartFP.read_stats(ws), kw.get("batch_norm_stats")))
            return y

        register_autograd_module(net, compress, flags)
        x = torch.randn(32, 3, 32, 32, device="cuda", requires_grad=True)
        loss = torch.nn.functional.cross_entropy(net(x), torch.arange(32, device="cuda") % 10)
        loss.backward()
        return loss.detach(), x.grad.detach().clone(), calls

    loss, grad, calls = run(SmartFP, True)
    assert torch.isfinite(loss) and len(calls) >= 20
    for xin, y, seed, off, st, bn in calls:
        xn = xin.cpu().numpy()
        u = orng.uniforms(seed, off, xn.size).reshape(xn.shape)
        bn_np = None if bn is None else (bn[0].cpu().numpy(), bn[1].cpu().numpy())
        y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], osmaq.SmaqConfig(), u, bn=bn_np)
        assert same_f32(y.cpu().numpy(), y_or), (xin.shape, n_diff_f32(y.cpu().numpy(), y_or))
    hp.use_batch_norm = False  # the packed container has no BN variant
    flags.use_batch_norm = False
    l1, g1, _ = run(SmartFP, False)
    l2, g2, _ = run(SmartFPPacked, False)
    assert torch.equal(l1, l2) and torch.equal(g1.view(torch.int32), g2.view(torch.int32))


@pytest.mark.parametrize("fused", [True, False])
def test_acc_quant_keeps_full_precision_accumulator(fused):
    """optimizer.py:63-67, 83-86, 101-107: with acc_quant the inner step updates weight_acc (swapped
    in as p.data) and the weights are quantised into NEW tensors — the accumulator keeps the full
    precision update. The fused weight launch must not write through p.data in that case."""
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.optimizer import OptimLP, TaggedQuant

    model = _model()
    base = torch.optim.SGD(_groups(model), lr=0.1, momentum=0.9)
    codec = SmartFP(smaq_hparams(smq_seed=3))
    if fused:
        wq = TaggedQuant(codec, "optimizer_weight")
    else:
        def wq(t, **kw):
            return codec(t, tag="optimizer_weight", **kw)
    opt = OptimLP(base, weight_quant=wq, acc_quant=lambda t, **kw: t)
    params = [p for g in opt.param_groups for p in g["params"]]
    _train(model, opt, steps=2)
    torch.cuda.synchronize()
    quantised = [g for g in opt.param_groups if not g.get("no_weight_compression", False)]
    for g in quantised:
        for p in g["params"]:
            acc = opt.weight_acc[p]
            assert p.data.data_ptr() != acc.data_ptr()  # p now holds a new, quantised tensor
            if p.numel() >= 8:
                # the accumulator is not on the SmaQ grid of its own statistics: quantising it
                # again changes it; the weights are already quantised values
                assert not torch.equal(acc, p.data)
    # BN group (no_weight_compression): p.data stays the accumulator itself
    for p in opt.param_groups[0]["params"]:
        assert p.data.data_ptr() == opt.weight_acc[p].data_ptr()
    assert len(params) == len(opt.weight_acc)
