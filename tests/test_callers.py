"""The reference's callers on the codec boundary, mirrored (autograd.py, hooks.py, the layer
tables of quantization.py): behaviour with a recording codec on the CPU."""

from argparse import Namespace

import pytest
import torch
import torch.nn as nn


class Recorder:
    def __init__(self, scale=1.0):
        self.calls = []
        self.scale = scale

    def __call__(self, x, tag=None, **kw):
        self.calls.append((tag, tuple(x.shape), sorted(kw)))
        return x * self.scale


def _flags(**over):
    d = dict(compress_forward=True, compress_backward=True, use_batch_norm=False)
    d.update(over)
    return Namespace(**d)


def test_compressor_directions_and_tags():
    from smart_compress_amd.util.pytorch.autograd import Compressor

    rec = Recorder(scale=2.0)
    x = torch.randn(3, 4, requires_grad=True)
    y = Compressor(rec)(x)
    y.sum().backward()
    assert [c[0] for c in rec.calls] == ["forward_autograd", "backward_autograd"]
    assert torch.equal(y, 2 * x.detach()) and torch.equal(x.grad, torch.full((3, 4), 2.0))
    for fwd, bwd in ((False, True), (True, False), (False, False)):
        rec = Recorder(scale=3.0)
        x = torch.randn(5, requires_grad=True)
        y = Compressor(rec, forward=fwd, backward=bwd)(x)
        y.sum().backward()
        assert [c[0] for c in rec.calls] == (["forward_autograd"] if fwd else []) + (
            ["backward_autograd"] if bwd else [])
        assert torch.equal(x.grad, torch.full((5,), 3.0 if bwd else 1.0))


def test_compressor_batch_norm_stats_kwarg_and_no_grad_input():
    from smart_compress_amd.util.pytorch.autograd import Compressor, process_input

    rec = Recorder()
    g, b = torch.ones(2), torch.zeros(2)
    x = torch.randn(1, 2, 3, 3, requires_grad=True)
    Compressor(rec)(x, {"batch_norm_stats": (g, b)}).sum().backward()
    assert rec.calls[0] == ("forward_autograd", (1, 2, 3, 3), ["batch_norm_stats"])
    assert process_input([1, {"other": 2}]) == ([1, {"other": 2}], {})
    rec = Recorder()
    Compressor(rec)(torch.randn(4))  # no grad needed: backward never runs
    assert [c[0] for c in rec.calls] == ["forward_autograd"]


def _net():
    return nn.Sequential(nn.Conv2d(3, 4, 3, padding=1), nn.BatchNorm2d(4), nn.ReLU(),
                         nn.Dropout(0.0), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(4, 2))


def test_register_autograd_module_selection_and_bn():
    from smart_compress_amd.util.pytorch.autograd import register_autograd_module
    from smart_compress_amd.util.pytorch.layers import is_valid_layer_type

    net = _net()
    valid = [type(m).__name__ for m in net.modules() if is_valid_layer_type(m)]
    # conv / bn / relu (activation path) / pool / linear / the Sequential container; not Dropout,
    # not Flatten (a plain module outside the selected tables)
    assert valid == ["Sequential", "Conv2d", "BatchNorm2d", "ReLU", "AdaptiveAvgPool2d", "Linear"]
    rec = Recorder()
    register_autograd_module(net, rec, _flags(use_batch_norm=True))
    x = torch.randn(2, 3, 8, 8, requires_grad=True)
    net(x).sum().backward()
    fwd = [c for c in rec.calls if c[0] == "forward_autograd"]
    assert len(fwd) == 6 and fwd[0][2] == [] and fwd[1][2] == ["batch_norm_stats"]  # conv, bn
    bn_calls = [c for c in fwd if c[2] == ["batch_norm_stats"]]
    assert len(bn_calls) == 1 and bn_calls[0][1] == (2, 4, 8, 8)
    assert sum(c[0] == "backward_autograd" for c in rec.calls) == 6


def test_global_forward_hooks():
    from smart_compress_amd.util.pytorch.hooks import register_global_hooks, wrap_optimizer

    rec = Recorder()
    assert register_global_hooks(rec, _flags(compress_forward=False)) == []
    handles = register_global_hooks(rec, _flags())
    try:
        _net()(torch.randn(2, 3, 8, 8))
    finally:
        for h in handles:
            h.remove()
    # default layer types: conv, linear, pool, normalization + activation / container paths
    assert [c[1] for c in rec.calls] == [(2, 4, 8, 8), (2, 4, 8, 8), (2, 4, 8, 8), (2, 4, 1, 1),
                                        (2, 2), (2, 2)]
    assert all(c[0] == "forward_hook" for c in rec.calls)
    n = len(rec.calls)
    _net()(torch.randn(2, 3, 8, 8))
    assert len(rec.calls) == n  # removed
    assert callable(wrap_optimizer)


def test_layer_tables_match_reference_names():
    from smart_compress_amd.util.pytorch import quantization as q

    assert q.DEFAULT_LAYER_TYPES == ["conv", "linear", "pool", "normalization"]
    assert set(q.LAYERS_TYPES) == {"conv", "linear", "pool", "pad", "activation", "normalization",
                                   "dropout", "loss"}
    assert q.is_valid_layer_type(nn.Dropout(), layer_types=["dropout"])
    with pytest.raises(AssertionError):
        q.is_valid_layer_type(nn.ReLU(), layer_types=["nope"])
