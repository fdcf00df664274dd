"""The C host path (csrc/torchfast.cpp, module _smqtorch) against the Python paths it shortcuts.

SmartFP.__call__ (smart.py:110-190) on a device tensor, S2FP8.__call__ (s2fp8.py:27-48) on an fp32
device tensor and Compressor.forward / backward with a SmartFP codec (autograd.py:18-47) go
through one C call each. Every value must equal the Python path's bit for bit: the same outputs,
the same random-stream positions, the same workspace header, the same gradients of a training
step — and the C path must actually be the one taken."""

from argparse import Namespace

import pytest
import torch
import torch.nn as nn

from helpers import smaq_hparams

pytestmark = pytest.mark.gpu


def _N():
    from smart_compress_amd import _native as N

    assert N.torch_fast() is not None, "_smqtorch was not built next to libsmq.so"
    return N


def _python_path(codec):
    """Force the codec onto its Python paths (the C state marked unavailable)."""
    object.__setattr__(codec, "_hot", False)
    return codec


def _pair(hp, seed=7, offset=123):
    from smart_compress_amd.compress.smart import SmartFP

    a, b = SmartFP(hp), _python_path(SmartFP(hp))
    for c in (a, b):
        c.rng.seed, c.rng.offset = seed, offset
    return a, b


def _eq(a, b):
    return torch.equal(a.view(torch.int32), b.view(torch.int32))


@pytest.mark.parametrize("dtype,precision", [(torch.float32, 32), (torch.bfloat16, 32),
                                             (torch.float16, 16), (torch.bfloat16, 16)])
@pytest.mark.parametrize("n", [9, 4099, 1 << 20, 3_000_001, 9_000_000])
def test_smartfp_c_path_equals_python_path(dtype, precision, n):
    _N()
    hp = smaq_hparams(precision=precision)
    fast, slow = _pair(hp)
    gen = torch.Generator(device="cuda").manual_seed(n)
    x = (torch.randn(n, generator=gen, device="cuda") * 2 + 0.3).to(dtype)
    for all_positive in (False, True, False):
        xi = x.abs() if all_positive else x
        y1 = fast(xi, all_positive=all_positive)
        y2 = slow(xi, all_positive=all_positive)
        torch.cuda.synchronize()
        assert y1.dtype == torch.float32 and y1.shape == xi.shape
        assert _eq(y1, y2)
        assert fast.rng.offset == slow.rng.offset
    assert fast._hot not in (None, False)  # the C path served these calls


def test_smartfp_c_path_header_and_views():
    """Same workspace header as the Python path; non-contiguous and offset views; shapes kept."""
    from smart_compress_amd.compress.smart import SmartFP

    N = _N()
    hp = smaq_hparams()
    fast, slow = _pair(hp)
    base = torch.randn(64, 3, 33, 35, device="cuda")
    for x in (base, base.transpose(1, 3), base[:, 1:], base.reshape(-1)[5:]):
        y1 = fast(x)
        torch.cuda.synchronize()
        h1 = SmartFP.read_stats(N._ws[("smaq", 0, N.stream_ptr(x.device))])
        y2 = slow(x)
        torch.cuda.synchronize()
        h2 = SmartFP.read_stats(N._ws[("smaq", 0, N.stream_ptr(x.device))])
        assert y1.shape == x.shape and _eq(y1, y2)
        assert h1 == h2


def test_smartfp_c_path_flags_changed_and_declined():
    """A flag changed between calls takes effect (the state is rebuilt); modes the C path does not
    serve (range / sampled statistics, tensors below min_size, CPU tensors, fp64) give what the
    Python path gives; replacing the random stream re-keys the C path."""
    from smart_compress_amd._native import RngState

    _N()
    hp = smaq_hparams()
    fast, slow = _pair(hp)
    x = torch.randn(70_000, device="cuda")
    for change in (dict(num_bits_main=4), dict(stochastic_rounding=False),
                   dict(use_range_std_dev=True), dict(use_range_std_dev=False),
                   dict(use_sample_stats=True), dict(use_sample_stats=False),
                   dict(min_size=100_000), dict(min_size=8), dict(outlier_std_dev_threshold=3.0)):
        for k, v in change.items():
            setattr(hp, k, v)
        y1, y2 = fast(x), slow(x)
        if hp.min_size > x.numel():
            assert y1 is x and y2 is x
        else:
            assert _eq(y1, y2), change
        assert fast.rng.offset == slow.rng.offset
    # the constants the reference reads per call (smart.py:154, 162), assigned after the first
    # call: the C state is rebuilt from them
    for attr, val in (("range_normal", 11.0), ("range_outlier", 30.0),
                      ("clamped_range", (1e-4, 1e4))):
        for c in (fast, slow):
            setattr(c, attr, val)
        _python_path(slow)
        y1, y2 = fast(x), slow(x)
        assert _eq(y1, y2), attr
        assert fast._hot not in (None, False)
    for c in (fast, slow):
        c.rng = RngState(1234)
    _python_path(slow)  # (replacing rng re-keys, i.e. resets, the C state)
    assert _eq(fast(x), slow(x)) and fast._hot not in (None, False)
    xc = torch.randn(5000)
    assert _eq(fast(xc), slow(xc))
    xd = torch.randn(5000, device="cuda", dtype=torch.float64)
    assert torch.equal(fast(xd), slow(xd))


def test_smartfp_c_path_graph_safe_and_capture():
    """graph_safe(True) takes the Python path (device counter); after graph_safe(False) the C path
    continues the same stream."""
    _N()
    hp = smaq_hparams()
    fast, slow = _pair(hp)
    x = torch.randn(1 << 18, device="cuda")
    fast.graph_safe(True, device="cuda")
    slow.graph_safe(True, device="cuda")
    assert _eq(fast(x), slow(x))
    assert fast._hot is False
    fast.graph_safe(False)
    slow.graph_safe(False)
    _python_path(slow)
    assert _eq(fast(x), slow(x)) and fast.rng.offset == slow.rng.offset
    assert fast._hot not in (None, False)


def _cnn(inplace=True):
    def block(cin, cout):
        return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout),
                             nn.ReLU(inplace=inplace))

    return nn.Sequential(block(3, 16), block(16, 16), nn.MaxPool2d(2), block(16, 32),
                         block(32, 32), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10))


@pytest.mark.parametrize("fwd,bwd", [(True, True), (True, False), (False, True)])
def test_autograd_c_node_equals_python_function(fwd, bwd):
    """register_autograd_module with the SmartFP codec itself (C node) vs the same codec behind a
    Python callable (the Python Function): loss, every parameter gradient and the input gradient
    bit for bit over two SGD steps, the same number of codec positions consumed."""
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.autograd import register_autograd_module

    _N()
    flags = Namespace(compress_forward=fwd, compress_backward=bwd, use_batch_norm=False)

    def run(direct):
        torch.manual_seed(3)
        # (without forward compression the Function returns its input, a view an in-place ReLU may
        # not modify — in the reference too: autograd.py:29-30)
        net = _cnn(inplace=fwd).cuda()
        codec = SmartFP(smaq_hparams())
        codec.rng.seed, codec.rng.offset = 99, 0
        fn = codec if direct else (lambda v, tag=None, **kw: codec(v, tag=tag, **kw))
        register_autograd_module(net, fn, flags)
        opt = torch.optim.SGD(net.parameters(), lr=0.05, momentum=0.9)
        g = torch.Generator(device="cuda").manual_seed(5)
        names = set()
        out = []
        for _ in range(2):
            x = torch.randn(16, 3, 32, 32, device="cuda", generator=g, requires_grad=True)
            opt.zero_grad()
            y = net(x)
            todo, seen = [y.grad_fn], set()
            while todo:  # every node of the graph
                fn_ = todo.pop()
                if fn_ is None or id(fn_) in seen:
                    continue
                seen.add(id(fn_))
                names.add(fn_.name())
                todo.extend(f for f, _ in fn_.next_functions)
            loss = nn.functional.cross_entropy(y, torch.arange(16, device="cuda") % 10)
            loss.backward()
            opt.step()
            out.append((loss.detach(), x.grad.clone(),
                        [p.grad.clone() for p in net.parameters()]))
        return out, codec.rng.offset, names

    # MIOpen's weight-gradient kernels split K with atomics: deterministic algorithms, so that the
    # parameter gradients of the two runs can be compared bit for bit
    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        a, off_a, names_a = run(True)
        b, off_b, names_b = run(False)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert off_a == off_b > 0
    if fwd:
        assert "SmaqCompressBackward" in names_a and "SmaqCompressBackward" not in names_b
    for (la, xa, ga), (lb, xb, gb) in zip(a, b):
        assert _eq(la, lb) and _eq(xa, xb)
        assert all(_eq(p, q) for p, q in zip(ga, gb))


def test_autograd_c_node_no_grad_and_half():
    """Under no_grad the C path returns a plain tensor; a bf16 activation gets an fp32 output and
    a bf16 input gradient (the engine's cast), equal to the Python Function's."""
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.autograd import Compressor

    _N()
    codec = SmartFP(smaq_hparams())
    comp = Compressor(codec)
    x = torch.randn(4096, device="cuda", requires_grad=True)
    with torch.no_grad():
        y = comp(x)
    assert y.grad_fn is None and not y.requires_grad
    res = []
    for direct in (True, False):
        codec.rng.seed, codec.rng.offset = 5, 0
        c = Compressor(codec if direct else (lambda v, tag=None, **kw: codec(v, tag=tag, **kw)))
        xb = torch.randn(128, 64, device="cuda", generator=torch.Generator(
            device="cuda").manual_seed(1)).to(torch.bfloat16).requires_grad_(True)
        yb = c(xb)
        (yb * torch.linspace(-1, 1, 64, device="cuda")).sum().backward()
        res.append((yb.detach(), xb.grad.clone()))
        assert yb.dtype == torch.float32 and xb.grad.dtype == torch.bfloat16
    assert _eq(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_s2fp8_c_path_equals_python_path():
    from smart_compress_amd.compress.s2fp8 import S2FP8
    from smart_compress_amd.util.pytorch import quantization as q

    N = _N()
    hp = S2FP8.add_argparse_args(__import__("argparse").ArgumentParser()).parse_args([])
    hp.precision = 32
    codec = S2FP8(hp)
    x = torch.randn(32, 128, 768, device="cuda")
    outs = []
    for use_c in (True, False):
        q.quant_rng().seed, q.quant_rng().offset = 11, 4096
        if not use_c:
            N._torch_fast, saved = None, N._torch_fast
        try:
            outs.append((codec(x), codec(x[:, :, 1:]), codec(x[:3]), q.quant_rng().offset))
        finally:
            if not use_c:
                N._torch_fast = saved
    for a, b in zip(outs[0][:3], outs[1][:3]):
        assert _eq(a, b)
    assert outs[0][3] == outs[1][3]


@pytest.mark.parametrize("field,value", [("min_size", 8.0), ("precision", "32")])
def test_smartfp_c_path_declines_non_int_hparams(field, value):
    """min_size / precision that are not Python ints (a hand-built Namespace, a config file): the C
    state declines instead of raising, and the Python path serves the call with the same result."""
    _N()
    hp = smaq_hparams()
    setattr(hp, field, value)
    fast, slow = _pair(hp)
    x = torch.randn(70_000, device="cuda")
    assert _eq(fast(x), slow(x))
    assert fast.rng.offset == slow.rng.offset
