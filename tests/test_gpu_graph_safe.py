"""Graph-safe random streams of the float codecs, S2FP8 and the multi-tensor SmaQ launch.

With a device offset counter the first kernel of a call reads the stream position (and the call
advances it), so nothing on the host changes between calls and a captured hipGraph replays with
fresh, consecutive random streams. Contract, bit-exact:
  * C ABI: a call with *offset_counter = K equals the host-offset call at offset K, and leaves
    K + n in the counter (float_quantize, S2FP8 at precision 32 and 16, multi-tensor SmaQ);
  * codecs: eager graph-safe calls and graph replays equal the host-offset sequence of calls, and
    graph_safe(False) continues on the host from the device position;
  * the fused precision-16 float_quantize (fp16 / bf16 / fp32 in, fp16 out, one launch) equals the
    reference's x.float() -> quantise -> .half() passes.
"""

from argparse import ArgumentParser

import pytest
import torch

from helpers import smaq_hparams

pytestmark = pytest.mark.gpu


def _g():
    import gpu_calls

    return gpu_calls


def _ctr(v):
    return torch.tensor([v], dtype=torch.int64, device="cuda")


def _bits(t):
    return t.view(torch.int16 if t.element_size() == 2 else torch.int32)


@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.bfloat16])
def test_float_quant_half_out_equals_two_passes(dt):
    g = _g()
    n = (1 << 18) + 3
    x = (torch.randn(n, device="cuda") * 3).to(dt)
    for base in (x, x[1:]):  # vector and unaligned paths
        for e, m in ((5, 2), (5, 10), (8, 7), (4, 3)):
            y = g.float_quant_any(base, e, m, out_dtype=torch.float16, seed=9, offset=4)
            ref = g.float_quant(base.float().contiguous(), e, m, seed=9, offset=4).half()
            assert torch.equal(_bits(y), _bits(ref)), (dt, e, m)
            y32 = g.float_quant_any(base, e, m, seed=9, offset=4)
            assert torch.equal(_bits(y32), _bits(g.float_quant(base.float().contiguous(), e, m,
                                                                seed=9, offset=4)))


def test_float_quant_counter_equals_host_offsets():
    g = _g()
    n = (1 << 20) + 5
    x = torch.randn(n, device="cuda")
    c = _ctr(1000)
    for k in range(3):
        y = g.float_quant_any(x, 5, 2, seed=3, offset=7, counter=c)
        ref = g.float_quant(x, 5, 2, seed=3, offset=7 + 1000 + k * n)
        assert torch.equal(_bits(y), _bits(ref))
    assert int(c.item()) == 1000 + 3 * n


@pytest.mark.parametrize("precision,dt", [(32, torch.float32), (16, torch.float16),
                                          (16, torch.bfloat16)])
def test_s2fp8_counter_equals_host_offsets(precision, dt):
    g = _g()
    n = (1 << 19) + 1
    x = torch.randn(n, device="cuda").to(dt)
    c = _ctr(555)
    for k in range(2):
        y, st = g.s2fp8(x, seed=4, offset=2, precision=precision, counter=c)
        ref, _ = g.s2fp8(x, seed=4, offset=2 + 555 + k * n, precision=precision)
        assert torch.equal(_bits(y), _bits(ref))
    assert int(c.item()) == 555 + 2 * n


def _capture(fn, x):
    """Warm up on a side stream, capture one call, return (graph, static output)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(x)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        y = fn(x)
    return graph, y


@pytest.mark.parametrize("codec,precision,dt", [("FP8", 32, torch.float32),
                                                ("FP8", 16, torch.float16),
                                                ("BF16", 32, torch.float32),
                                                ("S2FP8", 32, torch.float32),
                                                ("S2FP8", 16, torch.float16)])
def test_float_codec_graph_capture(codec, precision, dt):
    """Host-offset calls 1..3 == (graph-safe warm-up, replay, replay); then the host offset resumes
    after the device position."""
    import smart_compress_amd.compress as C
    from smart_compress_amd.util.pytorch import quantization as Q

    cls = getattr(C, codec)
    hp = cls.add_argparse_args(ArgumentParser()).parse_args([])
    hp.precision = precision
    c = cls(hp)
    n = (1 << 20) + 7
    x = (torch.randn(n, device="cuda") * 2).to(dt)
    r = Q.quant_rng()
    start = r.offset
    refs = [c(x).clone() for _ in range(3)]
    torch.cuda.synchronize()
    r.offset = start
    c.graph_safe(True, device="cuda")
    try:
        graph, y_static = _capture(c, x)
        outs = []
        for _ in range(2):
            graph.replay()
            outs.append(y_static.clone())
        torch.cuda.synchronize()
    finally:
        c.graph_safe(False)
    assert r.offset == start + 3 * n
    for o, ref in zip(outs, refs[1:]):
        assert torch.equal(_bits(o), _bits(ref))
    assert not torch.equal(outs[0], outs[1])


def test_multi_bound_graph_capture():
    """SmaqMulti.bind + graph_safe: eager calls equal the host-offset mode; replays of a captured
    bound call equal the next host-offset calls."""
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    hp = smaq_hparams()
    gen = torch.Generator(device="cuda").manual_seed(3)
    sizes = [4099, 1 << 16, 3, (1 << 18) + 1, 777]
    xs = [torch.randn(s, generator=gen, device="cuda") for s in sizes]
    ys_h = [torch.empty_like(x) if x.numel() >= hp.min_size else x for x in xs]
    ys_d = [torch.empty_like(x) if x.numel() >= hp.min_size else x for x in xs]
    host = SmaqMulti(hp, seed=11)
    dev = SmaqMulti(hp, seed=11).graph_safe(True, device="cuda")
    bh, bd = host.bind(xs, ys_h), dev.bind(xs, ys_d)
    for _ in range(2):
        bh()
        bd()
        for a, b in zip(ys_h, ys_d):
            assert torch.equal(_bits(a), _bits(b))
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):  # a bound call allocates nothing: no warm-up needed
        bd()
    for _ in range(3):
        graph.replay()
        bh()
        torch.cuda.synchronize()
        for a, b in zip(ys_h, ys_d):
            assert torch.equal(_bits(a), _bits(b))
    assert dev.rng.position() == host.rng.offset


def test_optimizer_step_graph_safe_matches_host():
    """OptimLP's fused SmaQ launch follows its codec's mode: a graph-safe codec's optimizer step
    equals the host-offset step bit for bit."""
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.optimizer import wrap_optimizer

    def run(graph_safe):
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(),
                                    torch.nn.Linear(256, 10)).cuda()
        hp = smaq_hparams()
        hp.compress_weights = True
        hp.compress_gradients = True
        hp.compress_momentum_vectors = True
        codec = SmartFP(hp)
        codec.rng.seed, codec.rng.offset = 5, 0
        if graph_safe:
            codec.graph_safe(True, device="cuda")
        opt = wrap_optimizer(torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9), codec, hp)
        x = torch.randn(32, 64, device="cuda")
        for _ in range(2):
            opt.zero_grad()
            model(x).square().mean().backward()
            opt.step()
        torch.cuda.synchronize()
        return [p.detach().clone() for p in model.parameters()], codec.rng.position()

    ph, oh = run(False)
    pd, od = run(True)
    assert oh == od
    for a, b in zip(ph, pd):
        assert torch.equal(_bits(a), _bits(b))


def test_workspace_created_in_capture_keeps_counters_across_replays():
    """A SmaQ workspace first requested while a graph is being captured (torch.cuda.graph's own
    capture stream) is allocated without a zero-fill node: replays leave its arrival counters as
    the last replay set them, so every call finds its own tag (a cleared word sent all 60 calls of
    the VGG autograd graph down the re-tagging path: 14 -> 53 us per 512-workgroup statistics
    launch). Outputs still equal the host-offset calls."""
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.smart import SmartFP

    n = 13 << 20  # above the deferred-statistics limit: the statistics launch counts arrivals
    x1 = torch.randn(n, device="cuda")
    x2 = torch.randn(n, device="cuda") * 3
    dev = SmartFP(smaq_hparams())
    dev.rng.seed, dev.rng.offset = 5, 0
    dev.graph_safe(device="cuda")
    host = SmartFP(smaq_hparams())
    host.rng.seed, host.rng.offset = 5, 0
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y1 = dev(x1)
        y2 = dev(x2)
        key = ("smaq", 0, N.stream_ptr(x1.device))  # the capture stream's workspace
    ws = N._ws[key]  # created in this capture, or by an earlier test's capture on this stream
    sentinel = N.SMQ_WS_SAMPLES_OFFSET + 8 * N.SMQ_MAX_DEVICE_SAMPLES - 1  # only device draws write it
    ws[sentinel] = 0xA5
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        assert int(ws[sentinel]) == 0xA5  # no captured clear of the workspace
    refs = []
    for _ in range(2):
        refs += [host(x1), host(x2)]
    torch.cuda.synchronize()
    # replay 2 equals the host's 3rd and 4th calls
    assert torch.equal(_bits(y1), _bits(refs[2])) and torch.equal(_bits(y2), _bits(refs[3]))


@pytest.mark.parametrize("check_inf", [True, False])
def test_s2fp8_class_eager_path_equals_c_abi(check_inf):
    """S2FP8.__call__'s fp32 device path (its own stream query and cached workspace) returns what
    smq_s2fp8_roundtrip returns for the same seed and stream position, for contiguous and strided
    inputs, and advances the host stream by n per call."""
    import smart_compress_amd.compress as C
    from smart_compress_amd.util.pytorch import quantization as Q

    g = _g()
    hp = C.S2FP8.add_argparse_args(ArgumentParser()).parse_args([])
    hp.precision = 32
    hp.float_quantize_check_inf = check_inf
    c = C.S2FP8(hp)
    r = Q.quant_rng()
    base = torch.randn(96, 4097, device="cuda") * 3
    for x in (base, base[:, 1:], base.t()):
        start = r.offset
        y = c(x, tag="t")
        assert r.offset == start + x.numel()
        ref, _ = g.s2fp8(x.contiguous(), check_inf=check_inf, seed=r.seed, offset=start)
        assert y.shape == x.shape and y.dtype == torch.float32
        assert torch.equal(_bits(y.contiguous()), _bits(ref))
