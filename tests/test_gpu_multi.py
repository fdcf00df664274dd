"""Multi-tensor SmaQ (smq_smaq_multi_f32): every tensor equals the oracle fed the tensor's own
device statistics and counter RNG stream, bit for bit; statistics within 1 ulp of fp64; in-place
aliasing; equality with the sequence of single-tensor calls."""

import numpy as np
import pytest
import torch

from helpers import same_f32, smaq_hparams, ulp_diff

pytestmark = pytest.mark.gpu

SHAPES = [(64, 3, 3, 3), (64,), (64,), (64, 64, 3, 3), (128, 64, 3, 3), (128,), (10, 512), (10,),
          (256, 128, 1, 1), (512, 256, 3, 3), (7,), (33, 17), (100003,)]


def _make(seed=0):
    gen = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.randn(s, generator=gen, device="cuda") * (0.1 + i) for i, s in enumerate(SHAPES)]


@pytest.mark.parametrize("sr", [True, False])
@pytest.mark.parametrize("inplace", [False, True])
def test_multi_vs_oracle(sr, inplace):
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    hp = smaq_hparams(stochastic_rounding=sr)
    xs = _make()
    x_np = [x.cpu().numpy() for x in xs]
    outs = [x if inplace else torch.empty_like(x) for x in xs]
    allpos = [i % 3 == 0 for i in range(len(xs))]
    m = SmaqMulti(hp, seed=42)
    m(xs, outs, all_positive=allpos)
    torch.cuda.synchronize()
    stats = m.read_stats()
    for t, (xn, y) in enumerate(zip(x_np, outs)):
        if xn.size < hp.min_size:
            assert torch.equal(y, xs[t]) if inplace else True
            continue
        st = stats[m.index_of(t)]
        mo, so = osmaq.full_stats(xn, osmaq.SmaqConfig())
        assert ulp_diff(st["mean"], mo) <= 1 and ulp_diff(st["raw_std"], so) <= 1
        cfg = osmaq.SmaqConfig(stochastic_rounding=sr)
        u = orng.uniforms(42, m.offset_of(t), xn.size) if sr else None
        y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], cfg, u, allpos[t])
        assert same_f32(y.cpu().numpy().reshape(xn.shape), y_or), t


def test_multi_repeated_calls_reuse_plan():
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    hp = smaq_hparams()
    xs = _make(1)
    ys = [torch.empty_like(x) for x in xs]
    m = SmaqMulti(hp, seed=1)
    for _ in range(3):
        m(xs, ys)
    torch.cuda.synchronize()
    assert all(torch.isfinite(y).all() for y in ys)


def test_bound_multi_equals_per_call():
    """SmaqMulti.bind (fixed buffers, no per-call Python checks) computes what the per-call path
    computes for the same random stream."""
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    torch.manual_seed(0)
    xs = [torch.randn(s, device="cuda") for s in ((300, 7), (5,), (4096 * 3 + 1,), (64, 64))]
    ys1 = [torch.empty_like(x) if x.numel() >= 8 else x for x in xs]
    ys2 = [torch.empty_like(x) if x.numel() >= 8 else x for x in xs]
    a, b = SmaqMulti(smaq_hparams(), seed=5), SmaqMulti(smaq_hparams(), seed=5)
    bound = b.bind(xs, ys2, all_positive=[False, False, True, False])
    for _ in range(2):
        a(xs, ys1, all_positive=[False, False, True, False])
        bound()
        torch.cuda.synchronize()
        for u, v in zip(ys1, ys2):
            assert torch.equal(u.view(torch.int32), v.view(torch.int32))


def test_multi_c5_full_resnet34_set():
    """BASELINE config 5 exactly as bench.py --config multi runs it: the 110 ResNet-34 (CIFAR)
    gradients + the 38 non-BN weights (fc bias included) = 148 tensors, 42,547,220 elements, in one
    bound SmaqMulti call. Every tensor equals the oracle fed its device statistics and counter
    stream bit for bit, statistics within 1 ulp of fp64, and the fused call equals the per-tensor
    SmartFP calls at the same stream offsets for EVERY tensor, bit for bit: the multi statistics
    launch computes each tensor's partials in the single-tensor partition and reduces them in its
    order (csrc/smaq_small.h, smaq_multi.hip)."""
    import bench
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    xs = bench.resnet34_c5_tensors(torch.device("cuda"), 0)
    assert len(xs) == 148 and sum(x.numel() for x in xs) == 42547220
    assert [tuple(x.shape) for x in xs] == bench.resnet34_c5_shapes()
    hp = smaq_hparams()
    ys = [torch.empty_like(x) for x in xs]
    m = SmaqMulti(hp, seed=21)
    m.bind(xs, ys)()
    torch.cuda.synchronize()
    stats = m.read_stats()
    single = SmartFP(hp)
    single.rng.seed = 21
    for t, (x, y) in enumerate(zip(xs, ys)):
        xn = x.cpu().numpy().ravel()
        st = stats[m.index_of(t)]
        mo, so = osmaq.full_stats(xn, osmaq.SmaqConfig())
        assert ulp_diff(st["mean"], mo) <= 1 and ulp_diff(st["raw_std"], so) <= 1, t
        y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], osmaq.SmaqConfig(),
                              orng.uniforms(21, m.offset_of(t), xn.size))
        assert same_f32(y.cpu().numpy().ravel(), y_or), t
        # the per-tensor path at the same offset
        single.rng.offset = m.offset_of(t)
        assert torch.equal(single(x).view(torch.int32), y.view(torch.int32)), t
        sst = SmartFP.read_stats(next(v for k, v in N._ws.items() if k[0] == "smaq"))
        assert (sst["mean"], sst["raw_std"]) == (st["mean"], st["raw_std"]), t


MODES = [dict(use_sample_stats=True), dict(use_sample_stats=True, num_samples=300),
         dict(use_sample_stats=True, use_range_std_dev=True), dict(use_range_std_dev=True),
         dict(stochastic_rounding=False, use_sample_stats=True)]


@pytest.mark.parametrize("mode", MODES, ids=lambda m: "-".join(f"{k}={v}" for k, v in m.items()))
@pytest.mark.parametrize("dt", ["f32", "f16", "bf16"])
def test_multi_modes_equal_single_calls(mode, dt):
    """Sampled (device-drawn, any k), range-std and half-input lists in one SmaqMulti call equal
    the per-tensor SmartFP calls at the same stream offsets bit for bit (statistics included)."""
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[dt]
    hp = smaq_hparams(precision=16 if dt == "f16" else 32, **mode)
    xs = [x.to(tdt) for x in _make(4)]
    m = SmaqMulti(hp, seed=8)
    ys = m(xs)
    torch.cuda.synchronize()
    stats = m.read_stats()
    single = SmartFP(hp)
    single.rng.seed = 8
    for t, (x, y) in enumerate(zip(xs, ys)):
        if x.numel() < hp.min_size:
            assert y is x
            continue
        assert y.dtype == torch.float32
        single.rng.offset = m.offset_of(t)
        ref = single(x)
        torch.cuda.synchronize()
        st = SmartFP.read_stats(N.workspace("smaq", x.device, 0))
        assert torch.equal(ref.view(torch.int32), y.view(torch.int32)), t
        assert stats[m.index_of(t)]["mean"] == st["mean"], t
        assert stats[m.index_of(t)]["raw_std"] == st["raw_std"], t


@pytest.mark.parametrize("mode", [dict(), dict(use_range_std_dev=True),
                                  dict(stochastic_rounding=False)],
                         ids=["full", "range", "trunc"])
@pytest.mark.parametrize("dt", ["f32", "f16", "bf16"])
def test_multi_full_stats_equal_single_calls(mode, dt):
    """Full statistics (the default): every size class — the small partition with one partial,
    runs of 4 / V partials per workgroup at V = 1 .. 4 (300,000; 1.18M; ResNet-34's 2,359,296;
    3M), one partial per workgroup with the lane-ahead loads (V = 5: 5M; V = 8: 8,388,611) and
    tensors above it (9M: the deferred grid; 13M: 512 workgroups), whose statistics are the
    single-tensor launch itself — equal the per-tensor SmartFP calls at the same stream offsets,
    outputs and statistics bit for bit."""
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[dt]
    hp = smaq_hparams(precision=16 if dt == "f16" else 32, **mode)
    gen = torch.Generator(device="cuda").manual_seed(31)
    sizes = [5, 4099, 65537, 300000, 1179655, 2359296, 3 * (1 << 20) + 5, 5 * (1 << 20) + 1,
             8388611, 9 << 20, 13 << 20]
    xs = [(torch.randn(n, generator=gen, device="cuda") * (0.5 + i)).to(tdt)
          for i, n in enumerate(sizes)]
    m = SmaqMulti(hp, seed=12)
    ys = m(xs)
    torch.cuda.synchronize()
    stats = m.read_stats()
    single = SmartFP(hp)
    single.rng.seed = 12
    for t, (x, y) in enumerate(zip(xs, ys)):
        if x.numel() < hp.min_size:
            assert y is x
            continue
        single.rng.offset = m.offset_of(t)
        ref = single(x)
        torch.cuda.synchronize()
        st = SmartFP.read_stats(N.workspace("smaq", x.device, 0))
        assert torch.equal(ref.view(torch.int32), y.view(torch.int32)), t
        for k in ("mean", "raw_std", "std_clamped"):
            assert stats[m.index_of(t)][k] == st[k], (t, k)


def test_multi_mixed_dtypes_one_call_per_group():
    """A list mixing fp32 / bf16 tensors: one launch pair per dtype, each tensor as its single
    call at its offset in the whole list."""
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    hp = smaq_hparams(use_sample_stats=True)
    base = _make(5)
    xs = [x if i % 2 else x.to(torch.bfloat16) for i, x in enumerate(base)]
    m = SmaqMulti(hp, seed=3)
    ys = m(xs)
    single = SmartFP(hp)
    single.rng.seed = 3
    for t, (x, y) in enumerate(zip(xs, ys)):
        if x.numel() < hp.min_size:
            continue
        single.rng.offset = m.offset_of(t)
        assert torch.equal(single(x).view(torch.int32), y.view(torch.int32)), t


def test_multi_sampled_graph_replays():
    """Graph-safe bound sampled multi call: eager calls and replays equal the host-offset calls
    (fresh index sets per replay, the draw at each tensor's offset)."""
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    hp = smaq_hparams(use_sample_stats=True, num_samples=50)
    gen = torch.Generator(device="cuda").manual_seed(3)
    sizes = [4099, 1 << 16, 3, (1 << 18) + 1, 777]
    xs = [torch.randn(s, generator=gen, device="cuda") for s in sizes]
    ys_h = [torch.empty_like(x) if x.numel() >= hp.min_size else x for x in xs]
    ys_d = [torch.empty_like(x) if x.numel() >= hp.min_size else x for x in xs]
    host = SmaqMulti(hp, seed=11)
    dev = SmaqMulti(hp, seed=11).graph_safe(True, device="cuda")
    bh, bd = host.bind(xs, ys_h), dev.bind(xs, ys_d)
    bh()
    bd()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        bd()
    outs = []
    for _ in range(3):
        graph.replay()
        bh()
        torch.cuda.synchronize()
        for a, b in zip(ys_h, ys_d):
            assert torch.equal(a.view(torch.int32), b.view(torch.int32))
        outs.append(ys_d[1].clone())
    assert not torch.equal(outs[0], outs[1])
    assert dev.rng.position() == host.rng.offset


def test_multi_half_in_place_rejected():
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    x = torch.randn(1000, device="cuda").half()
    with pytest.raises(RuntimeError):
        SmaqMulti(smaq_hparams(precision=16))([x], [x])
