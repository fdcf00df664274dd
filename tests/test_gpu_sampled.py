"""Device-drawn sampled statistics (SMQ_STATS_SAMPLED_DEVICE; smart.py:86-91 with the randperm of
line 88 drawn by Floyd's algorithm on the device from the call's stream position).

Contract, bit-exact: the indices a call records in its workspace equal oracle/rng.py
floyd_indices(seed, position, n, k) for any k (the reference has no cap; above SMQ_MAX_DEVICE_SAMPLES =
4096 the draw runs across workgroups, include/smq.h SMQ_WS_LARGE_SAMPLES_OFFSET); the statistics equal the oracle's over those indices (fp32 within 1 ulp
of the fp64 restatement); the output equals the oracle's apply with the device statistics and the
same counter RNG. Consecutive eager calls draw different sets, and so do consecutive replays of a
captured graph in graph-safe mode (round 1 reused one set there).
"""

import numpy as np
import pytest
import torch

from helpers import same_f32, smaq_hparams, ulp_diff

pytestmark = pytest.mark.gpu


def _idx(ws, k):
    from smart_compress_amd.compress.smart import SmartFP

    return SmartFP.sample_indices(ws, k)


def _check_call(x, y, ws, hp, seed, pos, k):
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import SmartFP

    n = x.numel()
    idx = _idx(ws, k)
    want = orng.floyd_indices(seed, pos, n, k)
    assert idx.tolist() == want.tolist()
    xn = x.detach().cpu().numpy().ravel()
    cfg = osmaq.SmaqConfig(use_sample_stats=True, num_samples=k,
                           use_range_std_dev=hp.use_range_std_dev)
    mo, so = osmaq.sampled_stats(xn, idx, cfg)
    st = SmartFP.read_stats(ws)
    assert ulp_diff(st["mean"], mo) <= 1 and ulp_diff(st["raw_std"], so) <= 1, (st, mo, so)
    assert st["n_used"] == k
    y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], cfg, orng.uniforms(seed, pos, n))
    assert same_f32(y.detach().cpu().numpy().ravel(), y_or)
    return idx


@pytest.mark.parametrize("n,k,rng_std", [(1 << 18, 16, False), (1 << 18, 64, False),
                                         (1 << 18, 65, False), (1 << 20, 1000, False),
                                         (1 << 20, 4096, False), (4096, 4096, False),
                                         (3000, 4096, False), (10, 16, False),
                                         (1 << 18, 16, True), (1 << 20, 2048, True),
                                         (1 << 20, 4097, False), (1 << 20, 10000, False),
                                         (10000, 10000, False), (11000, 10000, False),
                                         (1 << 22, 100000, True), (3 << 20, 10000, False)])
def test_device_draw_eager_calls(n, k, rng_std):
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.smart import SmartFP

    hp = smaq_hparams(use_sample_stats=True, num_samples=k, use_range_std_dev=rng_std)
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 77, 12345
    x = torch.randn(n, device="cuda") * 3 + 1
    keff = min(n, k)
    seen = []
    for _ in range(3):
        pos = codec.rng.offset
        y = codec(x)
        torch.cuda.synchronize()
        ws = N.workspace("smaq", x.device, 0)
        seen.append(tuple(_check_call(x, y, ws, hp, 77, pos, keff)))
    if keff < n:
        assert len(set(seen)) == 3  # a fresh set per call (smart.py:88)
    else:
        assert all(sorted(s) == list(range(n)) for s in seen)


def test_device_draw_half_inputs():
    """fp16 / bf16 inputs: the sample statistics run in the input type like the reference."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.smart import SmartFP

    for dt, name, prec in ((torch.float16, "f16", 16), (torch.bfloat16, "bf16", 32)):
        hp = smaq_hparams(use_sample_stats=True, num_samples=100, precision=prec)
        codec = SmartFP(hp)
        codec.rng.seed, codec.rng.offset = 5, 0
        x = torch.randn(1 << 16, device="cuda").to(dt)
        y = codec(x)
        torch.cuda.synchronize()
        ws = N.workspace("smaq", x.device, 0)
        idx = _idx(ws, 100)
        assert idx.tolist() == orng.floyd_indices(5, 0, x.numel(), 100).tolist()
        xn = x.float().cpu().numpy()
        cfg = osmaq.SmaqConfig(use_sample_stats=True, num_samples=100, precision=prec)
        mo, so = osmaq.sampled_stats(xn, idx, cfg, name)
        st = SmartFP.read_stats(ws)
        assert st["mean"] == mo and st["raw_std"] == so, (st, mo, so)
        assert y.dtype == torch.float32


def test_device_draw_large_k_half_and_heavy_repeats():
    """The multi-workgroup draw with fp16 input and with n barely above k (most steps are
    suspects, resolved 64 at a time in draw order), against the oracle's Floyd draw."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.smart import SmartFP

    for n, k, dt in ((1 << 18, 20000, torch.float16), (20001, 20000, torch.float32),
                     (40000, 20000, torch.float32)):
        hp = smaq_hparams(use_sample_stats=True, num_samples=k, precision=16)
        codec = SmartFP(hp)
        codec.rng.seed, codec.rng.offset = 31, 5
        x = (torch.randn(n, device="cuda") * 2).to(dt)
        y = codec(x)
        torch.cuda.synchronize()
        ws = N.workspace("smaq", x.device, 0)
        idx = _idx(ws, k)
        assert idx.tolist() == orng.floyd_indices(31, 5, n, k).tolist()
        name = "f16" if dt == torch.float16 else "f32"
        cfg = osmaq.SmaqConfig(use_sample_stats=True, num_samples=k, precision=16)
        mo, so = osmaq.sampled_stats(x.float().cpu().numpy(), idx, cfg, name)
        st = SmartFP.read_stats(ws)
        if dt == torch.float16:
            h = lambda v: int(np.array(v, np.float16).view(np.int16))
            assert abs(h(st["mean"]) - h(mo)) <= 1 and abs(h(st["raw_std"]) - h(so)) <= 1
        else:
            assert ulp_diff(st["mean"], mo) <= 1 and ulp_diff(st["raw_std"], so) <= 1
        assert st["n_used"] == k and y.dtype == torch.float32


def test_device_draw_graph_replays_draw_fresh_sets():
    """graph_safe() + --use_sample_stats: the eager warm-up and every replay of the captured call
    read the stream position from the device counter, so each draws its own index set (round 1:
    the same set on every replay)."""
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.smart import SmartFP

    hp = smaq_hparams(use_sample_stats=True, num_samples=32)
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 13, 1000
    n = (1 << 20) + 3
    x = torch.randn(n, device="cuda")
    codec.graph_safe(True, device="cuda")
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            y0 = codec(x)  # eager graph-safe call at position 1000
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        ws_eager = N._ws[("smaq", 0, s.cuda_stream)]
        first = _check_call(x, y0, ws_eager, hp, 13, 1000, 32)
        cap = torch.cuda.Stream()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=cap):
            y_static = codec(x)
        ws = N._ws[("smaq", 0, cap.cuda_stream)]
        sets = [tuple(first)]
        for r in range(3):
            graph.replay()
            torch.cuda.synchronize()
            sets.append(tuple(_check_call(x, y_static, ws, hp, 13, 1000 + (r + 1) * n, 32)))
        assert len(set(sets)) == 4
        assert codec.rng.position() == 1000 + 4 * n
    finally:
        codec.graph_safe(False)
