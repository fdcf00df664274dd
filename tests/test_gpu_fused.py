"""The single-launch SmaQ round trip (csrc/smaq_fused.hip) against the two-launch paths and the
oracle. smq_smaq_roundtrip takes it for tensors up to 8,388,611 elements (smart.py:110-190 on an
activation-sized tensor, autograd.py:30-42); the statistics partition of that size class
(csrc/smaq_small.h) is shared by every statistics path, so the single launch, the deferred
two-launch path, the two-launch path whose statistics launch finalises, and separate
smq_smaq_stats + smq_smaq_apply calls give the same header, stream position and outputs BIT FOR
BIT, by construction."""

import numpy as np
import pytest
import torch

from helpers import smaq_hparams

pytestmark = pytest.mark.gpu

# groups per lane V = ceil((n / 4) / 2^18): every V from 1 to 8 (V = 2 / 3 take the u0lds hand-off
# from waves 4..4+V-1; V = 7 splits its rounding draws between LDS and the transform and makes the
# largest LDS request), both sides of the 8,388,611 single-launch limit
SIZES = [5, 4095, 4099, 65536, 1 << 20, (1 << 20) + 3, 1_500_000, 2_500_000, 3 * (1 << 20) + 5,
         1 << 22, (1 << 22) + 16, 6 << 20, 6_500_000, 7 << 20, 8 << 20, 8388611, (8 << 20) + 4]
MODES = ["normal", "trunc", "range", "allpos", "counter", "count", "f16", "bf16"]


def _gpu():
    import gpu_calls

    return gpu_calls


def _input(n, mode, seed):
    gen = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(n, generator=gen, device="cuda") * 1.3 - 0.2
    if mode == "allpos":
        x = x.abs()
    dt = {"f16": torch.float16, "bf16": torch.bfloat16}.get(mode, torch.float32)
    return x.to(dt)


def _run(x, hp, mode, path, ws=None, flags=0):
    """One call on `path`: 'fused' (smq_smaq_roundtrip), 'split' / 'no_defer' (roundtrip_ex
    flags), 'stats_apply' (two entry points). Returns (y, header, counter, outliers)."""
    from smart_compress_amd import _native as N

    g = _gpu()
    n = x.numel()
    p = g.smaq_params(hp, n, all_positive=mode == "allpos", seed=99, offset=12345, dtype=x.dtype)
    if mode == "count":
        p.count_outliers = 1
    ctr = None
    if mode == "counter":
        ctr = torch.tensor([1 << 33], dtype=torch.int64, device="cuda")
        p.offset_counter = ctr.data_ptr()
    y = torch.empty(n, dtype=torch.float32, device="cuda")
    if ws is None:
        ws = torch.zeros(N.lib().smq_smaq_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    args = (x.data_ptr(), N.DTYPE_CODES[x.dtype])
    if path == "stats_apply":
        N.check(N.lib().smq_smaq_stats(*args, n, p, ws.data_ptr(), ws.numel(), g.stream()), "stats")
        N.check(N.lib().smq_smaq_apply(*args, y.data_ptr(), n, p, None, None, ws.data_ptr(),
                                       ws.numel(), g.stream()), "apply")
    else:
        fl = flags | {"fused": 0, "split": N.SMQ_SMAQ_SPLIT, "no_defer": N.SMQ_SMAQ_NO_DEFER}[path]
        N.check(N.lib().smq_smaq_roundtrip_ex(*args, y.data_ptr(), n, p, None, ws.data_ptr(),
                                              ws.numel(), fl, g.stream()), "roundtrip_ex")
    torch.cuda.synchronize()
    hdr = g.read_stats(ws)
    return y, hdr, (None if ctr is None else int(ctr.item())), hdr["n_outlier"]


def _hp(mode):
    hp = smaq_hparams(stochastic_rounding=mode != "trunc", use_range_std_dev=mode == "range")
    if mode == "f16":
        hp.precision = 16
    return hp


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("n", SIZES)
def test_single_launch_equals_two_launch_paths(n, mode):
    x = _input(n, mode, n % 997 + len(mode))
    hp = _hp(mode)
    res = {path: _run(x, hp, mode, path) for path in ("fused", "split", "no_defer", "stats_apply")}
    y0, h0, c0, o0 = res["fused"]
    for path, (y, h, c, o) in res.items():
        assert torch.equal(y.view(torch.int32), y0.view(torch.int32)), path
        for k in ("mean", "std_dev", "std_clamped", "raw_std", "n_used"):
            assert h[k] == h0[k] or (np.isnan(h[k]) and np.isnan(h0[k])), (path, k)
        if mode == "range":
            assert h["min"] == h0["min"] and h["max"] == h0["max"], path
        if mode == "counter":
            assert c == c0 == (1 << 33) + n, path
        if mode == "count":
            assert o == o0, path


@pytest.mark.parametrize("n", [(1 << 20) + 3, 2_500_000, (1 << 22) + 16, 6_500_000, 8388611])
@pytest.mark.parametrize("mode", ["normal", "range", "f16"])
def test_single_launch_vs_oracle(n, mode):
    """Device statistics within 1 ulp (fp32) / one half step of the fp64 oracle; outputs equal the
    oracle fed the device statistics and the counter RNG, bit for bit."""
    from oracle import rng as orng
    from oracle import smaq as osmaq

    x = _input(n, mode, 7 + n % 13)
    hp = _hp(mode)
    y, h, _, _ = _run(x, hp, mode, "fused")
    xn = x.float().cpu().numpy()
    dt = {"f16": "f16", "bf16": "bf16"}.get(mode, "f32")
    cfg = osmaq.SmaqConfig(use_range_std_dev=mode == "range", precision=hp.precision)
    mean, std = osmaq.full_stats(xn, cfg, dt)

    def bits(v):
        if dt == "f16":
            return int(np.float16(v).view(np.int16))
        b = int(np.float32(v).view(np.int32))
        return b >> 16 if dt == "bf16" else b

    for a, b in ((h["mean"], mean), (h["raw_std"], std)):
        assert abs(bits(a) - bits(b)) <= 1, (a, b)
    y_or, _ = osmaq.apply(xn, h["mean"], h["raw_std"], cfg, orng.uniforms(99, 12345, n), dtype=dt)
    yh = y.cpu().numpy()
    assert int((yh.view(np.uint32) != y_or.view(np.uint32)).sum()) == 0


@pytest.mark.parametrize("n", [1 << 20, 1_500_000, 2_500_000, (1 << 22) + 16, 6_500_000, 7 << 20,
                               8388611])
def test_single_launch_without_co_residency(n):
    """SMQ_SMAQ_TEST_LATE: half of the workgroups start ~500 us late and the others compute the
    partials they miss after 20 us. Same bytes as the undisturbed call."""
    from smart_compress_amd import _native as N

    x = _input(n, "normal", 3)
    hp = _hp("normal")
    y0, h0, _, _ = _run(x, hp, "normal", "fused")
    for _ in range(3):
        y1, h1, _, _ = _run(x, hp, "normal", "fused", flags=N.SMQ_SMAQ_TEST_LATE)
        assert torch.equal(y0.view(torch.int32), y1.view(torch.int32))
        assert h0["mean"] == h1["mean"] and h0["raw_std"] == h1["raw_std"]


def test_single_launch_poisoned_and_shared_workspace():
    """A workspace of random bytes (generation, arrival word, granules), then a sequence of calls of
    different sizes (grids of 1 .. 256 workgroups) on ONE workspace: every call equals the same
    call on a fresh zeroed workspace."""
    from smart_compress_amd import _native as N

    hp = _hp("normal")
    nb = N.lib().smq_smaq_workspace_bytes(1 << 20)
    gen = torch.Generator(device="cuda").manual_seed(5)
    ws = torch.randint(0, 256, (nb,), dtype=torch.uint8, device="cuda", generator=gen)
    for i, n in enumerate([8388611, 1 << 20, 4099, (1 << 22) + 16, 65536, 8 << 20, 1 << 20]):
        x = _input(n, "normal", 100 + i)
        y_ref, h_ref, _, _ = _run(x, hp, "normal", "fused")
        y, h, _, _ = _run(x, hp, "normal", "fused", ws=ws)
        assert torch.equal(y.view(torch.int32), y_ref.view(torch.int32)), n
        assert h["mean"] == h_ref["mean"] and h["raw_std"] == h_ref["raw_std"], n
        if i == 3:  # poison the exchange region again mid-sequence
            off = N.SMQ_WS_FUSED_OFFSET
            ws[off: off + 4096] = torch.randint(0, 256, (4096,), dtype=torch.uint8, device="cuda",
                                                generator=gen)


def test_single_launch_graph_replays_match_eager():
    """Three SmartFP calls (graph-safe random stream) captured into one hipGraph: two replays give
    the outputs of six consecutive eager calls, bit for bit, and fresh streams per replay."""
    from smart_compress_amd.compress.smart import SmartFP

    hp = _hp("normal")
    sizes = [(1 << 20) + 3, 3 * (1 << 20) + 5, 8 << 20]
    xs = [_input(n, "normal", 40 + i) for i, n in enumerate(sizes)]
    eager = SmartFP(hp)
    eager.rng.seed, eager.rng.offset = 77, 1000
    want = [[eager(x).clone() for x in xs] for _ in range(2)]
    torch.cuda.synchronize()
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 77, 1000
    codec.graph_safe(True, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm the workspace of the capture stream (not the stream position)
        codec.rng.counter("cuda")
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = [codec(x) for x in xs]
    for r in range(2):
        g.replay()
        torch.cuda.synchronize()
        for o, w in zip(outs, want[r]):
            assert torch.equal(o.view(torch.int32), w.view(torch.int32)), r
    codec.graph_safe(False)
