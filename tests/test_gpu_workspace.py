"""Self-healing workspaces: the cross-workgroup arrival counters are tagged per call
(smq_common.h block_arrive_tagged), so a workspace that was never zeroed, or whose counter a call
left mid-count (an aborted launch), still yields correct statistics on the next call — round 1
needed zero-filled workspaces and a single bad call poisoned every later one silently."""

import numpy as np
import pytest
import torch

from helpers import same_f32, smaq_hparams, ulp_diff

pytestmark = pytest.mark.gpu

# stale tags the host never hands out soon (tags run 1, 2, ... per slot, < 2^31); a word holding
# exactly the tag of the coming call is the one case the scheme cannot tell apart (smq_common.h)
POISON = [0xFFFFFFFFFFFFFFF0, (0x7FFFFFF0 << 32) | 5, 3, 0x7FFFFFFF00000000 | 12345, 1 << 63]


def _counter_words(ws):
    """The 64 tagged arrival counters at the end of the single-tensor workspace (smq.h layout)."""
    from smart_compress_amd import _native as N

    off = N.SMQ_WS_SAMPLES_OFFSET + 8 * N.SMQ_MAX_DEVICE_SAMPLES
    return off, off + 8 * 64


def _poison_counter(ws, value):
    lo, hi = _counter_words(ws)
    v = np.full(64, value, dtype=np.uint64).view(np.uint8)
    ws[lo:hi] = torch.from_numpy(v.copy()).to(ws.device)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("n", [(1 << 22) + 1, 1 << 24, 5000])
def test_stats_after_poisoned_counter(n, split):
    """split: smq_smaq_stats + smq_smaq_apply (the statistics launch always hands off through a
    counter); else smq_smaq_roundtrip, which defers the reduction below 12M elements."""
    import gpu_calls as g
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd import _native as N

    hp = smaq_hparams()
    x = torch.randn(n, device="cuda") * 2 + 0.5
    xn = x.cpu().numpy()
    mo, so = osmaq.full_stats(xn, osmaq.SmaqConfig())
    ws = torch.randint(0, 256, (N.lib().smq_smaq_workspace_bytes(n),), dtype=torch.uint8,
                       device="cuda")  # never zeroed: garbage everywhere
    y = torch.empty_like(x)
    for i, poison in enumerate(POISON + [None, None]):
        if poison is not None:
            _poison_counter(ws, poison)
        p = g.smaq_params(hp, n, seed=4, offset=i * n)
        if split:
            N.check(N.lib().smq_smaq_stats(x.data_ptr(), N.SMQ_DTYPE_F32, n, p, ws.data_ptr(),
                                           ws.numel(), g.stream()), "stats")
            N.check(N.lib().smq_smaq_apply(x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, p,
                                           None, None, ws.data_ptr(), ws.numel(), g.stream()),
                    "apply")
        else:
            N.check(N.lib().smq_smaq_roundtrip(x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, p,
                                               None, ws.data_ptr(), ws.numel(), g.stream()), "rt")
        torch.cuda.synchronize()
        st = g.read_stats(ws)
        assert ulp_diff(st["mean"], mo) <= 1 and ulp_diff(st["raw_std"], so) <= 1, (i, st)
        y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], osmaq.SmaqConfig(),
                              orng.uniforms(4, i * n, n))
        assert same_f32(y.cpu().numpy(), y_or), i
    # a call that counted arrivals leaves the next call's word tagged with a zero count
    lo, hi = _counter_words(ws)
    words = [int(w) for w in ws[lo:hi].cpu().numpy().view(np.uint64)]
    if split and n > 5000:
        assert any(w & 0xFFFFFFFF == 0 and w >> 32 != 0 for w in words)


def test_multi_after_poisoned_workspace():
    """Multi-tensor statistics: every per-tensor counter poisoned with garbage."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    hp = smaq_hparams()
    gen = torch.Generator(device="cuda").manual_seed(9)
    xs = [torch.randn(s, generator=gen, device="cuda") for s in (300000, 70000, 4096, 200001)]
    ys = [torch.empty_like(x) for x in xs]
    m = SmaqMulti(hp, seed=3)
    bound = m.bind(xs, ys)
    ws = m._plans[next(iter(m._plans))]["ws"]
    for rep in range(3):
        ws.copy_(torch.randint(0, 256, ws.shape, dtype=torch.uint8, device="cuda"))
        bound()
        torch.cuda.synchronize()
        stats = m.read_stats()
        for t, (x, y) in enumerate(zip(xs, ys)):
            xn = x.cpu().numpy()
            mo, so = osmaq.full_stats(xn, osmaq.SmaqConfig())
            st = stats[t]
            assert ulp_diff(st["mean"], mo) <= 1 and ulp_diff(st["raw_std"], so) <= 1, (rep, t)
            y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], osmaq.SmaqConfig(),
                                  orng.uniforms(3, m.offset_of(t), xn.size))
            assert same_f32(y.cpu().numpy(), y_or), (rep, t)
