"""The codecs on CPU tensors (libsmq's host path, smq_cpu_*): parity with the reference's golden
vectors and the oracle, on this machine (no GPU needed; these are product code, not the oracle).

Tolerances, as for the device path (tests/test_gpu_smaq.py, test_gpu_float.py):
  * SmaQ with the reference's statistics and uniforms injected: BIT-EXACT vs the reference;
  * library statistics vs the fp64 oracle: within 1 fp32 ulp (half types: one half step);
  * library statistics + counter RNG vs the oracle fed the same statistics and RNG: BIT-EXACT;
  * float_quantize with the reference's recorded words, or the counter RNG vs the oracle:
    BIT-EXACT;
  * S2FP8: E5M2 codes of Y against the reference's / oracle's (>= 99.99 % identical, never more
    than one code apart), outputs within 2 fp32 ulp where the codes agree.
The results do not depend on the thread count (fixed task split, fixed summation order).
"""

import ctypes
from argparse import ArgumentParser

import numpy as np
import pytest
import torch

from helpers import (float_meta, load_float, load_smaq, n_diff_f32, oracle_cfg, same_f32,
                     smaq_cases, smaq_hparams, ulp_diff)

CASES = smaq_cases()
ACTIVE = [k for k in sorted(CASES) if not k.startswith("n7")]
META = float_meta()
FMT = dict(fp8=(5, 2), fp16=(5, 10), bf16=(8, 7))
TORCH_DT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}


def _N():
    from smart_compress_amd import _native as N

    return N


def _params(hp, numel, all_positive=False, seed=0, offset=0, dtype=torch.float32):
    from smart_compress_amd.compress.smart import SmartFP

    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = seed, offset
    return codec._params(numel, all_positive, dtype)


def _stats_in(mean, std, hp, dtype="f32"):
    """SmqSmaqStats for injected (mean, std), as tests/gpu_calls.stats_struct builds it."""
    from oracle.smaq import round_to

    N = _N()
    s = N.SmqSmaqStats()
    lo = np.float32(round_to(np.float32(1e-4 if hp.precision == 16 else 1e-38), dtype))
    hi = np.float32(round_to(np.float32(1e4 if hp.precision == 16 else 1e38), dtype))
    sd = np.float32(std)
    std_dev = np.float32(1.0) if sd == 0 else sd
    sc = min(max(std_dev, lo), hi)
    s.mean, s.std_dev, s.std_clamped, s.raw_std = float(mean), float(std_dev), float(sc), float(sd)
    return s


def _roundtrip(x, p, uniforms=None, stats_in=None, threads=0):
    """smq_cpu_smaq_roundtrip on a CPU tensor; returns (y, ws, stats dict)."""
    from smart_compress_amd.compress.smart import SmartFP

    N = _N()
    n = x.numel()
    y = torch.empty(x.shape, dtype=torch.float32)
    ws = torch.zeros(N.lib().smq_smaq_workspace_bytes_sampled(n, max(p.num_samples, 1)),
                     dtype=torch.uint8)
    if stats_in is not None:
        p.stats_source = N.SMQ_STATS_INJECTED
    u = None
    if uniforms is not None:
        u = torch.from_numpy(np.ascontiguousarray(uniforms, np.float32).ravel())
    N.check(N.lib().smq_cpu_smaq_roundtrip(
        x.data_ptr(), N.DTYPE_CODES[x.dtype], y.data_ptr(), n, p,
        u.data_ptr() if u is not None else None,
        ctypes.byref(stats_in) if stats_in is not None else None,
        ws.data_ptr(), ws.numel(), threads), "cpu roundtrip")
    return y, ws, SmartFP.read_stats(ws)


def _golden_x(d, meta):
    return torch.from_numpy(d["x"].astype(np.float32)).to(TORCH_DT[meta.get("dtype", "f32")])


def _bind_bn(p, d, meta, keep):
    if "bn_gamma" not in d:
        return
    if meta["bn_scalar_params"]:
        g, b = d["bn_gamma_used"], d["bn_beta_used"]
    else:
        g, b = d["bn_gamma"], d["bn_beta"]
    g = torch.from_numpy(np.ascontiguousarray(g, np.float32).ravel())
    b = torch.from_numpy(np.ascontiguousarray(b, np.float32).ravel())
    keep += [g, b]
    p.bn_gamma, p.bn_beta = g.data_ptr(), b.data_ptr()
    p.bn_channels = g.numel()
    p.bn_inner = d["x"].shape[2] * d["x"].shape[3]


@pytest.mark.parametrize("name", ACTIVE)
def test_cpu_golden_injected_bitexact(name):
    """Reference statistics + reference uniforms -> the reference's output, bit for bit."""
    meta, d = CASES[name], load_smaq(name)
    hp = smaq_hparams(meta)
    x = _golden_x(d, meta).reshape(-1)
    p = _params(hp, x.numel(), all_positive=meta["all_positive"], dtype=x.dtype)
    p.count_outliers = 1
    keep = []
    _bind_bn(p, d, meta, keep)
    y, ws, st = _roundtrip(x, p, uniforms=d.get("uniforms"),
                           stats_in=_stats_in(d["mean"], d["std"], hp, meta["dtype"]))
    yh = y.numpy().reshape(d["y"].shape)
    assert same_f32(yh, d["y"]), f"{n_diff_f32(yh, d['y'])} elements differ"
    if "n_outlier" in d and int(d["n_outlier"]) >= 0:
        from smart_compress_amd.compress.smart import SmartFP

        assert SmartFP.outlier_count(ws) == int(d["n_outlier"])


def _assert_stats_close(ours, ref, dtype):
    if dtype == "f32":
        assert ulp_diff(ours, ref) <= 1, (ours, ref)
    else:
        step = float(np.spacing(np.float16(ref))) if dtype == "f16" else abs(float(ref)) * 2.0**-7
        assert abs(float(ours) - float(ref)) <= step + 1e-30, (ours, ref)


@pytest.mark.parametrize("name", [k for k in ACTIVE if CASES[k]["use_sample_stats"]])
def test_cpu_golden_sampled_indices(name):
    """Sampled statistics on the reference's own randperm draws (smart.py:86-91)."""
    N = _N()
    meta, d = CASES[name], load_smaq(name)
    hp = smaq_hparams(meta)
    x = _golden_x(d, meta).reshape(-1)
    p = _params(hp, x.numel(), dtype=x.dtype)
    p.stats_source = N.SMQ_STATS_SAMPLED
    for j, v in enumerate(d["sample_idx"]):
        p.sample_idx[j] = int(v)
    p.num_samples = len(d["sample_idx"])
    y, _, st = _roundtrip(x, p, uniforms=d.get("uniforms"))
    _assert_stats_close(st["mean"], d["mean"], meta["dtype"])
    _assert_stats_close(st["raw_std"], d["std"], meta["dtype"])
    if st["mean"] == d["mean"] and st["raw_std"] == d["std"]:
        assert same_f32(y.numpy(), d["y"].ravel())


@pytest.mark.parametrize("name", [k for k in ACTIVE if not CASES[k]["use_sample_stats"]])
def test_cpu_golden_full_pipeline(name):
    """Library statistics vs the oracle's fp64 statistics; with them the oracle's output."""
    from oracle import smaq as osmaq

    meta, d = CASES[name], load_smaq(name)
    hp = smaq_hparams(meta)
    x = _golden_x(d, meta).reshape(-1)
    p = _params(hp, x.numel(), all_positive=meta["all_positive"], dtype=x.dtype)
    keep = []
    _bind_bn(p, d, meta, keep)
    y, _, st = _roundtrip(x, p, uniforms=d.get("uniforms"))
    mo, so = osmaq.full_stats(d["x"], oracle_cfg(meta), meta["dtype"])
    _assert_stats_close(st["mean"], mo, meta["dtype"])
    _assert_stats_close(st["raw_std"], so, meta["dtype"])
    if st["mean"] == d["mean"] and st["raw_std"] == d["std"]:
        assert same_f32(y.numpy(), d["y"].ravel())


@pytest.mark.parametrize("n,shift", [(1 << 20, 0), (1000003, 1), (4099, 3), (8, 0)])
@pytest.mark.parametrize("sr", [True, False])
def test_cpu_smartfp_vs_oracle(n, shift, sr):
    """The drop-in SmartFP on a CPU tensor (incl. an unaligned view): statistics within 1 ulp of
    the oracle, output == oracle(x, those statistics, the counter RNG) bit for bit."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import SmartFP

    N = _N()
    g = torch.Generator().manual_seed(n + shift)
    x = (torch.randn(n + shift, generator=g) * 2.5 + 0.3)[shift:]
    hp = smaq_hparams(stochastic_rounding=sr)
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 1234, 777
    y = codec(x)
    assert y.shape == x.shape and y.dtype == torch.float32 and y.device.type == "cpu"
    ws = N.cpu_workspace("smaq", 0)
    st = SmartFP.read_stats(ws)
    xn = x.numpy()
    mo, so = osmaq.full_stats(xn, osmaq.SmaqConfig())
    assert ulp_diff(st["mean"], mo) <= 1 and ulp_diff(st["raw_std"], so) <= 1
    cfg = osmaq.SmaqConfig(stochastic_rounding=sr)
    u = orng.uniforms(1234, 777, n) if sr else None
    y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], cfg, u)
    assert same_f32(y.numpy(), y_or), n_diff_f32(y.numpy(), y_or)
    assert codec.rng.offset == 777 + n


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_cpu_thread_count_invariant(threads):
    """Fixed 64K-element tasks and a fixed summation order: the same bytes on any thread count."""
    n = 3 * (1 << 16) + 12345
    x = torch.randn(n, generator=torch.Generator().manual_seed(5)) * 3 - 1
    hp = smaq_hparams()
    ref, _, st_ref = _roundtrip(x, _params(hp, n, seed=9, offset=4), threads=1)
    y, _, st = _roundtrip(x, _params(hp, n, seed=9, offset=4), threads=threads)
    assert st["mean"] == st_ref["mean"] and st["raw_std"] == st_ref["raw_std"]
    assert torch.equal(y.view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("k,n", [(16, 200003), (1000, 200003), (4096, 200003), (4097, 200003),
                                 (10000, 200003), (10000, 10000), (10000, 11000)])
def test_cpu_sampled_draw_matches_device_draw(k, n):
    """SMQ_STATS_SAMPLED_DEVICE on the host: the same Floyd draw as the device (oracle/rng.py),
    recorded in the workspace (above SMQ_MAX_DEVICE_SAMPLES in the large-draw region), and the
    oracle's sampled statistics / output from those indices. k = n is a permutation; n close to k
    substitutes most steps."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import SmartFP

    N = _N()
    x = torch.randn(n, generator=torch.Generator().manual_seed(k)) + 0.5
    hp = smaq_hparams(use_sample_stats=True, num_samples=k)
    p = _params(hp, n, seed=77, offset=1000)
    assert p.stats_source == N.SMQ_STATS_SAMPLED_DEVICE
    y, ws, st = _roundtrip(x, p)
    idx = SmartFP.sample_indices(ws, min(n, k))
    assert np.array_equal(idx, orng.floyd_indices(77, 1000, n, k))
    if k >= n:
        assert sorted(idx.tolist()) == list(range(n))
    cfg = osmaq.SmaqConfig(use_sample_stats=True, num_samples=k)
    mo, so = osmaq.sampled_stats(x.numpy(), idx, cfg)
    assert ulp_diff(st["mean"], mo) <= 1 and ulp_diff(st["raw_std"], so) <= 1
    y_or, _ = osmaq.apply(x.numpy(), st["mean"], st["raw_std"], osmaq.SmaqConfig(),
                          orng.uniforms(77, 1000, n))
    assert same_f32(y.numpy(), y_or)


@pytest.mark.parametrize("dt", ["f16", "bf16"])
def test_cpu_half_inputs_vs_oracle(dt):
    """fp16 / bf16 inputs through SmartFP on CPU: the reference's dtype flow (statistics and z in
    the input type), against the oracle fed the library's statistics."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import SmartFP

    N = _N()
    n = 300007
    x = (torch.randn(n, generator=torch.Generator().manual_seed(2)) * 1.5).to(TORCH_DT[dt])
    hp = smaq_hparams(precision=16 if dt == "f16" else 32)
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 42, 0
    y = codec(x)
    st = SmartFP.read_stats(N.cpu_workspace("smaq", 0))
    xn = x.float().numpy()
    cfg = osmaq.SmaqConfig(precision=hp.precision)
    mo, so = osmaq.full_stats(xn, cfg, dt)
    _assert_stats_close(st["mean"], mo, dt)
    _assert_stats_close(st["raw_std"], so, dt)
    y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], cfg, orng.uniforms(42, 0, n),
                          dtype=dt)
    assert same_f32(y.numpy(), y_or), n_diff_f32(y.numpy(), y_or)


def _float_quant(x, e, m, check_inf=True, rand_bits=None, seed=0, offset=0, out=torch.float32):
    N = _N()
    y = torch.empty(x.shape, dtype=out)
    r = None if rand_bits is None else torch.from_numpy(np.ascontiguousarray(rand_bits).view(np.int32))
    N.check(N.lib().smq_cpu_float_quant(
        x.data_ptr(), N.DTYPE_CODES[x.dtype], y.data_ptr(), N.DTYPE_CODES[out], x.numel(), e, m,
        N.SMQ_ROUND_STOCHASTIC, 1 if check_inf else 0,
        r.data_ptr() if r is not None else None, seed, offset, 0), "cpu float_quant")
    return y


@pytest.mark.parametrize("key", sorted(k for k, m in META["cases"].items() if m["codec"] != "s2fp8"))
def test_cpu_golden_float_bitexact(key):
    """float_quantize with the reference's recorded random words -> its output, bit for bit."""
    m, d = META["cases"][key], load_float(key)
    y = _float_quant(torch.from_numpy(d["x"]), *FMT[m["codec"]], check_inf=m["check_inf"],
                     rand_bits=d["q_rand"])
    assert same_f32(y.numpy(), d["y"]), n_diff_f32(y.numpy(), d["y"])


@pytest.mark.parametrize("fmt", [(5, 2), (4, 3), (5, 10), (8, 7)])
def test_cpu_float_counter_rng_vs_oracle(fmt):
    from oracle import qtorch_float as qf
    from oracle import rng as orng

    n = 300001
    g = torch.Generator().manual_seed(3)
    x = torch.randn(n, generator=g) * torch.exp(torch.randn(n, generator=g) * 4)
    x[:8] = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), float("nan"), 57344.0, -57344.0,
                          1e-42])
    y = _float_quant(x, *fmt, seed=11, offset=2**32 - 5)
    y_or = qf.float_quantize(x.numpy(), *fmt, orng.rng_u32(11, 2**32 - 5, n), True)
    assert same_f32(y.numpy(), y_or), n_diff_f32(y.numpy(), y_or)


def _s2fp8(x, rand_bits=None, seed=0, offset=0, mu_m=None, flags=0, check_inf=True, precision=32):
    N = _N()
    half_out = precision == 16 and x.dtype == torch.float16
    y = torch.empty(x.shape, dtype=torch.float16 if half_out else torch.float32)
    ws = torch.zeros(64, dtype=torch.uint8)
    st_in = None
    if mu_m is not None:
        st_in = N.SmqS2fp8Stats()
        st_in.mu, st_in.m = float(mu_m[0]), float(mu_m[1])
    r = None if rand_bits is None else torch.from_numpy(np.ascontiguousarray(rand_bits).view(np.int32))
    N.check(N.lib().smq_cpu_s2fp8_roundtrip(
        x.data_ptr(), N.DTYPE_CODES[x.dtype], y.data_ptr(), x.numel(), precision,
        1 if check_inf else 0, r.data_ptr() if r is not None else None, seed, offset,
        ctypes.byref(st_in) if st_in is not None else None, ws.data_ptr(), ws.numel(), flags, 0),
        "cpu s2fp8")
    f = ws[:32].numpy().view(np.float32)
    return y, dict(mu=f[0], m=f[1], alpha=f[2], beta=f[3], beta_pow2=f[4])


def _codes_of(t):
    from test_gpu_float import _codes

    return _codes(t)


@pytest.mark.parametrize("key", sorted(k for k, m in META["cases"].items() if m["codec"] == "s2fp8"))
def test_cpu_golden_s2fp8(key):
    """With the reference's (mu, max) and words: alpha, beta, 2^beta bit-exact; Y within 4 fp32
    ulp of the reference's recorded quantiser input; T in the E5M2 code domain; outputs within 2 ulp
    where the codes agree. Then end to end with the library's own statistics."""
    from oracle import qtorch_float as qf
    from oracle import s2fp8 as os2
    from test_gpu_float import _assert_codes, _assert_code_domain, _ulps

    N = _N()
    m, d = META["cases"][key], load_float(key)
    x = torch.from_numpy(d["x"])
    kw = dict(check_inf=m["check_inf"], rand_bits=d["q_rand"], mu_m=(d["mu"], d["m"]))
    y, st = _s2fp8(x, **kw)
    for k in ("alpha", "beta", "beta_pow2"):
        assert st[k] == d[k], (k, st[k], d[k])
    Y, _ = _s2fp8(x, flags=N.SMQ_S2FP8_OUT_Y, **kw)
    T, _ = _s2fp8(x, flags=N.SMQ_S2FP8_OUT_T, **kw)
    ok = ~np.isnan(d["q_in"])
    assert _ulps(Y.numpy()[ok], d["q_in"][ok]).max() <= 4
    T_ref = qf.float_quantize(d["q_in"], 5, 2, d["q_rand"], m["check_inf"])
    _assert_codes(T.numpy(), T_ref)
    same = _codes_of(T.numpy()) == _codes_of(T_ref)
    yh = y.numpy()
    okk = same & ~np.isnan(d["y"])
    assert _ulps(yh[okk], d["y"][okk]).max() <= 2
    assert np.array_equal(np.isnan(yh), np.isnan(d["y"]))
    y2, st2 = _s2fp8(x, check_inf=m["check_inf"], rand_bits=d["q_rand"])
    assert abs(float(st2["mu"]) - float(d["mu"])) <= 2.0**-20 * max(1.0, abs(float(d["mu"])))
    assert ulp_diff(st2["m"], d["m"]) <= 1
    ref = os2.roundtrip(d["x"], d["q_rand"], m["check_inf"], st=os2.derive(st2["mu"], st2["m"]))
    _assert_code_domain(y2.numpy(), ref[0])


def test_cpu_s2fp8_counter_rng_vs_oracle():
    """C4's shape on CPU with the counter RNG: T codes against the oracle's qtorch(Y) with the same
    words, outputs within 2 ulp where the codes agree."""
    from oracle import qtorch_float as qf
    from oracle import rng as orng
    from oracle import s2fp8 as os2
    from test_gpu_float import _assert_codes, _ulps

    N = _N()
    x = torch.randn(32, 128, 768, generator=torch.Generator().manual_seed(4))
    T, st = _s2fp8(x, seed=8, offset=3, flags=N.SMQ_S2FP8_OUT_T)
    y, _ = _s2fp8(x, seed=8, offset=3)
    xn = x.numpy().ravel()
    so = os2.derive(st["mu"], st["m"])
    words = orng.rng_u32(8, 3, xn.size)
    T_or = qf.float_quantize(os2.transform(xn, so), 5, 2, words, True)
    _assert_codes(T.numpy().ravel(), T_or)
    y_or = os2.roundtrip(xn, words, True, st=so)[0]
    same = _codes_of(T.numpy().ravel()) == _codes_of(T_or)
    assert _ulps(y.numpy().ravel()[same], y_or[same]).max() <= 2


def test_cpu_codecs_dropin():
    """FP8 / FP16 / BF16 / S2FP8 / SmartFP on CPU tensors through the reference's plugin API:
    shapes and dtypes as the reference returns them, RNG offsets advanced, values close."""
    import smart_compress_amd.compress as C
    from smart_compress_amd.util.pytorch import quantization as Q

    x = torch.randn(64, 300, generator=torch.Generator().manual_seed(1))
    for name in ("FP8", "FP16", "BF16", "S2FP8", "SmartFP"):
        cls = getattr(C, name)
        hp = cls.add_argparse_args(ArgumentParser()).parse_args([])
        hp.precision = 32
        c = cls(hp)
        start = Q.quant_rng().offset
        y = c(x, tag="t")
        assert y.shape == x.shape and y.dtype == torch.float32 and y.device.type == "cpu"
        assert (y - x).abs().max().item() < 0.3 * x.abs().max().item(), name
        if name != "SmartFP":
            assert Q.quant_rng().offset == start + x.numel()
    # precision 16: half in -> half out (quantization.py:201-202)
    hp = C.FP8.add_argparse_args(ArgumentParser()).parse_args([])
    hp.precision = 16
    y = C.FP8(hp)(x.half())
    assert y.dtype == torch.float16
    hp = C.S2FP8.add_argparse_args(ArgumentParser()).parse_args([])
    hp.precision = 16
    y = C.S2FP8(hp)(x.half())
    assert y.dtype == torch.float16 and torch.isfinite(y).all()


def test_cpu_smartfp_batch_norm_and_outlier_count():
    """BN variant (per-channel fold) and --measure_compression_ratio on CPU tensors."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import SmartFP

    x = torch.randn(4, 8, 5, 5, generator=torch.Generator().manual_seed(3)) * 2
    gamma = torch.rand(8, generator=torch.Generator().manual_seed(4)) + 0.5
    beta = torch.randn(8, generator=torch.Generator().manual_seed(5))
    hp = smaq_hparams(use_batch_norm=True, measure_compression_ratio=True)
    codec = SmartFP(hp)
    logged = {}
    codec.log = lambda k, v, **_: logged.__setitem__(k, v)
    codec.rng.seed, codec.rng.offset = 3, 0
    y = codec(x, tag="bn", batch_norm_stats=(gamma, beta))
    st = SmartFP.read_stats(_N().cpu_workspace("smaq", 0))
    y_or, o = osmaq.apply(x.numpy(), st["mean"], st["raw_std"], osmaq.SmaqConfig(),
                          orng.uniforms(3, 0, x.numel()), bn=(gamma.numpy(), beta.numpy()))
    assert same_f32(y.numpy(), y_or), n_diff_f32(y.numpy(), y_or)
    n_out = int(np.asarray(o).sum())
    assert logged["new_size"] == n_out * 8 + (x.numel() - n_out) * 6


@pytest.mark.parametrize("special", ["nan", "inf", "-inf"])
def test_cpu_nonfinite_input_propagates_like_reference(special):
    """One NaN / +-inf element on the host path: statistics NaN / inf as the fp64 oracle's, every
    output NaN, bit-exact vs the oracle (as tests/test_gpu_smaq.py does on the device)."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import SmartFP

    N = _N()
    n = 200003
    x = torch.randn(n, generator=torch.Generator().manual_seed(5))
    x[n // 3] = float(special)
    codec = SmartFP(smaq_hparams())
    codec.rng.seed, codec.rng.offset = 8, 0
    y = codec(x)
    st = SmartFP.read_stats(N.cpu_workspace("smaq", 0))
    xn = x.numpy()
    with np.errstate(invalid="ignore"):  # inf - inf in the oracle's centred sums
        mo, so = osmaq.full_stats(xn, osmaq.SmaqConfig())
    assert same_f32(np.float32(st["mean"]), mo) and same_f32(np.float32(st["raw_std"]), so)
    y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], osmaq.SmaqConfig(), orng.uniforms(8, 0, n))
    assert same_f32(y.numpy(), y_or) and np.isnan(y.numpy()).all()


def test_cpu_rejected_call_consumes_no_stream_positions():
    """A call that fails validation (num_samples out of range or beyond what the workspace holds,
    missing injected statistics) leaves the graph-safe stream position where it was; a valid call
    advances it by n."""
    N = _N()
    n = 3 * N.SMQ_MAX_DEVICE_SAMPLES
    x = torch.randn(n)
    y = torch.empty(n)
    ws = torch.zeros(N.lib().smq_smaq_workspace_bytes(n), dtype=torch.uint8)
    ctr = torch.tensor([777], dtype=torch.int64)
    for src, k in ((N.SMQ_STATS_SAMPLED_DEVICE, N.SMQ_MAX_DEVICE_SAMPLES + 1),
                   (N.SMQ_STATS_SAMPLED_DEVICE, 0),
                   (N.SMQ_STATS_SAMPLED, N.SMQ_MAX_SAMPLES + 1), (N.SMQ_STATS_INJECTED, 16)):
        p = _params(smaq_hparams(), n)
        p.offset_counter = ctr.data_ptr()
        p.stats_source, p.num_samples = src, k
        rc = N.lib().smq_cpu_smaq_roundtrip(x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, p,
                                            None, None, ws.data_ptr(), ws.numel(), 1)
        assert rc != 0 and int(ctr.item()) == 777
    p = _params(smaq_hparams(), n)
    p.offset_counter = ctr.data_ptr()
    assert N.lib().smq_cpu_smaq_roundtrip(x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, p,
                                          None, None, ws.data_ptr(), ws.numel(), 1) == 0
    assert int(ctr.item()) == 777 + n


def test_sampled_workspace_sizes():
    """smq_smaq_workspace_bytes_sampled: the plain size up to SMQ_MAX_DEVICE_SAMPLES, the
    large-draw region above it (growing with k), 0 beyond SMQ_MAX_DRAW_SAMPLES."""
    N = _N()
    lib = N.lib()
    n = 1 << 30
    base = lib.smq_smaq_workspace_bytes(n)
    assert lib.smq_smaq_workspace_bytes_sampled(n, 16) == base
    assert lib.smq_smaq_workspace_bytes_sampled(n, N.SMQ_MAX_DEVICE_SAMPLES) == base
    assert N.SMQ_WS_LARGE_SAMPLES_OFFSET >= base
    a = lib.smq_smaq_workspace_bytes_sampled(n, N.SMQ_MAX_DEVICE_SAMPLES + 1)
    b = lib.smq_smaq_workspace_bytes_sampled(n, 10000)
    assert N.SMQ_WS_LARGE_SAMPLES_OFFSET + 8 * 4097 < a <= b
    assert lib.smq_smaq_workspace_bytes_sampled(5000, 10000) == lib.smq_smaq_workspace_bytes_sampled(5000, 5000)
    assert lib.smq_smaq_workspace_bytes_sampled(n, N.SMQ_MAX_DRAW_SAMPLES + 1) == 0
