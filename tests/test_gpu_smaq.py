"""SmaQ parity on the GPU, through the C-ABI and through the drop-in SmartFP class.

Tolerances (north_star: "within 1 ulp of the target low-precision format"):
  * injected statistics + injected uniforms (the reference's own draws): BIT-EXACT vs the
    reference's outputs (golden vectors from smart.py);
  * device statistics vs the fp64 oracle: mean and std within 1 fp32 ulp;
  * device statistics + counter RNG vs the oracle fed the same statistics and RNG: BIT-EXACT;
  * full pipeline vs the reference (its own float mean, our fp64 mean): every element within
    1.001 quantisation steps (step = std / range of the element's class).
"""

import ctypes

import numpy as np
import pytest
import torch

from helpers import (load_smaq, n_diff_f32, oracle_cfg, same_f32, smaq_cases, smaq_hparams,
                     ulp_diff)

pytestmark = pytest.mark.gpu

CASES = smaq_cases()
ACTIVE = [k for k in sorted(CASES) if not k.startswith("n7")]


def _gpu():
    import gpu_calls

    return gpu_calls


def _bn_args(d, meta):
    if "bn_gamma" not in d:
        return None
    if meta["bn_scalar_params"]:
        return d["bn_gamma_used"], d["bn_beta_used"]
    return d["bn_gamma"], d["bn_beta"]


def _bind_bn(p, d, meta, x_shape, keep):
    bn = _bn_args(d, meta)
    if bn is None:
        return
    g = _gpu().to_dev(bn[0].astype(np.float32).ravel())
    b = _gpu().to_dev(bn[1].astype(np.float32).ravel())
    keep += [g, b]
    p.bn_gamma, p.bn_beta = g.data_ptr(), b.data_ptr()
    p.bn_channels = g.numel()
    p.bn_inner = x_shape[2] * x_shape[3]


@pytest.mark.parametrize("name", ACTIVE)
def test_golden_injected_bitexact(name):
    """Reference statistics + reference uniforms -> the reference's output, bit for bit."""
    g = _gpu()
    meta, d = CASES[name], load_smaq(name)
    hp = smaq_hparams(meta)
    x = g.golden_x(d, meta)
    p = g.smaq_params(hp, x.numel(), all_positive=meta["all_positive"], dtype=x.dtype)
    p.count_outliers = 1
    keep = []
    _bind_bn(p, d, meta, d["x"].shape, keep)
    stats = g.stats_struct(d["mean"], d["std"], hp, meta["dtype"])
    u = g.to_dev(d["uniforms"].ravel()) if "uniforms" in d else None
    y, ws = g.smaq_apply(x.reshape(-1), p, uniforms=u, stats_in=stats)
    yh = y.cpu().numpy().reshape(d["y"].shape)
    assert same_f32(yh, d["y"]), f"{n_diff_f32(yh, d['y'])} elements differ"
    if "n_outlier" in d and int(d["n_outlier"]) >= 0:
        assert g.read_stats(ws)["n_outlier"] == int(d["n_outlier"])


@pytest.mark.parametrize("name", [k for k in ACTIVE if CASES[k]["use_sample_stats"]])
def test_golden_sampled_indices(name):
    """In-kernel sampled statistics on the reference's randperm draws (smart.py:86-91)."""
    g = _gpu()
    meta, d = CASES[name], load_smaq(name)
    hp = smaq_hparams(meta)
    x = g.golden_x(d, meta)
    p = g.smaq_params(hp, x.numel(), dtype=x.dtype)
    p.stats_source = g.N.SMQ_STATS_SAMPLED  # host-given indices: the reference's own draw
    idx = d["sample_idx"]
    for j, v in enumerate(idx):
        p.sample_idx[j] = int(v)
    p.num_samples = len(idx)
    u = g.to_dev(d["uniforms"].ravel()) if "uniforms" in d else None
    y, ws = g.smaq_apply(x, p, uniforms=u)
    st = g.read_stats(ws)
    _assert_stats_close(st["mean"], d["mean"], meta["dtype"])
    _assert_stats_close(st["raw_std"], d["std"], meta["dtype"])
    yh = y.cpu().numpy()
    if st["mean"] == d["mean"] and st["raw_std"] == d["std"]:
        assert same_f32(yh, d["y"])
    else:
        _assert_within_step(yh, d["y"], d["x"], st["raw_std"], hp)


def _assert_stats_close(ours, ref, dtype):
    """fp32: within 1 ulp; half types: equal or one step of the half type apart."""
    if dtype == "f32":
        assert ulp_diff(ours, ref) <= 1, (ours, ref)
    else:
        step = float(np.spacing(np.float16(ref))) if dtype == "f16" else abs(float(ref)) * 2.0**-7
        assert abs(float(ours) - float(ref)) <= step + 1e-30, (ours, ref)


def _assert_within_step(y, y_ref, x, std, hp, max_frac=1.0):
    from oracle import smaq as osmaq

    cfg = osmaq.SmaqConfig(num_bits_main=hp.num_bits_main, num_bits_outlier=hp.num_bits_outlier,
                           main_std_dev_threshold=hp.main_std_dev_threshold,
                           outlier_std_dev_threshold=hp.outlier_std_dev_threshold)
    s = np.float64(std if std != 0 else 1.0)
    step_out = s / np.float64(np.float32(cfg.range_outlier))
    step_main = s / np.float64(np.float32(cfg.range_normal))
    step = np.maximum(step_out, step_main)
    diff = np.abs(y.astype(np.float64) - y_ref.astype(np.float64))
    finite = np.isfinite(y_ref)
    assert np.all(np.isnan(y[~finite]) == np.isnan(y_ref[~finite]))
    assert np.all(diff[finite] <= 1.001 * step + 1e-6 * np.abs(y_ref[finite])), diff.max() / step


@pytest.mark.parametrize("name", [k for k in ACTIVE if not CASES[k]["use_sample_stats"]])
def test_golden_full_pipeline(name):
    """Device statistics (fp64) vs the reference's torch statistics, then outputs within a step."""
    g = _gpu()
    meta, d = CASES[name], load_smaq(name)
    hp = smaq_hparams(meta)
    x = g.golden_x(d, meta).reshape(-1)
    p = g.smaq_params(hp, x.numel(), all_positive=meta["all_positive"], dtype=x.dtype)
    keep = []
    _bind_bn(p, d, meta, d["x"].shape, keep)
    u = g.to_dev(d["uniforms"].ravel()) if "uniforms" in d else None
    y, ws = g.smaq_roundtrip(x, p, uniforms=u)
    st = g.read_stats(ws)
    from oracle import smaq as osmaq

    mo, so = osmaq.full_stats(d["x"], oracle_cfg(meta), meta["dtype"])
    _assert_stats_close(st["mean"], mo, meta["dtype"])
    _assert_stats_close(st["raw_std"], so, meta["dtype"])
    if meta["num_bits_main"] == 2:  # range_normal == 0 -> NaN like the reference
        assert np.isnan(y.cpu().numpy()).sum() == np.isnan(d["y"]).sum()
        return
    yh = y.cpu().numpy().reshape(d["y"].shape)
    if st["mean"] == d["mean"] and st["raw_std"] == d["std"]:
        assert same_f32(yh, d["y"])
    else:
        _assert_within_step(yh.ravel(), d["y"].ravel(), d["x"].ravel(), st["raw_std"], hp)


def _smaq_ws():
    from smart_compress_amd import _native as N

    # the current stream's workspace (earlier tests may have left others, e.g. a capture stream's)
    return N._ws[("smaq", 0, N.stream_ptr(torch.device("cuda")))]


def _oracle_check(x_np, y_dev, ws, hp, seed, offset, all_positive=False, window=None):
    """Device output == oracle(x, device stats, counter RNG), bit for bit."""
    from oracle import rng as orng
    from oracle import smaq as osmaq

    g = _gpu()
    st = g.read_stats(ws)
    cfg = osmaq.SmaqConfig(num_bits_main=hp.num_bits_main, num_bits_outlier=hp.num_bits_outlier,
                           main_std_dev_threshold=hp.main_std_dev_threshold,
                           outlier_std_dev_threshold=hp.outlier_std_dev_threshold,
                           stochastic_rounding=hp.stochastic_rounding)
    lo, hi = window if window else (0, x_np.size)
    u = orng.uniforms(seed, offset, hi - lo, start=lo) if hp.stochastic_rounding else None
    y_or, _ = osmaq.apply(x_np[lo:hi], st["mean"], st["raw_std"], cfg, u, all_positive)
    yh = y_dev[lo:hi].cpu().numpy()
    assert same_f32(yh, y_or), f"{n_diff_f32(yh, y_or)} of {hi - lo} differ in [{lo},{hi})"
    return st


@pytest.mark.parametrize("n,offset_elems", [(1 << 20, 0), (1000003, 0), (65537, 1), (4099, 3)])
@pytest.mark.parametrize("sr", [True, False])
def test_smartfp_vs_oracle(n, offset_elems, sr):
    """The drop-in class end to end (incl. unaligned/ragged views) vs the oracle."""
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import SmartFP

    g = _gpu()
    gen = torch.Generator(device="cuda").manual_seed(n + offset_elems)
    base = torch.randn(n + offset_elems, generator=gen, device="cuda") * 2.5 + 0.3
    x = base[offset_elems:]
    hp = smaq_hparams(stochastic_rounding=sr)
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 1234, 777
    y = codec(x)
    torch.cuda.synchronize()
    ws = _smaq_ws()
    xn = x.cpu().numpy()
    mo, so = osmaq.full_stats(xn, osmaq.SmaqConfig())
    st = g.read_stats(ws)
    assert ulp_diff(st["mean"], mo) <= 1 and ulp_diff(st["raw_std"], so) <= 1
    _oracle_check(xn, y, ws, hp, 1234, 777)
    assert y.shape == x.shape and y.dtype == x.dtype and y.data_ptr() != x.data_ptr()


def test_constant_and_small():
    from smart_compress_amd.compress.smart import SmartFP

    hp = smaq_hparams()
    codec = SmartFP(hp)
    x = torch.full((5000,), -2.25, device="cuda")
    assert torch.equal(codec(x), x)  # std == 0 -> 1, every z == 0
    x7 = torch.randn(7, device="cuda")
    assert codec(x7) is x7  # n < min_size: same object (smart.py:128)
    x8 = torch.randn(8, device="cuda")
    y8 = codec(x8)
    assert y8.shape == (8,) and torch.isfinite(y8).all()


def test_all_positive_and_shapes():
    from smart_compress_amd.compress.smart import SmartFP

    codec = SmartFP(smaq_hparams())
    x = torch.randn(3, 5, 7, 11, device="cuda") ** 2 * 1e-5
    y = codec(x, all_positive=True, tag="optimizer_momentum")
    assert y.shape == x.shape and (y >= 0).all()
    xt = torch.randn(64, 48, device="cuda").t()  # non-contiguous input
    yt = codec(xt)
    assert yt.shape == xt.shape


def test_sampled_mode_end_to_end():
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import SmartFP

    g = _gpu()
    hp = smaq_hparams(use_sample_stats=True)
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 99, 0
    x = torch.randn(1 << 18, device="cuda")
    from oracle import rng as orng0

    idx = orng0.floyd_indices(99, 0, x.numel(), 16)  # the draw the device makes at offset 0
    y = codec(x)
    torch.cuda.synchronize()
    xn = x.cpu().numpy()
    assert len(set(idx.tolist())) == 16
    mean, std = osmaq.sampled_stats(xn, idx, osmaq.SmaqConfig())
    from oracle import rng as orng

    cfg = osmaq.SmaqConfig()
    y_or, _ = osmaq.apply(xn, mean, std, cfg, orng.uniforms(99, 0, xn.size))
    assert same_f32(y.cpu().numpy(), y_or)


def test_measure_compression_ratio_logging():
    from smart_compress_amd.compress.smart import SmartFP

    hp = smaq_hparams(measure_compression_ratio=True)
    codec = SmartFP(hp)
    logged = {}
    codec.log = lambda k, v, **kw: logged.__setitem__(k, v)
    x = torch.randn(100000, device="cuda")
    codec(x, tag="forward_autograd")
    n_out = int(((x - x.mean()).abs() > x.std()).sum())
    expect_bits = n_out * 8 + (x.numel() - n_out) * 6
    assert abs(logged["new_size_forward_autograd"] - expect_bits) <= 8 * 2
    assert logged["orig_size"] == x.numel() * 32
    assert abs(logged["compression_ratio"] - x.numel() * 32 / expect_bits) < 1e-3


def test_sr_unbiased():
    """E[y] == x for stochastic rounding (test.py's drift idea, with full statistics)."""
    from smart_compress_amd.compress.smart import SmartFP

    codec = SmartFP(smaq_hparams())
    x = torch.randn(4096, device="cuda")
    acc = torch.zeros_like(x)
    reps = 400
    for _ in range(reps):
        acc += codec(x)
    err = (acc / reps - x).abs().max().item()
    assert err < 0.05  # step 1/15 std, sd of the mean ~ step/2/sqrt(400)*...


def _oracle_every_element(x, y, st, hp, seed, offset, chunk=1 << 24):
    """Every element of y vs the oracle fed x, the device statistics and the counter RNG, bit for
    bit: host chunks of 16M elements on a thread pool (numpy releases the GIL). Returns the number
    of elements compared."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import rng as orng
    from oracle import smaq as osmaq

    n = x.numel()
    xh = x.cpu().numpy()
    yh = y.cpu().numpy()
    cfg = osmaq.SmaqConfig(num_bits_main=hp.num_bits_main, num_bits_outlier=hp.num_bits_outlier,
                           main_std_dev_threshold=hp.main_std_dev_threshold,
                           outlier_std_dev_threshold=hp.outlier_std_dev_threshold,
                           stochastic_rounding=hp.stochastic_rounding)

    def one(lo):
        hi = min(n, lo + chunk)
        u = orng.uniforms(seed, offset, hi - lo, start=lo) if hp.stochastic_rounding else None
        y_or, _ = osmaq.apply(xh[lo:hi], st["mean"], st["raw_std"], cfg, u)
        return n_diff_f32(yh[lo:hi], y_or)

    with ThreadPoolExecutor(max_workers=8) as pool:
        bad = sum(pool.map(one, range(0, n, chunk)))
    assert bad == 0, f"{bad} of {n} elements differ from the oracle"
    return n


@pytest.mark.slow
def test_full_size_256m_every_element():
    """BASELINE config 2 (the headline: 268,435,456 fp32 N(0,1) elements): statistics vs fp64
    within 1 ulp, then EVERY output element vs the oracle (device statistics, same counter RNG),
    bit for bit; outlier share and SR bias as size-independent properties."""
    from smart_compress_amd.compress.smart import SmartFP

    n = 1 << 28
    gen = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(n, generator=gen, device="cuda")
    hp = smaq_hparams()
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 5, 0
    y = codec(x)
    torch.cuda.synchronize()
    st = _gpu().read_stats(_smaq_ws())
    xd = x.double()
    assert ulp_diff(st["mean"], np.float32(xd.mean().item())) <= 1
    assert ulp_diff(st["raw_std"], np.float32(xd.std().item())) <= 1
    del xd
    frac_out = ((x - st["mean"]).abs() / st["std_clamped"] > 1.0).float().mean().item()
    assert abs(frac_out - 0.3173) < 0.002
    assert abs((y - x).double().mean().item()) < 1e-4  # unbiased SR
    assert _oracle_every_element(x, y, st, hp, 5, 0) == n


def _laplace(n, seed, device="cuda"):
    """Laplace(0, 1) as the difference of two Exp(1) draws -log1p(-U), U in [0, 1) (SURVEY 8d
    C2's heavy-tailed variant; finite for every U)."""
    gen = torch.Generator(device=device).manual_seed(seed)
    x = -torch.log1p(-torch.rand(n, generator=gen, device=device))
    return x.sub_(-torch.log1p(-torch.rand(n, generator=gen, device=device)))


def test_full_size_256m_laplace_every_element():
    """C2's heavy-tailed variant at full size: Laplace(0, 1) puts ~24 % of the elements beyond
    1 std and a long tail beyond T_o = 2.5 std (outliers the 8-bit range clips). Statistics vs
    fp64, every element vs the oracle, outlier fraction vs the Laplace law."""
    from smart_compress_amd.compress.smart import SmartFP

    n = 1 << 28
    x = _laplace(n, 7)
    hp = smaq_hparams()
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 5, 0
    y = codec(x)
    torch.cuda.synchronize()
    st = _gpu().read_stats(_smaq_ws())
    xd = x.double()
    assert ulp_diff(st["mean"], np.float32(xd.mean().item())) <= 1
    assert ulp_diff(st["raw_std"], np.float32(xd.std().item())) <= 1
    del xd
    # P(|x| > sqrt(2)) = exp(-sqrt(2)) for Laplace(0, 1) (std sqrt(2))
    frac_out = ((x - st["mean"]).abs() / st["std_clamped"] > 1.0).float().mean().item()
    assert abs(frac_out - float(np.exp(-np.sqrt(2.0)))) < 0.002
    assert abs((y - x).double().mean().item()) < 1e-4
    assert _oracle_every_element(x, y, st, hp, 5, 0) == n


def test_full_size_256m_sampled_every_element():
    """C2 with --use_sample_stats (smart.py:86-91): the 16 indices the device draws equal
    oracle/rng.py floyd_indices, the statistics equal the oracle's over them, and every one of the
    268,435,456 outputs equals the oracle's, bit for bit."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.smart import SmartFP

    n = 1 << 28
    gen = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(n, generator=gen, device="cuda") * 0.7 + 0.1
    hp = smaq_hparams(use_sample_stats=True)
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 21, 1 << 30
    y = codec(x)
    torch.cuda.synchronize()
    ws = _smaq_ws()
    o = N.SMQ_WS_SAMPLES_OFFSET
    idx = ws[o: o + 8 * 16].cpu().numpy().view(np.int64).copy()
    assert idx.tolist() == orng.floyd_indices(21, 1 << 30, n, 16).tolist()
    st = _gpu().read_stats(ws)
    mo, so = osmaq.sampled_stats(x[torch.from_numpy(idx).cuda()].cpu().numpy(), np.arange(16),
                                 osmaq.SmaqConfig())
    assert ulp_diff(st["mean"], mo) <= 1 and ulp_diff(st["raw_std"], so) <= 1, (st, mo, so)
    assert _oracle_every_element(x, y, st, hp, 21, 1 << 30) == n


@pytest.mark.parametrize("dt", ["f16", "bf16"])
@pytest.mark.parametrize("offset_elems,n", [(0, 1 << 18), (4, (1 << 20) + 5), (1, 70001),
                                            (0, (3 << 22) + 8)])
def test_half_inputs_end_to_end(dt, offset_elems, n):
    """SmartFP on fp16 / bf16 tensors (Lightning precision=16): fp32 output, stats in the input
    type, bit-exact vs the oracle fed the device statistics and counter RNG. Offsets: 0 (16-B
    aligned: tile sweep with 16-B loads), 4 elements (8-B aligned: grid-stride sweep), 1 (element
    path); 12M runs the non-deferred round trip and several statistics tiles per workgroup."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import SmartFP

    g = _gpu()
    tdt = g.TORCH_DT[dt]
    gen = torch.Generator(device="cuda").manual_seed(11)
    base = (torch.randn(n + offset_elems, generator=gen, device="cuda") * 1.5 - 0.2).to(tdt)
    x = base[offset_elems:]
    hp = smaq_hparams(precision=16)
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 3, 10
    y = codec(x)
    torch.cuda.synchronize()
    assert y.dtype == torch.float32 and y.shape == x.shape
    st = g.read_stats(_smaq_ws())
    xn = x.float().cpu().numpy()
    cfg = osmaq.SmaqConfig(precision=16)
    mo, so = osmaq.full_stats(xn, cfg, dt)
    _assert_stats_close(st["mean"], mo, dt)
    _assert_stats_close(st["raw_std"], so, dt)
    y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], cfg, orng.uniforms(3, 10, xn.size),
                          dtype=dt)
    assert same_f32(y.cpu().numpy(), y_or)


@pytest.mark.parametrize("dt", ["f16", "bf16"])
def test_half_apply_fp32_quotient_extremes(dt):
    """The non-deferred half apply takes the two-op fp32 quotient q / range (smq_half_quot_split,
    checked over every reachable code): data whose std exceeds the precision-16 clamp (1e4) gives
    z-scores far beyond the thresholds — bf16 at 1e30 scale: codes up to ~1e27, fp16 near its
    maximum: z ~ 6 and every class — still bit-exact against the oracle."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.smart import SmartFP

    g = _gpu()
    n = (3 << 22) + 8  # above kDeferMaxN: the statistics + apply launches
    gen = torch.Generator(device="cuda").manual_seed(12)
    base = torch.randn(n, generator=gen, device="cuda")
    base = base * 1e30 if dt == "bf16" else (base * 2e4).clamp(-6e4, 6e4)
    x = base.to(g.TORCH_DT[dt])
    hp = smaq_hparams(precision=16)
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 5, 3
    out = (ctypes.c_float * 4)()
    assert N.lib().smq_half_quot_split(N.SMQ_DTYPE_F16 if dt == "f16" else N.SMQ_DTYPE_BF16,
                                       float(np.float32(hp.main_std_dev_threshold)),
                                       float(np.float32(codec.range_normal)),
                                       float(np.float32(codec.range_outlier)), 1, out) == 1
    y = codec(x)
    torch.cuda.synchronize()
    st = g.read_stats(_smaq_ws())
    assert st["std_clamped"] < st["raw_std"]  # the clamp is active
    xn = x.float().cpu().numpy()
    cfg = osmaq.SmaqConfig(precision=16)
    y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], cfg, orng.uniforms(5, 3, xn.size),
                          dtype=dt)
    assert same_f32(y.cpu().numpy(), y_or)


def test_half_precision_rules():
    from smart_compress_amd.compress.smart import SmartFP

    x = torch.randn(100, device="cuda").half()
    with pytest.raises(RuntimeError, match="Half without overflow"):
        SmartFP(smaq_hparams(precision=32))(x)  # std.clamp(1e-38, 1e38) overflows half
    y = SmartFP(smaq_hparams(precision=32))(x.bfloat16())  # bf16 holds 1e38
    assert y.dtype == torch.float32
    # fp64 data runs in fp64 and stays fp64 (smart.py's type flow; tests/test_f64.py)
    assert SmartFP(smaq_hparams())(torch.randn(100, device="cuda").double()).dtype == torch.float64
    with pytest.raises(NotImplementedError):
        SmartFP(smaq_hparams())(torch.ones(100, device="cuda", dtype=torch.int32))


def _subnormal_mix(n, seed):
    """Subnormal floats, tiny normals and ordinary values, both signs."""
    rs = np.random.default_rng(seed)
    bits = rs.integers(1, 1 << 23, n, dtype=np.uint32)  # subnormal patterns
    x = bits.view(np.float32).copy()
    x[1::4] = rs.uniform(1e-38, 1e-30, x[1::4].size).astype(np.float32)
    x[2::4] = rs.normal(0, 1, x[2::4].size).astype(np.float32)
    x[rs.random(n) < 0.5] *= -1
    return x


@pytest.mark.parametrize("sc", [3.0, 0.7, 6.0, 2.0**25])
def test_subnormal_z_paths(sc):
    """z = (x - mean) / std subnormal: the guard-free body (sc neither an even integer nor >= 2^24,
    proven exact by oracle/csrc/div_check.c) and the checked body both match IEEE division."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import quot_check_for

    g = _gpu()
    hp = smaq_hparams()
    x = _subnormal_mix(1 << 16, int(sc * 10))
    xd = g.to_dev(x)
    p = g.smaq_params(hp, x.size, seed=5, offset=11)
    stats = g.stats_struct(0.0, sc, hp)
    y, ws = g.smaq_apply(xd, p, stats_in=stats)
    torch.cuda.synchronize()
    from smart_compress_amd import _native as N

    o = N.SmqSmaqStats.quot_check.offset
    flag = int(ws[o:o + 4].cpu().numpy().view(np.uint32)[0])
    assert flag == quot_check_for(sc) == (1 if sc in (6.0, 2.0**25) else 0)
    y_or, _ = osmaq.apply(x, 0.0, sc, osmaq.SmaqConfig(), orng.uniforms(5, 11, x.size))
    assert same_f32(y.cpu().numpy(), y_or), n_diff_f32(y.cpu().numpy(), y_or)


def test_huge_range_ieee_quotient():
    """A range beyond 2^100 (main threshold 1e-37 -> r_main ~ 1.5e38) makes q / range subnormal:
    the launcher routes it to the IEEE-division variant; bit-exact vs the oracle."""
    from oracle import rng as orng
    from oracle import smaq as osmaq

    g = _gpu()
    hp = smaq_hparams(main_std_dev_threshold=1e-37)
    x = _subnormal_mix(1 << 14, 3)
    x[2::4] *= 1e-30
    p = g.smaq_params(hp, x.size, seed=9, offset=0)
    y, _ = g.smaq_apply(g.to_dev(x), p, stats_in=g.stats_struct(0.0, 1.0, hp))
    torch.cuda.synchronize()
    cfg = osmaq.SmaqConfig(main_std_dev_threshold=1e-37)
    y_or, _ = osmaq.apply(x, 0.0, 1.0, cfg, orng.uniforms(9, 0, x.size))
    yh = y.cpu().numpy()
    assert same_f32(yh, y_or), n_diff_f32(yh, y_or)
    assert np.any((np.abs(yh) < np.finfo(np.float32).tiny) & (yh != 0))  # subnormal q / range hit


def test_graph_safe_stream_eager_and_captured():
    """SmartFP.graph_safe(): the stream position lives in a device counter advanced by the first
    kernel of each call. Eager calls equal the host-offset mode; a captured torch.cuda graph draws
    fresh, consecutive streams on every replay (each replay equals the next host-mode call)."""
    from smart_compress_amd.compress.smart import SmartFP

    n = (1 << 20) + 3
    x = torch.randn(n, device="cuda") * 1.7
    host = SmartFP(smaq_hparams())
    host.rng.seed, host.rng.offset = 77, 5
    dev = SmartFP(smaq_hparams())
    dev.rng.seed, dev.rng.offset = 77, 5
    dev.graph_safe(device="cuda")
    for _ in range(3):  # eager: identical streams
        assert torch.equal(dev(x).view(torch.int32), host(x).view(torch.int32))
    torch.cuda.synchronize()
    # capture one call, replay three times
    static_x = x.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        dev(static_x)  # warm-up on the capture stream (workspace for this stream)
        host(static_x)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y_static = dev(static_x)
    outs = []
    for _ in range(3):
        g.replay()
        outs.append(y_static.clone())
    torch.cuda.synchronize()
    refs = [host(static_x) for _ in range(3)]
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert torch.equal(o.view(torch.int32), r.view(torch.int32))
    assert not torch.equal(outs[0], outs[1])  # fresh randomness per replay


@pytest.mark.parametrize("n", [65536 + 5, 1 << 20, 5 * (1 << 20) + 3, 9 * (1 << 20), 40 << 20])
@pytest.mark.parametrize("mode", ["sr", "trunc", "range", "f16", "bf16", "allpos", "counter"])
def test_deferred_statistics_equal_two_call_path(n, mode):
    """smq_smaq_roundtrip on tensors up to kDeferMaxN (12M) reduces the statistics partials in
    every apply workgroup (smaq.hip defer_consts) instead of in the last statistics workgroup.
    Outputs, header and graph-safe stream position equal the separate smq_smaq_stats +
    smq_smaq_apply calls bit for bit BY CONSTRUCTION: both statistics launches use the same grid
    (<= 256 workgroups up to 12M elements) and both reductions run reduce_partials_w0's one fixed
    order; 40M runs the non-deferred path through the same entry point."""
    from smart_compress_amd import _native as N

    g = _gpu()
    gen = torch.Generator(device="cuda").manual_seed(n % 1000 + len(mode))
    dt = {"f16": torch.float16, "bf16": torch.bfloat16}.get(mode, torch.float32)
    x = (torch.randn(n, generator=gen, device="cuda") * 1.3 - 0.2)
    if mode == "allpos":
        x = x.abs()
    x = x.to(dt)
    hp = smaq_hparams(stochastic_rounding=mode != "trunc", use_range_std_dev=mode == "range")
    outs, hdrs, ctrs = [], [], []
    for split in (False, True):
        p = g.smaq_params(hp, n, all_positive=mode == "allpos", seed=99, offset=12345, dtype=dt)
        ctr = None
        if mode == "counter":
            ctr = torch.tensor([1 << 33], dtype=torch.int64, device="cuda")
            p.offset_counter = ctr.data_ptr()
        y = torch.empty(n, dtype=torch.float32, device="cuda")
        ws = torch.zeros(N.lib().smq_smaq_workspace_bytes(n), dtype=torch.uint8, device="cuda")
        args = (x.data_ptr(), N.DTYPE_CODES[dt])
        if split:
            N.check(N.lib().smq_smaq_stats(*args, n, p, ws.data_ptr(), ws.numel(), g.stream()),
                    "stats")
            N.check(N.lib().smq_smaq_apply(*args, y.data_ptr(), n, p, None, None, ws.data_ptr(),
                                           ws.numel(), g.stream()), "apply")
        else:
            N.check(N.lib().smq_smaq_roundtrip(*args, y.data_ptr(), n, p, None, ws.data_ptr(),
                                               ws.numel(), g.stream()), "roundtrip")
        torch.cuda.synchronize()
        outs.append(y)
        hdrs.append(g.read_stats(ws))
        ctrs.append(None if ctr is None else int(ctr.item()))
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
    for k in ("mean", "std_dev", "std_clamped", "raw_std", "n_used"):
        assert hdrs[0][k] == hdrs[1][k], k
    if mode == "range":
        assert hdrs[0]["min"] == hdrs[1]["min"] and hdrs[0]["max"] == hdrs[1]["max"]
    if mode == "counter":
        assert ctrs[0] == ctrs[1] == (1 << 33) + n


@pytest.mark.parametrize("n", [100003, 5 << 20, 13 << 20])
@pytest.mark.parametrize("special", ["nan", "inf", "-inf"])
def test_nonfinite_input_propagates_like_reference(special, n):
    """One NaN / +-inf element: the reference's data.mean() / data.std() become NaN or inf
    (inf - inf), the clamp keeps NaN, and every output element is NaN (smart.py:130-182). The
    device statistics (deferred below 12M, counted hand-off above) equal the fp64 oracle's and
    the output equals the oracle's bit for bit (every NaN equal to every NaN)."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from smart_compress_amd.compress.smart import SmartFP

    gen = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(n, generator=gen, device="cuda")
    x[n // 3] = float(special)
    hp = smaq_hparams()
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = 8, 0
    y = codec(x)
    torch.cuda.synchronize()
    st = _gpu().read_stats(_smaq_ws())
    xn = x.cpu().numpy()
    with np.errstate(invalid="ignore"):  # inf - inf in the oracle's centred sums
        mo, so = osmaq.full_stats(xn, osmaq.SmaqConfig())
    assert same_f32(np.float32(st["mean"]), mo) and same_f32(np.float32(st["raw_std"]), so)
    y_or, _ = osmaq.apply(xn, st["mean"], st["raw_std"], osmaq.SmaqConfig(),
                          orng.uniforms(8, 0, n))
    yh = y.cpu().numpy()
    assert same_f32(yh, y_or)
    assert np.isnan(yh).all()
