"""The oracle pinned against golden vectors produced by the reference implementation itself
(tests/golden/make_golden.py ran smart_compress/compress/*.py in the build container).

* SmaQ: oracle.smaq.apply fed the reference's statistics and its recorded torch.rand_like draws
  reproduces the reference output BIT FOR BIT in every mode (SR/trunc, sampled, range-std, BN,
  all_positive, bit widths, thresholds) and the same outlier count.
* The oracle's own fp64 statistics: std within 1 ulp of torch's (fp64 Welford); the mean within
  the error bound of torch's fp32 cascade sum (|d| <= 2^-21 * (|mean| + std)).
* float_quantize wrapper (check_inf, max value) for fp8/fp16/bf16: BIT-EXACT given the recorded
  random words (the quantiser restates qtorch; its own arithmetic is parity-unpinned).
* S2FP8: alpha, beta, 2^beta bit-exact from the reference's (mu, max); E5M2 codes identical;
  outputs within 4 ulp (library pow).
"""

import numpy as np
import pytest

from helpers import (float_meta, load_float, load_s2p16, load_smaq, n_diff_f32, oracle_cfg, same_f32,
                     s2p16_meta, smaq_cases, ulp_diff)

CASES = smaq_cases()
FMETA = float_meta()


@pytest.mark.parametrize("name", sorted(CASES))
def test_smaq_oracle_bitexact(name):
    from oracle import smaq

    meta, d = CASES[name], load_smaq(name)
    cfg = oracle_cfg(meta)
    if bool(d["passthrough"]):
        assert d["x"].size < cfg.min_size
        assert same_f32(d["y"], d["x"])
        return
    bn = None
    if "bn_gamma" in d:
        bn = (d["bn_gamma_used"], d["bn_beta_used"]) if meta["bn_scalar_params"] else (
            d["bn_gamma"], d["bn_beta"])
    y, o = smaq.apply(d["x"], d["mean"], d["std"], cfg, d.get("uniforms"), meta["all_positive"], bn,
                      dtype=meta["dtype"])
    assert same_f32(y, d["y"]), n_diff_f32(y, d["y"])
    if int(d.get("n_outlier", -1)) >= 0:
        assert int(o.sum()) == int(d["n_outlier"])


@pytest.mark.parametrize("name", sorted(k for k in CASES if not k.startswith("n7")))
def test_smaq_oracle_stats(name):
    from oracle import smaq

    meta, d = CASES[name], load_smaq(name)
    cfg = oracle_cfg(meta)
    dt = meta["dtype"]
    if meta["use_sample_stats"]:
        m, s = smaq.sampled_stats(d["x"], d["sample_idx"], cfg, dt)
    else:
        m, s = smaq.full_stats(d["x"], cfg, dt)
    if dt == "f32":
        assert ulp_diff(s, d["std"]) <= 1
        bound = 2.0**-21 * (abs(float(d["mean"])) + float(d["std"]))
        assert abs(float(m) - float(d["mean"])) <= bound
    else:  # 0-dim results rounded to the half type: equal, or one half-ulp step apart
        for ours, ref in ((m, d["mean"]), (s, d["std"])):
            step = np.spacing(np.float16(ref)) if dt == "f16" else abs(float(ref)) * 2.0**-7
            assert abs(float(ours) - float(ref)) <= float(step) + 1e-30, (ours, ref)


def test_smaq_logged_sizes():
    """log_size keys/values the reference logged (compress/base.py:60-102)."""
    for name, meta in CASES.items():
        d = load_smaq(name)
        logged = meta["logged"]
        n = d["x"].size
        if n < meta["min_size"]:
            # reference bug kept: log_ratio(tag, orig_size, 32, 32) multiplies by 32 again
            assert logged["orig_size_golden"] == n * 32 * 32
            continue
        assert logged["orig_size"] == n * 32
        if int(d.get("n_outlier", -1)) >= 0:
            no = int(d["n_outlier"])
            assert logged["new_size"] == no * meta["num_bits_outlier"] + (n - no) * meta["num_bits_main"]
        assert set(logged) == {f"{k}{s}" for k in ("compression_ratio", "new_size", "orig_size")
                               for s in ("", "_golden")}


FMT = dict(fp8=(5, 2), fp16=(5, 10), bf16=(8, 7))


@pytest.mark.parametrize("key", sorted(k for k, m in FMETA["cases"].items() if m["codec"] != "s2fp8"))
def test_float_wrapper_bitexact(key):
    from oracle import qtorch_float as qf

    m, d = FMETA["cases"][key], load_float(key)
    y = qf.float_quantize(d["x"], *FMT[m["codec"]], d["q_rand"], m["check_inf"])
    assert same_f32(y, d["y"])


def test_max_values():
    from oracle import qtorch_float as qf

    for k, v in FMETA["max_values"].items():
        e, m = map(int, k.split("_"))
        assert float(qf.max_value(e, m)) == v


@pytest.mark.parametrize("key", sorted(k for k, m in FMETA["cases"].items() if m["codec"] == "s2fp8"))
def test_s2fp8_oracle(key):
    from oracle import qtorch_float as qf
    from oracle import s2fp8

    m, d = FMETA["cases"][key], load_float(key)
    st = s2fp8.derive(d["mu"], d["m"])
    for k in ("alpha", "beta", "beta_pow2"):
        assert st[k] == d[k], k
    own = s2fp8.stats(d["x"])
    assert ulp_diff(own["mu"], d["mu"]) <= 2 and ulp_diff(own["m"], d["m"]) <= 1
    Y = s2fp8.transform(d["x"], st)
    assert np.max(np.abs(Y.view(np.int32).astype(np.int64) - d["q_in"].view(np.int32))) <= 2
    T = qf.float_quantize(Y, 5, 2, d["q_rand"], m["check_inf"])
    T_ref = qf.float_quantize(d["q_in"], 5, 2, d["q_rand"], m["check_inf"])
    assert same_f32(T, T_ref)
    y = s2fp8.inverse(T_ref, d["x"], st)
    ok = (np.isnan(y) & np.isnan(d["y"])) | (np.abs(y.astype(np.float64) - d["y"])
                                             <= 4 * np.spacing(np.abs(d["y"])))
    assert ok.all()


@pytest.mark.parametrize("key", sorted(s2p16_meta()))
def test_s2fp8_p16_oracle(key):
    """S2FP8 at precision 16 (tests/golden/s2p16_*: the reference run with fp16 / bf16 / fp32
    tensors and hparams.precision = 16): alpha, beta, 2^beta from the reference's (mu, max) and the
    oracle's own (mu, max) bit-exact; the quantiser input Y bit-exact for fp16 / bf16 (rounded to
    the input type) and within 2 fp32 ulp for fp32; the half-precision inverse bit-exact."""
    from oracle import qtorch_float as qf
    from oracle import s2fp8

    m, d = s2p16_meta()[key], load_s2p16(key)
    dt = m["dtype"]
    st = s2fp8.derive_p16(d["mu"], d["m"], dt)
    for k in ("alpha", "beta", "beta_pow2"):
        assert same_f32(st[k], d[k]), k
    own = s2fp8.stats_p16(d["x"], dt)
    if dt == "f32":
        assert ulp_diff(own["mu"], d["mu"]) <= 2
    else:
        assert same_f32(own["mu"], d["mu"])
    assert same_f32(own["m"], d["m"])
    Y = s2fp8.transform_p16(d["x"], st, dt)
    if dt == "f32":
        fin = np.isfinite(d["q_in"])
        assert np.max(np.abs(Y[fin].view(np.int32).astype(np.int64)
                             - d["q_in"][fin].view(np.int32)), initial=0) <= 2
    else:
        assert same_f32(Y, d["q_in"])
    T_ref = qf.float_quantize(d["q_in"], 5, 2, d["q_rand"], m["check_inf"])
    y, out_dt = s2fp8.inverse_p16(T_ref, d["x"], st, dt)
    assert out_dt == m["out_dtype"]
    assert same_f32(y, d["y"]), n_diff_f32(y, d["y"])


def test_qtorch_known_answers():
    """E5M2 representable values are fixed points for any random word; saturation; subnormal
    spacing 2^-16; +-0 -> +0; inf/NaN saturate (qtorch treats them as exponent 255)."""
    from oracle import qtorch_float as qf

    rs = np.random.default_rng(0)
    vals = sorted({(1 + mnt / 4) * 2.0**e for e in range(-14, 16) for mnt in range(4)}
                  | {mnt / 4 * 2.0**-14 for mnt in range(4)})
    v = np.array(vals + [-a for a in vals], np.float32)
    for _ in range(4):
        r = rs.integers(0, 2**32, v.size, dtype=np.uint32)
        y = qf.quantize(v, 5, 2, r)
        assert np.all(y == v)
    x = np.array([57344, 1e9, -1e9, np.inf, -np.inf, np.nan, 0.0, -0.0], np.float32)
    y = qf.quantize(x, 5, 2, np.zeros(x.size, np.uint32))
    assert list(y[:5]) == [57344, 57344, -57344, 57344, -57344]
    assert abs(y[5]) == 57344
    assert y[6] == 0 and y[7] == 0 and not np.signbit(y[7])
    yc = qf.check_inf(y, 5, 2)
    assert yc[0] == np.inf and yc[2] == -57344
    sub = qf.quantize(np.array([3 * 2.0**-17], np.float32), 5, 2, np.array([0], np.uint32),
                      stochastic=False)
    assert sub[0] in (2 * 2.0**-16, 1 * 2.0**-16)


def test_rng_uniform_properties():
    from oracle import rng

    u = rng.uniforms(7, 0, 1 << 20)
    assert u.min() >= 0 and u.max() < 1
    assert abs(u.mean() - 0.5) < 2e-3
    assert abs(np.corrcoef(u[:-1], u[1:])[0, 1]) < 5e-3
    a = rng.rng_u32(1, 2**32 - 2, 4)
    b = np.concatenate([rng.rng_u32(1, 2**32 - 2, 2), rng.rng_u32(1, 2**32, 2)])
    assert np.array_equal(a, b)  # counter crosses the 32-bit boundary consistently


@pytest.mark.parametrize("name", ["normal", "laplace", "small_scale", "relu_allpos", "grad_like"])
def test_smaq_torch_restatement_bitexact(name):
    """oracle/smaq_torch.py (the torch-CPU op sequence bench.py times as the CPU baseline) equals the
    reference's outputs bit for bit with its recorded uniforms and statistics, and its own
    statistics are within 1 ulp of the reference's."""
    import torch

    from oracle import smaq_torch

    from helpers import smaq_cases

    meta = smaq_cases()[name]
    if (meta["use_sample_stats"] or meta["use_range_std_dev"] or meta["use_batch_norm"]
            or not meta["stochastic_rounding"] or meta["dtype"] != "f32"):
        pytest.skip("default-flag fp32 cases only")
    d = load_smaq(name)
    x = torch.from_numpy(d["x"])
    kw = dict(num_bits_main=meta["num_bits_main"], num_bits_outlier=meta["num_bits_outlier"],
              thr=meta["main_std_dev_threshold"], thr_outlier=meta["outlier_std_dev_threshold"],
              all_positive=meta["all_positive"], uniforms=torch.from_numpy(d["uniforms"]))
    y = smaq_torch.roundtrip(x, stats=(float(d["mean"]), float(d["std"])), **kw).numpy()
    assert np.array_equal(y.view(np.uint32), d["y"].astype(np.float32).view(np.uint32))
    m, s = x.mean().item(), x.std().item()
    for a, b in ((m, d["mean"]), (s, d["std"])):
        assert abs(int(np.float32(a).view(np.int32)) - int(np.float32(b).view(np.int32))) <= 1

