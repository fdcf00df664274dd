"""The host packer (smq_cpu_smaq_compress / smq_cpu_smaq_decompress, csrc/cpu_codecs.hip) behind
SmartFPPacked on CPU tensors (smart.py:110-190 runs on any device).

* the stream equals the format restatement (oracle/smaq_packed.py — which the GPU stream equals
  byte for byte in tests/test_gpu_packed.py) given the host statistics and the counter RNG: every
  byte, on the golden cases' inputs and on escape-heavy, ragged, BN, half and threshold variants;
* decompress(compress(x)) equals SmartFP on the same CPU tensor (same flags, same random stream)
  bit for bit, incl. sampled statistics above 4096 device-style draws;
* the result does not depend on the thread count.
"""

import numpy as np
import pytest
import torch

from helpers import load_smaq, n_diff_f32, same_f32, smaq_cases, smaq_hparams

CASES = smaq_cases()
PACKABLE = sorted(k for k in CASES if not k.startswith("n7"))


def _codecs(hp, seed=5, offset=77):
    from smart_compress_amd.compress import SmartFP, SmartFPPacked

    a, b = SmartFPPacked(hp), SmartFP(hp)
    for c in (a, b):
        c.rng.seed, c.rng.offset = seed, offset
    return a, b


def _oracle_stream(x, hp, seed, offset, all_positive=False, bn=None, dtype="f32"):
    """The restatement's stream with the host packer's own statistics (left in its workspace)."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from oracle import smaq_packed as P
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress import SmartFP

    ws = N.cpu_workspace("smaq", 1)
    st = SmartFP.read_stats(ws)
    cfg = osmaq.SmaqConfig(num_bits_main=hp.num_bits_main, num_bits_outlier=hp.num_bits_outlier,
                           main_std_dev_threshold=hp.main_std_dev_threshold,
                           outlier_std_dev_threshold=hp.outlier_std_dev_threshold,
                           stochastic_rounding=hp.stochastic_rounding,
                           use_range_std_dev=hp.use_range_std_dev, precision=hp.precision)
    u = orng.uniforms(seed, offset, x.size) if hp.stochastic_rounding else None
    return P.pack(x, st["mean"], st["raw_std"], cfg, u, all_positive, dtype, bn)


def _bytes(p):
    return p.data.numpy()


@pytest.mark.parametrize("name", PACKABLE)
def test_host_stream_equals_restatement_golden_inputs(name):
    meta, d = CASES[name], load_smaq(name)
    if meta.get("use_sample_stats"):
        pytest.skip("sampled: covered by test_host_packer_sampled (drawn indices)")
    hp = smaq_hparams(meta, measure_compression_ratio=False)
    dt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[meta["dtype"]]
    x = torch.from_numpy(np.ascontiguousarray(d["x"])).to(dt)
    bn = None
    if "bn_gamma" in d:
        hp.use_batch_norm = True
        bn = (torch.from_numpy(d["bn_gamma"]), torch.from_numpy(d["bn_beta"]))
    pk, ref = _codecs(hp)
    p = pk.compress(x, meta["all_positive"], bn)
    bn_np = None
    if bn is not None:
        g, b = (d["bn_gamma_used"], d["bn_beta_used"]) if meta["bn_scalar_params"] else (
            d["bn_gamma"], d["bn_beta"])
        bn_np = (g, b)
    want = _oracle_stream(d["x"] if dt == torch.float32 else x.float().numpy(), hp, 5, 77,
                          meta["all_positive"], bn_np, meta["dtype"])
    assert np.array_equal(_bytes(p), want)
    y = ref(x, all_positive=meta["all_positive"], batch_norm_stats=bn)
    yp = pk.decompress(p)
    assert same_f32(yp.numpy(), y.numpy()), n_diff_f32(yp.numpy(), y.numpy())


@pytest.mark.parametrize("n", [9, 4095, 4096, 4097, 3 * 4096 + 5, 70_001])
@pytest.mark.parametrize("bits,thr,sr", [((6, 8), 1.0, True), ((4, 6), 1.0, False),
                                         ((2, 3), 0.5, True), ((9, 12), -0.3, True),
                                         ((6, 4), 1.5, True), ((13, 25), 1.0, True)])
def test_host_stream_escapes_and_sizes(n, bits, thr, sr):
    rs = np.random.default_rng(n + bits[0])
    x = (rs.standard_t(1.5, n) * 3).astype(np.float32)  # heavy tails: wrong-sign / large codes
    hp = smaq_hparams(num_bits_main=bits[0], num_bits_outlier=bits[1],
                      main_std_dev_threshold=thr, stochastic_rounding=sr)
    for ap in (False, True):
        xi = np.abs(x) if ap else x
        pk, ref = _codecs(hp)
        p = pk.compress(torch.from_numpy(xi), ap)
        assert np.array_equal(_bytes(p), _oracle_stream(xi, hp, 5, 77, ap))
        y = ref(torch.from_numpy(xi), all_positive=ap)
        assert same_f32(pk.decompress(p).numpy(), y.numpy())


def test_host_stream_specials_and_half():
    """NaN / inf inputs (the reference's all-NaN output) and fp16 / bf16 inputs."""
    rs = np.random.default_rng(3)
    x = rs.standard_normal(20_000).astype(np.float32)
    x[17] = np.inf
    hp = smaq_hparams()
    pk, ref = _codecs(hp)
    p = pk.compress(torch.from_numpy(x))
    assert np.array_equal(_bytes(p), _oracle_stream(x, hp, 5, 77))
    assert same_f32(pk.decompress(p).numpy(), ref(torch.from_numpy(x)).numpy())
    for dt, name, prec in ((torch.float16, "f16", 16), (torch.bfloat16, "bf16", 32)):
        hp = smaq_hparams(precision=prec)
        pk, ref = _codecs(hp)
        xt = torch.from_numpy(rs.standard_normal(50_003).astype(np.float32) * 3).to(dt)
        p = pk.compress(xt)
        assert np.array_equal(_bytes(p), _oracle_stream(xt.float().numpy(), hp, 5, 77, dtype=name))
        assert same_f32(pk.decompress(p).numpy(), ref(xt).numpy())


def test_host_packer_bn_variant():
    rs = np.random.default_rng(4)
    x = torch.from_numpy(rs.standard_normal((4, 6, 9, 11)).astype(np.float32) * 2 + 1)
    g = torch.from_numpy(rs.uniform(0.5, 2.0, 6).astype(np.float32))
    b = torch.from_numpy(rs.standard_normal(6).astype(np.float32))
    for scalar in (False, True):
        hp = smaq_hparams(use_batch_norm=True, bn_scalar_params=scalar)
        pk, ref = _codecs(hp)
        p = pk.compress(x, False, (g, b))
        gg, bb = (g.mean().reshape(1), b.mean().reshape(1)) if scalar else (g, b)
        want = _oracle_stream(x.numpy(), hp, 5, 77, bn=(gg.numpy(), bb.numpy()))
        assert np.array_equal(_bytes(p), want)
        y = ref(x, batch_norm_stats=(g, b))
        assert same_f32(pk.decompress(p).numpy(), y.numpy())


@pytest.mark.parametrize("k", [16, 5000])
def test_host_packer_sampled(k):
    """Sampled statistics (smart.py:86-91) with the device-style draw, above 4096 samples too:
    decompress(compress(x)) equals SmartFP's output on the same stream position."""
    rs = np.random.default_rng(k)
    x = torch.from_numpy(rs.standard_normal(60_000).astype(np.float32))
    hp = smaq_hparams(use_sample_stats=True, num_samples=k)
    pk, ref = _codecs(hp)
    p = pk.compress(x)
    assert same_f32(pk.decompress(p).numpy(), ref(x).numpy())
    assert pk.rng.offset == ref.rng.offset


def test_host_packer_thread_invariant_and_ratio():
    from smart_compress_amd.compress import SmartFPPacked

    rs = np.random.default_rng(8)
    x = torch.from_numpy(rs.standard_normal(1 << 20).astype(np.float32))
    hp = smaq_hparams()
    outs = []
    prev = torch.get_num_threads()
    try:
        for t in (1, 3, 8):
            torch.set_num_threads(t)
            pk = SmartFPPacked(hp)
            pk.rng.seed, pk.rng.offset = 2, 0
            outs.append(_bytes(pk.compress(x)))
    finally:
        torch.set_num_threads(prev)
    assert all(np.array_equal(o, outs[0]) for o in outs)
    assert 4.0 < 32 * x.numel() / (8 * outs[0].size) < 4.6  # ~7.4 bits per element (N(0,1))


def test_host_decoder_rejects_other_streams():
    """A stream of another n, or a bad magic, is refused and y left untouched."""
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress import SmartFPPacked

    pk = SmartFPPacked(smaq_hparams())
    p = pk.compress(torch.randn(10_000))
    y = torch.full((9_999,), 7.0)
    with pytest.raises(RuntimeError):
        N.check(N.lib().smq_cpu_smaq_decompress(p.data.data_ptr(), y.data_ptr(), 9_999, 1),
                "smq_cpu_smaq_decompress")
    bad = p.data.clone()
    bad[0] ^= 1
    y = torch.full((10_000,), 7.0)
    with pytest.raises(RuntimeError):
        N.check(N.lib().smq_cpu_smaq_decompress(bad.data_ptr(), y.data_ptr(), 10_000, 1),
                "smq_cpu_smaq_decompress")
    assert bool((y == 7.0).all())
