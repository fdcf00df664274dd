"""float64 tensors in the packed SmaQ container (flag SMQ_PACK_FLAG_F64; csrc/smaq_pack_f64.hip and
its host twin in csrc/cpu_codecs.hip) behind SmartFPPacked — smart.py:110-190 on a float64 tensor,
as SmartFP runs it (the fp64 chain: z, q and the de-quantisation in fp64).

* the stream equals the format restatement (oracle/smaq_packed.py pack_f64) given the codec's own
  fp64 statistics (left in its workspace) and the counter RNG, byte for byte — host (CPU tensors)
  and device (ROCm tensors);
* decompress(compress(x)) equals SmartFP(x) on float64 bit for bit (NaN where SmartFP gives NaN),
  and the restatement's decoder agrees;
* escapes need the 3-word form: sampled statistics of a few samples leave |q| far beyond 2^24, and
  inf / NaN inputs escape too.
"""

import numpy as np
import pytest
import torch

from helpers import smaq_hparams


def _same64(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    na, nb = np.isnan(a), np.isnan(b)
    return bool(np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint64),
                                                          b[~nb].view(np.uint64)))


def _data(kind, n, seed=3):
    rs = np.random.default_rng(seed)
    x = rs.normal(0.5, 3.0, n)
    if kind == "extremes":
        x[::97] = 1e300
        x[5::97] = -1e300
        x[11::331] = np.inf
        x[17::331] = -np.inf
        x[23::541] = np.nan
        x[29::89] = -0.0
        x[31::89] = 5e-324
    elif kind == "outliers":
        x[::50] *= 1e6  # escapes at 6/8 bits
    elif kind == "relu":
        x = np.maximum(x, 0.0)
    return x


CASES = [
    ("default", {}, "normal", False, None),
    ("trunc", {"stochastic_rounding": False}, "normal", False, None),
    ("all_positive", {}, "relu", True, None),
    ("bits_4_8", {"num_bits_main": 4, "num_bits_outlier": 8}, "outliers", False, None),
    ("bits_8_8", {"num_bits_main": 8, "num_bits_outlier": 8}, "outliers", False, None),
    ("both_sides", {"main_std_dev_threshold": -0.5}, "normal", False, None),
    ("range_std", {"use_range_std_dev": True}, "outliers", False, None),
    ("sampled_k16", {"use_sample_stats": True, "num_samples": 16}, "outliers", False, None),
    ("extremes", {}, "extremes", False, None),
    ("bn", {"use_batch_norm": True}, "normal", False, (4, 6, 5)),
]


def _codecs(hp, seed=9, offset=1234):
    from smart_compress_amd.compress import SmartFP, SmartFPPacked

    pk, ref = SmartFPPacked(hp), SmartFP(hp)
    for c in (pk, ref):
        c.rng.seed, c.rng.offset = seed, offset
    return pk, ref


def _cfg(hp):
    from oracle import smaq as osmaq

    return osmaq.SmaqConfig(num_bits_main=hp.num_bits_main, num_bits_outlier=hp.num_bits_outlier,
                            main_std_dev_threshold=hp.main_std_dev_threshold,
                            outlier_std_dev_threshold=hp.outlier_std_dev_threshold,
                            stochastic_rounding=hp.stochastic_rounding,
                            use_range_std_dev=hp.use_range_std_dev, precision=hp.precision)


def _case(name, over, kind, n=70_001):
    hp = smaq_hparams(measure_compression_ratio=False, **over)
    x = _data(kind, n)
    bn = None
    if name == "bn":
        c = 6
        x = x[: 4 * c * 5 * 583].reshape(4, c, 5, 583)
        rs = np.random.default_rng(4)
        bn = (rs.uniform(0.5, 2.0, c), rs.normal(0.0, 0.3, c))
    return hp, x, bn


def _oracle_stream(x, hp, st, seed, offset, all_positive, bn):
    from oracle import smaq as osmaq
    from oracle import smaq_packed as P

    u = osmaq.uniforms_f64(seed, offset, x.size).reshape(x.shape) if hp.stochastic_rounding else None
    return P.pack_f64(x, st["mean"], st["raw_std"], _cfg(hp), u, all_positive, bn)


@pytest.mark.parametrize("name,over,kind,ap,_shape", CASES, ids=[c[0] for c in CASES])
def test_cpu_f64_stream_and_round_trip(name, over, kind, ap, _shape):
    from oracle import smaq_packed as P
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress import SmartFP

    hp, x, bn = _case(name, over, kind)
    pk, ref = _codecs(hp)
    xt = torch.from_numpy(x)
    bnt = tuple(torch.from_numpy(t) for t in bn) if bn is not None else None
    p = pk.compress(xt, ap, bnt)
    assert p.dtype == torch.float64 and p.header()["flags"] & N.SMQ_PACK_FLAG_F64
    st = SmartFP.read_stats_f64(N.cpu_workspace("smaq", 1))
    want = _oracle_stream(x, hp, st, 9, 1234, ap, bn)
    got = p.data.numpy()
    assert got.size == want.size and np.array_equal(got, want)
    y = pk.decompress(p)
    assert y.dtype == torch.float64
    yr = ref(xt, all_positive=ap, batch_norm_stats=bnt)
    assert _same64(y.numpy(), yr.numpy())
    assert _same64(P.unpack(got), yr.numpy().ravel())
    assert pk.rng.offset == ref.rng.offset


def test_cpu_f64_sampled_escapes_beyond_float32():
    """A few samples of a wide tensor: std from 16 values, z of the rest up to ~1e6, |q| far
    beyond 2^24 — kept exactly by the 3-word escapes (a float32 escape word would round them)."""
    from oracle import smaq_packed as P

    hp = smaq_hparams(measure_compression_ratio=False, use_sample_stats=True, num_samples=16)
    x = np.random.default_rng(8).normal(0, 1, 50_000)
    x[::7] *= 1e12
    pk, ref = _codecs(hp)
    p = pk.compress(torch.from_numpy(x))
    _, dirs, _, _ = P.regions(p.data.numpy())
    n_esc = int(sum(int(d) >> 51 for d in dirs))
    assert n_esc > 1000
    y = pk.decompress(p)
    assert _same64(y.numpy(), ref(torch.from_numpy(x)).numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("name,over,kind,ap,_shape", CASES, ids=[c[0] for c in CASES])
def test_gpu_f64_stream_and_round_trip(name, over, kind, ap, _shape):
    from oracle import smaq_packed as P
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress import SmartFP

    hp, x, bn = _case(name, over, kind)
    pk, ref = _codecs(hp)
    xt = torch.from_numpy(x).cuda()
    bnt = tuple(torch.from_numpy(t).cuda() for t in bn) if bn is not None else None
    p = pk.compress(xt, ap, bnt)
    stream = p.compact().data.cpu().numpy()
    ws = N._ws[("smaq_pack_f64", 0, N.stream_ptr(torch.device("cuda")))]
    st = SmartFP.read_stats_f64(ws)
    want = _oracle_stream(x, hp, st, 9, 1234, ap, bn)
    assert stream.size == want.size and np.array_equal(stream, want)
    y = pk.decompress(p)
    torch.cuda.synchronize()
    yr = ref(xt, all_positive=ap, batch_norm_stats=bnt)
    assert y.dtype == torch.float64
    assert _same64(y.cpu().numpy(), yr.cpu().numpy())
    # the host decoder reads the device stream, and the restatement's decoder agrees
    from smart_compress_amd.compress.packed import SmaqPacked

    yh = pk.decompress(SmaqPacked(torch.from_numpy(stream), p.shape, p.n, widths=p.widths,
                                  dtype=torch.float64))
    assert _same64(yh.numpy(), yr.cpu().numpy())
    assert _same64(P.unpack(stream), yr.cpu().numpy().ravel())


@pytest.mark.gpu
def test_gpu_f64_ragged_and_multi_block_sizes():
    """Sizes around the block and group boundaries, and a decoder call with the wrong widths
    (left undecoded)."""
    from smart_compress_amd import _native as N

    hp = smaq_hparams(measure_compression_ratio=False)
    for n in (4096, 4097, 8191, 64 * 4096 + 5, 1_000_003):
        x = torch.from_numpy(_data("outliers", n, seed=n)).cuda()
        pk, ref = _codecs(hp, seed=n, offset=n)
        y = pk.decompress(pk.compress(x))
        assert _same64(y.cpu().numpy(), ref(x).cpu().numpy()), n
    p = pk.compress(x)
    y = torch.full((x.numel(),), 7.0, dtype=torch.float64, device="cuda")
    N.check(N.lib().smq_smaq_decompress_f64(p.data.data_ptr(), y.data_ptr(), x.numel(), 5, 8,
                                            N.stream_ptr(y.device)), "decompress_f64")
    assert bool((y == 7.0).all())
