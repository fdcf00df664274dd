"""Packed SmaQ container on the GPU (smq_smaq_compress / smq_smaq_decompress, SmartFPPacked).

* The device stream equals the oracle's byte for byte (oracle/smaq_packed.py fed the device
  statistics and the same counter RNG): header, directory, every block image, escapes.
* decompress(compress(x)) equals SmartFP(x) bit for bit for the same flags and random stream,
  and equals the oracle's unpack of the same stream.
* Large tensors (16k+ blocks): the round-trip identity, the directory (monotone, consistent with
  each block's size) and sampled blocks' fixed and variable sections vs the oracle.
* Escape-heavy blocks whose variable section outgrows its scratch slot are re-coded by the var
  kernel: same bytes as the oracle.
"""

import numpy as np
import pytest
import torch

from helpers import n_diff_f32, same_f32, smaq_hparams

pytestmark = pytest.mark.gpu


def _codecs(seed=21, offset=3, **over):
    from smart_compress_amd.compress import SmartFP, SmartFPPacked

    hp = smaq_hparams(**over)
    a, b = SmartFPPacked(hp), SmartFP(hp)
    a.rng.seed, a.rng.offset = seed, offset
    b.rng.seed, b.rng.offset = seed, offset
    return hp, a, b


def _stats_of(packed):
    h = packed.header()
    return h["mean"], h["std_dev"]


def _oracle_stream(x_np, packed, hp, seed, offset, all_positive=False, dtype="f32"):
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from oracle import smaq_packed as P

    h = packed.header()
    cfg = osmaq.SmaqConfig(num_bits_main=hp.num_bits_main, num_bits_outlier=hp.num_bits_outlier,
                           main_std_dev_threshold=hp.main_std_dev_threshold,
                           outlier_std_dev_threshold=hp.outlier_std_dev_threshold,
                           stochastic_rounding=hp.stochastic_rounding, precision=hp.precision)
    u = orng.uniforms(seed, offset, x_np.size) if hp.stochastic_rounding else None
    # header.std_dev is after the ==0 rule; the codes only depend on it through std_clamped
    return P.pack(x_np, h["mean"], h["std_dev"], cfg, u, all_positive, dtype), cfg, u


def _heavy(n, seed):
    rs = np.random.default_rng(seed)
    x = (rs.standard_t(2.0, n) * 1.3 + 0.1).astype(np.float32)
    x[rs.random(n) < 0.001] = np.nan
    x[rs.random(n) < 0.001] = np.inf
    x[rs.random(n) < 0.001] = -np.inf
    return x


@pytest.mark.parametrize("n", [8, 1000, 4095, 4096, 4097, 1 << 16, 1000003])
@pytest.mark.parametrize("sr", [True, False])
def test_stream_bytes_and_roundtrip(n, sr):
    hp, pk, ref = _codecs(stochastic_rounding=sr)
    gen = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(n, generator=gen, device="cuda") * 2.0 + 0.5
    packed = pk.compress(x)
    y = pk.decompress(packed)
    y_ref = ref(x)
    torch.cuda.synchronize()
    assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy())
    stream, _, _ = _oracle_stream(x.cpu().numpy(), packed, hp, 21, 3)
    got = packed.compact().data.cpu().numpy()
    assert got.size == stream.size, (got.size, stream.size)
    assert np.array_equal(got, stream), int(np.argmax(got != stream))
    assert packed.bits_per_element < 8.0 or n < (1 << 16)  # per-block header amortised


@pytest.mark.parametrize("bits", [(6, 8), (4, 6), (2, 3), (5, 7), (9, 12)])
def test_escapes_bits_and_all_positive(bits):
    from oracle import smaq_packed as P

    hp, pk, ref = _codecs(num_bits_main=bits[0], num_bits_outlier=bits[1])
    x_np = _heavy(50_000, bits[0])
    x = torch.from_numpy(x_np).cuda()
    for all_pos in (False, True):
        packed = pk.compress(x, all_positive=all_pos)
        y = pk.decompress(packed)
        y_ref = ref(x, all_positive=all_pos)
        torch.cuda.synchronize()
        assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy()), n_diff_f32(
            y.cpu().numpy(), y_ref.cpu().numpy())
        got = packed.compact().data.cpu().numpy()
        assert P.header(got)["n"] == x_np.size
        assert same_f32(P.unpack(got), y.cpu().numpy())  # the oracle decodes the device stream


@pytest.mark.parametrize("dt", ["f16", "bf16"])
def test_half_inputs(dt):
    tdt = {"f16": torch.float16, "bf16": torch.bfloat16}[dt]
    hp, pk, ref = _codecs(precision=16)
    gen = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.randn(70_001, generator=gen, device="cuda") * 3).to(tdt)
    packed = pk.compress(x)
    y = pk.decompress(packed)
    y_ref = ref(x)
    torch.cuda.synchronize()
    assert y.dtype == torch.float32 and same_f32(y.cpu().numpy(), y_ref.cpu().numpy())
    stream, _, _ = _oracle_stream(x.float().cpu().numpy(), packed, hp, 21, 3, dtype=dt)
    assert np.array_equal(packed.compact().data.cpu().numpy(), stream)


def test_sampled_and_range_stats():
    for over in (dict(use_sample_stats=True), dict(use_range_std_dev=True),
                 dict(use_sample_stats=True, use_range_std_dev=True)):
        hp, pk, ref = _codecs(**over)
        x = torch.randn(123_457, device="cuda") * 0.3
        packed = pk.compress(x)
        y = pk.decompress(packed)
        y_ref = ref(x)
        torch.cuda.synchronize()
        assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy()), over


def test_codec_call_logs_real_size_and_passthrough():
    from argparse import Namespace

    hp, pk, ref = _codecs(measure_compression_ratio=True)
    logged = []
    pk.log = lambda k, v, **kw: logged.append((k, v))
    x = torch.randn(1 << 18, device="cuda")
    y = pk(x, tag="forward_autograd")
    ref.log = lambda k, v, **kw: None
    y_ref = ref(x, tag="forward_autograd")  # (the reference's log_size needs a tag, base.py:101)
    assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy())
    d = dict(logged)
    assert d["orig_size"] == 32 * x.numel()
    assert 6.0 * x.numel() < d["new_size"] < 8.0 * x.numel()  # real stream bits
    small = torch.randn(5, device="cuda")
    assert pk(small, tag="forward_autograd") is small  # smart.py:123-128
    p = pk.compress(small)
    assert p.raw and torch.equal(pk.decompress(p), small)


def test_rejections():
    from smart_compress_amd.compress import SmartFPPacked

    with pytest.raises(NotImplementedError):
        SmartFPPacked(smaq_hparams(main_std_dev_threshold=float("nan"))).compress(
            torch.randn(100, device="cuda"))
    with pytest.raises(RuntimeError):  # the BN variant needs NCHW (smart.py:145 permutes 4 dims)
        SmartFPPacked(smaq_hparams(use_batch_norm=True)).compress(
            torch.randn(2, 3, 16, device="cuda"),
            batch_norm_stats=(torch.ones(3, device="cuda"), torch.zeros(3, device="cuda")))


def _bn_stream_vs_oracle(x, packed, hp, seed, offset, bn, all_positive):
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from oracle import smaq_packed as P

    h = packed.header()
    cfg = osmaq.SmaqConfig(num_bits_main=hp.num_bits_main, num_bits_outlier=hp.num_bits_outlier,
                           main_std_dev_threshold=hp.main_std_dev_threshold,
                           outlier_std_dev_threshold=hp.outlier_std_dev_threshold,
                           stochastic_rounding=hp.stochastic_rounding, precision=hp.precision)
    u = orng.uniforms(seed, offset, x.numel()) if hp.stochastic_rounding else None
    x_np = x.float().cpu().numpy()
    bn_np = None if bn is None else tuple(t.float().cpu().numpy() for t in bn)
    dt = {torch.float32: "f32", torch.float16: "f16", torch.bfloat16: "bf16"}[x.dtype]
    return P.pack(x_np, h["mean"], h["std_dev"], cfg, u, all_positive, dt, bn_np)


@pytest.mark.parametrize("thr", [-0.5, -1.25, -3.0])
@pytest.mark.parametrize("bits", [(6, 8), (4, 6), (9, 12)])
@pytest.mark.parametrize("sr", [True, False])
def test_negative_threshold(thr, bits, sr):
    """main_std_dev_threshold < 0 (smart.py:157-161): elements above -T and below T at once are the
    third state (mask 0, main code, both sides in the decoder): round trip == SmartFP, stream ==
    the oracle's (whose unpack is pinned to the reference's thr_neg goldens)."""
    from oracle import smaq_packed as P

    hp, pk, ref = _codecs(seed=9, offset=4, main_std_dev_threshold=thr, num_bits_main=bits[0],
                          num_bits_outlier=bits[1], stochastic_rounding=sr)
    gen = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(3 * 4096 + 555, generator=gen, device="cuda") * 1.5 + 0.2
    packed = pk.compress(x)
    y = pk.decompress(packed)
    y_ref = ref(x)
    torch.cuda.synchronize()
    assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy()), n_diff_f32(y.cpu().numpy(),
                                                                      y_ref.cpu().numpy())
    raw = packed.compact().data.cpu().numpy()
    assert P.header(raw)["flags"] & P.FLAG_BOTH_SIDES
    assert np.array_equal(raw, _bn_stream_vs_oracle(x, packed, hp, 9, 4, None, False))


@pytest.mark.parametrize("shape", [(2, 8, 6, 5), (4, 64, 32, 32), (50, 1000, 1, 1), (3, 17, 7, 7),
                                   (1, 3, 100, 100)])
@pytest.mark.parametrize("bits", [(6, 8), (4, 6)])
def test_batch_norm_variant(shape, bits):
    """The BN variant (smart.py:136-149, 174-179): per-channel (x - beta) / gamma before the
    z-score, * gamma + beta after; the stream carries the parameters (decompress needs none).
    Channel runs shorter than, equal to and longer than a block (inner 1, 25, 49, 1024, 10000),
    the default widths (decode table) and others; all_positive after the BN term; scalar
    parameters; a negative threshold on top. Round trip == SmartFP, stream == the oracle's."""
    from oracle import smaq_packed as P

    C = shape[1]
    gen = torch.Generator(device="cuda").manual_seed(C)
    x = torch.randn(shape, generator=gen, device="cuda") * 2.0 + 0.3
    gam = torch.rand(C, generator=gen, device="cuda") + 0.5
    bet = torch.randn(C, generator=gen, device="cuda") * 0.1
    for over, allpos in ((dict(), False), (dict(), True), (dict(bn_scalar_params=True), False),
                         (dict(main_std_dev_threshold=-0.5), True),
                         (dict(stochastic_rounding=False), False)):
        hp, pk, ref = _codecs(seed=5, offset=2, use_batch_norm=True, num_bits_main=bits[0],
                              num_bits_outlier=bits[1], **over)
        packed = pk.compress(x, all_positive=allpos, batch_norm_stats=(gam, bet))
        y = pk.decompress(packed)
        y_ref = ref(x, all_positive=allpos, batch_norm_stats=(gam, bet))
        torch.cuda.synchronize()
        assert y.shape == x.shape
        assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy()), (over, allpos, n_diff_f32(
            y.cpu().numpy(), y_ref.cpu().numpy()))
        raw = packed.compact().data.cpu().numpy()
        h = P.header(raw)
        assert h["flags"] & P.FLAG_BN and h["bn_inner"] == shape[2] * shape[3]
        bn = (gam.mean().reshape(1), bet.mean().reshape(1)) if over.get("bn_scalar_params") \
            else (gam, bet)
        assert h["bn_channels"] == bn[0].numel()
        assert np.array_equal(raw, _bn_stream_vs_oracle(x, packed, hp, 5, 2, bn, allpos)), over
        if x.numel() <= 1 << 16:
            assert same_f32(P.unpack(raw).reshape(shape), y.cpu().numpy())


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_batch_norm_half_inputs(dt):
    """Half inputs with fp32 BN parameters: the data are promoted to fp32 (z-score in fp32)."""
    hp, pk, ref = _codecs(seed=3, offset=0, use_batch_norm=True, precision=16)
    gen = torch.Generator(device="cuda").manual_seed(4)
    x = (torch.randn(4, 16, 12, 12, generator=gen, device="cuda") * 3).to(dt)
    gam = torch.rand(16, generator=gen, device="cuda") + 0.5
    bet = torch.randn(16, generator=gen, device="cuda") * 0.1
    packed = pk.compress(x, batch_norm_stats=(gam, bet))
    y = pk.decompress(packed)
    y_ref = ref(x, batch_norm_stats=(gam, bet))
    torch.cuda.synchronize()
    assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy())
    assert np.array_equal(packed.compact().data.cpu().numpy(),
                          _bn_stream_vs_oracle(x, packed, hp, 3, 0, (gam, bet), False))


def test_large_multiblock():
    """64M elements = 16384 blocks: round trip == SmartFP, the directory matches each block's
    variable-section size, sampled blocks' fixed and variable sections equal the oracle's."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from oracle import smaq_packed as P

    n = 1 << 26
    hp, pk, ref = _codecs(seed=77, offset=1000)
    gen = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(n, generator=gen, device="cuda")
    x[::997] *= 40.0  # escapes sprinkled over every block
    packed = pk.compress(x)
    y = pk.decompress(packed)
    y_ref = ref(x)
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.int32), y_ref.view(torch.int32))
    del y, y_ref
    raw = packed.compact().data.cpu().numpy()
    h, dirs, fixed_w, var_w = P.regions(raw)
    nb = h["n_blocks"]
    assert nb == n // 4096 and h["error"] == 0 and h["total_bytes"] == raw.size
    assert h["version"] == 2 and var_w.size == h["data_words"]
    off = (dirs & np.uint64((1 << 38) - 1)).astype(np.int64)
    n_out = ((dirs >> np.uint64(38)) & np.uint64(0x1FFF)).astype(np.int64)
    n_esc = (dirs >> np.uint64(51)).astype(np.int64)
    size = (2 * n_out + 31) // 32 + 2 * n_esc
    assert off[0] == 0 and np.array_equal(np.diff(off), size[:-1])
    assert off[-1] + size[-1] == h["data_words"]
    assert n_esc.sum() > nb  # escapes present throughout
    F = P.fixed_words(5)
    mask_pop = np.unpackbits(fixed_w.reshape(nb, F)[:, :128].view(np.uint8), axis=1).sum(axis=1)
    assert np.array_equal(mask_pop, n_out)
    cfg = osmaq.SmaqConfig()
    xh = x.cpu().numpy()
    for b in (0, 1, 2, nb // 2, nb - 2, nb - 1):
        s = slice(b * 4096, (b + 1) * 4096)
        u = orng.uniforms(77, 1000 + b * 4096, 4096)
        fx, vr = P.pack_block(xh[s], h["mean"], h["std_dev"], cfg, u)
        assert np.array_equal(fixed_w[b * F:(b + 1) * F], fx), b
        assert np.array_equal(var_w[off[b]: off[b] + vr.size], vr), b


def test_compress_is_repeatable():
    """Same seed/offset twice on one workspace: identical streams."""
    hp, pk, _ = _codecs(seed=4, offset=0)
    x = torch.randn(3 * 4096 + 77, device="cuda")
    a = pk.compress(x).compact().data.clone()
    pk.rng.offset = 0
    b = pk.compress(x).compact().data
    assert torch.equal(a, b)


def _compress_raw(x, pk, flags, p, ws=None):
    """smq_smaq_compress_ex with explicit flags and params into a fresh buffer; returns the
    stream bytes."""
    from smart_compress_amd import _native as N

    lib = N.lib()
    n = x.numel()
    code = N.DTYPE_CODES[x.dtype]
    bound = lib.smq_smaq_pack_bound(n, pk.hparams.num_bits_main, pk.hparams.num_bits_outlier)
    if ws is None:
        ws = N.workspace("smaq_pack", x.device, lib.smq_smaq_pack_workspace_bytes(n))
    out = torch.zeros(bound, dtype=torch.uint8, device=x.device)
    N.check(lib.smq_smaq_compress_ex(x.data_ptr(), code, n, p, out.data_ptr(), out.numel(),
                                     ws.data_ptr(), ws.numel(), flags, N.stream_ptr(x.device)),
            "compress_ex")
    torch.cuda.synchronize()
    raw = out.cpu().numpy()
    to = N.SmqPackedHeader.total_bytes.offset
    eo = N.SmqPackedHeader.error.offset
    assert int(raw[eo:eo + 4].view(np.uint32)[0]) == 0
    return raw[:int(raw[to:to + 8].view(np.uint64)[0])]


def _oracle_of(raw, x, hp, seed, offset, dtype="f32"):
    from oracle import smaq_packed as P

    h = P.header(raw)
    packed = type("P", (), {"header": lambda self: h})()
    stream, _, _ = _oracle_stream(x.float().cpu().numpy(), packed, hp, seed, offset, dtype=dtype)
    return stream


@pytest.mark.parametrize("n", [8, 4095, 4096, 4097, 3 * 4096 + 77, (1 << 20) + 5])
@pytest.mark.parametrize("bits", [(6, 8), (4, 6), (9, 12), (15, 15), (16, 18), (3, 21), (10, 5)])
def test_packer_widths_escapes_and_flags(n, bits):
    """Heavy-tailed input (NaN, +-inf, |q| far beyond any budget) at widths from 2 to 20 bits
    (wo - wm from -5 to 18): the stream equals the oracle's byte for byte; the legacy flags
    (SMQ_PACK_SINGLE / TICKETED) give the same bytes; a second call on the same workspace too."""
    from smart_compress_amd import _native as N

    hp, pk, _ = _codecs(seed=3, offset=11, num_bits_main=bits[0], num_bits_outlier=bits[1])
    x_np = _heavy(n, n % 97)
    rs = np.random.default_rng(n)
    x_np[rs.random(n) < 0.002] *= 1e6
    x = torch.from_numpy(x_np).cuda()
    p = pk._params(n, False, x.dtype, x.device)
    a = _compress_raw(x, pk, 0, p)
    assert np.array_equal(a, _oracle_of(a, x, hp, 3, 11))
    for flags in (N.SMQ_PACK_SINGLE, N.SMQ_PACK_TICKETED, 0):
        assert np.array_equal(a, _compress_raw(x, pk, flags, p))


@pytest.mark.parametrize("frac", [0.2, 0.6, 1.0])
def test_escape_heavy_blocks_recoded(frac):
    """Blocks with more escapes than their 3 KiB scratch slot holds (> ~380 at 6/8 bits) are
    re-coded from x by the var kernel: mixed with ordinary blocks, the stream equals the oracle's
    and decodes to SmartFP's output."""
    hp, pk, ref = _codecs(seed=12, offset=7)
    n = 9 * 4096 + 333
    rs = np.random.default_rng(int(frac * 10))
    x_np = rs.standard_normal(n).astype(np.float32)
    for b in (1, 4, 8, 9):  # escape-heavy blocks (incl. the short last one)
        s = slice(b * 4096, min(n, (b + 1) * 4096))
        sel = rs.random(x_np[s].size) < frac
        x_np[s][sel] *= 1e4
    x = torch.from_numpy(x_np).cuda()
    p = pk._params(n, False, x.dtype, x.device)
    a = _compress_raw(x, pk, 0, p)
    assert np.array_equal(a, _oracle_of(a, x, hp, 12, 7))
    pk.rng.offset = 7  # (_params advanced it)
    packed = pk.compress(x)
    y = pk.decompress(packed)
    y_ref = ref(x)
    torch.cuda.synchronize()
    assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy())


@pytest.mark.parametrize("dt", ["f32", "f16", "bf16"])
def test_packer_unaligned_and_half(dt):
    """Element-path (misaligned x) and half inputs == the oracle."""
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[dt]
    hp, pk, _ = _codecs(seed=8, offset=0, precision=16 if dt != "f32" else 32)
    gen = torch.Generator(device="cuda").manual_seed(2)
    base = (torch.randn(3 * 4096 + 1000, generator=gen, device="cuda") * 2).to(tdt)
    x = base[1:]  # misaligned by one element
    assert x.data_ptr() % 16 != 0
    got = _compress_raw(x, pk, 0, pk._params(x.numel(), False, x.dtype, x.device))
    assert np.array_equal(got, _oracle_of(got, x, hp, 8, 0, dtype=dt))


@pytest.mark.parametrize("scale", [1e8, 3.0e-3])
def test_packer_quot_check_paths(scale):
    """std >= 2^24 makes the statistics ask for the per-element subnormal-quotient check
    (quot_check_for): the checked body gives the oracle's bytes; a small scale exercises the
    unchecked body."""
    hp, pk, _ = _codecs(seed=6, offset=2)
    n = 5 * 4096 + 123
    gen = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(n, generator=gen, device="cuda") * scale
    a = _compress_raw(x, pk, 0, pk._params(n, False, x.dtype, x.device))
    assert np.array_equal(a, _oracle_of(a, x, hp, 6, 2))


def test_decompress_with_and_without_caller_widths():
    """smq_smaq_decompress (widths from the stream header) and smq_smaq_decompress_ex (the
    caller's widths: no header wait) decode the same bytes; _ex with widths the stream was not
    written with leaves y untouched."""
    from smart_compress_amd import _native as N

    hp, pk, _ = _codecs(seed=31, offset=0, num_bits_main=4, num_bits_outlier=6)
    n = 7 * 4096 + 19
    x = torch.randn(n, device="cuda") * 2
    packed = pk.compress(x)
    lib = N.lib()
    st = N.stream_ptr(x.device)
    a = torch.full((n,), 7.0, device="cuda")
    b = torch.full((n,), 7.0, device="cuda")
    c = torch.full((n,), 7.0, device="cuda")
    N.check(lib.smq_smaq_decompress(packed.data.data_ptr(), a.data_ptr(), n, st), "dec")
    N.check(lib.smq_smaq_decompress_ex(packed.data.data_ptr(), b.data_ptr(), n, 4, 6, st), "dex")
    N.check(lib.smq_smaq_decompress_ex(packed.data.data_ptr(), c.data_ptr(), n, 6, 8, st), "dex2")
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    assert not torch.equal(a, torch.full_like(a, 7.0))
    assert torch.equal(c, torch.full_like(c, 7.0))


def test_decompress_wrong_n_leaves_y_untouched():
    """A caller's n larger than the stream's (a right-sized buffer, so the stream's directory and
    fixed region end well before the caller's n would reach): the decoder checks the header's magic
    and n before it reads any directory entry or section, leaves y alone and does not fault."""
    from smart_compress_amd import _native as N

    hp, pk, _ = _codecs(seed=5, offset=0)
    n = 7 * 4096 + 19
    packed = pk.compress(torch.randn(n, device="cuda")).compact()
    lib = N.lib()
    st = N.stream_ptr(packed.data.device)
    for n2 in (n + 1, 64 * 4096, 1 << 22):
        for ex in (False, True):
            y = torch.full((n2,), 7.0, device="cuda")
            if ex:
                N.check(lib.smq_smaq_decompress_ex(packed.data.data_ptr(), y.data_ptr(), n2, 6, 8,
                                                   st), "dex")
            else:
                N.check(lib.smq_smaq_decompress(packed.data.data_ptr(), y.data_ptr(), n2, st), "dec")
            torch.cuda.synchronize()
            assert torch.equal(y, torch.full_like(y, 7.0)), (n2, ex)


def test_stream_from_elsewhere_decodes_with_header_widths():
    """A SmaqPacked without recorded widths (a stream received from elsewhere) is decoded with the
    widths its header records, whatever the decoding codec's own flags."""
    from smart_compress_amd.compress.packed import SmaqPacked

    hp, pk, single = _codecs(seed=9, offset=0, num_bits_main=4, num_bits_outlier=6)
    x = torch.randn(5 * 4096 + 3, device="cuda")
    packed = pk.compress(x).compact()
    want = pk.decompress(packed)
    _, other, _ = _codecs(seed=1, offset=0)  # 6/8 bits
    got = other.decompress(SmaqPacked(packed.data, packed.shape, packed.n))
    assert torch.equal(got.view(torch.int32), want.view(torch.int32))


def test_compress_decompress_in_a_captured_graph():
    """compress + decompress never synchronise the host: the pair is captured into a hipGraph
    (graph-safe random stream) and two replays equal two eager round trips of SmartFP at the same
    stream positions, bit for bit; the stream size is read only when asked (nbytes)."""
    from smart_compress_amd.compress.packed import SmartFPPacked
    from smart_compress_amd.compress.smart import SmartFP

    hp = smaq_hparams()
    x = torch.randn(9 * 4096 + 5, device="cuda")
    eager = SmartFP(hp)
    eager.rng.seed, eager.rng.offset = 44, 0
    want = [eager(x).clone() for _ in range(2)]
    pk = SmartFPPacked(hp)
    pk.rng.seed, pk.rng.offset = 44, 0
    pk.graph_safe(True, device="cuda")
    pk.decompress(pk.compress(x))  # eager call: workspaces and the device counter exist
    torch.cuda.synchronize()
    pk.rng.load_state_dict({"seed": 44, "offset": 0})
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        packed = pk.compress(x)
        y = pk.decompress(packed)
    for r in range(2):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y.view(torch.int32), want[r].view(torch.int32)), r
    assert 0 < packed.nbytes < 4 * x.numel()
    pk.graph_safe(False)


@pytest.mark.parametrize("k", [5000, 100_000])
def test_sampled_above_4096_device_draw(k):
    """smart.py:86-91 with more samples than one workgroup draws: the multi-workgroup draw in the
    packer's workspace (smq_smaq_pack_workspace_bytes_sampled); the round trip equals SmartFP."""
    hp, pk, ref = _codecs(use_sample_stats=True, num_samples=k)
    x = torch.randn(1_000_003, device="cuda") * 0.7 + 0.2
    for _ in range(2):  # consecutive calls: fresh draws, same stream positions
        y = pk.decompress(pk.compress(x))
        y_ref = ref(x)
        torch.cuda.synchronize()
        assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy())
    assert pk.rng.offset == ref.rng.offset


def _golden_packable():
    from helpers import smaq_cases

    cases = smaq_cases()
    return sorted(k for k, m in cases.items()
                  if not k.startswith("n7") and not m.get("use_sample_stats"))


@pytest.mark.parametrize("name", _golden_packable())
def test_device_stream_equals_host_stream(name):
    """The host packer (smq_cpu_smaq_compress) and the device packer write the same bytes for the
    same input and random stream whenever their statistics agree (fp64 sums in two fixed orders:
    equal but for rare last-bit cases, where the header tells); either library decodes the other's
    stream to the same values."""
    from helpers import load_smaq, smaq_cases

    from smart_compress_amd.compress import SmartFPPacked

    meta, d = smaq_cases()[name], load_smaq(name)
    hp = smaq_hparams(meta, measure_compression_ratio=False)
    dt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[meta["dtype"]]
    x = torch.from_numpy(np.ascontiguousarray(d["x"])).to(dt)
    bn = None
    if "bn_gamma" in d:
        hp.use_batch_norm = True
        bn = (torch.from_numpy(d["bn_gamma"]), torch.from_numpy(d["bn_beta"]))
        if meta["bn_scalar_params"]:  # (averaged once: a device mean may round differently)
            bn = tuple(t.mean().reshape(1) for t in bn)
    streams = []
    for dev in ("cpu", "cuda"):
        pk = SmartFPPacked(hp)
        pk.rng.seed, pk.rng.offset = 13, 5
        xb = x.to(dev)
        bnb = None if bn is None else tuple(t.to(dev) for t in bn)
        streams.append(pk.compress(xb, meta["all_positive"], bnb).compact())
    hc, hd = streams[0].header(), streams[1].header()
    if (hc["mean"], hc["std_dev"]) == (hd["mean"], hd["std_dev"]):
        assert np.array_equal(streams[0].data.numpy(), streams[1].data.cpu().numpy())
    else:  # (rare) statistics a last bit apart: both within one ulp
        for k in ("mean", "std_dev"):
            assert abs(int(np.float32(hc[k]).view(np.int32)) -
                       int(np.float32(hd[k]).view(np.int32))) <= 1
    pk = SmartFPPacked(hp)
    for s in streams:  # each stream decoded on the other side equals its own decode
        other = type(s)(s.data.cuda() if not s.data.is_cuda else s.data.cpu(), s.shape, s.n,
                        widths=s.widths, total=s.nbytes)
        a, b = pk.decompress(s), pk.decompress(other)
        torch.cuda.synchronize()
        assert same_f32(a.cpu().numpy(), b.cpu().numpy())
