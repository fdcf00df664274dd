"""Packed SmaQ container on the GPU (smq_smaq_compress / smq_smaq_decompress, SmartFPPacked).

* The device stream equals the oracle's byte for byte (oracle/smaq_packed.py fed the device
  statistics and the same counter RNG): header, directory, every block image, escapes.
* decompress(compress(x)) equals SmartFP(x) bit for bit for the same flags and random stream,
  and equals the oracle's unpack of the same stream.
* Large tensors (16k+ blocks, the decoupled look-back under load): the round-trip identity, the
  directory (monotone, consistent with each block's size) and sampled block images vs the oracle.
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
    got = packed.data.cpu().numpy()
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
        got = packed.data.cpu().numpy()
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
    assert np.array_equal(packed.data.cpu().numpy(), stream)


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
        SmartFPPacked(smaq_hparams(main_std_dev_threshold=-1.0)).compress(
            torch.randn(100, device="cuda"))
    with pytest.raises(NotImplementedError):
        SmartFPPacked(smaq_hparams(use_batch_norm=True)).compress(
            torch.randn(2, 3, 4, 4, device="cuda"),
            batch_norm_stats=(torch.ones(3, device="cuda"), torch.zeros(3, device="cuda")))


def test_large_multiblock_lookback():
    """64M elements = 16384 blocks compacted by the look-back scan: round trip == SmartFP, the
    directory matches each block's size, sampled block images equal the oracle's."""
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
    raw = packed.data.cpu().numpy()
    h = P.header(raw)
    nb = h["n_blocks"]
    assert nb == n // 4096 and h["error"] == 0 and h["total_bytes"] == raw.size
    dent = raw[128: 128 + 8 * nb].view(np.uint64)
    dirs = (dent & np.uint64((1 << 38) - 1)).astype(np.int64)
    data = raw[128 + 8 * nb:].view(np.uint32)
    w0 = data[dirs]
    n_out, n_esc = (w0 & 0xFFFF).astype(np.int64), (w0 >> 16).astype(np.int64)
    assert np.array_equal((dent >> np.uint64(38)) & np.uint64(0x1FFF), n_out.astype(np.uint64))
    assert np.array_equal(dent >> np.uint64(51), n_esc.astype(np.uint64))
    size = 129 + (5 * 4096 + 2 * n_out + 31) // 32 + 2 * n_esc
    assert dirs[0] == 0 and np.array_equal(np.diff(dirs), size[:-1])
    assert dirs[-1] + size[-1] == h["data_words"]
    assert n_esc.sum() > nb  # escapes present throughout
    cfg = osmaq.SmaqConfig()
    xh = x.cpu().numpy()
    for b in (0, 1, 2, nb // 2, nb - 2, nb - 1):
        s = slice(b * 4096, (b + 1) * 4096)
        u = orng.uniforms(77, 1000 + b * 4096, 4096)
        img = P.pack_block(xh[s], h["mean"], h["std_dev"], cfg, u)
        got = data[dirs[b]: dirs[b] + img.size]
        assert np.array_equal(got, img), b


def test_compress_is_repeatable():
    """Same seed/offset twice (workspace counters reset by the last block): identical streams."""
    hp, pk, _ = _codecs(seed=4, offset=0)
    x = torch.randn(3 * 4096 + 77, device="cuda")
    a = pk.compress(x).data.clone()
    pk.rng.offset = 0
    b = pk.compress(x).data
    assert torch.equal(a, b)


@pytest.mark.parametrize("n", [4096, 3 * 4096 + 77, (1 << 22) + 5])
def test_ticketed_and_index_order_give_the_same_bytes(n):
    """smq_smaq_compress_ex: index-ordered block ids (default) and SMQ_PACK_TICKETED ids place
    block b after blocks 0..b-1 either way: byte-identical streams (twice each: the ticket counter
    resets itself)."""
    from smart_compress_amd import _native as N

    hp, pk, _ = _codecs(seed=9, offset=5)
    gen = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(n, generator=gen, device="cuda")
    x[::501] *= 30.0
    lib = N.lib()
    p = pk._params(n, False, x.dtype, x.device)
    bound = lib.smq_smaq_pack_bound(n, hp.num_bits_main, hp.num_bits_outlier)
    ws = torch.zeros(lib.smq_smaq_pack_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    outs = []
    for flags in (0, N.SMQ_PACK_TICKETED, N.SMQ_PACK_TICKETED, 0, N.SMQ_PACK_SINGLE):
        out = torch.zeros(bound, dtype=torch.uint8, device="cuda")
        N.check(lib.smq_smaq_compress_ex(x.data_ptr(), N.SMQ_DTYPE_F32, n, p, out.data_ptr(),
                                         out.numel(), ws.data_ptr(), ws.numel(), flags,
                                         N.stream_ptr(x.device)), "compress_ex")
        outs.append(out)
    torch.cuda.synchronize()
    to, eo = N.SmqPackedHeader.total_bytes.offset, N.SmqPackedHeader.error.offset
    total = int(outs[0][to:to + 8].cpu().numpy().view(np.uint64)[0])
    assert int(outs[0][eo:eo + 4].cpu().numpy().view(np.uint32)[0]) == 0
    assert total > 128
    for o in outs[1:]:
        assert torch.equal(o[:total], outs[0][:total])


def _compress_raw(x, pk, flags, p):
    """smq_smaq_compress_ex with explicit flags and params into a fresh buffer; returns the
    stream bytes."""
    from smart_compress_amd import _native as N

    lib = N.lib()
    n = x.numel()
    code = N.DTYPE_CODES[x.dtype]
    bound = lib.smq_smaq_pack_bound(n, pk.hparams.num_bits_main, pk.hparams.num_bits_outlier)
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


@pytest.mark.parametrize("n", [8, 4095, 4096, 4097, 3 * 4096 + 77, (1 << 20) + 5])
@pytest.mark.parametrize("bits", [(6, 8), (4, 6), (9, 12), (15, 15), (16, 18)])
def test_streaming_packer_equals_single_launch(n, bits):
    """Default (streaming: code records -> group scan -> block images) and SMQ_PACK_SINGLE (one
    look-back launch) give the same bytes, incl. escapes whose q does not fit a record (|q| > 4095,
    inf, NaN: re-derived from x), widths beyond the 14-bit records (both take the single launch),
    and repeated calls on one workspace."""
    from smart_compress_amd import _native as N

    hp, pk, _ = _codecs(seed=3, offset=11, num_bits_main=bits[0], num_bits_outlier=bits[1])
    x_np = _heavy(n, n % 97)
    rs = np.random.default_rng(n)
    x_np[rs.random(n) < 0.002] *= 1e6  # |q| far beyond 4095
    x = torch.from_numpy(x_np).cuda()
    p = pk._params(n, False, x.dtype, x.device)
    a = _compress_raw(x, pk, 0, p)
    b = _compress_raw(x, pk, N.SMQ_PACK_SINGLE, p)
    c = _compress_raw(x, pk, 0, p)
    m = min(a.size, b.size)
    assert a.size == b.size and np.array_equal(a, b), (a.size, b.size, int(np.argmax(a[:m] != b[:m])))
    assert np.array_equal(a, c)


@pytest.mark.parametrize("dt", ["f32", "f16", "bf16"])
def test_streaming_packer_unaligned_and_half(dt):
    """Element-path (misaligned x) and half inputs through the streaming packer == the oracle."""
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[dt]
    hp, pk, _ = _codecs(seed=8, offset=0, precision=16 if dt != "f32" else 32)
    gen = torch.Generator(device="cuda").manual_seed(2)
    base = (torch.randn(3 * 4096 + 1000, generator=gen, device="cuda") * 2).to(tdt)
    x = base[1:]  # misaligned by one element
    assert x.data_ptr() % 16 != 0
    got = _compress_raw(x, pk, 0, pk._params(x.numel(), False, x.dtype, x.device))
    from oracle import smaq_packed as P

    h = P.header(got)
    packed = type("P", (), {"header": lambda self: h})()
    stream, _, _ = _oracle_stream(x.float().cpu().numpy(), packed, hp, 8, 0, dtype=dt)
    assert np.array_equal(got, stream)


@pytest.mark.parametrize("scale", [1e8, 3.0e-3])
def test_streaming_packer_quot_check_paths(scale):
    """std >= 2^24 makes the statistics ask for the per-element subnormal-quotient check
    (quot_check_for): the streaming packer's checked body gives the oracle's bytes and the same
    bytes as the single launch; a small scale exercises the unchecked body."""
    from smart_compress_amd import _native as N

    hp, pk, _ = _codecs(seed=6, offset=2)
    n = 5 * 4096 + 123
    gen = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(n, generator=gen, device="cuda") * scale
    p = pk._params(n, False, x.dtype, x.device)
    a = _compress_raw(x, pk, 0, p)
    b = _compress_raw(x, pk, N.SMQ_PACK_SINGLE, p)
    assert np.array_equal(a, b)
    from oracle import smaq_packed as P

    h = P.header(a)
    packed = type("P", (), {"header": lambda self: h})()
    stream, _, _ = _oracle_stream(x.cpu().numpy(), packed, hp, 6, 2)
    assert np.array_equal(a, stream)
