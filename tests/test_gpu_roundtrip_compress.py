"""smq_smaq_roundtrip_compress / SmartFPPacked.roundtrip_compress on the GPU: y and the stream of one
call from one statistics pass.

* y equals SmartFP(x) bit for bit (same flags, seed and stream position) and the stream equals
  SmartFPPacked.compress(x)'s byte for byte — on the single-launch sizes (V = 1..8 groups per lane,
  one workgroup, ragged tails) and the two-launch sizes above 8,388,611 elements, for fp32 and
  half inputs, all_positive, the BN variant and sampled statistics;
* decompress(stream) == y, and the random stream advances once per call (a second call equals the
  second SmartFP call);
* a buffer below the bound: the stream is written when it fits (bytes equal), and when it does not
  the header's total_bytes exceeds the buffer and nothing is written past it.
Reference: smart.py:110-190 (y), smart.py:184-188 / README.md:25-28 (the codes kept).
"""


import ctypes

import numpy as np
import pytest
import torch

from helpers import same_f32, smaq_hparams

pytestmark = pytest.mark.gpu


def _codecs(seed=7, offset=11, **over):
    from smart_compress_amd.compress import SmartFP, SmartFPPacked

    hp = smaq_hparams(**over)
    a, b, c = SmartFPPacked(hp), SmartFP(hp), SmartFPPacked(hp)
    for k in (a, b, c):
        k.rng.seed, k.rng.offset = seed, offset
    return hp, a, b, c


def _stream(p):
    return p.data[:p.nbytes].cpu().numpy()


SIZES = [5, 1000, 4097, 70_000, 1 << 20, 1_500_000, 2_500_001, 4 << 20, 6_500_000, 7 << 20,
         8_388_608, 8_388_611, 9_000_003]


@pytest.mark.parametrize("n", SIZES)
def test_y_and_stream_equal_the_separate_calls(n):
    hp, rc, ref, pk = _codecs()
    gen = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(n, generator=gen, device="cuda") * 1.7 - 0.3
    y, p = rc.roundtrip_compress(x)
    y_ref = ref(x)
    q = pk.compress(x)
    y_dec = rc.decompress(p)
    torch.cuda.synchronize()
    assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy())
    assert same_f32(y_dec.cpu().numpy(), y_ref.cpu().numpy())
    a, b = _stream(p), _stream(q)
    assert a.size == b.size and np.array_equal(a, b), int(np.argmax(a[:b.size] != b[:a.size]))
    # the stream advanced once: the next call equals the next SmartFP call
    y2, _ = rc.roundtrip_compress(x)
    assert same_f32(y2.cpu().numpy(), ref(x).cpu().numpy())


@pytest.mark.parametrize("case", ["all_positive", "trunc", "range", "sampled", "f16", "bf16",
                                  "bits_4_6"])
def test_variants(case):
    over, dtype, ap = {}, torch.float32, False
    if case == "all_positive":
        ap = True
    elif case == "trunc":
        over["stochastic_rounding"] = False
    elif case == "range":
        over["use_range_std_dev"] = True
    elif case == "sampled":
        over.update(use_sample_stats=True, num_samples=64)
    elif case in ("f16", "bf16"):
        dtype = torch.float16 if case == "f16" else torch.bfloat16
        over["precision"] = 16
    elif case == "bits_4_6":
        over.update(num_bits_main=4, num_bits_outlier=6)
    hp, rc, ref, pk = _codecs(**over)
    gen = torch.Generator(device="cuda").manual_seed(5)
    for n in (300_001, 3 << 20, 9 << 20):
        x = (torch.randn(n, generator=gen, device="cuda") * 2.0 + 0.25).to(dtype)
        if ap:
            x = torch.relu(x)
        y, p = rc.roundtrip_compress(x, all_positive=ap)
        y_ref = ref(x, all_positive=ap)
        q = pk.compress(x, all_positive=ap)
        torch.cuda.synchronize()
        assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy()), (case, n)
        assert same_f32(rc.decompress(p).cpu().numpy(), y_ref.cpu().numpy()), (case, n)
        a, b = _stream(p), _stream(q)
        assert np.array_equal(a, b), (case, n)


def test_batch_norm_variant():
    hp, rc, ref, pk = _codecs(use_batch_norm=True)
    gen = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(32, 24, 20, 20, generator=gen, device="cuda") * 1.5
    g = torch.rand(24, generator=gen, device="cuda") + 0.5
    b = torch.randn(24, generator=gen, device="cuda") * 0.1
    y, p = rc.roundtrip_compress(x, batch_norm_stats=(g, b))
    y_ref = ref(x, batch_norm_stats=(g, b))
    q = pk.compress(x, batch_norm_stats=(g, b))
    torch.cuda.synchronize()
    assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy())
    assert np.array_equal(_stream(p), _stream(q))
    assert same_f32(rc.decompress(p).cpu().numpy(), y_ref.cpu().numpy())


def _raw_call(x, n, cap, guard=4096):
    """The C-ABI with a buffer of cap bytes followed by a guard region of 0xAB bytes."""
    from smart_compress_amd import _native as N

    hp, rc, _, _ = _codecs()
    lib = N.lib()
    p = rc._params(n, False, torch.float32, x.device)
    buf = torch.full((cap + guard,), 0xAB, dtype=torch.uint8, device="cuda")
    y = torch.empty(n, device="cuda")
    ws = torch.empty(lib.smq_smaq_pack_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    rc_ = lib.smq_smaq_roundtrip_compress(x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, p,
                                          buf.data_ptr(), cap, ws.data_ptr(), ws.numel(),
                                          N.stream_ptr(x.device))
    torch.cuda.synchronize()
    hdr = N.SmqPackedHeader.from_buffer_copy(bytes(buf[:128].cpu().numpy()))
    return rc_, buf.cpu().numpy(), hdr, y


def test_capacity_bounded_buffer():
    from smart_compress_amd import _native as N

    lib = N.lib()
    n = 1_000_003
    gen = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(n, generator=gen, device="cuda")
    bound = lib.smq_smaq_pack_bound(n, 6, 8)
    rc0, full, hdr0, y0 = _raw_call(x, n, bound, 0)
    assert rc0 == 0
    total = int(hdr0.total_bytes)
    fixed = lib.smq_smaq_pack_fixed_bytes(n, 6)
    assert fixed < total < bound
    # exactly the stream's size: the same bytes
    rc1, b1, hdr1, y1 = _raw_call(x, n, total)
    assert rc1 == 0 and int(hdr1.total_bytes) == total
    assert np.array_equal(b1[:total], full[:total]) and (b1[total:] == 0xAB).all()
    assert same_f32(y1.cpu().numpy(), y0.cpu().numpy())
    # too small: flagged by total_bytes, nothing written past the buffer, y still complete
    small = fixed + (total - fixed) // 3
    rc2, b2, hdr2, y2 = _raw_call(x, n, small)
    assert rc2 == 0 and int(hdr2.total_bytes) == total > small
    assert (b2[small:] == 0xAB).all()
    assert np.array_equal(b2[:fixed], full[:fixed])
    assert same_f32(y2.cpu().numpy(), y0.cpu().numpy())
    # below the fixed part: refused
    rc3, _, _, _ = _raw_call(x, n, fixed - 8)
    assert rc3 == -2  # SMQ_ERR_WORKSPACE
    assert b"smq_smaq_pack_fixed_bytes" in lib.smq_last_error()


def test_one_launch_packer_workspace_reuse():
    """The one-launch packer (up to 2048 blocks) and the three-launch form (above) alternating on
    ONE workspace that starts as random bytes: every stream equals the one a fresh zeroed
    workspace gives (the look-back's status granules carry the call's generation; nothing the
    other launches write lands in their region)."""
    from smart_compress_amd import _native as N

    lib = N.lib()
    hp, rc, _, _ = _codecs()
    gen = torch.Generator(device="cuda").manual_seed(13)
    # (64 and 32 blocks alternating: the layout of the workspace moves with n — the pattern that
    # once let a stale status granule pass for the current call's)
    sizes = [1_000_003, 9_000_000, 4096 * 2048, 70_000, 9_000_000, 1_000_003] + [262_144, 131_072] * 4
    xs = {n: torch.randn(n, generator=gen, device="cuda") * 1.3 for n in set(sizes)}
    big = max(lib.smq_smaq_pack_workspace_bytes(n) for n in sizes)
    ws = torch.randint(0, 256, (big,), dtype=torch.uint8, device="cuda", generator=gen)

    def stream(n, w):
        p = rc._params(n, False, torch.float32, xs[n].device)
        p.offset = 77  # the same draws for both workspaces
        bound = lib.smq_smaq_pack_bound(n, 6, 8)
        out = torch.empty(bound, dtype=torch.uint8, device="cuda")
        assert lib.smq_smaq_compress(xs[n].data_ptr(), N.SMQ_DTYPE_F32, n, p, out.data_ptr(),
                                     bound, w.data_ptr(), w.numel(),
                                     N.stream_ptr(xs[n].device)) == 0
        torch.cuda.synchronize()
        hdr = N.SmqPackedHeader.from_buffer_copy(bytes(out[:128].cpu().numpy()))
        return out[:int(hdr.total_bytes)].cpu().numpy()

    for n in sizes:
        fresh = torch.zeros(lib.smq_smaq_pack_workspace_bytes(n), dtype=torch.uint8,
                            device="cuda")
        assert np.array_equal(stream(n, ws), stream(n, fresh)), n


# The single launch that also packs (smaq_fused.hip PACK: fp32, n % 4 == 0, up to 4 groups per
# lane, T_m > 0, no BN / range statistics): block b * V + u is built from workgroup b's registers
# right after its transform, the variable sections placed by one granule per workgroup. Its stream
# must be the look-back packer's byte for byte (compress() never takes it: y == NULL there).
PACK_SIZES = [4096, 8192, 12_288, 4096 * 255 + 8, 262_144, (1 << 20) + 4, 2 << 20,
              3 * (1 << 20) + 4000, 4 << 20, 4_194_300]


@pytest.mark.parametrize("n", PACK_SIZES)
@pytest.mark.parametrize("case", ["default", "all_positive", "trunc", "bits_4_6", "bits_5_7"])
def test_fused_pack_stream_equals_compress(n, case):
    over, ap = {}, False
    if case == "all_positive":
        ap = True
    elif case == "trunc":
        over["stochastic_rounding"] = False
    elif case == "bits_4_6":
        over.update(num_bits_main=4, num_bits_outlier=6)
    elif case == "bits_5_7":
        over.update(num_bits_main=5, num_bits_outlier=7)
    hp, rc, ref, pk = _codecs(**over)
    gen = torch.Generator(device="cuda").manual_seed(n + len(case))
    x = torch.randn(n, generator=gen, device="cuda") * 1.7 - 0.3
    if ap:
        x = torch.relu(x)
    for _ in range(2):  # twice: consecutive calls on one workspace (epochs advance)
        y, p = rc.roundtrip_compress(x, all_positive=ap)
        y_ref = ref(x, all_positive=ap)
        q = pk.compress(x, all_positive=ap)
        torch.cuda.synchronize()
        assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy()), (n, case)
        a, b = _stream(p), _stream(q)
        assert a.size == b.size and np.array_equal(a, b), (n, case, int(np.argmax(a != b)))
        assert same_f32(rc.decompress(p).cpu().numpy(), y_ref.cpu().numpy()), (n, case)


@pytest.mark.parametrize("n", [1 << 20, 3 << 20, 4 << 20])
def test_fused_pack_escape_heavy_blocks(n):
    """Activations whose channels sit far from the tensor's mean escape by the hundreds per block
    (more than the block's LDS section holds, and than a segment's list): those blocks are re-coded
    from x into their place; every other block keeps its LDS section. Same bytes as compress()."""
    hp, rc, ref, pk = _codecs()
    gen = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(n, generator=gen, device="cuda")
    x[: n // 64] += 40.0            # a run of blocks far above the mean: every element escapes
    x[n // 2: n // 2 + 300] = -1e5  # one block with 300 escapes in a row
    x[n - 4096 + 17: n - 4096 + 60] = 3e4  # the last block: 43 escapes in one segment
    y, p = rc.roundtrip_compress(x)
    y_ref = ref(x)
    q = pk.compress(x)
    torch.cuda.synchronize()
    assert same_f32(y.cpu().numpy(), y_ref.cpu().numpy())
    a, b = _stream(p), _stream(q)
    assert a.size == b.size and np.array_equal(a, b)
    assert same_f32(rc.decompress(p).cpu().numpy(), y_ref.cpu().numpy())


def test_fused_pack_capacity_bounded_buffer():
    """The PACK launch with a buffer below the stream's size: total_bytes flags it, nothing is
    written past the buffer, the fixed part and y are complete."""
    from smart_compress_amd import _native as N

    lib = N.lib()
    n = 1_000_000
    gen = torch.Generator(device="cuda").manual_seed(19)
    x = torch.randn(n, generator=gen, device="cuda")
    rc0, full, hdr0, y0 = _raw_call(x, n, lib.smq_smaq_pack_bound(n, 6, 8), 0)
    total = int(hdr0.total_bytes)
    fixed = lib.smq_smaq_pack_fixed_bytes(n, 6)
    assert rc0 == 0 and fixed < total
    rc1, b1, hdr1, y1 = _raw_call(x, n, total)
    assert rc1 == 0 and int(hdr1.total_bytes) == total
    assert np.array_equal(b1[:total], full[:total]) and (b1[total:] == 0xAB).all()
    small = fixed + (total - fixed) // 3
    rc2, b2, hdr2, y2 = _raw_call(x, n, small)
    assert rc2 == 0 and int(hdr2.total_bytes) == total > small
    assert (b2[small:] == 0xAB).all() and np.array_equal(b2[:fixed], full[:fixed])
    assert same_f32(y2.cpu().numpy(), y0.cpu().numpy())


def test_fused_pack_workspace_of_random_bytes():
    """The PACK launch's aggregates are epoch-tagged granules: a workspace of random bytes, reused
    across sizes and by the other packers, gives the fresh workspace's streams."""
    from smart_compress_amd import _native as N

    lib = N.lib()
    hp, rc, _, _ = _codecs()
    gen = torch.Generator(device="cuda").manual_seed(23)
    sizes = [1 << 20, 4 << 20, 262_144, 9_000_000, 1 << 20, 65_536, 4 << 20]
    xs = {n: torch.randn(n, generator=gen, device="cuda") * 1.1 for n in set(sizes)}
    big = max(lib.smq_smaq_pack_workspace_bytes(n) for n in sizes)
    ws = torch.randint(0, 256, (big,), dtype=torch.uint8, device="cuda", generator=gen)

    def stream(n, w):
        p = rc._params(n, False, torch.float32, xs[n].device)
        p.offset = 91
        bound = lib.smq_smaq_pack_bound(n, 6, 8)
        out = torch.empty(bound, dtype=torch.uint8, device="cuda")
        y = torch.empty(n, device="cuda")
        assert lib.smq_smaq_roundtrip_compress(xs[n].data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n,
                                               p, out.data_ptr(), bound, w.data_ptr(), w.numel(),
                                               N.stream_ptr(xs[n].device)) == 0
        torch.cuda.synchronize()
        hdr = N.SmqPackedHeader.from_buffer_copy(bytes(out[:128].cpu().numpy()))
        return out[:int(hdr.total_bytes)].cpu().numpy(), y.cpu().numpy()

    for n in sizes:
        fresh = torch.zeros(lib.smq_smaq_pack_workspace_bytes(n), dtype=torch.uint8,
                            device="cuda")
        (a, ya), (b, yb) = stream(n, ws), stream(n, fresh)
        assert np.array_equal(a, b) and same_f32(ya, yb), n


# smq_smaq_roundtrip_compress_notify: the launch that writes the header also stores total_bytes
# into a host-mapped word (PackedActivations reads it instead of an event + copy per batch).
@pytest.mark.parametrize("n,case", [(1 << 20, "pack"), (4 << 20, "pack"), (6_000_000, "lookback"),
                                    (1_000_003, "lookback"), (9_000_000, "three_launch"),
                                    (1 << 20, "bn"), (1 << 20, "small_buffer"),
                                    (3 << 20, "escape_heavy")])
def test_notify_word_equals_header_total(n, case):
    from smart_compress_amd import _native as N

    lib = N.lib()
    hp, rc, _, _ = _codecs()
    gen = torch.Generator(device="cuda").manual_seed(n % 977 + len(case))
    x = torch.randn(n, generator=gen, device="cuda") * 1.4
    if case == "escape_heavy":
        x[: n // 64] += 40.0
    bn_args = None
    if case == "bn":
        x = x.view(64, 16, -1)
        g = torch.rand(16, generator=gen, device="cuda") + 0.5
        b = torch.randn(16, generator=gen, device="cuda") * 0.1
        bn_args = (g, b)
    words = lib.smq_notify_alloc(4)
    assert words
    try:
        w = np.ctypeslib.as_array((ctypes.c_uint32 * 4).from_address(words))
        assert (w == N.SMQ_NOTIFY_PENDING).all()  # armed by the allocation
        w[1] = 12345  # a neighbour the launch must leave alone
        p = rc._params(n, False, torch.float32, x.device)
        if bn_args is not None:  # the BN variant (smart.py:136-149): the general packer
            p.bn_gamma, p.bn_beta = bn_args[0].data_ptr(), bn_args[1].data_ptr()
            p.bn_channels, p.bn_inner = 16, x.shape[2]
        bound = (lib.smq_smaq_pack_bound_bn(n, 6, 8, 16) if bn_args is not None
                 else lib.smq_smaq_pack_bound(n, 6, 8))
        cap = bound
        if case == "small_buffer":
            cap = lib.smq_smaq_pack_fixed_bytes(n, 6) + 4096
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        y = torch.empty(n, device="cuda")
        ws = torch.zeros(lib.smq_smaq_pack_workspace_bytes(n), dtype=torch.uint8, device="cuda")
        assert lib.smq_smaq_roundtrip_compress_notify(
            x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, p, out.data_ptr(), cap,
            ws.data_ptr(), ws.numel(), ctypes.c_void_p(words), N.stream_ptr(x.device)) == 0, \
            lib.smq_last_error()
        torch.cuda.synchronize()
        hdr = N.SmqPackedHeader.from_buffer_copy(bytes(out[:128].cpu().numpy()))
        assert int(w[0]) == int(hdr.total_bytes), (case, int(w[0]), int(hdr.total_bytes))
        assert int(w[1]) == 12345 and int(w[2]) == N.SMQ_NOTIFY_PENDING
        if case == "small_buffer":
            assert int(w[0]) > cap  # did not fit: the word says so as the header does
        # a NULL word: the plain call's bytes
        out2 = torch.empty(cap, dtype=torch.uint8, device="cuda")
        assert lib.smq_smaq_roundtrip_compress_notify(
            x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, p, out2.data_ptr(), cap,
            ws.data_ptr(), ws.numel(), None, N.stream_ptr(x.device)) == 0
        torch.cuda.synchronize()
        t = min(int(hdr.total_bytes), cap)
        if case != "small_buffer":
            assert torch.equal(out[:t], out2[:t])
        # misaligned word: refused
        assert lib.smq_smaq_roundtrip_compress_notify(
            x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, p, out2.data_ptr(), cap,
            ws.data_ptr(), ws.numel(), ctypes.c_void_p(words + 2), N.stream_ptr(x.device)) != 0
    finally:
        lib.smq_notify_free(ctypes.c_void_p(words))
