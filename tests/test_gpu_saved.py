"""SmaQ-packed saved activations (util/pytorch/saved.py) against the unpacked SmaQ training step.

The reference keeps every compressed activation as fp32 (autograd.py:18-77); PackedActivations
keeps the ones autograd saves for backward as SmaQ streams and decodes them in backward. Because
decode(encode(x)) == SmartFP(x) bit for bit (include/smq.h "Packed SmaQ container"), the loss and
every gradient must equal the SmartFP run's bit for bit, while the saved bytes shrink."""

from argparse import Namespace

import pytest
import torch
import torch.nn as nn

from helpers import smaq_hparams

pytestmark = pytest.mark.gpu


def _net(inplace):
    def block(cin, cout):
        return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout),
                             nn.ReLU(inplace=inplace))

    return nn.Sequential(block(3, 32), block(32, 32), nn.MaxPool2d(2), block(32, 64),
                         block(64, 64), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(64, 10))


def _eq(a, b):
    return torch.equal(a.view(torch.int32), b.view(torch.int32))


@pytest.mark.parametrize("inplace,overlap", [(False, True), (True, True), (False, False),
                                             (True, False)])
def test_packed_saved_activations_bitexact(inplace, overlap):
    from smart_compress_amd.compress import SmartFP, SmartFPPacked
    from smart_compress_amd.util.pytorch.autograd import register_autograd_module
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    flags = Namespace(compress_forward=True, compress_backward=True, use_batch_norm=False)

    def run(packed):
        torch.manual_seed(3)
        net = _net(inplace).cuda()
        codec = (SmartFPPacked if packed else SmartFP)(smaq_hparams())
        codec.rng.seed, codec.rng.offset = 21, 0
        acts = PackedActivations(codec, verify_bytes=8 << 20, overlap=overlap) if packed else None
        register_autograd_module(net, acts if packed else codec, flags)
        opt = torch.optim.SGD(net.parameters(), lr=0.05, momentum=0.9)
        g = torch.Generator(device="cuda").manual_seed(9)
        out, peaks = [], []
        for _ in range(2):
            x = torch.randn(64, 3, 32, 32, device="cuda", generator=g, requires_grad=True)
            tgt = torch.arange(64, device="cuda") % 10
            opt.zero_grad()
            torch.cuda.synchronize()
            base = torch.cuda.memory_allocated()
            torch.cuda.reset_peak_memory_stats()
            if packed:
                with acts:
                    loss = nn.functional.cross_entropy(net(x), tgt)
            else:
                loss = nn.functional.cross_entropy(net(x), tgt)
            torch.cuda.synchronize()
            peaks.append(torch.cuda.memory_allocated() - base)  # held for backward
            loss.backward()
            opt.step()
            out.append((loss.detach(), x.grad.clone(), [p.grad.clone() for p in net.parameters()]))
        return out, codec.rng.offset, peaks, acts

    prev = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:  # (deterministic weight-gradient kernels: the parameter gradients compare bit for bit)
        a, off_a, held_a, _ = run(False)
        b, off_b, held_b, acts = run(True)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev
    assert off_a == off_b > 0
    for (la, xa, ga), (lb, xb, gb) in zip(a, b):
        assert _eq(la, lb) and _eq(xa, xb)
        assert all(_eq(p, q) for p, q in zip(ga, gb))
    acts.verify()  # (sizes not read by the last unpacks: nothing waits for them at the exit)
    st = acts.stats()
    # the second step skipped the packing of the outputs the first one did not save as streams
    assert st["skipped_packs"] > 0, st
    assert st["saved_packed"] >= 8 and 6.0 < st["bits_per_element"] < 9.0, st
    assert st["kept_fp32"] == 0 and st["allocated_bits_per_element"] < 10.5, st
    # in-place ReLUs on the BatchNorm outputs: their values saved as the BN output's stream with
    # the ReLU replayed on the decoded values
    assert (st["saved_replayed"] > 0) == inplace, st
    if not overlap:  # the C calls' sizes came through notify words, every word released since
        assert acts._notify is not None and not any(acts._notify.held)
        assert not acts._notified and not acts._inflight and not acts._pending
    # the memory held between forward and backward shrinks by the packed activations' share
    # (second step: the first one also allocates workspaces)
    assert held_b[1] < 0.8 * held_a[1], (held_a, held_b)


def test_stream_capacity_cut_keeps_the_activation():
    """A stream larger than its capacity (escape-heavy data: 8 % of the elements at +-1e6, whose
    outlier codes exceed the 8-bit budget: ~93 KB against a 71 KB capacity at 64K elements) is
    detected when the pending streams are checked: the saved value is then the activation itself,
    still exact."""
    from smart_compress_amd.compress import SmartFP, SmartFPPacked
    from smart_compress_amd.util.pytorch.autograd import Compressor
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(1 << 16, device="cuda", generator=g)
    x[::25] = 1e6
    x[12::25] = -1e6  # z ~ +-3.5: |q| ~ 105 > 63, escaped
    res = []
    for packed in (False, True):
        codec = (SmartFPPacked if packed else SmartFP)(smaq_hparams())
        codec.rng.seed, codec.rng.offset = 2, 0
        acts = PackedActivations(codec) if packed else None
        comp = Compressor(acts if packed else codec)
        w = torch.linspace(0.5, 1.5, x.numel(), device="cuda").requires_grad_(True)
        if packed:
            with acts:
                y = comp(x * w)
                loss = (y * y).sum()  # (y saved by the multiply)
        else:
            y = comp(x * w)
            loss = (y * y).sum()
        loss.backward()
        res.append((y.detach(), w.grad.clone()))
        if packed:
            acts.verify()  # (its size may still be unread: nothing waits at the context's exit)
            assert acts.stats()["kept_fp32"] == 1
    assert _eq(res[0][0], res[1][0]) and _eq(res[0][1], res[1][1])


def test_packed_saved_outside_context_and_backward_calls():
    """Outside the context (and for backward-direction calls) the compress_fn is the plain codec
    call: the same outputs and random stream as SmartFP."""
    from smart_compress_amd.compress import SmartFP, SmartFPPacked
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    x = torch.randn(100_000, device="cuda")
    ref = SmartFP(smaq_hparams())
    pk = SmartFPPacked(smaq_hparams())
    for c in (ref, pk):
        c.rng.seed, c.rng.offset = 4, 0
    acts = PackedActivations(pk)
    assert _eq(acts(x, tag="forward_autograd"), ref(x))
    with acts:
        assert _eq(acts(x, tag="backward_autograd"), ref(x))
        assert _eq(acts(x, tag="forward_autograd"), ref(x))
    assert pk.rng.offset == ref.rng.offset


@pytest.mark.parametrize("overlap", [True, False])
def test_backward_inside_the_context_waits_for_the_packer(overlap):
    """A backward run while the context is still open decodes streams whose packing launches ran on
    the side stream (overlap=True: _unpack joins the side stream first): the decode is ordered
    after them (the gradient equals SmartFP's)."""
    from smart_compress_amd.compress import SmartFP, SmartFPPacked
    from smart_compress_amd.util.pytorch.autograd import Compressor
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(3 << 20, device="cuda", generator=g)
    res = []
    for packed in (False, True):
        codec = (SmartFPPacked if packed else SmartFP)(smaq_hparams())
        codec.rng.seed, codec.rng.offset = 8, 0
        acts = (PackedActivations(codec, verify_bytes=1 << 10, overlap=overlap) if packed
                else None)
        comp = Compressor(acts if packed else codec)
        w = torch.linspace(0.5, 1.5, x.numel(), device="cuda").requires_grad_(True)
        if packed:
            with acts:
                y = comp(x * w)
                loss = (y * y).sum()
                acts.verify()  # the activation dropped: backward must decode the stream
                assert acts._joined == (not overlap)  # overlap: the side stream not joined yet
                loss.backward()
                assert acts._joined
        else:
            y = comp(x * w)
            (y * y).sum().backward()
        res.append((y.detach(), w.grad.clone()))
    assert _eq(res[0][0], res[1][0]) and _eq(res[0][1], res[1][1])


@pytest.mark.parametrize("when", ["held", "verified", "modified_then_verified"])
def test_inplace_change_after_save_raises(when):
    """saved_tensors_hooks switch off autograd's version check; PackedActivations repeats it, so an
    activation modified in place after a multiply saved it raises autograd's error in backward (as
    the reference, whose autograd saves y itself, autograd.py:30-42) — whether the saved value is
    still the held activation or already the stream, and whether the change came before or after
    the size check that dropped the activation."""
    from smart_compress_amd.compress import SmartFP, SmartFPPacked
    from smart_compress_amd.util.pytorch.autograd import Compressor
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    x = torch.randn(1 << 18, device="cuda")
    w = torch.linspace(0.5, 1.5, x.numel(), device="cuda").requires_grad_(True)
    # the reference behaviour: plain SmartFP, y saved by the multiply, then changed in place
    comp = Compressor(SmartFP(smaq_hparams()))
    y = comp(x * w)
    loss = (y * w).sum()
    y.add_(1.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        loss.backward()
    codec = SmartFPPacked(smaq_hparams())
    acts = PackedActivations(codec, verify_bytes=1 << 40)
    comp = Compressor(acts)
    with acts:
        y = comp(x * w)
        loss = (y * w).sum()  # saves y (held until its size is checked)
        if when == "verified":
            acts.verify()     # y dropped: the saved value is now the stream
            y.add_(1.0)
        elif when == "modified_then_verified":
            y.add_(1.0)
            acts.verify()
        else:
            y.add_(1.0)
        with pytest.raises(RuntimeError, match="modified by an inplace operation"):
            loss.backward()
    assert acts.stats()["saved_packed"] == 1


def test_skipped_site_that_gets_saved_stays_exact():
    """A call site whose stream went unsaved in one step runs as SmartFP's own call in the next
    (saved_tensors_hooks then see an output with no stream: it is saved as itself). When that
    step does save it, the values and gradients are still SmartFP's; the re-probe step packs it
    again."""
    from smart_compress_amd.compress import SmartFP, SmartFPPacked
    from smart_compress_amd.util.pytorch.autograd import Compressor
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(1 << 18, device="cuda", generator=g)
    ref = SmartFP(smaq_hparams())
    pk = SmartFPPacked(smaq_hparams())
    for c in (ref, pk):
        c.rng.seed, c.rng.offset = 5, 0
    acts = PackedActivations(pk)
    acts._REPROBE = 3
    comp_p, comp_r = Compressor(acts), Compressor(ref)
    for step, saves in enumerate((False, True, True, True)):
        res = []
        for comp in (comp_r, comp_p):
            w = torch.linspace(0.5, 1.5, x.numel(), device="cuda").requires_grad_(True)
            if comp is comp_p:
                with acts:
                    y = comp(x * w)
                    loss = (y * y).sum() if saves else y.sum()  # (y * y saves y; sum does not)
            else:
                y = comp(x * w)
                loss = (y * y).sum() if saves else y.sum()
            loss.backward()
            res.append((y.detach(), w.grad.clone()))
        assert _eq(res[0][0], res[1][0]) and _eq(res[0][1], res[1][1]), step
        acts.verify()
        st = acts.stats()
        # step 0 packs (unsaved); steps 1-2 skip the site; step 2 is the re-probe's last skipped
        # step (the skip set clears after 3 steps), step 3 packs and saves a stream again
        assert st["skipped_packs"] == {0: 0, 1: 1, 2: 2, 3: 2}[step], (step, st)
    assert st["saved_packed"] == 2 and pk.rng.offset == ref.rng.offset  # (y * y: y saved twice)


def test_packed_saved_float64_activations_bitexact():
    """A float64 model (autograd.py:64-72 compresses whatever dtype a layer produces): its saved
    activations are held as float64 streams (SMQ_PACK_FLAG_F64) and the gradients equal the
    SmartFP run's bit for bit."""
    from smart_compress_amd.compress import SmartFP, SmartFPPacked
    from smart_compress_amd.util.pytorch.autograd import register_autograd_module
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    flags = Namespace(compress_forward=True, compress_backward=True, use_batch_norm=False)

    def run(packed):
        torch.manual_seed(5)
        net = nn.Sequential(nn.Linear(256, 512), nn.ReLU(), nn.Linear(512, 512), nn.Tanh(),
                            nn.Linear(512, 10)).cuda().double()
        codec = (SmartFPPacked if packed else SmartFP)(smaq_hparams())
        codec.rng.seed, codec.rng.offset = 8, 0
        acts = PackedActivations(codec) if packed else None
        register_autograd_module(net, acts if packed else codec, flags)
        g = torch.Generator(device="cuda").manual_seed(4)
        x = torch.randn(512, 256, device="cuda", generator=g, dtype=torch.float64,
                        requires_grad=True)
        if packed:
            with acts:
                loss = net(x).square().mean()
        else:
            loss = net(x).square().mean()
        loss.backward()
        return (loss.detach(), x.grad.clone(), [p.grad.clone() for p in net.parameters()],
                codec.rng.offset, acts)

    la, xa, ga, off_a, _ = run(False)
    lb, xb, gb, off_b, acts = run(True)
    assert off_a == off_b > 0
    v = lambda t: t.view(torch.int64)  # noqa: E731
    assert torch.equal(v(la), v(lb)) and torch.equal(v(xa), v(xb))
    assert all(torch.equal(v(p), v(q)) for p, q in zip(ga, gb))
    acts.verify()
    st = acts.stats()
    assert st["saved_packed"] >= 2 and st["kept_fp32"] == 0, st


@pytest.mark.parametrize("act", ["relu", "leaky", "elu", "celu", "selu"])
def test_inplace_activation_replayed_bitexact(act):
    """An in-place activation module applied to a codec output (ResNet's relu(bn1(x))): its value
    is saved as the codec output's stream and the module replayed on the decoded values in
    backward; loss and every gradient equal the SmartFP run's bit for bit."""
    from smart_compress_amd.compress import SmartFP, SmartFPPacked
    from smart_compress_amd.util.pytorch.autograd import register_autograd_module
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    make = {"relu": lambda: nn.ReLU(inplace=True),
            "leaky": lambda: nn.LeakyReLU(0.1, inplace=True),
            "elu": lambda: nn.ELU(0.7, inplace=True),
            "celu": lambda: nn.CELU(1.3, inplace=True),
            "selu": lambda: nn.SELU(inplace=True)}[act]
    flags = Namespace(compress_forward=True, compress_backward=True, use_batch_norm=False)

    def run(packed):
        torch.manual_seed(11)
        net = nn.Sequential(nn.Linear(128, 1024), make(), nn.Linear(1024, 1024), nn.LayerNorm(1024),
                            make(), nn.Linear(1024, 10)).cuda()
        codec = (SmartFPPacked if packed else SmartFP)(smaq_hparams())
        codec.rng.seed, codec.rng.offset = 6, 0
        acts = PackedActivations(codec) if packed else None
        register_autograd_module(net, acts if packed else codec, flags)
        g = torch.Generator(device="cuda").manual_seed(2)
        out = []
        for _ in range(2):
            x = torch.randn(512, 128, device="cuda", generator=g, requires_grad=True)
            net.zero_grad()
            if packed:
                with acts:
                    loss = net(x).square().mean()
            else:
                loss = net(x).square().mean()
            loss.backward()
            out.append((loss.detach(), x.grad.clone(), [p.grad.clone() for p in net.parameters()]))
        return out, codec.rng.offset, acts

    a, off_a, _ = run(False)
    b, off_b, acts = run(True)
    assert off_a == off_b > 0
    for (la, xa, ga), (lb, xb, gb) in zip(a, b):
        assert _eq(la, lb) and _eq(xa, xb)
        assert all(_eq(p, q) for p, q in zip(ga, gb))
    acts.verify()
    st = acts.stats()
    assert st["saved_replayed"] >= 2 and st["kept_fp32"] == 0, st


def test_inplace_activation_then_modified_raises():
    """A replayed activation's value modified in place again after it was saved: backward raises
    autograd's in-place error (saved_tensors_hooks switch autograd's own check off)."""
    from smart_compress_amd.compress import SmartFPPacked
    from smart_compress_amd.util.pytorch.autograd import register_autograd_module
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    flags = Namespace(compress_forward=True, compress_backward=True, use_batch_norm=False)
    lin, relu = nn.Linear(64, 4096).cuda(), nn.ReLU(inplace=True)
    acts = PackedActivations(SmartFPPacked(smaq_hparams()))
    register_autograd_module(nn.Sequential(lin), acts, flags)
    x = torch.randn(64, 64, device="cuda", requires_grad=True)
    with acts:
        y = lin(x)
        acts.note_inplace(relu, y)
        z = torch.relu_(y)  # saved (the replayed handle)
        z.mul_(2.0)         # ... and modified after it was saved
        loss = z.sum()
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        loss.backward()
