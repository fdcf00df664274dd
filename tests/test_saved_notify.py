"""PackedActivations' size notification bookkeeping, on the CPU (no device launch): the notify ring
(util/pytorch/saved.py _NotifyRing: a word is re-armed only once nobody holds it and its last launch
has written it) and the harvest of notified handles (_poll: oldest first, a stream that fitted drops
its activation, one that did not keeps it, the host waits only while more than the budget waits).
The device side (the launch writes header.total_bytes into the word) is
tests/test_gpu_roundtrip_compress.py::test_notify_word_equals_header_total."""

import threading

import numpy as np
import torch

from helpers import smaq_hparams


def _ring(words=8):
    from smart_compress_amd.util.pytorch.saved import _NotifyRing

    r = _NotifyRing.__new__(_NotifyRing)  # (no host-mapped allocation: a plain array)
    r.WORDS = words
    r.words = np.zeros(words, dtype=np.uint32)
    r.held = bytearray(words)
    r.next = 0
    r.base = 0
    return r


def test_ring_rearms_only_free_written_words():
    from smart_compress_amd import _native as N

    r = _ring(8)
    got = [r.take() for _ in range(8)]
    assert got == list(range(8)) and (r.words == N.SMQ_NOTIFY_PENDING).all()
    assert r.take() is None  # every word held
    r.release(3, written=False)  # a declined call: no launch writes word 3
    assert r.words[3] == 0 and r.take() == 3
    r.release(5)  # released, but its launch has not written it yet: not re-armed under it
    assert r.take() is None
    r.words[5] = 1234  # the launch's store arrives
    assert r.take() == 5 and r.words[5] == N.SMQ_NOTIFY_PENDING


def _acts_with(ring):
    from smart_compress_amd.compress import SmartFPPacked
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    acts = PackedActivations(SmartFPPacked(smaq_hparams()), verify_bytes=1000)
    acts._notify = ring
    return acts


def _handle(acts, ring, n, cap):
    from smart_compress_amd.compress.packed import SmaqPacked
    from smart_compress_amd.util.pytorch.saved import _Saved

    i = ring.take()
    y = torch.zeros(n)
    h = _Saved(SmaqPacked(torch.zeros(cap, dtype=torch.uint8), (n,), n, widths=(6, 8)), y,
               acts.codec, y._version, None, i)
    acts._notified.append(h)
    acts._notified_bytes += 4 * n
    return h


def test_poll_finishes_written_words_in_order():
    from smart_compress_amd import _native as N

    ring = _ring(8)
    acts = _acts_with(ring)
    a = _handle(acts, ring, 100, 64)
    b = _handle(acts, ring, 100, 64)
    c = _handle(acts, ring, 100, 64)
    ring.words[b.slot] = 40  # b written before a: a (the oldest) still blocks the queue
    acts._poll(10_000)
    assert len(acts._notified) == 3 and a.y is not None and b.y is not None
    ring.words[a.slot] = 64  # fits exactly
    acts._poll(10_000)
    assert a.y is None and a.packed._total == 64 and b.y is None and b.packed._total == 40
    assert list(acts._notified) == [c] and acts._notified_bytes == 400
    assert not ring.held[0] and not ring.held[1] and ring.held[2]
    ring.words[c.slot] = 65  # one byte over its buffer: the activation stays the saved value
    acts._poll(0)
    assert c.packed is None and c.y is not None and acts.kept_fp32 == 1
    assert acts.saved_bytes == 104 and not any(ring.held)
    assert N.SMQ_NOTIFY_PENDING not in (int(ring.words[0]), int(ring.words[1]))


def test_poll_waits_for_the_oldest_only_over_budget():
    ring = _ring(8)
    acts = _acts_with(ring)  # budget 1000 bytes
    a = _handle(acts, ring, 200, 64)  # 800 bytes waiting: under the budget, no wait
    acts._poll(acts.verify_bytes)
    assert a.y is not None
    b = _handle(acts, ring, 200, 64)  # 1600 waiting: wait for a (written 20 ms later), not b
    t = threading.Timer(0.02, lambda: ring.words.__setitem__(a.slot, 10))
    t.start()
    acts._poll(acts.verify_bytes)
    t.join()
    assert a.y is None and b.y is not None and list(acts._notified) == [b]


def test_replayable_activation_modules():
    """The in-place activation modules whose result can be held as the codec output's stream plus
    the module (their in-place op saves its result): exact types, inplace=True only."""
    import torch.nn as nn

    from smart_compress_amd.util.pytorch.saved import replayable

    assert all(replayable(m) for m in (nn.ReLU(True), nn.LeakyReLU(0.2, True), nn.ELU(inplace=True),
                                       nn.CELU(inplace=True), nn.SELU(True)))
    # out of place, or in-place ops that save a clone of their input (nothing of the output's
    # storage is saved, so there is nothing to replay)
    assert not any(replayable(m) for m in (nn.ReLU(), nn.SiLU(True), nn.ReLU6(True),
                                           nn.Hardtanh(inplace=True), nn.Hardswish(True),
                                           nn.Conv2d(1, 1, 1)))

    class MyReLU(nn.ReLU):
        pass

    assert not replayable(MyReLU(True))  # (a subclass may change forward)


def test_autograd_wrapper_notes_inplace_activations_before_they_run():
    """register_autograd_module (autograd.py:50-77) tells a compress_fn with note_inplace about a
    replayable module's input before the module runs (the value not yet changed), and about no
    other module."""
    import torch.nn as nn
    from argparse import Namespace

    from smart_compress_amd.util.pytorch.autograd import register_autograd_module

    seen = []

    class Fn:
        def __call__(self, x, tag=None, **kw):
            return x.clone()

        def note_inplace(self, module, x):
            seen.append((type(module).__name__, x.clone()))

    net = nn.Sequential(nn.Linear(4, 4), nn.ReLU(inplace=True), nn.Tanh(), nn.ReLU())
    register_autograd_module(net, Fn(), Namespace(compress_forward=True, compress_backward=True))
    x = torch.randn(3, 4)
    h = net[0](x).detach()
    net(x)
    assert [s[0] for s in seen] == ["ReLU"] and torch.equal(seen[0][1], h)


def test_roundtrip_compress_side_stream_needs_private_workspace():
    """roundtrip_compress with pack_stream but no workspace raises (the shared per-stream
    workspace would be rewritten by the next call on the current stream while pack_stream reads
    it)."""
    import pytest

    from smart_compress_amd.compress import SmartFPPacked

    with pytest.raises(ValueError, match="private workspace"):
        SmartFPPacked(smaq_hparams()).roundtrip_compress(torch.randn(4096), pack_stream=object())
