"""SmaQ-packed activations for backward: the memory saving the reference only reports.

The reference compresses each layer output through autograd (smart_compress/util/pytorch/
autograd.py:18-77: ``y = compress_fn(x)``, smart.py:110-190) but keeps ``y`` as an fp32 tensor, so
the tensors autograd saves for backward take their full size; the memory saving the paper claims
("reduce the memory usage during training by up to 6.7x", README.md:25) exists only as the size
``log_size`` reports (smart.py:184-188).

``PackedActivations`` makes it real with identical numerics. Used as the ``compress_fn`` of
``register_autograd_module``, each forward call computes ``P = SmartFPPacked.compress(x)`` and
returns ``y = decompress(P)`` — bit for bit what ``SmartFP`` returns for the same input, flags and
random stream (include/smq.h "Packed SmaQ container"). Inside ``with activations:`` a
``torch.autograd.graph.saved_tensors_hooks`` pair replaces every saved tensor that IS such a ``y``
(same storage, shape, strides, and not modified in place since) by ``P``, and the backward decodes
it again: the gradients equal those of the unpacked SmaQ run bit for bit, while a saved activation
takes ~8 bits per element (6/8-bit codes) instead of 32.

Memory without host synchronisation per call or per step: ``y`` and its stream come from one call
(``SmartFPPacked.roundtrip_compress``: SmartFP's round trip, then the packing launches on its
statistics), the stream written straight into a buffer of ``capacity`` bytes — the fixed region
(known from n) plus room for every element being an outlier and 1 % escapes (``stream_capacity``).
Only a stream larger than that (escape-heavy data) does not fit, which its header records, so until
its size is checked the saved ``y`` is kept too. The size reaches the host without a
synchronisation: the C forward call (csrc/torchfast.cpp ``smaq_packed``) hands the library a word of
host-mapped coherent memory (``smq_smaq_roundtrip_compress_notify``) into which the launch that writes
the stream's header stores its total_bytes, and the host reads it with a load. Each save reads the
words that are there (oldest first: a stream that fit drops its ``y``) and waits — for the oldest
word only, i.e. an earlier call, usually done by then — while more than 64 MiB of activations are
still waiting (``verify_bytes`` sets it), at the context's exit too (the rest are read by later
saves, unpacks or the next entry: ``y`` stays the saved value until then). Calls that take the
Python path (no notify word) send their sizes in batches of ``verify_batch`` bytes instead (a device
gather, an asynchronous copy to pinned memory, an event; 32 MiB of held activations at most by
default), settled at the context's exit. A stream
that did not fit (never seen on N(0,1)-like data) keeps ``y`` as the saved value instead.
The forward call is one C call where it applies (csrc/torchfast.cpp ``smaq_packed``: SmartFP's
parameter template, the output allocations and ``smq_smaq_roundtrip_compress``). Overlap
(opt-in, ``overlap=True``): the packing launches of a forward call run on a side stream — they
wait for the call's statistics by an event and then run beside the next layers, each call with
one of a ring of workspaces the current stream waits for before reusing; backward (and the size
checks) are ordered after the side stream. It costs ~20 us of host time per call (events, stream
waits, record_stream), which an eager ResNet-34 step cannot spare (15.0 -> 19.2 ms/step,
profiles/r5x_saved_ab.txt).
float64 activations are held as float64 streams (``SmartFPPacked.compress`` then its decode: SmartFP's
fp64 chain bit for bit; autograd.py:64-72 compresses whatever dtype the layer produces).
Backward-direction calls (grad-maps, never saved) and calls outside the context run as SmartFP's
own call (the same values as the codec's decompress(compress(x)), one launch instead of five).
"""

import ctypes
import time
import weakref
from collections import deque
from typing import Deque, Dict, List, Optional

import numpy as np
import torch

from ... import _native as N
from ...compress.packed import SmaqPacked, SmartFPPacked, _HDR_BYTES, _TOTAL_OFF
from ...compress.smart import SmartFP
from ..globals import Globals

__all__ = ["PackedActivations", "stream_capacity"]

FORWARD_TAG = "forward_autograd"
ESCAPE_FRAC = 0.01  # a saved stream's capacity: every element an outlier and 1 % escapes


def stream_capacity(n: int, num_bits_main: int, num_bits_outlier: int, bn_channels: int = 0,
                    escape_frac: float = 0.01) -> int:
    """Bytes of a stream of n elements (format v2) with every element an outlier and up to
    ``escape_frac`` of them escaped: the header, the directory, the fixed region, per block the
    outlier bits above the plane (rounded up to a word), the escapes, the BN table."""
    nb = (n + N.SMQ_PACK_BLOCK - 1) // N.SMQ_PACK_BLOCK
    wm, wo = num_bits_main - 1, num_bits_outlier - 1
    we = max(0, wo - wm)
    fixed_words = 128 + 128 * wm
    var_words = (we * n + 31) // 32 + nb + 2 * int(escape_frac * n + nb)
    return (_HDR_BYTES + 8 * (nb + (nb & 1)) + 4 * (nb * fixed_words + var_words)
            + 8 * bn_channels)


class _NotifyRing:
    """Words of host-mapped coherent memory (smq_notify_alloc) into which the forward calls' packing
    launches store their stream's size (smq_smaq_roundtrip_compress_notify): the host reads whether
    a stream fitted its capacity with a load — no event, copy or synchronisation per call. One ring
    per process, never freed (a launch in flight may still write a word). A word is free to take
    again once no handle holds it and its last launch has written it (a word still pending may be
    written late: never re-armed under it)."""

    WORDS = 1 << 14

    def __init__(self):
        ptr = N.lib().smq_notify_alloc(self.WORDS)
        if not ptr:
            raise RuntimeError("smq_notify_alloc failed: "
                               + N.lib().smq_last_error().decode(errors="replace"))
        self.base = ptr
        self.words = np.ctypeslib.as_array((ctypes.c_uint32 * self.WORDS).from_address(ptr))
        self.words[:] = 0  # free
        self.held = bytearray(self.WORDS)
        self.next = 0

    def take(self) -> Optional[int]:
        """A word armed (SMQ_NOTIFY_PENDING) for the next call, or None when the next few are
        still busy (the call then takes the event path)."""
        w, held = self.words, self.held
        for _ in range(16):
            i = self.next
            self.next = (i + 1) % self.WORDS
            if not held[i] and w[i] != N.SMQ_NOTIFY_PENDING:
                held[i] = 1
                w[i] = N.SMQ_NOTIFY_PENDING
                return i
        return None

    def release(self, i: int, written: bool = True) -> None:
        """Nobody reads word i any more; written=False: no launch will write it (the call was
        declined or failed)."""
        if not written:
            self.words[i] = 0
        self.held[i] = 0


_RING: Optional[_NotifyRing] = None


def _notify_ring() -> Optional[_NotifyRing]:
    global _RING
    if _RING is None:
        try:
            _RING = _NotifyRing()
        except (RuntimeError, OSError, AttributeError):
            _RING = False  # no host-mapped memory here: every call takes the event path
    return _RING or None


def _drop_entry(live: dict, key: int, ring) -> None:
    """The weak reference's callback: a forward output died before (or after) being saved."""
    e = live.pop(key, None)
    if e is not None and e.slot is not None:
        ring.release(e.slot)
        e.slot = None


class _Saved:
    """What autograd holds instead of a saved activation: the stream (and, until its size is
    checked, the activation itself), the activation's version counter value when it was saved and
    a weak reference to it (saved_tensors_hooks turn off autograd's own in-place check: _unpack
    repeats it), and the notify word its size arrives in (None: the event path)."""

    __slots__ = ("packed", "y", "codec", "version", "ref", "modified", "slot", "replay")

    def __init__(self, packed: SmaqPacked, y: torch.Tensor, codec: SmartFPPacked, version: int,
                 ref, slot: Optional[int] = None, replay: Optional[torch.nn.Module] = None):
        self.packed, self.y, self.codec = packed, y, codec
        self.version, self.ref, self.modified = version, ref, None
        self.slot = slot
        # an in-place activation module the saved value went through after the codec (its class
        # forward is replayed on the decoded stream: the same op on the same bits)
        self.replay = replay

    def check_version(self) -> None:
        """Raise autograd's in-place error when the saved activation was modified after it was
        saved (checked on the activation while it is held, at the size check before it is dropped,
        and through the weak reference while it lives)."""
        if self.modified is None:
            y = self.y if self.y is not None else self.ref()
            if y is None or y._version == self.version:
                return
            self.modified = (tuple(y.shape), y._version)
        shape, v = self.modified
        raise RuntimeError(
            "one of the variables needed for gradient computation has been modified by an inplace "
            f"operation: [torch.cuda.FloatTensor {list(shape)}], which is a SmaQ-compressed "
            f"activation saved as a packed stream; is at version {v}; expected version "
            f"{self.version} instead. (util/pytorch/saved.py: PackedActivations repeats autograd's "
            "check, which saved_tensors_hooks disable.)")


class _Entry:
    __slots__ = ("ref", "packed", "version", "shape", "stride", "dtype", "handle", "slot", "site",
                 "post")


# In-place activation modules whose op on a codec output can be replayed on its decoded stream:
# deterministic elementwise functions of the values alone whose in-place ATen op (one version bump)
# saves its result for backward. (Hardtanh / ReLU6 / SiLU / Hardswish / Hardsigmoid / Mish save a
# clone of their input instead: nothing of the codec output's storage is saved.) Exact types only.
_REPLAYABLE = (torch.nn.ReLU, torch.nn.LeakyReLU, torch.nn.ELU, torch.nn.CELU, torch.nn.SELU)


def replayable(module: torch.nn.Module) -> bool:
    """Whether PackedActivations can hold the output of ``module`` applied in place to a codec
    output as that output's stream plus the module (util/pytorch/autograd.py asks, per module)."""
    return type(module) in _REPLAYABLE and bool(getattr(module, "inplace", False))


class PackedActivations:
    def __init__(self, codec: SmartFPPacked, verify_bytes: Optional[int] = None,
                 overlap: bool = False, verify_batch: Optional[int] = None,
                 replay_inplace: bool = True):
        if not isinstance(codec, SmartFPPacked):
            raise TypeError("PackedActivations needs a SmartFPPacked codec")
        self.codec = codec
        # activations held while their sizes are on their way, before the host waits: notified
        # calls (a load per size) and the event path's batches (whose requests cost host time).
        # A larger budget lets the host run further ahead of the device (fewer waits) and holds
        # more activations at once: ResNet-34 / VGG packed steps at 32 / 64 / 256 MiB — 1.21 /
        # 1.18 / 1.13 and 1.22 / 1.16 / 1.12 x their SmartFP step, peaks 273 / 275 / 273 and
        # 238 / 263 / 314 MiB against 333 and 292 uncompressed (profiles/r6zb_saved_budget.txt)
        self.notify_bytes = int(verify_bytes) if verify_bytes is not None else 64 << 20
        # at the context's exit: wait until at most this much is still unchecked; what is left is
        # held into backward (its size words are read by later unpacks). Waiting for all of it
        # holds the host until the device has run the whole forward (ResNet-34: +0.6 ms per step)
        self.exit_bytes = self.notify_bytes
        self.verify_bytes = int(verify_bytes) if verify_bytes is not None else 32 << 20
        # the event path (calls without a notify word): a size request per verify_batch bytes of
        # saved activations (default: the budget; smaller batches cost more host time per step
        # than the waits they save, profiles/r6p_saved_ab.txt)
        self.verify_batch = int(verify_batch) if verify_batch is not None else self.verify_bytes
        # overlap: the packing launches of each forward call on a side stream (they wait for the
        # call's statistics, then run beside the next layers), with a ring of _RING workspaces
        self.overlap = bool(overlap)
        # in-place activations on codec outputs (note_inplace): their values held as the output's
        # stream with the activation replayed in backward (ResNet-34: step peak 275 -> 215 MiB, at
        # +0.2 ms of codec device time per step: the streams of the BN outputs the in-place ReLUs
        # change are packed and decoded, and the ReLUs replayed); False: saved as fp32
        self.replay_inplace = bool(replay_inplace)
        self._side: Dict[int, torch.cuda.Stream] = {}
        self._ring: Dict[int, List[list]] = {}  # device -> [[workspace, event recorded after], ...]
        self._ring_next = 0
        self._joined = True
        self._getter = N.ws_getter("smaq_pack")
        self._live: Dict[int, _Entry] = {}  # data_ptr of a forward output -> its stream
        self._pending: List[_Saved] = []     # saved, size not yet checked (y still held)
        self._pending_bytes = 0
        # saved with a notify word: size not read yet (y still held), in call order
        self._notified: Deque[_Saved] = deque()
        self._notified_bytes = 0
        self._notify: Optional[_NotifyRing] = None  # the process's ring, at the first C call
        # call sites (the k-th forward call of a step): packed this step, saved as streams this
        # step, and those whose packing is skipped (see _take_site)
        self._site = 0
        self._packed_sites: set = set()
        self._used_sites: set = set()
        self._skip: frozenset = frozenset()
        self._steps = 0
        self.skipped_packs = 0
        self.saved_replayed = 0  # of saved_packed: with an in-place activation replayed
        # batches whose sizes are on their way to the host: (event, pinned sizes, handles, bytes)
        self._inflight: Deque[tuple] = deque()
        self._inflight_bytes = 0
        self._hooks = None
        self.saved_packed = 0    # saved tensors held as streams (since construction)
        self.saved_bytes = 0     # the distinct verified streams' bytes
        self.saved_capacity = 0  # and the bytes allocated for them
        self.saved_elements = 0  # and their elements
        self.kept_fp32 = 0       # streams cut at their capacity (the activation kept instead)
        self.size_waits = 0      # times the host waited for a notify word (over the budget)
        self.size_wait_s = 0.0   # and the seconds it waited

    # -- the compress_fn of register_autograd_module ---------------------------------------------
    def __call__(self, x: torch.Tensor, tag: str = None, all_positive=False,
                 batch_norm_stats=None, **kw):
        codec = self.codec
        hp = codec.hparams
        if (self._hooks is None or tag != FORWARD_TAG or x.numel() < hp.min_size
                or not x.is_cuda):
            # a value nobody keeps as a stream (a grad-map, a call outside the context): SmartFP's
            # own call (one launch up to 8.4M elements), the values decompress(compress(x)) has
            return SmartFP.__call__(codec, x, tag=tag, all_positive=all_positive,
                                    batch_norm_stats=batch_norm_stats, **kw)
        site = self._take_site()
        if site in self._skip:  # its output was never saved as a stream lately: SmartFP's call
            self.skipped_packs += 1
            return SmartFP.__call__(codec, x, tag=tag, all_positive=all_positive,
                                    batch_norm_stats=batch_norm_stats, **kw)
        if not self.overlap and (batch_norm_stats is None or not hp.use_batch_norm):
            # the C call (csrc/torchfast.cpp smaq_packed): y and its stream in one call
            hot = codec._hot
            if hot is None:
                hot = codec._build_hot()
            r = None
            if hot is not False and Globals.profiler is None and codec._trace is None:
                slot, addr = self._arm()
                try:
                    r = N._torch_fast.smaq_packed(hot, x, all_positive, self._getter, ESCAPE_FRAC,
                                                  addr)
                    if r is NotImplemented:  # a flag changed: rebuild the state
                        hot = codec._build_hot()
                        r = (N._torch_fast.smaq_packed(hot, x, all_positive, self._getter,
                                                       ESCAPE_FRAC, addr)
                             if hot is not False else None)
                finally:
                    if slot is not None and (r is None or r is NotImplemented):
                        self._notify.release(slot, written=False)
            if r is not None and r is not NotImplemented:
                y, data = r
                return self._register(y, SmaqPacked(data, x.shape, x.numel(),
                                                    widths=(hp.num_bits_main,
                                                            hp.num_bits_outlier)), slot, site)
        n = x.numel()
        bn = batch_norm_stats is not None and hp.use_batch_norm
        channels = (1 if hp.bn_scalar_params else x.shape[1]) if bn else 0
        cap = stream_capacity(n, hp.num_bits_main, hp.num_bits_outlier, channels, ESCAPE_FRAC)
        # y and its stream from one statistics pass, the stream straight into a buffer of the
        # capacity (a stream that does not fit is flagged by its header: verify() keeps y then)
        if self.overlap:
            side, ws = self._slot(x.device, n)
            self._joined = False
            y, full = codec.roundtrip_compress(x, all_positive, batch_norm_stats, capacity=cap,
                                               pack_stream=side, workspace=ws[0])
            ws[1].record(side)  # this slot's workspace is free again once side has passed here
        else:
            y, full = codec.roundtrip_compress(x, all_positive, batch_norm_stats, capacity=cap)
        codec.log_size(tag, n * 32, lambda: full.nbytes * 8)
        return self._register(y, full, None, site)

    def _autograd_fast(self, x: torch.Tensor, backward: bool):
        """Compressor.forward for this compress_fn in C (util/pytorch/autograd.py): inside the
        context, the packed forward call and a C++ autograd node whose backward is the codec's plain
        call on the grad-map (as __call__ serves backward-direction calls); outside it, the codec's
        own C autograd path. None when the C path does not take the call (the Python Function
        then does: the same calls and values)."""
        codec = self.codec
        if self._hooks is None:
            return codec._autograd_fast(x, backward)
        if self.overlap or not x.is_cuda or Globals.profiler is not None or codec._trace is not None:
            return None
        hot = codec._hot
        if hot is None:
            hot = codec._build_hot()
        if hot is False:
            return None
        site = self._take_site()
        if site in self._skip:  # its output was never saved as a stream lately: SmartFP's C call
            r = codec._autograd_fast(x, backward)
            if r is None:  # (the Python Function then calls __call__, which takes this site)
                self._site -= 1
            else:
                self.skipped_packs += 1
            return r
        T = N._torch_fast
        slot, addr = self._arm()
        r = None
        try:
            r = T.smaq_packed_autograd(hot, x, self, backward, self._getter, ESCAPE_FRAC, addr)
            if r is NotImplemented:  # a flag changed: rebuild the state
                hot = codec._build_hot()
                r = (T.smaq_packed_autograd(hot, x, self, backward, self._getter, ESCAPE_FRAC,
                                            addr) if hot is not False else None)
        finally:
            if slot is not None and (r is None or r is NotImplemented):
                self._notify.release(slot, written=False)
        if r is None or r is NotImplemented:
            self._site -= 1  # (the Python Function then calls __call__, which takes this site)
            return None
        y, data = r
        hp = codec.hparams
        return self._register(y, SmaqPacked(data, x.shape, x.numel(),
                                            widths=(hp.num_bits_main, hp.num_bits_outlier)), slot,
                              site)

    # Forward calls whose outputs the model saves only after changing them in place (an in-place
    # ReLU, BasicBlock's `out += identity`) are packed for nothing: their stream no longer describes
    # the saved tensor. A model calls its codec in the same order every step, so the k-th forward
    # call of a step (its "site") whose stream was not saved in the last step runs as SmartFP's
    # own call the next time (the same values and random stream; the output is then saved as
    # itself, as it would have been). Every _REPROBE steps every site packs again, so a site whose
    # output starts being saved is found. ResNet-34: 60 of 132 packs per step skipped.
    _REPROBE = 64

    def _take_site(self) -> int:
        site = self._site
        self._site += 1
        return site

    def _arm(self):
        """(word index, its address) for the next C call's size notification, or (None, None)."""
        ring = self._notify
        if ring is None:
            ring = self._notify = _notify_ring()
            if ring is None:
                return None, None
        i = ring.take()
        return (None, None) if i is None else (i, ring.base + 4 * i)

    def _register(self, y: torch.Tensor, packed: SmaqPacked, slot: Optional[int] = None,
                  site: int = -1) -> torch.Tensor:
        """Remember y's stream (and the notify word its size arrives in) until autograd saves y
        (or y dies)."""
        e = _Entry()
        key = y.data_ptr()
        old = self._live.get(key)
        if old is not None and old.slot is not None:
            self._notify.release(old.slot)
        e.ref = weakref.ref(y, lambda _r, k=key, d=self._live, g=self._notify: _drop_entry(d, k, g))
        e.packed = packed
        e.version = y._version
        e.shape, e.stride, e.dtype = y.shape, y.stride(), y.dtype
        e.handle = None
        e.slot = slot
        e.site = site
        e.post = None
        self._live[key] = e
        self._packed_sites.add(site)
        return y

    _RING = 4

    def _slot(self, device: torch.device, n: int):
        """The side stream of device and the next ring slot [workspace, event], its workspace at
        least the packer's for n elements. The current stream waits (on the device) until the
        side stream has finished the slot's previous call."""
        di = device.index if device.index is not None else torch.cuda.current_device()
        side = self._side.get(di)
        if side is None:
            side = self._side[di] = torch.cuda.Stream(device)
            self._ring[di] = [[None, torch.cuda.Event()] for _ in range(self._RING)]
        slot = self._ring[di][self._ring_next % self._RING]
        self._ring_next += 1
        cur = torch.cuda.current_stream(device)
        cur.wait_event(slot[1])  # (a never-recorded event is complete)
        lib = N.lib()
        hp = self.codec.hparams
        k = min(n, hp.num_samples) if hp.use_sample_stats else 0
        need = (lib.smq_smaq_pack_workspace_bytes_sampled(n, k) if k
                else lib.smq_smaq_pack_workspace_bytes(n))
        if slot[0] is None or slot[0].numel() < need:
            # zero-filled once (the workspace needs no initialisation, include/smq.h); allocated
            # on the current stream, which has just waited for the old one's last side use
            slot[0] = torch.zeros(max(need, 1 << 20), dtype=torch.uint8, device=device)
        return side, slot

    def _join(self) -> None:
        """Order the current stream after every packing launch enqueued on the side streams."""
        for di, side in self._side.items():
            torch.cuda.current_stream(di).wait_stream(side)
        self._joined = True

    def note_inplace(self, module: torch.nn.Module, x) -> None:
        """An in-place activation module (``replayable``) is about to run on x: when x is a codec
        output of this step not modified since, remember the module, so that the value it leaves
        (one version later) is saved as x's stream with the module replayed on the decoded values
        (ResNet's ``relu(bn1(...))``: the stream of bn1's output instead of the fp32 activation).
        Called by register_autograd_module's wrapper before the module's forward."""
        if self._hooks is None or not self.replay_inplace or type(x) is not torch.Tensor:
            return
        e = self._live.get(x.data_ptr())  # (shape, strides, dtype: checked by _pack)
        if e is not None and e.version == x._version:
            e.post = (module, e.version)

    # -- saved_tensors_hooks ------------------------------------------------------------------------
    def _pack(self, t: torch.Tensor):
        key = t.data_ptr() if t.is_cuda else None
        e = self._live.get(key) if key is not None else None
        if e is None:
            return t  # not a forward output of this codec
        if t._version != e.version:  # modified in place since (e.g. an in-place ReLU): its stream
            post = e.post            # (with the op replayed, when note_inplace saw it coming)
            if (post is not None and t._version == post[1] + 1 and t.shape == e.shape
                    and t.stride() == e.stride and t.dtype == e.dtype):
                return self._save_replayed(e, t, post[0])
            if e.handle is None:     # no longer describes it
                self._live.pop(key, None)
                if e.slot is not None:  # (its notify word: nobody reads it now)
                    self._notify.release(e.slot)
                    e.slot = None
            return t
        if t.shape != e.shape or t.stride() != e.stride or t.dtype != e.dtype:
            return t  # a view of it
        y = e.ref()
        if y is None:
            return t
        self.saved_packed += 1
        if e.handle is not None:  # saved again (another consumer): the same stream
            return e.handle
        h = e.handle = _Saved(e.packed, y, self.codec, e.version, e.ref, e.slot)
        return self._hold(e, h, y)

    def _save_replayed(self, e: _Entry, t: torch.Tensor, module: torch.nn.Module):
        """t: the codec output of entry e after the in-place module op note_inplace recorded (one
        version later): held as e's stream and the module, replayed in _unpack."""
        y = e.ref()
        if y is None:
            return t
        self.saved_packed += 1
        self.saved_replayed += 1
        e.post = None
        e.version = t._version  # (a later save of the same value shares the handle)
        slot = e.slot if e.handle is None else None  # (else the earlier handle holds the word)
        h = e.handle = _Saved(e.packed, y, self.codec, e.version, e.ref, slot, replay=module)
        return self._hold(e, h, y)

    def _hold(self, e: _Entry, h: _Saved, y: torch.Tensor):
        """A new handle: its size comes through its notify word or the event path's batches."""
        self._used_sites.add(e.site)
        if e.slot is not None:  # its size arrives in a notify word: read, never requested
            e.slot = None  # (the handle holds the word now)
            self._notified.append(h)
            self._notified_bytes += 4 * y.numel()
            # the streams whose sizes are there drop their activations; more than the budget
            # still waiting: wait for the oldest ones (earlier calls, usually done by then)
            self._poll(self.notify_bytes)
            return h
        self._pending.append(h)
        self._pending_bytes += 4 * y.numel()
        if self._pending_bytes > self.verify_batch:
            self._request_sizes()
            # the batches whose sizes have arrived drop their activations; more than the budget
            # still in flight: wait for the oldest batches only (their work is usually done by
            # then; the batch just requested is waited for only when it alone exceeds the budget)
            self._harvest(self.verify_bytes)
        return h

    def _unpack(self, h):
        if isinstance(h, _Saved):
            if self._notified:  # the sizes that are there by now drop their activations
                self._poll(self.notify_bytes)
            h.check_version()
            if h.y is not None:  # not checked yet, or cut at its capacity: the activation itself
                return h.y
            if not self._joined:  # a backward inside the context: after the packing launches
                self._join()
            p = h.packed
            T = N._torch_fast
            if T is not None and p.widths is not None and p.dtype == torch.float32 and not p.raw:
                d = T.smaq_unpacked(p.data, tuple(p.shape), p.n, p.widths[0], p.widths[1])
            else:
                d = h.codec.decompress(p)
            if h.replay is not None:  # the in-place activation the saved value went through
                with torch.no_grad():
                    d = type(h.replay).forward(h.replay, d)
            return d
        return h

    def verify(self) -> None:
        """Check every pending stream's size against its capacity (waiting for the sizes still on
        their way); a stream that fits drops its activation, one that does not keeps it."""
        self._request_sizes()
        self._harvest(0)
        self._poll(0)

    def _poll(self, max_waiting_bytes: int) -> None:
        """Finish the notified handles whose size words are written, oldest first; wait for the
        oldest while more than max_waiting_bytes of activations still wait on theirs."""
        q, ring = self._notified, self._notify
        words = ring.words if ring is not None else None
        while q:
            h = q[0]
            total = int(words[h.slot])
            if total == N.SMQ_NOTIFY_PENDING:
                if self._notified_bytes <= max_waiting_bytes:
                    return
                total = self._wait_word(h)
            q.popleft()
            self._notified_bytes -= 4 * h.packed.n
            ring.release(h.slot)
            h.slot = None
            if total == N.SMQ_NOTIFY_SATURATED:  # 4 GiB or more: the header has the size
                total = int(h.packed.data[_TOTAL_OFF:_TOTAL_OFF + 8].view(torch.int64).item())
            self._finish(h, total)

    def _wait_word(self, h: _Saved) -> int:
        """Spin on h's notify word (its launch is queued before everything enqueued since). After
        a second without it, the stream is synchronised and the header read instead (a launch
        that did not notify: never expected)."""
        words, i = self._notify.words, h.slot
        t0 = time.perf_counter()
        spins = 0
        self.size_waits += 1
        while True:
            v = int(words[i])
            if v != N.SMQ_NOTIFY_PENDING:
                self.size_wait_s += time.perf_counter() - t0
                return v
            spins += 1
            if spins > 256:  # past ~50 us: short sleeps (which also let other threads run)
                if time.perf_counter() - t0 > 1.0:
                    torch.cuda.synchronize(h.packed.data.device)
                    v = int(words[i])
                    if v != N.SMQ_NOTIFY_PENDING:
                        return v
                    return int(h.packed.data[_TOTAL_OFF:_TOTAL_OFF + 8].view(torch.int64).item())
                time.sleep(1e-5)

    def _finish(self, h: _Saved, total: int) -> None:
        """h's stream size is known: drop the activation if the stream fitted its buffer."""
        cap = h.packed.data.numel()
        if h.y._version != h.version:  # modified in place since saved: backward raises
            h.modified = (tuple(h.y.shape), h.y._version)
        if total <= cap:
            h.packed._total = int(total)
            h.y = None
            self.saved_bytes += int(total)
            self.saved_capacity += cap
            self.saved_elements += h.packed.n
        else:  # did not fit its capacity: the activation stays the saved value
            h.packed = None
            self.kept_fp32 += 1

    def _request_sizes(self) -> None:
        """Every pending stream's header total_bytes, gathered on the device and copied to pinned
        host memory without synchronising; an event marks when they are there."""
        hs = self._pending
        if not hs:
            return
        dev = hs[0].packed.data.device
        # the headers are written by the packing launches: read them on their stream
        st = self._side.get(dev.index) if self.overlap else None
        with torch.cuda.stream(st if st is not None else torch.cuda.current_stream(dev)):
            sizes = torch.cat([h.packed.data[_TOTAL_OFF:_TOTAL_OFF + 8] for h in hs])
            host = torch.empty(sizes.numel(), dtype=torch.uint8, pin_memory=True)
            host.copy_(sizes, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        self._inflight.append((ev, host, hs, self._pending_bytes))
        self._inflight_bytes += self._pending_bytes
        self._pending = []
        self._pending_bytes = 0

    def _harvest(self, max_inflight_bytes: int) -> None:
        """Finish the batches whose sizes have arrived, oldest first; wait for the oldest while
        more than max_inflight_bytes of activations still wait on theirs."""
        while self._inflight:
            ev, host, hs, nbytes = self._inflight[0]
            if not ev.query():
                if self._inflight_bytes <= max_inflight_bytes:
                    return
                ev.synchronize()
            self._inflight.popleft()
            self._inflight_bytes -= nbytes
            for h, total in zip(hs, host.view(torch.int64).tolist()):
                self._finish(h, total)

    def __enter__(self):
        if self._notified:  # (handles of an earlier step whose sizes nobody has read yet)
            self._poll(self.notify_bytes)
        self._site = 0
        self._packed_sites = set()
        self._used_sites = set()
        self._hooks = torch.autograd.graph.saved_tensors_hooks(self._pack, self._unpack)
        self._hooks.__enter__()
        return self

    def __exit__(self, *exc):
        hooks, self._hooks = self._hooks, None
        try:
            self._join()  # backward decodes the streams on the current stream
            # the event path's batches are settled here; notified handles are waited for only down
            # to exit_bytes (waiting for all would hold the host until the device has run the whole
            # forward, and backward could not be enqueued behind it): the rest keep their
            # activation until their words are read — by the next save, unpack or context entry
            self._request_sizes()
            self._harvest(0)
            self._poll(self.exit_bytes)
            # the sites packed this step whose stream nobody saved are skipped from now on (with
            # the ones skipped already), until the next re-probe step packs every site again
            self._steps += 1
            if self._steps % self._REPROBE == 0:
                self._skip = frozenset()
            else:
                self._skip = frozenset(self._skip | (self._packed_sites - self._used_sites))
        finally:
            ring = self._notify
            for e in self._live.values():
                if e.slot is not None:
                    ring.release(e.slot)
                    e.slot = None
            self._live.clear()
            hooks.__exit__(*exc)
        return False

    def stats(self) -> Dict[str, Optional[float]]:
        """Saved tensors held as streams; bits per element of the verified streams (their real
        size and the capacity allocated for them); streams cut and kept as fp32."""
        el = self.saved_elements
        return {"saved_packed": self.saved_packed, "saved_elements": el,
                "saved_stream_bytes": self.saved_bytes,
                "bits_per_element": 8.0 * self.saved_bytes / el if el else None,
                "allocated_bits_per_element": 8.0 * self.saved_capacity / el if el else None,
                "kept_fp32": self.kept_fp32, "skipped_packs": self.skipped_packs,
                "saved_replayed": self.saved_replayed,
                "size_waits": self.size_waits,
                "size_wait_s": self.size_wait_s}
