"""Multi-tensor SmaQ: one fused call for a list of tensors (grads / weights / momenta).

Reference: util/pytorch/optimizer.py:69-127 runs ``SmartFP.__call__`` once per parameter tensor
(a ResNet-34 step: 148 tensors, median 256 elements, each call ~24 ATen launches + 1 host sync).
``SmaqMulti`` computes exactly what those per-tensor calls compute — each tensor keeps its own
mean/std (full statistics), its own ``all_positive`` flag and passthrough below ``min_size`` — in
two launches of libsmq (``smq_smaq_multi_f32``) for the whole list.

The plan (descriptor table + chunk map) is cached by the list's pointers and sizes, so a training
loop whose parameter and gradient buffers stay put uploads it once.
"""

import copy
import ctypes
from typing import List, Optional, Sequence

import numpy as np
import torch

from ... import _native as N
from ...compress.smart import SmartFP


class SmaqMulti:
    def __init__(self, hparams, seed: Optional[int] = None, rng: Optional[N.RngState] = None):
        if hparams.use_sample_stats or hparams.use_range_std_dev:
            raise NotImplementedError("SmaqMulti supports full statistics only")
        self.hparams = hparams
        internal = copy.copy(hparams)
        internal.smq_seed = 0  # the internal codec only builds parameter blocks: no torch RNG draw
        self._codec = SmartFP(internal)
        if rng is None:
            rng = N.RngState(seed if seed is not None else getattr(hparams, "smq_seed", None))
        self.rng = rng  # shared with a SmartFP codec when fused into its optimizer calls
        self._plans = {}
        self._last = None
        self._p = None
        self._graph_safe = False

    def _plan(self, xs, ys, allpos, device):
        key = tuple((x.data_ptr(), y.data_ptr(), x.numel(), a) for x, y, a in zip(xs, ys, allpos))
        hit = self._plans.get(key)
        if hit is not None:
            return hit
        count = len(xs)
        descs = (N.SmqTensorDesc * count)()
        rel = 0
        offsets = []
        for i, (x, y, a) in enumerate(zip(xs, ys, allpos)):
            descs[i].x, descs[i].y, descs[i].n = x.data_ptr(), y.data_ptr(), x.numel()
            descs[i].all_positive = 1 if a else 0
            descs[i].rng_offset = rel
            offsets.append(rel)
            rel += x.numel()
        sizes = (ctypes.c_int64 * count)(*[x.numel() for x in xs])
        lib = N.lib()
        nbytes = lib.smq_smaq_multi_plan_bytes(sizes, count)
        host = (ctypes.c_uint8 * nbytes)()
        N.check(lib.smq_smaq_multi_plan_build(descs, count, host, nbytes), "multi_plan_build")
        host_t = torch.frombuffer(bytearray(bytes(host)), dtype=torch.uint8)
        dev_t = host_t.to(device)
        ws_bytes = lib.smq_smaq_multi_workspace_bytes(sizes, count)
        ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=device)
        plan = dict(host=host, dev=dev_t, ws=ws, offsets=offsets, total=rel, count=count)
        if len(self._plans) > 16:
            self._plans.clear()
        self._plans[key] = plan
        return plan

    def _select(self, xs, ys, all_positive):
        hp = self.hparams
        if all_positive is None:
            all_positive = [False] * len(xs)
        elif isinstance(all_positive, bool):
            all_positive = [all_positive] * len(xs)
        sel, sx, sy, sa = [], [], [], []
        for i, (x, y) in enumerate(zip(xs, ys)):
            if x.numel() < hp.min_size:
                if y is not x:
                    y.copy_(x)
                continue
            N.require_device_f32(x, "SmaqMulti")
            if not (x.is_contiguous() and y.is_contiguous() and y.dtype == torch.float32
                    and y.numel() == x.numel()):
                raise RuntimeError("SmaqMulti needs contiguous float32 tensors of equal size")
            sel.append(i)
            sx.append(x)
            sy.append(y)
            sa.append(bool(all_positive[i]))
        return sel, sx, sy, sa

    def _launch(self, plan, sel, device):
        p = self._p
        if p is None:  # built once: the C call reads it synchronously, only seed/offset change
            p = self._p = self._codec._params(1, False)
            p.stats_source = N.SMQ_STATS_WORKSPACE
            p.count_outliers = 1 if self.hparams.measure_compression_ratio else 0
        if self._graph_safe:
            p.seed, p.offset = self.rng.seed, 0
            p.offset_counter = self.rng.counter(device).data_ptr()
        else:
            p.seed, p.offset = self.rng.take(plan["total"])
            p.offset_counter = None
        N.check(N.lib().smq_smaq_multi_f32(
            plan["dev"].data_ptr(), ctypes.addressof(plan["host"]), p, plan["ws"].data_ptr(),
            plan["ws"].numel(), N.stream_ptr(device)), "smq_smaq_multi_f32")
        self._last = dict(plan=plan, sel=sel, base=None if self._graph_safe else p.offset)

    @torch.no_grad()
    def __call__(self, xs: Sequence[torch.Tensor], ys: Optional[Sequence[torch.Tensor]] = None,
                 all_positive=None) -> List[torch.Tensor]:
        """Quantise-dequantise every ``xs[i]`` into ``ys[i]`` (new tensors if ``ys`` is None; may
        alias ``xs`` for in-place). Tensors below ``min_size`` are passed through."""
        hp = self.hparams
        if ys is None:
            ys = [torch.empty_like(x) if x.numel() >= hp.min_size else x for x in xs]
        sel, sx, sy, sa = self._select(xs, ys, all_positive)
        self._last = None
        if not sel:
            return list(ys)
        device = sx[0].device
        self._launch(self._plan(sx, sy, sa, device), sel, device)
        return list(ys)

    def bind(self, xs: Sequence[torch.Tensor], ys: Sequence[torch.Tensor],
             all_positive=None) -> "BoundSmaqMulti":
        """Validate a FIXED list of buffers once (parameters, optimizer state, preallocated
        outputs) and return a callable that only draws the random stream and launches: no
        per-tensor Python work per call. The buffers must keep their storage while bound."""
        sel, sx, sy, sa = self._select(xs, ys, all_positive)
        for i, (x, y) in enumerate(zip(xs, ys)):
            if i not in sel and y is not x:
                raise RuntimeError("bind: tensors below min_size must be passed as ys[i] = xs[i]")
        device = sx[0].device if sx else None
        plan = self._plan(sx, sy, sa, device) if sel else None
        return BoundSmaqMulti(self, plan, sel, device, list(ys))

    # -- inspection (tests, logging) ---------------------------------------------------------------
    @property
    def last_selected(self) -> bool:
        """Whether the last call quantised at least one tensor (others were below min_size)."""
        return self._last is not None

    def index_of(self, t: int) -> int:
        return self._last["sel"].index(t)

    def graph_safe(self, enable: bool = True, device=None):
        """Device-counter random stream (``SmqSmaqParams.offset_counter``): bound calls captured
        in a hipGraph draw fresh streams on every replay. Shares ``self.rng`` (and so its counter)
        with the SmartFP codec it was built from. ``offset_of`` is unavailable in this mode."""
        self._graph_safe = bool(enable)
        if enable and device is not None:
            self.rng.counter(device)
        if not enable:
            self.rng.release_counters()
        return self

    def offset_of(self, t: int) -> int:
        last = self._last
        if last["base"] is None:
            raise RuntimeError("offset_of: the stream position is on the device (graph-safe mode)")
        return last["base"] + last["plan"]["offsets"][last["sel"].index(t)]

    def read_stats(self):
        plan = self._last["plan"]
        raw = plan["ws"][: 64 * plan["count"]].cpu().numpy()
        out = []
        for t in range(plan["count"]):
            r = raw[64 * t: 64 * (t + 1)]
            f = r[:24].view(np.float32)
            out.append(dict(mean=float(f[0]), std_dev=float(f[1]), std_clamped=float(f[2]),
                            raw_std=float(f[3]), n_outlier=int(r[32:40].view(np.uint64)[0])))
        return out


class BoundSmaqMulti:
    """``SmaqMulti.bind`` result: one call = the two launches of the bound list."""

    def __init__(self, multi: SmaqMulti, plan, sel, device, ys):
        self.multi, self.plan, self.sel, self.device, self.ys = multi, plan, sel, device, ys

    @torch.no_grad()
    def __call__(self) -> List[torch.Tensor]:
        if self.plan is not None:
            self.multi._launch(self.plan, self.sel, self.device)
        return self.ys
