"""Multi-tensor SmaQ: one fused call for a list of tensors (grads / weights / momenta).

Reference: util/pytorch/optimizer.py:69-127 runs ``SmartFP.__call__`` once per parameter tensor
(a ResNet-34 step: 148 tensors, median 256 elements, each call ~24 ATen launches + 1 host sync).
``SmaqMulti`` computes exactly what those per-tensor calls compute — each tensor keeps its own
statistics (full, range-std or device-drawn samples: smart.py:86-108), its own ``all_positive``
flag and passthrough below ``min_size`` — in two launches of libsmq (``smq_smaq_multi``) per input
dtype of the list (fp32 / fp16 / bf16; outputs fp32 like the single-tensor path), plus the
single-tensor statistics launch of each tensor above 8,388,611 elements. Each tensor's statistics
are computed in the single-tensor call's partition and reduction order, so the outputs equal the
per-tensor calls at the same stream offsets bit for bit.

The plan (descriptor table + chunk map) is cached by the list's pointers and sizes, so a training
loop whose parameter and gradient buffers stay put uploads it once.
"""

import copy
import ctypes
from typing import List, Optional, Sequence

import numpy as np
import torch

from ... import _native as N
from ...compress.smart import SmartFP, range_std_coef


class SmaqMulti:
    def __init__(self, hparams, seed: Optional[int] = None, rng: Optional[N.RngState] = None):
        if hparams.use_sample_stats and min(hparams.num_samples, 1 << 30) > N.SMQ_MAX_DEVICE_SAMPLES:
            raise NotImplementedError(
                f"--num_samples {hparams.num_samples} > {N.SMQ_MAX_DEVICE_SAMPLES} is not supported")
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

    def _plan(self, xs, ys, allpos, rels, device):
        """Plan of one dtype group; rels = each tensor's stream offset within the whole call."""
        key = tuple((x.data_ptr(), y.data_ptr(), x.numel(), a, r, x.dtype)
                    for x, y, a, r in zip(xs, ys, allpos, rels))
        hit = self._plans.get(key)
        if hit is not None:
            return hit
        hp = self.hparams
        count = len(xs)
        descs = (N.SmqTensorDesc * count)()
        for i, (x, y, a, r) in enumerate(zip(xs, ys, allpos, rels)):
            descs[i].x, descs[i].y, descs[i].n = x.data_ptr(), y.data_ptr(), x.numel()
            descs[i].all_positive = 1 if a else 0
            descs[i].rng_offset = r
            descs[i].range_std_coef = -1.0
            if hp.use_range_std_dev:  # C of the n (or k sampled) elements, in the tensor's dtype
                m = min(x.numel(), hp.num_samples) if hp.use_sample_stats else x.numel()
                descs[i].range_std_coef = range_std_coef(m, x.dtype)
        sizes = (ctypes.c_int64 * count)(*[x.numel() for x in xs])
        lib = N.lib()
        nbytes = lib.smq_smaq_multi_plan_bytes(sizes, count)
        host = (ctypes.c_uint8 * nbytes)()
        N.check(lib.smq_smaq_multi_plan_build(descs, count, host, nbytes), "multi_plan_build")
        host_t = torch.frombuffer(bytearray(bytes(host)), dtype=torch.uint8)
        dev_t = host_t.to(device)
        ws_bytes = lib.smq_smaq_multi_workspace_bytes(sizes, count)
        ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=device)
        plan = dict(host=host, dev=dev_t, ws=ws, count=count, dtype=N.DTYPE_CODES[xs[0].dtype],
                    n=torch.tensor([x.numel() for x in xs], dtype=torch.int64, device=device),
                    rels=list(rels))
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
            N.require_device(x, "SmaqMulti")
            if x.dtype not in N.DTYPE_CODES:
                raise NotImplementedError(f"SmaqMulti: dtype {x.dtype} is not supported")
            if x.dtype == torch.float16 and hp.precision != 16:
                # the reference's std.clamp(1e-38, 1e38) on a half tensor (smart.py:154)
                raise RuntimeError("value cannot be converted to type c10::Half without overflow")
            if not (x.is_contiguous() and y.is_contiguous() and y.dtype == torch.float32
                    and y.numel() == x.numel()):
                raise RuntimeError("SmaqMulti needs contiguous inputs and float32 outputs of equal "
                                   "size")
            if x.dtype != torch.float32 and y.data_ptr() == x.data_ptr():
                raise RuntimeError("SmaqMulti: fp16 / bf16 inputs give fp32 outputs; y cannot "
                                   "alias x")
            sel.append(i)
            sx.append(x)
            sy.append(y)
            sa.append(bool(all_positive[i]))
        return sel, sx, sy, sa

    def _groups(self, sx, sy, sa, device):
        """One plan per input dtype (list order kept inside each); rels over the whole list."""
        rels, rel = [], 0
        for x in sx:
            rels.append(rel)
            rel += x.numel()
        by = {}
        for j, x in enumerate(sx):
            by.setdefault(x.dtype, []).append(j)
        if len(by) > 1 and self._graph_safe:
            raise NotImplementedError("SmaqMulti: a graph-safe call takes one input dtype")
        plans = [self._plan([sx[j] for j in js], [sy[j] for j in js], [sa[j] for j in js],
                            [rels[j] for j in js], device) for js in by.values()]
        return plans, rels, rel

    def _params(self):
        p = self._p
        if p is None:  # built once: the C call reads it synchronously, only seed/offset change
            hp = self.hparams
            p = self._p = self._codec._params(1, False)
            if hp.use_sample_stats:
                p.stats_source = N.SMQ_STATS_SAMPLED_DEVICE
                p.num_samples = hp.num_samples
            else:
                p.stats_source = N.SMQ_STATS_WORKSPACE
            p.count_outliers = 1 if hp.measure_compression_ratio else 0
        return p

    def _launch(self, plans, rels, total, sel, device):
        p = self._params()
        if self._graph_safe:
            p.seed, p.offset = self.rng.seed, 0
            p.offset_counter = self.rng.counter(device).data_ptr()
        else:
            p.seed, p.offset = self.rng.take(total)
            p.offset_counter = None
        st = N.stream_ptr(device)
        lib = N.lib()
        fn = lib.smq_smaq_multi
        hp = self.hparams
        metrics = [] if hp.measure_compression_ratio else None
        for plan in plans:
            rc = fn(plan["dev"].data_ptr(), ctypes.addressof(plan["host"]), plan["dtype"], p,
                    plan["ws"].data_ptr(), plan["ws"].numel(), st)
            if rc:
                N.check(rc, "smq_smaq_multi")
            if metrics is not None:
                # the per-tensor log_size values on the device (no host synchronisation): one
                # small launch reads every tensor's outlier count from its statistics record
                out = torch.empty((plan["count"], 4), dtype=torch.float64, device=device)
                N.check(lib.smq_smaq_multi_size_metrics(
                    plan["ws"].data_ptr(), plan["n"].data_ptr(), plan["count"], hp.num_bits_main,
                    hp.num_bits_outlier, out.data_ptr(), st), "smq_smaq_multi_size_metrics")
                metrics.append(out)
        self._last = dict(plans=plans, rels=rels, sel=sel, metrics=metrics,
                          base=None if self._graph_safe else p.offset)

    @torch.no_grad()
    def __call__(self, xs: Sequence[torch.Tensor], ys: Optional[Sequence[torch.Tensor]] = None,
                 all_positive=None) -> List[torch.Tensor]:
        """Quantise-dequantise every ``xs[i]`` into ``ys[i]`` (new fp32 tensors if ``ys`` is None;
        may alias fp32 ``xs`` for in-place). Tensors below ``min_size`` are passed through."""
        hp = self.hparams
        if ys is None:
            ys = [torch.empty(x.shape, dtype=torch.float32, device=x.device)
                  if x.numel() >= hp.min_size else x for x in xs]
        sel, sx, sy, sa = self._select(xs, ys, all_positive)
        self._last = None
        if not sel:
            return list(ys)
        device = sx[0].device
        plans, rels, total = self._groups(sx, sy, sa, device)
        self._launch(plans, rels, total, sel, device)
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
        groups = self._groups(sx, sy, sa, device) if sel else None
        return BoundSmaqMulti(self, groups, sel, device, list(ys))

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
        return last["base"] + last["rels"][last["sel"].index(t)]

    def size_records(self):
        """--measure_compression_ratio: per selected tensor of the last call (list order), its fp64
        device values [n_outlier, new_size, compression_ratio, orig_size] (smart.py:184-188),
        written by smq_smaq_multi_size_metrics — read without a host synchronisation."""
        last = self._last
        if last is None or last["metrics"] is None:
            return None
        out = [None] * len(last["sel"])
        pos = {r: j for j, r in enumerate(last["rels"])}
        for plan, m in zip(last["plans"], last["metrics"]):
            for t, row in zip(range(plan["count"]), m.unbind()):
                out[pos[plan["rels"][t]]] = row
        return out

    def read_stats(self):
        """Statistics of the last call's selected tensors, in list order."""
        last = self._last
        out = [None] * len(last["sel"])
        # tensors of each plan in list order: map back through the rels (unique per tensor)
        pos = {r: j for j, r in enumerate(last["rels"])}
        for plan in last["plans"]:
            raw = plan["ws"][: 64 * plan["count"]].cpu().numpy()
            descs = np.frombuffer(bytes(plan["host"])[32: 32 + 40 * plan["count"]], dtype=np.uint8)
            for t in range(plan["count"]):
                r = raw[64 * t: 64 * (t + 1)]
                f = r[:24].view(np.float32)
                rel = int(descs[40 * t + 32: 40 * t + 40].view(np.uint64)[0])
                out[pos[rel]] = dict(mean=float(f[0]), std_dev=float(f[1]),
                                     std_clamped=float(f[2]), raw_std=float(f[3]),
                                     n_outlier=int(r[32:40].view(np.uint64)[0]))
        return out


class BoundSmaqMulti:
    """``SmaqMulti.bind`` result: one call = the two launches per dtype group of the bound list."""

    def __init__(self, multi: SmaqMulti, groups, sel, device, ys):
        self.multi, self.groups, self.sel, self.device, self.ys = multi, groups, sel, device, ys

    @torch.no_grad()
    def __call__(self) -> List[torch.Tensor]:
        if self.groups is not None:
            plans, rels, total = self.groups
            self.multi._launch(plans, rels, total, self.sel, self.device)
        return self.ys
