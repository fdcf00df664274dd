"""Low-precision optimizer wrapper with the reference's surface, fused on MI355X.

Reference: smart_compress/util/pytorch/optimizer.py:37-180 (``OptimLP``) and
util/pytorch/hooks.py:22-34 (``wrap_optimizer``). Same constructor, same order of work per step:

* before the inner step (inside the closure): gradients ``g <- Q(g * grad_scaling)`` for every
  parameter with a gradient, skipping groups flagged ``no_grad_compression``; optional accumulator
  swap-in;
* after the inner step: gradients again, then weights ``w <- Q(w)`` (groups without
  ``no_weight_compression``, every parameter of the group), then momenta (SGD ``momentum_buffer``
  unless ``momentum == 0``; Adam/AdamW ``exp_avg`` and ``exp_avg_sq`` with ``all_positive=True``),
  skipping ``no_momentum_compression`` groups.

Fusion: when a quantiser is this package's ``SmartFP`` (wrapped by ``wrap_optimizer`` below), each
of those loops becomes ONE ``SmaqMulti`` call (two launches) that
rewrites the tensors in place, instead of one ``SmartFP.__call__`` (two launches + allocation) per
tensor. Per tensor the arithmetic is identical: own mean/std, own ``all_positive``, ``min_size``
passthrough, and the same ``optimizer_*`` compression-ratio logs when measuring. Any other
quantiser (or non-contiguous / non-fp32 tensor) is called per tensor exactly like the reference.
"""

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
from torch.optim import SGD, Adam, AdamW, Optimizer

from ... import _native as N
from ...compress.smart import SmartFP
from .multi import SmaqMulti

__all__ = ["OptimLP", "TaggedQuant", "wrap_optimizer"]


class TaggedQuant:
    """``compress_fn`` with a fixed tag (hooks.py:15-19) that stays introspectable for fusion."""

    def __init__(self, codec: Callable, tag: str):
        self.codec = codec
        self.tag = tag

    def __call__(self, *args, **kwargs):
        return self.codec(*args, tag=self.tag, **kwargs)


def wrap_optimizer(optimizer: Optimizer, compress_fn, hparams):
    """hooks.py:22-34: wrap with OptimLP for the enabled optimizer data structures."""
    quant = {}
    for flag, key, tag in (("compress_weights", "weight_quant", "optimizer_weight"),
                           ("compress_gradients", "grad_quant", "optimizer_grad"),
                           ("compress_momentum_vectors", "momentum_quant", "optimizer_momentum")):
        if getattr(hparams, flag, False):
            quant[key] = TaggedQuant(compress_fn, tag)
    return OptimLP(optimizer, **quant) if quant else optimizer


def _fusable(fn) -> Optional[SmartFP]:
    """The SmartFP behind a wrap_optimizer quantiser (any statistics mode: full, range-std or
    sampled — SmaqMulti computes each exactly as the per-tensor call would)."""
    if isinstance(fn, TaggedQuant) and isinstance(fn.codec, SmartFP):
        hp = fn.codec.hparams
        if hp.use_sample_stats and hp.num_samples > N.SMQ_MAX_DEVICE_SAMPLES:
            return None  # the multi-workgroup draw runs per tensor (SmartFP)
        return fn.codec
    return None


def _fusable_tensor(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()


class OptimLP(Optimizer):
    def __init__(self, optim: Optimizer, weight_quant=None, grad_scaling=1.0, grad_quant=None,
                 momentum_quant=None, acc_quant=None):
        super().__init__(optim.param_groups, optim.defaults)
        self.param_groups = optim.param_groups  # shared with the inner optimizer
        self.optim = optim
        assert grad_scaling > 0, "gradient scaling must be positive"
        self.grad_scaling = grad_scaling
        self.weight_quant = weight_quant
        self.grad_quant = grad_quant
        self.momentum_quant = momentum_quant
        self.acc_quant = acc_quant
        if isinstance(optim, SGD):
            self.momentum_keys: List[Tuple[str, Dict]] = [("momentum_buffer", {})]
        elif isinstance(optim, (Adam, AdamW)):
            self.momentum_keys = [("exp_avg", {}), ("exp_avg_sq", {"all_positive": True})]
        else:
            raise NotImplementedError("Only supporting Adam and SGD for now. ")
        if acc_quant is not None:
            self.weight_acc = {p: p.detach().clone().type_as(p)
                               for g in self.param_groups for p in g["params"]}
        self._multi: Dict[int, SmaqMulti] = {}

    # -- helpers -----------------------------------------------------------------------------------
    def _apply(self, fn, tensors: Sequence[torch.Tensor], all_pos: Sequence[bool],
               assign: Callable[[int, torch.Tensor], None], inplace: bool = True):
        """Quantise ``tensors`` with ``fn``: one fused launch pair when possible (in place, or into
        new tensors handed to ``assign`` when the inputs' storage must survive), else the
        reference's per-tensor calls with their results handed to ``assign``."""
        codec = _fusable(fn)
        fused = [i for i, t in enumerate(tensors) if codec is not None and _fusable_tensor(t)]
        if fused:
            multi = self._multi.get(id(fn))
            if multi is None:
                multi = self._multi[id(fn)] = SmaqMulti(codec.hparams, rng=codec.rng)
            multi._graph_safe = codec._graph_safe  # same stream, same mode (device counter or host)
            xs = [tensors[i] for i in fused]
            ys = multi(xs, xs if inplace else None, all_positive=[all_pos[i] for i in fused])
            self._log_fused(codec, fn.tag, multi, xs)
            if not inplace:
                for i, y in zip(fused, ys):
                    if y is not tensors[i]:  # below min_size the reference returns the input
                        assign(i, y)
        done = set(fused)
        for i, t in enumerate(tensors):
            if i not in done:
                kwargs = {"all_positive": True} if all_pos[i] else {}
                assign(i, fn(t, **kwargs))

    # the per-tensor log_size values of a fused call stay on the device (SmaqMulti.size_records:
    # no host synchronisation per optimizer step); False: read the counts on the host instead
    device_metrics = True

    @classmethod
    def _log_fused(cls, codec: SmartFP, tag: str, multi: SmaqMulti, xs: Sequence[torch.Tensor]):
        hp = codec.hparams
        if not hp.measure_compression_ratio:
            return
        recs = multi.size_records() if cls.device_metrics and multi.last_selected else None
        stats = multi.read_stats() if recs is None and multi.last_selected else []
        for t, x in enumerate(xs):
            n = x.numel()
            if n < hp.min_size:
                codec.log_ratio(tag, n * 32, 32, 32)  # smart.py:125
                continue
            if recs is not None:
                _, new, ratio, orig = recs[multi.index_of(t)].unbind()
                codec._log_size_record(tag, ratio, new, orig)
                continue
            n_out = stats[multi.index_of(t)]["n_outlier"]
            codec.log_size(tag, n * 32, n_out * hp.num_bits_outlier + (n - n_out) * hp.num_bits_main)

    def _grads(self):
        ps = [p for g in self.param_groups if not g.get("no_grad_compression", False)
              for p in g["params"] if p.requires_grad and p.grad is not None]
        if not ps:
            return
        if self.grad_scaling != 1.0 and _fusable(self.grad_quant) is not None:
            for p in ps:
                p.grad.data.mul_(self.grad_scaling)
            tensors = [p.grad.data for p in ps]
        elif self.grad_scaling != 1.0:
            tensors = [p.grad.data * self.grad_scaling for p in ps]
        else:
            tensors = [p.grad.data for p in ps]

        def assign(i, q):
            ps[i].grad.data = q.data

        self._apply(self.grad_quant, tensors, [False] * len(ps), assign)

    def _pre_closure(self):
        if self.grad_quant is not None:
            self._grads()
        if self.acc_quant is not None:
            for g in self.param_groups:
                for p in g["params"]:
                    p.data = self.weight_acc[p].data

    def _post_closure(self):
        if self.grad_quant is not None:
            self._grads()
        if self.weight_quant is not None:
            ps = [p for g in self.param_groups if not g.get("no_weight_compression", False)
                  for p in g["params"]]

            def assign_w(i, q):
                ps[i].data = q.data

            # with an accumulator, p.data IS weight_acc[p] (swapped in by _pre_closure): the
            # reference's `p.data = weight_quant(p.data).data` leaves the full-precision
            # accumulator intact, so the fused launch must not write in place then
            self._apply(self.weight_quant, [p.data for p in ps], [False] * len(ps), assign_w,
                        inplace=self.acc_quant is None)
        if self.momentum_quant is not None:
            slots = []
            for g in self.param_groups:
                if g.get("no_momentum_compression", False):
                    continue
                if isinstance(self.optim, SGD) and g["momentum"] == 0:
                    continue
                for p in g["params"]:
                    if not p.requires_grad or p.grad is None:
                        continue
                    state = self.optim.state[p]
                    for key, kw in self.momentum_keys:
                        slots.append((state, key, bool(kw.get("all_positive", False))))
            if slots:
                def assign_m(i, q):
                    state, key, _ = slots[i]
                    state[key].data = q.data

                self._apply(self.momentum_quant, [s[key] for s, key, _ in slots],
                            [ap for _, _, ap in slots], assign_m)

    def step(self, closure=None):
        """Quantise gradients (inside the closure), step, then quantise gradients, weights and
        momenta. Unlike the reference, a missing closure does not raise: the gradients are then
        quantised before the inner step."""
        if closure is None:
            self._pre_closure()
            loss = self.optim.step()
        else:
            def closure_(*args, **kwargs):
                value = closure(*args, **kwargs)
                self._pre_closure()
                return value

            loss = self.optim.step(closure=closure_)
        self._post_closure()
        return loss

    def __repr__(self):
        return "LP Optimizer: {}".format(self.optim.__repr__())

    def __str__(self):
        return "LP Optimizer: {}".format(self.optim.__str__())
