"""SmaQ codec on MI355X: drop-in for smart_compress/compress/smart.py:10-190 (``SmartFP``).

Same class name, argparse flags and defaults (smart.py:11-70), hparams fields, constants
(smart.py:72-84), ``__call__(data, tag=None, all_positive=False, batch_norm_stats=None, **_)``
signature, passthrough of tensors with fewer than ``min_size`` elements (returns the same object,
smart.py:123-128) and ``log_size`` metrics (smart.py:184-188).

Below the boundary, the reference's ~24 ATen launches + one host sync (smart.py:151) become one or
two launches of libsmq (include/smq.h):

* full statistics (default): ``smq_smaq_roundtrip`` — up to 8,388,611 elements ONE launch that
  holds the tensor in registers (8 B/elem of traffic), above it statistics + apply (12 B/elem);
* ``--use_sample_stats``: ``smq_smaq_apply`` with ``SMQ_STATS_SAMPLED_DEVICE``: a one-workgroup
  launch draws k distinct indices (Floyd, on the device, from the call's stream position),
  gathers them and writes mean / biased std, then the apply launch (8 B/elem).

Randomness: the reference draws ``torch.rand_like`` (smart.py:94) and ``torch.randperm`` (88); here a
counter-based RNG keyed by ``(seed, offset)`` held on the codec (``self.rng``), for the rounding
draws and the sample indices alike — the seed comes from
torch's default generator at construction (so ``torch.manual_seed`` makes runs repeatable) or from
``hparams.smq_seed``; the offset advances by the elements consumed per call.
"""

import ctypes
from argparse import ArgumentParser, Namespace
from typing import Optional, Tuple

import numpy as np
import torch

from .. import _native as N
from ..util.globals import Globals, profile
from .base import CompressionAlgorithmBase, _reduce_fx

_F32 = {}
_WS_BYTES = {}  # (numel, device-drawn samples or -1) -> workspace bytes


def _f32(v: float) -> float:
    """The fp32 value of a Python number (what torch's fp32 scalar ops see), memoised: the flags'
    constants repeat on every call, and a numpy conversion costs ~0.75 us of host time each."""
    r = _F32.get(v)
    if r is None:
        if len(_F32) > 1024:  # (NaN keys never hit; keep the table bounded)
            _F32.clear()
        r = _F32[v] = float(np.float32(v))
    return r

# (flag, argparse kwargs) exactly as smart.py:11-70 declares them
_SMAQ_FLAGS = (
    ("--num_samples", dict(type=int, default=16,
                           help="number of samples to use for mean/std_dev calculation")),
    ("--use_sample_stats", dict(action="store_true",
                                help="use sample mean and std for smart compression")),
    ("--no_stochastic_rounding", dict(action="store_false", dest="stochastic_rounding",
                                      help="use stochastic rounding when quantizing")),
    ("--num_bits_main", dict(type=int, default=6,
                             help="number of bits for main data (within 1 std dev)")),
    ("--num_bits_outlier", dict(type=int, default=8,
                                help="number of bits for outlier data (more than 1 std dev)")),
    ("--main_std_dev_threshold", dict(type=float, default=1.0,
                                      help="std dev to consider something main")),
    ("--outlier_std_dev_threshold", dict(
        type=float, default=2.5,
        help="max std dev for outliers (everything else is clamped to this)")),
    ("--min_size", dict(type=int, default=8)),
    ("--use_range_std_dev", dict(action="store_true",
                                 help="use range std dev (from range batch norm paper)")),
    ("--use_batch_norm", dict(action="store_true", help="support BN acceleration")),
    ("--bn_scalar_params", dict(action="store_true", help="BN params should be scalar")),
)

_range_coef_cache = {}
_SIZE_FX = {"reduce_fx": _reduce_fx, "tbptt_reduce_fx": _reduce_fx}  # base.py's "*size*" metrics


def quot_check_for(sc: float) -> int:
    """Host mirror of smaq_elem.h ``quot_check_for`` (tests): 1 when the element transform keeps
    the subnormal-quotient check for this clamped std (an even integer, or >= 2^24)."""
    sc = float(np.float32(sc))
    h = float(np.float32(sc * 0.5))
    even_int = h == float(np.trunc(h)) and h != 0.0
    return 1 if (even_int or not abs(sc) < 2.0**24) else 0


def range_std_coef(n: int, dtype: torch.dtype = torch.float32) -> float:
    """C = 1 / sqrt(2 log n) evaluated with the reference's torch ops in the data's dtype
    (smart.py:101-106: ``torch.tensor(numel).type_as(range_)``; for half data n > 65504 becomes
    inf and C = 0, which the std == 0 rule then turns into std = 1, as in the reference)."""
    key = (n, dtype)
    c = _range_coef_cache.get(key)
    if c is None:
        t = torch.tensor(n).type_as(torch.tensor(0.0, dtype=dtype))
        c = float(1 / torch.sqrt(2.0 * torch.log(t)))
        _range_coef_cache[key] = c
    return c


class SmartFP(CompressionAlgorithmBase):
    @staticmethod
    def add_argparse_args(parent_parser: ArgumentParser) -> ArgumentParser:
        parser = ArgumentParser(
            parents=[CompressionAlgorithmBase.add_argparse_args(parent_parser)], add_help=False
        )
        for flag, kwargs in _SMAQ_FLAGS:
            parser.add_argument(flag, **kwargs)
        return parser

    def __init__(self, hparams: Namespace):
        super().__init__(hparams)
        hp = self.hparams
        # Python doubles, rounded to fp32 where the kernels use them (smart.py:72-84)
        main_codes = (2 ** (hp.num_bits_main - 2)) - 1
        outlier_codes = (2 ** (hp.num_bits_outlier - 2)) - 1
        self.range_outlier = outlier_codes / (
            hp.outlier_std_dev_threshold - hp.main_std_dev_threshold
        )
        self.range_normal = main_codes / hp.main_std_dev_threshold
        self.clamped_range = (1e-4, 1e4) if hp.precision == 16 else (1e-38, 1e38)
        self.rng = N.RngState(getattr(hp, "smq_seed", None))
        self._graph_safe = False
        self._templates = {}  # flag templates of the parameter block (_hot_params)

    # -- graph-safe random stream ----------------------------------------------------------------
    def graph_safe(self, enable: bool = True, device=None):
        """Keep the random-stream position in a device counter (``SmqSmaqParams.offset_counter``,
        ``self.rng.counter``) instead of advancing ``self.rng.offset`` on the host, so calls
        captured in a hipGraph (``torch.cuda.graph``) draw fresh, consecutive random streams on
        every replay. The stream continues from the host position; create the counter before
        capturing (pass ``device`` or make one eager call first). Values are identical to the
        host-offset mode for the same sequence of calls. ``graph_safe(False)`` continues on the
        host from the device position (one host synchronisation)."""
        self._graph_safe = bool(enable)
        if enable and device is not None:
            self.rng.counter(device)
        if not enable:
            self.rng.release_counters()
        return self

    # -- parameter block -------------------------------------------------------------------------
    def _params(self, numel: int, all_positive: bool,
                dtype: torch.dtype = torch.float32, device=None) -> N.SmqSmaqParams:
        hp = self.hparams
        p = self._flag_params(all_positive)
        self._stream_fields(p, numel, device)
        if hp.use_sample_stats:
            # smart.py:86-91: k indices drawn on the device (Floyd) from this call's stream
            # position, so eager calls and graph replays alike see a fresh set (smart.py:88)
            k = min(numel, hp.num_samples)
            if k > N.SMQ_MAX_DRAW_SAMPLES:
                raise NotImplementedError(
                    f"--num_samples {hp.num_samples} > {N.SMQ_MAX_DRAW_SAMPLES} is not supported"
                )
            p.stats_source = N.SMQ_STATS_SAMPLED_DEVICE
            p.num_samples = k
            if hp.use_range_std_dev:
                self._set_range_coef(p, k, dtype)
        elif hp.use_range_std_dev:
            self._set_range_coef(p, numel, dtype)
        return p

    def _flag_params(self, all_positive: bool) -> N.SmqSmaqParams:
        """The fields of the parameter block that follow from the flags alone (full statistics
        from the workspace; the caller adds the stream position and the per-size fields)."""
        hp = self.hparams
        p = N.SmqSmaqParams()
        p.num_bits_main = hp.num_bits_main
        p.num_bits_outlier = hp.num_bits_outlier
        p.main_std_dev_threshold = _f32(hp.main_std_dev_threshold)
        p.range_main = _f32(self.range_normal)
        p.range_outlier = _f32(self.range_outlier)
        p.clamp_lo = _f32(self.clamped_range[0])
        p.clamp_hi = _f32(self.clamped_range[1])
        # fp64 data: the Python doubles themselves (smart.py:82-84, 154-156)
        p.main_std_dev_threshold_f64 = float(hp.main_std_dev_threshold)
        p.clamp_lo_f64 = float(self.clamped_range[0])
        p.clamp_hi_f64 = float(self.clamped_range[1])
        p.range_std_coef_f64 = -1.0
        p.stochastic_rounding = 1 if hp.stochastic_rounding else 0
        p.all_positive = 1 if all_positive else 0
        p.use_range_std_dev = 1 if hp.use_range_std_dev else 0
        p.count_outliers = 1 if hp.measure_compression_ratio else 0
        p.range_std_coef = -1.0  # set by _set_range_coef in range mode (0.0 is a valid coefficient)
        p.stats_source = N.SMQ_STATS_WORKSPACE
        return p

    def _stream_fields(self, p: N.SmqSmaqParams, numel: int, device) -> None:
        """This call's random-stream position: the device counter (graph-safe) or a host offset."""
        if self._graph_safe and device is not None:
            p.seed, p.offset = self.rng.seed, 0
            p.offset_counter = self.rng.counter(device).data_ptr()
        else:
            p.seed, p.offset = self.rng.take(numel)

    def _hot_params(self, numel: int, all_positive: bool, dtype: torch.dtype, device):
        """_params for the hot path (full statistics): a copy of a cached flag template — keyed on
        every flag it reads, so a flag changed between calls takes effect — plus this call's stream
        position and range coefficient. ~40 % of _params' host time (the block has ~20 fields)."""
        hp = self.hparams
        key = (hp.num_bits_main, hp.num_bits_outlier, hp.main_std_dev_threshold,
               hp.stochastic_rounding, hp.use_range_std_dev, hp.measure_compression_ratio,
               self.range_normal, self.range_outlier, self.clamped_range, bool(all_positive))
        t = self._templates.get(key)
        if t is None:
            if len(self._templates) >= 64:
                self._templates.clear()
            t = self._templates[key] = self._flag_params(all_positive)
        p = N.SmqSmaqParams.from_buffer_copy(t)
        self._stream_fields(p, numel, device)
        if hp.use_range_std_dev:
            self._set_range_coef(p, numel, dtype)
        return p

    @staticmethod
    def _set_range_coef(p, count: int, dtype: torch.dtype):
        if dtype == torch.float64:
            p.range_std_coef_f64 = range_std_coef(count, torch.float64)
        else:
            p.range_std_coef = range_std_coef(count, dtype)

    def _bind_batch_norm(self, p, data: torch.Tensor, bn: Tuple[torch.Tensor, torch.Tensor]):
        """smart.py:136-149: per-channel (x - beta) / gamma on dim 1 of NCHW."""
        if data.dim() != 4:
            raise RuntimeError("use_batch_norm expects a 4-D NCHW tensor (smart.py:145 permutes 4 dims)")
        gamma, beta = bn
        if self.hparams.bn_scalar_params:
            gamma, beta = gamma.mean(), beta.mean()
        # fp32 parameters (fp64 for fp64 data: the promoted (x - beta) / gamma of smart.py:146)
        pdt = torch.float64 if data.dtype == torch.float64 else torch.float32
        gamma = gamma.detach().to(device=data.device, dtype=pdt).contiguous().reshape(-1)
        beta = beta.detach().to(device=data.device, dtype=pdt).contiguous().reshape(-1)
        channels = gamma.numel()
        if channels != beta.numel() or channels not in (1, data.shape[1]):
            raise RuntimeError(
                f"batch_norm_stats of size {channels} do not broadcast over {data.shape[1]} channels"
            )
        p.bn_gamma = gamma.data_ptr()
        p.bn_beta = beta.data_ptr()
        p.bn_channels = channels
        p.bn_inner = data.shape[2] * data.shape[3]
        return gamma, beta  # keep alive until the launch is enqueued

    # -- the C hot path (csrc/torchfast.cpp) --------------------------------------------------------
    # A capsule holding the flag templates of the parameter block and a snapshot of the hparams
    # they were built from; None: not built yet; False: unavailable (no binding, graph-safe random
    # stream, a subclass with its own __call__). Rebuilt when the hparams, the random stream or the
    # graph-safe switch are replaced (__setattr__), or when the C side finds a flag changed.
    _hot = None

    # the attributes the C state is built from: the hparams, the random stream, the graph-safe
    # switch and the constants the reference reads on every call (smart.py:154, 162)
    _HOT_INPUTS = frozenset(("hparams", "rng", "_graph_safe", "range_normal", "range_outlier",
                             "clamped_range"))

    def __setattr__(self, name, value):
        object.__setattr__(self, name, value)
        if name in SmartFP._HOT_INPUTS:
            object.__setattr__(self, "_hot", None)

    def _build_hot(self):
        T = N.torch_fast()
        hp = self.hparams
        d = hp if isinstance(hp, dict) else getattr(hp, "__dict__", None)
        hot = False
        call = type(self).__call__
        own = call is SmartFP.__call__
        if (T is not None and not self._graph_safe and type(d) is dict
                and (own or call is getattr(type(self), "_smartfp_call", None))):
            # a subclass whose __call__ returns SmartFP's values shares the C state, but not its
            # ratio logging (allow_count False: counted calls decline): the counted values are
            # SmartFP's bit counts, SmartFPPacked logs the real stream size
            hot = T.smaq_state(bytes(self._flag_params(False)), bytes(self._flag_params(True)),
                               d, self.rng.__dict__, N.ws_getter("smaq"), own)
        object.__setattr__(self, "_hot", hot)
        return hot

    def _autograd_fast(self, x: torch.Tensor, backward: bool):
        """Compressor.forward for this codec in C (util/pytorch/autograd.py): y = self(x) and a
        C++ autograd node whose backward is self(grad_y, tag="backward_autograd"); None when the C
        path does not take this call (the Python Function then does)."""
        hot = self._hot
        if hot is None:
            hot = self._build_hot()
        if hot is False or Globals.profiler is not None or self._trace is not None:
            return None
        y = N._torch_fast.smaq_autograd(hot, x, self, backward)
        if y is NotImplemented:  # a flag changed since the state was built
            if self._build_hot() is False:
                return None
            y = N._torch_fast.smaq_autograd(self._hot, x, self, backward)
        return y

    # -- call --------------------------------------------------------------------------------------
    def __call__(
        self,
        data: torch.Tensor,
        tag: str = None,
        all_positive=False,
        batch_norm_stats: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
        **_,
    ):
        # The hot path — a ROCm fp32 / fp16 / bf16 tensor of at least min_size elements, full
        # statistics, no BN term, no ratio logging, no profiler — is one C call on the tensor
        # (csrc/torchfast.cpp): an eager training step that compresses every layer is bound by the
        # host time of these calls (bench.py --config autograd_resnet34). No autograd op runs on
        # it (a fresh output the library writes), so it needs no grad-mode switch.
        hot = self._hot
        if hot is None:
            hot = self._build_hot()
        if hot is not False and Globals.profiler is None and self._trace is None:
            y = N._torch_fast.smaq(hot, data, all_positive, batch_norm_stats)
            if y is NotImplemented and self._build_hot() is not False:
                # a flag changed: rebuild, call again
                y = N._torch_fast.smaq(self._hot, data, all_positive, batch_norm_stats)
            if y is not None and y is not NotImplemented:
                if type(y) is tuple:  # --measure_compression_ratio: (y, its log_size values)
                    y, rec = y
                    self._log_size_record(tag, *rec)
                return y
        # Without the binding (or on graph-safe streams): the same call through the CPython
        # fast-call binding (ctypes' argument conversion costs ~4 us). Everything else: _call,
        # under torch.no_grad as smart.py:110.
        hp = self.hparams
        fast = N._fast if N._fast_tried else N.fast()
        if (fast is not None and data.is_cuda and not hp.measure_compression_ratio
                and Globals.profiler is None and self._trace is None
                and (batch_norm_stats is None or not hp.use_batch_norm)):
            code = N.DTYPE_CODES.get(data.dtype)
            numel = data.numel()
            if (code is not None and numel >= hp.min_size and not hp.use_sample_stats
                    and (data.dtype != torch.float16 or hp.precision == 16)):
                x = data if data.is_contiguous() else data.detach().contiguous()
                # (empty_like: half the host time of torch.empty with a shape and a device)
                y = (torch.empty_like(x) if code == N.SMQ_DTYPE_F32
                     else torch.empty(x.shape, dtype=torch.float32, device=x.device))
                p = self._hot_params(numel, all_positive, x.dtype, x.device)
                st = N.stream_ptr(x.device)
                ws = N.workspace("smaq", x.device, self.workspace_bytes(numel), st)
                rc = fast.smaq_roundtrip(x.data_ptr(), code, y.data_ptr(), numel,
                                         ctypes.addressof(p), ws.data_ptr(), ws.numel(), st)
                if rc:
                    N.check(rc, "smq_smaq_roundtrip")
                return y
        return self._call(data, tag, all_positive, batch_norm_stats)

    @torch.no_grad()
    def _call(self, data, tag, all_positive, batch_norm_stats):
        with profile("smaq"):
            hp = self.hparams
            numel = data.numel()
            if numel < hp.min_size:
                # same (double-counted) size the reference logs at smart.py:125
                self.log_ratio(tag, numel * 32, 32, 32)
                return data

            N.require_supported(data, "SmartFP")
            if data.dtype == torch.float64:
                return self._call_f64(data, tag, numel, all_positive, batch_norm_stats)
            code = N.DTYPE_CODES.get(data.dtype)
            if code is None:
                raise NotImplementedError(
                    f"SmartFP: dtype {data.dtype} is not supported "
                    "(float32/float16/bfloat16/float64)")
            if data.dtype == torch.float16 and hp.precision != 16:
                # the reference's std.clamp(1e-38, 1e38) on a half tensor (smart.py:154)
                raise RuntimeError("value cannot be converted to type c10::Half without overflow")
            if N.on_cpu(data):
                return self._call_cpu(data, tag, numel, code, all_positive, batch_norm_stats)
            if hp.measure_compression_ratio and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("SmartFP: --measure_compression_ratio reads the outlier count "
                                   "on the host; it cannot run inside a graph capture")
            x = data.contiguous()
            # half inputs: the bool*float scalars/ranges tensors promote the chain to fp32
            y = torch.empty(x.shape, dtype=torch.float32, device=x.device)
            p = self._params(numel, all_positive, x.dtype, x.device)
            keep = None
            if hp.use_batch_norm and batch_norm_stats is not None:
                keep = self._bind_batch_norm(p, x, batch_norm_stats)
            st = N.stream_ptr(x.device)
            ws = N.workspace("smaq", x.device, self.workspace_bytes(numel), st)
            self._launch(x, y, numel, p, ws, code, st)
            del keep

            def new_size():
                n_out = self.outlier_count(ws)
                return n_out * hp.num_bits_outlier + (numel - n_out) * hp.num_bits_main

            self.log_size(tag, numel * 32, new_size)
            return y

    def _call_cpu(self, data, tag, numel, code, all_positive, batch_norm_stats):
        """CPU tensors: the library's host path (smq_cpu_smaq_roundtrip), one synchronous call on
        torch's intra-op thread count; host RNG offsets (there is no graph to replay)."""
        hp = self.hparams
        x = data.contiguous()
        y = torch.empty(x.shape, dtype=torch.float32)
        p = self._params(numel, all_positive, x.dtype, None)
        keep = None
        if hp.use_batch_norm and batch_norm_stats is not None:
            keep = self._bind_batch_norm(p, x, batch_norm_stats)
        lib = N.lib()
        ws = N.cpu_workspace("smaq", self.workspace_bytes(numel))
        N.check(lib.smq_cpu_smaq_roundtrip(x.data_ptr(), code, y.data_ptr(), numel, p, None, None,
                                           ws.data_ptr(), ws.numel(), N.cpu_threads()),
                "smq_cpu_smaq_roundtrip")
        del keep
        if hp.measure_compression_ratio:
            n_out = self.outlier_count(ws)
            self.log_size(tag, numel * 32,
                          n_out * hp.num_bits_outlier + (numel - n_out) * hp.num_bits_main)
        else:
            self.log_size(tag, numel * 32, None)
        return y

    def _call_f64(self, data, tag, numel, all_positive, batch_norm_stats):
        """float64 data: smart.py:130-182 in fp64 (smq_smaq_roundtrip_f64 / its host twin), output
        float64; header SmqSmaqStatsF64 (read_stats_f64)."""
        hp = self.hparams
        x = data.contiguous()
        y = torch.empty(x.shape, dtype=torch.float64, device=x.device)
        cpu = N.on_cpu(x)
        p = self._params(numel, all_positive, torch.float64, None if cpu else x.device)
        keep = None
        if hp.use_batch_norm and batch_norm_stats is not None:
            keep = self._bind_batch_norm(p, x, batch_norm_stats)
        lib = N.lib()
        if cpu:
            ws = N.cpu_workspace("smaq", self.workspace_bytes(numel))
            N.check(lib.smq_cpu_smaq_roundtrip_f64(x.data_ptr(), y.data_ptr(), numel, p, None, None,
                                                   ws.data_ptr(), ws.numel(), N.cpu_threads()),
                    "smq_cpu_smaq_roundtrip_f64")
        else:
            if hp.measure_compression_ratio and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("SmartFP: --measure_compression_ratio reads the outlier count "
                                   "on the host; it cannot run inside a graph capture")
            st = N.stream_ptr(x.device)
            ws = N.workspace("smaq", x.device, self.workspace_bytes(numel), st)
            N.check(lib.smq_smaq_roundtrip_f64(x.data_ptr(), y.data_ptr(), numel, p, None, None,
                                               ws.data_ptr(), ws.numel(), st),
                    "smq_smaq_roundtrip_f64")
        del keep

        def new_size():
            n_out = self.outlier_count(ws)
            return n_out * hp.num_bits_outlier + (numel - n_out) * hp.num_bits_main

        self.log_size(tag, numel * 32, new_size if hp.measure_compression_ratio else None)
        return y

    _size_keys = {}  # tag -> the six metric names (the f-strings of base.log_size, built once)

    def _log_size_record(self, tag, ratio, new_size, orig_size):
        """log_size of a counted call (csrc/torchfast.cpp, smq_smaq_roundtrip_counted): the values
        are 0-dim fp64 device tensors the call itself wrote — the same values the host path logs
        as floats (smart.py:184-188, base.py:72-102), converted only when the logger consumes them,
        so a measuring step has no host synchronisation per call. Same keys, order, reduce_fx and
        log / log_custom routing as CompressionAlgorithmBase.log_size."""
        keys = SmartFP._size_keys.get(tag)
        if keys is None:
            keys = SmartFP._size_keys[tag] = (
                "compression_ratio", f"compression_ratio_{tag}", "new_size", f"new_size_{tag}",
                "orig_size", f"orig_size_{tag}", tag.startswith("optimizer_"))
        if keys[6] and self.log_custom is not None:
            self.log_custom({keys[0]: ratio, keys[1]: ratio, keys[2]: new_size,
                             keys[3]: new_size, keys[4]: orig_size, keys[5]: orig_size})
            return
        log, fx = self.log, _reduce_fx  # (= **_SIZE_FX, without a kwargs dict per call)
        log(keys[0], ratio)
        log(keys[1], ratio)
        log(keys[2], new_size, reduce_fx=fx, tbptt_reduce_fx=fx)
        log(keys[3], new_size, reduce_fx=fx, tbptt_reduce_fx=fx)
        log(keys[4], orig_size, reduce_fx=fx, tbptt_reduce_fx=fx)
        log(keys[5], orig_size, reduce_fx=fx, tbptt_reduce_fx=fx)

    # bench.py sets an event recorder here: an event pair on the codec's stream around the call's
    # launches (the product entry point either way)
    _trace = None

    def _launch(self, x: torch.Tensor, y: torch.Tensor, numel: int, p, ws: torch.Tensor,
                code: int = N.SMQ_DTYPE_F32, st: int = None):
        lib = N.lib()
        st = N.stream_ptr(x.device) if st is None else st
        tr = self._trace
        if tr is not None:
            tr.begin("call")
        if p.stats_source == N.SMQ_STATS_WORKSPACE:
            # one entry point: the single launch (tensors up to 8,388,611 elements), the deferred
            # two-launch path, or statistics + apply (smq.h smq_smaq_roundtrip)
            N.check(lib.smq_smaq_roundtrip(x.data_ptr(), code, y.data_ptr(), numel, p, None,
                                           ws.data_ptr(), ws.numel(), st), "smq_smaq_roundtrip")
        else:
            N.check(lib.smq_smaq_apply(x.data_ptr(), code, y.data_ptr(), numel, p, None, None,
                                       ws.data_ptr(), ws.numel(), st), "smq_smaq_apply")
        if tr is not None:
            tr.end("call")

    def workspace_bytes(self, numel: int) -> int:
        """Workspace of one call: above SMQ_MAX_DEVICE_SAMPLES device-drawn samples the
        multi-workgroup draw needs its own region (include/smq.h SMQ_WS_LARGE_SAMPLES_OFFSET)."""
        key = (numel, self.hparams.num_samples if self.hparams.use_sample_stats else -1)
        nb = _WS_BYTES.get(key)
        if nb is None:  # (one library query per size: ~1 us of host time per call otherwise)
            lib = N.lib()
            if key[1] >= 0:
                nb = lib.smq_smaq_workspace_bytes_sampled(numel, key[1])
            else:
                nb = lib.smq_smaq_workspace_bytes(numel)
            if len(_WS_BYTES) > 4096:
                _WS_BYTES.clear()
            _WS_BYTES[key] = nb
        return nb

    # -- inspection helpers (tests / bench) --------------------------------------------------------
    @staticmethod
    def sample_indices(ws: torch.Tensor, k: int) -> np.ndarray:
        """The k indices the last device-drawn sampled call on ``ws`` drew, in draw order."""
        off = N.SMQ_WS_SAMPLES_OFFSET if k <= N.SMQ_MAX_DEVICE_SAMPLES else N.SMQ_WS_LARGE_SAMPLES_OFFSET
        return ws[off: off + 8 * k].cpu().numpy().view(np.int64).copy()

    @staticmethod
    def outlier_count(ws: torch.Tensor) -> int:
        """Sum of the SMQ_WS_OUTLIER_SLOTS outlier-count slots (include/smq.h)."""
        off = N.SMQ_WS_OUTLIER_SLOTS_OFFSET
        slots = ws[off: off + 8 * N.SMQ_WS_OUTLIER_SLOTS].cpu().numpy().view(np.uint64)
        return int(slots.sum())

    @staticmethod
    def read_stats_f64(ws: torch.Tensor) -> dict:
        """The SmqSmaqStatsF64 header of an fp64 call."""
        raw = ws[:80].cpu().numpy()
        d = raw[:48].view(np.float64)
        return {
            "mean": float(d[0]), "std_dev": float(d[1]), "std_clamped": float(d[2]),
            "raw_std": float(d[3]), "min": float(d[4]), "max": float(d[5]),
            "n_used": int(raw[48:52].view(np.uint32)[0]),
            "rng_offset": int(raw[56:64].view(np.uint64)[0]),
            "n_outlier": SmartFP.outlier_count(ws),
        }

    @staticmethod
    def read_stats(ws: torch.Tensor) -> dict:
        raw = ws[:64].cpu().numpy()
        f = raw[:24].view(np.float32)
        return {
            "mean": float(f[0]), "std_dev": float(f[1]), "std_clamped": float(f[2]),
            "raw_std": float(f[3]), "min": float(f[4]), "max": float(f[5]),
            "n_used": int(raw[24:28].view(np.uint32)[0]),
            "n_outlier": SmartFP.outlier_count(ws),
        }
