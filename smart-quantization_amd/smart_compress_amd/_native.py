"""ctypes binding of libsmq.so, the C-ABI declared in include/smq.h.

This is the only place the Python host touches the native library. There is no fallback: if the
library is missing or a device tensor is not on a ROCm GPU, the codecs raise. The structures below
mirror include/smq.h field for field.
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict, Tuple

import torch

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "SMQ_LIB", os.path.join(os.path.dirname(_PKG_DIR), "lib", "libsmq.so")
)

SMQ_ABI_VERSION = 8
SMQ_MAX_SAMPLES = 64
SMQ_MAX_DEVICE_SAMPLES = 4096
SMQ_MAX_DRAW_SAMPLES = 1 << 28
SMQ_WS_FUSED_OFFSET = 99584
SMQ_WS_LARGE_SAMPLES_OFFSET = 199168
SMQ_WS_OUTLIER_SLOTS_OFFSET = 128
SMQ_WS_OUTLIER_SLOTS = 64
SMQ_WS_SAMPLES_OFFSET = 66176
SMQ_STATS_WORKSPACE = 0
SMQ_STATS_SAMPLED = 1
SMQ_STATS_INJECTED = 2
SMQ_STATS_SAMPLED_DEVICE = 3
SMQ_SMAQ_SPLIT = 1
SMQ_SMAQ_NO_DEFER = 2
SMQ_SMAQ_TEST_LATE = 4
SMQ_S2FP8_OUT_Y = 1
SMQ_S2FP8_OUT_T = 2
SMQ_S2FP8_EXACT_POW = 4
SMQ_S2FP8_SPLIT = 8
SMQ_S2FP8_TEST_LATE = 16
SMQ_PACK_TICKETED = 1
SMQ_PACK_SINGLE = 2
SMQ_DTYPE_F32 = 0
SMQ_DTYPE_F16 = 1
SMQ_DTYPE_BF16 = 2
SMQ_DTYPE_F64 = 3
SMQ_ROUND_NEAREST = 0
SMQ_ROUND_STOCHASTIC = 1


class SmqSmaqParams(ctypes.Structure):
    _fields_ = [
        ("num_bits_main", ctypes.c_int32),
        ("num_bits_outlier", ctypes.c_int32),
        ("main_std_dev_threshold", ctypes.c_float),
        ("range_main", ctypes.c_float),
        ("range_outlier", ctypes.c_float),
        ("clamp_lo", ctypes.c_float),
        ("clamp_hi", ctypes.c_float),
        ("range_std_coef", ctypes.c_float),
        ("stochastic_rounding", ctypes.c_int32),
        ("all_positive", ctypes.c_int32),
        ("use_range_std_dev", ctypes.c_int32),
        ("stats_source", ctypes.c_int32),
        ("count_outliers", ctypes.c_int32),
        ("num_samples", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("offset", ctypes.c_uint64),
        ("bn_gamma", ctypes.c_void_p),
        ("bn_beta", ctypes.c_void_p),
        ("bn_channels", ctypes.c_int64),
        ("bn_inner", ctypes.c_int64),
        ("sample_idx", ctypes.c_int64 * SMQ_MAX_SAMPLES),
        ("offset_counter", ctypes.c_void_p),
        ("main_std_dev_threshold_f64", ctypes.c_double),
        ("clamp_lo_f64", ctypes.c_double),
        ("clamp_hi_f64", ctypes.c_double),
        ("range_std_coef_f64", ctypes.c_double),
    ]


class SmqSmaqStats(ctypes.Structure):
    _fields_ = [
        ("mean", ctypes.c_float),
        ("std_dev", ctypes.c_float),
        ("std_clamped", ctypes.c_float),
        ("raw_std", ctypes.c_float),
        ("min_val", ctypes.c_float),
        ("max_val", ctypes.c_float),
        ("n_used", ctypes.c_uint32),
        ("quot_check", ctypes.c_uint32),
        ("n_outlier", ctypes.c_ulonglong),
        ("inv_std_clamped", ctypes.c_double),
        ("rng_offset", ctypes.c_ulonglong),
        ("inv_std_clamped_f32", ctypes.c_float),
        ("reserved", ctypes.c_uint32),
    ]


class SmqPackedHeader(ctypes.Structure):
    _fields_ = [
        ("magic", ctypes.c_uint32),
        ("version", ctypes.c_uint32),
        ("n", ctypes.c_int64),
        ("block_elems", ctypes.c_uint32),
        ("n_blocks", ctypes.c_uint32),
        ("num_bits_main", ctypes.c_int32),
        ("num_bits_outlier", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("thr", ctypes.c_float),
        ("range_main", ctypes.c_float),
        ("range_outlier", ctypes.c_float),
        ("mean", ctypes.c_float),
        ("std_dev", ctypes.c_float),
        ("inv_range_main", ctypes.c_double),
        ("inv_range_outlier", ctypes.c_double),
        ("data_words", ctypes.c_uint64),
        ("total_bytes", ctypes.c_uint64),
        ("error", ctypes.c_uint32),
        ("bn_channels", ctypes.c_uint32),
        ("bn_inner", ctypes.c_int64),
        ("mean_f64", ctypes.c_double),
        ("std_dev_f64", ctypes.c_double),
        ("reserved", ctypes.c_uint32 * 2),
    ]


SMQ_PACK_MAGIC = 0x50514D53
SMQ_PACK_BLOCK = 4096
SMQ_NOTIFY_PENDING = 0xFFFFFFFF    # a notify word not written yet (smq_smaq_roundtrip_compress_notify)
SMQ_NOTIFY_SATURATED = 0xFFFFFFFE  # a stream of 2^32 - 1 bytes or more
SMQ_PACK_FLAG_ALL_POSITIVE = 1
SMQ_PACK_FLAG_SAFE_Q = 2
SMQ_PACK_FLAG_BOTH_SIDES = 4
SMQ_PACK_FLAG_BN = 8
SMQ_PACK_FLAG_F64 = 16


class SmqSizeRecord(ctypes.Structure):
    """include/smq.h SmqSizeRecord: a counted call's outlier count and log_size values (fp64, on
    the device; smq_smaq_roundtrip_counted)."""
    _fields_ = [
        ("slots", ctypes.c_uint64 * 8),
        ("arrived", ctypes.c_uint64),
        ("reserved", ctypes.c_uint64 * 3),
        ("n_outlier", ctypes.c_double),
        ("new_size", ctypes.c_double),
        ("compression_ratio", ctypes.c_double),
        ("orig_size", ctypes.c_double),
    ]


class SmqTensorDesc(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_void_p),
        ("y", ctypes.c_void_p),
        ("n", ctypes.c_int64),
        ("all_positive", ctypes.c_int32),
        ("range_std_coef", ctypes.c_float),
        ("rng_offset", ctypes.c_uint64),
    ]


class SmqS2fp8Stats(ctypes.Structure):
    _fields_ = [
        ("mu", ctypes.c_float),
        ("m", ctypes.c_float),
        ("alpha", ctypes.c_float),
        ("beta", ctypes.c_float),
        ("beta_pow2", ctypes.c_float),
        ("inv_beta_pow2", ctypes.c_float),
        ("inv_alpha", ctypes.c_float),
        ("n_used", ctypes.c_uint32),
        ("rng_offset", ctypes.c_uint64),
        ("reserved", ctypes.c_uint32 * 6),
    ]


class SmqSmaqStatsF64(ctypes.Structure):
    _fields_ = [
        ("mean", ctypes.c_double),
        ("std_dev", ctypes.c_double),
        ("std_clamped", ctypes.c_double),
        ("raw_std", ctypes.c_double),
        ("min_val", ctypes.c_double),
        ("max_val", ctypes.c_double),
        ("n_used", ctypes.c_uint32),
        ("reserved0", ctypes.c_uint32),
        ("rng_offset", ctypes.c_ulonglong),
        ("reserved", ctypes.c_ulonglong * 2),
    ]


class SmqS2fp8StatsF64(ctypes.Structure):
    _fields_ = [
        ("mu", ctypes.c_double),
        ("m", ctypes.c_double),
        ("alpha", ctypes.c_double),
        ("beta", ctypes.c_double),
        ("beta_pow2", ctypes.c_double),
        ("inv_beta_pow2", ctypes.c_double),
        ("inv_alpha", ctypes.c_double),
        ("n_used", ctypes.c_uint32),
        ("reserved0", ctypes.c_uint32),
        ("rng_offset", ctypes.c_uint64),
        ("reserved", ctypes.c_uint64 * 3),
    ]


assert ctypes.sizeof(SmqSmaqStats) == 64
assert ctypes.sizeof(SmqSmaqStatsF64) == 80
assert ctypes.sizeof(SmqS2fp8StatsF64) == 96
assert ctypes.sizeof(SmqTensorDesc) == 40
assert ctypes.sizeof(SmqS2fp8Stats) == 64

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int
_U64 = ctypes.c_uint64
_U32 = ctypes.c_uint32
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); every function declared in include/smq.h
SIGNATURES = {
    "smq_abi_version": (_I32, []),
    "smq_last_error": (ctypes.c_char_p, []),
    "smq_smaq_params_init": (None, [ctypes.POINTER(SmqSmaqParams)]),
    "smq_smaq_params_set": (
        _I32,
        [ctypes.POINTER(SmqSmaqParams), _I32, _I32, ctypes.c_double, ctypes.c_double, _I32],
    ),
    "smq_smaq_draw_samples": (_I32, [ctypes.POINTER(SmqSmaqParams), _I64, _I32]),
    "smq_smaq_workspace_bytes": (_SZ, [_I64]),
    "smq_smaq_workspace_bytes_sampled": (_SZ, [_I64, _I64]),
    "smq_smaq_stats_f32": (_I32, [_P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _SZ, _P]),
    "smq_smaq_apply_f32": (
        _I32,
        [_P, _P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _P, _P, _SZ, _P],
    ),
    "smq_smaq_roundtrip_f32": (
        _I32,
        [_P, _P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _P, _SZ, _P],
    ),
    "smq_smaq_stats": (_I32, [_P, _I32, _I64, ctypes.POINTER(SmqSmaqParams), _P, _SZ, _P]),
    "smq_smaq_apply": (
        _I32,
        [_P, _I32, _P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _P, _P, _SZ, _P],
    ),
    "smq_smaq_roundtrip": (
        _I32,
        [_P, _I32, _P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _P, _SZ, _P],
    ),
    "smq_smaq_roundtrip_ex": (
        _I32,
        [_P, _I32, _P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _P, _SZ, _U32, _P],
    ),
    "smq_smaq_roundtrip_counted": (
        _I32,
        [_P, _I32, _P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _SZ, _P, _P],
    ),
    "smq_smaq_size_metrics": (_I32, [_P, _I64, _I32, _I32, _P, _P]),
    "smq_smaq_multi_size_metrics": (_I32, [_P, _P, _I32, _I32, _I32, _P, _P]),
    "smq_smaq_multi_plan_bytes": (_SZ, [ctypes.POINTER(_I64), _I32]),
    "smq_smaq_multi_plan_build": (_I32, [ctypes.POINTER(SmqTensorDesc), _I32, _P, _SZ]),
    "smq_smaq_multi_workspace_bytes": (_SZ, [ctypes.POINTER(_I64), _I32]),
    "smq_smaq_multi_f32": (_I32, [_P, _P, ctypes.POINTER(SmqSmaqParams), _P, _SZ, _P]),
    "smq_smaq_multi": (_I32, [_P, _P, _I32, ctypes.POINTER(SmqSmaqParams), _P, _SZ, _P]),
    "smq_float_quant_f32": (
        _I32,
        [_P, _P, _I64, _I32, _I32, _I32, _I32, _P, _U64, _U64, _P],
    ),
    "smq_float_quant_max_value": (ctypes.c_float, [_I32, _I32]),
    "smq_s2fp8_workspace_bytes": (_SZ, [_I64]),
    "smq_s2fp8_roundtrip_f32": (
        _I32,
        [_P, _P, _I64, _I32, _P, _U64, _U64, _P, _P, _SZ, _P],
    ),
    "smq_s2fp8_roundtrip": (
        _I32,
        [_P, _I32, _P, _I64, _I32, _I32, _P, _U64, _U64, _P, _P, _P, _SZ, _P],
    ),
    "smq_s2fp8_roundtrip_ex": (
        _I32,
        [_P, _I32, _P, _I64, _I32, _I32, _P, _U64, _U64, _P, _P, _P, _SZ, _U32, _P],
    ),
    "smq_float_quant": (
        _I32,
        [_P, _I32, _P, _I32, _I64, _I32, _I32, _I32, _I32, _P, _U64, _U64, _P, _P],
    ),
    "smq_rng_u32": (ctypes.c_uint32, [_U64, _U64]),
    "smq_smaq_u24": (ctypes.c_uint32, [_U64, _U64]),
    "smq_half_quot_split": (ctypes.c_int, [ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_int, _P]),
    "smq_smaq_pack_bound": (_SZ, [_I64, _I32, _I32]),
    "smq_smaq_pack_bound_bn": (_SZ, [_I64, _I32, _I32, _I64]),
    "smq_smaq_pack_workspace_bytes": (_SZ, [_I64]),
    "smq_smaq_compress": (_I32, [_P, _I32, _I64, ctypes.POINTER(SmqSmaqParams),
                                         _P, _SZ, _P, _SZ, _P]),
    "smq_smaq_compress_ex": (_I32, [_P, _I32, _I64, ctypes.POINTER(SmqSmaqParams),
                                     _P, _SZ, _P, _SZ, _U32, _P]),
    "smq_smaq_decompress": (_I32, [_P, _P, _I64, _P]),
    "smq_smaq_pack_fixed_bytes": (_SZ, [_I64, _I32]),
    "smq_smaq_roundtrip_compress": (_I32, [_P, _I32, _P, _I64, ctypes.POINTER(SmqSmaqParams),
                                           _P, _SZ, _P, _SZ, _P]),
    "smq_smaq_roundtrip_compress_ex": (_I32, [_P, _I32, _P, _I64, ctypes.POINTER(SmqSmaqParams),
                                              _P, _SZ, _P, _SZ, _P, _P]),
    "smq_smaq_roundtrip_compress_notify": (_I32, [_P, _I32, _P, _I64,
                                                  ctypes.POINTER(SmqSmaqParams), _P, _SZ, _P, _SZ,
                                                  _P, _P]),
    "smq_notify_alloc": (_P, [_I64]),
    "smq_notify_free": (None, [_P]),
    "smq_smaq_pack_workspace_bytes_sampled": (_SZ, [_I64, _I64]),
    "smq_cpu_smaq_compress": (_I32, [_P, _I32, _I64, ctypes.POINTER(SmqSmaqParams), _P, _SZ, _P,
                                     _SZ, _I32]),
    "smq_cpu_smaq_decompress": (_I32, [_P, _P, _I64, _I32]),
    "smq_smaq_decompress_ex": (_I32, [_P, _P, _I64, _I32, _I32, _P]),
    "smq_smaq_pack_bound_f64": (_SZ, [_I64, _I32, _I32, _I64]),
    "smq_smaq_pack_workspace_bytes_f64": (_SZ, [_I64, _I64]),
    "smq_smaq_compress_f64": (_I32, [_P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _SZ, _P, _SZ,
                                     _P]),
    "smq_smaq_decompress_f64": (_I32, [_P, _P, _I64, _I32, _I32, _P]),
    "smq_cpu_smaq_compress_f64": (_I32, [_P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _SZ, _P,
                                         _SZ, _I32]),
    "smq_cpu_smaq_decompress_f64": (_I32, [_P, _P, _I64, _I32]),
    "smq_cpu_threads": (_I32, []),
    "smq_cpu_smaq_roundtrip": (
        _I32,
        [_P, _I32, _P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _P, _P, _SZ, _I32],
    ),
    "smq_cpu_float_quant": (
        _I32,
        [_P, _I32, _P, _I32, _I64, _I32, _I32, _I32, _I32, _P, _U64, _U64, _I32],
    ),
    "smq_cpu_s2fp8_roundtrip": (
        _I32,
        [_P, _I32, _P, _I64, _I32, _I32, _P, _U64, _U64, _P, _P, _SZ, _U32, _I32],
    ),
    "smq_smaq_roundtrip_f64": (
        _I32,
        [_P, _P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _P, _P, _SZ, _P],
    ),
    "smq_cpu_smaq_roundtrip_f64": (
        _I32,
        [_P, _P, _I64, ctypes.POINTER(SmqSmaqParams), _P, _P, _P, _SZ, _I32],
    ),
    "smq_s2fp8_roundtrip_f64": (
        _I32,
        [_P, _P, _I64, _I32, _I32, _P, _U64, _U64, _P, _P, _P, _SZ, _U32, _P],
    ),
    "smq_cpu_s2fp8_roundtrip_f64": (
        _I32,
        [_P, _P, _I64, _I32, _I32, _P, _U64, _U64, _P, _P, _SZ, _U32, _I32],
    ),
}

_lib = None
_lib_lock = threading.Lock()


class NativeLibraryError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load libsmq.so once. Raises NativeLibraryError if it is missing: there is no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeLibraryError(
                    f"libsmq.so not found at {LIB_PATH}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)"
                )
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            if handle.smq_abi_version() != SMQ_ABI_VERSION:
                raise NativeLibraryError("libsmq ABI version mismatch")
            _lib = handle
    return _lib


_fast = None
_fast_tried = False


def _load_binding(name: str):
    """A binding module built next to the library being used (lib/<name><EXT_SUFFIX>), or None
    when there is none (an experiment library elsewhere, SMQ_LIB). Bindings call the same
    libsmq.so (rpath $ORIGIN = the directory of LIB_PATH)."""
    lib()  # the ABI check, and the library every entry point shares
    import importlib.machinery
    import importlib.util
    import sysconfig

    path = os.path.join(os.path.dirname(LIB_PATH), name + sysconfig.get_config_var("EXT_SUFFIX"))
    if not os.path.exists(path):
        return None
    loader = importlib.machinery.ExtensionFileLoader(name, path)
    spec = importlib.util.spec_from_file_location(name, path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


def fast():
    """The CPython fast-call binding of smq_smaq_roundtrip / smq_s2fp8_roundtrip
    (csrc/pyfast.cpp), or None (then ctypes): the same calls without ctypes' ~4 us of argument
    conversion per call."""
    global _fast, _fast_tried
    if _fast_tried:
        return _fast
    _fast = _load_binding("_smqfast")
    _fast_tried = True
    return _fast


_torch_fast = None
_torch_fast_tried = False


def torch_fast():
    """The at::Tensor-level binding (csrc/torchfast.cpp: the eager SmartFP / S2FP8 call and the
    SmartFP autograd node), or None (then the Python hot paths). SMQ_TORCHFAST=0 disables it (the
    A/B switch of tools/host_cost_smaq.py)."""
    global _torch_fast, _torch_fast_tried
    if _torch_fast_tried:
        return _torch_fast
    if os.environ.get("SMQ_TORCHFAST", "1") != "0":
        _torch_fast = _load_binding("_smqtorch")
    _torch_fast_tried = True
    return _torch_fast


def ws_getter(kind: str):
    """The workspace callback of the C hot paths: (device index, stream, nbytes) -> the
    (kind, device, stream) workspace of this table."""
    def get(dev: int, stream: int, nbytes: int) -> torch.Tensor:
        return workspace(kind, torch.device("cuda", dev), nbytes, stream)
    return get


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().smq_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (rc={rc}): {msg}")


DTYPE_CODES = {torch.float32: SMQ_DTYPE_F32, torch.float16: SMQ_DTYPE_F16,
               torch.bfloat16: SMQ_DTYPE_BF16}


def require_device(t: torch.Tensor, who: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(
            f"{who}: smart_compress_amd runs on ROCm device tensors only (got device={t.device}); "
            "move the tensor to the GPU"
        )


def on_cpu(t: torch.Tensor) -> bool:
    """CPU tensors run on the library's host path (smq_cpu_*), ROCm tensors on the kernels."""
    return t.device.type == "cpu"


def require_supported(t: torch.Tensor, who: str) -> None:
    """A ROCm device tensor or a CPU tensor (the reference's plugins run on either)."""
    if not (t.is_cuda or on_cpu(t)):
        raise RuntimeError(f"{who}: tensors on {t.device} are not supported (ROCm device or CPU)")


def cpu_threads() -> int:
    """Threads a host-path call uses: torch's intra-op setting, like the reference's CPU ops."""
    return max(1, torch.get_num_threads())


_cpu_ws = threading.local()


def cpu_workspace(kind: str, nbytes: int) -> torch.Tensor:
    """A host workspace of at least nbytes for the calling thread (host calls are synchronous)."""
    cache = getattr(_cpu_ws, "bufs", None)
    if cache is None:
        cache = _cpu_ws.bufs = {}
    buf = cache.get(kind)
    if buf is None or buf.numel() < nbytes:
        buf = cache[kind] = torch.zeros(max(nbytes, 256), dtype=torch.uint8)
    return buf


def require_device_f32(t: torch.Tensor, who: str) -> None:
    require_device(t, who)
    if t.dtype != torch.float32:
        raise NotImplementedError(
            f"{who}: dtype {t.dtype} is not supported by the gfx950 kernels yet (float32 only)"
        )


# the current stream's raw handle without building a torch.cuda.Stream object (~0.2 vs ~2 us)
_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def device_index(device: torch.device) -> int:
    return device.index if device.index is not None else torch.cuda.current_device()


def raw_stream(index: int) -> int:
    """The current stream of device ``index`` as a hipStream_t value (one C call)."""
    if _raw_stream is not None:
        return _raw_stream(index)
    return torch.cuda.current_stream(index).cuda_stream


def stream_ptr(device: torch.device) -> int:
    if _raw_stream is not None:
        return _raw_stream(device_index(device))
    return torch.cuda.current_stream(device).cuda_stream


# ---- per (device, stream) workspaces (the library needs them neither zeroed nor reset) ----------
# Keyed by the raw stream handle, which the table does not own: a program that creates streams
# without end would grow it without end, so it holds at most WORKSPACE_LIMIT entries. A new entry
# past the limit evicts the oldest one after synchronising that device (its stream may still have
# calls queued). A captured graph keeps using the buffers its calls were given, so eviction stops
# for good once graph-safe random streams (the precondition of capturing a codec call) exist in
# the process (RngState.counter) or a workspace is created during a capture.
WORKSPACE_LIMIT = 256  # above torch's per-device stream pool (2 x 32) times the workspace kinds
_ws: Dict[Tuple[str, int, int], torch.Tensor] = {}
_ws_evictable = True
_ws_lock = threading.Lock()


def pin_workspaces() -> None:
    """Stop evicting workspaces (a hipGraph may hold any of them from now on)."""
    global _ws_evictable
    _ws_evictable = False


def workspace(kind: str, device: torch.device, nbytes: int, stream: int = None) -> torch.Tensor:
    """The (kind, device, stream) workspace of at least nbytes. The hit path takes no lock (a dict
    read is atomic under the GIL); creation does."""
    key = (kind, device_index(device), stream_ptr(device) if stream is None else stream)
    buf = _ws.get(key)
    if buf is not None and buf.numel() >= nbytes:
        # a capture may hold this buffer from now on (even one taken without graph-safe streams):
        # stop evicting. (Only while eviction is still on; the C hot path keeps its own reference.)
        if _ws_evictable and torch.device(device).type == "cuda" and \
                torch.cuda.is_current_stream_capturing():
            pin_workspaces()
        return buf
    with _ws_lock:
        capturing = (torch.device(device).type == "cuda"
                     and torch.cuda.is_current_stream_capturing())
        if capturing:
            pin_workspaces()
        buf = _ws.get(key)
        if buf is None or buf.numel() < nbytes:
            # Allocated while a graph is being captured, a zero-fill would become a graph node
            # that clears the buffer on every replay: each replay's calls would then find their
            # arrival counters cleared and take the slow re-tagging path (include/smq.h: the
            # SmaQ and S2FP8 workspaces need no initialisation). The packed codec's look-back
            # status words do need it; for them a per-replay clear is only a redundant memset.
            if capturing and kind in ("smaq", "s2fp8"):
                buf = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
            else:
                buf = torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=device)
            if key not in _ws and len(_ws) >= WORKSPACE_LIMIT and _ws_evictable:
                # (a thread still holding the evicted tensor keeps its memory; when it drops it,
                # the caching allocator reuses the block only in the order of the stream the
                # buffer was made and used on, i.e. after that thread's queued calls)
                old = next(iter(_ws))
                if old[1] >= 0 and torch.cuda.is_available():
                    torch.cuda.synchronize(old[1])
                del _ws[old]
            _ws[key] = buf
    return buf


class RngState:
    """(seed, offset) of a counter-based RNG stream; offset advances by the elements consumed.

    Graph-safe mode keeps the position in a device uint64 per GPU (``counter(device)``, created
    from ``offset``); the kernels read and advance it, so hipGraph replays draw fresh streams.
    ``release_counters`` returns to host offsets, continuing from the device position."""

    def __init__(self, seed: int | None = None):
        if seed is None:
            seed = int(torch.randint(0, 2**62, (1,), generator=torch.default_generator).item())
        self.seed = int(seed) & (2**64 - 1)
        self.offset = 0
        self._lock = threading.Lock()
        self._counters = {}

    def take(self, n: int) -> Tuple[int, int]:
        with self._lock:
            off = self.offset
            self.offset = (self.offset + int(n)) & (2**64 - 1)
        return self.seed, off

    def counter(self, device) -> torch.Tensor:
        device = torch.device(device)
        idx = device.index if device.index is not None else torch.cuda.current_device()
        c = self._counters.get(idx)
        if c is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("graph-safe random stream: create the device counter before "
                                   "capture (graph_safe(device=...) or one eager call)")
            v = self.offset - 2**64 if self.offset >= 2**63 else self.offset  # int64 bit pattern
            c = torch.tensor([v], dtype=torch.int64, device=torch.device("cuda", idx))
            self._counters[idx] = c
            pin_workspaces()  # calls may now be captured: their workspaces must stay alive
        return c

    def position(self) -> int:
        """The stream position: the host offset, or the furthest device counter (a host sync)."""
        pos = self.offset
        for c in self._counters.values():
            pos = max(pos, int(c.item()) & (2**64 - 1))
        return pos

    def release_counters(self) -> None:
        self.offset = self.position()
        self._counters.clear()

    def state_dict(self):
        return {"seed": self.seed, "offset": self.position()}

    def load_state_dict(self, d):
        self.seed = int(d["seed"])
        self.offset = int(d["offset"])
        v = self.offset - 2**64 if self.offset >= 2**63 else self.offset
        for c in self._counters.values():
            c.fill_(v)
