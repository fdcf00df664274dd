"""Thin wrappers that drive the C-ABI (include/smq.h) directly from tests, with the parity-only
inputs (injected statistics, uniforms, random words) the Python codecs never pass."""

import ctypes

import numpy as np
import torch

from smart_compress_amd import _native as N
from smart_compress_amd.compress.smart import SmartFP

DEV = "cuda:0"


def stream():
    return torch.cuda.current_stream().cuda_stream


TORCH_DT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}


def smaq_params(hp, numel, all_positive=False, seed=0, offset=0, dtype=torch.float32):
    codec = SmartFP(hp)
    codec.rng.seed, codec.rng.offset = seed, offset
    return codec._params(numel, all_positive, dtype)


def stats_struct(mean, std, hp, dtype="f32"):
    """SmqSmaqStats as the kernel's finaliser would write it for (mean, std) (smart.py:151-154)."""
    from oracle.smaq import round_to

    s = N.SmqSmaqStats()
    lo = np.float32(round_to(np.float32(1e-4 if hp.precision == 16 else 1e-38), dtype))
    hi = np.float32(round_to(np.float32(1e4 if hp.precision == 16 else 1e38), dtype))
    sd = np.float32(std)
    std_dev = np.float32(1.0) if sd == 0 else sd
    sc = std_dev
    if sc < lo:
        sc = lo
    if sc > hi:
        sc = hi
    s.mean, s.std_dev, s.std_clamped, s.raw_std = float(mean), float(std_dev), float(sc), float(sd)
    raw = np.frombuffer(ctypes.string_at(ctypes.addressof(s), 64), dtype=np.uint8).copy()
    return torch.from_numpy(raw).to(DEV)


def read_stats(ws):
    return SmartFP.read_stats(ws)


def smaq_apply(x, p, uniforms=None, stats_in=None, y=None):
    """One smq_smaq_apply launch (input dtype from x, fp32 output); returns (y, ws)."""
    n = x.numel()
    y = torch.empty(x.shape, dtype=torch.float32, device=x.device) if y is None else y
    ws = torch.zeros(N.lib().smq_smaq_workspace_bytes(n), dtype=torch.uint8, device=x.device)
    if stats_in is not None:
        p.stats_source = N.SMQ_STATS_INJECTED
    N.check(N.lib().smq_smaq_apply(
        x.data_ptr(), N.DTYPE_CODES[x.dtype], y.data_ptr(), n, p,
        uniforms.data_ptr() if uniforms is not None else None,
        stats_in.data_ptr() if stats_in is not None else None,
        ws.data_ptr(), ws.numel(), stream()), "apply")
    return y, ws


def smaq_roundtrip(x, p, uniforms=None, y=None):
    n = x.numel()
    y = torch.empty(x.shape, dtype=torch.float32, device=x.device) if y is None else y
    ws = torch.zeros(N.lib().smq_smaq_workspace_bytes(n), dtype=torch.uint8, device=x.device)
    N.check(N.lib().smq_smaq_roundtrip(
        x.data_ptr(), N.DTYPE_CODES[x.dtype], y.data_ptr(), n, p,
        uniforms.data_ptr() if uniforms is not None else None,
        ws.data_ptr(), ws.numel(), stream()), "roundtrip")
    return y, ws


def float_quant_any(x, exp_bits, man_bits, out_dtype=torch.float32, rounding=N.SMQ_ROUND_STOCHASTIC,
                    check_inf=True, rand_bits=None, seed=0, offset=0, counter=None):
    """smq_float_quant: any input dtype, fp32 or fp16 output, optional device offset counter."""
    y = torch.empty(x.shape, dtype=out_dtype, device=x.device)
    N.check(N.lib().smq_float_quant(
        x.data_ptr(), N.DTYPE_CODES[x.dtype], y.data_ptr(), N.DTYPE_CODES[out_dtype], x.numel(),
        exp_bits, man_bits, rounding, 1 if check_inf else 0,
        rand_bits.data_ptr() if rand_bits is not None else None, seed, offset,
        counter.data_ptr() if counter is not None else None, stream()), "float_quant")
    return y


def float_quant(x, exp_bits, man_bits, rounding=N.SMQ_ROUND_STOCHASTIC, check_inf=True,
                rand_bits=None, seed=0, offset=0):
    y = torch.empty_like(x)
    N.check(N.lib().smq_float_quant_f32(
        x.data_ptr(), y.data_ptr(), x.numel(), exp_bits, man_bits, rounding,
        1 if check_inf else 0, rand_bits.data_ptr() if rand_bits is not None else None,
        seed, offset, stream()), "float_quant")
    return y


def s2fp8(x, check_inf=True, rand_bits=None, seed=0, offset=0, mu_m=None, precision=32,
          counter=None, flags=0, ws=None):
    """smq_s2fp8_roundtrip_ex on a device tensor of any supported dtype (precision 16: fp16 in ->
    fp16 out, fp32 / bf16 in -> fp32 out); flags = SMQ_S2FP8_* (OUT_Y / OUT_T: y holds Y or T)."""
    n = x.numel()
    half_out = precision == 16 and x.dtype == torch.float16
    y = torch.empty(x.shape, dtype=torch.float16 if half_out else torch.float32, device=x.device)
    if ws is None:
        ws = torch.zeros(N.lib().smq_s2fp8_workspace_bytes(n), dtype=torch.uint8, device=x.device)
    st_in = None
    if mu_m is not None:
        s = N.SmqS2fp8Stats()
        s.mu, s.m, s.n_used = float(mu_m[0]), float(mu_m[1]), n
        raw = np.frombuffer(ctypes.string_at(ctypes.addressof(s), 64), dtype=np.uint8).copy()
        st_in = torch.from_numpy(raw).to(x.device)
    N.check(N.lib().smq_s2fp8_roundtrip_ex(
        x.data_ptr(), N.DTYPE_CODES[x.dtype], y.data_ptr(), n, precision, 1 if check_inf else 0,
        rand_bits.data_ptr() if rand_bits is not None else None, seed, offset,
        counter.data_ptr() if counter is not None else None,
        st_in.data_ptr() if st_in is not None else None, ws.data_ptr(), ws.numel(), flags,
        stream()), "s2fp8")
    hdr = ws[:32].cpu().numpy().view(np.float32)
    stats = dict(mu=hdr[0], m=hdr[1], alpha=hdr[2], beta=hdr[3], beta_pow2=hdr[4],
                 inv_beta_pow2=hdr[5], inv_alpha=hdr[6],
                 gave_up=int(ws[40:44].cpu().numpy().view(np.uint32)[0]))
    return y, stats


def golden_x(d, meta):
    """The golden input on the device in the case's dtype (fixtures store exact float32 values)."""
    return to_dev(d["x"].astype(np.float32), TORCH_DT[meta.get("dtype", "f32")])


def to_dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV)
