"""Generate golden vectors by running the REFERENCE implementation (container-only tooling).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
Needs /root/reference (read-only); on the GPU box it is absent and this script is never run —
only its outputs (tests/golden/*.npz, *.json, committed) travel.

What is executed from the reference, unmodified:
  smart_compress/compress/smart.py       SmartFP (all modes), argparse flags
  smart_compress/compress/{fp8,fp16,bf16,s2fp8}.py, util/pytorch/quantization.py (float_quantize
  wrapper with check_inf), compress/base.py (log_ratio / log_size metric keys)

Two missing dependencies are substituted, and only those:
  * smart_compress.util.globals imports pytorch_lightning (absent) for a type annotation; it is
    replaced by a module exposing the same `Globals` with a no-op `profiler.profile()`.
  * qtorch 0.2.0 (absent, un-vendored) is replaced by oracle/qtorch_float.py (the restated
    quantiser) whose random words are recorded. Fixtures that pass through it pin the REFERENCE'S
    wrapper and S2FP8 transform code, not qtorch itself (see oracle/__init__.py).

Randomness is captured, not reproduced: torch.rand_like / torch.randperm are wrapped so that the
uniforms and sample indices the reference drew are saved next to its outputs.
"""

import contextlib
import json
import os
import sys
import types
from argparse import ArgumentParser

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def _install_stubs(record):
    g = types.ModuleType("smart_compress.util.globals")

    class _Prof:
        @contextlib.contextmanager
        def profile(self, name):
            yield

    class Globals:
        compression = None
        profiler = _Prof()

    g.Globals = Globals
    sys.modules["smart_compress.util.globals"] = g

    from oracle import qtorch_float as qf

    qmod = types.ModuleType("qtorch.quant.quant_function")
    record["_rs"] = np.random.default_rng(1234)

    def float_quantize(x, exp, man, rounding="stochastic"):
        xn = x.detach().cpu().numpy().astype(np.float32)
        if rounding == "nearest":
            y = qf.quantize(xn, exp, man, stochastic=False)
        else:
            r = record["_rs"].integers(0, 2**31 - 1, size=xn.shape, dtype=np.uint32)  # randint_like(INT_MAX)
            record.setdefault("q_in", []).append(xn.copy())
            record.setdefault("q_rand", []).append(r)
            y = qf.quantize(xn, exp, man, r, stochastic=True)
        # fp64 input (gen_f64 only): the dtype-generic extension qtorch's data_ptr<float>() kernel
        # lacks — zeros_like(x) filled with the quantised fp32(x) (include/smq.h SMQ_DTYPE_F64)
        dt = torch.float64 if x.dtype == torch.float64 else torch.float32
        return torch.from_numpy(y).to(device=x.device, dtype=dt)

    qmod.float_quantize = float_quantize
    for name in ("qtorch", "qtorch.quant"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["qtorch.quant.quant_function"] = qmod
    sys.path.insert(0, REF)


class Capture:
    """Wrap torch.rand_like / torch.randperm to record the reference's draws."""

    def __init__(self):
        self.uniforms = []
        self.perms = []

    def __enter__(self):
        self._rl, self._rp = torch.rand_like, torch.randperm
        cap = self

        def rand_like(*a, **k):
            out = cap._rl(*a, **k)
            cap.uniforms.append(out.detach().cpu().numpy().copy())
            return out

        def randperm(*a, **k):
            out = cap._rp(*a, **k)
            cap.perms.append(out.detach().cpu().numpy().copy())
            return out

        torch.rand_like, torch.randperm = rand_like, randperm
        return self

    def __exit__(self, *exc):
        torch.rand_like, torch.randperm = self._rl, self._rp


def smaq_hparams(SmartFP, argv, precision=32):
    hp = SmartFP.add_argparse_args(ArgumentParser()).parse_args(argv)
    hp.precision = precision
    return hp


def gen_smaq(out_dir):
    from smart_compress.compress.smart import SmartFP

    g = torch.Generator().manual_seed(20250310)

    def normal(n, mu=0.0, sd=1.0):
        return (torch.randn(n, generator=g) * sd + mu).float()

    cases = []

    def case(name, x, argv=(), all_positive=False, bn=None, dtype=torch.float32, precision=32):
        cases.append((name, x.to(dtype), list(argv), all_positive, bn, precision))

    n = 16384
    case("normal", normal(n))
    case("normal_trunc", normal(n), ["--no_stochastic_rounding"])
    case("small_scale", normal(n, 0.01, 0.05))
    lap = torch.distributions.Laplace(0.0, 1.0).sample((n,))
    case("laplace", lap.float())
    st = torch.distributions.StudentT(2.0).sample((n,))
    case("student_t2", st.float())
    case("student_t2_trunc", st.float(), ["--no_stochastic_rounding"])
    case("relu_allpos", torch.relu(normal(n)), all_positive=True)
    case("adam_exp_avg_sq", (normal(n) ** 2 * 1e-6).float(), all_positive=True)
    case("constant", torch.full((4096,), 0.75))
    case("n7_passthrough", normal(7))
    case("n8", normal(8))
    case("ragged_1001", normal(1001, 3.0, 2.0))
    for bm, bo in ((4, 6), (5, 7), (3, 5), (3, 3), (2, 3)):
        case(f"bits_{bm}_{bo}", normal(n), ["--num_bits_main", str(bm), "--num_bits_outlier", str(bo)])
    case("thresholds_0.8_3.0", normal(n), ["--main_std_dev_threshold", "0.8",
                                           "--outlier_std_dev_threshold", "3.0"])
    case("range_std", normal(n), ["--use_range_std_dev"])
    case("range_std_trunc", normal(n), ["--use_range_std_dev", "--no_stochastic_rounding"])
    case("sampled", normal(n), ["--use_sample_stats"])
    case("sampled_trunc", normal(n), ["--use_sample_stats", "--no_stochastic_rounding"])
    case("sampled_range", normal(n), ["--use_sample_stats", "--use_range_std_dev"])
    case("sampled_32", normal(n), ["--use_sample_stats", "--num_samples", "32"])
    case("large_mean", normal(n, 1000.0, 0.5))
    case("grad_like", normal(65536, 0.0, 1e-3))
    x4 = normal(2 * 8 * 6 * 5).reshape(2, 8, 6, 5)
    gam = (torch.rand(8, generator=g) + 0.5).float()
    bet = (torch.randn(8, generator=g) * 0.1).float()
    case("bn", x4, ["--use_batch_norm"], bn=(gam, bet))
    case("bn_scalar", x4, ["--use_batch_norm", "--bn_scalar_params"], bn=(gam, bet))
    case("bn_trunc", x4, ["--use_batch_norm", "--no_stochastic_rounding"], bn=(gam, bet))
    # half inputs (Lightning precision=16): stats and z-score in the input type, fp32 output
    h16 = dict(dtype=torch.float16, precision=16)
    case("f16_normal", normal(n), **h16)
    case("f16_trunc", normal(n, 0.5, 3.0), ["--no_stochastic_rounding"], **h16)
    case("f16_sampled", normal(n), ["--use_sample_stats"], **h16)
    case("f16_range", normal(n), ["--use_range_std_dev"], **h16)
    case("f16_range_big", normal(70000), ["--use_range_std_dev"], **h16)  # half(n) = inf -> std 1
    case("f16_relu_allpos", torch.relu(normal(n)), all_positive=True, **h16)
    case("f16_constant", torch.full((4096,), 0.75), **h16)
    case("f16_thresholds", normal(n), ["--main_std_dev_threshold", "0.8",
                                       "--outlier_std_dev_threshold", "3.0"], **h16)
    case("f16_bn", x4, ["--use_batch_norm"], bn=(gam, bet), **h16)
    case("bf16_normal", normal(n), dtype=torch.bfloat16, precision=16)
    case("bf16_normal_p32", normal(n, 0.1, 2.0), dtype=torch.bfloat16, precision=32)
    case("bf16_trunc", normal(n), ["--no_stochastic_rounding"], dtype=torch.bfloat16, precision=16)
    case("bf16_sampled", normal(n), ["--use_sample_stats"], dtype=torch.bfloat16, precision=16)
    case("bf16_range", normal(n), ["--use_range_std_dev"], dtype=torch.bfloat16, precision=16)
    # negative thresholds (T = 0 divides by zero at smart.py:78; T < 0 gives, smart.py:157-161,
    # elements above -T and below T at once) — appended, so the cases above keep their draws
    case("thr_neg", normal(n), ["--main_std_dev_threshold", "-0.5"])
    case("thr_neg_trunc", normal(n), ["--main_std_dev_threshold", "-1.25", "--no_stochastic_rounding"])
    case("f16_thr_neg", normal(n), ["--main_std_dev_threshold", "-0.5"], **h16)
    case("bn_thr_neg", x4, ["--use_batch_norm", "--main_std_dev_threshold", "-0.5"], bn=(gam, bet),
         all_positive=True)

    index = {}
    for name, x, argv, allpos, bn, precision in cases:
        hp = smaq_hparams(SmartFP, argv + ["--measure_compression_ratio"], precision)
        codec = SmartFP(hp)
        logged = {}
        codec.log = lambda k, v, **kw: logged.__setitem__(k, v)
        torch.manual_seed(len(index) + 7)
        with Capture() as cap:
            kwargs = dict(all_positive=allpos)
            if bn is not None:
                kwargs["batch_norm_stats"] = bn
            y = codec(x, tag="golden", **kwargs)
        rec = dict(x=x.float().numpy(), y=y.float().numpy(), passthrough=np.array(y is x),
                   y_dtype=np.array(str(y.dtype)))
        if cap.uniforms:
            rec["uniforms"] = cap.uniforms[0].astype(np.float32)
        if x.numel() >= hp.min_size:
            if cap.perms:  # the reference's own sampled statistics on the recorded indices
                idx = cap.perms[0][: min(x.numel(), hp.num_samples)]
                rec["sample_idx"] = idx.astype(np.int64)
                sample = x.reshape(-1)[torch.from_numpy(idx)]
                mean, std = sample.mean(), codec._get_std(sample, unbiased=False)
            else:
                mean, std = x.mean(), codec._get_std(x)
            rec["mean"] = np.float32(mean.float().item())
            rec["std"] = np.float32(std.float().item())
        if bn is not None:
            rec["bn_gamma"], rec["bn_beta"] = bn[0].numpy(), bn[1].numpy()
            if hp.bn_scalar_params:  # what smart.py:146-148 actually applies
                rec["bn_gamma_used"] = np.array([bn[0].mean().item()], dtype=np.float32)
                rec["bn_beta_used"] = np.array([bn[1].mean().item()], dtype=np.float32)
        new_size = logged.get("new_size")
        if new_size is not None and x.numel() >= hp.min_size:
            n_el = x.numel()
            rec["n_outlier"] = np.int64(round((new_size - n_el * hp.num_bits_main)
                                              / (hp.num_bits_outlier - hp.num_bits_main))) \
                if hp.num_bits_outlier != hp.num_bits_main else np.int64(-1)
        np.savez_compressed(os.path.join(out_dir, f"smaq_{name}.npz"), **rec)
        meta = vars(hp).copy()
        meta.update(all_positive=allpos, logged={k: float(v) for k, v in logged.items()},
                    range_outlier=codec.range_outlier, range_normal=codec.range_normal,
                    dtype={torch.float32: "f32", torch.float16: "f16", torch.bfloat16: "bf16"}[x.dtype])
        index[name] = meta
    with open(os.path.join(out_dir, "smaq_cases.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


def gen_float(out_dir, record):
    from smart_compress.compress.fp8 import FP8
    from smart_compress.compress.fp16 import FP16
    from smart_compress.compress.bf16 import BF16
    from smart_compress.compress.s2fp8 import S2FP8
    from smart_compress.util.pytorch import quantization as Q

    g = torch.Generator().manual_seed(77)
    n = 8192
    specials = torch.tensor([0.0, -0.0, 57344.0, -57344.0, 60000.0, -70000.0, 1e-6, -3e-5,
                             2.0**-14, 2.0**-16, 3 * 2.0**-17, 65504.0, float("inf"), float("-inf"),
                             1.0, -1.5, 0.3, 3.4e38, -3.4e38, 1e-40])
    inputs = {
        "normal": torch.randn(n, generator=g),
        "relu": torch.relu(torch.randn(n, generator=g)),
        "wide": torch.randn(n, generator=g) * torch.exp(torch.randn(n, generator=g) * 6),
        "specials": specials,
    }
    index = {}
    for cname, cls in (("fp8", FP8), ("fp16", FP16), ("bf16", BF16), ("s2fp8", S2FP8)):
        for check_inf in (True, False):
            argv = [] if check_inf else ["--no_float_quantize_check_inf"]
            hp = cls.add_argparse_args(ArgumentParser()).parse_args(argv)
            hp.precision = 32
            codec = cls(hp)
            for iname, x in inputs.items():
                if cname == "s2fp8" and iname == "specials":
                    continue
                _clear(record)
                y = codec(x.float(), tag="golden")
                rec = dict(x=x.float().numpy(), y=y.numpy(),
                           q_in=record["q_in"][0], q_rand=record["q_rand"][0])
                if cname == "s2fp8":  # the statistics s2fp8.py:31-43 computes, same torch ops
                    xa = x.float().abs()
                    lg = torch.where(xa == 0.0, xa, torch.log2(xa))
                    mu, mx = torch.mean(lg), torch.max(lg)
                    alpha = 15.0 / (mx - mu)
                    beta = -alpha * mu
                    rec.update(mu=np.float32(mu.item()), m=np.float32(mx.item()),
                               alpha=np.float32(alpha.item()), beta=np.float32(beta.item()),
                               beta_pow2=np.float32((2.0 ** beta).item()))
                key = f"{cname}_{iname}_{'inf' if check_inf else 'noinf'}"
                np.savez_compressed(os.path.join(out_dir, f"float_{key}.npz"), **rec)
                index[key] = dict(codec=cname, check_inf=check_inf, input=iname)
    maxv = {f"{e}_{m}": float(Q._get_max_value(e, m)) for e, m in ((5, 2), (5, 10), (8, 7), (4, 3))}
    argd = {c.__name__: vars(c.add_argparse_args(ArgumentParser()).parse_args([]))
            for c in (FP8, FP16, BF16, S2FP8)}
    with open(os.path.join(out_dir, "float_cases.json"), "w") as f:
        json.dump(dict(cases=index, max_values=maxv, argparse_defaults=argd), f, indent=1,
                  sort_keys=True)


def _clear(record):
    for k in [k for k in record if not k.startswith("_")]:
        del record[k]


def gen_s2fp8_p16(out_dir, record):
    """S2FP8 at Lightning precision 16 (s2fp8.py:27-48 with quantization.py:187-204's half branch):
    fp16 / bf16 inputs run the statistics and the forward transform in their own type, fp32 inputs
    in fp32; float_quantize returns half, so the inverse transform runs in half; `* signs` gives
    the output type (fp16 for fp16 inputs, fp32 otherwise). Own random stream and index file."""
    from smart_compress.compress.s2fp8 import S2FP8

    record["_rs"] = np.random.default_rng(4321)
    g = torch.Generator().manual_seed(1616)
    n = 8192
    base = {
        "normal": torch.randn(n, generator=g),
        "relu": torch.relu(torch.randn(n, generator=g)),
        "wide": torch.randn(n, generator=g) * torch.exp(torch.randn(n, generator=g) * 2),
        "tiny": torch.randn(n, generator=g) * 1e-3,
    }
    dtypes = {"f16": torch.float16, "bf16": torch.bfloat16, "f32": torch.float32}
    index = {}
    for check_inf in (True, False):
        argv = [] if check_inf else ["--no_float_quantize_check_inf"]
        hp = S2FP8.add_argparse_args(ArgumentParser()).parse_args(argv)
        hp.precision = 16
        codec = S2FP8(hp)
        for dname, dt in dtypes.items():
            for iname, x0 in base.items():
                x = x0.to(dt)
                _clear(record)
                y = codec(x.clone(), tag="golden")
                xa = x.abs()  # the statistics s2fp8.py:31-43 computes, same torch ops and dtype
                lg = torch.where(xa == 0.0, xa, torch.log2(xa))
                mu, mx = torch.mean(lg), torch.max(lg)
                alpha = 15.0 / (mx - mu)
                beta = -alpha * mu
                rec = dict(x=x.float().numpy(), y=y.float().numpy(),
                           q_in=record["q_in"][0], q_rand=record["q_rand"][0],
                           mu=np.float32(mu.item()), m=np.float32(mx.item()),
                           alpha=np.float32(alpha.item()), beta=np.float32(beta.item()),
                           beta_pow2=np.float32((2.0 ** beta).item()))
                key = f"{dname}_{iname}_{'inf' if check_inf else 'noinf'}"
                np.savez_compressed(os.path.join(out_dir, f"s2p16_{key}.npz"), **rec)
                index[key] = dict(dtype=dname, out_dtype={torch.float16: "f16",
                                  torch.float32: "f32"}[y.dtype], check_inf=check_inf, input=iname)
    with open(os.path.join(out_dir, "s2fp8_p16_cases.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


def gen_f64(out_dir, record):
    """float64 tensors through SmartFP (every statistics mode, BN, thresholds that fp32 cannot
    hold), FP8 (precision 32: dtype-generic quantiser; 16: x.float() / .half()) and S2FP8 (both
    precisions). Own random streams and index file; the SmaQ uniforms are the fp64 draws."""
    from smart_compress.compress.fp8 import FP8
    from smart_compress.compress.s2fp8 import S2FP8
    from smart_compress.compress.smart import SmartFP

    g = torch.Generator().manual_seed(6464)

    def normal(n, mu=0.0, sd=1.0):
        return torch.randn(n, generator=g, dtype=torch.float64) * sd + mu

    n = 16384
    x4 = normal(2 * 8 * 6 * 5).reshape(2, 8, 6, 5)
    gam = torch.rand(8, generator=g, dtype=torch.float64) + 0.5
    bet = torch.randn(8, generator=g, dtype=torch.float64) * 0.1
    smaq = [
        ("normal", normal(n), [], False, None, 32),
        ("trunc", normal(n, 0.3, 2.0), ["--no_stochastic_rounding"], False, None, 32),
        ("range", normal(n), ["--use_range_std_dev"], False, None, 32),
        ("sampled", normal(n), ["--use_sample_stats"], False, None, 32),
        ("sampled_range", normal(n), ["--use_sample_stats", "--use_range_std_dev"], False, None, 32),
        ("relu_allpos", torch.relu(normal(n)), [], True, None, 32),
        ("thresholds", normal(n), ["--main_std_dev_threshold", "0.7",
                                   "--outlier_std_dev_threshold", "2.9"], False, None, 32),
        ("bits_3_5", normal(n), ["--num_bits_main", "3", "--num_bits_outlier", "5"], False, None, 32),
        ("large_mean", normal(n, 1e6, 0.25), [], False, None, 32),
        ("tiny", normal(n, 0.0, 1e-30), [], False, None, 16),
        ("p16", normal(n, 2.0, 3.0), [], False, None, 16),
        ("bn", x4, ["--use_batch_norm"], False, (gam, bet), 32),
        ("constant", torch.full((4096,), 0.75, dtype=torch.float64), [], False, None, 32),
    ]
    index = {}
    for name, x, argv, allpos, bn, precision in smaq:
        hp = smaq_hparams(SmartFP, argv + ["--measure_compression_ratio"], precision)
        codec = SmartFP(hp)
        logged = {}
        codec.log = lambda k, v, **kw: logged.__setitem__(k, v)
        torch.manual_seed(len(index) + 64)
        with Capture() as cap:
            kwargs = dict(all_positive=allpos)
            if bn is not None:
                kwargs["batch_norm_stats"] = bn
            y = codec(x, tag="golden", **kwargs)
        rec = dict(x=x.numpy(), y=y.numpy(), y_dtype=np.array(str(y.dtype)))
        if cap.uniforms:
            rec["uniforms"] = cap.uniforms[0].astype(np.float64)
        if cap.perms:
            idx = cap.perms[0][: min(x.numel(), hp.num_samples)]
            rec["sample_idx"] = idx.astype(np.int64)
            sample = x.reshape(-1)[torch.from_numpy(idx)]
            mean, std = sample.mean(), codec._get_std(sample, unbiased=False)
        else:
            mean, std = x.mean(), codec._get_std(x)
        rec["mean"], rec["std"] = np.float64(mean.item()), np.float64(std.item())
        if bn is not None:
            rec["bn_gamma"], rec["bn_beta"] = bn[0].numpy(), bn[1].numpy()
        new_size = logged.get("new_size")
        if new_size is not None:
            rec["n_outlier"] = np.int64(round((new_size - x.numel() * hp.num_bits_main)
                                              / (hp.num_bits_outlier - hp.num_bits_main)))
        np.savez_compressed(os.path.join(out_dir, f"f64_smaq_{name}.npz"), **rec)
        meta = vars(hp).copy()
        meta.update(all_positive=allpos, kind="smaq")
        index[f"smaq_{name}"] = meta
    record["_rs"] = np.random.default_rng(6400)
    inputs = {
        "normal": torch.randn(4096, generator=g, dtype=torch.float64),
        "wide": torch.randn(4096, generator=g, dtype=torch.float64)
        * torch.exp(torch.randn(4096, generator=g, dtype=torch.float64) * 3),
    }
    # S2FP8 at precision 16 computes `t1 ** (1 / alpha)` on half values (s2fp8.py:48); on this draw
    # (found by a 400-draw search against the reference) a float pow that is not correctly
    # rounded (a libm powf) moves 23 elements by one half ulp, while double pow rounded to float
    # then half reproduces every element: it decides which pow the oracle and the device follow
    g2 = torch.Generator().manual_seed(1015)
    pow_case = torch.randn(4096, generator=g2, dtype=torch.float64) * 3.0
    for cname, cls in (("fp8", FP8), ("s2fp8", S2FP8)):
        for precision in (32, 16):
            if cname == "s2fp8" and precision == 16:
                inputs["powcase"] = pow_case
            else:
                inputs.pop("powcase", None)
            hp = cls.add_argparse_args(ArgumentParser()).parse_args([])
            hp.precision = precision
            codec = cls(hp)
            for iname, x in inputs.items():
                _clear(record)
                y = codec(x.clone(), tag="golden")
                rec = dict(x=x.numpy(), y=y.double().numpy(), y_dtype=np.array(str(y.dtype)),
                           q_in=record["q_in"][0], q_rand=record["q_rand"][0])
                if cname == "s2fp8":
                    xa = x.abs()
                    lg = torch.where(xa == 0.0, xa, torch.log2(xa))
                    mu, mx = torch.mean(lg), torch.max(lg)
                    alpha = 15.0 / (mx - mu)
                    beta = -alpha * mu
                    rec.update(mu=np.float64(mu.item()), m=np.float64(mx.item()),
                               alpha=np.float64(alpha.item()), beta=np.float64(beta.item()),
                               beta_pow2=np.float64((2.0 ** beta).item()))
                key = f"{cname}_p{precision}_{iname}"
                np.savez_compressed(os.path.join(out_dir, f"f64_{key}.npz"), **rec)
                index[key] = dict(kind=cname, precision=precision, input=iname,
                                  y_dtype=str(y.dtype))
    with open(os.path.join(out_dir, "f64_cases.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True, default=str)


def main():
    if not os.path.isdir(REF):
        print("reference not present; nothing to do")
        return
    record = {}
    _install_stubs(record)
    out_dir = HERE
    only = sys.argv[1] if len(sys.argv) > 1 else None  # e.g. `s2fp8_p16`: one generator
    if only in (None, "smaq"):
        gen_smaq(out_dir)
    if only in (None, "float"):
        gen_float(out_dir, record)
    if only in (None, "s2fp8_p16"):
        gen_s2fp8_p16(out_dir, record)
    if only in (None, "f64"):
        gen_f64(out_dir, record)
    print("golden vectors written to", out_dir)


if __name__ == "__main__":
    main()
