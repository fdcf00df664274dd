"""Dump precision-16 S2FP8 device outputs + stats for offline comparison with the oracle."""
import sys
import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
sys.path.insert(0, "smart-quantization_amd")
import gpu_calls as g

out = {}
for dt in ("f16", "bf16", "f32"):
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[dt]
    n = 1 << 20 | 3
    gen = torch.Generator(device="cuda").manual_seed(5)
    base = torch.randn(n + 1, generator=gen, device="cuda").to(tdt)
    base[::9] = 0.0
    for tag, x in (("a", base[:n]), ("u", base[1:])):
        y, st = g.s2fp8(x, check_inf=True, seed=21, offset=7, precision=16)
        out[f"{dt}_{tag}_x"] = x.float().cpu().numpy()
        out[f"{dt}_{tag}_y"] = y.float().cpu().numpy()
        out[f"{dt}_{tag}_st"] = np.array([st[k] for k in ("mu", "m", "alpha", "beta", "beta_pow2",
                                                           "inv_beta_pow2", "inv_alpha")])
np.savez_compressed("gpurun_out/diag_s2p16.npz", **out)
print("ok")
