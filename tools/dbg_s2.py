import sys, os
sys.path[:0] = ["/root/repo", "/root/repo/smart-quantization_amd", "/root/repo/tests"]
import numpy as np, torch
import gpu_calls as g
from oracle import s2fp8 as os2
from test_gpu_float import _ulps
gen = torch.Generator(device="cuda").manual_seed(4)
x = torch.randn(32, 128, 768, generator=gen, device="cuda")
Y, st = g.s2fp8(x, seed=8, offset=3, flags=g.N.SMQ_S2FP8_OUT_Y)
xn = x.cpu().numpy().ravel()
so = os2.derive(st["mu"], st["m"])
Yo = os2.transform(xn, so)
Yd = Y.cpu().numpy().ravel()
u = _ulps(Yd, Yo)
bad = np.argsort(-u)[:8]
print("st", st)
for i in bad:
    print(i, u[i], xn[i], Yd[i], Yo[i])
print("n bad>128:", int((u > 128).sum()))
badi = np.nonzero(u > 128)[0]
if badi.size:
    j = badi // 4
    import collections
    print("comp", collections.Counter((badi % 4).tolist()))
    print("u-slot", collections.Counter(((j % 1024) // 256).tolist()))
    print("tiles", len(set((j // 1024).tolist())), "lanes", len(set((j % 256).tolist())))
    print("per tile counts", sorted(collections.Counter((j // 1024).tolist()).values())[:10])
    print("wave", collections.Counter(((j % 256) // 64).tolist()))
