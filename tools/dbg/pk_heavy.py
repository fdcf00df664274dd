import sys, numpy as np, torch
sys.path[:0] = ["tests", ".", "smart-quantization_amd"]
from helpers import smaq_hparams, n_diff_f32
from smart_compress_amd.compress import SmartFP, SmartFPPacked
from oracle import smaq_packed as P
hp = smaq_hparams()
pk, ref = SmartFPPacked(hp), SmartFP(hp)
for c in (pk, ref):
    c.rng.seed, c.rng.offset = 12, 7
n = 9 * 4096 + 333
rs = np.random.default_rng(2)
x_np = rs.standard_normal(n).astype(np.float32)
for b in (1, 4, 8, 9):
    s = slice(b * 4096, min(n, (b + 1) * 4096))
    sel = rs.random(x_np[s].size) < 0.2
    x_np[s][sel] *= 1e4
x = torch.from_numpy(x_np).cuda()
packed = pk.compress(x)
y = pk.decompress(packed).cpu().numpy()
yr = ref(x).cpu().numpy()
raw = packed.data.cpu().numpy()
yo = P.unpack(raw)
print("gpu vs ref", n_diff_f32(y, yr), "oracle-unpack vs ref", n_diff_f32(yo, yr), "gpu vs oracle-unpack", n_diff_f32(y, yo))
bad = np.nonzero(y.view(np.uint32) != yo.view(np.uint32))[0]
print("bad idx", bad[:20], "blocks", np.unique(bad // 4096))
print(y[bad[:5]], yo[bad[:5]])
h, dirs, fx, vw = P.regions(raw)
print([(int(d) & ((1<<38)-1), (int(d)>>38)&0x1fff, int(d)>>51) for d in dirs])
