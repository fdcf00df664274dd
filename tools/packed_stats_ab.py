"""Why the packed compress's statistics launch takes longer than the headline's (measurement script,
not product): 256M fp32 N(0,1), two alternating inputs, K iterations of one mode, meant to run under
`rocprofv3 --kernel-trace --stats` (one process per mode) so smaq_stats_kernel's average can be
compared between modes:
  compress      compress only
  packed        compress + decompress (bench.py --config packed)
  packed_nt     compress + decompress, then a 1 GiB read-only sweep before the next statistics
  roundtrip     smq_smaq_roundtrip (the headline)

python tools/packed_stats_ab.py <mode> [iters]"""

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

from helpers import smaq_hparams  # noqa: E402
from smart_compress_amd import _native as N  # noqa: E402
from smart_compress_amd.compress.packed import SmartFPPacked  # noqa: E402


def main():
    mode = sys.argv[1]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda", 0)
    n = 1 << 28
    hp = smaq_hparams()
    codec = SmartFPPacked(hp)
    gen = torch.Generator(device=dev).manual_seed(0)
    xs = [torch.randn(n, generator=gen, device=dev) for _ in range(2)]
    lib = N.lib()
    bound = lib.smq_smaq_pack_bound(n, hp.num_bits_main, hp.num_bits_outlier)
    packed = torch.empty(bound, dtype=torch.uint8, device=dev)
    ws = torch.zeros(lib.smq_smaq_pack_workspace_bytes(n), dtype=torch.uint8, device=dev)
    y = torch.empty(n, dtype=torch.float32, device=dev)
    other = torch.empty(n, dtype=torch.float32, device=dev).fill_(1.0)
    st = torch.cuda.current_stream(dev).cuda_stream
    for i in range(iters):
        x = xs[i & 1]
        p = codec._params(n, False)
        if mode == "roundtrip":
            N.check(lib.smq_smaq_roundtrip(x.data_ptr(), N.SMQ_DTYPE_F32, y.data_ptr(), n, p, None,
                                           ws.data_ptr(), ws.numel(), st), "roundtrip")
            continue
        N.check(lib.smq_smaq_compress(x.data_ptr(), N.SMQ_DTYPE_F32, n, p, packed.data_ptr(),
                                      bound, ws.data_ptr(), ws.numel(), st), "compress")
        if mode in ("packed", "packed_nt"):
            N.check(lib.smq_smaq_decompress_ex(packed.data_ptr(), y.data_ptr(), n,
                                               hp.num_bits_main, hp.num_bits_outlier, st),
                    "decompress")
        if mode == "packed_nt":
            other.sum()
    torch.cuda.synchronize()
    print(mode, "done", flush=True)


if __name__ == "__main__":
    main()
