"""Benchmark of the SmaQ 6/8-bit compress->decompress round trip on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): one contiguous 268,435,456-element fp32 tensor
(1 GiB, x ~ N(0,1), generated on the device), SmartFP defaults (6/8 bits, thresholds 1.0/2.5,
full statistics, stochastic rounding), through the drop-in SmartFP.__call__ -> libsmq C-ABI.
A "step" = one round trip of that tensor (stats launch + apply launch, output tensor allocated by
the codec like the reference). value = algorithmic bytes (12 B/elem: stats read + apply read +
write) over all ranks / max-over-ranks wall time of the K timed steps.

Multi-GPU: one process per GPU (torchrun), each rank owns its own 256M tensor (independent
units, "weak" scaling, no data-path collective; the only collectives are the timing barrier and
the max-over-ranks reduction of the elapsed time).

Other configs (--config fp8 | s2fp8 | multi | smaq_sampled) are measurement aids, not the line
the driver records.

roofline: the dominant kernel is smaq_apply_kernel (8 B/elem algorithmic); its average duration is
measured with events on the codec's stream around every launch inside the timed region.
cpu_baseline: the oracle (numpy restatement of smart.py, single thread) on a bounded sample.
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "smart-quantization_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "SmaQ 6/8-bit quant+dequant round-trip GB/s (and % HBM peak), 256M fp32"


def _hip_runtime():
    """The HIP runtime this process already uses (torch's copy), for events with flags torch does
    not expose."""
    import ctypes

    path = None
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                path = line.split()[-1]
                break
    lib = ctypes.CDLL(path or "libamdhip64.so")
    lib.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    lib.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.hipEventSynchronize.argtypes = [ctypes.c_void_p]
    lib.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                        ctypes.c_void_p]
    lib.hipEventDestroy.argtypes = [ctypes.c_void_p]
    return lib


HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000  # hip_runtime_api.h


class EventTrace:
    """HIP events recorded on the current stream around each named kernel launch. Created with
    hipEventDisableSystemFence: a default timing event's system-scope release writes back and
    invalidates the caches at every record, which lengthened the bracketed apply launch by ~3 %
    (0.352 vs rocprofv3's 0.342 ms)."""

    def __init__(self):
        self.pairs = {}
        self.enabled = True
        self._hip = _hip_runtime()  # resolved here, never inside a timed region

    def _event(self):
        import ctypes

        ev = ctypes.c_void_p()
        if self._hip.hipEventCreateWithFlags(ctypes.byref(ev), HIP_EVENT_DISABLE_SYSTEM_FENCE):
            raise RuntimeError("hipEventCreateWithFlags failed")
        if self._hip.hipEventRecord(ev, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)):
            raise RuntimeError("hipEventRecord failed")
        return ev

    def begin(self, name):
        if self.enabled:
            self.pairs.setdefault(name, []).append([self._event(), None])

    def end(self, name):
        if self.enabled:
            self.pairs[name][-1][1] = self._event()

    def mean_ms(self, name):
        import ctypes

        ps = self.pairs.get(name, [])
        if not ps:
            return None
        out = []
        for a, b in ps:
            self._hip.hipEventSynchronize(b)
            ms = ctypes.c_float()
            if self._hip.hipEventElapsedTime(ctypes.byref(ms), a, b):
                raise RuntimeError("hipEventElapsedTime failed")
            out.append(ms.value)
        return float(np.mean(out))

    def reset(self):
        for ps in self.pairs.values():
            for a, b in ps:
                self._hip.hipEventDestroy(a)
                self._hip.hipEventDestroy(b)
        self.pairs = {}


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("SMQ_BENCH_SHARE_DEVICE") == "1":
        local = 0  # rehearsal of the N>1 flow on a 1-GPU box (gloo collectives, shared card)
    if world > 1:
        import torch.distributed as dist

        backend = os.environ.get("SMQ_BENCH_BACKEND", "nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def _coll_device(device):
    import torch.distributed as dist

    return device if dist.get_backend() == "nccl" else torch.device("cpu")


def max_over_ranks(value, world, device):
    if world == 1:
        return value
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, world, device):
    if world == 1:
        return value
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def smaq_hparams(**over):
    from argparse import ArgumentParser

    from smart_compress_amd.compress.smart import SmartFP

    hp = SmartFP.add_argparse_args(ArgumentParser()).parse_args([])
    hp.precision = 32
    for k, v in over.items():
        setattr(hp, k, v)
    return hp


HOST = {}
PREWARM_S = 0.5


def prewarm(step, device):
    """Setup, not measurement: run the step untimed for ~PREWARM_S seconds so every buffer of the
    workload (2 inputs, the recycled outputs, workspaces: ~4 GiB at the default size) has been
    touched and its address translations are warm before the W warmup steps. Measured on MI355X:
    with only 3 warm-up steps the apply kernel ran 12 % slower than in steady state."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < PREWARM_S:
        step()
        torch.cuda.synchronize()


def time_steps(step, steps, warmup, world, device, region=None):
    """region: optional (start, end) EventTrace pair recorded on the launch stream at the two ends
    of the timed region (no event between the steps)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if region is not None:
        region.begin("region")
    for _ in range(steps):
        step()
    if region is not None:
        region.end("region")
    HOST["enqueue_ms_per_step"] = (time.perf_counter() - t0) / steps * 1e3
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    return max_over_ranks(elapsed, world, device)


def cpu_baseline_smaq(sample_elems, budget_s):
    """The reference's algorithm on the host cores: oracle/smaq_torch.py, smart.py's own torch-CPU
    op sequence (full stats, torch.rand_like SR; bit-exact with the reference's outputs on the
    golden fixtures), on a bounded sample, with as many intra-op threads as this job's CPU share
    (OMP_NUM_THREADS, 16 on the GPU box; os.cpu_count() counts the whole machine there)."""
    from oracle import smaq_torch

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        g = torch.Generator().manual_seed(0)
        x = torch.randn(sample_elems, generator=g)
        smaq_torch.roundtrip(x)  # warm-up (allocator, thread pool)
        reps, t_tot = 0, 0.0
        while t_tot < budget_s or reps < 2:
            t0 = time.perf_counter()
            smaq_torch.roundtrip(x)
            t_tot += time.perf_counter() - t0
            reps += 1
    finally:
        torch.set_num_threads(prev)
    gbps = 12.0 * sample_elems * reps / t_tot / 1e9
    return {"value": round(gbps, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x {sample_elems} fp32 N(0,1) round trips, oracle/smaq_torch.py "
                      f"(smart.py's torch-CPU op sequence, full stats + rand_like SR), "
                      f"{threads} threads, {t_tot:.1f} s"}


def traffic_from_profile(config):
    path = os.path.join(REPO, "profiles", f"traffic_{config}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("apply_bytes_per_launch")


def run_smaq(args, world, rank, device):
    from smart_compress_amd.compress.smart import SmartFP

    n = args.elements or (1 << 28)
    sampled = args.config == "smaq_sampled"
    hp = smaq_hparams(use_sample_stats=sampled)
    codec = SmartFP(hp)
    codec.rng.seed = 1000 + rank
    gen = torch.Generator(device=device).manual_seed(rank)
    # two input tensors, alternated per step, so a step never finds the previous step's input in
    # the 256 MB Infinity Cache (in training every call sees a different tensor)
    xs = [torch.randn(n, generator=gen, device=device) for _ in range(2)]
    # measurement knob SMQ_BENCH_DTYPE=f16|bf16: half-precision inputs (statistics and apply read
    # 2 B/elem, the output stays fp32: 8 B/elem of algorithmic traffic)
    in_dt = {"f16": torch.float16, "bf16": torch.bfloat16}.get(os.environ.get("SMQ_BENCH_DTYPE", ""))
    if in_dt is not None:
        xs = [x.to(in_dt) for x in xs]
        if in_dt == torch.float16:
            codec.hparams.precision = 16
    trace = EventTrace()
    codec._trace = trace
    out = {"i": 0}

    def step():
        out["y"] = codec(xs[out["i"] & 1])
        out["i"] += 1

    trace.enabled = False
    prewarm(step, device)
    for _ in range(args.warmup):
        step()
    # the K timed steps carry no per-launch event markers (an event pair between two launches
    # costs a few us per step); the apply launch duration for `roofline` is then measured with an
    # event pair around each apply launch over K more steps of the same workload, on the codec's
    # stream (SMQ_BENCH_EVENTS_IN_TIMED=1: events inside the timed steps instead)
    in_timed = os.environ.get("SMQ_BENCH_EVENTS_IN_TIMED") == "1"
    trace.enabled = in_timed
    elapsed = time_steps(step, args.steps, 0, world, device)
    if not in_timed:
        trace.enabled = True
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    in_bytes = 4 if in_dt is None else 2
    alg_per_elem = (in_bytes + 4) if sampled else (2 * in_bytes + 4)
    total_bytes = sum_over_ranks(alg_per_elem * n * args.steps, world, device)
    value = total_bytes / elapsed / 1e9
    apply_ms = trace.mean_ms("apply")
    apply_gbps = (in_bytes + 4.0) * n / (apply_ms * 1e-3) / 1e9
    res = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "fp32" if in_dt is None else f"{os.environ['SMQ_BENCH_DTYPE']} in, fp32 out",
        "data": "synthetic",
        "config": {"workload": "smaq_6_8_roundtrip_256M_fp32" if not sampled else
                   "smaq_6_8_roundtrip_sampled_stats", "elements_per_gpu": n,
                   "stats": "sampled(16)" if sampled else "full", "rounding": "stochastic",
                   "bits": "6/8", "alg_bytes_per_elem": alg_per_elem,
                   "parallelism": f"replicas{world}"},
        "pct_hbm_peak": round(100.0 * value / world / HBM_PEAK_GBPS, 2),
        "roofline": {"bound": "hbm", "kernel": "smaq_apply_kernel",
                     "achieved": round(apply_gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(apply_gbps / HBM_PEAK_GBPS, 4),
                     "alg_bytes_per_launch": int((in_bytes + 4) * n),
                     "avg_launch_ms": round(apply_ms, 5),
                     "traffic": traffic_from_profile(args.config)},
        # the statistics launch is not bracketed by events (an event between the two launches
        # costs ~1 %); its duration is in the committed rocprofv3 summary (profiles/)
        "host_enqueue_ms_per_step": round(HOST.get("enqueue_ms_per_step", 0.0), 4),
        "input_buffers": 2,
    }
    return res


def run_fp8(args, world, rank, device):
    """Config 3: FP8 (E5M2, fp8.py) on [128,256,28,28], rotating 8 buffer pairs (> MALL)."""
    from smart_compress_amd import _native as N

    shape = (128, 256, 28, 28)
    n = int(np.prod(shape))
    nbuf = 8
    gen = torch.Generator(device=device).manual_seed(rank)
    xs = [torch.relu(torch.randn(shape, generator=gen, device=device)) for _ in range(nbuf)]
    ys = [torch.empty_like(x) for x in xs]
    lib = N.lib()
    st = torch.cuda.current_stream(device).cuda_stream
    trace = EventTrace()
    it = [0]

    def step():
        i = it[0] % nbuf
        it[0] += 1
        N.check(lib.smq_float_quant_f32(xs[i].data_ptr(), ys[i].data_ptr(), n, 5, 2,
                                        N.SMQ_ROUND_STOCHASTIC, 1, None, 7, it[0] * n, st), "fq")

    prewarm(step, device)
    # one launch per step: events only at the two ends of the timed region (an event pair per
    # launch cost ~7 us of a 43 us step); the average launch time then includes its boundary
    elapsed = time_steps(step, args.steps, args.warmup, world, device, region=trace)
    total = sum_over_ranks(8.0 * n * args.steps, world, device)
    k_ms = trace.mean_ms("region") / args.steps
    gbps = 8.0 * n / (k_ms * 1e-3) / 1e9
    return {"metric": "FP8 E5M2 round-trip GB/s, [128,256,28,28] fp32", "value": round(total / elapsed / 1e9, 2),
            "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "host_enqueue_ms_per_step": round(HOST.get("enqueue_ms_per_step", 0.0), 4),
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "fp8_e5m2_roundtrip_resnet34_act", "shape": list(shape),
                       "rotating_buffers": nbuf},
            "roofline": {"bound": "hbm", "kernel": "float_quant_kernel", "achieved": round(gbps, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(gbps / HBM_PEAK_GBPS, 4),
                         "avg_launch_ms": round(k_ms, 5), "traffic": traffic_from_profile("fp8")}}


def run_s2fp8(args, world, rank, device):
    """Config 4: S2FP8 on [32,128,768], rotating 48 buffers (> MALL)."""
    from smart_compress_amd.compress.s2fp8 import S2FP8
    from argparse import ArgumentParser

    shape = (32, 128, 768)
    n = int(np.prod(shape))
    nbuf = int(os.environ.get("SMQ_BENCH_NBUF", "48"))  # measurement knob: 1 = MALL/TLB-warm
    hp = S2FP8.add_argparse_args(ArgumentParser()).parse_args([])
    hp.precision = 32
    codec = S2FP8(hp)
    gen = torch.Generator(device=device).manual_seed(rank)
    xs = [torch.randn(shape, generator=gen, device=device) for _ in range(nbuf)]
    it = [0]

    def step():
        codec(xs[it[0] % nbuf])
        it[0] += 1

    prewarm(step, device)
    elapsed = time_steps(step, args.steps, args.warmup, world, device)
    total = sum_over_ranks(12.0 * n * args.steps, world, device)
    return {"metric": "S2FP8 round-trip GB/s, [32,128,768] fp32", "value": round(total / elapsed / 1e9, 2),
            "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "host_enqueue_ms_per_step": round(HOST.get("enqueue_ms_per_step", 0.0), 4),
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "s2fp8_roundtrip_bert_hidden", "shape": list(shape),
                       "rotating_buffers": nbuf}}


RESNET34_PARAMS = (
    [(512, 512, 3, 3)] * 5 + [(512, 256, 3, 3)] + [(256, 256, 3, 3)] * 11 + [(256, 128, 3, 3)]
    + [(128, 128, 3, 3)] * 7 + [(512, 256, 1, 1), (128, 64, 3, 3)] + [(64, 64, 3, 3)] * 6
    + [(256, 128, 1, 1), (128, 64, 1, 1), (10, 512), (64, 3, 3, 3)] + [(512,)] * 14
    + [(256,)] * 26 + [(128,)] * 18 + [(64,)] * 14 + [(10,)]
)


def run_multi(args, world, rank, device):
    """Config 5: fused multi-tensor SmaQ over ResNet-34 (CIFAR) grads (110) + non-BN weights (38)."""
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    gen = torch.Generator(device=device).manual_seed(rank)
    grads = [torch.randn(s, generator=gen, device=device) * 1e-3 for s in RESNET34_PARAMS]
    weights = [torch.randn(s, generator=gen, device=device) * 0.05 for s in RESNET34_PARAMS
               if len(s) != 1]
    tensors = grads + weights
    n = sum(t.numel() for t in tensors)
    outs = [torch.empty_like(t) for t in tensors]
    m = SmaqMulti(smaq_hparams(), seed=rank)
    bound = m.bind(tensors, outs)  # fixed buffers: validated once, one call = two launches

    def step():
        bound()

    prewarm(step, device)
    elapsed = time_steps(step, args.steps, args.warmup, world, device)
    total = sum_over_ranks(12.0 * n * args.steps, world, device)
    return {"metric": "Fused multi-tensor SmaQ GB/s, ResNet-34 weights+grads per step",
            "value": round(total / elapsed / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "host_enqueue_ms_per_step": round(HOST.get("enqueue_ms_per_step", 0.0), 4),
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "smaq_multi_resnet34_weights_grads", "tensors": len(tensors),
                       "elements_per_gpu": n}}


def run_packed(args, world, rank, device):
    """Packed SmaQ container on the 256M config: compress (statistics + packing
    launch) then decompress, both through the C-ABI into preallocated buffers (no host sync)."""
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.packed import SmartFPPacked

    n = args.elements or (1 << 28)
    hp = smaq_hparams()
    codec = SmartFPPacked(hp)
    codec.rng.seed = 2000 + rank
    gen = torch.Generator(device=device).manual_seed(rank)
    xs = [torch.randn(n, generator=gen, device=device) for _ in range(2)]
    lib = N.lib()
    bound = lib.smq_smaq_pack_bound(n, hp.num_bits_main, hp.num_bits_outlier)
    packed = torch.empty(bound, dtype=torch.uint8, device=device)
    ws = torch.zeros(lib.smq_smaq_pack_workspace_bytes(n), dtype=torch.uint8, device=device)
    y = torch.empty(n, dtype=torch.float32, device=device)
    st = torch.cuda.current_stream(device).cuda_stream
    trace = EventTrace()
    it = [0]
    # SMQ_BENCH_PACK_FLAGS: smq_smaq_compress_ex flags (2 = SMQ_PACK_SINGLE, the one-launch packer)
    pack_flags = int(os.environ.get("SMQ_BENCH_PACK_FLAGS", "0"))

    def step():
        x = xs[it[0] & 1]
        it[0] += 1
        p = codec._params(n, False)
        trace.begin("compress")
        N.check(lib.smq_smaq_compress_ex(x.data_ptr(), N.SMQ_DTYPE_F32, n, p, packed.data_ptr(),
                                         bound, ws.data_ptr(), ws.numel(), pack_flags, st),
                "compress")
        trace.end("compress")
        trace.begin("unpack")
        N.check(lib.smq_smaq_decompress(packed.data_ptr(), y.data_ptr(), n, st), "decompress")
        trace.end("unpack")

    trace.enabled = False
    prewarm(step, device)
    for _ in range(args.warmup):
        step()
    # timed steps without event markers; compress / decompress durations from K more steps with an
    # event pair around each call (as for the headline)
    elapsed = time_steps(step, args.steps, 0, world, device)
    trace.enabled = True
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    hdr = N.SmqPackedHeader.from_buffer_copy(bytes(packed[:128].cpu().numpy()))
    sbytes = int(hdr.total_bytes)
    # algorithmic bytes: stats read 4n, pack read 4n + stream write, unpack stream read + 4n write
    alg = 12.0 * n + 2.0 * sbytes
    total = sum_over_ranks(alg * args.steps, world, device)
    c_ms, u_ms = trace.mean_ms("compress"), trace.mean_ms("unpack")
    u_gbps = (sbytes + 4.0 * n) / (u_ms * 1e-3) / 1e9
    return {"metric": "Packed SmaQ 6/8 compress+decompress GB/s, 256M fp32",
            "value": round(total / elapsed / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "host_enqueue_ms_per_step": round(HOST.get("enqueue_ms_per_step", 0.0), 4),
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "smaq_6_8_packed_256M_fp32", "elements_per_gpu": n,
                       "stream_bytes": sbytes, "bits_per_element": round(8.0 * sbytes / n, 3),
                       "compression_ratio_vs_fp32": round(32.0 * n / (8.0 * sbytes), 3),
                       "pack_flags": pack_flags},
            "compress_ms": round(c_ms, 4), "decompress_ms": round(u_ms, 4),
            "roofline": {"bound": "hbm", "kernel": "smaq_unpack_kernel",
                         "achieved": round(u_gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(u_gbps / HBM_PEAK_GBPS, 4),
                         "alg_bytes_per_launch": sbytes + 4 * n, "avg_launch_ms": round(u_ms, 5),
                         "traffic": None}}


def _vgg_cifar():
    import torch.nn as nn

    def stage(cin, cout):
        return [nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(),
                nn.Conv2d(cout, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout), nn.ReLU()]

    layers = stage(3, 64) + [nn.MaxPool2d(2)] + stage(64, 128) + [nn.MaxPool2d(2)] + \
        stage(128, 256) + [nn.MaxPool2d(2)] + stage(256, 512) + \
        [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(512, 10)]
    return nn.Sequential(*layers)


def run_autograd(args, world, rank, device):
    """SURVEY 8f-2 at model scale: a CIFAR-shaped VGG-style CNN (batch 128) trained with SmaQ on
    every selected layer's activation (forward) and grad-map (backward) through the mirrored
    register_autograd_module (autograd.py:50-77). Three variants: no compression, codec calls
    eager, and the whole training step captured in a hipGraph (SmartFP.graph_safe: fresh random
    streams per replay)."""
    from argparse import Namespace

    import torch.nn.functional as F

    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.autograd import register_autograd_module

    batch = 128
    torch.manual_seed(rank)
    x = torch.randn(batch, 3, 32, 32, device=device)
    t = torch.randint(0, 10, (batch,), device=device)
    flags = Namespace(compress_forward=True, compress_backward=True, use_batch_norm=False)
    calls = {"n": 0, "elems": 0}

    def build(compress):
        torch.manual_seed(0)
        net = _vgg_cifar().to(device)
        opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
        codec = None
        if compress:
            codec = SmartFP(smaq_hparams())
            codec.rng.seed = 3000 + rank

            def fn(v, tag=None, **kw):
                calls["n"] += 1
                calls["elems"] += v.numel()
                return codec(v, tag=tag, **kw)

            register_autograd_module(net, fn, flags)
        return net, opt, codec

    def step_fn(net, opt):
        def step():
            opt.zero_grad(set_to_none=False)
            loss = F.cross_entropy(net(x), t)
            loss.backward()
            opt.step()
        return step

    results = {}
    for name in ("uncompressed", "smaq_eager", "smaq_graph"):
        net, opt, codec = build(name != "uncompressed")
        step = step_fn(net, opt)
        if name == "smaq_graph":
            codec.graph_safe(device=device)
            s = torch.cuda.Stream(device)
            s.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(s):
                for _ in range(3):
                    step()
            torch.cuda.current_stream(device).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            run = g.replay
        else:
            run = step
        calls["n"] = calls["elems"] = 0
        run()
        torch.cuda.synchronize()
        per_step = (calls["n"], calls["elems"])
        for _ in range(args.warmup):
            run()
        elapsed = time_steps(run, args.steps, 0, world, device)
        results[name] = {"ms_per_step": round(elapsed / args.steps * 1e3, 4)}
        if name != "uncompressed" and per_step[0]:
            results[name].update(codec_calls_per_step=per_step[0],
                                 compressed_elements_per_step=per_step[1])
    calls_per, elems = results["smaq_eager"]["codec_calls_per_step"], \
        results["smaq_eager"]["compressed_elements_per_step"]
    g_ms = results["smaq_graph"]["ms_per_step"]
    return {"metric": "Training step with SmaQ on every layer (activations + grad-maps), ms/step",
            "value": g_ms, "unit": "ms/step", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": g_ms, "higher_is_better": False,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "vgg_cifar_b128_register_autograd_module",
                       "codec_calls_per_step": calls_per,
                       "compressed_elements_per_step": elems},
            "variants": results}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="smaq",
                    choices=["smaq", "smaq_sampled", "fp8", "s2fp8", "multi", "packed",
                             "autograd"])
    ap.add_argument("--elements", type=int, default=0, help="override elements (smaq configs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1 << 24)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    args = ap.parse_args()

    world, rank, local = dist_setup()
    device = torch.device("cuda", local)
    runner = {"smaq": run_smaq, "smaq_sampled": run_smaq, "fp8": run_fp8, "s2fp8": run_s2fp8,
              "multi": run_multi, "packed": run_packed, "autograd": run_autograd}[args.config]
    res = runner(args, world, rank, device)
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline and args.config.startswith("smaq"):
            res["cpu_baseline"] = cpu_baseline_smaq(args.cpu_sample, args.cpu_budget)
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
