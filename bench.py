"""Benchmark of the SmaQ 6/8-bit compress->decompress round trip on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): one contiguous 268,435,456-element fp32 tensor
(1 GiB, x ~ N(0,1), generated on the device), SmartFP defaults (6/8 bits, thresholds 1.0/2.5,
full statistics, stochastic rounding), through the drop-in SmartFP.__call__ -> libsmq C-ABI.
A "step" = one round trip of that tensor (stats launch + apply launch, output tensor allocated by
the codec like the reference). value = algorithmic bytes (12 B/elem: stats read + apply read +
write) over all ranks / max-over-ranks wall time of the K timed steps.

Multi-GPU (independent units, no data-path collective): one process per GPU, each with
its own tensors and seed ("weak" scaling). `bench.py --gpus N` launches the N rank processes itself
(before any GPU call) when no launcher did; under torchrun (RANK / WORLD_SIZE set) each process is
one rank. Ranks meet in a CPU (gloo) process group that only carries the start/stop barriers and
the reduction of the timings: no RCCL. Rank 0 prints the one JSON line with every rank's time.

Other configs (--config smaq_sampled | fp8 | s2fp8 | multi | packed | autograd | autograd_resnet34 |
smaq_cpu) are measurement
aids (BASELINE configs 1 and 3-5), not the line the driver records; each carries its own
`roofline` and, at N=1, a `cpu_baseline`.

roofline: the call's launches (at 256M the statistics + apply kernels, 12 B/elem algorithmic) timed
with an event pair on the codec's stream around each call (over K steps after the timed ones).
cpu_baseline: the CPU restatement in oracle/ (kind "port"): smart.py's own torch-CPU op sequence
(oracle/smaq_torch.py, 16 intra-op threads) for SmaQ, the numpy qtorch / s2fp8 restatements (one
thread) for FP8 / S2FP8, on a bounded sample.
"""

import argparse
import collections
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
SMALL_MAX_N = 8388611  # smq_smaq_roundtrip: one register-resident launch up to this many elements
METRIC = "SmaQ 6/8-bit quant+dequant round-trip GB/s (and % HBM peak), {size} fp32"


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
    """This process's rank. World > 1: a CPU (gloo) process group over 127.0.0.1 — it carries the
    start/stop barriers and the timing reductions only; the codecs never communicate."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if os.environ.get("SMQ_BENCH_SHARE_DEVICE") == "1":
        local = 0  # rehearsal of the N>1 flow on a 1-GPU box (shared card)
    if world > 1:
        import datetime

        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=300))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(value, world, device=None):
    if world == 1:
        return value
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, world, device=None):
    if world == 1:
        return value
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_over_ranks(value, world):
    """Every rank's value, in rank order (on every rank)."""
    if world == 1:
        return [value]
    import torch.distributed as dist

    t = torch.zeros(world, dtype=torch.float64)
    t[dist.get_rank()] = value
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (RANK,
    LOCAL_RANK = i, WORLD_SIZE = N, rendezvous on 127.0.0.1) and wait for them. This process never
    touches the GPU (the children are started before anything initialises HIP). Rank 0's stdout —
    the one JSON line — goes to a temporary file (never a pipe: a rank writing more than a pipe
    buffer would block on it while the others wait at a barrier) and is relayed after the ranks
    exit; if a rank fails, the others are stopped. Returns the exit code."""
    import subprocess
    import tempfile

    port = str(_free_port())
    procs = []
    out0 = tempfile.TemporaryFile()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True))
    rc = 0
    try:
        pending = set(range(n))
        while pending:
            for r in sorted(pending):
                code = procs[r].poll()
                if code is None:
                    continue
                pending.discard(r)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:  # a rank died: the others would wait at a barrier
                        procs[q].terminate()
            time.sleep(0.05)
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    out0.seek(0)
    out = out0.read().decode(errors="replace")
    out0.close()
    for line in out.splitlines():  # the JSON line to stdout, anything else (gloo chatter) to stderr
        (sys.stdout if line.startswith("{") else sys.stderr).write(line + "\n")
    sys.stdout.flush()
    return rc


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


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


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
    _sync()
    barrier(world)
    _sync()
    t0 = time.perf_counter()
    if region is not None:
        region.begin("region")
    for _ in range(steps):
        step()
    if region is not None:
        region.end("region")
    HOST["enqueue_ms_per_step"] = (time.perf_counter() - t0) / steps * 1e3
    _sync()
    own = time.perf_counter() - t0  # this rank's own work, before it waits for the others
    barrier(world)
    elapsed = time.perf_counter() - t0
    HOST["rank_ms_per_step"] = [round(v / steps * 1e3, 4) for v in gather_over_ranks(own, world)]
    return max_over_ranks(elapsed, world, device)


def _cpu_threads():
    """Intra-op threads of this job's CPU share (OMP_NUM_THREADS, 16 on the GPU box; os.cpu_count()
    counts the whole machine there)."""
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)


def _host_info():
    """What the CPU baseline ran on: the host CPU model, the machine's logical CPUs and its load
    (the baseline moves between boxes with both)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    load = os.getloadavg() if hasattr(os, "getloadavg") else None
    return {"cpu_model": model, "machine_cpus": os.cpu_count(),
            "loadavg_1m": None if load is None else round(load[0], 2)}


def _spread(per_rep_bytes, ts):
    """min / median / max of the per-repetition rate (GB/s) over the timed repetitions."""
    r = sorted(per_rep_bytes / t / 1e9 for t in ts)
    return {"min": round(r[0], 4), "median": round(float(np.median(r)), 4), "max": round(r[-1], 4),
            "reps": len(r)}


def _time_reps(fn, budget_s, min_reps=2):
    fn()  # warm-up (allocator, thread pool)
    reps, t_tot, ts = 0, 0.0, []
    while t_tot < budget_s or reps < min_reps:
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        ts.append(dt)
        t_tot += dt
        reps += 1
    return reps, t_tot, ts


def cpu_baseline_smaq(args, sampled=False):
    """The reference's algorithm on the host cores: oracle/smaq_torch.py, smart.py's own torch-CPU
    op sequence (full stats — or randperm-sampled ones —, torch.rand_like SR; bit-exact with the
    reference's outputs on the golden fixtures), on a bounded sample of the workload, plus the
    reference's own CPU config C1 (1M elements, median of >= 30 calls) for BASELINE.md."""
    from oracle import smaq_torch

    threads = _cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    ns = 16 if sampled else 0
    try:
        x = torch.randn(args.cpu_sample, generator=torch.Generator().manual_seed(0))
        reps, t_tot, ts = _time_reps(lambda: smaq_torch.roundtrip(x, num_samples=ns),
                                     args.cpu_budget)
        torch.manual_seed(0)
        x1 = torch.randn(1 << 20)
        _, _, t1 = _time_reps(lambda: smaq_torch.roundtrip(x1, num_samples=ns), 0.0, min_reps=30)
    finally:
        torch.set_num_threads(prev)
    per = 8.0 if sampled else 12.0
    gbps = per * args.cpu_sample * reps / t_tot / 1e9
    c1_ms = float(np.median(t1)) * 1e3
    return {"value": round(gbps, 4), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x {args.cpu_sample} fp32 N(0,1) round trips, oracle/smaq_torch.py "
                      f"(smart.py's torch-CPU op sequence, {'sampled(16)' if sampled else 'full'} "
                      f"stats + rand_like SR), {threads} threads, {t_tot:.1f} s",
            "spread_gbps": _spread(per * args.cpu_sample, ts),
            "c1_1M": {"ms_median": round(c1_ms, 3), "ms_min": round(min(t1) * 1e3, 3),
                      "ms_max": round(max(t1) * 1e3, 3),
                      "gbps": round(per * (1 << 20) / (c1_ms * 1e-3) / 1e9, 4), "reps": len(t1)}}


def cpu_baseline_float(args, codec):
    """FP8 / S2FP8 on the host: the numpy restatements (oracle/qtorch_float.py with check_inf,
    oracle/s2fp8.py) — the reference's CPU path would be qtorch's single-thread C++ loop, absent
    here — one thread, on a bounded sample."""
    from oracle import qtorch_float as qf
    from oracle import rng as orng
    from oracle import s2fp8 as os2

    n = min(args.cpu_sample, 1 << 22)
    x = np.random.default_rng(0).standard_normal(n).astype(np.float32)
    if codec == "fp8":
        x = np.maximum(x, 0)
        r = orng.rng_u32(7, 0, n)
        fn, per = (lambda: qf.float_quantize(x, 5, 2, r, True)), 8.0
    else:
        r = orng.rng_u32(7, 0, n)
        fn, per = (lambda: os2.roundtrip(x, r, True)), 12.0
    reps, t_tot, _ = _time_reps(fn, args.cpu_budget)
    return {"value": round(per * n * reps / t_tot / 1e9, 4), "unit": "GB/s", "cores": 1,
            "kind": "port",
            "sample": f"{reps} x {n} fp32 elements, numpy restatement "
                      f"({'oracle/qtorch_float.py E5M2 SR + check_inf' if codec == 'fp8' else 'oracle/s2fp8.py'}),"
                      f" 1 thread, {t_tot:.1f} s"}


def cpu_baseline_multi(args):
    """C5 on the host: the reference's per-tensor calls (optimizer.py:79-127 -> smart.py) as
    oracle/smaq_torch.py over the same 148 ResNet-34 tensors, all host threads."""
    from oracle import smaq_torch

    threads = _cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        g = torch.Generator().manual_seed(0)
        ts = [torch.randn(s, generator=g) * 1e-3 for s in resnet34_c5_shapes()]
        n = sum(t.numel() for t in ts)

        def step():
            for t in ts:
                if t.numel() >= 8:
                    smaq_torch.roundtrip(t)

        reps, t_tot, _ = _time_reps(step, args.cpu_budget)
    finally:
        torch.set_num_threads(prev)
    return {"value": round(12.0 * n * reps / t_tot / 1e9, 4), "unit": "GB/s", "cores": threads,
            "kind": "port",
            "sample": f"{reps} steps x 148 tensors ({n} elements), oracle/smaq_torch.py per tensor "
                      f"(the reference's per-parameter SmartFP calls), {threads} threads, "
                      f"{t_tot:.1f} s"}


def cpu_baseline_packed(args):
    """Packed container on the host: the numpy restatement (oracle/smaq_packed.py: full statistics,
    counter-RNG codes, block images, then the decoder), one thread, on a bounded sample; the same
    algorithmic bytes as the GPU line (12 B/elem + the stream written and read)."""
    from oracle import rng as orng
    from oracle import smaq as osmaq
    from oracle import smaq_packed as opk

    n = min(args.cpu_sample, 1 << 20)
    x = np.random.default_rng(0).standard_normal(n).astype(np.float32)
    cfg = osmaq.SmaqConfig()
    u = orng.uniforms(7, 0, n)
    box = {}

    def step():
        mean, std = osmaq.full_stats(x, cfg)
        box["s"] = opk.pack(x, mean, std, cfg, u)
        opk.unpack(box["s"])

    reps, t_tot, _ = _time_reps(step, args.cpu_budget)
    alg = 12.0 * n + 2.0 * box["s"].size
    return {"value": round(alg * reps / t_tot / 1e9, 4), "unit": "GB/s", "cores": 1,
            "kind": "port",
            "sample": f"{reps} x {n} fp32 N(0,1) compress + decompress, numpy restatement "
                      f"(oracle/smaq_packed.py), 1 thread, {t_tot:.1f} s"}


CPU_BASELINES = {
    "packed": lambda a: cpu_baseline_packed(a),
    "smaq": lambda a: cpu_baseline_smaq(a),
    "smaq_cpu": lambda a: cpu_baseline_smaq(a),
    "smaq_sampled": lambda a: cpu_baseline_smaq(a, sampled=True),
    "fp8": lambda a: cpu_baseline_float(a, "fp8"),
    "s2fp8": lambda a: cpu_baseline_float(a, "s2fp8"),
    "multi": lambda a: cpu_baseline_multi(a),
}


def traffic_from_profile(config, elements, dtype="f32", whole_call=False, profile=None):
    """HBM bytes per launch from the committed PMC passes (profiles/traffic_<profile>.json): the
    dominant kernel's, or (whole_call) the sum over the call's kernels. Reported only when the
    profiled run was this workload (same config, element count and input dtype); otherwise None —
    counter bytes of another size say nothing about this run."""
    path = os.path.join(REPO, "profiles", f"traffic_{profile or config}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    if (d.get("config"), d.get("elements"), d.get("dtype", "f32")) != (config, int(elements), dtype):
        return None
    if whole_call:
        return float(sum(d.get("kernels", {}).values())) or None
    return d.get("apply_bytes_per_launch")


def size_label(n):
    """'256M' for whole multiples of 2^20 elements, else the exact count."""
    return f"{n >> 20}M" if n % (1 << 20) == 0 else str(n)


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
    # SMQ_BENCH_DIST=laplace: C2's heavy-tailed variant, Laplace(0, 1) as the
    # difference of two Exp(1) draws
    dist = os.environ.get("SMQ_BENCH_DIST", "normal")
    if dist == "laplace":
        xs = []
        for _ in range(2):
            x = -torch.log1p(-torch.rand(n, generator=gen, device=device))
            xs.append(x.sub_(-torch.log1p(-torch.rand(n, generator=gen, device=device))))
    else:
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
    # the K timed steps carry no event markers; the call's device time for `roofline` is then
    # measured with an event pair around each call (the product entry point smq_smaq_roundtrip: its
    # statistics and apply launches) over K more steps of the same workload, on the codec's stream
    # (SMQ_BENCH_EVENTS_IN_TIMED=1: events inside the timed steps instead)
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
    call_ms = trace.mean_ms("call")
    # the launches of one call: one register-resident launch up to 8,388,611 elements (full
    # statistics: x read once, y written = in_bytes + 4 per element), else the statistics launch +
    # the apply launch (include/smq.h). `value` keeps the metric's convention (alg_per_elem);
    # the roofline divides the bytes the call's launches must move.
    moved_per_elem = alg_per_elem
    if sampled:
        kernels = "smaq_draw_stats_kernel+smaq_apply_kernel"
    elif n <= SMALL_MAX_N:
        kernels = "smaq_fused_kernel"
        moved_per_elem = in_bytes + 4
    else:
        kernels = "smaq_stats_kernel+smaq_apply_kernel"
    call_gbps = moved_per_elem * n / (call_ms * 1e-3) / 1e9
    res = {
        "metric": METRIC.format(size=size_label(n)), "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "fp32" if in_dt is None else f"{os.environ['SMQ_BENCH_DTYPE']} in, fp32 out",
        "data": "synthetic",
        "config": {"workload": f"smaq_6_8_roundtrip_{size_label(n)}_fp32" if not sampled else
                   f"smaq_6_8_roundtrip_sampled_stats_{size_label(n)}", "elements_per_gpu": n,
                   "stats": "sampled(16)" if sampled else "full", "rounding": "stochastic",
                   "bits": "6/8", "alg_bytes_per_elem": alg_per_elem,
                   "parallelism": f"replicas{world}",
                   **({"dist": dist} if dist != "normal" else {})},
        "pct_hbm_peak": round(100.0 * value / world / HBM_PEAK_GBPS, 2),
        # the same time read as tensor GB/s (in_bytes * n per step) and as HBM-read
        # GB/s (statistics read + apply read: the north star's "HBM-read roofline" reading)
        "tensor_gbps": round(value * in_bytes / alg_per_elem, 2),
        "read_gbps": round(value * (alg_per_elem - 4) / alg_per_elem, 2),
        # the whole call (all of its launches) over its algorithmic bytes; traffic = the sum of
        # the call's kernels' PMC bytes (profiles/traffic_<config>.json)
        "roofline": {"bound": "hbm", "kernel": kernels,
                     "achieved": round(call_gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(call_gbps / HBM_PEAK_GBPS, 4),
                     "alg_bytes_per_launch": int(moved_per_elem * n),
                     "avg_launch_ms": round(call_ms, 5),
                     "traffic": traffic_from_profile(
                         args.config, n, "f32" if in_dt is None else os.environ["SMQ_BENCH_DTYPE"],
                         whole_call=True,
                         profile=args.config if in_dt is None
                         else f"{args.config}_{os.environ['SMQ_BENCH_DTYPE']}")},
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
                         "avg_launch_ms": round(k_ms, 5), "traffic": traffic_from_profile("fp8", n)}}


def run_s2fp8(args, world, rank, device):
    """Config 4: S2FP8 on [32,128,768], rotating 48 buffers (> MALL). Two variants of the same
    calls: eager S2FP8.__call__ (the reference's usage; `value`), and the 48 calls of one rotation
    captured in a hipGraph and replayed (graph_safe random stream), which removes the host path
    and shows the device time per call."""
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

    trace = EventTrace()
    prewarm(step, device)
    elapsed = time_steps(step, args.steps, args.warmup, world, device, region=trace)
    enqueue = HOST.get("enqueue_ms_per_step", 0.0)
    eager_dev_ms = trace.mean_ms("region") / args.steps
    # hipGraph variant: one graph = one rotation of nbuf calls
    codec.graph_safe(True, device=device)
    try:
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            for x in xs:
                codec(x)
        torch.cuda.current_stream(device).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for x in xs:
                codec(x)
        reps = max(1, -(-args.steps // nbuf))
        gtrace = EventTrace()
        g_elapsed = time_steps(g.replay, reps, max(1, args.warmup // nbuf), world, device,
                               region=gtrace)
        g_ms = g_elapsed / (reps * nbuf) * 1e3
        g_dev_ms = gtrace.mean_ms("region") / (reps * nbuf)
    finally:
        codec.graph_safe(False)
    total = sum_over_ranks(12.0 * n * args.steps, world, device)
    # S2FP8 algorithmic bytes are 12 B/elem (log2 statistics read + read + write) over
    # all launches of the call; the single launch (s2fp8_fused_kernel) moves 8 of them (x is read
    # once into registers), so HBM traffic / alg bytes = 0.68
    gbps = 12.0 * n / (g_dev_ms * 1e-3) / 1e9
    # in-MALL variant ("in-MALL vs rotated"): one input buffer, eager calls
    xs1 = xs[:1]
    it1 = [0]

    def step1():
        codec(xs1[0])
        it1[0] += 1

    t1 = time_steps(step1, args.steps, args.warmup, world, device)
    return {"metric": "S2FP8 round-trip GB/s, [32,128,768] fp32", "value": round(total / elapsed / 1e9, 2),
            "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "host_enqueue_ms_per_step": round(enqueue, 4),
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "s2fp8_roundtrip_bert_hidden", "shape": list(shape),
                       "rotating_buffers": nbuf, "alg_bytes_per_elem": 12,
                       "parallelism": f"replicas{world}"},
            "variants": {"eager": {"ms_per_step": round(elapsed / args.steps * 1e3, 4),
                                   "device_ms_per_step": round(eager_dev_ms, 5)},
                         "graph": {"ms_per_step": round(g_ms, 5),
                                   "device_ms_per_step": round(g_dev_ms, 5)},
                         "in_mall_1buf": {"ms_per_step": round(t1 / args.steps * 1e3, 5)}},
            # one call = one launch, timed over graph replays (no host gaps)
            "roofline": {"bound": "hbm", "kernel": "s2fp8_fused_kernel",
                         "achieved": round(gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(gbps / HBM_PEAK_GBPS, 4), "alg_bytes_per_launch": int(12 * n),
                         "avg_launch_ms": round(g_dev_ms, 5), "traffic": traffic_from_profile("s2fp8", n, whole_call=True)}}


def resnet34_cifar_params():
    """(shape, in the BN group) of every parameter of the reference's CIFAR ResNet-34, in module
    order (models/pytorch/resnet.py:133-260: 3x3 stem, BasicBlock layers [3, 4, 6, 3] with 1x1
    downsample shortcuts, fc 512 -> 10): 110 tensors, 21,282,122 elements."""
    out = [((64, 3, 3, 3), False), ((64,), True), ((64,), True)]
    cin = 64
    for planes, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(blocks):
            s = stride if b == 0 else 1
            out += [((planes, cin, 3, 3), False), ((planes,), True), ((planes,), True),
                    ((planes, planes, 3, 3), False), ((planes,), True), ((planes,), True)]
            if b == 0 and (s != 1 or cin != planes):
                out += [((planes, cin, 1, 1), False), ((planes,), True), ((planes,), True)]
            cin = planes
    out += [((10, 512), False), ((10,), False)]
    return out


def resnet34_c5_shapes():
    """BASELINE config 5, one optimizer step's SmaQ tensors: the 110 gradients (every parameter)
    then the 38 weights of the non-BN group (models/base.py:139-150 puts BatchNorm2d parameters in
    a no_weight_compression group; the fc bias stays): 148 tensors, 42,547,220 elements."""
    ps = resnet34_cifar_params()
    return [s for s, _ in ps] + [s for s, bn in ps if not bn]


def resnet34_c5_tensors(device, seed):
    """C5 values: gradients ~ N(0, 1e-3); conv weights Kaiming-normal fan_out (resnet.py:186-188),
    fc weight / bias U(-1/sqrt(512), 1/sqrt(512)) (nn.Linear's default)."""
    gen = torch.Generator(device=device).manual_seed(seed)
    ps = resnet34_cifar_params()
    grads = [torch.randn(s, generator=gen, device=device) * 1e-3 for s, _ in ps]
    weights = []
    for s, bn in ps:
        if bn:
            continue
        if len(s) == 4:
            std = (2.0 / (s[0] * s[2] * s[3])) ** 0.5
            weights.append(torch.randn(s, generator=gen, device=device) * std)
        else:
            b = 1.0 / 512 ** 0.5
            weights.append((torch.rand(s, generator=gen, device=device) * 2 - 1) * b)
    return grads + weights


def run_multi(args, world, rank, device):
    """Config 5: fused multi-tensor SmaQ over ResNet-34 (CIFAR) grads (110) + non-BN weights (38),
    one bound SmaqMulti call (two launches) per step."""
    from smart_compress_amd.util.pytorch.multi import SmaqMulti

    tensors = resnet34_c5_tensors(device, rank)
    n = sum(t.numel() for t in tensors)
    outs = [torch.empty_like(t) for t in tensors]
    m = SmaqMulti(smaq_hparams(), seed=rank)
    bound = m.bind(tensors, outs)  # fixed buffers: validated once, one call = two launches
    trace = EventTrace()

    def step():
        bound()

    prewarm(step, device)
    elapsed = time_steps(step, args.steps, args.warmup, world, device, region=trace)
    total = sum_over_ranks(12.0 * n * args.steps, world, device)
    k_ms = trace.mean_ms("region") / args.steps
    gbps = 12.0 * n / (k_ms * 1e-3) / 1e9
    return {"metric": "Fused multi-tensor SmaQ GB/s, ResNet-34 weights+grads per step",
            "value": round(total / elapsed / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "host_enqueue_ms_per_step": round(HOST.get("enqueue_ms_per_step", 0.0), 4),
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "smaq_multi_resnet34_weights_grads", "tensors": len(tensors),
                       "elements_per_gpu": n, "alg_bytes_per_elem": 12,
                       "parallelism": f"replicas{world}"},
            # one call = the statistics + apply launches: timed together by events at the two ends
            # of the timed region (the per-kernel split is in profiles/*_multi_summary.json)
            "roofline": {"bound": "hbm", "kernel": "smaq_multi_stats_kernel+smaq_multi_apply_kernel",
                         "achieved": round(gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(gbps / HBM_PEAK_GBPS, 4), "alg_bytes_per_launch": int(12 * n),
                         "avg_launch_ms": round(k_ms, 5), "traffic": traffic_from_profile("multi", n, whole_call=True)}}


def run_packed(args, world, rank, device):
    """Packed SmaQ container on the 256M config: compress (statistics + packing
    launch) then decompress, both through the C-ABI into preallocated buffers (no host sync)."""
    from smart_compress_amd import _native as N
    from smart_compress_amd.compress.packed import SmartFPPacked

    n = args.elements or (1 << 28)
    # measurement knob SMQ_BENCH_SR=0: truncation instead of stochastic rounding
    hp = smaq_hparams(stochastic_rounding=os.environ.get("SMQ_BENCH_SR", "1") != "0")
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
    # SMQ_BENCH_PACK_FLAGS: smq_smaq_compress_ex flags (legacy, no effect since format version 2)
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
        N.check(lib.smq_smaq_decompress_ex(packed.data_ptr(), y.data_ptr(), n, hp.num_bits_main,
                                           hp.num_bits_outlier, st), "decompress")
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
    # compress: statistics read (4n) + the packer's read of x (4n) + the stream written; decompress:
    # the stream read + 4n written
    c_alg = 8.0 * n + sbytes
    c_gbps = c_alg / (c_ms * 1e-3) / 1e9
    u_gbps = (sbytes + 4.0 * n) / (u_ms * 1e-3) / 1e9
    traffic = None
    tp = os.path.join(REPO, "profiles", "traffic_packed.json")
    if os.path.exists(tp):
        with open(tp) as f:
            d = json.load(f)
        if (d.get("config"), d.get("elements")) == ("packed", n):
            ks = d.get("kernels", {})
            unpack = ("smaq_unpack_kernel", "smaq_unpack_big_kernel")
            comp = [v for k, v in ks.items() if k not in unpack and v]
            dec = [ks[k] for k in unpack if ks.get(k)]
            traffic = {"compress": float(sum(comp)) if comp else None,
                       "decompress": float(sum(dec)) if dec else None}
    return {"metric": f"Packed SmaQ 6/8 compress+decompress GB/s, {size_label(n)} fp32",
            "value": round(total / elapsed / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "host_enqueue_ms_per_step": round(HOST.get("enqueue_ms_per_step", 0.0), 4),
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": f"smaq_6_8_packed_{size_label(n)}_fp32", "elements_per_gpu": n,
                       "stream_bytes": sbytes, "bits_per_element": round(8.0 * sbytes / n, 3),
                       "compression_ratio_vs_fp32": round(32.0 * n / (8.0 * sbytes), 3),
                       "format_version": int(hdr.version), "pack_flags": pack_flags},
            "compress_ms": round(c_ms, 4), "decompress_ms": round(u_ms, 4),
            # compress (all its launches: statistics, block codes, scan, variable sections) over
            # its algorithmic bytes; traffic = the sum of those kernels' PMC bytes per call
            "roofline": {"bound": "hbm",
                         "kernel": "smaq_stats_kernel+smaq_pack_block_kernel+smaq_pack_scan_kernel"
                                   "+smaq_pack_var_kernel",
                         "achieved": round(c_gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(c_gbps / HBM_PEAK_GBPS, 4), "alg_bytes_per_launch": int(c_alg),
                         "avg_launch_ms": round(c_ms, 5),
                         "traffic": None if traffic is None else traffic["compress"]},
            # decompress: both launches (blocks whose variable section is in LDS, then the rare
            # others), timed by one event pair around the call
            "roofline_decompress": {"bound": "hbm",
                                    "kernel": "smaq_unpack_kernel+smaq_unpack_big_kernel",
                                    "achieved": round(u_gbps, 1), "peak": HBM_PEAK_GBPS,
                                    "unit": "GB/s", "frac": round(u_gbps / HBM_PEAK_GBPS, 4),
                                    "alg_bytes_per_launch": int(sbytes + 4 * n),
                                    "avg_launch_ms": round(u_ms, 5),
                                    "traffic": None if traffic is None else traffic["decompress"]}}


def _vgg_cifar():
    import torch.nn as nn

    def stage(cin, cout):
        return [nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(),
                nn.Conv2d(cout, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout), nn.ReLU()]

    layers = stage(3, 64) + [nn.MaxPool2d(2)] + stage(64, 128) + [nn.MaxPool2d(2)] + \
        stage(128, 256) + [nn.MaxPool2d(2)] + stage(256, 512) + \
        [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(512, 10)]
    return nn.Sequential(*layers)


class _BasicBlock(torch.nn.Module):
    """The reference's CIFAR ResNet BasicBlock (models/pytorch/resnet.py:31-79), written here (the
    reference's model zoo is not imported): conv3x3-BN-ReLU(inplace)-conv3x3-BN, identity or the
    1x1-conv + BN downsample, in-place add, ReLU."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        nn = torch.nn
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out += identity
        return self.relu(out)


class _ResNet(torch.nn.Module):
    """The reference's CIFAR ResNet (models/pytorch/resnet.py:133-260): 3x3 stride-1 stem, BN,
    ReLU, 3x3 / 2 max-pool, four BasicBlock layers, average pool, fc; Kaiming fan-out init."""

    def __init__(self, layers=(3, 4, 6, 3), num_classes=10):
        super().__init__()
        nn = torch.nn
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], 2)
        self.layer3 = self._make_layer(256, layers[2], 2)
        self.layer4 = self._make_layer(512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def _make_layer(self, planes, blocks, stride=1):
        nn = torch.nn
        down = None
        if stride != 1 or self.inplanes != planes:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride, bias=False),
                                 nn.BatchNorm2d(planes))
        layers = [_BasicBlock(self.inplanes, planes, stride, down)]
        self.inplanes = planes
        layers += [_BasicBlock(planes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = self.avgpool(x)
        return self.fc(x.reshape(x.size(0), -1))


# quantization.py:164-180 always wraps the classes of the reference's model zoo (module path
# smart_compress.models.pytorch.*): BasicBlock and the whole ResNet get their outputs compressed
# too (132 module outputs per forward). These stand-ins carry that module path so the
# mirrored is_valid_layer_type selects exactly the reference's call set.
_BasicBlock.__module__ = _ResNet.__module__ = "smart_compress.models.pytorch.resnet"


def run_autograd(args, world, rank, device):
    """SURVEY 8f-2 at model scale: a CIFAR network at batch 128 trained with SmaQ on every selected
    module's activation (forward) and grad-map (backward) through the mirrored
    register_autograd_module (autograd.py:50-77). --config autograd_resnet34: the reference's
    CIFAR ResNet-34 (models/pytorch/resnet.py:133-303, SURVEY 3B: the reference's own model);
    --config autograd: a VGG-style CNN. Three variants: no compression, codec calls eager, and the
    whole training step captured in a hipGraph (SmartFP.graph_safe: fresh random streams per
    replay). The codec's share of a step = compressed - uncompressed, reported with its
    algorithmic bytes (12 B per compressed element)."""
    from argparse import Namespace

    import torch.nn.functional as F

    from smart_compress_amd.compress.packed import SmartFPPacked
    from smart_compress_amd.compress.smart import SmartFP
    from smart_compress_amd.util.pytorch.autograd import register_autograd_module
    from smart_compress_amd.util.pytorch.saved import PackedActivations

    batch = 128
    resnet = args.config == "autograd_resnet34"
    torch.manual_seed(rank)
    x = torch.randn(batch, 3, 32, 32, device=device)
    t = torch.randint(0, 10, (batch,), device=device)
    flags = Namespace(compress_forward=True, compress_backward=True, use_batch_norm=False)

    def build(compress, sizes=None, packed=False, ratio=False):
        """The network; with compression the SmartFP codec itself is registered (train.py:198-213
        passes the codec instance), so Compressor takes the codec's C autograd path. sizes: a list
        that records the element count of every codec call instead (one counting step). packed:
        the activations autograd saves are held as SmaQ streams (util/pytorch/saved.py). ratio:
        --measure_compression_ratio, as every reference training script runs (scripts/train.ps1),
        logging into a bounded in-memory sink (the logger's own cost is not the codec's)."""
        torch.manual_seed(0)
        net = (_ResNet() if resnet else _vgg_cifar()).to(device)
        opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
        codec = None
        if compress:
            codec = (SmartFPPacked if packed else SmartFP)(
                smaq_hparams(measure_compression_ratio=ratio))
            codec.rng.seed = 3000 + rank
            if ratio:
                sink = collections.deque(maxlen=1 << 14)
                codec.log = lambda k, v, _s=sink, **kw: _s.append((k, v))
            fn = codec
            if packed:
                fn = PackedActivations(codec, verify_bytes=(args.saved_budget << 20
                                                            if args.saved_budget else None))
                if args.saved_exit >= 0:  # (measurement option: the exit's wait, MiB)
                    fn.exit_bytes = args.saved_exit << 20
                fn.replay_inplace = not args.saved_no_replay  # (measurement option)
            if sizes is not None:
                def fn(v, tag=None, **kw):
                    sizes.append(v.numel())
                    return codec(v, tag=tag, **kw)
            register_autograd_module(net, fn, flags)
            if packed:
                codec = fn
        return net, opt, codec

    def step_fn(net, opt, acts=None):
        def step():
            opt.zero_grad(set_to_none=False)
            if acts is None:
                loss = F.cross_entropy(net(x), t)
            else:
                with acts:  # saved activations held as streams
                    loss = F.cross_entropy(net(x), t)
            loss.backward()
            opt.step()
        return step

    # the codec calls of one step and their sizes (a separate, counting network)
    sizes = []
    net, opt, _ = build(True, sizes)
    step_fn(net, opt)()
    torch.cuda.synchronize()
    calls_per, elems = len(sizes), sum(sizes)
    # bytes the calls must move: 8 B/elem for the single launch (x read once, y written), 12 B/elem
    # for the two-launch calls above SMALL_MAX_N (statistics read + apply read and write)
    alg_bytes = sum(8 * n if n <= SMALL_MAX_N else 12 * n for n in sizes)
    del net, opt

    results = {}
    # (the graph variant last: its capture keeps a private memory pool alive, which would count in
    # the following variants' allocated memory)
    variants = ["uncompressed", "smaq_eager", "smaq_eager_ratio", "smaq_eager_packed_saved",
                "smaq_graph"]
    if args.variants:  # a subset (profiling passes), always with the uncompressed baseline
        keep = set(args.variants.split(",")) | {"uncompressed"}
        variants = [v for v in variants if v in keep]
    for name in variants:
        packed = name == "smaq_eager_packed_saved"
        net, opt, codec = build(name != "uncompressed", packed=packed,
                                ratio=name == "smaq_eager_ratio")
        step = step_fn(net, opt, codec if packed else None)
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
        run()
        torch.cuda.synchronize()
        mem = None
        if name != "smaq_graph":  # peak allocated over one step, and its excess over the memory
            # resident before the step (parameters, gradients, optimizer state, workspaces); a
            # graph's memory is its private pool, allocated at capture
            before = torch.cuda.memory_allocated(device)
            torch.cuda.reset_peak_memory_stats(device)
            run()
            torch.cuda.synchronize()
            peak = torch.cuda.max_memory_allocated(device)
            mem = {"peak_allocated_mib": round(peak / 2**20, 1),
                   "step_peak_above_resident_mib": round((peak - before) / 2**20, 1)}
        for _ in range(args.warmup):
            run()
        elapsed = time_steps(run, args.steps, 0, world, device)
        results[name] = {"ms_per_step": round(elapsed / args.steps * 1e3, 4)}
        if mem:
            results[name]["memory"] = mem
        if name != "uncompressed":
            results[name].update(codec_calls_per_step=calls_per,
                                 compressed_elements_per_step=elems)
        if packed:
            codec.verify()  # (the last step's sizes: nothing waits for them at the context's exit)
            st = codec.stats()
            results[name]["saved_streams"] = {
                "saved_tensors_packed_per_step": round(st["saved_packed"] / (args.steps + args.warmup + 2), 1),
                "bits_per_element": round(st["bits_per_element"], 3) if st["bits_per_element"] else None}
        del net, opt, codec, run
    base_ms = results["uncompressed"]["ms_per_step"]
    for name in variants[1:]:
        codec_ms = results[name]["ms_per_step"] - base_ms
        results[name]["codec_ms_per_step"] = round(codec_ms, 4)
        results[name]["codec_gbps_12B"] = round(12.0 * elems / (codec_ms * 1e-3) / 1e9, 1) \
            if codec_ms > 0 else None
        results[name]["codec_gbps_alg"] = round(alg_bytes / (codec_ms * 1e-3) / 1e9, 1) \
            if codec_ms > 0 else None
    if "smaq_eager_ratio" in results and "smaq_eager" in results:
        results["smaq_eager_ratio"]["vs_smaq_eager"] = round(
            results["smaq_eager_ratio"]["ms_per_step"] / results["smaq_eager"]["ms_per_step"], 4)
    tpk = os.path.join(REPO, "profiles", f"traffic_{args.config}_packed.json")
    if "smaq_eager_packed_saved" in results and os.path.exists(tpk):
        # HBM bytes per step of the packed-saved variant's codec launches (PMC passes,
        # tools/saved_traffic.py)
        with open(tpk) as f:
            results["smaq_eager_packed_saved"]["traffic"] = json.load(f)["hbm_bytes_per_step"]
    if "smaq_eager_packed_saved" in results and "smaq_eager" in results:
        results["smaq_eager_packed_saved"]["vs_smaq_eager"] = round(
            results["smaq_eager_packed_saved"]["ms_per_step"] / results["smaq_eager"]["ms_per_step"],
            4)
    head = "smaq_graph" if "smaq_graph" in results else variants[-1]
    g_ms = results[head]["ms_per_step"]
    g_codec = results[head]["codec_ms_per_step"]
    g_gbps = results[head]["codec_gbps_alg"]
    # HBM bytes of the step's SmaQ launches from the committed PMC passes
    # (tools/autograd_profile.py -> profiles/traffic_<config>.json)
    traffic = None
    tp = os.path.join(REPO, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tp):
        with open(tp) as f:
            tj = json.load(f)
        if tj.get("calls_per_step") == calls_per and tj.get("elements_per_step") == elems:
            traffic = tj["hbm_bytes_per_step"]
    return {"metric": "Training step with SmaQ on every layer (activations + grad-maps), ms/step",
            "value": g_ms, "unit": "ms/step", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": g_ms, "higher_is_better": False,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": ("resnet34" if resnet else "vgg") +
                       "_cifar_b128_register_autograd_module",
                       "codec_calls_per_step": calls_per,
                       "compressed_elements_per_step": elems,
                       "alg_bytes_per_step": alg_bytes},
            "variants": results,
            # the codec's share of the graph step (compressed - uncompressed) over the bytes its
            # calls must move (8 B/elem single launch, 12 B/elem above): every call as one number
            "roofline": {"bound": "hbm", "kernel": "all SmaQ launches of the step",
                         "variant": head,
                         "achieved": g_gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(g_gbps / HBM_PEAK_GBPS, 4) if g_gbps else None,
                         "alg_bytes_per_launch": int(alg_bytes), "avg_launch_ms": g_codec,
                         "traffic": traffic}}


def run_smaq_cpu(args, world, rank, device):
    """BASELINE config 1 on the library's own CPU path: SmartFP.__call__ on a 1,048,576-element fp32
    CPU tensor (defaults: 6/8 bits, full statistics, stochastic rounding) -> smq_cpu_smaq_roundtrip,
    median of >= 30 calls after warm-up, on this job's CPU share (torch intra-op threads). Also a
    16M-element tensor for throughput. The reference on the container's 8 cores: 6.56 ms = 1.92 GB/s
    at 1M; its torch op sequence is timed in the same run as cpu_baseline."""
    from smart_compress_amd.compress.smart import SmartFP

    threads = _cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        codec = SmartFP(smaq_hparams())
        torch.manual_seed(0)
        x1 = torch.randn(1 << 20)
        _, _, t1 = _time_reps(lambda: codec(x1), 0.0, min_reps=max(30, args.steps))
        n16 = args.elements or (1 << 24)
        x16 = torch.randn(n16, generator=torch.Generator().manual_seed(1))
        reps, t_tot, _ = _time_reps(lambda: codec(x16), min(args.cpu_budget, 5.0))
    finally:
        torch.set_num_threads(prev)
    ms = float(np.median(t1)) * 1e3
    gbps = 12.0 * (1 << 20) / (ms * 1e-3) / 1e9
    return {"metric": "SmaQ 6/8-bit quant+dequant round-trip GB/s on CPU, 1M fp32 (BASELINE config 1)",
            "value": round(gbps, 3), "unit": "GB/s", "n_gpus": 0, "steps": len(t1), "warmup": 1,
            "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "none",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "smaq_6_8_roundtrip_1M_fp32_cpu", "elements": 1 << 20,
                       "threads": threads, "path": "smq_cpu_smaq_roundtrip (libsmq host code)"},
            "vs_reference_in_container": {"reference_ms": 6.56, "reference_threads": 8,
                                          "speedup": round(6.56 / ms, 2)},
            "large": {"elements": n16, "gbps": round(12.0 * n16 * reps / t_tot / 1e9, 3),
                      "reps": reps}}


def run_mock(args, world, rank, device):
    """Device-free step (CPU tests of the N-rank launcher, tests/test_dist_gloo.py): a fixed amount
    of numpy work per step on each rank's own seeded data; reports what each rank saw."""
    if os.environ.get("SMQ_BENCH_MOCK_FAIL_RANK") == str(rank):
        raise RuntimeError(f"rank {rank}: injected failure (SMQ_BENCH_MOCK_FAIL_RANK)")
    chatter = int(os.environ.get("SMQ_BENCH_MOCK_CHATTER", "0"))  # bytes of non-JSON stdout
    if chatter:
        sys.stdout.write(("x" * 1023 + "\n") * (chatter // 1024))
        sys.stdout.flush()
    rng = np.random.default_rng(1000 + rank)
    a = rng.standard_normal(1 << 16).astype(np.float32)

    def step():
        np.sort(a)

    elapsed = time_steps(step, args.steps, args.warmup, world, device)
    seeds = gather_over_ranks(1000 + rank, world)
    pids = gather_over_ranks(os.getpid(), world)
    ranks = gather_over_ranks(rank, world)
    return {"metric": "mock", "value": round(world * args.steps / elapsed, 2), "unit": "steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "mock"}, "ranks": [int(r) for r in ranks],
            "seeds": [int(v) for v in seeds], "pids": [int(v) for v in pids],
            "rank_ms_per_step": HOST.get("rank_ms_per_step")}


def run_mock_multi(args, world, rank, device):
    """Device-free stand-in of run_multi for the launcher tests: 148 numpy tensors per rank (its own
    seed) summed per step; the same line keys."""
    rng = np.random.default_rng(2000 + rank)
    ts = [rng.standard_normal(1 << 10).astype(np.float32) for _ in range(148)]
    n = sum(t.size for t in ts)

    def step():
        for t in ts:
            t.sum()

    elapsed = time_steps(step, args.steps, args.warmup, world, device)
    total = sum_over_ranks(12.0 * n * args.steps, world, device)
    return {"metric": "mock multi", "value": round(total / elapsed / 1e9, 6), "unit": "GB/s",
            "n_gpus": world, "steps": args.steps, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "scaling": "weak", "config": {"workload": "mock_multi", "tensors": len(ts),
                                          "elements_per_gpu": n, "parallelism": f"replicas{world}"},
            "roofline": None}


# BASELINE config 5 is the one the weak-scaling curve is quoted on (fused multi-tensor SmaQ over
# every ResNet-34 weight + grad tensor, each rank its own tensors): the headline config's N-rank job
# measures it after the headline, so a `--gpus N` run carries both curves' points. Nested, so
# `value` stays the headline metric the driver computes its scaling from.
NESTED = {"smaq": ("c5_multi", run_multi), "mock": ("c5_multi", run_mock_multi)}


def attach_nested(res, nested, args, world, rank, device):
    """Run the nested workload on every rank (the same barriers and max-over-ranks timing) and put
    its line under res[name] with every rank's own ms/step."""
    name, runner = nested
    m = runner(args, world, rank, device)
    out = {k: m[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "ms_per_step",
                             "scaling", "config", "roofline")}
    out["rank_ms_per_step"] = HOST.get("rank_ms_per_step")
    out["pct_hbm_peak"] = round(100.0 * m["value"] / world / HBM_PEAK_GBPS, 4)
    res[name] = out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="smaq",
                    choices=["smaq", "smaq_sampled", "fp8", "s2fp8", "multi", "packed",
                             "autograd", "autograd_resnet34", "smaq_cpu", "mock"])
    ap.add_argument("--elements", type=int, default=0, help="override elements (smaq configs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--variants", default="",
                    help="--config autograd*: comma list of variants to run (uncompressed always)")
    ap.add_argument("--saved-budget", type=int, default=0,
                    help="autograd packed-saved variant: PackedActivations verify_bytes, MiB "
                         "(0: its default)")
    ap.add_argument("--saved-exit", type=int, default=-1,
                    help="autograd packed-saved variant: PackedActivations exit_bytes, MiB "
                         "(-1: its default)")
    ap.add_argument("--saved-no-replay", action="store_true",
                    help="autograd packed-saved variant: in-place activations of codec outputs "
                         "saved as fp32 (PackedActivations replay_inplace=False)")
    ap.add_argument("--no-multi", action="store_true",
                    help="--config smaq: skip the nested C5 multi-tensor line (c5_multi)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 24)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: this process starts the ranks and relays rank 0's line
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = dist_setup()
    on_host = args.config in ("mock", "smaq_cpu")
    device = torch.device("cuda", local) if not on_host else torch.device("cpu")
    runner = {"smaq": run_smaq, "smaq_sampled": run_smaq, "fp8": run_fp8, "s2fp8": run_s2fp8,
              "multi": run_multi, "packed": run_packed, "autograd": run_autograd,
              "autograd_resnet34": run_autograd,
              "smaq_cpu": run_smaq_cpu, "mock": run_mock}[args.config]
    res = runner(args, world, rank, device)
    if world > 1:
        res.setdefault("rank_ms_per_step", HOST.get("rank_ms_per_step"))
    if args.config in NESTED and not args.no_multi and not args.elements:
        attach_nested(res, NESTED[args.config], args, world, rank, device)
        res["launcher"] = "self" if os.environ.get("TORCHELASTIC_RUN_ID") is None else "torchrun"
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline and args.config in CPU_BASELINES:
            res["cpu_baseline"] = CPU_BASELINES[args.config](args)
            res["cpu_baseline"]["host"] = _host_info()
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
