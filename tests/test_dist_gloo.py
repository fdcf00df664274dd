"""N>1 path of bench.py on CPU (no GPU needed):

* the launcher itself: `python bench.py --gpus N --config mock` starts N rank processes (no
  torchrun), the ranks meet in a gloo group, and rank 0's one JSON line says n_gpus = N with one
  time per rank, distinct ranks, pids and seeds (each rank owns its own units: "weak" scaling);
* the same flow under torch.distributed.run (the driver's declared launcher);
* the timing helpers (barrier, max / sum / gather over ranks) on a world_size-2 gloo group.
No data-path collective exists: the group carries barriers and timing reductions only.
"""

import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _clean_env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    return env


def _last_json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launch_n_ranks(n):
    res = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n),
                          "--config", "mock", "--steps", "4", "--warmup", "1"],
                         env=_clean_env(), cwd=REPO, capture_output=True, timeout=240)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    line = _last_json(res.stdout.decode())
    assert line["n_gpus"] == n and line["launcher"] == "self"
    assert line["ranks"] == list(range(n))
    assert len(set(line["pids"])) == n and os.getpid() not in line["pids"]
    assert len(set(line["seeds"])) == n
    assert len(line["rank_ms_per_step"]) == n and all(t > 0 for t in line["rank_ms_per_step"])
    assert line["scaling"] == "weak"
    # the nested multi-tensor line (BASELINE config 5's weak-scaling curve; run_multi on a GPU box)
    m = line["c5_multi"]
    assert m["n_gpus"] == n and m["scaling"] == "weak" and m["config"]["tensors"] == 148
    assert m["config"]["parallelism"] == f"replicas{n}"
    assert len(m["rank_ms_per_step"]) == n and all(t > 0 for t in m["rank_ms_per_step"])
    # value = every rank's bytes / the slowest rank's time (its ms_per_step)
    total = 12.0 * m["config"]["elements_per_gpu"] * n * m["steps"]
    assert m["value"] == pytest.approx(total / (m["ms_per_step"] * 1e-3 * m["steps"]) / 1e9,
                                       rel=2e-3, abs=2e-6)
    assert m["ms_per_step"] >= max(m["rank_ms_per_step"]) * 0.999


def test_bench_self_launch_failing_rank_propagates():
    """A rank that fails makes the launcher fail: the rank waiting at the start barrier is stopped
    instead of being left there."""
    env = _clean_env()
    env["SMQ_BENCH_MOCK_FAIL_RANK"] = "1"
    res = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                          "--config", "mock", "--steps", "3"],
                         env=env, cwd=REPO, capture_output=True, timeout=120)
    assert res.returncode != 0
    assert b"injected failure" in res.stderr


def test_bench_self_launch_rank0_chatter_does_not_block():
    """Rank 0 writing more than a pipe buffer (2 MiB of non-JSON stdout) before its barrier: the
    launcher must not deadlock (rank 0's stdout goes to a file, not a pipe read after exit), and
    the JSON line is still relayed."""
    env = _clean_env()
    env["SMQ_BENCH_MOCK_CHATTER"] = str(2 << 20)
    res = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                          "--config", "mock", "--steps", "3", "--warmup", "1"],
                         env=env, cwd=REPO, capture_output=True, timeout=120)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    assert _last_json(res.stdout.decode())["n_gpus"] == 2
    assert len(res.stderr) >= 2 << 20  # the chatter went to stderr, whole


def test_bench_traffic_only_for_the_profiled_workload():
    """roofline.traffic comes from a committed PMC profile only when that profile measured this
    workload (config, element count, dtype); any other size reports null, and the metric string
    names the size actually run."""
    sys.path[:0] = [REPO]
    import bench

    full = bench.traffic_from_profile("smaq", 1 << 28)
    assert full is not None and 2.1e9 < full < 2.2e9
    assert bench.traffic_from_profile("smaq", 1 << 26) is None
    assert bench.traffic_from_profile("smaq", 1 << 28, "bf16", profile="smaq_bf16") is not None
    assert bench.traffic_from_profile("smaq", 1 << 28, "f16", profile="smaq_bf16") is None
    assert bench.traffic_from_profile("fp8", 25690112) is not None
    assert bench.traffic_from_profile("s2fp8", 3145728, whole_call=True) is not None
    assert bench.traffic_from_profile("s2fp8", 1 << 20, whole_call=True) is None
    assert bench.METRIC.format(size=bench.size_label(1 << 26)).endswith("64M fp32")
    assert bench.size_label(1000) == "1000"


def test_bench_under_torchrun():
    res = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                          str(_free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
                          "--config", "mock", "--steps", "3", "--warmup", "1"],
                         env=_clean_env(), cwd=REPO, capture_output=True, timeout=240)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    line = _last_json(res.stdout.decode())
    assert line["n_gpus"] == 2 and line["launcher"] == "torchrun" and line["ranks"] == [0, 1]


def _worker(rank, world, port, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist

    import bench

    w, r, _ = bench.dist_setup()
    assert (w, r) == (world, rank) and dist.get_backend() == "gloo"
    bench.barrier(w)
    elapsed = bench.max_over_ranks(0.5 + rank, w)
    total = bench.sum_over_ranks(12.0 * (1000 + rank), w)
    each = bench.gather_over_ranks(10.0 * rank, w)
    q.put((rank, elapsed, total, each))
    dist.destroy_process_group()


def test_bench_rank_aggregation_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, elapsed, total, each in res:
        assert elapsed == 1.5  # max over ranks
        assert total == 12.0 * (1000 + 1001)  # sum of both ranks' bytes
        assert each == [0.0, 10.0]  # per-rank values in rank order
