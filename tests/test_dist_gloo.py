"""N>1 path of bench.py on CPU: world_size-2 gloo process group, the same helpers the GPU bench
uses for its barrier, max-over-ranks elapsed time and sum-over-ranks bytes ("weak" scaling: each
rank processes its own units; no data-path collective)."""

import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "smart-quantization_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), SMQ_BENCH_BACKEND="gloo")
    import bench

    w, r, _ = bench.dist_setup()
    assert (w, r) == (world, rank)
    dev = torch.device("cpu")
    bench.barrier(w)
    elapsed = bench.max_over_ranks(0.5 + rank, w, dev)
    total = bench.sum_over_ranks(12.0 * (1000 + rank), w, dev)
    # each rank draws its own units (seed = rank), so the data differs across ranks
    x = torch.randn(4, generator=torch.Generator().manual_seed(rank))
    gathered = [torch.zeros(4) for _ in range(world)]
    dist.all_gather(gathered, x)
    q.put((rank, elapsed, total, [g.tolist() for g in gathered]))
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
    for rank, elapsed, total, gathered in res:
        assert elapsed == 1.5  # max over ranks
        assert total == 12.0 * (1000 + 1001)  # sum of both ranks' bytes
        assert gathered[0] != gathered[1]  # independent units per rank
