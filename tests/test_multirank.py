"""The N > 1 path of bench.py on CPU: world_size-2 gloo processes run the same per-step
counter exchange and max-over-ranks timing the GPU run uses over RCCL, and each rank's
input stream is disjoint from the others (weak scaling, no data-path collective)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from oracle_lib import Oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank r decodes its own stream: here its counters are synthetic but rank-specific
    total = torch.zeros(6, dtype=torch.int64)
    steps = 3
    for s in range(steps):
        step = torch.tensor([rank + 1, 10 * (rank + 1), 100 + s, 7, 5, 1000], dtype=torch.int64)
        bench.reduce_step(step, total, world, dist)
    el = bench.max_over_ranks(0.5 + rank, world, dist, torch.device("cpu"))
    q.put((rank, total.tolist(), el))
    dist.destroy_process_group()


def test_counter_exchange_and_max_timing_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, total, el in out:
        # 3 steps x sum over ranks, never re-reducing the running total
        assert total == [3 * 3, 3 * 30, 2 * (100 + 101 + 102), 3 * 14, 3 * 10, 3 * 2000]
        assert el == 1.5


def test_rank_streams_are_disjoint():
    o = Oracle(6, 6)
    _, y0 = o.stream(bench.rank_seed(1, 0), 64, 5.0)
    _, y1 = o.stream(bench.rank_seed(1, 1), 64, 5.0)
    assert not np.any(np.all(y0[:, None, :] == y1[None, :, :], axis=2))
