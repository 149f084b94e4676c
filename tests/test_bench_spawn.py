"""bench.py's multi-rank entry on the CPU (no GPU): `--gpus N` run without a launcher starts its
own N rank processes (the driver's scaling run is exactly `bench.py --gpus N`), ranks decode
disjoint jump-ahead ranges of the one reference stream, and rank 0 prints ONE line whose
counters are the sum of the N shards. The device decoder is replaced by the C oracle
(BCHK_BENCH_STUB, tests/bench_stub.py) -- this checks the plumbing, not the kernels (those are
tests/test_bench_multirank_gpu.py and tests/test_timed_path.py on the GPU)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import bench
from bchk_pkg import load
from bench_stub import stub_counters
from oracle_lib import Oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(args, extra_env=None, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(BCHK_BENCH_STUB="1", OMP_NUM_THREADS="2")
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO,
                          capture_output=True, text=True, timeout=timeout, env=env)


def json_lines(out):
    return [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]


def shard_counters(m, t, J, snr, B, world, seed=1):
    F, o = load(), Oracle(m, t)
    want = np.zeros(6, np.int64)
    for r in range(world):
        start, budget = bench.rank_stream_start(F, seed, r, world)
        tx, y = o.stream(start, B, snr)
        assert o.stream_draws(start, B, snr)[0] <= budget
        want += stub_counters(o, J, tx, y)
    return want


COMMON = ["--m", "5", "--t", "3", "--snr", "3.0", "--points", "", "--steps", "2", "--warmup", "1",
          "--cpu-seconds", "0", "--backend", "gloo"]


def test_gpus3_spawns_three_ranks_one_line_counters_equal_shards():
    B = 384
    out = run_bench(["--gpus", "3", "--batch", str(B)] + COMMON)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = json_lines(out)
    assert len(lines) == 1, out.stdout  # rank 0 only
    rec = lines[0]
    assert rec["n_gpus"] == 3 and rec["scaling"] == "weak"
    assert rec["config"]["launch"] == "bench.py --gpus" and rec["config"]["parallelism"] == "dp3"
    assert rec["config"]["batch_per_gpu"] == B and rec["config"]["global_batch"] == 3 * B
    assert rec["stub_decoder"] and "cpu_baseline" not in rec
    want = shard_counters(5, 3, 15, 3.0, B, 3)
    np.testing.assert_array_equal(np.array(rec["points"][0]["counters"], np.int64), want)
    assert want[5] == 3 * B and rec["points"][0]["words"] == 3 * B
    assert rec["counters_complete"]


def test_global_batch_splits_over_ranks_strong_scaling():
    G = 1024
    out = run_bench(["--gpus", "2", "--global-batch", str(G)] + COMMON)
    assert out.returncode == 0, out.stderr[-4000:]
    (rec,) = json_lines(out)
    assert rec["n_gpus"] == 2 and rec["scaling"] == "strong"
    assert rec["config"]["batch_per_gpu"] == G // 2 and rec["config"]["global_batch"] == G
    assert rec["metric"].endswith("batch=2^10")
    want = shard_counters(5, 3, 15, 3.0, G // 2, 2)
    np.testing.assert_array_equal(np.array(rec["points"][0]["counters"], np.int64), want)


def test_gpus_must_equal_launcher_world():
    # a launcher (torchrun) set WORLD_SIZE: --gpus is checked against it, not obeyed
    out = run_bench(["--gpus", "2", "--batch", "64"] + COMMON,
                    extra_env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0 and "--gpus 2 but the launcher started 1 ranks" in out.stderr
    out = run_bench(["--gpus", "3", "--global-batch", "1000"] + COMMON)
    assert out.returncode != 0 and "does not split" in out.stderr


def test_single_rank_default_line():
    out = run_bench(["--batch", "256"] + COMMON)
    assert out.returncode == 0, out.stderr[-4000:]
    (rec,) = json_lines(out)
    assert rec["n_gpus"] == 1 and rec["config"]["launch"] == "single"
    want = shard_counters(5, 3, 15, 3.0, 256, 1)
    np.testing.assert_array_equal(np.array(rec["points"][0]["counters"], np.int64), want)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_config5_global_batch_fits_rank_draw_budget(world):
    """BASELINE config 5 (BCH(255,139,31), 2^20 words on 8 GPUs): as a global batch, every
    rank's 2^20 / N words stay inside its 1/N of the minstd_rand0 period (the per-rank 2^20
    of weak scaling would not at N = 8: ~829 M draws against 268 M)."""
    F = load()
    o = Oracle(8, 15)

    class A:
        global_batch, batch = 1 << 20, 1 << 20
    B, scaling = bench.rank_batch(A, world)
    assert B == (1 << 20) // world and scaling == "strong"
    for r in range(world):
        start, budget = bench.rank_stream_start(F, 1, r, world)
        _, draws = F.stream_skip(o.k, o.n, start, B)
        bench.check_rank_draws(draws, budget, world)
    if world == 8:  # weak scaling at 2^20 per rank overflows the share: bench.py refuses it
        _, draws = F.stream_skip(o.k, o.n, bench.rank_stream_start(F, 1, 0, 8)[0], 1 << 20)
        with pytest.raises(SystemExit):
            bench.check_rank_draws(draws, F.MINSTD_PERIOD // 8, 8)


def test_headline_weak_scaling_fits_rank_draw_budget_at_8():
    """Config 4 (BCH(63,30,13), 2^20 per rank, 8 ranks = 2^23): weak scaling fits."""
    F = load()
    o = Oracle(6, 6)
    for r in (0, 7):
        start, budget = bench.rank_stream_start(F, 1, r, 8)
        _, draws = F.stream_skip(o.k, o.n, start, 1 << 20)
        bench.check_rank_draws(draws, budget, 8)
