"""bench.py's N > 1 branch executed on the GPU (verdict r3 item 5): two ranks on the box's one
GPU under torchrun, the per-step counter exchange over the gloo backend (the same
reduce_step / barrier / max-over-ranks code the RCCL run takes; only the transport differs).
The all-reduced counters of one pass must equal the two jump-ahead shards decoded separately
in this process. This is not a scaling measurement: both ranks share one GPU."""
import importlib.util
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from bchk_pkg import load

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_module():
    spec = importlib.util.spec_from_file_location("bench_under_test_mr", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


BENCH_ARGS = ["--gpus", "2", "--backend", "gloo", "--steps", "3", "--warmup", "1", "--points", "",
              "--cpu-seconds", "0"]  # BCH(63,30,13) at 5 dB: bench.py's defaults
# (no --m / --t: torch.distributed.run's parser would take them as abbreviations of its own)


def run_two_ranks(cmd):
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"))
    out = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints one line
    rec = json.loads(lines[0])
    print(json.dumps({k: rec[k] for k in ("value", "ms_per_step", "n_gpus", "config")}))
    return rec


@pytest.mark.parametrize("m,t,snr", [(6, 6, 5.0)])
def test_bench_two_ranks_gloo_counters_equal_shards(m, t, snr):
    B = 1 << 16
    rec = run_two_ranks([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                         "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py",
                         *BENCH_ARGS, "--batch", str(B)])
    assert rec["config"]["launch"] == "torchrun"
    check_counters_equal_shards(rec, m, t, snr, B)


def test_bench_gpus2_spawns_its_ranks_counters_equal_shards():
    """`python bench.py --gpus 2` with no launcher: bench.py starts both ranks itself (the
    driver's scaling command without torchrun), one line, the two shards' counters."""
    B = 1 << 16
    rec = run_two_ranks([sys.executable, "bench.py", *BENCH_ARGS, "--batch", str(B)])
    assert rec["config"]["launch"] == "bench.py --gpus"
    check_counters_equal_shards(rec, 6, 6, 5.0, B)


def check_counters_equal_shards(rec, m, t, snr, B):
    import torch
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 2 * B
    assert rec["config"]["backend"] == "gloo" and rec["config"]["parallelism"] == "dp2"
    assert rec["value"] > 0 and rec["points"][0]["words"] == 2 * B
    # the two shards, decoded here one after the other (the fused call bench.py makes)
    bench = bench_module()
    F = load()
    d = F.KanekoKernelProcessor(m, t, J=15)
    want = np.zeros(6, np.int64)
    for r in range(2):
        start, budget = bench.rank_stream_start(F, 1, r, 2)
        tx, y, _, used = d.generate_draws(snr, B, state=start)
        assert used <= budget
        dy, dtx = torch.from_numpy(y).cuda(), torch.from_numpy(tx).cuda()
        dres = torch.zeros((B, d.n), dtype=torch.uint8, device="cuda")
        c6 = torch.zeros(6, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        d.decode_count_device(dy.data_ptr(), dtx.data_ptr(), B, dres.data_ptr(), 0, 0, c6.data_ptr())
        d.sync()
        want += c6.cpu().numpy()
    np.testing.assert_array_equal(np.array(rec["points"][0]["counters"], np.int64), want)
    assert want[5] == 2 * B
