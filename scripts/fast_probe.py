#!/usr/bin/env python3
"""Per-stage timing of the n <= 63 decode call (HIP events on every launch), for the
environment knobs of the fast kernel (BCHK_FAST_RING, BCHK_FAST_RING_WAVES, BCHK_FAST_MODE,
BCHK_CONCURRENT_FIRST, ...) set by the caller: one JSON line.

    BCHK_FAST_MODE=1 python scripts/fast_probe.py --snr 5 --steps 20 --tag nodma

Experiment modes give wrong results by design; the line then only carries times.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=6)
    ap.add_argument("--t", type=int, default=6)
    ap.add_argument("--snr", type=float, default=5.0)
    ap.add_argument("--J", type=int, default=15)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    import torch
    import bench
    bchk = bench.load_pkg()
    dec = bchk.KanekoKernelProcessor(a.m, a.t, J=a.J)
    start, _ = bench.rank_stream_start(bchk, 1, 0, 1)
    tx, y, _, _ = dec.generate_draws(a.snr, a.batch, state=start)
    dy, dtx = torch.from_numpy(y).cuda(), torch.from_numpy(tx).cuda()
    dres = torch.zeros((a.batch, dec.n), dtype=torch.uint8, device="cuda")
    dl0 = torch.zeros(a.batch, dtype=torch.float64, device="cuda")
    cnt = torch.zeros(6, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def step():
        dec.decode_count_device(dy.data_ptr(), dtx.data_ptr(), a.batch, dres.data_ptr(), dl0.data_ptr(), 0,
                                cnt.data_ptr(), dec.stream)

    for _ in range(3):
        step()
    dec.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    dec.sync()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    dec.profile(True)
    for _ in range(a.steps):
        step()
    dec.sync()
    ms4, launches = dec.profile_read_stages()
    dec.profile(False)
    n_exact, n_coop = dec.path_counts()
    env = {k: v for k, v in os.environ.items() if k.startswith("BCHK_")}
    print(json.dumps({"tag": a.tag, "env": env, "snr_db": a.snr, "J": a.J, "batch": a.batch,
                      "ms_per_step": round(wall, 4),
                      "stages_ms": {"fast": round(ms4[0] / launches, 4), "first_pass": round(ms4[1] / launches, 4),
                                    "coop": round(ms4[2] / launches, 4), "tail": round(ms4[3] / launches, 4)},
                      "to_exact": n_exact, "to_coop": n_coop, "to_tail": dec.tail_count()}), flush=True)


if __name__ == "__main__":
    main()
