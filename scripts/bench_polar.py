#!/usr/bin/env python3
"""Throughput of the GPU SC-list decoder (csrc/polar_sclist.hip) on one MI355X.

A step = one bchk_polar_decode_device call over B resident codewords' LLRs (float32) of an
Arikan polar code (PW frozen set, optional dynamic constraints), AWGN at --snr. Timed with
HIP events on the decoder's own stream. Prints one JSON line: codewords/s, the kernel's
average duration, the algorithmic HBM bytes per codeword (4N LLR read + L(K + N) bytes of
information/codeword rows + 4L metrics + 4 count written) against the 8 TB/s roof, FER of
the best path, and the oracle (oracle/polar_oracle.c, one host core) on a bounded sample.

    python scripts/bench_polar.py --n 10 --K 512 --L 8 --snr 2.0 --batch 65536
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--dyn", type=int, default=0)
    ap.add_argument("--snr", type=float, default=2.0)
    ap.add_argument("--batch", type=int, default=1 << 16)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cw", action="store_true", help="do not write the codeword rows")
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    a = ap.parse_args()

    import torch
    from bchk_pkg import load
    from polar_lib import PolarOracle, arikan_spec, awgn_llr

    spec = arikan_spec(a.n, a.K, dyn=a.dyn, seed=1)
    o = PolarOracle(spec)
    d = load().PolarListDecoder(spec, a.L)
    N, K, L, B = d.N, d.K, d.L, a.batch
    rng = np.random.default_rng(1)
    base = min(B, 1 << 14)
    info = rng.integers(0, 2, (base, K)).astype(np.uint8)
    llr = awgn_llr(d.encode(info), a.snr, K / N, seed=2)
    reps = (B + base - 1) // base
    dev = torch.device("cuda:0")
    t_llr = torch.from_numpy(np.tile(llr, (reps, 1))[:B]).to(dev)
    t_info = torch.zeros((B, L, K), dtype=torch.uint8, device=dev)
    t_cw = None if a.no_cw else torch.zeros((B, L, N), dtype=torch.uint8, device=dev)
    t_met = torch.zeros((B, L), dtype=torch.float32, device=dev)
    t_cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    st = torch.cuda.ExternalStream(d.stream)

    def run():
        d.decode_device(t_llr.data_ptr(), B, t_info.data_ptr(),
                        0 if t_cw is None else t_cw.data_ptr(), t_met.data_ptr(),
                        t_cnt.data_ptr())

    for _ in range(a.warmup):
        run()
    d.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(st)
    for _ in range(a.steps):
        run()
    e1.record(st)
    d.sync()
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / a.steps
    cps = B / (ms * 1e-3)
    fer = float((t_info[:base, 0].cpu().numpy() != info).any(axis=1).mean())
    algo = 4 * N + L * (K + (0 if a.no_cw else N)) + 4 * L + 4
    gbs = algo * B / (ms * 1e-3) / 1e9

    # parity spot check + CPU baseline on a bounded sample (oracle, one core)
    cpu = None
    if a.cpu_seconds > 0:
        t = time.perf_counter()
        done = 0
        want = []
        while time.perf_counter() - t < a.cpu_seconds and done < base:
            want.append(o.decode(llr[done], L))
            done += 1
        cpu_s = time.perf_counter() - t
        cpu = {"value": done / cpu_s, "unit": "codewords/s", "cores": 1, "kind": "port",
               "sample": f"{done} codewords of the same batch, oracle/polar_oracle.c"}
        got_i = t_info[:done].cpu().numpy()
        got_m = t_met[:done].cpu().numpy()
        for b, (c, wi, wc, wm) in enumerate(want):
            assert np.array_equal(got_i[b, :c], wi[:c]), f"info mismatch row {b}"
            assert np.array_equal(got_m[b, :c].view(np.uint32), wm[:c].view(np.uint32))
    print(json.dumps({
        "metric": "SC-list codewords/s", "value": cps, "unit": "codewords/s",
        "config": {"workload": f"Arikan polar ({N},{K}) dyn={a.dyn}, L={L}, Eb/N0={a.snr} dB",
                   "batch": B, "write_codewords": not a.no_cw},
        "ms_per_step": ms, "wall_s": wall, "fer_best_path": fer,
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs / HBM_PEAK_GBS, "algo_bytes_per_codeword": algo},
        "cpu_baseline": cpu}))


if __name__ == "__main__":
    main()
