#!/usr/bin/env python3
"""Headline batch (2^20, BCH(63,30,13), J = 15) per Eb/N0: ms per fused decode+count call
for 1..4 sub-batch pipelines (GPU box)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

from bchk_pkg import load  # noqa: E402

F = load()
B = 1 << 20
for snr in (5.0, 4.0, 6.0):
    for K in (1, 2, 3, 4, 6):
        os.environ["BCHK_PIPES"] = str(K)
        os.environ["BCHK_PIPE_MIN"] = "65536"
        d = F.KanekoKernelProcessor(6, 6, J=15)
        tx, y, _ = d.generate(snr, B, seed=1)
        dy, dtx = torch.from_numpy(y).cuda(), torch.from_numpy(tx).cuda()
        dres = torch.zeros((B, 63), dtype=torch.uint8, device="cuda")
        dl0 = torch.empty(B, dtype=torch.float64, device="cuda")
        c6 = torch.zeros(6, dtype=torch.int64, device="cuda")
        call = lambda: d.decode_count_device(dy.data_ptr(), dtx.data_ptr(), B, dres.data_ptr(), dl0.data_ptr(), 0,
                                             c6.data_ptr())
        for _ in range(3):
            call()
        d.sync()
        t0 = time.perf_counter()
        for _ in range(10):
            call()
        d.sync()
        ms = (time.perf_counter() - t0) / 10 * 1e3
        d.profile(True)
        for _ in range(3):
            call()
        d.sync()
        st, n = d.profile_read_stages()
        d.profile(False)
        print(json.dumps({"snr": snr, "pipes": K, "ms_per_call": round(ms, 4),
                          "stage_ms_sum": [round(x / n, 4) for x in st], "counts": c6.cpu().tolist()}), flush=True)
        del d
