#!/usr/bin/env python3
"""The analytic tail inside the first pass (BCHK_TAIL_INLINE=1) against the default separate
tail kernel: identical rows / l0 / counters on the bench's 2^20 batch, and ms per call (GPU)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from bchk_pkg import load  # noqa: E402

F = load()
import torch  # noqa: E402


def mk(inline, m=6, t=6, J=15):
    os.environ["BCHK_TAIL_INLINE"] = "1" if inline else "0"
    try:
        return F.KanekoKernelProcessor(m, t, J=J)
    finally:
        os.environ.pop("BCHK_TAIL_INLINE", None)


bad = 0
for (m, t, J, snr) in [(6, 6, 15, 5.0), (6, 6, 15, 4.0), (6, 6, 15, 6.0), (6, 6, -1, 5.0), (5, 3, 15, 2.0),
                       (5, 3, -1, 2.0)]:
    B = 1 << 20 if m == 6 else 1 << 18
    a, b = mk(False, m, t, J), mk(True, m, t, J)
    tx, y, _ = a.generate(snr, B, seed=1)
    dy, dtx = torch.from_numpy(y).cuda(), torch.from_numpy(tx).cuda()
    outs = []
    for d in (a, b):
        dres = torch.zeros((B, d.n), dtype=torch.uint8, device="cuda")
        dl0 = torch.empty(B, dtype=torch.float64, device="cuda")
        dst = torch.zeros((B, 56), dtype=torch.uint8, device="cuda")
        c6 = torch.zeros(6, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        d.decode_device(dy.data_ptr(), B, dres.data_ptr(), dl0.data_ptr(), dst.data_ptr())
        d.sync()
        r1 = (dres.cpu().numpy(), dl0.cpu().numpy(), dst.cpu().numpy())
        for _ in range(3):
            d.decode_count_device(dy.data_ptr(), dtx.data_ptr(), B, dres.data_ptr(), dl0.data_ptr(), 0, c6.data_ptr())
        d.sync()
        t0 = time.perf_counter()
        for _ in range(10):
            d.decode_count_device(dy.data_ptr(), dtx.data_ptr(), B, dres.data_ptr(), dl0.data_ptr(), 0, c6.data_ptr())
        d.sync()
        ms = (time.perf_counter() - t0) / 10 * 1e3
        d.profile(True)
        for _ in range(5):
            d.decode_count_device(dy.data_ptr(), dtx.data_ptr(), B, dres.data_ptr(), dl0.data_ptr(), 0, c6.data_ptr())
        d.sync()
        st, nc = d.profile_read_stages()
        d.profile(False)
        outs.append((r1, ms, [round(x / nc, 4) for x in st], d.tail_stats(), d.path_counts()))
    (ra, msa, sta, tsa, pca), (rb, msb, stb, tsb, pcb) = outs
    same = (np.array_equal(ra[0], rb[0]) and np.array_equal(ra[1].view(np.uint64), rb[1].view(np.uint64))
            and np.array_equal(ra[2], rb[2]))
    bad += not same
    print(json.dumps({"m": m, "t": t, "J": J, "snr": snr, "identical": same, "ms_separate": round(msa, 4),
                      "ms_inline": round(msb, 4), "stages_separate": sta, "stages_inline": stb,
                      "tail_stats_separate": tsa, "tail_stats_inline": tsb, "to_coop": [pca[1], pcb[1]]}), flush=True)
sys.exit(1 if bad else 0)
