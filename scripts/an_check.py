#!/usr/bin/env python3
"""Analytic tail: every path against the cooperative (pattern-by-pattern) path and the oracle
on the heavy rows, then per-stage timing of the headline batch (GPU box)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from bchk_pkg import load  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

F = load()


def mk(m, t, J, analytic, limit=None):
    d = F.KanekoKernelProcessor(m, t, J=J)
    d.set_analytic(analytic)
    if limit is not None:
        d.set_chunk_limit(limit)
    return d


def same(a, b):
    return (np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint64), b[1].view(np.uint64))
            and np.array_equal(a[2], b[2]))


bad = 0
PARITY = os.environ.get("AN_PARITY", "1") == "1"
for (m, t, J, snr, B) in [] if not PARITY else [(6, 6, 15, 5.0, 1 << 16), (6, 6, 15, 4.0, 1 << 16), (6, 6, 15, 3.0, 1 << 13),
                          (6, 6, -1, 5.0, 1 << 15), (6, 6, -1, 4.0, 1 << 12), (6, 6, 15, 6.0, 1 << 16),
                          (5, 3, 15, 2.0, 1 << 15), (5, 3, -1, 3.0, 1 << 14), (6, 4, 15, 4.0, 1 << 14),
                          (5, 5, 15, 3.0, 1 << 14), (4, 2, 15, 1.0, 1 << 14)]:
    mode = int(snr * 2 + m) % 3  # the tail launch modes: sequential, concurrent, hybrid
    os.environ["BCHK_TAIL_CONCURRENT"] = str(int(mode == 1))
    os.environ["BCHK_TAIL_MIN_BOUND"] = "1023" if mode == 2 else "0"
    on, off = mk(m, t, J, True), mk(m, t, J, False)
    _, y, _ = on.generate(snr, B, seed=12345)
    if J < 0:
        on.set_max_decodes(1 << 22)
        off.set_max_decodes(1 << 22)
    t0 = time.perf_counter()
    a = on.decode(y)
    t1 = time.perf_counter()
    b = off.decode(y)
    t2 = time.perf_counter()
    ok = same(a, b)
    ntail = on.tail_count()
    decs = a[2]["decodes"].astype(np.int64)
    heavy = np.flatnonzero(decs > 128)
    rows = heavy[:120]
    orc = True
    if len(rows):
        o = Oracle(m, t)
        r2, l2, s2, a2 = o.kaneko_batch(y[rows], J=J)
        acc = (a[2]["flags"][rows] & F.F_ACCEPTED) != 0
        orc = (np.array_equal(acc, a2.astype(bool)) and np.array_equal(a[0][rows][acc], r2[acc])
               and np.array_equal(a[1][rows][acc].view(np.uint64), l2[acc].view(np.uint64))
               and np.array_equal(a[2]["decodes"][rows], s2[:, 0])
               and np.array_equal(a[2]["comparisons"][rows], s2[:, 1])
               and np.array_equal(a[2]["sums"][rows], s2[:, 2]))
    bad += (not ok) + (not orc)
    print(json.dumps({"m": m, "t": t, "J": J, "snr": snr, "B": B, "same_as_coop": ok, "oracle_heavy": orc,
                      "heavy_rows": int(len(heavy)), "to_tail": ntail, "t_analytic": round(t1 - t0, 4),
                      "t_coop": round(t2 - t1, 4)}), flush=True)

# timing of the headline batch per stage
for J, snr in [(15, 5.0), (15, 4.0), (15, 6.0), (-1, 5.0)]:
    lims = [int(x) for x in os.environ.get("AN_LIMITS", "8").split(",")]
    confs = [(False, 4, 0, 0)] + [(True, L, 0, 0) for L in lims]
    for blocks in [int(x) for x in os.environ.get("AN_CONC_BLOCKS", "").split(",") if x]:
        confs.append((True, lims[0], blocks, 0))
    for analytic, limit, conc, hyb in confs:
        os.environ["BCHK_TAIL_CONCURRENT"] = str(int(conc > 0))
        os.environ["BCHK_TAIL_BLOCKS"] = str(conc or 64)
        os.environ["BCHK_TAIL_MIN_BOUND"] = str(hyb)
        d = mk(6, 6, J, analytic, limit)
        _, y, _ = d.generate(snr, 1 << 20, seed=1)
        import torch
        dy = torch.from_numpy(y).cuda()
        dres = torch.zeros((1 << 20, 63), dtype=torch.uint8, device="cuda")
        dl0 = torch.empty(1 << 20, dtype=torch.float64, device="cuda")
        dst = torch.empty((1 << 20, 56), dtype=torch.uint8, device="cuda")
        for _ in range(2):
            d.decode_device(dy.data_ptr(), 1 << 20, dres.data_ptr(), dl0.data_ptr(), dst.data_ptr())
        d.sync()
        t0 = time.perf_counter()
        for _ in range(5):
            d.decode_device(dy.data_ptr(), 1 << 20, dres.data_ptr(), dl0.data_ptr(), dst.data_ptr())
        d.sync()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        d.profile(True)
        for _ in range(3):
            d.decode_device(dy.data_ptr(), 1 << 20, dres.data_ptr(), dl0.data_ptr(), dst.data_ptr())
        d.sync()
        st, n = d.profile_read_stages()
        d.profile(False)
        ex, co = d.path_counts()
        print(json.dumps({"J": J, "snr": snr, "analytic": analytic, "chunk_limit": limit, "conc": conc, "hybrid": hyb,
                          "ms_per_call": round(ms, 4),
                          "stage_ms": [round(x / n, 4) for x in st], "to_exact": ex, "to_tail": d.tail_count(), "tail_stats": d.tail_stats(),
                          "to_coop": co}), flush=True)
sys.exit(1 if bad else 0)
