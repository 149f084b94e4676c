#!/usr/bin/env python3
"""Analytic tail diagnostics (GPU box): per-codeword phase cycles of the tail kernel for the
headline batch -- the kernel's critical path (start stamps), the slowest codewords and the
plan's stages."""
import json
import os
import sys

import numpy as np

os.environ["BCHK_TAIL_DIAG"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from bchk_pkg import load  # noqa: E402

F = load()
cfgs = [(15, 5.0, 8), (15, 4.0, 8), (-1, 5.0, 8), (15, 5.0, 4)]
if len(sys.argv) > 1:
    cfgs = cfgs[:int(sys.argv[1])]
for J, snr, limit in cfgs:
    d = F.KanekoKernelProcessor(6, 6, J=J)
    d.set_chunk_limit(limit)
    _, y, _ = d.generate(snr, 1 << 20, seed=1)
    d.decode(y)
    d.decode(y)
    r = d.tail_diag(1 << 15).astype(np.uint64)
    r = r[:min(len(r), (1 << 15) - 1)]
    pf = d.tail_prof(len(r)).astype(np.int64) if "anprof" in os.environ.get("BCHK_LIB", "") else None
    cw = (r[:, 0] & np.uint64(0xFFFFFF)).astype(np.int64)
    xcd = ((r[:, 0] >> np.uint64(24)) & np.uint64(15)).astype(np.int64)
    start = (r[:, 0] >> np.uint64(28)).astype(np.int64)
    for x in np.unique(xcd):  # one clock per XCD
        start[xcd == x] -= start[xcd == x].min()
    prep = r[:, 1].astype(np.int64)
    st = r[:, 2]
    elim, cls, tab, setup = [((st >> np.uint64(s)) & np.uint64(0xFFFF)).astype(np.int64) for s in (0, 16, 32, 48)]
    plan = r[:, 3].astype(np.int64)
    iters = (r[:, 4] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    pre = (r[:, 4] >> np.uint64(32)).astype(np.int64)
    modef = r[:, 5].astype(np.int64)
    mode, why, split, fails = modef & 0xFF, (modef >> 8) & 0xFF, (modef >> 16) & 0xFF, modef >> 24
    after = r[:, 6].astype(np.int64)
    dec = r[:, 7].astype(np.int64)
    tot = prep + pre + plan + after
    end = start + tot
    span = int(end.max())
    order = np.argsort(-end)
    pct = lambda x: [int(np.percentile(x, q)) for q in (50, 90, 99, 100)]
    out = {"J": J, "snr": snr, "limit": limit, "n": int(len(r)), "stats": d.tail_stats(),
           "span_cycles": span, "start_p50_p90_max": [int(np.percentile(start, q)) for q in (50, 90, 100)],
           "started_after_half_span": int((start > span // 2).sum()),
           "mean": {"prep": float(prep.mean()), "elim": float(elim.mean()), "cls": float(cls.mean()),
                    "tab": float(tab.mean()), "setup": float(setup.mean()), "plan": float(plan.mean()),
                    "after": float(after.mean()), "iters": float(iters.mean()), "total": float(tot.mean())},
           "total_p50_p90_p99_max": pct(tot), "plan_p50_p90_p99_max": pct(plan), "after_p50_p90_p99_max": pct(after),
           "why_hist": {int(k): int(v) for k, v in zip(*np.unique(why[mode == 0], return_counts=True))},
           "mode_hist": {int(k): int(v) for k, v in zip(*np.unique(mode, return_counts=True))},
           "fails_hist": {int(k): int(v) for k, v in zip(*np.unique(fails, return_counts=True))},
           "last_to_end": [{"cw": int(cw[i]), "start": int(start[i]), "prep": int(prep[i]), "plan": int(plan[i]),
                            "setup": int(setup[i]), "iters": int(iters[i]), "mode": int(mode[i]),
                            "split": int(split[i]), "after": int(after[i]), "decodes": int(dec[i])}
                           for i in order[:10]],
           "slowest": [{"cw": int(cw[i]), "start": int(start[i]), "prep": int(prep[i]), "plan": int(plan[i]),
                        "setup": int(setup[i]), "iters": int(iters[i]), "mode": int(mode[i]),
                        "split": int(split[i]), "after": int(after[i]), "decodes": int(dec[i])}
                       for i in np.argsort(-tot)[:10]]}
    if pf is not None:  # enumeration cycles by step phase (experiment build)
        names = ["pop", "single", "leafrun", "push", "emits", "emit_cyc", "leaf_rounds", "steps"]
        out["prof_sum"] = {k: int(v) for k, v in zip(names, pf.sum(axis=0))}
        out["prof_slowest"] = [{k: int(v) for k, v in zip(names, pf[i])} for i in np.argsort(-tot)[:5]]
        fp = d.tail_prof(1 << 15)[-1].astype(np.int64)  # the first pass, summed (last record)
        out["first_pass"] = {k: int(v) for k, v in zip(["prep", "decode", "accept", "outputs", "chunks", "codewords"], fp[:6])}
    print(json.dumps(out), flush=True)
