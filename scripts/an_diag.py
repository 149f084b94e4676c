#!/usr/bin/env python3
"""Analytic tail diagnostics (GPU box): per-codeword phase cycles of the tail kernel for the
headline batch, summarised (slowest codewords, hand-off reasons)."""
import json
import os
import sys

import numpy as np

os.environ["BCHK_TAIL_DIAG"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from bchk_pkg import load  # noqa: E402

F = load()
for J, snr, limit in [(15, 5.0, 4), (15, 5.0, 2), (15, 4.0, 4), (-1, 5.0, 4)]:
    d = F.KanekoKernelProcessor(6, 6, J=J)
    d.set_chunk_limit(limit)
    _, y, _ = d.generate(snr, 1 << 20, seed=1)
    d.decode(y)
    d.decode(y)
    r = d.tail_diag(1 << 16).astype(np.int64)
    mode = r[:, 5] & 0xFF
    why = (r[:, 5] >> 8) & 0xFF
    tot = r[:, 1] + r[:, 3] + r[:, 6]
    order = np.argsort(-tot)
    out = {"J": J, "snr": snr, "limit": limit, "n": int(len(r)), "stats": d.tail_stats(),
           "mean_cycles": {"cls": float((r[:, 1] & 0xFFFFF).mean()), "tab": float((r[:, 1] >> 20).mean()),
                           "elim": float((r[:, 2] & 0xFFFFF).mean()),
                           "setup": float((r[:, 2] >> 20).mean()),
                           "plan": float(r[:, 3].mean()), "after": float(r[:, 6].mean()),
                           "iters": float(r[:, 4].mean())},
           "why_hist": {int(k): int(v) for k, v in zip(*np.unique(why[mode == 0], return_counts=True))},
           "fails_hist": {int(k): int(v) for k, v in zip(*np.unique(r[:, 5] >> 24, return_counts=True))},
           "plan_cycles_p50_p90_p99_max": [int(np.percentile(r[:, 3], q)) for q in (50, 90, 99, 100)],
           "slowest": [{"cw": int(r[i, 0]), "prep": int(r[i, 1]), "elim": int(r[i, 2] & 0xFFFFF),
                        "setup": int(r[i, 2] >> 20), "plan": int(r[i, 3]),
                        "iters": int(r[i, 4]), "mode": int(mode[i]), "why": int(why[i]),
                        "split_chunks": int((r[i, 5] >> 16) & 0xFF), "fails": int(r[i, 5] >> 24),
                        "after": int(r[i, 6]), "decodes": int(r[i, 7])}
                       for i in order[:12]]}
    print(json.dumps(out), flush=True)
