#!/usr/bin/env python3
"""First-pass timeline (round 6 diagnostic; GPU box): the bench call at BCH(63,30,13), 2^20
words, with the BCHK_FP_TRACE library (per codeword: dequeue, prep, pattern loop, outputs on
the 100 MHz clock). Prints one JSON line: phase percentiles, by chunk count, concurrency."""
import json
import os
import sys

import numpy as np

os.environ["BCHK_TAIL_DIAG"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402

snr = float(sys.argv[1]) if len(sys.argv) > 1 else 5.0
F = bench.load_pkg()
d = F.KanekoKernelProcessor(6, 6, J=15)
start, _ = bench.rank_stream_start(F, 1, 0, 1)
tx, y, _, _ = d.generate_draws(snr, 1 << 20, state=start)
dy, dtx = torch.from_numpy(y).cuda(), torch.from_numpy(tx).cuda()
dres = torch.zeros((1 << 20, 63), dtype=torch.uint8, device="cuda")
cnt = torch.zeros(6, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
for _ in range(3):
    d.decode_count_device(dy.data_ptr(), dtx.data_ptr(), 1 << 20, dres.data_ptr(), 0, 0, cnt.data_ptr(), d.stream)
d.sync()
r = d.tail_diag(1 << 15).astype(np.uint64)
np.save(os.path.join(REPO, "gpurun_out", f"fptrace_raw_{snr:g}.npy"), r)
fp = r[(r[:, 0] >> np.uint64(60)) == np.uint64(0xF)].astype(np.int64)
# tail records can carry 0xF there by chance (their word 0 holds clock bits): keep ordered,
# short (< 10 ms) first-pass timelines only
ok = (fp[:, 1] <= fp[:, 2]) & (fp[:, 2] <= fp[:, 5]) & (fp[:, 5] - fp[:, 1] < 1_000_000) & (fp[:, 1] > 0)
fp = fp[ok]
fp = fp[np.abs(fp[:, 1] - np.median(fp[:, 1])) < 1_000_000]
t0, t1, f0, f1, t4 = fp[:, 1], fp[:, 2], fp[:, 3], fp[:, 4], fp[:, 5]
chunks = fp[:, 6] & 0xFFFF
handed = (fp[:, 6] >> 16) & 1
hw = (fp[:, 6] >> 32)
base = t0.min()
ten = 10.0  # ns per 100 MHz tick
ph = {"dequeue": (t1 - t0) * ten / 1e3, "prep": (f0 - t1) * ten / 1e3, "patterns": (f1 - f0) * ten / 1e3,
      "outputs": (t4 - f1) * ten / 1e3, "total": (t4 - t0) * ten / 1e3}
pct = lambda a: [round(float(np.percentile(a, q)), 2) for q in (10, 50, 90, 99)] + [round(float(a.max()), 2)]
out = {"snr": snr, "records": int(len(fp)), "span_us": round(float((t4.max() - base) * ten / 1e3), 2),
       "clock_GHz": round(float(np.median(fp[:, 7] / ((t4 - t0) * ten + 1e-9))), 3),
       "phase_us_p10_50_90_99_max": {k: pct(v) for k, v in ph.items()},
       "phase_mean_us": {k: round(float(v.mean()), 3) for k, v in ph.items()},
       "by_chunks": {}}
for c in sorted(set(chunks.tolist()))[:12]:
    s = chunks == c
    out["by_chunks"][int(c)] = {"n": int(s.sum()), "mean_total_us": round(float(ph["total"][s].mean()), 2),
                                "mean_patterns_us": round(float(ph["patterns"][s].mean()), 2)}
out["handed"] = int(handed.sum())
# concurrency: codewords in flight over time (1 us bins), waves with records
ev = np.zeros(int((t4.max() - base) // 100) + 2)
for a, b in zip((t0 - base) // 100, (t4 - base) // 100):
    ev[a] += 1
    ev[b + 1] -= 1
inflight = np.cumsum(ev)
out["inflight_p50_max"] = [float(np.percentile(inflight[:-1], 50)), float(inflight.max())]
out["waves"] = int(len(np.unique(hw)))
ends = np.sort((t4 - base) * ten / 1e3)
out["end_us_p50_p90_p99_last"] = [round(float(np.percentile(ends, q)), 2) for q in (50, 90, 99)] + [round(float(ends[-1]), 2)]
starts = (t0 - base) * ten / 1e3
out["last_starters"] = [{"start_us": round(float(starts[i]), 2), "total_us": round(float(ph["total"][i]), 2),
                         "chunks": int(chunks[i])} for i in np.argsort(-(t4 - base))[:8]]
print(json.dumps(out))
