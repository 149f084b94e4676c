"""Diagnostic: where does the cooperative kernel's time go at 5 dB, J=15, B=2^20?"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from bchk_pkg import load  # noqa: E402

bchk = load()
d = bchk.KanekoKernelProcessor(6, 6, J=15)
tx, y, _ = d.generate(5.0, 1 << 20, seed=1)
res, l0, st = d.decode(y)
dec = st["decodes"].astype(np.int64)
order = np.argsort(-dec)
out = {"top_decodes": dec[order[:32]].tolist(),
       "count_ge": {str(k): int((dec >= k).sum()) for k in (64, 256, 1024, 4096, 16384, 32767)},
       "total_decodes": int(dec.sum())}


def timed(rows, reps=3):
    yy = np.ascontiguousarray(y[rows])
    d.decode(yy)
    d.profile(True)
    for _ in range(reps):
        d.decode(yy)
    ms, calls = d.profile_read()
    d.profile(False)
    return [round(m / calls, 4) for m in ms], d.path_counts()


for k in (1, 4, 16, 64, 256, 1024, 1778):
    ms, counts = timed(order[:k])
    out[f"top{k}"] = {"ms": ms, "counts": counts}
for i in range(3):
    ms, counts = timed(order[i:i + 1])
    out[f"single{i}"] = {"decodes": int(dec[order[i]]), "ms": ms}
print(json.dumps(out))
