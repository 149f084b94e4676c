"""Diagnostic: the codeword flagged TRUNCATED in the uncapped 5 dB batch -- alone, and in
growing sub-batches of the heavy codewords (with and without the syndrome table)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
from bchk_pkg import load  # noqa: E402

bchk = load()
d = bchk.KanekoKernelProcessor(6, 6, J=-1)
tx, y, _ = d.generate(5.0, 1 << 20, seed=1)
out = {}
for tab in (True, False):
    d.set_syndrome_table(tab)
    t0 = time.perf_counter()
    res, l0, st = d.decode(y)
    w = time.perf_counter() - t0
    tr = np.flatnonzero(st["flags"] & bchk.F_TRUNCATED)
    out[f"full_tab{int(tab)}"] = {"wall_s": w, "truncated": tr.tolist(),
                                   "decodes": st["decodes"][tr].tolist()}
d.set_syndrome_table(True)
dec = st["decodes"].astype(np.int64)
order = np.argsort(-dec)
tr = out["full_tab1"]["truncated"] + out["full_tab0"]["truncated"]
for i in tr[:2]:
    t0 = time.perf_counter()
    r, l, s = d.decode(np.ascontiguousarray(y[i:i + 1]))
    out[f"alone_{i}"] = {"wall_s": time.perf_counter() - t0, "decodes": int(s["decodes"][0]),
                         "flags": int(s["flags"][0])}
for k in (16, 256, 2048, 32768):
    rows = np.sort(np.unique(np.concatenate([order[:k], np.array(tr, dtype=np.int64)])))
    t0 = time.perf_counter()
    r, l, s = d.decode(np.ascontiguousarray(y[rows]))
    out[f"top{k}"] = {"wall_s": time.perf_counter() - t0,
                      "truncated": int(((s["flags"] & bchk.F_TRUNCATED) != 0).sum())}
print(json.dumps(out))
