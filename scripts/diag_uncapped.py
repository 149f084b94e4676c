"""Diagnostic: the heaviest codewords of the uncapped (J = inf) search at 5 dB, B = 2^20:
their decode counts and flags, and each one's cooperative-kernel time alone."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
from bchk_pkg import load  # noqa: E402

bchk = load()
snr = float(sys.argv[1]) if len(sys.argv) > 1 else 5.0
d = bchk.KanekoKernelProcessor(6, 6, J=-1)
tx, y, _ = d.generate(snr, 1 << 20, seed=1)
t0 = time.perf_counter()
res, l0, st = d.decode(y)
wall = time.perf_counter() - t0
dec = st["decodes"].astype(np.int64)
order = np.argsort(-dec)
out = {"wall_s": wall, "top_decodes": dec[order[:16]].tolist(),
       "top_flags": st["flags"][order[:16]].tolist(),
       "truncated": int(((st["flags"] & bchk.F_TRUNCATED) != 0).sum()),
       "total_decodes": int(dec.sum())}
for i in range(4):
    yy = np.ascontiguousarray(y[order[i:i + 1]])
    d.profile(True)
    t0 = time.perf_counter()
    d.decode(yy)
    w = time.perf_counter() - t0
    ms, calls = d.profile_read()
    d.profile(False)
    out[f"single{i}"] = {"decodes": int(dec[order[i]]), "ms": ms, "wall_s": w}
for tab in (False,):
    d.set_syndrome_table(tab)
    yy = np.ascontiguousarray(y[order[0:1]])
    d.profile(True)
    d.decode(yy)
    ms, calls = d.profile_read()
    d.profile(False)
    out["single0_no_table_ms"] = ms
print(json.dumps(out))
