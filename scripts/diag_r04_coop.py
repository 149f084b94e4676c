"""Round-4 diagnostic: BCH(255) t=4 at 4 dB (128 words, J=15) through each execution path,
with per-row decodes from the exact-only path (no cooperative kernel)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from bchk_pkg import load  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

F = load()
m, t, snr, B = (int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (8, 4, 4.0, 128)
o = Oracle(m, t)
_, y = o.stream(101, B, snr)
for name, lim, fast, an in (("exact-only", "0", False, True), ("coop-heavy", "1", True, False),
                            ("default", None, True, True)):
    if lim is not None:
        os.environ["BCHK_CHUNK_LIMIT"] = lim
    d = F.KanekoKernelProcessor(m, t, J=15)
    os.environ.pop("BCHK_CHUNK_LIMIT", None)
    d.set_fast_path(fast)
    d.set_analytic(an)
    t0 = time.time()
    try:
        res, l0, st = d.decode(y)
        print(name, "ok", f"{time.time() - t0:.2f}s", "decodes max", int(st["decodes"].max()), "sum",
              int(st["decodes"].sum()), "paths", d.path_counts(), flush=True)
        if name == "exact-only":
            print("  rows > 512 decodes:", np.sort(st["decodes"][st["decodes"] > 512])[::-1][:20].tolist(), flush=True)
            ref = (res, l0, st)
        else:
            print("  equal to exact-only:", bool(np.array_equal(res, ref[0]) and np.array_equal(st, ref[2])), flush=True)
            bad = np.flatnonzero((res != ref[0]).any(axis=1) | (st != ref[2]))
            for r in bad[:4]:
                print("   row", int(r), "exact", {k: int(ref[2][k][r]) for k in ("decodes", "jsteps", "improvements", "flags")},
                      "this", {k: int(st[k][r]) for k in ("decodes", "jsteps", "improvements", "flags")},
                      "l0", float(ref[1][r]), float(l0[r]), flush=True)
    except Exception as e:
        print(name, "FAILED", f"{time.time() - t0:.2f}s", e, flush=True)
