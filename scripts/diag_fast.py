"""Diagnostic (libbchk_diag.so): where the fast kernel's cycles go, per wave (s_memtime
stamps: stage+keys, sort, S0, decode i=0 + accept, i=1, outputs)."""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BCHK_LIB"] = os.path.join(REPO, "polar-codes-with-bch-kernel_amd", "lib", "libbchk_diag.so")
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from bchk_pkg import load  # noqa: E402

bchk = load()
L = bchk.lib()
L.bchk_diag_read.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
B = 1 << 20
d = bchk.KanekoKernelProcessor(6, 6, J=15)
tx, y, _ = d.generate(5.0, B, seed=1)
res, l0, st = d.decode(y)
waves = B // 64
off = (1 << 20) // 8  # fast stamps start at u64 offset 1<<20 = item 131072
buf = np.zeros((off + waves, 8), np.uint64)
assert L.bchk_diag_read(d.handle, buf.ctypes.data, off + waves) == 0
f = buf[off:, :6].astype(np.float64)
names = ["stage_keys", "sort", "S0", "dec0_accept", "dec1", "outputs"]
out = {"waves": waves, "mean": {k: round(float(f[:, i].mean()), 1) for i, k in enumerate(names)},
       "p90": {k: round(float(np.percentile(f[:, i], 90)), 1) for i, k in enumerate(names)},
       "total_mean": round(float(f.sum(1).mean()), 1)}
print(json.dumps(out))
