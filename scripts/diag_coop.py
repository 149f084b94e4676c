"""Diagnostic (libbchk_diag.so): per heavy codeword, where the cooperative kernel's cycles go."""
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
m, t, snr, J, B = 6, 6, 5.0, 15, 1 << 20
if len(sys.argv) > 5:
    m, t, snr, J, B = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
d = bchk.KanekoKernelProcessor(m, t, J=J)
tx, y, _ = d.generate(snr, B, seed=1)
res, l0, st = d.decode(y)
_, n_coop = d.path_counts()
buf = np.zeros((n_coop, 8), np.uint64)
assert L.bchk_diag_read(d.handle, buf.ctypes.data, n_coop) == 0
dec = st["decodes"][buf[:, 7].astype(np.int64)]
# chunks_decoded: chunks decoded by all waves (m <= 6), decode rounds of 64 packed patterns (m >= 7)
names = ["prep", "wait_chunks", "accept", "chunks_decoded", "chunks_accepted", "improvements", "total"]
if m >= 7:  # decoders' cycles in claims and waiting, summed over the decoder waves
    names = ["prep", "wait_chunks", "accept", "decode_rounds", "dec_claim_cycles", "dec_wait_cycles", "total"]
out = {"n": int(n_coop), "sum": {k: int(buf[:, i].sum()) for i, k in enumerate(names)}}
top = np.argsort(-buf[:, 6].astype(np.int64))[:8]
out["top"] = [{**{k: int(buf[j, i]) for i, k in enumerate(names)}, "decodes": int(dec[j])} for j in top]
out["config"] = {"m": m, "t": t, "snr": snr, "J": J, "B": B}
tot = buf[:, 6].astype(np.float64)
out["total_cycles_pct"] = {q: float(np.percentile(tot, q)) for q in (50, 90, 99, 100)}
out["decodes_pct"] = {q: float(np.percentile(dec, q)) for q in (50, 90, 99, 100)}
print(json.dumps(out))
