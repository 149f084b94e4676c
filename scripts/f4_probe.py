#!/usr/bin/env python3
"""SC-list over the 64 x 64 eBCH kernel ((64, 32), L = 8, 2 dB by default): GPU codewords/s and
FER of the library in BCHK_LIB (experiment builds of the ordered-statistics search). One JSON line."""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

from bchk_pkg import load  # noqa: E402
from polar_lib import PolarOracle, awgn_llr  # noqa: E402
from test_polar_mixed import KERNELS, _kernel_text, mixed_spec  # noqa: E402

F = load()
kdir = tempfile.mkdtemp()
for name, K in KERNELS.items():
    open(os.path.join(kdir, f"{name}.txt"), "w").write(_kernel_text(K))
B = int(os.environ.get("BENCH_B", "2048"))
L = int(os.environ.get("F4_L", "8"))
snr = float(os.environ.get("F4_SNR", "2.0"))
K = 32
spec = mixed_spec(("bch64f",), K, dyn=0, seed=1)
o = PolarOracle(spec, kdir)
d = F.PolarListDecoder(spec, L, kernel_dir=kdir)
info = np.random.default_rng(2).integers(0, 2, (B, K)).astype(np.uint8)
llr = awgn_llr(o.encode(info), snr, K / o.N, seed=3)
d.decode(llr[:64])
t0 = time.perf_counter()
got = d.decode(llr)
g = time.perf_counter() - t0
fer = float(np.mean(np.any(got[1][:, 0, :] != info, axis=1)))
print(json.dumps({"lib": os.path.basename(os.environ.get("BCHK_LIB", "libbchk.so")), "N": o.N, "K": K, "L": L,
                  "snr_db": snr, "B": B, "gpu_cw_s": round(B / g, 1), "fer_best_path": fer,
                  "got_md5": __import__("hashlib").md5(got[1].tobytes()).hexdigest()}), flush=True)
