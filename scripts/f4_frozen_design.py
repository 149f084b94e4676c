#!/usr/bin/env python3
"""A (x) eBCH64 (N = 128, K = 64, L = 8, 2.5 dB): frame error rate of the test construction
(`mixed_spec`: the U - K LOWEST indices frozen, a few swaps near the boundary) against frozen
sets that keep information in both Arikan branches. u = 64 a + b (the eBCH64 kernel acts on
each 64-block, then A with stride 64): the lowest 64 indices are the whole first branch, so
the test construction leaves the information in branch 1 only -- the codeword is (v, v) for
an unrestricted 64-bit v, minimum distance 2. GPU decoder; prints JSON lines."""
import json
import os
import sys
import tempfile

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
K, L, snr = 64, 8, 2.5


def spec_keep(k0):
    """information: the k0 highest rows of branch 0 and the 64 - k0 highest of branch 1"""
    frozen = [b for b in range(64 - k0)] + [64 + b for b in range(k0)]
    lines = [f"128 {K} 0 2 0 0", "A -bch64f.txt"] + [f"1 {f}" for f in sorted(frozen)]
    return "\n".join(lines) + "\n"


designs = [("mixed_spec (test construction)", mixed_spec(("A", "bch64f"), K, dyn=0, seed=1))]
designs += [(f"branch 0 keeps {k0} rows, branch 1 keeps {64 - k0}", spec_keep(k0)) for k0 in (0, 8, 16, 24)]
for name, spec in designs:
    o = PolarOracle(spec, kdir)
    d = F.PolarListDecoder(spec, L, kernel_dir=kdir)
    info = np.random.default_rng(2).integers(0, 2, (B, K)).astype(np.uint8)
    llr = awgn_llr(o.encode(info), snr, K / o.N, seed=3)
    got = d.decode(llr)
    fer = float(np.mean(np.any(got[1][:, 0, :] != info, axis=1)))
    print(json.dumps({"design": name, "N": o.N, "K": K, "L": L, "snr_db": snr, "B": B, "fer_best_path": fer}),
          flush=True)
