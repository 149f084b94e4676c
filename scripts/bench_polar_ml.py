#!/usr/bin/env python3
"""SC-list decoding over the 64 x 64 extended-BCH kernel (root bchCoder.cpp makeMatrix, field
order), kernel LLRs by the exact ordered-statistics search (polar_mixed.hip ml_llr): GPU
codewords/s and frame error rate, the C restatement on one core beside it, and equality of
the two on the sampled codewords (GPU box). Prints JSON lines."""
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
B = int(os.environ.get("BENCH_B", "16384"))
CASES = [(("bch64f",), 32, 8, 2.0), (("bch64f",), 32, 8, 3.0), (("bch64f",), 32, 1, 3.0), (("bch64f",), 32, 4, 3.0),
         (("A", "bch64f"), 64, 8, 2.5), (("bch64f", "A"), 64, 8, 2.5)]
if os.environ.get("BENCH_CASES"):  # e.g. "0,4": a subset of CASES
    CASES = [CASES[int(i)] for i in os.environ["BENCH_CASES"].split(",")]
for layers, K, L, snr in CASES:
    spec = mixed_spec(layers, K, dyn=0, seed=1)
    o = PolarOracle(spec, kdir)
    d = F.PolarListDecoder(spec, L, kernel_dir=kdir)
    info = np.random.default_rng(2).integers(0, 2, (B, K)).astype(np.uint8)
    llr = awgn_llr(o.encode(info), snr, K / o.N, seed=3)
    d.decode(llr[:64])
    t0 = time.perf_counter()
    got = d.decode(llr)
    g = time.perf_counter() - t0
    n_cpu = int(os.environ.get("BENCH_CPU", "16"))
    t0 = time.perf_counter()
    want = o.decode_batch(llr[:n_cpu], L, threads=1)
    c = time.perf_counter() - t0
    same = all(np.array_equal(a[:n_cpu], b) for a, b in zip(got, want))
    fer = float(np.mean(np.any(got[1][:, 0, :] != info, axis=1)))
    print(json.dumps({"layers": "-".join(layers), "N": o.N, "K": K, "L": L, "snr_db": snr, "B": B,
                      "gpu_cw_s": round(B / g, 1), "oracle_cw_s_1core": round(n_cpu / c, 3),
                      "ratio": round((B / g) / (n_cpu / c), 1), "fer_best_path": fer,
                      "same_as_oracle": same, "launches": d.last_launches(),
                      "budget_ms": os.environ.get("BCHK_POLAR_BUDGET_MS", "50 (default)")}), flush=True)
