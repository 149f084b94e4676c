#!/usr/bin/env python3
"""SC-list over mixed kernels (csrc/polar_mixed.hip) with the reference's extended-BCH kernels:
GPU codewords/s against the C restatement on one core (GPU box). Prints JSON lines."""
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
# (layers, K, L, batch, trellis threshold): matrix layers of at least that size take their LLRs
# from the trellis (default 16), smaller ones enumerate the coset
CASES = [(("A",) * 5 + ("bch8",), 128, 8, 4096, 16), (("A",) * 5 + ("bch8",), 128, 8, 4096, 2),
         (("bch8",) + ("A",) * 5, 128, 8, 4096, 16), (("bch8",) + ("A",) * 5, 128, 8, 4096, 2),
         (("A",) * 4 + ("bch16",), 128, 4, 4096, 16), (("A",) * 4 + ("bch16",), 128, 8, 4096, 16),
         (("bch16",) + ("A",) * 4, 128, 8, 4096, 16), (("A",) * 7 + ("bch8",), 512, 8, 1024, 16),
         (("A",) * 3 + ("bch32f",), 128, 4, 1024, 16), (("bch32f",) + ("A",) * 3, 128, 4, 1024, 16)]
for layers, K, L, B, tmin in CASES:
    os.environ["BCHK_POLAR_TRELLIS"] = str(tmin)
    spec = mixed_spec(layers, K, dyn=4, seed=1)
    o = PolarOracle(spec, kdir)
    d = F.PolarListDecoder(spec, L, kernel_dir=kdir)
    info = np.random.default_rng(2).integers(0, 2, (B, K)).astype(np.uint8)
    llr = awgn_llr(o.encode(info), 2.0, K / o.N, seed=3)
    d.decode(llr[:64])
    t0 = time.perf_counter()
    got = d.decode(llr)
    g = time.perf_counter() - t0
    n_cpu = 32 if o.U <= 256 else 8
    t0 = time.perf_counter()
    want = o.decode_batch(llr[:n_cpu], L, threads=1)
    c = time.perf_counter() - t0
    same = all(np.array_equal(a[:n_cpu], b) for a, b in zip(got, want))
    print(json.dumps({"layers": "-".join(layers), "U": o.U, "K": K, "L": L, "B": B, "trellis_min_size": tmin,
                      "gpu_cw_s": B / g,
                      "oracle_cw_s_1core": n_cpu / c, "ratio": (B / g) / (n_cpu / c), "same_as_oracle": same}),
          flush=True)
