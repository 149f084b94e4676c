#!/usr/bin/env python3
"""fun() end to end on the GPU (bchk_sweep_device): BCH(63,30,13), J = 15, 0..5 dB, p words
per point, words generated on the GPU. Prints the CSV, wall time and words/s (GPU box)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from bchk_pkg import load  # noqa: E402

F = load()
p = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
m, t, J = 6, 6, 15
d = F.KanekoKernelProcessor(m, t, J=J)
d.sweep_device(1 << 16, 1 << 30, max_snr=0.5, seed=99)  # warm-up (tables, buffers)
csv, secs, words = d.sweep_device(p, 1 << 40, max_snr=5.0, seed=1)
print(csv)
print(json.dumps({"p": p, "seconds": secs, "words": words, "words_per_s": words / secs}))
