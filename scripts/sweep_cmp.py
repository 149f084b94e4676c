import os, sys
sys.path.insert(0, "tests")
from bchk_pkg import load
F = load()
d = F.KanekoKernelProcessor(6, 6, J=15)
print("host", d.sweep(200000, 1 << 30, max_snr=1.0, seed=1))
csv, s, w = d.sweep_device(200000, 1 << 30, max_snr=1.0, seed=7)
print("gpu", csv)
