"""Round 6 debug: one batch over the 64 x 64 kernel decoded with and without time-budgeted
launches; which codewords differ."""
import os
import sys
import tempfile
sys.path.insert(0, "tests")
import numpy as np
from bchk_pkg import load
from polar_lib import PolarOracle, awgn_llr
from test_polar_mixed import KERNELS, _kernel_text, mixed_spec

kdir = tempfile.mkdtemp()
for name, K in KERNELS.items():
    open(os.path.join(kdir, f"{name}.txt"), "w").write(_kernel_text(K))
layers, K, dyn, L = ("bch64f",), 40, 3, int(sys.argv[1]) if len(sys.argv) > 1 else 1
spec = mixed_spec(layers, K, dyn, (), seed=len(layers) * 19 + K)
o = PolarOracle(spec, kdir)
rng = np.random.default_rng(L * 3 + K)
info = rng.integers(0, 2, (16, K)).astype(np.uint8)
llr = awgn_llr(o.encode(info), 1.0, K / o.N, seed=10 + L)
res = {}
for tag, env in [("b0", {"BCHK_POLAR_BUDGET_MS": "0"}), ("b5_nomid", {"BCHK_POLAR_BUDGET_MS": "5", "BCHK_POLAR_NO_MID": "1"}),
                 ("b5", {"BCHK_POLAR_BUDGET_MS": "5"}), ("b50", {"BCHK_POLAR_BUDGET_MS": "50"})]:
    for k in ("BCHK_POLAR_BUDGET_MS", "BCHK_POLAR_NO_MID"):
        os.environ.pop(k, None)
    os.environ.update(env)
    d = load().PolarListDecoder(spec, L, kernel_dir=kdir)
    res[tag] = d.decode(llr)
    diff = [b for b in range(16) if not (np.array_equal(res[tag][1][b], res["b0"][1][b]) and
                                          np.array_equal(res[tag][3][b], res["b0"][3][b]))]
    print(tag, "launches", d.last_launches(), "differ", diff, flush=True)
