"""Timing of the fast kernel cut after successive phases (libbchk_cut{N}.so builds, see
scripts/gpu_fast_cut.sh): the difference between cuts is the cost of a phase. The call is the
bench's (bchk_decode_count_device, no stats record: the 16-key selection kernel)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bchk_pkg import load  # noqa: E402

bchk = load()
B = 1 << 20
d = bchk.KanekoKernelProcessor(6, 6, J=15)
tx, y, _ = d.generate(5.0, B, seed=1)
dev = torch.device("cuda", 0)
d_y = torch.from_numpy(y).to(dev)
d_res = torch.zeros((B, d.n), dtype=torch.uint8, device=dev)
d_l0 = torch.empty(B, dtype=torch.float64, device=dev)
d_tx = torch.from_numpy(tx).to(dev)
d_cnt = torch.zeros(6, dtype=torch.int64, device=dev)
torch.cuda.synchronize()
d.set_fast_path(True)


def step():
    d.decode_count_device(d_y.data_ptr(), d_tx.data_ptr(), B, d_res.data_ptr(), d_l0.data_ptr(), 0,
                          d_cnt.data_ptr(), d.stream)


for _ in range(2):
    step()
d.sync()
d.profile(True)
for _ in range(5):
    step()
d.sync()
ms3, calls = d.profile_read()
print(json.dumps({"lib": os.environ.get("BCHK_LIB", "default"), "fast_ms": ms3[0] / calls,
                  "exact_ms": ms3[1] / calls, "coop_ms": ms3[2] / calls}))
