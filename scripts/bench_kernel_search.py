"""Column-permutation search (csrc/kernel_search.hip) vs the literal trellis oracle: the
exhaustive m = 5 search (2^20 L.U column maps of the 32 x 32 extended-BCH kernel in
field-element order) on the GPU, and the oracle's per-candidate time on one core."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from bchk_pkg import load  # noqa: E402
from test_kernel_search import llrs_like_reference, o_counts, o_perm  # noqa: E402  (checker)

bchk = load()
out = []
for power in (3, 4, 5):
    F = bchk.kernel_field_order(power, bchk.kernel_ebch(power))
    y = llrs_like_reference(1 << power, 1)
    bchk.kernel_column_costs(power, F, y)  # warm-up (module load, first launch)
    reps = 5
    t = time.perf_counter()
    for _ in range(reps):
        r = bchk.kernel_column_search(power, F, y)
    gpu_s = (time.perf_counter() - t) / reps
    n = 1 << (power * (power - 1))
    sample = min(n, 40)
    t = time.perf_counter()
    for code in range(sample):
        o_counts(F[:, o_perm(power, code)], y)
    cpu_per = (time.perf_counter() - t) / sample
    rec = dict(power=power, kernel=1 << power, candidates=n, gpu_search_s=gpu_s,
               gpu_candidates_per_s=n / gpu_s, oracle_s_per_candidate_1core=cpu_per,
               oracle_est_search_s=cpu_per * n, best_index=r["index"], best_sum=r["sum"],
               best_cmp=r["cmp"], identity_cost=list(bchk.kernel_trellis_cost(F, y)))
    print(json.dumps(rec), flush=True)
    out.append(rec)
