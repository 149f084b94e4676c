"""Per-kernel SQ counter summary of rocprofv3 --pmc passes (DIR_sq1, DIR_sq2, ...): mean per
dispatch, and per-wave instruction counts. Usage: sq_summary.py PREFIX KERNEL_SUBSTRING"""
import collections
import csv
import glob
import sys

pre, sub = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(pre + "_sq*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            acc[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
m = {c: sum(d.values()) / len(d) for c, d in acc.items()}
for c, v in sorted(m.items()):
    print(f"{c:24s} {v / 1e6:10.2f} M")
w = m.get("SQ_WAVES", 0)
if w:
    print("per wave:", {c: round(m[c] / w) for c in m if c.startswith("SQ_INSTS")})
