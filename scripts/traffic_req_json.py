"""profiles/traffic.json from per-request-size TCC counters (rocprofv3 --pmc CSVs of the
bench's call): memory-side bytes per launch of each kernel = 128 x RDREQ_128B + 64 x
RDREQ_64B + 32 x RDREQ_32B (reads) + 64 x WRREQ_64B + 32 x (WRREQ - WRREQ_64B) (writes).
Unlike FETCH_SIZE (RDREQ x 64 B, which halves 128-B requests on gfx950) this needs no
correction. Infinity-Cache hits are counted (the counters sit at the L2's memory side).
Usage: traffic_req_json.py RD.csv WR.csv BATCH SNR J > profiles/traffic.json"""
import collections
import csv
import datetime
import json
import re
import sys


def per_launch(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        m = re.search(r"bchk::(\w+<[^>]*>)", r["Kernel_Name"])
        if not m:
            continue
        acc[(m.group(1), r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = collections.defaultdict(dict)
    for (k, c), d in acc.items():
        out[k][c] = sum(d.values()) / len(d)
    return out


rd, wr = per_launch(sys.argv[1]), per_launch(sys.argv[2])
res = {"batch": int(sys.argv[3]), "snr_db": float(sys.argv[4]), "J": int(sys.argv[5]),
       "source": f"{sys.argv[1].split('gpurun_out/')[-1]} + {sys.argv[2].split('gpurun_out/')[-1]} "
                 "(TCC_EA0_RDREQ/WRREQ by request size)",
       "date": datetime.date.today().isoformat(), "kernels": {}, "read_bytes": {}, "write_bytes": {}}
for k in sorted(set(rd) & set(wr)):
    r, w = rd[k], wr[k]
    rb = 128 * r.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * r.get("TCC_EA0_RDREQ_64B_sum", 0) + \
        32 * r.get("TCC_EA0_RDREQ_32B_sum", 0)
    w64 = w.get("TCC_EA0_WRREQ_64B_sum", 0)
    wb = 64 * w64 + 32 * (w.get("TCC_EA0_WRREQ_sum", 0) - w64)
    key = re.sub(r"\s+", "", k)
    # bench.py's names: without the template flags; the search kernel's analytic-tail
    # instance (its last flag set) named as bench.py names it
    tail = key.startswith("kaneko_search_kernel") and key.endswith(",true>")
    key = re.sub(r",(true|false)", "", key) + ("analytictail" if tail else "")
    res["kernels"][key] = round(rb + wb)
    res["read_bytes"][key] = round(rb)
    res["write_bytes"][key] = round(wb)
print(json.dumps(res, indent=1))
