"""Summarise rocprofv3 --pmc counter CSVs (one directory per pass) per kernel: mean over
dispatches of each counter, plus derived per-wave instruction counts and HBM bytes
(FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 correction; WRITE_SIZE as read)."""
import collections
import csv
import glob
import json
import sys


def main(prefix):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(prefix + "_p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bchk::", "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            acc[k]["dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            acc[k]["VGPR"].append(float(r["VGPR_Count"]))
    out = {}
    for k, d in acc.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        w = m.get("SQ_WAVES", 0) or 1
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
            if c in m:
                m[c + "_per_wave"] = m[c] / w
        if "FETCH_SIZE" in m:
            m["hbm_read_bytes"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            m["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        out[k] = {c: round(v, 2) for c, v in sorted(m.items())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
