"""profiles/traffic.json from a pmc_summary.py output: HBM bytes per launch of each kernel
(FETCH_SIZE doubled per the gfx950 correction + WRITE_SIZE), for bench.py's roofline
`traffic` field. Usage: traffic_json.py SUMMARY.json BATCH SNR J > profiles/traffic.json"""
import datetime
import json
import re
import sys

summ = json.load(open(sys.argv[1]))
out = {"batch": int(sys.argv[2]), "snr_db": float(sys.argv[3]), "J": int(sys.argv[4]),
       "source": sys.argv[1].split("gpurun_out/")[-1], "date": datetime.date.today().isoformat(),
       "kernels": {}}
for name, v in summ.items():
    if "hbm_read_bytes" in v and "hbm_write_bytes" in v:
        key = re.sub(r"\s+", "", name).replace(",true>", ">").replace(",false>", ">")
        out["kernels"][key] = round(v["hbm_read_bytes"] + v["hbm_write_bytes"])
print(json.dumps(out, indent=1))
