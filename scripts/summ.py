"""One line per bench JSON line: workload, codewords/s, ms/step, decodes/codeword, stages."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        try:
            d = json.loads(line)
        except ValueError:
            continue
        ks = " ".join(f"{k['name'].split('<')[0]}={k['ms']}ms/{int(k['codewords'])}" for k in d["kernels"])
        print(f"{d['config']['workload']}: {d['value']:.4g} cw/s, {d['ms_per_step']} ms/step, "
              f"dec/cw {d['decodes_per_codeword']:.3f}, fer {d['fer']} | {ks}")
