#!/usr/bin/env python3
"""Register / scratch / occupancy table of every kernel in one HIP source, from the
compiler's kernel-resource-usage remarks (gfx950, the Makefile's product flags).

    python scripts/kernel_resources.py polar-codes-with-bch-kernel_amd/csrc/bchk_fast.hip [-D...] [filter]
"""
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "polar-codes-with-bch-kernel_amd"


def main():
    src = sys.argv[1]
    defs = [a for a in sys.argv[2:] if a.startswith("-D")]
    flt = [a for a in sys.argv[2:] if not a.startswith("-D")]
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
           f"-I{REPO / 'include'}", f"-I{PKG / 'csrc'}", "--offload-arch=gfx950",
           "-munsafe-fp-atomics", *defs, "-c", src, "-o", "/tmp/kernel_resources.o",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?):\s+(.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"name": val}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    try:
        from subprocess import check_output
        names = check_output(["c++filt"], input="\n".join(r["name"] for r in rows), text=True).splitlines()
    except Exception:
        names = [r["name"] for r in rows]
    print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'spill':>5s} {'scr':>5s} {'SGspill':>7s} {'occ':>4s} {'LDS':>6s}")
    for r, n in zip(rows, names):
        if flt and not any(f in n for f in flt):
            continue
        print(f"{n[:70]:70s} {r.get('VGPRs', ''):>5s} {r.get('AGPRs', ''):>5s} {r.get('VGPRs Spill', ''):>5s} "
              f"{r.get('ScratchSize [bytes/lane]', ''):>5s} {r.get('SGPRs Spill', ''):>7s} "
              f"{r.get('Occupancy [waves/SIMD]', ''):>4s} {r.get('LDS Size [bytes/block]', ''):>6s}")


if __name__ == "__main__":
    main()
