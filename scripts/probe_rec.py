"""Probe (round 6): cooperative dense re-decodes and stage times of BCH(255) at low Eb/N0."""
import os, sys, time
sys.path.insert(0, "tests")
from bchk_pkg import load
F = load()
rec = sys.argv[1] if len(sys.argv) > 1 else ""
if rec:
    os.environ["BCHK_LONG_REC"] = rec
cases = [(8, 15, 15, 3.0, 1 << 11), (8, 15, 15, 2.0, 256), (8, 15, 15, 3.0, 256), (7, 10, 15, 2.0, 1024)]
for m, t, J, snr, B in cases:
    d = F.KanekoKernelProcessor(m, t, J=J)
    _, y, _ = d.generate(snr, B, seed=59)
    d.profile(True)
    t0 = time.time(); res, l0, st = d.decode(y); dt = time.time() - t0
    ms, n = d.profile_read_stages()
    print(f"rec={rec or 'def'} m={m} t={t} J={J} snr={snr} B={B} coop={d.coop_stats()} paths={d.path_counts()} "
          f"wall={dt:.2f}s stages(fast,exact,coop,tail)={[round(x, 2) for x in ms]} "
          f"decodes={int(st['decodes'].sum())} max={int(st['decodes'].max())}", flush=True)
    d.close()
