#!/usr/bin/env python3
"""oracle/make_golden.py -- TEST INFRASTRUCTURE ONLY.

Regenerates the golden fixtures under tests/golden/ by RUNNING THE REFERENCE ITSELF:
oracle/_ref/ref_golden and oracle/_ref/kaneko are compiled by oracle/Makefile from the
unmodified sources under /root/reference (this container only). The fixtures are data
(inputs and the reference's outputs); no reference source text is stored.

    make -C oracle ref && python oracle/make_golden.py

Fixture formats (gzip text, one record per line):
  vectors_*.txt.gz   '# code n k t m gsize G seed S snr X count C' header, then per word
                     'W <tx bits> <y_0..y_{n-1} as %a> <res bits | -> <l0 %a> <decodes>
                      <comparisons> <sums> <accepted>'  (src/KanekoKernelProcessor.cpp:335)
  infile_m6t6.txt    the in/infile.txt known answer, same 'W' line (counters absolute)
  algdec_*.txt.gz    'A <word bits> <ok> <answer bits | ->'  (src/Decoder.cpp:298)
  sweep_*.csv        the reference CLI `kaneko m t file p e` output (src/dataForPlot.cpp:80)
  cli_*.txt          stdout of the reference CLI modes 1 and 3 (src/main.cpp:100-172)
  infile_input.txt   the reference's in/infile.txt fixture (input data of mode 3)
"""
import gzip
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden")
REF = os.path.join(HERE, "_ref")

# (m, t, seed, count, snr_db). J = infinity (the shipped build). Seeds vary the stream.
VECTORS = [
    (4, 2, 1, 256, 0.0), (4, 2, 7, 256, 3.0),
    (5, 3, 1, 256, 1.0), (5, 3, 11, 256, 4.0),
    (6, 6, 1, 128, 4.0), (6, 6, 13, 192, 4.5), (6, 6, 17, 256, 5.0), (6, 6, 19, 256, 6.0),
    (8, 15, 1, 48, 6.0), (8, 15, 23, 48, 7.0),
]
ALGDEC = [(4, 2, "exhaustive", 0, 0), (5, 3, "exhaustive", 0, 0),
          (6, 6, "random", 20000, 31), (8, 15, "random", 3000, 37)]
SWEEPS = [(4, 2, 10000, 10000), (5, 3, 10000, 100)]


def run(args, cwd=None):
    return subprocess.run(args, check=True, capture_output=True, text=True, cwd=cwd).stdout


def main():
    if not os.path.exists(os.path.join(REF, "ref_golden")):
        sys.exit("build the reference first: make -C oracle ref")
    os.makedirs(GOLD, exist_ok=True)
    for m, t, seed, count, snr in VECTORS:
        out = run([os.path.join(REF, "ref_golden"), "vectors", str(m), str(t), str(seed),
                   str(count), repr(snr)])
        name = f"vectors_m{m}t{t}_s{seed}_snr{snr:g}.txt.gz"
        with gzip.open(os.path.join(GOLD, name), "wt") as f:
            f.write(out)
        print(name, len(out))
    out = run([os.path.join(REF, "ref_golden"), "file", "6", "6",
               "/root/reference/in/infile.txt"])
    with open(os.path.join(GOLD, "infile_m6t6.txt"), "w") as f:
        f.write(out.replace("/root/reference/in/infile.txt", "in/infile.txt"))
    for m, t, what, count, seed in ALGDEC:
        out = run([os.path.join(REF, "ref_golden"), "algdec", str(m), str(t), what,
                   str(count), str(seed)])
        name = f"algdec_m{m}t{t}_{what}.txt.gz"
        with gzip.open(os.path.join(GOLD, name), "wt") as f:
            f.write(out)
        print(name, len(out))
    # CLI modes 1 and 3 of src/main.cpp (stdout), and the mode-3 input itself (data)
    for args, name in ((["6", "6", "0.0", "/root/reference/in/infile.txt"], "cli_infile_m6t6.txt"),
                       (["6", "6", "3.0"], "cli_random_m6t6_snr3.txt"),
                       (["4", "2", "4.0"], "cli_random_m4t2_snr4.txt")):
        with open(os.path.join(GOLD, name), "w") as f:
            f.write(run([os.path.join(REF, "kaneko")] + args))
    with open("/root/reference/in/infile.txt") as src, \
            open(os.path.join(GOLD, "infile_input.txt"), "w") as dst:
        dst.write(src.read())
    tmp = os.path.join(REF, "sweep_tmp")
    os.makedirs(tmp, exist_ok=True)
    for m, t, p, e in SWEEPS:
        run([os.path.join(REF, "kaneko"), str(m), str(t), "out", str(p), str(e)], cwd=tmp)
        name = f"sweep_m{m}t{t}_p{p}_e{e}.csv"
        with open(os.path.join(tmp, "out.csv")) as src, open(os.path.join(GOLD, name), "w") as dst:
            dst.write(src.read())
        print(name)


if __name__ == "__main__":
    main()
