"""The drop-in boundary at the reference's own level: its src/main.cpp (and, for
kaneko_refsweep, its src/dataForPlot.cpp) compiled UNCHANGED against include/bchk_dropin/
and linked with libbchk_dropin.so + libbchk.so. The CLI output and the CSV files must be
the reference's, byte for byte (fixtures in tests/golden/ made by the reference binary)."""
import hashlib
import os
import re
import subprocess

import pytest

from bchk_pkg import PKG_DIR, REPO
from golden import GOLD

BIN = os.path.join(PKG_DIR, "bin")
LIB = os.path.join(PKG_DIR, "lib")
HAVE_REF = os.path.exists("/root/reference/src/main.cpp")


def _build_dropin():
    targets = ["dropin"] + (["refbins"] if HAVE_REF else [])
    subprocess.run(["make", "-s", "-C", PKG_DIR] + targets, check=True)


def _need_bins():
    if HAVE_REF:
        _build_dropin()
    for b in ("kaneko", "kaneko_refsweep"):
        if not os.path.exists(os.path.join(BIN, b)):
            pytest.skip(f"{b} not built (needs /root/reference at build time)")


def test_dropin_library_exports_reference_api():
    _build_dropin()
    out = subprocess.run(["nm", "-DC", "--defined-only", os.path.join(LIB, "libbchk_dropin.so")],
                         capture_output=True, text=True, check=True).stdout
    for sym in ("KanekoKernelProcessor::KanekoKernelProcessor(long, long, long, long, unsigned long*, unsigned long*, double)",
                "KanekoKernelProcessor::decode(unsigned char const*, double const*, unsigned char*)",
                "KanekoKernelProcessor::decode(double const*, unsigned char*)",
                "KanekoKernelProcessor::calcL(unsigned char const*) const",
                "KanekoKernelProcessor::getDecodingCount() const",
                "Decoder::Decoder(long, long, long, long, unsigned long*, unsigned long*)",
                "Decoder::decode(unsigned char const*, unsigned char*)",
                "Decoder::findSyndromPoly(unsigned char const*)",
                "Decoder::alterSyndromPoly(unsigned char const*)",
                "findMinimalPolynomial(int, int, unsigned long const*, int*, unsigned char*)",
                "lcm(unsigned char const*, int, unsigned char const*, int, int*)",
                "addNoise(double, unsigned char const*, double*, unsigned long)",
                "fun(std::__cxx11::basic_string<char, std::char_traits<char>, std::allocator<char> > const&, KanekoKernelProcessor&, unsigned char const*, unsigned long, long, long, double)"):
        assert sym in out, sym


@pytest.mark.skipif(not HAVE_REF, reason="needs /root/reference to compile its main.cpp")
def test_reference_main_compiles_unchanged_against_dropin_headers():
    _build_dropin()
    for b in ("kaneko", "kaneko_refsweep"):
        assert os.path.exists(os.path.join(BIN, b))


def _run(args, cwd, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([os.path.join(BIN, args[0])] + args[1:], cwd=cwd, env=e,
                          capture_output=True, text=True, timeout=600)


def _strip_timing(s):
    return re.sub(r"Общее время: .*", "", s)


@pytest.mark.gpu
@pytest.mark.parametrize("binary", ["kaneko", "kaneko_refsweep"])
@pytest.mark.parametrize("m,t,p,e", [(4, 2, 10000, 10000), (5, 3, 10000, 100)])
def test_cli_sweep_csv_is_the_references(binary, m, t, p, e, tmp_path):
    _need_bins()
    r = _run([binary, str(m), str(t), "out", str(p), str(e)], cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    want = open(os.path.join(GOLD, f"sweep_m{m}t{t}_p{p}_e{e}.csv")).read()
    assert open(tmp_path / "out.csv").read() == want
    lines = _strip_timing(r.stdout).split("\n")
    assert "(%d, " % ((1 << m) - 1) in r.stdout and "0.5" in lines and "5" in lines


@pytest.mark.gpu
@pytest.mark.parametrize("m,t,md5", [
    (5, 3, "105c77e4bb47a243054121d9c907feae"),
    # the headline configuration (SURVEY.md §6.4 / BASELINE.md): BCH(63,30,13), J=15,
    # p=10^6 e=100 -- md5 of the reference binary's CSV as recorded there
    (6, 6, "e0beb7a4b884a4d0b8393c270827b028")])
def test_cli_sweep_j15_md5(m, t, md5, tmp_path):
    _need_bins()
    r = _run(["kaneko", str(m), str(t), "j15", "1000000", "100"], cwd=tmp_path,
             env={"BCHK_J": "15"})
    assert r.returncode == 0, r.stderr
    csv = open(tmp_path / "j15.csv").read()
    assert hashlib.md5(csv.encode()).hexdigest() == md5


@pytest.mark.gpu
def test_cli_sweep_bch15_shipped_md5(tmp_path):
    """`kaneko 4 2 x 1000000 1000` with the shipped (uncapped) search: md5 of the reference
    binary's CSV recorded in SURVEY.md §6.2."""
    _need_bins()
    r = _run(["kaneko", "4", "2", "x", "1000000", "1000"], cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    csv = open(tmp_path / "x.csv").read()
    assert hashlib.md5(csv.encode()).hexdigest() == "82dcef4a50ad04e68ac2385ebafdcd06"


@pytest.mark.gpu
@pytest.mark.parametrize("binary", ["kaneko", "kaneko_refsweep"])
@pytest.mark.parametrize("args,fixture", [
    (["6", "6", "0.0", "{infile}"], "cli_infile_m6t6.txt"),
    (["6", "6", "3.0"], "cli_random_m6t6_snr3.txt"),
    (["4", "2", "4.0"], "cli_random_m4t2_snr4.txt")])
def test_cli_single_word_modes_match_reference_stdout(binary, args, fixture, tmp_path):
    _need_bins()
    args = [a.format(infile=os.path.join(GOLD, "infile_input.txt")) for a in args]
    r = _run([binary] + args, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert r.stdout == open(os.path.join(GOLD, fixture)).read()
