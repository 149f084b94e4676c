"""The C restatement of the vendored SC-list decoder (oracle/polar_oracle.c) checked by
properties -- its parity is unpinned: the vendored library cannot be built here and ships
no fixtures.

* encoder / information extraction are inverse (MixedKernelEncoder.cpp:142-177, :209-238);
* noiseless words decode to themselves at metric 0, for every list size;
* L = 1 equals an independent recursive SC decoder (f/g of SoftProcessing.cpp:39-80);
* with a list as large as the code, the best path is the ML codeword and its metric is
  minus the correlation discrepancy (min-sum SC keeps exact path metrics);
* a 2x2 matrix kernel equal to Arikan's, decoded by the trellis min-sum processor
  (TrellisKernelProcessor.cpp:234-294), gives the f/g processor's results bit for bit;
* dynamic frozen constraints and puncturing round-trip.
"""
import itertools
import os

import numpy as np
import pytest

from polar_lib import PolarOracle, arikan_spec, awgn_llr, pw_order


def rand_info(K, B, seed):
    return np.random.default_rng(seed).integers(0, 2, (B, K)).astype(np.uint8)


@pytest.mark.parametrize("n,K,dyn,punct", [(4, 8, 0, ()), (6, 32, 4, ()), (8, 128, 10, ()),
                                           (7, 40, 3, (0, 5, 9))])
def test_encode_extract_roundtrip(n, K, dyn, punct):
    o = PolarOracle(arikan_spec(n, K, dyn=dyn, punct=punct, seed=n))
    for info in rand_info(K, 20, n):
        u = o.encode_unshortened(info)
        np.testing.assert_array_equal(o.extract_info(u), info)


@pytest.mark.parametrize("n,K,dyn", [(5, 16, 0), (6, 30, 5), (8, 100, 12)])
@pytest.mark.parametrize("L", [1, 4, 8])
def test_noiseless_words_decode_to_themselves(n, K, dyn, L):
    o = PolarOracle(arikan_spec(n, K, dyn=dyn, seed=3))
    info = rand_info(K, 6, 7)
    cw = o.encode(info)
    for b in range(len(info)):
        llr = np.where(cw[b] != 0, -4.0, 4.0).astype(np.float32)
        cnt, inf, c, met = o.decode(llr, L)
        np.testing.assert_array_equal(inf[0], info[b])
        np.testing.assert_array_equal(c[0], cw[b])
        assert met[0] == 0.0 and cnt == min(L, 1 << K)


def recursive_sc(llr, frozen):
    """Plain recursive SC over the same transform (first half a, second half b; f then g),
    float32 arithmetic, static frozen symbols = 0. Returns (u, metric)."""
    u = []
    metric = [np.float32(0.0)]

    def rec(l, fr):
        n = len(l)
        if n == 1:
            bit = 0 if fr[0] else int(l[0] < 0)
            if fr[0] and l[0] < 0:
                metric[0] = np.float32(metric[0] - np.abs(l[0]))
            u.append(bit)
            return np.array([bit], np.uint8)
        a, b = l[: n // 2], l[n // 2:]
        f = (np.sign(a) * np.sign(b) * np.minimum(np.abs(a), np.abs(b))).astype(np.float32)
        f = np.where((np.signbit(a) != np.signbit(b)), -np.minimum(np.abs(a), np.abs(b)),
                     np.minimum(np.abs(a), np.abs(b))).astype(np.float32)
        x0 = rec(f, fr[: n // 2])
        g = np.where(x0 != 0, b - a, b + a).astype(np.float32)
        x1 = rec(g, fr[n // 2:])
        return np.concatenate([x0 ^ x1, x1])

    rec(llr.astype(np.float32), frozen)
    return np.array(u, np.uint8), metric[0]


@pytest.mark.parametrize("n,K,snr", [(5, 16, 1.0), (6, 32, 2.0), (7, 64, 2.5)])
def test_list1_equals_recursive_sc(n, K, snr):
    o = PolarOracle(arikan_spec(n, K, seed=1))
    frozen = np.zeros(1 << n, bool)
    frozen[pw_order(n)[:(1 << n) - K]] = True
    info = rand_info(K, 40, 11)
    cw = o.encode(info)
    llr = awgn_llr(cw, snr, K / (1 << n), seed=5)
    for b in range(len(info)):
        u, m = recursive_sc(llr[b], frozen)
        cnt, inf, c, met = o.decode(llr[b], 1)
        np.testing.assert_array_equal(inf[0], u[~frozen])
        assert met[0] == m


def ml_discrepancy(o, llr):
    """min over all 2^K codewords of sum |llr_i| over positions disagreeing with the LLR's
    hard decision (bit 1 when llr < 0)."""
    infos = np.array(list(itertools.product([0, 1], repeat=o.K)), np.uint8)
    cws = o.encode(infos)
    hd = (llr < 0).astype(np.uint8)
    d = ((cws != hd[None, :]) * np.abs(llr)[None, :]).sum(axis=1)
    return infos, cws, d


@pytest.mark.parametrize("spec_kind", ["arikan", "matrix4"])
def test_full_list_finds_the_ml_codeword(spec_kind, tmp_path):
    if spec_kind == "arikan":
        spec, kdir = arikan_spec(4, 5, seed=2), None
    else:
        # a 4x4 kernel (rows of A (x) A with a column swap) over one Arikan layer, N = 8
        (tmp_path / "k4.txt").write_text("4\n1 0 0 0\n1 0 1 0\n1 1 0 0\n1 1 1 1\n")
        spec = "8 4 0 2 0 0\n-k4.txt A\n1 0\n1 1\n1 2\n1 4\n"
        kdir = str(tmp_path)
    o = PolarOracle(spec, kdir)
    rng = np.random.default_rng(9)
    for trial in range(30):
        info = rng.integers(0, 2, (1, o.K)).astype(np.uint8)
        llr = awgn_llr(o.encode(info), 0.0, o.K / o.N, seed=100 + trial)[0]
        cnt, inf, cw, met = o.decode(llr, 1 << o.K)
        infos, cws, d = ml_discrepancy(o, llr)
        assert cnt == 1 << o.K
        best = np.argmin(d)
        if np.sum(d == d[best]) == 1:
            np.testing.assert_array_equal(inf[0], infos[best])
        np.testing.assert_allclose(-met[0], d[best], rtol=1e-5, atol=1e-5)
        # every codeword is in the list, metrics = -discrepancy
        got = {tuple(c): -m for c, m in zip(cw[:cnt], met[:cnt])}
        for c, dd in zip(cws, d):
            assert abs(got[tuple(c)] - dd) <= 1e-4 * max(1.0, dd)


def test_matrix_kernel_equal_to_arikan_gives_identical_results(tmp_path):
    (tmp_path / "a2.txt").write_text("2\n1 0\n1 1\n")
    n, K = 6, 28
    base = arikan_spec(n, K, dyn=4, seed=4)
    head, kern, rest = base.split("\n", 2)
    o_a = PolarOracle(base)
    o_m = PolarOracle(head + "\n" + " ".join(["-a2.txt"] * n) + "\n" + rest, str(tmp_path))
    info = rand_info(K, 25, 3)
    llr = awgn_llr(o_a.encode(info), 1.5, K / 64, seed=8)
    for L in (1, 4):
        for b in range(len(info)):
            ra, rm = o_a.decode(llr[b], L), o_m.decode(llr[b], L)
            assert ra[0] == rm[0]
            np.testing.assert_array_equal(ra[1], rm[1])
            np.testing.assert_array_equal(ra[3], rm[3])


def test_list_decoding_helps_at_low_snr():
    n, K = 7, 64
    o = PolarOracle(arikan_spec(n, K, seed=5))
    info = rand_info(K, 150, 21)
    llr = awgn_llr(o.encode(info), 2.0, K / 128, seed=22)
    err = {}
    for L in (1, 8):
        err[L] = sum(int(np.any(o.decode(llr[b], L)[1][0] != info[b])) for b in range(len(info)))
    assert err[8] <= err[1] and err[1] > 0


def test_spec_errors_are_reported(tmp_path):
    with pytest.raises(ValueError, match="length mismatch"):
        PolarOracle("10 5 0 3 0 0\nA A A\n1 0\n1 1\n1 2\n")
    with pytest.raises(ValueError, match="Unknown kernel"):
        PolarOracle("3 1 0 1 0 0\nG\n1 0\n1 1\n")
    (tmp_path / "sing.txt").write_text("2\n1 1\n1 1\n")
    with pytest.raises(ValueError, match="singular"):
        PolarOracle("2 1 0 1 0 0\n-sing.txt\n1 0\n", str(tmp_path))
