"""Kernel LLRs of large BCH kernels by an exact ordered-statistics search.

The reference's trellis processor stops below 64 (out/external/TrellisKernelProcessor.cpp:
70-71), so the 64 x 64 nested extended-BCH kernel (root bchCoder.cpp:356-389 makeMatrix) has
no reference LLR processor. Its LLRs here are CTrellisKernelProcessor's value (best[1] -
best[0] over the coset, :234-294) computed by a certified search: the GPU's (polar_mixed.hip
ml_llr) and the oracle's restatement (oracle/polar_oracle.c ml_minsum_llr). This file pins
that search, bit for bit in float, to the coset enumeration and to the literal trellis
(extended to 65 columns for the 64 x 64 kernel):

* CPU: the oracle's search == enumeration == trellis, every phase, for 8 .. 32 kernels; for
  the 64 x 64 kernel == enumeration wherever the coset has <= 2^18 words and == the trellis
  at middle phases (field order: <= 2^23 states);
* GPU: SC-list decoding through the search (forced onto 8 .. 32 kernels, whose oracle LLRs
  come from enumeration / trellis) == the oracle; codes over the 64 x 64 kernel == the oracle.

Parity unpinned (as all of §8f): the vendored library has no 64 x 64 processor and ships no
fixtures.
"""
import ctypes as C
import os

import numpy as np
import pytest

from bchk_pkg import load
from polar_lib import PolarOracle, awgn_llr
from polar_lib import lib as plib
from test_polar_mixed import KERNELS, _lower_kernel, _plr_kernel, _same, kdir, mixed_spec  # noqa: F401

BY_ENUM, BY_TRELLIS, BY_ML = 0, 1, 2


def _lib():
    L = plib()
    L.plr_minsum_llr_by.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int]
    L.plr_minsum_llr_by.restype = C.c_float
    L.plr_ml_nodes.restype = C.c_long
    return L


def _llr(k, ph, y, method):
    y = np.ascontiguousarray(y, np.float32)
    return np.float32(_lib().plr_minsum_llr_by(C.byref(k), ph, y.ctypes.data_as(C.c_void_p), method))


def _vectors(l, seed, count):
    """AWGN-like kernel outputs plus adversarial rows: exact |y| ties, zeros (punctured),
    100000 (shortened), mixed scales."""
    rng = np.random.default_rng(seed)
    out = [rng.normal(0, 1.5, l) * 2.0 for _ in range(count)]
    y = rng.normal(0, 1.0, l)
    y[::3] = np.abs(y[1]) * np.sign(y[::3] + 0.1)  # many exact ties
    out.append(y)
    y = rng.normal(0, 1.0, l)
    y[rng.choice(l, l // 4, replace=False)] = 0.0
    out.append(y)
    y = rng.normal(1.0, 1.0, l) * 3
    y[rng.choice(l, 3, replace=False)] = 100000.0
    out.append(y)
    return [np.asarray(v, np.float32) for v in out]


@pytest.mark.parametrize("name", ["k3", "k8", "bch8", "k16", "bch16", "bch32f"])
def test_oracle_ml_search_equals_enumeration_and_trellis(name):
    K = KERNELS[name]
    l = len(K)
    k = _plr_kernel(K)
    for y in _vectors(l, l, 3):
        for ph in range(l):
            ml = _llr(k, ph, y, BY_ML)
            tr = _llr(k, ph, y, BY_TRELLIS)
            assert ml.view(np.uint32) == tr.view(np.uint32), (name, ph, ml, tr)
            if l - ph - 1 <= 16:
                en = _llr(k, ph, y, BY_ENUM)
                assert ml.view(np.uint32) == en.view(np.uint32), (name, ph, ml, en)


def test_oracle_64_kernel_search_equals_enumeration():
    # every phase whose coset has <= 2^17 words (46..63), both column orders
    for name in ("bch64f", "bch64"):
        k = _plr_kernel(KERNELS[name])
        for y in _vectors(64, 7, 1):
            for ph in range(46, 64):
                ml, en = _llr(k, ph, y, BY_ML), _llr(k, ph, y, BY_ENUM)
                assert ml.view(np.uint32) == en.view(np.uint32), (name, ph, ml, en)


def test_oracle_64_kernel_search_equals_literal_trellis():
    # middle phases through CTrellisKernelProcessor's trellis with 65 columns (field order:
    # at most 2^23 states, ~0.3 s per LLR); low / high phases in power order too
    k = _plr_kernel(KERNELS["bch64f"])
    for y in _vectors(64, 9, 1)[:2]:
        for ph in (3, 13, 22, 31, 40):
            ml, tr = _llr(k, ph, y, BY_ML), _llr(k, ph, y, BY_TRELLIS)
            assert ml.view(np.uint32) == tr.view(np.uint32), ("bch64f", ph, ml, tr)
    k = _plr_kernel(KERNELS["bch64"])
    y = _vectors(64, 11, 1)[0]
    for ph in (0, 5, 12, 50, 58):
        ml, tr = _llr(k, ph, y, BY_ML), _llr(k, ph, y, BY_TRELLIS)
        assert ml.view(np.uint32) == tr.view(np.uint32), ("bch64", ph, ml, tr)


def test_64_kernel_is_the_nested_construction():
    # the test kernels == the oracle's makeMatrix restatement (kernel_oracle.c) and the
    # product's (bchk_kernel_ebch / bchk_kernel_field_order, power 6)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    KL = C.CDLL(os.path.join(repo, "oracle", "build", "libkernel_oracle.so"))
    K = np.zeros((64, 64), np.uint8)
    assert KL.kor_make_ebch(6, K.ctypes.data_as(C.c_void_p)) == 0
    np.testing.assert_array_equal(K, KERNELS["bch64"])
    F = np.zeros_like(K)
    KL.kor_field_order(6, K.ctypes.data_as(C.c_void_p), F.ctypes.data_as(C.c_void_p))
    np.testing.assert_array_equal(F, KERNELS["bch64f"])
    B = load()
    np.testing.assert_array_equal(B.kernel_ebch(6), K)
    np.testing.assert_array_equal(B.kernel_field_order(6, K), F)


# ---- GPU: SC-list decoding through the search
FORCED = [
    (("bch16", "A"), 16, 2, ()),
    (("A", "k16"), 16, 2, ()),
    (("bch8", "A", "A"), 16, 2, (3,)),
    (("bch32f", "A"), 32, 2, ()),
]
CODES64 = [
    (("bch64f",), 32, 0, ()),
    (("bch64f",), 40, 3, ()),
    (("bch64",), 24, 2, ()),
    (("A", "bch64f"), 64, 2, ()),
    (("bch64f", "A"), 60, 2, (5, 77)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("layers,K,dyn,punct", FORCED, ids=["-".join(c[0]) for c in FORCED])
@pytest.mark.parametrize("L", [1, 4, 8])
def test_gpu_search_forced_on_small_kernels_matches_oracle(kdir, layers, K, dyn, punct, L, monkeypatch):
    # BCHK_POLAR_ML=2: every matrix layer through the GPU search; the oracle takes these
    # kernels' LLRs from enumeration / the trellis -- an independent method
    monkeypatch.setenv("BCHK_POLAR_ML", "2")
    spec = mixed_spec(layers, K, dyn, punct, seed=len(layers) * 17 + K)
    o = PolarOracle(spec, kdir)
    d = load().PolarListDecoder(spec, L, kernel_dir=kdir)
    rng = np.random.default_rng(L + K + 5)
    info = rng.integers(0, 2, (32, K)).astype(np.uint8)
    cw = o.encode(info)
    for snr in (0.0, 2.0):
        llr = awgn_llr(cw, snr, K / o.N, seed=int(snr * 10) + L + 7)
        _same(d.decode(llr), o.decode_batch(llr, L))


@pytest.mark.gpu
@pytest.mark.parametrize("layers,K,dyn,punct", CODES64, ids=["-".join(c[0]) + f"-{c[1]}" for c in CODES64])
@pytest.mark.parametrize("L", [1, 4, 8])
def test_gpu_64x64_kernel_matches_oracle(kdir, layers, K, dyn, punct, L):
    spec = mixed_spec(layers, K, dyn, punct, seed=len(layers) * 19 + K)
    o = PolarOracle(spec, kdir)
    d = load().PolarListDecoder(spec, L, kernel_dir=kdir)
    assert (d.N, d.K, d.U) == (o.N, o.K, o.U)
    rng = np.random.default_rng(L * 3 + K)
    info = rng.integers(0, 2, (16, K)).astype(np.uint8)
    cw = o.encode(info)
    np.testing.assert_array_equal(d.encode(info), cw)
    for snr in (1.0, 3.0):
        llr = awgn_llr(cw, snr, K / o.N, seed=int(snr * 10) + L)
        _same(d.decode(llr), o.decode_batch(llr, L))


@pytest.mark.gpu
@pytest.mark.parametrize("budget_ms", ["1", "20"])
def test_gpu_64x64_budgeted_launches_equal_one_launch(kdir, budget_ms, monkeypatch):
    # A decode call over the 64 x 64 kernel is a series of launches of ~budget each: codewords
    # are suspended between two search items and resumed by the next launch. Lists, metrics and
    # counts equal one unbounded launch bit for bit (and the oracle), and the call did take
    # several launches.
    layers, K, dyn, punct = CODES64[0]
    spec = mixed_spec(layers, K, dyn, punct, seed=len(layers) * 19 + K)
    o = PolarOracle(spec, kdir)
    L = 8
    rng = np.random.default_rng(61)
    info = rng.integers(0, 2, (24, K)).astype(np.uint8)
    llr = awgn_llr(o.encode(info), 2.0, K / o.N, seed=62)
    monkeypatch.setenv("BCHK_POLAR_BUDGET_MS", "0")
    one = load().PolarListDecoder(spec, L, kernel_dir=kdir)
    a = one.decode(llr)
    assert one.last_launches() == 1
    monkeypatch.setenv("BCHK_POLAR_BUDGET_MS", budget_ms)
    many = load().PolarListDecoder(spec, L, kernel_dir=kdir)
    b = many.decode(llr)
    print(f"\nbudget {budget_ms} ms: {many.last_launches()} launches")
    assert many.last_launches() > 1
    _same(b, a)
    _same(b, o.decode_batch(llr, L))
    b2 = many.decode(llr[::-1].copy())  # state of a previous call is not reused
    _same(b2, o.decode_batch(llr[::-1].copy(), L))
