"""BCH polar-kernel construction and the column-permutation search:
root bchCoder.cpp:356-389 (makeMatrix), :478-496 (swapColumns' field-element order),
:541-699 (randomSwapColumns) scored by CTrellisKernelProcessor's operation counts
(out/external/TrellisKernelProcessor.cpp:69-294).

The checker is oracle/kernel_oracle.c, which builds and walks the reference's trellis state
by state; its LLRs are pinned here to an independent coset enumeration (the min-sum the
trellis computes), its kernel to the restatement in test_polar_mixed.py. The operation
counts themselves are parity unpinned: the vendored library cannot be built here and the
SectionedTrellisKernelProcessor randomSwapColumns names is absent from the reference.
The GPU (csrc/kernel_search.hip, closed form from the minimum-span structure) must match the
oracle's counts exactly."""
import ctypes as C
import itertools
import os
import subprocess

import numpy as np
import pytest

from bchk_pkg import REPO, load
from test_polar_mixed import _bch_kernel

PRIM = {2: 0b111, 3: 0b1011, 4: 0b10011, 5: 0b100101}
_klib = None


def klib():
    global _klib
    if _klib is None:
        path = os.path.join(REPO, "oracle", "build", "libkernel_oracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "oracle"], check=True)
        L = C.CDLL(path)
        vp, u64p = C.c_void_p, C.POINTER(C.c_uint64)
        L.kor_make_ebch.argtypes = [C.c_int, vp]
        L.kor_field_order.argtypes = [C.c_int, vp, vp]
        L.kor_trellis_counts.argtypes = [vp, C.c_int, vp, u64p, u64p, vp]
        L.kor_lu_perm.argtypes = [C.c_int, C.c_uint64, vp]
        L.kor_random_codes.argtypes = [C.c_int, C.c_size_t, u64p, vp]
        L.kor_column_search.argtypes = [C.c_int, vp, vp, vp, C.c_size_t, vp, vp, u64p, u64p]
        L.kor_column_search.restype = C.c_long
        _klib = L
    return _klib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def o_ebch(power):
    n = 1 << power
    K = np.zeros((n, n), np.uint8)
    assert klib().kor_make_ebch(power, _p(K)) == 0
    return K


def o_field(power, K):
    out = np.zeros_like(K)
    klib().kor_field_order(power, _p(np.ascontiguousarray(K)), _p(out))
    return out


def o_counts(K, y, want_llr=False):
    K = np.ascontiguousarray(K, np.uint8)
    y = np.ascontiguousarray(y, np.float32)
    s, c = C.c_uint64(), C.c_uint64()
    llr = np.zeros(len(K))
    assert klib().kor_trellis_counts(_p(K), len(K), _p(y), C.byref(s), C.byref(c),
                                     _p(llr) if want_llr else None) == 0
    return (s.value, c.value, llr) if want_llr else (s.value, c.value)


def o_perm(m, code):
    perm = np.zeros(64, np.uint32)
    klib().kor_lu_perm(m, code, _p(perm))
    return perm[:1 << m]


def o_random_codes(m, count, state):
    codes = np.zeros(count, np.uint64)
    st = C.c_uint64(state)
    klib().kor_random_codes(m, count, C.byref(st), _p(codes))
    return codes, st.value


def o_search(m, K, y, codes):
    n = 1 << m
    best = np.zeros((n, n), np.uint8)
    perm = np.zeros(n, np.uint32)
    s, c = C.c_uint64(), C.c_uint64()
    codes = np.ascontiguousarray(codes, np.uint64)
    i = klib().kor_column_search(m, _p(np.ascontiguousarray(K, np.uint8)), _p(np.ascontiguousarray(y, np.float32)),
                                 _p(codes), len(codes), _p(best), _p(perm), C.byref(s), C.byref(c))
    return dict(index=i, best=best, perm=perm, sum=s.value, cmp=c.value)


def coset_llrs(K, y):
    """min-sum LLR of every kernel input with zero known inputs, by enumerating the coset
    of rows phase+1.. (what the trellis computes: correlation discrepancy, Y < 0 -> 1)."""
    l = len(K)
    hd = (np.asarray(y) < 0).astype(np.uint8)
    a = np.abs(np.asarray(y, np.float64))
    out = []
    for ph in range(l):
        rows = K[ph + 1:]
        best = [np.inf, np.inf]
        for b in (0, 1):
            for bits in itertools.product((0, 1), repeat=l - 1 - ph):
                c = (K[ph] * b).astype(np.uint8)
                for bb, r in zip(bits, rows):
                    if bb:
                        c = c ^ r
                best[b] = min(best[b], a[c != hd].sum())
        out.append(best[1] - best[0])
    return np.array(out)


def rand_invertible(l, rng):
    while True:
        K = rng.integers(0, 2, (l, l)).astype(np.uint8)
        if np.linalg.matrix_rank(K.astype(float)) < l:  # a quick real-rank filter
            continue
        rows = [int("".join(str(v) for v in r[::-1]), 2) for r in K]
        basis = []
        for v in rows:
            for b in basis:
                v = min(v, v ^ b)
            if v:
                basis.append(v)
                basis.sort(reverse=True)
        if len(basis) == l:
            return K


def llrs_like_reference(l, seed):
    """(rand() % 10) - 5 per position (root bchCoder.cpp:563-565), from a seeded generator."""
    return (np.random.default_rng(seed).integers(0, 10, l) - 5).astype(np.float32)


# ---------------------------------------------------------------- oracle (CPU)

@pytest.mark.parametrize("power", [2, 3, 4, 5])
def test_oracle_ebch_matches_restatement(power):
    assert np.array_equal(o_ebch(power), _bch_kernel(power, PRIM[power]))


@pytest.mark.parametrize("power", [2, 3, 4, 5])
def test_kernel_construction_host_matches_oracle(power):
    bchk = load()
    K = bchk.kernel_ebch(power)
    assert np.array_equal(K, o_ebch(power))
    assert np.array_equal(bchk.kernel_field_order(power, K), o_field(power, K))


def test_field_order_is_a_column_permutation():
    for power in (3, 4, 5):
        K = o_ebch(power)
        F = o_field(power, K)
        cols = {K[:, j].tobytes() for j in range(len(K))}
        assert {F[:, j].tobytes() for j in range(len(K))} == cols
        assert np.array_equal(F[:, :3], K[:, :3])


@pytest.mark.parametrize("power", [2, 3, 4])
def test_oracle_trellis_llrs_are_the_coset_min_sum(power):
    K = o_ebch(power)
    for seed in range(3):
        y = llrs_like_reference(len(K), seed)
        _, _, llr = o_counts(K, y, want_llr=True)
        assert np.allclose(llr, coset_llrs(K, y))
        Fk = o_field(power, K)
        _, _, llr = o_counts(Fk, y, want_llr=True)
        assert np.allclose(llr, coset_llrs(Fk, y))


@pytest.mark.parametrize("l", [3, 5, 8, 10])
def test_oracle_trellis_llrs_random_kernels(l):
    rng = np.random.default_rng(l)
    for _ in range(3):
        K = rand_invertible(l, rng)
        y = rng.normal(0, 2, l).astype(np.float32)
        _, _, llr = o_counts(K, y, want_llr=True)
        assert np.allclose(llr, coset_llrs(K, y))


def test_oracle_counts_closed_form_identity():
    """Cmp counts the valid edges (independent of the LLRs); with every column of every
    phase's code non-zero, each depth sends half its edges against the hard decision."""
    K = o_ebch(4)
    a = o_counts(K, llrs_like_reference(16, 1))
    b = o_counts(K, -llrs_like_reference(16, 1))
    assert a[1] == b[1]
    assert 2 * a[0] == a[1]


@pytest.mark.parametrize("m", [2, 3, 4])
def test_lu_maps_are_distinct_linear_bijections(m):
    seen = set()
    for code in range(1 << (m * (m - 1))):
        p = o_perm(m, code)
        assert sorted(p.tolist()) == list(range(1 << m)) and p[0] == 0
        for a in range(1 << m):  # linear: p[a ^ b] = p[a] ^ p[b]
            for b in range(1 << m):
                assert p[a ^ b] == p[a] ^ p[b]
        seen.add(p.tobytes())
    assert len(seen) == 1 << (m * (m - 1))  # L.U decompositions are unique


def test_random_codes_follow_the_reference_engine():
    """Bits of candidate codes are uniform_int_distribution<unsigned short>(0, 1) draws on
    minstd_rand0 (seed 1): the first draws of that stream are the reference's first
    information bits, whose golden values the GPU parity tests already pin; here, the
    engine restatement's state after k draws equals 16807^k mod (2^31 - 1) when no
    rejection occurs, and draws split evenly."""
    codes, st = o_random_codes(3, 4000, 1)
    bits = np.array([(int(c) >> d) & 1 for c in codes for d in range(6)])
    assert abs(bits.mean() - 0.5) < 0.02
    c1, s1 = o_random_codes(3, 1, 1)
    assert s1 == pow(16807, 6, 2147483647)
    c2, _ = o_random_codes(3, 1, s1)
    assert c2[0] == codes[1] and c1[0] == codes[0]


def test_oracle_search_accepts_strict_improvements_in_order():
    K = o_field(3, o_ebch(3))
    y = llrs_like_reference(8, 7)
    codes = np.arange(1 << 6, dtype=np.uint64)
    r = o_search(3, K, y, codes)
    costs = [o_counts(K[:, o_perm(3, int(c))], y) for c in codes]
    ms = mc = None
    bi = -1
    for i, (s, c) in enumerate(costs):
        if ms is None or (s < ms and c < mc):
            ms, mc, bi = s, c, i
    assert r["index"] == bi and (r["sum"], r["cmp"]) == (ms, mc)
    assert np.array_equal(r["best"], K[:, r["perm"]])


# ---------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("l", [2, 3, 5, 8, 12, 16, 24, 32])
def test_gpu_trellis_cost_matches_oracle_random_kernels(l):
    bchk = load()
    rng = np.random.default_rng(100 + l)
    for it in range(4 if l < 24 else 2):
        K = rand_invertible(l, rng)
        y = llrs_like_reference(l, it)
        assert bchk.kernel_trellis_cost(K, y) == o_counts(K, y)


@pytest.mark.gpu
@pytest.mark.parametrize("power", [2, 3, 4, 5])
def test_gpu_trellis_cost_matches_oracle_ebch(power):
    bchk = load()
    K = bchk.kernel_ebch(power)
    F = bchk.kernel_field_order(power, K)
    for seed in range(2):
        y = llrs_like_reference(1 << power, seed)
        assert bchk.kernel_trellis_cost(K, y) == o_counts(K, y)
        assert bchk.kernel_trellis_cost(F, y) == o_counts(F, y)


@pytest.mark.gpu
@pytest.mark.parametrize("power", [2, 3, 4])
def test_gpu_column_costs_match_oracle_every_candidate(power):
    bchk = load()
    F = bchk.kernel_field_order(power, bchk.kernel_ebch(power))
    y = llrs_like_reference(1 << power, 3)
    s, c = bchk.kernel_column_costs(power, F, y)
    n = 1 << (power * (power - 1))
    idx = range(n) if n <= 64 else np.random.default_rng(0).choice(n, 64, replace=False)
    for code in idx:
        assert (int(s[code]), int(c[code])) == o_counts(F[:, o_perm(power, int(code))], y)


@pytest.mark.gpu
def test_gpu_column_costs_32x32_sampled():
    bchk = load()
    F = bchk.kernel_field_order(5, bchk.kernel_ebch(5))
    y = llrs_like_reference(32, 11)
    s, c = bchk.kernel_column_costs(5, F, y)
    assert len(s) == 1 << 20 and s.min() > 0
    for code in np.random.default_rng(5).choice(1 << 20, 6, replace=False):
        assert (int(s[code]), int(c[code])) == o_counts(F[:, o_perm(5, int(code))], y)


@pytest.mark.gpu
@pytest.mark.parametrize("power", [3, 4])
def test_gpu_exhaustive_search_matches_oracle(power):
    bchk = load()
    F = bchk.kernel_field_order(power, bchk.kernel_ebch(power))
    y = llrs_like_reference(1 << power, 5)
    r = bchk.kernel_column_search(power, F, y, mode=bchk.KSEARCH_EXHAUSTIVE)
    codes = np.arange(1 << (power * (power - 1)), dtype=np.uint64)
    o = o_search(power, F, y, codes)
    assert (r["index"], r["sum"], r["cmp"]) == (o["index"], o["sum"], o["cmp"])
    assert np.array_equal(r["perm"], o["perm"]) and np.array_equal(r["best"], o["best"])
    assert bchk.kernel_trellis_cost(r["best"], y) == (r["sum"], r["cmp"])


@pytest.mark.gpu
@pytest.mark.parametrize("power,count", [(3, 500), (4, 3000), (5, 200)])
def test_gpu_random_search_matches_oracle(power, count):
    """mode RANDOM replays randomSwapColumns' draws: same candidates, same acceptance, same
    engine state afterwards."""
    bchk = load()
    F = bchk.kernel_field_order(power, bchk.kernel_ebch(power))
    y = llrs_like_reference(1 << power, 9)
    r = bchk.kernel_column_search(power, F, y, mode=bchk.KSEARCH_RANDOM, count=count, rng_state=12345)
    codes, st = o_random_codes(power, count, 12345)
    o = o_search(power, F, y, codes)
    assert r["rng_state"] == st
    assert (r["index"], r["sum"], r["cmp"]) == (o["index"], o["sum"], o["cmp"])
    assert np.array_equal(r["best"], o["best"])


@pytest.mark.gpu
def test_gpu_search_rejects_singular_kernel():
    bchk = load()
    K = np.eye(8, dtype=np.uint8)
    K[3] = K[2]
    with pytest.raises(bchk.BchkError):
        bchk.kernel_trellis_cost(K, np.ones(8, np.float32))
