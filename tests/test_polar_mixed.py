"""SC-list decoding over MIXED kernels on the GPU (csrc/polar_mixed.hip): Arikan layers and
matrix kernels (the reference's kernel files, Kernel.cpp:93-107 -- e.g. BCH-derived kernels),
whose kernel LLRs are the trellis min-sum of out/external/TrellisKernelProcessor.cpp:234-294.
Bit for bit against the C restatement (oracle/polar_oracle.c; its parity is unpinned, as
for the Arikan decoder -- SURVEY.md §8c): list counts, information vectors, codewords, f32
path metrics."""
import os

import numpy as np
import pytest

from bchk_pkg import load
from polar_lib import PolarOracle, awgn_llr


def _kernel_text(K):
    return f"{len(K)}\n" + "\n".join(" ".join(str(int(v)) for v in row) for row in K) + "\n"


def _lower_kernel(l, seed):
    """An invertible l x l kernel: unit lower-triangular with random entries below, rows
    then permuted among equal-weight classes so it is not a Kronecker power."""
    rng = np.random.default_rng(seed)
    K = np.tril(rng.integers(0, 2, (l, l)), -1).astype(np.uint8)
    np.fill_diagonal(K, 1)
    K[-1, :] = 1  # the all-ones row last, as polarising kernels have
    return K


def _bch_kernel(power, prim):
    """The reference's nested extended-BCH kernel (root bchCoder.cpp:356-389 makeMatrix):
    column 0 all ones, row 1 = x^0 shifted, row deg(g) of each growing generator
    g = lcm(M_2, ..., M_i) holds g (from column 1), the rows between hold shifts of the previous
    generator; GF(2^power) from the primitive polynomial `prim`."""
    n = (1 << power) - 1
    el, x = [], 1
    for _ in range(n):
        el.append(x)
        x <<= 1
        if x >> power:
            x ^= prim
    log = {v: k for k, v in enumerate(el)}

    def minpoly(i):
        coset, j = [], i % n
        while j not in coset:
            coset.append(j)
            j = 2 * j % n
        poly = [1]
        for j in coset:  # multiply by (x + alpha^j)
            q = [0] * (len(poly) + 1)
            for k, c in enumerate(poly):
                if c:
                    q[k] ^= el[(log[c] + j) % n]
                q[k + 1] ^= c
            poly = q
        return [int(c) for c in poly]

    def mul(a, b):
        r = [0] * (len(a) + len(b) - 1)
        for i, u in enumerate(a):
            for j, v in enumerate(b):
                r[i + j] ^= u & v
        return r

    def divides(a, b):  # b | a over GF(2)
        a = list(a)
        while len(a) >= len(b):
            if a[-1]:
                for k, c in enumerate(b):
                    a[len(a) - len(b) + k] ^= c
            a.pop()
        return not any(a)

    M = np.zeros((n + 1, n + 1), np.uint8)
    M[:, 0] = 1
    M[1, 1] = 1
    g, gold = [1], 1
    for i in range(2, (n - 1) // 2 + 1 if power != 2 else 3):
        poly = minpoly(i)
        if gold >= len(poly) and divides(g, poly):
            continue
        gnew = len(poly) + gold - 1
        M[gnew, 1:1 + gnew] = mul(poly, g)
        for cnt, j in enumerate(range(gold, gnew - 1), start=1):
            M[j + 1, cnt + 1:cnt + 1 + gold] = g[:gold]
        g, gold = list(M[gnew, 1:gnew + 1]), gnew
    return M


def _field_order(K, power, prim):
    """swapColumns' reordering (root bchCoder.cpp:478-496): column i >= 3 takes the column
    of the field element i (column j + 1 holds alpha^j)."""
    n = 1 << power
    el, x = [], 1
    for _ in range(n - 1):
        el.append(x)
        x <<= 1
        if x >> power:
            x ^= prim
    F = K.copy()
    for i in range(3, n):
        F[:, i] = K[:, el.index(i) + 1]
    return F


KERNELS = {
    "bch64f": _field_order(_bch_kernel(6, 0b1000011), 6, 0b1000011),  # exact ordered-statistics LLRs
    "bch64": _bch_kernel(6, 0b1000011),
    "bch8": _bch_kernel(3, 0b1011),
    "bch32f": _field_order(_bch_kernel(5, 0b100101), 5, 0b100101),  # trellis: 2^12 states
    "bch16": _bch_kernel(4, 0b10011),
    "k4": np.array([[1, 0, 0, 0], [1, 0, 1, 0], [1, 1, 0, 0], [1, 1, 1, 1]], np.uint8),
    "a2": np.array([[1, 0], [1, 1]], np.uint8),
    "k8": _lower_kernel(8, 3),
    "k16": _lower_kernel(16, 5),
    "k3": np.array([[1, 0, 0], [1, 1, 0], [1, 0, 1]], np.uint8),
}


@pytest.fixture(scope="module")
def kdir(tmp_path_factory):
    d = tmp_path_factory.mktemp("kernels")
    for name, K in KERNELS.items():
        (d / f"{name}.txt").write_text(_kernel_text(K))
    return str(d)


def mixed_spec(layers, K, dyn=0, punct=(), seed=0):
    """Spec text over the given layer names ("A" or a kernel file name): the U - K lowest
    indices frozen except a few swapped for variety, `dyn` of them dynamically frozen."""
    sizes = [2 if name == "A" else len(KERNELS[name]) for name in layers]
    U = int(np.prod(sizes))
    rng = np.random.default_rng(seed)
    order = list(range(U))
    for _ in range(U // 8):  # a few swaps near the boundary
        i = int(rng.integers(max(0, U - K - 4), min(U, U - K + 4)))
        j = int(rng.integers(max(0, U - K - 4), min(U, U - K + 4)))
        order[i], order[j] = order[j], order[i]
    frozen = sorted(order[:U - K])
    dynset = set(rng.choice([f for f in frozen if f >= 2], size=min(dyn, len([f for f in frozen if f >= 2])),
                            replace=False).tolist()) if dyn else set()
    names = ["A" if n == "A" else f"-{n}.txt" for n in layers]
    lines = [f"{U - len(punct)} {K} 0 {len(layers)} 0 {len(punct)}", " ".join(names)]
    if punct:
        lines.append(" ".join(str(p) for p in punct))
    for f in frozen:
        if f in dynset:
            a, b = sorted(rng.choice(f, size=2, replace=False).tolist())
            lines.append(f"3 {a} {b} {f}")
        else:
            lines.append(f"1 {f}")
    return "\n".join(lines) + "\n"


def _same(got, want):
    gc, gi, gw, gm = got
    wc, wi, ww, wm = want
    np.testing.assert_array_equal(gc, wc)
    for b in range(len(wc)):
        c = wc[b]
        np.testing.assert_array_equal(gi[b, :c], wi[b, :c], err_msg=f"info, codeword {b}")
        np.testing.assert_array_equal(gw[b, :c], ww[b, :c], err_msg=f"codeword, row {b}")
        np.testing.assert_array_equal(gm[b, :c].view(np.uint32), wm[b, :c].view(np.uint32),
                                      err_msg=f"metrics, row {b}")


def test_spec_errors_before_the_device(kdir, tmp_path):
    # matrix kernels are parsed and checked on the host, with or without a GPU
    F = load()
    (tmp_path / "sing.txt").write_text("3\n1 0 0\n1 0 0\n0 1 1\n")
    (tmp_path / "big.txt").write_text(_kernel_text(_lower_kernel(20, 1)))
    (tmp_path / "wide.txt").write_text(_kernel_text(_lower_kernel(32, 1)))
    (tmp_path / "huge.txt").write_text("70\n" + "\n".join(" ".join("1" if c <= r else "0" for c in range(70))
                                                         for r in range(70)) + "\n")
    for name, msg, n in [("sing", "singular", 3), ("wide", "GPU limit", 32), ("huge", "size", 70),
                         ("missing", "Error reading kernel file", 20)]:
        spec = f"{n} {n // 2} 0 1 0 0\n-{name}.txt\n" + "".join(f"1 {i}\n" for i in range(n - n // 2))
        with pytest.raises(F.BchkError, match=msg):
            F.PolarListDecoder(spec, 4, kernel_dir=str(tmp_path))
    with pytest.raises(F.BchkError, match="Unknown kernel"):
        F.PolarListDecoder("4 2 0 1 0 0\nB\n1 0\n1 1\n", 4)


CODES = [
    (("k4", "A"), 4, 0, ()),            # the oracle test's matrix4 code, N = 8
    (("k8", "A", "A"), 16, 2, ()),      # U = 32
    (("A", "k8", "A"), 14, 3, (5, 9)),  # punctured
    (("k16", "A"), 16, 2, ()),          # a 16 x 16 matrix kernel, U = 32
    (("A", "A", "k16"), 32, 4, ()),     # U = 64, the matrix layer innermost
    (("k3", "k4", "A"), 12, 2, ()),     # odd kernel size, U = 24
    (("bch16", "A"), 16, 2, ()),        # the reference's 16 x 16 extended-BCH kernel
    (("A", "bch8", "A"), 16, 2, (3,)),  # its 8 x 8 one, between Arikan layers
    (("bch16", "bch8"), 64, 4, ()),     # two BCH kernels, U = 128
]
# 32 x 32: the extended-BCH kernel in field-element order, through its trellis
CODES32 = [
    (("bch32f", "A"), 32, 2, ()),
    (("A", "bch32f"), 30, 2, (7,)),
]


def test_bch_kernels_are_the_nested_construction():
    # row weights / triangular shape of root bchCoder.cpp's makeMatrix output, and invertible
    for name in ("bch8", "bch16"):
        M = KERNELS[name].astype(np.int64)
        l = len(M)
        assert (M[:, 0] == 1).all() and M[-1].sum() == l
        assert all(M[r, r] == 1 and not M[r, r + 1:].any() for r in range(l))  # lower triangular
        assert abs(round(np.linalg.det(M))) % 2 == 1


@pytest.mark.gpu
@pytest.mark.parametrize("layers,K,dyn,punct", CODES, ids=["-".join(c[0]) for c in CODES])
@pytest.mark.parametrize("L", [1, 2, 4, 8, 16])
def test_gpu_mixed_matches_oracle(kdir, layers, K, dyn, punct, L):
    spec = mixed_spec(layers, K, dyn, punct, seed=len(layers) * 11 + K)
    o = PolarOracle(spec, kdir)
    d = load().PolarListDecoder(spec, L, kernel_dir=kdir)
    assert (d.N, d.K, d.U) == (o.N, o.K, o.U)
    rng = np.random.default_rng(L + K)
    info = rng.integers(0, 2, (40, K)).astype(np.uint8)
    cw = o.encode(info)
    np.testing.assert_array_equal(d.encode(info), cw)  # the host encoder over mixed layers
    for snr in (0.0, 2.0):
        llr = awgn_llr(cw, snr, K / o.N, seed=int(snr * 10) + L)
        _same(d.decode(llr), o.decode_batch(llr, L))


@pytest.mark.gpu
def test_matrix_arikan_kernel_equals_the_arikan_decoder(kdir):
    # 2x2 matrix kernels equal to Arikan's through the mixed decoder give the Arikan decoder's
    # (polar_sclist.hip) lists exactly
    from polar_lib import arikan_spec
    base = arikan_spec(6, 28, dyn=4, seed=4)
    head, kern, rest = base.split("\n", 2)
    mixed = head + "\n" + " ".join(["-a2.txt"] * 6) + "\n" + rest
    F = load()
    da, dm = F.PolarListDecoder(base, 8), F.PolarListDecoder(mixed, 8, kernel_dir=kdir)
    o = PolarOracle(base)
    info = np.random.default_rng(1).integers(0, 2, (64, 28)).astype(np.uint8)
    llr = awgn_llr(o.encode(info), 1.5, 28 / 64, seed=8)
    _same(dm.decode(llr), da.decode(llr))


def _plr_kernel(K):
    import ctypes as C

    class PK(C.Structure):
        _fields_ = [("size", C.c_int), ("arikan", C.c_int), ("K", C.c_uint8 * 4096), ("Kinv", C.c_uint8 * 4096)]

    k = PK()
    k.size, k.arikan = len(K), 0
    for i, v in enumerate(np.asarray(K, np.uint8).ravel()):
        k.K[i] = int(v)
    return k


@pytest.mark.parametrize("name", ["k3", "k4", "k8", "bch8", "k16", "bch16"])
def test_oracle_trellis_equals_coset_enumeration(name):
    """The oracle's literal trellis (TrellisKernelProcessor.cpp:69-294, used for large
    cosets) against its coset enumeration, bit for bit in float, every phase."""
    import ctypes as C
    from polar_lib import lib as plib
    L = plib()
    L.plr_minsum_llr.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    L.plr_minsum_llr.restype = C.c_float
    thr = C.c_int.in_dll(L, "plr_trellis_nfree")
    K = KERNELS[name]
    k = _plr_kernel(K)
    rng = np.random.default_rng(len(K))
    old = thr.value
    try:
        for _ in range(4):
            y = rng.normal(0, 1.5, len(K)).astype(np.float32)
            for ph in range(len(K)):
                thr.value = 64
                a = L.plr_minsum_llr(C.byref(k), ph, y.ctypes.data_as(C.c_void_p))
                thr.value = -1
                b = L.plr_minsum_llr(C.byref(k), ph, y.ctypes.data_as(C.c_void_p))
                assert np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32), (name, ph, a, b)
    finally:
        thr.value = old


@pytest.mark.gpu
@pytest.mark.parametrize("layers,K,dyn,punct", CODES, ids=["-".join(c[0]) for c in CODES])
@pytest.mark.parametrize("L", [1, 4, 8])
def test_gpu_mixed_trellis_everywhere_matches_oracle(kdir, layers, K, dyn, punct, L, monkeypatch):
    """Every matrix layer (3 x 3 up) through its trellis (BCHK_POLAR_TRELLIS=2) instead of
    the coset enumeration: same lists, bit for bit."""
    monkeypatch.setenv("BCHK_POLAR_TRELLIS", "2")
    spec = mixed_spec(layers, K, dyn, punct, seed=len(layers) * 11 + K)
    o = PolarOracle(spec, kdir)
    d = load().PolarListDecoder(spec, L, kernel_dir=kdir)
    rng = np.random.default_rng(L + K + 1)
    info = rng.integers(0, 2, (24, K)).astype(np.uint8)
    cw = o.encode(info)
    for snr in (0.0, 2.0):
        llr = awgn_llr(cw, snr, K / o.N, seed=int(snr * 10) + L + 3)
        _same(d.decode(llr), o.decode_batch(llr, L))


@pytest.mark.gpu
@pytest.mark.parametrize("layers,K,dyn,punct", CODES32, ids=["-".join(c[0]) for c in CODES32])
@pytest.mark.parametrize("L", [1, 4])
def test_gpu_mixed_32x32_kernel_matches_oracle(kdir, layers, K, dyn, punct, L):
    spec = mixed_spec(layers, K, dyn, punct, seed=len(layers) * 13 + K)
    o = PolarOracle(spec, kdir)
    d = load().PolarListDecoder(spec, L, kernel_dir=kdir)
    rng = np.random.default_rng(L + K)
    info = rng.integers(0, 2, (12, K)).astype(np.uint8)
    cw = o.encode(info)
    np.testing.assert_array_equal(d.encode(info), cw)
    for snr in (1.0, 3.0):
        llr = awgn_llr(cw, snr, K / o.N, seed=int(snr * 10) + L)
        _same(d.decode(llr), o.decode_batch(llr, L))
