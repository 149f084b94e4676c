"""The GPU SC-list decoder (csrc/polar_sclist.hip, bchk_polar_* C ABI) against the C
restatement of the vendored decoder (oracle/polar_oracle.c): list size, information
vectors, codewords, path metrics (f32 bits) and list counts, bit for bit.

Codes are length-2^n Arikan polar codes in the reference's specification format
(out/external/MixedKernelEncoder.cpp:7-98) with static and dynamic frozen symbols and
puncturing; LLRs come from BPSK over AWGN as in the reference's simulator
(headers/external/Modem.h:64-78). The oracle's own parity is unpinned (no fixtures ship
with the vendored library) -- see tests/test_polar_oracle.py.
"""
import numpy as np
import pytest

from bchk_pkg import load
from polar_lib import PolarOracle, arikan_spec, awgn_llr

_dec = {}


def gpu_decoder(spec, L):
    key = (spec, L)
    if key not in _dec:
        _dec[key] = load().PolarListDecoder(spec, L)
    return _dec[key]


def workload(n, K, dyn, punct, snr, B, seed):
    spec = arikan_spec(n, K, dyn=dyn, punct=punct, seed=seed)
    o = PolarOracle(spec)
    info = np.random.default_rng(seed).integers(0, 2, (B, K)).astype(np.uint8)
    llr = awgn_llr(o.encode(info), snr, K / o.N, seed=seed + 1)
    return spec, o, info, llr


def assert_same(got, want):
    gc, gi, gw, gm = got
    wc, wi, ww, wm = want
    np.testing.assert_array_equal(gc, wc)
    for b in range(len(wc)):
        c = wc[b]
        np.testing.assert_array_equal(gi[b, :c], wi[b, :c], err_msg=f"info, codeword {b}")
        np.testing.assert_array_equal(gw[b, :c], ww[b, :c], err_msg=f"codeword, row {b}")
        np.testing.assert_array_equal(gm[b, :c].view(np.uint32), wm[b, :c].view(np.uint32),
                                      err_msg=f"metrics, row {b}")


# ---------------------------------------------------------------- host side (no GPU needed)

def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(load().BchkError, match="device|HIP"):
        load().PolarListDecoder(arikan_spec(5, 16), 4)


@pytest.mark.parametrize("spec,L,msg", [
    (arikan_spec(5, 16), 0, "list size"),
    (arikan_spec(5, 16), 33, "list size"),
    (arikan_spec(11, 1024), 32, "LDS"),
    ("10 5 0 3 0 0\nA A A\n1 0\n1 1\n1 2\n", 4, "mismatch|length"),
    ("8 4 0 2 0 0\n-k4.txt A\n1 0\n1 1\n1 2\n1 4\n", 4, "Error reading kernel file"),
    ("garbage", 4, "header"),
])
def test_bad_codes_are_rejected_before_touching_the_device(spec, L, msg):
    with pytest.raises(load().BchkError, match=msg):
        load().PolarListDecoder(spec, L)


# ---------------------------------------------------------------- GPU parity

CODES = [  # n, K, dynamic constraints, punctured positions
    (3, 4, 0, ()),
    (4, 8, 2, ()),
    (5, 16, 3, ()),
    (6, 32, 5, (1, 7)),
    (7, 64, 8, ()),
    (8, 128, 12, (0, 3, 17, 40)),
    (9, 256, 10, ()),
    (10, 512, 20, ()),
]


@pytest.mark.gpu
@pytest.mark.parametrize("n,K,dyn,punct", CODES)
@pytest.mark.parametrize("L", [1, 2, 4, 8, 16, 32])
def test_gpu_sclist_matches_oracle(n, K, dyn, punct, L):
    if (1 << n) * L > 8192 and n >= 10 and L > 16:
        pytest.skip("exceeds the LDS budget")
    B = 48 if n >= 9 else 96
    spec, o, info, llr = workload(n, K, dyn, punct, 1.0 + 0.25 * n, B, seed=n * 7 + L)
    assert_same(gpu_decoder(spec, L).decode(llr), o.decode_batch(llr, L))


@pytest.mark.gpu
@pytest.mark.parametrize("snr", [-2.0, 0.0, 2.0, 4.0, 8.0])
def test_gpu_sclist_matches_oracle_across_snr(snr):
    spec, o, info, llr = workload(8, 128, 6, (), snr, 128, seed=int(snr * 10) + 50)
    for L in (4, 8):
        assert_same(gpu_decoder(spec, L).decode(llr), o.decode_batch(llr, L))


@pytest.mark.gpu
def test_gpu_sclist_ties_and_zeros():
    """Quantised LLRs produce equal path metrics (the (score, index) ordering decides) and
    zero LLRs (hard decision 0, no penalty)."""
    spec, o, info, llr = workload(7, 64, 4, (), 1.0, 96, seed=77)
    q = np.round(llr / 4.0).astype(np.float32)
    assert_same(gpu_decoder(spec, 8).decode(q), o.decode_batch(q, 8))


@pytest.mark.gpu
def test_gpu_sclist_small_codes_full_list():
    """A list as large as the code keeps every codeword (count = 2^K)."""
    for n, K in ((3, 3), (4, 5)):
        spec, o, info, llr = workload(n, K, 0, (), 0.0, 40, seed=n)
        got = gpu_decoder(spec, 1 << K).decode(llr)
        assert np.all(got[0] == 1 << K)
        assert_same(got, o.decode_batch(llr, 1 << K))


@pytest.mark.gpu
def test_gpu_encoder_matches_oracle():
    for n, K, dyn, punct in CODES:
        spec = arikan_spec(n, K, dyn=dyn, punct=punct, seed=n)
        o = PolarOracle(spec)
        info = np.random.default_rng(n).integers(0, 2, (30, K)).astype(np.uint8)
        np.testing.assert_array_equal(gpu_decoder(spec, 1).encode(info), o.encode(info))


@pytest.mark.gpu
def test_gpu_sclist_large_batch_noiseless_and_sampled_parity():
    """A batch far larger than the persistent grid: noiseless rows decode to themselves at
    metric 0; a sample of noisy rows matches the oracle."""
    spec, o, info, llr = workload(10, 512, 16, (), 2.5, 20000, seed=5)
    d = gpu_decoder(spec, 8)
    cw = o.encode(info)
    clean = np.where(cw != 0, -6.0, 6.0).astype(np.float32)
    cnt, inf, c, met = d.decode(clean)
    np.testing.assert_array_equal(inf[:, 0], info)
    np.testing.assert_array_equal(c[:, 0], cw)
    assert np.all(met[:, 0] == 0.0) and np.all(cnt == 8)
    got = d.decode(llr)
    idx = np.random.default_rng(1).choice(len(llr), 400, replace=False)
    want = o.decode_batch(llr[idx], 8)
    assert_same(tuple(g[idx] for g in got), want)


@pytest.mark.gpu
def test_gpu_sclist_device_entry_point():
    import torch
    spec, o, info, llr = workload(8, 128, 6, (7,), 2.0, 300, seed=9)
    d = gpu_decoder(spec, 4)
    dev = torch.device("cuda:0")
    t_llr = torch.from_numpy(llr).to(dev)
    t_info = torch.zeros((300, 4, o.K), dtype=torch.uint8, device=dev)
    t_cw = torch.zeros((300, 4, o.N), dtype=torch.uint8, device=dev)
    t_met = torch.zeros((300, 4), dtype=torch.float32, device=dev)
    t_cnt = torch.zeros(300, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    d.decode_device(t_llr.data_ptr(), 300, t_info.data_ptr(), t_cw.data_ptr(), t_met.data_ptr(),
                    t_cnt.data_ptr())
    d.sync()
    got = (t_cnt.cpu().numpy(), t_info.cpu().numpy(), t_cw.cpu().numpy(), t_met.cpu().numpy())
    assert_same(got, o.decode_batch(llr, 4))
