"""Syndrome decoding table (csrc/bchk_syndtab.h) against the reference decoder.

The search kernels decode a test pattern (n <= 63) by looking its normalised syndrome up
in a table of the weight <= t coset leaders instead of running Berlekamp-Massey + Chien.
That is the reference's Decoder::decode (src/Decoder.cpp:298-321) exactly when, for every
syndrome, the lookup succeeds iff the decoder does and returns the positions it flips.
Checked here on the host (bchk_syndrome_table_query, no GPU) against the C oracle's
restatement of Decoder::decode (orc_alg_decode, pinned to the reference's own decoder
tables in test_oracle.py) on words at every distance from the code, and exhaustively
against the definition (syndromes of the weight 1..t patterns) for the small codes.
"""
import itertools

import numpy as np
import pytest

from bchk_pkg import load
from oracle_lib import Oracle


def odd_syndromes(o, words):
    """[B][t] odd syndromes S_1, S_3, ..., S_{2t-1} of binary words (Decoder.cpp:184-207)."""
    n, t = o.n, o.t
    alog = np.array(o.code.alog[:n], np.uint32)
    pos = np.arange(n)
    syn = np.zeros((words.shape[0], t), np.uint32)
    for q in range(t):
        colq = alog[((2 * q + 1) * pos) % n]
        syn[:, q] = np.bitwise_xor.reduce(np.where(words != 0, colq[None, :], 0), axis=1)
    return syn


def mask_of(rows):
    return (rows.astype(np.uint64) << np.arange(rows.shape[1], dtype=np.uint64)).sum(
        axis=1, dtype=np.uint64)


@pytest.mark.parametrize("m,t", [(3, 1), (4, 2), (4, 3), (5, 2), (5, 3)])
def test_table_exhaustive_small(m, t):
    """Every syndrome tuple: decodes iff some pattern of weight 1..t has it, to that one."""
    o = Oracle(m, t)
    n = o.n
    pats = []
    for w in range(1, t + 1):
        for c in itertools.combinations(range(n), w):
            row = np.zeros(n, np.uint8)
            row[list(c)] = 1
            pats.append(row)
    pats = np.array(pats)
    leader = {tuple(s): int(mk) for s, mk in zip(odd_syndromes(o, pats), mask_of(pats))}
    assert len(leader) == len(pats)  # unique coset leaders (d = 2t + 1)
    allsyn = np.array(list(itertools.product(range(1 << m), repeat=t)), np.uint32)
    ok, err = load().syndrome_table_query(m, t, allsyn)
    want = np.array([tuple(s) in leader for s in allsyn])
    np.testing.assert_array_equal(ok, want)
    got = {tuple(s): int(e) for s, e, k in zip(allsyn, err, ok) if k}
    assert got == leader


@pytest.mark.parametrize("m,t,count", [(4, 2, 3000), (5, 3, 3000), (5, 7, 600), (6, 6, 2500),
                                       (6, 4, 1500), (6, 2, 800)])
def test_table_matches_decoder(m, t, count):
    """table(syndrome(word)) == the reference decoder (success and corrected word), on
    words at every distance from the code (a codeword's own zero syndrome included)."""
    o = Oracle(m, t)
    n, k = o.n, o.k
    rng = np.random.default_rng(1000 * m + t)
    words = np.zeros((count, n), np.uint8)
    for b in range(count):
        info = rng.integers(0, 2, k, dtype=np.uint8)
        cw = np.zeros(n, np.uint8)
        for i in np.nonzero(info)[0]:
            cw[i:i + len(o.g)] ^= o.g
        w = int(rng.integers(0, t + 4)) if b % 5 else int(rng.integers(0, n))
        cw[rng.choice(n, size=w, replace=False)] ^= 1
        words[b] = cw
    ok, err = load().syndrome_table_query(m, t, odd_syndromes(o, words))
    ref = [o.alg_decode(wd) for wd in words]
    np.testing.assert_array_equal(ok, [r[0] for r in ref])
    for b in np.flatnonzero(ok):
        np.testing.assert_array_equal(mask_of((ref[b][1] ^ words[b])[None, :])[0], err[b])
    assert 0 < ok.sum() < count


def test_table_size_and_probes():
    keys, nbytes, probe = load().syndrome_table_info(6, 6)
    # one key per (cyclic shift x Frobenius) orbit of the 75.6 M weight <= 6 patterns of
    # length 63: ~75.6 M / (63 * 6), plus orbits smaller than 378 and raw-region keys
    assert 195_000 < keys < 215_000
    # 8-B slots in 64-B buckets at load <= 1/2: 4 MiB, the size of one XCD's L2
    assert nbytes <= 4 << 20 and 1 <= probe <= 16


def test_table_rejects_infeasible():
    with pytest.raises(load().BchkError):
        load().syndrome_table_query(8, 15, np.zeros((1, 15), np.uint32))
