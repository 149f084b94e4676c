"""Readers for the reference-generated fixtures in tests/golden/ (see oracle/make_golden.py)."""
import glob
import gzip
import os
from dataclasses import dataclass

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _open(path):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def _bits(s, n):
    if s == "-":
        return None
    assert len(s) == n
    return np.frombuffer(s.encode(), dtype=np.uint8) - ord("0")


@dataclass
class Vectors:
    name: str
    m: int
    t: int
    n: int
    k: int
    snr: float
    g: np.ndarray       # generator polynomial coefficients (low -> high)
    tx: np.ndarray      # [B, n] u8 transmitted codeword
    y: np.ndarray       # [B, n] f64 channel samples
    res: np.ndarray     # [B, n] u8 decoded word (rows with accepted == 0 are undefined)
    l0: np.ndarray      # [B] f64 path metric of res (inf when not accepted)
    decodes: np.ndarray  # [B] u64 counter deltas
    cmp: np.ndarray
    sums: np.ndarray
    accepted: np.ndarray  # [B] u8


def load_vectors(path):
    tx, y, res, l0, dec, cmp, sums, acc = [], [], [], [], [], [], [], []
    g = None
    snr = float("nan")
    with _open(path) as f:
        for line in f:
            p = line.split()
            if p[0] == "#":
                if p[1] == "code":
                    n, k, t, m = (int(v) for v in p[2:6])
                    if "snr" in p:
                        snr = float.fromhex(p[p.index("snr") + 1])
                elif p[1] == "g":
                    g = _bits(p[2], len(p[2]))
                continue
            assert p[0] == "W"
            tx.append(_bits(p[1], n))
            y.append([float.fromhex(v) for v in p[2:2 + n]])
            r = _bits(p[2 + n], n)
            res.append(r if r is not None else np.zeros(n, np.uint8))
            l0.append(float.fromhex(p[3 + n]) if p[3 + n] != "inf" else float("inf"))
            dec.append(int(p[4 + n]))
            cmp.append(int(p[5 + n]))
            sums.append(int(p[6 + n]))
            acc.append(int(p[7 + n]))
    return Vectors(os.path.basename(path), m, t, n, k, snr, g, np.array(tx, np.uint8),
                   np.array(y, np.float64), np.array(res, np.uint8), np.array(l0),
                   np.array(dec, np.uint64), np.array(cmp, np.uint64),
                   np.array(sums, np.uint64), np.array(acc, np.uint8))


def vector_files():
    return sorted(glob.glob(os.path.join(GOLD, "vectors_*.txt.gz")))


@dataclass
class AlgDec:
    name: str
    m: int
    t: int
    n: int
    words: np.ndarray    # [N, n] u8
    ok: np.ndarray       # [N] u8
    answer: np.ndarray   # [N, n] u8 (zeros where ok == 0)


def load_algdec(path):
    words, ok, ans = [], [], []
    with _open(path) as f:
        for line in f:
            p = line.split()
            if p[0] == "#":
                n, k, t = int(p[2]), int(p[3]), int(p[4])
                continue
            words.append(_bits(p[1], n))
            ok.append(int(p[2]))
            a = _bits(p[3], n)
            ans.append(a if a is not None else np.zeros(n, np.uint8))
    m = {15: 4, 31: 5, 63: 6, 255: 8}[n]
    return AlgDec(os.path.basename(path), m, t, n, np.array(words, np.uint8),
                  np.array(ok, np.uint8), np.array(ans, np.uint8))


def algdec_files():
    return sorted(glob.glob(os.path.join(GOLD, "algdec_*.txt.gz")))


def sweep_files():
    return sorted(glob.glob(os.path.join(GOLD, "sweep_*.csv")))
