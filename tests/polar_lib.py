"""Polar-code helpers for the SC-list tests: the ctypes binding to the C restatement of the
vendored SC-list decoder (oracle/build/libpolar_oracle.so -- the CHECKER only), a code
specification builder in the reference's spec format (out/external/MixedKernelEncoder.cpp:
7-98), and an AWGN channel producing the decoder's LLRs.

Only tests/ import this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "oracle", "build", "libpolar_oracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "oracle"], check=True)
        L = C.CDLL(LIB)
        vp = C.c_void_p
        L.plr_create.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]
        L.plr_create.restype = vp
        L.plr_destroy.argtypes = [vp]
        L.plr_dims.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.plr_encode.argtypes = [vp, vp, vp]
        L.plr_encode_unshortened.argtypes = [vp, vp, vp]
        L.plr_extract_info.argtypes = [vp, vp, vp]
        L.plr_decode.argtypes = [vp, C.c_int, vp, vp, vp, vp]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class PolarOracle:
    """One code from its specification text; SC-list decode with list size L."""

    def __init__(self, spec, kernel_dir=None):
        msg = C.create_string_buffer(512)
        self.h = lib().plr_create(spec.encode(), (kernel_dir or "").encode(), msg, 512)
        if not self.h:
            raise ValueError(msg.value.decode())
        n, k, u = C.c_int(), C.c_int(), C.c_int()
        lib().plr_dims(self.h, C.byref(n), C.byref(k), C.byref(u))
        self.N, self.K, self.U = n.value, k.value, u.value

    def __del__(self):
        if getattr(self, "h", None):
            lib().plr_destroy(self.h)
            self.h = None

    def encode(self, info):
        info = np.ascontiguousarray(info, np.uint8)
        out = np.zeros((info.shape[0], self.N), np.uint8)
        for b in range(info.shape[0]):
            lib().plr_encode(self.h, _p(info[b]), _p(out[b]))
        return out

    def encode_unshortened(self, info):
        info = np.ascontiguousarray(info, np.uint8)
        out = np.zeros(self.U, np.uint8)
        lib().plr_encode_unshortened(self.h, _p(info), _p(out))
        return out

    def extract_info(self, ucw):
        ucw = np.ascontiguousarray(ucw, np.uint8)
        out = np.zeros(self.K, np.uint8)
        lib().plr_extract_info(self.h, _p(ucw), _p(out))
        return out

    def decode(self, llr, L):
        """llr [N] float32 -> (count, info [L][K], codewords [L][N], metrics [L])."""
        llr = np.ascontiguousarray(llr, np.float32)
        info = np.zeros((L, self.K), np.uint8)
        cw = np.zeros((L, self.N), np.uint8)
        met = np.zeros(L, np.float32)
        n = lib().plr_decode(self.h, L, _p(llr), _p(info), _p(cw), _p(met))
        assert n >= 1
        return n, info, cw, met

    def decode_batch(self, llrs, L, threads=None):
        """Rows decoded independently, over host threads (plr_decode keeps no global state;
        ctypes releases the GIL during the call)."""
        from concurrent.futures import ThreadPoolExecutor

        from oracle_lib import host_threads
        B = llrs.shape[0]
        cnt = np.zeros(B, np.int32)
        info = np.zeros((B, L, self.K), np.uint8)
        cw = np.zeros((B, L, self.N), np.uint8)
        met = np.zeros((B, L), np.float32)

        def one(b):
            cnt[b], info[b], cw[b], met[b] = self.decode(llrs[b], L)

        with ThreadPoolExecutor(max_workers=min(threads or host_threads(), max(1, B))) as ex:
            list(ex.map(one, range(B)))
        return cnt, info, cw, met


def pw_order(n):
    """Polarization-weight reliability of the 2^n bit channels (index bits weighted by
    2^(b/4)); least reliable first. A standard construction, used here only to pick
    frozen sets for test and benchmark codes."""
    U = 1 << n
    w = [sum(((i >> b) & 1) * 2.0 ** (b / 4.0) for b in range(n)) for i in range(U)]
    return sorted(range(U), key=lambda i: (w[i], i))


def arikan_spec(n, K, dyn=0, punct=(), seed=0):
    """Spec text of a length-2^n Arikan polar code of dimension K: the U - K least reliable
    symbols frozen (`dyn` of them dynamically, each as the XOR of two earlier symbols),
    `punct` punctured positions (N = U - len(punct))."""
    U = 1 << n
    rng = np.random.default_rng(seed)
    frozen = sorted(pw_order(n)[:U - K])
    dynset = set(rng.choice([f for f in frozen if f >= 2], size=min(dyn, len(frozen)),
                            replace=False).tolist()) if dyn else set()
    lines = [f"{U - len(punct)} {K} 0 {n} 0 {len(punct)}", " ".join(["A"] * n)]
    if punct:
        lines.append(" ".join(str(p) for p in punct))
    for f in frozen:
        if f in dynset:
            a, b = sorted(rng.choice(f, size=2, replace=False).tolist())
            lines.append(f"3 {a} {b} {f}")
        else:
            lines.append(f"1 {f}")
    return "\n".join(lines) + "\n"


def awgn_llr(cw, snr_db, rate, seed):
    """BPSK with bit 1 -> +1 (headers/external/Modem.h:64) over AWGN at Eb/N0 snr_db, LLR
    -2y/sigma^2 (Modem.h:78): positive favours 0, as the decoder reads it."""
    rng = np.random.default_rng(seed)
    sigma = np.sqrt(1.0 / (2.0 * rate * 10.0 ** (snr_db / 10.0)))
    x = np.where(cw != 0, 1.0, -1.0)
    y = x + sigma * rng.standard_normal(cw.shape)
    return (-2.0 * y / sigma ** 2).astype(np.float32)
