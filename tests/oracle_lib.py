"""ctypes binding to the C oracle (oracle/build/liboracle.so) -- the CHECKER only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "oracle", "build", "liboracle.so")

ORC_MAXN = 255
ORC_MAXT = 32


class OrcCode(C.Structure):
    _fields_ = [("m", C.c_int), ("n", C.c_int), ("t", C.c_int), ("k", C.c_int),
                ("gsize", C.c_int), ("alog", C.c_uint * (ORC_MAXN + 1)),
                ("log_", C.c_int * (ORC_MAXN + 2)), ("g", C.c_ubyte * (ORC_MAXN + 1))]


class OrcStats(C.Structure):
    _fields_ = [("decodes", C.c_uint64), ("cmp", C.c_uint64), ("sum", C.c_uint64),
                ("iters", C.c_uint64), ("jsteps", C.c_uint64), ("improvements", C.c_uint64),
                ("accepted", C.c_int), ("returned", C.c_int)]


_lib = None


def host_threads():
    """Checker threads: this process's CPU affinity, capped by the job share a GPU box
    exports (OMP_NUM_THREADS; os.cpu_count() there is the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(share))) if share.isdigit() and int(share) > 0 else max(1, n)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "oracle"],
                           check=True)
        L = C.CDLL(LIB)
        P = C.POINTER
        L.orc_code_init.argtypes = [P(OrcCode), C.c_int, C.c_int]
        L.orc_alg_decode.argtypes = [P(OrcCode), C.c_void_p, C.c_void_p]
        L.orc_alg_decode_bm.argtypes = [P(OrcCode), C.c_void_p, C.c_void_p]
        L.orc_kaneko_decode.argtypes = [P(OrcCode), C.c_double, C.c_int, C.c_void_p,
                                        C.c_void_p, P(C.c_double), P(OrcStats)]
        L.orc_kaneko_batch.argtypes = [P(OrcCode), C.c_double, C.c_int, C.c_void_p, C.c_long,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_sweep.argtypes = [P(OrcCode), C.c_double, C.c_int, C.c_long, C.c_long,
                                C.c_double, C.c_uint64, C.c_char_p, C.c_long]
        L.orc_sweep.restype = C.c_long
        L.orc_sigma.argtypes = [P(OrcCode), C.c_double]
        L.orc_sigma.restype = C.c_double
        L.orc_rng_seed.argtypes = [C.c_void_p, C.c_uint64]
        L.orc_gen_info.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.orc_encode.argtypes = [P(OrcCode), C.c_void_p, C.c_void_p]
        L.orc_add_noise.argtypes = [C.c_void_p, C.c_double, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_stream_draws.argtypes = [P(OrcCode), C.POINTER(C.c_uint64), C.c_long, C.c_double]
        L.orc_stream_draws.restype = C.c_uint64
        L.orc_sweep_block.argtypes = [P(OrcCode), C.c_double, C.c_int, C.c_double, C.POINTER(C.c_uint64),
                                      C.c_long, C.c_long, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p]
        L.orc_sweep_range.argtypes = [P(OrcCode), C.c_double, C.c_int, C.c_double, C.POINTER(C.c_uint64),
                                      C.c_uint64, C.c_long, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p]
        L.orc_sweep_range.restype = C.c_long
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    """One BCH(n, k) code: GF tables, g(x), and the reference-semantics routines."""

    def __init__(self, m, t):
        self.code = OrcCode()
        if lib().orc_code_init(C.byref(self.code), m, t) != 0:
            raise ValueError(f"invalid code m={m} t={t}")
        self.m, self.t, self.n, self.k = m, t, self.code.n, self.code.k
        self.g = np.array(self.code.g[: self.code.gsize], np.uint8)

    def sigma(self, snr_db):
        return lib().orc_sigma(C.byref(self.code), snr_db)

    def s2(self, decoder_snr_db=0.5):
        # pow(sd, 2) as src/KanekoKernelProcessor.cpp:337 (glibc pow via ctypes-free math)
        import math
        return math.pow(self.sigma(decoder_snr_db), 2)

    def alg_decode(self, word, bm=False):
        word = np.ascontiguousarray(word, np.uint8)
        ans = np.zeros(self.n, np.uint8)
        f = lib().orc_alg_decode_bm if bm else lib().orc_alg_decode
        ok = f(C.byref(self.code), _p(word), _p(ans))
        return bool(ok), ans

    def kaneko(self, y, J=-1, s2=None):
        y = np.ascontiguousarray(y, np.float64)
        res = np.full(self.n, 0xFF, np.uint8)
        l0 = C.c_double()
        st = OrcStats()
        lib().orc_kaneko_decode(C.byref(self.code), self.s2() if s2 is None else s2, J,
                                _p(y), _p(res), C.byref(l0), C.byref(st))
        return res, l0.value, st

    def kaneko_batch(self, Y, J=-1, threads=None):
        """Rows of Y decoded independently (orc_kaneko_batch, POSIX threads): res (0xFF rows
        where nothing was accepted), l0, stats [B][6] (decodes, cmp, sum, iters, jsteps,
        improvements), accepted."""
        Y = np.ascontiguousarray(Y, np.float64)
        B = Y.shape[0]
        res = np.full((B, self.n), 0xFF, np.uint8)
        l0 = np.zeros(B)
        stats = np.zeros((B, 6), np.uint64)
        acc = np.zeros(B, np.uint8)
        if B:
            lib().orc_kaneko_batch(C.byref(self.code), self.s2(), J, _p(Y), B, _p(res), _p(l0),
                                   _p(stats), _p(acc), threads or host_threads())
        return res, l0, stats, acc

    def sweep(self, p, e, J=-1, max_snr=5.0, seed=1, decoder_snr_db=0.5):
        buf = C.create_string_buffer(1 << 16)
        r = lib().orc_sweep(C.byref(self.code), decoder_snr_db, J, p, e, max_snr, seed,
                            buf, len(buf))
        assert r >= 0
        return buf.raw[:r].decode()

    def stream_draws(self, state, count, snr_db):
        """(engine draws of `count` stream words from `state`, the state after them)."""
        st = C.c_uint64(state)
        d = lib().orc_stream_draws(C.byref(self.code), C.byref(st), count, snr_db)
        return int(d), st.value

    def sweep_block(self, J, snr_db, state, skip, B, decoder_snr_db=0.5):
        """fun()'s loop body over one block (orc_sweep_block): the block source of
        sweep_dist.sharded_sweep."""
        tx = np.zeros((B, self.n), np.uint8)
        res = np.zeros((B, self.n), np.uint8)
        acc = np.zeros(B, np.uint8)
        ops = np.zeros((B, 3), np.uint64)
        states = np.zeros(B, np.uint64)
        st = C.c_uint64(state)
        lib().orc_sweep_block(C.byref(self.code), decoder_snr_db, J, snr_db, C.byref(st), skip, B,
                              _p(tx), _p(res), _p(acc), _p(ops), _p(states))
        return tx, res, acc, ops, states, st.value

    def sweep_range(self, J, snr_db, state, draws, max_words, decoder_snr_db=0.5):
        """fun()'s loop body over the words of `draws` engine draws (orc_sweep_range)."""
        tx = np.zeros((max_words, self.n), np.uint8)
        res = np.zeros((max_words, self.n), np.uint8)
        acc = np.zeros(max_words, np.uint8)
        ops = np.zeros((max_words, 3), np.uint64)
        states = np.zeros(max_words, np.uint64)
        st = C.c_uint64(state)
        B = lib().orc_sweep_range(C.byref(self.code), decoder_snr_db, J, snr_db, C.byref(st), draws, max_words,
                                  _p(tx), _p(res), _p(acc), _p(ops), _p(states))
        assert B >= 0, "the range does not end on a word boundary"
        return tx[:B], res[:B], acc[:B], ops[:B], states[:B], st.value

    def stream(self, seed, count, snr_db):
        """The reference's fun() input stream: (tx [count,n], y [count,n])."""
        rng = (C.c_uint64 * 1)()
        lib().orc_rng_seed(rng, seed)
        info = np.zeros(self.k, np.uint8)
        tx = np.zeros((count, self.n), np.uint8)
        y = np.zeros((count, self.n))
        sd = self.sigma(snr_db)
        for w in range(count):
            lib().orc_gen_info(rng, _p(info), self.k)
            row = np.zeros(self.n, np.uint8)
            lib().orc_encode(C.byref(self.code), _p(info), _p(row))
            yy = np.zeros(self.n)
            lib().orc_add_noise(rng, sd, _p(row), _p(yy), self.n)
            tx[w], y[w] = row, yy
        return tx, y
