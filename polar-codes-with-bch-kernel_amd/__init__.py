"""bchk_amd -- Python view of libbchk.so (MI355X Kaneko/BCH soft decoder), via ctypes.

The product is the C ABI in include/bchk.h (HIP kernels for gfx950 + C++ host runtime);
this module only marshals numpy arrays / device pointers for tests, bench.py and
__graft_entry__. It mirrors the reference's KanekoKernelProcessor / Decoder / fun()
surface (headers/KanekoKernelProcessor.h:47-68, headers/Decoder.h:67-78,
headers/dataForPlot.h:8) with batched calls. There is no CPU fallback: if the HIP library
or a gfx950 device is missing, constructing a KanekoKernelProcessor raises.

Load it by path (the directory name is not an identifier):
    spec = importlib.util.spec_from_file_location("bchk_amd", ".../__init__.py")
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
# BCHK_LIB selects another build of the same ABI (e.g. lib/libbchk_diag.so)
LIB_PATH = os.environ.get("BCHK_LIB") or os.path.join(PKG_DIR, "lib", "libbchk.so")

BCHK_J_SHIPPED = -1
VARIANT_ANSWER, VARIANT_WORD = 0, 1
F_ACCEPTED, F_RETURNED, F_TRUNCATED, F_TIE, F_SCAN_UB = 1, 2, 4, 8, 16

# Every exported entry point of include/bchk.h.
EXPORTS = (
    "bchk_create", "bchk_destroy", "bchk_code_params", "bchk_generator",
    "bchk_set_max_decodes", "bchk_decode_host", "bchk_decode_device",
    "bchk_decode_variant_host", "bchk_alg_decode_host", "bchk_count_device", "bchk_decode_count_device",
    "bchk_generate_host", "bchk_generate_host_draws", "bchk_generate_device", "bchk_sweep_device", "bchk_rng_jump", "bchk_sweep_block", "bchk_sweep_range", "bchk_stream_skip",
    "bchk_stream_sync", "bchk_sweep", "bchk_sync", "bchk_stream", "bchk_profile",
    "bchk_profile_read", "bchk_profile_read_stages", "bchk_path_counts", "bchk_tail_count",
    "bchk_tail_stats", "bchk_coop_stats", "bchk_tail_diag_read", "bchk_tail_prof_read", "bchk_set_fast_path", "bchk_set_analytic",
    "bchk_set_chunk_limit", "bchk_set_syndrome_table",
    "bchk_syndrome_table_query", "bchk_syndrome_table_info", "bchk_polar_create", "bchk_polar_create_kdir",
    "bchk_polar_destroy", "bchk_polar_params", "bchk_polar_decode_host", "bchk_polar_decode_device",
    "bchk_polar_encode_host", "bchk_polar_sync", "bchk_polar_stream", "bchk_polar_last_launches",
    "bchk_kernel_ebch", "bchk_kernel_field_order", "bchk_kernel_trellis_cost", "bchk_kernel_column_costs",
    "bchk_kernel_column_search", "bchk_last_error", "bchk_version",
)

STATS_DTYPE = np.dtype([("decodes", "<u8"), ("comparisons", "<u8"), ("sums", "<u8"),
                        ("iterations", "<u8"), ("jsteps", "<u8"), ("improvements", "<u8"),
                        ("flags", "<u4"), ("reserved", "<u4")])


class BchkError(RuntimeError):
    pass


def build(force=False):
    """Compile libbchk.so in-tree (hipcc --offload-arch=gfx950)."""
    if force or not os.path.exists(LIB_PATH):
        jobs = os.environ.get("MAX_JOBS", "8")
        subprocess.run(["make", "-s", "-C", PKG_DIR, f"-j{min(int(jobs), 16)}"], check=True)
    return LIB_PATH


_lib = None


def lib():
    """Load libbchk.so. If torch is importable it is imported first so that one HIP
    runtime (torch's libamdhip64.so.7) serves both torch and libbchk in this process."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BchkError(f"{LIB_PATH} missing: run make -C {PKG_DIR} (no CPU fallback)")
    if "torch" not in sys.modules and os.environ.get("BCHK_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401
        except Exception:
            pass
    L = C.CDLL(LIB_PATH)
    vp, sz, i32, u64, dbl = C.c_void_p, C.c_size_t, C.c_int, C.c_uint64, C.c_double
    L.bchk_create.argtypes = [i32, i32, i32, dbl, i32, C.POINTER(vp)]
    L.bchk_destroy.argtypes = [vp]
    L.bchk_destroy.restype = None
    L.bchk_code_params.argtypes = [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]
    L.bchk_generator.argtypes = [vp, vp]
    L.bchk_set_max_decodes.argtypes = [vp, u64]
    L.bchk_decode_host.argtypes = [vp, vp, sz, vp, vp, vp]
    L.bchk_decode_device.argtypes = [vp, vp, sz, vp, vp, vp, vp]
    L.bchk_decode_variant_host.argtypes = [vp, i32, vp, sz, vp, vp, vp]
    L.bchk_alg_decode_host.argtypes = [vp, vp, vp, sz, vp, vp]
    L.bchk_count_device.argtypes = [vp, vp, vp, vp, sz, vp, vp]
    L.bchk_decode_count_device.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, vp]
    L.bchk_generate_device.argtypes = [vp, C.c_double, sz, u64, u64, vp, vp, vp]
    L.bchk_sweep_device.argtypes = [vp, C.c_long, C.c_long, C.c_double, u64, sz, C.c_char_p, sz,
                                    C.POINTER(C.c_double), C.POINTER(u64)]
    L.bchk_generate_host.argtypes = [vp, dbl, sz, C.POINTER(u64), u64, vp, vp]
    L.bchk_generate_host_draws.argtypes = [vp, dbl, sz, C.POINTER(u64), u64, vp, vp, C.POINTER(u64)]
    L.bchk_rng_jump.argtypes = [u64, u64]
    L.bchk_rng_jump.restype = u64
    L.bchk_sweep_block.argtypes = [vp, dbl, C.POINTER(u64), sz, sz, vp, vp, vp, vp, vp]
    L.bchk_sweep_range.argtypes = [vp, dbl, C.POINTER(u64), u64, sz, vp, vp, vp, vp, vp, C.POINTER(sz)]
    L.bchk_stream_skip.argtypes = [i32, i32, u64, u64, C.POINTER(u64), C.POINTER(u64)]
    L.bchk_stream_sync.argtypes = [i32, i32, u64, u64, u64, C.POINTER(u64), C.POINTER(u64)]
    L.bchk_sweep.argtypes = [vp, C.c_long, C.c_long, dbl, C.POINTER(u64), u64, sz, C.c_char_p, sz]
    L.bchk_sync.argtypes = [vp]
    L.bchk_stream.argtypes = [vp]
    L.bchk_stream.restype = vp
    L.bchk_profile.argtypes = [vp, i32]
    L.bchk_profile_read.argtypes = [vp, C.POINTER(dbl), C.POINTER(u64)]
    L.bchk_set_fast_path.argtypes = [vp, i32]
    L.bchk_set_syndrome_table.argtypes = [vp, i32]
    L.bchk_polar_create.argtypes = [C.c_char_p, i32, i32, C.POINTER(vp)]
    L.bchk_polar_create_kdir.argtypes = [C.c_char_p, C.c_char_p, i32, i32, C.POINTER(vp)]
    L.bchk_polar_destroy.argtypes = [vp]
    L.bchk_polar_destroy.restype = None
    L.bchk_polar_params.argtypes = [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]
    L.bchk_polar_decode_host.argtypes = [vp, vp, sz, vp, vp, vp, vp]
    L.bchk_polar_decode_device.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp]
    L.bchk_polar_encode_host.argtypes = [vp, vp, sz, vp]
    L.bchk_polar_sync.argtypes = [vp]
    L.bchk_polar_stream.argtypes = [vp]
    L.bchk_polar_stream.restype = vp
    L.bchk_syndrome_table_query.argtypes = [i32, i32, vp, sz, vp, vp]
    L.bchk_syndrome_table_info.argtypes = [i32, i32, C.POINTER(u64), C.POINTER(u64),
                                           C.POINTER(C.c_uint32)]
    L.bchk_path_counts.argtypes = [vp, C.POINTER(u64), C.POINTER(u64)]
    L.bchk_tail_count.argtypes = [vp, C.POINTER(u64)]
    L.bchk_tail_stats.argtypes = [vp, C.POINTER(u64)]
    L.bchk_coop_stats.argtypes = [vp, C.POINTER(u64)]
    L.bchk_tail_diag_read.argtypes = [vp, C.POINTER(u64), sz, C.POINTER(u64)]
    L.bchk_tail_prof_read.argtypes = [vp, C.POINTER(u64), sz]
    L.bchk_profile_read_stages.argtypes = [vp, C.POINTER(dbl), C.POINTER(u64)]
    L.bchk_set_analytic.argtypes = [vp, i32]
    L.bchk_set_chunk_limit.argtypes = [vp, C.c_uint32]
    L.bchk_kernel_ebch.argtypes = [i32, vp]
    L.bchk_kernel_field_order.argtypes = [i32, vp, vp]
    L.bchk_kernel_trellis_cost.argtypes = [vp, i32, vp, i32, C.POINTER(u64), C.POINTER(u64)]
    L.bchk_kernel_column_costs.argtypes = [i32, vp, vp, i32, vp, vp]
    L.bchk_kernel_column_search.argtypes = [i32, vp, vp, i32, u64, C.POINTER(u64), i32, vp, vp,
                                            C.POINTER(u64), C.POINTER(u64), C.POINTER(C.c_int64)]
    L.bchk_last_error.restype = C.c_char_p
    L.bchk_version.restype = C.c_char_p
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise BchkError(f"bchk error {rc}: {lib().bchk_last_error().decode()}")


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class KanekoKernelProcessor:
    """Batched KanekoKernelProcessor (headers/KanekoKernelProcessor.h:47-68) for one
    BCH(n, k) code with t = designed correction capability, on one gfx950 device."""

    def __init__(self, m, t, J=BCHK_J_SHIPPED, decoder_snr_db=0.5, device=0):
        L = lib()
        h = C.c_void_p()
        _check(L.bchk_create(m, t, J, decoder_snr_db, device, C.byref(h)))
        self._h = h
        n, k, gs = C.c_int(), C.c_int(), C.c_int()
        _check(L.bchk_code_params(h, C.byref(n), C.byref(k), C.byref(gs)))
        self.m, self.t, self.J = m, t, J
        self.n, self.k = n.value, k.value
        self.g = np.zeros(gs.value, np.uint8)
        _check(L.bchk_generator(h, _p(self.g)))

    def close(self):
        if getattr(self, "_h", None):
            lib().bchk_destroy(self._h)
            self._h = None

    def __del__(self):
        # at interpreter shutdown the module globals may already be gone: the process
        # teardown releases the device memory then
        try:
            self.close()
        except (TypeError, AttributeError):
            pass

    @property
    def handle(self):
        return self._h

    def set_max_decodes(self, md):
        _check(lib().bchk_set_max_decodes(self._h, int(md)))

    def decode(self, y, res=None, variant=VARIANT_ANSWER):
        """y [B, n] f64 -> (res [B, n] u8, l0 [B] f64, stats [B] STATS_DTYPE).
        Rows that are never accepted keep the incoming `res` content (default 0)."""
        y = np.ascontiguousarray(np.atleast_2d(y), np.float64)
        B = y.shape[0]
        assert y.shape[1] == self.n
        res = np.zeros((B, self.n), np.uint8) if res is None else np.ascontiguousarray(res, np.uint8)
        l0 = np.zeros(B, np.float64)
        st = np.zeros(B, STATS_DTYPE)
        _check(lib().bchk_decode_variant_host(self._h, variant, _p(y), B, _p(res), _p(l0), _p(st)))
        return res, l0, st

    def decode_device(self, d_y, B, d_res, d_l0, d_st, stream=None):
        _check(lib().bchk_decode_device(self._h, C.c_void_p(d_y), B, C.c_void_p(d_res),
                                        C.c_void_p(d_l0), C.c_void_p(d_st),
                                        C.c_void_p(stream) if stream else None))

    def count_device(self, d_tx, d_res, d_st, B, d_out6, stream=None):
        _check(lib().bchk_count_device(self._h, C.c_void_p(d_tx), C.c_void_p(d_res),
                                       C.c_void_p(d_st), B, C.c_void_p(d_out6),
                                       C.c_void_p(stream) if stream else None))

    def decode_count_device(self, d_y, d_tx, B, d_res, d_l0, d_st, d_out6, stream=None):
        """decode_device + count_device fused (bchk_decode_count_device); d_st may be 0."""
        _check(lib().bchk_decode_count_device(self._h, C.c_void_p(d_y), C.c_void_p(d_tx), B, C.c_void_p(d_res),
                                              C.c_void_p(d_l0), C.c_void_p(d_st) if d_st else None,
                                              C.c_void_p(d_out6), C.c_void_p(stream) if stream else None))

    def alg_decode(self, words, syndromes=None):
        """Decoder::decode batch: words [N, n] u8 -> (ok [N] bool, answers [N, n] u8)."""
        words = np.ascontiguousarray(np.atleast_2d(words), np.uint8)
        N = words.shape[0]
        ans = np.zeros_like(words)
        ok = np.zeros(N, np.uint8)
        sp = None
        if syndromes is not None:
            syndromes = np.ascontiguousarray(syndromes, np.uint32)
            sp = _p(syndromes)
        _check(lib().bchk_alg_decode_host(self._h, _p(words), sp, N, _p(ans), _p(ok)))
        return ok.astype(bool), ans

    def generate(self, snr_db, B, seed=1, state=0):
        """The reference input stream: (tx [B, n] u8, y [B, n] f64, next_state)."""
        tx = np.zeros((B, self.n), np.uint8)
        y = np.zeros((B, self.n), np.float64)
        st = C.c_uint64(state)
        _check(lib().bchk_generate_host(self._h, snr_db, B, C.byref(st), seed, _p(tx), _p(y)))
        return tx, y, st.value

    def generate_draws(self, snr_db, B, seed=1, state=0):
        """generate() and the engine draws it consumed: (tx, y, next_state, draws)."""
        tx = np.zeros((B, self.n), np.uint8)
        y = np.zeros((B, self.n), np.float64)
        st, dr = C.c_uint64(state), C.c_uint64()
        _check(lib().bchk_generate_host_draws(self._h, snr_db, B, C.byref(st), seed, _p(tx), _p(y),
                                              C.byref(dr)))
        return tx, y, st.value, dr.value

    def sweep_block(self, snr_db, state, skip, B):
        """One block of a sharded fun() sweep (bchk_sweep_block): (tx, res, accepted,
        ops [B, 3] = decodes/comparisons/sums, states [B] after each word, state after)."""
        tx = np.zeros((B, self.n), np.uint8)
        res = np.zeros((B, self.n), np.uint8)
        acc = np.zeros(B, np.uint8)
        ops = np.zeros((B, 3), np.uint64)
        states = np.zeros(B, np.uint64)
        st = C.c_uint64(state)
        _check(lib().bchk_sweep_block(self._h, snr_db, C.byref(st), skip, B, _p(tx), _p(res), _p(acc),
                                      _p(ops), _p(states)))
        return tx, res, acc, ops, states, st.value

    def sweep_range(self, snr_db, state, draws, max_words):
        """The words of `draws` engine draws from word start `state` (bchk_sweep_range), as
        sweep_block: (tx, res, accepted, ops, states, state after)."""
        tx = np.zeros((max_words, self.n), np.uint8)
        res = np.zeros((max_words, self.n), np.uint8)
        acc = np.zeros(max_words, np.uint8)
        ops = np.zeros((max_words, 3), np.uint64)
        states = np.zeros(max_words, np.uint64)
        st, nw = C.c_uint64(state), C.c_size_t()
        _check(lib().bchk_sweep_range(self._h, snr_db, C.byref(st), draws, max_words, _p(tx), _p(res), _p(acc),
                                      _p(ops), _p(states), C.byref(nw)))
        B = nw.value
        return tx[:B], res[:B], acc[:B], ops[:B], states[:B], st.value

    def sweep(self, p, e, max_snr=5.0, seed=1, batch=0, state=0, return_state=False):
        """fun() on the GPU: the reference CSV text (and the engine state after it)."""
        buf = C.create_string_buffer(1 << 16)
        st = C.c_uint64(state)
        _check(lib().bchk_sweep(self._h, p, e, max_snr, C.byref(st), seed, batch, buf, len(buf)))
        return (buf.value.decode(), st.value) if return_state else buf.value.decode()

    def generate_device(self, snr, B, d_tx, d_y, seed=1, word0=0, stream=None):
        """On-GPU channel: words [word0, word0 + B) of the counter-based stream into d_tx, d_y."""
        _check(lib().bchk_generate_device(self._h, snr, B, seed, word0, C.c_void_p(d_tx), C.c_void_p(d_y),
                                          C.c_void_p(stream) if stream else None))

    def sweep_device(self, p, e, max_snr=5.0, seed=1, batch=0):
        """fun() with GPU-generated words: (CSV text, seconds, words decoded)."""
        buf = C.create_string_buffer(1 << 16)
        secs, words = C.c_double(0.0), C.c_uint64(0)
        _check(lib().bchk_sweep_device(self._h, p, e, max_snr, seed, batch, buf, len(buf), C.byref(secs),
                                       C.byref(words)))
        return buf.value.decode(), secs.value, words.value

    def sync(self):
        _check(lib().bchk_sync(self._h))

    @property
    def stream(self):
        return lib().bchk_stream(self._h)

    def profile(self, enable=True):
        _check(lib().bchk_profile(self._h, 1 if enable else 0))

    def profile_read(self):
        """([fast, exact, coop] kernel ms summed, decode calls) since the last read."""
        ms = (C.c_double * 3)()
        n = C.c_uint64()
        _check(lib().bchk_profile_read(self._h, ms, C.byref(n)))
        return list(ms), n.value

    def profile_read_stages(self):
        """([fast, exact first pass, coop, analytic tail] kernel ms, decode calls)."""
        ms = (C.c_double * 4)()
        n = C.c_uint64()
        _check(lib().bchk_profile_read_stages(self._h, ms, C.byref(n)))
        return list(ms), n.value

    def tail_count(self):
        """Codewords the last call's first pass handed to the analytic tail kernel."""
        a = C.c_uint64()
        _check(lib().bchk_tail_count(self._h, C.byref(a)))
        return a.value

    def tail_stats(self):
        """Last call's analytic tail outcomes: [handed on, finished, split, split chunks,
        enumeration steps, max steps per codeword]."""
        a = (C.c_uint64 * 6)()
        _check(lib().bchk_tail_stats(self._h, a))
        return list(a)

    def coop_stats(self):
        """Last call's cooperative-kernel counters (m >= 7): [dense re-decodes served,
        heavy codewords started]."""
        a = (C.c_uint64 * 2)()
        _check(lib().bchk_coop_stats(self._h, a))
        return list(a)

    def tail_diag(self, items=65536):
        """Diagnostics (context created with BCHK_TAIL_DIAG=1): per-codeword tail records."""
        import numpy as np
        out = np.zeros((items, 8), np.uint64)
        n = C.c_uint64()
        _check(lib().bchk_tail_diag_read(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), items,
                                         C.byref(n)))
        return out[:min(items, n.value)]

    def tail_prof(self, items=65536):
        """Experiment builds (BCHK_AN_PROF): enumeration cycles by step phase per tail record."""
        import numpy as np
        out = np.zeros((items, 8), np.uint64)
        _check(lib().bchk_tail_prof_read(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), items))
        return out

    def set_analytic(self, enable=True):
        """Analytic tail of heavy codewords (results identical either way)."""
        _check(lib().bchk_set_analytic(self._h, 1 if enable else 0))

    def set_chunk_limit(self, chunks):
        """64-pattern chunks of the exact first pass before the tail / hand-off."""
        _check(lib().bchk_set_chunk_limit(self._h, int(chunks)))

    def path_counts(self):
        """(codewords handed to the exact kernel, to the cooperative kernel) last call."""
        a, b = C.c_uint64(), C.c_uint64()
        _check(lib().bchk_path_counts(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def set_fast_path(self, enable=True):
        _check(lib().bchk_set_fast_path(self._h, 1 if enable else 0))

    def set_syndrome_table(self, enable=True):
        """Syndrome decoding table of the search kernels (results identical either way)."""
        _check(lib().bchk_set_syndrome_table(self._h, 1 if enable else 0))


class PolarListDecoder:
    """CMixedKernelListDecoder(Spec, ListSize) + Decode (out/external/MixedKernelListDecoder.cpp
    :9, :211-268) on the GPU: batched SC-list decoding of a polar code given by the
    reference's specification text (Arikan layers)."""

    def __init__(self, spec, L, device=0, kernel_dir=None):
        h = C.c_void_p()
        _check(lib().bchk_polar_create_kdir(spec.encode(), kernel_dir.encode() if kernel_dir else None, L, device,
                                            C.byref(h)))
        self._h = h
        n, k, u, l = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _check(lib().bchk_polar_params(h, C.byref(n), C.byref(k), C.byref(u), C.byref(l)))
        self.N, self.K, self.U, self.L = n.value, k.value, u.value, l.value

    def close(self):
        if getattr(self, "_h", None):
            lib().bchk_polar_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def stream(self):
        return lib().bchk_polar_stream(self._h)

    def encode(self, info):
        info = np.ascontiguousarray(info, np.uint8)
        cw = np.zeros((info.shape[0], self.N), np.uint8)
        _check(lib().bchk_polar_encode_host(self._h, _p(info), info.shape[0], _p(cw)))
        return cw

    def decode(self, llr):
        """llr [B][N] float32 -> (count [B], info [B][L][K], codewords [B][L][N], metrics [B][L])."""
        llr = np.ascontiguousarray(llr, np.float32)
        B = llr.shape[0]
        info = np.zeros((B, self.L, self.K), np.uint8)
        cw = np.zeros((B, self.L, self.N), np.uint8)
        met = np.zeros((B, self.L), np.float32)
        cnt = np.zeros(B, np.int32)
        _check(lib().bchk_polar_decode_host(self._h, _p(llr), B, _p(info), _p(cw), _p(met), _p(cnt)))
        return cnt, info, cw, met

    def decode_device(self, d_llr, B, d_info, d_cw, d_metric, d_count, stream=None):
        _check(lib().bchk_polar_decode_device(self._h, d_llr, B, d_info, d_cw, d_metric, d_count,
                                              stream))

    def sync(self):
        _check(lib().bchk_polar_sync(self._h))

    def last_launches(self):
        """Kernel launches the last decode call took (time-budgeted codes with search layers)."""
        n = C.c_uint64()
        _check(lib().bchk_polar_last_launches(self._h, C.byref(n)))
        return n.value


def stream_skip(k, n, state, words):
    """(engine state, draws) after `words` stream words from `state` (no samples, no device)."""
    st, dr = C.c_uint64(), C.c_uint64()
    _check(lib().bchk_stream_skip(k, n, state, words, C.byref(st), C.byref(dr)))
    return st.value, dr.value


def stream_sync(k, n, state, offset, limit):
    """A word start in [offset, offset + limit) draws from word start `state` that depends only
    on (state, offset, limit) -- where every parse possible at `offset` has merged, not
    necessarily the first start at or after it -- found without parsing the draws before
    `offset`: (draws from state, engine state), or None when unresolved."""
    off, st = C.c_uint64(), C.c_uint64()
    rc = lib().bchk_stream_sync(k, n, state, offset, limit, C.byref(off), C.byref(st))
    if rc == 1:
        return None
    _check(rc)
    return off.value, st.value


def rng_jump(state, draws):
    """The reference engine's state `draws` draws after `state` (a seed is a state)."""
    return int(lib().bchk_rng_jump(int(state), int(draws)))


MINSTD_PERIOD = 2147483646  # minstd_rand0: 2^31 - 2


def syndrome_table_query(m, t, syndromes):
    """Host-side Decoder::decode through the syndrome table (no GPU): syndromes [N][t] odd
    syndromes S_1, S_3, ... as uint32 -> (ok [N] bool, flipped-position masks [N] uint64)."""
    syn = np.ascontiguousarray(syndromes, np.uint32)
    N = syn.shape[0]
    ok = np.zeros(N, np.uint8)
    err = np.zeros(N, np.uint64)
    _check(lib().bchk_syndrome_table_query(m, t, _p(syn), N, _p(ok), _p(err)))
    return ok.astype(bool), err


def syndrome_table_info(m, t):
    """(distinct keys, bytes, longest probe sequence) of the (m, t) syndrome table."""
    k, b, p = C.c_uint64(), C.c_uint64(), C.c_uint32()
    _check(lib().bchk_syndrome_table_info(m, t, C.byref(k), C.byref(b), C.byref(p)))
    return k.value, b.value, p.value


def kernel_ebch(power):
    """makeMatrix (root bchCoder.cpp:356-389): the nested extended-BCH kernel, 2^power square."""
    n = 1 << power
    K = np.zeros((n, n), np.uint8)
    _check(lib().bchk_kernel_ebch(power, _p(K)))
    return K


def kernel_field_order(power, K):
    """swapColumns' column reordering (root bchCoder.cpp:478-496)."""
    K = np.ascontiguousarray(K, np.uint8)
    out = np.zeros_like(K)
    _check(lib().bchk_kernel_field_order(power, _p(K), _p(out)))
    return out


def kernel_trellis_cost(K, llr, device=0):
    """(SumCount, CmpCount) of CTrellisKernelProcessor::GetLLRs over every phase with zero known
    inputs (the column search's score), computed on the GPU."""
    K = np.ascontiguousarray(K, np.uint8)
    y = np.ascontiguousarray(llr, np.float32)
    s, c = C.c_uint64(), C.c_uint64()
    _check(lib().bchk_kernel_trellis_cost(_p(K), K.shape[0], _p(y), device, C.byref(s), C.byref(c)))
    return s.value, c.value


def kernel_column_costs(power, K, llr, device=0):
    """Scores of every L.U column map (indexed by candidate code), from one GPU launch."""
    K = np.ascontiguousarray(K, np.uint8)
    y = np.ascontiguousarray(llr, np.float32)
    n = 1 << (power * (power - 1))
    s = np.zeros(n, np.uint64)
    c = np.zeros(n, np.uint64)
    _check(lib().bchk_kernel_column_costs(power, _p(K), _p(y), device, _p(s), _p(c)))
    return s, c


KSEARCH_EXHAUSTIVE, KSEARCH_RANDOM = 0, 1


def kernel_column_search(power, K, llr, mode=KSEARCH_EXHAUSTIVE, count=0, rng_state=1, device=0):
    """randomSwapColumns (root bchCoder.cpp:541-699) -> dict(best, perm, sum, cmp, index,
    rng_state)."""
    K = np.ascontiguousarray(K, np.uint8)
    y = np.ascontiguousarray(llr, np.float32)
    n = 1 << power
    best = np.zeros((n, n), np.uint8)
    perm = np.zeros(n, np.uint32)
    st, s, c, i = C.c_uint64(rng_state), C.c_uint64(), C.c_uint64(), C.c_int64()
    _check(lib().bchk_kernel_column_search(power, _p(K), _p(y), mode, count, C.byref(st), device,
                                           _p(best), _p(perm), C.byref(s), C.byref(c), C.byref(i)))
    return dict(best=best, perm=perm, sum=s.value, cmp=c.value, index=i.value, rng_state=st.value)


def version():
    return lib().bchk_version().decode()

from . import sweep_dist  # noqa: E402,F401  (sharded fun() sweep over ranks)
