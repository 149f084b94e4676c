"""CPU stand-in for libbchk's KanekoKernelProcessor in bench.py's plumbing tests
(BCHK_BENCH_STUB=1, tests/test_bench_spawn.py): the C oracle (the checker) decodes each rank's
batch from host pointers so that bench.py's rank launch, jump-ahead stream ranges, per-step
counter exchange and single JSON line can run on a machine without a GPU. Test
infrastructure only: bench.py marks such a line `stub_decoder`, and it is no measurement."""
import ctypes as C

import numpy as np

from oracle_lib import Oracle


def host_array(ptr, shape, dtype):
    dtype = np.dtype(dtype)
    count = int(np.prod(shape))
    buf = (C.c_ubyte * (count * dtype.itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=count).reshape(shape)


def stub_counters(o, J, tx, y):
    """The six fused counters of one batch ({frame errors, bit errors, decodes, comparisons,
    sums, words}, src/dataForPlot.cpp:55-74): a row nothing was accepted for counts as wrong."""
    res, _, stats, acc = o.kaneko_batch(y, J=J)
    wrong = (res != tx) | (acc == 0)[:, None]
    return np.array([int(wrong.any(axis=1).sum()), int(wrong.sum()), int(stats[:, 0].sum()),
                     int(stats[:, 1].sum()), int(stats[:, 2].sum()), len(y)], np.int64)


class StubDecoder:
    stream = 0

    def __init__(self, m, t, J=-1):
        self.o = Oracle(m, t)
        self.m, self.t, self.J, self.n, self.k = m, t, J, self.o.n, self.o.k
        self._calls = 0

    def generate_draws(self, snr_db, B, seed=1, state=0):
        tx, y = self.o.stream(state, B, snr_db)
        draws, after = self.o.stream_draws(state, B, snr_db)
        return tx, y, after, draws

    def decode_count_device(self, d_y, d_tx, B, d_res, d_l0, d_st, d_out6, stream=None):
        y = host_array(d_y, (B, self.n), np.float64)
        tx = host_array(d_tx, (B, self.n), np.uint8)
        out = host_array(d_out6, (6,), np.int64)
        out += stub_counters(self.o, self.J, tx, y)
        self._calls += 1

    def sync(self):
        pass

    def profile(self, enable=True):
        self._calls = 0

    def profile_read_stages(self):
        return [0.0, 0.0, 0.0, 0.0], self._calls

    def path_counts(self):
        return 0, 0

    def tail_count(self):
        return 0

    def tail_stats(self):
        return [0] * 6
