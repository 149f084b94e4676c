"""The timed path at the timed configuration, pinned to the oracle (GPU box).

bench.py times one call per step: bchk_decode_count_device (decode + fused FER/op
counters, no stats record, the selection fast kernel, chunk limit, analytic tail,
cooperative kernel) over rank r's 2^20 words of the reference stream, BCH(63,30,13), J=15,
at 4 / 5 / 6 dB. These tests make exactly that call on exactly that input and check it
against the C oracle (the restatement of src/KanekoKernelProcessor.cpp:335-407, pinned to
the reference binary by tests/test_oracle.py):

* 5 and 6 dB: every one of the 2^20 rows (word, l0 bits) and the six fused counters equal
  to the oracle's sums; the per-row counters (from the same inputs decoded with a stats
  record) equal to the oracle's on every row.
* 4 dB: every row the fast path and the first exact pass did not finish (known from the
  stats run: ~20 000 analytic-tail / cooperative rows, the oracle's threads take about a
  minute) plus 4096 random rows go to the oracle; all 2^20 rows equal the cooperative path
  without the analytic tail; the fused counters equal the stats run's sums.
* Config 4's data shape on one GPU: the 2^23-word batch (the eight ranks' jump-ahead 2^20
  shards of bench.py, concatenated) decoded in ONE call gives the sum of the eight shard
  calls' counters and the same rows.
"""
import importlib.util
import os

import numpy as np
import pytest

from bchk_pkg import load
from oracle_lib import Oracle

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = 1 << 20
M, T, J = 6, 6, 15
CHUNK = 64


def bench_module():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


_dec = {}


def decoder():
    # the bench's decoder: default knobs (bench.py main: KanekoKernelProcessor(m, t, J=J))
    if "d" not in _dec:
        _dec["d"] = load().KanekoKernelProcessor(M, T, J=J)
    return _dec["d"]


def rank_words(d, snr, rank, world, count=B):
    """bench.py run_point's input for `rank` of `world`: its jump-ahead start in the one
    reference stream (bench.rank_stream_start), `count` words, draw budget checked."""
    bench = bench_module()
    start, budget = bench.rank_stream_start(load(), 1, rank, world)
    tx, y, _, used = d.generate_draws(snr, count, state=start)
    assert used <= budget
    return tx, y


def bench_step(d, dy, dtx, n_rows):
    """One bench step (bench.py run_point step(), world 1): fused decode + counters into a
    zero-initialised res, counters accumulated into a zeroed [6] int64 vector."""
    import torch
    dres = torch.zeros((n_rows, d.n), dtype=torch.uint8, device="cuda")
    dl0 = torch.empty(n_rows, dtype=torch.float64, device="cuda")
    cnt = torch.zeros(6, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    d.decode_count_device(dy.data_ptr(), dtx.data_ptr(), n_rows, dres.data_ptr(), dl0.data_ptr(), 0,
                          cnt.data_ptr(), d.stream)
    d.sync()
    return dres.cpu().numpy(), dl0.cpu().numpy(), cnt.cpu().numpy()


def stats_run(d, dy, n_rows):
    """The same rows decoded with a per-codeword stats record (bchk_decode_device)."""
    import torch
    dres = torch.zeros((n_rows, d.n), dtype=torch.uint8, device="cuda")
    dl0 = torch.empty(n_rows, dtype=torch.float64, device="cuda")
    dst = torch.zeros((n_rows, load().STATS_DTYPE.itemsize), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    d.decode_device(dy.data_ptr(), n_rows, dres.data_ptr(), dl0.data_ptr(), dst.data_ptr(), d.stream)
    d.sync()
    return dres.cpu().numpy(), dl0.cpu().numpy(), dst.cpu().numpy().view(load().STATS_DTYPE).reshape(n_rows)


def counters_from(tx, res, dec, cmp, sums):
    err = (res != tx).sum(axis=1)
    return np.array([int((err > 0).sum()), int(err.sum()), int(dec.sum()), int(cmp.sum()), int(sums.sum()),
                     len(tx)], np.int64)


def assert_rows_equal_oracle(rows, res, l0, st, r2, l2, s2, a2):
    acc = a2.astype(bool)
    np.testing.assert_array_equal(res[rows][acc], r2[acc])
    np.testing.assert_array_equal(res[rows][~acc], 0)  # never accepted: the caller's zeros
    np.testing.assert_array_equal(l0[rows][acc].view(np.uint64), l2[acc].view(np.uint64))
    if st is not None:
        np.testing.assert_array_equal(st["decodes"][rows], s2[:, 0])
        np.testing.assert_array_equal(st["comparisons"][rows], s2[:, 1])
        np.testing.assert_array_equal(st["sums"][rows], s2[:, 2])
        np.testing.assert_array_equal((st["flags"][rows] & load().F_ACCEPTED) != 0, acc)


@pytest.mark.parametrize("snr", [5.0, 6.0, 4.0])
def test_bench_step_matches_oracle(snr):
    import torch
    F = load()
    d = decoder()
    tx, y = rank_words(d, snr, 0, 1)
    dy, dtx = torch.from_numpy(y).cuda(), torch.from_numpy(tx).cuda()
    res, l0, cnt = bench_step(d, dy, dtx, B)
    to_exact, to_coop = d.path_counts()
    to_tail = d.tail_count()
    sres, sl0, st = stats_run(d, dy, B)
    # (the full sort without selection may queue a few more codewords for the exact kernel:
    # its early exit uses the same bound, but it sends every prefix tie on; the analytic
    # tail and cooperative kernels see the same codewords)
    assert (to_coop, to_tail) == (d.path_counts()[1], d.tail_count())
    # the stats run takes the same decisions (full sort instead of the 16-key selection)
    np.testing.assert_array_equal(sres, res)
    np.testing.assert_array_equal(sl0.view(np.uint64), l0.view(np.uint64))
    assert not np.any(st["flags"] & (F.F_TIE | F.F_TRUNCATED))
    # fused counters == the per-row stats' sums (and FER/BER from the rows)
    np.testing.assert_array_equal(cnt, counters_from(tx, res, st["decodes"], st["comparisons"], st["sums"]))
    o = Oracle(M, T)
    heavy = np.flatnonzero(st["decodes"] > 2 + 8 * CHUNK)  # past the first pass's chunks
    if snr >= 5.0:
        rows = np.arange(B)
    else:  # every heavy row (the analytic tail's and the cooperative kernel's) + 4096 others
        rng = np.random.default_rng(11)
        rows = np.unique(np.concatenate([heavy, rng.choice(B, 4096, replace=False)]))
        # and every row against the cooperative path without the analytic tail (hand-off
        # to the cooperative kernel after the first chunk: test_gpu_parity.PATHS coop-heavy)
        import os
        old_lim = os.environ.get("BCHK_CHUNK_LIMIT")
        os.environ["BCHK_CHUNK_LIMIT"] = "1"
        try:
            dc = F.KanekoKernelProcessor(M, T, J=J)
        finally:
            os.environ.pop("BCHK_CHUNK_LIMIT")
            if old_lim is not None:
                os.environ["BCHK_CHUNK_LIMIT"] = old_lim
        dc.set_analytic(False)
        cres, cl0, cst = stats_run(dc, dy, B)
        np.testing.assert_array_equal(cres, res)
        np.testing.assert_array_equal(cl0.view(np.uint64), l0.view(np.uint64))
        np.testing.assert_array_equal(cst, st)
        assert dc.path_counts()[1] >= len(heavy)
        dc.close()
    r2, l2, s2, a2 = o.kaneko_batch(y[rows], J=J)
    assert_rows_equal_oracle(rows, res, l0, st, r2, l2, s2, a2)
    if snr >= 5.0:  # every row: the fused counters are the oracle's
        acc = a2.astype(bool)
        ores = np.where(acc[:, None], r2, 0)
        np.testing.assert_array_equal(cnt, counters_from(tx, ores, s2[:, 0], s2[:, 1], s2[:, 2]))
    # the heavy rows really went through the tail / cooperative kernels
    if snr <= 5.0:
        assert to_tail > 0 and len(heavy) > 0
    print(f"\n{snr} dB: to_exact {to_exact} to_tail {to_tail} to_coop {to_coop}; oracle rows {len(rows)}"
          f" (heavy {len(heavy)}); counters {cnt.tolist()}")


def test_config5_bench_step_jinf_matches_oracle():
    # Config 5's 6 dB J = inf bench line (bench.py --m 8 --t 15 --snr 6 --J -1): the bench's own
    # 2^20 BCH(255,139,31) words through the bench's fused call. Every row against the
    # exact-only path (one wave per codeword, every pattern in order), and every row that left
    # the first-pattern kernel (decodes > 4: the search / cooperative kernels' rows, including
    # the uncapped ~2^17-decode codeword that dominates the step) plus 8192 others against the
    # oracle (src/KanekoKernelProcessor.cpp:361-405, the shipped non-monotone bound).
    import torch
    F = load()
    m, t, Jinf, snr = 8, 15, -1, 6.0
    d = F.KanekoKernelProcessor(m, t, J=Jinf)
    old = os.environ.get("BCHK_CHUNK_LIMIT")
    os.environ["BCHK_CHUNK_LIMIT"] = "0"
    try:
        ex = F.KanekoKernelProcessor(m, t, J=Jinf)
    finally:
        os.environ.pop("BCHK_CHUNK_LIMIT")
        if old is not None:
            os.environ["BCHK_CHUNK_LIMIT"] = old
    ex.set_fast_path(False)
    try:
        tx, y = rank_words(d, snr, 0, 1)
        dy, dtx = torch.from_numpy(y).cuda(), torch.from_numpy(tx).cuda()
        res, l0, cnt = bench_step(d, dy, dtx, B)
        to_exact, to_coop = d.path_counts()
        sres, sl0, st = stats_run(ex, dy, B)
        np.testing.assert_array_equal(sres, res)
        np.testing.assert_array_equal(sl0.view(np.uint64), l0.view(np.uint64))
        assert not np.any(st["flags"] & (F.F_TIE | F.F_TRUNCATED))
        np.testing.assert_array_equal(cnt, counters_from(tx, res, st["decodes"], st["comparisons"], st["sums"]))
        heavy = np.flatnonzero(st["decodes"] > 4)
        big = int(st["decodes"].max())
        assert to_coop >= 1 and big > 8 * CHUNK and (st["decodes"] > 5000).sum() >= 1
        rng = np.random.default_rng(13)
        rows = np.unique(np.concatenate([heavy, rng.choice(B, 8192, replace=False)]))
        r2, l2, s2, a2 = Oracle(m, t).kaneko_batch(y[rows], J=Jinf)
        assert_rows_equal_oracle(rows, res, l0, st, r2, l2, s2, a2)
        print(f"\nBCH(255,139,31) 6 dB J=inf: to_exact {to_exact} to_coop {to_coop}; oracle rows {len(rows)}"
              f" (decodes > 4: {len(heavy)}, > 5000: {int((st['decodes'] > 5000).sum())}, max {big})")
    finally:
        d.close()
        ex.close()


def test_config4_batch_equals_eight_shards():
    # BASELINE config 4: 2^23 words = the eight ranks' 2^20 jump-ahead shards. One call over
    # all of them (one GPU) == the eight shard calls (what eight GPUs run), row for row, and
    # its counters == the sum of theirs == what the RCCL all-reduce adds up.
    import torch
    d = decoder()
    W, snr = 8, 5.0
    dy = torch.empty((W * B, d.n), dtype=torch.float64, device="cuda")
    dtx = torch.empty((W * B, d.n), dtype=torch.uint8, device="cuda")
    for r in range(W):
        tx, y = rank_words(d, snr, r, W)
        dy[r * B:(r + 1) * B].copy_(torch.from_numpy(y))
        dtx[r * B:(r + 1) * B].copy_(torch.from_numpy(tx))
        del tx, y
    torch.cuda.synchronize()
    big_res, big_l0, big_cnt = bench_step(d, dy, dtx, W * B)
    tail_big = d.tail_count()
    total = np.zeros(6, np.int64)
    tails = 0
    for r in range(W):
        res, l0, cnt = bench_step(d, dy[r * B:(r + 1) * B], dtx[r * B:(r + 1) * B], B)
        tails += d.tail_count()
        np.testing.assert_array_equal(big_res[r * B:(r + 1) * B], res)
        np.testing.assert_array_equal(big_l0[r * B:(r + 1) * B].view(np.uint64), l0.view(np.uint64))
        total += cnt
    np.testing.assert_array_equal(big_cnt, total)
    assert big_cnt[5] == W * B and tail_big == tails
    print(f"\nconfig 4 (2^23 words, 5 dB, J=15): counters {big_cnt.tolist()}, FER {big_cnt[0] / big_cnt[5]:.3e}")
