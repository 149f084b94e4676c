"""Sharded fun() sweep: the reference's Monte-Carlo FER loop (src/dataForPlot.cpp:16-116) over
ranks, with output identical to the single-process sweep.

The reference consumes one sequential stream: per Eb/N0 point it draws words until `p` words
or `e` frame errors (`while (count < p && countErr < e)`, :43), and the next point continues
from the word after the stop. Here every round splits the next `world * nb` words of the
stream into contiguous blocks, block r to rank r; each rank generates and decodes its own
block (generating the earlier blocks of the round only to advance the engine: the stream
is sequential), then one all-gather of per-block (words, frame errors, last decoded row)
fixes where the point stops, in stream order, and one all-reduce sums the counters of the
words before the stop. The rank holding the stop word broadcasts the engine state after it.

Quirks kept: countE (bit errors) is never reset (:20, :90-95); the `decoded` buffer is shared
by all words and only written on acceptance (:25, :52), so a word whose search never accepts
is counted against the previous word's decision -- across block and rank boundaries too.

`source.block(snr, state, skip, B)` returns (tx, res, accepted, ops[B, 3], states[B],
state_after); libbchk's KanekoKernelProcessor.sweep_block (GPU) is the product source; the
tests also drive it with the C oracle on CPU.
"""
import numpy as np

MINSTD_M = 2147483647


def _g(x):
    return "%g" % x  # std::ostream << double: defaultfloat, precision 6


class _Comm:
    """The exchange: torch.distributed (gloo or RCCL) or a single process."""

    def __init__(self, dist, world, rank, device):
        self.dist, self.world, self.rank, self.device = dist, world, rank, device

    def all_gather_i64(self, vals):
        import torch
        t = torch.tensor(vals, dtype=torch.int64, device=self.device)
        if self.world == 1:
            return [list(vals)]
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.cpu().tolist() for o in out]

    def all_gather_u8(self, row):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(row)).to(self.device)
        if self.world == 1:
            return [row]
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.cpu().numpy() for o in out]

    def all_reduce_i64(self, vals):
        import torch
        t = torch.tensor(vals, dtype=torch.int64, device=self.device)
        if self.world > 1:
            self.dist.all_reduce(t)
        return t.cpu().tolist()


def sharded_sweep(source, n, p, e, max_snr=5.0, seed=1, dist=None, world=1, rank=0, device="cpu",
                  block=1 << 16):
    """The CSV text of fun(file, decoder, g, gSize, p, e, maxSTNR); every rank returns it."""
    comm = _Comm(dist, world, rank, device)
    state = int(seed) % MINSTD_M or 1
    decoded = np.zeros(n, np.uint8)  # fun()'s `decoded` buffer (zeros, as bchk_sweep)
    countE = 0
    out = []
    stnr = 0.0
    while stnr <= max_snr:
        count = count_err = 0
        D = Cc = Ss = words = 0
        fer_est = 0.5
        while count < p and count_err < e:
            want = 2.0 * (e - count_err) / max(fer_est, 1e-7)
            nb = max(256, int(min(want / world, float(block))))
            total = min(world * nb, p - count)
            lo, hi = min(rank * nb, total), min((rank + 1) * nb, total)
            tx, res, acc, ops, states, st_after = source.block(stnr, state, lo, hi - lo)
            B = hi - lo
            acc = acc.astype(bool)
            # the buffer entering this block: the last accepted row of an earlier block of
            # this round, else the one carried from before the round
            last = np.flatnonzero(acc)
            mine = res[last[-1]] if len(last) else np.zeros(n, np.uint8)
            rows = comm.all_gather_u8(mine)
            flags = comm.all_gather_i64([1 if len(last) else 0, B])
            incoming = decoded
            for r in range(rank):
                if flags[r][0]:
                    incoming = rows[r]
            # each word's `decoded`: its own result if accepted, else the buffer as it stands
            idx = np.maximum.accumulate(np.where(acc, np.arange(B), -1)) if B else np.zeros(0, np.int64)
            eff = np.where((idx >= 0)[:, None], res[np.maximum(idx, 0)], incoming[None, :]) if B else res
            diff = tx != eff
            fe = diff.any(axis=1).astype(np.int64)
            be = diff.sum(axis=1).astype(np.int64)
            # where the point stops, in stream order over the blocks
            tot = comm.all_gather_i64([B, int(fe.sum())])
            c_run, e_run, stop_rank = count, count_err, -1
            for r in range(world):
                w_r, f_r = tot[r]
                if w_r and (c_run + w_r >= p or e_run + f_r >= e):
                    stop_rank = r
                    break
                c_run += w_r
                e_run += f_r
            take = 0  # words of my block before the stop (inclusive)
            if stop_rank < 0 or rank < stop_rank:
                take = B
            elif rank == stop_rank:
                cum = count_err + sum(tot[r][1] for r in range(rank)) + np.cumsum(fe)
                cnt = count + sum(tot[r][0] for r in range(rank)) + np.arange(1, B + 1)
                take = int(np.flatnonzero((cnt >= p) | (cum >= e))[0]) + 1
            sums = [take, int(fe[:take].sum()), int(be[:take].sum()), int(ops[:take, 0].sum()),
                    int(ops[:take, 1].sum()), int(ops[:take, 2].sum())]
            # the owner of the last consumed word hands on the engine state and the buffer
            owner = stop_rank if stop_rank >= 0 else max(r for r in range(world) if tot[r][0])
            handoff = [0] * 2
            if rank == owner and take:
                handoff = [int(states[take - 1]), 1]
            buf = eff[take - 1] if (rank == owner and take) else np.zeros(n, np.uint8)
            red = comm.all_reduce_i64(sums + handoff)
            buf = comm.all_gather_u8(buf)[owner]
            used, errs = red[0], red[1]
            count += used
            count_err += errs
            countE += red[2]
            D += red[3]
            Cc += red[4]
            Ss += red[5]
            words += used
            state = red[6]
            decoded = buf
            fer_est = max(1e-7, (errs + 1) / (used + 1))
        out.append(f"{_g(stnr)},{_g(count_err / count)},{_g(countE / count / n)},{_g(D / words)},"
                   f"{_g(Cc / words)},{_g(Ss / words)}\n")
        stnr += 0.5
    return "".join(out)
