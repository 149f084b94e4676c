#!/usr/bin/env python3
"""Throughput of the Kaneko BCH soft decoder on MI355X (one process per GPU).

A step = one pass of the hot path over one resident batch: Kaneko decode of B codewords
(libbchk search kernel) + FER/op counter reduction (+ one RCCL all-reduce of the 6
counters when N > 1). Inputs are the reference's own channel stream (minstd_rand0 +
libstdc++ distributions; rank r starts (2^31-2)/N draws after rank r-1 in it), generated on the host and resident in HBM
before timing. Weak scaling: every rank decodes its own B codewords.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--global-batch G]
    torchrun --nproc-per-node N bench.py --gpus N ...

`--gpus N` without a launcher (no WORLD_SIZE in the environment) starts the N rank processes
itself, before anything touches a GPU, and exits with their status; under torchrun `--gpus`
must equal the world size. `--batch B` is per rank (weak scaling, the default);
`--global-batch G` fixes the job's total instead (strong scaling: G / N codewords per rank),
which is how config 5's 2^20 words fit eight ranks' shares of the minstd_rand0 period.

Rank 0 prints one JSON line (driver contract) with `roofline` (HIP-event kernel time of
the dominant kernel vs the 8 TB/s HBM roof at 9n+8 algorithmic bytes per codeword),
`points` (the same measurement at each Eb/N0 of --points: the FER/throughput curve) and
`cpu_baseline` (the reference itself, compiled into oracle/_ref, one process per host core
on disjoint ranges of the same stream, on a bounded sample of the same workload).
"""
import argparse
import contextlib
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "tests"))



def metric_name(n, k, t, batch):
    """BASELINE.json's metric string for the code that actually ran (the default run gives
    exactly BASELINE's "codewords/s + FER vs Eb/N0, BCH(63,30,13) L=8 batch=2^20")."""
    b = f"2^{batch.bit_length() - 1}" if batch & (batch - 1) == 0 else str(batch)
    return f"codewords/s + FER vs Eb/N0, BCH({n},{k},{2 * t + 1}) L=8 batch={b}"


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: the launcher's world size, 1 without one")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--m", type=int, default=6)
    ap.add_argument("--t", type=int, default=6)
    ap.add_argument("--snr", type=float, default=5.0, help="Eb/N0 in dB (the headline point)")
    ap.add_argument("--points", default="4,5,6",
                    help="Eb/N0 points (dB) of the FER/throughput curve; '' = the headline only")
    ap.add_argument("--J", type=int, default=15, help="test-pattern cap; -1 = shipped (uncapped)")
    ap.add_argument("--batch", type=int, default=1 << 20, help="codewords per rank (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="codewords of the whole job, split evenly over the ranks (strong "
                         "scaling); 0 = --batch per rank")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target wall time of the cpu_baseline sample (0 = skip)")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="reference processes for the CPU baseline (0 = the host's core share)")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo: the "
                         "same exchange staged through the host, e.g. several ranks on one GPU)")
    ap.add_argument("--unfused", action="store_true",
                    help="decode_device + count_device (re-reads res and stats) instead of the fused call")
    return ap.parse_args()


def load_pkg():
    import importlib.util
    pkg = os.path.join(REPO, "polar-codes-with-bch-kernel_amd")
    spec = importlib.util.spec_from_file_location("bchk_amd", os.path.join(pkg, "__init__.py"),
                                                  submodule_search_locations=[pkg])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["bchk_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def dec_tmax(t):
    """TMAX bucket of the instantiated kernels (csrc/bchk_kernels.hip select_kernels)."""
    return t if t in (1, 2, 3, 6, 15) else next(b for b in (7, 8, 12, 16, 31, 32) if b >= t)


def rank_stream_start(bchk, seed, rank, world):
    """Rank r decodes draws [r D, r D + used) of the one reference stream (minstd_rand0 from
    `seed`), D = the engine period / world: a jump-ahead, so the ranks' inputs never overlap
    as long as every rank uses at most D draws (checked by check_rank_draws)."""
    D = bchk.MINSTD_PERIOD // world
    return bchk.rng_jump(seed, rank * D), D


def check_rank_draws(used, budget, world):
    if used > budget:
        raise SystemExit(f"rank stream overlap: one batch uses {used} engine draws, more than the "
                         f"{budget} per rank that {world} ranks leave in minstd_rand0's period 2^31-2; "
                         "use fewer codewords per rank")


def reduce_step(step_cnt, total_cnt, world, dist):
    """One FER exchange per step: the 6 counters of this step are summed over ranks (RCCL
    all-reduce over xGMI for the nccl backend; gloo on CPU in tests) and accumulated."""
    if world > 1:
        dist.all_reduce(step_cnt)
    total_cnt += step_cnt


def max_over_ranks(value, world, dist, device):
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_cores():
    """CPUs this process may use: its affinity set, capped by the job share the GPU box
    exports (OMP_NUM_THREADS = 16 there: os.cpu_count() is the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(share))) if share and share.isdigit() else max(1, n)


def cpu_baseline(args, gpu_rate, bchk):
    """The reference decode(answer, word, res) timed on the host's cores: one reference
    process per core, each on its own range of the reference stream (jump-ahead), same
    code/SNR/J; per-core and aggregate codewords/s."""
    if args.cpu_seconds <= 0:
        return None
    exe = os.path.join(REPO, "oracle", "_ref", "ref_golden_j15" if args.J == 15 else "ref_golden")
    kind = "reference"
    if args.J not in (15, -1) or not os.path.exists(exe):
        exe, kind = None, "port"
    # size the sample from a short probe so the whole leg takes ~cpu_seconds (long codes: a
    # heavy BCH(255) codeword costs the reference ~1 s at 5 dB, J = 15)
    probe = 2000 if args.m <= 6 else 64
    if exe:
        procs = args.cpu_procs or host_cores()

        def cmd(seed, count):
            return [exe, "bench", str(args.m), str(args.t), str(seed), str(count), repr(args.snr)]

        r = json.loads(subprocess.run(cmd(args.seed, probe), capture_output=True, text=True,
                                      check=True).stdout.strip().splitlines()[-1])
        count = int(max(probe, min(2_000_000, r["codewords_per_s"] * args.cpu_seconds)))
        span = bchk.MINSTD_PERIOD // procs  # disjoint stream ranges (>> count words' draws)
        ps = [subprocess.Popen(cmd(bchk.rng_jump(args.seed, i * span), count), stdout=subprocess.PIPE,
                               text=True) for i in range(procs)]
        t0 = time.perf_counter()
        outs = [json.loads(pp.communicate()[0].strip().splitlines()[-1]) for pp in ps]
        wall = time.perf_counter() - t0
        if any(pp.returncode for pp in ps):
            raise RuntimeError("reference baseline process failed")
        per_core = [o["codewords_per_s"] for o in outs]
        # aggregate: all words over the slowest process's decode time (generation excluded)
        rate = procs * count / max(o["seconds"] for o in outs)
        return {"value": round(rate, 3), "unit": "codewords/s", "cores": procs,
                "nproc": os.cpu_count(), "per_core": round(sum(per_core) / procs, 3),
                "per_core_min": round(min(per_core), 3), "kind": kind,
                "sample": f"{procs} reference processes x {count} codewords, each from its own "
                          f"range of the reference stream (seed {args.seed}, jump-ahead), "
                          f"Eb/N0={args.snr} dB, J={'inf' if args.J < 0 else args.J}, "
                          f"BCH({(1 << args.m) - 1}) t={args.t}; decode calls only; wall "
                          f"{wall:.1f} s incl. generation",
                "gpu_over_cpu": round(gpu_rate / rate, 1) if rate > 0 else None}
    else:
        from oracle_lib import Oracle
        o = Oracle(args.m, args.t)
        _, y = o.stream(args.seed, probe, args.snr)
        t0 = time.perf_counter()
        o.kaneko_batch(y, J=args.J)
        rate = probe / (time.perf_counter() - t0)
        count = int(max(probe, min(200_000, rate * args.cpu_seconds)))
        _, y = o.stream(args.seed, count, args.snr)
        t0 = time.perf_counter()
        o.kaneko_batch(y, J=args.J)
        rate, words = count / (time.perf_counter() - t0), count
    return {"value": round(rate, 3), "unit": "codewords/s", "cores": 1, "nproc": os.cpu_count(),
            "kind": kind,
            "sample": f"first {words} codewords of the reference stream (seed {args.seed}) at "
                      f"Eb/N0={args.snr} dB, J={'inf' if args.J < 0 else args.J}, BCH("
                      f"{(1 << args.m) - 1}) t={args.t}; decode calls only, 1 thread",
            "gpu_over_cpu": round(gpu_rate / rate, 1) if rate > 0 else None}


def run_point(args, bchk, dec, snr, world, rank, dist, dev):
    """One Eb/N0 point: the rank's batch generated into HBM, W warmup + K timed steps (max over
    ranks), per-kernel HIP-event durations from K more steps, FER/op counters."""
    import numpy as np
    import torch

    n, B = dec.n, args.batch
    start, budget = rank_stream_start(bchk, args.seed, rank, world)
    t_gen = time.perf_counter()
    tx, y, _, used = dec.generate_draws(snr, B, state=start)
    t_gen = time.perf_counter() - t_gen
    check_rank_draws(used, budget, world)
    d_y = torch.from_numpy(y).to(dev)
    d_tx = torch.from_numpy(tx).to(dev)
    del tx, y
    d_res = torch.zeros((B, n), dtype=torch.uint8, device=dev)
    d_l0 = torch.empty(B, dtype=torch.float64, device=dev)
    d_st = torch.empty((B, bchk.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    d_step = torch.zeros(6, dtype=torch.int64, device=dev)
    d_cnt = torch.zeros(6, dtype=torch.int64, device=dev)
    cuda = dev.type == "cuda"  # cpu only under BCHK_BENCH_STUB (plumbing tests)
    stream = torch.cuda.ExternalStream(dec.stream, device=dev) if cuda else None

    def on_stream():
        return torch.cuda.stream(stream) if cuda else contextlib.nullcontext()

    def device_sync():
        if cuda:
            torch.cuda.synchronize()

    device_sync()

    def step():
        # everything below is enqueued on the decoder's stream (torch ops via ExternalStream)
        if world == 1 and not args.unfused:
            # one GPU: the fused call adds this step's counters straight into the totals
            # (bchk_decode_count_device accumulates), no separate zero / add launches
            dec.decode_count_device(d_y.data_ptr(), d_tx.data_ptr(), B, d_res.data_ptr(), d_l0.data_ptr(), 0,
                                    d_cnt.data_ptr(), dec.stream)
            return
        d_step.zero_()
        if args.unfused:  # decode, then the counters from a re-read of res / stats
            dec.decode_device(d_y.data_ptr(), B, d_res.data_ptr(), d_l0.data_ptr(), d_st.data_ptr(),
                              dec.stream)
            dec.count_device(d_tx.data_ptr(), d_res.data_ptr(), d_st.data_ptr(), B, d_step.data_ptr(),
                             dec.stream)
        else:  # counters fused into the decode kernels (no per-codeword stats stored)
            dec.decode_count_device(d_y.data_ptr(), d_tx.data_ptr(), B, d_res.data_ptr(), d_l0.data_ptr(), 0,
                                    d_step.data_ptr(), dec.stream)
        reduce_step(d_step, d_cnt, world, dist)

    with on_stream():
        for _ in range(args.warmup):
            step()
        dec.sync()
        d_cnt.zero_()
        dec.sync()
        if world > 1:
            dist.barrier()
        device_sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        dec.sync()
        device_sync()
        elapsed = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        # per-kernel durations: the same steps again with HIP events around every launch
        # (outside the timed region, so event records do not perturb `value`)
        dec.profile(True)
        for _ in range(args.steps):
            step()
        dec.sync()
        device_sync()
    ms4, launches = dec.profile_read_stages()  # fast, exact first pass, coop, analytic tail
    dec.profile(False)
    # FER / op counters of the batch itself: every step re-decodes the same resident words,
    # so the counts come from ONE more step on zeroed counters (world * B distinct words)
    with on_stream():
        dec.sync()
        d_cnt.zero_()
        dec.sync()
        step()
        dec.sync()
        device_sync()
    n_exact, n_coop = dec.path_counts()
    n_tail = dec.tail_count()
    tail_stats = dec.tail_stats()
    elapsed = max_over_ranks(elapsed, world, dist, dev)
    cnt = d_cnt.cpu().numpy().astype(np.int64)  # one pass over the batch, summed over ranks (N > 1)
    # every word counted once -- unless an experiment library that cuts a kernel short (it
    # finishes no word; scripts/gpu_first_cut.sh) is loaded instead of the product libbchk.so:
    # then the record says so (counters_complete false), it cannot pass as a result
    complete = int(cnt[5]) == world * B
    cut_build = os.path.basename(bchk.LIB_PATH) != "libbchk.so" and bool(os.environ.get("BCHK_CUT_BUILD"))
    assert complete or cut_build, "counters must cover every word once"
    total_words = world * B * args.steps
    value = total_words / elapsed
    # Algorithmic bytes per codeword: 8n B of f64 samples in, n B decoded bits and 8 B l0
    # out (9n + 8, the roofline's `achieved`); the fused step also reads the
    # n-B sent word for its counters (10n + 8, reported beside it as `achieved_fused`).
    # The fast kernel moves them for all B codewords; the exact, tail and cooperative
    # kernels re-read/write them for the codewords handed to them.
    bytes_per_cw = 9 * n + 8
    bytes_fused = bytes_per_cw + (0 if args.unfused else n)
    launches = max(1, launches)
    tm = dec_tmax(args.t)
    # the lane-per-codeword fast kernel exists for n <= 63 and small t (csrc/bchk_fast.hip
    # select_fast); without it stage 0 is only the control-block memset
    # (n > 63: kaneko_first_kernel, the first test patterns of every codeword)
    has_fast = args.m >= 7 or args.t <= {3: 3, 4: 7, 5: 8, 6: 6}.get(args.m, -1)
    # n <= 63: the ring kernel serves calls without a stats record where the 16-key selection
    # covers the decision (csrc/bchk_fast.hip launch_fast_impl), else the staged kernel
    ring = (min(2 * tm, n - 1) + 2 <= 16 and not args.unfused and os.environ.get("BCHK_FAST_RING", "1") != "0")
    # n > 63, t <= 15 (m = 7: TMAX 8): the lane pre-pass decides the rows that return at test
    # pattern 0 or 1, the first kernel the others (stage 0 = both launches)
    lane = (args.m == 8 and tm <= 15) or (args.m == 7 and tm <= 8)
    lane = lane and os.environ.get("BCHK_LANE_PRE", "1") != "0"
    tsuf = f"<{args.m},{tm}>"
    fast_name = (("kaneko_fast_ring_kernel" if ring else "kaneko_fast_kernel") + tsuf if args.m <= 6
                 else (f"kaneko_lane_kernel{tsuf} + kaneko_first_kernel{tsuf}" if lane else "kaneko_first_kernel" + tsuf))
    fast_on = has_fast and ms4[0] > 0 and n_exact < B
    # per launch: average duration (HIP events on the launching stream) and the codewords
    # one launch processes
    kern = [{"name": fast_name if has_fast else "control memset",
             "ms": ms4[0] / launches, "codewords": B if has_fast else 0},
            {"name": f"kaneko_search_kernel<{args.m},{tm}>", "ms": ms4[1] / launches,
             "codewords": n_exact if fast_on else B},
            {"name": f"kaneko_search_kernel<{args.m},{tm}> analytic tail", "ms": ms4[3] / launches,
             "codewords": n_tail},
            {"name": f"kaneko_coop_kernel<{args.m},{tm}>", "ms": ms4[2] / launches,
             "codewords": n_coop}]
    for k in kern:
        k["GB_s"] = (bytes_per_cw * k["codewords"] / (k["ms"] / 1e3) / 1e9) if k["ms"] > 0 else 0.0
        k["GB_s_fused"] = (bytes_fused * k["codewords"] / (k["ms"] / 1e3) / 1e9) if k["ms"] > 0 else 0.0
    dom = max(kern, key=lambda k: k["ms"])
    words = int(cnt[5])
    return {
        "snr_db": snr, "value": value, "ms_per_step": elapsed / args.steps * 1e3,
        "fer": (int(cnt[0]) / words) if words else None,
        "ber": (int(cnt[1]) / words / n) if words else None,
        "frame_errors": int(cnt[0]), "words": words, "counters": [int(c) for c in cnt],
        "decodes_per_codeword": (int(cnt[2]) / words) if words else None,
        "kernels": [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in kk.items()} for kk in kern],
        "dominant_kernel": dom["name"], "dominant_GB_s": dom["GB_s"],
        "dominant_GB_s_fused": dom["GB_s_fused"], "bytes_per_codeword": bytes_per_cw,
        "bytes_per_codeword_fused": bytes_fused, "counters_complete": complete, "cut_build": cut_build,
        "frac": dom["GB_s"] / HBM_PEAK_GBS,
        "kernel_ms_per_step": sum(k["ms"] for k in kern),
        "tail": {"to_tail": n_tail, "finished": tail_stats[1], "split": tail_stats[2],
                 "handed_on": tail_stats[0], "split_chunks": tail_stats[3],
                 "enum_steps_max": tail_stats[5]},
        "host_generation_s": t_gen, "rank_draws": used, "rank_draw_budget": budget,
    }


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n_ranks, argv):
    """`bench.py --gpus N` run directly: start the N rank processes here (the torchrun
    environment: RANK / LOCAL_RANK / WORLD_SIZE, rendezvous on 127.0.0.1), wait for them and
    return the job's exit status. Called before anything in this process touches a GPU; the
    children are ordinary child processes (no exec), rank 0 prints the JSON line. A rank that
    fails ends the others (by their own PIDs) so the job cannot hang on a dead peer."""
    port = str(free_port())
    procs = []
    for r in range(n_ranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n_ranks),
                   LOCAL_WORLD_SIZE=str(n_ranks), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, BCHK_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def rank_batch(args, world):
    """Codewords this rank decodes per step: --batch (weak scaling) or --global-batch / N
    (strong scaling; the total must split evenly)."""
    if args.global_batch:
        if args.global_batch % world:
            raise SystemExit(f"--global-batch {args.global_batch} does not split over {world} ranks")
        return args.global_batch // world, "strong"
    return args.batch, "weak"


def main():
    args = parse()
    launched = "WORLD_SIZE" in os.environ
    if args.gpus is not None and args.gpus > 1 and not launched:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started {world} ranks")
    args.batch, scaling = rank_batch(args, world)
    import torch
    import torch.distributed as dist

    bchk = load_pkg()
    stub = os.environ.get("BCHK_BENCH_STUB")
    if stub:
        # CPU plumbing tests only (tests/test_bench_spawn.py): the oracle stands in for the
        # device decoder so the rank launch, stream ranges and counter exchange run without a
        # GPU; the line says so and is no measurement
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from bench_stub import StubDecoder
        if args.backend != "gloo":
            raise SystemExit("BCHK_BENCH_STUB runs on the CPU: --backend gloo")
        gpu, dev = None, torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
        dec = StubDecoder(args.m, args.t, J=args.J)
    else:
        # one rank per GPU; more ranks than GPUs (a rehearsal of the N > 1 path on one GPU,
        # gloo only: RCCL refuses two ranks on one device) share them round-robin
        ndev = max(1, torch.cuda.device_count())
        if world > ndev and args.backend == "nccl":
            raise SystemExit(f"{world} ranks on {ndev} GPUs: nccl (RCCL) needs one GPU per rank; "
                             "--backend gloo rehearses several ranks per GPU")
        gpu = local % ndev
        torch.cuda.set_device(gpu)
        if world > 1:
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
            else:
                dist.init_process_group("gloo")
        dec = bchk.KanekoKernelProcessor(args.m, args.t, J=args.J, device=gpu)
        dev = torch.device("cuda", gpu)
    n, B = dec.n, args.batch
    snrs = [float(x) for x in args.points.split(",") if x.strip()] if args.points else []
    if args.snr not in snrs:
        snrs.append(args.snr)
    pts = {snr: run_point(args, bchk, dec, snr, world, rank, dist, dev) for snr in sorted(snrs)}
    head = pts[args.snr]
    dom = next(k for k in head["kernels"] if k["name"] == head["dominant_kernel"])
    # HBM bytes per launch of the dominant kernel, from the committed PMC passes of the same
    # workload (scripts/gpu_final6.sh -> scripts/traffic_req_json.py, rocprofv3 --pmc memory-
    # side requests by size); null when no profile of this workload exists. It is a stored
    # measurement (rocprofv3 cannot run inside this process): its source is named. A stage of
    # two launches (lane pre-pass + first kernel) sums both.
    traffic, traffic_src, traffic_read = None, None, None
    if os.path.exists(args.traffic):
        try:
            tr = json.load(open(args.traffic))
            if tr.get("batch") == B and tr.get("snr_db") == args.snr and tr.get("J") == args.J:
                names = [k.replace(" ", "") for k in dom["name"].split(" + ")]
                parts = [tr.get("kernels", {}).get(k) for k in names]
                traffic = None if any(v is None for v in parts) else sum(parts)
                rparts = [tr.get("read_bytes", {}).get(k) for k in names]
                traffic_read = None if any(v is None for v in rparts) else sum(rparts)
                traffic_src = f"{tr.get('source')} ({tr.get('date', 'undated')})"
        except Exception:
            traffic = None
    if rank == 0:
        out = {
            "metric": metric_name(n, dec.k, args.t, world * B if scaling == "strong" else B),
            "value": round(head["value"], 3),
            "unit": "codewords/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(head["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: the reference's AWGN stream (minstd_rand0 + libstdc++ "
                    "distributions), BPSK, generated on host, resident in HBM; rank r decodes "
                    "its own jump-ahead range of the one stream",
            "config": {"workload": f"Kaneko ML soft decoding of BCH({n},{dec.k},{2 * args.t + 1}), "
                                   f"Eb/N0={args.snr} dB, J={'inf' if args.J < 0 else args.J}",
                       "code": f"BCH({n},{dec.k},{2 * args.t + 1})", "batch_per_gpu": B,
                       "global_batch": world * B, "snr_db": args.snr, "J": args.J,
                       "L_inert": 8, "parallelism": f"dp{world}",
                       "launch": ("bench.py --gpus" if os.environ.get("BCHK_BENCH_SPAWNED") else
                                  "torchrun" if launched else "single"),
                       "backend": args.backend if world > 1 else None},
            "fer": head["fer"],
            "ber": head["ber"],
            "decodes_per_codeword": head["decodes_per_codeword"],
            "kernels": head["kernels"],
            "dominant_kernel": head["dominant_kernel"],
            "kernel_ms_per_step": round(head["kernel_ms_per_step"], 4),
            "roofline": {"bound": "hbm", "achieved": round(head["dominant_GB_s"], 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(head["frac"], 6), "traffic": traffic,
                         "traffic_source": traffic_src,
                         # its HBM reads against the inputs it streams: the rows (8n B per
                         # codeword) and, in the fused step, the sent words (n B)
                         "traffic_read": traffic_read,
                         "read_over_inputs": (round(traffic_read / ((8.0 * n + (0 if args.unfused else n)) * B), 4)
                                              if traffic_read else None),
                         "bytes_per_codeword": head["bytes_per_codeword"],
                         "achieved_fused": round(head["dominant_GB_s_fused"], 3),
                         "frac_fused": round(head["dominant_GB_s_fused"] / HBM_PEAK_GBS, 6),
                         "bytes_per_codeword_fused": head["bytes_per_codeword_fused"]},
            "points": [{"snr_db": p["snr_db"], "value": round(p["value"], 3),
                        "ms_per_step": round(p["ms_per_step"], 4), "fer": p["fer"],
                        "frame_errors": p["frame_errors"], "words": p["words"],
                        "counters": p["counters"], "decodes_per_codeword": p["decodes_per_codeword"],
                        "dominant_kernel": p["dominant_kernel"], "frac": round(p["frac"], 6),
                        "kernels": p["kernels"], "tail": p["tail"]} for p in pts.values()],
            "tail": head["tail"],
            "host_generation_s": round(head["host_generation_s"], 2),
            "counters_complete": head["counters_complete"],
            **({"cut_build": True} if head["cut_build"] else {}),
            **({"stub_decoder": "tests/bench_stub.py (CPU oracle, plumbing test; not a measurement)"}
               if stub else {}),
            "rank_draws": head["rank_draws"], "rank_draw_budget": head["rank_draw_budget"],
        }
        if world == 1 and not stub:
            out["cpu_baseline"] = cpu_baseline(args, head["value"], bchk)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
