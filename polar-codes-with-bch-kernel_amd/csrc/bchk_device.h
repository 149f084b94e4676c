// bchk_device.h -- structures shared by the host runtime (bchk_host.cpp) and the gfx950
// kernels (bchk_kernels.hip). Plain C++, no HIP types.
#pragma once
#include <stdint.h>

#include "bchk.h"
#include "bchk_syndtab.h"

namespace bchk {

constexpr int kMaxM = 8;
constexpr int kMaxT = 32;
constexpr int kWaveSize = 64;
constexpr int kWavesPerBlock = 4;
constexpr uint32_t kEmptySlot = 0xFFFFFFFFu;
// fault bits (SearchParams::fault)
constexpr uint32_t kFaultHeavySlot = 1u, kFaultHeavyWait = 2u, kFaultTailSlot = 4u, kFaultTailWait = 8u,
                   kFaultCoopRing = 16u;

// Per-code lookup tables, one device blob, copied into LDS by every workgroup.
//   exp8 [2n]        alpha^i for i < 2n-1, exp8[2n-1] = 0 (log sums are clamped to
//                    2n-1 = log(0), bchk_core.h gf_exp2); m >= 7: [4n], zero from 2n-1 on
//                    (any sum of two logs in [0, n) or 2n-1 indexes it, no clamp)
//   log16[2^m]       log_alpha(v); log16[0] = 2n-1
//   col  [n][W]      odd-syndrome column of position p: byte j of word j/4 =
//                    alpha^((2j+1) p mod n), j < t   (Decoder::alterSyndromPoly :210-230)
//   chien[t+1][2][m][8] (m <= 6 only) bit-planes of v * alpha^(j k) over k = 0..n-1:
//                    the Chien search of Decoder::locatorsAndRoots (:279-296) as a
//                    GF(2)-linear map. v splits into its low and high 3-bit halves
//                    (v = lo + 8 hi), each indexing an 8-entry table per (j, plane b):
//                    rows of 8 u64 = 16 LDS banks, so lanes never conflict.
struct TableDesc {
    uint32_t off_exp, off_log, off_col, off_chien, bytes;
    int32_t W;   // u32 words per packed odd-syndrome vector
    int32_t EW;  // unused (kept for the struct layout)
};

// A codeword's search state where the exact first pass hands it to the analytic tail
// kernel, which resumes from it (no exact chunk decoded twice).
struct TailRec {
    double l0;
    uint64_t bound, jsteps, impr, best;
    int32_t T, m0;
    uint32_t chunks, flags;  // flags: 1 firstOK, 2 accepted
};

struct SearchParams {
    const double *y;       // [B][n]
    uint8_t *res;          // [B][n]
    double *l0;            // [B] or null
    bchk_stats *st;        // [B] or null
    const uint8_t *tables; // device blob, TableDesc layout
    TableDesc td;
    double s2;             // pow(sd0, 2), host glibc (src/KanekoKernelProcessor.cpp:337)
    uint64_t max_decodes;  // 0 = unlimited
    uint32_t count;        // codewords
    // slow-path work queue (null = process codewords [0, count) in place):
    //   queue[0 .. *qcount) codeword indices, dequeued through 8 per-XCD heads
    //   heads[32 * x] (one 128-B line each), zeroed before the launch.
    const uint32_t *queue;
    const uint32_t *qcount;
    uint32_t *heads;
    uint32_t *qtail;       // fast path: append unresolved codewords here (with queue_out)
    uint32_t *queue_out;
    // fast path, two-ended queue (null: all at the front): codewords likely to be heavy
    // (the hard decision does not decode) take slots 0, 1, ... (qfront), the others slots
    // count-1, count-2, ... (qback); *qtail stays the total. The first pass reads items
    // below *qfront_n from the front, the rest from the back, so it starts the likely heavy
    // codewords first and hands them to a concurrent tail kernel early.
    uint32_t *qfront;
    uint32_t *qback;
    const uint32_t *qfront_n;
    // long codes (m >= 7): the lane pre-pass (kaneko_lane_kernel) sets bit k of word c when
    // it finished codeword 64 c + k; kaneko_first_kernel skips those (null: no pre-pass)
    uint64_t *pre_mask;
    // its hard-decision syndrome table: [ceil(n/8)][256][W] words, entry (j, v) = the
    // syndrome of byte value v at positions 8j .. 8j + 7
    const uint32_t *syn8;
    // m >= 7: GF(2^m) products [2^m][2^m] then inverses [2^m] (bytes), which the
    // cooperative kernel stages into LDS for its decoders (GfMul, bchk_core.h)
    const uint8_t *gfmul;
    // heavy codewords: the wave kernel hands a codeword still running after chunk_limit
    // steps of 64 patterns to the cooperative kernel, which may run concurrently with it
    // (heavy_tail == null disables the hand-off). Longest-first: codewords whose loop bound
    // at the hand-off is >= heavy_big go to the front queue (slots 0, 1, ...), the others to
    // the back queue (slots count-1, count-2, ...). A producer reserves a slot with its
    // tail, then stores the codeword index; empty slots hold kEmptySlot, and consumers
    // (who reserve with the heads) put it back, so the array stays clean between calls.
    // exact_done counts the codewords the wave kernel has finished or handed off; once it
    // reaches *exact_total (null: count) the tails are final.
    uint32_t *heavy_queue;
    uint32_t *heavy_tail;
    uint32_t *heavy_tail2;
    uint32_t *heavy_head;
    uint32_t *heavy_head2;
    uint32_t *exact_done;
    const uint32_t *exact_total;
    uint64_t heavy_big;
    uint32_t chunk_limit;
    // diagnostic builds only (-DBCHK_DIAG): per heavy-queue item, 8 u64 timing counters
    unsigned long long *diag;
    uint32_t *diag_count;
    // syndrome-indexed decoding table (bchk_syndtab.h) for the search kernels' test
    // patterns; slots == null: Berlekamp-Massey + Chien
    SyndTable tab;
    int32_t t;
    int32_t J;             // < 0: shipped
    int32_t variant;       // BCHK_VARIANT_*
    // search kernel: after chunk_limit exact chunks, finish the codeword from its candidate
    // codewords (bchk_kernels.hip, analytic tail) instead of handing it off; 0 = hand off
    int32_t analytic;
    // analytic tail kernel: waves of a block whose queue is exhausted help a sibling decode
    // the exact chunks of a split codeword (bchk_kernels.hip, HelpCtl); 0 = off
    int32_t an_help;
    // analytic tail outcomes (null = not counted): [0] handed on to the cooperative kernel,
    // [1] finished from the candidates, [2] split (exact chunks, then the candidates),
    // [3] exact chunks of the splits
    uint32_t *tail_stats;
    // diagnostics: per codeword through the analytic tail, 8 u64 (codeword, cycles of prep,
    // exact chunks, plan, enumeration steps, mode | why << 8 | split chunks << 16, cycles
    // after the plan, decodes); null = off
    // first pass -> analytic tail: the state of each hand-off, by its queue slot (null = the
    // tail kernel starts codewords from scratch)
    TailRec *tail_rec;
    // the analytic tail kernel's input when it runs concurrently with the first pass (null:
    // the static queue/qcount above): slots in_queue[k] (kEmptySlot until stored), the
    // producer's tail, this kernel's ticket counter, the producer's 8 per-XCD done counts
    // and their final total (null: count)
    uint32_t *in_queue;
    const uint32_t *in_tail;
    uint32_t *in_head;
    const uint32_t *in_done;
    const uint32_t *in_total;
    unsigned long long *tail_diag;
    uint32_t *tail_diag_count;
    uint32_t tail_diag_cap;
    // sticky per-context fault word (null = off): a bounded queue wait that ran out sets a
    // bit (kFault*), since its codeword is then not finished; bchk_sync / the host decode
    // calls report it as BCHK_EHIP and clear it
    uint32_t *fault;
    // FER/BER/op counters fused into the decode (null = off): every kernel that finishes a
    // codeword compares its row with the sent word tx [B][n] and adds {frame errors, bit
    // errors, decodes, comparisons, sums, words} to the partial counters
    // cnt[kCntSlots][kCntStride] (slot by codeword, spreading the atomics), which
    // cnt_reduce_kernel folds into the caller's totals
    const uint8_t *tx;
    unsigned long long *cnt;
    // fast ring kernel (bchk_fast.hip): waves per workgroup (0: all 16 -- 1 loader + 15
    // compute; fewer leave room for a concurrent kernel), and experiment modes (0: normal;
    // 1: the loader publishes slots without loading them, 2: compute waves only read their
    // slot -- timing builds of the two halves, wrong results; 3: the slot held through the
    // i = 0 tests, 6: flipped positions' values all re-read from HBM -- correct, slower or
    // more bytes, measured)
    uint32_t fast_waves;
    uint32_t fast_mode;
    uint32_t heavy_t;  // fast path: estimated loop-bound exponent sending an ok0 codeword to the front (0: kHeavyT)
    uint32_t heavy_tmax;  // ... and at most this one (0: no upper limit; experiments)
    // cooperative kernel, m >= 7: candidate records a ring slot keeps (0..2; a chunk with more
    // is decoded again densely on the acceptor's request), and its counters (null = off):
    // [0] dense re-decodes served, [1] heavy codewords started
    int32_t long_rec;
    uint32_t *coop_stats;
    // cooperative kernel, m >= 7: cross-workgroup help (null: off). Workgroup b's codeword
    // is job b: its control line (jobctl, 128 B each, zeroed per launch) and its data
    // (jobs, KernelSet::long_job_bytes each: result tags and records, the prep tables).
    // Workgroups left without a heavy codeword decode chunks of the published ones.
    void *long_jobctl;     // [gridDim + 1] lines: the last one counts the workgroups owning a codeword
    void *long_jobs;
    uint32_t long_epoch;      // launch count (the high bits of the jobs' tag generations)
    uint32_t long_help_max;   // helpers per job (0: kHelpersMax)
    uint32_t long_share_min;  // chunks left for a job to be offered (0: kShareMinChunks)
};
constexpr int kCntSlots = 512;
constexpr int kCntStride = 16;  // u64 per slot: one 128-B line

// on-GPU channel (bchk_channel.hip): words [word0, word0 + count) of the counter-based
// stream `seed`: tx [count][n] (0/1), y [count][n] = BPSK(tx) + N(0, sd)
struct ChanParams {
    uint8_t *tx;
    double *y;
    uint64_t word0;
    uint32_t count;
    int32_t n, k;
    uint32_t seed_lo, seed_hi;
    double sd;
    uint64_t g[4];  // generator polynomial, bit j = coefficient of x^j
};

struct AlgParams {
    const uint8_t *words;   // [N][n]
    const uint32_t *synd;   // [N][t] or null
    uint8_t *answers;       // [N][n]
    uint8_t *ok;            // [N]
    const uint8_t *tables;
    TableDesc td;
    uint32_t count;
    int32_t t;
};

}  // namespace bchk
