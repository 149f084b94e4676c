// bchk_fast.hip -- lane-per-codeword fast path of the Kaneko search (n <= 63).
//
// At the SNRs where the decoder is used, most codewords leave the reference loop
// (src/KanekoKernelProcessor.cpp:361-405) through `l < calcRightSide()` at test pattern
// i = 0 (the hard decision lies within t of a codeword) or i = 1 (the hard decision is a
// codeword: its zero syndrome fails, flipping the least reliable bit succeeds). This kernel
// gives every lane its own codeword and decides exactly those two cases:
//   - the row is staged through LDS in 8-position slices (coalesced 8-B loads), each lane
//     builds 32-bit sort keys (26-bit monotone prefix of |y|, 6-bit position) and sorts
//     them with a 64-key bitonic network in registers;
//   - distinct prefixes order alpha = |2y/s2| exactly; a prefix tie within the sorted
//     prefix calcRightSide can touch (2t+1 entries) sends the codeword to the exact slow
//     path; calcL sums exact alphas (IEEE f64 division of the samples at the flipped
//     positions, gathered on demand); calcRightSide is bounded below from the keys alone;
//   - decodes i = 0 and i = 1 run per lane (binary BM + Chien table);
//   - calcL / calcRightSide are summed in the reference's order.
// Codewords not resolved here (no early return at i <= 1, or any doubt) are appended to a
// queue that the wave-per-codeword kernel (bchk_kernels.hip) processes from scratch, so
// every result is the reference's.
#include <algorithm>
#include <cstdlib>

#include "bchk_core.h"
#include "bchk_launch.h"

namespace bchk {

namespace {
constexpr int kRowD = 9;  // doubles per staged row slice (8 + 1 pad: conflict-free b64)
constexpr int kSlice = 8;
constexpr int kFastWaves = 8;  // waves per persistent block
constexpr int kStageBytes = 64 * kRowD * 8;
}  // namespace

// Ascending compare-exchange of key[I], key[J] (static indices: stays in registers).
#define BCHK_CAS(I, J)                                                  \
    {                                                                   \
        const uint32_t a_ = key[I], b_ = key[J];                        \
        key[I] = a_ < b_ ? a_ : b_;                                     \
        key[J] = a_ < b_ ? b_ : a_;                                     \
    }

// Sort of key[O .. O+16), ascending: Green's 60-comparator network (10 layers; checked on
// all 2^16 zero-one inputs), 20 compare-exchanges fewer than the bitonic one.
__device__ constexpr uint8_t kGreen16[60][2] = {
    {0, 13}, {1, 12}, {2, 15}, {3, 14}, {4, 8},  {5, 6},  {7, 11}, {9, 10},
    {0, 5},  {1, 7},  {2, 9},  {3, 4},  {6, 13}, {8, 14}, {10, 15}, {11, 12},
    {0, 1},  {2, 3},  {4, 5},  {6, 8},  {7, 9},  {10, 11}, {12, 13}, {14, 15},
    {0, 2},  {1, 3},  {4, 10}, {5, 11}, {6, 7},  {8, 9},  {12, 14}, {13, 15},
    {1, 2},  {3, 12}, {4, 6},  {5, 7},  {8, 10}, {9, 11}, {13, 14},
    {1, 4},  {2, 6},  {5, 8},  {7, 10}, {9, 13}, {11, 14},
    {2, 4},  {3, 6},  {9, 12}, {11, 13},
    {3, 5},  {6, 8},  {7, 9},  {10, 12},
    {3, 4},  {5, 6},  {7, 8},  {9, 10}, {11, 12},
    {6, 7},  {8, 9}};
template <int O>
__device__ __forceinline__ void sort16(uint32_t *key) {
#pragma unroll
    for (int c = 0; c < 60; ++c) BCHK_CAS(O + kGreen16[c][0], O + kGreen16[c][1])
}

// key[A..A+16) and key[B..B+16) sorted -> key[A..A+16) = the 16 smallest of both, sorted:
// min(A_i, B_15-i) is bitonic, then a bitonic merge.
template <int A, int B>
__device__ __forceinline__ void merge_low16(uint32_t *key) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t a = key[A + i], b = key[B + 15 - i];
        key[A + i] = a < b ? a : b;
    }
#pragma unroll
    for (int j = 8; j > 0; j >>= 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (!(i & j)) BCHK_CAS(A + i, A + i + j)
    }
}

// 32-bit sort key: a monotone 26-bit prefix of |y| (5 exponent bits covering
// [2^-27, 2^5) + 21 mantissa bits) above the 6-bit position. |y| below the range maps to
// prefix 0 or 1, above it (and inf/NaN) to the all-ones prefix; both are detected after the sort.
// Five VALU operations: the biased exponent minus 996 saturates at 0 (|y| < 2^-27 then gives
// prefix 0 or 1 -- the lo word's top bit -- and prefixes <= 1 are sent to the slow path), the
// funnel shift appends the 21st mantissa bit, and the min saturates |y| >= 32 / inf / NaN.
__device__ __forceinline__ uint32_t sort_key(uint32_t hi, uint32_t lo, int pos) {
    const uint32_t ahi = hi & 0x7FFFFFFFu;
    const uint32_t d = __builtin_elementwise_sub_sat(ahi, (uint32_t)(1023 - 27) << 20);
    const uint32_t mid = __builtin_amdgcn_alignbit(d, lo, 31);  // (d:lo) >> 31 = d << 1 | lo >> 31
    const uint32_t pre = mid < 0x3FFFFFFu ? mid : 0x3FFFFFFu;
    return (pre << 6) | (uint32_t)pos;
}

// Blocks of kFastWaves waves, one 64-codeword chunk per wave: the code tables are staged
// into LDS once per 512 codewords, and two blocks per CU give 4 waves per SIMD (<= 128
// VGPRs; the kernel is latency-bound, so occupancy wins).
// SEL (no per-codeword stats requested, 2 TMAX + 2 <= 16): only the 16 smallest keys are
// put in order (four sorted groups of 16, then low-half merges) -- the fast-path exits read
// ranks 0..2t and the least reliable position, so an exact tie beyond rank 2t + 1 cannot
// change a result, only the BCHK_F_TIE flag of the stats record; SEL = false sorts all 64
// keys and sends any tie to the exact path, so the flags match it.
template <int M, int TMAX, bool SEL>
__global__ void __launch_bounds__(kWaveSize * kFastWaves, 4)
kaneko_fast_kernel(SearchParams p) {
    constexpr int N = Geo<M>::N;
    static_assert(N <= 63, "fast path covers n <= 63");
    constexpr int W = (TMAX + 3) / 4;
    // calcRightSide takes the first border = 2t+1-m agreeing sorted positions; with m0 == m
    // (both fast-path exits) and m positions disagreeing, they lie within ranks 0..2t (KMAX).
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    load_tables(smem, p.tables, p.td.bytes);
    __syncthreads();
    const uint8_t *ex = smem + p.td.off_exp;
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(smem + p.td.off_log);
    const uint32_t *col = reinterpret_cast<const uint32_t *>(smem + p.td.off_col);
    const uint64_t *chien = reinterpret_cast<const uint64_t *>(smem + p.td.off_chien);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double *stage = reinterpret_cast<double *>(smem + ((p.td.bytes + 15) & ~15u) + wid * kStageBytes);
    const uint32_t cw0 = (blockIdx.x * kFastWaves + wid) * 64u;
    if (cw0 >= p.count) return;
    // experiment (BCHK_FAST_STAGGER): the first round's second block on each CU starts
    // p.fast_stagger cycles late, so the CU's two blocks load and compute out of phase
    if (p.fast_stagger && blockIdx.x >= p.fast_blocks / 2 && blockIdx.x < p.fast_blocks) {
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        while (__builtin_amdgcn_s_memtime() - t0 < p.fast_stagger) __builtin_amdgcn_s_sleep(8);
    }
    const uint32_t cw = cw0 + (uint32_t)lane;
    const bool live = cw < p.count;
    const int t = p.t;
    (void)M;
    const double s2 = p.s2;
    const double *yrow = p.y + (size_t)(live ? cw : cw0) * N;
    static_assert(64 * N + 256 <= kStageBytes, "output block and row errors fit the stage");

#ifdef BCHK_DIAG
    // stamps: [0] stage+keys, [1] sort, [2] S0, [3] decode i=0 + accept, [4] i=1, [5] outputs
    unsigned long long dg[6], tp = __builtin_amdgcn_s_memtime();
#define BCHK_STAMP(i)                                          \
    {                                                          \
        const unsigned long long tn = __builtin_amdgcn_s_memtime(); \
        dg[i] = tn - tp;                                       \
        tp = tn;                                               \
    }
#else
#define BCHK_STAMP(i)
#endif
    // ---- stage rows, build keys and the hard decision yH = (2y/s2 > 0) (:336-342).
    // Slice loads run kAhead slices ahead of the slice being turned into keys, so a wave
    // waits for one memory round trip instead of one per slice.
    const uint32_t last_row = p.count - 1u - cw0;  // rows past the batch end clamp (unused)
    constexpr int NS = (N + kSlice - 1) / kSlice;
    constexpr int kAhead = 2;
    uint32_t key[64];
    uint32_t yHl = 0, yHh = 0;
    double v[kAhead + 1][kSlice];
    auto load_slice = [&](int c, double *dst) {
#pragma unroll
        for (int it = 0; it < kSlice; ++it) {
            const int flat = it * 64 + lane;
            const uint32_t r = (uint32_t)(flat >> 3);
            const int pos = kSlice * c + (flat & 7);
            const uint32_t rr = r < last_row ? r : last_row;
            dst[it] = p.y[(size_t)(cw0 + rr) * N + (pos < N ? pos : N - 1)];
        }
    };
#pragma unroll
    for (int c = 0; c < kAhead && c < NS; ++c) load_slice(c, v[c]);
#pragma unroll
    for (int c = 0; c < NS; ++c) {
        if (c + kAhead < NS) load_slice(c + kAhead, v[(c + kAhead) % (kAhead + 1)]);
#pragma unroll
        for (int it = 0; it < kSlice; ++it) {
            const int flat = it * 64 + lane;
            stage[(flat >> 3) * kRowD + (flat & 7)] = v[c % (kAhead + 1)][it];
        }
        wave_sync();
#pragma unroll
        for (int k = 0; k < kSlice; ++k) {
            const int pos = kSlice * c + k;
            if (pos < N) {
                const uint64_t b = (uint64_t)__double_as_longlong(stage[lane * kRowD + k]);
                const uint32_t hi = (uint32_t)(b >> 32), lo = (uint32_t)b;
                key[pos] = sort_key(hi, lo, pos);
                // y > 0 is the clear sign bit: y = +0 (and tiny/subnormal y, whose alpha
                // could underflow) has prefix 0 and is sent to the slow path below
                // sign bits shifted in from the top (no per-position constants)
                if (pos < 32) yHl = (yHl >> 1) | (hi & 0x80000000u);
                else yHh = (yHh >> 1) | (hi & 0x80000000u);
            }
        }
        wave_sync();
    }
#pragma unroll
    for (int q = N; q < 64; ++q) key[q] = 0xFFFFFFFFu;
    // yHl/yHh hold the sign bits of positions 0..31 / 32..N-1, last position at bit 31
    if constexpr (N < 32) {
        yHl >>= 32 - N;
        yHh = 0;
    } else if constexpr (N < 64) {
        yHh >>= 64 - N;
    }
    const uint64_t yH = ~(((uint64_t)yHh << 32) | yHl) & ((1ull << N) - 1ull);
    BCHK_STAMP(0)
#if defined(BCHK_FAST_CUT) && BCHK_FAST_CUT == 1
    if (p.l0 && live) p.l0[cw] = (double)(key[5] ^ key[17] ^ key[40] ^ (uint32_t)yH);
    return;
#endif

    constexpr int KMAX = (2 * TMAX < N - 1) ? 2 * TMAX : N - 1;
    static_assert(!SEL || KMAX + 2 <= 16, "selection keeps 16 ranks");
    uint32_t kmax_real = 0;  // the largest key of a real position (SEL)
    if constexpr (SEL) {
        // ---- the 16 smallest keys in order: four sorted groups, low halves merged
        sort16<0>(key);
        sort16<16>(key);
        sort16<32>(key);
        sort16<48>(key);
        // padding keys (positions >= N) are all-ones and sort to the top of their group
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int cnt = N - 16 * g < 0 ? 0 : (N - 16 * g > 16 ? 16 : N - 16 * g);
            if (cnt > 0) kmax_real = key[16 * g + cnt - 1] > kmax_real ? key[16 * g + cnt - 1] : kmax_real;
        }
        merge_low16<0, 16>(key);
        merge_low16<32, 48>(key);
        merge_low16<0, 32>(key);
    } else {
        // ---- bitonic sort of the 64 keys, ascending
#pragma unroll
        for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
                for (int i = 0; i < 64; ++i) {
                    const int l = i ^ j;
                    if (l > i) {
                        const uint32_t a = key[i], b = key[l];
                        const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
                        key[i] = (i & k) ? hi : lo;
                        key[l] = (i & k) ? lo : hi;
                    }
                }
            }
        }
        kmax_real = key[N - 1];
    }

    BCHK_STAMP(1)
#if defined(BCHK_FAST_CUT) && BCHK_FAST_CUT == 2
    if (p.l0 && live) p.l0[cw] = (double)(key[5] ^ key[17] ^ key[40] ^ (uint32_t)yH);
    return;
#endif
    // ---- sorted prefix. Distinct 26-bit prefixes imply |y| values >= 2^-21 apart
    // (relative), so their alphas are strictly ordered exactly as the reference's
    // (|alpha|, position) order. Any equal prefix sends the codeword to the exact slow
    // path: beyond rank KMAX+1 the order cannot change this path's result, but an exact
    // tie anywhere is flagged (BCHK_F_TIE) there, so every path reports the same flags.
    bool bad = (key[0] >> 6) <= 1u                       // some |y| < 2^-27 (or zero)
               || (kmax_real >> 6) == 0x3FFFFFFu;        // some |y| >= 32, inf or NaN
    constexpr int NTIE = SEL ? KMAX + 1 : N - 1;         // adjacent pairs checked for ties
#pragma unroll
    for (int r = 0; r < NTIE; ++r) bad |= ((key[r] ^ key[r + 1]) >> 6) == 0u;
    {   // materialise the flag here, so the sorted keys past the prefix die now
        uint32_t b = bad ? 1u : 0u;
        asm volatile("" : "+v"(b));
        bad = b != 0u;
    }

    // ---- the sorted prefix calcRightSide can touch: positions packed 5 per word, and a
    // lower bound of each alpha from its key alone: the prefix is |y| truncated to 21
    // mantissa bits, so ylo <= |y| < ylo (1 + 2^-20), and lo = ylo * RN(2/s2) lies below
    // alpha = RN(2|y|/s2) by at most a relative 2^-51. The row is not re-read: the fast
    // path returns only when l < (sum of lo) (1 - 2^-40) <= calcRightSide(), and queues
    // every other case (a relative window of 2^-19 more than the exact test) for the
    // exact kernel.
    constexpr int NPF = KMAX + 1;
    constexpr int NPW = (NPF + 4) / 5;
    uint32_t ppk[NPW];
#pragma unroll
    for (int w = 0; w < NPW; ++w) ppk[w] = 0;
#pragma unroll
    for (int r = 0; r < NPF; ++r) ppk[r / 5] |= (key[r] & 63u) << (6 * (r % 5));
    auto ppos = [&](int r) { return (int)((ppk[r / 5] >> (6 * (r % 5))) & 63u); };
    const int o0 = (int)(key[0] & 63u);
    double alo[NPF];
    {
        const double c2 = 2.0 / s2;
#pragma unroll
        for (int r = 0; r < NPF; ++r) {
            const uint32_t pre = key[r] >> 6;  // eb (5 bits) | 21 mantissa bits
            const uint64_t bits = ((uint64_t)((pre >> 21) + (1023u - 27u)) << 52) |
                                  ((uint64_t)(pre & 0x1FFFFFu) << 31);
            alo[r] = __longlong_as_double((long long)bits) * c2;
        }
    }
    // ---- syndrome of the hard decision (Decoder::findSyndromPoly :184-207)
    uint32_t S0[W];
#pragma unroll
    for (int w = 0; w < W; ++w) S0[w] = 0;
#pragma unroll
    for (int pos = 0; pos < N; ++pos) {
        const uint32_t on = ((yH >> pos) & 1ull) ? 0xFFFFFFFFu : 0u;
#pragma unroll
        for (int w = 0; w < W; ++w) S0[w] ^= col[pos * W + w] & on;
    }

    BCHK_STAMP(2)
#if defined(BCHK_FAST_CUT) && BCHK_FAST_CUT == 3
    if (p.l0 && live) p.l0[cw] = (double)(alo[0] + alo[NPF - 1] + (double)(S0[0] ^ ppk[0] ^ (uint32_t)bad));
    return;
#endif
    // calcL (:69-77, index order) and calcRightSide (:54-67, sorted order) for `diff`
    // (at most t + 1 positions: the error pattern, plus the flipped bit at i = 1).
    auto accept = [&](uint64_t diff, double &l, bool &ret) {
        constexpr int LMAX = TMAX + 1;
        const int m = __popcll(diff);
        const int border = (2 * t + 1) - m;  // m0 == m on both fast-path exits
        double g[LMAX];
        uint64_t v = diff;
#pragma unroll
        for (int j = 0; j < LMAX; ++j) {  // independent loads, issued together; only the
            g[j] = 0.0;                    // flipped positions' (no line fetched for others)
            if (v) g[j] = yrow[(int)__builtin_ctzll(v)];
            v &= v - 1;
        }
        l = 0.0;
        v = diff;
#pragma unroll
        for (int j = 0; j < LMAX; ++j) {
            if (v) l += fabs((2.0 * g[j]) / s2);
            v &= v - 1;
        }
        double rs_lo = 0.0;  // lower bound of calcRightSide() (:54-67)
        int taken = 0;
#pragma unroll
        for (int r = 0; r < NPF; ++r) {
            const bool ag = !((diff >> ppos(r)) & 1ull);
            if (ag && taken < border) {
                rs_lo += alo[r];
                ++taken;
            }
        }
        // a certain return only: l < rs_lo (1 - 2^-40) <= rs; the exact path decides the rest
        ret = (taken >= border) && (l < rs_lo * (1.0 - 0x1p-40));
    };

    // ---- i = 0 (:361-382)
    int state = 0;  // 0 unresolved, 1 returned at i = 0, 2 returned at i = 1
    uint64_t best = 0;
    double l0 = DBL_MAX;
    Mask<1> E;
#ifdef BCHK_FAST_VALU  // experiment: Berlekamp-Massey on the VALU (spread GF products)
    const bool ok0 = alg_core_valu<M, TMAX>(chien, S0, t, E);
#else
    const bool ok0 = alg_core<M, TMAX>(ex, lg, chien, S0, t, E);
#endif
    if (!bad && ok0) {
        double l;
        bool ret;
        accept(E.w[0], l, ret);
        if (ret) { state = 1; best = E.w[0]; l0 = l; }
    }
    BCHK_STAMP(3)
#if defined(BCHK_FAST_CUT) && BCHK_FAST_CUT == 4
    if (p.l0 && live) p.l0[cw] = (double)(l0 + (double)(state ^ (uint32_t)best));
    return;
#endif
    // ---- i = 1: only where i = 0 failed (firstDecodingSuccessful = false, :371). When the
    // hard decision is a codeword (zero syndrome, which the decoder rejects), pattern 1 flips
    // the least reliable position o0 and its syndrome is o0's single column: the decoder
    // corrects that one error, back to yH, so D = 0 (l = 0) without a decode.
    bool zero0 = true;
#pragma unroll
    for (int w = 0; w < W; ++w) zero0 = zero0 && S0[w] == 0u;
    if (live && !bad && !ok0 && zero0) {
        double l;
        bool ret;
        accept(0ull, l, ret);
        if (ret) { state = 2; best = 0ull; l0 = l; }
    }
    const bool need1 = live && !bad && !ok0 && !zero0;
    if (ballot(need1)) {
        uint32_t S1[W];
#pragma unroll
        for (int w = 0; w < W; ++w) S1[w] = S0[w] ^ col[o0 * W + w];
#ifdef BCHK_FAST_VALU
        const bool ok1 = alg_core_valu<M, TMAX>(chien, S1, t, E);
#else
        const bool ok1 = alg_core<M, TMAX>(ex, lg, chien, S1, t, E);
#endif
        if (need1 && ok1) {
            const uint64_t diff = (1ull << o0) ^ E.w[0];
            double l;
            bool ret;
            accept(diff, l, ret);
            if (ret) { state = 2; best = diff; l0 = l; }
        }
    }

    BCHK_STAMP(4)
    // ---- outputs: resolved rows through LDS, one coalesced 64-row block per wave. The
    // unresolved rows of the block are read back and written unchanged (the exact kernel,
    // which runs after this one on the same stream, then owns them): measured against
    // writing only the resolved rows (16-B chunks that also touch an unresolved row stored
    // byte by byte) the read-back is 8 % faster at 5 dB -- 84 % of waves hold an unresolved row
    const bool resolved = live && state != 0;
    uint8_t *out = reinterpret_cast<uint8_t *>(stage);
    const uint64_t x = yH ^ best;
    if (resolved) {
#pragma unroll
        for (int pos = 0; pos < N; ++pos) out[lane * N + pos] = (uint8_t)((x >> pos) & 1ull);
    } else if (live) {  // unresolved: keep the caller's row as it is
        for (int pos = 0; pos < N; ++pos) out[lane * N + pos] = p.res[(size_t)cw * N + pos];
    }
    wave_sync();
    uint8_t *dst = p.res + (size_t)cw0 * N;
    if (cw0 + 64u <= p.count && ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0)) {
        const uint4 *src4 = reinterpret_cast<const uint4 *>(out);
        uint4 *dst4 = reinterpret_cast<uint4 *>(dst);
        for (int i = lane; i < 4 * N; i += 64) dst4[i] = src4[i];
    } else {
        const int rows = (int)((p.count - cw0) < 64u ? (p.count - cw0) : 64u);
        for (int i = lane; i < rows * N; i += 64) dst[i] = out[i];
    }
    if (p.cnt) {
        // fused counters (src/dataForPlot.cpp:55-74) of the resolved rows: the sent words'
        // block against the output block, 16 B at a time; differing bytes are rare
        uint32_t *rowerr = reinterpret_cast<uint32_t *>(out + 64 * N);
        rowerr[lane] = 0u;
        wave_sync();
        const uint8_t *txb = p.tx + (size_t)cw0 * N;
        if (cw0 + 64u <= p.count && ((reinterpret_cast<uintptr_t>(txb) & 15u) == 0)) {
            const uint4 *a4 = reinterpret_cast<const uint4 *>(txb);
            const uint4 *b4 = reinterpret_cast<const uint4 *>(out);
            for (int v = lane; v < 4 * N; v += 64) {
                const uint4 a = a4[v], b = b4[v];
                const uint32_t xx[4] = {a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (!xx[k]) continue;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if ((xx[k] >> (8 * q)) & 0xFFu) atomicAdd(&rowerr[(16 * v + 4 * k + q) / N], 1u);
                }
            }
        } else {
            const int rows = (int)((p.count - cw0) < 64u ? (p.count - cw0) : 64u);
            for (int i = lane; i < rows * N; i += 64)
                if (txb[i] != out[i]) atomicAdd(&rowerr[i / N], 1u);
        }
        wave_sync();
        const uint32_t e = resolved ? rowerr[lane] : 0u;
        const uint64_t it = state == 2 ? 1ull : 0ull;
        const uint64_t pro = p.variant == BCHK_VARIANT_WORD ? (uint64_t)(2 * N + 1) : 0ull;
        unsigned long long c[6] = {e ? 1ull : 0ull, e, resolved ? it + 1 : 0ull,
                                   resolved ? pro + it * (uint64_t)(N + 6) : 0ull,
                                   resolved ? pro + it * (uint64_t)(N + 1) : 0ull, resolved ? 1ull : 0ull};
        // frame / bit errors are rare: a ballot decides whether they need a reduction
        const bool anyerr = ballot(e != 0u) != 0ull;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            if (k < 2 && !anyerr) continue;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) c[k] += (unsigned long long)__shfl_xor((long long)c[k], o, 64);
        }
        if (lane == 0) {
            unsigned long long *dst6 = p.cnt + (size_t)((cw0 >> 6) % (uint32_t)kCntSlots) * kCntStride;
#pragma unroll
            for (int k = 0; k < 6; ++k)
                if (c[k]) atomicAdd(dst6 + k, c[k]);
        }
    }
    if (resolved) {
        const bool word = p.variant == BCHK_VARIANT_WORD;
        const uint64_t pro = word ? (uint64_t)(2 * N + 1) : 0ull;
        const uint64_t iters = state == 2 ? 1ull : 0ull;
        if (p.l0) p.l0[cw] = l0;
        if (p.st) {
            bchk_stats st;
            st.decodes = iters + 1;
            st.comparisons = pro + iters * (uint64_t)(N + 6);
            st.sums = pro + iters * (uint64_t)(N + 1);
            st.iterations = iters;
            st.jsteps = 0;
            st.improvements = 0;
            st.flags = BCHK_F_ACCEPTED | BCHK_F_RETURNED;
            st.reserved = 0;
            p.st[cw] = st;
        }
    }
    BCHK_STAMP(5)
#ifdef BCHK_DIAG
    if (p.diag && lane == 0)
        for (int q = 0; q < 6; ++q) p.diag[(size_t)(cw0 / 64) * 8 + q] = dg[q];
#endif
#undef BCHK_STAMP
    // ---- everything else goes to the exact wave-per-codeword path
    const bool unres = live && state == 0;
    const uint64_t um = ballot(unres);
    if (um && p.qfront) {
        // likely heavy: the hard decision itself does not decode (nor is it a codeword)
        const bool hv = unres && !bad && !ok0 && !zero0;
        const uint64_t hm = ballot(hv), om = um & ~hm;
        const uint64_t below = (1ull << lane) - 1ull;
        uint32_t bf = 0, bb = 0;
        if (lane == 0) {
            if (hm) bf = atomicAdd(p.qfront, (uint32_t)__popcll(hm));
            if (om) bb = atomicAdd(p.qback, (uint32_t)__popcll(om));
            atomicAdd(p.qtail, (uint32_t)__popcll(um));
        }
        bf = (uint32_t)__shfl((int)bf, 0, 64);
        bb = (uint32_t)__shfl((int)bb, 0, 64);
        if (hv) p.queue_out[bf + (uint32_t)__popcll(hm & below)] = cw;
        else if (unres) p.queue_out[p.count - 1u - (bb + (uint32_t)__popcll(om & below))] = cw;
    } else if (um) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(p.qtail, (uint32_t)__popcll(um));
        base = (uint32_t)__shfl((int)base, 0, 64);
        if (unres) p.queue_out[base + (uint32_t)__popcll(um & ((1ull << lane) - 1ull))] = cw;
    }
}

template <int M, int TMAX, bool SEL>
static hipError_t launch_fast_sel(const SearchParams &p, size_t lds, hipStream_t s) {
    const uint32_t chunks = (p.count + 63u) / 64u;
    const int blocks = (int)((chunks + kFastWaves - 1) / kFastWaves);
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void *)&kaneko_fast_kernel<M, TMAX, SEL>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((kaneko_fast_kernel<M, TMAX, SEL>), dim3(blocks), dim3(kWaveSize * kFastWaves),
                       lds, s, p);
    return hipGetLastError();
}

template <int M, int TMAX>
static hipError_t launch_fast_impl(const SearchParams &p, size_t lds, hipStream_t s) {
    constexpr int N = Geo<M>::N;
    constexpr int KMAX = (2 * TMAX < N - 1) ? 2 * TMAX : N - 1;
    if constexpr (KMAX + 2 <= 16) {
        // no stats record: the flags are not observable, selection suffices
        if (!p.st && !getenv("BCHK_FAST_FULLSORT")) return launch_fast_sel<M, TMAX, true>(p, lds, s);
    }
    return launch_fast_sel<M, TMAX, false>(p, lds, s);
}

size_t fast_wave_bytes() { return (size_t)kStageBytes; }
int fast_block_waves() { return kFastWaves; }

// Fast-path instantiations (n <= 63, small t): (m, TMAX) as in select_kernels.
bool select_fast(int m, int t, FastFn *out) {
    if (m >= 7) return select_first_long(m, t, out);  // bchk_kernels.hip
#define BCHK_FAST(MM, TT) \
    if (m == MM && t <= TT) { *out = &launch_fast_impl<MM, TT>; return true; }
    BCHK_FAST(3, 3)
    BCHK_FAST(4, 2) BCHK_FAST(4, 7)
    BCHK_FAST(5, 3) BCHK_FAST(5, 8)
    BCHK_FAST(6, 6)
#undef BCHK_FAST
    return false;
}

}  // namespace bchk
