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
#include <cfloat>
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
// accept: leave the flipped-position loops once no lane of the wave has another position
#ifndef BCHK_ACC_BREAK
#define BCHK_ACC_BREAK 1
#endif

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

// kept[0..16) and nk[0..16) sorted -> kept = the 16 smallest of both, sorted (as merge_low16)
__device__ __forceinline__ void merge_low16_2(uint32_t (&kept)[16], const uint32_t (&nk)[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t a = kept[i], b = nk[15 - i];
        kept[i] = a < b ? a : b;
    }
    uint32_t *key = kept;
#pragma unroll
    for (int j = 8; j > 0; j >>= 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (!(i & j)) BCHK_CAS(i, i + j)
    }
}

// 32-bit sort key: a monotone 26-bit prefix of |y| (5 exponent bits covering
// [2^-27, 2^5) + 21 mantissa bits) above the 6-bit position. |y| below the range maps to
// prefix 0, above it (and inf/NaN) to the all-ones prefix; both are detected after the sort.
// Four VALU operations: the funnel shift drops the sign and appends the 21st mantissa bit
// ((hi:lo) >> 31 = |y|'s top 32 bits below the sign), the biased exponent minus 996 (in that
// shifted form) saturates at 0 (|y| < 2^-27: prefix 0, sent to the slow path like every
// prefix <= 1), and the min saturates |y| >= 32 / inf / NaN.
__device__ __forceinline__ uint32_t sort_key(uint32_t hi, uint32_t lo, int pos) {
    const uint32_t top = __builtin_amdgcn_alignbit(hi, lo, 31);  // hi << 1 | lo >> 31
    const uint32_t mid = __builtin_elementwise_sub_sat(top, (uint32_t)(1023 - 27) << 21);
    const uint32_t pre = mid < 0x3FFFFFFu ? mid : 0x3FFFFFFu;
    return (pre << 6) | (uint32_t)pos;
}

// the hard decision yH = (2y/s2 > 0) (:336-342) from the sign bits shifted in from the top
// (yHl: positions 0..31, yHh: 32..N-1, last position at bit 31)
template <int N>
__device__ __forceinline__ uint64_t hard_decision(uint32_t yHl, uint32_t yHh);
// the same from sign bits shifted in from the bottom, one funnel shift per position
// (yH = yH << 1 | hi >> 31: the last position at bit 0): bit-reversed, they are the above
template <int N>
__device__ __forceinline__ uint64_t hard_decision_rev(uint32_t yHl, uint32_t yHh) {
    return hard_decision<N>(__builtin_bitreverse32(yHl), __builtin_bitreverse32(yHh));
}
template <int N>
__device__ __forceinline__ uint64_t hard_decision(uint32_t yHl, uint32_t yHh) {
    if constexpr (N < 32) {
        yHl >>= 32 - N;
        yHh = 0;
    } else if constexpr (N < 64) {
        yHh >>= 64 - N;
    }
    // y > 0 is the clear sign bit: y = +0 (and tiny/subnormal y, whose alpha could
    // underflow) has prefix 0 and is sent to the slow path by fast_decide
    return ~(((uint64_t)yHh << 32) | yHl) & ((1ull << N) - 1ull);
}

// ------------------------------------------------------------------ the per-lane decision
// What the fast path decides for one codeword (lane), from its 64 sort keys (positions N..63
// all-ones) and its hard decision yH: returned at i = 0 (state 1) or i = 1 (state 2) with the
// decoded difference `best` and path metric l0, or unresolved (state 0: the exact kernel
// decides). bad / ok0 / zero0 classify it for the queue.
struct FastRes {
    int state;
    uint64_t best;
    double l0;
    bool bad, ok0, zero0;
    bool heavy;  // unresolved, likely to run >= 127 test patterns (queue order only)
};
// An unresolved codeword whose hard decision decodes (ok0) runs to the loop bound of that
// first improvement, (1 << T) - 1 with T from calcT's scan (:110-126, :383-390), unless a
// later improvement moves it (rare). T estimated from the keys of ranks 0..15 (lower bounds
// of alpha) at or above this flags the codeword for the front of the exact kernel's queue, so
// the first pass starts it early (its last starters set its length). Queue order only: every
// result is unchanged. 2^18 words at 5 dB (oracle): the estimate equals the true T for every
// such word up to T = 9; a list-scheduling model of the first pass, 350 -> 280 us.
constexpr int kHeavyT = 7;

// Sort of the 64 keys (positions N..63 all-ones) into the 16 smallest in order, k[0..15].
// SEL (no per-codeword stats requested, 2 TMAX + 2 <= 16): only the 16 smallest keys are
// put in order (four sorted groups of 16, then low-half merges) -- the fast-path exits read
// ranks 0..2t and the least reliable position, so an exact tie beyond rank 2t + 1 cannot
// change a result, only the BCHK_F_TIE flag of the stats record; SEL = false sorts all 64
// keys and sends any tie to the exact path, so the flags match it. bad: some |y| outside
// the keys' range, or (SEL = false) a prefix tie anywhere.
template <int M, int TMAX, bool SEL>
__device__ __forceinline__ void fast_sort64(uint32_t (&key)[64], uint32_t &kmax_real, bool &bad) {
    constexpr int N = Geo<M>::N;
    kmax_real = 0;  // the largest key of a real position
    bad = false;
    if constexpr (SEL) {
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
#pragma unroll
        for (int r = 0; r < N - 1; ++r) bad |= ((key[r] ^ key[r + 1]) >> 6) == 0u;
    }
}

// The decision from the sorted prefix k[0..15] (ranks 0..15 of the 64 keys), the largest
// real key and the sorter's flags: returned at i = 0 / i = 1, or unresolved.
// Row values are read through rd0 for the i = 0 tests and through rd1 for i = 1; `between`
// runs after the i = 0 tests (the ring kernel gives its LDS slot back there).
template <int M, int TMAX, class Rd0, class Rd1, class Between>
__device__ __forceinline__ FastRes fast_decide(const uint8_t *ex, const uint16_t *lg, const uint32_t *col,
                                               const uint64_t *chien, const uint32_t *k, uint32_t kmax_real,
                                               bool bad, uint64_t yH, Rd0 rd0, Rd1 rd1, Between between,
                                               bool live, int t, double s2, const uint32_t *lo = nullptr,
                                               bool have_lo = false, const uint32_t *syn8 = nullptr,
                                               int heavy_t = kHeavyT, int heavy_tmax = 64) {
    constexpr int N = Geo<M>::N;
    constexpr int W = (TMAX + 3) / 4;
    // calcRightSide takes the first border = 2t+1-m agreeing sorted positions; with m0 == m
    // (both fast-path exits) and m positions disagreeing, they lie within ranks 0..2t (KMAX).
    constexpr int KMAX = (2 * TMAX < N - 1) ? 2 * TMAX : N - 1;
    // (k holds at least ranks 0..KMAX+1: 16 from the selection, 64 from the full sort)
    // ---- sorted prefix. Distinct 26-bit prefixes imply |y| values >= 2^-21 apart
    // (relative), so their alphas are strictly ordered exactly as the reference's
    // (|alpha|, position) order. Any equal prefix sends the codeword to the exact slow
    // path: beyond rank KMAX+1 the order cannot change this path's result, but an exact
    // tie anywhere is flagged (BCHK_F_TIE) there, so every path reports the same flags.
    bad = bad || (k[0] >> 6) <= 1u                       // some |y| < 2^-27 (or zero)
              || (kmax_real >> 6) == 0x3FFFFFFu;         // some |y| >= 32, inf or NaN
#pragma unroll
    for (int r = 0; r < KMAX + 1; ++r) bad |= ((k[r] ^ k[r + 1]) >> 6) == 0u;
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
    // exact kernel. The bounds are formed from the prefix keys where they are summed.
    constexpr int NPF = KMAX + 1;
    uint32_t pre[NPF];
#pragma unroll
    for (int r = 0; r < NPF; ++r) pre[r] = k[r];
    const int o0 = (int)(k[0] & 63u);
    const double c2 = 2.0 / s2;
    // ---- syndrome of the hard decision (Decoder::findSyndromPoly :184-207): from the byte
    // table when given (syn8[j][v]: byte value v at positions 8j .. 8j + 7; one L1-resident
    // load per byte of yH instead of a select and W XORs per position), else per position
    uint32_t S0[W];
#pragma unroll
    for (int w = 0; w < W; ++w) S0[w] = 0;
    if (syn8) {
#pragma unroll
        for (int j = 0; 8 * j < N; ++j) {
            const uint32_t v = (uint32_t)(yH >> (8 * j)) & 255u;
            const uint32_t *e = syn8 + ((uint32_t)j * 256u + v) * (uint32_t)W;
#pragma unroll
            for (int w = 0; w < W; ++w) S0[w] ^= e[w];
        }
    } else {
#pragma unroll
        for (int pos = 0; pos < N; ++pos) {
            const uint32_t on = ((yH >> pos) & 1ull) ? 0xFFFFFFFFu : 0u;
#pragma unroll
            for (int w = 0; w < W; ++w) S0[w] ^= col[pos * W + w] & on;
        }
    }
    // calcL (:69-77, index order) and calcRightSide (:54-67, sorted order) for `diff`
    // (at most t + 1 positions: the error pattern, plus the flipped bit at i = 1).
    auto accept = [&](auto rd, uint64_t diff, double &l, bool &ret) {
        constexpr int LMAX = TMAX + 1;
        const int m = __popcll(diff);
        const int border = (2 * t + 1) - m;  // m0 == m on both fast-path exits
        double g[LMAX];
#pragma unroll
        for (int j = 0; j < LMAX; ++j) g[j] = 0.0;
        uint64_t v = diff;
#pragma unroll
        for (int j = 0; j < LMAX; ++j) {  // independent loads, issued together; only the
                                           // flipped positions' (no line fetched for others)
#if BCHK_ACC_BREAK
            if (!ballot(v != 0ull)) break;  // no lane has a j-th flipped position
#endif
            const int pj = (int)__builtin_ctzll(v);
            bool found = false;
            if (have_lo) {
                // |y| of a prefix rank rebuilt exactly: its key's exponent and 21 mantissa bits
                // (the hi word's 20 below the top) and the row's lo word, gathered before the
                // slot was given back (a non-bad key: 2^-27 <= |y| < 32)
                uint64_t bits = 0;
#pragma unroll
                for (int r = 0; r < NPF; ++r) {
                    const bool hit = (pre[r] & 63u) == (uint32_t)pj;
                    found = found || hit;
                    bits = hit ? ((uint64_t)((pre[r] >> 7) + (996u << 20)) << 32) | lo[r] : bits;
                }
                if (v) g[j] = __longlong_as_double((long long)bits);
            }
            if (v && !found) g[j] = rd(pj);
            v &= v - 1;
        }
        l = 0.0;
        v = diff;
#pragma unroll
        for (int j = 0; j < LMAX; ++j) {
#if BCHK_ACC_BREAK
            if (!ballot(v != 0ull)) break;
#endif
            if (v) l += fabs((2.0 * g[j]) / s2);
            v &= v - 1;
        }
        double rs_lo = 0.0;  // lower bound of calcRightSide() (:54-67)
        int taken = 0;
#pragma unroll
        for (int r = 0; r < NPF; ++r) {
            const bool ag = !((diff >> (pre[r] & 63u)) & 1ull);
            if (ag && taken < border) {
                const uint32_t pr = pre[r] >> 6;  // eb (5 bits) | 21 mantissa bits
                const uint64_t bits = ((uint64_t)((pr >> 21) + (1023u - 27u)) << 52) |
                                      ((uint64_t)(pr & 0x1FFFFFu) << 31);
                rs_lo += __longlong_as_double((long long)bits) * c2;
                ++taken;
            }
        }
        // a certain return only: l < rs_lo (1 - 2^-40) <= rs; the exact path decides the rest
        ret = (taken >= border) && (l < rs_lo * (1.0 - 0x1p-40));
    };

    FastRes R;
    // ---- i = 0 (:361-382)
    R.state = 0;  // 0 unresolved, 1 returned at i = 0, 2 returned at i = 1
    R.best = 0;
    R.l0 = DBL_MAX;
    R.heavy = false;
    Mask<1> E;
    const bool ok0 = alg_core<M, TMAX>(ex, lg, chien, S0, t, E);
    double lE = 0.0;
    if (!bad && ok0) {
        bool ret;
        accept(rd0, E.w[0], lE, ret);
        if (ret) { R.state = 1; R.best = E.w[0]; R.l0 = lE; }
    }
    // ---- the loop bound of an unresolved ok0 codeword, estimated (queue order, FastRes::heavy):
    // calcT(j) = the first t - (m + m0) / 2 agreeing sorted alphas + alpha of ranks j .. j + t,
    // m = m0 = |E|; T = the first j with l < calcT(j). Ranks up to 15 from the keys.
    if (ballot(live && !bad && ok0 && R.state == 0)) {
        constexpr int RK = 16;
        double al[RK];
#pragma unroll
        for (int r = 0; r < RK; ++r) {
            const uint32_t pr = k[r] >> 6;
            const uint64_t bits = ((uint64_t)((pr >> 21) + (1023u - 27u)) << 52) | ((uint64_t)(pr & 0x1FFFFFu) << 31);
            al[r] = __longlong_as_double((long long)bits) * c2;
        }
        int need = t - __popcll(E.w[0]);
        double A = 0.0;
#pragma unroll
        for (int r = 0; r < RK; ++r) {
            const bool ag = !((E.w[0] >> (k[r] & 63u)) & 1ull);
            if (ag && need > 0) {
                A += al[r];
                --need;
            }
        }
        int T = RK - t;  // past the keys: at least this
        bool found = false;
#pragma unroll
        for (int j = RK - 1; j >= 0; --j) {  // the first j with l < calcT(j), scanned from the top
            double Wj = A;
#pragma unroll
            for (int i = 0; i <= TMAX; ++i)
                if (j + i < RK && i <= t) Wj += al[j + i];
            const bool below = j + t < RK && lE < Wj;
            T = below ? j : T;
            found = found || below;
        }
        (void)found;
        R.heavy = live && !bad && ok0 && R.state == 0 && T >= heavy_t && T <= heavy_tmax;
    }
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
        accept(rd0, 0ull, l, ret);
        if (ret) { R.state = 2; R.best = 0ull; R.l0 = l; }
    }
    between();
    const bool need1 = live && !bad && !ok0 && !zero0;
#ifdef BCHK_FAST_NO_I1  // experiment builds: the i = 1 decode left to the exact kernels
    if (false) {
#else
    if (ballot(need1)) {
#endif
        uint32_t S1[W];
#pragma unroll
        for (int w = 0; w < W; ++w) S1[w] = S0[w] ^ col[o0 * W + w];
        const bool ok1 = alg_core<M, TMAX>(ex, lg, chien, S1, t, E);
        if (need1 && ok1) {
            const uint64_t diff = (1ull << o0) ^ E.w[0];
            double l;
            bool ret;
            accept(rd1, diff, l, ret);
            if (ret) { R.state = 2; R.best = diff; R.l0 = l; }
        }
    }
    R.bad = bad;
    R.ok0 = ok0;
    R.zero0 = zero0;
    return R;
}

// The fused counters of a wave's 64 codewords (src/dataForPlot.cpp:55-74): e = bit errors of
// a resolved row (0 otherwise); one reduction per counter, the error ones only when a row has
// errors (rare: ballot); partial slot by chunk.
__device__ __forceinline__ void fast_counters(const SearchParams &p, uint32_t cw0, int N, bool resolved, int state,
                                              uint32_t e) {
    // per-codeword counts are 0/1 flags times constants: wave sums by ballot popcounts (no
    // cross-lane reductions); the bit-error sum only when a row has errors (rare)
    const uint64_t nres = (uint64_t)__popcll(ballot(resolved));
    const uint64_t nit = (uint64_t)__popcll(ballot(resolved && state == 2));
    const uint64_t pro = p.variant == BCHK_VARIANT_WORD ? (uint64_t)(2 * N + 1) : 0ull;
    const uint64_t em = ballot(e != 0u);
    unsigned long long c[6] = {(unsigned long long)__popcll(em), 0ull, nres + nit,
                               pro * nres + nit * (uint64_t)(N + 6), pro * nres + nit * (uint64_t)(N + 1), nres};
    for (uint64_t mm = em; mm; mm &= mm - 1) c[1] += rdl(e, (int)__builtin_ctzll(mm));
    if ((threadIdx.x & 63) == 0) {
        unsigned long long *dst6 = p.cnt + (size_t)((cw0 >> 6) % (uint32_t)kCntSlots) * kCntStride;
#pragma unroll
        for (int k = 0; k < 6; ++k)
            if (c[k]) atomicAdd(dst6 + k, c[k]);
    }
}

// l0 and the stats record of a resolved codeword, then every unresolved one into the exact
// kernel's queue (likely heavy ones -- the hard decision neither decodes nor is a codeword --
// at the front when the queue is two-ended)
__device__ __forceinline__ void fast_finish(const SearchParams &p, uint32_t cw, int N, bool live, const FastRes &R) {
    const bool resolved = live && R.state != 0;
    if (resolved) {
        const bool word = p.variant == BCHK_VARIANT_WORD;
        const uint64_t pro = word ? (uint64_t)(2 * N + 1) : 0ull;
        const uint64_t iters = R.state == 2 ? 1ull : 0ull;
        if (p.l0) p.l0[cw] = R.l0;
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
    const int lane = threadIdx.x & 63;
    const bool unres = live && R.state == 0;
    const uint64_t um = ballot(unres);
    if (um && p.qfront) {
        const bool hv = unres && ((!R.bad && !R.ok0 && !R.zero0) || R.heavy);
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

// ------------------------------------------------------------ staged kernel (BCHK_FAST_RING=0)
// Blocks of kFastWaves waves, one 64-codeword chunk per wave: the code tables are staged
// into LDS once per 512 codewords, and two blocks per CU give 4 waves per SIMD (<= 128
// VGPRs). Each wave stages its rows through LDS in 8-position slices (coalesced 8-B loads
// via registers).
template <int M, int TMAX, bool SEL>
__global__ void __launch_bounds__(kWaveSize * kFastWaves, 4)
kaneko_fast_kernel(SearchParams p) {
    constexpr int N = Geo<M>::N;
    static_assert(N <= 63, "fast path covers n <= 63");
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
    const uint32_t cw = cw0 + (uint32_t)lane;
    const bool live = cw < p.count;
    const double *yrow = p.y + (size_t)(live ? cw : cw0) * N;
    static_assert(64 * N + 256 <= kStageBytes, "output block and row errors fit the stage");

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
    const uint64_t yH = hard_decision<N>(yHl, yHh);
    uint32_t kmax_real;
    bool bad;
    fast_sort64<M, TMAX, SEL>(key, kmax_real, bad);
    auto rdg = [&](int pos) { return yrow[pos]; };
    const FastRes R = fast_decide<M, TMAX>(ex, lg, col, chien, key, kmax_real, bad, yH, rdg, rdg, [] {}, live,
                                           p.t, p.s2);

    // ---- outputs: resolved rows through LDS, one coalesced 64-row block per wave. The
    // unresolved rows of the block are read back and written unchanged (the exact kernel,
    // which runs after this one on the same stream, then owns them): measured against
    // writing only the resolved rows (16-B chunks that also touch an unresolved row stored
    // byte by byte) the read-back is 8 % faster at 5 dB -- 84 % of waves hold an unresolved row
    const bool resolved = live && R.state != 0;
    uint8_t *out = reinterpret_cast<uint8_t *>(stage);
    const uint64_t x = yH ^ R.best;
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
        // fused counters of the resolved rows: the sent words' block against the output
        // block, 16 B at a time; differing bytes are rare
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
        fast_counters(p, cw0, N, resolved, R.state, resolved ? rowerr[lane] : 0u);
    }
    fast_finish(p, cw, N, live, R);
}

// ------------------------------------------------------------------ ring kernel (default)
// Workgroups of kRingWaves waves, kRingPerCU per CU, persistent over the batch's 64-codeword
// chunks (chunk b, b + G, b + 2G, ... for workgroup b of G). Wave 0 is the loader: it copies each chunk's
// rows -- 64 x n contiguous f64, exactly the caller's layout -- from HBM into a ring of LDS
// slots with gfx950 direct-to-LDS loads (global_load_lds_dwordx4: no VGPRs, one 1-KiB
// wave-instruction per 1 KiB, every line read once, fully coalesced), up to two chunks in
// flight, and publishes a slot once its loads have landed (a counted vmcnt wait, then the
// slot's tag in LDS). The other waves compute: each claims the workgroup's next chunk, reads its
// 64 rows from the slot (lane r reads row r: row stride 8n bytes keeps ds_read_b64
// conflict-free), turns them into sort keys -- selecting the 16 smallest on the way, 32 keys
// held at a time -- and gives the slot back, then runs the same decision as the staged kernel
// (fast_decide). Selection only (no stats record: the staged kernel serves those calls). So the chip streams the next chunks while it
// computes the current ones, instead of every wave loading, then computing, in step with
// the others. Outputs leave without an LDS row image: each lane's decoded word is one 64-bit
// mask, and the block's 16-B pieces are expanded from the masks (the caller's bytes kept
// for unresolved rows, which are not written) and stored coalesced.
// default: one 16-wave workgroup per CU with 4 slots (147 KB of LDS at n = 63). Measured at
// 5 dB / 6 dB (fast kernel alone, profiles/r05_fast/): 16 waves / 4 slots 0.233-0.235 /
// 0.163 ms, 2 x 12 waves / 2 slots 0.241 / 0.177, 2 x 10 waves 0.238 / 0.213, staged
// kernel 0.237 / 0.190
#ifndef BCHK_FAST_RING_SLOTS
#define BCHK_FAST_RING_SLOTS 4
#endif
#ifndef BCHK_FAST_RING_WAVES
#define BCHK_FAST_RING_WAVES 16
#endif
#ifndef BCHK_FAST_RING_PER_CU
#define BCHK_FAST_RING_PER_CU 1
#endif
constexpr int kRingSlots = BCHK_FAST_RING_SLOTS;
constexpr int kRingWaves = BCHK_FAST_RING_WAVES;  // 1 loader + the compute waves
constexpr int kRingPerCU = BCHK_FAST_RING_PER_CU; // workgroups per CU (LDS and VGPRs sized for it)
constexpr int kRingWPE = (kRingWaves * kRingPerCU + 3) / 4;  // waves per SIMD
constexpr int kRingWaveBytes = 64 * 8 + 64 * 4;  // decoded masks + row error counts
struct RingCtl {
    uint32_t tag[kRingSlots];  // chunk + 1 once the slot holds that chunk's rows, 0 = free
    uint32_t claim;            // next chunk for a compute wave
    uint32_t pad[3];
};
template <int M>
constexpr size_t ring_slot_bytes() { return (size_t)64 * Geo<M>::N * 8; }
template <int M>
constexpr size_t ring_lds_bytes(size_t tables) {
    return ((tables + 15) & ~size_t(15)) + kRingSlots * ring_slot_bytes<M>() + sizeof(RingCtl) +
           (kRingWaves - 1) * kRingWaveBytes;
}

__device__ __forceinline__ void glds16(const void *src, uint8_t *lds_dst) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void *)lds_dst, 16, 0, 0);
}
__device__ __forceinline__ uint32_t lds_ld32(const uint32_t *a) {
    return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st32(uint32_t *a, uint32_t v) {
    __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
constexpr uint32_t kRingSpin = 1u << 24;  // bounded waits: a guard against logic errors
constexpr uint32_t kFaultFastRing = 32u;

// 4 bits -> 4 bytes of 0/1 (bit k to byte k)
__device__ __forceinline__ uint32_t nib_bytes(uint32_t nib) { return (nib * 0x00204081u) & 0x01010101u; }

template <int M, int TMAX>
__global__ void __launch_bounds__(kWaveSize * kRingWaves) __attribute__((amdgpu_waves_per_eu(kRingWPE, kRingWPE)))
kaneko_fast_ring_kernel(SearchParams p) {
    constexpr int N = Geo<M>::N;
    static_assert(N <= 63, "fast path covers n <= 63");
    constexpr int KMAX = (2 * TMAX < N - 1) ? 2 * TMAX : N - 1;
    static_assert(KMAX + 2 <= 16, "the 16-key selection covers the decision's ranks");
    constexpr uint32_t SLOT = (uint32_t)ring_slot_bytes<M>();
    static_assert(SLOT % 512 == 0, "a slot is whole half-instructions of 16-B pieces");
    constexpr int NG = (int)((SLOT + 1023) / 1024);  // glds wave-instructions per chunk
    static_assert(NG <= 32, "two chunks in flight fit the vmcnt field");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    load_tables(smem, p.tables, p.td.bytes);
    uint8_t *ring = smem + ((p.td.bytes + 15) & ~15u);
    RingCtl *ctl = reinterpret_cast<RingCtl *>(ring + kRingSlots * SLOT);
    if (threadIdx.x < sizeof(RingCtl) / 4) reinterpret_cast<uint32_t *>(ctl)[threadIdx.x] = 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = uni((int)(threadIdx.x >> 6));  // wave-uniform: SGPRs
    const uint32_t nch = (p.count + 63u) / 64u, nfull = p.count / 64u;
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint32_t K = b < nch ? (nch - b + G - 1u) / G : 0u;  // this workgroup's chunks

    if (wid == 0) {
        // ------------------------------------------------------------------ loader
        uint32_t issued = 0, published = 0, spins = 0;
        while (published < K) {
            while (issued < K && issued - published < 2u) {
                const uint32_t s = issued % kRingSlots;
                if (lds_ld32(&ctl->tag[s]) != 0u) break;  // still held by a compute wave
                const uint32_t gk = b + issued * G;
                if (gk < nfull && p.fast_mode != 1u) {  // a partial last chunk: read by its compute wave
                    const uint8_t *src = reinterpret_cast<const uint8_t *>(p.y) + (size_t)gk * SLOT + 16u * lane;
                    uint8_t *dst = ring + s * SLOT;
#pragma unroll
                    for (int i = 0; i < NG; ++i)
                        if (1024u * i + 16u * lane < SLOT) glds16(src + 1024u * i, dst + 1024u * i);
                }
                ++issued;
            }
            if (issued == published) {  // no slot free yet
                if (++spins > kRingSpin) {
                    if (lane == 0 && p.fault) atomicOr(p.fault, kFaultFastRing);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            spins = 0;
            // the oldest chunk in flight has landed once at most the newer one's loads remain
            const bool newer = issued - published == 2u && b + (published + 1u) * G < nfull;
            if (newer) {
                asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NG) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (lane == 0) lds_st32(&ctl->tag[published % kRingSlots], published + 1u);
            ++published;
        }
        return;
    }
    // ---------------------------------------------------------------------- compute
    const uint8_t *ex = smem + p.td.off_exp;
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(smem + p.td.off_log);
    const uint32_t *col = reinterpret_cast<const uint32_t *>(smem + p.td.off_col);
    const uint64_t *chien = reinterpret_cast<const uint64_t *>(smem + p.td.off_chien);
    uint8_t *wb = reinterpret_cast<uint8_t *>(ctl + 1) + (wid - 1) * kRingWaveBytes;
    uint64_t *xm = reinterpret_cast<uint64_t *>(wb);
    uint32_t *rowerr = reinterpret_cast<uint32_t *>(wb + 64 * 8);
    for (;;) {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(&ctl->claim, 1u);
        k = (uint32_t)uni((int)__shfl((int)k, 0, 64));
        if (k >= K) break;
        const uint32_t gk = b + k * G, cw0 = 64u * gk;
        const uint32_t cw = cw0 + (uint32_t)lane;
        const bool live = cw < p.count;
        const bool full = gk < nfull;
        const uint32_t s = k % kRingSlots;
        {   // the slot: published by the loader
            uint32_t sp = 0;
            while (lds_ld32(&ctl->tag[s]) != k + 1u && ++sp < kRingSpin) __builtin_amdgcn_s_sleep(1);
            if (sp >= kRingSpin) {
                if (lane == 0 && p.fault) atomicOr(p.fault, kFaultFastRing);
                break;
            }
        }
        // ---- keys and the hard decision yH = (2y/s2 > 0) (:336-342) from the rows, 16
        // positions at a time: each group of 16 keys is sorted (Green's network) and merged
        // into the 16 smallest so far, so only 32 keys are ever held (registers for more
        // waves per SIMD); the same selection as fast_sort64's
        uint32_t kept[16];
        uint32_t kmax_real = 0, yHl = 0, yHh = 0;
        auto build = [&](auto rd) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                uint32_t nk[16];
#pragma unroll
                for (int h = 0; h < 2; ++h) {  // 8 reads in flight at a time
                    double v8[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const int pos = 16 * g + 8 * h + i;
                        if (pos < N) v8[i] = rd(pos);
                    }
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const int pos = 16 * g + 8 * h + i;
                        if (pos < N) {
                            const uint64_t bb = (uint64_t)__double_as_longlong(v8[i]);
                            const uint32_t hi = (uint32_t)(bb >> 32), lo = (uint32_t)bb;
                            nk[8 * h + i] = sort_key(hi, lo, pos);
                            if (pos < 32) yHl = __builtin_amdgcn_alignbit(yHl, hi, 31);
                            else yHh = __builtin_amdgcn_alignbit(yHh, hi, 31);
                        } else {
                            nk[8 * h + i] = 0xFFFFFFFFu;
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                sort16<0>(nk);
                const int cnt = N - 16 * g < 0 ? 0 : (N - 16 * g > 16 ? 16 : N - 16 * g);
                if (cnt > 0) kmax_real = nk[cnt - 1] > kmax_real ? nk[cnt - 1] : kmax_real;
                if (g == 0) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) kept[i] = nk[i];
                } else {
                    merge_low16_2(kept, nk);
                }
            }
        };
        typedef __attribute__((address_space(3))) const double *LdsF64;
        LdsF64 lrow = (LdsF64)(ring + s * SLOT);  // a C cast: generic -> LDS address space
        lrow += lane * N;
        const double *yrow = p.y + (size_t)(live ? cw : cw0) * N;
        if (full) {  // the slot (LDS)
            build([&](int pos) { return lrow[pos]; });
        } else {     // the partial last chunk, from HBM
            build([&](int pos) { return yrow[pos]; });
        }
        // the slot goes back once every read of it has returned: now (the tests rebuild the
        // prefix ranks' values from their keys and lo words; other flipped positions' values
        // are read again from HBM), or in experiment mode 3 after the i = 0 tests, which
        // then read them from the slot (the slot is held through the decode: slower, measured)
        // the lo words of the prefix ranks' values (the accept tests rebuild those exactly:
        // re-reading a flipped position from HBM fetches a 128-B line the stream has long
        // evicted from L2 -- 0.32 GB per 2^20 rows at 5 dB, measured; experiment mode 6 does)
        constexpr int NPF = KMAX + 1;
        uint32_t lo[NPF] = {};
        const bool use_lo = full && p.fast_mode != 6u;
        if (use_lo) {
            typedef __attribute__((address_space(3))) const uint32_t *LdsU32;
            LdsU32 lw = (LdsU32)(ring + s * SLOT);
            lw += lane * 2 * N;
#pragma unroll
            for (int r = 0; r < NPF; ++r) lo[r] = lw[2 * (kept[r] & 63u)];
        }
        auto release = [&] {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            wave_sync();
            if (lane == 0) lds_st32(&ctl->tag[s], 0u);
        };
        const bool hold = full && p.fast_mode == 3u;
        if (!hold) release();
        const uint64_t yH = hard_decision_rev<N>(yHl, yHh);
        if (p.fast_mode == 2u) {  // experiment: the rows' path alone (wrong results)
            if (hold) release();
            if (p.l0 && live) p.l0[cw] = (double)(kept[3] ^ kmax_real ^ (uint32_t)yH);
            continue;
        }
        // t and s2 re-read opaquely per chunk: nothing derived from them is hoisted out of
        // the persistent loop (it would stay live through the selection and spill)
        int t = p.t;
        double s2 = p.s2;
        asm volatile("" : "+s"(t), "+s"(s2));
        const FastRes R = fast_decide<M, TMAX>(
            ex, lg, col, chien, kept, kmax_real, false, yH, [&](int pos) { return hold ? lrow[pos] : yrow[pos]; },
            [&](int pos) { return yrow[pos]; }, [&] { if (hold) release(); }, live, t, s2,
            lo, use_lo, p.syn8, p.heavy_t ? (int)p.heavy_t : kHeavyT, p.heavy_tmax ? (int)p.heavy_tmax : 64);

        // ---- outputs
        const bool resolved = live && R.state != 0;
        const uint64_t x = yH ^ R.best;
        uint32_t e = 0;
        uint8_t *dst = p.res + (size_t)cw0 * N;
        const uint8_t *txb = p.tx ? p.tx + (size_t)cw0 * N : nullptr;
        if (N >= 16 && full && ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(txb)) & 15u) == 0) {
            // the block's 4n 16-B pieces from the 64 masks: piece q holds bytes 16q .. 16q + 15
            // = positions o .. of row r1 = 16q / n (and the first ones of row r1 + 1: n >= 16)
            const uint64_t rm = ballot(resolved);
            xm[lane] = x;
            rowerr[lane] = 0u;
            wave_sync();
            bool anyerr = false;
            for (int q = lane; q < 4 * N; q += 64) {
                const int b0 = 16 * q, r1 = b0 / N, o = b0 - N * r1;
                const bool span = o > N - 16;  // the piece reaches row r1 + 1
                const int r2 = span ? r1 + 1 : r1;
                const uint64_t x1 = xm[r1], x2 = xm[r2];
                const uint64_t w = (x1 >> o) | (span ? x2 << (N - o) : 0ull);
                uint32_t nw[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) nw[d] = nib_bytes((uint32_t)(w >> (4 * d)) & 15u);
                // bytes of unresolved rows are not written (the exact kernel owns them, and
                // may run concurrently on another XCD: no stale byte may be stored over its
                // result); a piece shared with one goes out byte by byte (rare)
                const uint32_t in2 = span ? (0xFFFFu << (N - o)) & 0xFFFFu : 0u;  // bytes of r2
                const uint32_t keep = (((rm >> r1) & 1ull) ? 0u : (~in2 & 0xFFFFu)) |
                                      (((rm >> r2) & 1ull) ? 0u : in2);
                if (!keep) {
                    reinterpret_cast<uint4 *>(dst)[q] = make_uint4(nw[0], nw[1], nw[2], nw[3]);
                } else if (keep != 0xFFFFu) {
                    for (uint32_t wm = ~keep & 0xFFFFu; wm; wm &= wm - 1) {
                        const int i = __builtin_ctz(wm);
                        dst[16 * q + i] = (uint8_t)(nw[i >> 2] >> (8 * (i & 3)));
                    }
                }
                if (txb) {  // fused counters: bytes that differ from the sent word (rare)
                    const uint4 a = reinterpret_cast<const uint4 *>(txb)[q];
                    const uint32_t xx[4] = {a.x ^ nw[0], a.y ^ nw[1], a.z ^ nw[2], a.w ^ nw[3]};
                    if (xx[0] | xx[1] | xx[2] | xx[3]) {
                        anyerr = true;
#pragma unroll
                        for (int i = 0; i < 16; ++i)
                            if ((xx[i >> 2] >> (8 * (i & 3))) & 0xFFu) atomicAdd(&rowerr[i < N - o ? r1 : r2], 1u);
                    }
                }
            }
            if (txb) {
                if (ballot(anyerr)) {
                    wave_sync();
                    e = resolved ? rowerr[lane] : 0u;
                }
            }
        } else if (resolved) {  // partial chunk (or unaligned buffers): the row byte by byte
            for (int pos = 0; pos < N; ++pos) {
                const uint8_t bit = (uint8_t)((x >> pos) & 1ull);
                dst[lane * N + pos] = bit;
                if (txb) e += txb[lane * N + pos] != bit ? 1u : 0u;
            }
        }
        if (p.cnt) fast_counters(p, cw0, N, resolved, R.state, e);
        fast_finish(p, cw, N, live, R);
        wave_sync();  // xm / rowerr are rewritten by the next chunk
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

// the ring kernel: one workgroup per CU (persistent), LDS sized by ring_lds_bytes
static int device_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}
template <int M, int TMAX>
static hipError_t launch_fast_ring(const SearchParams &p, hipStream_t s) {
    const uint32_t chunks = (p.count + 63u) / 64u;
    const int blocks = (int)std::min<uint32_t>(chunks, (uint32_t)(kRingPerCU * device_cus()));
    const size_t lds = ring_lds_bytes<M>(p.td.bytes);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)&kaneko_fast_ring_kernel<M, TMAX>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    const int waves = p.fast_waves ? std::min((int)p.fast_waves, kRingWaves) : kRingWaves;
    hipLaunchKernelGGL((kaneko_fast_ring_kernel<M, TMAX>), dim3(blocks), dim3(kWaveSize * waves), lds, s, p);
    return hipGetLastError();
}

// BCHK_FAST_RING=0 in the environment selects the staged kernel (measurements)
static bool use_ring() {
    static int r = -1;
    if (r < 0) {
        const char *e = getenv("BCHK_FAST_RING");
        r = (e && atoi(e) == 0) ? 0 : 1;
    }
    return r != 0;
}

template <int M, int TMAX>
static hipError_t launch_fast_impl(const SearchParams &p, size_t lds, hipStream_t s) {
    constexpr int N = Geo<M>::N;
    constexpr int KMAX = (2 * TMAX < N - 1) ? 2 * TMAX : N - 1;
    if constexpr (KMAX + 2 <= 16) {
        // no stats record: the flags are not observable, selection suffices
        if (!p.st && !getenv("BCHK_FAST_FULLSORT")) {
            const bool ring = use_ring() && kRingPerCU * ring_lds_bytes<M>(p.td.bytes) <= 160 * 1024;
            return ring ? launch_fast_ring<M, TMAX>(p, s) : launch_fast_sel<M, TMAX, true>(p, lds, s);
        }
    }
    return launch_fast_sel<M, TMAX, false>(p, lds, s);
}

// ---------------------------------------------------------------------------------------
// Long codes (m >= 7, TMAX <= 15): the lane-per-codeword pre-pass of kaneko_first_kernel.
// The wave-per-codeword first kernel spends ~1 700 wave instructions on each codeword (a
// 64-lane selection network, cross-lane syndromes and key equations) although at the SNRs
// of use nearly every codeword returns at test pattern 0 or 1. This kernel gives each lane
// one codeword of a 64-row chunk and decides exactly those two exits, as the n <= 63 fast
// kernel does (fast_decide: the same certified tests), and marks the rows it finished in
// pre_mask; the first kernel then takes only the others, from scratch.
//   - rows stream through a per-wave LDS buffer 16 positions at a time (8-B loads, four
//     rows of 128 contiguous bytes per wave instruction; the next segment's loads are in
//     flight while this one is keyed), each lane reading its own row back;
//   - 32-bit keys: a 24-bit monotone prefix of |y| (5 exponent bits over [2^-27, 2^5), 19
//     mantissa bits) above the 8-bit position; the 32 smallest are kept sorted (Green's
//     16-key network per segment, then a bitonic merge into the kept 32), which covers the
//     ranks KMAX + 2 <= 32 the decision reads;
//   - hard-decision syndromes from the LDS column table; the decodes per lane
//     (alg_decode_lanes: binary BM, split test, wave-spread Chien scan of each success).
constexpr int kLaneWaves = 8;                   // waves per workgroup (2 workgroups per CU)
constexpr int kLaneSeg = 16;                    // positions per staged segment
constexpr int kLaneRowD = kLaneSeg + 1;         // hi words per staged row (pad: conflict-free reads)
constexpr int kLaneKeep = 32;
// the row buffer (64 x kLaneRowD hi words), then the parked keys (64 x 33), then the masks
constexpr int kLaneWaveBytes = 64 * (kLaneKeep + 1) * 4;

// 24-bit prefix (5 exponent bits, 19 mantissa bits; 0: |y| < 2^-27 or zero, all ones:
// |y| >= 32, inf, NaN) above the 8-bit position
__device__ __forceinline__ uint32_t sort_key8(uint32_t hi, int pos) {
    const uint32_t ahi = hi & 0x7FFFFFFFu;
    const uint32_t d = __builtin_elementwise_sub_sat(ahi, (uint32_t)(1023 - 27) << 20) >> 1;
    const uint32_t pre = d < 0xFFFFFFu ? d : 0xFFFFFFu;
    return (pre << 8) | (uint32_t)pos;
}

// kept[0..32) and nk[0..16) sorted -> kept = the 32 smallest of both, sorted: kept with the
// reversed nk (padded with +inf) taken elementwise by min is bitonic, then a bitonic merge
__device__ __forceinline__ void merge_low32_16(uint32_t (&kept)[32], const uint32_t (&nk)[16]) {
#pragma unroll
    for (int i = 16; i < 32; ++i) {
        const uint32_t a = kept[i], b = nk[31 - i];
        kept[i] = a < b ? a : b;
    }
    uint32_t *key = kept;
#pragma unroll
    for (int j = 16; j > 0; j >>= 1) {
#pragma unroll
        for (int i = 0; i < 32; ++i)
            if (!(i & j)) BCHK_CAS(i, i + j)
    }
}

template <int NW>
struct LaneRes {
    int state;  // 0 unresolved, 1 returned at i = 0, 2 returned at i = 1
    Mask<NW> best;
    double l0;
};

// bit pos of a mask: the words masked arithmetically (a select chain over the words is
// turned into a dynamically indexed stack copy -- scratch)
template <int NW>
__device__ __forceinline__ bool mask_bit(const Mask<NW> &m, int pos) {
    uint32_t b = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const uint32_t in = (uint32_t)((pos >> 6) == s);
        b |= (uint32_t)(m.w[s] >> (pos & 63)) & in;
    }
    return b & 1u;
}

// Decoder::decode (src/Decoder.cpp:298-321) of one word per lane for the pre-pass, where
// nearly every lane succeeds: binary BM (bm_locator); the roots of a locator of degree 1
// (1 + C1 x: x = 1/C1) and 2 (1 + C1 x + C2 x^2 = 0 with x = (C1/C2) z: z^2 + z = C2/C1^2,
// solved by the table quad[c] = a root z, 0 when there is none; C1 = 0 is a double root)
// in closed form, degree 3 too (below); degree >= 4 by the wave-spread Chien scan of
// alg_decode_lanes_g, one scan per such lane. Success and flipped positions as alg_core's (a root alpha^k flips
// position (n - k) mod n, :287): L <= t, deg >= 1 distinct roots in GF(2^m)*.
template <int M, int TMAX>
__device__ __forceinline__ bool lane_alg_decode(const uint8_t *ex, const uint16_t *lg, const uint8_t *quad,
                                                const uint32_t *cub, const uint32_t *Sw, int t, Mask<Geo<M>::NW> &E,
                                                bool act) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    const int lane = (int)__lane_id();
    uint32_t C[TMAX + 1];
    int L;
    bm_locator<M, TMAX>(ex, lg, Sw, t, C, L);
    int deg = 0;
#pragma unroll
    for (int i = 1; i <= TMAX; ++i) deg = C[i] ? i : deg;
    bool ok = act && (L <= t) && (deg >= 1);
#pragma unroll
    for (int s = 0; s < NW; ++s) E.w[s] = 0;
    auto pos_of = [&](int k) { return k ? N - k : 0; };  // root alpha^k, k in [0, n)
    if (ok && deg == 1) {
        const int l1 = lg[C[1]];
        mask_set<NW>(E, pos_of(l1 ? N - l1 : 0));  // x = 1 / C1
    } else if (ok && deg == 2) {
        if (C[1] == 0u) {
            ok = false;
        } else {
            const int l1 = lg[C[1]], l2 = lg[C[2]];
            int lc = l2 - 2 * l1;
            lc += lc < 0 ? N : 0;
            lc += lc < 0 ? N : 0;
            const uint32_t z0 = quad[ex[lc]];
            if (z0 == 0u) {
                ok = false;
            } else {
                int base = l1 - l2;
                base += base < 0 ? N : 0;
                int k0 = base + lg[z0], k1 = base + lg[z0 ^ 1u];
                k0 -= k0 >= N ? N : 0;
                k1 -= k1 >= N ? N : 0;
                mask_set<NW>(E, pos_of(k0));
                mask_set<NW>(E, pos_of(k1));
            }
        }
    } else if (ok && deg == 3) {
        // sigma(X) = X^3 + a X^2 + b X + c (X = 1/x, the error locators): X = Y + a gives
        // Y^3 + p Y + q with p = a^2 + b, q = a b + c; q = 0: a double root; p = 0: Y^3 = q
        // (three roots iff 3 | n and q is a cube); else Y = sqrt(p) W, W^3 + W = q / p^(3/2)
        // (cub[r]: its roots, three or fewer)
        const uint32_t a = C[1], b = C[2], c = C[3];
        const int la = lg[a], lb = lg[b];
        const uint32_t P = (a ? (uint32_t)ex[2 * la] : 0u) ^ b;
        const uint32_t Q = (a && b ? (uint32_t)ex[la + lb] : 0u) ^ c;
        uint32_t Y0 = 0, Y1 = 0, Y2 = 0;
        bool three = false;
        if (Q != 0u) {
            const int lq = lg[Q];
            if (P == 0u) {
                if constexpr (N % 3 == 0) {
                    if (lq % 3 == 0) {
                        const int c3 = lq / 3;
                        Y0 = ex[c3];
                        Y1 = ex[c3 + N / 3];
                        Y2 = ex[c3 + 2 * (N / 3)];
                        three = true;
                    }
                }
            } else {
                const int lp = lg[P];
                const int ls = (lp & 1) ? (lp + N) >> 1 : lp >> 1;  // log sqrt(p)
                int lr = lq - 3 * ls;
                lr += lr < 0 ? N : 0;
                lr += lr < 0 ? N : 0;
                lr += lr < 0 ? N : 0;
                const uint32_t e3 = cub[ex[lr]];
                if ((e3 >> 24) == 3u) {
                    const uint32_t w0 = e3 & 255u, w1 = (e3 >> 8) & 255u, w2 = (e3 >> 16) & 255u;
                    Y0 = w0 ? ex[lg[w0] + ls] : 0u;
                    Y1 = w1 ? ex[lg[w1] + ls] : 0u;
                    Y2 = w2 ? ex[lg[w2] + ls] : 0u;
                    three = true;
                }
            }
        }
        const uint32_t X0 = Y0 ^ a, X1 = Y1 ^ a, X2 = Y2 ^ a;
        if (!three || !X0 || !X1 || !X2) {
            ok = false;
        } else {
            mask_set<NW>(E, lg[X0]);
            mask_set<NW>(E, lg[X1]);
            mask_set<NW>(E, lg[X2]);
        }
    }
    const bool scan = ok && deg >= 4;
    int lc[TMAX + 1];
#pragma unroll
    for (int i = 0; i <= TMAX; ++i) lc[i] = lg[C[i]];
    for (uint64_t sm = ballot(scan); sm; sm &= sm - 1) {
        const int src = (int)__builtin_ctzll(sm);
        const int dg = uni(__shfl(deg, src, 64));
        int kk[NW], ik[NW];
        uint32_t v[NW];
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int pos = lane + 64 * s;
            kk[s] = pos ? N - pos : 0;
            ik[s] = 0;
            v[s] = 0;
        }
#pragma unroll
        for (int i = 0; i <= TMAX; ++i) {
            if (i <= dg) {
                const int lti = __builtin_amdgcn_readlane(lc[i], src);
#pragma unroll
                for (int s = 0; s < NW; ++s) {
                    v[s] ^= gf_exp2<M>(ex, lti, ik[s]);
                    ik[s] += kk[s];
                    ik[s] = ik[s] >= N ? ik[s] - N : ik[s];
                }
            }
        }
        int cnt = 0;
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const uint64_t r = ballot(lane + 64 * s < N && v[s] == 0u);
            cnt += __popcll(r);
            if (lane == src) E.w[s] = r;
        }
        if (lane == src && cnt != dg) ok = false;
    }
    return ok;
}

// fast_decide for n <= 255 (NW words): the same exits, tests and bounds from k[0..KMAX+1]
// (k: the lane's kept keys, parked in LDS while the decoders hold their registers)
template <int M, int TMAX>
__device__ __forceinline__ LaneRes<Geo<M>::NW> lane_decide(const uint8_t *ex, const uint16_t *lg, const uint32_t *col,
                                                           const uint8_t *quad, const uint32_t *cub,
                                                           const uint32_t *syn8, const uint32_t *k, uint32_t kmax_real,
                                                           const Mask<Geo<M>::NW> &yH, const double *yrow, bool live,
                                                           int t, double s2) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    constexpr int W = (TMAX + 3) / 4;
    constexpr int KMAX = 2 * TMAX;
    static_assert(KMAX + 2 <= kLaneKeep, "the kept keys cover the decision's ranks");
    constexpr int NPF = KMAX + 1;
    bool bad = (k[0] >> 8) == 0u || (kmax_real >> 8) == 0xFFFFFFu;
#pragma unroll
    for (int r = 0; r < KMAX + 1; ++r) bad |= ((k[r] ^ k[r + 1]) >> 8) == 0u;
    const uint32_t *pre = k;
    const int o0 = (int)(k[0] & 255u);
    const double c2 = 2.0 / s2;
    // syndrome of the hard decision (Decoder::findSyndromPoly :184-207): the XOR of the
    // byte table's entries (syn8[j][v] = the syndrome of byte value v at positions 8j ..
    // 8j + 7; L2-resident, one 16-B load per byte of the row)
    uint32_t S0[W];
#pragma unroll
    for (int w = 0; w < W; ++w) S0[w] = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const int j = 8 * s + b;
            if (8 * j < N) {
                const uint32_t v = (uint32_t)(yH.w[s] >> (8 * b)) & 255u;
                const uint32_t *e = syn8 + ((size_t)j * 256 + v) * W;
#pragma unroll
                for (int w = 0; w < W; ++w) S0[w] ^= e[w];
            }
        }
    }
    // calcL (:69-77, index order) and calcRightSide (:54-67, sorted order) for `diff`, as
    // fast_decide's accept
    auto accept = [&](const Mask<NW> &diff, double &l, bool &ret) {
        constexpr int LMAX = TMAX + 1;
        const int m = mask_popc<NW>(diff);
        const int border = (2 * t + 1) - m;
        double g[LMAX];
#pragma unroll
        for (int j = 0; j < LMAX; ++j) g[j] = 0.0;
        Mask<NW> v = diff;
#pragma unroll
        for (int j = 0; j < LMAX; ++j) {  // the j-th flipped position, ascending
#if BCHK_ACC_BREAK
            if (!ballot(j < m)) break;  // no lane has a j-th flipped position
#endif
            int pj = -1;
#pragma unroll
            for (int s = NW - 1; s >= 0; --s)
                if (v.w[s]) pj = 64 * s + (int)__builtin_ctzll(v.w[s]);
#pragma unroll
            for (int s = 0; s < NW; ++s)
                if ((pj >> 6) == s && pj >= 0) v.w[s] &= v.w[s] - 1;
            if (pj >= 0) g[j] = yrow[pj];
        }
        l = 0.0;
#pragma unroll
        for (int j = 0; j < LMAX; ++j) {
#if BCHK_ACC_BREAK
            if (!ballot(j < m)) break;
#endif
            if (j < m) l += fabs((2.0 * g[j]) / s2);
        }
        double rs_lo = 0.0;
        int taken = 0;
#pragma unroll
        for (int r = 0; r < NPF; ++r) {
            const bool ag = !mask_bit<NW>(diff, (int)(pre[r] & 255u));
            if (ag && taken < border) {
                const uint32_t pr = pre[r] >> 8;  // eb (5 bits) | 19 mantissa bits
                const uint64_t bits = (uint64_t)((pr << 1) + (996u << 20)) << 32;
                rs_lo += __longlong_as_double((long long)bits) * c2;
                ++taken;
            }
        }
        ret = (taken >= border) && (m <= LMAX) && (l < rs_lo * (1.0 - 0x1p-40));
    };

    LaneRes<NW> R;
    R.state = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) R.best.w[s] = 0;
    R.l0 = DBL_MAX;
    bool zero0 = true;
#pragma unroll
    for (int w = 0; w < W; ++w) zero0 = zero0 && S0[w] == 0u;
    Mask<NW> E;
    const bool ok0 = lane_alg_decode<M, TMAX>(ex, lg, quad, cub, S0, t, E, live && !bad && !zero0);
    if (live && !bad && ok0) {
        double l;
        bool ret;
        accept(E, l, ret);
        if (ret) { R.state = 1; R.best = E; R.l0 = l; }
    }
    // i = 1 where i = 0 failed (:371): a codeword hard decision (zero syndrome) returns to
    // itself (D = 0, l = 0); otherwise pattern 1 flips rank 0 and is decoded
    if (live && !bad && !ok0 && zero0) {
        Mask<NW> z;
#pragma unroll
        for (int s = 0; s < NW; ++s) z.w[s] = 0;
        double l;
        bool ret;
        accept(z, l, ret);
        if (ret) { R.state = 2; R.l0 = l; }
    }
    const bool need1 = live && !bad && !ok0 && !zero0;
    if (ballot(need1)) {
        uint32_t S1[W];
#pragma unroll
        for (int w = 0; w < W; ++w) S1[w] = S0[w] ^ col[o0 * W + w];
        const bool ok1 = lane_alg_decode<M, TMAX>(ex, lg, quad, cub, S1, t, E, need1);
        if (need1 && ok1) {
            Mask<NW> diff = E;
#pragma unroll
            for (int s = 0; s < NW; ++s) diff.w[s] ^= (o0 >> 6) == s ? 1ull << (o0 & 63) : 0ull;
            double l;
            bool ret;
            accept(diff, l, ret);
            if (ret) { R.state = 2; R.best = diff; R.l0 = l; }
        }
    }
    return R;
}

template <int M, int TMAX>
#ifndef BCHK_LANE_WPE
#define BCHK_LANE_WPE 4  // waves per SIMD (two workgroups per CU; LDS allows four)
#endif
__global__ void __launch_bounds__(kWaveSize * kLaneWaves) __attribute__((amdgpu_waves_per_eu(BCHK_LANE_WPE, BCHK_LANE_WPE)))
kaneko_lane_kernel(SearchParams p) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    static_assert(kLaneSeg == 16, "segment = four rows of 16 positions per wave instruction");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    load_tables(smem, p.tables, p.td.bytes);
    const uint32_t tb = (p.td.bytes + 15) & ~15u;
    uint32_t *cub = reinterpret_cast<uint32_t *>(smem + tb);  // [2^m]: roots of W^3 + W = r
    uint8_t *quad = smem + tb + 4 * (1 << M);  // [2^m]: a root z of z^2 + z = c, 0 when there is none
    for (int c = threadIdx.x; c < (1 << M); c += blockDim.x) {
        quad[c] = 0;
        cub[c] = 0;
    }
    __syncthreads();
    const uint8_t *ex = smem + p.td.off_exp;
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(smem + p.td.off_log);
    const uint32_t *col = reinterpret_cast<const uint32_t *>(smem + p.td.off_col);
    for (int z = threadIdx.x; z < (1 << M); z += blockDim.x) {
        // c = z^2 + z; z and z + 1 give the same c (either root serves)
        const uint32_t z2 = z ? ex[2 * lg[z]] : 0u;
        if (z != 1) quad[z2 ^ (uint32_t)z] = (uint8_t)z;
        // r = z^3 + z: up to three roots (bytes 0..2) and their count (byte 3)
        int l3 = z ? 3 * lg[z] : 0;  // the exp table is zero from 2n - 1 on: reduce mod n
        l3 -= l3 >= Geo<M>::N ? Geo<M>::N : 0;
        l3 -= l3 >= Geo<M>::N ? Geo<M>::N : 0;
        const uint32_t z3 = z ? ex[l3] : 0u;
        const uint32_t r = z3 ^ (uint32_t)z;
        const uint32_t old = atomicAdd(&cub[r], 1u << 24) >> 24;
        if (old < 3u) atomicOr(&cub[r], (uint32_t)z << (8 * old));
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = uni((int)(threadIdx.x >> 6));  // wave-uniform: SGPRs
    uint8_t *wb = smem + tb + 5 * (1 << M) + wid * kLaneWaveBytes;
    uint32_t *seg = reinterpret_cast<uint32_t *>(wb);  // hi words, [64][kLaneRowD]
    const uint32_t gk = blockIdx.x * kLaneWaves + (uint32_t)wid;  // this wave's chunk
    const uint32_t nch = (p.count + 63u) / 64u;
    if (gk >= nch) return;
    const uint32_t cw0 = 64u * gk, cw = cw0 + (uint32_t)lane;
    const bool live = cw < p.count;
    const uint32_t rows = p.count - cw0 < 64u ? p.count - cw0 : 64u;
    // segment loads: instruction i, lane l -> row r = 4 i + l / 16, slot l % 16 of the row's
    // segment g. Segments follow the 128-B lines, not the positions: row r's position 0 sits
    // at 8-B slot a_r = (c0 + r N) mod 16 of its line, so segment g holds positions
    // 16 g - a_r .. 16 g - a_r + 15, one whole line fetched once (position-aligned segments
    // straddle two lines whose second half L2 had often dropped before the next segment
    // asked for it: 1.6x the input read). Positions outside [0, n) are masked out; the
    // offsets are all in the lane's VGPR (no scalar offset), so anything past the chunk's
    // rows, or before them, is out of range and reads 0.
    const int lr = lane >> 4, lj = lane & 15;
    const __amdgpu_buffer_rsrc_t ysrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(p.y + (size_t)cw0 * N), (short)0, (int)(rows * (uint32_t)N * 8u), 0x00020000);
    const uint32_t c0 = (uint32_t)(reinterpret_cast<uintptr_t>(p.y + (size_t)cw0 * N) >> 3) & 15u;
    int vo[4];  // row 4 q + lr (and every 16th row on): its segment 0's offset (hi word)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = 4 * q + lr;
        const int a = (int)((c0 + (uint32_t)(r * N)) & 15u);
        vo[q] = (r * N + lj - a) * 8 + 4;
    }
    const int aself = (int)((c0 + (uint32_t)(lane * N)) & 15u);
    constexpr int NSEG = (N + 15 + kLaneSeg - 1) / kLaneSeg;
    // (the keys and the hard decision need the hi words only: half the registers and LDS;
    // the acceptance tests read exact values from the rows again)
    uint32_t pf[16];
    auto load_seg = [&](int g) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            pf[i] = __builtin_amdgcn_raw_buffer_load_b32(ysrc, vo[i & 3] + kLaneSeg * 8 * g + (i >> 2) * 16 * N * 8, 0, 0);
    };
    load_seg(0);
    uint32_t kept[kLaneKeep];
#pragma unroll
    for (int i = 0; i < kLaneKeep; ++i) kept[i] = 0xFFFFFFFFu;
    uint32_t kmax_real = 0;
    Mask<NW> yH;
#pragma unroll
    for (int s = 0; s < NW; ++s) yH.w[s] = 0;
#pragma nounroll
    for (int g = 0; g < NSEG; ++g) {
        wave_sync();  // the previous segment's reads are done
#pragma unroll
        for (int i = 0; i < 16; ++i) seg[(4 * i + lr) * kLaneRowD + lj] = pf[i];
        wave_sync();
        if (g + 1 < NSEG) load_seg(g + 1);
        const int p0 = kLaneSeg * g - aself;  // this lane's first position of the segment
        uint32_t nk[16];
        uint32_t sb = 0;  // sign bits of the segment (position p0 + i -> bit i)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int pos = p0 + i;
            const bool in = pos >= 0 && pos < N;
            const uint32_t hi = seg[lane * kLaneRowD + i];
            nk[i] = in ? sort_key8(hi, pos) : 0xFFFFFFFFu;
            sb |= (in ? (~hi >> 31) : 0u) << i;
        }
        sort16<0>(nk);
        // the real keys sort below the padding: the largest is rank cnt - 1
        const int hiend = p0 + 16 < N ? p0 + 16 : N, loend = p0 > 0 ? p0 : 0;
        const int cnt = hiend - loend;
        uint32_t top = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) top = cnt == i + 1 ? nk[i] : top;
        kmax_real = top > kmax_real ? top : kmax_real;
        merge_low32_16(kept, nk);
        // y > 0 is the clear sign bit (the hard decision, :336-342); y = +0 has prefix 0 and
        // is sent to the slow path by lane_decide. Bits p0 .. p0 + 15 may span two words.
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int sh = p0 - 64 * s;
            const uint64_t c = (sh >= 0 && sh < 64) ? (uint64_t)sb << (sh & 63)
                             : (sh < 0 && sh > -16) ? (uint64_t)sb >> ((-sh) & 63) : 0ull;
            yH.w[s] |= c;
        }
    }
    // the kept keys into the (now free) row buffer, lane-major with stride 33 (conflict-free)
    wave_sync();
    static_assert(64 * (kLaneKeep + 1) * 4 <= kLaneWaveBytes, "the parked keys fit the row buffer");
    uint32_t *kl = reinterpret_cast<uint32_t *>(wb) + lane * (kLaneKeep + 1);
#pragma unroll
    for (int i = 0; i < kLaneKeep; ++i) kl[i] = kept[i];
    int t = p.t;
    double s2 = p.s2;
    asm volatile("" : "+s"(t), "+s"(s2));
    const double *yrow = p.y + (size_t)(live ? cw : cw0) * N;
    const LaneRes<NW> R = lane_decide<M, TMAX>(ex, lg, col, quad, cub, p.syn8, kl, kmax_real, yH, yrow, live, t, s2);

    // ---- outputs: decoded rows of the finished codewords (others untouched: the first
    // kernel writes them), their l0, the fused counters and the chunk's pre_mask word
    const bool resolved = live && R.state != 0;
    Mask<NW> x;
#pragma unroll
    for (int s = 0; s < NW; ++s) x.w[s] = yH.w[s] ^ R.best.w[s];
    uint32_t e = 0;
    uint8_t *dst = p.res + (size_t)cw0 * N;
    const uint8_t *txb = p.tx ? p.tx + (size_t)cw0 * N : nullptr;
    wave_sync();  // the segment buffer becomes the masks' area
    uint64_t *xm = reinterpret_cast<uint64_t *>(wb);            // [64][NW]
    uint32_t *rowerr = reinterpret_cast<uint32_t *>(wb + 64 * NW * 8);
    if (rows == 64u && ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(txb)) & 15u) == 0) {
        const uint64_t rm = ballot(resolved);
#pragma unroll
        for (int s = 0; s < NW; ++s) xm[lane * NW + s] = x.w[s];
        rowerr[lane] = 0u;
        wave_sync();
        bool anyerr = false;
        for (int q = lane; q < 4 * N; q += 64) {
            const int b0 = 16 * q, r1 = b0 / N, o = b0 - N * r1;
            const bool span = o > N - 16;
            const int r2 = span ? r1 + 1 : r1;
            const int wi = o >> 6, sh = o & 63;
            const uint64_t a0 = xm[r1 * NW + wi];
            const uint64_t a1 = (wi + 1 < NW && sh) ? xm[r1 * NW + wi + 1] : 0ull;
            uint64_t w = (a0 >> sh) | (sh ? a1 << (64 - sh) : 0ull);
            if (span) w = (w & ((1ull << (N - o)) - 1ull)) | (xm[r2 * NW] << (N - o));
            uint32_t nw[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) nw[d] = nib_bytes((uint32_t)(w >> (4 * d)) & 15u);
            const uint32_t in2 = span ? (0xFFFFu << (N - o)) & 0xFFFFu : 0u;
            const uint32_t keep = (((rm >> r1) & 1ull) ? 0u : (~in2 & 0xFFFFu)) |
                                  (((rm >> r2) & 1ull) ? 0u : in2);
            if (!keep) {
                reinterpret_cast<uint4 *>(dst)[q] = make_uint4(nw[0], nw[1], nw[2], nw[3]);
            } else if (keep != 0xFFFFu) {
                for (uint32_t wm = ~keep & 0xFFFFu; wm; wm &= wm - 1) {
                    const int i = __builtin_ctz(wm);
                    dst[16 * q + i] = (uint8_t)(nw[i >> 2] >> (8 * (i & 3)));
                }
            }
            if (txb) {
                const uint4 a = reinterpret_cast<const uint4 *>(txb)[q];
                const uint32_t xx[4] = {a.x ^ nw[0], a.y ^ nw[1], a.z ^ nw[2], a.w ^ nw[3]};
                if (xx[0] | xx[1] | xx[2] | xx[3]) {
                    anyerr = true;
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        if ((xx[i >> 2] >> (8 * (i & 3))) & 0xFFu) atomicAdd(&rowerr[i < N - o ? r1 : r2], 1u);
                }
            }
        }
        if (txb && ballot(anyerr)) {
            wave_sync();
            e = resolved ? rowerr[lane] : 0u;
        }
    } else if (resolved) {  // partial chunk (or unaligned buffers): the row byte by byte
        for (int pos = 0; pos < N; ++pos) {
            const uint8_t bit = mask_bit<NW>(x, pos) ? 1u : 0u;
            dst[lane * N + pos] = bit;
            if (txb) e += txb[lane * N + pos] != bit ? 1u : 0u;
        }
    }
    if (p.cnt) fast_counters(p, cw0, N, resolved, R.state, e);
    if (resolved && p.l0) p.l0[cw] = R.l0;
    const uint64_t done = ballot(resolved);
    if (lane == 0) p.pre_mask[gk] = done;
}

template <int M, int TMAX>
static hipError_t launch_lane_impl(const SearchParams &p, size_t, hipStream_t s) {
    const uint32_t chunks = (p.count + 63u) / 64u;
    const int blocks = (int)((chunks + kLaneWaves - 1) / kLaneWaves);
    const size_t lds = ((p.td.bytes + 15) & ~size_t(15)) + 5 * (1u << M) + (size_t)kLaneWaves * kLaneWaveBytes;
    static bool attr = false;
    if (!attr && lds > 65536) {
        (void)hipFuncSetAttribute((const void *)&kaneko_lane_kernel<M, TMAX>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    if (blocks > 0) hipLaunchKernelGGL((kaneko_lane_kernel<M, TMAX>), dim3(blocks), dim3(kWaveSize * kLaneWaves), lds, s, p);
    return hipGetLastError();
}

// the same (m, TMAX) buckets as select_first_long (the column table's stride)
bool select_lane(int m, int t, FastFn *out) {
    if (m == 7 && t <= 8) { *out = &launch_lane_impl<7, 8>; return true; }
    if (m == 8 && t <= 15) { *out = &launch_lane_impl<8, 15>; return true; }
    return false;
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
