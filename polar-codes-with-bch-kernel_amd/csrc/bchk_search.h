// bchk_search.h -- the device side of the wave-per-codeword Kaneko search (prep, test
// pattern decoding, the reference's ordered acceptance, the analytic tail, the work queues),
// shared by the search / cooperative kernels (bchk_kernels.hip) and the fast ring kernel
// (bchk_fast.hip), whose waves run the first pass beside the fast path. Reference:
// src/KanekoKernelProcessor.cpp:335-407, src/Decoder.cpp:184-321.
#pragma once
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdlib.h>
#include <stdint.h>

#include "bchk_core.h"
#include "bchk_launch.h"

// Tuning knobs (experiment builds override them): chunks per syndrome-table lookup group,
// and calcL terms whose LDS loads are issued together.
#ifndef BCHK_TAB_GROUP
#define BCHK_TAB_GROUP 1
#endif
#ifndef BCHK_LSUM_BATCH
#define BCHK_LSUM_BATCH 8
#endif

namespace bchk {

// -------------------------------------------------------------- LDS layout
template <int M, int TMAX>
struct Smem {
    static constexpr int NP = 64 * Geo<M>::NW;     // padded positions per wave
    // sorted |alpha| (f64), |alpha| by position (f64), order (u8)
    static constexpr int WAVE_BYTES = NP * 8 * 2 + NP;
};
#ifndef BCHK_COOP_WAVES
#define BCHK_COOP_WAVES 16
#endif
constexpr int kCoopWaves = BCHK_COOP_WAVES;  // waves that share one heavy codeword (1024 threads)
// long codes: test patterns decoded one at a time by the whole wave before the 64-pattern
// chunks (search_codeword)
#ifndef BCHK_SEQ_PATTERNS
#define BCHK_SEQ_PATTERNS 4
#endif
constexpr int kSeqPatterns = BCHK_SEQ_PATTERNS;
static_assert(kSeqPatterns >= 1 && kSeqPatterns <= 64, "sequential patterns lie in chunk 0");

// ------------------------------------------------------- per-codeword prep
// Reference: KanekoKernelProcessor::decode(answer, word, res) prologue and set-up,
// src/KanekoKernelProcessor.cpp:336-359 (and :213-234 for decode(word, res)).
template <int M, int TMAX>
struct Prep {
    static constexpr int NW = Geo<M>::NW, W = (TMAX + 3) / 4;
    double av[NW];     // |alpha| of position lane + 64 s
    double asv[NW];    // sorted |alpha|, rank lane + 64 s
    int ordv[NW];      // position of rank lane + 64 s
    Mask<NW> yH;       // hard decision (wave-uniform)
    uint32_t S0[W];    // odd syndromes of yH (wave-uniform)
    uint32_t scol[W];  // lane b: odd-syndrome column of position ord[b]
    int ordb;          // lane b: ord[b]
    uint32_t Lo[W];    // syndrome contribution of pattern bits 0..5 = lane
    Mask<NW> Plo;      // flipped positions of pattern bits 0..5 = lane
    bool tie;          // two |alpha| exactly equal
};

template <int M, int TMAX>
__device__ __forceinline__ void prep_syndromes(const uint32_t *col, int lane, Prep<M, TMAX> &P);

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

// One compare-exchange step of the bitonic network at lane distance J < 64.
template <int J, int NW>
__device__ __forceinline__ void bitonic_lane_step(uint64_t (&key)[NW], int kk, int lane) {
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int e = lane + 64 * s;
        const uint64_t o = lane_xor64<J>(key[s], lane);
        const bool takemin = ((lane & J) == 0) == ((e & kk) == 0);
        const bool lt = o < key[s];
        key[s] = (takemin == lt) ? o : key[s];
    }
}

// Ascending bitonic sort of a wave's 64 NW keys, element e = lane + 64 s in key[s]:
// partners at distance < 64 are exchanged across lanes, larger distances within a lane.
// Unrolled by template recursion, so every register index is a constant (a runtime index
// would put the keys in scratch memory).
template <int KK, int J, int NW>
__device__ __forceinline__ void bitonic_merge_steps(uint64_t (&key)[NW], int lane) {
    if constexpr (J >= 64) {
        constexpr int js = J >> 6;
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            if (s & js) continue;  // s is the lower element of the pair (s, s | js)
            const bool up = ((64 * s) & KK) == 0;
            const uint64_t a = key[s], b = key[s | js];
            const bool sw = up ? (a > b) : (a < b);
            key[s] = sw ? b : a;
            key[s | js] = sw ? a : b;
        }
    } else {
        bitonic_lane_step<J, NW>(key, KK, lane);
    }
    if constexpr (J > 1) bitonic_merge_steps<KK, J / 2, NW>(key, lane);
}
template <int KK, int NW>
__device__ __forceinline__ void bitonic_stages(uint64_t (&key)[NW], int lane) {
    bitonic_merge_steps<KK, KK / 2, NW>(key, lane);
    if constexpr (KK < 64 * NW) bitonic_stages<2 * KK, NW>(key, lane);
}
template <int NW>
__device__ __forceinline__ void wave_bitonic_sort(uint64_t (&key)[NW], int lane) {
    bitonic_stages<2, NW>(key, lane);
}

// the channel samples of codeword cw: yv[s] = position lane + 64 s (0 past n)
template <int M>
__device__ __forceinline__ void load_row(const SearchParams &p, uint32_t cw, int lane,
                                         double (&yv)[Geo<M>::NW]) {
    constexpr int N = Geo<M>::N;
    const double *y = p.y + (size_t)cw * N;
#pragma unroll
    for (int s = 0; s < Geo<M>::NW; ++s) yv[s] = lane + 64 * s < N ? y[lane + 64 * s] : 0.0;
}

// prep from a row already loaded (yv[s] = sample of position lane + 64 s)
template <int M, int TMAX>
__device__ __forceinline__ void prep_loaded(const SearchParams &p, const uint32_t *col, double *as,
                                            double *ap, uint8_t *ordl, const double (&yv)[Geo<M>::NW],
                                            int lane, Prep<M, TMAX> &P);

template <int M, int TMAX>
__device__ __forceinline__ void prep_codeword(const SearchParams &p, const uint32_t *col, double *as, double *ap,
                              uint8_t *ordl, uint32_t cw, int lane, Prep<M, TMAX> &P) {
    double yv[Geo<M>::NW];
    load_row<M>(p, cw, lane, yv);
    prep_loaded<M, TMAX>(p, col, as, ap, ordl, yv, lane, P);
}

template <int M, int TMAX>
__device__ __forceinline__ void prep_loaded(const SearchParams &p, const uint32_t *col, double *as,
                                            double *ap, uint8_t *ordl, const double (&yv)[Geo<M>::NW],
                                            int lane, Prep<M, TMAX> &P) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    // alpha = 2*word/pow(sd,2); yH; |alpha| (:336-342)
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        const bool valid = pos < N;
        const double yy = yv[s];
        const double al = (2.0 * yy) / p.s2;
        P.av[s] = valid ? fabs(al) : 0.0;
        P.yH.w[s] = ballot(valid && !(al <= 0.0));
    }
    // exact rank by (|alpha|, position): the stable order of std::sort's keys (:343).
    // |alpha| by position goes to LDS first.
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        if (pos < N) ap[pos] = P.av[s];
    }
    wave_sync();
    {
        // sort the wave's 64 NW keys (f64 bits of |alpha| with the low 8 mantissa bits
        // replaced by the position) with a bitonic network. Keys whose 55-bit |alpha|
        // prefixes all differ are ordered exactly as (|alpha|, position); a prefix tie between
        // sorted neighbours -- an exact tie or a near one -- takes the exact rank below. (Round
        // 3: also for n <= 63, where the O(n^2) rank cost ~10 instructions per position.)
        uint64_t key[NW];
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int pos = lane + 64 * s;
            key[s] = pos < N ? (((uint64_t)__double_as_longlong(P.av[s]) & ~0xFFull) | (uint64_t)pos)
                             : ~0ull;
        }
        wave_bitonic_sort<NW>(key, lane);
        bool ptie = false;
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            uint64_t nx = shfl64(key[s], (lane + 1) & 63);
            if (s + 1 < NW) nx = lane == 63 ? rdl64(key[s + 1 < NW ? s + 1 : s], 0) : nx;
            const int e = lane + 64 * s;
            ptie |= e + 1 < N && (key[s] >> 8) == (nx >> 8);
        }
        if (ballot(ptie) == 0ull) {
#pragma unroll
            for (int s = 0; s < NW; ++s) {
                const int q = lane + 64 * s;
                const int pos = (int)(key[s] & 0xFFull);
                P.ordv[s] = q < N ? pos : 0;
                P.asv[s] = q < N ? ap[pos] : 0.0;
                if (q < N) {
                    as[q] = P.asv[s];
                    ordl[q] = (uint8_t)pos;
                }
            }
            P.tie = false;
            wave_sync();
            prep_syndromes<M, TMAX>(col, lane, P);
            return;
        }
    }
    int rk[NW];
    bool tie = false;
#pragma unroll
    for (int s = 0; s < NW; ++s) rk[s] = 0;
#pragma unroll 8
    for (int q = 0; q < N; ++q) {
        const double aq = ap[q];
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int pos = lane + 64 * s;
            const bool lt = aq < P.av[s];
            const bool eq = aq == P.av[s];
            rk[s] += (lt || (eq && q < pos)) ? 1 : 0;
            tie |= eq && (q != pos) && (pos < N);
        }
    }
    P.tie = ballot(tie) != 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        if (pos < N) {
            as[rk[s]] = P.av[s];
            ordl[rk[s]] = (uint8_t)pos;
        }
    }
    wave_sync();
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int q = lane + 64 * s;
        P.asv[s] = q < N ? as[q] : 0.0;
        P.ordv[s] = q < N ? ordl[q] : 0;
    }
    prep_syndromes<M, TMAX>(col, lane, P);
}

// The hard decision's syndromes and the test-pattern syndrome columns (the prep's tail,
// after the order is known).
template <int M, int TMAX>
__device__ __forceinline__ void prep_syndromes(const uint32_t *col, int lane, Prep<M, TMAX> &P) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW, W = Prep<M, TMAX>::W;
    constexpr int NB = N < 31 ? N : 31;  // pattern bits in use (i < 2^31)
    // syndrome of the hard decision (Decoder::findSyndromPoly :184-207)
#pragma unroll
    for (int w = 0; w < W; ++w) P.S0[w] = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        if (pos < N && ((P.yH.w[s] >> lane) & 1ull)) {
#pragma unroll
            for (int w = 0; w < W; ++w) P.S0[w] ^= col[pos * W + w];
        }
    }
#pragma unroll
    for (int w = 0; w < W; ++w) P.S0[w] = wave_xor(P.S0[w]);
    // test patterns (calcError :36-51): bit b of i flips position ord[b]
    P.ordb = P.ordv[0];
#pragma unroll
    for (int w = 0; w < W; ++w) P.scol[w] = lane < NB ? col[P.ordb * W + w] : 0u;
#pragma unroll
    for (int w = 0; w < W; ++w) P.Lo[w] = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) P.Plo.w[s] = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
        if (b < NB) {
            const bool on = (lane >> b) & 1;
            const int pb = (int)rdl((uint32_t)P.ordb, b);
#pragma unroll
            for (int w = 0; w < W; ++w) P.Lo[w] ^= on ? rdl(P.scol[w], b) : 0u;
            if (on) mask_set<NW>(P.Plo, pb);
        }
    }
}

// Long codes, first kernel: what the first test patterns read of the order is the least
// reliable ranks -- patterns 0..3 flip ranks 0 and 1, calcRightSide takes at most 2t + 1
// agreeing ranks past at most t + 2 disagreeing ones, and the calcT scan decides small T
// from ranks <= t + 2 (accept_success bails out to the search kernel past the selection).
// So instead of sorting all n reliabilities (a 256-key bitonic network, ~1 100 VALU per
// codeword) the kernel selects the KSEL <= 64 smallest: a binary search over the high word of
// the |alpha| bits for a bound that between KSEL and 64 keys lie at or below (wave-uniform,
// ballot counts), then those keys -- one per lane -- are sorted by the 64-lane network.
template <int M, int TMAX>
constexpr int first_ksel() { return 3 * TMAX + 4 < 31 ? 31 : 3 * TMAX + 4; }
template <int M, int TMAX>
constexpr bool first_sel_capable() { return Geo<M>::NW > 1 && first_ksel<M, TMAX>() <= 64; }

// prep_loaded's state with ranks 0 .. nsel-1 exact (lane = rank, s = 0); false (nothing
// decided) when no such bound exists or two selected keys share their 55-bit prefix -- the
// caller then takes prep_loaded, whose exact rank resolves ties.
template <int M, int TMAX>
__device__ __forceinline__ bool prep_select(const SearchParams &p, const uint32_t *col, double *as,
                                            double *ap, uint8_t *ordl, const double (&yv)[Geo<M>::NW],
                                            int lane, Prep<M, TMAX> &P, int &nsel) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW, KLO = first_ksel<M, TMAX>();
    uint32_t kh[NW];
#pragma unroll
    for (int s = 0; s < NW; ++s) {  // :336-342
        const int pos = lane + 64 * s;
        const bool valid = pos < N;
        const double al = (2.0 * yv[s]) / p.s2;
        P.av[s] = valid ? fabs(al) : 0.0;
        P.yH.w[s] = ballot(valid && !(al <= 0.0));
        if (valid) ap[pos] = P.av[s];
        kh[s] = valid ? (uint32_t)((uint64_t)__double_as_longlong(P.av[s]) >> 32) : 0xFFFFFFFFu;
    }
    auto count = [&](uint32_t h) {
        int c = 0;
#pragma unroll
        for (int s = 0; s < NW; ++s) c += __popcll(ballot(kh[s] <= h));
        return c;
    };
    uint32_t h = 0x7FF00000u;  // +inf: every finite |alpha| lies at or below
    int c = count(h);
    if (c < KLO) return false;  // NaN samples
    // invariant: fewer than KLO keys below lo, at least KLO at or below h
    for (uint32_t lo = 0; c > 64 && lo < h;) {
        const uint32_t mid = lo + ((h - lo) >> 1);
        const int cm = count(mid);
        if (cm >= KLO) {
            h = mid;
            c = cm;
        } else {
            lo = mid + 1;
        }
    }
    if (c > 64) return false;
    // the selected keys, one per lane, then the 64-lane network
    double *scratch = as;  // the sorted ranks are written there after the exchange
    int base = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const bool sel = kh[s] <= h;
        const uint64_t bal = ballot(sel);
        const int r = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (sel)
            scratch[r] = __longlong_as_double(
                (long long)(((uint64_t)__double_as_longlong(P.av[s]) & ~0xFFull) | (uint64_t)(lane + 64 * s)));
        base += __popcll(bal);
    }
    wave_sync();
    uint64_t key[1];
    key[0] = lane < c ? (uint64_t)__double_as_longlong(scratch[lane]) : ~0ull;
    wave_sync();
    wave_bitonic_sort<1>(key, lane);
    const uint64_t nx = shfl64(key[0], (lane + 1) & 63);
    if (ballot(lane + 1 < c && (key[0] >> 8) == (nx >> 8))) return false;  // a prefix tie
    const int pos = (int)(key[0] & 0xFFull);
    P.ordv[0] = lane < c ? pos : 0;
    P.asv[0] = lane < c ? ap[pos] : 0.0;
#pragma unroll
    for (int s = 1; s < NW; ++s) {
        P.ordv[s] = 0;
        P.asv[s] = 0.0;
    }
    if (lane < c) {
        as[lane] = P.asv[0];
        ordl[lane] = (uint8_t)pos;
    }
    P.tie = false;
    wave_sync();
    prep_syndromes<M, TMAX>(col, lane, P);
    nsel = c;
    return true;
}

// The best codeword so far as a skip key: bit 63 valid, bits 32..39 u = its differences
// from the hard decision outside the NB <= 31 least reliable positions, bits 0..30 dR = its
// differences on them (bit b: sorted position b, the bit test pattern i flips, :36-51).
template <int M, int TMAX>
__device__ __forceinline__ uint64_t skip_key(const Mask<Geo<M>::NW> &best, const Prep<M, TMAX> &P, int lane) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    constexpr int NB = N < 31 ? N : 31;
    const int op = P.ordb;  // lane b: position of sorted rank b
    uint64_t dw = 0;
#pragma unroll
    for (int u = 0; u < NW; ++u) dw = (u == (op >> 6)) ? best.w[u] : dw;
    const uint32_t dR = (uint32_t)ballot(lane < NB && ((dw >> (op & 63)) & 1ull));
    const int u = mask_popc<NW>(best) - __popc(dR);
    return (1ull << 63) | ((uint64_t)(u > 255 ? 255 : u) << 32) | dR;
}
// pattern i re-finds the key's codeword (distance <= t): |D ^ P_i| = u + popc(dR ^ i)
__device__ __forceinline__ bool skip_lane(uint64_t skey, uint64_t i, int t) {
    const int u = (int)((skey >> 32) & 0xFFu);
    const uint32_t dR = (uint32_t)skey & 0x7FFFFFFFu;
    return (skey >> 63) && u + __popc(dR ^ ((uint32_t)i & 0x7FFFFFFFu)) <= t;
}

// Decode test patterns i = base + lane (base a multiple of 64) of G consecutive chunks
// (bases base, base + 64, ...): success and diff = yH ^ x (flipped pattern positions ^
// error locations); for successful lanes also m = calcM (:89-97) and l = calcL (:69-77),
// summed over diff in index order from the wave's |alpha|-by-position LDS slice
// (lane-parallel; the ordered acceptance only compares them). With the syndrome table the
// G lookups are issued together, so a wave has G bucket loads in flight.
//
// Long codes: a pattern whose word lies within distance t of a codeword found at an EARLIER
// pattern decodes to that codeword again (unique decoding, d >= 2t + 1; at distance 0 it
// fails) and cannot be an improvement, since l0 <= its l from then on; nothing else in the
// reference loop depends on a non-improving success (m0 only matters at an improvement,
// where :374 re-reads it). skey (skip_key) describes the best codeword so far; such
// patterns are reported as failures without decoding them -- same acceptance, same
// counters. At 5 dB on BCH(255,139,31) a third of a heavy codeword's patterns re-find its
// best codeword.
template <int M, int TMAX, int G, bool TAB>
__device__ __forceinline__ void decode_chunks(const Prep<M, TMAX> &P, uint64_t base, int t,
                                              const uint8_t *ex, const uint16_t *lg,
                                              const uint64_t *chien, const double *ap,
                                              const SyndTable &T, Mask<Geo<M>::NW> (&diff)[G],
                                              int (&m)[G], double (&l)[G], bool (&ok)[G],
                                              uint64_t skey = 0) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW, W = Prep<M, TMAX>::W;
    constexpr int NB = N < 31 ? N : 31;
    uint32_t Sw[G][W];
    Mask<NW> Pm[G], E[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        Pm[g] = P.Plo;
#pragma unroll
        for (int w = 0; w < W; ++w) Sw[g][w] = P.S0[w] ^ P.Lo[w];
        for (uint64_t hb = (base >> 6) + (uint64_t)g; hb; hb &= hb - 1) {  // wave-uniform
            const int b = 6 + (int)__builtin_ctzll(hb);
            if (b >= NB) continue;
            const int pb = (int)rdl((uint32_t)P.ordb, b);
#pragma unroll
            for (int w = 0; w < W; ++w) Sw[g][w] ^= rdl(P.scol[w], b);
            mask_set<NW>(Pm[g], pb);
        }
    }
    if constexpr (TAB) {
        // the decoder as a table lookup (bchk_syndtab.h): identical result
        SyndKey K[G];
        TabHome H[G];
        TabBucket B[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            K[g] = synd_key<M, TMAX>(Sw[g], t, lg);
            H[g] = tab_home(K[g].key, T);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) tab_load(T, H[g].b, B[g]);
#pragma unroll
        for (int g = 0; g < G; ++g) ok[g] = tab_finish<M, TMAX>(T, K[g], H[g], B[g], E[g].w[0]);
    } else {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            bool act = true;
            if constexpr (M >= 7) act = !skip_lane(skey, base + 64ull * (uint64_t)g + (uint64_t)(__lane_id()), t);
            ok[g] = alg_decode_word<M, TMAX>(ex, lg, chien, Sw[g], t, E[g], act);
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int s = 0; s < NW; ++s) diff[g].w[s] = Pm[g].w[s] ^ E[g].w[s];
        m[g] = 0;
        l[g] = 0.0;
        if (ok[g]) {
            m[g] = mask_popc<NW>(diff[g]);
            if constexpr (NW == 1 && BCHK_LSUM_BATCH > 0) {
                // calcL in index order (:69-77): the first KL terms' LDS loads are issued
                // together, then summed in order (one LDS round trip instead of one per term)
                constexpr int KL = BCHK_LSUM_BATCH > 0 ? BCHK_LSUM_BATCH : 1;
                double v[KL];
                uint64_t d = diff[g].w[0];
#pragma unroll
                for (int k = 0; k < KL; ++k) {
                    v[k] = ap[d ? (int)__builtin_ctzll(d) : 0];
                    d &= d - 1;
                }
                uint64_t e = diff[g].w[0];
#pragma unroll
                for (int k = 0; k < KL; ++k) {
                    if (e) l[g] += v[k];
                    e &= e - 1;
                }
                for (; d; d &= d - 1) l[g] += ap[(int)__builtin_ctzll(d)];
            } else {
#pragma unroll
                for (int s = 0; s < NW; ++s)
                    for (uint64_t v = diff[g].w[s]; v; v &= v - 1) l[g] += ap[64 * s + (int)__builtin_ctzll(v)];
            }
        }
    }
}

// Chunks decoded per step (G). Measured on MI355X (profiles/r01_syndtab): G = 2 and 4
// issue more lookups per wave but run slower (more registers, chunks published later), so
// both kernels decode one chunk per step; the knob stays for experiment builds.
template <bool TAB>
constexpr int chunk_group() { return TAB ? BCHK_TAB_GROUP : 1; }
// kernels with the table path exist for n <= 63 and t <= 8 (bchk_syndtab.h)
template <int M, int TMAX>
constexpr bool tab_capable() { return M <= 6 && TMAX <= 8; }

// ----------------------------------------------------- sequential search state
template <int NW>
struct SearchState {
    double l0;
    uint64_t bound, jsteps, impr, i_end;
    Mask<NW> best;
    int T, m0;
    bool firstOK, accepted, returned, truncated, scan_ub, done;
};

template <int M>
__device__ __forceinline__ void init_state(SearchState<Geo<M>::NW> &S, int variant) {
    constexpr int N = Geo<M>::N;
    S.T = N;  // :354 (ANSWER); LONG_MAX sentinel for WORD (:229)
    S.bound = variant == BCHK_VARIANT_WORD ? 0x7FFFFFFFFFFFFFFFull : ((1ull << (S.T & 31)) - 1ull);
    S.l0 = DBL_MAX;
    S.m0 = 0;
    S.jsteps = S.impr = S.i_end = 0;
#pragma unroll
    for (int s = 0; s < Geo<M>::NW; ++s) S.best.w[s] = 0;
    S.firstOK = true;
    S.accepted = S.returned = S.truncated = S.scan_ub = S.done = false;
}

// One successful decode at test pattern ii, in pattern order: the body of the reference
// loop after `success` (:372-398). Wave-uniform inputs; the calcT scan is lane-parallel.
// Sets S.done when the reference loop would end after this iteration.
// Long-code first kernel (prep_select): only ranks 0 .. nsel-1 of the order are known (lane
// = rank, s = 0). Where calcRightSide or the calcT scan would need a rank beyond them,
// *bail is set and nothing else is decided: the codeword goes to the search kernel, which
// starts it from scratch with the full order.
template <int M, int TMAX>
__device__ __forceinline__ void accept_success(SearchState<Geo<M>::NW> &S, const Prep<M, TMAX> &P,
                               const Mask<Geo<M>::NW> &d, int m, double l, uint64_t ii,
                               const double *as, const SearchParams &p, int lane,
                               int nsel = Geo<M>::N, bool *bail = nullptr) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    const int t = p.t;
    if (ii == 0 || !S.firstOK) S.m0 = m; // :374 (m = calcM, l = calcL of this candidate)
    if (!(l < S.l0)) return;             // :377
    S.best = d;                          // res = x; l0 = l (:378-379)
    S.l0 = l;
    S.accepted = true;
    // calcRightSide :54-67 and the calcT prefix (:110-121) over agreeing sorted positions;
    // both are prefixes of the same sequential sum.
    const int border = (2 * t + 1) - (m + S.m0) / 2;
    const int border2 = t - (m + S.m0) / 2;
    if (nsel < N) {
        // selected ranks (lane = rank): the return is certain when l lies below the
        // border-term sum formed in any order by more than its rounding (the terms are
        // positive: the two sums differ by < 2^-47 relative at border <= 64)
        const int op = P.ordv[0];
        uint64_t dw = 0;
#pragma unroll
        for (int u = 0; u < NW; ++u) dw = (u == (op >> 6)) ? d.w[u] : dw;
        const bool ag = lane < nsel && !((dw >> (op & 63)) & 1ull);
        const uint64_t agm = ballot(ag);
        if (__popcll(agm) < border) {  // needs a rank past the selection
            *bail = true;
            return;
        }
        const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(agm >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)agm, 0u));
        const double sum = rdlf(wave_sum_f64((ag && pre < border) ? P.asv[0] : 0.0), 0);
        if (l < sum * (1.0 - 0x1p-40)) {  // :380-382
            S.returned = true;
            S.i_end = ii + 1;
            S.done = true;
            return;
        }
    }
    double rs = 0.0, base2 = 0.0;
    int taken = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int q = lane + 64 * s;
        const int op = P.ordv[s];
        uint64_t dw = 0;
#pragma unroll
        for (int u = 0; u < NW; ++u) dw = (u == (op >> 6)) ? d.w[u] : dw;
        const bool ag = q < N && q < nsel && !((dw >> (op & 63)) & 1ull);
        uint64_t agm = ballot(ag);
        while (agm && taken < border) {
            const int b = (int)__builtin_ctzll(agm);
            agm &= agm - 1;
            rs += rdlf(P.asv[s], b);
            ++taken;
            if (taken == border2) base2 = rs;
        }
    }
    if (l < rs) {                        // :380-382
        S.returned = true;
        S.i_end = ii + 1;
        S.done = true;
        return;
    }
    // calcT scan (:384): while (l >= calcT(j) && j <= n-1-t) ++j, one j per lane; with a
    // selection only j + t < nsel is known (then jstar is exact if the scan stops there)
    const int scan_last = N - 1 - t;
    const int jlim = nsel < N ? (nsel - 1 - t < scan_last ? nsel - 1 - t : scan_last) : scan_last;
    int first = 0x7FFFFFFF;
#pragma unroll
    for (int s = 0; s < (N + 63) / 64; ++s) {
        const int j = lane + 64 * s;
        bool stop = jlim == scan_last;  // j beyond the scan range stops it
        if (j <= jlim) {
            double ct = base2;
            for (int u = 0; u <= t; ++u) ct += as[j + u];
            stop = !(l >= ct);
        }
        const uint64_t sm = ballot(stop && j < N);
        if (sm && first == 0x7FFFFFFF) first = 64 * s + (int)__builtin_ctzll(sm);
    }
    if (first == 0x7FFFFFFF && jlim < scan_last) {
        *bail = true;
        return;
    }
    const int jstar = first > scan_last + 1 ? scan_last + 1 : first;
    const bool word_variant = p.variant == BCHK_VARIANT_WORD;
    if (word_variant && jstar == scan_last + 1) S.scan_ub = true;  // :257 unbounded
    S.jsteps += (uint64_t)jstar;
    ++S.impr;
    if (word_variant) {
        S.T = jstar;                                     // :264
        S.bound = 1ull << (S.T & 63);
    } else {
        S.T = (p.J >= 0 && jstar > p.J) ? p.J : jstar;   // :392 / :393
        S.bound = (1ull << (S.T & 31)) - 1ull;           // (1 << T) - 1 in int32 (:361)
    }
    if (S.bound <= ii + 1) {
        S.i_end = ii + 1;
        S.done = true;
    }
}

// The sent word's positions lane + 64 s, loaded when the codeword's search starts (its
// latency then hides under the search instead of the output step's).
template <int NW>
struct TxPre {
    uint8_t v[NW];
    bool valid;
};
template <int M>
__device__ __forceinline__ TxPre<Geo<M>::NW> tx_prefetch(const SearchParams &p, uint32_t cw, int lane) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    TxPre<NW> t;
    t.valid = p.cnt != nullptr;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        t.v[s] = (t.valid && pos < N) ? p.tx[(size_t)cw * N + pos] : (uint8_t)0;
    }
    return t;
}

template <int M, int TMAX>
__device__ __forceinline__ void write_outputs(const SearchState<Geo<M>::NW> &S, const Prep<M, TMAX> &P,
                              const SearchParams &p, uint32_t cw, int lane,
                              TxPre<Geo<M>::NW> txp = TxPre<Geo<M>::NW>{{}, false},
                              unsigned long long *acc = nullptr) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    const bool word_variant = p.variant == BCHK_VARIANT_WORD;
    const uint64_t decodes = S.i_end;
    const uint64_t iters = S.returned ? S.i_end - 1 : S.i_end;
    const uint64_t pro = word_variant ? (uint64_t)(2 * N + 1) : 0ull;  // :221-224
    uint32_t bit_errors = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        uint8_t x = 0;
        if (S.accepted) {
            x = (uint8_t)(((P.yH.w[s] ^ S.best.w[s]) >> lane) & 1ull);
            if (pos < N) p.res[(size_t)cw * N + pos] = x;
        } else if (p.cnt && pos < N) {
            x = p.res[(size_t)cw * N + pos];  // not accepted: the row stays the caller's
        }
        if (p.cnt) {
            const uint8_t tv = txp.valid ? txp.v[s] : (pos < N ? p.tx[(size_t)cw * N + pos] : (uint8_t)0);
            bit_errors += (uint32_t)__popcll(ballot(pos < N && x != tv));
        }
    }
    if (p.cnt && acc) {  // the caller's per-wave sums (wave-uniform), flushed once per wave
        acc[0] += bit_errors ? 1ull : 0ull;
        acc[1] += (unsigned long long)bit_errors;
        acc[2] += (unsigned long long)decodes;
        acc[3] += (unsigned long long)(pro + iters * (uint64_t)(N + 6) + S.jsteps + S.impr);
        acc[4] += (unsigned long long)(pro + iters * (uint64_t)(N + 1) + S.jsteps);
        acc[5] += 1ull;
    } else if (p.cnt && lane == 0) {  // src/dataForPlot.cpp:55-74
        unsigned long long *c = p.cnt + (size_t)(cw % (uint32_t)kCntSlots) * kCntStride;
        if (bit_errors) {
            atomicAdd(c + 0, 1ull);
            atomicAdd(c + 1, (unsigned long long)bit_errors);
        }
        atomicAdd(c + 2, (unsigned long long)decodes);
        atomicAdd(c + 3, (unsigned long long)(pro + iters * (uint64_t)(N + 6) + S.jsteps + S.impr));
        atomicAdd(c + 4, (unsigned long long)(pro + iters * (uint64_t)(N + 1) + S.jsteps));
        atomicAdd(c + 5, 1ull);
    }
    if (lane == 0) {
        if (p.l0) p.l0[cw] = S.l0;
        if (p.st) {
            bchk_stats st;
            st.decodes = decodes;
            st.comparisons = pro + iters * (uint64_t)(N + 6) + S.jsteps + S.impr;
            st.sums = pro + iters * (uint64_t)(N + 1) + S.jsteps;
            st.iterations = iters;
            st.jsteps = S.jsteps;
            st.improvements = S.impr;
            st.flags = (S.accepted ? BCHK_F_ACCEPTED : 0u) | (S.returned ? BCHK_F_RETURNED : 0u) |
                       (S.truncated ? BCHK_F_TRUNCATED : 0u) | (P.tie ? BCHK_F_TIE : 0u) |
                       (S.scan_ub ? BCHK_F_SCAN_UB : 0u);
            st.reserved = 0;
            p.st[cw] = st;
        }
    }
}

// Long codes: the first kSeqPatterns test patterns (the hard decision, :363-379, then
// single flips of the least reliable positions -- at high SNR the hard decision is often a
// codeword already, which Decoder::decode rejects) are decoded one at a time by the whole
// wave, and most codewords leave the reference loop among them through
// `l < calcRightSide()` (:380-382) without decoding a 64-pattern chunk. Otherwise the chunk
// at base 0 decodes these patterns again to the same results; none of them is an
// improvement a second time (l0 <= their l), so the state advances exactly as in the
// reference. Sets S.done when the codeword's search has ended.
template <int M, int TMAX, bool PRE0 = false>
__device__ __forceinline__ void first_patterns(SearchState<Geo<M>::NW> &S, const Prep<M, TMAX> &P,
                                               const SearchParams &p, const uint8_t *ex,
                                               const uint16_t *lg, const double *as,
                                               const double *ap, int lane,
                                               int nsel = Geo<M>::N, bool *bail = nullptr,
                                               const Mask<Geo<M>::NW> *E0 = nullptr, bool ok0 = false) {
    constexpr int NW = Geo<M>::NW, W = Prep<M, TMAX>::W;
    for (int i = 0; i < kSeqPatterns; ++i) {
        if ((uint64_t)i >= S.bound) {  // the loop ends at its bound (:361)
            S.i_end = S.bound;
            S.done = true;
            return;
        }
        uint32_t Sw[W];  // pattern i < 64: flips Plo of lane i, syndrome S0 ^ Lo of lane i
#pragma unroll
        for (int w = 0; w < W; ++w) Sw[w] = P.S0[w] ^ rdl(P.Lo[w], i);
        Mask<NW> E;
        bool ok;
        if (PRE0 && i == 0) {  // pattern 0 decoded by the caller (alg_decode_wave4)
            ok = ok0;
            E = *E0;
        } else {
            ok = alg_decode_wave<M, TMAX>(ex, lg, Sw, p.t, lane, E);
        }
        if (i == 0 && !ok) S.firstOK = false;  // :371
        if (ok) {
#pragma unroll
            for (int s = 0; s < NW; ++s) E.w[s] ^= rdl64(P.Plo.w[s], i);  // yH ^ x
            // calcL (:69-77) in index order; position lane + 64 s holds its |alpha| in
            // P.av[s], so the terms come by readlane instead of dependent LDS loads
            double l = 0.0;
#pragma unroll
            for (int s = 0; s < NW; ++s)
                for (uint64_t v = E.w[s]; v; v &= v - 1) l += rdlf(P.av[s], (int)__builtin_ctzll(v));
            if (l < S.l0)
                accept_success<M, TMAX>(S, P, E, mask_popc<NW>(E), l, (uint64_t)i, as, p, lane, nsel, bail);
            else if (i == 0 || !S.firstOK) S.m0 = mask_popc<NW>(E);  // :374 without improvement
        }
        if (S.done || (bail && *bail)) return;
    }
}

// ------------------------------------------ analytic tail of the search (n <= 63)
// Test pattern i flips the positions ord[b] of the set bits b of i, all among the NB least
// reliable positions R (i < 2^NB). It succeeds exactly when some codeword c lies within
// distance 1..t of yH ^ P_i (Decoder::decode, src/Decoder.cpp:298-321), and then yields c.
// Write D = yH ^ c = D_U + D_R (U: the other positions). c is reached by some pattern iff
// |D_U| <= t, and syn(D_R) = S0 ^ syn(D_U) (c is a codeword), i.e. S0 ^ syn(D_U) lies in the
// span V of R's syndrome columns; D_R then follows from the column basis (plus the kernel
// of R's columns). The first pattern that yields c is D_R with its t - |D_U| highest bits
// cleared. Only first occurrences can improve l0 (a later one has the same l), and an
// improvement needs l(c) < l0, where l(c) >= sum of a over D_U. So the rest of the
// reference loop (src/KanekoKernelProcessor.cpp:361-405) is decided by the codewords whose
// D_U has at most t elements and reliability sum below l0: a depth-first enumeration over U
// in ascending reliability order, pruned at l0, finds all of them, and the reference's
// acceptance logic is replayed over them in first-pattern order -- same result, same
// counters, without decoding the thousands of test patterns in between.
// When l0 is too loose for the node budget, the enumeration runs at a tighter bound lim
// (the sum of the k least reliable U positions): the earliest candidate c* with
// l(c*) <= lim at pattern i* splits the search -- patterns below i* are decoded exactly
// (chunks, as before), and from i* on every improvement has l < l0 <= lim, so it is among
// the enumerated candidates. Nothing fits (stack, candidate list, kernel dimension,
// budget): the codeword is handed to the cooperative kernel as before.
#ifndef BCHK_AN_STACK
#define BCHK_AN_STACK 448
#endif
#ifndef BCHK_AN_CAND
#define BCHK_AN_CAND 128
#endif
constexpr int kAnStack = BCHK_AN_STACK;  // pending nodes of the enumeration (64 lanes x depth)
constexpr int kAnCand = BCHK_AN_CAND;    // candidate codewords kept for the replay
constexpr int kAnKern = 3;               // kernel dimension of R's columns (2^3 combinations)
constexpr uint32_t kAnBudget = 4096;     // enumeration nodes per attempt
constexpr uint32_t kAnExactChunks = 32;  // exact chunks below the split pattern
constexpr int kAnMaxU = 32;              // |U| <= 32 (n = 63 with NB = 31)

struct AnNode {  // enumeration node: D_U = sel (bits over U indices)
    uint64_t rem;       // residual syndrome (zero: a codeword)
    int64_t sum;        // sum of a over D_U, fixed point (a lower bound)
    uint32_t sel, comb; // U indices; pattern bits of D_R for this D_U
    uint32_t next, cls; // the next child to generate; the residual's class (leaf runs)
};
struct AnCand {
    uint64_t D;  // yH ^ c (positions)
    double l;    // calcL(c), index order
    uint32_t i, m;
};
struct AnPend {  // a codeword met by the enumeration, emitted in batches of 64
    uint32_t sel, comb;
    int64_t usum;
};
constexpr int kAnPend = 64 + 5 * 64;  // below 64 between steps, + 5 pushes of a wave
struct AnWave {
    AnNode stack[kAnStack];
    AnCand cand[kAnCand];
    AnPend pend[kAnPend];
    // pattern bits -> positions and fixed-point reliability sums, per nibble of D_R; U
    // indices -> positions, per nibble of sel
    uint64_t dpos[128];
    int64_t dsum[128];
    uint64_t upos[128];
    int64_t afix[kAnMaxU + 1];  // a of U index q, fixed point (2^40), sentinel at NU
    uint64_t ru[kAnMaxU];
    uint32_t cu[kAnMaxU];
    uint32_t kern[kAnKern];
    uint32_t ncand;
    uint8_t pu[kAnMaxU];
    // residual classes: the residuals all lie in the span of the U columns' residuals and
    // rem0, identified by their bits at the span's pivot positions (cbits of them): cmask[c]
    // = the U elements whose residual has class c
    uint32_t cmask[32];
    uint8_t ucls[kAnMaxU];  // class of U element q's residual (classes are linear)
    uint8_t cpiv[5];
    int32_t cbits;
#ifdef BCHK_AN_PROF
    // experiment builds: cycles of the enumeration by step phase (scripts/an_diag.py)
    uint64_t prof[8];
#endif
};
template <int M, int TMAX>
constexpr bool an_capable() { return Geo<M>::NW == 1 && TMAX <= 8; }
template <int M, int TMAX>
constexpr int an_bytes() { return an_capable<M, TMAX>() ? (int)((sizeof(AnWave) + 15) & ~size_t(15)) : 0; }

// floor(a 2^40) (a lower bound of a in fixed point; huge values clamp low, still a bound)
__device__ __forceinline__ int64_t an_fix(double a) {
    return a < 0x1p17 ? (int64_t)(a * 0x1p40) : (int64_t)1 << 57;
}
// a fixed-point bound at least lim 2^40 (no pruning for huge bounds)
__device__ __forceinline__ int64_t an_fix_up(double lim) {
    return lim < 0x1p17 ? (int64_t)(lim * 0x1p40) + 1 : (int64_t)0x7FFFFFFFFFFFFFFFll;
}

// One enumerated codeword with residual zero: its D_R options (kernel combinations), first
// pattern, filters (not yet processed exactly, below every possible bound, l < l0), and the
// candidate list (per lane, divergent).
template <int TMAX>
__device__ __forceinline__ void an_emit(AnWave *A, uint32_t sel, int64_t usum, uint32_t comb, int wU, int t,
                                        int nkern, uint64_t ifrom, uint64_t BM, int jb, double l0, double lcap,
                                        const double *ap) {
    for (uint32_t ks = 0; ks < (1u << nkern); ++ks) {
        uint32_t DR = comb;
#pragma unroll
        for (int q = 0; q < kAnKern; ++q)
            if (q < nkern && ((ks >> q) & 1u)) DR ^= A->kern[q];
        const int r = t - wU;
        // more than r bits at or above bit jb stay set after clearing the top r: first
        // pattern >= 2^jb >= BM (most codewords the enumeration meets at n = 63)
        if (__popc(DR >> jb) > r) continue;
        uint32_t ifirst;
        if (__popc(DR) <= r) {
            ifirst = (wU == 0 && DR == 0u) ? 1u : 0u;  // c = yH: the hard decision fails
        } else {
            uint32_t v = DR;
#pragma unroll
            for (int k = 0; k < TMAX; ++k)
                if (k < r) v &= ~(1u << (31 - __builtin_clz(v)));
            ifirst = v;
        }
        if ((uint64_t)ifirst < ifrom || (uint64_t)ifirst >= BM) continue;
        uint64_t D = 0;
        int64_t lsum = usum;  // fixed-point lower bound of l(c)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t v = (DR >> (4 * j)) & 15u, u = (sel >> (4 * j)) & 15u;
            D |= A->dpos[16 * j + v] | A->upos[16 * j + u];
            lsum += A->dsum[16 * j + v];
        }
        if ((double)lsum * 0x1p-40 > lcap * (1.0 + 0x1p-40)) continue;  // cannot matter
        double l = 0.0;  // calcL (:69-77): index order
        for (uint64_t v = D; v; v &= v - 1) l += ap[__builtin_ctzll(v)];
        if (!(l < l0 && l <= lcap)) continue;
        const uint32_t slot = atomicAdd(&A->ncand, 1u);
        if (slot < (uint32_t)kAnCand) {
            AnCand c;
            c.D = D;
            c.l = l;
            c.i = ifirst;
            c.m = (uint32_t)__popcll(D);
            A->cand[slot] = c;
        }
    }
}

// Depth-first enumeration of D_U (sum <= limfix, |D_U| <= t) from the root residual. Every
// lane owns one node and generates its children one per step in ascending order (the first
// child over the bound ends the node: the reliabilities ascend). A child that has children
// of its own becomes the lane's node, and the parent goes on the wave's LDS stack as a
// continuation (its next child); lanes without a node take continuations from the top. So
// each step visits up to 64 nodes, and the stack holds about a descent path per lane.
// Returns 0, or why the candidate list is partial: 1 node budget, 2 stack, 3 list full.
template <int TMAX>
__device__ int an_enumerate(AnWave *A, int NU, int t, int64_t limfix, uint64_t rem0, uint32_t comb0,
                             uint32_t cls0, int nkern, uint64_t ifrom, uint64_t BM, double l0, double lcap,
                             const double *ap, uint32_t budget, int lane, uint32_t &iters) {
    const int jb = BM > 1ull ? 64 - __builtin_clzll(BM - 1ull) : 0;  // patterns < BM: bits < jb
#ifdef BCHK_AN_PROF
    // [0] pops, [1] loads + single child + its drain, [2] leaf runs, [3] stack pushes,
    // [4] emission batches, [5] their cycles, [6] leaf-run rounds, [7] steps
    uint64_t pf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tq = __builtin_amdgcn_s_memtime();
#define AN_PF(i)                                            \
    {                                                       \
        const uint64_t tn_ = __builtin_amdgcn_s_memtime(); \
        pf[i] += tn_ - tq;                                  \
        tq = tn_;                                           \
    }
    auto pf_flush = [&]() {
        if (lane == 0)
            for (int i = 0; i < 8; ++i) A->prof[i] += pf[i];
    };
#else
#define AN_PF(i)
    auto pf_flush = [&]() {};
#endif
    const int cbits = A->cbits;
    if (lane == 0) A->ncand = 0u;
    wave_sync();
    if (lane == 0 && rem0 == 0ull) an_emit<TMAX>(A, 0u, 0, comb0, 0, t, nkern, ifrom, BM, jb, l0, lcap, ap);
    AnNode nd;  // lane 0 starts on the root
    nd.rem = rem0;
    nd.sum = 0;
    nd.sel = 0;
    nd.comb = comb0;
    nd.next = 0;
    nd.cls = cls0;
    bool have = lane == 0 && t >= 1;
    int sp = 0, np = 0;  // stack and pending-emission counts
    uint32_t steps = 0;
    const uint64_t below = (1ull << lane) - 1ull;
    for (;;) {
        const uint64_t idle = ballot(!have);
        const int nidle = __popcll(idle);
        const int take = nidle < sp ? nidle : sp;
        {   // every lane loads a slot (clamped) and the idle ones below `take` keep it: no
            // exec-mask branch around the loads
            const int k = __popcll(idle & below);
            const int slot = sp - 1 - k;
            const AnNode c = A->stack[slot > 0 ? slot : 0];
            const bool tk = !have & (k < take);
            if (tk) nd = c;
            have = have | tk;
        }
        sp -= take;
        if (ballot(have) == 0ull) {  // done: emit what is still pending
            wave_sync();
            if (lane < np) {
                const AnPend e = A->pend[lane];
                an_emit<TMAX>(A, e.sel, e.usum, e.comb, __popc(e.sel), t, nkern, ifrom, BM, jb, l0, lcap, ap);
            }
            wave_sync();
            break;
        }
        ++iters;
        wave_sync();  // the pops are read before this step's pushes reuse their slots
        AN_PF(0)
        const int depth = __popc(nd.sel);
        const int next = (int)nd.next;
        const int q = next < NU ? next : NU;  // NU: the sentinel (never fits)
        const int qr = next < NU ? next : 0;
        // every load of the step at once: the child's reliability and the next one's, its
        // residual and pattern bits, the class mask of this node's residual
        const int64_t aq = A->afix[q];
        const int64_t anext = A->afix[q + 1 <= NU ? q + 1 : NU];
        const uint64_t rq = A->ru[qr];
        const uint32_t cq = A->cu[qr];
        const uint32_t uq = A->ucls[qr];
        // the node carries its residual's class: no dependent load for the class mask
        const uint32_t cmk = A->cmask[cbits >= 0 ? nd.cls : 0];
        // (flags combined with & and |, not && and ||: every operand is at hand, and the
        // short-circuit forms compiled to exec-mask branches)
        const int64_t X = limfix - nd.sum;
        const bool valid = have & (next < NU) & (depth < t) & (aq <= X);
        const int64_t cs = nd.sum + aq;
        const bool expand = valid & (depth + 1 < t) & (q + 1 < NU) & (anext <= limfix - cs);
        // no child from q on can expand (the pair sums ascend): all of them are leaves, and
        // the ones whose residual matches are found from the class masks at once
        const bool run = valid & !expand & (cbits >= 0);
        const bool single = valid & !run;
        // a single child (visited one per step)
        const uint64_t crem = nd.rem ^ rq;
        const uint32_t ccomb = nd.comb ^ cq;
        const uint32_t csel = nd.sel | (1u << qr);
        const uint32_t ccls = nd.cls ^ uq;
        // codewords (zero residual) that can still reach a pattern below BM wait for the
        // next batch of emissions (a whole wave processes 64 together)
        auto push = [&](bool c, uint32_t sel, uint32_t comb, int64_t sum) {
            const uint64_t pm = ballot(c);
            if (c) {
                AnPend e;
                e.sel = sel;
                e.comb = comb;
                e.usum = sum;
                A->pend[np + __popcll(pm & below)] = e;
            }
            np += __popcll(pm);
        };
        auto drain = [&]() {
            while (np >= 64) {
#ifdef BCHK_AN_PROF
                const uint64_t te_ = __builtin_amdgcn_s_memtime();
#endif
                wave_sync();
                const AnPend e = A->pend[np - 1 - lane];
                an_emit<TMAX>(A, e.sel, e.usum, e.comb, __popc(e.sel), t, nkern, ifrom, BM, jb, l0, lcap, ap);
                np -= 64;
                wave_sync();
#ifdef BCHK_AN_PROF
                pf[4] += 1;
                pf[5] += __builtin_amdgcn_s_memtime() - te_;
#endif
            }
        };
        push(single & (crem == 0ull) & ((nkern > 0) | (__popc(ccomb >> jb) <= t - depth - 1)), csel, ccomb, cs);
        drain();
        AN_PF(1)
        // a leaf run from q on: of the remaining children only those whose residual
        // matches can be codewords, ascending until one is over the bound; kAnLeaf per
        // round (one LDS round trip), the pushes (rare: most fail the pattern filter) only
        // when some lane has one
        uint32_t mm = run ? (cmk & ~((1u << qr) - 1u)) : 0u;
        while (ballot(mm != 0u)) {
#ifdef BCHK_AN_PROF
            pf[6] += 1;
#endif
            constexpr int kAnLeaf = 4;  // measured: 8 per round visits more slots for the same rounds
            int mi[kAnLeaf];
#pragma unroll
            for (int i = 0; i < kAnLeaf; ++i) {
                mi[i] = mm ? (int)__builtin_ctz(mm) : NU;
                mm &= mm - 1u;
            }
            int64_t av[kAnLeaf];
            uint32_t cv[kAnLeaf];
#pragma unroll
            for (int i = 0; i < kAnLeaf; ++i) {
                av[i] = A->afix[mi[i]];
                cv[i] = A->cu[mi[i] < NU ? mi[i] : 0];
            }
            uint32_t alive = 1u, pm = 0u;  // below the bound so far; elements to push
            const uint32_t anyk = nkern > 0 ? 1u : 0u;
#pragma unroll
            for (int i = 0; i < kAnLeaf; ++i) {
                alive &= av[i] <= X ? 1u : 0u;  // the sentinel at NU never fits
                const uint32_t pc = nd.comb ^ cv[i];
                const uint32_t pass = anyk | (__popc(pc >> jb) <= t - depth - 1 ? 1u : 0u);
                pm |= (alive & pass) << i;
            }
            mm = alive ? mm : 0u;
            if (ballot(pm != 0u)) {
#pragma unroll
                for (int i = 0; i < kAnLeaf; ++i) {
                    push(((pm >> i) & 1u) != 0u, nd.sel | (1u << (mi[i] & 31)), nd.comb ^ cv[i], nd.sum + av[i]);
                    if (i % 4 == 3) drain();  // the pending list holds < 64 + 5 x 64
                }
            }
        }
        AN_PF(2)
        // the parent stays open iff its next child fits too
        const bool cont = expand & (anext <= X);
        const uint64_t em = ballot(cont);
        const int cnt = __popcll(em);
        if (sp + cnt > kAnStack) {
            pf_flush();
            return 2;
        }
        if (cont) {
            AnNode c = nd;
            c.next = (uint32_t)(q + 1);
            A->stack[sp + __popcll(em & below)] = c;
        }
        sp += cnt;
        if (expand) {  // descend
            nd.rem = crem;
            nd.sum = cs;
            nd.sel = csel;
            nd.comb = ccomb;
            nd.cls = ccls;
        }
        nd.next = (uint32_t)(q + 1);
        const bool valid_next = single;  // a leaf run ends the node
        have = valid_next;
        wave_sync();
#ifdef BCHK_AN_PROF
        pf[7] += 1;
#endif
        AN_PF(3)
        if (++steps > budget / 8) {  // the DP bound keeps real enumerations far below
            pf_flush();
            return 1;
        }
    }
    pf_flush();
#undef AN_PF
    return A->ncand <= (uint32_t)kAnCand ? 0 : 3;
}

// First chunk boundary at or after the earliest candidate with l <= lim (~0 if none): from
// that candidate's pattern on, l0 <= lim.
__device__ __forceinline__ uint64_t an_earliest(const AnWave *A, double lim, int lane) {
    const uint32_t nc = A->ncand;
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t e = (uint32_t)lane; e < nc && e < (uint32_t)kAnCand; e += 64) {
        const AnCand c = A->cand[e];
        if (c.l <= lim && c.i < best) best = c.i;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t x = (uint32_t)__shfl_xor((int)best, o, 64);
        best = x < best ? x : best;
    }
    return best == 0xFFFFFFFFu ? ~0ull : (((uint64_t)best + 63ull) & ~63ull);
}

// Candidates of a code with n <= 31 when every position can be flipped by some pattern (the
// loop bound uncapped, or no improvement yet: NB = n). The flip columns' kernel then has the
// code's dimension, too large for an_enumerate; instead the codewords that can still
// improve l0 are listed directly by an ordered-statistics search. Gauss-Jordan over the
// syndrome bits (one column per lane, lane = reliability rank, lane n the hard decision's
// syndrome) picks pivot columns (least reliable first); every other rank j then has a
// representation comb_j over the pivots (its own bit included) and S0 has comb0, so the
// codewords are c = yH ^ D with D = comb0 ^ XOR_{j in E} comb_j over the sets E of non-pivot
// ranks. D includes E, so l(c) >= sum_E a: a depth-first search over E (non-pivot ranks in
// ascending reliability, 64 nodes per step from a LIFO in the wave's stack) that drops a
// subtree once that sum exceeds l0 lists every codeword with l(c) < l0. Each one's first
// pattern is D (as rank bits) with its t highest bits cleared (1 when D = 0: the hard
// decision is a codeword and pattern 0 fails on it), as an_emit. The candidates then go to
// an_replay exactly as an_enumerate's. Returns 0, or 1 budget / 2 stack / 3 list full.
template <int M, int TMAX>
__device__ int an_osd(const SearchState<1> &S, const Prep<M, TMAX> &P, AnWave *A, const uint32_t *col,
                      const uint8_t *ordl, const double *ap, uint64_t ifrom, uint64_t BM, int t, int lane,
                      uint32_t &iters) {
    constexpr int N = Geo<M>::N, W = Prep<M, TMAX>::W;
    static_assert(N <= 31, "rank masks are 32-bit");
    uint64_t v = 0;
    if (lane < N) {
        const int pos = P.ordv[0];
#pragma unroll
        for (int w = 0; w < W; ++w) v |= (uint64_t)col[pos * W + w] << (32 * w);
    } else if (lane == N) {
#pragma unroll
        for (int w = 0; w < W; ++w) v |= (uint64_t)P.S0[w] << (32 * w);
    }
    uint32_t comb = lane < N ? (1u << lane) : 0u;
    bool used = false;
#pragma unroll
    for (int q = 0; q < TMAX; ++q) {
        if (q >= t) break;
#pragma unroll
        for (int b = 0; b < M; ++b) {
            const int bit = 8 * q + b;
            const bool has = (v >> bit) & 1ull;
            const uint64_t cm = ballot(has && lane < N && !used);
            if (!cm) continue;
            const int k = (int)__builtin_ctzll(cm);
            const uint64_t pv = rdl64(v, k);
            const uint32_t pc = rdl(comb, k);
            if (has && lane != k) {
                v ^= pv;
                comb ^= pc;
            }
            used = used || lane == k;
        }
    }
    const uint32_t comb0 = rdl(comb, N);
    const uint64_t freem = ballot(lane < N && !used);  // non-pivot ranks, ascending reliability
    const int nf = __popcll(freem);
    const double a_me = P.asv[0];                       // a of rank `lane`
    // per free index f (ascending rank): its comb and cost, through the stack's spare words
    uint32_t *fcomb = reinterpret_cast<uint32_t *>(A->cmask);  // 32 entries: nf <= 31
    double *fcost = reinterpret_cast<double *>(A->dsum);      // 128 entries
    if (lane < N && !used) {
        const int f = __popcll(freem & ((1ull << lane) - 1ull));
        fcomb[f] = comb;
        fcost[f] = a_me;
    }
    if (lane == 0) A->ncand = 0u;
    wave_sync();
    const double lim = S.l0 * (1.0 + 0x1p-40);  // sums of <= 31 terms in another order
    const double l0 = S.l0;
    // a codeword D (rank bits): its candidate record when it can improve l0
    auto consider = [&](bool live, uint32_t D) {
        uint64_t Dp = 0;
        double l = 0.0;
        uint32_t ifirst = 0;
        bool ok = live;
        if (live) {
            for (uint32_t x = D; x; x &= x - 1) Dp |= 1ull << ordl[__builtin_ctz(x)];
            for (uint64_t x = Dp; x; x &= x - 1) l += ap[__builtin_ctzll(x)];  // calcL, index order
            if (__popc(D) <= t) {
                ifirst = D == 0u ? 1u : 0u;
            } else {
                uint32_t x = D;
                for (int k = 0; k < t; ++k) x &= ~(1u << (31 - __builtin_clz(x)));
                ifirst = x;
            }
            ok = l < l0 && (uint64_t)ifirst >= ifrom && (uint64_t)ifirst < BM;
        }
        if (ok) {
            const uint32_t slot = atomicAdd(&A->ncand, 1u);
            if (slot < (uint32_t)kAnCand) {
                AnCand c;
                c.D = Dp;
                c.l = l;
                c.i = ifirst;
                c.m = (uint32_t)__popcll(Dp);
                A->cand[slot] = c;
            }
        }
    };
    consider(lane == 0, comb0);  // E empty
    // nodes: the words D ^ fcomb[f] (f = next) and below them; lb = cost of E so far
    int sp = 0;
    if (nf > 0 && lane == 0) {
        AnNode r;
        r.rem = comb0;
        r.sum = __double_as_longlong(0.0);
        r.sel = 0;
        r.comb = 0;
        r.next = 0;
        r.cls = 0;
        A->stack[0] = r;
    }
    sp = nf > 0 ? 1 : 0;
    wave_sync();
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t steps = 0;
    while (sp > 0) {
        int n = sp < 64 ? sp : 64;
        const int room = kAnStack - 64 - sp;
        if (room < n) n = room > 1 ? room : 1;
        const bool have = lane < n;
        AnNode e;
        e.rem = 0;
        e.sum = 0;
        e.next = 0;
        if (have) e = A->stack[sp - n + lane];
        sp -= n;
        wave_sync();
        const int f = (int)e.next;
        const double lb = __longlong_as_double(e.sum);
        const double lb2 = have ? lb + fcost[f] : 0.0;
        const bool live = have && lb2 <= lim;
        const uint32_t D2 = (uint32_t)e.rem ^ fcomb[f < 31 ? f : 0];
        consider(live, D2);
        const bool more = live && f + 1 < nf;
        const double nc = more ? fcost[f + 1] : 0.0;
        const bool psib = more && lb + nc <= lim;
        const bool pch = more && lb2 + nc <= lim;
        const uint64_t ms = ballot(psib), mc = ballot(pch);
        const int nsib = __popcll(ms);
        if (sp + nsib + __popcll(mc) > kAnStack) return 2;
        if (psib) {
            AnNode c = e;
            c.next = (uint32_t)(f + 1);
            A->stack[sp + __popcll(ms & below)] = c;
        }
        if (pch) {
            AnNode c = e;
            c.rem = D2;
            c.sum = __double_as_longlong(lb2);
            c.next = (uint32_t)(f + 1);
            A->stack[sp + nsib + __popcll(mc & below)] = c;
        }
        sp += nsib + __popcll(mc);
        wave_sync();
        ++iters;
        if (++steps > 4096u) return 1;
    }
    return A->ncand <= (uint32_t)kAnCand ? 0 : 3;
}

struct AnPlan {
    int mode;       // 0: hand off, 1: candidates complete from ifrom, 2: exact below stop
    uint64_t stop;  // mode 2: first pattern the replay takes over (a chunk boundary)
    int why;        // mode 0: 1 geometry, 2 kernel dimension, 3 no split within the
                    // budget, 4 split too far
    int fails;      // enumeration failures seen: bit 1 budget, 2 stack, 3 candidates
    uint32_t t_elim, t_setup;  // diagnostics: cycles to the end of the elimination, the setup
    uint32_t t_cls, t_tab;     // ... the residual classes, the nibble tables
};

// Plan the rest of the search of one codeword from pattern ifrom (a chunk boundary, every
// earlier pattern processed exactly); candidates land in A.
template <int M, int TMAX>
__device__ AnPlan an_plan(const SearchState<1> &S, const Prep<M, TMAX> &P, const SearchParams &p,
                          AnWave *A, const uint32_t *col, const uint8_t *ordl, const double *as,
                          const double *ap, uint64_t ifrom, int lane, uint32_t &iters) {
    constexpr int N = Geo<M>::N, W = Prep<M, TMAX>::W;
    const int t = p.t, J = p.J;
    AnPlan plan{0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t t_0 = p.tail_diag ? __builtin_amdgcn_s_memtime() : 0;
#ifdef BCHK_AN_PROF
    if (lane < 8) A->prof[lane] = 0;
    wave_sync();
#endif
    // NB pattern bits: every pattern any future bound admits, and |U| <= 32
    int NB;
    if (N >= 63) NB = 31;
    else NB = (J >= 0 && J < 31 && S.impr > 0) ? (J < N ? J : N) : (N < 31 ? N : 31);
    const int NU = N - NB;
    if (NU > kAnMaxU || NU < 0) { plan.why = 1; return plan; }
    uint64_t BM;  // patterns at or past BM are never processed
    if (S.impr == 0) BM = S.bound;
    else BM = (J >= 0 && J < 31) ? (1ull << J) - 1ull : 0x7FFFFFFFull;
    if constexpr (N <= 31) {
        if (NB >= N) {  // every position flippable: list the improving codewords directly
            const int er = an_osd<M, TMAX>(S, P, A, col, ordl, ap, ifrom, BM, t, lane, iters);
            if (!er) {
                plan.mode = 1;
                return plan;
            }
            plan.fails |= 1 << er;
            plan.why = 2;
            return plan;
        }
    }
    if (NB < 31 && BM > (1ull << NB)) { plan.why = 1; return plan; }
    // Gaussian elimination over GF(2), one column per lane: lanes r < NB the flip columns
    // (rank r), NB <= r < N the U columns, lane N the hard decision's syndrome S0
    uint64_t v = 0;
    if (lane < N) {
        const int pos = P.ordv[0];
#pragma unroll
        for (int w = 0; w < W; ++w) v |= (uint64_t)col[pos * W + w] << (32 * w);
    } else if (lane == N) {
#pragma unroll
        for (int w = 0; w < W; ++w) v |= (uint64_t)P.S0[w] << (32 * w);
    }
    uint32_t comb = lane < NB ? (1u << lane) : 0u;
    bool used = false;
    uint64_t pivbits = 0;  // bits that hold a pivot of the flip columns
#pragma unroll
    for (int q = 0; q < TMAX; ++q) {
        if (q >= t) break;
#pragma unroll
        for (int b = 0; b < M; ++b) {
            const int bit = 8 * q + b;
            const bool has = (v >> bit) & 1ull;
            const uint64_t cm = ballot(has && lane < NB && !used);
            if (!cm) continue;
            pivbits |= 1ull << bit;
            const int k = (int)__builtin_ctzll(cm);
            const uint64_t pv = rdl64(v, k);
            const uint32_t pc = rdl(comb, k);
            if (has && lane != k) {
                v ^= pv;
                comb ^= pc;
            }
            used = used || lane == k;
        }
    }
    const uint64_t km = ballot(lane < NB && !used);  // dependent flip columns: the kernel
    const int nkern = __popcll(km);
    if (nkern > kAnKern) { plan.why = 2; return plan; }
    {
        uint64_t kk = km;
        for (int q = 0; q < nkern; ++q) {
            const int k = (int)__builtin_ctzll(kk);
            kk &= kk - 1;
            const uint32_t kc = rdl(comb, k);
            if (lane == 0) A->kern[q] = kc;
        }
    }
    const uint64_t rem0 = rdl64(v, N);
    const uint32_t comb0 = rdl(comb, N);
    uint32_t cls0 = 0;
    if (p.tail_diag) plan.t_elim = (uint32_t)(__builtin_amdgcn_s_memtime() - t_0);
    if (lane >= NB && lane < N) {
        const int q = lane - NB;
        A->afix[q] = an_fix(P.asv[0]);
        A->ru[q] = v;
        A->cu[q] = comb;
        A->pu[q] = (uint8_t)P.ordv[0];
    }
    if (lane == 0) A->afix[NU] = (int64_t)0x7FFFFFFFFFFFFFFFll;
    // residual classes (leaf runs of the enumeration): a reduced basis of the span of the U
    // residuals and rem0; a residual's bits at its pivots identify it within the span
    {
        uint64_t w = (lane >= NB && lane <= N) ? v : 0ull;
        bool used2 = false;
        int cb = 0;
        int piv[5] = {0, 0, 0, 0, 0};
        // residuals are zero at the flip pivots: only the other bits can hold a pivot
        uint64_t cand_bits = 0;
#pragma unroll
        for (int q = 0; q < TMAX; ++q)
            if (q < t) cand_bits |= (uint64_t)((1u << M) - 1u) << (8 * q);
        cand_bits &= ~pivbits;
        for (uint64_t bb = cand_bits; bb && cb <= 5; bb &= bb - 1) {  // wave-uniform
            const int bit = (int)__builtin_ctzll(bb);
            const bool has = (w >> bit) & 1ull;
            const uint64_t cm = ballot(has && !used2);
            if (!cm) continue;
            const int k = (int)__builtin_ctzll(cm);
            const uint64_t pv = rdl64(w, k);
            if (has && lane != k) w ^= pv;
            used2 = used2 || lane == k;
            if (cb < 5) piv[cb] = bit;
            ++cb;
        }
        const int cbits = cb <= 5 ? cb : -1;  // too many classes: no leaf runs
        uint32_t cls = 0;
#pragma unroll
        for (int i = 0; i < 5; ++i)
            if (i < cbits) cls |= (uint32_t)((v >> piv[i]) & 1ull) << i;
        if (cbits >= 0) {
            for (int c = 0; c < (1 << cbits); ++c) {
                const uint64_t bm = ballot(lane >= NB && lane < N && cls == (uint32_t)c);
                if (lane == 0) A->cmask[c] = (uint32_t)(bm >> NB);
            }
        }
        if (lane >= NB && lane < N) A->ucls[lane - NB] = (uint8_t)cls;
        cls0 = rdl(cls, N);  // rem0's class
        if (lane == 0) {
            A->cbits = cbits;
#pragma unroll
            for (int i = 0; i < 5; ++i) A->cpiv[i] = (uint8_t)piv[i];
        }
    }
    if (p.tail_diag) plan.t_cls = (uint32_t)(__builtin_amdgcn_s_memtime() - t_0);
    // nibble tables of the flip set: entry 16 j + v covers pattern bits 4 j .. 4 j + 3 set in v
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int e = lane + 64 * h, j = e >> 4, v = e & 15;
        uint64_t dp = 0;
        int64_t ds = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int b = 4 * j + k;
            if (((v >> k) & 1) && b < NB) {
                dp |= 1ull << ordl[b];
                ds += an_fix(as[b]);
            }
        }
        A->dpos[e] = dp;
        A->dsum[e] = ds;
        uint64_t up = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = 4 * j + k;
            if (((v >> k) & 1) && q < NU) up |= 1ull << ordl[NB + q];
        }
        A->upos[e] = up;
    }
    wave_sync();
    if (p.tail_diag) plan.t_tab = (uint32_t)(__builtin_amdgcn_s_memtime() - t_0);
    const double l0 = S.l0;
    const double full = l0 * (1.0 + 0x1p-40);
    // No U subset of 4 or more fits under l0: at most 1 + 32 + 496 + 4960 nodes, so the
    // complete enumeration goes ahead without counting.
    if (NU < 4 || t <= 3 ||
        rdlf(P.asv[0], NB) + rdlf(P.asv[0], NB + 1) + rdlf(P.asv[0], NB + 2) + rdlf(P.asv[0], NB + 3) > full) {
        if (p.tail_diag) plan.t_setup = (uint32_t)(__builtin_amdgcn_s_memtime() - t_0);
        const int er = an_enumerate<TMAX>(A, NU, t, an_fix_up(full), rem0, comb0, cls0, nkern, ifrom, BM, l0, l0, ap,
                                          2 * kAnBudget, lane, iters);
        if (!er) {
            plan.mode = 1;
            return plan;
        }
        plan.fails |= 1 << er;
    }
    // Bound from a count: subsets of U of size <= t by floored bin sum (bins of width
    // hi / 64, lane = bin; a DP over the ascending reliabilities), an upper bound of the
    // enumeration's nodes at every bin edge. The largest bound within the budget is taken:
    // l0 itself when it fits (the candidates are then complete), else a tighter one.
    double prefix_t = 0.0;  // sum of the t least reliable U positions
    for (int q = 0; q < t && q < NU; ++q) prefix_t += rdlf(P.asv[0], NB + q);
    const double hi = full < 2.0 * prefix_t ? full : 2.0 * prefix_t;
    const double delta = hi / 63.0;  // sums <= hi land in bins 0..63
    // counts by subset size w packed two per word (dp[2i] | dp[2i+1] << 16), saturating at
    // 2^16 - 1: every budget compared below is < 2^16, so a saturated count decides the same
    // (half the permutes and adds of 32-bit counts)
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    constexpr int NPK = (TMAX + 2) / 2;
    uint32_t pk[NPK];
#pragma unroll
    for (int i = 0; i < NPK; ++i) pk[i] = (i == 0 && lane == 0) ? 1u : 0u;
    uint32_t wmask[NPK];  // weights <= t
#pragma unroll
    for (int i = 0; i < NPK; ++i) wmask[i] = (2 * i <= t ? 0xFFFFu : 0u) | (2 * i + 1 <= t ? 0xFFFF0000u : 0u);
    // bin of every U element (lane NB + q), all at once
    int mybin = 64;
    {
        const double inv = delta > 0.0 ? 1.0 / delta : 0.0;
        const double bq = P.asv[0] * inv;
        if (delta > 0.0 && lane >= NB && lane < N && bq < 64.0) mybin = (int)bq;
    }
    for (int q = 0; q < NU; ++q) {
        const int b = (int)rdl((uint32_t)mybin, NB + q);
        if (b >= 64) break;  // ascending: no later element fits a bin either
        // every pair's shifted counts first (the permutes issue back to back), then the adds:
        // size w gains the subsets of size w - 1 whose sum lies b bins lower
        uint32_t sh[NPK];
        const int src = ((lane - b) & 63) << 2;
#pragma unroll
        for (int i = 0; i < NPK; ++i) sh[i] = 2 * i < t ? (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pk[i]) : 0u;
#pragma unroll
        for (int i = 0; i < NPK; ++i) sh[i] = lane >= b ? sh[i] : 0u;
#pragma unroll
        for (int i = NPK - 1; i >= 0; --i) {
            // (dp'[2i - 1], dp'[2i]) -> the pair (2i, 2i + 1)
            const uint32_t add = __builtin_amdgcn_alignbit(sh[i], i > 0 ? sh[i - 1] : 0u, 16) & wmask[i];
            const u16x2 r = __builtin_elementwise_add_sat(__builtin_bit_cast(u16x2, pk[i]), __builtin_bit_cast(u16x2, add));
            pk[i] = __builtin_bit_cast(uint32_t, r);
        }
    }
    uint32_t cnt = 0;  // < 2^32: at most 64 bins x (TMAX + 1) counts of < 2^16
#pragma unroll
    for (int i = 0; i < NPK; ++i) cnt += (pk[i] & 0xFFFFu) + (pk[i] >> 16);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // inclusive prefix over the bins
        const uint32_t x = (uint32_t)__shfl((int)cnt, (lane - o) & 63, 64);
        cnt += lane >= o ? x : 0u;
    }
    static_assert(4 * kAnBudget < 0xFFFFu, "budgets compared against 16-bit saturated counts");
    if (p.tail_diag) plan.t_setup = (uint32_t)(__builtin_amdgcn_s_memtime() - t_0);
    uint32_t budget = kAnBudget;
    for (int attempt = 0; attempt < 2; ++attempt, budget *= 4) {
        const uint64_t fit = ballot(cnt <= budget);  // bins 0..L fit: a prefix of the lanes
        if (!fit) continue;
        const int L = 63 - (int)__builtin_clzll(fit);
        const bool whole = L == 63 && hi >= full;
        const double lim = whole ? full : (double)(L + 1) * delta * (1.0 - 0x1p-30);
        const int er = an_enumerate<TMAX>(A, NU, t, an_fix_up(whole ? full : lim), rem0, comb0, cls0, nkern, ifrom, BM,
                                          l0, whole ? l0 : lim, ap, budget * 2, lane, iters);
        if (er) {
            plan.fails |= 1 << er;
            continue;
        }
        if (whole) {
            plan.mode = 1;
            return plan;
        }
        // earliest candidate with l <= lim: from its pattern on, l0 <= lim, and every
        // improvement after it is among the enumerated candidates
        const uint64_t stop = an_earliest(A, lim, lane);
        if (stop == ~0ull) continue;
        if (stop - ifrom > 64ull * kAnExactChunks) {
            plan.why = 4;
            return plan;
        }
        plan.mode = 2;
        plan.stop = stop;
        return plan;
    }
    plan.why = 3;
    return plan;
}

// The reference loop from pattern `from` on, over the candidates (first patterns >= from)
// in pattern order; the loop ends at its bound or, chunk-granular, at the decode cap.
template <int M, int TMAX>
__device__ void an_replay(SearchState<1> &S, const Prep<M, TMAX> &P, const AnWave *A, uint64_t from,
                          const double *as, const SearchParams &p, int lane) {
    const uint64_t capc = p.max_decodes ? ((p.max_decodes + 63ull) & ~63ull) : ~0ull;
    const uint32_t nc = A->ncand < (uint32_t)kAnCand ? A->ncand : (uint32_t)kAnCand;
    constexpr int KW = kAnCand / 64;
    static_assert(kAnCand % 64 == 0 && kAnCand <= 256, "candidate keys: (pattern << 8) | index");
    uint64_t key[KW];
#pragma unroll
    for (int s = 0; s < KW; ++s) {
        const uint32_t e = (uint32_t)(lane + 64 * s);
        key[s] = ~0ull;
        if (e < nc && (uint64_t)A->cand[e].i >= from) key[s] = ((uint64_t)A->cand[e].i << 8) | (uint64_t)e;
    }
    wave_bitonic_sort<KW>(key, lane);
    for (int k = 0; k < 64 * KW; ++k) {
        uint64_t kk = 0;
#pragma unroll
        for (int s = 0; s < KW; ++s) kk = (k >> 6) == s ? rdl64(key[s], k & 63) : kk;
        if (kk == ~0ull) break;
        const uint64_t ii = kk >> 8;
        if (ii >= S.bound || ii >= capc) break;
        const AnCand c = A->cand[kk & 255ull];
        Mask<1> d;
        d.w[0] = c.D;
        accept_success<M, TMAX>(S, P, d, (int)c.m, c.l, ii, as, p, lane);
        if (S.done) return;
    }
    if (((S.bound + 63ull) & ~63ull) <= capc) {
        S.i_end = S.bound;
    } else {
        S.i_end = capc;
        S.truncated = true;
    }
    S.done = true;
}

// A TailRec crosses XCDs (L2s not coherent) when the tail kernel runs beside the first
// pass: written and read as device-scope relaxed atomics, and the writer waits for its
// stores before it publishes the queue slot.
static_assert(sizeof(TailRec) % 8 == 0, "TailRec as u64 words");
__device__ __forceinline__ void tail_rec_store(TailRec *dst, const TailRec &r) {
    const uint64_t *src = reinterpret_cast<const uint64_t *>(&r);
    uint64_t *d = reinterpret_cast<uint64_t *>(dst);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(TailRec) / 8); ++i)
        __hip_atomic_store(d + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ TailRec tail_rec_load(const TailRec *src) {
    TailRec r;
    uint64_t *d = reinterpret_cast<uint64_t *>(&r);
    const uint64_t *s = reinterpret_cast<const uint64_t *>(src);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(TailRec) / 8); ++i)
        d[i] = __hip_atomic_load(s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return r;
}

__device__ __forceinline__ uint32_t lds_ld(const uint32_t *a) {
    return __hip_atomic_load(a, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t *a, uint32_t v) {
    __hip_atomic_store(a, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint64_t lds_ld64(const uint64_t *a) {
    return __hip_atomic_load(a, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st64(uint64_t *a, uint64_t v) {
    __hip_atomic_store(a, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

constexpr uint32_t kSpinLimit = 1u << 24;  // ~1 s of polling: a guard against logic errors
// A bounded wait ran out (a logic error: its codeword stays unfinished): tell the host.
__device__ __forceinline__ void flag_fault(const SearchParams &p, uint32_t bit) {
    if (p.fault) atomicOr(p.fault, bit);
}

// ----------------------------------------- helper waves of the analytic tail kernel
// At 5 dB the tail kernel holds about one heavy codeword per wave, most of them finish
// within ~1.3e5 cycles, and the kernel's time is its slowest codeword's critical path. A
// split codeword (plan mode 2) then decodes up to kAnExactChunks exact chunks one after
// another. Waves of the same block whose queue is exhausted help: the owner publishes its
// decode state (the pattern-syndrome inputs of decode_chunks) and the chunk range; helpers
// claim chunks in order with a CAS on `next` (generation << 16 | chunk) and leave each one's
// per-lane results in a ring slot tagged generation << 16 | chunk + 1; the owner consumes
// the chunks in order -- the acceptance stays the owner's, in pattern order -- and decodes
// a chunk itself whenever nobody has claimed it, so it never waits on an absent helper.
// Every result is decode_chunks' own for that chunk: the output is unchanged.
constexpr int kHelpSlots = 4;
constexpr uint32_t kHelpNone = 0xFFFFu;  // chunk field: no chunk claimable
struct HelpSlot {
    uint64_t diff[64];
    double l[64];
    uint8_t m[64];
    uint64_t okm;
    uint32_t tag, pad;
};
struct HelpCtl {
    uint32_t idle;      // waves of the block past their last codeword
    uint32_t owner;     // wave id + 1 of the job's owner, 0: no job
    uint32_t gen;       // the current job's generation (low 16 bits in next and the tags)
    uint32_t next;      // gen << 16 | next unclaimed chunk (kHelpNone: closed or being set up)
    uint32_t consumed;  // chunks the owner has taken, in order
    uint32_t nch;       // chunks in the job
    uint64_t base;      // first test pattern of chunk 0
    int32_t t;
    uint32_t jown;      // wave id + 1 of the job's owner, part of the job state (read with it)
    uint32_t S0[2];
    uint32_t Lo[2][64], scol[2][64];
    uint64_t Plo[64];
    int32_t ordb[64];
    HelpSlot slot[kHelpSlots];
};
template <int M, int TMAX>
constexpr int help_bytes() { return an_capable<M, TMAX>() ? (int)((sizeof(HelpCtl) + 15) & ~size_t(15)) : 0; }

__device__ __forceinline__ uint32_t help_gen_next(uint32_t g) { return (g + 1u) & 0xFFFFu ? (g + 1u) & 0xFFFFu : 1u; }

// Owner: publish a job of nch chunks from pattern base, when some sibling is idle (then
// true: the caller takes its chunks through help_take and ends with help_close).
template <int M, int TMAX>
__device__ bool help_open(HelpCtl *H, const Prep<M, TMAX> &P, uint64_t base, uint32_t nch, int t, int wid,
                          int lane) {
    constexpr int W = Prep<M, TMAX>::W;
    static_assert(W <= 2 && Geo<M>::NW == 1, "helper jobs: n <= 63, t <= 8");
    uint32_t got = 0;
    if (lane == 0 && nch >= 2u && lds_ld(&H->idle) > 0u) got = atomicCAS(&H->owner, 0u, (uint32_t)wid + 1u) == 0u;
    got = (uint32_t)__shfl((int)got, 0, 64);
    if (!got) return false;
    const uint32_t g = help_gen_next(H->gen);  // only the owner writes gen
    if (lane == 0) {
        H->gen = g;
        lds_st(&H->next, (g << 16) | kHelpNone);  // generation first: readers re-check it
    }
    wave_sync();
#pragma unroll
    for (int w = 0; w < W; ++w) {
        H->Lo[w][lane] = P.Lo[w];
        H->scol[w][lane] = P.scol[w];
    }
    H->Plo[lane] = P.Plo.w[0];
    H->ordb[lane] = P.ordb;
    if (lane == 0) {
#pragma unroll
        for (int w = 0; w < W; ++w) H->S0[w] = P.S0[w];
        H->base = base;
        H->nch = nch;
        H->t = t;
        H->jown = (uint32_t)wid + 1u;
        H->consumed = 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wave_sync();
    if (lane == 0) lds_st(&H->next, g << 16);
    return true;
}

// Owner: the results of chunk k (in order). true: read from a helper's slot; false: the
// owner claimed it and decodes it itself.
__device__ bool help_take(HelpCtl *H, uint32_t k, uint64_t &diff, double &l, int &m, bool &ok, int lane,
                          const SearchParams &p) {
    const uint32_t g = H->gen;
    HelpSlot &S = H->slot[k % kHelpSlots];
    const uint32_t want = (g << 16) | (k + 1u);
    for (uint32_t spin = 0; spin < kSpinLimit; ++spin) {
        uint32_t st = 0;  // 1 ready in the slot, 2 claimed by the owner
        if (lane == 0) {
            if (lds_ld(&S.tag) == want) {
                st = 1;
            } else {
                const uint32_t nx = lds_ld(&H->next);
                if (nx == ((g << 16) | k) && atomicCAS(&H->next, nx, nx + 1u) == nx) st = 2;
            }
        }
        st = (uint32_t)__shfl((int)st, 0, 64);
        if (st == 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            diff = S.diff[lane];
            l = S.l[lane];
            m = S.m[lane];
            ok = (S.okm >> lane) & 1ull;
            wave_sync();
            if (lane == 0) lds_st(&H->consumed, k + 1u);
            return true;
        }
        if (st == 2) {
            if (lane == 0) lds_st(&H->consumed, k + 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    flag_fault(p, kFaultTailWait);  // a claimed chunk never arrived (a logic error)
    return false;
}

// Owner: close the job -- no further claims; wait for the chunks already claimed (their
// slots are written exactly once), then give the block's job slot back.
__device__ void help_close(HelpCtl *H, int lane, const SearchParams &p) {
    if (lane == 0) {
        const uint32_t g = H->gen;
        const uint32_t old = atomicExch(&H->next, (g << 16) | kHelpNone);
        const uint32_t claimed = old & 0xFFFFu, from = H->consumed;
        for (uint32_t j = from; j < claimed && claimed != kHelpNone; ++j) {
            uint32_t spin = 0;
            while (lds_ld(&H->slot[j % kHelpSlots].tag) != ((g << 16) | (j + 1u)) && ++spin < kSpinLimit)
                __builtin_amdgcn_s_sleep(1);
            if (spin >= kSpinLimit) flag_fault(p, kFaultTailWait);
        }
        lds_st(&H->owner, 0u);
    }
    wave_sync();
}

// Helper: after its last codeword, a wave decodes claimed chunks of its siblings' jobs
// until every wave of the block is past its last codeword and no job is open.
template <int M, int TMAX, bool TAB>
__device__ void help_loop(HelpCtl *H, const SearchParams &p, const uint8_t *ex, const uint16_t *lg,
                          const uint64_t *chien, const uint8_t *waves0, int wave_stride, int lane) {
    constexpr int W = Prep<M, TMAX>::W;
    Prep<M, TMAX> Q;
    uint32_t mygen = 0xFFFFFFFFu, qnch = 0;
    uint64_t qbase = 0;
    int qt = 0;
    const double *qap = nullptr;
    for (uint32_t spin = 0; spin < kSpinLimit; ++spin) {
        const uint32_t own = lds_ld(&H->owner);
        if (own == 0u) {
            if (lds_ld(&H->idle) >= (uint32_t)kWavesPerBlock) return;
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        const uint32_t nx = lds_ld(&H->next);
        const uint32_t g = nx >> 16, j = nx & 0xFFFFu;
        if (j == kHelpNone) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        if (g != mygen) {  // a new job: its decode state, re-checked against the generation
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
            for (int w = 0; w < W; ++w) {
                Q.S0[w] = H->S0[w];
                Q.Lo[w] = H->Lo[w][lane];
                Q.scol[w] = H->scol[w][lane];
            }
            Q.Plo.w[0] = H->Plo[lane];
            Q.ordb = H->ordb[lane];
            qbase = H->base;
            qnch = H->nch;
            qt = H->t;
            // the owner's |alpha| slice from the job state, not from `owner` (read before
            // `next`: the job may have changed hands in between); the generation re-check
            // below covers everything read here
            const uint32_t jo = H->jown;
            qap = reinterpret_cast<const double *>(waves0 + (size_t)((jo ? jo : 1u) - 1u) * wave_stride) +
                  Smem<M, TMAX>::NP;
            wave_sync();
            if ((lds_ld(&H->next) >> 16) != g) continue;
            mygen = g;
        }
        if (j >= qnch || j >= lds_ld(&H->consumed) + (uint32_t)kHelpSlots) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint32_t won = 0;
        if (lane == 0) won = atomicCAS(&H->next, nx, nx + 1u) == nx;
        won = (uint32_t)__shfl((int)won, 0, 64);
        if (!won) continue;
        Mask<1> diff[1];
        int m[1];
        double l[1];
        bool ok[1];
        decode_chunks<M, TMAX, 1, TAB>(Q, qbase + 64ull * j, qt, ex, lg, chien, qap, p.tab, diff, m, l, ok);
        HelpSlot &S = H->slot[j % kHelpSlots];
        S.diff[lane] = diff[0].w[0];
        S.l[lane] = l[0];
        S.m[lane] = (uint8_t)m[0];
        const uint64_t okm = ballot(ok[0]);
        if (lane == 0) S.okm = okm;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        wave_sync();
        if (lane == 0) lds_st(&S.tag, (g << 16) | (j + 1u));
        spin = 0;
    }
}

// ------------------------------------------------ wave-per-codeword search
// 64 consecutive test patterns per step, acceptance in pattern order. A codeword still
// running after p.chunk_limit steps finishes through the analytic tail (above) or is handed
// to the cooperative kernel (heavy queue).
template <int M, int TMAX, bool TAB, bool AN>
__device__ void search_codeword(const SearchParams &p, const uint8_t *ex, const uint16_t *lg,
                                const uint32_t *col, const uint64_t *chien, double *as,
                                double *ap, uint8_t *ordl, uint32_t cw, int lane, AnWave *an,
                                uint32_t item, HelpCtl *help, int wid, uint64_t *fpt = nullptr) {
    constexpr int NW = Geo<M>::NW;
    (void)fpt;  // BCHK_FP_TRACE (diagnostic builds): [0] prep done, [1] patterns done, [2] chunks
    // analytic tail: exact chunks end at an_stop, then the candidates decide the rest
    bool an_tried = false, an_exact = false;
    uint64_t an_stop = 0;
    bool helped = false;  // the exact chunks below an_stop with the block's idle waves
    uint64_t help_base = 0;
    (void)an_tried;
    // analytic-tail timing records (p.tail_diag, diagnostics only): cycles per phase
    uint64_t dg_t0 = 0, dg_t1 = 0, dg_t2 = 0, dg_t3 = 0, dg_stage = 0;
    uint32_t dg_iters = 0, dg_mode = 0;
    if (AN && p.tail_diag) dg_t0 = __builtin_amdgcn_s_memtime();
#ifdef BCHK_AN_PROF
    // experiment builds: the first pass's cycles by phase, summed over its codewords into
    // the last prof record of the tail diagnostics ([0] prep, [1] decode, [2] acceptance,
    // [3] outputs, [4] chunks, [5] codewords)
    uint64_t fq = __builtin_amdgcn_s_memtime(), fp[6] = {0, 0, 0, 0, 0, 1};
#define FP_STAMP(i)                                         \
    {                                                       \
        const uint64_t tn_ = __builtin_amdgcn_s_memtime(); \
        fp[i] += tn_ - fq;                                  \
        fq = tn_;                                           \
    }
    auto fp_flush = [&]() {
        if (!AN && p.tail_diag && lane == 0) {
            unsigned long long *q = p.tail_diag + (size_t)p.tail_diag_cap * 8 + (size_t)(p.tail_diag_cap - 1) * 8;
            for (int i = 0; i < 6; ++i) atomicAdd(q + i, (unsigned long long)fp[i]);
        }
    };
#else
#define FP_STAMP(i)
    auto fp_flush = [&]() {};
#endif
    const TxPre<NW> txp = tx_prefetch<M>(p, cw, lane);
    Prep<M, TMAX> P;
    prep_codeword<M, TMAX>(p, col, as, ap, ordl, cw, lane, P);
#ifdef BCHK_FP_TRACE
    if (fpt) fpt[0] = __builtin_amdgcn_s_memrealtime();
#endif
    FP_STAMP(0)
    if (AN && p.tail_diag) dg_t1 = __builtin_amdgcn_s_memtime();
    SearchState<NW> S;
    init_state<M>(S, p.variant);
    (void)an;
    auto tail_record = [&]() {
        if (AN && p.tail_diag && an_tried && lane == 0) {
            const uint32_t r = atomicAdd(p.tail_diag_count, 1u);
            if (r < p.tail_diag_cap) {
                unsigned long long *d = p.tail_diag + (size_t)r * 8;
                const uint64_t t4 = __builtin_amdgcn_s_memtime();
                d[0] = cw | (uint64_t)xcc_id() << 24 | (dg_t0 & 0xFFFFFFFFFull) << 28;  // + XCD, start
                d[1] = dg_t1 - dg_t0;                         // prep (+ resume)
                d[2] = dg_stage;                              // plan stages (packed)
                d[3] = dg_t3 - dg_t2;                         // plan
                d[4] = dg_iters | (uint64_t)(dg_t2 - dg_t1) << 32;  // steps, exact chunks before
                d[5] = dg_mode;
                d[6] = t4 - dg_t3;                            // split chunks + replay + outputs
                d[7] = S.i_end;
#ifdef BCHK_AN_PROF
                // second half of the buffer: the enumeration's step-phase cycles
                unsigned long long *q = p.tail_diag + (size_t)p.tail_diag_cap * 8 + (size_t)r * 8;
                if (an)
                    for (int i = 0; i < 8; ++i) q[i] = an->prof[i];
#endif
            }
        }
    };
    if constexpr (M >= 7) {
        // long codes: the first test patterns one at a time, unless kaneko_first_kernel has
        // done so already (it queued this codeword)
        if (!p.queue) {
            first_patterns<M, TMAX>(S, P, p, ex, lg, as, ap, lane);
            if (S.done) {
                write_outputs<M, TMAX>(S, P, p, cw, lane, txp);
                return;
            }
        }
    }
    constexpr int G = chunk_group<TAB>();
    uint32_t chunks = 0;
    uint64_t base00 = 0;
    if constexpr (AN && G == 1) {
        if (p.tail_rec && (p.queue || p.in_queue)) {  // resume where the first pass handed it off
            const TailRec r = tail_rec_load(p.tail_rec + item);
            S.l0 = r.l0;
            S.bound = r.bound;
            S.jsteps = r.jsteps;
            S.impr = r.impr;
            S.best.w[0] = r.best;
            S.T = r.T;
            S.m0 = r.m0;
            S.firstOK = (r.flags & 1u) != 0;
            S.accepted = (r.flags & 2u) != 0;
            chunks = r.chunks;
            base00 = 64ull * r.chunks;
        }
    }
    for (uint64_t base0 = base00;; base0 += 64 * G) {
        // the checks of the next chunk before any decode (no group started past the end)
        if (base0 >= S.bound) { S.i_end = S.bound; break; }
        if (p.max_decodes && base0 >= p.max_decodes) { S.i_end = base0; S.truncated = true; break; }
        if constexpr (AN && an_capable<M, TMAX>() && G == 1) {
            if (p.analytic && p.heavy_tail && chunks >= p.chunk_limit && !an_tried &&
                p.variant == BCHK_VARIANT_ANSWER) {
                an_tried = true;
                uint32_t iters = 0;
                if (p.tail_diag) dg_t2 = __builtin_amdgcn_s_memtime();
                const AnPlan plan = an_plan<M, TMAX>(S, P, p, an, col, ordl, as, ap, base0, lane, iters);
                if (p.tail_diag) {
                    dg_t3 = __builtin_amdgcn_s_memtime();
                    dg_iters = iters;
                    const auto c16 = [](uint32_t x) { return (uint64_t)(x < 0xFFFFu ? x : 0xFFFFu); };
                    dg_stage = c16(plan.t_elim) | c16(plan.t_cls) << 16 | c16(plan.t_tab) << 32 |
                               c16(plan.t_setup) << 48;  // cycles from the plan's start
                    dg_mode = (uint32_t)plan.mode | ((uint32_t)plan.why << 8) |
                              (uint32_t)(((plan.stop > base0 ? plan.stop - base0 : 0) >> 6) << 16) |
                              ((uint32_t)plan.fails << 24);
                }
                if (p.tail_stats && lane == 0) {
                    atomicAdd(p.tail_stats + plan.mode, 1u);
                    if (plan.mode == 2) atomicAdd(p.tail_stats + 3, (uint32_t)((plan.stop - base0) >> 6));
                    atomicAdd(p.tail_stats + 4, iters);
                    atomicMax(p.tail_stats + 5, iters);
                }
                if (plan.mode == 1) {
                    an_replay<M, TMAX>(S, P, an, base0, as, p, lane);
                    break;
                }
                if (plan.mode == 2) {
                    an_exact = true;
                    an_stop = plan.stop;
                    if (help) {
                        helped = help_open<M, TMAX>(help, P, base0, (uint32_t)((an_stop - base0) >> 6), p.t, wid, lane);
                        help_base = base0;
                    }
                }
            }
            if (an_exact && base0 >= an_stop) {
                an_replay<M, TMAX>(S, P, an, an_stop, as, p, lane);
                break;
            }
        }
        const bool hand_off = p.heavy_tail && chunks >= p.chunk_limit && !an_exact;
        Mask<NW> diff[G];
        int m[G];
        double l[G];
        bool ok[G];
        bool handed = false;
        if (!hand_off) {
            bool got = false;
            if constexpr (AN && G == 1 && an_capable<M, TMAX>()) {
                if (helped && base0 < an_stop)
                    got = help_take(help, (uint32_t)((base0 - help_base) >> 6), diff[0].w[0], l[0], m[0], ok[0], lane, p);
            }
            if (!got) {
                const uint64_t skey = (M >= 7 && S.accepted) ? skip_key<M, TMAX>(S.best, P, lane) : 0ull;
                decode_chunks<M, TMAX, G, TAB>(P, base0, p.t, ex, lg, chien, ap, p.tab, diff, m, l, ok, skey);
            }
        }
        FP_STAMP(1)
#ifdef BCHK_AN_PROF
        fp[4] += 1;
#endif
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint64_t base = base0 + 64ull * (uint64_t)g;
            if (base >= S.bound) { S.i_end = S.bound; S.done = true; break; }
            if (p.max_decodes && base >= p.max_decodes) {
                S.i_end = base;
                S.truncated = true;
                S.done = true;
                break;
            }
            if (hand_off) {
                if (lane == 0) {  // longest-first: large remaining bounds to the front queue
                    uint32_t *slot;
                    if (S.bound >= p.heavy_big) {
                        const uint32_t k = atomicAdd(p.heavy_tail, 1u);
                        slot = p.heavy_queue + k;
                        if constexpr (!AN && NW == 1) {
                            if (p.tail_rec) {  // the analytic tail kernel resumes from here
                                TailRec r;
                                r.l0 = S.l0;
                                r.bound = S.bound;
                                r.jsteps = S.jsteps;
                                r.impr = S.impr;
                                r.best = S.best.w[0];
                                r.T = S.T;
                                r.m0 = S.m0;
                                r.chunks = chunks;
                                r.flags = (S.firstOK ? 1u : 0u) | (S.accepted ? 2u : 0u);
                                tail_rec_store(p.tail_rec + k, r);  // complete before the slot store
                            }
                        }
                    } else {
                        slot = p.heavy_queue + (p.count - 1u - atomicAdd(p.heavy_tail2, 1u));
                    }
                    __hip_atomic_store(slot, cw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                handed = true;  // redone from scratch by kaneko_coop_kernel
                break;
            }
            ++chunks;
            const uint64_t okm = ballot(ok[g]);
            if (base == 0 && !(okm & 1ull)) S.firstOK = false;  // :371
            // Only improvements (l < l0) change the state: m0 at an improvement is the fixed
            // i = 0 value or, once i = 0 has failed, the improving candidate's own m (:374),
            // and l0 only decreases, so successes with l >= l0 can be skipped wholesale. The
            // loop bound is NOT monotone (T comes from the calcT scan of each improvement,
            // and (1 << T) - 1 wraps at 32 bits), so lanes meet the current bound.
            uint64_t imp = ballot(ok[g] && l[g] < S.l0);
            while (imp) {
                const int L = (int)__builtin_ctzll(imp);
                const uint64_t ii = base + (uint64_t)L;
                if (ii >= S.bound) break;
                const double lL = rdlf(l[g], L);
                const int mL = (int)rdl((uint32_t)m[g], L);
                Mask<NW> d;
#pragma unroll
                for (int s = 0; s < NW; ++s) d.w[s] = rdl64(diff[g].w[s], L);
                accept_success<M, TMAX>(S, P, d, mL, lL, ii, as, p, lane);
                if (S.done) break;
                // l0 dropped: re-filter the later lanes of this chunk
                imp = ballot(ok[g] && l[g] < S.l0) & ~((2ull << L) - 1ull);
            }
            if (S.done) break;
        }
        FP_STAMP(2)
        if (handed) {
#ifdef BCHK_FP_TRACE
            if (fpt) {
                fpt[1] = __builtin_amdgcn_s_memrealtime();
                fpt[2] = chunks | 0x10000u;
            }
#endif
            fp_flush();
            tail_record();
            return;
        }
        if (S.done) break;
    }
    if (helped) help_close(help, lane, p);
#ifdef BCHK_FP_TRACE
    if (fpt) {
        fpt[1] = __builtin_amdgcn_s_memrealtime();
        fpt[2] = chunks;
    }
#endif
    write_outputs<M, TMAX>(S, P, p, cw, lane, txp);
    FP_STAMP(3)
    fp_flush();
#undef FP_STAMP
    tail_record();
}

// Relaxed device-scope atomics only: acquire/release at agent scope would write back or
// invalidate this XCD's whole L2 on every use (L2s are not coherent across XCDs), and the
// only data handed over are the atomic words themselves.
__device__ __forceinline__ uint32_t ld_rlx(const uint32_t *a) {
    return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// s_waitcnt vmcnt(0): this wave's earlier memory operations (gfx9: loads and stores) have
// completed before any later one issues; the asm is also a compiler barrier.
__device__ __forceinline__ void mem_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// A wave of the exact kernel exits after `ndone` codewords (finished or handed off): it
// adds them to its XCD's count (8 counters on separate lines: no single hot address). Its
// hand-offs' tail increments have returned (their values addressed the slots) before the
// count is issued, so a consumer that sees the counts complete sees final tails.
__device__ __forceinline__ void wave_done(const SearchParams &p, int lane, uint32_t ndone) {
    if (p.exact_done && lane == 0 && ndone) {
        mem_drain();
        __hip_atomic_fetch_add(p.exact_done + 32 * xcc_id(), ndone, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The analytic tail kernel running concurrently with the first pass: the next codeword the
// first pass hands off (one ticket per codeword; the first pass reserves a slot with its
// tail, then stores the codeword; consumers restore empty slots), kEmptySlot once the
// first pass has finished (its per-XCD done counts reach *in_total) and no ticket is left.
// Every wait is bounded (a logic error ends the wave instead of hanging it).

__device__ uint32_t tail_dequeue(const SearchParams &p, uint32_t &item) {
    constexpr uint32_t kTailSpin = 1u << 24;  // ~1 s of polling: a guard against logic errors
    const uint32_t total = p.in_total ? *p.in_total : p.count;
    const uint32_t k = atomicAdd(p.in_head, 1u);
    for (uint32_t spins = 0; spins < kTailSpin; ++spins) {
        if (k < ld_rlx(p.in_tail)) {
            uint32_t *slot = p.in_queue + k;
            for (uint32_t w = 0; w < kTailSpin; ++w) {
                const uint32_t cw = ld_rlx(slot);
                if (cw != kEmptySlot) {
                    __hip_atomic_store(slot, kEmptySlot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    item = k;
                    return cw;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            flag_fault(p, kFaultTailSlot);
            return kEmptySlot;
        }
        uint32_t done = 0;
#pragma unroll
        for (int x = 0; x < 8; ++x) done += ld_rlx(p.in_done + 32 * x);
        const bool final = done >= total;
        mem_drain();
        if (k < ld_rlx(p.in_tail)) continue;
        if (final) return kEmptySlot;
        __builtin_amdgcn_s_sleep(16);
    }
    flag_fault(p, kFaultTailWait);
    return kEmptySlot;
}

}  // namespace bchk
