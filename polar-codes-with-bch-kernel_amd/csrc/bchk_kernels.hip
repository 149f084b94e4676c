// bchk_kernels.hip -- gfx950 (CDNA4) kernels for Kaneko's soft-decision search over a
// binary BCH(n, k) code, the hot path of src/KanekoKernelProcessor.cpp:335-407 and
// src/Decoder.cpp:184-321 of the reference.
//
// Execution model (one 64-lane wave per codeword, persistent waves):
//   prep    lane = channel position: alpha = 2y/s2 (IEEE f64 division), hard decision,
//           |alpha|; exact rank by (|alpha|, position) with wave-uniform readlanes; the
//           sorted reliabilities are scattered to the wave's LDS slice.
//   search  lane = test pattern: 64 consecutive test patterns i = base + lane are decoded
//           speculatively in parallel. A pattern's syndrome is the XOR of the hard
//           decision's syndrome with the odd-syndrome columns of its flipped positions
//           (GF(2)-linear, 3 XORs per word per lane); the key equation is solved with
//           inversionless binary Berlekamp-Massey (== the reference's Euclid, see
//           oracle/bchk_oracle.c:orc_alg_decode_bm) and roots are found by a GF(2)-linear
//           Chien map (table XOR) or an incremental Chien scan (m >= 7).
//   accept  the reference's sequential acceptance logic (m0, l0, calcRightSide, calcT
//           scan, loop bound) runs wave-uniformly over the successful lanes in pattern
//           order; its f64 sums are formed in exactly the reference's order. calcT(j) for
//           all j is evaluated lane-parallel (one j per lane).
// No MFMA: there is no dense contraction here; the work is GF table/bit arithmetic.
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdint.h>

#include "bchk_core.h"
#include "bchk_launch.h"

namespace bchk {

// -------------------------------------------------------------- LDS layout
template <int M, int TMAX>
struct Smem {
    static constexpr int NP = 64 * Geo<M>::NW;     // padded positions per wave
    // sorted |alpha| (f64), |alpha| by position (f64), order (u8)
    static constexpr int WAVE_BYTES = NP * 8 * 2 + NP;
};
constexpr int kCoopWaves = 16;  // waves that share one heavy codeword (1024 threads)

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
__device__ void prep_codeword(const SearchParams &p, const uint32_t *col, double *as, double *ap,
                              uint8_t *ordl, uint32_t cw, int lane, Prep<M, TMAX> &P) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW, W = Prep<M, TMAX>::W;
    constexpr int NB = N < 31 ? N : 31;  // pattern bits in use (i < 2^31)
    const double *y = p.y + (size_t)cw * N;
    // alpha = 2*word/pow(sd,2); yH; |alpha| (:336-342)
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        const bool valid = pos < N;
        const double yy = valid ? y[pos] : 0.0;
        const double al = (2.0 * yy) / p.s2;
        P.av[s] = valid ? fabs(al) : 0.0;
        P.yH.w[s] = ballot(valid && !(al <= 0.0));
    }
    // exact rank by (|alpha|, position): the stable order of std::sort's keys (:343).
    // |alpha| by position goes to LDS first; every lane then streams all N values with
    // broadcast reads (uniform address, no bank conflict) and counts those ranked before it.
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        if (pos < N) ap[pos] = P.av[s];
    }
    wave_sync();
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

// Decode test patterns i = base + lane (base a multiple of 64): returns success and
// diff = yH ^ x (flipped pattern positions ^ error locations); for successful lanes also
// m = calcM (:89-97) and l = calcL (:69-77), summed over diff in index order from the
// wave's |alpha|-by-position LDS slice (lane-parallel; the ordered acceptance only
// compares them).
template <int M, int TMAX>
__device__ __forceinline__ bool decode_chunk(const Prep<M, TMAX> &P, uint64_t base, int t,
                                             const uint8_t *ex, const uint16_t *lg,
                                             const uint64_t *chien, const double *ap,
                                             Mask<Geo<M>::NW> &diff, int &m, double &l) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW, W = Prep<M, TMAX>::W;
    constexpr int NB = N < 31 ? N : 31;
    uint32_t Sw[W];
    Mask<NW> Pm = P.Plo;
#pragma unroll
    for (int w = 0; w < W; ++w) Sw[w] = P.S0[w] ^ P.Lo[w];
    for (uint64_t hb = base >> 6; hb; hb &= hb - 1) {  // high pattern bits: wave-uniform
        const int b = 6 + (int)__builtin_ctzll(hb);
        if (b >= NB) continue;
        const int pb = (int)rdl((uint32_t)P.ordb, b);
#pragma unroll
        for (int w = 0; w < W; ++w) Sw[w] ^= rdl(P.scol[w], b);
        mask_set<NW>(Pm, pb);
    }
    Mask<NW> E;
    const bool ok = alg_decode_word<M, TMAX>(ex, lg, chien, Sw, t, E);
#pragma unroll
    for (int s = 0; s < NW; ++s) diff.w[s] = Pm.w[s] ^ E.w[s];
    m = 0;
    l = 0.0;
    if (ok) {
        m = mask_popc<NW>(diff);
#pragma unroll
        for (int s = 0; s < NW; ++s)
            for (uint64_t v = diff.w[s]; v; v &= v - 1) l += ap[64 * s + (int)__builtin_ctzll(v)];
    }
    return ok;
}

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
template <int M, int TMAX>
__device__ void accept_success(SearchState<Geo<M>::NW> &S, const Prep<M, TMAX> &P,
                               const Mask<Geo<M>::NW> &d, int m, double l, uint64_t ii,
                               const double *as, const SearchParams &p, int lane) {
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
    double rs = 0.0, base2 = 0.0;
    int taken = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int q = lane + 64 * s;
        const int op = P.ordv[s];
        uint64_t dw = 0;
#pragma unroll
        for (int u = 0; u < NW; ++u) dw = (u == (op >> 6)) ? d.w[u] : dw;
        const bool ag = q < N && !((dw >> (op & 63)) & 1ull);
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
    // calcT scan (:384): while (l >= calcT(j) && j <= n-1-t) ++j, one j per lane
    const int scan_last = N - 1 - t;
    int first = 0x7FFFFFFF;
#pragma unroll
    for (int s = 0; s < (N + 63) / 64; ++s) {
        const int j = lane + 64 * s;
        bool stop = true;  // j beyond the scan range stops it
        if (j <= scan_last) {
            double ct = base2;
            for (int u = 0; u <= t; ++u) ct += as[j + u];
            stop = !(l >= ct);
        }
        const uint64_t sm = ballot(stop && j < N);
        if (sm && first == 0x7FFFFFFF) first = 64 * s + (int)__builtin_ctzll(sm);
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

template <int M, int TMAX>
__device__ void write_outputs(const SearchState<Geo<M>::NW> &S, const Prep<M, TMAX> &P,
                              const SearchParams &p, uint32_t cw, int lane) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    const bool word_variant = p.variant == BCHK_VARIANT_WORD;
    const uint64_t decodes = S.i_end;
    const uint64_t iters = S.returned ? S.i_end - 1 : S.i_end;
    const uint64_t pro = word_variant ? (uint64_t)(2 * N + 1) : 0ull;  // :221-224
    if (S.accepted) {
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int pos = lane + 64 * s;
            if (pos < N)
                p.res[(size_t)cw * N + pos] = (uint8_t)(((P.yH.w[s] ^ S.best.w[s]) >> lane) & 1ull);
        }
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

// ------------------------------------------------ wave-per-codeword search
// 64 consecutive test patterns per step, acceptance in pattern order. A codeword still
// running after p.chunk_limit steps is handed to the cooperative kernel (heavy queue).
template <int M, int TMAX>
__device__ void search_codeword(const SearchParams &p, const uint8_t *ex, const uint16_t *lg,
                                const uint32_t *col, const uint64_t *chien, double *as,
                                double *ap, uint8_t *ordl, uint32_t cw, int lane) {
    constexpr int NW = Geo<M>::NW;
    Prep<M, TMAX> P;
    prep_codeword<M, TMAX>(p, col, as, ap, ordl, cw, lane, P);
    SearchState<NW> S;
    init_state<M>(S, p.variant);
    uint32_t chunks = 0;
    for (uint64_t base = 0;; base += 64, ++chunks) {
        if (base >= S.bound) { S.i_end = S.bound; break; }
        if (p.max_decodes && base >= p.max_decodes) { S.i_end = base; S.truncated = true; break; }
        if (p.heavy_tail && chunks == p.chunk_limit) {
            if (lane == 0) p.heavy_queue[atomicAdd(p.heavy_tail, 1u)] = cw;
            return;  // redone from scratch by kaneko_coop_kernel
        }
        Mask<NW> diff;
        int m;
        double l;
        const bool ok = decode_chunk<M, TMAX>(P, base, p.t, ex, lg, chien, ap, diff, m, l);
        const bool live = ok && base + (uint64_t)lane < S.bound;
        const uint64_t okm = ballot(live);
        if (base == 0 && !(okm & 1ull)) S.firstOK = false;  // :371
        // Only improvements (l < l0) change the state: m0 at an improvement is the fixed
        // i = 0 value or, once i = 0 has failed, the improving candidate's own m (:374), and
        // l0 only decreases, so successes with l >= l0 can be skipped wholesale.
        uint64_t imp = ballot(live && l < S.l0);
        while (imp) {
            const int L = (int)__builtin_ctzll(imp);
            const uint64_t ii = base + (uint64_t)L;
            if (ii >= S.bound) break;
            const double lL = rdlf(l, L);
            const int mL = (int)rdl((uint32_t)m, L);
            Mask<NW> d;
#pragma unroll
            for (int s = 0; s < NW; ++s) d.w[s] = rdl64(diff.w[s], L);
            accept_success<M, TMAX>(S, P, d, mL, lL, ii, as, p, lane);
            if (S.done) break;
            // l0 dropped: re-filter the later lanes of this chunk
            imp = ballot(live && l < S.l0) & ~((2ull << L) - 1ull);
        }
        if (S.done) break;
    }
    write_outputs<M, TMAX>(S, P, p, cw, lane);
}

template <int M, int TMAX>
__global__ void __launch_bounds__(kWaveSize * kWavesPerBlock)
kaneko_search_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    load_tables(smem, p.tables, p.td.bytes);
    __syncthreads();
    const uint8_t *ex = smem + p.td.off_exp;
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(smem + p.td.off_log);
    const uint32_t *col = reinterpret_cast<const uint32_t *>(smem + p.td.off_col);
    const uint64_t *chien = reinterpret_cast<const uint64_t *>(smem + p.td.off_chien);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int NP = Smem<M, TMAX>::NP;
    uint8_t *wbase = smem + ((p.td.bytes + 15) & ~15u) + wid * Smem<M, TMAX>::WAVE_BYTES;
    double *as = reinterpret_cast<double *>(wbase);
    double *ap = as + NP;
    uint8_t *ordl = wbase + NP * 16;
    if (!p.queue) {
        const uint32_t stride = gridDim.x * kWavesPerBlock;
        for (uint32_t cw = blockIdx.x * kWavesPerBlock + wid; cw < p.count; cw += stride)
            search_codeword<M, TMAX>(p, ex, lg, col, chien, as, ap, ordl, cw, lane);
        return;
    }
    // Work queue left by the fast path: sub-queue x holds items x, x+8, x+16, ...; a wave
    // drains its own XCD's sub-queue first (one L2-local atomic per codeword), then steals.
    const uint32_t total = *p.qcount;
    if ((blockIdx.x * kWavesPerBlock + wid) >= total) return;  // more waves than work
    int x = xcc_id();
    for (int exhausted = 0; exhausted < 8;) {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(p.heads + 32 * x, 1u);
        k = (uint32_t)__shfl((int)k, 0, 64);
        const uint32_t item = (uint32_t)x + 8u * k;
        if (item >= total) {
            x = (x + 1) & 7;
            ++exhausted;
            continue;
        }
        search_codeword<M, TMAX>(p, ex, lg, col, chien, as, ap, ordl, p.queue[item], lane);
    }
}

// ---------------------------------------- cooperative search of heavy codewords
// One workgroup of kCoopWaves waves per codeword: every round, wave w decodes patterns
// [base + 64 w, base + 64 w + 64); wave 0 then applies the reference's sequential
// acceptance to all successes of the round in pattern order (:361-405) and publishes the
// new loop bound. Results are identical to the single-wave search.
template <int M, int TMAX>
__global__ void __launch_bounds__(kWaveSize * kCoopWaves)
kaneko_coop_kernel(SearchParams p) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    constexpr int NP = Smem<M, TMAX>::NP;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    load_tables(smem, p.tables, p.td.bytes);
    const uint8_t *ex = smem + p.td.off_exp;
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(smem + p.td.off_log);
    const uint32_t *col = reinterpret_cast<const uint32_t *>(smem + p.td.off_col);
    const uint64_t *chien = reinterpret_cast<const uint64_t *>(smem + p.td.off_chien);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint8_t *shared0 = smem + ((p.td.bytes + 15) & ~15u);
    uint64_t *okm_l = reinterpret_cast<uint64_t *>(shared0);                    // [waves]
    uint64_t *diff_l = okm_l + kCoopWaves;                                      // [waves][64][NW]
    double *l_l = reinterpret_cast<double *>(diff_l + kCoopWaves * 64 * NW);    // [waves][64]
    uint32_t *m_l = reinterpret_cast<uint32_t *>(l_l + kCoopWaves * 64);        // [waves][64]
    uint64_t *ctl = reinterpret_cast<uint64_t *>(m_l + kCoopWaves * 64);  // bound, done, item, l0
    uint64_t *cand_l = ctl + 4;                                           // [waves]
    uint8_t *wbase = reinterpret_cast<uint8_t *>(cand_l + kCoopWaves) + wid * Smem<M, TMAX>::WAVE_BYTES;
    double *as = reinterpret_cast<double *>(wbase);
    double *ap = as + NP;
    uint8_t *ordl = wbase + NP * 16;
    const uint32_t total = *p.heavy_tail;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) ctl[2] = atomicAdd(p.heavy_head, 1u);
        __syncthreads();
        const uint32_t item = (uint32_t)ctl[2];
        if (item >= total) return;
        const uint32_t cw = p.heavy_queue[item];
#ifdef BCHK_DIAG
        // stamps (wave 0): [0] prep, [1] own decodes, [2] wait for the other waves,
        // [3] ordered acceptance, [4] rounds, [5] improvements, [6] total
        unsigned long long dg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
        Prep<M, TMAX> P;  // every wave builds the same prep (its own LDS slice)
        prep_codeword<M, TMAX>(p, col, as, ap, ordl, cw, lane, P);
#ifdef BCHK_DIAG
        unsigned long long t_prev = __builtin_amdgcn_s_memtime();
        dg[0] = t_prev - t_start;
#endif
        SearchState<NW> S;
        init_state<M>(S, p.variant);
        if (threadIdx.x == 0) {
            ctl[0] = S.bound;
            ctl[1] = 0;
            ctl[3] = (uint64_t)__double_as_longlong(S.l0);
        }
        for (uint64_t rbase = 0;; rbase += 64 * kCoopWaves) {
            __syncthreads();
            const uint64_t bound = ctl[0];
            if (ctl[1]) break;
            const double l0r = __longlong_as_double((long long)ctl[3]);  // l0 at round start
            const uint64_t base = rbase + 64 * (uint64_t)wid;
            uint64_t okm = 0, cand = 0;
            if (base < bound && !(p.max_decodes && base >= p.max_decodes)) {
                Mask<NW> diff;
                int m;
                double l;
                const bool ok = decode_chunk<M, TMAX>(P, base, p.t, ex, lg, chien, ap, diff, m, l);
                const bool live = ok && base + (uint64_t)lane < bound;
                okm = ballot(live);
                // candidates: the strict running minima of l over this wave's successes,
                // below the round-start l0. The round's improvements are the running minima
                // over all its successes in pattern order, so they are a subset of these.
                const uint64_t cm = ballot(live && l < l0r);
                double run = l0r;
                for (uint64_t mm = cm; mm; mm &= mm - 1) {
                    const int L = (int)__builtin_ctzll(mm);
                    const double lv = rdlf(l, L);
                    if (lv < run) {
                        cand |= 1ull << L;
                        run = lv;
                    }
                }
                if ((cand >> lane) & 1ull) {
#pragma unroll
                    for (int s = 0; s < NW; ++s) diff_l[(wid * 64 + lane) * NW + s] = diff.w[s];
                    m_l[wid * 64 + lane] = (uint32_t)m;
                }
                l_l[wid * 64 + lane] = l;
            }
            if (lane == 0) { okm_l[wid] = okm; cand_l[wid] = cand; }
#ifdef BCHK_DIAG
            const unsigned long long t_dec = __builtin_amdgcn_s_memtime();
#endif
            __syncthreads();
#ifdef BCHK_DIAG
            const unsigned long long t_bar = __builtin_amdgcn_s_memtime();
            dg[1] += t_dec - t_prev;
            dg[2] += t_bar - t_dec;
            dg[4] += 1;
            const uint64_t impr0 = S.impr;
#endif
            if (wid == 0) {
                // Visit the round's candidates in pattern order; accept_success runs for
                // those that still improve on the current l0 (rare).
                if (rbase == 0 && !(okm_l[0] & 1ull)) S.firstOK = false;  // :371
                // patterns this round may run to: the loop bound, or the safety cap rounded
                // up to its 64-pattern chunk (as the single-wave kernel applies it)
                const uint64_t capc = p.max_decodes ? ((p.max_decodes + 63) & ~63ull) : ~0ull;
                // lane w < 16 holds wave w's candidate mask: one LDS read, one ballot
                const uint64_t cv = lane < kCoopWaves ? cand_l[lane] : 0ull;
                for (uint64_t wm = ballot(cv != 0ull); wm && !S.done; wm &= wm - 1) {
                    const int w = (int)__builtin_ctzll(wm);
                    uint64_t im = rdl64(cv, w);
                    while (im && !S.done) {
                        const int fl = (int)__builtin_ctzll(im);
                        im &= im - 1;
                        const uint64_t ii = rbase + 64 * (uint64_t)w + (uint64_t)fl;
                        const uint64_t stop = S.bound < capc ? S.bound : capc;
                        if (ii >= stop) { im = 0; break; }
                        const double lL = l_l[w * 64 + fl];
                        if (!(lL < S.l0)) continue;
                        const int mL = (int)m_l[w * 64 + fl];
                        Mask<NW> d;
#pragma unroll
                        for (int s2 = 0; s2 < NW; ++s2) d.w[s2] = diff_l[(w * 64 + fl) * NW + s2];
                        accept_success<M, TMAX>(S, P, d, mL, lL, ii, as, p, lane);
                    }
                }
                // the loop ends in this round when it reaches the bound, or is cut at the
                // cap; whichever chunk comes first (the bound wins a tie), as the
                // single-wave kernel decides at its chunk starts
                if (!S.done) {
                    const uint64_t rend = rbase + 64 * (uint64_t)kCoopWaves;
                    const uint64_t nb = (S.bound + 63) & ~63ull;
                    if (nb <= capc) {
                        if (S.bound <= rend) { S.i_end = S.bound; S.done = true; }
                    } else if (capc <= rend) {
                        S.i_end = capc;
                        S.truncated = true;
                        S.done = true;
                    }
                }
                if (lane == 0) {
                    ctl[0] = S.bound;
                    ctl[1] = S.done ? 1u : 0u;
                    ctl[3] = (uint64_t)__double_as_longlong(S.l0);
                }
            }
#ifdef BCHK_DIAG
            t_prev = __builtin_amdgcn_s_memtime();
            dg[3] += t_prev - t_bar;
            dg[5] += S.impr - impr0;
#endif
        }
        if (wid == 0) write_outputs<M, TMAX>(S, P, p, cw, lane);
#ifdef BCHK_DIAG
        dg[6] = __builtin_amdgcn_s_memtime() - t_start;
        dg[7] = cw;
        if (p.diag && threadIdx.x == 0)
            for (int q = 0; q < 8; ++q) p.diag[(size_t)item * 8 + q] = dg[q];
#endif
        (void)N;
    }
}

// ------------------------------------------------- batched algebraic decoder
// Decoder::decode (src/Decoder.cpp:298-321), one word per lane.
template <int M, int TMAX>
__global__ void __launch_bounds__(256) alg_decode_kernel(AlgParams p) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    constexpr int W = (TMAX + 3) / 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    load_tables(smem, p.tables, p.td.bytes);
    __syncthreads();
    const uint8_t *ex = smem + p.td.off_exp;
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(smem + p.td.off_log);
    const uint32_t *col = reinterpret_cast<const uint32_t *>(smem + p.td.off_col);
    const uint64_t *chien = reinterpret_cast<const uint64_t *>(smem + p.td.off_chien);
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = idx < p.count;
    const uint32_t wi = live ? idx : 0u;
    const uint8_t *w = p.words + (size_t)wi * N;
    uint32_t Sw[W];
#pragma unroll
    for (int j = 0; j < W; ++j) Sw[j] = 0;
    if (p.synd) {
        for (int j = 0; j < p.t; ++j) Sw[j >> 2] |= (p.synd[(size_t)wi * p.t + j] & 0xFFu) << (8 * (j & 3));
    } else {
        for (int pos = 0; pos < N; ++pos) {
            const uint32_t on = w[pos] ? 0xFFFFFFFFu : 0u;
#pragma unroll
            for (int j = 0; j < W; ++j) Sw[j] ^= col[pos * W + j] & on;
        }
    }
    Mask<NW> E;
    const bool ok = alg_decode_word<M, TMAX>(ex, lg, chien, Sw, p.t, E);
    if (!live) return;
    p.ok[idx] = ok ? 1 : 0;
    if (ok)
        for (int pos = 0; pos < N; ++pos)
            p.answers[(size_t)idx * N + pos] = w[pos] ^ (uint8_t)((E.w[pos >> 6] >> (pos & 63)) & 1ull);
}

// --------------------------------------------------------- FER counters
// src/dataForPlot.cpp:55-74: frame errors, bit errors, decodes, comparisons, sums, words.
template <int N>
__global__ void __launch_bounds__(256) count_kernel(const uint8_t *tx, const uint8_t *res,
                                                    const bchk_stats *st, uint32_t B,
                                                    unsigned long long *out6) {
    __shared__ unsigned long long part[6][4];
    unsigned long long c[6] = {0, 0, 0, 0, 0, 0};
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x) {
        int be = 0;
        for (int i = 0; i < N; ++i) be += tx[(size_t)b * N + i] != res[(size_t)b * N + i];
        c[0] += be ? 1 : 0;
        c[1] += be;
        if (st) { c[2] += st[b].decodes; c[3] += st[b].comparisons; c[4] += st[b].sums; }
        c[5] += 1;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        unsigned long long v = c[k];
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) part[k][wid] = v;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        unsigned long long v = 0;
        for (int w = 0; w < (int)(blockDim.x / 64); ++w) v += part[threadIdx.x][w];
        atomicAdd(out6 + threadIdx.x, v);
    }
}

// ------------------------------------------------------------- launchers
template <int M, int TMAX>
static hipError_t launch_search_impl(const SearchParams &p, int grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((kaneko_search_kernel<M, TMAX>), dim3(grid), dim3(kWaveSize * kWavesPerBlock),
                       lds, s, p);
    return hipGetLastError();
}
template <int M, int TMAX>
static hipError_t launch_coop_impl(const SearchParams &p, int grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((kaneko_coop_kernel<M, TMAX>), dim3(grid), dim3(kWaveSize * kCoopWaves),
                       lds, s, p);
    return hipGetLastError();
}
template <int M, int TMAX>
static hipError_t launch_alg_impl(const AlgParams &p, size_t lds, hipStream_t s) {
    const int grid = (int)((p.count + 255) / 256);
    hipLaunchKernelGGL((alg_decode_kernel<M, TMAX>), dim3(grid), dim3(256), lds, s, p);
    return hipGetLastError();
}
template <int M, int TMAX>
static const void *search_fn() { return reinterpret_cast<const void *>(&kaneko_search_kernel<M, TMAX>); }
template <int M, int TMAX>
static const void *coop_fn() { return reinterpret_cast<const void *>(&kaneko_coop_kernel<M, TMAX>); }

template <int M, int TMAX>
static KernelSet make_set() {
    constexpr int NW = Geo<M>::NW;
    const size_t coop = (size_t)kCoopWaves * 8 + (size_t)kCoopWaves * 64 * NW * 8 +
                        (size_t)kCoopWaves * 64 * 12 + 32 + (size_t)kCoopWaves * 8 +
                        (size_t)kCoopWaves * Smem<M, TMAX>::WAVE_BYTES;
    return KernelSet{&launch_search_impl<M, TMAX>, &launch_coop_impl<M, TMAX>, &coop_fn<M, TMAX>, coop,
                     &launch_alg_impl<M, TMAX>, &search_fn<M, TMAX>, TMAX,
                     (size_t)Smem<M, TMAX>::WAVE_BYTES};
}

// TMAX buckets: smallest instantiated bucket >= t.
bool select_kernels(int m, int t, KernelSet *out) {
#define BCHK_TRY(MM, TT) \
    if (m == MM && t <= TT) { *out = make_set<MM, TT>(); return true; }
    BCHK_TRY(2, 1)
    BCHK_TRY(3, 3)
    BCHK_TRY(4, 2) BCHK_TRY(4, 7)
    BCHK_TRY(5, 3) BCHK_TRY(5, 8) BCHK_TRY(5, 15)
    BCHK_TRY(6, 6) BCHK_TRY(6, 12) BCHK_TRY(6, 31)
    BCHK_TRY(7, 8) BCHK_TRY(7, 16) BCHK_TRY(7, 32)
    BCHK_TRY(8, 15) BCHK_TRY(8, 16) BCHK_TRY(8, 32)
#undef BCHK_TRY
    return false;
}

hipError_t launch_search(const KernelSet &k, const SearchParams &p, int grid, size_t lds, hipStream_t s) {
    return k.search(p, grid, lds, s);
}
hipError_t launch_alg(const KernelSet &k, const AlgParams &p, size_t lds, hipStream_t s) {
    return k.alg(p, lds, s);
}
hipError_t launch_count(int n, const uint8_t *tx, const uint8_t *res, const bchk_stats *st,
                        uint32_t B, uint64_t *out6, hipStream_t s) {
    const int grid = (int)((B + 255) / 256) < 2048 ? (int)((B + 255) / 256) : 2048;
    unsigned long long *o = reinterpret_cast<unsigned long long *>(out6);
    switch (n) {
#define BCHK_CNT(NN) \
    case NN: hipLaunchKernelGGL((count_kernel<NN>), dim3(grid > 0 ? grid : 1), dim3(256), 0, s, tx, res, st, B, o); break;
        BCHK_CNT(3) BCHK_CNT(7) BCHK_CNT(15) BCHK_CNT(31) BCHK_CNT(63) BCHK_CNT(127) BCHK_CNT(255)
#undef BCHK_CNT
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace bchk
