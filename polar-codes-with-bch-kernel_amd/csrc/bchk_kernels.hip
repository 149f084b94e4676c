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
    static constexpr int WAVE_BYTES = NP * 8 + NP; // sorted |alpha| (f64) + order (u8)
};

// ---------------------------------------------------------- Kaneko search
// One codeword per wave. Reference: KanekoKernelProcessor::decode(answer, word, res)
// src/KanekoKernelProcessor.cpp:335-407 (variant ANSWER) and decode(word, res) :212-276
// (variant WORD).
template <int M, int TMAX>
__device__ void search_codeword(const SearchParams &p, const uint8_t *ex, const uint16_t *lg,
                                const uint32_t *col, const uint64_t *chien, double *as,
                                uint8_t *ordl, uint32_t cw, int lane) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    constexpr int W = (TMAX + 3) / 4;
    constexpr int NB = N < 31 ? N : 31;  // pattern bits in use (i < 2^31)
    const int t = p.t;
    const double *y = p.y + (size_t)cw * N;

    // ---- prologue :336-343: alpha = 2*word/pow(sd,2); yH; |alpha|
    double av[NW];
    Mask<NW> yH;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        const bool valid = pos < N;
        const double yy = valid ? y[pos] : 0.0;
        const double al = (2.0 * yy) / p.s2;
        av[s] = valid ? fabs(al) : 0.0;
        yH.w[s] = ballot(valid && !(al <= 0.0));
    }
    // exact rank by (|alpha|, position): the stable order of std::sort's keys (:343)
    int rk[NW];
    bool tie = false;
#pragma unroll
    for (int s = 0; s < NW; ++s) rk[s] = 0;
#pragma unroll
    for (int q = 0; q < N; ++q) {
        const double aq = rdlf(av[q >> 6], q & 63);
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int pos = lane + 64 * s;
            const bool lt = aq < av[s];
            const bool eq = aq == av[s];
            rk[s] += (lt || (eq && q < pos)) ? 1 : 0;
            tie |= eq && (q != pos) && (pos < N);
        }
    }
    const bool any_tie = ballot(tie) != 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        if (pos < N) {
            as[rk[s]] = av[s];
            ordl[rk[s]] = (uint8_t)pos;
        }
    }
    wave_sync();
    double asv[NW];  // sorted |alpha|, lane owns q = lane + 64 s
    int ordv[NW];
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int q = lane + 64 * s;
        asv[s] = q < N ? as[q] : 0.0;
        ordv[s] = q < N ? ordl[q] : 0;
    }

    // ---- syndrome of the hard decision (Decoder::findSyndromPoly :184-207)
    uint32_t S0[W];
#pragma unroll
    for (int w = 0; w < W; ++w) S0[w] = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        if (pos < N && ((yH.w[s] >> lane) & 1ull)) {
#pragma unroll
            for (int w = 0; w < W; ++w) S0[w] ^= col[pos * W + w];
        }
    }
#pragma unroll
    for (int w = 0; w < W; ++w) S0[w] = wave_xor(S0[w]);

    // ---- test patterns (calcError :36-51): bit b of i flips position ord[b].
    // lane b < NB holds ord[b] and its syndrome column.
    const int ordb = ordv[0];
    uint32_t scol[W];
#pragma unroll
    for (int w = 0; w < W; ++w) scol[w] = lane < NB ? col[ordb * W + w] : 0u;
    uint32_t Lo[W];
    Mask<NW> Plo;
#pragma unroll
    for (int w = 0; w < W; ++w) Lo[w] = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) Plo.w[s] = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
        if (b < NB) {
            const bool on = (lane >> b) & 1;
            const int pb = (int)rdl((uint32_t)ordb, b);
#pragma unroll
            for (int w = 0; w < W; ++w) Lo[w] ^= on ? rdl(scol[w], b) : 0u;
            if (on) mask_set<NW>(Plo, pb);
        }
    }

    // ---- search state (:351-358)
    const bool word_variant = p.variant == BCHK_VARIANT_WORD;
    const uint64_t kInfBound = 0x7FFFFFFFFFFFFFFFull;
    int T = N;
    uint64_t bound = word_variant ? kInfBound : ((1ull << (T & 31)) - 1ull);
    double l0 = DBL_MAX;
    bool firstOK = true, accepted = false, returned = false, truncated = false, scan_ub = false;
    int m0 = 0;
    Mask<NW> best;
#pragma unroll
    for (int s = 0; s < NW; ++s) best.w[s] = 0;
    uint64_t jsteps = 0, impr = 0, i_end = 0;
    const int scan_last = N - 1 - t;  // j <= n-1-t (:384)

    for (uint64_t base = 0;; base += 64) {
        if (base >= bound) { i_end = bound; break; }
        if (p.max_decodes && base >= p.max_decodes) { i_end = base; truncated = true; break; }
        // high pattern bits of base (bits >= 6): wave-uniform
        uint32_t Sw[W];
        Mask<NW> P = Plo;
#pragma unroll
        for (int w = 0; w < W; ++w) Sw[w] = S0[w] ^ Lo[w];
        for (uint64_t hb = base >> 6; hb; hb &= hb - 1) {
            const int b = 6 + (int)__builtin_ctzll(hb);
            if (b >= NB) continue;
            const int pb = (int)rdl((uint32_t)ordb, b);
#pragma unroll
            for (int w = 0; w < W; ++w) Sw[w] ^= rdl(scol[w], b);
            mask_set<NW>(P, pb);
        }
        Mask<NW> E;
        const bool ok = alg_core<M, TMAX>(ex, lg, chien, Sw, t, E);
        Mask<NW> diff;  // yH ^ x = pattern ^ error locations
#pragma unroll
        for (int s = 0; s < NW; ++s) diff.w[s] = P.w[s] ^ E.w[s];
        const uint64_t i_lane = base + (uint64_t)lane;
        uint64_t okm = ballot(ok && i_lane < bound);
        if (base == 0 && !(okm & 1ull)) firstOK = false;  // :371

        bool done = false;
        while (okm) {
            const int L = (int)__builtin_ctzll(okm);
            okm &= okm - 1;
            const uint64_t ii = base + (uint64_t)L;
            if (ii >= bound) break;
            Mask<NW> d;
#pragma unroll
            for (int s = 0; s < NW; ++s) d.w[s] = rdl64(diff.w[s], L);
            const int m = mask_popc<NW>(d);                 // calcM :89-97
            if (ii == 0 || !firstOK) m0 = m;                 // :374
            double l = 0.0;                                  // calcL :69-77, index order
#pragma unroll
            for (int s = 0; s < NW; ++s)
                for (uint64_t v = d.w[s]; v; v &= v - 1) l += rdlf(av[s], (int)__builtin_ctzll(v));
            if (!(l < l0)) continue;                         // :377
            // res = x; l0 = l (:378-379)
            best = d;
            l0 = l;
            accepted = true;
            // calcRightSide :54-67 and the calcT prefix (:110-121) over agreeing sorted
            // positions; both are prefixes of the same sequential sum.
            const int border = (2 * t + 1) - (m + m0) / 2;
            const int border2 = t - (m + m0) / 2;
            double rs = 0.0, base2 = 0.0;
            int taken = 0;
            if (border2 <= 0) base2 = 0.0;
#pragma unroll
            for (int s = 0; s < NW; ++s) {
                const int q = lane + 64 * s;
                const int op = ordv[s];
                uint64_t dw = 0;
#pragma unroll
                for (int u = 0; u < NW; ++u) dw = (u == (op >> 6)) ? d.w[u] : dw;
                const bool ag = q < N && !((dw >> (op & 63)) & 1ull);
                uint64_t agm = ballot(ag);
                while (agm && taken < border) {
                    const int b = (int)__builtin_ctzll(agm);
                    agm &= agm - 1;
                    rs += rdlf(asv[s], b);
                    ++taken;
                    if (taken == border2) base2 = rs;
                }
            }
            if (l < rs) { returned = true; i_end = ii + 1; done = true; break; }  // :380
            // calcT scan (:384): while (l >= calcT(j) && j <= n-1-t) ++j, lane-parallel
            int jstar;
            {
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
                jstar = first;
                if (jstar > scan_last + 1) jstar = scan_last + 1;
            }
            if (word_variant && jstar == scan_last + 1) scan_ub = true;  // :257 unbounded
            jsteps += (uint64_t)jstar;
            ++impr;
            if (word_variant) {
                T = jstar;                                   // :264
                bound = 1ull << (T & 63);
            } else {
                T = (p.J >= 0 && jstar > p.J) ? p.J : jstar;  // :392 / :393
                bound = (1ull << (T & 31)) - 1ull;           // (1 << T) - 1 in int32 (:361)
            }
            if (bound <= ii + 1) { i_end = ii + 1; done = true; break; }
        }
        if (done) break;
    }

    // ---- outputs
    const uint64_t decodes = i_end;
    const uint64_t iters = returned ? i_end - 1 : i_end;
    const uint64_t pro = word_variant ? (uint64_t)(2 * N + 1) : 0ull;  // :221-224
    if (accepted) {
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int pos = lane + 64 * s;
            if (pos < N)
                p.res[(size_t)cw * N + pos] = (uint8_t)(((yH.w[s] ^ best.w[s]) >> lane) & 1ull);
        }
    }
    if (lane == 0) {
        if (p.l0) p.l0[cw] = l0;
        if (p.st) {
            bchk_stats st;
            st.decodes = decodes;
            st.comparisons = pro + iters * (uint64_t)(N + 6) + jsteps + impr;
            st.sums = pro + iters * (uint64_t)(N + 1) + jsteps;
            st.iterations = iters;
            st.jsteps = jsteps;
            st.improvements = impr;
            st.flags = (accepted ? BCHK_F_ACCEPTED : 0u) | (returned ? BCHK_F_RETURNED : 0u) |
                       (truncated ? BCHK_F_TRUNCATED : 0u) | (any_tie ? BCHK_F_TIE : 0u) |
                       (scan_ub ? BCHK_F_SCAN_UB : 0u);
            st.reserved = 0;
            p.st[cw] = st;
        }
    }
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
    uint8_t *ordl = wbase + NP * 8;
    if (!p.queue) {
        const uint32_t stride = gridDim.x * kWavesPerBlock;
        for (uint32_t cw = blockIdx.x * kWavesPerBlock + wid; cw < p.count; cw += stride)
            search_codeword<M, TMAX>(p, ex, lg, col, chien, as, ordl, cw, lane);
        return;
    }
    // Work queue left by the fast path: sub-queue x holds items x, x+8, x+16, ...; a wave
    // drains its own XCD's sub-queue first (one L2-local atomic per codeword), then steals.
    const uint32_t total = *p.qcount;
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
        search_codeword<M, TMAX>(p, ex, lg, col, chien, as, ordl, p.queue[item], lane);
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
    const bool ok = alg_core<M, TMAX>(ex, lg, chien, Sw, p.t, E);
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
static hipError_t launch_alg_impl(const AlgParams &p, size_t lds, hipStream_t s) {
    const int grid = (int)((p.count + 255) / 256);
    hipLaunchKernelGGL((alg_decode_kernel<M, TMAX>), dim3(grid), dim3(256), lds, s, p);
    return hipGetLastError();
}
template <int M, int TMAX>
static const void *search_fn() { return reinterpret_cast<const void *>(&kaneko_search_kernel<M, TMAX>); }


template <int M, int TMAX>
static KernelSet make_set() {
    return KernelSet{&launch_search_impl<M, TMAX>, &launch_alg_impl<M, TMAX>, &search_fn<M, TMAX>,
                     TMAX, (size_t)Smem<M, TMAX>::WAVE_BYTES};
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
