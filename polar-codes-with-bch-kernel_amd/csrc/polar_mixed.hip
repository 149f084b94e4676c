// polar_mixed.hip -- batched SC-list decoding of polar codes over MIXED binary kernels (Arikan
// layers and matrix kernels, e.g. BCH-derived ones) on gfx950.
//
// Reference: CMixedKernelListDecoder (out/external/MixedKernelListDecoder.cpp:61-268) over
// CListKernelEngine (out/external/KernelListEngine.cpp:266-447); Arikan layers by the f/g of
// SoftProcessing.cpp:39-80; matrix layers by CTrellisKernelProcessor::GetLLRs
// (out/external/TrellisKernelProcessor.cpp:234-294): the offset state accumulates the known
// kernel inputs times their rows, and the LLR of input `phase` is the min-sum difference
// best[1] - best[0] over the coset of the remaining rows (each word's metric a left-to-right
// float sum of |y| over its disagreeing positions -- the trellis's value bit for bit, see
// oracle/polar_oracle.c). Same decisions, arithmetic and path indices as the CPU restatement.
//
// Execution model: one wave per codeword (persistent). Every path's S (per layer, outer[λ]
// floats), C (kernel inputs per layer) and matrix offset states live in LDS; lane q < L holds
// path q's scalars (metric, leaf LLR, dynamic-freezing mask, record word, stack slot). A
// matrix LLR's coset is split over lanes when there are fewer (path, element) items than lanes
// (float min is exact, so any split gives the same value). The all-Arikan kernel
// (polar_sclist.hip) stays the fast path for codes without matrix layers.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "polar_device.h"

namespace bchk {

namespace {

constexpr uint32_t kUninitM = 0xFFFFFFFFu;

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ float rdlf_m(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint32_t rdlu_m(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t rdlu64_m(uint64_t v, int l) {
    return (uint64_t)rdlu_m((uint32_t)v, l) | ((uint64_t)rdlu_m((uint32_t)(v >> 32), l) << 32);
}

struct MStack {  // TVMemoryEngine's path-index stack with lazy initialisation (misc.h:212-226)
    uint32_t slot;
    int top;
    __device__ __forceinline__ void reset(int L, int lane) {
        top = L;
        if (lane == L) slot = kUninitM;
    }
    __device__ __forceinline__ uint32_t pop(int lane) {
        const uint32_t v = rdlu_m(slot, top);
        if (v == kUninitM) {
            const int r = top - 1;
            top = r;
            if (r > 0 && lane == r) slot = kUninitM;
            return (uint32_t)r;
        }
        --top;
        return v;
    }
    __device__ __forceinline__ void push(uint32_t x, int lane) {
        ++top;
        if (lane == top) slot = x;
    }
};

// min over the words of one half of the coset (CTrellisKernelProcessor::GetLLRs, :272-292):
// words c = XOR of rows phase+1 .. l-1 selected by v, v = first, first + step, ...; metric of
// c (b = 0) and c ^ row[phase] (b = 1) against the hard decision (l <= 32)
__device__ __forceinline__ void coset_min(const uint64_t *rows, int l, int phase, const float *ay, uint64_t hd,
                                          uint32_t first, uint32_t step, float &b0, float &b1) {
    const int nfree = l - phase - 1;
    const uint32_t nw = 1u << nfree;
    for (uint32_t v = first; v < nw; v += step) {
        uint64_t c = 0;
        for (int r = 0; r < nfree; ++r)
            if ((v >> r) & 1u) c ^= rows[phase + 1 + r];
        const uint64_t d0 = c ^ hd, d1 = d0 ^ rows[phase];
        float m0 = 0.0f, m1 = 0.0f;  // left to right (:279-282)
        for (int j = 0; j < l; ++j) {
            if ((d0 >> j) & 1ull) m0 += ay[j];
            if ((d1 >> j) & 1ull) m1 += ay[j];
        }
        b0 = m0 < b0 ? m0 : b0;
        b1 = m1 < b1 ? m1 : b1;
    }
}


// ---- exact kernel LLRs by an ordered-statistics search (matrix kernels beyond the trellis
// limit, e.g. the 64 x 64 extended-BCH kernel of root bchCoder.cpp:356-389 makeMatrix).
// The value is CTrellisKernelProcessor's (:234-294): best[1] - best[0], best[b] the least
// left-to-right float sum of |y| over the disagreeing positions of a word of rows phase+1..l-1
// (b = 0) or of those words plus row `phase` (b = 1). Gauss-Jordan over the positions in
// decreasing |y| gives the most reliable basis of rows phase+1..l-1 (the pivots); a word of
// half b is fixed by its pivot values, and the one matching the hard decision there is the
// root. Flipping a set E of pivots costs at least the sum of their |y| (those positions then
// disagree), so a search over E, cheapest pivot first, that drops every subtree whose flip cost
// exceeds the best metric found (less a float-rounding margin) still visits every word that
// can be a minimum: the result is the coset enumeration's, bit for bit. The wave works on one
// item: 64 lanes sort the positions and eliminate (a lane per row), then evaluate 64 search
// nodes per round (a node per lane) from a LIFO in LDS.
struct MlNode {  // the words c ^ G[i] (and below them): flip cost so far lb, half b
    uint32_t clo, chi;
    uint32_t lbib;  // lb's float bits with the low 7 mantissa bits replaced by i << 1 | b
};                  // (truncating a non-negative float lowers it: still a lower bound)
__device__ __forceinline__ MlNode ml_node(uint64_t c, float lb, int i, int b) {
    return MlNode{(uint32_t)c, (uint32_t)(c >> 32), (__float_as_uint(lb) & ~0x7Fu) | ((uint32_t)i << 1) | (uint32_t)b};
}
struct MlScratch {
    uint64_t *G;   // [64] reduced basis, by increasing flip cost
    uint64_t *U;   // [65] U[i]: non-pivot positions rows i.. can change (suffix unions)
    float *cost;   // [64] flip cost of each basis row (|y| at its pivot)
    float *ay;     // [64] |y| by position
    MlNode *stk;   // [kMlStack]
};
// a subtree is dropped when lb * kMlShrink > best: a float sum of at most 64 non-negative terms
// is within 64 u (u = 2^-24) of the exact sum, for lb and for every metric, so the margin
// 2^-15 > 2 * 64 u keeps every word whose float metric could be <= best
constexpr float kMlShrink = 1.0f - 1.0f / 32768.0f;

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
// v from lane ^ J without the LDS crossbar: DPP quad permutes (J = 1, 2), row rotates (J = 4,
// 8) and the gfx950 row / half swaps (J = 16, 32)
template <int J>
__device__ __forceinline__ uint32_t xlane(uint32_t v, int lane) {
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    } else if constexpr (J == 4) {
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x12C, 0xF, 0xF, false);
        return (lane & 4) ? dn : up;
    } else if constexpr (J == 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);
    } else if constexpr (J == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else {
        static_assert(J == 32, "lane distance");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
}
// minimum over the wave of non-negative floats or +inf (their bit patterns order as the
// values do), by DPP / permlane steps
__device__ __forceinline__ float wave_minf(float v) {
    const int lane = (int)__lane_id();
    uint32_t b = __float_as_uint(v), o;
    o = xlane<1>(b, lane);  b = o < b ? o : b;
    o = xlane<2>(b, lane);  b = o < b ? o : b;
    o = xlane<4>(b, lane);  b = o < b ? o : b;
    o = xlane<8>(b, lane);  b = o < b ? o : b;
    o = xlane<16>(b, lane); b = o < b ? o : b;
    o = xlane<32>(b, lane); b = o < b ? o : b;
    return __uint_as_float(b);
}
__device__ __forceinline__ uint64_t wave_xor64(uint64_t v) {
    for (int m = 1; m < 64; m <<= 1) v ^= shfl_xor64(v, m);
    return v;
}
// the metric of the word whose disagreement mask is dis: |y| summed in index order (adding
// +0 where a position agrees leaves the sum unchanged, so this is the trellis's path sum)
// Only the set positions are visited, in ascending order: the +0 terms of the index-order
// sum leave a float sum of non-negative terms unchanged, so the bits are the same, and a lane
// runs popc(dis) steps instead of l.
__device__ __forceinline__ uint64_t ml_below(int l) { return l >= 64 ? ~0ull : ((1ull << l) - 1ull); }
__device__ __forceinline__ float ml_metric(uint64_t dis, const float *ay, int l) {
    float m = 0.0f;
    for (uint64_t v = dis & ml_below(l); v; v &= v - 1) m += ay[__builtin_ctzll(v)];
    return m;
}
// the same, and (fx) the sum over the subset fix of dis
__device__ __forceinline__ void ml_metric2(uint64_t dis, uint64_t fix, const float *ay, int l, float &m, float &fx) {
    m = ml_metric(dis, ay, l);
    fx = ml_metric(fix, ay, l);
}

// A search suspended between two rounds (time-budgeted launches): the wave-uniform state
// beside the scratch (G, U, cost, ay, the stack's first sp nodes), which the caller saves
// and restores with it.
struct MlResume {
    int sp;
    float best0, best1;
    uint64_t hd, lrb;
};

// rs == null: the whole search in this call. Otherwise *resume says whether the scratch and
// *rs hold a suspended search to continue, and past the deadline (t_launch + budget on the
// 100 MHz clock), after at least one round of this call, the search stops between two rounds:
// *rs filled, *suspended set, the return value meaningless.
__device__ float ml_llr(const uint64_t *kr, int l, int loc, const float *src, const uint8_t *off, int d, int s,
                        int lane, const MlScratch &ms, MlResume *rs = nullptr, bool resume = false,
                        uint64_t t_launch = 0, uint64_t budget = 0, bool *suspended = nullptr) {
    const float kInf = __int_as_float(0x7F800000);
    const uint64_t lt = (1ull << lane) - 1ull;
    const int nf = l - loc - 1;
    uint64_t hd, lrb;
    float best0, best1;
    int sp;
    if (rs && resume) {
        hd = rs->hd;
        lrb = rs->lrb;
        best0 = rs->best0;
        best1 = rs->best1;
        sp = rs->sp;
    } else {
        // the layer's LLRs with the known inputs' sign flips (:240-262), HD = Y < 0 (:270-276)
        float a = 0.0f;
        bool neg = false;
        if (lane < l) {
            const float v = src[lane * d + s];
            const float yv = off[lane * d + s] ? -v : v;
            neg = yv < 0.0f;
            a = fabsf(yv);
            ms.ay[lane] = a;
        }
        hd = __ballot(neg);
        wsync();
        if (nf <= kMlEnumBits) {  // small coset: enumerated, words spread over the lanes
            float b0 = kInf, b1 = kInf;
            for (uint32_t v = (uint32_t)lane; v < (1u << nf); v += 64) {
                uint64_t c = 0;
                for (int r = 0; r < nf; ++r)
                    if ((v >> r) & 1u) c ^= kr[loc + 1 + r];
                const float m0 = ml_metric(c ^ hd, ms.ay, l), m1 = ml_metric(c ^ hd ^ kr[loc], ms.ay, l);
                b0 = m0 < b0 ? m0 : b0;
                b1 = m1 < b1 ? m1 : b1;
            }
            return wave_minf(b1) - wave_minf(b0);
        }
        // positions by decreasing |y| (bitonic across the lanes; key: |y| bits, valid, position)
        uint64_t key = lane < l ? (((uint64_t)__float_as_uint(a) << 8) | 0x80ull | (uint64_t)(63 - lane)) : 0ull;
        for (int k = 2; k <= 64; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                const uint64_t o = shfl_xor64(key, j);
                const bool desc = (lane & k) == 0, lower = (lane & j) == 0;
                key = (lower == desc) ? (o > key ? o : key) : (o < key ? o : key);
            }
        const int pos = 63 - (int)(key & 63ull);
        // Gauss-Jordan: lane i < nf holds row loc + 1 + i; pivots in decreasing |y|
        uint64_t g = lane < nf ? kr[loc + 1 + lane] : 0ull;
        bool used = false;
        int t = 0, piv = 0;
        for (int si = 0, np = 0; si < l && np < nf; ++si) {
            const int p = __builtin_amdgcn_readlane(pos, si);
            const uint64_t cand = __ballot(lane < nf && !used && ((g >> p) & 1ull));
            if (!cand) continue;
            const int r = (int)__builtin_ctzll(cand);
            const uint64_t gr = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)g, r) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(g >> 32), r) << 32);
            if (lane == r) {
                used = true;
                t = np;
                piv = p;
            } else if (lane < nf && ((g >> p) & 1ull)) {
                g ^= gr;
            }
            ++np;
        }
        if (lane < nf) {  // found in decreasing |y|: index nf - 1 - t runs by increasing cost
            ms.G[nf - 1 - t] = g;
            ms.cost[nf - 1 - t] = ms.ay[piv];
        }
        // non-pivot positions; below a word that has taken rows up to i - 1, every non-pivot
        // disagreement outside U[i] is fixed, so its |y| bounds the subtree from below too
        uint64_t pm = lane < nf ? (1ull << piv) : 0ull;
        for (int o = 1; o < 64; o <<= 1) pm |= shfl_xor64(pm, o);
        lrb = ~pm & (l >= 64 ? ~0ull : ((1ull << l) - 1ull));
        wsync();
        if (lane <= nf) {
            uint64_t u = 0ull;
            for (int q = lane; q < nf; ++q) u |= ms.G[q] & lrb;
            ms.U[lane] = u;
        }
        // the roots: the word of each half that matches the hard decision on the pivots
        const uint64_t root0 = wave_xor64(lane < nf && ((hd >> piv) & 1ull) ? g : 0ull);
        const uint64_t t1 = hd ^ kr[loc];
        const uint64_t root1 = kr[loc] ^ wave_xor64(lane < nf && ((t1 >> piv) & 1ull) ? g : 0ull);
        best0 = ml_metric(root0 ^ hd, ms.ay, l);
        best1 = ml_metric(root1 ^ hd, ms.ay, l);
        if (lane == 0) {
            ms.stk[0] = ml_node(root0, 0.0f, 0, 0);
            ms.stk[1] = ml_node(root1, 0.0f, 0, 1);
        }
        sp = 2;
        wsync();
    }
    // a guard only (the search tree is finite): past 2^20 rounds the LLR is NaN, never a hang
    for (uint32_t rounds = 0; sp > 0; ++rounds) {
        if (rounds >= (1u << 20)) return __int_as_float(0x7FC00000);
        if (rs && rounds > 0 && __builtin_amdgcn_s_memrealtime() - t_launch > budget) {
            rs->sp = sp;  // past the launch's deadline: stop between two rounds
            rs->best0 = best0;
            rs->best1 = best1;
            rs->hd = hd;
            rs->lrb = lrb;
            *suspended = true;
            return 0.0f;
        }
        // the top n nodes, one per lane; n shrinks near the stack's end so that the pushes of a
        // round (at most 2 per node) and of one depth-first descent (< 64) always fit
        int n = sp < 64 ? sp : 64;
        const int room = kMlStack - 128 - sp;
        if (room < n) n = room > 1 ? room : 1;
        const bool have = lane < n;
        MlNode e{0u, 0u, 0u};
        if (have) e = ms.stk[sp - n + lane];
        sp -= n;
        wsync();
        const uint64_t ec = (uint64_t)e.clo | ((uint64_t)e.chi << 32);
        const float elb = __uint_as_float(e.lbib & ~0x7Fu);
        const int i = (int)((e.lbib >> 1) & 63u);
        const bool hb = (e.lbib & 1u) != 0;
        const float bound = hb ? best1 : best0;
        const float l2 = have ? elb + ms.cost[i] : kInf;
        const bool live = have && l2 * kMlShrink <= bound;
        uint64_t c2 = 0ull;
        float m = kInf, fx = 0.0f;
        if (live) {
            c2 = ec ^ ms.G[i];
            const uint64_t dis = c2 ^ hd;
            ml_metric2(dis, dis & lrb & ~ms.U[i + 1], ms.ay, l, m, fx);
        }
        const float n0 = wave_minf(live && !hb ? m : kInf), n1 = wave_minf(live && hb ? m : kInf);
        best0 = n0 < best0 ? n0 : best0;
        best1 = n1 < best1 ? n1 : best1;
        const float nb = hb ? best1 : best0;
        const bool more = live && i + 1 < nf;
        const float nc = more ? ms.cost[i + 1] : 0.0f;
        const bool psib = more && (elb + nc) * kMlShrink <= nb;     // the next pivot instead of this one
        const bool pch = more && (l2 + fx + nc) * kMlShrink <= nb;  // this one and a later one
        const uint64_t ms_ = __ballot(psib), mc = __ballot(pch);
        const int nsib = __builtin_popcountll(ms_);
        if (psib) ms.stk[sp + __builtin_popcountll(ms_ & lt)] = ml_node(ec, elb, i + 1, hb ? 1 : 0);
        if (pch) ms.stk[sp + nsib + __builtin_popcountll(mc & lt)] = ml_node(c2, l2, i + 1, hb ? 1 : 0);
        sp += nsib + __builtin_popcountll(mc);
        wsync();
    }
    return best1 - best0;  // (:292)
}

}  // namespace

__global__ void __launch_bounds__(64) polar_mixed_kernel(PolarMixedParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)threadIdx.x;
    const int U = p.U, nl = p.nl, L = p.L, K = p.K;
    const int RW = polar_rec_words(K);
    // LDS: polar_mixed_lds_bytes (polar_device.h)
    const PolarMixedLayout lo = polar_mixed_layout(U, L, p.ssize, p.csize, p.osize, nl, RW);
    const int o_S = lo.o_S, o_C = lo.o_C, o_O = lo.o_O, o_ph = lo.o_ph, o_rows = lo.o_rows, o_act = lo.o_act,
              o_tm = lo.o_tm;
    float *chan = reinterpret_cast<float *>(smem);
    float *S = reinterpret_cast<float *>(smem + o_S);
    uint8_t *C = smem + o_C;
    uint8_t *O = smem + o_O;
    uint16_t *ph = reinterpret_cast<uint16_t *>(smem + o_ph);
    uint64_t *rows = reinterpret_cast<uint64_t *>(smem + o_rows);  // [layer][row] bitmasks
    uint32_t *act = reinterpret_cast<uint32_t *>(smem + o_act);
    uint32_t *rec = act + L;
    float *tmet = reinterpret_cast<float *>(smem + o_tm);  // trellis state metrics, 2 x tstates
    uint8_t *mls = smem + ((o_tm + 8 * p.tstates + 15) & ~15);  // ordered-statistics search scratch
    MlScratch ms{reinterpret_cast<uint64_t *>(mls), reinterpret_cast<uint64_t *>(mls + 512),
                 reinterpret_cast<float *>(mls + 1040), reinterpret_cast<float *>(mls + 1296),
                 reinterpret_cast<MlNode *>(mls + 1552)};
    const bool mine = lane < L;
    for (int i = lane; i < U; i += 64) ph[i] = p.phase[i];
    for (int i = lane; i < kPolarMaxKernel * nl; i += 64) rows[i] = p.krows[i];
    auto Sof = [&](int q, int lam) -> float * { return lam == 0 ? chan : S + (size_t)q * p.ssize + p.soff[lam]; };
    auto Cof = [&](int q, int lam) -> uint8_t * { return C + (size_t)q * p.csize + p.coff[lam]; };
    auto Oof = [&](int q, int j) -> uint8_t * { return O + (size_t)q * p.osize + p.ooff[j]; };
    auto list_act = [&](uint32_t active) {
        if (mine && ((active >> lane) & 1u)) act[__builtin_popcount(active & ((1u << lane) - 1u))] = (uint32_t)lane;
        wsync();
        return __builtin_popcount(active);
    };
    const int lastsz = p.ksize[nl - 1];
    const int lastc = p.coff[nl];
    MStack st;
    st.slot = 0;
    wsync();
    // time-budgeted launches (PolarMixedParams::budget): this launch's start on the 100 MHz clock
    const bool budgeted = p.budget != 0 && p.rstate != nullptr;
    const uint64_t t_launch = __builtin_amdgcn_s_memrealtime();
    auto expired = [&]() { return budgeted && __builtin_amdgcn_s_memrealtime() - t_launch > p.budget; };
    for (uint32_t cw = blockIdx.x; cw < p.B; cw += gridDim.x) {
        const uint32_t cst = budgeted ? __builtin_amdgcn_readfirstlane(p.rstate[cw]) : 0u;
        if (cst == 2u) continue;  // finished by an earlier launch
        if (expired()) {          // past the budget: start (or resume) nothing more
            if (lane == 0) atomicAdd(p.unfinished, 1u);
            continue;
        }
        uint8_t *sv = budgeted ? p.rsave + (size_t)cw * p.rstride : nullptr;
        uint32_t active;
        float R = 0.0f, lv = 0.0f;
        uint64_t dm = 0;
        uint32_t rw = 0;
        int k = 0, phi0 = 0, rj = -1, rit = 0;  // rj >= 0: resume in layer rj at item rit
        if (cst == 1u) {
            // resume a suspended codeword: header, registers, the list state's LDS
            const uint32_t *hd = reinterpret_cast<const uint32_t *>(sv);
            phi0 = (int)__builtin_amdgcn_readfirstlane(hd[0]);
            rj = (int)__builtin_amdgcn_readfirstlane(hd[1]);
            rit = (int)__builtin_amdgcn_readfirstlane(hd[2]);
            k = (int)__builtin_amdgcn_readfirstlane(hd[3]);
            active = __builtin_amdgcn_readfirstlane(hd[4]);
            st.top = (int)__builtin_amdgcn_readfirstlane(hd[5]);
            const uint32_t *rg = hd + 16 + 6 * lane;
            R = __uint_as_float(rg[0]);
            lv = __uint_as_float(rg[1]);
            dm = (uint64_t)rg[2] | ((uint64_t)rg[3] << 32);
            rw = rg[4];
            st.slot = rg[5];
            const uint8_t *ls = sv + 64 + 64 * 24;
            for (int i = 4 * lane; i < o_ph; i += 256) *reinterpret_cast<uint32_t *>(smem + i) = *reinterpret_cast<const uint32_t *>(ls + i);
            for (int i = 4 * lane; i < o_tm - o_act; i += 256)
                *reinterpret_cast<uint32_t *>(smem + o_act + i) = *reinterpret_cast<const uint32_t *>(ls + o_ph + i);
        } else {
            const float *y = p.llr + (size_t)cw * p.N;  // LoadLLRs (MixedKernelEncoder.cpp:181-207)
            for (int i = lane; i < U; i += 64) {
                const int m = p.symmap[i];
                chan[i] = m >= 0 ? y[m] : (m == -1 ? 100000.0f : 0.0f);
            }
            st.reset(L, lane);
            const uint32_t pid = st.pop(lane);
            active = 1u << pid;
        }
        wsync();
        int nact = list_act(active);
        bool progressed = false, yielded = false;
        // suspend between two search items (the list state is complete there: every layer
        // before rj done, layer rj's offset state applied, items before it done)
        MlResume mr{0, 0.0f, 0.0f, 0ull, 0ull};
        bool rmid = false;  // resuming inside a search item (its scratch saved too)
        if (cst == 1u) {
            const uint32_t *hd = reinterpret_cast<const uint32_t *>(sv);
            rmid = __builtin_amdgcn_readfirstlane(hd[6]) != 0u;
            if (rmid) {
                mr.sp = (int)__builtin_amdgcn_readfirstlane(hd[7]);
                mr.best0 = __uint_as_float(__builtin_amdgcn_readfirstlane(hd[8]));
                mr.best1 = __uint_as_float(__builtin_amdgcn_readfirstlane(hd[9]));
                // (readfirstlane returns int: through uint32_t, or the low word sign-extends)
                mr.hd = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(hd[10]) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(hd[11]) << 32);
                mr.lrb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(hd[12]) |
                         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(hd[13]) << 32);
                const uint8_t *ml = sv + 64 + 64 * 24 + o_ph + (o_tm - o_act);
                const int mb = (int)kMlHeadBytes + 12 * mr.sp;  // G, U, cost, ay, stack[0, sp)
                for (int i = 4 * lane; i < mb; i += 256) *reinterpret_cast<uint32_t *>(mls + i) = *reinterpret_cast<const uint32_t *>(ml + i);
                wsync();
            }
        }
        // mid: inside a search item, whose scratch and MlResume go along
        auto suspend = [&](int phi, int j, int it, bool mid) {
            uint32_t *hd = reinterpret_cast<uint32_t *>(sv);
            if (lane == 0) {
                hd[0] = (uint32_t)phi;
                hd[1] = (uint32_t)j;
                hd[2] = (uint32_t)it;
                hd[3] = (uint32_t)k;
                hd[4] = active;
                hd[5] = (uint32_t)st.top;
                hd[6] = mid ? 1u : 0u;
                hd[7] = (uint32_t)mr.sp;
                hd[8] = __float_as_uint(mr.best0);
                hd[9] = __float_as_uint(mr.best1);
                hd[10] = (uint32_t)mr.hd;
                hd[11] = (uint32_t)(mr.hd >> 32);
                hd[12] = (uint32_t)mr.lrb;
                hd[13] = (uint32_t)(mr.lrb >> 32);
            }
            if (mid) {
                uint8_t *ml = sv + 64 + 64 * 24 + o_ph + (o_tm - o_act);
                const int mb = (int)kMlHeadBytes + 12 * mr.sp;
                for (int i = 4 * lane; i < mb; i += 256) *reinterpret_cast<uint32_t *>(ml + i) = *reinterpret_cast<const uint32_t *>(mls + i);
            }
            uint32_t *rg = hd + 16 + 6 * lane;
            rg[0] = __float_as_uint(R);
            rg[1] = __float_as_uint(lv);
            rg[2] = (uint32_t)dm;
            rg[3] = (uint32_t)(dm >> 32);
            rg[4] = rw;
            rg[5] = st.slot;
            uint8_t *ls = sv + 64 + 64 * 24;
            for (int i = 4 * lane; i < o_ph; i += 256) *reinterpret_cast<uint32_t *>(ls + i) = *reinterpret_cast<const uint32_t *>(smem + i);
            for (int i = 4 * lane; i < o_tm - o_act; i += 256)
                *reinterpret_cast<uint32_t *>(ls + o_ph + i) = *reinterpret_cast<const uint32_t *>(smem + o_act + i);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            if (lane == 0) {
                p.rstate[cw] = 1u;
                atomicAdd(p.unfinished, 1u);
            }
            yielded = true;
        };
        for (int phi = phi0; phi < U && !yielded; ++phi) {
            const uint32_t e = __builtin_amdgcn_readfirstlane((uint32_t)ph[phi]);
            // ---- IterativelyCalcS (KernelListEngine.cpp:370-447)
            int m = nl - 1;
            uint32_t pq = (uint32_t)phi;
            while (m > 0 && pq % (uint32_t)p.ksize[m] == 0) {
                pq /= (uint32_t)p.ksize[m];
                --m;
            }
            for (int j = m; j < nl; ++j) {
                if (rj >= 0 && j < rj) continue;  // done before the suspension
                const bool resume_here = rj == j;
                const int loc = (j == m) ? (int)(pq % (uint32_t)p.ksize[j]) : 0;
                const int d = p.outer[j + 1], l = p.ksize[j];
                const int tot = nact * d;
                if (p.arikan[j]) {
                    for (int it = lane; it < tot; it += 64) {
                        const int q = (int)act[it / d], s = it % d;
                        const float *src = Sof(q, j);
                        float *dst = Sof(q, j + 1);
                        const float a = src[s], b = src[d + s];
                        float r;
                        if (loc) {  // SoftCombine (:39-50)
                            r = Cof(q, j + 1)[s] ? b - a : b + a;
                        } else {    // SoftXOR (:54-80)
                            const float fa = fabsf(a), fb = fabsf(b), mn = fa < fb ? fa : fb;
                            r = __uint_as_float(__float_as_uint(mn) |
                                                ((__float_as_uint(a) ^ __float_as_uint(b)) & 0x80000000u));
                        }
                        dst[s] = r;
                    }
                    wsync();
                    continue;
                }
                // matrix layer: offset state (:240-262), then the min-sum LLR per element
                const uint64_t *kr = rows + kPolarMaxKernel * j;
                for (int it = lane; it < tot && !resume_here; it += 64) {  // (applied before a suspension)
                    const int q = (int)act[it / d], s = it % d;
                    uint8_t *off = Oof(q, j);
                    if (!loc) {
                        for (int i = 0; i < l; ++i) off[i * d + s] = 0;
                    } else {
                        const uint8_t kn = Cof(q, j + 1)[(loc - 1) * d + s];
                        if (kn)
                            for (int i = 0; i < l; ++i)
                                if ((kr[loc - 1] >> i) & 1ull) off[i * d + s] ^= 1u;
                    }
                }
                wsync();
                if (p.ml[j]) {
                    // exact ordered-statistics search (kernels larger than the trellis limit):
                    // one item at a time, the whole wave on it
                    for (int it = resume_here ? rit : 0; it < tot; ++it) {
                        if (progressed && expired()) {  // past the launch's budget: suspend here
                            suspend(phi, j, it, false);
                            break;
                        }
                        const int q = (int)act[it / d], s = it % d;
                        const bool mid = resume_here && it == rit && rmid;  // continue a suspended search
                        bool susp = false;
                        const float v = ml_llr(kr, l, loc, Sof(q, j), Oof(q, j), d, s, lane, ms,
                                               budgeted && !p.no_mid ? &mr : nullptr, mid, t_launch, p.budget,
                                               &susp);
                        if (susp) {  // the search itself ran past the budget: suspended inside it
                            suspend(phi, j, it, true);
                            break;
                        }
                        if (lane == 0) Sof(q, j + 1)[s] = v;
                        wsync();
                        progressed = true;
                    }
                    rj = -1;
                    if (yielded) break;
                    continue;
                }
                if (p.trellis[j]) {
                    // CTrellisKernelProcessor::GetLLRs (:260-292) as a pull-form Viterbi: a state
                    // of depth dd + 1 takes the smaller of its (at most two) predecessors' metrics,
                    // each plus |Y| when its edge label differs from the hard decision (min
                    // commutes with the monotone float add, so the values are the reference's).
                    // G lanes per item (G = states of the phase's widest depth, at most 64).
                    const int tp = j * kPolarMaxKernel + loc;
                    const uint8_t *lgp = p.tlog + (size_t)tp * (kPolarMaxKernel + 1);
                    const uint32_t *ent0 = p.tent + p.tbase[tp];
                    int ab = 0;
                    for (int dd = 1; dd <= l; ++dd) ab = lgp[dd] > ab ? lgp[dd] : ab;
                    const int stride = 1 << ab, G = stride < 64 ? stride : 64, ipr = 64 / G;
                    const int slot = lane / G, sub = lane % G;
                    for (int base = 0; base < tot; base += ipr) {
                        const int it = base + slot;
                        const bool have = slot < ipr && it < tot;
                        int q = 0, s = 0;
                        if (have) {
                            q = (int)act[it / d];
                            s = it % d;
                        }
                        const float *src = Sof(q, j);
                        const uint8_t *off = Oof(q, j);
                        float *m0 = tmet + slot * stride, *m1 = tmet + p.tstates + slot * stride;
                        if (have && sub == 0) m0[0] = 0.0f;
                        wsync();
                        const uint32_t *e = ent0;
                        for (int dd = 0; dd < l; ++dd) {
                            const int n1 = 1 << lgp[dd + 1];
                            if (have) {
                                const float v = src[dd * d + s];
                                const float yv = off[dd * d + s] ? -v : v;
                                const bool hd = yv < 0.0f;  // HD = Y < 0 (:270)
                                const float ay = fabsf(yv);
                                for (int S1 = sub; S1 < n1; S1 += G) {
                                    const uint32_t w = e[S1], a = w & 0xFFFFu, b = w >> 16;
                                    float x = m0[a & kTrellisState];
                                    if (((a & kTrellisZ) != 0u) != hd) x = x + ay;
                                    if (b & kTrellisValid) {
                                        float xb = m0[b & kTrellisState];
                                        if (((b & kTrellisZ) != 0u) != hd) xb = xb + ay;
                                        x = xb < x ? xb : x;
                                    }
                                    m1[S1] = x;
                                }
                            }
                            wsync();
                            float *tt = m0;
                            m0 = m1;
                            m1 = tt;
                            e += n1;
                        }
                        if (have && sub == 0) Sof(q, j + 1)[s] = m0[1] - m0[0];  // (:292)
                        wsync();
                    }
                    continue;
                }
                // lanes per item: the coset split when items are fewer than lanes
                int lpi = 1;
                const int nfree = l - loc - 1;
                while (lpi * 2 * tot <= 64 && (lpi * 2) <= (1 << (nfree < 6 ? nfree : 6))) lpi *= 2;
                const int span = 64 / lpi * lpi;  // lanes used per round
                for (int base = 0; base < tot * lpi; base += span) {
                    const int g = base + lane;
                    const bool have = lane < span && g < tot * lpi;
                    const int it = g / lpi, sub = g % lpi;
                    float b0 = __int_as_float(0x7F800000), b1 = __int_as_float(0x7F800000);
                    int q = 0, s = 0;
                    if (have) {
                        q = (int)act[it / d];
                        s = it % d;
                        const float *src = Sof(q, j);
                        const uint8_t *off = Oof(q, j);
                        float ay[kPolarMaxTrellisKernel];  // enumerated layers: l <= 32
                        uint64_t hd = 0;
                        for (int jj = 0; jj < l; ++jj) {
                            const float v = src[jj * d + s];
                            const float yv = off[jj * d + s] ? -v : v;
                            if (yv < 0.0f) hd |= 1ull << jj;  // HD = Y < 0 (:276)
                            ay[jj] = fabsf(yv);
                        }
                        coset_min(kr, l, loc, ay, hd, (uint32_t)sub, (uint32_t)lpi, b0, b1);
                    }
                    for (int o = 1; o < lpi; o <<= 1) {  // min over the item's lanes (exact)
                        const float x0 = __shfl_xor(b0, o, 64), x1 = __shfl_xor(b1, o, 64);
                        b0 = x0 < b0 ? x0 : b0;
                        b1 = x1 < b1 ? x1 : b1;
                    }
                    if (have && sub == 0) Sof(q, j + 1)[s] = b1 - b0;  // (:292)
                }
                wsync();
            }
            if (yielded) break;
            const bool on = mine && ((active >> lane) & 1u);
            if (on) lv = Sof(lane, nl)[0];
            const uint64_t corr = (e & kPhaseCorr) ? p.dfcorr[phi] : 0ull;
            uint32_t dec = 0;
            if (e & kPhaseFrozen) {
                // ---- ContinuePathsFrozen (MixedKernelListDecoder.cpp:61-98)
                const int db = (int)((e >> 1) & 127u) - 1;
                if (on) {
                    dec = db >= 0 ? (uint32_t)((dm >> db) & 1ull) : 0u;
                    if ((dec != 0) ^ (lv < 0.0f)) R -= fabsf(lv);
                }
            } else {
                // ---- ContinuePathsUnfrozen (:100-185): candidate 2q + b in lane 2q + b
                const int q = lane >> 1, b = lane & 1;
                const float vq = __shfl(lv, q & 31), Rq = __shfl(R, q & 31);
                const bool valid = q < L && ((active >> q) & 1u);
                float sc = 0.0f;
                if (valid) sc = (b == (vq < 0.0f ? 1 : 0)) ? Rq : Rq - fabsf(vq);
                int rank = 0;  // std::greater<pair<float, unsigned>> (:125)
                for (uint64_t mm = __ballot(valid); mm; mm &= mm - 1) {
                    const int o = (int)__builtin_ctzll(mm);
                    const float so = rdlf_m(sc, o);
                    rank += (sc < so || (!(so < sc) && lane < o)) ? 1 : 0;
                }
                const int J = 2 * nact, keep = J < L ? J : L;
                const uint64_t sel = __ballot(valid && rank < keep);
                const uint32_t cont = mine ? (uint32_t)((sel >> (2 * lane)) & 3ull) : 0u;
                const uint32_t cont_any = (uint32_t)__ballot(cont != 0);
                const uint32_t clones = (uint32_t)__ballot(cont == 3u);
                for (uint32_t kill = active & ~cont_any; kill; kill &= kill - 1) st.push((uint32_t)__builtin_ctz(kill), lane);
                active &= cont_any;
                dec = cont == 2u ? 1u : (cont == 3u ? (lv < 0.0f ? 1u : 0u) : 0u);
                for (uint32_t cl = clones; cl; cl &= cl - 1) {
                    const int l = __builtin_ctz(cl);
                    const int l1 = (int)st.pop(lane);  // ClonePath: the whole path state
                    for (int i = lane; i < p.ssize; i += 64) S[(size_t)l1 * p.ssize + i] = S[(size_t)l * p.ssize + i];
                    for (int i = lane; i < p.csize; i += 64) C[(size_t)l1 * p.csize + i] = C[(size_t)l * p.csize + i];
                    for (int i = lane; i < p.osize; i += 64) O[(size_t)l1 * p.osize + i] = O[(size_t)l * p.osize + i];
                    for (int i = lane; i < (k >> 5); i += 64) rec[l1 * RW + i] = rec[l * RW + i];
                    const float Rl = rdlf_m(R, l), vl = rdlf_m(lv, l);
                    const uint64_t dml = rdlu64_m(dm, l);
                    const uint32_t rwl = rdlu_m(rw, l), decl = rdlu_m(dec, l);
                    if (lane == l1) {
                        R = Rl - fabsf(vl);
                        dm = dml;
                        rw = rwl;
                        dec = decl ^ 1u;
                        lv = vl;
                    }
                    active |= 1u << l1;
                }
                wsync();
            }
            const bool now = mine && ((active >> lane) & 1u);
            if (now) {
                C[(size_t)lane * p.csize + lastc + (phi % lastsz)] = (uint8_t)dec;
                if (dec) dm ^= corr;
            }
            if (!(e & kPhaseFrozen)) {
                if (now) rw |= dec << (k & 31);
                ++k;
                if ((k & 31) == 0) {
                    if (now) rec[lane * RW + (k >> 5) - 1] = rw;
                    rw = 0;
                }
                nact = list_act(active);
            } else {
                wsync();
            }
            // ---- IterativelyUpdateC (KernelListEngine.cpp:266-315): finished blocks are
            // multiplied by their kernel into the parent layer's inputs
            {
                int lam = nl, stride = 1;
                uint32_t ph2 = (uint32_t)phi;
                while (lam > 0 && (ph2 + 1) % (uint32_t)p.ksize[lam - 1] == 0) {
                    const int l = p.ksize[lam - 1];
                    const uint32_t psi = ph2 / (uint32_t)l;
                    const int next = stride * l;
                    const int phi0 = lam > 1 ? (int)(psi % (uint32_t)p.ksize[lam - 2]) * next : 0;
                    const uint64_t *kr = rows + kPolarMaxKernel * (lam - 1);
                    const int tot = nact * stride;
                    for (int it = lane; it < tot; it += 64) {
                        const int q = (int)act[it / stride], s = it % stride;
                        const uint8_t *x = Cof(q, lam);
                        uint8_t *yo = Cof(q, lam - 1) + phi0;
                        // (y_i) = (x_j) K: y_i = XOR over rows j with K[j][i] (LinAlg.cpp:685-709)
                        uint64_t yv = 0;
                        for (int jj = 0; jj < l; ++jj)
                            if (x[jj * stride + s] & 1u) yv ^= kr[jj];
                        for (int i = 0; i < l; ++i) yo[i * stride + s] = (uint8_t)((yv >> i) & 1ull);
                    }
                    wsync();
                    stride = next;
                    ph2 = psi;
                    --lam;
                }
            }
        }
        if (yielded) {  // suspended: outputs when it finishes in a later launch
            wsync();
            continue;
        }
        if ((k & 31) && mine && ((active >> lane) & 1u)) rec[lane * RW + (k >> 5)] = rw;
        wsync();
        // ---- final order (:249-267): active paths by (R, index), descending
        int rk = 0;
        const bool me = mine && ((active >> lane) & 1u);
        for (uint64_t mm = __ballot(me); mm; mm &= mm - 1) {
            const int o = (int)__builtin_ctzll(mm);
            const float ro = rdlf_m(R, o);
            rk += (R < ro || (!(ro < R) && lane < o)) ? 1 : 0;
        }
        for (int r = 0; r < nact; ++r) {
            const int q = (int)__builtin_ctzll(__ballot(me && rk == r));
            const uint8_t *cq = C + (size_t)q * p.csize;  // C_0: the unshortened codeword
            const uint32_t *rq = rec + q * RW;
            const size_t row = (size_t)cw * L + r;
            for (int kk = lane; kk < K; kk += 64) p.info[row * K + kk] = (uint8_t)((rq[kk >> 5] >> (kk & 31)) & 1u);
            if (p.cw)
                for (int i = lane; i < p.N; i += 64) p.cw[row * p.N + i] = cq[p.cwpos[i]];
            if (lane == 0) p.metric[row] = rdlf_m(R, q);
        }
        if (lane == 0) p.count[cw] = nact;
        if (budgeted && lane == 0) p.rstate[cw] = 2u;
        wsync();
    }
}

hipError_t launch_polar_mixed(const PolarMixedParams &p, int grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(polar_mixed_kernel, dim3(grid), dim3(64), lds, s, p);
    return hipGetLastError();
}

const void *polar_mixed_kernel_ptr() { return reinterpret_cast<const void *>(&polar_mixed_kernel); }

}  // namespace bchk
