// bchk_core.h -- device-side building blocks shared by the gfx950 kernels: code geometry,
// wave helpers and the per-lane algebraic BCH decoder (Decoder::decode of the reference,
// src/Decoder.cpp:184-321). Included by .hip translation units only.
#pragma once
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdint.h>

#include "bchk_device.h"

namespace bchk {

template <int M>
struct Geo {
    static constexpr int N = (1 << M) - 1;
    static constexpr int NW = (N + 63) / 64;    // u64 words per position mask
    static constexpr int ZL = 2 * N - 1;        // log(0) sentinel
    static constexpr int EW = (M + 1) & ~1;     // Chien row u64 words (16-B aligned)
};

template <int NW>
struct Mask {
    uint64_t w[NW];
};

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int l) {
    return ((uint64_t)rdl((uint32_t)(v >> 32), l) << 32) | rdl((uint32_t)v, l);
}
__device__ __forceinline__ double rdlf(double v, int l) {
    return __longlong_as_double((long long)rdl64((uint64_t)__double_as_longlong(v), l));
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// LDS written by some lanes of a wave and read by other lanes of the same wave: DS
// instructions of one wave execute in order; the fences stop the compiler reordering.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}

__device__ __forceinline__ int xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return (int)(v & 7u);
}

// alpha^(la + lb) with log(0) = ZL = 2n-1: the sum is clamped to ZL so the exp table has
// 2n entries (exp[2n-1] = 0) -- at most 32 dwords for n <= 63, one per LDS bank, so
// byte lookups from 32 lanes never conflict.
template <int M>
__device__ __forceinline__ uint32_t gf_exp2(const uint8_t *ex, int la, int lb) {
    constexpr int ZL = 2 * ((1 << M) - 1) - 1;
    const int s = la + lb;
    return ex[s < ZL ? s : ZL];
}

template <int NW>
__device__ __forceinline__ void mask_set(Mask<NW> &m, int p) {
#pragma unroll
    for (int s = 0; s < NW; ++s)
        if (s == (p >> 6)) m.w[s] |= 1ull << (p & 63);
}
template <int NW>
__device__ __forceinline__ int mask_popc(const Mask<NW> &m) {
    int c = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) c += __popcll(m.w[s]);
    return c;
}

// ------------------------------------------------------------ algebraic decode
// Decoder::decode (src/Decoder.cpp:298-321) for one test word, from its packed odd
// syndromes Sw (byte j = S_{2j+1}). Success iff the syndrome is nonzero, the BM register
// length L <= t and the locator has deg C >= 1 distinct roots in GF(2^m)*; E = flipped
// positions ((n - k) mod n for each root alpha^k, :287).
template <int M, int TMAX>
__device__ __forceinline__ bool alg_core(const uint8_t *__restrict__ ex,
                                         const uint16_t *__restrict__ lg,
                                         const uint64_t *__restrict__ chien,
                                         const uint32_t *Sw, int t,
                                         Mask<Geo<M>::NW> &E) {
    constexpr int N = Geo<M>::N, ZL = Geo<M>::ZL, NW = Geo<M>::NW;
    int lS[2 * TMAX];  // lS[j-1] = log S_j
#pragma unroll
    for (int j = 0; j < TMAX; ++j) lS[2 * j] = lg[(Sw[j >> 2] >> (8 * (j & 3))) & 0xFFu];
#pragma unroll
    for (int e = 2; e <= 2 * TMAX - 1; e += 2) {  // S_{2i} = S_i^2
        const int h = lS[e / 2 - 1];
        int sq = 2 * h;
        sq = sq >= N ? sq - N : sq;
        lS[e - 1] = (h == ZL) ? ZL : sq;
    }
    // inversionless binary Berlekamp-Massey over S_1, S_3, ... (even steps vanish)
    uint32_t C[TMAX + 1];
    int lB[TMAX + 1];
#pragma unroll
    for (int i = 0; i <= TMAX; ++i) { C[i] = i ? 0u : 1u; lB[i] = i ? ZL : 0; }
    int lgam = 0, L = 0;
#pragma unroll
    for (int k = 0; k < TMAX; ++k) {
        if (k < t) {
            const int r = 2 * k;
            int lC[TMAX + 1];
#pragma unroll
            for (int i = 0; i <= TMAX; ++i) lC[i] = lg[C[i]];
            uint32_t d = 0;
#pragma unroll
            for (int i = 0; i <= (r < TMAX ? r : TMAX); ++i) d ^= gf_exp2<M>(ex, lC[i], lS[r - i]);
            const int ld = lg[d];
            const bool chg = (d != 0u) && (2 * L <= r);
#pragma unroll
            for (int i = TMAX; i >= 0; --i) {
                const uint32_t g = gf_exp2<M>(ex, lgam, lC[i]);
                C[i] = i ? (g ^ gf_exp2<M>(ex, ld, lB[i - 1])) : g;
            }
            // B <- C_old (length change) or x*B; then x*B for the skipped odd step
#pragma unroll
            for (int i = TMAX; i >= 0; --i) {
                const int shifted1 = i ? lB[i - 1] : ZL;
                const int next = chg ? lC[i] : shifted1;
                lB[i] = next;
            }
#pragma unroll
            for (int i = TMAX; i >= 1; --i) lB[i] = lB[i - 1];
            lB[0] = ZL;
            L = chg ? r + 1 - L : L;
            lgam = chg ? ld : lgam;
        }
    }
    int deg = 0;
#pragma unroll
    for (int i = 1; i <= TMAX; ++i) deg = C[i] ? i : deg;
    bool ok = (L <= t) && (deg >= 1);

    if constexpr (M <= 6) {
        constexpr int EW = Geo<M>::EW;
        uint64_t pl[EW];
#pragma unroll
        for (int w = 0; w < EW; ++w) pl[w] = 0;
#pragma unroll
        for (int j = 0; j <= TMAX; ++j) {
            if (j <= t) {
                const uint64_t *row = chien + (size_t)((j << M) + (int)C[j]) * EW;
#pragma unroll
                for (int w = 0; w < EW; ++w) pl[w] ^= row[w];
            }
        }
        uint64_t any = 0;
#pragma unroll
        for (int b = 0; b < M; ++b) any |= pl[b];
        const uint64_t zero = ~any & ((1ull << N) - 1ull);
        ok = ok && (__popcll(zero) == deg);
        uint64_t e = __builtin_bitreverse64(zero) >> (63 - N);  // root k -> bit n - k
        if ((e >> N) & 1ull) e = (e & ((1ull << N) - 1ull)) | 1ull;  // k = 0 -> position 0
        E.w[0] = e;
    } else {
        int lt[TMAX + 1];
#pragma unroll
        for (int i = 0; i <= TMAX; ++i) lt[i] = lg[C[i]];
#pragma unroll
        for (int s = 0; s < NW; ++s) E.w[s] = 0;
        int cnt = 0;
        for (int k = 0; k < N; ++k) {
            uint32_t v = 0;
#pragma unroll
            for (int i = 0; i <= TMAX; ++i) v ^= ex[lt[i]];
            if (v == 0u) {
                ++cnt;
                mask_set<NW>(E, k ? N - k : 0);
            }
#pragma unroll
            for (int i = 1; i <= TMAX; ++i) {
                int u = lt[i] + i;
                u = u >= N ? u - N : u;
                lt[i] = lt[i] == ZL ? ZL : u;
            }
        }
        ok = ok && (cnt == deg);
    }
    return ok;
}

__device__ __forceinline__ void load_tables(uint8_t *dst, const uint8_t *src, uint32_t bytes) {
    const uint32_t n16 = bytes / 16;
    const uint4 *s = reinterpret_cast<const uint4 *>(src);
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x) d[i] = s[i];
}

}  // namespace bchk
