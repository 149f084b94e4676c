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
};

// Chien map (m <= 6): planes pl[b] ^= T[j][lo][b] ^ T[j][hi][b], value = lo + 8 hi.
template <int M>
__device__ __forceinline__ void chien_add(const uint64_t *__restrict__ chien, int j, uint32_t lo,
                                          uint32_t hi, uint64_t (&pl)[M]) {
    const uint64_t *tl = chien + (size_t)j * (2 * M * 8);
#pragma unroll
    for (int b = 0; b < M; ++b) {
        uint64_t v = tl[b * 8 + lo];
        if constexpr (M > 3) v ^= tl[(M + b) * 8 + hi];
        pl[b] ^= v;
    }
}

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
// v from lane ^ J, without the LDS crossbar: DPP quad permutes (J = 1, 2), row rotates
// (J = 4: by 12 or 4 as bit 2 of the lane says; J = 8: by 8), and the gfx950 row/half swaps
// v_permlane16_swap / v_permlane32_swap (J = 16, 32).
template <int J>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v, int lane) {
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
    } else if constexpr (J == 4) {
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x12C, 0xF, 0xF, false);
        return (lane & 4) ? dn : up;  // row_ror:4 reads lane - 4, row_ror:12 lane + 4
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
template <int J>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t v, int lane) {
    return ((uint64_t)lane_xor<J>((uint32_t)(v >> 32), lane) << 32) | lane_xor<J>((uint32_t)v, lane);
}

// v of lane - 1 (DPP wave_shr:1); lane 0 gets `fill`
__device__ __forceinline__ int wave_shr1(int v, int fill) {
    return __builtin_amdgcn_update_dpp(fill, v, 0x138, 0xF, 0xF, false);
}

// XOR over the wave
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
    const int lane = (int)__lane_id();
    v ^= lane_xor<32>(v, lane);
    v ^= lane_xor<16>(v, lane);
    v ^= lane_xor<8>(v, lane);
    v ^= lane_xor<4>(v, lane);
    v ^= lane_xor<2>(v, lane);
    v ^= lane_xor<1>(v, lane);
    return v;
}

// f64 sum over the wave by recursive doubling (each lane's rounding order differs: callers
// that branch on it take one lane's value)
__device__ __forceinline__ double wave_sum_f64(double v) {
    const int lane = (int)__lane_id();
    uint64_t b = (uint64_t)__double_as_longlong(v);
    b = (uint64_t)__double_as_longlong(__longlong_as_double((long long)b) +
                                       __longlong_as_double((long long)lane_xor64<32>(b, lane)));
    b = (uint64_t)__double_as_longlong(__longlong_as_double((long long)b) +
                                       __longlong_as_double((long long)lane_xor64<16>(b, lane)));
    b = (uint64_t)__double_as_longlong(__longlong_as_double((long long)b) +
                                       __longlong_as_double((long long)lane_xor64<8>(b, lane)));
    b = (uint64_t)__double_as_longlong(__longlong_as_double((long long)b) +
                                       __longlong_as_double((long long)lane_xor64<4>(b, lane)));
    b = (uint64_t)__double_as_longlong(__longlong_as_double((long long)b) +
                                       __longlong_as_double((long long)lane_xor64<2>(b, lane)));
    b = (uint64_t)__double_as_longlong(__longlong_as_double((long long)b) +
                                       __longlong_as_double((long long)lane_xor64<1>(b, lane)));
    return __longlong_as_double((long long)b);
}

__device__ __forceinline__ int xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return (int)(v & 7u);
}

// alpha^(la + lb) with log(0) = ZL = 2n-1 (la, lb in [0, n) or ZL). m <= 6: the sum is
// clamped to ZL so the exp table has 2n entries (exp[2n-1] = 0) -- at most 32 dwords for
// n <= 63, one per LDS bank, so byte lookups from 32 lanes never conflict. m >= 7: the table
// has 4n entries, zero from 2n-1 on (bchk_host.cpp make_tables), so no clamp: one add per
// product, in the decoders' innermost loops.
template <int M>
__device__ __forceinline__ uint32_t gf_exp2(const uint8_t *ex, int la, int lb) {
    constexpr int ZL = 2 * ((1 << M) - 1) - 1;
    const int s = la + lb;
    if constexpr (M >= 7) return ex[s];
    else return ex[s < ZL ? s : ZL];
}

// GF(2^m) table views for the per-lane decoders (bm_locator, split_test, alg_decode_lanes).
// A view hands out log "handles" and forms products from two of them; the arithmetic the
// decoders need on logs (division, doubling, the log(0) sentinel) goes through it.
//   GfPlain: the packed tables (exp u8 with 4n entries for m >= 7, log u16): handle = log.
//   GfRep (m >= 7, bchk_kernels.hip's cooperative kernel): the same tables replicated 16
//     times with one 4-B entry per replica, entry e of replica r at byte 64 e + 4 r, lanes
//     reading replica lane & 15 -- a 32-lane LDS group then touches each bank at most twice
//     (lanes l and l + 16), against ~3.5 distinct dwords per bank for random byte lookups
//     into the packed table (the cooperative kernel's LDS array was 88 % busy, half of it
//     in bank conflicts, r05 PMC). handle = 64 log + 4 r, so a product is one
//     v_add3 (a + b - 4 r) and one ds_read_b32, as before one add and one ds_read_u8.
//   GfMul (m >= 7, the cooperative kernel's decoders, round 6): the whole product table
//     [2^m][2^m] (64 KiB at m = 8) and the inverses in LDS; handle = the element itself, so
//     lg() is free and a product is one lookup. The decoders' log lookups go away: Berlekamp-
//     Massey re-logs C at every step (169 of its ~520 lookups at t = 15), the split test
//     logs every coefficient it squares or reduces by (~120 of ~1 050).
// Besides the products: val(h) = the element of handle h; pdiv(b) / div_by(a, pdiv(b)) =
// a / b with the divisor's part computed once (a log for the log views, its inverse for GfMul).
template <int M>
struct GfPlain {
    static constexpr int N = Geo<M>::N, ZL = Geo<M>::ZL;
    const uint8_t *ex;
    const uint16_t *lg_;
    __device__ __forceinline__ int lg(uint32_t g) const { return lg_[g]; }
    __device__ __forceinline__ uint32_t mul(int a, int b) const { return gf_exp2<M>(ex, a, b); }
    __device__ __forceinline__ uint32_t val(int h) const { return gf_exp2<M>(ex, h, 0); }
    __device__ __forceinline__ int pdiv(int b) const { return b; }
    __device__ __forceinline__ int div_by(int a, int pb) const { return div(a, pb); }
    __device__ __forceinline__ int zl() const { return ZL; }
    __device__ __forceinline__ int one() const { return 0; }
    __device__ __forceinline__ bool is_zl(int h) const { return h == ZL; }
    // log(x / y) for x, y != 0
    __device__ __forceinline__ int div(int a, int b) const { const int d = a - b; return d < 0 ? d + N : d; }
    // log(x^2) for x != 0
    __device__ __forceinline__ int dbl(int h) const { const int s2 = 2 * h; return s2 >= N ? s2 - N : s2; }
    __device__ __forceinline__ int plain(int h) const { return h; }  // the packed table's log
};
constexpr int kGfRepStride = 64;   // bytes per entry (16 replicas x 4 B)
template <int M>
constexpr int gf_rep_exp_entries() { return 4 * Geo<M>::N; }  // the 4n-entry exp table (m >= 7)
template <int M>
constexpr int gf_rep_bytes() { return (gf_rep_exp_entries<M>() + (1 << M)) * kGfRepStride; }
template <int M>
struct GfRep {
    static constexpr int N = Geo<M>::N, ZL = Geo<M>::ZL, S = kGfRepStride;
    const uint8_t *rep;  // LDS: exp entries 0 .. 4n-1, then log entries 0 .. 2^m - 1
    int lo;              // 4 (lane & 15)
    __device__ __forceinline__ int lg(uint32_t g) const {
        return *reinterpret_cast<const int *>(rep + (gf_rep_exp_entries<M>() + (int)g) * S + lo);
    }
    __device__ __forceinline__ uint32_t mul(int a, int b) const {
        return *reinterpret_cast<const uint32_t *>(rep + (a + b - lo));
    }
    __device__ __forceinline__ uint32_t val(int h) const { return mul(h, one()); }
    __device__ __forceinline__ int pdiv(int b) const { return b; }
    __device__ __forceinline__ int div_by(int a, int pb) const { return div(a, pb); }
    __device__ __forceinline__ int zl() const { return ZL * S + lo; }
    __device__ __forceinline__ int one() const { return lo; }
    __device__ __forceinline__ bool is_zl(int h) const { return h == ZL * S + lo; }
    __device__ __forceinline__ int div(int a, int b) const {
        const int d = a - b;
        return (d < 0 ? d + N * S : d) + lo;
    }
    __device__ __forceinline__ int dbl(int h) const {
        const int s2 = 2 * h - lo;
        return s2 >= N * S + lo ? s2 - N * S : s2;
    }
    // any lane's handle (64 log + 4 r, 4 r < 64): the log alone
    __device__ __forceinline__ int plain(int h) const { return h / S; }
};
template <int M>
constexpr int gf_mul_bytes() { return (1 << (2 * M)) + (1 << M); }  // products, then inverses
template <int M>
struct GfMul {
    const uint8_t *mt;    // LDS: mt[a 2^m + b] = a b, then iv[a] = 1 / a (iv[0] = 0)
    const uint16_t *lg_;  // the packed log table (plain logs for the Chien scan)
    __device__ __forceinline__ int lg(uint32_t g) const { return (int)g; }
    __device__ __forceinline__ uint32_t mul(int a, int b) const { return mt[(a << M) | b]; }
    __device__ __forceinline__ uint32_t val(int h) const { return (uint32_t)h; }
    __device__ __forceinline__ int zl() const { return 0; }
    __device__ __forceinline__ int one() const { return 1; }
    __device__ __forceinline__ bool is_zl(int h) const { return h == 0; }
    __device__ __forceinline__ int pdiv(int b) const { return mt[(1 << (2 * M)) + b]; }
    __device__ __forceinline__ int div_by(int a, int pb) const { return mt[(a << M) | pb]; }
    __device__ __forceinline__ int div(int a, int b) const { return div_by(a, pdiv(b)); }
    __device__ __forceinline__ int dbl(int h) const { return mt[(h << M) | h]; }  // h^2
    __device__ __forceinline__ int plain(int h) const { return lg_[h]; }
};
// fills the replicated tables from the packed ones (a whole workgroup, before a barrier)
template <int M>
__device__ __forceinline__ void gf_rep_fill(uint8_t *rep, const uint8_t *ex, const uint16_t *lg) {
    constexpr int NE = gf_rep_exp_entries<M>(), NL = 1 << M;
    for (int i = threadIdx.x; i < (NE + NL) * 16; i += blockDim.x) {
        const int e = i >> 4, r = i & 15;
        const uint32_t v = e < NE ? (uint32_t)ex[e] : (uint32_t)(lg[e - NE] * kGfRepStride + 4 * r);
        *reinterpret_cast<uint32_t *>(rep + i * 4) = v;
    }
}

template <int NW>
__device__ __forceinline__ void mask_set(Mask<NW> &m, int p) {
#pragma unroll
    for (int s = 0; s < NW; ++s)  // branch-free: a guarded store becomes a runtime index
        m.w[s] |= (uint64_t)((p >> 6) == s) << (p & 63);
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
// Binary Berlekamp-Massey over the table GF(2^m): connection polynomial C (TMAX + 1
// coefficients, C_0 = 1) and register length L of the syndromes S_1 .. S_2t. The update
// C <- C + (d / b) x B (b: the discrepancy of the last length change) takes one product per
// coefficient; the inversionless form (gamma C + d x B, two products) gives the same C up to
// a nonzero scalar at every step (by induction: its C, B and gamma are this form's times
// the same running product of discrepancies), so the same L, degree and roots.
template <int M, int TMAX, class GF>
__device__ __forceinline__ void bm_locator_g(const GF &gf, const uint32_t *Sw, int t, uint32_t (&C)[TMAX + 1],
                                             int &Lout) {
    int lS[2 * TMAX];  // lS[j-1] = log S_j
#pragma unroll
    for (int j = 0; j < TMAX; ++j) lS[2 * j] = gf.lg((Sw[j >> 2] >> (8 * (j & 3))) & 0xFFu);
#pragma unroll
    for (int e = 2; e <= 2 * TMAX - 1; e += 2) {  // S_{2i} = S_i^2
        const int h = lS[e / 2 - 1];
        lS[e - 1] = gf.is_zl(h) ? h : gf.dbl(h);
    }
    // binary Berlekamp-Massey over S_1, S_3, ... (even steps vanish)
    int lB[TMAX + 1];
#pragma unroll
    for (int i = 0; i <= TMAX; ++i) { C[i] = i ? 0u : 1u; lB[i] = i ? gf.zl() : gf.one(); }
    int lb = gf.one(), L = 0;
#pragma unroll
    for (int k = 0; k < TMAX; ++k) {
        if (k < t) {
            const int r = 2 * k;
            int lC[TMAX + 1];
            // C_i = 0 for i > 2k - 1 before step k (deg C <= L <= 2k - 1): their logs are the
            // zero sentinel without a table lookup (71 of the 240 lookups at t = TMAX = 15)
#pragma unroll
            for (int i = 0; i <= TMAX; ++i) lC[i] = (i <= 2 * k - 1 || i == 0) ? gf.lg(C[i]) : gf.zl();
            // before step k, deg C <= L <= 2k-1; after it, deg C <= 2k+1 (terms beyond are
            // zero whenever the final L <= t, the only case that can succeed)
            uint32_t d = 0;
#pragma unroll
            for (int i = 0; i <= (2 * k - 1 > 0 ? (2 * k - 1 < TMAX ? 2 * k - 1 : TMAX) : 0); ++i)
                d ^= gf.mul(lC[i], lS[r - i]);
            const int ld = gf.lg(d);
            const bool chg = (d != 0u) && (2 * L <= r);
            const int lf = d ? gf.div(ld, lb) : gf.zl();  // log(d / b); d = 0 leaves C as it is
#pragma unroll
            for (int i = TMAX; i >= 1; --i) {
                if (i > 2 * k + 1) { C[i] = 0u; continue; }
                C[i] ^= gf.mul(lf, lB[i - 1]);
            }
            // B <- C_old (length change) or x*B; then x*B for the skipped odd step
#pragma unroll
            for (int i = TMAX; i >= 0; --i) {
                const int shifted1 = i ? lB[i - 1] : gf.zl();
                const int next = chg ? lC[i] : shifted1;
                lB[i] = next;
            }
#pragma unroll
            for (int i = TMAX; i >= 1; --i) lB[i] = lB[i - 1];
            lB[0] = gf.zl();
            L = chg ? r + 1 - L : L;
            lb = chg ? ld : lb;
        }
    }
    Lout = L;
}
template <int M, int TMAX>
__device__ __forceinline__ void bm_locator(const uint8_t *__restrict__ ex,
                                           const uint16_t *__restrict__ lg, const uint32_t *Sw,
                                           int t, uint32_t (&C)[TMAX + 1], int &Lout) {
    bm_locator_g<M, TMAX>(GfPlain<M>{ex, lg}, Sw, t, C, Lout);
}

template <int M, int TMAX>
__device__ __forceinline__ bool alg_core(const uint8_t *__restrict__ ex,
                                         const uint16_t *__restrict__ lg,
                                         const uint64_t *__restrict__ chien,
                                         const uint32_t *Sw, int t,
                                         Mask<Geo<M>::NW> &E) {
    constexpr int N = Geo<M>::N, ZL = Geo<M>::ZL, NW = Geo<M>::NW;
    uint32_t C[TMAX + 1];
    int L;
    bm_locator<M, TMAX>(ex, lg, Sw, t, C, L);
    int deg = 0;
#pragma unroll
    for (int i = 1; i <= TMAX; ++i) deg = C[i] ? i : deg;
    bool ok = (L <= t) && (deg >= 1);

    if constexpr (M <= 6) {
        uint64_t pl[M];
#pragma unroll
        for (int b = 0; b < M; ++b) pl[b] = 0;
#pragma unroll
        for (int j = 0; j <= TMAX; ++j)
            if (j <= t) chien_add<M>(chien, j, C[j] & 7u, C[j] >> 3, pl);
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

// ---------------------------------------------------------------------------
// GF(2^m) on the VALU, m <= 6, no tables: an element is kept "spread", bit b at bit 3b.
// A 24-bit integer multiply of two spread elements is their carry-less product (every
// 3-bit slot sums at most m <= 6 terms, so slots never carry into each other; the slot's
// low bit is the XOR), then x^m = q(x) folds the high slots back. ~5 VALU per product.
template <int M>
struct Spread {
    static constexpr unsigned kPrim[9] = {0, 3, 7, 11, 19, 37, 67, 137, 285};  // main.cpp:14
    static constexpr uint32_t Q = kPrim[M] ^ (1u << M);
    static constexpr uint32_t mask_slots(int n) {
        uint32_t v = 0;
        for (int k = 0; k < n; ++k) v |= 1u << (3 * k);
        return v;
    }
    static constexpr uint32_t ELEM = mask_slots(M);
    static constexpr uint32_t PROD = mask_slots(2 * M - 1);
    static constexpr int deg_q() {
        int d = 0;
        for (int b = 0; b < M; ++b)
            if ((Q >> b) & 1u) d = b;
        return d;
    }
    // folds needed: after one fold the top slot is (m-2) + deg q
    static constexpr int FOLDS = (M - 2) + deg_q() < M ? 1 : 2;
};

template <int M>
__device__ __forceinline__ uint32_t sp_mul(uint32_t a, uint32_t b) {
    static_assert(M <= 6, "spread GF arithmetic needs m <= 6");
    uint32_t r = __umul24(a, b) & Spread<M>::PROD;
#pragma unroll
    for (int f = 0; f < Spread<M>::FOLDS; ++f) {
        const uint32_t h = r >> (3 * M);
        r &= Spread<M>::ELEM;
#pragma unroll
        for (int b = 0; b < M; ++b)
            if ((Spread<M>::Q >> b) & 1u) r ^= h << (3 * b);
    }
    return r;
}
// Reduction of a raw product, or of the XOR of several raw products (the slot parities
// add, the bits between slots are junk that never reaches a slot): one fold per product
// sum instead of one per product ("lazy" reduction).
template <int M>
__device__ __forceinline__ uint32_t sp_red(uint32_t r) {
    static_assert(M <= 6, "spread GF arithmetic needs m <= 6");
    if constexpr (Spread<M>::FOLDS == 1) {
        // x^(m+k) = x^k q(x): the high slots shifted by 3b for every term x^b of q; junk
        // bits move by multiples of 3 and stay between slots, so one final mask suffices
        const uint32_t h = r >> (3 * M);
        uint32_t f = r;
#pragma unroll
        for (int b = 0; b < M; ++b)
            if ((Spread<M>::Q >> b) & 1u) f ^= h << (3 * b);
        return f & Spread<M>::ELEM;
    } else {
        r &= Spread<M>::PROD;
#pragma unroll
        for (int f = 0; f < Spread<M>::FOLDS; ++f) {
            const uint32_t h = r >> (3 * M);
            r &= Spread<M>::ELEM;
#pragma unroll
            for (int b = 0; b < M; ++b)
                if ((Spread<M>::Q >> b) & 1u) r ^= h << (3 * b);
        }
        return r;
    }
}
// raw carry-less product of two reduced spread elements (no reduction)
__device__ __forceinline__ uint32_t sp_raw(uint32_t a, uint32_t b) { return __umul24(a, b); }

__device__ __forceinline__ uint32_t sp_from(uint32_t v) {  // 6-bit element -> spread
    v &= 0x3Fu;
    v = (v | (v << 8)) & 0x0000F00Fu;
    v = (v | (v << 4)) & 0x000C30C3u;
    v = (v | (v << 2)) & 0x00009249u;
    return v;
}
__device__ __forceinline__ uint32_t sp_to(uint32_t v) {  // spread -> 6-bit element
    v &= 0x00009249u;
    v = (v | (v >> 2)) & 0x000C30C3u;
    v = (v | (v >> 4)) & 0x0000F00Fu;
    v = (v | (v >> 8)) & 0x3Fu;
    return v;
}

// Same decision as alg_core (inversionless binary BM + Chien table), with BM on the VALU.
template <int M, int TMAX>
__device__ __forceinline__ bool alg_core_valu(const uint64_t *__restrict__ chien, const uint32_t *Sw,
                                              int t, Mask<1> &E) {
    constexpr int N = (1 << M) - 1;
    static_assert(N <= 63, "m <= 6");
    uint32_t S[2 * TMAX];  // S[j-1] = S_j, spread
#pragma unroll
    for (int j = 0; j < TMAX; ++j) S[2 * j] = sp_from((Sw[j >> 2] >> (8 * (j & 3))) & 0xFFu);
#pragma unroll
    for (int e = 2; e <= 2 * TMAX - 1; e += 2)
        S[e - 1] = sp_red<M>(sp_raw(S[e / 2 - 1], S[e / 2 - 1]));
    uint32_t C[TMAX + 1], B[TMAX + 1];
#pragma unroll
    for (int i = 0; i <= TMAX; ++i) { C[i] = i ? 0u : 1u; B[i] = i ? 0u : 1u; }
    uint32_t gam = 1;
    int L = 0;
#pragma unroll
    for (int k = 0; k < TMAX; ++k) {
        if (k < t) {
            const int r = 2 * k;
            uint32_t dr = 0;  // discrepancy: XOR of raw products, reduced once
#pragma unroll
            for (int i = 0; i <= (2 * k - 1 > 0 ? (2 * k - 1 < TMAX ? 2 * k - 1 : TMAX) : 0); ++i)
                dr ^= sp_raw(C[i], S[r - i]);
            const uint32_t d = sp_red<M>(dr);
            const bool chg = (d != 0u) && (2 * L <= r);
            uint32_t Cn[TMAX + 1];
#pragma unroll
            for (int i = 0; i <= TMAX; ++i) {
                if (i > 2 * k + 1) { Cn[i] = 0u; continue; }
                const uint32_t g = sp_raw(gam, C[i]);
                Cn[i] = sp_red<M>(i ? (g ^ sp_raw(d, B[i - 1])) : g);
            }
#pragma unroll
            for (int i = TMAX; i >= 0; --i) {
                const uint32_t sh = i ? B[i - 1] : 0u;
                B[i] = chg ? C[i] : sh;
            }
#pragma unroll
            for (int i = TMAX; i >= 1; --i) B[i] = B[i - 1];
            B[0] = 0u;
            L = chg ? r + 1 - L : L;
            gam = chg ? d : gam;
#pragma unroll
            for (int i = 0; i <= TMAX; ++i) C[i] = Cn[i];
        }
    }
    int deg = 0;
#pragma unroll
    for (int i = 1; i <= TMAX; ++i) deg = C[i] ? i : deg;
    bool ok = (L <= t) && (deg >= 1);
    uint64_t pl[M];
#pragma unroll
    for (int b = 0; b < M; ++b) pl[b] = 0;
#pragma unroll
    for (int j = 0; j <= TMAX; ++j) {
        if (j <= t) {
            // spread bits 0,3,6 (and 9,12,15) gathered into 3-bit indices by one multiply:
            // x * 21 = x + 4x + 16x puts spread bits 0/3/6 at 4/5/6 with no carries
            const uint32_t lo = (((C[j] & 0x49u) * 21u) >> 4) & 7u;
            const uint32_t hi = ((((C[j] >> 9) & 0x49u) * 21u) >> 4) & 7u;
            chien_add<M>(chien, j, lo, hi, pl);
        }
    }
    uint64_t any = 0;
#pragma unroll
    for (int b = 0; b < M; ++b) any |= pl[b];
    const uint64_t zero = ~any & ((1ull << N) - 1ull);
    ok = ok && (__popcll(zero) == deg);
    uint64_t e = __builtin_bitreverse64(zero) >> (63 - N);
    if ((e >> N) & 1ull) e = (e & ((1ull << N) - 1ull)) | 1ull;
    E.w[0] = e;
    return ok;
}

// ---------------------------------------------------------------------------
// Long codes (m >= 7): the root test without the Chien scan.
// Decoder::locatorsAndRoots (src/Decoder.cpp:279-296) accepts iff lambda has deg distinct
// roots among alpha^0 .. alpha^(n-1), i.e. iff lambda splits into distinct linear factors
// over GF(2^m)* -- iff lambda divides x^(2^m) - x = prod_a (x - a) (square-free; a = 0 is
// excluded because lambda(0) = C_0 != 0: the inversionless BM multiplies C_0 = 1 by nonzero
// discrepancies only). The scan costs n (t + 1) table lookups per test word (4080 at
// BCH(255,139,31)); x^(2^m) mod lambda costs about (m - 4) (t + 1)^2 (~1 100 there), and a
// failing word -- nearly every test pattern of a heavy codeword -- needs nothing more.
// Registers are indexed by compile-time constants only, so the arithmetic is modulo the
// reversed locator rho(x) = x^TMAX lambda(1/x) = sum_i C_i x^(TMAX - i), whose degree is
// TMAX whatever deg lambda is (leading coefficient C_0): rho = x^s lambda_rev with
// s = TMAX - deg, and lambda_rev (roots 1/X) divides x^(2^m) - x iff
// x^(2^m + s) == x^(1 + s) (mod rho). Checked against the root count on random and split
// locators for m = 7, 8 and every TMAX bucket (scripts/proto_m8_skip.c's companion
// experiment, and the GPU parity tests through the exhaustive/random decoder tables).
//
// x g mod rho-hat (rho / C_0, monic: x^TMAX = sum_j q_j x^j), g linear, lq = log q
template <int M, int TMAX, class GF>
__device__ __forceinline__ void mulx_mod(const GF &gf, const int (&lq)[TMAX], uint32_t (&g)[TMAX]) {
    const int lt = gf.lg(g[TMAX - 1]);
#pragma unroll
    for (int j = TMAX - 1; j >= 0; --j) g[j] = (j ? g[j - 1] : 0u) ^ gf.mul(lt, lq[j]);
}
// g^2 mod rho-hat: squares of the coefficients (Frobenius), then the top-down reduction of
// degrees 2 TMAX - 2 .. TMAX
template <int M, int TMAX, class GF>
__device__ __forceinline__ void sqr_mod(const GF &gf, const int (&lq)[TMAX], uint32_t (&g)[TMAX]) {
    uint32_t sq[2 * TMAX - 1];
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {
        const int l = gf.lg(g[j]);
        sq[2 * j] = gf.mul(l, l);
        if (j + 1 < TMAX) sq[2 * j + 1] = 0u;
    }
#pragma unroll
    for (int k = 2 * TMAX - 2; k >= TMAX; --k) {
        const int lk = gf.lg(sq[k]);
#pragma unroll
        for (int j = 0; j < TMAX; ++j) sq[k - TMAX + j] ^= gf.mul(lk, lq[j]);
    }
#pragma unroll
    for (int j = 0; j < TMAX; ++j) g[j] = sq[j];
}
constexpr int floor_pow2(int v) { return v < 2 ? 1 : 2 * floor_pow2(v / 2); }
constexpr int ilog2c(int v) { return v < 2 ? 0 : 1 + ilog2c(v / 2); }

// lambda = C (logs lc), deg >= 1, C_0 != 0: true iff lambda has deg distinct roots in GF(2^m)*
// (lanes with act = false give an unspecified answer)
template <int M, int TMAX, class GF>
__device__ __forceinline__ bool split_test(const GF &gf, const int (&lc)[TMAX + 1], int deg, bool act) {
    static_assert(TMAX >= 2, "split test needs TMAX >= 2");
    int lq[TMAX];
    const int pc0 = gf.pdiv(lc[0]);
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {  // q_j = C_(TMAX - j) / C_0
        const int v = lc[TMAX - j];
        lq[j] = gf.is_zl(v) ? v : gf.div_by(v, pc0);
    }
    // x^(2P) for the largest power of two P <= TMAX - 1 (so 2P >= TMAX): x^TMAX = q, then
    // 2P - TMAX multiplications by x; then squarings up to x^(2^m)
    constexpr int P = floor_pow2(TMAX - 1);
    constexpr int SQ = M - ilog2c(2 * P);
    static_assert(SQ >= 1, "2P < 2^m");
    uint32_t g[TMAX];
#pragma unroll
    for (int j = 0; j < TMAX; ++j) g[j] = gf.val(lq[j]);
#pragma unroll
    for (int e = TMAX; e < 2 * P; ++e) mulx_mod<M, TMAX>(gf, lq, g);
#pragma unroll
    for (int s = 0; s < SQ; ++s) sqr_mod<M, TMAX>(gf, lq, g);
    // times x^s, s = TMAX - deg (per lane; the wave runs the largest s of its active lanes)
    const int sh = (act && deg >= 2) ? TMAX - deg : 0;
    for (int st = 0; ballot(st < sh); ++st) {
        uint32_t h[TMAX];
#pragma unroll
        for (int j = 0; j < TMAX; ++j) h[j] = g[j];
        mulx_mod<M, TMAX>(gf, lq, h);
#pragma unroll
        for (int j = 0; j < TMAX; ++j) g[j] = st < sh ? h[j] : g[j];
    }
    bool eq = true;
#pragma unroll
    for (int j = 0; j < TMAX; ++j) eq = eq && (g[j] == (j == 1 + sh ? 1u : 0u));
    return deg == 1 || eq;  // a linear lambda with lambda(0) != 0 has its one root in GF*
}

// Decoder::decode for m >= 7, one test word per lane (wave-collective: every lane of the
// wave must call it): BM (bm_locator), the split test, and for the lanes that pass -- rare
// among test patterns -- the positions by a Chien scan spread over the wave (lane l tests
// positions l + 64 s, as alg_decode_wave), one scan per successful lane. Same decision and
// flipped positions as alg_core. Lanes with act = false report failure without the tests
// (the caller knows their outcome cannot matter).
template <int M, int TMAX, class GF>
__device__ __forceinline__ bool alg_decode_lanes_g(const GF &gf, const uint8_t *__restrict__ ex, const uint32_t *Sw,
                                                   int t, Mask<Geo<M>::NW> &E, bool act = true) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    const int lane = (int)__lane_id();
    uint32_t C[TMAX + 1];
    int L;
    bm_locator_g<M, TMAX>(gf, Sw, t, C, L);
    int deg = 0;
#pragma unroll
    for (int i = 1; i <= TMAX; ++i) deg = C[i] ? i : deg;
    int lc[TMAX + 1];
#pragma unroll
    for (int i = 0; i <= TMAX; ++i) lc[i] = gf.lg(C[i]);
    bool ok = act && (L <= t) && (deg >= 1);
#if defined(BCHK_SPLIT_CUT)  // experiment builds only (wrong results): Berlekamp-Massey alone
    ok = ok && lc[0] == 12345;
#else
    if (ballot(ok)) ok = split_test<M, TMAX>(gf, lc, deg, ok) && ok;
#endif
#pragma unroll
    for (int s = 0; s < NW; ++s) E.w[s] = 0;
    for (uint64_t sm = ballot(ok); sm; sm &= sm - 1) {
        const int src = (int)__builtin_ctzll(sm);
        const int dg = uni(__shfl(deg, src, 64));
        int kk[NW], ik[NW];
        uint32_t v[NW];
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int pos = lane + 64 * s;
            kk[s] = pos ? N - pos : 0;  // lambda(alpha^k) at k = (n - pos) mod n (:287)
            ik[s] = 0;
            v[s] = 0;
        }
#pragma unroll
        for (int i = 0; i <= TMAX; ++i) {
            if (i <= dg) {
                // the scan reads the packed exp table: plain logs (a lookup for GfMul, only
                // for the rare successful lanes)
                const int lti = gf.plain(__builtin_amdgcn_readlane(lc[i], src));
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
        if (lane == src && cnt != dg) ok = false;  // never: the split test said deg roots
    }
    return ok;
}

template <int M, int TMAX>
__device__ __forceinline__ bool alg_decode_lanes(const uint8_t *__restrict__ ex,
                                                 const uint16_t *__restrict__ lg, const uint32_t *Sw,
                                                 int t, Mask<Geo<M>::NW> &E, bool act = true) {
    return alg_decode_lanes_g<M, TMAX>(GfPlain<M>{ex, lg}, ex, Sw, t, E, act);
}

// The decoder a kernel uses: VALU BM for m <= 6 unless BCHK_GF_LDS is defined; m >= 7 the
// split test (wave-collective).
template <int M, int TMAX>
__device__ __forceinline__ bool alg_decode_word(const uint8_t *ex, const uint16_t *lg,
                                                const uint64_t *chien, const uint32_t *Sw, int t,
                                                Mask<Geo<M>::NW> &E, bool act = true) {
#ifndef BCHK_GF_LDS
    if constexpr (M <= 6) return alg_core_valu<M, TMAX>(chien, Sw, t, E);
    else
#endif
    if constexpr (M >= 7) return alg_decode_lanes<M, TMAX>(ex, lg, Sw, t, E, act);
    else return alg_core<M, TMAX>(ex, lg, chien, Sw, t, E);
}

// Decoder::decode of ONE test word by a whole wave (its syndromes Sw wave-uniform): the
// same decision and flipped positions as alg_core. Long codes (m >= 7) only, where one
// lane's decode costs ~(t + 1)(n + 4t) table lookups and the LDS pipe, shared by the CU's
// four SIMDs, is the bottleneck:
//   * Berlekamp-Massey with lane i holding coefficient i of C (and B): per step one log
//     lookup, one product per lane for the discrepancy -- summed by a DPP/permlane XOR --
//     and one product per lane for the update; the recurrence of bm_locator.
//   * the Chien search of Decoder::locatorsAndRoots (:279-296) spread over the lanes: lane
//     l tests the points of positions p = l + 64 s (root alpha^k flips position
//     (n - k) mod n, :287), the locator's logs broadcast from lanes 0..deg.
template <int M>
__device__ __forceinline__ uint32_t wave_xor_bits(uint32_t v) {
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < M; ++b) r |= (uint32_t)(__popcll(ballot((v >> b) & 1u)) & 1) << b;
    return r;
}

template <int M, int TMAX>
__device__ __forceinline__ bool alg_decode_wave(const uint8_t *__restrict__ ex,
                                                const uint16_t *__restrict__ lg,
                                                const uint32_t *Sw, int t, int lane,
                                                Mask<Geo<M>::NW> &E) {
    constexpr int N = Geo<M>::N, ZL = Geo<M>::ZL, NW = Geo<M>::NW, W = (TMAX + 3) / 4;
    static_assert(2 * TMAX <= 64, "one syndrome per lane");
    // lane q: log S_{q+1}; S_{2^e o} = S_o^(2^e) from the odd syndrome S_o (byte (o-1)/2)
    int lSq;
    {
        const int j1 = lane + 1;
        const int e = __builtin_ctz(j1);
        const int o = j1 >> e;
        const int jb = (o - 1) >> 1;  // odd-syndrome index
        uint32_t wv = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) wv = (w == (jb >> 2)) ? Sw[w] : wv;
        const uint32_t so = jb < TMAX ? (wv >> (8 * (jb & 3))) & 0xFFu : 0u;
        const int ls = lg[so];
        lSq = ls == ZL ? ZL : (int)(((uint32_t)ls << e) % (uint32_t)N);
    }
    uint32_t C = lane == 0 ? 1u : 0u;  // coefficient `lane` of C
    int lB = lane == 0 ? 0 : ZL;       // log of coefficient `lane` of B
    int lgam = 0, L = 0;
    // lane i holds log S_{r - i + 1} at step k (r = 2k): two lanes further up per step, the
    // two new syndromes entering at lanes 0 and 1. Lane moves by DPP wave shifts and the
    // discrepancy by a DPP/permlane XOR over the wave -- no LDS crossbar (ds_bpermute) on the
    // step's dependency chain.
    int lsv = lane == 0 ? (int)rdl((uint32_t)lSq, 0) : ZL;
    for (int k = 0; k < t; ++k) {
        const int r = 2 * k;
        const int lC = lg[C];
        const int top = 2 * k - 1 > 0 ? (2 * k - 1 < TMAX ? 2 * k - 1 : TMAX) : 0;
        const uint32_t term = lane <= top ? gf_exp2<M>(ex, lC, lsv) : 0u;
        const uint32_t d = uni((int)wave_xor(term));
        const int ld = lg[d];
        const bool chg = (d != 0u) && (2 * L <= r);
        const int lBm1 = wave_shr1(lB, ZL);  // B_{lane-1}
        const int lBm2 = wave_shr1(lBm1, ZL);
        const int lCm1 = wave_shr1(lC, ZL);
        int lf = ld - lgam;  // log(d / b), bm_locator's update with division
        lf = lf < 0 ? lf + N : lf;
        lf = d ? lf : ZL;
        const uint32_t Cn = lane ? (C ^ gf_exp2<M>(ex, lf, lBm1)) : C;
        C = (lane > 2 * k + 1 || lane > TMAX) ? 0u : Cn;
        // B <- C_old (length change) or x B, then x B for the vanishing odd step
        lB = lane == 0 ? ZL : (chg ? lCm1 : (lane >= 2 ? lBm2 : ZL));
        L = chg ? r + 1 - L : L;
        lgam = chg ? ld : lgam;
        if (k + 1 < t) {
            const int s2 = wave_shr1(wave_shr1(lsv, ZL), ZL);
            const int n0 = (int)rdl((uint32_t)lSq, (r + 2) & 63), n1 = (int)rdl((uint32_t)lSq, (r + 1) & 63);
            lsv = lane == 0 ? n0 : (lane == 1 ? n1 : s2);
        }
    }
    const uint64_t nz = ballot(C != 0u && lane <= TMAX) & ~1ull;
    const int deg = nz ? 63 - (int)__builtin_clzll(nz) : 0;
    const int ltl = lg[C];
    int kk[NW], ik[NW];
    uint32_t v[NW];
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        kk[s] = pos ? N - pos : 0;  // lambda(alpha^k) = sum_i C_i alpha^(i k)
        ik[s] = 0;
        v[s] = 0;
    }
    for (int i = 0; i <= deg; ++i) {  // wave-uniform trip count
        const int lti = __builtin_amdgcn_readlane(ltl, i);
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            v[s] ^= gf_exp2<M>(ex, lti, ik[s]);  // log(0) clamps to exp = 0
            ik[s] += kk[s];
            ik[s] = ik[s] >= N ? ik[s] - N : ik[s];
        }
    }
    int cnt = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        E.w[s] = ballot(lane + 64 * s < N && v[s] == 0u);
        cnt += __popcll(E.w[s]);
    }
    return (L <= t) && (deg >= 1) && (cnt == deg);
}

// v of lane - 1 within the lane's DPP row of 16 (row_shr:1); the row's lane 0 gets `fill`
__device__ __forceinline__ int row_shr1(int v, int fill) {
    return __builtin_amdgcn_update_dpp(fill, v, 0x111, 0xF, 0xF, false);
}

// Decoder::decode of FOUR test words by one wave (long codes, TMAX <= 15): DPP row r (lanes
// 16r .. 16r+15) solves word r's key equation with lane j holding coefficient j -- the
// recurrence of alg_decode_wave, its lane moves and discrepancy XOR kept inside the row --
// so one chain of dependent LDS lookups serves four words; then each word's Chien search by
// the whole wave, as alg_decode_wave. Sw4[r] = word r's packed odd syndromes (wave-uniform);
// Eout (LDS): [r][NW] word r's flipped positions, [4 NW + r] its success.
template <int M, int TMAX>
__device__ __forceinline__ void alg_decode_wave4(const uint8_t *__restrict__ ex,
                                                 const uint16_t *__restrict__ lg,
                                                 const uint32_t (&Sw4)[4][(TMAX + 3) / 4], int t, int lane,
                                                 uint64_t *Eout) {
    constexpr int N = Geo<M>::N, ZL = Geo<M>::ZL, NW = Geo<M>::NW, W = (TMAX + 3) / 4;
    static_assert(TMAX <= 15, "16 coefficients per DPP row");
    const int r = lane >> 4, j = lane & 15;
    // lane j of row r: log S_{j+1} (lo) and log S_{j+17} (hi) of word r
    int lSlo, lShi;
    {
        uint32_t wv[W];
#pragma unroll
        for (int w = 0; w < W; ++w)
            wv[w] = r == 0 ? Sw4[0][w] : (r == 1 ? Sw4[1][w] : (r == 2 ? Sw4[2][w] : Sw4[3][w]));
        auto lsq = [&](int q) {
            const int j1 = q + 1;
            const int e = __builtin_ctz(j1);
            const int o = j1 >> e;
            const int jb = (o - 1) >> 1;
            uint32_t x = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) x = (w == (jb >> 2)) ? wv[w] : x;
            const uint32_t so = jb < TMAX ? (x >> (8 * (jb & 3))) & 0xFFu : 0u;
            const int ls = lg[so];
            return ls == ZL ? ZL : (int)(((uint32_t)ls << e) % (uint32_t)N);
        };
        lSlo = lsq(j);
        lShi = lsq(j + 16);
    }
    const int rowbase = lane & 48;
    uint32_t C = j == 0 ? 1u : 0u;
    int lB = j == 0 ? 0 : ZL;
    int lgam = 0, L = 0;
    int lsv = j == 0 ? lSlo : ZL;  // lane j: log S_{2k - j + 1} at step k
    for (int k = 0; k < t; ++k) {
        const int r2 = 2 * k;
        const int lC = lg[C];
        const int top = 2 * k - 1 > 0 ? (2 * k - 1 < TMAX ? 2 * k - 1 : TMAX) : 0;
        uint32_t d = j <= top ? gf_exp2<M>(ex, lC, lsv) : 0u;
        d ^= lane_xor<1>(d, lane);
        d ^= lane_xor<2>(d, lane);
        d ^= lane_xor<4>(d, lane);
        d ^= lane_xor<8>(d, lane);
        const int ld = lg[d];
        const bool chg = (d != 0u) && (2 * L <= r2);
        const int lBm1 = row_shr1(lB, ZL);
        const int lBm2 = row_shr1(lBm1, ZL);
        const int lCm1 = row_shr1(lC, ZL);
        int lf = ld - lgam;
        lf = lf < 0 ? lf + N : lf;
        lf = d ? lf : ZL;
        const uint32_t Cn = j ? (C ^ gf_exp2<M>(ex, lf, lBm1)) : C;
        C = (j > 2 * k + 1 || j > TMAX) ? 0u : Cn;
        lB = j == 0 ? ZL : (chg ? lCm1 : (j >= 2 ? lBm2 : ZL));
        L = chg ? r2 + 1 - L : L;
        lgam = chg ? ld : lgam;
        if (k + 1 < t) {
            const int q0 = r2 + 2, q1 = r2 + 1;  // log S_{r2+3}, log S_{r2+2} of the row
            const int n0 = __shfl(q0 < 16 ? lSlo : lShi, rowbase + (q0 & 15), 64);
            const int n1 = __shfl(q1 < 16 ? lSlo : lShi, rowbase + (q1 & 15), 64);
            const int s2 = row_shr1(row_shr1(lsv, ZL), ZL);
            lsv = j == 0 ? n0 : (j == 1 ? n1 : s2);
        }
    }
    const uint64_t nz = ballot(C != 0u && j <= TMAX && j >= 1);
    const int ltl = lg[C];
#pragma unroll
    for (int w4 = 0; w4 < 4; ++w4) {
        const uint32_t mr = (uint32_t)(nz >> (16 * w4)) & 0xFFFFu;
        const int deg = mr ? 31 - __builtin_clz(mr) : 0;
        const int Lr = (int)rdl((uint32_t)L, 16 * w4);
        int kk[NW], ik[NW];
        uint32_t v[NW];
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int pos = lane + 64 * s;
            kk[s] = pos ? N - pos : 0;
            ik[s] = 0;
            v[s] = 0;
        }
        for (int i = 0; i <= deg; ++i) {
            const int lti = (int)rdl((uint32_t)ltl, 16 * w4 + i);
#pragma unroll
            for (int s = 0; s < NW; ++s) {
                v[s] ^= gf_exp2<M>(ex, lti, ik[s]);
                ik[s] += kk[s];
                ik[s] = ik[s] >= N ? ik[s] - N : ik[s];
            }
        }
        int cnt = 0;
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const uint64_t e = ballot(lane + 64 * s < N && v[s] == 0u);
            cnt += __popcll(e);
            if (lane == 0) Eout[w4 * NW + s] = e;
        }
        if (lane == 0) Eout[4 * NW + w4] = ((Lr <= t) && (deg >= 1) && (cnt == deg)) ? 1ull : 0ull;
    }
}

__device__ __forceinline__ void load_tables(uint8_t *dst, const uint8_t *src, uint32_t bytes) {
    const uint32_t n16 = bytes / 16;
    const uint4 *s = reinterpret_cast<const uint4 *>(src);
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x) d[i] = s[i];
}

}  // namespace bchk
