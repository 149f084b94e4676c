// bchk_syndtab.h -- syndrome-indexed decoding table (coset leaders of weight <= t) for
// the algebraic decoder inside the Kaneko loop, n <= 63.
//
// Decoder::decode (src/Decoder.cpp:298-321) succeeds on a test word exactly when its
// syndrome equals the syndrome of an error pattern e of weight 1..t, and then flips e:
// Euclid / BM return the locator of that pattern, whose deg lambda distinct roots lie in
// GF(2^m)*; any other syndrome makes the locator fail (lambda(0) = 0, deg > t, or too few
// roots). e is unique (two such patterns would differ by a codeword of weight <= 2t < d).
// So the whole decoder is a map syndrome -> e on the correctable syndromes, and the
// heavy part of the search -- thousands of test patterns per codeword, ~17 % of them
// correctable -- looks e up instead of running Berlekamp-Massey + Chien.
//
// The map commutes with cyclic shifts: shifting e by s multiplies S_j by alpha^(j s). A
// syndrome is normalised before lookup: with q* the first odd index j coprime to n whose
// S_j is nonzero, the shift s with alpha^(j s) S_j = 1 is applied to all syndromes; S_j
// (= 1) and the zero syndromes before it leave the key. The key is (region k = ordinal of
// q*, packed remaining syndromes); syndromes whose coprime entries are all zero form the
// last region, keyed by the raw remaining syndromes (s = 0). The table stores, per key,
// the error mask of the normalised pattern; the caller rotates it back by s. For
// BCH(63,30,13) that is ~1.2 M keys (one per shift orbit of the 75.6 M patterns), held in
// an open-addressed table of 64-B buckets (4 slots of {key, mask}), 64 MiB: one bucket
// load per lookup in the common case, resident in the 256 MB Infinity Cache while the
// search kernels run. Built once per (m, t) on the host, uploaded once per device.
//
// tests/test_filter.py checks every lookup against the oracle's Decoder::decode (the small
// codes exhaustively); tests/test_gpu_parity.py runs every path with and without it.
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

namespace bchk {

constexpr int kTabMaxBits = 30;  // m * (t - 1) <= 30: region index fits 30 bits
constexpr int kTabSlots = 4;     // slots per 64-B bucket

// Device view: buckets of kTabSlots slots {key (0 = empty), error mask}.
struct SyndTable {
    const uint64_t *slots;  // [nbuckets][kTabSlots][2], null = no table (BM + Chien)
    uint32_t bbits;         // log2(nbuckets)
    uint32_t max_probe;     // longest probe sequence of any key, in buckets (from the build)
};

__host__ __device__ constexpr int f_gcd(int a, int b) { return b ? f_gcd(b, a % b) : a; }
__host__ __device__ constexpr int f_inv(int j, int n) {  // j^-1 mod n (gcd(j, n) = 1)
    int r = 1;
    while ((j * r) % n != 1) ++r;
    return r;
}
__host__ __device__ constexpr bool f_coprime(int q, int n) { return f_gcd(2 * q + 1, n) == 1; }

inline bool syndtab_feasible(int m, int t) {
    return m <= 6 && t >= 1 && m * (t - 1) <= kTabMaxBits;  // masks are one u64 (n <= 63)
}

// Per-(n, TMAX) constants, evaluated at compile time: coprimality of j = 2q + 1 and its
// inverse mod n.
template <int N, int TMAX>
struct TabConsts {
    bool cop[TMAX];
    int inv[TMAX];
    __host__ __device__ constexpr TabConsts() : cop(), inv() {
        for (int q = 0; q < TMAX; ++q) {
            cop[q] = f_coprime(q, N);
            inv[q] = cop[q] ? f_inv(2 * q + 1, N) : 0;
        }
    }
};

struct SyndKey {
    uint64_t key;  // (region << 32 | packed syndromes) + 1, never 0
    int s;         // normalising shift
};

// Normalised key of packed odd syndromes Sw (byte q of word q/4 is S_(2q+1)), runtime
// t <= TMAX. lg: log table with lg[0] = 2n - 1; ex: exp table over [0, 2n) with
// ex[2n - 1] = 0 (bchk_device.h TableDesc). Branch-free; identical on host and device.
template <int M, int TMAX>
__host__ __device__ __forceinline__ SyndKey synd_key(const uint32_t *Sw, int t,
                                                     const uint16_t *lg, const uint8_t *ex) {
    constexpr int N = (1 << M) - 1;
    constexpr TabConsts<N, TMAX> C{};
    uint32_t S[TMAX];
    int ls[TMAX];
#pragma unroll
    for (int q = 0; q < TMAX; ++q) {
        S[q] = q < t ? (Sw[q >> 2] >> (8 * (q & 3))) & 0xFFu : 0u;
        ls[q] = lg[S[q]];
    }
    // region k (ordinal of the first nonzero coprime syndrome) and the shift s
    int k = 0, s = 0;
    bool found = false;
#pragma unroll
    for (int q = 0; q < TMAX; ++q) {
        if (!C.cop[q]) continue;
        const bool nz = S[q] != 0u;
        const int sq = ((N - ls[q]) * C.inv[q]) % N;  // used only when nz
        s = (nz && !found) ? sq : s;
        k += (!nz && !found && q < t) ? 1 : 0;
        found = found || nz;
    }
    // remaining syndromes times alpha^(j s): the exponent ls + (j s mod n) is < 2n - 1
    // when S_j != 0 and >= 2n - 1 (clamped to the zero entry) when S_j = 0
    const int d2 = (2 * s >= N) ? 2 * s - N : 2 * s;  // 2 s mod n
    int r = s;                                         // j s mod n for j = 1, 3, 5, ...
    uint64_t idx = 0;
    int ord = 0;
#pragma unroll
    for (int q = 0; q < TMAX; ++q) {
        const bool incl = q < t && (!C.cop[q] || ord > k);
        ord += C.cop[q] ? 1 : 0;
        int e = ls[q] + r;
        e = e < 2 * N - 1 ? e : 2 * N - 1;
        const uint64_t v = ex[e];
        idx = incl ? ((idx << M) | v) : idx;
        r += d2;
        r = r >= N ? r - N : r;
    }
    SyndKey out;
    out.key = (((uint64_t)k << 32) | idx) + 1ull;
    out.s = s;
    return out;
}

__host__ __device__ __forceinline__ uint32_t tab_hash(uint64_t key, uint32_t bbits) {
    return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - bbits));
}

// rotate an n-bit mask (n <= 63) right by s in [0, n): position p -> p - s (mod n)
template <int N>
__host__ __device__ __forceinline__ uint64_t rotr_n(uint64_t v, int s) {
    constexpr uint64_t FULL = (1ull << N) - 1ull;
    return s ? (((v >> s) | (v << (N - s))) & FULL) : v;
}

// Decoder::decode of one test word from its odd syndromes, by table lookup: true and E =
// the flipped positions iff the syndrome is correctable. Probes at most T.max_probe
// buckets (linear probing: no key sits further from its home bucket).
template <int M, int TMAX>
__host__ __device__ __forceinline__ bool tab_decode(const SyndTable &T, const uint32_t *Sw, int t,
                                                    const uint16_t *lg, const uint8_t *ex,
                                                    uint64_t &E) {
    constexpr int N = (1 << M) - 1;
    const SyndKey K = synd_key<M, TMAX>(Sw, t, lg, ex);
    const uint32_t bm = (1u << T.bbits) - 1u;
    uint32_t b = tab_hash(K.key, T.bbits);
    uint64_t mask = 0;
    bool hit = false;
    for (uint32_t p = 0; p < T.max_probe; ++p) {
        const uint64_t *bk = T.slots + (size_t)b * (2 * kTabSlots);
        bool open = false;
#pragma unroll
        for (int j = 0; j < kTabSlots; ++j) {
            const uint64_t k = bk[2 * j], v = bk[2 * j + 1];
            mask = (k == K.key) ? v : mask;
            hit = hit || k == K.key;
            open = open || k == 0ull;
        }
        if (hit || open) break;
        b = (b + 1u) & bm;
    }
    E = hit ? rotr_n<N>(mask, K.s) : 0ull;
    return hit;
}

}  // namespace bchk
