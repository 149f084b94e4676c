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
// last region, keyed by the raw remaining syndromes (s = 0). Squaring all syndromes (the
// Frobenius map: positions times 2 mod n) also preserves correctability, so keys are
// canonical over that orbit too: ~0.2 M keys for BCH(63,30,13) (of 75.6 M patterns).
//
// Slots are 8 B, as a quotient table: the key (region, canonical fields) is mixed by an
// invertible multiplication mod 2^kbits; the top bbits of the product pick the home bucket
// and only the rest (the quotient) is stored, with the slot's distance from home (linear
// probing over 64-B buckets of 8 slots, at most 8 buckets) and all t position fields. The
// low 32 bits hold the tag (occupied bit | quotient | distance), so a slot test is one
// 32-bit compare; the fields sit above it (BCH(63,30,13): 20-bit tag + 36 field bits). At load
// <= 1/2 the table is 4 MiB at BCH(63,30,13) (the 16-B {key, positions} slots of rounds 1-2
// made it 8 MiB), one 64-B request per lookup in the common case. Built once per (m, t) on
// the host, uploaded once per device.
//
// tests/test_syndtab.py checks every lookup against the oracle's Decoder::decode (the small
// codes exhaustively); tests/test_gpu_parity.py runs every path with and without it.
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

namespace bchk {

constexpr int kTabMaxBits = 30;  // m * (t - 1) <= 30
constexpr int kTabSlots = 8;     // 8-B slots per 64-B bucket

// Device view: buckets of kTabSlots slots (layout above; 0 = empty).
struct SyndTable {
    const uint64_t *slots;  // [nbuckets][kTabSlots], null = no table (BM + Chien)
    uint32_t bbits;         // log2(nbuckets)
    uint32_t max_probe;     // longest probe sequence of any key, in buckets (from the build)
    uint32_t kbits;         // bits of a canonical key (tab_kbits)
    uint32_t tbits;         // bits of a slot's tag (tab_tbits)
};

__host__ __device__ constexpr int f_gcd(int a, int b) { return b ? f_gcd(b, a % b) : a; }
__host__ __device__ constexpr int f_inv(int j, int n) {  // j^-1 mod n (gcd(j, n) = 1)
    int r = 1;
    while ((j * r) % n != 1) ++r;
    return r;
}
__host__ __device__ constexpr bool f_coprime(int q, int n) { return f_gcd(2 * q + 1, n) == 1; }

constexpr int kTabDistBits = 3;  // slot distance from its home bucket: < 8 buckets
constexpr uint64_t kTabMult = 0x9E3779B97F4A7C15ull;  // odd: invertible mod 2^kbits

// bits of the canonical key: region above m (t - 1) field bits (synd_key)
__host__ __device__ __forceinline__ int tab_vbits(int m, int t) { return m * (t - 1); }
inline int tab_kbits(int m, int t) {
    const int n = (1 << m) - 1;
    int K = 0;  // coprime odd indices: the last region's ordinal
    for (int q = 0; q < t; ++q) K += f_coprime(q, n) ? 1 : 0;
    int rb = 0;
    while ((1 << rb) < K + 1) ++rb;
    return tab_vbits(m, t) + rb;
}
// a slot: t fields of m bits | tag = occupied bit | quotient (kbits - bbits) | distance (3)
inline int tab_tbits(int m, int t, int bbits) { return 1 + (tab_kbits(m, t) - bbits) + kTabDistBits; }
inline bool tab_fits(int m, int t, int bbits) {
    // < 32: tab_finish masks the tag with (1u << tbits) - 1u
    return tab_tbits(m, t, bbits) < 32 && tab_tbits(m, t, bbits) + m * t <= 64;
}
constexpr int kTabMaxBucketBits = 20;  // 64 MiB
inline bool syndtab_feasible(int m, int t) {  // n <= 63: one u64 mask; a layout within 64 MiB
    if (m > 6 || t < 1 || m * (t - 1) > kTabMaxBits) return false;
    const int kb = tab_kbits(m, t);
    return tab_fits(m, t, kb < kTabMaxBucketBits ? kb : kTabMaxBucketBits);
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
    uint64_t key;  // region << m (t - 1) | canonical packed log-syndromes
    int s;         // normalising shift
    int kf;        // Frobenius power of the canonical form
    int t;         // position fields in a table entry
};

// rotate an m-bit field left by k in [0, m) (= multiply by 2^k mod n for values < n; the
// all-ones value n, used as "zero element" / "no position", is fixed)
template <int M>
__host__ __device__ __forceinline__ int rotl_m(int v, int k) {
    constexpr int N = (1 << M) - 1;
    return ((v << k) | (v >> (M - k))) & N;
}

// Canonical key of packed odd syndromes Sw (byte q of word q/4 is S_(2q+1)), runtime
// t <= TMAX. lg: log table with lg[0] = 2n - 1 (bchk_device.h TableDesc). The key packs,
// for every odd index left in it, the log of the normalised syndrome (n for a zero one),
// m bits each. Squaring every syndrome (the Frobenius map, = the pattern's positions times
// 2 mod n) rotates each field left by one bit, so the least of the m rotations is a key
// shared by the whole (shift x Frobenius) orbit; kf records which rotation it was.
// Branch-free; identical on host and device.
template <int M, int TMAX>
__host__ __device__ __forceinline__ SyndKey synd_key(const uint32_t *Sw, int t,
                                                     const uint16_t *lg) {
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
    // log of alpha^(j s) S_j = ls + (j s mod n), reduced mod n; n marks S_j = 0
    const int d2 = (2 * s >= N) ? 2 * s - N : 2 * s;  // 2 s mod n
    int r = s;                                         // j s mod n for j = 1, 3, 5, ...
    uint64_t idx = 0;
    int ord = 0;
    uint64_t lo = 0;  // bit 0 of every field: the SWAR field-rotation masks
#pragma unroll
    for (int q = 0; q < TMAX; ++q) {
        const bool incl = q < t && (!C.cop[q] || ord > k);
        ord += C.cop[q] ? 1 : 0;
        int e = ls[q] + r;
        e = e >= N ? e - N : e;
        e = S[q] ? e : N;
        idx = incl ? ((idx << M) | (uint64_t)e) : idx;
        lo = incl ? ((lo << M) | 1ull) : lo;
        r += d2;
        r = r >= N ? r - N : r;
    }
    // least rotation over the m Frobenius conjugates (each field rotated by the same k)
    const uint64_t top = lo << (M - 1);       // bit m-1 of every field
    const uint64_t full = lo * (uint64_t)N;   // every field bit
    uint64_t best = idx, cur = idx;
    int kf = 0;
#pragma unroll
    for (int f = 1; f < M; ++f) {
        cur = (((cur << 1) & ~lo) | ((cur & top) >> (M - 1))) & full;
        kf = cur < best ? f : kf;
        best = cur < best ? cur : best;
    }
    SyndKey out;
    out.key = ((uint64_t)k << tab_vbits(M, t)) | best;
    out.s = s;
    out.kf = kf;
    out.t = t;
    return out;
}

// Home bucket and quotient of a key: h = key * kTabMult mod 2^kbits (a bijection), home =
// its top bbits, quotient = the rest.
struct TabHome {
    uint32_t b;     // home bucket
    uint32_t tag;   // the slot's tag at distance 0: 1 | quotient | 0
};
__host__ __device__ __forceinline__ TabHome tab_home(uint64_t key, const SyndTable &T) {
    const uint64_t h = (key * kTabMult) & ((1ull << T.kbits) - 1ull);
    const int qb = (int)T.kbits - (int)T.bbits;
    TabHome r;
    r.b = (uint32_t)(h >> qb);
    r.tag = (1u << (T.tbits - 1u)) | ((uint32_t)(h & ((1ull << qb) - 1ull)) << kTabDistBits);
    return r;
}

// Stored pattern: t position fields of m bits (unused fields all ones) of the canonical
// syndrome's leader P = 2^kf (e + s), ascending. Back to e: p = 2^-kf p' - s (mod n).
template <int M, int TMAX>
__host__ __device__ __forceinline__ uint64_t tab_unmap(uint64_t packed, int s, int kf, int t) {
    constexpr int N = (1 << M) - 1;
    uint64_t E = 0;
#pragma unroll
    for (int f = 0; f < TMAX; ++f) {
        const int pp = f < t ? (int)((packed >> (M * f)) & (uint64_t)N) : N;
        int p = rotl_m<M>(pp, kf ? M - kf : 0) - s;
        p = p < 0 ? p + N : p;
        E |= (pp != N) ? (1ull << p) : 0ull;
    }
    return E;
}

// One 64-B bucket: kTabSlots slots.
struct TabBucket {
    uint64_t k[kTabSlots];
};

__host__ __device__ __forceinline__ void tab_load(const SyndTable &T, uint32_t b, TabBucket &B) {
    const uint64_t *bk = T.slots + (size_t)b * kTabSlots;
#pragma unroll
    for (int j = 0; j < kTabSlots; ++j) B.k[j] = bk[j];
}

// Finish a lookup from its home bucket (already loaded): a slot matches when its bits above
// the fields are the key's tag at the bucket's distance from home; further buckets only
// when the home bucket is full without the key (no key sits more than T.max_probe - 1
// buckets past its home).
template <int M, int TMAX>
__host__ __device__ __forceinline__ bool tab_finish(const SyndTable &T, const SyndKey &K, const TabHome &H,
                                                    const TabBucket &B0, uint64_t &E) {
    const uint32_t tm = (1u << T.tbits) - 1u;
    uint64_t v = 0;
    bool hit = false, open = false;
#pragma unroll
    for (int j = 0; j < kTabSlots; ++j) {
        const uint32_t lo = (uint32_t)B0.k[j];
        const bool h = (lo & tm) == H.tag;
        v = h ? B0.k[j] : v;
        hit = hit || h;
        open = open || lo == 0u;
    }
    if (!hit && !open) {
        const uint32_t bm = (1u << T.bbits) - 1u;
        uint32_t b = H.b;
        for (uint32_t p = 1; p < T.max_probe; ++p) {
            b = (b + 1u) & bm;
            const uint32_t tag = H.tag | p;
            TabBucket B;
            tab_load(T, b, B);
#pragma unroll
            for (int j = 0; j < kTabSlots; ++j) {
                const uint32_t lo = (uint32_t)B.k[j];
                const bool h = (lo & tm) == tag;
                v = h ? B.k[j] : v;
                hit = hit || h;
                open = open || lo == 0u;
            }
            if (hit || open) break;
        }
    }
    E = hit ? tab_unmap<M, TMAX>(v >> T.tbits, K.s, K.kf, K.t) : 0ull;
    return hit;
}

// Decoder::decode of one test word from its odd syndromes, by table lookup: true and E =
// the flipped positions iff the syndrome is correctable.
template <int M, int TMAX>
__host__ __device__ __forceinline__ bool tab_decode(const SyndTable &T, const uint32_t *Sw, int t,
                                                    const uint16_t *lg, uint64_t &E) {
    const SyndKey K = synd_key<M, TMAX>(Sw, t, lg);
    const TabHome H = tab_home(K.key, T);
    TabBucket B;
    tab_load(T, H.b, B);
    return tab_finish<M, TMAX>(T, K, H, B, E);
}

}  // namespace bchk
