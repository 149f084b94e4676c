/* kernel_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker of csrc/kernel_search.hip).
 *
 * A literal C restatement of the reference's BCH polar-kernel construction and of the
 * column-permutation search's objective, used by tests/ to check the GPU search:
 *
 *   kor_make_ebch        root bchCoder.cpp:356-389  makeMatrix (nested extended-BCH kernel)
 *   kor_field_order      root bchCoder.cpp:478-496  swapColumns' column reordering
 *   kor_trellis_counts   out/external/TrellisKernelProcessor.cpp:7-67 (MinimumSpan),
 *                        :69-179 (trellis construction), :234-294 (GetLLRs with the
 *                        SUM_COUNT / CMP_COUNT counters of headers/external/misc.h:84-93),
 *                        every phase evaluated once with zero known inputs, as the search
 *                        loops do (root bchCoder.cpp:505-515, :645-647)
 *   kor_lu_perm          root bchCoder.cpp:766-785 randomInvertibleMatrix (L.U over GF(2)),
 *                        :608-626 the column map it induces
 *   kor_random_codes     the draws randomSwapColumns makes (:603, :768-775)
 *   kor_column_search    root bchCoder.cpp:541-699 randomSwapColumns: column map
 *                        j -> B j (:608-630), accept when Sum AND Cmp strictly improve (:651)
 *
 * The trellis is built and walked state by state exactly as the reference does (states
 * up to 2^MaxNumOfActiveBits), so the counts are the reference's by construction; the GPU
 * computes them in closed form and is compared with this.
 *
 * Parity: the active randomSwapColumns calls a SectionedTrellisKernelProcessor whose header
 * and source are absent from the reference; the objective restated here is
 * that of CTrellisKernelProcessor, the processor CMatrixBinaryKernel::GetProcessor(0)
 * returns (out/external/Kernel.cpp:276-281) and the one the earlier exhaustive swapColumns
 * (root bchCoder.cpp:413-475) used. The vendored library cannot be built here, so these
 * counts are parity unpinned; kor_trellis_counts' LLRs are checked against an independent
 * coset enumeration in tests/test_kernel_search.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const unsigned kPrim[16] = {3, 7, 11, 19, 37, 67, 137, 285, 529, 1033,
                                   2053, 4179, 8219, 17475, 32771, 69643}; /* src/main.cpp:14 */

typedef uint64_t Word;

/* ---- GF(2^m) power table (src/main.cpp:59-72): alog[i] = alpha^i */
static void gf_alog(int m, unsigned *alog) {
    const int n = (1 << m) - 1;
    unsigned v = 1;
    for (int i = 0; i < n; ++i) {
        alog[i] = v;
        v <<= 1;
        if (v >> m) v ^= kPrim[m - 1];
    }
}

/* minimal polynomial of alpha^i over GF(2), coefficients low degree first
 * (root bchCoder.cpp findMinimalPolynomial: product over the cyclotomic coset of i) */
static int minpoly(int m, const unsigned *alog, const int *lg, int i, unsigned char *out) {
    const int n = (1 << m) - 1;
    int coset[32], cs = 0, j = i % n;
    for (;;) {
        int seen = 0;
        for (int q = 0; q < cs; ++q) seen |= coset[q] == j;
        if (seen) break;
        coset[cs++] = j;
        j = (2 * j) % n;
    }
    unsigned poly[34] = {1};
    int deg = 0;
    for (int q = 0; q < cs; ++q) { /* poly *= (x + alpha^coset[q]) */
        unsigned nx[34] = {0};
        for (int k = 0; k <= deg; ++k) {
            if (poly[k]) nx[k] ^= alog[(lg[poly[k]] + coset[q]) % n];
            nx[k + 1] ^= poly[k];
        }
        ++deg;
        memcpy(poly, nx, sizeof poly);
    }
    for (int k = 0; k <= deg; ++k) out[k] = (unsigned char)(poly[k] & 1u);
    return deg + 1;
}

/* remainder of a(x) mod b(x) over GF(2) is zero? */
static int divides(const unsigned char *a, int na, const unsigned char *b, int nb) {
    unsigned char r[130];
    memcpy(r, a, (size_t)na);
    for (int d = na - 1; d >= nb - 1; --d)
        if (r[d])
            for (int k = 0; k < nb; ++k) r[d - (nb - 1) + k] ^= b[k];
    for (int k = 0; k < nb - 1 && k < na; ++k)
        if (r[k]) return 0;
    return 1;
}

/* root bchCoder.cpp:356-389: column 0 all ones, K[1][1] = 1, then for each new minimal
 * polynomial the generator g <- g * M_i is written to row deg(g_new) from column 1 and the
 * rows between the old and the new degree hold the previous g shifted by 1, 2, ... */
int kor_make_ebch(int power, uint8_t *K) {
    if (power < 2 || power > 6) return -1;
    const int len = (1 << power) - 1, N = len + 1;
    const int amount = (power != 2) ? ((1 << power) - 2) / 2 : 2;
    unsigned alog[64];
    int lg[64];
    gf_alog(power, alog);
    for (int i = 0; i < len; ++i) lg[alog[i]] = i;
    memset(K, 0, (size_t)N * N);
    for (int i = 0; i < N; ++i) K[i * N] = 1;
    K[len + 2] = 1; /* row 1, column 1 */
    unsigned char g[130] = {1}, poly[34], prod[130];
    int gOld = 1;
    for (int i = 2; i <= amount; ++i) {
        const int ps = minpoly(power, alog, lg, i, poly);
        if (gOld >= ps && divides(g, gOld, poly, ps)) continue; /* :372 */
        const int gNew = ps + gOld - 1;
        memset(prod, 0, sizeof prod);
        for (int a = 0; a < ps; ++a)
            if (poly[a])
                for (int b = 0; b < gOld; ++b) prod[a + b] ^= g[b];
        if (gNew >= N) return -2;
        for (int k = 0; k < gNew; ++k) K[gNew * N + k + 1] = prod[k]; /* :374, offset 1 (:125-139) */
        int count = 1;
        for (int j = gOld; j < gNew - 1; ++j, ++count) /* :376-381 */
            for (int k = count; k < count + gOld; ++k) K[(j + 1) * N + k + 1] = g[k - count];
        for (int j = 1; j <= gNew; ++j) g[j - 1] = K[gNew * N + j]; /* :382-384 */
        gOld = gNew;
    }
    return 0;
}

/* root bchCoder.cpp:481-496: columns 0..2 stay, column i >= 3 takes the old column j + 1
 * where fieldElements[j] == i (fieldElements = the power table alpha^j) */
int kor_field_order(int power, const uint8_t *K, uint8_t *out) {
    const int n = 1 << power;
    unsigned alog[64];
    gf_alog(power, alog);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= 2; ++j) out[i * n + j] = K[i * n + j];
    for (int i = 3; i < n; ++i) {
        int j = 2;
        for (; j < n - 1; ++j)
            if ((int)alog[j] == i) break;
        for (int k = 0; k < n; ++k) out[k * n + i] = K[k * n + j + 1];
    }
    return 0;
}

/* ---- MinimumSpan (TrellisKernelProcessor.cpp:7-67) */
static int minimum_span(unsigned K, unsigned N, Word *M, unsigned *start, unsigned *end) {
    for (unsigned c = 0; c < N; ++c) start[c] = end[c] = ~0u;
    unsigned C = 0;
    for (unsigned i = 0; i < K; ++i) {
        int found = 0;
        for (; C < N; ++C) {
            if (!((M[i] >> C) & 1)) {
                for (unsigned j = i + 1; j < K; ++j)
                    if ((M[j] >> C) & 1) {
                        M[i] ^= M[j];
                        found = 1;
                        break;
                    }
                if (found) {
                    start[C] = i;
                    break;
                }
            } else {
                start[C] = i;
                found = 1;
                break;
            }
        }
        if (!found) return -1; /* "Matrix is not full rank" */
        for (unsigned j = i + 1; j < K; ++j)
            if ((M[j] >> C) & 1ull) M[j] ^= M[i];
    }
    for (int i = (int)K - 1; i >= 0; --i)
        for (int j = (int)N - 1; j >= 0; --j)
            if ((M[i] >> j) & 1) {
                end[j] = (unsigned)i;
                for (int s = 0; s < i; ++s)
                    if ((M[s] >> j) & 1) M[s] ^= M[i];
                break;
            }
    return 0;
}

/* Trellis of phase `ph` (:85-158) walked by GetLLRs (:260-292) with zero known inputs
 * (offset 0, :246-247 / :258) for channel LLRs y; returns the LLR, adds the counters. */
static int phase_llr(const uint8_t *Kmat, unsigned l, unsigned ph, const float *y, uint64_t *sum,
                     uint64_t *cmp, double *llr) {
    const unsigned N = l + 1, K = l - ph;
    Word ext[64];
    unsigned start[65], end[65], active[64];
    for (unsigned j = ph; j < l; ++j) {
        Word r = 0;
        for (unsigned s = 0; s < l; ++s)
            if (Kmat[j * l + s]) r |= 1ull << s;
        ext[j - ph] = r;
    }
    ext[0] |= 1ull << l;
    Word gm[64];
    memcpy(gm, ext, sizeof(Word) * K);
    if (minimum_span(K, N, gm, start, end)) return -1;
    /* pCW0 / pCW1 hold the codeword prefix of each state; the construction runs once to get
     * each depth's edges, the metric pass follows it depth by depth */
    size_t cap = 1;
    {   /* the largest state count, to size the arrays */
        unsigned na = 0, mx = 0;
        unsigned tmp[64];
        for (unsigned j = 0; j <= l; ++j) {
            unsigned B = na;
            for (unsigned q = 0; q < na; ++q)
                if (tmp[q] == end[j]) { B = q; break; }
            if (start[j] != ~0u) tmp[na++] = start[j];
            if (na > mx) mx = na;
            if (end[j] != ~0u) {
                memmove(tmp + B, tmp + B + 1, sizeof(unsigned) * (na - B));
                --na;
            }
        }
        if (mx > 26) return -2;
        cap = (size_t)1 << (mx + 1);
    }
    Word *cw0 = calloc(cap, sizeof(Word)), *cw1 = calloc(cap, sizeof(Word));
    double *m0 = malloc(cap * sizeof(double)), *m1 = malloc(cap * sizeof(double));
    uint64_t *nxt = malloc(cap * 2 * sizeof(uint64_t));
    if (!cw0 || !cw1 || !m0 || !m1 || !nxt) {
        free(cw0); free(cw1); free(m0); free(m1); free(nxt);
        return -3;
    }
    unsigned na = 0;
    m0[0] = 0.0;
    cw0[0] = 0;
    for (unsigned j = 0; j < l; ++j) { /* GetLLRs walks depths 0..l-1 only */
        unsigned B = na;
        for (unsigned q = 0; q < na; ++q)
            if (active[q] == end[j]) { B = q; break; }
        const uint64_t emask = (end[j] == ~0u) ? ~0ull : ((1ull << B) - 1);
        const uint64_t ns = 1ull << na;
        if (start[j] == ~0u) { /* :112-123 */
            for (uint64_t S = 0; S < ns; ++S) {
                const Word bit = (cw0[S] >> j) & 1;
                const uint64_t nx = (S & emask) | ((S >> 1) & ~emask);
                cw1[nx] = cw0[S];
                nxt[2 * S + bit] = nx;
                nxt[2 * S + (1 - bit)] = ~0ull;
            }
        } else { /* :128-146 */
            for (uint64_t S = 0; S < ns; ++S) {
                uint64_t n0 = S, n1 = S ^ (1ull << na);
                n0 = (n0 & emask) | ((n0 >> 1) & ~emask);
                n1 = (n1 & emask) | ((n1 >> 1) & ~emask);
                const Word c1 = cw0[S] ^ gm[start[j]];
                cw1[n0] = cw0[S];
                cw1[n1] = c1;
                nxt[2 * S + ((cw0[S] >> j) & 1)] = n0;
                nxt[2 * S + ((c1 >> j) & 1)] = n1;
            }
            active[na++] = start[j];
        }
        { Word *t = cw0; cw0 = cw1; cw1 = t; }
        if (end[j] != ~0u) {
            memmove(active + B, active + B + 1, sizeof(unsigned) * (na - B));
            --na;
        }
        /* metric step (:263-290) on the edges just built */
        const uint64_t ns1 = 1ull << na;
        for (uint64_t S = 0; S < ns1; ++S) m1[S] = 1e300;
        const double Y = (double)y[j];
        const unsigned HD = Y < 0;
        for (uint64_t S = 0; S < ns; ++S)
            for (unsigned z = 0; z < 2; ++z) {
                const uint64_t S1 = nxt[2 * S + z];
                if (S1 == ~0ull) continue;
                double sc;
                if (z ^ HD) {
                    sc = m0[S] + (Y < 0 ? -Y : Y);
                    ++*sum;
                } else
                    sc = m0[S];
                ++*cmp;
                if (sc < m1[S1]) m1[S1] = sc;
            }
        { double *t = m0; m0 = m1; m1 = t; }
    }
    *llr = m0[1] - m0[0];
    free(cw0); free(cw1); free(m0); free(m1); free(nxt);
    return 0;
}

/* Every phase 0..l-1 once (root bchCoder.cpp:513-515): total SUM / CMP counts and the
 * phase LLRs (llr may be NULL). */
int kor_trellis_counts(const uint8_t *Kmat, int l, const float *y, uint64_t *sum, uint64_t *cmp,
                       double *llr) {
    if (l < 2 || l > 63) return -1;
    *sum = *cmp = 0;
    for (int ph = 0; ph < l; ++ph) {
        double v;
        const int rc = phase_llr(Kmat, (unsigned)l, (unsigned)ph, y, sum, cmp, &v);
        if (rc) return rc;
        if (llr) llr[ph] = v;
    }
    return 0;
}

/* Candidate `code` -> B = L.U (root bchCoder.cpp:766-785): the draws randomInvertibleMatrix
 * makes, in its order (row i: l[i][0..i-1], then u[i][i+1..m-1]), are bits 0, 1, ... of
 * code. Returns the column map perm[j] = B j (:608-626) for j < 2^m. */
void kor_lu_perm(int m, uint64_t code, uint32_t *perm) {
    unsigned char L[64] = {0}, U[64] = {0}, Bm[64];
    int d = 0;
    for (int i = 0; i < m; ++i) {
        L[i * m + i] = U[i * m + i] = 1;
        for (int j = 0; j < i; ++j) L[i * m + j] = (unsigned char)((code >> d++) & 1);
        for (int j = i + 1; j < m; ++j) U[i * m + j] = (unsigned char)((code >> d++) & 1);
    }
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) {
            unsigned char b = 0;
            for (int k = 0; k < m; ++k) b ^= L[i * m + k] & U[k * m + j];
            Bm[i * m + j] = b;
        }
    uint32_t basis[8];
    for (int j = 0; j < m; ++j) { /* newBasis[j] = sum_k oldBasis[k] b[k][j] (:608-613) */
        basis[j] = 0;
        for (int k = 0; k < m; ++k) basis[j] ^= (Bm[k * m + j] ? 1u : 0u) << k;
    }
    for (int j = 0; j < (1 << m); ++j) {
        uint32_t t = 0;
        for (int k = 0; k < m; ++k)
            if (j & (1 << k)) t ^= basis[k];
        perm[j] = t;
    }
}

/* randomSwapColumns over an explicit candidate sequence codes[0..count): tempMatrix[k][j] =
 * matrix[k][perm[j]] (:627-629), accepted when both counts strictly drop (:651-657).
 * Returns the index of the accepted candidate (-1 if none). */
long kor_column_search(int m, const uint8_t *Kmat, const float *y, const uint64_t *codes, size_t count,
                       uint8_t *best, uint32_t *best_perm, uint64_t *best_sum, uint64_t *best_cmp) {
    const int n = 1 << m;
    uint64_t mins = ~0ull, minc = ~0ull;
    long bi = -1;
    uint8_t *tmp = malloc((size_t)n * n);
    uint32_t perm[64];
    for (size_t c = 0; c < count; ++c) {
        kor_lu_perm(m, codes[c], perm);
        for (int k = 0; k < n; ++k)
            for (int j = 0; j < n; ++j) tmp[k * n + j] = Kmat[k * n + perm[j]];
        uint64_t s, cm;
        if (kor_trellis_counts(tmp, n, y, &s, &cm, NULL)) {
            free(tmp);
            return -2;
        }
        if (s < mins && cm < minc) {
            mins = s;
            minc = cm;
            bi = (long)c;
            if (best) memcpy(best, tmp, (size_t)n * n);
            if (best_perm) memcpy(best_perm, perm, sizeof(uint32_t) * n);
        }
    }
    free(tmp);
    *best_sum = mins;
    *best_cmp = minc;
    return bi;
}

/* The candidate codes randomSwapColumns draws (root bchCoder.cpp:603 -> :768-775): bits
 * 0, 1, ... of code r are its m (m - 1) uniform_int_distribution<unsigned short>(0, 1)
 * draws on the reference's minstd_rand0 (libstdc++ downscaling: reject >= 2 scaling).
 * *state in / out (the engine's state = its last output). */
void kor_random_codes(int m, size_t count, uint64_t *state, uint64_t *codes) {
    const uint64_t M = 2147483647ull, urngrange = 2147483645ull, scaling = urngrange / 2u,
                   past = 2u * scaling;
    uint64_t x = *state % M;
    if (!x) x = 1;
    const int bits = m * (m - 1);
    for (size_t r = 0; r < count; ++r) {
        uint64_t c = 0;
        for (int d = 0; d < bits; ++d) {
            uint64_t v;
            do {
                x = x * 16807ull % M;
                v = x - 1u;
            } while (v >= past);
            c |= (uint64_t)(v / scaling) << d;
        }
        codes[r] = c;
    }
    *state = x;
}
