/* scripts/proto_analytic.c -- EXPERIMENT: Kaneko search without decoding every test pattern.
 *
 * After the first test patterns are decoded exactly (phase A), the rest of the search is
 * replayed from the candidate codewords instead of decoding patterns one by one:
 *   pattern i succeeds  <=>  some codeword c has 1 <= |yH ^ P_i ^ c| <= t,
 * and P_i only flips the NB least reliable positions R. Writing D = yH ^ c = D_U + D_R
 * (U = the other positions), c is reachable iff |D_U| <= t, and syn(D_R) = S0 ^ syn(D_U)
 * must lie in V = span of R's syndrome columns. Its first pattern is D_R with its top
 * t - |D_U| bits cleared. Improvements need l(c) < l0 and l(c) >= sum_{D_U} a, so a
 * depth-first enumeration of D_U (ascending reliabilities, pruned at l0) finds every
 * codeword that can still improve. The replay applies the reference's acceptance logic to
 * those codewords in first-pattern order.
 *
 * Checks every codeword against orc_kaneko_decode and prints enumeration statistics.
 *   gcc -O2 -std=c11 -I oracle scripts/proto_analytic.c oracle/bchk_oracle.c -lm
 *   ./a.out m t snr J count [seed]
 */
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bchk_oracle.h"

#define BOUND(T_) ((long)((1UL << ((T_) & 31)) - 1UL))

typedef struct {
    long i;
    uint64_t D;
    double l;
    int m;
    double su;
} cand_t;

static int cmp_cand(const void *a, const void *b) {
    const cand_t *x = a, *y = b;
    return x->i < y->i ? -1 : x->i > y->i;
}

static uint64_t col_of(const orc_code *c, int p) {
    uint64_t v = 0;
    for (int q = 0; q < c->t; ++q) v |= (uint64_t)c->alog[((long)(2 * q + 1) * p) % c->n] << (8 * q);
    return v;
}

typedef struct {
    const orc_code *c;
    const double *a;
    const int *ord;
    int NB, n, t;
    uint64_t remU[64], combU[64];
    uint64_t kern[64];
    int nkern;
    double lim;
    long i0;
    cand_t *cands;
    int ncand, cap;
    long nodes;
    long depth[16];
} enum_t;

static void emit(enum_t *E, uint64_t posU, int wU, uint64_t comb, double su) {
    for (uint64_t ks = 0; ks < (1ull << E->nkern); ++ks) {
        uint64_t DR = comb;
        for (int q = 0; q < E->nkern; ++q)
            if ((ks >> q) & 1) DR ^= E->kern[q];
        const int r = E->t - wU;
        long ifirst;
        if (__builtin_popcountll(DR) <= r) {
            ifirst = (wU == 0 && DR == 0) ? 1 : 0;
        } else {
            uint64_t v = DR;
            for (int q = 0; q < r; ++q) v &= ~(1ull << (63 - __builtin_clzll(v)));
            ifirst = (long)v;
        }
        if (ifirst < E->i0) continue;
        uint64_t D = posU;
        for (uint64_t v = DR; v; v &= v - 1) D |= 1ull << E->ord[__builtin_ctzll(v)];
        double l = 0;
        for (uint64_t v = D; v; v &= v - 1) l += E->a[__builtin_ctzll(v)];
        if (E->ncand == E->cap) {
            E->cap = E->cap ? 2 * E->cap : 64;
            E->cands = realloc(E->cands, sizeof(cand_t) * E->cap);
        }
        E->cands[E->ncand++] = (cand_t){ifirst, D, l, __builtin_popcountll(D), su};
    }
}

static long count_sub(const double *v, int k, int from, int left, double sum, double lim) {
    long c = 1;
    if (!left) return c;
    for (int u = from; u < k; ++u) {
        if (sum + v[u] > lim) break;
        c += count_sub(v, k, u + 1, left - 1, sum + v[u], lim);
    }
    return c;
}

static void dfs(enum_t *E, int from, int wU, double sum, uint64_t posU, uint64_t rem, uint64_t comb) {
    ++E->nodes;
    ++E->depth[wU];
    if (rem == 0) emit(E, posU, wU, comb, sum);
    if (wU == E->t) return;
    for (int u = from; u < E->n; ++u) {
        const double s = sum + E->a[E->ord[u]];
        if (s > E->lim) break; /* ascending: no later u fits either */
        dfs(E, u + 1, wU + 1, s, posU | (1ull << E->ord[u]), rem ^ E->remU[u], comb ^ E->combU[u]);
    }
}

typedef struct {
    long nodes, cands, heavy;
    long depth[16];
    long maxn5, maxn4;
    long mitm, maxmitm;
    long surv, maxsurv;
} stat_t;

/* analytic Kaneko; returns 0 and fills res/l0/st */
static void analytic(const orc_code *c, double s2, int J, const double *y, unsigned char *res,
                     double *l0_out, orc_stats *st, long i0max, stat_t *S) {
    const int n = c->n, t = c->t;
    double a[64];
    unsigned char yH[64], e[64], x[64];
    int ord[64];
    orc_stats s;
    memset(&s, 0, sizeof s);
    for (int i = 0; i < n; ++i) {
        double al = 2 * y[i] / s2;
        a[i] = fabs(al);
        yH[i] = (al <= 0.0) ? 0 : 1;
        ord[i] = i;
    }
    for (int i = 1; i < n; ++i) {
        int p = ord[i], j = i - 1;
        while (j >= 0 && a[ord[j]] > a[p]) { ord[j + 1] = ord[j]; --j; }
        ord[j + 1] = p;
    }
    long i = 0, T = n;
    double l0 = DBL_MAX;
    int firstOK = 1;
    long m0 = 0;
    /* the acceptance body: returns 1 when the loop ends (early return) */
    uint64_t yHm = 0;
    for (int p = 0; p < n; ++p) yHm |= (uint64_t)yH[p] << p;
#define ACCEPT(DM, LL, MM, II)                                                              \
    do {                                                                                    \
        if (!(II) || !firstOK) m0 = (MM);                                                   \
        if ((LL) < l0) {                                                                    \
            for (int q = 0; q < n; ++q) res[q] = yH[q] ^ (unsigned char)(((DM) >> q) & 1);  \
            l0 = (LL);                                                                      \
            s.accepted = 1;                                                                 \
            long border = (2 * t + 1) - ((MM) + m0) / 2, border2 = t - ((MM) + m0) / 2;     \
            double rs = 0, b2 = 0;                                                          \
            long tk = 0;                                                                    \
            for (int q = 0; q < n && tk < border; ++q)                                      \
                if (!(((DM) >> ord[q]) & 1)) { rs += a[ord[q]]; ++tk; if (tk == border2) b2 = rs; } \
            if (border2 <= 0) b2 = 0; else if (tk < border2) b2 = rs;                     \
            if ((LL) < rs) { s.returned = 1; ret = 1; break; }                              \
            long j = 0;                                                                     \
            for (;;) {                                                                      \
                if (!(j <= n - 1 - t)) break;                                               \
                double ct = b2;                                                             \
                for (int u = 0; u <= t; ++u) ct += (j + u < n) ? a[ord[j + u]] : 0.0;        \
                if (!((LL) >= ct)) break;                                                   \
                ++j; ++s.jsteps;                                                            \
            }                                                                               \
            T = (J >= 0 && j > J) ? J : j;                                                  \
            ++s.improvements;                                                               \
        }                                                                                   \
    } while (0)
    int ret = 0;
    /* phase A: exact decodes until i0max patterns AND at least one success */
    int any = 0;
    while (i < BOUND(T)) {
        if (i >= i0max && any) break;
        memcpy(e, yH, (size_t)n);
        for (long b = 0, v = i; v > 0; ++b, v >>= 1)
            if (v & 1) e[ord[b]] ^= 1;
        s.decodes++;
        int ok = orc_alg_decode(c, e, x);
        if (!i && !ok) firstOK = 0;
        if (ok) {
            any = 1;
            uint64_t D = 0;
            for (int q = 0; q < n; ++q) D |= (uint64_t)(yH[q] != x[q]) << q;
            double l = 0;
            for (int q = 0; q < n; ++q) if ((D >> q) & 1) l += a[q];
            ACCEPT(D, l, (long)__builtin_popcountll(D), i);
            if (ret) break;
        }
        ++i;
        ++s.iters;
    }
    if (!ret && i < BOUND(T)) {
        /* phase B */
        S->heavy++;
        enum_t E;
        memset(&E, 0, sizeof E);
        E.c = c; E.a = a; E.ord = ord; E.n = n; E.t = t;
        E.NB = getenv("NB") ? atoi(getenv("NB")) : ((J >= 0 && J < 31) ? J : 31);
        if (E.NB > n) E.NB = n;
        E.i0 = i;
        E.lim = l0 * (1.0 + 1e-12);
        uint64_t bv[64], bc[64];
        int piv[64], nb = 0;
        for (int b = 0; b < E.NB; ++b) {
            uint64_t v = col_of(c, ord[b]), cm = 1ull << b;
            for (int k = 0; k < nb; ++k)
                if ((v >> piv[k]) & 1) { v ^= bv[k]; cm ^= bc[k]; }
            if (v) { piv[nb] = __builtin_ctzll(v); bv[nb] = v; bc[nb] = cm; ++nb; }
            else E.kern[E.nkern++] = cm;
        }
        uint64_t S0 = 0;
        for (int p = 0; p < n; ++p) if (yH[p]) S0 ^= col_of(c, p);
        uint64_t rem0 = S0, comb0 = 0;
        for (int k = 0; k < nb; ++k)
            if ((rem0 >> piv[k]) & 1) { rem0 ^= bv[k]; comb0 ^= bc[k]; }
        for (int u = E.NB; u < n; ++u) {
            uint64_t v = col_of(c, ord[u]), cm = 0;
            for (int k = 0; k < nb; ++k)
                if ((v >> piv[k]) & 1) { v ^= bv[k]; cm ^= bc[k]; }
            E.remU[u] = v; E.combU[u] = cm;
        }
        dfs(&E, E.NB, 0, 0.0, 0, rem0, comb0);
        {
            double ve[64], vo[64];
            int ke = 0, ko = 0;
            for (int u = E.NB; u < n; ++u) { if ((u - E.NB) & 1) vo[ko++] = a[ord[u]]; else ve[ke++] = a[ord[u]]; }
            long le = count_sub(ve, ke, 0, t, 0.0, E.lim), lo = count_sub(vo, ko, 0, t, 0.0, E.lim);
            long d4 = 0; for (int d = 0; d <= t - 2; ++d) d4 += E.depth[d];
            if (getenv("VERB")) printf("  heavy: patterns_left %ld nodes %ld d<=t-2 %ld Le %ld Lo %ld cands %d\n", (long)BOUND(T) - i, E.nodes, d4, le, lo, E.ncand);
            S->mitm += le + lo; if (le + lo > S->maxmitm) S->maxmitm = le + lo;
        }
        S->nodes += E.nodes;
        { long a5=0,a4=0; for (int d=0; d<16; ++d) { S->depth[d]+=E.depth[d]; if (d<=t-1) a5+=E.depth[d]; if (d<=t-2) a4+=E.depth[d]; }
          if (a5>S->maxn5) S->maxn5=a5; if (a4>S->maxn4) S->maxn4=a4; }
        S->cands += E.ncand;
        {
            const long BM = (J >= 0 && J < 31) ? (1L << J) - 1 : 2147483647L;
            long sv = 0;
            for (int q = 0; q < E.ncand; ++q) sv += E.cands[q].i < BM && E.cands[q].l < l0;
            S->surv += sv; if (sv > S->maxsurv) S->maxsurv = sv;
            if (getenv("TIGHT") && E.nodes > 20000) {
                /* iterative tightening: lim1 = sum of the first k U reliabilities */
                printf("  bad: nodes %ld l0/aU0 %.2f i0 %ld bound %ld:", E.nodes, l0 / a[ord[E.NB]], i, (long)BOUND(T));
                double lim1 = 0;
                for (int k = 1; k <= t + 1 && E.NB + k - 1 < n; ++k) {
                    lim1 += a[ord[E.NB + k - 1]];
                    long istar = -1;
                    for (int q = 0; q < E.ncand; ++q)
                        if (E.cands[q].su < lim1 && E.cands[q].l <= lim1 && E.cands[q].i < BM && (istar < 0 || E.cands[q].i < istar)) istar = E.cands[q].i;
                    enum_t E2 = E; E2.nodes = 0; memset(E2.depth, 0, sizeof E2.depth); E2.lim = lim1; E2.cands = 0; E2.ncand = E2.cap = 0;
                    dfs(&E2, E.NB, 0, 0.0, 0, rem0, comb0); free(E2.cands);
                    printf(" [k=%d nodes %ld i* %ld]", k, E2.nodes, istar);
                }
                printf("\n");
            }
        }
        qsort(E.cands, (size_t)E.ncand, sizeof(cand_t), cmp_cand);
        long iend = -1;
        for (int q = 0; q < E.ncand && !ret; ++q) {
            const cand_t *cd = &E.cands[q];
            if (cd->i >= BOUND(T)) break;
            ACCEPT(cd->D, cd->l, (long)cd->m, cd->i);
            if (ret) { iend = cd->i + 1; break; }
            if (BOUND(T) <= cd->i + 1) { iend = cd->i + 1; break; }
        }
        if (ret) { s.decodes = iend; s.iters = iend - 1; }
        else {
            if (iend < 0) iend = BOUND(T);
            if (iend < i) iend = i; /* bound fell below the processed prefix: cannot happen */
            s.decodes = iend; s.iters = iend;
        }
        free(E.cands);
    }
    s.cmp = s.iters * (uint64_t)(n + 6) + s.jsteps + s.improvements;
    s.sum = s.iters * (uint64_t)(n + 1) + s.jsteps;
    *l0_out = l0;
    *st = s;
#undef ACCEPT
}

int main(int argc, char **argv) {
    if (argc < 6) { fprintf(stderr, "usage: m t snr J count [seed] [i0]\n"); return 2; }
    const int m = atoi(argv[1]), t = atoi(argv[2]);
    const double snr = atof(argv[3]);
    const int J = atoi(argv[4]);
    const long count = atol(argv[5]);
    const uint64_t seed = argc > 6 ? strtoull(argv[6], 0, 10) : 1;
    const long i0 = argc > 7 ? atol(argv[7]) : 64;
    orc_code c;
    orc_code_init(&c, m, t);
    const int n = c.n;
    orc_rng rng;
    orc_rng_seed(&rng, seed);
    const double sd = orc_sigma(&c, snr), s2 = pow(orc_sigma(&c, 0.5), 2);
    unsigned char info[256], tx[256], r1[256], r2[256];
    double y[256];
    stat_t S;
    memset(&S, 0, sizeof S);
    long bad = 0, heavy_dec = 0, maxnodes = 0;
    for (long w = 0; w < count; ++w) {
        orc_gen_info(&rng, info, c.k);
        orc_encode(&c, info, tx);
        orc_add_noise(&rng, sd, tx, y, n);
        memset(r1, 0, n); memset(r2, 0, n);
        double l1, l2;
        orc_stats s1, s2s;
        orc_kaneko_decode(&c, s2, J, y, r1, &l1, &s1);
        long before = S.nodes;
        analytic(&c, s2, J, y, r2, &l2, &s2s, i0, &S);
        if (S.nodes - before > maxnodes) maxnodes = S.nodes - before;
        if (s1.decodes > (uint64_t)i0) heavy_dec += s1.decodes;
        if (memcmp(r1, r2, n) || memcmp(&l1, &l2, 8) || s1.decodes != s2s.decodes || s1.cmp != s2s.cmp ||
            s1.sum != s2s.sum || s1.accepted != s2s.accepted) {
            if (bad < 10)
                printf("MISMATCH w=%ld dec %lu/%lu cmp %lu/%lu sum %lu/%lu l %.17g/%.17g acc %d/%d res %d\n", w,
                       (unsigned long)s1.decodes, (unsigned long)s2s.decodes, (unsigned long)s1.cmp,
                       (unsigned long)s2s.cmp, (unsigned long)s1.sum, (unsigned long)s2s.sum, l1, l2,
                       s1.accepted, s2s.accepted, memcmp(r1, r2, n) != 0);
            ++bad;
        }
    }
    printf("m=%d t=%d snr=%g J=%d count=%ld: mismatches %ld; heavy %ld (patterns %ld), dfs nodes %ld "
           "(%.1f per heavy, max %ld), candidates %ld\n",
           m, t, snr, J, count, bad, S.heavy, heavy_dec, S.nodes, S.heavy ? (double)S.nodes / S.heavy : 0.0,
           maxnodes, S.cands);
    printf("  depth:");
    for (int d = 0; d <= t; ++d) printf(" %ld", S.depth[d]);
    printf("  max(depth<=t-1) %ld max(depth<=t-2) %ld; mitm lists total %ld max %ld\n", S.maxn5, S.maxn4, S.mitm, S.maxmitm);
    printf("  survivors %ld max %ld\n", S.surv, S.maxsurv);
    return bad != 0;
}
