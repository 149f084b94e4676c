/* scripts/proto_analytic2.c -- EXPERIMENT: the analytic Kaneko tail with a node budget.
 *
 * Exact test-pattern decoding for a prefix, then candidate codewords from a depth-first
 * enumeration of D_U (see proto_analytic.c). When the bound l0 is too loose for the budget,
 * the enumeration runs at a tighter bound lim (the sum of the k smallest U reliabilities)
 * and the earliest candidate c* with l(c*) <= lim splits the rest: patterns below its first
 * pattern i* are decoded exactly, and from i* on every possible improvement has l < lim,
 * so the enumeration at lim covers it.
 *
 *   gcc -O2 -std=gnu11 -I oracle scripts/proto_analytic2.c oracle/bchk_oracle.c -lm
 *   ./a.out m t snr J count [seed] [i0] [budget] [NB]
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
    /* code / codeword */
    const orc_code *c;
    int n, t, J;
    double a[64];
    int ord[64];
    unsigned char yH[64];
    /* Kaneko state */
    long i, T, m0;
    double l0;
    int firstOK, done, ret, accepted;
    long jsteps, impr, iend;
    uint64_t best;
    /* costs */
    long exact, nodes;
} ks_t;

/* the body of the reference loop for a success at pattern ii (m0, improvement, return,
 * calcT scan) */
static void accept(ks_t *k, uint64_t D, double l, long m, long ii) {
    const int n = k->n, t = k->t;
    if (!ii || !k->firstOK) k->m0 = m;
    if (!(l < k->l0)) return;
    k->best = D;
    k->l0 = l;
    k->accepted = 1;
    long border = (2 * t + 1) - (m + k->m0) / 2, border2 = t - (m + k->m0) / 2;
    double rs = 0, b2 = 0;
    long tk = 0;
    for (int q = 0; q < n && tk < border; ++q)
        if (!((D >> k->ord[q]) & 1)) {
            rs += k->a[k->ord[q]];
            ++tk;
            if (tk == border2) b2 = rs;
        }
    if (border2 <= 0) b2 = 0;
    else if (tk < border2) b2 = rs;
    if (l < rs) {
        k->ret = 1;
        k->done = 1;
        k->iend = ii + 1;
        return;
    }
    long j = 0;
    while (j <= n - 1 - t) {
        double ct = b2;
        for (int u = 0; u <= t; ++u) ct += (j + u < n) ? k->a[k->ord[j + u]] : 0.0;
        if (!(l >= ct)) break;
        ++j;
        ++k->jsteps;
    }
    k->T = (k->J >= 0 && j > k->J) ? k->J : j;
    ++k->impr;
    if (BOUND(k->T) <= ii + 1) {
        k->done = 1;
        k->iend = ii + 1;
    }
}

/* exact decoding of patterns [k->i, to) (stops at the bound or an early return) */
static void exact_range(ks_t *k, long to, int until_success) {
    const int n = k->n;
    unsigned char e[64], x[64];
    int any = 0;
    while (!k->done) {
        if (k->i >= BOUND(k->T)) { k->done = 1; k->iend = BOUND(k->T); return; }
        if (k->i >= to && (!until_success || any)) return;
        const long i = k->i;
        memcpy(e, k->yH, (size_t)n);
        for (long b = 0, v = i; v > 0; ++b, v >>= 1)
            if (v & 1) e[k->ord[b]] ^= 1;
        ++k->exact;
        int ok = orc_alg_decode(k->c, e, x);
        if (!i && !ok) k->firstOK = 0;
        if (ok) {
            any = 1;
            uint64_t D = 0;
            for (int q = 0; q < n; ++q) D |= (uint64_t)(k->yH[q] != x[q]) << q;
            double l = 0;
            for (int q = 0; q < n; ++q)
                if ((D >> q) & 1) l += k->a[q];
            accept(k, D, l, __builtin_popcountll(D), i);
        }
        ++k->i;
    }
}

typedef struct {
    int NB, NU, t;
    double au[64];
    int posu[64];
    uint64_t remU[64], combU[64], kern[64];
    int nkern;
    const int *ord;
    const double *a;
    long ifrom, BM;
    double lim, l0;
    cand_t *cands;
    int ncand, cap;
    long nodes, budget;
} en_t;

static void emit(en_t *E, uint64_t posU, int wU, uint64_t comb) {
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
        if (ifirst < E->ifrom || ifirst >= E->BM) continue;
        uint64_t D = posU;
        for (uint64_t v = DR; v; v &= v - 1) D |= 1ull << E->ord[__builtin_ctzll(v)];
        double l = 0;
        for (uint64_t v = D; v; v &= v - 1) l += E->a[__builtin_ctzll(v)];
        if (!(l < E->l0)) continue;
        if (E->ncand == E->cap) {
            E->cap = E->cap ? 2 * E->cap : 64;
            E->cands = realloc(E->cands, sizeof(cand_t) * E->cap);
        }
        E->cands[E->ncand++] = (cand_t){ifirst, D, l, __builtin_popcountll(D)};
    }
}

static void dfs(en_t *E, int from, int wU, double sum, uint64_t posU, uint64_t rem, uint64_t comb) {
    ++E->nodes;
    if (rem == 0) emit(E, posU, wU, comb);
    if (wU == E->t) return;
    for (int q = from; q < E->NU; ++q) {
        const double s = sum + E->au[q];
        if (s > E->lim) break;
        dfs(E, q + 1, wU + 1, s, posU | (1ull << E->posu[q]), rem ^ E->remU[q], comb ^ E->combU[q]);
    }
}

/* subsets of size <= t with sum <= lim (count, capped) */
static long count_nodes(const double *v, int k, int from, int left, double sum, double lim, long cap) {
    long c = 1;
    if (!left) return c;
    for (int u = from; u < k && c < cap; ++u) {
        if (sum + v[u] > lim) break;
        c += count_nodes(v, k, u + 1, left - 1, sum + v[u], lim, cap - c);
    }
    return c;
}

typedef struct {
    long words, heavy, exact_total, nodes_total, max_nodes, fallback, tight, max_exact_heavy;
    long worst_cost;
} st_t;

static void decode2(const orc_code *c, double s2, int J, const double *y, unsigned char *res,
                    double *l0_out, orc_stats *st, long i0, long budget, int NBo, st_t *S) {
    const int n = c->n, t = c->t;
    ks_t k;
    memset(&k, 0, sizeof k);
    k.c = c; k.n = n; k.t = t; k.J = J;
    for (int i = 0; i < n; ++i) {
        double al = 2 * y[i] / s2;
        k.a[i] = fabs(al);
        k.yH[i] = (al <= 0.0) ? 0 : 1;
        k.ord[i] = i;
    }
    for (int i = 1; i < n; ++i) {
        int p = k.ord[i], j = i - 1;
        while (j >= 0 && k.a[k.ord[j]] > k.a[p]) { k.ord[j + 1] = k.ord[j]; --j; }
        k.ord[j + 1] = p;
    }
    k.T = n;
    k.l0 = DBL_MAX;
    k.firstOK = 1;
    exact_range(&k, i0, 1);
    if (!k.done) {
        ++S->heavy;
        const long exact_before = k.exact;
        en_t E;
        memset(&E, 0, sizeof E);
        E.t = t; E.ord = k.ord; E.a = k.a;
        E.NB = NBo > 0 ? NBo : 31;
        if (E.NB > n) E.NB = n;
        E.NU = n - E.NB;
        E.BM = (J >= 0 && J < 31) ? (1L << J) - 1 : 2147483647L;
        if (!k.impr && BOUND(k.T) > E.BM) E.BM = BOUND(k.T);
        uint64_t bv[64], bc[64];
        int piv[64], nb = 0;
        for (int b = 0; b < E.NB; ++b) {
            uint64_t v = col_of(c, k.ord[b]), cm = 1ull << b;
            for (int q = 0; q < nb; ++q)
                if ((v >> piv[q]) & 1) { v ^= bv[q]; cm ^= bc[q]; }
            if (v) { piv[nb] = __builtin_ctzll(v); bv[nb] = v; bc[nb] = cm; ++nb; }
            else E.kern[E.nkern++] = cm;
        }
        uint64_t S0 = 0;
        for (int p = 0; p < n; ++p)
            if (k.yH[p]) S0 ^= col_of(c, p);
        uint64_t rem0 = S0, comb0 = 0;
        for (int q = 0; q < nb; ++q)
            if ((rem0 >> piv[q]) & 1) { rem0 ^= bv[q]; comb0 ^= bc[q]; }
        for (int u = 0; u < E.NU; ++u) {
            const int p = k.ord[E.NB + u];
            uint64_t v = col_of(c, p), cm = 0;
            for (int q = 0; q < nb; ++q)
                if ((v >> piv[q]) & 1) { v ^= bv[q]; cm ^= bc[q]; }
            E.remU[u] = v; E.combU[u] = cm;
            E.au[u] = k.a[p];
            E.posu[u] = p;
        }
        /* bound selection: the full l0 if within budget, else the largest prefix sum */
        const double full = k.l0 * (1.0 + 1e-12);
        double lim = full;
        int complete = 1;
        E.ifrom = k.i;
        E.l0 = k.l0;
        int q0 = 0;
        for (long bud = budget;; bud *= 4) {
            complete = 1;
            lim = full;
            if (count_nodes(E.au, E.NU, 0, t, 0.0, full, bud + 1) > bud) {
                complete = 0;
                double pre = 0;
                lim = 0;
                for (int q = 0; q < E.NU && q <= t; ++q) {
                    const double p2 = pre + E.au[q];
                    if (count_nodes(E.au, E.NU, 0, t, 0.0, p2 * (1.0 + 1e-12), bud + 1) > bud) break;
                    pre = p2;
                    lim = p2;
                }
                if (bud == budget) ++S->tight;
            }
            E.lim = complete ? full : lim * (1.0 + 1e-12);
            E.ncand = 0;
            if (lim > 0) dfs(&E, 0, 0, 0.0, 0, rem0, comb0);
            qsort(E.cands, (size_t)E.ncand, sizeof(cand_t), cmp_cand);
            if (complete) break;
            long istar = -1;
            for (int q = 0; q < E.ncand; ++q)
                if (E.cands[q].l <= lim) { istar = E.cands[q].i; q0 = q; break; }
            if (istar >= 0) { exact_range(&k, istar, 0); break; }
            if (bud > 64 * budget) {
                ++S->fallback;
                exact_range(&k, E.BM + 1, 0); /* everything, exactly */
                q0 = E.ncand;
                break;
            }
        }
        k.nodes += E.nodes;
        for (int q = q0; q < E.ncand && !k.done; ++q) {
            const cand_t *cd = &E.cands[q];
            if (cd->i >= BOUND(k.T)) break;
            accept(&k, cd->D, cd->l, cd->m, cd->i);
        }
        if (!k.done) { k.done = 1; k.iend = BOUND(k.T); }
        free(E.cands);
        const long ex = k.exact - exact_before;
        if (ex > S->max_exact_heavy) S->max_exact_heavy = ex;
        if (E.nodes > S->max_nodes) S->max_nodes = E.nodes;
        if (ex * 30 + E.nodes > S->worst_cost) S->worst_cost = ex * 30 + E.nodes;
    }
    S->exact_total += k.exact;
    S->nodes_total += k.nodes;
    orc_stats s;
    memset(&s, 0, sizeof s);
    s.decodes = (uint64_t)k.iend;
    s.iters = (uint64_t)(k.ret ? k.iend - 1 : k.iend);
    s.jsteps = (uint64_t)k.jsteps;
    s.improvements = (uint64_t)k.impr;
    s.accepted = k.accepted;
    s.returned = k.ret;
    s.cmp = s.iters * (uint64_t)(n + 6) + s.jsteps + s.improvements;
    s.sum = s.iters * (uint64_t)(n + 1) + s.jsteps;
    if (k.accepted)
        for (int q = 0; q < n; ++q) res[q] = k.yH[q] ^ (unsigned char)((k.best >> q) & 1);
    *l0_out = k.l0;
    *st = s;
}

int main(int argc, char **argv) {
    if (argc < 6) { fprintf(stderr, "usage: m t snr J count [seed] [i0] [budget] [NB]\n"); return 2; }
    const int m = atoi(argv[1]), t = atoi(argv[2]);
    const double snr = atof(argv[3]);
    const int J = atoi(argv[4]);
    const long count = atol(argv[5]);
    const uint64_t seed = argc > 6 ? strtoull(argv[6], 0, 10) : 1;
    const long i0 = argc > 7 ? atol(argv[7]) : 64;
    const long budget = argc > 8 ? atol(argv[8]) : 4096;
    const int NB = argc > 9 ? atoi(argv[9]) : 0;
    orc_code c;
    orc_code_init(&c, m, t);
    const int n = c.n;
    orc_rng rng;
    orc_rng_seed(&rng, seed);
    const double sd = orc_sigma(&c, snr), s2 = pow(orc_sigma(&c, 0.5), 2);
    unsigned char info[256], tx[256], r1[256], r2[256];
    double y[256];
    st_t S;
    memset(&S, 0, sizeof S);
    long bad = 0, ref_patterns = 0, ref_heavy_patterns = 0;
    for (long w = 0; w < count; ++w) {
        orc_gen_info(&rng, info, c.k);
        orc_encode(&c, info, tx);
        orc_add_noise(&rng, sd, tx, y, n);
        memset(r1, 0, n);
        memset(r2, 0, n);
        double l1, l2;
        orc_stats s1, s2s;
        orc_kaneko_decode(&c, s2, J, y, r1, &l1, &s1);
        ref_patterns += (long)s1.decodes;
        if (s1.decodes > (uint64_t)i0) ref_heavy_patterns += (long)s1.decodes;
        decode2(&c, s2, J, y, r2, &l2, &s2s, i0, budget, NB, &S);
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
    printf("m=%d t=%d snr=%g J=%d count=%ld i0=%ld budget=%ld: mismatches %ld\n"
           "  reference patterns %ld (heavy %ld); exact %ld; heavy %ld, tightened %ld, fallback %ld\n"
           "  dfs nodes %ld (max %ld), max exact per heavy %ld, worst cost %ld\n",
           m, t, snr, J, count, i0, budget, bad, ref_patterns, ref_heavy_patterns, S.exact_total, S.heavy, S.tight,
           S.fallback, S.nodes_total, S.max_nodes, S.max_exact_heavy, S.worst_cost);
    return bad != 0;
}
