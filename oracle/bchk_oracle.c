/* oracle/bchk_oracle.c -- TEST INFRASTRUCTURE ONLY (see bchk_oracle.h).
 *
 * A from-scratch C11 restatement of the reference hot path. Every function cites
 * the reference file:line it follows (paths relative to the reference repo root).
 * It is the checker for the HIP path; nothing in the product links it.
 *
 * Known, documented divergence: the reference orders reliabilities with std::sort on
 * |alpha| only (src/KanekoKernelProcessor.cpp:148,343), which leaves the order of
 * EXACTLY equal |alpha| values unspecified. This restatement (and the GPU) break such
 * ties by position index. Continuous AWGN never produces such ties in practice; the
 * golden vectors contain none (tests check this).
 */
#include "bchk_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <pthread.h>

static const unsigned kPrim[16] = {3, 7, 11, 19, 37, 67, 137, 285, 529, 1033,
                                   2053, 4179, 8219, 17475, 32771, 69643}; /* main.cpp:14 */

static inline unsigned gf_mul(const orc_code *c, unsigned a, unsigned b) {
    if (!a || !b) return 0;
    int s = c->log_[a] + c->log_[b];
    if (s >= c->n) s -= c->n;
    return c->alog[s];
}
static inline unsigned gf_pow_alpha(const orc_code *c, long e) { /* alpha^e, e >= 0 */
    return c->alog[e % c->n];
}

/* ---------------------------------------------------------------- code setup */
/* GF(2^m) tables: src/main.cpp:59-78. g(x) = lcm of the minimal polynomials of
 * alpha^1..alpha^(2t-1) (main.cpp:84-92; bchCoder.cpp:25-91 minimal polynomial,
 * :217 lcm). The lcm of irreducibles is the product of the distinct ones, so we
 * multiply the minimal polynomial of each distinct cyclotomic coset once. */
int orc_code_init(orc_code *c, int m, int t) {
    if (m < 2 || m > 8 || t <= 0 || t >= (1 << (m - 1))) return -1; /* main.cpp:55 */
    memset(c, 0, sizeof *c);
    c->m = m; c->t = t; c->n = (1 << m) - 1;
    const int n = c->n;
    c->alog[0] = 1;
    for (int i = 1; i < n; ++i) {
        unsigned v = c->alog[i - 1] << 1;
        if (v >> m) v ^= kPrim[m - 1];
        c->alog[i] = v;
    }
    c->log_[0] = -1;
    for (int i = 0; i < n; ++i) c->log_[c->alog[i]] = i;

    unsigned char g[ORC_MAXN + 1] = {1};
    int gdeg = 0;
    unsigned char seen[ORC_MAXN + 1] = {0};
    for (int i = 1; i < 2 * t; ++i) {
        if (seen[i % n]) continue;
        /* minimal polynomial of alpha^i: prod over the coset {i*2^j} of (x + alpha^e) */
        unsigned mp[ORC_MAXN + 1] = {1};
        int mdeg = 0;
        int e = i % n;
        do {
            seen[e] = 1;
            unsigned root = c->alog[e];
            /* mp <- mp * (x + root) */
            for (int d = mdeg + 1; d >= 0; --d) {
                unsigned hi = d > 0 ? mp[d - 1] : 0;
                unsigned lo = d <= mdeg ? gf_mul(c, mp[d], root) : 0;
                mp[d] = hi ^ lo;
            }
            ++mdeg;
            e = (e * 2) % n;
        } while (e != i % n);
        /* coefficients are 0/1 field elements; g <- g * mp over GF(2) */
        unsigned char tmp[ORC_MAXN + 1];
        memset(tmp, 0, sizeof tmp);
        for (int a = 0; a <= gdeg; ++a)
            if (g[a])
                for (int b = 0; b <= mdeg; ++b) tmp[a + b] ^= (unsigned char)(mp[b] & 1);
        gdeg += mdeg;
        memcpy(g, tmp, sizeof g);
    }
    c->gsize = gdeg + 1;
    memcpy(c->g, g, (size_t)c->gsize);
    c->k = n - c->gsize + 1; /* main.cpp:93 */
    return 0;
}

/* ---------------------------------------------------------------- RNG stream */
/* minstd_rand0: x <- 16807 x mod (2^31 - 1), default seed 1. */
static inline uint64_t minstd(orc_rng *r) {
    r->x = (r->x * 16807u) % 2147483647u;
    return r->x;
}
void orc_rng_seed(orc_rng *r, uint64_t seed) {
    seed %= 2147483647u;
    r->x = seed ? seed : 1u;
}
/* uniform_int_distribution<unsigned short>(0,1), libstdc++ 11 "downscaling
 * fallback": urngrange = 2^31-3, scaling = urngrange/2, reject >= 2*scaling. */
static inline unsigned uniform01(orc_rng *r) {
    const uint64_t urngrange = 2147483646u - 1u;
    const uint64_t scaling = urngrange / 2u;
    const uint64_t past = 2u * scaling;
    uint64_t v;
    do v = minstd(r) - 1u; while (v >= past);
    return (unsigned)(v / scaling);
}
/* std::generate_canonical<double, 53>(minstd_rand0): two draws, base r = 2^31-2. */
static inline double canonical(orc_rng *r) {
    const long double R = 2147483646.0L;
    double sum = 0.0, tmp = 1.0;
    for (int k = 0; k < 2; ++k) {
        sum += (double)(minstd(r) - 1u) * tmp;
        tmp = (double)((long double)tmp * R);
    }
    double ret = sum / tmp;
    if (ret >= 1.0) ret = nextafter(1.0, 0.0);
    return ret;
}
void orc_gen_info(orc_rng *r, unsigned char *info, int k) {
    for (int i = 0; i < k; ++i) info[i] = (unsigned char)uniform01(r);
}
/* c(x) = info(x) g(x) over GF(2): bchCoder.cpp:120-132 (non-systematic). */
void orc_encode(const orc_code *c, const unsigned char *info, unsigned char *cw) {
    memset(cw, 0, (size_t)c->n);
    for (int i = 0; i < c->k; ++i)
        if (info[i])
            for (int j = 0; j < c->gsize; ++j) cw[i + j] ^= c->g[j];
}
/* addNoise: bchCoder.cpp:243-250 with a FRESH normal_distribution (its cached
 * second polar variate dies with it): Marsaglia polar method as libstdc++. */
void orc_add_noise(orc_rng *r, double sd, const unsigned char *cw, double *y, int n) {
    int saved_ok = 0;
    double saved = 0.0;
    for (int i = 0; i < n; ++i) {
        double v;
        if (saved_ok) {
            saved_ok = 0;
            v = saved;
        } else {
            double x, yy, r2;
            do {
                x = 2.0 * canonical(r) - 1.0;
                yy = 2.0 * canonical(r) - 1.0;
                r2 = x * x + yy * yy;
            } while (r2 > 1.0 || r2 == 0.0);
            const double mult = sqrt(-2 * log(r2) / r2);
            saved = x * mult;
            saved_ok = 1;
            v = yy * mult;
        }
        v = v * sd + 0.0;
        y[i] = (cw[i] ? 1 : -1) + v;
    }
}
double orc_sigma(const orc_code *c, double snr_db) {
    long k = c->k, n = c->n;
    return sqrt(1 / (pow(10, snr_db / 10) * 2 * k / n));
}

/* ------------------------------------------------------ algebraic decoder */
/* Syndromes S_j = w(alpha^j), j = 1..2t: Decoder::findSyndromPoly :184-207. */
static void syndromes(const orc_code *c, const unsigned char *w, unsigned *S) {
    for (int j = 1; j <= 2 * c->t; ++j) {
        unsigned s = 0;
        for (int i = 0; i < c->n; ++i)
            if (w[i]) s ^= gf_pow_alpha(c, (long)i * j);
        S[j] = s;
    }
}
static int pdeg(const unsigned *p, int cap) {
    for (int d = cap; d >= 0; --d)
        if (p[d]) return d;
    return -1;
}
/* Chien search + acceptance rule of Decoder::locatorsAndRoots :279-296: success iff
 * the number of roots alpha^k (k = 0..n-1) equals deg(lambda) >= 1; each root alpha^k
 * flags error position (n-k) mod n; decode :309-319 flips them. */
static int chien_apply(const orc_code *c, const unsigned *lam, int deg,
                       const unsigned char *word, unsigned char *answer) {
    if (deg < 1) return 0;
    int pos[ORC_MAXN + 1], cnt = 0;
    for (int k = 0; k < c->n; ++k) {
        unsigned x = c->alog[k], v = lam[deg];
        for (int i = deg - 1; i >= 0; --i) v = gf_mul(c, v, x) ^ lam[i];
        if (!v) pos[cnt++] = (c->n - k) % c->n;
    }
    if (cnt != deg) return 0;
    memcpy(answer, word, (size_t)c->n);
    for (int i = 0; i < cnt; ++i) answer[pos[i]] ^= 1;
    return 1;
}

/* Sugiyama / Euclid key-equation solver, Decoder::euclid :233-277 (with
 * dividePolynomial :112, multiplyPolynomials :94, addPolynomials :71):
 * r_{-1} = x^{2t}, r_0 = S(x) = sum S_{j+1} x^j; lambda_{-1} = 0, lambda_0 = 1;
 * iterate while deg r >= t (the reference's `sizeP > t`); fail if lambda(0) = 0. */
int orc_alg_decode(const orc_code *c, const unsigned char *word, unsigned char *answer) {
    const int t = c->t, L2 = 2 * t;
    unsigned S[2 * ORC_MAXT + 2];
    syndromes(c, word, S);
    unsigned a[2 * ORC_MAXT + 2] = {0}, b[2 * ORC_MAXT + 2] = {0};
    unsigned la[2 * ORC_MAXT + 2] = {0}, lb[2 * ORC_MAXT + 2] = {0};
    a[L2] = 1;                                  /* r_{-1} = x^{2t}   (:234-238) */
    for (int j = 0; j < L2; ++j) b[j] = S[j + 1]; /* r_0 = S(x)        (:241)     */
    lb[0] = 1;                                   /* lambda_0 = 1     (:248-249) */
    int db = pdeg(b, L2);
    while (db >= t) {
        /* q, rem = divmod(a, b) */
        unsigned q[2 * ORC_MAXT + 2] = {0};
        int da = pdeg(a, L2);
        int lead_inv_log = (c->n - c->log_[b[db]]) % c->n;
        while (da >= db) {
            unsigned coef = gf_mul(c, a[da], c->alog[lead_inv_log]);
            int sh = da - db;
            q[sh] = coef;
            for (int i = 0; i <= db; ++i) a[i + sh] ^= gf_mul(c, coef, b[i]);
            da = pdeg(a, L2);
        }
        /* lambda_new = lambda_prev + q * lambda_cur */
        unsigned ln[2 * ORC_MAXT + 2];
        memcpy(ln, la, sizeof ln);
        for (int i = 0; i <= L2; ++i)
            if (q[i])
                for (int j = 0; i + j <= L2; ++j) ln[i + j] ^= gf_mul(c, q[i], lb[j]);
        /* shift: (a, b) <- (b, rem); (la, lb) <- (lb, ln) */
        unsigned rem[2 * ORC_MAXT + 2];
        memcpy(rem, a, sizeof rem);
        memcpy(a, b, sizeof a);
        memcpy(b, rem, sizeof b);
        memcpy(la, lb, sizeof la);
        memcpy(lb, ln, sizeof lb);
        db = pdeg(b, L2);
    }
    if (!lb[0]) return 0; /* :270-273 */
    return chien_apply(c, lb, pdeg(lb, L2), word, answer);
}

/* The GPU kernel's formulation: inversionless binary Berlekamp-Massey over the odd
 * syndromes (even discrepancies vanish for binary codes), then the same root rule.
 * Equivalence to Euclid: if BM's register length L <= t, its connection polynomial is a
 * scalar multiple of Euclid's lambda (key-equation uniqueness); if L > t, Euclid's lambda
 * has lambda(0) = 0 and fails. Hence success <=> S != 0, L <= t, #roots == deg C. */
int orc_alg_decode_bm(const orc_code *c, const unsigned char *word, unsigned char *answer) {
    const int t = c->t;
    enum { CAP = 2 * ORC_MAXT + 4 };
    unsigned S[2 * ORC_MAXT + 2];
    syndromes(c, word, S);
    unsigned C[CAP] = {1}, B[CAP] = {1}, Cn[CAP];
    unsigned gamma = 1;
    int L = 0;
    for (int k = 0; k < t; ++k) {
        const int r = 2 * k;
        unsigned d = 0;
        for (int i = 0; i <= r && i < CAP; ++i)
            if (C[i]) d ^= gf_mul(c, C[i], S[r + 1 - i]);
        for (int i = 0; i < CAP; ++i)
            Cn[i] = gf_mul(c, gamma, C[i]) ^ (i ? gf_mul(c, d, B[i - 1]) : 0);
        if (d && 2 * L <= r) {
            memcpy(B, C, sizeof B);
            L = r + 1 - L;
            gamma = d;
        } else {
            memmove(B + 1, B, sizeof(unsigned) * (CAP - 1));
            B[0] = 0;
        }
        memcpy(C, Cn, sizeof C);
        memmove(B + 1, B, sizeof(unsigned) * (CAP - 1)); /* the skipped odd step */
        B[0] = 0;
    }
    if (L > t) return 0;
    return chien_apply(c, C, pdeg(C, CAP - 1), word, answer);
}

/* ------------------------------------------------------------ Kaneko search */
typedef struct {
    const orc_code *c;
    const double *a;      /* |alpha_i| by position            */
    const int *ord;       /* positions sorted by |alpha| asc  */
    const unsigned char *yH, *x;
    long m, m0;
} kctx;

/* calcRightSide, src/KanekoKernelProcessor.cpp:54-67 */
static double calc_right_side(const kctx *k) {
    const long n = k->c->n, t = k->c->t;
    long border = (2 * t + 1) - (k->m + k->m0) / 2;
    double l = 0;
    long i = 0, j = 0;
    while (i < border && j < n) {
        int p = k->ord[j];
        if (k->yH[p] == k->x[p]) { l += k->a[p]; ++i; }
        ++j;
    }
    return l;
}
/* calcT(j), :110-126. Callers never use the value at j = n - t (out of range). */
static double calc_T(const kctx *k, long j) {
    const long n = k->c->n, t = k->c->t;
    long border = t - (k->m + k->m0) / 2;
    double l = 0;
    long i = 0, q = 0;
    while (i < border && q < n) {
        int p = k->ord[q];
        if (k->yH[p] == k->x[p]) { l += k->a[p]; ++i; }
        ++q;
    }
    for (i = 0; i <= t; ++i) l += (j + i < n) ? k->a[k->ord[j + i]] : 0.0;
    return l;
}

/* decode(answer, word, res), src/KanekoKernelProcessor.cpp:335-407 */
void orc_kaneko_decode(const orc_code *c, double s2, int J, const double *y,
                       unsigned char *res, double *l0_out, orc_stats *st) {
    const long n = c->n, t = c->t;
    double a[ORC_MAXN + 1];
    unsigned char yH[ORC_MAXN + 1], e[ORC_MAXN + 1], x[ORC_MAXN + 1];
    int ord[ORC_MAXN + 1];
    orc_stats s;
    memset(&s, 0, sizeof s);
    /* prologue :336-343 */
    for (long i = 0; i < n; ++i) {
        double al = 2 * y[i] / s2;
        a[i] = fabs(al);
        yH[i] = (al <= 0.0) ? 0 : 1;
        ord[i] = (int)i;
    }
    /* insertion sort by (|alpha|, index): stable ascending order */
    for (long i = 1; i < n; ++i) {
        int p = ord[i];
        long j = i - 1;
        while (j >= 0 && a[ord[j]] > a[p]) { ord[j + 1] = ord[j]; --j; }
        ord[j + 1] = p;
    }
    kctx k = {c, a, ord, yH, x, 0, 0};
    long i = 0, j = 0, T = n;
    double l0 = DBL_MAX;
    int firstOK = 1;
    /* loop bound (1 << T) - 1 in 32-bit int as shipped (-O0 == -O2 -fwrapv): :361 */
#define BOUND(T_) ((long)((1UL << ((T_) & 31)) - 1UL))
    while (i < BOUND(T)) {
        memcpy(e, yH, (size_t)n); /* calcError(i) ^ yH, :36-51, :362-365 */
        for (long b = 0, v = i; v > 0; ++b, v >>= 1)
            if (v & 1) e[ord[b]] ^= 1;
        s.decodes++;
        int ok = orc_alg_decode(c, e, x);
        if (!i && !ok) firstOK = 0;
        if (ok) {
            long mm = 0;
            for (long q = 0; q < n; ++q) mm += yH[q] != x[q]; /* calcM :89-97 */
            k.m = mm;
            if (!i || !firstOK) k.m0 = mm;
            double l = 0; /* calcL :69-77 (index order) */
            for (long q = 0; q < n; ++q)
                if (yH[q] != x[q]) l += a[q];
            if (l < l0) {
                memcpy(res, x, (size_t)n);
                l0 = l;
                s.accepted = 1;
                if (l < calc_right_side(&k)) {
                    s.returned = 1;
                    break;
                }
                while (j <= n - 1 - t && l >= calc_T(&k, j)) { ++j; ++s.jsteps; }
                T = (J >= 0 && j > J) ? J : j;
                j = 0;
                ++s.improvements;
            }
        }
        ++i;
        ++s.iters;
    }
#undef BOUND
    s.cmp = s.iters * (uint64_t)(n + 6) + s.jsteps + s.improvements;
    s.sum = s.iters * (uint64_t)(n + 1) + s.jsteps;
    if (l0_out) *l0_out = l0;
    if (st) *st = s;
}

/* ------------------------------------------------------ batch (threaded) */
typedef struct {
    const orc_code *c;
    double s2;
    int J;
    const double *Y;
    long B;
    unsigned char *res, *acc;
    double *l0;
    uint64_t *st6;
    long next; /* next unclaimed row (claimed in chunks under `mu`) */
    pthread_mutex_t mu;
} orc_batch_job;

static void *orc_batch_worker(void *arg) {
    orc_batch_job *j = (orc_batch_job *)arg;
    const long n = j->c->n, chunk = 16;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const long b0 = j->next;
        j->next += chunk;
        pthread_mutex_unlock(&j->mu);
        if (b0 >= j->B) break;
        const long b1 = b0 + chunk < j->B ? b0 + chunk : j->B;
        for (long b = b0; b < b1; ++b) {
            orc_stats s;
            orc_kaneko_decode(j->c, j->s2, j->J, j->Y + b * n, j->res + b * n, &j->l0[b], &s);
            uint64_t *o = j->st6 + 6 * b;
            o[0] = s.decodes; o[1] = s.cmp; o[2] = s.sum;
            o[3] = s.iters; o[4] = s.jsteps; o[5] = s.improvements;
            j->acc[b] = (unsigned char)s.accepted;
        }
    }
    return NULL;
}

void orc_kaneko_batch(const orc_code *c, double s2, int J, const double *Y, long B,
                      unsigned char *res, double *l0, uint64_t *stats6, unsigned char *acc,
                      int threads) {
    enum { MAXTH = 256 };
    if (threads < 1) threads = 1;
    if (threads > MAXTH) threads = MAXTH;
    pthread_t th[MAXTH];
    int started[MAXTH] = {0};
    /* rows are claimed dynamically: a heavy codeword (up to 2^31 - 1 test patterns) must not
     * hold up a statically assigned range */
    orc_batch_job job = {c, s2, J, Y, B, res, acc, l0, stats6, 0, PTHREAD_MUTEX_INITIALIZER};
    for (int q = 1; q < threads; ++q)
        started[q] = pthread_create(&th[q], NULL, orc_batch_worker, &job) == 0;
    orc_batch_worker(&job);
    for (int q = 1; q < threads; ++q)
        if (started[q]) pthread_join(th[q], NULL);
}

/* ------------------------------------------------------------------- sweep */
/* fun(), src/dataForPlot.cpp:16-116 (COUNT on, DEBUG off). Note the reference
 * quirks kept here: countE is never reset (:20,95); `decoded` is reused across
 * words and is only overwritten on acceptance. */
long orc_sweep(const orc_code *c, double decoder_snr_db, int J, long p, long e,
               double max_snr, uint64_t seed, char *out, long cap) {
    const int n = c->n, k = c->k;
    orc_rng rng;
    orc_rng_seed(&rng, seed);
    double sd0 = orc_sigma(c, decoder_snr_db);
    double s2 = pow(sd0, 2);
    unsigned char info[ORC_MAXN + 1], tx[ORC_MAXN + 1], dec[ORC_MAXN + 1] = {0};
    double y[ORC_MAXN + 1];
    int count = 0, countErr = 0, countE = 0;
    uint64_t wordCount = 0, D = 0, Cc = 0, Ss = 0;
    long off = 0;
    for (double stnr = 0.0; stnr <= max_snr; stnr += 0.5) {
        while (count < p && countErr < e) {
            double sd = orc_sigma(c, stnr);
            orc_gen_info(&rng, info, k);
            orc_encode(c, info, tx);
            orc_add_noise(&rng, sd, tx, y, n);
            orc_stats st;
            orc_kaneko_decode(c, s2, J, y, dec, NULL, &st);
            D += st.decodes; Cc += st.cmp; Ss += st.sum;
            if (memcmp(tx, dec, (size_t)n)) ++countErr;
            for (int q = 0; q < n; ++q) countE += tx[q] != dec[q];
            ++count;
            ++wordCount;
        }
        int w = snprintf(out + off, (size_t)(cap - off), "%g,%g,%g,%g,%g,%g\n", stnr,
                         ((double)countErr) / count, ((double)countE) / count / n,
                         ((double)D) / wordCount, ((double)Cc) / wordCount,
                         ((double)Ss) / wordCount);
        if (w < 0 || off + w >= cap) return -1;
        off += w;
        D = Cc = Ss = 0;
        wordCount = 0;
        count = 0;
        countErr = 0;
    }
    return off;
}

/* ------------------------------------------------------- stream helpers (tests) */
uint64_t orc_stream_draws(const orc_code *c, uint64_t *state, long count, double snr_db) {
    /* counts minstd() calls by re-deriving them: the engine is x <- 16807 x mod (2^31 - 1),
     * so the draws between two states are found by stepping a copy alongside */
    orc_rng r = {*state}, probe;
    unsigned char info[ORC_MAXN + 1], tx[ORC_MAXN + 1];
    double y[ORC_MAXN + 1];
    const double sd = orc_sigma(c, snr_db);
    uint64_t draws = 0;
    for (long w = 0; w < count; ++w) {
        probe = r;
        orc_gen_info(&r, info, c->k);            /* bchCoder.cpp:236-240 */
        orc_encode(c, info, tx);
        orc_add_noise(&r, sd, tx, y, c->n);      /* bchCoder.cpp:243-250 */
        while (probe.x != r.x) {                 /* the draws this word consumed */
            probe.x = (probe.x * 16807u) % 2147483647u;
            ++draws;
        }
    }
    *state = r.x;
    return draws;
}

void orc_sweep_block(const orc_code *c, double decoder_snr_db, int J, double snr_db, uint64_t *state,
                     long skip, long B, unsigned char *tx, unsigned char *res, unsigned char *acc,
                     uint64_t *ops, uint64_t *states) {
    orc_rng r = {*state};
    unsigned char info[ORC_MAXN + 1], junk[ORC_MAXN + 1];
    double y[ORC_MAXN + 1];
    const double sd = orc_sigma(c, snr_db), s2 = pow(orc_sigma(c, decoder_snr_db), 2);
    const int n = c->n;
    for (long w = 0; w < skip + B; ++w) {
        unsigned char *row = w < skip ? junk : tx + (w - skip) * n;
        orc_gen_info(&r, info, c->k);            /* dataForPlot.cpp:47-50 */
        orc_encode(c, info, row);
        orc_add_noise(&r, sd, row, y, n);
        if (w < skip) continue;
        const long b = w - skip;
        orc_stats st;
        memset(res + b * n, 0, (size_t)n);
        orc_kaneko_decode(c, s2, J, y, res + b * n, NULL, &st);  /* :52 */
        acc[b] = (unsigned char)st.accepted;
        ops[3 * b] = st.decodes;
        ops[3 * b + 1] = st.cmp;
        ops[3 * b + 2] = st.sum;
        states[b] = r.x;
    }
    *state = r.x;
}

/* fun()'s loop body over the words of a stretch of `draws` engine draws from word start *state
 * (advanced): words generated one by one (their draws counted by stepping a copy of the
 * engine, as orc_stream_draws) until exactly `draws` are consumed. Returns the word count,
 * -1 if the stretch does not end on a word boundary or holds more than max_words words. */
long orc_sweep_range(const orc_code *c, double decoder_snr_db, int J, double snr_db, uint64_t *state,
                     uint64_t draws, long max_words, unsigned char *tx, unsigned char *res, unsigned char *acc,
                     uint64_t *ops, uint64_t *states) {
    orc_rng r = {*state}, probe;
    unsigned char info[ORC_MAXN + 1];
    double y[ORC_MAXN + 1];
    const double sd = orc_sigma(c, snr_db), s2 = pow(orc_sigma(c, decoder_snr_db), 2);
    const int n = c->n;
    uint64_t used = 0;
    long b = 0;
    while (used < draws) {
        if (b >= max_words) return -1;
        probe = r;
        orc_gen_info(&r, info, c->k);            /* dataForPlot.cpp:47-50 */
        orc_encode(c, info, tx + b * n);
        orc_add_noise(&r, sd, tx + b * n, y, n);
        while (probe.x != r.x) {
            probe.x = (probe.x * 16807u) % 2147483647u;
            ++used;
        }
        orc_stats st;
        memset(res + b * n, 0, (size_t)n);
        orc_kaneko_decode(c, s2, J, y, res + b * n, NULL, &st);  /* :52 */
        acc[b] = (unsigned char)st.accepted;
        ops[3 * b] = st.decodes;
        ops[3 * b + 1] = st.cmp;
        ops[3 * b + 2] = st.sum;
        states[b] = r.x;
        ++b;
    }
    if (used != draws) return -1;
    *state = r.x;
    return b;
}

