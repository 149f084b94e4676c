/* polar_oracle.c -- CPU restatement of the reference's vendored SC-list decoder for polar
 * codes over mixed binary kernels. TEST INFRASTRUCTURE (the GPU path's checker): built into
 * oracle/build/libpolar_oracle.so and loaded only by tests/.
 *
 * Follows (paths in the reference repo; the library under out/external is vendored and
 * never built by the reference itself):
 *   spec format, encoder, info extraction  out/external/MixedKernelEncoder.cpp:7-98, :142-177, :209-238
 *   dynamic-freezing masks                 out/external/KernelListEngine.cpp:6-39
 *   list decoder                           out/external/MixedKernelListDecoder.cpp:61-185, :211-268
 *   S / C recursions                       out/external/KernelListEngine.cpp:266-315, :370-447
 *   path-index stack                       out/external/TVMemoryEngine.cpp:85-142, headers/external/misc.h:212-226
 *   Arikan f / g                           out/external/SoftProcessing.cpp:39-80, headers/external/KernProc.h:89-102
 *   matrix kernels                         out/external/Kernel.cpp:93-176 (file, inverse), LinAlg.cpp:685-709
 *   kernel LLRs of a matrix kernel         out/external/TrellisKernelProcessor.cpp:234-294 (min-sum Viterbi)
 * A cloned path gets copies of its parent's arrays instead of the reference's copy-on-write
 * (TVMemoryEngine, KernelListEngine.cpp:318-367): every array a path reads holds the same
 * values either way. The trellis min-sum is evaluated by enumerating the coset: each
 * word's metric is a left-to-right float sum of |Y| over disagreeing positions, and min
 * commutes with adding a constant under round-to-nearest, so the minimum is the trellis's
 * bit for bit.
 *
 * PARITY UNPINNED: the vendored library needs GSL, Windows.h, MSVC-only constructs and 10
 * headers absent from the reference, and no fixtures exist; this file is
 * checked by properties in tests/test_polar_oracle.py.
 */
#include "polar_oracle.h"

#include <ctype.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void setmsg(char *msg, int len, const char *fmt, ...) {
    if (!msg || len <= 0) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, (size_t)len, fmt, ap);
    va_end(ap);
}

/* ------------------------------------------------------------------- tokens */
typedef struct {
    const char *p;
} tok_t;

static int next_tok(tok_t *t, char *buf, int cap) {
    while (*t->p && isspace((unsigned char)*t->p)) t->p++;
    if (!*t->p) return 0;
    int n = 0;
    while (*t->p && !isspace((unsigned char)*t->p)) {
        if (n < cap - 1) buf[n++] = *t->p;
        t->p++;
    }
    buf[n] = 0;
    return 1;
}

static int next_int(tok_t *t, int *v) {
    char b[64], *e;
    if (!next_tok(t, b, sizeof b)) return 0;
    long x = strtol(b, &e, 10);
    if (*e) return 0;
    *v = (int)x;
    return 1;
}

/* ------------------------------------------------------------------ kernels */
/* GF(2) inverse by Gauss-Jordan (the matrix Kernel.cpp:155-176 computes) */
static int gf2_inverse(int n, const uint8_t *K, uint8_t *inv) {
    static uint8_t a[PLR_MAXKERNEL][2 * PLR_MAXKERNEL];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            a[i][j] = K[i * n + j];
            a[i][n + j] = (uint8_t)(i == j);
        }
    for (int c = 0; c < n; ++c) {
        int p = c;
        while (p < n && !a[p][c]) ++p;
        if (p == n) return -1; /* "Kernel is singular" (:165) */
        if (p != c)
            for (int j = 0; j < 2 * n; ++j) {
                uint8_t x = a[p][j];
                a[p][j] = a[c][j];
                a[c][j] = x;
            }
        for (int r = 0; r < n; ++r)
            if (r != c && a[r][c])
                for (int j = 0; j < 2 * n; ++j) a[r][j] ^= a[c][j];
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) inv[i * n + j] = a[i][n + j];
    return 0;
}

/* GetKernelByName (Kernel.cpp:235-252): "A" (any case) or a matrix file "-path" / "<path"
 * holding the size and size^2 entries (Kernel.cpp:93-107). "G" and "A5" are not restated. */
static int kernel_by_name(plr_kernel *k, const char *name, const char *kdir, char *msg, int ml) {
    memset(k, 0, sizeof *k);
    if ((name[0] == 'A' || name[0] == 'a') && name[1] == 0) {
        k->size = 2;
        k->arikan = 1;
        k->K[0] = 1; k->K[1] = 0; k->K[2] = 1; k->K[3] = 1; /* Kernel.cpp:8-12 */
        memcpy(k->Kinv, k->K, 4);                           /* InverseMultiply == Multiply */
        return 0;
    }
    if (name[0] == '-' || name[0] == '<') {
        char path[1024];
        if (name[1] == '/' || !kdir || !kdir[0])
            snprintf(path, sizeof path, "%s", name + 1);
        else
            snprintf(path, sizeof path, "%s/%s", kdir, name + 1);
        FILE *f = fopen(path, "r");
        if (!f) {
            setmsg(msg, ml, "Error reading kernel file %s", path);
            return -1;
        }
        int n = 0;
        if (fscanf(f, "%d", &n) != 1 || n < 2 || n > PLR_MAXKERNEL) {
            fclose(f);
            setmsg(msg, ml, "Error reading kernel file %s (size)", path);
            return -1;
        }
        for (int i = 0; i < n * n; ++i) {
            unsigned c;
            if (fscanf(f, "%u", &c) != 1) {
                fclose(f);
                setmsg(msg, ml, "Error parsing kernel file %s", path);
                return -1;
            }
            k->K[i] = (uint8_t)(c != 0);
        }
        fclose(f);
        k->size = n;
        if (gf2_inverse(n, k->K, k->Kinv)) {
            setmsg(msg, ml, "Kernel is singular (%s)", path);
            return -1;
        }
        return 0;
    }
    setmsg(msg, ml, "Unknown kernel %s", name);
    return -2;
}

/* (y_i, y_{i+d}, ...) = (x_i, x_{i+d}, ...) M, 0 <= i < d (Kernel.h:31-36, LinAlg.cpp:685-709) */
static void kmul(int l, const uint8_t *M, int d, const uint8_t *x, uint8_t *y) {
    memset(y, 0, (size_t)l * (size_t)d);
    for (int j = 0; j < l; ++j)
        for (int i = 0; i < l; ++i)
            if (M[j * l + i])
                for (int s = 0; s < d; ++s) y[i * d + s] ^= x[j * d + s];
}

/* --------------------------------------------------------------------- spec */
plr_code *plr_create(const char *spec, const char *kdir, char *msg, int ml) {
    plr_code *P = (plr_code *)calloc(1, sizeof *P);
    if (!P) return NULL;
    tok_t t = {spec};
    if (!next_int(&t, &P->N) || !next_int(&t, &P->K) || !next_int(&t, &P->dmin) ||
        !next_int(&t, &P->layers) || !next_int(&t, &P->nshort) || !next_int(&t, &P->npunct)) {
        setmsg(msg, ml, "Error reading file header");
        goto bad;
    }
    if (P->K > P->N || P->K < 0 || P->N <= 0) {
        setmsg(msg, ml, "Code dimension cannot exceed code length");
        goto bad;
    }
    if (P->layers < 1 || P->layers > PLR_MAXLAYERS) {
        setmsg(msg, ml, "bad number of layers %d", P->layers);
        goto bad;
    }
    P->U = 1;
    for (int i = 0; i < P->layers; ++i) {
        char name[512];
        if (!next_tok(&t, name, sizeof name)) {
            setmsg(msg, ml, "missing kernel name %d", i);
            goto bad;
        }
        if (kernel_by_name(&P->kern[i], name, kdir, msg, ml)) goto bad;
        P->U *= P->kern[i].size;
        if (P->U > PLR_MAXU) {
            setmsg(msg, ml, "length %d exceeds %d", P->U, PLR_MAXU);
            goto bad;
        }
    }
    if (P->N + P->nshort + P->npunct != P->U) {
        setmsg(msg, ml, "Code length mismatch");
        goto bad;
    }
    for (int i = 0; i < P->nshort + P->npunct; ++i) {
        int s;
        if (!next_int(&t, &s) || s < 0 || s >= P->U) {
            setmsg(msg, ml, "Invalid shortened / punctured symbol");
            goto bad;
        }
        P->symtype[s] = (uint8_t)(i < P->nshort ? 1 : 2);
    }
    for (int i = 0; i < P->U; ++i) {
        P->decision[i] = -1;
        P->dfbit[i] = -1;
    }
    int nt = 0;
    for (int c = 0; c < P->U - P->K; ++c) {
        int w;
        if (!next_int(&t, &w) || w < 1) {
            setmsg(msg, ml, "Error reading freezing constraint %d", c);
            goto bad;
        }
        P->fc_start[c] = nt;
        for (int j = 0; j < w; ++j) {
            int v;
            if (!next_int(&t, &v) || v < 0 || v >= P->U || nt >= PLR_MAXU * 8 ||
                (j > 0 && v <= P->fc_terms[nt - 1])) {
                setmsg(msg, ml, "Invalid freezing constraint %d", c);
                goto bad;
            }
            P->fc_terms[nt++] = v;
        }
        const int last = P->fc_terms[nt - 1];
        if (P->decision[last] != -1) {
            setmsg(msg, ml, "Duplicate freezing constraint on symbol %d", last);
            goto bad;
        }
        P->decision[last] = c;
    }
    P->fc_start[P->U - P->K] = nt;
    P->outer[0] = P->U;
    for (int i = 0; i < P->layers; ++i) P->outer[i + 1] = P->outer[i] / P->kern[i].size;
    /* dynamic-freezing value bits (KernelListEngine.cpp:6-39): a constraint gets the least
     * free mask bit at its first term and releases it at its frozen symbol */
    uint64_t avail = ~0ull;
    for (int i = 0; i < P->U; ++i) {
        if (P->dfbit[i] >= 0) avail |= 1ull << P->dfbit[i];
        for (int j = i + 1; j < P->U; ++j) {
            const int c = P->decision[j];
            if (c < 0 || P->fc_terms[P->fc_start[c]] != i) continue;
            if (!avail) {
                setmsg(msg, ml, "Too many dynamic freezing constraints are simultaneously active");
                goto bad;
            }
            const int B = __builtin_ctzll(avail);
            avail &= ~(1ull << B);
            P->dfbit[j] = B;
            for (int q = P->fc_start[c]; P->fc_terms[q] != j; ++q) P->dfcorr[P->fc_terms[q]] ^= 1ull << B;
            P->dfcorr[j] ^= 1ull << B;
        }
    }
    return P;
bad:
    free(P);
    return NULL;
}

void plr_destroy(plr_code *P) { free(P); }

void plr_dims(const plr_code *P, int *N, int *K, int *U) {
    if (N) *N = P->N;
    if (K) *K = P->K;
    if (U) *U = P->U;
}

/* ---------------------------------------------------------- encode / extract */
void plr_encode_unshortened(const plr_code *P, const uint8_t *info, uint8_t *ucw) {
    const int U = P->U;
    uint8_t *a = (uint8_t *)malloc((size_t)U), *b = (uint8_t *)malloc((size_t)U);
    int k = 0;
    for (int i = 0; i < U; ++i) { /* frozen symbols from their constraints (:147-157) */
        const int c = P->decision[i];
        if (c >= 0) {
            uint8_t v = 0;
            for (int q = P->fc_start[c]; P->fc_terms[q] != i; ++q) v ^= a[P->fc_terms[q]];
            a[i] = v;
        } else {
            a[i] = info[k++] & 1;
        }
    }
    int stride = 1; /* innermost layer first (:159-170) */
    for (int L = P->layers - 1; L >= 0; --L) {
        const int l = P->kern[L].size, next = stride * l;
        for (int blk = 0; blk < U / next; ++blk) kmul(l, P->kern[L].K, stride, a + blk * next, b + blk * next);
        uint8_t *x = a; a = b; b = x;
        stride = next;
    }
    memcpy(ucw, a, (size_t)U);
    free(a);
    free(b);
}

void plr_encode(const plr_code *P, const uint8_t *info, uint8_t *cw) {
    uint8_t *u = (uint8_t *)malloc((size_t)P->U);
    plr_encode_unshortened(P, info, u);
    for (int i = 0, j = 0; i < P->U; ++i) /* Shorten (:104-130) */
        if (P->symtype[i] == 0) cw[j++] = u[i];
    free(u);
}

void plr_extract_info(const plr_code *P, const uint8_t *ucw, uint8_t *info) {
    const int U = P->U;
    uint8_t *a = (uint8_t *)malloc((size_t)U), *b = (uint8_t *)malloc((size_t)U);
    memcpy(a, ucw, (size_t)U);
    int nb = 1, prev = U;
    for (int L = 0; L < P->layers; ++L) {
        const int l = P->kern[L].size, st = prev / l;
        for (int blk = 0; blk < nb; ++blk) kmul(l, P->kern[L].Kinv, st, a + blk * prev, b + blk * prev);
        prev = st;
        nb *= l;
        uint8_t *x = a; a = b; b = x;
    }
    for (int i = 0, k = 0; i < U; ++i)
        if (P->decision[i] < 0) info[k++] = a[i];
    free(a);
    free(b);
}

/* ------------------------------------------------------------- kernel LLRs */
/* SoftXOR / SoftCombine (SoftProcessing.cpp:39-80): a = first block, b = second block */
static void arikan_llr(int phase, int d, const uint8_t *known, const float *src, float *dst) {
    for (int s = 0; s < d; ++s) {
        const float a = src[s], b = src[d + s];
        if (!phase) {
            const float fa = fabsf(a), fb = fabsf(b);
            const float m = fa < fb ? fa : fb;
            dst[s] = ((signbit(a) != 0) != (signbit(b) != 0)) ? -m : m;
        } else {
            dst[s] = known[s] ? b - a : b + a;
        }
    }
}

/* The trellis itself, for cosets too large to enumerate: CTrellisKernelProcessor's
 * construction (TrellisKernelProcessor.cpp:69-179, MinimumSpan :7-67) and walk (:260-292)
 * state by state, float metrics. Same value as the enumeration (min commutes with the
 * monotone float add along each word's left-to-right sum). */
typedef unsigned __int128 u128; /* kernel rows plus the extension column (size <= 64) */

static float trellis_minsum_llr(const plr_kernel *k, int phase, const float *y) {
    const unsigned l = (unsigned)k->size, N = l + 1, K = l - (unsigned)phase;
    u128 M[PLR_MAXKERNEL] = {0};
    for (unsigned i = 0; i < K; ++i) {
        M[i] = 0;
        for (unsigned j = 0; j < l; ++j)
            if (k->K[(phase + i) * l + j]) M[i] |= (u128)1 << j;
    }
    M[0] |= (u128)1 << l;
    unsigned start[PLR_MAXKERNEL + 1], end[PLR_MAXKERNEL + 1], C = 0;
    for (unsigned c = 0; c < N; ++c) start[c] = end[c] = ~0u;
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
        for (unsigned j = i + 1; j < K; ++j)
            if ((M[j] >> C) & 1) M[j] ^= M[i];
    }
    for (int i = (int)K - 1; i >= 0; --i)
        for (int j = (int)N - 1; j >= 0; --j)
            if ((M[i] >> j) & 1) {
                end[j] = (unsigned)i;
                for (int s = 0; s < i; ++s)
                    if ((M[s] >> j) & 1) M[s] ^= M[i];
                break;
            }
    unsigned most = 0;
    for (unsigned j = 0, a = 0; j < l; ++j) { /* states of the widest depth, edges included */
        if (a + 1 > most) most = a + 1;
        a += (start[j] != ~0u) - (end[j] != ~0u);
    }
    const size_t cap = (size_t)1 << (most + 1);
    /* labels are read at positions < l only: a state's word fits 64 bits without the extension */
    uint64_t *cw0 = calloc(cap, 8), *cw1 = calloc(cap, 8);
    float *m0 = malloc(cap * 4), *m1 = malloc(cap * 4);
    unsigned active[PLR_MAXKERNEL + 1], na = 0;
    m0[0] = 0.0f;
    for (unsigned j = 0; j < l; ++j) {
        unsigned B = na;
        for (unsigned q = 0; q < na; ++q)
            if (active[q] == end[j]) { B = q; break; }
        const uint64_t emask = (end[j] == ~0u) ? ~0ull : ((1ull << B) - 1);
        const uint64_t ns = 1ull << na;
        const unsigned na1 = na + (start[j] != ~0u) - (end[j] != ~0u);
        for (uint64_t S = 0; S < (1ull << na1); ++S) m1[S] = INFINITY;
        const float Y = y[j], aY = fabsf(Y);
        const unsigned HD = Y < 0;
        const uint64_t rowj = start[j] == ~0u ? 0 : (uint64_t)M[start[j]];
        for (uint64_t S = 0; S < ns; ++S) {
            uint64_t nx[2];
            uint64_t lab[2];
            int ne;
            if (start[j] == ~0u) {
                nx[0] = (S & emask) | ((S >> 1) & ~emask);
                lab[0] = (cw0[S] >> j) & 1;
                cw1[nx[0]] = cw0[S];
                ne = 1;
            } else {
                uint64_t n0 = S, n1 = S ^ (1ull << na);
                nx[0] = (n0 & emask) | ((n0 >> 1) & ~emask);
                nx[1] = (n1 & emask) | ((n1 >> 1) & ~emask);
                const uint64_t c1 = cw0[S] ^ rowj;
                cw1[nx[0]] = cw0[S];
                cw1[nx[1]] = c1;
                lab[0] = (cw0[S] >> j) & 1;
                lab[1] = (c1 >> j) & 1;
                ne = 2;
            }
            for (int e = 0; e < ne; ++e) {
                const float sc = (lab[e] ^ HD) ? m0[S] + aY : m0[S];
                if (sc < m1[nx[e]]) m1[nx[e]] = sc;
            }
        }
        if (start[j] != ~0u) active[na++] = start[j];
        if (end[j] != ~0u) {
            memmove(active + B, active + B + 1, sizeof(unsigned) * (na - B - 1));
            --na;
        }
        { uint64_t *t = cw0; cw0 = cw1; cw1 = t; }
        { float *t = m0; m0 = m1; m1 = t; }
    }
    const float r = m0[1] - m0[0];
    free(cw0); free(cw1); free(m0); free(m1);
    return r;
}

/* metric of a word: the left-to-right float sum of |y| over its disagreeing positions
 * (TrellisKernelProcessor.cpp:279-282 along one path) */
static float word_metric(uint64_t dis, const float *ay, int l) {
    float m = 0.0f;
    for (int j = 0; j < l; ++j)
        if ((dis >> j) & 1) m += ay[j];
    return m;
}

static void kernel_rows(const plr_kernel *k, uint64_t *rows) {
    const int l = k->size;
    for (int r = 0; r < l; ++r) {
        rows[r] = 0;
        for (int j = 0; j < l; ++j)
            if (k->K[r * l + j]) rows[r] |= 1ull << j;
    }
}

/* the coset enumerated: every word of rows phase+1..l-1 (Gray order, one row per step) */
static float enum_minsum_llr(const plr_kernel *k, int phase, const float *y) {
    const int l = k->size, nfree = l - phase - 1;
    uint64_t rows[PLR_MAXKERNEL], hd = 0;
    float ay[PLR_MAXKERNEL];
    kernel_rows(k, rows);
    for (int j = 0; j < l; ++j) {
        if (y[j] < 0) hd |= 1ull << j; /* HD = Y < 0 (TrellisKernelProcessor.cpp:276) */
        ay[j] = fabsf(y[j]);
    }
    float best[2] = {INFINITY, INFINITY};
    uint64_t c = 0;
    for (uint64_t v = 0; v < (1ull << nfree); ++v) {
        if (v) c ^= rows[phase + 1 + __builtin_ctzll(v)];
        for (int b = 0; b < 2; ++b) {
            const float m = word_metric((b ? c ^ rows[phase] : c) ^ hd, ay, l);
            if (m < best[b]) best[b] = m;
        }
    }
    return best[1] - best[0]; /* :292 */
}

/* Exact ordered-statistics search, each half b of the coset on its own: Gauss-Jordan on rows
 * phase+1..l-1 over the positions in decreasing |y| gives the most reliable basis (pivots); a
 * word of half b is fixed by its pivot values, and the one matching the hard decision there
 * is the root. Flipping a set E of pivots costs at least the sum of their |y| (they then
 * disagree), so a depth-first search over E, cheapest pivot first, pruning every subtree whose
 * flip cost exceeds the best metric found (less a float-rounding margin), visits every word
 * that can be the minimum: the value is the enumeration's. */
static __thread long ml_nodes_last, ml_nodes_total, ml_calls_total;
long plr_ml_nodes(void) { return ml_nodes_last; }
/* totals over this thread's searches since the last call (diagnostics) */
long plr_ml_nodes_total(long *calls) {
    const long t = ml_nodes_total;
    if (calls) *calls = ml_calls_total;
    ml_nodes_total = ml_calls_total = 0;
    return t;
}

static float ml_minsum_llr(const plr_kernel *k, int phase, const float *y) {
    const int l = k->size, nf = l - phase - 1;
    uint64_t rows[PLR_MAXKERNEL], G[PLR_MAXKERNEL], hd = 0;
    float ay[PLR_MAXKERNEL];
    int piv[PLR_MAXKERNEL], used[PLR_MAXKERNEL] = {0}, ord[PLR_MAXKERNEL], po[PLR_MAXKERNEL];
    kernel_rows(k, rows);
    for (int j = 0; j < l; ++j) {
        if (y[j] < 0) hd |= 1ull << j;
        ay[j] = fabsf(y[j]);
        ord[j] = j;
    }
    for (int i = 1; i < l; ++i) { /* positions by decreasing |y| (insertion sort) */
        const int p = ord[i];
        int j = i - 1;
        while (j >= 0 && ay[ord[j]] < ay[p]) { ord[j + 1] = ord[j]; --j; }
        ord[j + 1] = p;
    }
    for (int i = 0; i < nf; ++i) G[i] = rows[phase + 1 + i];
    int np = 0;
    for (int s = 0; s < l && np < nf; ++s) {
        const int p = ord[s];
        int r = -1;
        for (int i = 0; i < nf; ++i)
            if (!used[i] && ((G[i] >> p) & 1)) { r = i; break; }
        if (r < 0) continue;
        used[r] = 1;
        piv[r] = p;
        po[nf - 1 - np] = r; /* found in decreasing |y|: po runs by increasing flip cost */
        ++np;
        for (int i = 0; i < nf; ++i)
            if (i != r && ((G[i] >> p) & 1)) G[i] ^= G[r];
    }
    /* a float sum of at most 64 non-negative terms is within 64 u (u = 2^-24) of the exact
     * sum: a subtree is pruned only when its exact cost exceeds best by more than that */
    const double shrink = 1.0 - 1.0 / 32768.0;
    /* U[i]: the non-pivot positions rows po[i..] can still change; below a word that has
     * taken pivots up to po[i - 1], every other non-pivot disagreement is fixed */
    uint64_t pivm = 0, U[PLR_MAXKERNEL + 1];
    for (int i = 0; i < nf; ++i) pivm |= 1ull << piv[i];
    const uint64_t lrb = ~pivm & (l == 64 ? ~0ull : ((1ull << l) - 1));
    U[nf] = 0;
    for (int i = nf - 1; i >= 0; --i) U[i] = U[i + 1] | (G[po[i]] & lrb);
    float best[2];
    typedef struct { uint64_t c; double lb; int i; } node;
    node *st = malloc(sizeof(node) * (size_t)(nf + 2));
    long nodes = 0;
    for (int b = 0; b < 2; ++b) {
        const uint64_t base = b ? rows[phase] : 0, target = hd ^ base;
        uint64_t c = base;
        for (int i = 0; i < nf; ++i)
            if ((target >> piv[i]) & 1) c ^= G[i];
        best[b] = word_metric(c ^ hd, ay, l);
        ++nodes;
        int sp = 0;
        if (nf > 0) st[sp++] = (node){c, 0.0, 0};
        while (sp) { /* (c, lb, i): the words c ^ G[po[j]] for j = i, i+1, ... and below them */
            const node n = st[--sp];
            for (int i = n.i; i < nf; ++i) {
                const double lb2 = n.lb + ay[piv[po[i]]];
                if (lb2 * shrink > best[b]) break; /* costs increase with i */
                const uint64_t c2 = n.c ^ G[po[i]];
                /* c2 and everything below it disagree at least at its fixed non-pivot positions */
                const double fx = word_metric((c2 ^ hd) & lrb & ~U[i + 1], ay, l);
                if ((lb2 + fx) * shrink > best[b]) continue;
                const float m = word_metric(c2 ^ hd, ay, l);
                ++nodes;
                if (m < best[b]) best[b] = m;
                if (i + 1 < nf) st[sp++] = (node){c2, lb2, i + 1};
            }
        }
    }
    free(st);
    ml_nodes_last = nodes;
    ml_nodes_total += nodes;
    ++ml_calls_total;
    return best[1] - best[0]; /* :292 */
}

/* cosets of more than 2^plr_trellis_nfree words go through the trellis (tests set it to
 * compare the two) when the kernel has at most 32 rows, else through the ordered-statistics
 * search (the reference's trellis processor takes kernels below 64 only) */
int plr_trellis_nfree = 12;

float plr_minsum_llr_by(const plr_kernel *k, int phase, const float *y, int method) {
    if (method == PLR_BY_ENUM) return enum_minsum_llr(k, phase, y);
    if (method == PLR_BY_TRELLIS) return trellis_minsum_llr(k, phase, y);
    return ml_minsum_llr(k, phase, y);
}

float plr_minsum_llr(const plr_kernel *k, int phase, const float *y) {
    const int l = k->size, nfree = l - phase - 1;
    if (nfree <= plr_trellis_nfree) return enum_minsum_llr(k, phase, y);
    return l <= 32 ? trellis_minsum_llr(k, phase, y) : ml_minsum_llr(k, phase, y);
}

/* CTrellisKernelProcessor::GetLLRs (:234-294): the offset state accumulates the known
 * inputs times their kernel rows; output LLRs flip sign where it is set. */
static void matrix_llr(const plr_kernel *k, int phase, int d, const uint8_t *known,
                       const float *src, float *dst, uint8_t *off) {
    const int l = k->size;
    if (!phase) {
        memset(off, 0, (size_t)l * (size_t)d);
    } else {
        for (int i = 0; i < l; ++i)
            if (k->K[(phase - 1) * l + i])
                for (int s = 0; s < d; ++s) off[i * d + s] ^= known[(phase - 1) * d + s];
    }
    float y[PLR_MAXKERNEL];
    for (int s = 0; s < d; ++s) {
        for (int j = 0; j < l; ++j) {
            const float v = src[j * d + s];
            y[j] = off[j * d + s] ? -v : v;
        }
        dst[s] = plr_minsum_llr(k, phase, y);
    }
}

/* ------------------------------------------------------------------ decoder */
typedef struct {
    float r;
    unsigned i;
} cand_t;

/* std::sort with std::greater<pair<float, unsigned>> (MixedKernelListDecoder.cpp:125,257,
 * headers/external/misc.h:166): descending score, then descending index */
static int cand_cmp(const void *pa, const void *pb) {
    const cand_t *x = (const cand_t *)pa, *y = (const cand_t *)pb;
    if (y->r < x->r) return -1;
    if (x->r < y->r) return 1;
    if (y->i < x->i) return -1;
    if (x->i < y->i) return 1;
    return 0;
}

typedef struct {
    const plr_code *P;
    int L, nl;
    int soff[PLR_MAXLAYERS + 1], ssize; /* per path: S layers 1..nl */
    int coff[PLR_MAXLAYERS + 1], csize; /* per path: C layers 0..nl */
    int ooff[PLR_MAXLAYERS], osize;     /* per path: kernel offset states, layers 0..nl-1 */
    float *S0, *S, *R;
    uint8_t *C, *O, *active;
    uint64_t *dfm;
    unsigned *stack;
} dec_t;

static float *S_of(dec_t *D, int l, int lam) {
    return lam == 0 ? D->S0 : D->S + (size_t)l * D->ssize + D->soff[lam];
}
static uint8_t *C_of(dec_t *D, int l, int lam) { return D->C + (size_t)l * D->csize + D->coff[lam]; }
static uint8_t *O_of(dec_t *D, int l, int j) { return D->O + (size_t)l * D->osize + D->ooff[j]; }

/* misc.h:206-226 */
static void st_push(unsigned x, unsigned *s) { s[++s[0]] = x; }
static unsigned st_pop(unsigned *s) {
    if (s[s[0]] == ~0u) {
        const unsigned v = --s[0];
        if (v > 0) s[s[0]] = ~0u;
        return v;
    }
    return s[s[0]--];
}

/* IterativelyCalcS (KernelListEngine.cpp:370-447) */
static float calc_s(dec_t *D, int l, unsigned phi) {
    const plr_code *P = D->P;
    int m = D->nl - 1;
    while (m > 0 && phi % (unsigned)P->kern[m].size == 0) {
        phi /= (unsigned)P->kern[m].size;
        --m;
    }
    for (int j = m; j < D->nl; ++j) {
        const int local = (j == m) ? (int)(phi % (unsigned)P->kern[j].size) : 0;
        const int d = P->outer[j + 1];
        const float *src = S_of(D, l, j);
        float *dst = S_of(D, l, j + 1);
        const uint8_t *known = C_of(D, l, j + 1);
        if (P->kern[j].arikan)
            arikan_llr(local, d, known, src, dst);
        else
            matrix_llr(&P->kern[j], local, d, known, src, dst, O_of(D, l, j));
    }
    return S_of(D, l, D->nl)[0];
}

/* IterativelyUpdateC (KernelListEngine.cpp:266-315) */
static void update_c(dec_t *D, int l, unsigned phi) {
    const plr_code *P = D->P;
    int lam = D->nl, stride = 1;
    while (lam > 0 && (phi + 1) % (unsigned)P->kern[lam - 1].size == 0) {
        const unsigned psi = phi / (unsigned)P->kern[lam - 1].size;
        const int next = stride * P->kern[lam - 1].size;
        const int phi0 = lam > 1 ? (int)(psi % (unsigned)P->kern[lam - 2].size) * next : 0;
        kmul(P->kern[lam - 1].size, P->kern[lam - 1].K, stride, C_of(D, l, lam), C_of(D, l, lam - 1) + phi0);
        stride = next;
        phi = psi;
        --lam;
    }
}

static void clone_arrays(dec_t *D, int from, int to) {
    memcpy(D->S + (size_t)to * D->ssize, D->S + (size_t)from * D->ssize, sizeof(float) * (size_t)D->ssize);
    memcpy(D->C + (size_t)to * D->csize, D->C + (size_t)from * D->csize, (size_t)D->csize);
    if (D->osize) memcpy(D->O + (size_t)to * D->osize, D->O + (size_t)from * D->osize, (size_t)D->osize);
}

int plr_decode(const plr_code *P, int L, const float *llr, uint8_t *info, uint8_t *cw,
               float *metric) {
    if (L < 1 || L > 1024) return -1;
    dec_t D;
    memset(&D, 0, sizeof D);
    D.P = P;
    D.L = L;
    D.nl = P->layers;
    int s = 0, c = 0, o = 0;
    for (int lam = 1; lam <= D.nl; ++lam) {
        D.soff[lam] = s;
        s += P->outer[lam];
    }
    for (int lam = 0; lam <= D.nl; ++lam) {
        D.coff[lam] = c;
        c += lam ? P->outer[lam] * P->kern[lam - 1].size : P->outer[0];
    }
    for (int j = 0; j < D.nl; ++j) {
        D.ooff[j] = o;
        if (!P->kern[j].arikan) o += P->kern[j].size * P->outer[j + 1];
    }
    D.ssize = s;
    D.csize = c;
    D.osize = o;
    D.S0 = (float *)calloc((size_t)P->U, sizeof(float));
    D.S = (float *)calloc((size_t)L * (size_t)(s ? s : 1), sizeof(float));
    D.C = (uint8_t *)calloc((size_t)L * (size_t)c, 1);
    D.O = (uint8_t *)calloc((size_t)L * (size_t)(o ? o : 1), 1);
    D.R = (float *)calloc((size_t)L, sizeof(float));
    D.dfm = (uint64_t *)calloc((size_t)L, sizeof(uint64_t));
    D.active = (uint8_t *)calloc((size_t)L, 1);
    D.stack = (unsigned *)calloc((size_t)L + 1, sizeof(unsigned));
    cand_t *buf = (cand_t *)calloc(2 * (size_t)L, sizeof(cand_t));
    uint8_t *cont = (uint8_t *)calloc((size_t)L, 1);
    /* Cleanup + AssignInitialPath (TVMemoryEngine.cpp:58-94) */
    D.stack[0] = (unsigned)L;
    D.stack[L] = ~0u;
    const unsigned pid = st_pop(D.stack);
    D.active[pid] = 1;
    /* LoadLLRs (MixedKernelEncoder.cpp:181-207) */
    for (int i = 0, I = 0; i < P->U; ++i) {
        switch (P->symtype[i]) {
            case 0: D.S0[i] = llr[I++]; break;
            case 1: D.S0[i] = 100000.0f; break; /* MTYPE_UPPER_BOUND, SeqConfigOrig.h:173 */
            default: D.S0[i] = 0.0f; break;
        }
    }
    const int lastsz = P->kern[D.nl - 1].size;
    for (unsigned phi = 0; phi < (unsigned)P->U; ++phi) {
        uint8_t *Cl;
        if (P->decision[phi] >= 0) { /* ContinuePathsFrozen (:61-98) */
            for (int l = 0; l < L; ++l) {
                if (!D.active[l]) continue;
                const float v = calc_s(&D, l, phi);
                uint8_t C = 0;
                if (P->dfbit[phi] >= 0) C = (uint8_t)((D.dfm[l] >> P->dfbit[phi]) & 1);
                if ((C > 0) ^ (v < 0)) D.R[l] -= fabsf(v);
                C_of(&D, l, D.nl)[phi % (unsigned)lastsz] = C;
                if (C) D.dfm[l] ^= P->dfcorr[phi];
                update_c(&D, l, phi);
            }
            continue;
        }
        /* ContinuePathsUnfrozen (:100-185) */
        int J = 0;
        for (int l = 0; l < L; ++l) {
            if (!D.active[l]) continue;
            const float v = calc_s(&D, l, phi);
            const unsigned Dd = v < 0;
            buf[J].r = D.R[l];
            buf[J].i = 2u * (unsigned)l + Dd;
            buf[J + 1].r = D.R[l] - fabsf(v);
            buf[J + 1].i = 2u * (unsigned)l + (Dd ^ 1u);
            J += 2;
        }
        qsort(buf, (size_t)J, sizeof(cand_t), cand_cmp);
        memset(cont, 0, (size_t)L);
        for (int i = 0; i < (J < L ? J : L); ++i) cont[buf[i].i >> 1] |= (uint8_t)(1u << (buf[i].i & 1));
        for (int i = 0; i < L; ++i)
            if (D.active[i] && !cont[i]) { /* KillPath */
                st_push((unsigned)i, D.stack);
                D.active[i] = 0;
            }
        for (int l = 0; l < L; ++l) {
            switch (cont[l]) {
                case 1:
                    C_of(&D, l, D.nl)[phi % (unsigned)lastsz] = 0;
                    break;
                case 2:
                    C_of(&D, l, D.nl)[phi % (unsigned)lastsz] = 1;
                    D.dfm[l] ^= P->dfcorr[phi];
                    break;
                case 3: {
                    const float v = S_of(&D, l, D.nl)[0];
                    const uint8_t C = v < 0;
                    C_of(&D, l, D.nl)[phi % (unsigned)lastsz] = C;
                    const unsigned l1 = st_pop(D.stack); /* ClonePath */
                    clone_arrays(&D, l, (int)l1);
                    Cl = C_of(&D, (int)l1, D.nl);
                    Cl[phi % (unsigned)lastsz] = (uint8_t)(C ^ 1);
                    D.active[l1] = 1;
                    D.R[l1] = D.R[l] - fabsf(v);
                    D.dfm[l1] = D.dfm[l];
                    if (C)
                        D.dfm[l] ^= P->dfcorr[phi];
                    else
                        D.dfm[l1] ^= P->dfcorr[phi];
                    break;
                }
                default:
                    break;
            }
        }
        for (int l = 0; l < L; ++l)
            if (D.active[l]) update_c(&D, l, phi);
    }
    /* final ordering and outputs (:249-267) */
    int J = 0;
    for (int l = 0; l < L; ++l)
        if (D.active[l]) {
            buf[J].r = D.R[l];
            buf[J].i = (unsigned)l;
            ++J;
        }
    qsort(buf, (size_t)J, sizeof(cand_t), cand_cmp);
    for (int r = 0; r < J; ++r) {
        const uint8_t *ucw = C_of(&D, (int)buf[r].i, 0);
        if (cw)
            for (int i = 0, j = 0; i < P->U; ++i)
                if (P->symtype[i] == 0) cw[(size_t)r * P->N + j++] = ucw[i];
        plr_extract_info(P, ucw, info + (size_t)r * P->K);
        if (metric) metric[r] = buf[r].r;
    }
    free(D.S0);
    free(D.S);
    free(D.C);
    free(D.O);
    free(D.R);
    free(D.dfm);
    free(D.active);
    free(D.stack);
    free(buf);
    free(cont);
    return J;
}
