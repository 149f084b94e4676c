/* scripts/proto_m8_skip.c -- experiment (not product): how much of the Kaneko loop on a long
 * code is re-decoding a codeword already found?
 *
 * A test pattern P whose word yH ^ P lies within distance t of a codeword c found by an
 * EARLIER pattern decodes to c (unique decoding, d >= 2t + 1), and l(c) >= l0 at that point,
 * so P cannot be an improvement (src/KanekoKernelProcessor.cpp:372-399: only l < l0 calls
 * calcRightSide / calcT; m0 changes on non-improving successes only matter at the next
 * improvement, where !firstOK sets m0 = m again). This counts, per codeword, the patterns
 * skipped by that test, how many of the rest pass Berlekamp-Massey (L <= t) and how many
 * succeed.  Build: gcc -O2 -o /tmp/proto_m8_skip scripts/proto_m8_skip.c -lm -lpthread
 */
#include "../oracle/bchk_oracle.c"

#include <stdlib.h>

static int bm_L(const orc_code *c, const unsigned char *word, int *deg_out) {
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
        memmove(B + 1, B, sizeof(unsigned) * (CAP - 1));
        B[0] = 0;
    }
    *deg_out = pdeg(C, CAP - 1);
    return L;
}

int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 8, t = argc > 2 ? atoi(argv[2]) : 15;
    const double snr = argc > 3 ? atof(argv[3]) : 5.0;
    const long words = argc > 4 ? atol(argv[4]) : 2000;
    const int J = argc > 5 ? atoi(argv[5]) : 15;
    orc_code c;
    orc_code_init(&c, m, t);
    const int n = c.n;
    const double sd0 = orc_sigma(&c, 0.5), s2 = pow(sd0, 2), sd = orc_sigma(&c, snr);
    orc_rng r;
    orc_rng_seed(&r, 1);
    unsigned char info[256], cw[256], e[256], x[256], yH[256], res[256];
    double y[256], a[256];
    int ord[256];
    long tot_dec = 0, tot_skip = 0, tot_bm = 0, tot_ok = 0, heavy = 0, heavy_dec = 0, heavy_rest = 0,
         heavy_bm = 0, deg_hist[40] = {0};
    for (long w = 0; w < words; ++w) {
        orc_gen_info(&r, info, c.k);
        orc_encode(&c, info, cw);
        orc_add_noise(&r, sd, cw, y, n);
        for (int i = 0; i < n; ++i) {
            double al = 2 * y[i] / s2;
            a[i] = fabs(al);
            yH[i] = al <= 0.0 ? 0 : 1;
            ord[i] = i;
        }
        for (int i = 1; i < n; ++i) {
            int p = ord[i], j = i - 1;
            while (j >= 0 && a[ord[j]] > a[p]) { ord[j + 1] = ord[j]; --j; }
            ord[j + 1] = p;
        }
        /* known codewords as D = yH ^ c: weight outside the first 31 sorted positions, and
         * the bit image over them */
        enum { KMAX = 64 };
        int ku[KMAX];
        uint32_t kr[KMAX];
        int nk = 0;
        kctx k = {&c, a, ord, yH, x, 0, 0};
        long i = 0, j = 0, T = n, dec = 0, skip = 0, bm = 0, okc = 0;
        double l0 = DBL_MAX;
        int firstOK = 1;
#define BOUND(T_) ((long)((1UL << ((T_) & 31)) - 1UL))
        while (i < BOUND(T)) {
            ++dec;
            int sk = 0;
            for (int q = 0; q < nk && !sk; ++q) sk = ku[q] + __builtin_popcount(kr[q] ^ (uint32_t)i) <= t;
            if (sk) { ++skip; ++i; continue; }
            memcpy(e, yH, (size_t)n);
            for (long b = 0, v = i; v > 0; ++b, v >>= 1)
                if (v & 1) e[ord[b]] ^= 1;
            int deg;
            const int L = bm_L(&c, e, &deg);
            if (L <= t) { ++bm; if (deg >= 0 && deg < 40) deg_hist[deg]++; }
            int ok = orc_alg_decode(&c, e, x);
            if (!i && !ok) firstOK = 0;
            if (ok) {
                ++okc;
                /* remember the codeword */
                int u = 0;
                uint32_t rb = 0;
                for (int q = 0; q < n; ++q) {
                    if (yH[ord[q]] == x[ord[q]]) continue;
                    if (q < 31) rb |= 1u << q; else ++u;
                }
                int seen = 0;
                for (int q = 0; q < nk; ++q) seen |= ku[q] == u && kr[q] == rb;
                if (!seen && nk < KMAX) { ku[nk] = u; kr[nk] = rb; ++nk; }
                long mm = 0;
                for (long q = 0; q < n; ++q) mm += yH[q] != x[q];
                k.m = mm;
                if (!i || !firstOK) k.m0 = mm;
                double l = 0;
                for (long q = 0; q < n; ++q)
                    if (yH[q] != x[q]) l += a[q];
                if (l < l0) {
                    memcpy(res, x, (size_t)n);
                    l0 = l;
                    if (l < calc_right_side(&k)) break;
                    while (j <= n - 1 - t && l >= calc_T(&k, j)) ++j;
                    T = (J >= 0 && j > J) ? J : j;
                    j = 0;
                }
            }
            ++i;
        }
        tot_dec += dec; tot_skip += skip; tot_bm += bm; tot_ok += okc;
        if (dec > 64) { ++heavy; heavy_dec += dec; heavy_rest += dec - skip; heavy_bm += bm; }
        if (dec > 1000 && heavy <= 20)
            printf("w %ld: dec %ld skip %ld rest %ld bm-pass %ld ok %ld known %d\n", w, dec, skip,
                   dec - skip, bm, okc, nk);
    }
    printf("words %ld: decodes %.2f/w, skipped %.1f%%, bm-pass among rest %.1f%%, ok %.3f%%\n", words,
           (double)tot_dec / words, 100.0 * tot_skip / tot_dec, 100.0 * tot_bm / (tot_dec - tot_skip),
           100.0 * tot_ok / (tot_dec - tot_skip));
    printf("heavy (>64): %ld words, decodes %ld, rest %ld (%.1f%%), bm-pass %ld\n", heavy, heavy_dec,
           heavy_rest, 100.0 * heavy_rest / heavy_dec, heavy_bm);
    printf("deg hist (bm pass):");
    for (int d = 0; d < 40; ++d) if (deg_hist[d]) printf(" %d:%ld", d, deg_hist[d]);
    printf("\n");
    return 0;
}
