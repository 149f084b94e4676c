/* oracle/bchk_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C11) of the reference hot path of
 * lizmoscow/polar-codes-with-bch-kernel, used exclusively as the CHECKER by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg. It is never linked into,
 * called by, or substituted for the product library (libbchk.so).
 *
 * Parity pinning: tests/test_oracle.py checks this restatement against the golden
 * vectors in tests/golden/, which oracle/make_golden.py produced by running the
 * REFERENCE itself (compiled from /root/reference by oracle/Makefile into oracle/_ref).
 */
#ifndef BCHK_ORACLE_H
#define BCHK_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#define ORC_MAXN 255
#define ORC_MAXT 32

typedef struct {
    int m, n, t, k, gsize;
    unsigned alog[ORC_MAXN + 1]; /* alpha^i, i in [0,n)            main.cpp:63-78 */
    int log_[ORC_MAXN + 2];      /* log(a), log(0) = -1           main.cpp:67-78 */
    unsigned char g[ORC_MAXN + 1];
} orc_code;

typedef struct {
    uint64_t decodes;      /* decodingCount delta                              */
    uint64_t cmp;          /* comparisonCount delta                            */
    uint64_t sum;          /* summCount delta                                  */
    uint64_t iters;        /* completed iterations (no early return)           */
    uint64_t jsteps;       /* calcT scan steps                                 */
    uint64_t improvements; /* accepted candidates that did not return          */
    int accepted;          /* res was written at least once                    */
    int returned;          /* left through the l < calcRightSide() exit        */
} orc_stats;

/* code construction: src/main.cpp:59-93, src/bchCoder.cpp:25-226 */
int orc_code_init(orc_code *c, int m, int t);

/* RNG stream: std::default_random_engine (minstd_rand0, seed 1 by default,
 * src/bchCoder.cpp:20), uniform_int_distribution<unsigned short>(0,1)
 * (src/bchCoder.cpp:22) and a fresh normal_distribution per addNoise call
 * (src/bchCoder.cpp:243-250), restated from libstdc++ 11 <bits/random.tcc>. */
typedef struct { uint64_t x; } orc_rng;
void orc_rng_seed(orc_rng *r, uint64_t seed);
void orc_gen_info(orc_rng *r, unsigned char *info, int k);        /* bchCoder.cpp:236 */
void orc_encode(const orc_code *c, const unsigned char *info, unsigned char *cw); /* :120 */
void orc_add_noise(orc_rng *r, double sd, const unsigned char *cw, double *y, int n); /* :243 */
double orc_sigma(const orc_code *c, double snr_db); /* dataForPlot.cpp:45 / Kaneko ctor :20 */

/* algebraic BCH hard decoder, src/Decoder.cpp:184-321 (Sugiyama/Euclid + Chien).
 * Returns 1 on success and writes answer = word ^ error pattern. */
int orc_alg_decode(const orc_code *c, const unsigned char *word, unsigned char *answer);
/* Same decision made the way the GPU kernel makes it (binary Berlekamp-Massey +
 * all-element root test). Exposed so tests can check the equivalence the GPU relies on. */
int orc_alg_decode_bm(const orc_code *c, const unsigned char *word, unsigned char *answer);

/* Kaneko soft decoder, decode(answer, word, res), src/KanekoKernelProcessor.cpp:335-407.
 * s2 = pow(sd0, 2) with sd0 the ctor sigma at the decoder SNR (0.5 dB in main.cpp).
 * J < 0: shipped (uncapped) bound; J >= 0: the commented `T = (j > J) ? J : j` (:392).
 * res is written only on acceptance (as the reference). l0 = DBL_MAX if none. */
void orc_kaneko_decode(const orc_code *c, double s2, int J, const double *y,
                       unsigned char *res, double *l0, orc_stats *st);

/* B independent decodes of the rows of Y [B][n] (orc_kaneko_decode each), split over
 * `threads` POSIX threads (the oracle keeps no global state). res rows are written only on
 * acceptance (callers pre-fill them); stats6 [B][6] = decodes, cmp, sum, iters, jsteps,
 * improvements; acc [B] = accepted. Test infrastructure: the checker for full batches. */
void orc_kaneko_batch(const orc_code *c, double s2, int J, const double *Y, long B,
                      unsigned char *res, double *l0, uint64_t *stats6, unsigned char *acc,
                      int threads);

/* Monte-Carlo FER sweep fun(), src/dataForPlot.cpp:16-116, into a text buffer
 * (CSV). Returns the number of bytes written (or -1 if cap is too small). */
/* Engine draws of `count` stream words from state *state (advanced), at Eb/N0 snr_db:
 * the words of src/dataForPlot.cpp:47-50 (generateRandomPoly + addNoise). */
uint64_t orc_stream_draws(const orc_code *c, uint64_t *state, long count, double snr_db);
/* One block of fun()'s loop body (src/dataForPlot.cpp:47-53): from engine state *state
 * (advanced), `skip` words dropped, then B words generated and decoded (res rows zeroed first,
 * written on acceptance): tx, res [B][n], acc [B], ops [B][3] = decodes/cmp/sums, states [B]
 * = the engine state after each word. */
void orc_sweep_block(const orc_code *c, double decoder_snr_db, int J, double snr_db, uint64_t *state,
                     long skip, long B, unsigned char *tx, unsigned char *res, unsigned char *acc,
                     uint64_t *ops, uint64_t *states);
long orc_sweep_range(const orc_code *c, double decoder_snr_db, int J, double snr_db, uint64_t *state,
                     uint64_t draws, long max_words, unsigned char *tx, unsigned char *res, unsigned char *acc,
                     uint64_t *ops, uint64_t *states);
long orc_sweep(const orc_code *c, double decoder_snr_db, int J, long p, long e,
               double max_snr, uint64_t seed, char *out, long cap);

#endif
