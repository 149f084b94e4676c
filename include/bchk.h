/* include/bchk.h -- C ABI of libbchk.so, the MI355X (gfx950) Kaneko/BCH soft decoder.
 *
 * This is the drop-in boundary for the reference's hot path. The reference has no FFI;
 * its boundary is the C++ class API below, which the headers in include/bchk_dropin/ re-declare
 * on top of these entry points. Each entry point names the
 * reference interface it replaces (paths relative to the reference repo root).
 *
 * Conventions
 *  - Every function returns 0 on success and a negative BCHK_E* code on failure;
 *    bchk_last_error() describes the last failure of the calling thread. Nothing throws.
 *  - One context = one (code, J, decoder SNR, device); it owns a HIP stream. A context
 *    is not thread-safe; use one per host thread. It also owns the work queues, control
 *    words and fused-counter slots of its decode calls: at most ONE decode call per
 *    context may be in flight on the device at a time. Calls enqueued on the same stream
 *    serialise by themselves; a caller that passes different streams to consecutive calls
 *    must order them (an event, or bchk_sync) -- otherwise one call's counter reduction
 *    can fold and zero the other's partial counts. Use one context per concurrent stream.
 *  - Kernels never hang on a work-queue wait: every wait is bounded, and a wait that runs
 *    out leaves its codeword unfinished and sets the context's fault word. bchk_sync (and
 *    every synchronous *_host call) then fails with BCHK_EHIP and clears it.
 *  - Bit vectors are one byte per position (0/1), position i = coefficient of x^i,
 *    exactly as the reference's unsigned char arrays.
 *  - *_host functions take host pointers and are synchronous. *_device functions take
 *    device pointers, enqueue on `stream` (a hipStream_t, NULL = the context's stream)
 *    and return immediately.
 *  - There is NO CPU fallback: without a usable gfx950 device every compute call fails
 *    with BCHK_ENODEV.
 */
#ifndef BCHK_H
#define BCHK_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BCHK_OK 0
#define BCHK_EINVAL -1   /* bad argument / unsupported (m, t)                       */
#define BCHK_ENODEV -2   /* no HIP device, or the gfx950 code object failed to load */
#define BCHK_EHIP -3     /* a HIP runtime call failed                               */
#define BCHK_ENOMEM -4

/* J: the reference's test-pattern exponent cap.
 *   BCHK_J_SHIPPED (-1): as shipped, `T = j` (src/KanekoKernelProcessor.cpp:393);
 *   J >= 0: the commented-out `T = (j > J) ? J : j` (:392, J = 15 in the header :35). */
#define BCHK_J_SHIPPED (-1)

/* Decoder variants of KanekoKernelProcessor::decode */
#define BCHK_VARIANT_ANSWER 0 /* decode(answer, word, res) :335-407 (used by fun())       */
#define BCHK_VARIANT_WORD 1   /* decode(word, res)         :212-276 (main.cpp file mode)  */

/* per-codeword flags (bchk_stats.flags) */
#define BCHK_F_ACCEPTED 1u   /* res was written (else the row is left untouched)       */
#define BCHK_F_RETURNED 2u   /* left through `l < calcRightSide()` (:380-382)          */
#define BCHK_F_TRUNCATED 4u  /* stopped at the context's max_decodes safety cap:        */
                             /* result is NOT the reference's                           */
#define BCHK_F_TIE 8u        /* two |alpha| exactly equal: std::sort order unspecified  */
#define BCHK_F_SCAN_UB 16u   /* VARIANT_WORD only: the unbounded calcT scan (:257)      */
                             /* would read past alphaSorted[n-1] (UB in the reference)  */

typedef struct bchk_stats {
    uint64_t decodes;      /* += decodingCount                                (:368) */
    uint64_t comparisons;  /* += comparisonCount                       (:387,396,402) */
    uint64_t sums;         /* += summCount                                 (:388,403) */
    uint64_t iterations;   /* completed loop iterations                               */
    uint64_t jsteps;       /* calcT scan steps                                        */
    uint64_t improvements; /* accepted candidates that did not return                 */
    uint32_t flags;        /* BCHK_F_*                                                */
    uint32_t reserved;
} bchk_stats;

typedef struct bchk_ctx bchk_ctx;

/* Replaces KanekoKernelProcessor::KanekoKernelProcessor(pw, n, t, k, antilog, log, snr)
 * (headers/KanekoKernelProcessor.h:47-50, src/KanekoKernelProcessor.cpp:17-26) plus the
 * GF/generator setup of src/main.cpp:59-93. Supported: 2 <= m <= 8, 1 <= t <= 32,
 * t < 2^(m-1) (main.cpp:55). decoder_snr_db is 0.5 in every reference call site. */
int bchk_create(int m, int t, int J, double decoder_snr_db, int device, bchk_ctx **out);
void bchk_destroy(bchk_ctx *ctx);

/* n, k (= n - deg g, main.cpp:93) and deg g + 1. */
int bchk_code_params(const bchk_ctx *ctx, int *n, int *k, int *gsize);
/* g(x) coefficients low -> high (gsize bytes), as printVec(g, gSize) in main.cpp:95. */
int bchk_generator(const bchk_ctx *ctx, uint8_t *g);
/* Safety cap on algebraic decodes per codeword (0 = unlimited, the default). Codewords
 * that hit it are flagged BCHK_F_TRUNCATED. */
int bchk_set_max_decodes(bchk_ctx *ctx, uint64_t max_decodes);

/* Replaces KanekoKernelProcessor::decode(answer, word, res)
 * (headers/KanekoKernelProcessor.h:55, src/KanekoKernelProcessor.cpp:335-407), batched:
 *   y   [B][n] channel samples (double), row b = `word` of codeword b
 *   res [B][n] decoded words; row b is written only if flags & BCHK_F_ACCEPTED
 *   l0  [B]    path metric of res (calcL(res)), DBL_MAX if not accepted   (may be NULL)
 *   st  [B]    counters / flags                                           (may be NULL)
 * `answer` is not an input: the reference ignores it (:345 computes an unused value). */
int bchk_decode_host(bchk_ctx *ctx, const double *y, size_t B, uint8_t *res, double *l0,
                     bchk_stats *st);
int bchk_decode_device(bchk_ctx *ctx, const double *d_y, size_t B, uint8_t *d_res,
                       double *d_l0, bchk_stats *d_st, void *stream);
/* As above for another decode() variant (BCHK_VARIANT_*). */
int bchk_decode_variant_host(bchk_ctx *ctx, int variant, const double *y, size_t B,
                             uint8_t *res, double *l0, bchk_stats *st);

/* Replaces Decoder::decode(word, answer) (headers/Decoder.h:78, src/Decoder.cpp:298-321),
 * batched. The reference decodes from its stored syndrome (findSyndromPoly/
 * alterSyndromPoly, src/Decoder.cpp:184-230) and flips bits of `word`; syndromes (may be
 * NULL) carries that stored state as the t odd syndromes S_1, S_3, ..., S_{2t-1} per word
 * ([N][t] GF elements as uint32). NULL = syndromes of `words` themselves.
 *   ok [N] 1 on success; answers [N][n] written only where ok. */
int bchk_alg_decode_host(bchk_ctx *ctx, const uint8_t *words, const uint32_t *syndromes,
                         size_t N, uint8_t *answers, uint8_t *ok);

/* FER/BER/op-counter accumulation of one batch (src/dataForPlot.cpp:55-74), on device:
 *   out6 += {frame errors, bit errors, decodes, comparisons, sums, words}
 * tx/res [B][n]; st [B] from bchk_decode_device. d_out6 is a device uint64_t[6]. */
int bchk_count_device(bchk_ctx *ctx, const uint8_t *d_tx, const uint8_t *d_res,
                      const bchk_stats *d_st, size_t B, uint64_t *d_out6, void *stream);
/* bchk_decode_device and bchk_count_device in one pass (the body of the reference's fun()
 * loop over a batch, src/dataForPlot.cpp:55-74): every kernel that finishes a codeword
 * compares its row with tx and adds to the counters, so res and st are not read back.
 *   d_st may be NULL (then no per-codeword stats are stored; the counters still include
 *   decodes, comparisons and sums); out6 += {frame errors, bit errors, decodes,
 *   comparisons, sums, words}. Rows never accepted keep the caller's contents and are
 *   counted as such, exactly as bchk_count_device after bchk_decode_device. */
int bchk_decode_count_device(bchk_ctx *ctx, const double *d_y, const uint8_t *d_tx, size_t B, uint8_t *d_res,
                             double *d_l0, bchk_stats *d_st, uint64_t *d_out6, void *stream);

/* The reference's input stream (src/bchCoder.cpp:228-250 in fun() order): minstd_rand0
 * seeded with `seed`, B words at Eb/N0 snr_db: tx [B][n], y [B][n]. rng_state (in/out,
 * may be NULL) is the engine state: pass 0 to start from `seed`. Host-side, sequential. */
int bchk_generate_host(const bchk_ctx *ctx, double snr_db, size_t B, uint64_t *rng_state,
                       uint64_t seed, uint8_t *tx, double *y);
/* As above, and draws = the engine draws the B words consumed. */
int bchk_generate_host_draws(const bchk_ctx *ctx, double snr_db, size_t B, uint64_t *rng_state,
                             uint64_t seed, uint8_t *tx, double *y, uint64_t *draws);
/* The engine state `draws` draws after `state` (minstd_rand0: state * 16807^draws mod
 * 2^31 - 1; a seed is a state): disjoint ranges of the one reference stream per rank or
 * process. */
uint64_t bchk_rng_jump(uint64_t state, uint64_t draws);
/* One block of a (sharded) fun() sweep (src/dataForPlot.cpp:41-74): from engine state
 * *rng_state (in/out), `skip` words are passed over (their engine draws only, no samples),
 * then B words are generated at Eb/N0 snr_db and decoded on the GPU:
 *   tx [B][n], res [B][n] (zero where not accepted), accepted [B], ops [B][3] = decodes,
 *   comparisons, sums, states [B] = engine state after word b (where a sweep resumes when
 *   it stops after word b). */
int bchk_sweep_block(bchk_ctx *ctx, double snr_db, uint64_t *rng_state, size_t skip, size_t B,
                     uint8_t *tx, uint8_t *res, uint8_t *accepted, uint64_t *ops, uint64_t *states);
/* The same over the words of a stretch of the stream given in engine draws: from *rng_state
 * (a word start; in/out) words are generated until exactly `draws` draws are consumed (an
 * error if the stretch does not end on a word boundary or holds more than max_words words);
 * *words = their count. A sharded sweep's rank decodes the stretch between two word starts
 * found by bchk_stream_sync. */
int bchk_sweep_range(bchk_ctx *ctx, double snr_db, uint64_t *rng_state, uint64_t draws, size_t max_words,
                     uint8_t *tx, uint8_t *res, uint8_t *accepted, uint64_t *ops, uint64_t *states,
                     size_t *words);
/* The reference stream's draw structure for a code of dimension k and length n (host only,
 * no device): a word is k information draws (uniform_int_distribution<unsigned short>(0, 1),
 * src/bchCoder.cpp:236-240, redrawn only for the two largest engine values) and polar-method
 * attempts of four draws until ceil(n/2) pairs are accepted (normal_distribution, :243-250).
 * bchk_stream_skip: the engine state and draws after `words` words from `state` (no samples).
 * bchk_stream_sync: from a word start `state`, a word start in [offset, offset + limit) draws
 * on the stream's own parse that depends only on (state, offset, limit) -- the start where
 * every parse state possible at `offset` has merged, not necessarily the first start at or
 * after `offset` -- found WITHOUT parsing the draws before `offset` (neighbouring ranks make
 * the identical call for a shared boundary, so parts tile the stream; a redrawn information bit before
 * `offset`, or no merge before offset + limit, returns 1 = unresolved): *word_offset (draws
 * from `state`) and *word_state. */
int bchk_stream_skip(int k, int n, uint64_t state, uint64_t words, uint64_t *state_out, uint64_t *draws);
int bchk_stream_sync(int k, int n, uint64_t state, uint64_t offset, uint64_t limit, uint64_t *word_offset,
                     uint64_t *word_state);

/* fun(file, decoder, g, gSize, p, e, maxSTNR) (headers/dataForPlot.h:8,
 * src/dataForPlot.cpp:16-116) on the GPU: identical CSV text, written to csv (cap bytes,
 * NUL-terminated). The stream starts from *rng_state (engine state; NULL or 0 = seed) and
 * *rng_state receives the state after the last word consumed, exactly where the
 * reference's global engine would be. batch = codewords per GPU launch (0 = auto). */
int bchk_sweep(bchk_ctx *ctx, long p, long e, double max_snr, uint64_t *rng_state,
               uint64_t seed, size_t batch, char *csv, size_t cap);

/* On-GPU channel front-end (the encode + AWGN step of src/bchCoder.cpp:120-132,243-250 as a
 * batched kernel): words [word0, word0 + B) of a counter-based stream (Philox4x32-10 keyed
 * by seed; word w depends only on (seed, w)) at Eb/N0 snr_db -- uniform information bits,
 * c(x) = info(x) g(x), y = BPSK(c) + N(0, sd) with sd as src/dataForPlot.cpp:45. The same
 * distribution as the reference's words, NOT its minstd_rand0 stream (bchk_generate_host is
 * the bit-exact one). d_tx [B][n] u8, d_y [B][n] f64 on device. */
int bchk_generate_device(bchk_ctx *ctx, double snr_db, size_t B, uint64_t seed, uint64_t word0,
                         uint8_t *d_tx, double *d_y, void *stream);
/* fun() (src/dataForPlot.cpp:16-74) end to end on the GPU: words from bchk_generate_device,
 * decode and counters fused (bchk_decode_count_device), Eb/N0 0..max_snr step 0.5, each point
 * until p words or e frame errors (the e-th error cut exactly in word order). CSV lines as
 * bchk_sweep (statistically the reference's, not byte-identical); seconds = wall time,
 * words = words decoded. One divergence in the BER column: a word the decoder never accepts
 * is compared against the row left at its index in the batch buffer (zero in the first batch,
 * else that row's last accepted word), whereas fun() compares it against the previous word's
 * decision (its `decoded` buffer is shared, src/dataForPlot.cpp:25,52). FER, decodes,
 * comparisons and sums are unaffected only when every word is accepted; unaccepted words are
 * rare (none in the fixtures at n <= 63). bchk_sweep keeps fun()'s carry exactly. */
int bchk_sweep_device(bchk_ctx *ctx, long p, long e, double max_snr, uint64_t seed, size_t batch,
                      char *csv, size_t cap, double *seconds, uint64_t *words);

int bchk_sync(bchk_ctx *ctx);
/* the context's HIP stream (hipStream_t) */
void *bchk_stream(bchk_ctx *ctx);
/* Kernel-time profiling with HIP events recorded on the launch stream around each decode
 * call's three stages: [0] the lane-per-codeword fast kernel (+ the control memset),
 * [1] the exact wave-per-codeword kernel, [2] the workgroup-cooperative kernel for heavy
 * codewords. read() returns the summed milliseconds per stage since the last read and the
 * number of decode calls, then resets. */
int bchk_profile(bchk_ctx *ctx, int enable);
int bchk_profile_read(bchk_ctx *ctx, double *ms3, uint64_t *launches);
/* The same per stage: [0] fast, [1] exact first pass, [2] cooperative, [3] analytic tail
 * kernel (bchk_set_analytic); bchk_profile_read's exact stage is [1] + [3]. */
int bchk_profile_read_stages(bchk_ctx *ctx, double *ms4, uint64_t *launches);
/* Codewords the last decode call handed from the fast path to the exact kernel, and from
 * the exact kernel to the cooperative kernel (synchronises the context's stream). */
int bchk_path_counts(bchk_ctx *ctx, uint64_t *to_exact, uint64_t *to_coop);
/* Codewords the last decode call's exact first pass handed to the analytic tail kernel. */
int bchk_tail_count(bchk_ctx *ctx, uint64_t *to_tail);
/* Outcomes of the last call's analytic tail: [0] handed on to the cooperative kernel,
 * [1] finished from the candidate codewords, [2] split (exact chunks below the earliest
 * candidate within the tightened bound, then the candidates), [3] exact chunks of [2],
 * [4] enumeration steps (64 nodes each) summed, [5] their maximum over codewords. */
int bchk_tail_stats(bchk_ctx *ctx, uint64_t *out6);
/* The last call's cooperative-kernel counters (m >= 7): [0] chunks decoded again densely on
 * the acceptor's request (more candidates than a ring slot keeps; BCHK_LONG_REC=0..2 in the
 * environment at bchk_create sets the records per slot, default 2), [1] heavy codewords the
 * cooperative kernel started. */
int bchk_coop_stats(bchk_ctx *ctx, uint64_t *out2);
/* Diagnostics (context created with BCHK_TAIL_DIAG=1 in the environment): the last call's
 * per-codeword analytic-tail records, 8 u64 each -- codeword, cycles of prep, of the exact
 * chunks, of the plan, enumeration steps, mode | reason << 8 | split chunks << 16, cycles
 * after the plan, decodes. count = records written (may exceed items). */
int bchk_tail_diag_read(bchk_ctx *ctx, uint64_t *out, size_t items, uint64_t *count);
/* Diagnostics of experiment builds (BCHK_AN_PROF, lib/libbchk_anprof.so): per record of
 * bchk_tail_diag_read, 8 u64 of enumeration cycles by step phase -- pops, loads and single
 * children, leaf runs, stack pushes, emission batches, their cycles, leaf-run rounds, steps;
 * the record at index items - 1 of a 32768-record read holds the first pass's cycles summed
 * over its codewords -- prep, decode, acceptance, outputs, chunks, codewords (zeros in the
 * product build). */
int bchk_tail_prof_read(bchk_ctx *ctx, uint64_t *out, size_t items);
/* Enable (default) or disable the fast path; results are identical either way. */
int bchk_set_fast_path(bchk_ctx *ctx, int enable);
/* Enable (default) or disable the analytic tail of the exact kernel (n <= 63, decode
 * variant): a codeword still searching after the chunk limit is finished from its candidate
 * codewords -- those within t of some test pattern whose path metric can still improve
 * (KanekoKernelProcessor.cpp:361-405 replayed over them) -- instead of decoding every test
 * pattern in the cooperative kernel. Results are identical either way. */
int bchk_set_analytic(bchk_ctx *ctx, int enable);
/* 64-pattern chunks the exact kernel decodes before the analytic tail / the hand-off to
 * the cooperative kernel (default 1; 0 = neither: the exact kernel decodes everything). */
int bchk_set_chunk_limit(bchk_ctx *ctx, uint32_t chunks);

/* Enable (default) or disable the syndrome decoding table of the search kernels: for
 * n <= 63 and m (t - 1) <= 30, Decoder::decode of a test pattern is a lookup of its
 * normalised syndrome in a table of the weight <= t coset leaders (csrc/bchk_syndtab.h)
 * instead of Berlekamp-Massey + Chien. Results are identical either way. */
int bchk_set_syndrome_table(bchk_ctx *ctx, int enable);
/* Host-side decode through that table (no GPU): for odd syndromes synd[i][0..t) =
 * S_1, S_3, ..., S_{2t-1}, ok[i] = 1 iff Decoder::decode succeeds, and err[i] (may be
 * NULL) = the flipped positions as a bit mask. BCHK_EINVAL when (m, t) has no table.
 * Test/diagnostic entry point. */
int bchk_syndrome_table_query(int m, int t, const uint32_t *synd, size_t N, uint8_t *ok,
                              uint64_t *err);
/* Size of that table: distinct keys, bytes, longest probe sequence (buckets). */
int bchk_syndrome_table_info(int m, int t, uint64_t *keys, uint64_t *bytes, uint32_t *max_probe);

/* ---- SC-list decoding of polar codes (the reference's vendored library, never built by
 * the reference itself: headers/external/MixedKernelListDecoder.h:10-42). */
typedef struct bchk_polar bchk_polar;
/* Replaces CMixedKernelListDecoder(std::istream& Spec, unsigned ListSize)
 * (out/external/MixedKernelListDecoder.cpp:9): spec is the text of the reference's code
 * specification (out/external/MixedKernelEncoder.cpp:7-98: "N K d layers #shortened
 * #punctured", kernel names, shortened / punctured symbols, U - K freezing constraints).
 * Kernels: Arikan ("A") layers, and matrix kernels ("-file" / "<file", a size and size^2
 * entries, Kernel.cpp:93-107 -- e.g. BCH-derived kernels) of size <= 64, whose kernel LLRs are
 * the trellis min-sum of out/external/TrellisKernelProcessor.cpp:234-294 (polar_mixed.hip):
 * coset enumeration below 16, the trellis for 16..32 (at most 2^12 states per depth), and an
 * exact ordered-statistics search above 32 (the 64 x 64 extended-BCH kernel; the reference's
 * trellis processor stops below 64) -- the same value bit for bit;
 * 1 <= list_size <= 32, lengths whose per-wave state fits the 160 KiB LDS (U <= 1024 at
 * L = 16, 2048 at L = 8 for all-Arikan codes). Kernel files are read relative to kdir. */
int bchk_polar_create(const char *spec, int list_size, int device, bchk_polar **out);
int bchk_polar_create_kdir(const char *spec, const char *kdir, int list_size, int device, bchk_polar **out);
void bchk_polar_destroy(bchk_polar *pc);
/* N (transmitted length), K, U (unshortened length), L */
int bchk_polar_params(const bchk_polar *pc, int *n, int *k, int *unshortened, int *list_size);
/* Replaces Decode(pLLR, pInfVectorList, pCodewordList) (MixedKernelListDecoder.cpp:211-268),
 * batched: llr [B][N] float, log P(0)/P(1) as the decoder reads them (bit 1 when < 0);
 * per codeword the list, best path first: info [B][L][K], cw [B][L][N] (may be NULL),
 * metric [B][L] (path metrics, 0 = the hard decision), count [B] (rows written; rows past
 * it are left as they were). */
int bchk_polar_decode_host(bchk_polar *pc, const float *llr, size_t B, uint8_t *info,
                           uint8_t *cw, float *metric, int32_t *count);
int bchk_polar_decode_device(bchk_polar *pc, const float *d_llr, size_t B, uint8_t *d_info,
                             uint8_t *d_cw, float *d_metric, int32_t *d_count, void *stream);
/* Codes with a search layer (a matrix kernel above 32, e.g. the 64 x 64 extended-BCH kernel):
 * one codeword's list decode can take seconds, so a decode call is a series of kernel launches
 * of about 50 ms each (environment BCHK_POLAR_BUDGET_MS; 0 = one launch per call): a codeword
 * is suspended between two search items and resumed by the next launch, with identical
 * results. Such a call returns when the batch is decoded (it synchronises its stream). The
 * launches the last call took (1 for codes without a search layer or with the budget off). */
int bchk_polar_last_launches(const bchk_polar *pc, uint64_t *launches);
/* CMixedKernelEncoder::Encode (MixedKernelEncoder.cpp:142-177), host side: info [B][K] ->
 * codewords [B][N]. */
int bchk_polar_encode_host(const bchk_polar *pc, const uint8_t *info, size_t B, uint8_t *cw);
int bchk_polar_sync(bchk_polar *pc);
void *bchk_polar_stream(bchk_polar *pc);

/* ---- BCH polar-kernel construction and the column-permutation search (root bchCoder.cpp;
 * csrc/kernel_search.hip). Kernels are row-major l x l bytes (0/1). */
/* makeMatrix (root bchCoder.cpp:356-389): the nested extended-BCH kernel of size 2^power
 * (2 <= power <= 6), GF(2^power) from the reference's primitive polynomials
 * (src/main.cpp:14-15). Columns in power order: column 0 the extension, column p + 1 the
 * position of alpha^p. */
int bchk_kernel_ebch(int power, uint8_t *K);
/* swapColumns' reordering (root bchCoder.cpp:478-496): columns 0..2 kept, column i >= 3
 * takes the column of the field element i. */
int bchk_kernel_field_order(int power, const uint8_t *K, uint8_t *out);
/* The operation counts (SumCount, CmpCount; headers/external/misc.h:84-93) a
 * CTrellisKernelProcessor (out/external/TrellisKernelProcessor.cpp:69-294) spends on
 * GetLLRs(1, phase, zero known inputs, llr) for every phase 0..l-1 of the invertible kernel
 * K (2 <= l <= 32), the score the column search minimises (root bchCoder.cpp:505-515). */
int bchk_kernel_trellis_cost(const uint8_t *K, int l, const float *llr, int device, uint64_t *sum,
                             uint64_t *cmp);
/* The same score for every column map j -> B j with B = L.U (randomInvertibleMatrix, root
 * bchCoder.cpp:766-785) of a 2^power kernel: sum / cmp hold 2^(power (power - 1)) entries,
 * indexed by the candidate code whose bit d is the d-th bit randomInvertibleMatrix draws
 * (row i: l[i][0..i-1], then u[i][i+1..power-1]). */
int bchk_kernel_column_costs(int power, const uint8_t *K, const float *llr, int device, uint64_t *sum,
                             uint64_t *cmp);
#define BCHK_KSEARCH_EXHAUSTIVE 0 /* every L.U product, in code order                    */
#define BCHK_KSEARCH_RANDOM 1     /* randomSwapColumns: `count` random L.U products drawn  */
                                  /* from the reference's engine (state *rng_state, in/out) */
/* randomSwapColumns (root bchCoder.cpp:541-699): the candidate accepted last under the
 * reference's rule (both counts strictly below the best so far, :651-657), its permuted
 * kernel best[k][j] = K[k][perm[j]] (:627-629; best / perm may be NULL), its counts and its
 * index in the candidate sequence (-1: none). Scores come from the GPU (one launch over all
 * candidates), the acceptance is replayed on the host in candidate order. */
int bchk_kernel_column_search(int power, const uint8_t *K, const float *llr, int mode, uint64_t count,
                              uint64_t *rng_state, int device, uint8_t *best, uint32_t *perm,
                              uint64_t *best_sum, uint64_t *best_cmp, int64_t *best_index);

const char *bchk_last_error(void);
const char *bchk_version(void);

#ifdef __cplusplus
}
#endif
#endif
