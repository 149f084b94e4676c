/* polar_oracle.h -- CPU restatement of the reference's vendored SC-list decoder for polar
 * codes over mixed binary kernels. TEST INFRASTRUCTURE ONLY: the checker of the GPU path
 * (polar-codes-with-bch-kernel_amd/csrc/polar_sclist.hip); nothing in the product links it.
 * See polar_oracle.c for the reference lines each routine follows. PARITY UNPINNED: the
 * vendored library cannot be built here and ships no fixtures. */
#ifndef POLAR_ORACLE_H
#define POLAR_ORACLE_H
#include <stdint.h>

#define PLR_MAXLAYERS 16
#define PLR_MAXU 4096
#define PLR_MAXKERNEL 64 /* matrix kernels up to 64 x 64 (the 2^6 extended-BCH kernel) */

typedef struct {
    int size;
    int arikan; /* "A": f/g processor (headers/external/KernProc.h:78-107) */
    uint8_t K[PLR_MAXKERNEL * PLR_MAXKERNEL];    /* row-major, 0/1 */
    uint8_t Kinv[PLR_MAXKERNEL * PLR_MAXKERNEL];
} plr_kernel;

typedef struct {
    int N, K, dmin, layers, nshort, npunct, U;
    plr_kernel kern[PLR_MAXLAYERS];
    uint8_t symtype[PLR_MAXU];   /* 0 normal, 1 shortened, 2 punctured */
    int decision[PLR_MAXU];      /* freezing constraint of symbol i, or -1 (unfrozen) */
    int fc_start[PLR_MAXU + 1];  /* constraint c: terms fc_terms[fc_start[c] .. fc_start[c+1]) */
    int fc_terms[PLR_MAXU * 8];
    uint64_t dfcorr[PLR_MAXU];   /* dynamic-freezing correction masks */
    int dfbit[PLR_MAXU];         /* mask bit holding the value of frozen symbol i, or -1 */
    int outer[PLR_MAXLAYERS + 1];
} plr_code;

/* Parse a code specification (MixedKernelEncoder.cpp:7-98); kernel files named "-path" or
 * "<path" are read relative to kernel_dir. NULL on error (msg filled). */
plr_code *plr_create(const char *spec, const char *kernel_dir, char *msg, int msglen);
void plr_destroy(plr_code *P);
void plr_dims(const plr_code *P, int *N, int *K, int *U);
/* info [K] -> codeword [N] (shortened / punctured symbols removed), Encode :142-177 */
void plr_encode(const plr_code *P, const uint8_t *info, uint8_t *cw);
/* info [K] -> unshortened codeword [U] */
void plr_encode_unshortened(const plr_code *P, const uint8_t *info, uint8_t *ucw);
/* unshortened codeword [U] -> info [K], ExtractInformationBitsUnshortened :209-238 */
void plr_extract_info(const plr_code *P, const uint8_t *ucw, uint8_t *info);
/* SC-list decode (MixedKernelListDecoder.cpp:211-268) of N channel LLRs (log P(0)/P(1)
 * as the decoder treats them). Writes count <= L entries, best first: info [L][K],
 * codewords [L][N] (may be NULL), path metrics [L] (may be NULL). Returns count or <0. */
int plr_decode(const plr_code *P, int L, const float *llr, uint8_t *info, uint8_t *cw,
               float *metric);
/* one kernel-input LLR of a matrix kernel: the min-sum value of CTrellisKernelProcessor::GetLLRs
 * (out/external/TrellisKernelProcessor.cpp:234-294), best[1] - best[0] over the coset of rows
 * phase+1..size-1, each word's metric the left-to-right float sum of |y| where it differs
 * from the hard decision. y = the kernel's output LLRs with the known inputs' signs applied.
 * Method: coset enumeration for cosets of at most 2^plr_trellis_nfree words; above that the
 * literal trellis for sizes <= 32 and the exact ordered-statistics search for larger kernels
 * (the reference's trellis processor stops below 64, TrellisKernelProcessor.cpp:70-71). */
float plr_minsum_llr(const plr_kernel *k, int phase, const float *y);
/* The same value by a given method (tests): PLR_BY_ENUM (2^(size-1-phase) words),
 * PLR_BY_TRELLIS (the trellis, any size <= 64: 65 columns with the extension), PLR_BY_ML
 * (exact ordered-statistics search with a lower-bound certificate). */
#define PLR_BY_ENUM 0
#define PLR_BY_TRELLIS 1
#define PLR_BY_ML 2
float plr_minsum_llr_by(const plr_kernel *k, int phase, const float *y, int method);
/* nodes (candidate codewords) the last PLR_BY_ML call of this thread evaluated */
long plr_ml_nodes(void);
/* nodes and searches of this thread since the previous call (then reset) */
long plr_ml_nodes_total(long *calls);

#endif
