// polar_device.h -- structures shared by the host runtime (polar_host.cpp) and the gfx950
// SC-list kernel (polar_sclist.hip). Plain C++, no HIP types.
#pragma once
#include <stdint.h>

namespace bchk {

constexpr int kPolarMaxList = 32;    // 2 L candidates, one per lane of a wave
constexpr int kPolarMaxLayers = 14;  // U <= 2^14 (LDS bounds it further)

// One SC-list decode launch: B codewords, one wave each, every path's arrays in LDS.
struct PolarParams {
    const float *llr;       // [B][N] channel LLRs, log P(0)/P(1) (the decoder's reading)
    uint8_t *info;          // [B][L][K] information vectors, best path first
    uint8_t *cw;            // [B][L][N] codewords (may be null)
    float *metric;          // [B][L] path metrics
    int32_t *count;         // [B] list entries written
    const int16_t *symmap;  // [U] LoadLLRs: index into the LLR row; -1 shortened, -2 punctured
    const uint16_t *phase;  // [U] bit 0 frozen | (dynamic-freezing bit + 1) << 1 | has-correction << 8
    const uint64_t *dfcorr; // [U] dynamic-freezing correction masks
    const int16_t *cwpos;   // [N] transmitted (neither shortened nor punctured) symbols
    uint32_t B;
    int32_t n, U, N, K, L;
    int32_t pathCw;                       // packed partial-sum words per path
    int32_t cwoff[kPolarMaxLayers + 1];   // word offset of C_λ in a path's packed array
};

constexpr uint16_t kPhaseFrozen = 1u, kPhaseCorr = 0x100u;


// (constexpr: usable from device code too.) Per-path strides in LDS, padded by 16 bytes so that the same element of consecutive paths
// falls in different banks (64 x 4 B banks): S holds U floats, C 3U bytes.
constexpr int polar_path_s(int U) { return ((U + 3) & ~3) + 4; }
constexpr int polar_path_c(int U) { return ((3 * U + 15) & ~15) + 16; }
constexpr int polar_rec_words(int K) { return K > 0 ? (K + 31) / 32 : 1; }

// Mixed kernels (polar_mixed.hip): layer j has a kernel of size ksize[j] (Arikan or a
// matrix, rows as 64-bit masks krows[j * kPolarMaxKernel + r], bit c = K[r][c]); outer[λ] =
// U / (ksize[0] ... ksize[λ-1]); per path S layer λ at soff[λ] (outer[λ] floats, λ >= 1), C
// layer λ at coff[λ] (outer[λ] ksize[λ-1] bytes, C_0 = U), matrix offset states at ooff[j].
constexpr int kPolarMaxKernel = 64;
constexpr int kPolarMaxMatrixGpu = 64;  // the 2^6 extended-BCH kernel (CTrellisKernelProcessor: < 64)
constexpr int kPolarMaxTrellisKernel = 32;  // the trellis is built for kernels up to 32 only
// Matrix layers of size > 32 (or from BCHK_POLAR_ML up) take their LLRs from an exact
// ordered-statistics search instead (one wave per item, polar_mixed.hip ml_llr): per wave an
// LDS scratch of kMlStack 12-byte search nodes, the reduced basis and the suffix unions of its
// non-pivot parts (64 + 65 u64), flip costs and |y| (64 floats each). Phases whose coset has
// at most 2^kMlEnumBits words are enumerated.
#ifndef BCHK_ML_STACK
#define BCHK_ML_STACK 768  // (64,32) L=8 2 dB, 8 192 words: 1536 nodes 950, 768 1 159, 512 1 116 codewords/s (profiles/r05_f4/ml_stack_variants.jsonl)
#endif
constexpr int kMlStack = BCHK_ML_STACK;
constexpr int kMlEnumBits = 10;
constexpr uint32_t kMlScratchBytes = 12u * kMlStack + 8u * 64u + 8u * 65u + 8u + 4u * 64u + 4u * 64u;
// the scratch before the stack (G, U, cost, ay: polar_mixed.hip MlScratch), saved with a
// suspended search together with the stack's live nodes
constexpr uint32_t kMlHeadBytes = 8u * 64u + 8u * 65u + 8u + 4u * 64u + 4u * 64u;
// Matrix layers of size >= the trellis threshold (default 16, BCHK_POLAR_TRELLIS) take their
// LLRs from CTrellisKernelProcessor's trellis (pull-form Viterbi over predecessor lists);
// smaller ones enumerate the coset (2^(size - 1 - phase) words per LLR). Per (layer, phase):
// tlog[(layer * kPolarMaxKernel + phase) * (kPolarMaxKernel + 1) + d] = log2 of the states at
// depth d (d = 0..size), tbase[layer * kPolarMaxKernel + phase] = first entry of the phase in
// tent; entries run depth by depth, one per state of depth d + 1, two 16-bit predecessors
// (state | z << 13 | valid << 14).
constexpr int kPolarTrellisMaxBits = 12;
constexpr uint32_t kTrellisZ = 1u << 13, kTrellisValid = 1u << 14, kTrellisState = kTrellisZ - 1u;
struct PolarMixedParams {
    const float *llr;
    uint8_t *info, *cw;
    float *metric;
    int32_t *count;
    const int16_t *symmap;
    const uint16_t *phase;
    const uint64_t *dfcorr;
    const int16_t *cwpos;
    const uint64_t *krows;  // [nl][kPolarMaxKernel]
    const uint32_t *tent, *tbase;  // trellis predecessor lists (see above)
    const uint8_t *tlog;
    int32_t tstates;               // largest state count of any trellis layer (>= 64 if any)
    uint32_t B;
    int32_t nl, U, N, K, L;
    int32_t ssize, csize, osize;
    int32_t ksize[kPolarMaxLayers], outer[kPolarMaxLayers + 1];
    int32_t soff[kPolarMaxLayers + 1], coff[kPolarMaxLayers + 1], ooff[kPolarMaxLayers];
    uint8_t arikan[kPolarMaxLayers];
    uint8_t trellis[kPolarMaxLayers];  // matrix layer decoded through its trellis
    uint8_t ml[kPolarMaxLayers];       // matrix layer decoded by the ordered-statistics search
    int32_t any_ml;                    // LDS holds the search scratch
    // Time-budgeted launches (round 6; codes with search layers): a wave past `budget` ticks
    // of the 100 MHz clock since its launch began suspends its codeword between two search
    // items (its LDS state and registers to rsave, rstate[cw] = 1) and starts no other; the
    // host launches again until `unfinished` stays 0. rstate: 0 not started, 1 suspended,
    // 2 done. budget 0 (or rstate null): every codeword runs to its end in one launch.
    uint32_t *rstate;
    uint8_t *rsave;
    uint32_t rstride;       // bytes of rsave per codeword (polar_mixed_save_bytes)
    uint32_t *unfinished;   // codewords left suspended or not started by this launch
    uint64_t budget;
    int32_t no_mid;         // experiments: suspend between search items only (BCHK_POLAR_NO_MID)
};

// The kernel's LDS offsets (polar_mixed.hip), shared with the host's save-area size.
struct PolarMixedLayout {
    int o_S, o_C, o_O, o_ph, o_rows, o_act, o_tm;
};
__host__ __device__ inline PolarMixedLayout polar_mixed_layout(int U, int L, int ssize, int csize, int osize, int nl,
                                                               int rec_words) {
    PolarMixedLayout o;
    o.o_S = (4 * U + 15) & ~15;
    o.o_C = o.o_S + 4 * ssize * L;
    o.o_O = o.o_C + csize * L;
    o.o_ph = (o.o_O + osize * L + 15) & ~15;
    o.o_rows = (o.o_ph + 2 * U + 15) & ~15;
    o.o_act = o.o_rows + 8 * kPolarMaxKernel * nl;
    o.o_tm = (o.o_act + 4 * L + 4 * L * rec_words + 15) & ~15;
    return o;
}
// a suspended codeword: header (64 B), six registers per lane (64 x 24 B), then the LDS of
// the list state: channel / S / C / O ([0, o_ph)) and act / rec ([o_act, o_tm))
// (+ a suspended search's scratch: kMlScratchBytes)
__host__ __device__ inline uint32_t polar_mixed_save_bytes(const PolarMixedLayout &o) {
    return (uint32_t)((64 + 64 * 24 + o.o_ph + (o.o_tm - o.o_act) + kMlScratchBytes + 15) & ~15);
}

inline uint32_t polar_mixed_lds_bytes(int U, int L, int K, int ssize, int csize, int osize, int nl,
                                      int tstates, bool ml) {
    uint32_t b = (4u * (uint32_t)U + 15u) & ~15u;                                     // channel
    b += 4u * (uint32_t)ssize * (uint32_t)L + (uint32_t)csize * (uint32_t)L;           // S, C
    b = (b + (uint32_t)osize * (uint32_t)L + 15u) & ~15u;                              // offsets
    b = (b + 2u * (uint32_t)U + 15u) & ~15u;                                           // phases
    b += 8u * (uint32_t)kPolarMaxKernel * (uint32_t)nl;                                // rows
    b += 4u * (uint32_t)L + 4u * (uint32_t)L * (uint32_t)polar_rec_words(K);            // act, rec
    b = (b + 15u) & ~15u;
    b += 8u * (uint32_t)tstates;  // trellis state metrics: two buffers of tstates floats
    b = (b + 15u) & ~15u;
    if (ml) b += kMlScratchBytes;  // ordered-statistics search scratch
    return (b + 15u) & ~15u;
}

// Packed partial sums of the all-Arikan kernel (polar_sclist.hip): per path C_0 (U bits,
// the codeword) then C_λ (U >> (λ-1) bits, λ = 1..n), each starting on a 32-bit word; the
// path stride is odd, so the same word of different paths falls in different banks. Writes
// the word offsets (n + 1 entries) when off is given; returns the stride in words.
inline int polar_cw_layout(int U, int32_t *off) {
    int n = 0;
    while ((1 << n) < U) ++n;
    int w = 0;
    for (int lam = 0; lam <= n; ++lam) {
        if (off) off[lam] = w;
        const int bits = lam == 0 ? U : (U >> (lam - 1));
        w += (bits + 31) / 32;
    }
    return w | 1;
}

// LDS bytes of one wave's state (see polar_sclist.hip): per path S (floats) and the packed
// partial sums, the active-path list and per path the information bits decided so far. The
// channel LLRs and the phase table are read from global memory (layer 0 is read at two
// phases per codeword, the phase word once per phase).
inline uint32_t polar_lds_bytes(int U, int L, int K) {
    uint32_t b = 4u * (uint32_t)polar_path_s(U) * (uint32_t)L;             // S
    b += 4u * (uint32_t)polar_cw_layout(U, nullptr) * (uint32_t)L;          // C (bits)
    b = (b + 15u) & ~15u;
    b += 4u * (uint32_t)L;                                                  // active list
    b += 4u * (uint32_t)L * (uint32_t)polar_rec_words(K);                   // information bits
    return (b + 15u) & ~15u;
}

}  // namespace bchk
