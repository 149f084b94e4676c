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
    const uint8_t *frozen;  // [U] 1 = (dynamic) frozen symbol
    const int8_t *dfbit;    // [U] mask bit holding a frozen symbol's value, -1 = static
    const uint64_t *dfcorr; // [U] dynamic-freezing correction masks
    const int16_t *infopos; // [K] unfrozen symbols
    const int16_t *cwpos;   // [N] transmitted (neither shortened nor punctured) symbols
    uint32_t B;
    int32_t n, U, N, K, L;
};

// LDS bytes of one wave's state (see polar_sclist.hip): channel LLRs, per path S (U floats,
// padded) and C (3U bytes, padded) arrays, per path metric / LLR / mask, the path stack,
// the list of active paths and a U-byte scratch row.
inline uint32_t polar_lds_bytes(int U, int L) {
    uint32_t b = 4u * (uint32_t)U;                  // channel
    b += 4u * (uint32_t)U * (uint32_t)L;            // S
    b += 4u * (uint32_t)L * 2u;                     // R, llr
    b = (b + 7u) & ~7u;
    b += 8u * (uint32_t)L;                          // DF masks
    b += 4u * (uint32_t)(L + 1) + 4u * (uint32_t)L; // stack, active list
    b = (b + 15u) & ~15u;
    b += 3u * (uint32_t)U * (uint32_t)L;            // C
    b += (uint32_t)U;                               // scratch
    return (b + 15u) & ~15u;
}

}  // namespace bchk
