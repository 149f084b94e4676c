// bchk_channel.hip -- on-GPU channel front-end for throughput sweeps: the reference's
// encode and AWGN step (src/bchCoder.cpp:120-132 encode c(x) = info(x) g(x); :243-250
// y = BPSK(c) + N(0, sd)) with a counter-based generator instead of the reference's
// sequential minstd_rand0 stream. The words are statistically the reference's (uniform
// information bits, Gaussian noise of the same sd) but not its bit-exact stream; parity
// runs keep using the host stream (bchk_generate_host). Word w of a (seed, Eb/N0) stream
// depends only on (seed, w), so any range of words can be generated anywhere.
//
// chan_kernel: one wave per 64 words. Each lane draws its word's information bits (Philox
// 4x32-10, counter (word, 0xFFFFFFFF)) and multiplies by g over GF(2) (shifted XORs of the
// packed generator); the 64 x n bits go to LDS, and the wave then writes tx and y for the
// block element by element: element G of the stream (flat index over [word][position]) takes
// one of the Box-Muller pair of Philox counter G / 2 (coalesced stores of y).
#include <hip/hip_runtime.h>

#include "bchk_device.h"
#include "bchk_launch.h"

namespace bchk {

namespace {

struct U4 {
    uint32_t x, y, z, w;
};

// Philox4x32-10 (Salmon et al., SC'11): 10 rounds of the 4x32 bijection keyed by (k0, k1)
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t h0 = __umulhi(M0, c.x), l0 = M0 * c.x;
        const uint32_t h1 = __umulhi(M1, c.z), l1 = M1 * c.z;
        c = U4{h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// (0, 1] with 53 random bits
__device__ __forceinline__ double unit53(uint32_t a, uint32_t b) {
    const uint64_t v = ((uint64_t)a << 21) ^ (uint64_t)(b >> 11);  // 53 bits
    return ((double)(v & ((1ull << 53) - 1ull)) + 1.0) * 0x1p-53;
}

constexpr int kChanWaves = 4;
constexpr int kMaxWords64 = 4;  // n <= 255

template <int NW64>
__global__ void __launch_bounds__(64 * kChanWaves) chan_kernel(ChanParams cp) {
    extern __shared__ __attribute__((aligned(16))) uint8_t csm[];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int n = cp.n;
    uint8_t *bits = csm + (size_t)wid * 64 * (size_t)n;  // [64][n] codeword bits
    const uint32_t w0 = (blockIdx.x * kChanWaves + wid) * 64u;
    if (w0 >= cp.count) return;
    const uint32_t rows = cp.count - w0 < 64u ? cp.count - w0 : 64u;
    // ---- information bits and c(x) = info(x) g(x) (bchCoder.cpp:120-132), lane = word
    {
        const uint64_t word = cp.word0 + w0 + (uint64_t)lane;
        uint64_t c[NW64];
#pragma unroll
        for (int q = 0; q < NW64; ++q) c[q] = 0;
        for (int i0 = 0; i0 < cp.k; i0 += 128) {
            const U4 r = philox(U4{(uint32_t)word, (uint32_t)(word >> 32), 0xFFFFFFFFu, (uint32_t)i0},
                                cp.seed_lo, cp.seed_hi);
            const uint32_t rw[4] = {r.x, r.y, r.z, r.w};
            for (int i = i0; i < cp.k && i < i0 + 128; ++i) {
                if (!((rw[(i - i0) >> 5] >> ((i - i0) & 31)) & 1u)) continue;
                // c ^= g << i
#pragma unroll
                for (int q = 0; q < NW64; ++q) {
                    uint64_t v = 0;
#pragma unroll
                    for (int j = 0; j < NW64; ++j) {
                        const int s = i + 64 * j - 64 * q;  // bit offset of g word j in c word q
                        if (s >= 64 || s <= -64) continue;
                        v ^= s >= 0 ? (cp.g[j] << s) : (cp.g[j] >> (-s));
                    }
                    c[q] ^= v;
                }
            }
        }
        if ((uint32_t)lane < rows)
            for (int pos = 0; pos < n; ++pos)
                bits[lane * n + pos] = (uint8_t)((c[pos >> 6] >> (pos & 63)) & 1ull);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- tx rows (the block is contiguous) and y = BPSK + noise, element-parallel
    const uint32_t elems = rows * (uint32_t)n;
    uint8_t *tx = cp.tx + (size_t)w0 * n;
    for (uint32_t e = (uint32_t)lane; e < elems; e += 64) tx[e] = bits[e];
    double *y = cp.y + (size_t)w0 * n;
    // global element G = word * n + position; the Box-Muller pair of Philox counter G / 2
    // gives elements 2 p and 2 p + 1 (a pair may straddle two blocks: each computes it)
    const uint64_t ebase = (cp.word0 + w0) * (uint64_t)n;
    const uint64_t p0 = ebase >> 1, pend = (ebase + elems + 1) >> 1;
    for (uint64_t pr = p0 + (uint64_t)lane; pr < pend; pr += 64) {
        const U4 r = philox(U4{(uint32_t)pr, (uint32_t)(pr >> 32), 0x5EEDu, 0u}, cp.seed_lo, cp.seed_hi);
        const double u1 = unit53(r.x, r.y), u2 = unit53(r.z, r.w);
        const double rad = sqrt(-2.0 * log(u1));
        double sn, cs;
        sincospi(2.0 * u2, &sn, &cs);
        const double z[2] = {rad * cs, rad * sn};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t el = (int64_t)(2 * pr + (uint64_t)h) - (int64_t)ebase;  // within the block
            if (el < 0 || el >= (int64_t)elems) continue;
            y[el] = (bits[el] ? 1.0 : -1.0) + cp.sd * z[h];
        }
    }
}

// per word: does the decoded row differ from the sent one (frame error flag)
__global__ void __launch_bounds__(256) frame_err_kernel(const uint8_t *tx, const uint8_t *res, uint32_t B, int n,
                                                          uint8_t *flags) {
    const uint32_t w = blockIdx.x * 256u + threadIdx.x;
    if (w >= B) return;
    uint8_t d = 0;
    for (int i = 0; i < n; ++i) d |= (uint8_t)(tx[(size_t)w * n + i] != res[(size_t)w * n + i]);
    flags[w] = d;
}

}  // namespace

hipError_t launch_channel(const ChanParams &cp, hipStream_t s) {
    if (cp.count == 0) return hipSuccess;
    const int words64 = (cp.n + 63) / 64;
    const uint32_t waves = (cp.count + 63u) / 64u;
    const dim3 grid((waves + kChanWaves - 1) / kChanWaves), block(64 * kChanWaves);
    const size_t lds = (size_t)kChanWaves * 64 * (size_t)cp.n;
    if (lds > 65536) {
        static bool done[kMaxWords64 + 1] = {false, false, false, false, false};
        if (!done[words64]) {
            const void *fn = words64 == 3 ? (const void *)&chan_kernel<3> : (const void *)&chan_kernel<4>;
            (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            done[words64] = true;
        }
    }
    switch (words64) {
        case 1: hipLaunchKernelGGL(chan_kernel<1>, grid, block, lds, s, cp); break;
        case 2: hipLaunchKernelGGL(chan_kernel<2>, grid, block, lds, s, cp); break;
        case 3: hipLaunchKernelGGL(chan_kernel<3>, grid, block, lds, s, cp); break;
        case 4: hipLaunchKernelGGL(chan_kernel<4>, grid, block, lds, s, cp); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_frame_errors(const uint8_t *tx, const uint8_t *res, uint32_t B, int n, uint8_t *flags,
                               hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(frame_err_kernel, dim3((B + 255) / 256), dim3(256), 0, s, tx, res, B, n, flags);
    return hipGetLastError();
}

static_assert(kMaxWords64 * 64 >= 255, "n <= 255");

}  // namespace bchk
