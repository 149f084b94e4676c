// polar_sclist.hip -- batched SC-list decoding of polar codes over the Arikan kernel (with
// dynamic frozen constraints, shortening and puncturing) on gfx950.
//
// Reference: the vendored CMixedKernelListDecoder (out/external/MixedKernelListDecoder.cpp:
// 61-268) over CListKernelEngine (out/external/KernelListEngine.cpp:266-447), the f/g
// processor of headers/external/KernProc.h:89-102 (SoftProcessing.cpp:39-80) and the
// path-index stack of out/external/TVMemoryEngine.cpp:85-142. Same decisions, same float
// arithmetic and the same path indices (the list sorts break ties on them), so the output
// lists equal the CPU restatement (oracle/polar_oracle.c) bit for bit.
//
// Execution model: one 64-lane wave per codeword (persistent over the batch).
//   * LDS holds every path's LLRs S_λ (U >> λ floats) and partial sums C_λ (kernel inputs
//     of the current block, U >> (λ-1) bits packed in 32-bit words, each layer word-aligned;
//     C_0 = the codeword) and the information bits decided so far (packed, flushed every 32
//     decisions). The channel LLRs (read at two phases per codeword) and the phase table
//     come from global memory, so (1024, 512) at L = 8 fits 4 waves per CU.
//   * Lane q < L holds path q's scalar state in registers: metric R, leaf LLR, dynamic-
//     freezing mask, the current record word and slot q of the path-index stack (pushes and
//     pops are v_writelane / v_readlane on a wave-uniform top).
//   * Each phase: the LLR recursion from the first layer whose block changed, lanes over
//     (active path x element); decisions (frozen: lane = path; unfrozen: the 2 L candidates
//     ranked in lanes 2q + b with the reference's std::greater<pair> order); kills, then
//     clones in path order, a clone copying only the parent's live S layers, live C halves
//     and record words; then the partial-sum butterflies of the finished blocks.
// No MFMA: the work is float min/add and byte XOR on short vectors.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "polar_device.h"

namespace bchk {

namespace {

constexpr uint32_t kUninit = 0xFFFFFFFFu;

__device__ __forceinline__ void wave_sync_p() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// offset of S_λ (λ >= 1) inside one path's LLR array
__device__ __forceinline__ int s_off(int U, int lam) { return U - (U >> (lam - 1)); }

// SoftXOR (SoftProcessing.cpp:54-80): sign(a) sign(b) min(|a|, |b|)
__device__ __forceinline__ float f_minsum(float a, float b) {
    const float fa = fabsf(a), fb = fabsf(b);
    const float m = fa < fb ? fa : fb;
    return __uint_as_float(__float_as_uint(m) | ((__float_as_uint(a) ^ __float_as_uint(b)) & 0x80000000u));
}

__device__ __forceinline__ float rdl_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint32_t rdl_u(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t rdl_u64(uint64_t v, int l) {
    return (uint64_t)rdl_u((uint32_t)v, l) | ((uint64_t)rdl_u((uint32_t)(v >> 32), l) << 32);
}

// The path-index stack of TVMemoryEngine (headers/external/misc.h:212-226) with its lazy
// initialisation: slot i lives in lane i's `slot`, `top` is wave-uniform.
struct PathStack {
    uint32_t slot;
    int top;
    __device__ __forceinline__ void reset(int L, int lane) {
        top = L;
        if (lane == L) slot = kUninit;
    }
    __device__ __forceinline__ uint32_t pop(int lane) {
        const uint32_t v = rdl_u(slot, top);
        if (v == kUninit) {  // never pushed: hand out top - 1
            const int r = top - 1;
            top = r;
            if (r > 0 && lane == r) slot = kUninit;
            return (uint32_t)r;
        }
        --top;
        return v;
    }
    __device__ __forceinline__ void push(uint32_t x, int lane) {
        ++top;
        if (lane == top) slot = x;
    }
};

// act[k] = index of the k-th active path; returns their number
__device__ __forceinline__ int list_active(uint32_t active, uint32_t *act, int lane, int L) {
    if (lane < L && ((active >> lane) & 1u)) act[__builtin_popcount(active & ((1u << lane) - 1u))] = (uint32_t)lane;
    wave_sync_p();
    return __builtin_popcount(active);
}

}  // namespace

__global__ void __launch_bounds__(64) polar_sclist_kernel(PolarParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)threadIdx.x;
    const int U = p.U, n = p.n, L = p.L, K = p.K;
    const int pathS = polar_path_s(U), pathC = p.pathCw, RW = polar_rec_words(K);
    // LDS layout: polar_lds_bytes (polar_device.h)
    // (byte offsets from smem, never through integer casts of the pointers, which would
    // lose the LDS address space and turn every access into a FLAT one)
    const int o_C = 4 * pathS * L;
    const int o_act = (o_C + 4 * pathC * L + 15) & ~15;
    float *S = reinterpret_cast<float *>(smem);
    uint32_t *C = reinterpret_cast<uint32_t *>(smem + o_C);  // packed bits, words per path
    uint32_t *act = reinterpret_cast<uint32_t *>(smem + o_act);
    uint32_t *rec = act + L;
    const int lastc = p.cwoff[n];  // C_n: the two inputs of the last Arikan block (one word)
    const bool mine = lane < L;
    auto cbit = [&](int q, int lam, int s) -> uint32_t {
        const int b = s;
        return (C[(size_t)q * pathC + p.cwoff[lam] + (b >> 5)] >> (b & 31)) & 1u;
    };

    PathStack st;
    st.slot = 0;
    for (uint32_t cw = blockIdx.x; cw < p.B; cw += gridDim.x) {
        // ---- LoadLLRs (MixedKernelEncoder.cpp:181-207), applied where layer 0 is read
        const float *y = p.llr + (size_t)cw * p.N;
        auto chan = [&](int i) -> float {
            const int m = p.symmap[i];
            return m >= 0 ? y[m] : (m == -1 ? 100000.0f : 0.0f);
        };
        // ---- Cleanup + AssignInitialPath (TVMemoryEngine.cpp:58-94)
        st.reset(L, lane);
        const uint32_t pid = st.pop(lane);
        uint32_t active = 1u << pid;
        float R = 0.0f, lv = 0.0f;
        uint64_t dm = 0;
        uint32_t rw = 0;
        int k = 0;  // unfrozen decisions so far
        wave_sync_p();
        int nact = list_active(active, act, lane, L);

        for (int phi = 0; phi < U; ++phi) {
            const uint32_t e = __builtin_amdgcn_readfirstlane((uint32_t)p.phase[phi]);
            // ---- IterativelyCalcS (KernelListEngine.cpp:370-447): from layer m, where the
            // block of phase phi starts, down to the single LLR of layer n
            int m = 0, local = 0;
            if (phi) {
                m = n - 1 - __builtin_ctz((unsigned)phi);
                local = 1;
            }
            for (int j = m; j < n; ++j) {
                const int loc = (j == m) ? local : 0;
                const int lgd = n - 1 - j;  // d = U >> (j + 1)
                const int d = 1 << lgd;
                const int tot = nact << lgd;
                for (int it = lane; it < tot; it += 64) {
                    const int q = (int)act[it >> lgd], s = it & (d - 1);
                    float *dst = S + (size_t)q * pathS + s_off(U, j + 1);
                    float a, b;
                    if (j == 0) {
                        a = chan(s);
                        b = chan(d + s);
                    } else {
                        const float *src = S + (size_t)q * pathS + s_off(U, j);
                        a = src[s];
                        b = src[d + s];
                    }
                    float r;
                    if (loc) {  // SoftCombine (:39-50): b - a if u = 1 else b + a
                        r = cbit(q, j + 1, s) ? b - a : b + a;
                    } else {
                        r = f_minsum(a, b);
                    }
                    dst[s] = r;
                }
                wave_sync_p();
            }
            const bool on = mine && ((active >> lane) & 1u);
            if (on) lv = S[(size_t)lane * pathS + U - 2];
            const uint64_t corr = (e & kPhaseCorr) ? p.dfcorr[phi] : 0ull;
            uint32_t dec = 0;

            if (e & kPhaseFrozen) {
                // ---- ContinuePathsFrozen (MixedKernelListDecoder.cpp:61-98)
                const int db = (int)((e >> 1) & 127u) - 1;
                if (on) {
                    dec = db >= 0 ? (uint32_t)((dm >> db) & 1ull) : 0u;
                    if ((dec != 0) ^ (lv < 0.0f)) R -= fabsf(lv);
                }
            } else {
                // ---- ContinuePathsUnfrozen (:100-185). Candidate 2q + b (bit b of path q)
                // sits in lane 2q + b; its score is R (b = hard decision) or R - |llr|.
                const int q = lane >> 1, b = lane & 1;
                const float vq = __shfl(lv, q & 31), Rq = __shfl(R, q & 31);
                const bool valid = q < L && ((active >> q) & 1u);
                float sc = 0.0f;
                if (valid) sc = (b == (vq < 0.0f ? 1 : 0)) ? Rq : Rq - fabsf(vq);
                // rank under std::greater<pair<float, unsigned>> (:125): score, then index
                int rank = 0;
                for (uint64_t mm = __ballot(valid); mm; mm &= mm - 1) {
                    const int o = (int)__builtin_ctzll(mm);
                    const float so = rdl_f(sc, o);
                    rank += (sc < so || (!(so < sc) && lane < o)) ? 1 : 0;
                }
                const int J = 2 * nact, keep = J < L ? J : L;
                const uint64_t sel = __ballot(valid && rank < keep);
                const uint32_t cont = mine ? (uint32_t)((sel >> (2 * lane)) & 3ull) : 0u;
                const uint32_t cont_any = (uint32_t)__ballot(cont != 0);
                const uint32_t clones = (uint32_t)__ballot(cont == 3u);
                // KillPath, in path order (:129-136)
                for (uint32_t kill = active & ~cont_any; kill; kill &= kill - 1) st.push((uint32_t)__builtin_ctz(kill), lane);
                active &= cont_any;
                // continuations (:138-178): 1 -> bit 0, 2 -> bit 1, 3 -> the hard decision
                // here and its complement in a clone; the score changes only in the clone
                dec = cont == 2u ? 1u : (cont == 3u ? (lv < 0.0f ? 1u : 0u) : 0u);
                for (uint32_t cl = clones; cl; cl &= cl - 1) {
                    const int l = __builtin_ctz(cl);
                    const int l1 = (int)st.pop(lane);  // ClonePath: copy the live state of l
                    {
                        // S_j (j >= 1) is read again iff bit n-1-j of phi is 0; copy from the
                        // first such layer on. The packed partial sums are copied whole
                        // (3U bits).
                        const uint32_t zs = ~(uint32_t)phi & ((1u << (n - 1)) - 1u);
                        const int s0 = zs ? (s_off(U, n - 1 - (31 - __builtin_clz(zs))) & ~3) : pathS;
                        const int ns4 = (((U + 3) & ~3) - s0) >> 2;
                        const int nc = pathC;
                        const int nr = k >> 5;
                        const uint4 *sS = reinterpret_cast<const uint4 *>(S + (size_t)l * pathS + s0);
                        uint4 *dS = reinterpret_cast<uint4 *>(S + (size_t)l1 * pathS + s0);
                        const uint32_t *sC = C + (size_t)l * pathC;
                        uint32_t *dC = C + (size_t)l1 * pathC;
                        int top = ns4 > nc ? ns4 : nc;
                        top = top > nr ? top : nr;
                        for (int i = lane; i < top; i += 64) {
                            uint4 vs;
                            uint32_t vc = 0, vr = 0;
                            if (i < ns4) vs = sS[i];
                            if (i < nc) vc = sC[i];
                            if (i < nr) vr = rec[l * RW + i];
                            if (i < ns4) dS[i] = vs;
                            if (i < nc) dC[i] = vc;
                            if (i < nr) rec[l1 * RW + i] = vr;
                        }
                    }
                    const float Rl = rdl_f(R, l), vl = rdl_f(lv, l);
                    const uint64_t dml = rdl_u64(dm, l);
                    const uint32_t rwl = rdl_u(rw, l), decl = rdl_u(dec, l);
                    if (lane == l1) {
                        R = Rl - fabsf(vl);
                        dm = dml;
                        rw = rwl;
                        dec = decl ^ 1u;
                        lv = vl;
                    }
                    active |= 1u << l1;
                }
                wave_sync_p();
            }
            const bool now = mine && ((active >> lane) & 1u);
            if (now) {  // the path's own word: no other lane writes it
                uint32_t &w = C[(size_t)lane * pathC + lastc];
                const uint32_t bit = 1u << (phi & 1);
                w = dec ? (w | bit) : (w & ~bit);
                if (dec) dm ^= corr;
            }
            if (!(e & kPhaseFrozen)) {
                if (now) rw |= dec << (k & 31);
                ++k;
                if ((k & 31) == 0) {
                    if (now) rec[lane * RW + (k >> 5) - 1] = rw;
                    rw = 0;
                }
                nact = list_active(active, act, lane, L);
            } else {
                wave_sync_p();
            }

            // ---- IterativelyUpdateC (KernelListEngine.cpp:266-315): the blocks this phase
            // completes are encoded into their parents' slots
            {
                int lam = n, lgs = 0, ph2 = phi;
                while (lam > 0 && (ph2 & 1)) {
                    const int psi = ph2 >> 1;
                    const int stride = 1 << lgs, next = stride << 1;
                    const int phi0 = (lam > 1) ? (psi & 1) * next : 0;
                    if (stride >= 32) {  // whole words: (x0, x1) -> (x0 ^ x1, x1), 32 at a time
                        const int lw = lgs - 5, sw = 1 << lw, tot = nact << lw;
                        for (int it = lane; it < tot; it += 64) {
                            const int q = (int)act[it >> lw], s = it & (sw - 1);
                            const uint32_t *src = C + (size_t)q * pathC + p.cwoff[lam];
                            uint32_t *dst = C + (size_t)q * pathC + p.cwoff[lam - 1] + (phi0 >> 5);
                            const uint32_t x0 = src[s], x1 = src[sw + s];
                            dst[s] = x0 ^ x1;
                            dst[sw + s] = x1;
                        }
                    } else if (mine && ((active >> lane) & 1u)) {  // one word per path, its lane
                        const uint32_t v = C[(size_t)lane * pathC + p.cwoff[lam]];
                        const uint32_t mk = (1u << stride) - 1u;
                        const uint32_t x0 = v & mk, x1 = (v >> stride) & mk;
                        const uint32_t r = (x0 ^ x1) | (x1 << stride);  // 2 stride bits
                        uint32_t &w = C[(size_t)lane * pathC + p.cwoff[lam - 1] + (phi0 >> 5)];
                        if (next == 32) {
                            w = r;
                        } else {
                            const int sh = phi0 & 31;
                            const uint32_t m2 = ((1u << next) - 1u) << sh;
                            w = (w & ~m2) | (r << sh);
                        }
                    }
                    wave_sync_p();
                    ++lgs;
                    ph2 = psi;
                    --lam;
                }
            }
        }
        if ((k & 31) && mine && ((active >> lane) & 1u)) rec[lane * RW + (k >> 5)] = rw;
        wave_sync_p();

        // ---- final order (:249-267): active paths by (R, index), descending
        int rk = 0;
        const bool me = mine && ((active >> lane) & 1u);
        for (uint64_t mm = __ballot(me); mm; mm &= mm - 1) {
            const int o = (int)__builtin_ctzll(mm);
            const float ro = rdl_f(R, o);
            rk += (R < ro || (!(ro < R) && lane < o)) ? 1 : 0;
        }
        for (int r = 0; r < nact; ++r) {
            const int q = (int)__builtin_ctzll(__ballot(me && rk == r));
            const uint32_t *cq = C + (size_t)q * pathC;  // C_0: the unshortened codeword (bits)
            const uint32_t *rq = rec + q * RW;
            const size_t row = (size_t)cw * L + r;
            if ((K & 3) == 0) {  // information bits, four per lane and store
                uint32_t *o4 = reinterpret_cast<uint32_t *>(p.info + row * K);
                for (int w = lane; w < (K >> 2); w += 64) {
                    const uint32_t bits = (rq[w >> 3] >> ((w & 7) * 4)) & 15u;
                    o4[w] = (bits & 1u) | ((bits & 2u) << 7) | ((bits & 4u) << 14) | ((bits & 8u) << 21);
                }
            } else {
                for (int kk = lane; kk < K; kk += 64) p.info[row * K + kk] = (uint8_t)((rq[kk >> 5] >> (kk & 31)) & 1u);
            }
            if (p.cw) {
                if ((p.N & 3) == 0) {
                    uint32_t *o4 = reinterpret_cast<uint32_t *>(p.cw + row * p.N);
                    for (int w = lane; w < (p.N >> 2); w += 64) {
                        const int i0 = 4 * w;
                        auto bitat = [&](int i) { return (cq[i >> 5] >> (i & 31)) & 1u; };
                        o4[w] = bitat(p.cwpos[i0]) | (bitat(p.cwpos[i0 + 1]) << 8) |
                                (bitat(p.cwpos[i0 + 2]) << 16) | (bitat(p.cwpos[i0 + 3]) << 24);
                    }
                } else {
                    for (int i = lane; i < p.N; i += 64) {
                        const int ci = p.cwpos[i];
                        p.cw[row * p.N + i] = (uint8_t)((cq[ci >> 5] >> (ci & 31)) & 1u);
                    }
                }
            }
            if (lane == 0) p.metric[row] = rdl_f(R, q);
        }
        if (lane == 0) p.count[cw] = nact;
        wave_sync_p();
    }
}

hipError_t launch_polar(const PolarParams &p, int grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(polar_sclist_kernel, dim3(grid), dim3(64), lds, s, p);
    return hipGetLastError();
}

const void *polar_kernel_ptr() { return reinterpret_cast<const void *>(&polar_sclist_kernel); }

}  // namespace bchk
