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
// Execution model: one 64-lane wave per codeword (persistent over the batch), every path's
// state in LDS. Layer λ of path p keeps its LLRs S_λ (U >> λ floats) and partial sums C_λ
// (kernel inputs of the current block, U >> (λ-1) bytes; C_0 = the codeword). Each phase:
//   * the LLR recursion from the first layer whose block changed, lanes over
//     (active path x element);
//   * decisions: frozen symbols per path (lane = path); unfrozen ones rank the 2 L
//     candidates (lane = path x bit) with the reference's std::greater<pair> order,
//     then kills and clones run wave-uniformly in path order (clone = LDS copy of the
//     parent's arrays);
//   * the partial-sum butterflies of the finished blocks.
// No MFMA: the work is float min/add and byte XOR on short vectors.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "polar_device.h"

namespace bchk {

namespace {

__device__ __forceinline__ void wave_sync_p() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// offsets inside one path's arrays: S_λ (λ >= 1) and C_λ
__device__ __forceinline__ int s_off(int U, int lam) { return U - (U >> (lam - 1)); }
__device__ __forceinline__ int c_off(int U, int lam) {
    return lam == 0 ? 0 : (lam == 1 ? U : 3 * U - (U >> (lam - 2)));
}

// SoftXOR (SoftProcessing.cpp:54-80): sign(a) sign(b) min(|a|, |b|)
__device__ __forceinline__ float f_minsum(float a, float b) {
    const float fa = fabsf(a), fb = fabsf(b);
    const float m = fa < fb ? fa : fb;
    return __uint_as_float(__float_as_uint(m) | ((__float_as_uint(a) ^ __float_as_uint(b)) & 0x80000000u));
}

__device__ __forceinline__ float rdl_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// The path stack of TVMemoryEngine (headers/external/misc.h:212-226), in LDS: every lane
// reads, lane 0 writes.
__device__ __forceinline__ uint32_t st_pop(uint32_t *s, int lane) {
    const uint32_t top = s[0], v = s[top];
    uint32_t r;
    wave_sync_p();
    if (v == 0xFFFFFFFFu) {  // not yet initialised: hand out top - 1
        r = top - 1u;
        if (lane == 0) {
            s[0] = r;
            if (r > 0) s[r] = 0xFFFFFFFFu;
        }
    } else {
        r = v;
        if (lane == 0) s[0] = top - 1u;
    }
    wave_sync_p();
    return r;
}
__device__ __forceinline__ void st_push(uint32_t x, uint32_t *s, int lane) {
    const uint32_t top = s[0] + 1u;
    wave_sync_p();
    if (lane == 0) {
        s[top] = x;
        s[0] = top;
    }
    wave_sync_p();
}

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
    const int U = p.U, n = p.n, L = p.L;
    const int pathS = U, pathC = 3 * U;  // padded per-path strides (floats, bytes)
    // LDS layout: polar_lds_bytes (polar_device.h)
    float *chan = reinterpret_cast<float *>(smem);
    float *S = chan + U;
    float *Rv = S + (size_t)pathS * L;
    float *lv = Rv + L;
    uintptr_t a8 = (reinterpret_cast<uintptr_t>(lv + L) + 7u) & ~uintptr_t(7);
    uint64_t *dfm = reinterpret_cast<uint64_t *>(a8);
    uint32_t *stack = reinterpret_cast<uint32_t *>(dfm + L);
    uint32_t *act = stack + L + 1;
    uintptr_t a16 = (reinterpret_cast<uintptr_t>(act + L) + 15u) & ~uintptr_t(15);
    uint8_t *C = reinterpret_cast<uint8_t *>(a16);
    uint8_t *tmp = C + (size_t)pathC * L;
    const int lastc = c_off(U, n);  // C_n: the two inputs of the last Arikan block

    for (uint32_t cw = blockIdx.x; cw < p.B; cw += gridDim.x) {
        // ---- LoadLLRs (MixedKernelEncoder.cpp:181-207)
        const float *y = p.llr + (size_t)cw * p.N;
        for (int i = lane; i < U; i += 64) {
            const int m = p.symmap[i];
            chan[i] = m >= 0 ? y[m] : (m == -1 ? 100000.0f : 0.0f);
        }
        // ---- Cleanup + AssignInitialPath (TVMemoryEngine.cpp:58-94)
        if (lane == 0) {
            stack[0] = (uint32_t)L;
            stack[L] = 0xFFFFFFFFu;
        }
        wave_sync_p();
        const uint32_t pid = st_pop(stack, lane);
        uint32_t active = 1u << pid;
        if (lane == 0) {
            Rv[pid] = 0.0f;
            dfm[pid] = 0ull;
        }
        wave_sync_p();
        int nact = list_active(active, act, lane, L);

        for (int phi = 0; phi < U; ++phi) {
            // ---- IterativelyCalcS (KernelListEngine.cpp:370-447): from layer m, where the
            // block of phase phi starts, down to the single LLR of layer n
            int m = 0, local = 0;
            if (phi) {
                const int tz = __builtin_ctz((unsigned)phi);
                m = n - 1 - tz;
                local = 1;
            }
            for (int j = m; j < n; ++j) {
                const int loc = (j == m) ? local : 0;
                const int lgd = n - 1 - j;  // d = U >> (j + 1)
                const int d = 1 << lgd;
                const int tot = nact << lgd;
                for (int it = lane; it < tot; it += 64) {
                    const int q = (int)act[it >> lgd], s = it & (d - 1);
                    const float *src = (j == 0) ? chan : S + (size_t)q * pathS + s_off(U, j);
                    float *dst = S + (size_t)q * pathS + s_off(U, j + 1);
                    const float a = src[s], b = src[d + s];
                    float r;
                    if (loc) {  // SoftCombine (:39-50): b - a if u = 1 else b + a
                        r = C[(size_t)q * pathC + c_off(U, j + 1) + s] ? b - a : b + a;
                    } else {
                        r = f_minsum(a, b);
                    }
                    dst[s] = r;
                }
                wave_sync_p();
            }
            if (lane < L && ((active >> lane) & 1u)) lv[lane] = S[(size_t)lane * pathS + U - 2];
            wave_sync_p();

            if (p.frozen[phi]) {
                // ---- ContinuePathsFrozen (MixedKernelListDecoder.cpp:61-98)
                const int db = p.dfbit[phi];
                const uint64_t corr = p.dfcorr[phi];
                if (lane < L && ((active >> lane) & 1u)) {
                    const float v = lv[lane];
                    const int cb = db >= 0 ? (int)((dfm[lane] >> db) & 1ull) : 0;
                    if ((cb > 0) ^ (v < 0.0f)) Rv[lane] -= fabsf(v);
                    C[(size_t)lane * pathC + lastc + (phi & 1)] = (uint8_t)cb;
                    if (cb) dfm[lane] ^= corr;
                }
                wave_sync_p();
            } else {
                // ---- ContinuePathsUnfrozen (:100-185). Candidate 2q + b (bit b of path q)
                // sits in lane 2q + b; its score is R (b = hard decision) or R - |llr|.
                const int q = lane >> 1, b = lane & 1;
                const bool valid = q < L && ((active >> q) & 1u);
                float sc = 0.0f;
                if (valid) {
                    const float v = lv[q];
                    const int hd = v < 0.0f;
                    sc = (b == hd) ? Rv[q] : Rv[q] - fabsf(v);
                }
                // rank under std::greater<pair<float, unsigned>> (:125): score, then index
                int rank = 0;
                for (uint64_t mm = __ballot(valid); mm; mm &= mm - 1) {
                    const int o = (int)__builtin_ctzll(mm);
                    const float so = rdl_f(sc, o);
                    rank += (sc < so || (!(so < sc) && lane < o)) ? 1 : 0;
                }
                const int J = 2 * nact, keep = J < L ? J : L;
                const uint64_t sel = __ballot(valid && rank < keep);
                const uint64_t corr = p.dfcorr[phi];
                for (int i = 0; i < L; ++i)  // KillPath, in path order (:129-136)
                    if (((active >> i) & 1u) && !((sel >> (2 * i)) & 3ull)) {
                        st_push((uint32_t)i, stack, lane);
                        active &= ~(1u << i);
                    }
                for (int l = 0; l < L; ++l) {  // continuations, in path order (:138-178)
                    const int cont = (int)((sel >> (2 * l)) & 3ull);
                    if (!cont) continue;
                    uint8_t *cl = C + (size_t)l * pathC + lastc + (phi & 1);
                    if (cont == 1) {
                        if (lane == 0) *cl = 0;
                    } else if (cont == 2) {
                        if (lane == 0) {
                            *cl = 1;
                            dfm[l] ^= corr;
                        }
                    } else {
                        const float v = lv[l];
                        const uint8_t cb = v < 0.0f;
                        if (lane == 0) *cl = cb;
                        wave_sync_p();
                        const uint32_t l1 = st_pop(stack, lane);  // ClonePath
                        {
                            const uint32_t *s4 = reinterpret_cast<const uint32_t *>(S + (size_t)l * pathS);
                            uint32_t *d4 = reinterpret_cast<uint32_t *>(S + (size_t)l1 * pathS);
                            for (int i = lane; i < pathS; i += 64) d4[i] = s4[i];
                            const uint32_t *c4 = reinterpret_cast<const uint32_t *>(C + (size_t)l * pathC);
                            uint32_t *e4 = reinterpret_cast<uint32_t *>(C + (size_t)l1 * pathC);
                            for (int i = lane; i < pathC / 4; i += 64) e4[i] = c4[i];
                        }
                        wave_sync_p();
                        if (lane == 0) {
                            C[(size_t)l1 * pathC + lastc + (phi & 1)] = (uint8_t)(cb ^ 1u);
                            Rv[l1] = Rv[l] - fabsf(v);
                            const uint64_t dm = dfm[l];
                            dfm[l1] = cb ? dm : dm ^ corr;
                            dfm[l] = cb ? dm ^ corr : dm;
                        }
                        active |= 1u << l1;
                    }
                    wave_sync_p();
                }
                nact = list_active(active, act, lane, L);
            }

            // ---- IterativelyUpdateC (KernelListEngine.cpp:266-315): the blocks this phase
            // completes are encoded into their parents' slots
            {
                int lam = n, lgs = 0, ph = phi;
                while (lam > 0 && (ph & 1)) {
                    const int psi = ph >> 1;
                    const int stride = 1 << lgs, next = stride << 1;
                    const int phi0 = (lam > 1) ? (psi & 1) * next : 0;
                    const int tot = nact << lgs;
                    for (int it = lane; it < tot; it += 64) {
                        const int q = (int)act[it >> lgs], s = it & (stride - 1);
                        const uint8_t *src = C + (size_t)q * pathC + c_off(U, lam);
                        uint8_t *dst = C + (size_t)q * pathC + c_off(U, lam - 1) + phi0;
                        const uint8_t x0 = src[s], x1 = src[stride + s];
                        dst[s] = (uint8_t)(x0 ^ x1);
                        dst[stride + s] = x1;
                    }
                    wave_sync_p();
                    ++lgs;
                    ph = psi;
                    --lam;
                }
            }
        }

        // ---- final order (:249-267): active paths by (R, index), descending
        int rk = 0;
        float rv = 0.0f;
        const bool me = lane < L && ((active >> lane) & 1u);
        if (me) rv = Rv[lane];
        for (uint64_t mm = __ballot(me); mm; mm &= mm - 1) {
            const int o = (int)__builtin_ctzll(mm);
            const float ro = rdl_f(rv, o);
            rk += (rv < ro || (!(ro < rv) && lane < o)) ? 1 : 0;
        }
        const uint64_t mme = __ballot(me);
        for (int r = 0; r < nact; ++r) {
            const uint64_t who = __ballot(me && rk == r);
            const int q = (int)__builtin_ctzll(who);
            const uint8_t *cq = C + (size_t)q * pathC;  // C_0: the unshortened codeword
            // information bits: the inverse transform (= the transform, stages commute)
            for (int i = lane; i < U; i += 64) tmp[i] = cq[i];
            wave_sync_p();
            for (int st = 1; st < U; st <<= 1) {
                for (int i = lane; i < U / 2; i += 64) {
                    const int lo = ((i & ~(st - 1)) << 1) | (i & (st - 1));
                    tmp[lo] ^= tmp[lo + st];
                }
                wave_sync_p();
            }
            const size_t row = (size_t)cw * L + r;
            for (int k = lane; k < p.K; k += 64) p.info[row * p.K + k] = tmp[p.infopos[k]];
            if (p.cw)
                for (int i = lane; i < p.N; i += 64) p.cw[row * p.N + i] = cq[p.cwpos[i]];
            if (lane == 0) p.metric[row] = Rv[q];
            wave_sync_p();
        }
        (void)mme;
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
