// polar_mixed.hip -- batched SC-list decoding of polar codes over MIXED binary kernels (Arikan
// layers and matrix kernels, e.g. BCH-derived ones) on gfx950.
//
// Reference: CMixedKernelListDecoder (out/external/MixedKernelListDecoder.cpp:61-268) over
// CListKernelEngine (out/external/KernelListEngine.cpp:266-447); Arikan layers by the f/g of
// SoftProcessing.cpp:39-80; matrix layers by CTrellisKernelProcessor::GetLLRs
// (out/external/TrellisKernelProcessor.cpp:234-294): the offset state accumulates the known
// kernel inputs times their rows, and the LLR of input `phase` is the min-sum difference
// best[1] - best[0] over the coset of the remaining rows (each word's metric a left-to-right
// float sum of |y| over its disagreeing positions -- the trellis's value bit for bit, see
// oracle/polar_oracle.c). Same decisions, arithmetic and path indices as the CPU restatement.
//
// Execution model: one wave per codeword (persistent). Every path's S (per layer, outer[λ]
// floats), C (kernel inputs per layer) and matrix offset states live in LDS; lane q < L holds
// path q's scalars (metric, leaf LLR, dynamic-freezing mask, record word, stack slot). A
// matrix LLR's coset is split over lanes when there are fewer (path, element) items than lanes
// (float min is exact, so any split gives the same value). The all-Arikan kernel
// (polar_sclist.hip) stays the fast path for codes without matrix layers.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "polar_device.h"

namespace bchk {

namespace {

constexpr uint32_t kUninitM = 0xFFFFFFFFu;

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ float rdlf_m(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint32_t rdlu_m(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t rdlu64_m(uint64_t v, int l) {
    return (uint64_t)rdlu_m((uint32_t)v, l) | ((uint64_t)rdlu_m((uint32_t)(v >> 32), l) << 32);
}

struct MStack {  // TVMemoryEngine's path-index stack with lazy initialisation (misc.h:212-226)
    uint32_t slot;
    int top;
    __device__ __forceinline__ void reset(int L, int lane) {
        top = L;
        if (lane == L) slot = kUninitM;
    }
    __device__ __forceinline__ uint32_t pop(int lane) {
        const uint32_t v = rdlu_m(slot, top);
        if (v == kUninitM) {
            const int r = top - 1;
            top = r;
            if (r > 0 && lane == r) slot = kUninitM;
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

// min over the words of one half of the coset (CTrellisKernelProcessor::GetLLRs, :272-292):
// words c = XOR of rows phase+1 .. l-1 selected by v, v = first, first + step, ...; metric of
// c (b = 0) and c ^ row[phase] (b = 1) against the hard decision
__device__ __forceinline__ void coset_min(const uint32_t *rows, int l, int phase, const float *ay, uint32_t hd,
                                          uint32_t first, uint32_t step, float &b0, float &b1) {
    const int nfree = l - phase - 1;
    const uint32_t nw = 1u << nfree;
    for (uint32_t v = first; v < nw; v += step) {
        uint32_t c = 0;
        for (int r = 0; r < nfree; ++r)
            if ((v >> r) & 1u) c ^= rows[phase + 1 + r];
        const uint32_t d0 = c ^ hd, d1 = d0 ^ rows[phase];
        float m0 = 0.0f, m1 = 0.0f;  // left to right (:279-282)
        for (int j = 0; j < l; ++j) {
            if ((d0 >> j) & 1u) m0 += ay[j];
            if ((d1 >> j) & 1u) m1 += ay[j];
        }
        b0 = m0 < b0 ? m0 : b0;
        b1 = m1 < b1 ? m1 : b1;
    }
}

}  // namespace

__global__ void __launch_bounds__(64) polar_mixed_kernel(PolarMixedParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)threadIdx.x;
    const int U = p.U, nl = p.nl, L = p.L, K = p.K;
    const int RW = polar_rec_words(K);
    // LDS: polar_mixed_lds_bytes (polar_device.h)
    const int o_S = (4 * U + 15) & ~15;
    const int o_C = o_S + 4 * p.ssize * L;
    const int o_O = o_C + p.csize * L;
    const int o_ph = (o_O + p.osize * L + 15) & ~15;
    const int o_rows = (o_ph + 2 * U + 15) & ~15;
    const int o_act = o_rows + 4 * kPolarMaxKernel * nl;
    const int o_tm = (o_act + 4 * L + 4 * L * RW + 15) & ~15;
    float *chan = reinterpret_cast<float *>(smem);
    float *S = reinterpret_cast<float *>(smem + o_S);
    uint8_t *C = smem + o_C;
    uint8_t *O = smem + o_O;
    uint16_t *ph = reinterpret_cast<uint16_t *>(smem + o_ph);
    uint32_t *rows = reinterpret_cast<uint32_t *>(smem + o_rows);  // [layer][row] bitmasks
    uint32_t *act = reinterpret_cast<uint32_t *>(smem + o_act);
    uint32_t *rec = act + L;
    float *tmet = reinterpret_cast<float *>(smem + o_tm);  // trellis state metrics, 2 x tstates
    const bool mine = lane < L;
    for (int i = lane; i < U; i += 64) ph[i] = p.phase[i];
    for (int i = lane; i < kPolarMaxKernel * nl; i += 64) rows[i] = p.krows[i];
    auto Sof = [&](int q, int lam) -> float * { return lam == 0 ? chan : S + (size_t)q * p.ssize + p.soff[lam]; };
    auto Cof = [&](int q, int lam) -> uint8_t * { return C + (size_t)q * p.csize + p.coff[lam]; };
    auto Oof = [&](int q, int j) -> uint8_t * { return O + (size_t)q * p.osize + p.ooff[j]; };
    auto list_act = [&](uint32_t active) {
        if (mine && ((active >> lane) & 1u)) act[__builtin_popcount(active & ((1u << lane) - 1u))] = (uint32_t)lane;
        wsync();
        return __builtin_popcount(active);
    };
    const int lastsz = p.ksize[nl - 1];
    const int lastc = p.coff[nl];
    MStack st;
    st.slot = 0;
    wsync();
    for (uint32_t cw = blockIdx.x; cw < p.B; cw += gridDim.x) {
        const float *y = p.llr + (size_t)cw * p.N;  // LoadLLRs (MixedKernelEncoder.cpp:181-207)
        for (int i = lane; i < U; i += 64) {
            const int m = p.symmap[i];
            chan[i] = m >= 0 ? y[m] : (m == -1 ? 100000.0f : 0.0f);
        }
        st.reset(L, lane);
        const uint32_t pid = st.pop(lane);
        uint32_t active = 1u << pid;
        float R = 0.0f, lv = 0.0f;
        uint64_t dm = 0;
        uint32_t rw = 0;
        int k = 0;
        wsync();
        int nact = list_act(active);
        for (int phi = 0; phi < U; ++phi) {
            const uint32_t e = __builtin_amdgcn_readfirstlane((uint32_t)ph[phi]);
            // ---- IterativelyCalcS (KernelListEngine.cpp:370-447)
            int m = nl - 1;
            uint32_t pq = (uint32_t)phi;
            while (m > 0 && pq % (uint32_t)p.ksize[m] == 0) {
                pq /= (uint32_t)p.ksize[m];
                --m;
            }
            for (int j = m; j < nl; ++j) {
                const int loc = (j == m) ? (int)(pq % (uint32_t)p.ksize[j]) : 0;
                const int d = p.outer[j + 1], l = p.ksize[j];
                const int tot = nact * d;
                if (p.arikan[j]) {
                    for (int it = lane; it < tot; it += 64) {
                        const int q = (int)act[it / d], s = it % d;
                        const float *src = Sof(q, j);
                        float *dst = Sof(q, j + 1);
                        const float a = src[s], b = src[d + s];
                        float r;
                        if (loc) {  // SoftCombine (:39-50)
                            r = Cof(q, j + 1)[s] ? b - a : b + a;
                        } else {    // SoftXOR (:54-80)
                            const float fa = fabsf(a), fb = fabsf(b), mn = fa < fb ? fa : fb;
                            r = __uint_as_float(__float_as_uint(mn) |
                                                ((__float_as_uint(a) ^ __float_as_uint(b)) & 0x80000000u));
                        }
                        dst[s] = r;
                    }
                    wsync();
                    continue;
                }
                // matrix layer: offset state (:240-262), then the min-sum LLR per element
                const uint32_t *kr = rows + kPolarMaxKernel * j;
                for (int it = lane; it < tot; it += 64) {
                    const int q = (int)act[it / d], s = it % d;
                    uint8_t *off = Oof(q, j);
                    if (!loc) {
                        for (int i = 0; i < l; ++i) off[i * d + s] = 0;
                    } else {
                        const uint8_t kn = Cof(q, j + 1)[(loc - 1) * d + s];
                        if (kn)
                            for (int i = 0; i < l; ++i)
                                if ((kr[loc - 1] >> i) & 1u) off[i * d + s] ^= 1u;
                    }
                }
                wsync();
                if (p.trellis[j]) {
                    // CTrellisKernelProcessor::GetLLRs (:260-292) as a pull-form Viterbi: a state
                    // of depth dd + 1 takes the smaller of its (at most two) predecessors' metrics,
                    // each plus |Y| when its edge label differs from the hard decision (min
                    // commutes with the monotone float add, so the values are the reference's).
                    // G lanes per item (G = states of the phase's widest depth, at most 64).
                    const int tp = j * kPolarMaxKernel + loc;
                    const uint8_t *lgp = p.tlog + (size_t)tp * (kPolarMaxKernel + 1);
                    const uint32_t *ent0 = p.tent + p.tbase[tp];
                    int ab = 0;
                    for (int dd = 1; dd <= l; ++dd) ab = lgp[dd] > ab ? lgp[dd] : ab;
                    const int stride = 1 << ab, G = stride < 64 ? stride : 64, ipr = 64 / G;
                    const int slot = lane / G, sub = lane % G;
                    for (int base = 0; base < tot; base += ipr) {
                        const int it = base + slot;
                        const bool have = slot < ipr && it < tot;
                        int q = 0, s = 0;
                        if (have) {
                            q = (int)act[it / d];
                            s = it % d;
                        }
                        const float *src = Sof(q, j);
                        const uint8_t *off = Oof(q, j);
                        float *m0 = tmet + slot * stride, *m1 = tmet + p.tstates + slot * stride;
                        if (have && sub == 0) m0[0] = 0.0f;
                        wsync();
                        const uint32_t *e = ent0;
                        for (int dd = 0; dd < l; ++dd) {
                            const int n1 = 1 << lgp[dd + 1];
                            if (have) {
                                const float v = src[dd * d + s];
                                const float yv = off[dd * d + s] ? -v : v;
                                const bool hd = yv < 0.0f;  // HD = Y < 0 (:270)
                                const float ay = fabsf(yv);
                                for (int S1 = sub; S1 < n1; S1 += G) {
                                    const uint32_t w = e[S1], a = w & 0xFFFFu, b = w >> 16;
                                    float x = m0[a & kTrellisState];
                                    if (((a & kTrellisZ) != 0u) != hd) x = x + ay;
                                    if (b & kTrellisValid) {
                                        float xb = m0[b & kTrellisState];
                                        if (((b & kTrellisZ) != 0u) != hd) xb = xb + ay;
                                        x = xb < x ? xb : x;
                                    }
                                    m1[S1] = x;
                                }
                            }
                            wsync();
                            float *tt = m0;
                            m0 = m1;
                            m1 = tt;
                            e += n1;
                        }
                        if (have && sub == 0) Sof(q, j + 1)[s] = m0[1] - m0[0];  // (:292)
                        wsync();
                    }
                    continue;
                }
                // lanes per item: the coset split when items are fewer than lanes
                int lpi = 1;
                const int nfree = l - loc - 1;
                while (lpi * 2 * tot <= 64 && (lpi * 2) <= (1 << (nfree < 6 ? nfree : 6))) lpi *= 2;
                const int span = 64 / lpi * lpi;  // lanes used per round
                for (int base = 0; base < tot * lpi; base += span) {
                    const int g = base + lane;
                    const bool have = lane < span && g < tot * lpi;
                    const int it = g / lpi, sub = g % lpi;
                    float b0 = __int_as_float(0x7F800000), b1 = __int_as_float(0x7F800000);
                    int q = 0, s = 0;
                    if (have) {
                        q = (int)act[it / d];
                        s = it % d;
                        const float *src = Sof(q, j);
                        const uint8_t *off = Oof(q, j);
                        float ay[kPolarMaxKernel];
                        uint32_t hd = 0;
                        for (int jj = 0; jj < l; ++jj) {
                            const float v = src[jj * d + s];
                            const float yv = off[jj * d + s] ? -v : v;
                            if (yv < 0.0f) hd |= 1u << jj;  // HD = Y < 0 (:276)
                            ay[jj] = fabsf(yv);
                        }
                        coset_min(kr, l, loc, ay, hd, (uint32_t)sub, (uint32_t)lpi, b0, b1);
                    }
                    for (int o = 1; o < lpi; o <<= 1) {  // min over the item's lanes (exact)
                        const float x0 = __shfl_xor(b0, o, 64), x1 = __shfl_xor(b1, o, 64);
                        b0 = x0 < b0 ? x0 : b0;
                        b1 = x1 < b1 ? x1 : b1;
                    }
                    if (have && sub == 0) Sof(q, j + 1)[s] = b1 - b0;  // (:292)
                }
                wsync();
            }
            const bool on = mine && ((active >> lane) & 1u);
            if (on) lv = Sof(lane, nl)[0];
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
                // ---- ContinuePathsUnfrozen (:100-185): candidate 2q + b in lane 2q + b
                const int q = lane >> 1, b = lane & 1;
                const float vq = __shfl(lv, q & 31), Rq = __shfl(R, q & 31);
                const bool valid = q < L && ((active >> q) & 1u);
                float sc = 0.0f;
                if (valid) sc = (b == (vq < 0.0f ? 1 : 0)) ? Rq : Rq - fabsf(vq);
                int rank = 0;  // std::greater<pair<float, unsigned>> (:125)
                for (uint64_t mm = __ballot(valid); mm; mm &= mm - 1) {
                    const int o = (int)__builtin_ctzll(mm);
                    const float so = rdlf_m(sc, o);
                    rank += (sc < so || (!(so < sc) && lane < o)) ? 1 : 0;
                }
                const int J = 2 * nact, keep = J < L ? J : L;
                const uint64_t sel = __ballot(valid && rank < keep);
                const uint32_t cont = mine ? (uint32_t)((sel >> (2 * lane)) & 3ull) : 0u;
                const uint32_t cont_any = (uint32_t)__ballot(cont != 0);
                const uint32_t clones = (uint32_t)__ballot(cont == 3u);
                for (uint32_t kill = active & ~cont_any; kill; kill &= kill - 1) st.push((uint32_t)__builtin_ctz(kill), lane);
                active &= cont_any;
                dec = cont == 2u ? 1u : (cont == 3u ? (lv < 0.0f ? 1u : 0u) : 0u);
                for (uint32_t cl = clones; cl; cl &= cl - 1) {
                    const int l = __builtin_ctz(cl);
                    const int l1 = (int)st.pop(lane);  // ClonePath: the whole path state
                    for (int i = lane; i < p.ssize; i += 64) S[(size_t)l1 * p.ssize + i] = S[(size_t)l * p.ssize + i];
                    for (int i = lane; i < p.csize; i += 64) C[(size_t)l1 * p.csize + i] = C[(size_t)l * p.csize + i];
                    for (int i = lane; i < p.osize; i += 64) O[(size_t)l1 * p.osize + i] = O[(size_t)l * p.osize + i];
                    for (int i = lane; i < (k >> 5); i += 64) rec[l1 * RW + i] = rec[l * RW + i];
                    const float Rl = rdlf_m(R, l), vl = rdlf_m(lv, l);
                    const uint64_t dml = rdlu64_m(dm, l);
                    const uint32_t rwl = rdlu_m(rw, l), decl = rdlu_m(dec, l);
                    if (lane == l1) {
                        R = Rl - fabsf(vl);
                        dm = dml;
                        rw = rwl;
                        dec = decl ^ 1u;
                        lv = vl;
                    }
                    active |= 1u << l1;
                }
                wsync();
            }
            const bool now = mine && ((active >> lane) & 1u);
            if (now) {
                C[(size_t)lane * p.csize + lastc + (phi % lastsz)] = (uint8_t)dec;
                if (dec) dm ^= corr;
            }
            if (!(e & kPhaseFrozen)) {
                if (now) rw |= dec << (k & 31);
                ++k;
                if ((k & 31) == 0) {
                    if (now) rec[lane * RW + (k >> 5) - 1] = rw;
                    rw = 0;
                }
                nact = list_act(active);
            } else {
                wsync();
            }
            // ---- IterativelyUpdateC (KernelListEngine.cpp:266-315): finished blocks are
            // multiplied by their kernel into the parent layer's inputs
            {
                int lam = nl, stride = 1;
                uint32_t ph2 = (uint32_t)phi;
                while (lam > 0 && (ph2 + 1) % (uint32_t)p.ksize[lam - 1] == 0) {
                    const int l = p.ksize[lam - 1];
                    const uint32_t psi = ph2 / (uint32_t)l;
                    const int next = stride * l;
                    const int phi0 = lam > 1 ? (int)(psi % (uint32_t)p.ksize[lam - 2]) * next : 0;
                    const uint32_t *kr = rows + kPolarMaxKernel * (lam - 1);
                    const int tot = nact * stride;
                    for (int it = lane; it < tot; it += 64) {
                        const int q = (int)act[it / stride], s = it % stride;
                        const uint8_t *x = Cof(q, lam);
                        uint8_t *yo = Cof(q, lam - 1) + phi0;
                        // (y_i) = (x_j) K: y_i = XOR over rows j with K[j][i] (LinAlg.cpp:685-709)
                        uint32_t xin = 0;
                        for (int jj = 0; jj < l; ++jj) xin |= (uint32_t)(x[jj * stride + s] & 1u) << jj;
                        for (int i = 0; i < l; ++i) {
                            uint32_t acc = 0;
                            for (int jj = 0; jj < l; ++jj) acc ^= ((xin >> jj) & (kr[jj] >> i)) & 1u;
                            yo[i * stride + s] = (uint8_t)acc;
                        }
                    }
                    wsync();
                    stride = next;
                    ph2 = psi;
                    --lam;
                }
            }
        }
        if ((k & 31) && mine && ((active >> lane) & 1u)) rec[lane * RW + (k >> 5)] = rw;
        wsync();
        // ---- final order (:249-267): active paths by (R, index), descending
        int rk = 0;
        const bool me = mine && ((active >> lane) & 1u);
        for (uint64_t mm = __ballot(me); mm; mm &= mm - 1) {
            const int o = (int)__builtin_ctzll(mm);
            const float ro = rdlf_m(R, o);
            rk += (R < ro || (!(ro < R) && lane < o)) ? 1 : 0;
        }
        for (int r = 0; r < nact; ++r) {
            const int q = (int)__builtin_ctzll(__ballot(me && rk == r));
            const uint8_t *cq = C + (size_t)q * p.csize;  // C_0: the unshortened codeword
            const uint32_t *rq = rec + q * RW;
            const size_t row = (size_t)cw * L + r;
            for (int kk = lane; kk < K; kk += 64) p.info[row * K + kk] = (uint8_t)((rq[kk >> 5] >> (kk & 31)) & 1u);
            if (p.cw)
                for (int i = lane; i < p.N; i += 64) p.cw[row * p.N + i] = cq[p.cwpos[i]];
            if (lane == 0) p.metric[row] = rdlf_m(R, q);
        }
        if (lane == 0) p.count[cw] = nact;
        wsync();
    }
}

hipError_t launch_polar_mixed(const PolarMixedParams &p, int grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(polar_mixed_kernel, dim3(grid), dim3(64), lds, s, p);
    return hipGetLastError();
}

const void *polar_mixed_kernel_ptr() { return reinterpret_cast<const void *>(&polar_mixed_kernel); }

}  // namespace bchk
