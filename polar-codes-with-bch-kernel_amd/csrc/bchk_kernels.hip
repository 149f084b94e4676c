// bchk_kernels.hip -- gfx950 (CDNA4) kernels for Kaneko's soft-decision search over a
// binary BCH(n, k) code, the hot path of src/KanekoKernelProcessor.cpp:335-407 and
// src/Decoder.cpp:184-321 of the reference.
//
// Execution model (one 64-lane wave per codeword, persistent waves):
//   prep    lane = channel position: alpha = 2y/s2 (IEEE f64 division), hard decision,
//           |alpha|; exact rank by (|alpha|, position) with wave-uniform readlanes; the
//           sorted reliabilities are scattered to the wave's LDS slice.
//   search  lane = test pattern: 64 consecutive test patterns i = base + lane are decoded
//           speculatively in parallel. A pattern's syndrome is the XOR of the hard
//           decision's syndrome with the odd-syndrome columns of its flipped positions
//           (GF(2)-linear, 3 XORs per word per lane); the key equation is solved with
//           inversionless binary Berlekamp-Massey (== the reference's Euclid, see
//           oracle/bchk_oracle.c:orc_alg_decode_bm) and roots are found by a GF(2)-linear
//           Chien map (table XOR) or an incremental Chien scan (m >= 7).
//   accept  the reference's sequential acceptance logic (m0, l0, calcRightSide, calcT
//           scan, loop bound) runs wave-uniformly over the successful lanes in pattern
//           order; its f64 sums are formed in exactly the reference's order. calcT(j) for
//           all j is evaluated lane-parallel (one j per lane).
// No MFMA: there is no dense contraction here; the work is GF table/bit arithmetic.
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdlib.h>
#include <stdint.h>

#include "bchk_core.h"
#include "bchk_launch.h"
#include "bchk_search.h"

namespace bchk {

// Waves per SIMD the registers must allow: 5 for the first pass with the syndrome table
// (its LDS allows 5 workgroups per CU; left alone it takes 98 VGPRs, 4 waves), the compiler's
// choice otherwise (the tail instance needs ~220). BCHK_SEARCH_WPE: experiment builds.
#ifdef BCHK_SEARCH_WPE
#define BCHK_SEARCH_ATTR __attribute__((amdgpu_waves_per_eu(BCHK_SEARCH_WPE)))
#else
#ifndef BCHK_FIRST_WPE
#define BCHK_FIRST_WPE 5  // measured: 6 / 7 / 8 (spilling) are slower (profiles/r03_help/bench_fwpe*.json)
#endif
#define BCHK_SEARCH_ATTR __attribute__((amdgpu_waves_per_eu((TAB && !AN) ? BCHK_FIRST_WPE : 1)))
#endif
template <int M, int TMAX, bool TAB, bool AN>
__global__ void __launch_bounds__(kWaveSize * kWavesPerBlock) BCHK_SEARCH_ATTR
kaneko_search_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // the first pass with the syndrome table never runs the Chien search: its tables stop
    // before the Chien rows (the last table), which leaves LDS for more waves
    const uint32_t tbytes = (TAB && !AN) ? p.td.off_chien : p.td.bytes;
    load_tables(smem, p.tables, tbytes);
    constexpr int WB0 = Smem<M, TMAX>::WAVE_BYTES, SB0 = WB0 + (AN ? an_bytes<M, TMAX>() : 0);
    if constexpr (AN && an_capable<M, TMAX>()) {
        if (p.an_help && threadIdx.x < 64) {  // the helper job control: no job, nobody idle
            HelpCtl *h = reinterpret_cast<HelpCtl *>(smem + ((p.td.bytes + 15) & ~15u) + kWavesPerBlock * SB0);
            if (threadIdx.x == 0) {
                h->idle = 0u;
                h->owner = 0u;
                h->gen = 0u;
                h->next = kHelpNone;
                h->consumed = 0u;
            }
            if (threadIdx.x < kHelpSlots) h->slot[threadIdx.x].tag = 0u;
        }
    }
    __syncthreads();
    const uint8_t *ex = smem + p.td.off_exp;
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(smem + p.td.off_log);
    const uint32_t *col = reinterpret_cast<const uint32_t *>(smem + p.td.off_col);
    const uint64_t *chien = (TAB && !AN) ? nullptr : reinterpret_cast<const uint64_t *>(smem + p.td.off_chien);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int NP = Smem<M, TMAX>::NP;
    // per wave: the prep's LDS slice, then the analytic tail's state (n <= 63)
    constexpr int WB = Smem<M, TMAX>::WAVE_BYTES, SB = WB + (AN ? an_bytes<M, TMAX>() : 0);
    uint8_t *wbase = smem + ((tbytes + 15) & ~15u) + wid * SB;
    double *as = reinterpret_cast<double *>(wbase);
    double *ap = as + NP;
    uint8_t *ordl = wbase + NP * 16;
    AnWave *an = (AN && an_capable<M, TMAX>()) ? reinterpret_cast<AnWave *>(wbase + WB) : nullptr;
    // helper waves (analytic tail kernel): the block's job control after the wave slices
    uint8_t *waves0 = smem + ((p.td.bytes + 15) & ~15u);
    HelpCtl *help = nullptr;
    if constexpr (AN && an_capable<M, TMAX>()) {
        if (p.an_help) help = reinterpret_cast<HelpCtl *>(waves0 + kWavesPerBlock * SB);
    }
    // Three sources of codewords -- the first pass's hand-offs as they come (the analytic
    // tail beside the first pass), grid-stride over the batch (no queue), or the work queue
    // left by the fast path (sub-queue x holds items x, x+8, ...; a wave drains its own
    // XCD's sub-queue first, one L2-local atomic per codeword, then steals) -- feeding ONE
    // call of search_codeword: with a single call site it is inlined, so the LDS state and
    // the parameters stay in their own address spaces (ds_* and scalar loads). A second call
    // site made it an outlined function taking generic pointers: every LDS access a flat
    // access and the parameter block spilled to scratch.
    const bool live = AN && p.in_queue;
    const uint32_t stride = gridDim.x * kWavesPerBlock;
    uint32_t gs = blockIdx.x * kWavesPerBlock + wid;
    const uint32_t total = (!live && p.queue) ? *p.qcount : 0u;
    const uint32_t nfront = (!live && p.queue && p.qfront_n) ? *p.qfront_n : total;  // past it: the back
    // more waves than work: nothing to take (a helper wave of the tail kernel still helps)
    const bool none = !live && p.queue && gs >= total;
    if (none && !help) return;
    int x = xcc_id(), exhausted = none ? 8 : 0;
    uint32_t ndone = 0;
    for (;;) {
        uint32_t cw = kEmptySlot, item = 0;
#ifdef BCHK_FP_TRACE
        // diagnostic build (never the product): per-codeword timeline of the first pass on
        // the 100 MHz clock into the tail diagnostics buffer, tagged 0xF in word 0's top nibble
        // (scripts/fp_trace.py, profiles/r06_fp/)
        uint64_t fpt[3] = {0, 0, 0};
        const uint64_t fp_t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t fp_c0 = __builtin_amdgcn_s_memtime();
#endif
        if (live) {
            if (lane == 0) cw = tail_dequeue(p, item);
            cw = (uint32_t)__shfl((int)cw, 0, 64);
            item = (uint32_t)__shfl((int)item, 0, 64);
            if (cw == kEmptySlot) break;
            if (cw >= p.count) continue;  // never a valid slot value
        } else if (!p.queue) {
            if (gs >= p.count) break;
            cw = gs;
            item = gs;
            gs += stride;
        } else {
            if (exhausted >= 8) break;
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(p.heads + 32 * x, 1u);
            k = (uint32_t)__shfl((int)k, 0, 64);
            item = (uint32_t)x + 8u * k;
            if (item >= total) {
                x = (x + 1) & 7;
                ++exhausted;
                continue;
            }
            const uint32_t qi = item < nfront ? item : p.count - 1u - (item - nfront);
            cw = p.queue[qi];
        }
        if (cw < p.count)  // never otherwise: no access outside the batch
        {
#ifdef BCHK_FP_TRACE
            const uint64_t fp_t1 = __builtin_amdgcn_s_memrealtime();
            search_codeword<M, TMAX, TAB, AN>(p, ex, lg, col, chien, as, ap, ordl, cw, lane, an, item, help, wid,
                                              AN ? nullptr : fpt);
            if (!AN && p.tail_diag && p.tail_diag_count && lane == 0) {
                const uint64_t fp_t4 = __builtin_amdgcn_s_memrealtime(), fp_c4 = __builtin_amdgcn_s_memtime();
                const uint32_t r = atomicAdd(p.tail_diag_count, 1u);
                if (r < p.tail_diag_cap) {
                    unsigned long long *d = p.tail_diag + (size_t)r * 8;
                    uint32_t hw;
                    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                    d[0] = (0xFull << 60) | cw;
                    d[1] = fp_t0;
                    d[2] = fp_t1;
                    d[3] = fpt[0];
                    d[4] = fpt[1];
                    d[5] = fp_t4;
                    d[6] = fpt[2] | (uint64_t)xcc_id() << 20 | (uint64_t)hw << 32;
                    d[7] = fp_c4 - fp_c0;
                }
            }
#else
            search_codeword<M, TMAX, TAB, AN>(p, ex, lg, col, chien, as, ap, ordl, cw, lane, an, item, help, wid);
#endif
        }
        ++ndone;
    }
    wave_done(p, lane, ndone);
    if constexpr (AN && an_capable<M, TMAX>()) {
        if (help) {  // past its last codeword: help the siblings until all of them are
            if (lane == 0) atomicAdd(&help->idle, 1u);
            help_loop<M, TMAX, TAB>(help, p, ex, lg, chien, waves0, SB, lane);
        }
    }
}

// --------------------------------------- long codes: first patterns of every codeword
// The counterpart of the n <= 63 fast path (bchk_fast.hip) for m >= 7: one wave per
// codeword, grid-stride over the batch, with only the prep and first_patterns in the
// kernel, so it holds fewer registers than the search kernel and keeps more waves in flight
// to hide the channel loads. A codeword whose search has not ended goes to the exact
// kernel's queue (one atomic per queued codeword), which starts it from scratch.
// The hard decision's odd syndromes of codeword cw (prep_syndromes' S0, from the row alone:
// yH = (2y/s2 > 0), :336-342, Decoder::findSyndromPoly :184-207)
template <int M, int TMAX>
__device__ __forceinline__ void hard_syndromes(const SearchParams &p, const uint32_t *col, uint32_t cw, int lane,
                                               uint32_t (&S0)[Prep<M, TMAX>::W]) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW, W = Prep<M, TMAX>::W;
    double yv[NW];
    load_row<M>(p, cw, lane, yv);
#pragma unroll
    for (int w = 0; w < W; ++w) S0[w] = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int pos = lane + 64 * s;
        const double al = (2.0 * yv[s]) / p.s2;
        if (pos < N && !(al <= 0.0)) {
#pragma unroll
            for (int w = 0; w < W; ++w) S0[w] ^= col[pos * W + w];
        }
    }
#pragma unroll
    for (int w = 0; w < W; ++w) S0[w] = wave_xor(S0[w]);
}

// SEL (no stats record requested, so an exact tie beyond the selection is not observable):
// the order by prep_select, and the fused counters summed per wave (one set of atomics per
// wave instead of per codeword).
// Each wave decodes kFirstPerWave consecutive codewords. Without a stats record their sent
// words come into LDS, and their decoded words leave it, as one contiguous block of
// kFirstPerWave rows moved with 8-B accesses (the row of one codeword is n bytes at an odd
// offset: byte accesses, one per lane per 64 positions, cost the memory pipe more than the
// bytes); rows not finished here (queued) are left to the search kernel and stored by it.
constexpr uint32_t kFirstPerWave = 8;
constexpr int kFirstBlockBytes = 2048;  // kFirstPerWave rows of n <= 255 bytes
constexpr int kFirstWaveExtra = 2 * kFirstBlockBytes + 256;  // + four words' pattern-0 results
#ifndef BCHK_LONGFIRST_WPE  // experiment builds set it (waves per SIMD the allocation targets)
#define BCHK_LONGFIRST_WPE 4
#endif
template <int M, int TMAX, bool SEL>
__global__ void __launch_bounds__(kWaveSize * kWavesPerBlock) __attribute__((amdgpu_waves_per_eu(BCHK_LONGFIRST_WPE)))
kaneko_first_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    load_tables(smem, p.tables, p.td.bytes);
    __syncthreads();
    const uint8_t *ex = smem + p.td.off_exp;
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(smem + p.td.off_log);
    const uint32_t *col = reinterpret_cast<const uint32_t *>(smem + p.td.off_col);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int NP = Smem<M, TMAX>::NP, NW = Geo<M>::NW, N = Geo<M>::N;
    static_assert(kFirstPerWave * N <= kFirstBlockBytes, "a wave's rows fit its block");
    uint8_t *wbase = smem + ((p.td.bytes + 15) & ~15u) + wid * Smem<M, TMAX>::WAVE_BYTES;
    double *as = reinterpret_cast<double *>(wbase);
    double *ap = as + NP;
    uint8_t *ordl = wbase + NP * 16;
    // the wave's row blocks (SEL): sent words, decoded words
    uint8_t *txs = smem + ((p.td.bytes + 15) & ~15u) + kWavesPerBlock * Smem<M, TMAX>::WAVE_BYTES +
                   wid * kFirstWaveExtra;
    uint8_t *rss = txs + kFirstBlockBytes;
    uint64_t *e4s = reinterpret_cast<uint64_t *>(rss + kFirstBlockBytes);  // [4][NW] + ok flags
    const uint32_t cw0 = (blockIdx.x * kWavesPerBlock + wid) * kFirstPerWave;
    if (cw0 >= p.count) return;
    const uint32_t nrows = p.count - cw0 < kFirstPerWave ? p.count - cw0 : kFirstPerWave;
    const uint32_t nbytes = nrows * (uint32_t)N;
    // rows the lane pre-pass finished (kaneko_lane_kernel) are not touched
    static_assert(64 % kFirstPerWave == 0, "a wave's rows lie in one pre_mask word");
    const uint32_t rmask = (1u << nrows) - 1u;
    const uint32_t skip = p.pre_mask ? (uint32_t)(p.pre_mask[cw0 >> 6] >> (cw0 & 63u)) & rmask : 0u;
    if (skip == rmask) return;
    const uint32_t todo = rmask & ~skip;
    // 8-B pieces: row blocks start at a multiple of 8 rows (8 N bytes); the tail of a ragged
    // last block byte by byte
    const bool wide = nrows == kFirstPerWave && ((reinterpret_cast<uintptr_t>(p.tx) | reinterpret_cast<uintptr_t>(p.res)) & 7u) == 0;
    if (SEL && p.cnt) {
        const uint8_t *src = p.tx + (size_t)cw0 * N;
        if (wide) {
            for (uint32_t q = (uint32_t)lane; q < nbytes / 8u; q += 64u)
                reinterpret_cast<uint64_t *>(txs)[q] = reinterpret_cast<const uint64_t *>(src)[q];
        } else {
            for (uint32_t q = (uint32_t)lane; q < nbytes; q += 64u) txs[q] = src[q];
        }
    }
    // the next codeword's row is loaded while this one is decoded (its latency hidden)
    // (and its sent word, for the fused counters at the output step, with a stats record)
    double ynext[NW];
    TxPre<NW> txnext{{}, false};
    const uint32_t kfirst = (uint32_t)__builtin_ctz(todo);
    load_row<M>(p, cw0 + kfirst, lane, ynext);
    if (!SEL) txnext = tx_prefetch<M>(p, cw0 + kfirst, lane);
    unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
    uint32_t fin = 0;     // SEL: rows finished here (bit k: codeword cw0 + k)
    double l0k = 0.0;     // SEL: lane k holds codeword cw0 + k's l0
    for (uint32_t k = kfirst; k < nrows; ++k) {
        if (!((todo >> k) & 1u)) continue;
        const uint32_t cw = cw0 + k;
        double yv[NW];
#pragma unroll
        for (int s = 0; s < NW; ++s) yv[s] = ynext[s];
        const TxPre<NW> txp = txnext;
        const uint32_t rest = todo & ~((2u << k) - 1u);  // the next row to decode
        if (rest) {
            const uint32_t kn = (uint32_t)__builtin_ctz(rest);
            load_row<M>(p, cw0 + kn, lane, ynext);
            if (!SEL) txnext = tx_prefetch<M>(p, cw0 + kn, lane);
        }
#if defined(BCHK_FIRST_CUT) && BCHK_FIRST_CUT == 1
        // experiment builds only (wrong results, timing of the phases): channel loads
        if (yv[0] + yv[NW - 1] == 12345.0) p.l0[cw] = 0.0;  // keeps the loads
        continue;
#endif
        if constexpr (TMAX <= 15) {
            const uint32_t kb = k & ~3u;
            if (k == (uint32_t)__builtin_ctz(todo & (0xFu << kb))) {
                // test pattern 0 of the four words of this row's group (its first row to
                // decode): one four-row key-equation solve (their rows are read again, from
                // the cache, for the prep)
                constexpr int W = Prep<M, TMAX>::W;
                uint32_t *s4s = reinterpret_cast<uint32_t *>(e4s + 5 * NW);  // [4][W]
#pragma nounroll
                for (int q = 0; q < 4; ++q) {  // one row at a time (registers)
                    uint32_t Sq[W];
                    if (((todo >> (kb + (uint32_t)q)) & 1u) != 0u) {
                        hard_syndromes<M, TMAX>(p, col, cw0 + kb + (uint32_t)q, lane, Sq);
                    } else {
#pragma unroll
                        for (int w = 0; w < W; ++w) Sq[w] = 0;
                    }
                    if (lane == 0) {
#pragma unroll
                        for (int w = 0; w < W; ++w) s4s[q * W + w] = Sq[w];
                    }
                }
                wave_sync();
                uint32_t S4[4][W];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
#pragma unroll
                    for (int w = 0; w < W; ++w) S4[q][w] = s4s[q * W + w];
                }
                alg_decode_wave4<M, TMAX>(ex, lg, S4, p.t, lane, e4s);
                wave_sync();
            }
        }
        Prep<M, TMAX> P;
        int nsel = Geo<M>::N;
        bool selected = false;
        if constexpr (SEL) selected = prep_select<M, TMAX>(p, col, as, ap, ordl, yv, lane, P, nsel);
        if (!selected) {
            nsel = Geo<M>::N;
            prep_loaded<M, TMAX>(p, col, as, ap, ordl, yv, lane, P);
        }
#if defined(BCHK_FIRST_CUT) && BCHK_FIRST_CUT == 2
        ap[lane] = P.asv[0] + (double)P.S0[0] + (double)P.Lo[0];  // + prep (sort, syndromes)
        continue;
#endif
#if defined(BCHK_FIRST_CUT) && BCHK_FIRST_CUT == 3
        {  // + one wave decode
            Mask<NW> E;
            const bool ok = alg_decode_wave<M, TMAX>(ex, lg, P.S0, p.t, lane, E);
            ap[lane] = P.asv[0] + (ok ? (double)E.w[0] : 0.0);
        }
        continue;
#endif
        SearchState<NW> S;
        init_state<M>(S, p.variant);
        bool bail = false;
        if constexpr (TMAX <= 15) {
            Mask<NW> E0;
#pragma unroll
            for (int s2 = 0; s2 < NW; ++s2) E0.w[s2] = rdl64(e4s[(k & 3u) * NW + s2], 0);  // uniform (SGPRs)
            const bool ok0 = uni((int)e4s[4 * NW + (k & 3u)]) != 0;
            first_patterns<M, TMAX, true>(S, P, p, ex, lg, as, ap, lane, nsel, &bail, &E0, ok0);
        } else {
            first_patterns<M, TMAX>(S, P, p, ex, lg, as, ap, lane, nsel, &bail);
        }
#if defined(BCHK_FIRST_CUT) && BCHK_FIRST_CUT == 4
        ap[lane] = S.l0 + (double)(S.done ? 1 : 0) + (double)(bail ? 2 : 0);  // + the first patterns
        continue;
#endif
        if (S.done && !bail) {
            if constexpr (SEL) {
                // the decoded row into the block (the accepted word: a finished codeword
                // returned or ran to its bound after an acceptance -- or, never accepted,
                // keeps the caller's row, which the block then reads back), counters from
                // the sent words' block (src/dataForPlot.cpp:55-74)
                uint32_t bit_errors = 0;
                const bool accp = S.accepted;
#pragma unroll
                for (int s2 = 0; s2 < NW; ++s2) {
                    const int pos = lane + 64 * s2;
                    if (pos < N) {
                        uint8_t x;
                        if (accp) {
                            x = (uint8_t)(((P.yH.w[s2] ^ S.best.w[s2]) >> lane) & 1ull);
                        } else {
                            x = p.res[(size_t)cw * N + pos];
                        }
                        rss[k * N + pos] = x;
                        if (p.cnt) bit_errors += (uint32_t)__popcll(ballot(x != txs[k * N + pos]));
                    }
                }
                if (p.cnt) {
                    const bool word_variant = p.variant == BCHK_VARIANT_WORD;
                    const uint64_t iters = S.returned ? S.i_end - 1 : S.i_end;
                    const uint64_t pro = word_variant ? (uint64_t)(2 * N + 1) : 0ull;
                    acc[0] += bit_errors ? 1ull : 0ull;
                    acc[1] += (unsigned long long)bit_errors;
                    acc[2] += (unsigned long long)S.i_end;
                    acc[3] += (unsigned long long)(pro + iters * (uint64_t)(N + 6) + S.jsteps + S.impr);
                    acc[4] += (unsigned long long)(pro + iters * (uint64_t)(N + 1) + S.jsteps);
                    acc[5] += 1ull;
                }
                fin |= 1u << k;
                l0k = lane == (int)k ? S.l0 : l0k;
            } else {
                write_outputs<M, TMAX>(S, P, p, cw, lane, txp);
            }
        } else if (lane == 0) {
            p.queue_out[atomicAdd(p.qtail, 1u)] = cw;
        }
    }
    if constexpr (SEL) {
        wave_sync();
        uint8_t *dst = p.res + (size_t)cw0 * N;
        const uint32_t all = (1u << nrows) - 1u;
        if (fin == all && wide) {
            for (uint32_t q = (uint32_t)lane; q < nbytes / 8u; q += 64u)
                reinterpret_cast<uint64_t *>(dst)[q] = reinterpret_cast<const uint64_t *>(rss)[q];
        } else {
            for (uint32_t q = (uint32_t)lane; q < nbytes; q += 64u)
                if ((fin >> (q / (uint32_t)N)) & 1u) dst[q] = rss[q];
        }
        if (p.l0 && lane < (int)nrows && ((fin >> lane) & 1u)) p.l0[cw0 + (uint32_t)lane] = l0k;
        if (p.cnt && lane == 0) {
            unsigned long long *c = p.cnt + (size_t)(cw0 / kFirstPerWave % (uint32_t)kCntSlots) * kCntStride;
#pragma unroll
            for (int q = 0; q < 6; ++q)
                if (acc[q]) atomicAdd(c + q, acc[q]);
        }
    }
}

// ---------------------------------------- cooperative search of heavy codewords
// One workgroup per codeword: kCoopWaves - 1 decoder waves and one acceptor wave.
// Decoders take 64-pattern chunks from an LDS counter (the oldest waves, which the SIMD
// favours, simply take more) and decode them speculatively ahead of the acceptance; each
// finished chunk lands in a ring of kCoopSlots slots (success mask, candidates). The
// acceptor walks the chunks strictly in pattern order, applies the reference's sequential
// acceptance (:361-405) to the candidates, and publishes the loop bound and l0 that the
// decoders read to stop early and filter candidates. No workgroup barrier per chunk.
// Results are identical to the single-wave search.
// Ring slots: chunks in flight between the decoders and the acceptor. With 15 decoder
// waves each holding G chunks while a table lookup is outstanding, the ring -- not the
// decoders -- bounds the rate (chunks in flight / chunk latency): n <= 63 gets a deep ring
// (1.3 KB per slot), longer codes keep 16.
#ifndef BCHK_COOP_SLOTS
#define BCHK_COOP_SLOTS 48
#endif
// Long-code ring slots and tail claims (experiment builds vary them; BCH(255,139,31), 2^20,
// cooperative kernel at 5 dB J=15 / 6 dB J=inf: 128 slots 85.1 / 11.0 ms, 256 slots 82.9 /
// 9.9, + 4-chunk claims in the last 60 chunks 81.1-81.6 / 9.8-9.9, 384 slots 81.1 / 9.7;
// profiles/r04_long/coop_ring*.jsonl). Round 5, with helper workgroups (the ring is also the
// window of chunks helpers may run ahead): 256 slots 64.2 / 1.57 ms, 512 64.2 / 1.17, 1024
// 64.3 / 1.07 (profiles/r05_long/help_ring_slots.jsonl). With the decoders' product table
// (BCHK_LONG_GFMUL, 64 KiB of LDS at m = 8) 1024 slots (123 KiB at m = 8) no longer fit: 512.
// The decoders' GF arithmetic (m >= 7): 0 = log / exp tables (GfPlain), 1 = the product
// table (GfMul: no log lookups, ~18 % fewer lookups per test word). Measured (round 6,
// profiles/r06_long/coop_gfmul_rejected.jsonl): cooperative kernel 5 dB J = 15 64.6 -> 89.8
// ms, 6 dB J = inf 1.05 -> 1.63 ms. Random byte lookups spread over 64 KiB meet more bank
// conflicts than sums of two logs into the 1-KiB exp table, where lanes often share a dword
// (a broadcast), so the product table is an experiment build only (make gm1).
#ifndef BCHK_LONG_GFMUL
#define BCHK_LONG_GFMUL 0
#endif
#ifndef BCHK_LONG_SLOTS
#define BCHK_LONG_SLOTS (BCHK_LONG_GFMUL ? 512 : 1024)
#endif
#ifndef BCHK_LONG_TAIL
#define BCHK_LONG_TAIL 60
#endif
#ifndef BCHK_LONG_TAIL_CLAIM
#define BCHK_LONG_TAIL_CLAIM 2
#endif
constexpr int kCoopSlotsMax = BCHK_LONG_SLOTS > 128 ? BCHK_LONG_SLOTS : 128;
// Long codes (m >= 7): a decoder wave claims kLongClaim chunks at once and decodes only
// their patterns that can still matter -- the ones skip_lane does not rule out -- packed 64
// to a round (lane i no longer decodes pattern base + i). At 5 dB on BCH(255,139,31) the
// skip rules out 46 % of a heavy codeword's patterns but whole 64-pattern chunks rarely
// (6 %: scripts/proto_m8_skip.c), so without packing most of that stayed lanes doing
// nothing. Successes are rare (almost every pattern of a heavy codeword fails), so a ring
// slot holds only the chunk's success mask and up to kLongRec candidate records. A chunk
// with more candidates is decoded again, on the acceptor's request (when it reaches that
// chunk), by a decoder wave into the one dense result buffer. A claim that lies past the
// published loop bound waits -- the bound may rise again -- until the codeword is done or
// the bound passes it.
// Chunks per decoder claim (experiment builds vary it). BCH(255,139,31), 2^20, cooperative
// kernel at 5 dB J=15 / 6 dB J=inf: 16 chunks 96.6 / 12.0 ms, 8: 81.7 / 9.9, 4: 78.1 / 9.5
// (77.4 / 9.5 on a second box), 2: 75.6 / 9.5, 1: 82.3 / 11.5
// (profiles/r04_long/coop_claim_size_variants*.jsonl)
#ifndef BCHK_LONG_CLAIM
#define BCHK_LONG_CLAIM 2
#endif
constexpr int kLongClaim = BCHK_LONG_CLAIM;
static_assert(kLongClaim >= 1 && kLongClaim <= 16 && (kLongClaim & (kLongClaim - 1)) == 0 &&
                  BCHK_LONG_TAIL_CLAIM <= kLongClaim, "claim sizes");
constexpr int kLongSlots = BCHK_LONG_SLOTS;
constexpr int kLongRec = 2;
template <int NW>
constexpr int coop_slots() { return NW == 1 ? BCHK_COOP_SLOTS : kLongSlots; }
static_assert(BCHK_COOP_SLOTS <= 64, "ring flags are polled one slot per lane");
// m >= 7: waves of the cooperative workgroup (1 acceptor + decoders). 12 waves = 3 per SIMD
// leave each wave 168 VGPRs, which the packed decoder (Berlekamp-Massey and the split test
// per lane) needs without spilling; at 16 waves (128 VGPRs) it spilled 184-332 B per lane.
// (The helper path of round 5 spills 168 B per lane at 12 waves too. Round 6 measured 16
// waves: BCH(255,139,31) 2^20, 5 dB J = 15 cooperative kernel 64.4 -> 62.0 ms but 6 dB J = inf
// 1.05 -> 1.35 ms; 8 waves 73.9 / 0.99 ms -- 12 stays; profiles/r06_long/coop_waves.jsonl.)
#ifndef BCHK_LONG_COOP_WAVES
#define BCHK_LONG_COOP_WAVES 12
#endif
// the packed decoders' GF tables: 1 = replicated (GfRep, bank-spread), 0 = the packed tables
#ifndef BCHK_LONG_GFREP
#define BCHK_LONG_GFREP 0
#endif
static_assert(!(BCHK_LONG_GFREP && BCHK_LONG_GFMUL), "one GF view for the packed decoders");
template <int M>
constexpr size_t coop_gf_bytes() {
    return BCHK_LONG_GFREP ? (size_t)gf_rep_bytes<M>() : BCHK_LONG_GFMUL ? (size_t)gf_mul_bytes<M>() : 0;
}
template <int M>
constexpr int coop_waves() { return Geo<M>::NW > 1 ? BCHK_LONG_COOP_WAVES : kCoopWaves; }
static_assert(kLongSlots <= kCoopSlotsMax && kLongSlots >= (BCHK_LONG_COOP_WAVES - 1) * kLongClaim + 8,
              "every decoder's claim fits");

template <int NW>
struct CoopSlot {  // one decoded chunk
    uint64_t okm, cand;
    uint64_t diff[64 * NW];
    double l[64];
    uint32_t m[64];
};
template <int NW>
struct LongRec {  // a candidate (m >= 7): pattern base + lane
    uint64_t diff[NW];
    double l;
    uint32_t m, lane;
};
template <int NW>
struct LongSlot {
    uint64_t okm;    // successes (lanes = patterns of the chunk)
    uint32_t ncand;  // candidates found; > kLongRec: only the first kLongRec stored
    uint32_t pad;
    double run;      // the decoder's running minimum of l (candidates lie below it)
    LongRec<NW> rec[kLongRec];
};
template <int NW>
struct LongDense {  // one chunk decoded for the acceptor: every lane's result
    uint64_t okm;
    uint64_t diff[64 * NW];
    double l[64];
    uint32_t m[64];
};
template <int NW>
constexpr size_t coop_ring_bytes() {
    return NW == 1 ? sizeof(CoopSlot<NW>) * coop_slots<NW>()
                   : sizeof(LongSlot<NW>) * kLongSlots + ((sizeof(LongDense<NW>) + 15) & ~size_t(15));
}

// the cooperative kernel's per-wave LDS: n <= 63 one prep slice per wave; m >= 7 ONE prep
// slice (every wave builds the same prep, so all of them write the same values), a 128-B
// scratch per wave (long_decode_claim's chunk masks and syndromes), then the replicated GF
// tables of the packed decoders (GfRep)
constexpr int kCoopScratch = 128;  // 8 G + 4 G W bytes (G = kLongClaim, W <= 8)
template <int M, int TMAX>
struct PrepTab;
template <int M, int TMAX>
constexpr size_t coop_wave_area() {
    return Geo<M>::NW == 1 ? (size_t)kCoopWaves * Smem<M, TMAX>::WAVE_BYTES
                           : (size_t)Smem<M, TMAX>::WAVE_BYTES + (size_t)coop_waves<M>() * kCoopScratch +
                                 coop_gf_bytes<M>() + sizeof(PrepTab<M, TMAX>);
}

struct CoopCtl {
    uint32_t next;      // next chunk to hand out
    uint32_t consumed;  // chunks the acceptor has finished
    uint32_t done;      // the codeword's search has ended
    uint32_t item;      // the heavy codeword of this workgroup
    uint32_t drec;      // diagnostic builds: its record index
    uint64_t bound;     // the acceptor's current loop bound (diagnostics; may rise again)
    double l0;          // current l0 (monotone non-increasing)
    uint64_t skey;      // skip_key of the best codeword so far (0: none yet)
    uint32_t go;        // m >= 7: the acceptor has decoded the first patterns and published
    uint32_t redo;      // m >= 7: chunk + 1 the acceptor wants decoded densely (0: none)
    uint32_t redo_done; // chunk + 1 whose results the dense buffer holds
    uint32_t ready[kCoopSlotsMax];  // chunk index + 1 once the slot holds that chunk
};


__device__ __forceinline__ uint32_t exact_finished(const SearchParams &p) {
    uint32_t v = 0;
#pragma unroll
    for (int x = 0; x < 8; ++x) v += ld_rlx(p.exact_done + 32 * x);
    return v;
}

// Next heavy codeword for this workgroup (one thread), kEmptySlot when none is left. A
// ticket of the front queue first: it is served as soon as the k-th big codeword is handed
// off; once the exact kernel has finished and the front queue holds no k-th item, a ticket
// of the back queue. One atomic per ticket (no compare-and-swap retries); every wait is
// bounded, so a logic error ends the workgroup instead of hanging it.
__device__ uint32_t next_heavy(const SearchParams &p) {
    const uint32_t total = p.exact_total ? *p.exact_total : p.count;
    for (int q = 0; q < 2; ++q) {
        uint32_t *head = q ? p.heavy_head2 : p.heavy_head;
        const uint32_t *tail = q ? p.heavy_tail2 : p.heavy_tail;
        const uint32_t k = atomicAdd(head, 1u);
        bool have = false, final = false;
        for (uint32_t spins = 0; spins < kSpinLimit; ++spins) {
            if (k < ld_rlx(tail)) { have = true; break; }
            // the counts first (and waited for): if complete, the tail read after is final
            final = exact_finished(p) >= total;
            mem_drain();
            if (k < ld_rlx(tail)) { have = true; break; }
            if (final) break;
            __builtin_amdgcn_s_sleep(32);
        }
        if (!have && !final) flag_fault(p, kFaultHeavyWait);
        if (!have) continue;
        uint32_t *slot = q ? p.heavy_queue + (p.count - 1u - k) : p.heavy_queue + k;
        for (uint32_t w = 0; w < kSpinLimit; ++w) {  // the producer stores after reserving
            const uint32_t cw = ld_rlx(slot);
            if (cw != kEmptySlot) {
                __hip_atomic_store(slot, kEmptySlot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return cw;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        flag_fault(p, kFaultHeavySlot);
        return kEmptySlot;
    }
    return kEmptySlot;
}

// k-th set bit (k from 0, k < popc(mk)) of mk, per lane, branch-free
__device__ __forceinline__ int select_bit(uint64_t mk, int k) {
    const uint32_t lo = (uint32_t)mk;
    int c = __popc(lo);
    const bool up = k >= c;
    k = up ? k - c : k;
    uint32_t v = up ? (uint32_t)(mk >> 32) : lo;
    int pos = up ? 32 : 0;
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        const uint32_t low = v & ((1u << w) - 1u);
        c = __popc(low);
        const bool u2 = k >= c;
        k = u2 ? k - c : k;
        v = u2 ? (v >> w) : low;
        pos += u2 ? w : 0;
    }
    return pos;
}

template <int NW>
__device__ __forceinline__ void mask_flip(Mask<NW> &m, int p) {
#pragma unroll
    for (int s = 0; s < NW; ++s) m.w[s] ^= (uint64_t)((p >> 6) == s) << (p & 63);
}

// The prep's test-pattern tables in the workgroup's LDS (m >= 7, written once per codeword by
// the acceptor wave): the decoder waves read them there instead of holding the Prep fields in
// registers and moving them between lanes (readlane / ds_bpermute). Round 4's attempt to
// serve dense re-decodes through the claim's own call site decoded BCH(127, t = 10) words
// wrongly: lanes read P.Lo values of other lanes as 0 or as another lane's value
// (gpurun_out/diag_m7dbg.log) -- cross-lane reads of register-resident prep fields in a kernel
// that spilled 58-90 VGPRs; with the tables here no decoder reads another lane's register.
template <int M, int TMAX>
struct PrepTab {
    static constexpr int W = Prep<M, TMAX>::W, NW = Geo<M>::NW;
    uint32_t scol[64 * W];  // rank b: odd-syndrome column of position ord[b] (b < NB)
    uint32_t Lo[64 * W];    // pattern bits 0..5 = l: their syndrome contribution
    uint64_t Plo[64 * NW];  // pattern bits 0..5 = l: their flipped positions
    uint32_t S0[W];         // odd syndromes of the hard decision
};
template <int M, int TMAX>
__device__ __forceinline__ void prep_tab_store(PrepTab<M, TMAX> *pt, const Prep<M, TMAX> &P, int lane) {
    constexpr int W = Prep<M, TMAX>::W, NW = Geo<M>::NW;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        pt->scol[lane * W + w] = P.scol[w];
        pt->Lo[lane * W + w] = P.Lo[w];
    }
#pragma unroll
    for (int s2 = 0; s2 < NW; ++s2) pt->Plo[lane * NW + s2] = P.Plo.w[s2];
    if (lane < W) {
        uint32_t v = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) v = lane == w ? P.S0[w] : v;
        pt->S0[lane] = v;
    }
}

// ---- cross-workgroup help for long codewords (m >= 7, round 5). A codeword with many chunks
// left is published as workgroup b's job: its prep tables, and its loop state mirrored from
// the acceptor (bound, l0, skip key, chunks consumed, done). Workgroups left without a heavy
// codeword attach to a job, claim chunks from the job's counter (which the owner's decoders
// claim from too), decode them exactly as the owner's decoders would (long_decode, into their
// own LDS ring) and hand each chunk's slot record over through the job's data: `sc1` stores,
// `s_waitcnt vmcnt(0)`, then the chunk's tag (`sc1`). The owner's acceptor polls the tags of
// the chunks its own ring does not hold yet (only while helpers are attached), copies a
// tagged record into its ring slot and marks it ready, so the acceptance is unchanged. A
// dense re-decode is always served by the owner's decoders. The owner re-uses its job only
// after every helper has left (they leave at `done`).
constexpr uint32_t kShareMinChunks = 64;  // published / helped while at least this many chunks are left
constexpr uint32_t kHelpersMax = 16;       // helpers per job (the ring window bounds the useful number)
struct alignas(128) JobCtl {
    uint32_t state;     // 1: published (prep tables valid), 0: not
    uint32_t helpers;   // helper workgroups attached
    uint32_t done;      // the codeword's search has ended
    uint32_t consumed;  // chunks the acceptor has finished
    uint32_t next;      // chunk claim counter (owner's decoders and helpers)
    uint32_t helped;    // some helper has attached to this codeword (sticky until the next)
    uint64_t bound;     // published loop bound
    uint64_t l0bits;    // published l0 (f64 bits)
    uint64_t skey;      // published skip key
    uint32_t gen;       // this publication's generation: the high word of its tags
    uint32_t pad[19];
};
static_assert(sizeof(JobCtl) == 128, "one control line per job");
template <int M, int TMAX>
struct JobData {
    uint64_t tag[kLongSlots];                 // gen << 32 | chunk + 1 once rec[chunk % kLongSlots] is stored
    LongSlot<Geo<M>::NW> rec[kLongSlots];
    PrepTab<M, TMAX> pt;
    uint64_t ordl[32];                        // the order's first 256 positions (bytes)
    double ap[256];                           // |alpha| by position
};
__device__ __forceinline__ uint32_t g_ld32(const uint32_t *a) {
    return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_st32(uint32_t *a, uint32_t v) {
    __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t g_ld64(const uint64_t *a) {
    return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_st64(uint64_t *a, uint64_t v) {
    __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// n 8-B words, one wave: LDS -> job data (sc1) or job data -> LDS (sc1 loads)
__device__ __forceinline__ void job_put(uint64_t *dst, const uint64_t *src, int n, int lane) {
    for (int i = lane; i < n; i += 64) g_st64(dst + i, src[i]);
}
__device__ __forceinline__ void job_get(uint64_t *dst, const uint64_t *src, int n, int first, int stride) {
    for (int i = first; i < n; i += stride) dst[i] = g_ld64(src + i);
}

// A decoder wave's work (m >= 7), one call site for both kinds:
//  * a claim of nch <= kLongClaim chunks c .. c + nch - 1: the patterns skip_lane leaves,
//    packed 64 per round (the k-th of them in lane k), decoded; each success goes, in pattern
//    order, into its chunk's success mask and -- when it is a strict running minimum of l
//    below l0 as published (the candidates of the dense ring) -- into the chunk's slot.
//    Chunks past the cap are not published.
//  * dense (the acceptor's request for a chunk with more candidates than its slot keeps):
//    every pattern of chunk c, lane = pattern, every lane's result into the dense buffer.
template <int M, int TMAX, class GF>
__device__ __forceinline__ int long_decode(const PrepTab<M, TMAX> *pt, const uint8_t *ordl, uint32_t c, uint64_t capc,
                                           double l0r, uint64_t skey, int t, const uint8_t *ex,
                                           const GF &gfr, const double *ap, uint8_t *wscratch,
                                           LongSlot<Geo<M>::NW> *ring, LongDense<Geo<M>::NW> *dn, CoopCtl *ctl,
                                           int lane, uint32_t nch, int lrec, bool dense) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW, W = Prep<M, TMAX>::W, G = kLongClaim;
    constexpr int NB = N < 31 ? N : 31;
    static_assert(G <= 64 && (G & (G - 1)) == 0, "lanes 0..G-1 form the claim's chunk syndromes");
    static_assert(8 * G + 4 * G * W <= kCoopScratch, "the wave's scratch holds the claim's masks and syndromes");
    // per-wave LDS scratch: the chunks' pattern masks and the syndromes of the hard decision
    // ^ pattern bits >= 6
    uint64_t *actl = reinterpret_cast<uint64_t *>(wscratch);
    uint32_t *hl = reinterpret_cast<uint32_t *>(actl + G);
    int pre[G + 1];
    pre[0] = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint64_t b = 64ull * (uint64_t)(c + (uint32_t)g);
        const bool own = (uint32_t)g < nch;  // chunks past nch belong to later claims
        uint64_t a = (!dense && own && b < capc) ? ballot(!skip_lane(skey, b + (uint64_t)lane, t)) : 0ull;
        a = (dense && g == 0) ? ~0ull : a;
        if (lane == 0) actl[g] = a;
        pre[g + 1] = pre[g] + __popcll(a);
        if (!dense && own && b < capc && lane == 0) {  // the slot's running state (the ring space is ours)
            LongSlot<NW> &S = ring[(c + (uint32_t)g) % kLongSlots];
            S.okm = 0ull;
            S.ncand = 0u;
            S.run = l0r;
        }
    }
    {   // lane g < G: the syndrome of pattern bits >= 6 for chunk c + g
        uint32_t h[W];
#pragma unroll
        for (int w = 0; w < W; ++w) h[w] = pt->S0[w];
        const uint32_t hb = (c + (uint32_t)(lane & (G - 1))) << 6;
        for (int b = 6; b < NB; ++b) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint32_t col_b = pt->scol[b * W + w];  // a broadcast read, then the select
                h[w] ^= ((hb >> b) & 1u) ? col_b : 0u;
            }
        }
        if (lane < G) {
#pragma unroll
            for (int w = 0; w < W; ++w) hl[lane * W + w] = h[w];
        }
    }
    wave_sync();
    const int A = pre[G];
    for (int r = 0; 64 * r < A; ++r) {
        const int idx = 64 * r + lane;
        const bool valid = idx < A;
        int g = 0, pg = 0;
#pragma unroll
        for (int gg = 1; gg < G; ++gg) {
            g = idx >= pre[gg] ? gg : g;
            pg = idx >= pre[gg] ? pre[gg] : pg;
        }
        const int bit = valid ? select_bit(actl[g], idx - pg) : 0;
        uint32_t Sw[W];
#pragma unroll
        for (int w = 0; w < W; ++w) Sw[w] = hl[g * W + w] ^ pt->Lo[bit * W + w];
        Mask<NW> E;
        const bool ok = alg_decode_lanes_g<M, TMAX>(gfr, ex, Sw, t, E, valid) && valid;
        const uint64_t okb = ballot(ok);
        if (!okb && !dense) continue;
        // the successes: diff = flipped positions ^ error locations, m, calcL (:69-77)
        const uint32_t ii = 64u * (c + (uint32_t)g) + (uint32_t)bit;
        Mask<NW> d = E;
        double l = 0.0;
        int m = 0;
        if (ok) {
            for (int b = 0; b < NB; ++b)
                if ((ii >> b) & 1u) mask_flip<NW>(d, (int)ordl[b]);
            m = mask_popc<NW>(d);
#pragma unroll
            for (int s2 = 0; s2 < NW; ++s2)
                for (uint64_t v = d.w[s2]; v; v &= v - 1) l += ap[64 * s2 + (int)__builtin_ctzll(v)];
        }
        if (dense) {  // lane = pattern: every lane's result (the acceptor reads okm's lanes)
#pragma unroll
            for (int s2 = 0; s2 < NW; ++s2) dn->diff[lane * NW + s2] = d.w[s2];
            dn->l[lane] = l;
            dn->m[lane] = (uint32_t)m;
            if (lane == 0) dn->okm = okb;
            continue;
        }
        for (uint64_t sm = okb; sm; sm &= sm - 1) {  // pattern order (lane order in a round)
            const int L = (int)__builtin_ctzll(sm);
            const int gL = (int)rdl((uint32_t)g, L), bL = (int)rdl((uint32_t)bit, L);
            const double lL = rdlf(l, L);
            LongSlot<NW> &S = ring[(c + (uint32_t)gL) % kLongSlots];
            const bool cand = lL < S.run;
            const uint32_t slot_n = S.ncand;
            wave_sync();
            if (lane == 0) {
                S.okm |= 1ull << bL;
                if (cand) {
                    S.run = lL;
                    S.ncand = slot_n + 1u;
                }
            }
            if (cand && slot_n < (uint32_t)lrec && lane == L) {
                LongRec<NW> &R = S.rec[slot_n];
#pragma unroll
                for (int s2 = 0; s2 < NW; ++s2) R.diff[s2] = d.w[s2];
                R.l = l;
                R.m = (uint32_t)m;
                R.lane = (uint32_t)bL;
            }
            wave_sync();
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (!dense) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t cg = c + (uint32_t)g;
            if ((uint32_t)g >= nch || 64ull * cg >= capc) break;  // not ours / never read by the acceptor
            if (lane == 0) lds_st(&ctl->ready[cg % kLongSlots], cg + 1u);
        }
    }
    wave_sync();
    return (A + 63) >> 6;  // decode rounds
}

template <int M, int TMAX, bool TAB>
__global__ void __launch_bounds__(kWaveSize * coop_waves<M>())
kaneko_coop_kernel(SearchParams p) {
    constexpr int NW = Geo<M>::NW;
    constexpr int NP = Smem<M, TMAX>::NP;
    constexpr int kAcceptor = 0;  // the oldest wave: the SIMD arbiter favours it
    constexpr int kCoopSlots = coop_slots<NW>();
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    {   // nothing handed off and every producer finished (the usual case at high SNR): the
        // block leaves before staging the tables
        __shared__ uint32_t idle;
        if (threadIdx.x == 0) {
            const uint32_t total = p.exact_total ? *p.exact_total : p.count;
            const bool fin = exact_finished(p) >= total;
            mem_drain();
            idle = fin && ld_rlx(p.heavy_tail) == 0u && ld_rlx(p.heavy_tail2) == 0u ? 1u : 0u;
        }
        __syncthreads();
        if (idle) return;
    }
    load_tables(smem, p.tables, p.td.bytes);
    const uint8_t *ex = smem + p.td.off_exp;
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(smem + p.td.off_log);
    const uint32_t *col = reinterpret_cast<const uint32_t *>(smem + p.td.off_col);
    const uint64_t *chien = reinterpret_cast<const uint64_t *>(smem + p.td.off_chien);
    [[maybe_unused]] const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    uint8_t *shared0 = smem + ((p.td.bytes + 15) & ~15u);
    CoopSlot<NW> *ring = reinterpret_cast<CoopSlot<NW> *>(shared0);    // n <= 63
    LongSlot<NW> *lring = reinterpret_cast<LongSlot<NW> *>(shared0);   // m >= 7
    LongDense<NW> *ldense = reinterpret_cast<LongDense<NW> *>(shared0 + sizeof(LongSlot<NW>) * kLongSlots);
    CoopCtl *ctl = reinterpret_cast<CoopCtl *>(shared0 + coop_ring_bytes<NW>());
    // n <= 63: a prep slice per wave; m >= 7: one shared slice, per-wave scratch, GfRep
    uint8_t *area = reinterpret_cast<uint8_t *>(ctl + 1);
    uint8_t *wbase = NW == 1 ? area + wid * Smem<M, TMAX>::WAVE_BYTES : area;
    uint8_t *wscr = area + Smem<M, TMAX>::WAVE_BYTES + wid * kCoopScratch;  // m >= 7
    uint8_t *grep = area + Smem<M, TMAX>::WAVE_BYTES + coop_waves<M>() * kCoopScratch;  // m >= 7
    PrepTab<M, TMAX> *ptab =
        reinterpret_cast<PrepTab<M, TMAX> *>(grep + coop_gf_bytes<M>());  // m >= 7
    if constexpr (NW > 1 && BCHK_LONG_GFREP) {
        __syncthreads();  // the packed tables are in LDS
        gf_rep_fill<M>(grep, ex, lg);
    }
    if constexpr (NW > 1 && BCHK_LONG_GFMUL) {
        // the product table from HBM (built by the host; L2-resident after the first CU)
        static_assert(gf_mul_bytes<M>() % 4 == 0, "dwords");
        const uint32_t *src = reinterpret_cast<const uint32_t *>(p.gfmul);
        uint32_t *dst = reinterpret_cast<uint32_t *>(grep);
        for (int i = (int)threadIdx.x; i < gf_mul_bytes<M>() / 4; i += (int)blockDim.x) dst[i] = src[i];
    }
    double *as = reinterpret_cast<double *>(wbase);
    double *ap = as + NP;
    uint8_t *ordl = wbase + NP * 16;
    const uint64_t capc = p.max_decodes ? ((p.max_decodes + 63) & ~63ull) : ~0ull;
    // m >= 7: this workgroup's job (cross-workgroup help), null when off
    JobCtl *const jcb = (NW > 1) ? reinterpret_cast<JobCtl *>(p.long_jobctl) : nullptr;
    JobData<M, TMAX> *const jdb = (NW > 1) ? reinterpret_cast<JobData<M, TMAX> *>(p.long_jobs) : nullptr;
    JobCtl *const jc = jcb ? jcb + blockIdx.x : nullptr;
    JobData<M, TMAX> *const jd = jdb ? jdb + blockIdx.x : nullptr;
    uint32_t hidle = 0;  // helper scans in a row that found no job
    // the workgroups owning a codeword (helpers keep looking while any does)
    uint32_t *const owners = jcb ? reinterpret_cast<uint32_t *>(jcb + gridDim.x) : nullptr;
    const uint32_t help_max = p.long_help_max ? p.long_help_max : kHelpersMax;
    const uint32_t share_min = p.long_share_min ? p.long_share_min : kShareMinChunks;
    bool owning = false;  // thread 0: this workgroup counts among the owners
    uint32_t *const idle_wgs = owners ? owners + 1 : nullptr;  // workgroups that have turned helper
    bool was_helper = false;  // thread 0: counted in idle_wgs
    // publication generations: the launch's epoch above a per-workgroup count (a tag of an
    // earlier publication, or of an earlier launch, never matches)
    uint32_t jgen = (p.long_epoch & 0xFFFFFu) << 12;
    for (;;) {
        // the lane index and t re-read opaquely per codeword: values derived from them are not
        // hoisted out of this persistent loop (they stayed live through the whole body and
        // spilled)
        int lane_o = (int)(threadIdx.x & 63), t_o = p.t;
        asm volatile("" : "+v"(lane_o), "+v"(t_o));
        const int lane = lane_o, tt = uni(t_o);
#if BCHK_LONG_GFREP
        const GfRep<M> gfr{grep, 4 * (lane & 15)};
#elif BCHK_LONG_GFMUL
        const GfMul<M> gfr{grep, lg};
#else
        const GfPlain<M> gfr{ex, lg};
#endif
        (void)tt;
        __syncthreads();
        if (threadIdx.x == 0) {
            if (jc) {  // the previous codeword's job: closed, and every helper gone
                g_st32(&jc->done, 1u);
                g_st32(&jc->state, 0u);
                uint32_t sp = 0;
                while (g_ld32(&jc->helpers) != 0u && ++sp < kSpinLimit) __builtin_amdgcn_s_sleep(8);
                if (sp >= kSpinLimit) flag_fault(p, kFaultCoopRing);
                g_st32(&jc->next, 0u);
                g_st32(&jc->consumed, 0u);
                g_st32(&jc->helped, 0u);
                g_st32(&jc->done, 0u);
            }
            if (owning) {
                atomicSub(owners, 1u);
                owning = false;
            }
            ctl->item = next_heavy(p);
            if (owners && ctl->item != kEmptySlot && ctl->item < p.count) {
                atomicAdd(owners, 1u);
                owning = true;
            }
#ifdef BCHK_DIAG
            ctl->drec = atomicAdd(p.diag_count, 1u);
#endif
            ctl->next = 0;
            ctl->consumed = 0;
            ctl->done = 0;
            ctl->redo = 0;
            ctl->redo_done = 0;
            ctl->go = 0;
        }
        for (uint32_t k = threadIdx.x; k < (uint32_t)kCoopSlots; k += blockDim.x) ctl->ready[k] = 0;
        __syncthreads();
        const uint32_t item = ctl->item;
        JobCtl *hq = nullptr;  // helper mode (m >= 7): the job this workgroup helps
        if (item == kEmptySlot) {
            if constexpr (NW > 1) {
                if (jc) {
                    // ---------------------------------------------- helper (m >= 7)
                    // wave 0 picks the published job with the most chunks left and attaches;
                    // the workgroup loads its tables and runs the decoder loop below on it
                    __shared__ uint32_t hjob;
                    if (threadIdx.x < 64) {
                        uint64_t key = 0;
                        for (uint32_t j = (uint32_t)lane; j < gridDim.x; j += 64) {
                            const JobCtl *q = jcb + j;
                            if (j == blockIdx.x || g_ld32(&q->state) != 1u || g_ld32(&q->done) ||
                                g_ld32(&q->helpers) >= help_max)
                                continue;
                            const uint64_t bch = (g_ld64(&q->bound) + 63ull) >> 6, nx = g_ld32(&q->next);
                            const uint64_t left = bch > nx ? bch - nx : 0ull;
                            const uint64_t kj = ((left < (1ull << 39) ? left : (1ull << 39) - 1ull) << 24) | j;
                            if (left >= share_min && kj > key) key = kj;
                        }
#pragma unroll
                        for (int o = 32; o; o >>= 1) {
                            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)key, o, 64);
                            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(key >> 32), o, 64);
                            const uint64_t other = ((uint64_t)hi << 32) | lo;
                            key = other > key ? other : key;
                        }
                        if (lane == 0) {
                            uint32_t pick = kEmptySlot;
                            if (key) {
                                const uint32_t j = (uint32_t)(key & 0xFFFFFFu);
                                JobCtl *q = jcb + j;
                                const uint32_t h = atomicAdd(&q->helpers, 1u);
                                // attached first, then the state: an owner that saw no helper may
                                // have closed it, or published its next codeword (whose tables
                                // were stored before its state)
                                if (h < help_max && g_ld32(&q->state) == 1u && !g_ld32(&q->done)) {
                                    pick = j;
                                    g_st32(&q->helped, 1u);  // the acceptor polls tags from now on
                                } else {
                                    atomicSub(&q->helpers, 1u);
                                }
                            }
                            hjob = pick;
                        }
                    }
                    if (threadIdx.x == 0 && !was_helper) {
                        atomicAdd(idle_wgs, 1u);  // owners publish their long codewords from now on
                        was_helper = true;
                    }
                    __syncthreads();
                    const uint32_t jb = (uint32_t)uni((int)hjob);
                    if (jb == kEmptySlot) {
                        // no job now: wait while some workgroup still owns a codeword (it may
                        // publish one), leave when none does (bounded: a logic error ends it)
                        if (uni((int)g_ld32(owners)) == 0 || ++hidle > (1u << 16)) return;
                        __builtin_amdgcn_s_sleep(127);
                        continue;
                    }
                    hidle = 0;
                    hq = jcb + jb;
                    const JobData<M, TMAX> *qd = jdb + jb;
                    // the job's tables into this workgroup's LDS (sc1 loads, behind the barrier
                    // that follows wave 0's state poll)
                    job_get(reinterpret_cast<uint64_t *>(ptab), reinterpret_cast<const uint64_t *>(&qd->pt),
                            (int)(sizeof(PrepTab<M, TMAX>) / 8), (int)threadIdx.x, (int)blockDim.x);
                    job_get(reinterpret_cast<uint64_t *>(ordl), qd->ordl, NP / 8, (int)threadIdx.x, (int)blockDim.x);
                    job_get(reinterpret_cast<uint64_t *>(ap), reinterpret_cast<const uint64_t *>(qd->ap), NP,
                            (int)threadIdx.x, (int)blockDim.x);
                    __syncthreads();
                }
            }
            if (!hq) return;
        } else if (item >= p.count) {
            continue;  // never a valid slot value: no access outside the batch
        }
        const bool helper = hq != nullptr;
        JobData<M, TMAX> *const hqd = helper ? jdb + (hq - jcb) : nullptr;
        if (threadIdx.x == 0 && p.coop_stats && !helper) atomicAdd(p.coop_stats + 1, 1u);
        const uint32_t cw = item;
#ifdef BCHK_DIAG
        const uint32_t drec = ctl->drec;  // this codeword's diagnostic record
#endif
#ifdef BCHK_DIAG
        // stamps (acceptor): [0] prep, [1] waiting for chunks, [2] acceptance, [3] chunks
        // decoded (all waves), [4] chunks accepted, [5] improvements, [6] total
        unsigned long long dg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
        Prep<M, TMAX> P;  // every wave builds the same prep (its own LDS slice)
        SearchState<NW> S;
        bool pub = false;  // the acceptor: this codeword was published as a job
        // the acceptor wave publishes its codeword as a job: tables, loop state, generation
        // (drained), then the state word
        auto publish = [&](uint64_t sk, uint32_t cons) {
            jgen = (jgen & ~0xFFFu) | ((jgen + 1u) & 0xFFFu);
            job_put(reinterpret_cast<uint64_t *>(&jd->pt), reinterpret_cast<const uint64_t *>(ptab),
                    (int)(sizeof(PrepTab<M, TMAX>) / 8), lane);
            job_put(jd->ordl, reinterpret_cast<const uint64_t *>(ordl), NP / 8, lane);
            job_put(reinterpret_cast<uint64_t *>(jd->ap), reinterpret_cast<const uint64_t *>(ap), NP, lane);
            if (lane == 0) {
                g_st32(&jc->gen, jgen);
                g_st64(&jc->bound, S.bound);
                g_st64(&jc->l0bits, (uint64_t)__double_as_longlong(S.l0));
                g_st64(&jc->skey, sk);
                g_st32(&jc->consumed, cons);
            }
            mem_drain();
            if (lane == 0) g_st32(&jc->state, 1u);
            pub = true;
        };
        if (!helper) {
        prep_codeword<M, TMAX>(p, col, as, ap, ordl, cw, lane, P);
        init_state<M>(S, p.variant);
        if (threadIdx.x == 0) {
            ctl->bound = S.bound;
            ctl->l0 = S.l0;
            ctl->skey = 0ull;
        }
        if constexpr (NW > 1)  // the decoders' pattern tables (m >= 7)
            if (wid == kAcceptor) prep_tab_store<M, TMAX>(ptab, P, lane);
        __syncthreads();
#ifdef BCHK_DIAG
        unsigned long long t_prev = __builtin_amdgcn_s_memtime();
        dg[0] = t_prev - t_start;
#endif
        if constexpr (NW > 1) {
            // m >= 7: the acceptor decodes the first kSeqPatterns patterns itself before the
            // decoders start (first_patterns; chunk 0 decodes them again, none of them is an
            // improvement a second time), so the loop bound and the skip key of the best
            // codeword -- at 5 dB usually the hard decision's -- are known from the first
            // claim on: otherwise the first claims (15 x 8 chunks) decode, and Chien-scan,
            // every pattern that only re-finds that codeword
            if (wid == kAcceptor) {
                first_patterns<M, TMAX>(S, P, p, ex, lg, as, ap, lane);
                const uint64_t skey0 = S.accepted ? skip_key<M, TMAX>(S.best, P, lane) : 0ull;
                if (jc && !S.done && ((S.bound + 63ull) >> 6) >= share_min && uni((int)g_ld32(idle_wgs)) != 0)
                    publish(skey0, 0u);
                if (lane == 0) {
                    lds_st64(&ctl->bound, S.bound);
                    lds_st64(reinterpret_cast<uint64_t *>(&ctl->l0), (uint64_t)__double_as_longlong(S.l0));
                    lds_st64(&ctl->skey, skey0);
                    if (S.done) lds_st(&ctl->done, 1u);
                    lds_st(&ctl->go, 1u);
                }
            } else {
                uint32_t sp = 0;
                while (!lds_ld(&ctl->go) && ++sp < kSpinLimit) __builtin_amdgcn_s_sleep(2);
                if (sp >= kSpinLimit) {  // never expected: fail the codeword, no hang
                    if (lane == 0) {
                        flag_fault(p, kFaultCoopRing);
                        lds_st(&ctl->done, 1u);
                    }
                    wave_sync();
                }
            }
        }
        }  // !helper
        if (NW > 1 && (helper || wid != kAcceptor)) {
            // ------------------------------------------------ decoder, m >= 7 (packed)
            // One call site of long_decode for both jobs: a dense re-decode the acceptor asks
            // for (served first: it waits on it), else the wave's claim once it fits the ring
            // and lies below the published loop bound (which may rise again) and the cap; the
            // codeword's end (done) releases the wave. Nothing of the Prep is read here: the
            // pattern tables are in LDS (PrepTab), so the decoders hold no prep registers.
          if constexpr (NW > 1) {
            bool have = false;
            uint32_t c = 0, nch = (uint32_t)kLongClaim, spins = 0;
#ifdef BCHK_DIAG
            unsigned long long tw0 = __builtin_amdgcn_s_memtime();
#endif
            for (;;) {
                if (!have) {
                    if (lane == 0) {
                        // the last BCHK_LONG_TAIL chunks below the published bound in smaller
                        // claims: the codeword ends with its slowest claim
                        nch = (uint32_t)kLongClaim;
                        if (BCHK_LONG_TAIL > 0 && !helper) {
                            const uint64_t bch = (lds_ld64(&ctl->bound) + 63ull) >> 6;
                            const uint32_t nx = jc ? g_ld32(&jc->next) : lds_ld(&ctl->next);
                            if ((uint64_t)nx + (uint64_t)BCHK_LONG_TAIL >= bch)
                                nch = (uint32_t)BCHK_LONG_TAIL_CLAIM;
                        }
                        // (the job's counter when help is on: helpers claim from it too)
                        JobCtl *const src = helper ? hq : jc;
                        c = src ? atomicAdd(&src->next, nch) : atomicAdd(&ctl->next, nch);
                    }
                    c = (uint32_t)uni(__shfl((int)c, 0, 64));
                    nch = (uint32_t)uni(__shfl((int)nch, 0, 64));
                    have = true;
                    spins = 0;
                }
                // the loop state: this workgroup's LDS, or (helper) the job's mirror, read
                // wave-uniform (readfirstlane)
                const bool fin = helper ? uni((int)g_ld32(&hq->done)) != 0 : lds_ld(&ctl->done) != 0u;
                if (fin || (helper && 64ull * c >= capc)) break;
                uint32_t r = 0;  // a pending dense request (chunk + 1), taken by one wave
                if (lane == 0 && !helper) {
                    r = lds_ld(&ctl->redo);
                    if (r && atomicCAS(&ctl->redo, r, 0u) != r) r = 0;
                }
                r = (uint32_t)__shfl((int)r, 0, 64);
                const uint64_t b0 = 64ull * c;
                uint32_t cons;
                uint64_t bnd;
                if (helper) {
                    cons = (uint32_t)uni((int)g_ld32(&hq->consumed));
                    const uint64_t b = g_ld64(&hq->bound);
                    bnd = ((uint64_t)(uint32_t)uni((int)(uint32_t)(b >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)b);
                } else {
                    cons = lds_ld(&ctl->consumed);
                    bnd = lds_ld64(&ctl->bound);
                }
                const bool ready = c + (uint32_t)(kLongClaim - 1) < cons + kLongSlots && b0 < bnd && b0 < capc;
                if (!r && !ready) {
                    if (++spins > kSpinLimit) {
#ifdef BCHK_COOP_DEBUG
                        if (lane == 0)
                            printf("dec wid %d cw %u claim %u consumed %u bound %llu done %u redo %u/%u next %u\n", wid, cw, c,
                                   lds_ld(&ctl->consumed), (unsigned long long)lds_ld64(&ctl->bound),
                                   lds_ld(&ctl->done), lds_ld(&ctl->redo), lds_ld(&ctl->redo_done), lds_ld(&ctl->next));
#endif
                        flag_fault(p, kFaultCoopRing);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                    continue;
                }
#ifdef BCHK_DIAG
                const unsigned long long tw1 = __builtin_amdgcn_s_memtime();
                dg[5] += tw1 - tw0;  // m >= 7 decoders: cycles waiting (ring space, bound, done)
#endif
                const double l0r = __longlong_as_double((long long)(helper ? g_ld64(&hq->l0bits) : lds_ld64(
                    reinterpret_cast<const uint64_t *>(&ctl->l0))));
                // a codeword found before chunk c
                const uint64_t skey = helper ? g_ld64(&hq->skey) : lds_ld64(&ctl->skey);
                const bool dense = r != 0u;
                const int rounds = long_decode<M, TMAX>(ptab, ordl, dense ? r - 1u : c, capc, l0r, skey, tt, ex, gfr,
                                                        ap, wscr, lring, ldense, ctl, lane, dense ? 1u : nch,
                                                        p.long_rec, dense);
                if (helper) {
                    // hand the chunks over: slot records (sc1), drained, then their tags
                    constexpr int SW = (int)(sizeof(LongSlot<NW>) / 8);
                    for (uint32_t g = 0; g < nch; ++g) {
                        const uint32_t cg = c + g;
                        if (64ull * cg < capc && lane < SW)
                            g_st64(reinterpret_cast<uint64_t *>(&hqd->rec[cg % kLongSlots]) + lane,
                                   reinterpret_cast<const uint64_t *>(&lring[cg % kLongSlots])[lane]);
                    }
                    mem_drain();
                    if (lane == 0) {
                        const uint64_t tg = (uint64_t)g_ld32(&hq->gen) << 32;  // fixed while attached
                        for (uint32_t g = 0; g < nch; ++g) {
                            const uint32_t cg = c + g;
                            if (64ull * cg < capc) g_st64(&hqd->tag[cg % kLongSlots], tg | ((uint64_t)cg + 1ull));
                        }
                    }
                }
                if (dense) {
                    if (lane == 0) {
                        lds_st(&ctl->redo_done, r);
                        if (p.coop_stats) atomicAdd(p.coop_stats, 1u);
                    }
                } else {
                    have = false;
                }
                spins = 0;
#ifdef BCHK_DIAG
                dg[3] += (unsigned long long)rounds;  // m >= 7: decode rounds of 64 packed patterns
                tw0 = __builtin_amdgcn_s_memtime();
                dg[4] += tw0 - tw1;  // m >= 7 decoders: cycles in claims
#endif
                (void)rounds;
            }
          }
        } else if (wid != kAcceptor) {
            // ------------------------------------------------------------ decoder
            constexpr int G = chunk_group<TAB>();
            for (;;) {
                uint32_t c = 0;  // this wave decodes chunks c .. c + G - 1
                if (lane == 0) c = atomicAdd(&ctl->next, (uint32_t)G);
                c = (uint32_t)__shfl((int)c, 0, 64);
                const uint64_t base = 64ull * c;
                // no early stop on the published loop bound: it can rise again after a later
                // improvement (T is not monotone), so only the acceptor decides the end; the
                // ring keeps decoders at most kCoopSlots chunks ahead of it
                if (base >= capc || lds_ld(&ctl->done)) break;
                // the slots are free once the acceptor has finished chunk c + G - 1 - kCoopSlots
                bool stop = false;
                for (uint32_t spins = 0; c + (uint32_t)(G - 1) >= lds_ld(&ctl->consumed) + kCoopSlots; ++spins) {
                    if (lds_ld(&ctl->done) || spins > kSpinLimit) { stop = true; break; }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (stop) break;
                const double l0r = __longlong_as_double((long long)lds_ld64(
                    reinterpret_cast<const uint64_t *>(&ctl->l0)));
                // any published key is a codeword found in a chunk the acceptor has consumed,
                // i.e. before chunk c (consumed <= c: chunk c is not decoded yet)
                const uint64_t skey = M >= 7 ? lds_ld64(&ctl->skey) : 0ull;
                Mask<NW> diff[G];
                int m[G];
                double l[G];
                bool ok[G];
                decode_chunks<M, TMAX, G, TAB>(P, base, p.t, ex, lg, chien, ap, p.tab, diff, m, l, ok, skey);
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const uint32_t cg = c + (uint32_t)g;
                    if (64ull * cg >= capc) break;  // past the cap: never read by the acceptor
                    const uint64_t okm = ballot(ok[g]);
                    // candidates: the strict running minima of l over this chunk's successes,
                    // below l0 as last published. The improvements are the running minima
                    // over all successes in pattern order, so they are a subset of these.
                    const uint64_t cm = ballot(ok[g] && l[g] < l0r);
                    uint64_t cand = 0;
                    double run = l0r;
                    for (uint64_t mm = cm; mm; mm &= mm - 1) {
                        const int L = (int)__builtin_ctzll(mm);
                        const double lv = rdlf(l[g], L);
                        if (lv < run) {
                            cand |= 1ull << L;
                            run = lv;
                        }
                    }
                    CoopSlot<NW> &sl = ring[cg % kCoopSlots];
                    if ((cand >> lane) & 1ull) {
#pragma unroll
                        for (int s2 = 0; s2 < NW; ++s2) sl.diff[lane * NW + s2] = diff[g].w[s2];
                        sl.m[lane] = (uint32_t)m[g];
                        sl.l[lane] = l[g];
                    }
                    if (lane == 0) {
                        sl.okm = okm;
                        sl.cand = cand;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0) lds_st(&ctl->ready[cg % kCoopSlots], cg + 1u);
#ifdef BCHK_DIAG
                    dg[3] += 1;
#endif
                }
            }
        } else {
            // ------------------------------------------------------------ acceptor
            __builtin_amdgcn_s_setprio(3);
            uint32_t spins = 0;
            for (uint32_t c = 0; !S.done;) {
                // the loop ends at the bound, or is cut at the cap (chunk-granular, the
                // bound winning a tie) exactly as the single-wave kernel decides
                {
                    const uint64_t nb = (S.bound + 63) & ~63ull;  // first chunk past the bound
                    if (64ull * c >= nb || 64ull * c >= capc) {
                        if (nb <= capc) {
                            S.i_end = S.bound;
                        } else {
                            S.i_end = capc;
                            S.truncated = true;
                        }
                        break;
                    }
                }
#ifdef BCHK_DIAG
                const unsigned long long t_w = __builtin_amdgcn_s_memtime();
#endif
                // lane j looks at chunk c + j: the run of consecutive finished chunks is
                // taken in one batch (one LDS round trip for flags, one for the masks)
                const uint32_t cj = c + (uint32_t)lane;
                bool rdy = lane < kCoopSlots && lds_ld(&ctl->ready[cj % kCoopSlots]) == cj + 1u;
                if constexpr (NW > 1) {
                    // chunks a helper decoded (only while helpers are attached): its record
                    // into our ring slot, then the slot is ready like our decoders' ones
                    // (sticky: a helper that delivered and left still has tags to be read)
                    if (pub && uni((int)g_ld32(&jc->helped)) != 0) {
                        constexpr int HC = 32;  // chunks c .. c + HC - 1 looked up
                        const bool hit =
                            lane < HC && !rdy &&
                            g_ld64(&jd->tag[cj % kLongSlots]) == (((uint64_t)jgen << 32) | ((uint64_t)cj + 1ull));
                        // the tagged records, all words in flight at once: word w of chunk j at
                        // index j SW + w, lane = index mod 64
                        constexpr int SW = (int)(sizeof(LongSlot<NW>) / 8);
                        const uint64_t hm = ballot(hit);
                        if (hm) {
                            uint64_t v[(HC * SW + 63) / 64];
#pragma unroll
                            for (int k = 0; k < (HC * SW + 63) / 64; ++k) {
                                const int idx = lane + 64 * k, j = idx / SW, w = idx - SW * (idx / SW);
                                const uint32_t cc = c + (uint32_t)j;
                                v[k] = (idx < HC * SW && ((hm >> j) & 1ull))
                                           ? g_ld64(reinterpret_cast<const uint64_t *>(&jd->rec[cc % kLongSlots]) + w)
                                           : 0ull;
                            }
#pragma unroll
                            for (int k = 0; k < (HC * SW + 63) / 64; ++k) {
                                const int idx = lane + 64 * k, j = idx / SW, w = idx - SW * (idx / SW);
                                const uint32_t cc = c + (uint32_t)j;
                                if (idx < HC * SW && ((hm >> j) & 1ull))
                                    reinterpret_cast<uint64_t *>(&lring[cc % kLongSlots])[w] = v[k];
                            }
                        }
                        wave_sync();
                        if (hit) {
                            lds_st(&ctl->ready[cj % kCoopSlots], cj + 1u);
                            rdy = true;
                        }
                    }
                }
                const uint64_t rm = ballot(rdy);
                // chunks c .. c + run - 1 ready (all 64 polled: the long-code ring has 128
                // slots, and ctz of 0 is undefined -- -1 on gfx950)
                const int run = ~rm ? (int)__builtin_ctzll(~rm) : 64;
                if (run == 0) {
                    if (++spins > kSpinLimit) {  // never expected: fail the codeword, no hang
#ifdef BCHK_COOP_DEBUG
                        if (lane == 0)
                            printf("acc cw %u c %u bound %llu next %u ready[c] %u l0 %g redo %u/%u\n", cw, c,
                                   (unsigned long long)S.bound, lds_ld(&ctl->next), lds_ld(&ctl->ready[c % kCoopSlots]),
                                   S.l0, lds_ld(&ctl->redo), lds_ld(&ctl->redo_done));
#endif
                        if (lane == 0) flag_fault(p, kFaultCoopRing);
                        S.i_end = 64ull * c;
                        S.truncated = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                spins = 0;
#ifdef BCHK_DIAG
                const unsigned long long t_a = __builtin_amdgcn_s_memtime();
                dg[1] += t_a - t_w;
                const uint64_t impr0 = S.impr;
#endif
                uint32_t cdone = c + (uint32_t)run;
                if constexpr (NW > 1) {
                    // m >= 7: the candidate records, or the chunk decoded here (marked past
                    // the bound, or more candidates than the slot holds)
                    // (firstOK, :371, was decided by first_patterns: pattern 0 may be skipped here)
                    const bool need = lane < run && lring[cj % kLongSlots].ncand != 0u;
                    for (uint64_t jm = ballot(need); jm; jm &= jm - 1) {
                        const int j = (int)__builtin_ctzll(jm);
                        const uint32_t cc = c + (uint32_t)j;
                        const uint64_t base = 64ull * cc;
                        if (base >= S.bound || base >= capc) { cdone = cc; break; }
                        const LongSlot<NW> &sl = lring[cc % kLongSlots];
                        if (sl.ncand > (uint32_t)p.long_rec) {
                            // more candidates than the slot holds: a decoder wave decodes the
                            // chunk densely for us (all earlier chunks are consumed, so no
                            // decoder is waiting on us for it)
                            if (lane == 0) lds_st(&ctl->redo, cc + 1u);
                            uint32_t sp = 0;
                            while (lds_ld(&ctl->redo_done) != cc + 1u && ++sp < kSpinLimit) __builtin_amdgcn_s_sleep(1);
                            if (sp >= kSpinLimit) {
#ifdef BCHK_COOP_DEBUG
                                if (lane == 0)
                                    printf("acc dense wait cw %u cc %u redo %u/%u\n", cw, cc, lds_ld(&ctl->redo),
                                           lds_ld(&ctl->redo_done));
#endif
                                if (lane == 0) flag_fault(p, kFaultCoopRing);
                                S.i_end = base;
                                S.truncated = true;
                                S.done = true;
                                cdone = cc;
                                break;
                            }
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                            for (uint64_t im = ldense->okm; im; im &= im - 1) {
                                const int L = (int)__builtin_ctzll(im);
                                const uint64_t ii = base + (uint64_t)L;
                                if (ii >= S.bound) break;
                                const double lL = ldense->l[L];
                                if (!(lL < S.l0)) continue;
                                Mask<NW> d;
#pragma unroll
                                for (int s2 = 0; s2 < NW; ++s2) d.w[s2] = ldense->diff[L * NW + s2];
                                accept_success<M, TMAX>(S, P, d, (int)ldense->m[L], lL, ii, as, p, lane);
                                if (S.done) break;
                            }
                            if (lane == 0) lds_st(&ctl->redo_done, 0u);
                        } else {
                            const int nc = (int)sl.ncand;
                            for (int q = 0; q < nc; ++q) {
                                const LongRec<NW> &R = sl.rec[q];
                                const uint64_t ii = base + (uint64_t)R.lane;
                                if (ii >= S.bound) break;
                                const double lL = R.l;
                                if (!(lL < S.l0)) continue;
                                Mask<NW> d;
#pragma unroll
                                for (int s2 = 0; s2 < NW; ++s2) d.w[s2] = R.diff[s2];
                                accept_success<M, TMAX>(S, P, d, (int)R.m, lL, ii, as, p, lane);
                                if (S.done) break;
                            }
                        }
                        if (S.done) { cdone = cc + 1u; break; }
                    }
                }
                const uint64_t candj = (NW == 1 && lane < run) ? ring[cj % kCoopSlots].cand : 0ull;
                if (NW == 1 && c == 0 && !(ring[0].okm & 1ull)) S.firstOK = false;  // :371
                for (uint64_t jm = ballot(candj != 0ull); jm; jm &= jm - 1) {
                    const int j = (int)__builtin_ctzll(jm);
                    const uint32_t cc = c + (uint32_t)j;
                    const uint64_t base = 64ull * cc;
                    if (base >= S.bound || base >= capc) { cdone = cc; break; }
                    const CoopSlot<NW> &sl = ring[cc % kCoopSlots];
                    for (uint64_t im = rdl64(candj, j); im; im &= im - 1) {
                        const int L = (int)__builtin_ctzll(im);
                        const uint64_t ii = base + (uint64_t)L;
                        if (ii >= S.bound) break;
                        const double lL = sl.l[L];
                        if (!(lL < S.l0)) continue;
                        Mask<NW> d;
#pragma unroll
                        for (int s2 = 0; s2 < NW; ++s2) d.w[s2] = sl.diff[L * NW + s2];
                        accept_success<M, TMAX>(S, P, d, (int)sl.m[L], lL, ii, as, p, lane);
                        if (S.done) break;
                    }
                    if (S.done) { cdone = cc + 1u; break; }
                }
                c = cdone;
                const uint64_t skey = (M >= 7 && S.accepted) ? skip_key<M, TMAX>(S.best, P, lane) : 0ull;
                if (lane == 0) {
                    lds_st64(&ctl->bound, S.bound);
                    lds_st64(reinterpret_cast<uint64_t *>(&ctl->l0),
                             (uint64_t)__double_as_longlong(S.l0));
                    if (M >= 7) lds_st64(&ctl->skey, skey);
                    lds_st(&ctl->consumed, c);
                    if (pub) {  // the job's mirror for its helpers
                        g_st64(&jc->bound, S.bound);
                        g_st64(&jc->l0bits, (uint64_t)__double_as_longlong(S.l0));
                        g_st64(&jc->skey, skey);
                        g_st32(&jc->consumed, c);
                    }
                }
                // published once some workgroup has run out of codewords and enough chunks
                // are left (a codeword started earlier is published mid-way)
                if (jc && !pub && !S.done && ((S.bound + 63ull) >> 6) >= (uint64_t)c + share_min &&
                    uni((int)g_ld32(idle_wgs)) != 0)
                    publish(skey, c);
#ifdef BCHK_DIAG
                dg[2] += __builtin_amdgcn_s_memtime() - t_a;
                dg[4] += (uint64_t)run;
                dg[5] += S.impr - impr0;
#endif
            }
            __builtin_amdgcn_s_setprio(0);
            if (lane == 0) {
                lds_st(&ctl->done, 1u);
                if (jc) g_st32(&jc->done, 1u);  // helpers leave
            }
            write_outputs<M, TMAX>(S, P, p, cw, lane);
        }
        if constexpr (NW > 1) {
            if (helper) {  // every wave has left the job: detach, then look for another
                __syncthreads();
                if (threadIdx.x == 0) atomicSub(&hq->helpers, 1u);
                continue;
            }
        }
#ifdef BCHK_DIAG
        // chunk counts of every wave into the acceptor's record
        if (lane == 0) atomicAdd(reinterpret_cast<unsigned long long *>(&p.diag[(size_t)drec * 8 + 3]), dg[3]);
        if (NW > 1 && wid != kAcceptor && lane == 0) {  // m >= 7: [4] claim, [5] wait cycles of all decoders
            atomicAdd(reinterpret_cast<unsigned long long *>(&p.diag[(size_t)drec * 8 + 4]), dg[4]);
            atomicAdd(reinterpret_cast<unsigned long long *>(&p.diag[(size_t)drec * 8 + 5]), dg[5]);
        }
        if (wid == kAcceptor && lane == 0) {
            dg[6] = __builtin_amdgcn_s_memtime() - t_start;
            dg[7] = cw;
            for (int q = 0; q < 8; ++q)
                if (q != 3 && !(NW > 1 && (q == 4 || q == 5))) p.diag[(size_t)drec * 8 + q] = dg[q];
        }
#endif
    }
}

template <int M, int TMAX>
__global__ void __launch_bounds__(256) alg_decode_kernel(AlgParams p) {
    constexpr int N = Geo<M>::N, NW = Geo<M>::NW;
    constexpr int W = (TMAX + 3) / 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    load_tables(smem, p.tables, p.td.bytes);
    __syncthreads();
    const uint8_t *ex = smem + p.td.off_exp;
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(smem + p.td.off_log);
    const uint32_t *col = reinterpret_cast<const uint32_t *>(smem + p.td.off_col);
    const uint64_t *chien = reinterpret_cast<const uint64_t *>(smem + p.td.off_chien);
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = idx < p.count;
    const uint32_t wi = live ? idx : 0u;
    const uint8_t *w = p.words + (size_t)wi * N;
    uint32_t Sw[W];
#pragma unroll
    for (int j = 0; j < W; ++j) Sw[j] = 0;
    if (p.synd) {
        for (int j = 0; j < p.t; ++j) Sw[j >> 2] |= (p.synd[(size_t)wi * p.t + j] & 0xFFu) << (8 * (j & 3));
    } else {
        for (int pos = 0; pos < N; ++pos) {
            const uint32_t on = w[pos] ? 0xFFFFFFFFu : 0u;
#pragma unroll
            for (int j = 0; j < W; ++j) Sw[j] ^= col[pos * W + j] & on;
        }
    }
    Mask<NW> E;
    const bool ok = alg_decode_word<M, TMAX>(ex, lg, chien, Sw, p.t, E);
    if (!live) return;
    p.ok[idx] = ok ? 1 : 0;
    if (ok)
        for (int pos = 0; pos < N; ++pos)
            p.answers[(size_t)idx * N + pos] = w[pos] ^ (uint8_t)((E.w[pos >> 6] >> (pos & 63)) & 1ull);
}

// --------------------------------------------------------- FER counters
// src/dataForPlot.cpp:55-74: frame errors, bit errors, decodes, comparisons, sums, words.
// One wave per 64 rows: the rows' bytes are read as 16-B vectors (the 64-row block of
// 64n bytes is contiguous and 16-B aligned when the arrays are), differing bytes -- rare at
// the SNRs of interest -- are tallied per row in LDS, then lane r owns row r.
// The fused counters' partial slots into the caller's totals (one block), slots zeroed for
// the next call.
__global__ void __launch_bounds__(256) cnt_reduce_kernel(unsigned long long *cnt, unsigned long long *out6) {
    __shared__ unsigned long long part[6][4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long c[6] = {0, 0, 0, 0, 0, 0};
    for (int sl = threadIdx.x; sl < kCntSlots; sl += 256) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            c[k] += cnt[(size_t)sl * kCntStride + k];
            cnt[(size_t)sl * kCntStride + k] = 0ull;
        }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) c[k] += (unsigned long long)__shfl_xor((long long)c[k], o, 64);
        if (lane == 0) part[k][wid] = c[k];
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        out6[k] += part[k][0] + part[k][1] + part[k][2] + part[k][3];
    }
}

hipError_t launch_cnt_reduce(unsigned long long *cnt, unsigned long long *out6, hipStream_t s) {
    hipLaunchKernelGGL(cnt_reduce_kernel, dim3(1), dim3(256), 0, s, cnt, out6);
    return hipGetLastError();
}

template <int N>
__global__ void __launch_bounds__(256) count_kernel(const uint8_t *tx, const uint8_t *res,
                                                    const bchk_stats *st, uint32_t B,
                                                    unsigned long long *out6) {
    __shared__ uint32_t rowerr[4][64];
    __shared__ unsigned long long part[6][4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long c[6] = {0, 0, 0, 0, 0, 0};
    const bool vec = ((reinterpret_cast<uintptr_t>(tx) | reinterpret_cast<uintptr_t>(res)) & 15u) == 0;
    const uint32_t stride = gridDim.x * 4u * 64u;
    for (uint32_t r0 = (blockIdx.x * 4u + (uint32_t)wid) * 64u; r0 < B; r0 += stride) {
        rowerr[wid][lane] = 0;
        wave_sync();
        const uint32_t rows = (B - r0) < 64u ? (B - r0) : 64u;
        const size_t base = (size_t)r0 * N;
        const uint32_t bytes = rows * (uint32_t)N;
        if (vec && rows == 64u) {  // 64 N bytes = 4 N vectors
            const uint4 *a4 = reinterpret_cast<const uint4 *>(tx + base);
            const uint4 *b4 = reinterpret_cast<const uint4 *>(res + base);
            for (uint32_t v = (uint32_t)lane; v < 4u * N; v += 64u) {
                const uint4 a = a4[v], b = b4[v];
                const uint32_t x[4] = {a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (!x[k]) continue;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if ((x[k] >> (8 * q)) & 0xFFu)
                            atomicAdd(&rowerr[wid][(16u * v + 4u * k + q) / N], 1u);
                }
            }
        } else {
            for (uint32_t o = (uint32_t)lane; o < bytes; o += 64u)
                if (tx[base + o] != res[base + o]) atomicAdd(&rowerr[wid][o / N], 1u);
        }
        wave_sync();
        if ((uint32_t)lane < rows) {
            const uint32_t e = rowerr[wid][lane];
            c[0] += e ? 1 : 0;
            c[1] += e;
            if (st) {
                const bchk_stats &s = st[r0 + lane];
                c[2] += s.decodes;
                c[3] += s.comparisons;
                c[4] += s.sums;
            }
            c[5] += 1;
        }
        wave_sync();
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        unsigned long long v = c[k];
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) part[k][wid] = v;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        unsigned long long v = 0;
        for (int w = 0; w < (int)(blockDim.x / 64); ++w) v += part[threadIdx.x][w];
        atomicAdd(out6 + threadIdx.x, v);
    }
}

// ------------------------------------------------------------- launchers
template <int M, int TMAX, bool TAB, bool AN>
static hipError_t launch_search_impl(const SearchParams &p, int grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((kaneko_search_kernel<M, TMAX, TAB, AN>), dim3(grid),
                       dim3(kWaveSize * kWavesPerBlock), lds, s, p);
    return hipGetLastError();
}
template <int M, int TMAX, bool TAB>
static hipError_t launch_coop_impl(const SearchParams &p, int grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((kaneko_coop_kernel<M, TMAX, TAB>), dim3(grid), dim3(kWaveSize * coop_waves<M>()),
                       lds, s, p);
    return hipGetLastError();
}
template <int M, int TMAX>
static hipError_t launch_alg_impl(const AlgParams &p, size_t lds, hipStream_t s) {
    const int grid = (int)((p.count + 255) / 256);
    hipLaunchKernelGGL((alg_decode_kernel<M, TMAX>), dim3(grid), dim3(256), lds, s, p);
    return hipGetLastError();
}
template <int M, int TMAX, bool TAB, bool AN>
static const void *search_fn() { return reinterpret_cast<const void *>(&kaneko_search_kernel<M, TMAX, TAB, AN>); }
template <int M, int TMAX, bool TAB>
static const void *coop_fn() { return reinterpret_cast<const void *>(&kaneko_coop_kernel<M, TMAX, TAB>); }

// kaneko_first_kernel: kFirstPerWave consecutive codewords per wave; its row blocks after
// the search kernel's LDS layout
template <int M, int TMAX>
static hipError_t launch_first_impl(const SearchParams &p, size_t lds0, hipStream_t s) {
    const uint32_t per_block = kWavesPerBlock * kFirstPerWave;
    const int blocks = (int)((p.count + per_block - 1) / per_block);
    const size_t lds = lds0 + (size_t)kWavesPerBlock * kFirstWaveExtra;
    if constexpr (first_sel_capable<M, TMAX>()) {
        if (!p.st && !getenv("BCHK_FIRST_FULLSORT")) {
            hipLaunchKernelGGL((kaneko_first_kernel<M, TMAX, true>), dim3(blocks > 0 ? blocks : 1),
                               dim3(kWaveSize * kWavesPerBlock), lds, s, p);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((kaneko_first_kernel<M, TMAX, false>), dim3(blocks > 0 ? blocks : 1),
                       dim3(kWaveSize * kWavesPerBlock), lds, s, p);
    return hipGetLastError();
}

// Long-code first-pattern kernels (m >= 7), same (m, TMAX) buckets as select_kernels.
bool select_first_long(int m, int t, FastFn *out) {
#define BCHK_FIRST(MM, TT) \
    if (m == MM && t <= TT) { *out = &launch_first_impl<MM, TT>; return true; }
#if defined(BCHK_ISA_ONLY) && BCHK_ISA_ONLY == 8
    BCHK_FIRST(8, 15)
#elif !defined(BCHK_ISA_ONLY)
    BCHK_FIRST(7, 8) BCHK_FIRST(7, 16) BCHK_FIRST(7, 32)
    BCHK_FIRST(8, 15) BCHK_FIRST(8, 16) BCHK_FIRST(8, 32)
#endif
#undef BCHK_FIRST
    return false;
}

template <int M, int TMAX>
static KernelSet make_set() {
    constexpr int NW = Geo<M>::NW;
    const size_t coop = coop_ring_bytes<NW>() + sizeof(CoopCtl) + coop_wave_area<M, TMAX>();
    KernelSet k{};
    k.search = &launch_search_impl<M, TMAX, false, false>;
    k.coop = &launch_coop_impl<M, TMAX, false>;
    k.coop_ptr = &coop_fn<M, TMAX, false>;
    k.search_ptr = &search_fn<M, TMAX, false, false>;
    if constexpr (tab_capable<M, TMAX>()) {
        k.search_tab = &launch_search_impl<M, TMAX, true, false>;
        k.coop_tab = &launch_coop_impl<M, TMAX, true>;
        k.coop_tab_ptr = &coop_fn<M, TMAX, true>;
        k.search_tab_ptr = &search_fn<M, TMAX, true, false>;
    }
    if constexpr (an_capable<M, TMAX>()) {
        k.tail = &launch_search_impl<M, TMAX, false, true>;
        k.tail_ptr = &search_fn<M, TMAX, false, true>;
        if constexpr (tab_capable<M, TMAX>()) {
            k.tail_tab = &launch_search_impl<M, TMAX, true, true>;
            k.tail_tab_ptr = &search_fn<M, TMAX, true, true>;
        }
        k.tail_wave_bytes = (size_t)(Smem<M, TMAX>::WAVE_BYTES + an_bytes<M, TMAX>());
        k.tail_block_bytes = (size_t)help_bytes<M, TMAX>();
    }
    k.coop_threads = kWaveSize * coop_waves<M>();
    k.long_job_bytes = Geo<M>::NW > 1 ? sizeof(JobData<M, TMAX>) : 0;
    k.gfmul = Geo<M>::NW > 1 && BCHK_LONG_GFMUL;
    k.coop_bytes = coop;
    k.alg = &launch_alg_impl<M, TMAX>;
    k.tmax = TMAX;
    k.wave_bytes = (size_t)Smem<M, TMAX>::WAVE_BYTES;
    return k;
}

// TMAX buckets: smallest instantiated bucket >= t.
bool select_kernels(int m, int t, KernelSet *out) {
#define BCHK_TRY(MM, TT) \
    if (m == MM && t <= TT) { *out = make_set<MM, TT>(); return true; }
#if defined(BCHK_ISA_ONLY) && BCHK_ISA_ONLY == 8  // ISA inspection builds: one code's kernels only
    BCHK_TRY(8, 15)
#elif defined(BCHK_ISA_ONLY)
    BCHK_TRY(6, 6)
#else
    BCHK_TRY(2, 1)
    BCHK_TRY(3, 3)
    BCHK_TRY(4, 2) BCHK_TRY(4, 7)
    BCHK_TRY(5, 3) BCHK_TRY(5, 8) BCHK_TRY(5, 15)
    BCHK_TRY(6, 6) BCHK_TRY(6, 12) BCHK_TRY(6, 31)
    BCHK_TRY(7, 8) BCHK_TRY(7, 16) BCHK_TRY(7, 32)
    BCHK_TRY(8, 15) BCHK_TRY(8, 16) BCHK_TRY(8, 32)
#endif
#undef BCHK_TRY
    return false;
}

hipError_t launch_search(const KernelSet &k, const SearchParams &p, int grid, size_t lds, hipStream_t s) {
    return (p.tab.slots && k.search_tab) ? k.search_tab(p, grid, lds, s) : k.search(p, grid, lds, s);
}
hipError_t launch_tail(const KernelSet &k, const SearchParams &p, int grid, size_t lds, hipStream_t s) {
    return (p.tab.slots && k.tail_tab) ? k.tail_tab(p, grid, lds, s) : k.tail(p, grid, lds, s);
}
hipError_t launch_coop(const KernelSet &k, const SearchParams &p, int grid, size_t lds, hipStream_t s) {
    return (p.tab.slots && k.coop_tab) ? k.coop_tab(p, grid, lds, s) : k.coop(p, grid, lds, s);
}
hipError_t launch_alg(const KernelSet &k, const AlgParams &p, size_t lds, hipStream_t s) {
    return k.alg(p, lds, s);
}
hipError_t launch_count(int n, const uint8_t *tx, const uint8_t *res, const bchk_stats *st,
                        uint32_t B, uint64_t *out6, hipStream_t s) {
    // grid-stride: every block ends with 6 atomics on the same 6 words, so the grid is capped
    // (1024 blocks: 43.6 us at 2^20 x 63 vs 67.8 us with one block per 256 rows,
    // profiles/r01_long/count_grid.jsonl)
    // (BCHK_COUNT_GRID overrides the cap for experiments)
    static const int cap = getenv("BCHK_COUNT_GRID") ? atoi(getenv("BCHK_COUNT_GRID")) : 1024;
    const int grid = (int)((B + 255) / 256) < cap ? (int)((B + 255) / 256) : cap;
    unsigned long long *o = reinterpret_cast<unsigned long long *>(out6);
    switch (n) {
#define BCHK_CNT(NN) \
    case NN: hipLaunchKernelGGL((count_kernel<NN>), dim3(grid > 0 ? grid : 1), dim3(256), 0, s, tx, res, st, B, o); break;
        BCHK_CNT(3) BCHK_CNT(7) BCHK_CNT(15) BCHK_CNT(31) BCHK_CNT(63) BCHK_CNT(127) BCHK_CNT(255)
#undef BCHK_CNT
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace bchk
