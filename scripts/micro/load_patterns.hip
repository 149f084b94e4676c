// Read-bandwidth microbenchmark for the fast kernel's row layout ([B][63] f64, 504-B rows):
// how fast can a wave bring its 64 rows into registers lane-per-row, by access pattern?
//   slice8  : the fast kernel's pattern -- 8-B loads, 8 lanes per row (64 B), 8 rows per
//             instruction, 8-position slices staged through LDS
//   slice16 : 16-B loads, 4 lanes per row-slice of 64 B, 16 rows per instruction
//   wide16  : 16-position slices (128 B per row) with 16-B loads, 8 lanes per row
//   stream  : contiguous 16 B per lane over the whole array (the streaming ceiling)
// Each variant folds what it loaded into one value per lane (no dead code) and writes it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int N = 63;
constexpr int kWaves = 8;

// LDS doubles per wave of each pattern (the fast kernel's 8-position stage, 16-position
// stage, the 32-row key ring)
__host__ __device__ constexpr int wave_doubles(int pat) {
    return pat == 2 ? 64 * 17 : pat == 5 ? 32 * 68 / 2 : pat == 3 ? 0 : 64 * 9;
}
template <int PATTERN>
__global__ void __launch_bounds__(512) rows_kernel(const double *__restrict__ y, uint32_t count, double *out) {
    extern __shared__ double stage_dyn[];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t cw0 = (blockIdx.x * kWaves + wid) * 64u;
    if (cw0 >= count) return;
    double *st = stage_dyn + wid * wave_doubles(PATTERN);
    double acc = 0.0;
    if constexpr (PATTERN == 0) {  // slice8
        constexpr int NS = 8;
        for (int c = 0; c < NS; ++c) {
            double v[8];
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                const int flat = it * 64 + lane;
                const int r = flat >> 3, pos = 8 * c + (flat & 7);
                v[it] = y[(size_t)(cw0 + r) * N + (pos < N ? pos : N - 1)];
            }
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                const int flat = it * 64 + lane;
                st[(flat >> 3) * 9 + (flat & 7)] = v[it];
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += st[lane * 9 + k];
            __builtin_amdgcn_wave_barrier();
        }
    } else if constexpr (PATTERN == 1) {  // slice16: 16-B loads of 64-B row slices
        // a row slice of 8 doubles = 4 x 16 B; 64 lanes cover 16 rows per instruction
        const char *base = reinterpret_cast<const char *>(y);
        for (int c = 0; c < 8; ++c) {
            double v[8];
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const int flat = it * 64 + lane;
                const int r = flat >> 2, q = flat & 3;
                const int pos = 8 * c + 2 * q;
                // rows are 8-B aligned only: two 8-B loads when the pair straddles the end
                const size_t off = ((size_t)(cw0 + r) * N + (pos < N - 1 ? pos : N - 2)) * 8;
                const double2 d = *reinterpret_cast<const double2 *>(base + (off & ~(size_t)15)) ;
                v[2 * it] = d.x;
                v[2 * it + 1] = d.y;
            }
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const int flat = it * 64 + lane;
                st[(flat >> 2) * 9 + 2 * (flat & 3)] = v[2 * it];
                st[(flat >> 2) * 9 + 2 * (flat & 3) + 1] = v[2 * it + 1];
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += st[lane * 9 + k];
            __builtin_amdgcn_wave_barrier();
        }
    } else if constexpr (PATTERN == 2) {  // wide16: 16-position slices, 8-B loads, 4 rows/instr
        for (int c = 0; c < 4; ++c) {
            double v[16];
#pragma unroll
            for (int it = 0; it < 16; ++it) {
                const int flat = it * 64 + lane;
                const int r = flat >> 4, pos = 16 * c + (flat & 15);
                v[it] = y[(size_t)(cw0 + r) * N + (pos < N ? pos : N - 1)];
            }
#pragma unroll
            for (int it = 0; it < 16; ++it) {
                const int flat = it * 64 + lane;
                st[(flat >> 4) * 17 + (flat & 15)] = v[it];
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < 16; ++k) acc += st[lane * 17 + k];
            __builtin_amdgcn_wave_barrier();
        }
    } else if constexpr (PATTERN == 4) {  // slice8 + sort keys (the fast kernel's stage phase)
        uint32_t key[64];
        uint32_t yl = 0, yh = 0;
        for (int c = 0; c < 8; ++c) {
            double v[8];
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                const int flat = it * 64 + lane;
                const int r = flat >> 3, pos = 8 * c + (flat & 7);
                v[it] = y[(size_t)(cw0 + r) * N + (pos < N ? pos : N - 1)];
            }
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                const int flat = it * 64 + lane;
                st[(flat >> 3) * 9 + (flat & 7)] = v[it];
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint64_t b = (uint64_t)__double_as_longlong(st[lane * 9 + k]);
                const uint32_t hi = (uint32_t)(b >> 32), lo = (uint32_t)b;
                const uint32_t d = __builtin_elementwise_sub_sat(hi & 0x7FFFFFFFu, (uint32_t)(1023 - 27) << 20);
                const uint32_t mid = __builtin_amdgcn_alignbit(d, lo, 31);
                const uint32_t pre = mid < 0x3FFFFFFu ? mid : 0x3FFFFFFu;
                key[8 * c + k] = (pre << 6) | (uint32_t)(8 * c + k);
                if (8 * c + k < 32) yl = (yl >> 1) | (hi & 0x80000000u); else yh = (yh >> 1) | (hi & 0x80000000u);
            }
            __builtin_amdgcn_wave_barrier();
        }
        uint32_t x = yl ^ yh;
#pragma unroll
        for (int k = 0; k < 63; ++k) x += key[k] * (uint32_t)(k + 1);
        acc = (double)x;
    } else if constexpr (PATTERN == 5) {  // stream + element-parallel keys + 32-row LDS ring
        // key = prefix(25) << 7 | pos << 1 | sign: lanes of pass p (rows 16p..16p+15) read
        // their row's 63 keys once the instruction completing row 16p+15 has been written
        uint32_t *kb = reinterpret_cast<uint32_t *>(st);  // [32][68]
        const double2 *b2 = reinterpret_cast<const double2 *>(y + (size_t)cw0 * N);
        uint32_t key[64];
        // element e0 = 2 (64 i + lane): row / pos, advanced by 128 elements per instruction
        int e0 = 2 * lane;
        int row = e0 / 63, pos = e0 - 63 * row;
        constexpr int NI = (64 * N / 2 + 63) / 64;
        constexpr int AH = 6;
        double2 buf[AH];
#pragma unroll
        for (int i = 0; i < AH; ++i) buf[i] = (64 * i + lane < 64 * N / 2) ? b2[64 * i + lane] : make_double2(0.0, 0.0);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const double2 d = buf[i % AH];
            if (i + AH < NI) buf[i % AH] = (64 * (i + AH) + lane < 64 * N / 2) ? b2[64 * (i + AH) + lane] : make_double2(0.0, 0.0);
            if (64 * i + lane < 64 * N / 2) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint64_t b = (uint64_t)__double_as_longlong(j ? d.y : d.x);
                    const uint32_t hi = (uint32_t)(b >> 32), lo = (uint32_t)b;
                    const uint32_t dd = __builtin_elementwise_sub_sat(hi & 0x7FFFFFFFu, (uint32_t)(1023 - 27) << 20);
                    const uint32_t mid = __builtin_amdgcn_alignbit(dd, lo, 31) >> 1;
                    const uint32_t pre = mid < 0x1FFFFFFu ? mid : 0x1FFFFFFu;
                    const int pj = j ? (pos + 1 == 63 ? 0 : pos + 1) : pos;
                    const int rj = j ? (pos + 1 == 63 ? row + 1 : row) : row;
                    kb[(rj & 31) * 68 + pj] = (pre << 7) | ((uint32_t)pj << 1) | (hi >> 31);
                }
            }
            pos += 2;
            const bool wrap = pos >= 63;
            pos -= wrap ? 63 : 0;
            row += wrap ? 3 : 2;
            // rows 16p .. 16p+15 complete after instruction (1008 p + 1007) / 128
#pragma unroll
            for (int pp = 0; pp < 4; ++pp) {
                if (i == (1008 * pp + 1007) / 128) {
                    __builtin_amdgcn_wave_barrier();
                    if ((lane >> 4) == pp) {
                        const uint4 *r4 = reinterpret_cast<const uint4 *>(kb + (lane & 31) * 68);
#pragma unroll
                        for (int q = 0; q < 16; ++q) {
                            const uint4 w = r4[q];
                            key[4 * q] = w.x; key[4 * q + 1] = w.y; key[4 * q + 2] = w.z; key[4 * q + 3] = w.w;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 63; ++k) x += key[k] * (uint32_t)(k + 1);
        acc = (double)x;
    } else {  // stream: the wave's 64 rows as contiguous 16-B pieces
        const double2 *b2 = reinterpret_cast<const double2 *>(y + (size_t)cw0 * N);
        const int pieces = 64 * N / 2;  // 2016
        for (int i = lane; i < pieces; i += 64) {
            const double2 d = b2[i];
            acc += d.x + d.y;
        }
    }
    out[cw0 + lane] = acc;
}

int main(int argc, char **argv) {
    const uint32_t B = 1u << 20;
    double *y, *out;
    hipMalloc(&y, (size_t)B * N * 8 + 64);
    hipMalloc(&out, (size_t)B * 8);
    hipMemset(y, 0, (size_t)B * N * 8);
    const int blocks = (int)((B / 64 + kWaves - 1) / kWaves);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[6] = {"slice8", "slice16", "wide16", "stream", "slice8_keys", "stream_keys_ring"};
    for (int pat = 0; pat < 6; ++pat) {
        for (int rep = 0; rep < 2; ++rep) {
            float best = 1e9f;
            for (int k = 0; k < 10; ++k) {
                hipEventRecord(e0);
                switch (pat) {
                    case 0: rows_kernel<0><<<blocks, 512, kWaves * wave_doubles(0) * 8>>>(y, B, out); break;
                    case 1: rows_kernel<1><<<blocks, 512, kWaves * wave_doubles(1) * 8>>>(y, B, out); break;
                    case 2: rows_kernel<2><<<blocks, 512, kWaves * wave_doubles(2) * 8>>>(y, B, out); break;
                    case 4: rows_kernel<4><<<blocks, 512, kWaves * wave_doubles(4) * 8>>>(y, B, out); break;
                    case 5: rows_kernel<5><<<blocks, 512, kWaves * wave_doubles(5) * 8>>>(y, B, out); break;
                    default: rows_kernel<3><<<blocks, 512, 0>>>(y, B, out); break;
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            if (rep == 1)
                printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"GB_s\": %.1f}\n", names[pat], best,
                       (double)B * N * 8 / (best * 1e-3) / 1e9);
        }
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
