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

template <int PATTERN>
__global__ void __launch_bounds__(512) rows_kernel(const double *__restrict__ y, uint32_t count, double *out) {
    __shared__ double stage[kWaves][64 * 17];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t cw0 = (blockIdx.x * kWaves + wid) * 64u;
    if (cw0 >= count) return;
    double *st = stage[wid];
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
    const char *names[4] = {"slice8", "slice16", "wide16", "stream"};
    for (int pat = 0; pat < 4; ++pat) {
        for (int rep = 0; rep < 2; ++rep) {
            float best = 1e9f;
            for (int k = 0; k < 10; ++k) {
                hipEventRecord(e0);
                switch (pat) {
                    case 0: rows_kernel<0><<<blocks, 512>>>(y, B, out); break;
                    case 1: rows_kernel<1><<<blocks, 512>>>(y, B, out); break;
                    case 2: rows_kernel<2><<<blocks, 512>>>(y, B, out); break;
                    default: rows_kernel<3><<<blocks, 512>>>(y, B, out); break;
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
