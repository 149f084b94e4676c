// FETCH_SIZE calibration for the fast kernel's load shape.
// Streams rows of 63 f64 (2^20 rows, 528 MB) two ways and writes one double per lane:
//   rowslice: kaneko_fast_kernel's staging pattern, 8 lanes x 8 B per row chunk, 64 rows
//             per wave, 8 slices of 8 positions (csrc/bchk_fast.hip load_slice)
//   stream16: 16 B per lane, contiguous, grid-stride
// Comparing their FETCH_SIZE says whether the guide's x2 gfx950 correction (measured for
// 16 B/lane streaming) applies to the rowslice shape.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int N = 63;
constexpr unsigned ROWS = 1u << 20;

__global__ void __launch_bounds__(256) rowslice(const double *__restrict__ y, double *out) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned cw0 = (blockIdx.x * 4u + wid) * 64u;
    if (cw0 >= ROWS) return;
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int flat = it * 64 + lane;
            const unsigned r = (unsigned)(flat >> 3);
            const int pos = 8 * c + (flat & 7);
            acc += y[(size_t)(cw0 + r) * N + (pos < N ? pos : N - 1)];
        }
    }
    out[cw0 + lane] = acc;
}

__global__ void __launch_bounds__(256) stream16(const double2 *__restrict__ y, size_t n2,
                                                double *out) {
    const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    double acc = 0.0;
    for (size_t i = tid; i < n2; i += stride) {
        const double2 v = y[i];
        acc += v.x + v.y;
    }
    out[tid] = acc;
}

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
            return 1;                                                               \
        }                                                                           \
    } while (0)

int main() {
    const size_t elems = (size_t)ROWS * N;  // even, so double2 covers it exactly
    double *y, *out;
    CK(hipMalloc(&y, elems * sizeof(double)));
    CK(hipMalloc(&out, (size_t)ROWS * sizeof(double)));
    CK(hipMemset(y, 0, elems * sizeof(double)));
    const unsigned rs_blocks = ROWS / 256;  // 4 waves x 64 rows per block
    const unsigned st_blocks = 2048;        // 2048 x 256 lanes <= ROWS outputs
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int rep = 0; rep < 3; ++rep) {
        float ms_rs, ms_st;
        CK(hipEventRecord(a));
        rowslice<<<rs_blocks, 256>>>(y, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms_rs, a, b));
        CK(hipEventRecord(a));
        stream16<<<st_blocks, 256>>>(reinterpret_cast<const double2 *>(y), elems / 2, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms_st, a, b));
        printf("rep %d bytes %zu rowslice %.4f ms (%.0f GB/s) stream16 %.4f ms (%.0f GB/s)\n",
               rep, elems * 8, ms_rs, elems * 8 / ms_rs / 1e6, ms_st,
               elems * 8 / ms_st / 1e6);
    }
    CK(hipGetLastError());
    CK(hipFree(y));
    CK(hipFree(out));
    return 0;
}
