// kernel_search.hip -- BCH polar-kernel construction and the column-permutation search on
// the GPU, behind the bchk_kernel_* C ABI (include/bchk.h).
//
// Reference: root bchCoder.cpp:356-389 (makeMatrix: the nested extended-BCH kernel),
// :478-496 (swapColumns: columns into field-element order), :541-699 (randomSwapColumns:
// 2*10^7 random column maps j -> B j, B = L.U over GF(2) from randomInvertibleMatrix
// :766-785, each scored by the SumCount / CmpCount a trellis kernel processor spends on
// GetLLRs for every phase, the first strict improvement of both kept, :651-657).
//
// The score is that of CTrellisKernelProcessor (out/external/TrellisKernelProcessor.cpp:
// 69-294), the processor CMatrixBinaryKernel::GetProcessor(0) returns (Kernel.cpp:276-281;
// the SectionedTrellisKernelProcessor randomSwapColumns names is absent from the reference).
// The reference builds that trellis state by state for every candidate (2^(max active rows)
// states per depth); here it is evaluated in closed form from the code's minimum-span
// structure, one lane per candidate:
//   * phase ph's trellis is that of the code spanned by kernel rows ph..l-1, row ph extended
//     by a 1 at position l (:89-98). MinimumSpan (:7-67) leaves rows with distinct starts and
//     distinct ends; those sets are the code's canonical ones: depth j starts a row iff
//     column j is independent of columns 0..j-1, and ends one iff it is independent of
//     columns j+1..l (the extension column included);
//   * a_j, the active rows entering depth j, is #starts - #ends before j, and the walk of
//     GetLLRs (:263-289) visits 2^a_j states there: a start depth has two edges per state
//     (CMP twice, exactly one label differs from the hard decision: SUM once); any other
//     depth has one edge per state whose label is the active rows' combination at column j
//     -- half the states differ from the hard decision when that column is non-zero, none
//     or all (by the hard decision) when it is zero.
// Known inputs are zero in the search (:504-509), so the offset of :246-258 is zero.
// oracle/kernel_oracle.c walks the reference's trellis literally; tests compare the two.
//
// Roofline: compute (integer VALU + LDS), no HBM traffic beyond 16 B of counts per
// candidate; 2^20 candidates (m = 5, every L.U product) are one launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "bchk.h"

namespace bchk {
void set_last_error(const char *msg);  // bchk_host.cpp
}

namespace {

constexpr int kMaxL = 32;        // columns as u32 row masks; the trellis processor needs < 64
constexpr int kBlock = 128;      // lanes per workgroup, one candidate each
constexpr unsigned kPrimKS[6] = {3, 7, 11, 19, 37, 67};  // src/main.cpp:14, m = 1..6

struct KsParams {
    uint32_t col[kMaxL];  // column c of the input kernel as a row mask (bit r = K[r][c])
    uint64_t hd;          // bit j: channel LLR j < 0 (TrellisKernelProcessor.cpp:270)
    uint64_t ncodes;      // candidates (codes 0 .. ncodes-1)
    int l;                // kernel size
    int m;                // l = 2^m for the L.U column maps; 0: identity map (score K itself)
    unsigned long long *sum, *cmp;
};

int kfail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    bchk::set_last_error(buf);
    return code;
}

// B = L.U from a candidate code, drawn bits in randomInvertibleMatrix's order (row i:
// l[i][0..i-1], then u[i][i+1..m-1]; root bchCoder.cpp:768-775); returns newBasis[j] =
// column j of B as a bit mask (:608-613).
__host__ __device__ inline void lu_basis(int m, uint64_t code, uint32_t *basis) {
    uint32_t Lr[8], Uc[8];
    for (int i = 0; i < m; ++i) {
        Lr[i] = 1u << i;
        Uc[i] = 1u << i;
    }
    int d = 0;
    for (int i = 0; i < m; ++i) {
        for (int j = 0; j < i; ++j) Lr[i] |= (uint32_t)((code >> d++) & 1u) << j;       // L[i][j]
        for (int j = i + 1; j < m; ++j) Uc[j] |= (uint32_t)((code >> d++) & 1u) << i;   // U[i][j]
    }
    for (int j = 0; j < m; ++j) {
        uint32_t b = 0;
        for (int k = 0; k < m; ++k) b |= (uint32_t)(__builtin_popcount(Lr[k] & Uc[j]) & 1) << k;
        basis[j] = b;
    }
}

__host__ __device__ inline uint32_t map_column(int m, const uint32_t *basis, uint32_t j) {
    uint32_t t = 0;  // temp = sum over the bits k of j of newBasis[k] (:617-623)
    for (int k = 0; k < m; ++k)
        if (j & (1u << k)) t ^= basis[k];
    return t;
}

// One lane per candidate. The per-lane column list and XOR basis live in LDS ([slot][lane],
// so a wave's accesses hit 64 distinct banks), indexed by data-dependent positions.
__global__ void __launch_bounds__(kBlock) trellis_cost_kernel(KsParams p) {
    __shared__ uint32_t cols[kMaxL + 1][kBlock];
    __shared__ uint32_t bas[kMaxL][kBlock];
    const int tid = threadIdx.x;
    const uint64_t code = (uint64_t)blockIdx.x * kBlock + (uint64_t)tid;
    if (code >= p.ncodes) return;  // no block-wide barrier follows
    const int l = p.l;
    uint32_t basis[8];
    if (p.m > 0) lu_basis(p.m, code, basis);
    for (int j = 0; j < l; ++j)
        cols[j][tid] = p.col[p.m > 0 ? map_column(p.m, basis, (uint32_t)j) : (uint32_t)j];
    unsigned long long sum = 0, cmp = 0;
    for (int ph = 0; ph < l; ++ph) {
        // independent-column tests (rank increments) over rows ph..l-1, leading bit = the
        // highest row index of the reduced vector
        auto clear = [&]() {
            for (int b = 0; b < l - ph; ++b) bas[b][tid] = 0u;
        };
        auto independent = [&](uint32_t v) {
            while (v) {
                const int hb = 31 - __builtin_clz(v);
                const uint32_t b = bas[hb][tid];
                if (!b) {
                    bas[hb][tid] = v;
                    return true;
                }
                v ^= b;
            }
            return false;
        };
        uint64_t st = 0, en = 0, nz = 0;
        clear();
        for (int j = 0; j < l; ++j) {
            const uint32_t v = cols[j][tid] >> ph;
            if (v) nz |= 1ull << j;
            if (independent(v)) st |= 1ull << j;
        }
        clear();
        (void)independent(1u);  // the extension column (row ph only) is the last column
        for (int j = l - 1; j >= 0; --j)
            if (independent(cols[j][tid] >> ph)) en |= 1ull << j;
        int a = 0;  // active rows entering depth j
        for (int j = 0; j < l; ++j) {
            const unsigned long long s = 1ull << a;
            const bool sj = (st >> j) & 1ull;
            cmp += sj ? 2 * s : s;
            sum += sj ? s : (((nz >> j) & 1ull) ? s >> 1 : (((p.hd >> j) & 1ull) ? s : 0ull));
            a += (int)sj - (int)((en >> j) & 1ull);
        }
    }
    p.sum[code] = sum;
    p.cmp[code] = cmp;
}

bool invertible(const uint8_t *K, int l) {
    uint64_t rows[64];
    for (int r = 0; r < l; ++r) {
        rows[r] = 0;
        for (int c = 0; c < l; ++c)
            if (K[r * l + c]) rows[r] |= 1ull << c;
    }
    int rank = 0;
    for (int c = 0; c < l && rank < l; ++c) {
        int piv = -1;
        for (int r = rank; r < l; ++r)
            if ((rows[r] >> c) & 1ull) { piv = r; break; }
        if (piv < 0) continue;
        std::swap(rows[rank], rows[piv]);
        for (int r = 0; r < l; ++r)
            if (r != rank && ((rows[r] >> c) & 1ull)) rows[r] ^= rows[rank];
        ++rank;
    }
    return rank == l;
}

// Score ncodes candidates of kernel K on the GPU; sum/cmp: host arrays of ncodes.
int run_costs(const uint8_t *K, int l, int m, const float *llr, uint64_t ncodes, int device,
              uint64_t *sum, uint64_t *cmp) {
    if (l < 2 || l > kMaxL) return kfail(BCHK_EINVAL, "kernel size %d unsupported (2..%d)", l, kMaxL);
    if (!K || !llr || !sum || !cmp) return kfail(BCHK_EINVAL, "NULL argument");
    for (int i = 0; i < l * l; ++i)
        if (K[i] > 1) return kfail(BCHK_EINVAL, "kernel entries must be 0 or 1");
    if (!invertible(K, l)) return kfail(BCHK_EINVAL, "kernel is singular");  // MinimumSpan throws
    KsParams p{};
    for (int c = 0; c < l; ++c) {
        uint32_t v = 0;
        for (int r = 0; r < l; ++r)
            if (K[r * l + c]) v |= 1u << r;
        p.col[c] = v;
    }
    for (int j = 0; j < l; ++j)
        if (llr[j] < 0) p.hd |= 1ull << j;
    p.ncodes = ncodes;
    p.l = l;
    p.m = m;
    if (hipSetDevice(device) != hipSuccess) return kfail(BCHK_ENODEV, "hipSetDevice(%d) failed", device);
    void *d = nullptr;
    const size_t bytes = (size_t)ncodes * sizeof(unsigned long long);
    if (hipMalloc(&d, 2 * bytes) != hipSuccess) return kfail(BCHK_ENOMEM, "hipMalloc(%zu) failed", 2 * bytes);
    p.sum = (unsigned long long *)d;
    p.cmp = p.sum + ncodes;
    const uint64_t blocks = (ncodes + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(trellis_cost_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, 0, p);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(sum, p.sum, bytes, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(cmp, p.cmp, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return kfail(BCHK_EHIP, "trellis_cost_kernel: %s", hipGetErrorString(e));
    return BCHK_OK;
}

}  // namespace

extern "C" {

int bchk_kernel_ebch(int power, uint8_t *K) {
    if (power < 2 || power > 6 || !K) return kfail(BCHK_EINVAL, "power %d unsupported (2..6)", power);
    const int len = (1 << power) - 1, N = len + 1, n = len;
    const int amount = (power != 2) ? ((1 << power) - 2) / 2 : 2;
    std::vector<unsigned> alog(n);
    std::vector<int> lg(N, -1);
    for (unsigned i = 0, v = 1; i < (unsigned)n; ++i) {
        alog[i] = v;
        lg[v] = (int)i;
        v <<= 1;
        if (v >> power) v ^= kPrimKS[power - 1];
    }
    std::memset(K, 0, (size_t)N * N);
    for (int i = 0; i < N; ++i) K[i * N] = 1;  // column 0 (:363-368)
    K[len + 2] = 1;                             // row 1, column 1 (:369)
    std::vector<uint8_t> g(1, 1);
    for (int i = 2; i <= amount; ++i) {
        // minimal polynomial of alpha^i: product of (x + alpha^j) over i's cyclotomic coset
        std::vector<unsigned> poly(1, 1u);
        std::vector<int> coset;
        for (int j = i % n; std::find(coset.begin(), coset.end(), j) == coset.end(); j = 2 * j % n) {
            coset.push_back(j);
            std::vector<unsigned> nx(poly.size() + 1, 0u);
            for (size_t k = 0; k < poly.size(); ++k) {
                if (poly[k]) nx[k] ^= alog[(lg[poly[k]] + j) % n];
                nx[k + 1] ^= poly[k];
            }
            poly.swap(nx);
        }
        const int ps = (int)poly.size(), gOld = (int)g.size();
        if (gOld >= ps) {  // skip a minimal polynomial g already contains (:372)
            std::vector<uint8_t> r(g);
            for (int dd = gOld - 1; dd >= ps - 1; --dd)
                if (r[dd])
                    for (int k = 0; k < ps; ++k) r[dd - (ps - 1) + k] ^= (uint8_t)(poly[k] & 1u);
            bool zero = true;
            for (int k = 0; k < ps - 1; ++k) zero = zero && !r[k];
            if (zero) continue;
        }
        const int gNew = ps + gOld - 1;
        std::vector<uint8_t> prod(gNew, 0);
        for (int a = 0; a < ps; ++a)
            if (poly[a] & 1u)
                for (int b = 0; b < gOld; ++b) prod[a + b] ^= g[b];
        for (int k = 0; k < gNew; ++k) K[gNew * N + 1 + k] = prod[k];  // :374 (offset 1)
        for (int j = gOld, cnt = 1; j < gNew - 1; ++j, ++cnt)           // :375-381
            for (int k = cnt; k < cnt + gOld; ++k) K[(j + 1) * N + k + 1] = g[k - cnt];
        g = prod;                                                       // :382-384
    }
    return BCHK_OK;
}

int bchk_kernel_field_order(int power, const uint8_t *K, uint8_t *out) {
    if (power < 2 || power > 6 || !K || !out) return kfail(BCHK_EINVAL, "power %d unsupported (2..6)", power);
    const int n = 1 << power;
    std::vector<unsigned> alog(n - 1);
    for (unsigned i = 0, v = 1; i < (unsigned)(n - 1); ++i) {
        alog[i] = v;
        v <<= 1;
        if (v >> power) v ^= kPrimKS[power - 1];
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= 2; ++j) out[i * n + j] = K[i * n + j];
    for (int i = 3; i < n; ++i) {  // column i <- old column j + 1 with fieldElements[j] == i
        int j = 2;
        for (; j < n - 1; ++j)
            if ((int)alog[j] == i) break;
        for (int k = 0; k < n; ++k) out[k * n + i] = K[k * n + j + 1];
    }
    return BCHK_OK;
}

int bchk_kernel_trellis_cost(const uint8_t *K, int l, const float *llr, int device, uint64_t *sum,
                             uint64_t *cmp) {
    return run_costs(K, l, 0, llr, 1, device, sum, cmp);
}

int bchk_kernel_column_costs(int power, const uint8_t *K, const float *llr, int device, uint64_t *sum,
                             uint64_t *cmp) {
    if (power < 1 || power > 5) return kfail(BCHK_EINVAL, "power %d unsupported (1..5)", power);
    return run_costs(K, 1 << power, power, llr, 1ull << (power * (power - 1)), device, sum, cmp);
}

int bchk_kernel_column_search(int power, const uint8_t *K, const float *llr, int mode, uint64_t count,
                              uint64_t *rng_state, int device, uint8_t *best, uint32_t *perm,
                              uint64_t *best_sum, uint64_t *best_cmp, int64_t *best_index) {
    if (power < 1 || power > 5) return kfail(BCHK_EINVAL, "power %d unsupported (1..5)", power);
    if (mode != BCHK_KSEARCH_EXHAUSTIVE && mode != BCHK_KSEARCH_RANDOM)
        return kfail(BCHK_EINVAL, "mode %d unknown", mode);
    if (mode == BCHK_KSEARCH_RANDOM && !rng_state) return kfail(BCHK_EINVAL, "rng_state is NULL");
    if (!best_sum || !best_cmp) return kfail(BCHK_EINVAL, "NULL argument");
    const int n = 1 << power, bits = power * (power - 1);
    const uint64_t ncodes = 1ull << bits;
    std::vector<uint64_t> sum(ncodes), cmp(ncodes);
    int rc = run_costs(K, n, power, llr, ncodes, device, sum.data(), cmp.data());
    if (rc) return rc;
    // the reference's acceptance, in candidate order (:651-657)
    uint64_t mins = ~0ull, minc = ~0ull;
    int64_t bi = -1;
    uint64_t bcode = 0;
    auto consider = [&](uint64_t idx, uint64_t code) {
        if (sum[code] < mins && cmp[code] < minc) {
            mins = sum[code];
            minc = cmp[code];
            bi = (int64_t)idx;
            bcode = code;
        }
    };
    if (mode == BCHK_KSEARCH_EXHAUSTIVE) {
        for (uint64_t c = 0; c < ncodes; ++c) consider(c, c);
    } else {
        // randomInvertibleMatrix's draws (:768-775): uniform_int_distribution<unsigned
        // short>(0, 1) on the reference's default_random_engine, bits * count draws
        // (minstd_rand0: the engine's state is its last output; *rng_state in and out)
        struct Rec {
            using result_type = std::default_random_engine::result_type;
            std::default_random_engine e;
            result_type last;
            static constexpr result_type min() { return std::default_random_engine::min(); }
            static constexpr result_type max() { return std::default_random_engine::max(); }
            result_type operator()() { return last = e(); }
        };
        const uint64_t s0 = *rng_state % 2147483647ull;
        Rec eng{std::default_random_engine(s0 ? (unsigned)s0 : 1u), (unsigned)(s0 ? s0 : 1u)};
        std::uniform_int_distribution<unsigned short> bit(0, 1);
        for (uint64_t i = 0; i < count; ++i) {
            uint64_t code = 0;
            for (int d = 0; d < bits; ++d) code |= (uint64_t)bit(eng) << d;
            consider(i, code);
        }
        *rng_state = eng.last;
    }
    *best_sum = mins;
    *best_cmp = minc;
    if (best_index) *best_index = bi;
    if (bi >= 0) {
        uint32_t basis[8];
        lu_basis(power, bcode, basis);
        for (int j = 0; j < n; ++j) {
            const uint32_t t = map_column(power, basis, (uint32_t)j);
            if (perm) perm[j] = t;
            if (best)
                for (int k = 0; k < n; ++k) best[k * n + j] = K[k * n + t];  // :627-629
        }
    }
    return BCHK_OK;
}

}  // extern "C"
