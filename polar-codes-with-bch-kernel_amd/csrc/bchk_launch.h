// bchk_launch.h -- kernel dispatch table shared by bchk_kernels.hip and bchk_host.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "bchk_device.h"

namespace bchk {

// Kernel entry points of one (m, TMAX) instantiation. The *_tab variants decode test
// patterns through the syndrome table (bchk_syndtab.h); null where (m, TMAX) has none.
struct KernelSet {
    hipError_t (*search)(const SearchParams &, int, size_t, hipStream_t);
    hipError_t (*coop)(const SearchParams &, int, size_t, hipStream_t);
    const void *(*coop_ptr)();
    const void *(*search_ptr)();
    hipError_t (*search_tab)(const SearchParams &, int, size_t, hipStream_t);
    hipError_t (*coop_tab)(const SearchParams &, int, size_t, hipStream_t);
    const void *(*coop_tab_ptr)();
    const void *(*search_tab_ptr)();
    size_t coop_bytes;  // LDS bytes of the cooperative kernel beyond the tables
    hipError_t (*alg)(const AlgParams &, size_t, hipStream_t);
    int tmax;
    size_t wave_bytes;  // LDS bytes per wave of the search kernel
    // analytic-tail instance of the search kernel (n <= 63, TMAX <= 8; null elsewhere): it
    // takes the codewords the first pass hands off and finishes them from their candidate
    // codewords, handing only the rest on to the cooperative kernel
    hipError_t (*tail)(const SearchParams &, int, size_t, hipStream_t);
    hipError_t (*tail_tab)(const SearchParams &, int, size_t, hipStream_t);
    const void *(*tail_ptr)();
    const void *(*tail_tab_ptr)();
    size_t tail_wave_bytes;
    size_t tail_block_bytes;  // the block's helper-job control (HelpCtl) after the waves
    int coop_threads;         // the cooperative kernel's workgroup size
    size_t long_job_bytes;    // m >= 7: one job's data (SearchParams::long_jobs), 0 otherwise
    bool gfmul;               // the cooperative kernel reads SearchParams::gfmul (BCHK_LONG_GFMUL builds)
};

typedef hipError_t (*FastFn)(const SearchParams &, size_t, hipStream_t);

// Fast path: lane per codeword for n <= 63 (bchk_fast.hip), first test patterns of every
// codeword for m >= 7 (kaneko_first_kernel, bchk_kernels.hip); false when (m, t) has none.
bool select_fast(int m, int t, FastFn *out);
bool select_first_long(int m, int t, FastFn *out);
// the lane pre-pass of the long-code first kernel (m >= 7, t <= 15; false: none)
bool select_lane(int m, int t, FastFn *out);
size_t fast_wave_bytes();
int fast_block_waves();  // waves per block of the fast kernel

// Picks the (m, TMAX) instantiation for runtime t (smallest TMAX >= t).
bool select_kernels(int m, int t, KernelSet *out);
// search / cooperative kernel: the table variant when p.tab.slots is set and it exists
hipError_t launch_search(const KernelSet &k, const SearchParams &p, int grid, size_t lds, hipStream_t s);
hipError_t launch_coop(const KernelSet &k, const SearchParams &p, int grid, size_t lds, hipStream_t s);
hipError_t launch_tail(const KernelSet &k, const SearchParams &p, int grid, size_t lds, hipStream_t s);
constexpr int kCoopThreads = 1024;
hipError_t launch_alg(const KernelSet &k, const AlgParams &p, size_t lds, hipStream_t s);
hipError_t launch_count(int n, const uint8_t *tx, const uint8_t *res, const bchk_stats *st,
                        uint32_t B, uint64_t *out6, hipStream_t s);
// on-GPU channel words (bchk_channel.hip) and per-word frame-error flags (tx != res)
hipError_t launch_channel(const ChanParams &cp, hipStream_t s);
hipError_t launch_frame_errors(const uint8_t *tx, const uint8_t *res, uint32_t B, int n, uint8_t *flags,
                               hipStream_t s);
// the fused counters (SearchParams::cnt) into out6, slots zeroed
hipError_t launch_cnt_reduce(unsigned long long *cnt, unsigned long long *out6, hipStream_t s);

}  // namespace bchk
