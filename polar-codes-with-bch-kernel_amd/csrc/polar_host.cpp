// polar_host.cpp -- host runtime of the GPU SC-list decoder behind the C ABI (bchk_polar_*
// in include/bchk.h): the reference's code specification, the dynamic-freezing masks, the
// device tables and the batched launch. Replaces CMixedKernelListDecoder(Spec, ListSize)
// and Decode(pLLR, pInfVectorList, pCodewordList) (headers/external/MixedKernelListDecoder.h:
// 27-39, out/external/MixedKernelListDecoder.cpp:9, :211-268) and CMixedKernelEncoder::Encode
// (out/external/MixedKernelEncoder.cpp:142-177). All decoding runs on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "bchk.h"
#include "polar_device.h"

using namespace bchk;

namespace bchk {
hipError_t launch_polar(const PolarParams &p, int grid, size_t lds, hipStream_t s);
const void *polar_kernel_ptr();
void set_last_error(const char *msg);  // bchk_host.cpp: the message bchk_last_error returns
}  // namespace bchk

namespace {

int pfail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    set_last_error(buf);
    return code;
}

#define PHIP_TRY(expr)                                                                  \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return pfail(BCHK_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),     \
                         __FILE__, __LINE__);                                           \
    } while (0)

struct PBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, bytes) != hipSuccess) return pfail(BCHK_ENOMEM, "hipMalloc(%zu) failed", bytes);
        cap = bytes;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

struct bchk_polar {
    int N = 0, K = 0, U = 0, n = 0, L = 0, device = 0;
    std::vector<int16_t> symmap, infopos, cwpos;
    std::vector<uint8_t> frozen;
    std::vector<int8_t> dfbit;
    std::vector<uint64_t> dfcorr;
    std::vector<std::vector<int>> fc;  // freezing constraints (terms, frozen symbol last)
    std::vector<int> decision;         // constraint of each symbol, -1 = unfrozen
    uint8_t *d_tab = nullptr;          // one blob: symmap | phase | cwpos | dfcorr
    size_t off_symmap = 0, off_phase = 0, off_cwpos = 0, off_dfcorr = 0;
    hipStream_t stream = nullptr;
    size_t lds = 0;
    int grid = 0;
    PBuf llr, info, cw, metric, count;
};

namespace {

// The specification (MixedKernelEncoder.cpp:7-98): header, kernel names, shortened and
// punctured symbols, then U - K freezing constraints "w t_1 ... t_w" (ascending, the frozen
// symbol last). The GPU decoder takes Arikan layers ("A"); other kernels are rejected.
int parse_spec(bchk_polar *c, const char *spec) {
    std::istringstream in(spec);
    int N, K, dmin, layers, nsh, npu;
    if (!(in >> N >> K >> dmin >> layers >> nsh >> npu)) return pfail(BCHK_EINVAL, "Error reading file header");
    if (K > N || K < 0 || N <= 0) return pfail(BCHK_EINVAL, "Code dimension cannot exceed code length");
    if (layers < 1 || layers > kPolarMaxLayers) return pfail(BCHK_EINVAL, "%d layers unsupported", layers);
    for (int i = 0; i < layers; ++i) {
        std::string name;
        if (!(in >> name)) return pfail(BCHK_EINVAL, "missing kernel name %d", i);
        if (!(name == "A" || name == "a"))
            return pfail(BCHK_EINVAL, "kernel %s: the GPU SC-list decoder takes Arikan (A) layers only",
                         name.c_str());
    }
    const int U = 1 << layers;
    if (N + nsh + npu != U) return pfail(BCHK_EINVAL, "Code length mismatch");
    c->N = N;
    c->K = K;
    c->U = U;
    c->n = layers;
    std::vector<uint8_t> type(U, 0);
    for (int i = 0; i < nsh + npu; ++i) {
        int s;
        if (!(in >> s) || s < 0 || s >= U) return pfail(BCHK_EINVAL, "Invalid shortened / punctured symbol");
        type[s] = (uint8_t)(i < nsh ? 1 : 2);
    }
    c->decision.assign(U, -1);
    c->fc.assign(U - K, {});
    for (int i = 0; i < U - K; ++i) {
        int w;
        if (!(in >> w) || w < 1) return pfail(BCHK_EINVAL, "Error reading freezing constraint %d", i);
        for (int j = 0; j < w; ++j) {
            int v;
            if (!(in >> v) || v < 0 || v >= U || (j && v <= c->fc[i].back()))
                return pfail(BCHK_EINVAL, "Invalid freezing constraint %d", i);
            c->fc[i].push_back(v);
        }
        const int last = c->fc[i].back();
        if (c->decision[last] != -1) return pfail(BCHK_EINVAL, "Duplicate freezing constraint on symbol %d", last);
        c->decision[last] = i;
    }
    // dynamic-freezing value bits (KernelListEngine.cpp:6-39)
    c->dfbit.assign(U, -1);
    c->dfcorr.assign(U, 0);
    uint64_t avail = ~0ull;
    for (int i = 0; i < U; ++i) {
        if (c->dfbit[i] >= 0) avail |= 1ull << c->dfbit[i];
        for (int j = i + 1; j < U; ++j) {
            const int ci = c->decision[j];
            if (ci < 0 || c->fc[ci][0] != i) continue;
            if (!avail) return pfail(BCHK_EINVAL, "Too many dynamic freezing constraints are simultaneously active");
            const int B = __builtin_ctzll(avail);
            avail &= ~(1ull << B);
            c->dfbit[j] = (int8_t)B;
            for (int t : c->fc[ci]) {
                if (t == j) break;
                c->dfcorr[t] ^= 1ull << B;
            }
            c->dfcorr[j] ^= 1ull << B;
        }
    }
    c->symmap.assign(U, 0);
    c->frozen.assign(U, 0);
    c->infopos.clear();
    c->cwpos.clear();
    for (int i = 0, I = 0; i < U; ++i) {
        c->symmap[i] = (int16_t)(type[i] == 0 ? I++ : (type[i] == 1 ? -1 : -2));
        if (type[i] == 0) c->cwpos.push_back((int16_t)i);
        c->frozen[i] = c->decision[i] >= 0;
        if (c->decision[i] < 0) c->infopos.push_back((int16_t)i);
    }
    return 0;
}

}  // namespace

extern "C" {

int bchk_polar_create(const char *spec, int list_size, int device, bchk_polar **out) {
    if (!out || !spec) return pfail(BCHK_EINVAL, "NULL argument");
    *out = nullptr;
    if (list_size < 1 || list_size > kPolarMaxList)
        return pfail(BCHK_EINVAL, "list size %d unsupported (1..%d)", list_size, kPolarMaxList);
    // the specification is checked first, so malformed codes are reported with or without a GPU
    bchk_polar *c = new bchk_polar();
    c->L = list_size;
    c->device = device;
    if (int rc = parse_spec(c, spec)) {
        delete c;
        return rc;
    }
    c->lds = polar_lds_bytes(c->U, c->L, c->K);
    if (c->lds > 160 * 1024) {
        const size_t need = c->lds;
        const int U = c->U;
        delete c;
        return pfail(BCHK_EINVAL, "length %d with list %d needs %zu B of LDS (> 160 KiB)", U, list_size, need);
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        delete c;
        return pfail(BCHK_ENODEV, "no HIP device visible (the SC-list decoder has no CPU fallback)");
    }
    if (device < 0 || device >= ndev) {
        delete c;
        return pfail(BCHK_EINVAL, "device %d out of range", device);
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        delete c;
        return pfail(BCHK_ENODEV, "device %d is not gfx950; libbchk is built for gfx950 only", device);
    }
    if (hipSetDevice(device) != hipSuccess) {
        delete c;
        return pfail(BCHK_EHIP, "hipSetDevice(%d) failed", device);
    }
    // device tables, one blob
    auto al = [](size_t v) { return (v + 15) & ~size_t(15); };
    size_t o = 0;
    c->off_symmap = o; o = al(o + 2 * (size_t)c->U);
    c->off_phase = o; o = al(o + 2 * (size_t)c->U);
    c->off_cwpos = o; o = al(o + 2 * (size_t)c->N);
    c->off_dfcorr = o; o = al(o + 8 * (size_t)c->U);
    std::vector<uint8_t> blob(o, 0);
    memcpy(blob.data() + c->off_symmap, c->symmap.data(), 2 * (size_t)c->U);
    {
        uint16_t *ph = reinterpret_cast<uint16_t *>(blob.data() + c->off_phase);
        for (int i = 0; i < c->U; ++i)
            ph[i] = (uint16_t)((c->frozen[i] ? kPhaseFrozen : 0u) | ((uint16_t)(c->dfbit[i] + 1) << 1) |
                               (c->dfcorr[i] ? kPhaseCorr : 0u));
    }
    memcpy(blob.data() + c->off_cwpos, c->cwpos.data(), 2 * (size_t)c->N);
    memcpy(blob.data() + c->off_dfcorr, c->dfcorr.data(), 8 * (size_t)c->U);
    if (hipMalloc(&c->d_tab, o) != hipSuccess ||
        hipMemcpy(c->d_tab, blob.data(), o, hipMemcpyHostToDevice) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        bchk_polar_destroy(c);
        return pfail(BCHK_EHIP, "device setup failed");
    }
    const void *fn = polar_kernel_ptr();
    if (c->lds > 65536) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, c->lds) != hipSuccess || per_cu <= 0) {
        per_cu = 1;
        (void)hipGetLastError();
    }
    c->grid = per_cu * prop.multiProcessorCount;
    if (const char *g = getenv("BCHK_POLAR_GRID")) c->grid = std::max(1, atoi(g));
    if (getenv("BCHK_POLAR_DEBUG"))
        fprintf(stderr, "bchk_polar: U=%d L=%d lds=%u per_cu=%d CUs=%d grid=%d\n", c->U, c->L, c->lds, per_cu,
                prop.multiProcessorCount, c->grid);
    *out = c;
    return 0;
}

void bchk_polar_destroy(bchk_polar *c) {
    if (!c) return;
    c->llr.release();
    c->info.release();
    c->cw.release();
    c->metric.release();
    c->count.release();
    if (c->d_tab) (void)hipFree(c->d_tab);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int bchk_polar_params(const bchk_polar *c, int *n, int *k, int *unshortened, int *list_size) {
    if (!c) return pfail(BCHK_EINVAL, "NULL argument");
    if (n) *n = c->N;
    if (k) *k = c->K;
    if (unshortened) *unshortened = c->U;
    if (list_size) *list_size = c->L;
    return 0;
}

int bchk_polar_decode_device(bchk_polar *c, const float *d_llr, size_t B, uint8_t *d_info,
                             uint8_t *d_cw, float *d_metric, int32_t *d_count, void *stream) {
    if (!c || (B && (!d_llr || !d_info || !d_metric || !d_count))) return pfail(BCHK_EINVAL, "NULL argument");
    if (B == 0) return 0;
    if (B > 0xFFFFFFFFull) return pfail(BCHK_EINVAL, "batch too large");
    PolarParams p{};
    p.llr = d_llr;
    p.info = d_info;
    p.cw = d_cw;
    p.metric = d_metric;
    p.count = d_count;
    p.symmap = reinterpret_cast<const int16_t *>(c->d_tab + c->off_symmap);
    p.phase = reinterpret_cast<const uint16_t *>(c->d_tab + c->off_phase);
    p.cwpos = reinterpret_cast<const int16_t *>(c->d_tab + c->off_cwpos);
    p.dfcorr = reinterpret_cast<const uint64_t *>(c->d_tab + c->off_dfcorr);
    p.B = (uint32_t)B;
    p.n = c->n;
    p.U = c->U;
    p.N = c->N;
    p.K = c->K;
    p.L = c->L;
    const int grid = (int)std::min<size_t>((size_t)c->grid, B);
    PHIP_TRY(launch_polar(p, grid, c->lds, stream ? (hipStream_t)stream : c->stream));
    return 0;
}

int bchk_polar_decode_host(bchk_polar *c, const float *llr, size_t B, uint8_t *info, uint8_t *cw,
                           float *metric, int32_t *count) {
    if (!c || (B && (!llr || !info || !metric || !count))) return pfail(BCHK_EINVAL, "NULL argument");
    if (B == 0) return 0;
    const size_t L = (size_t)c->L;
    int rc;
    if ((rc = c->llr.ensure(B * c->N * sizeof(float))) || (rc = c->info.ensure(B * L * std::max(c->K, 1))) ||
        (rc = c->metric.ensure(B * L * sizeof(float))) || (rc = c->count.ensure(B * sizeof(int32_t))) ||
        (cw && (rc = c->cw.ensure(B * L * c->N))))
        return rc;
    PHIP_TRY(hipMemcpyAsync(c->llr.p, llr, B * c->N * sizeof(float), hipMemcpyHostToDevice, c->stream));
    // list rows past each count keep the caller's contents, as the reference leaves them
    PHIP_TRY(hipMemcpyAsync(c->info.p, info, B * L * c->K, hipMemcpyHostToDevice, c->stream));
    PHIP_TRY(hipMemcpyAsync(c->metric.p, metric, B * L * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if (cw) PHIP_TRY(hipMemcpyAsync(c->cw.p, cw, B * L * c->N, hipMemcpyHostToDevice, c->stream));
    if ((rc = bchk_polar_decode_device(c, (const float *)c->llr.p, B, (uint8_t *)c->info.p,
                                       cw ? (uint8_t *)c->cw.p : nullptr, (float *)c->metric.p,
                                       (int32_t *)c->count.p, c->stream)))
        return rc;
    PHIP_TRY(hipMemcpyAsync(info, c->info.p, B * L * c->K, hipMemcpyDeviceToHost, c->stream));
    PHIP_TRY(hipMemcpyAsync(metric, c->metric.p, B * L * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    PHIP_TRY(hipMemcpyAsync(count, c->count.p, B * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    if (cw) PHIP_TRY(hipMemcpyAsync(cw, c->cw.p, B * L * c->N, hipMemcpyDeviceToHost, c->stream));
    PHIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

// CMixedKernelEncoder::Encode (MixedKernelEncoder.cpp:142-177) for Arikan layers, host side:
// frozen symbols from their constraints, the transform, then the transmitted symbols.
int bchk_polar_encode_host(const bchk_polar *c, const uint8_t *info, size_t B, uint8_t *cw) {
    if (!c || (B && (!info || !cw))) return pfail(BCHK_EINVAL, "NULL argument");
    std::vector<uint8_t> u(c->U);
    for (size_t b = 0; b < B; ++b) {
        const uint8_t *in = info + b * c->K;
        int k = 0;
        for (int i = 0; i < c->U; ++i) {
            const int ci = c->decision[i];
            if (ci >= 0) {
                uint8_t v = 0;
                for (int t : c->fc[ci]) {
                    if (t == i) break;
                    v ^= u[t];
                }
                u[i] = v;
            } else {
                u[i] = in[k++] & 1;
            }
        }
        for (int st = 1; st < c->U; st <<= 1)
            for (int i = 0; i < c->U; ++i)
                if (!(i & st)) u[i] ^= u[i + st];
        for (int i = 0; i < c->N; ++i) cw[b * c->N + i] = u[c->cwpos[i]];
    }
    return 0;
}

int bchk_polar_sync(bchk_polar *c) {
    if (!c) return pfail(BCHK_EINVAL, "NULL argument");
    PHIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

void *bchk_polar_stream(bchk_polar *c) { return c ? (void *)c->stream : nullptr; }

}  // extern "C"
