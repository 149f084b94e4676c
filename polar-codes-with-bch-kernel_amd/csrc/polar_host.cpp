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
hipError_t launch_polar_mixed(const PolarMixedParams &p, int grid, size_t lds, hipStream_t s);
const void *polar_mixed_kernel_ptr();
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
    // layers: kernel size, Arikan flag, rows as bitmasks (bit c = K[r][c]); mixed = any
    // matrix layer (decoded by polar_mixed_kernel)
    bool mixed = false;
    std::vector<int> ksize;
    std::vector<uint8_t> arikan;
    std::vector<uint64_t> krows;  // [layer][kPolarMaxKernel]
    PolarMixedParams mp{};        // the mixed layout (sizes, offsets)
    size_t off_krows = 0;
    std::vector<uint32_t> tent, tbase;  // matrix-layer trellises (polar_device.h)
    std::vector<uint8_t> tlog;
    size_t off_tent = 0, off_tbase = 0, off_tlog = 0;
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
    // time-budgeted launches of codes with search layers (PolarMixedParams::budget)
    PBuf rstate, rsave, unfinished;
    uint64_t budget_ticks = 0;  // 100 MHz ticks per launch, 0 = one launch per call
    uint64_t launches_last = 0; // launches the last budgeted call took
};

namespace {

// The specification (MixedKernelEncoder.cpp:7-98): header, kernel names, shortened and
// punctured symbols, then U - K freezing constraints "w t_1 ... t_w" (ascending, the frozen
// symbol last). The GPU decoder takes Arikan layers ("A"); other kernels are rejected.
// GetKernelByName (Kernel.cpp:235-252): "A" (any case), or a matrix file "-path" / "<path"
// (relative to kdir) holding the size and size^2 entries (Kernel.cpp:93-107); the kernel must
// be invertible (Kernel.cpp:155-176).
int read_kernel(const std::string &name, const char *kdir, int *size, uint64_t *rows, bool *arikan) {
    if (name == "A" || name == "a") {
        *size = 2;
        rows[0] = 1u;       // 1 0
        rows[1] = 3u;       // 1 1  (Kernel.cpp:8-12)
        *arikan = true;
        return 0;
    }
    if (name.empty() || (name[0] != '-' && name[0] != '<')) return pfail(BCHK_EINVAL, "Unknown kernel %s", name.c_str());
    std::string path = name.substr(1);
    if (!path.empty() && path[0] != '/' && kdir && kdir[0]) path = std::string(kdir) + "/" + path;
    FILE *f = fopen(path.c_str(), "r");
    if (!f) return pfail(BCHK_EINVAL, "Error reading kernel file %s", path.c_str());
    int l = 0;
    if (fscanf(f, "%d", &l) != 1 || l < 2 || l > kPolarMaxKernel) {
        fclose(f);
        return pfail(BCHK_EINVAL, "Error reading kernel file %s (size)", path.c_str());
    }
    for (int r = 0; r < l; ++r) {
        rows[r] = 0;
        for (int q = 0; q < l; ++q) {
            unsigned v;
            if (fscanf(f, "%u", &v) != 1) {
                fclose(f);
                return pfail(BCHK_EINVAL, "Error parsing kernel file %s", path.c_str());
            }
            if (v) rows[r] |= 1ull << q;
        }
    }
    fclose(f);
    std::vector<uint64_t> a(rows, rows + l);  // GF(2) rank
    for (int col = 0, r0 = 0; col < l; ++col) {
        int piv = r0;
        while (piv < l && !((a[piv] >> col) & 1ull)) ++piv;
        if (piv == l) return pfail(BCHK_EINVAL, "Kernel is singular (%s)", path.c_str());
        std::swap(a[piv], a[r0]);
        for (int r = 0; r < l; ++r)
            if (r != r0 && ((a[r] >> col) & 1ull)) a[r] ^= a[r0];
        ++r0;
    }
    if (l > kPolarMaxMatrixGpu)
        return pfail(BCHK_EINVAL, "matrix kernel of size %d: the GPU SC-list decoder takes sizes up to %d", l,
                     kPolarMaxMatrixGpu);
    *size = l;
    *arikan = false;
    return 0;
}

// CTrellisKernelProcessor's trellis of every phase of an l x l kernel (out/external/
// TrellisKernelProcessor.cpp:69-179: MinimumSpan :7-67 of rows phase..l-1 with row `phase`
// extended by a 1 at position l, states = active rows, state bits compressed as rows end),
// stored as predecessor lists for the GPU's pull-form Viterbi (polar_device.h). Appends to
// ent; base[phase], lg[phase * (kPolarMaxKernel + 1) + d]; returns the largest state count
// (0 and a message when a depth needs more than 2^kPolarTrellisMaxBits states).
int build_trellis(const uint64_t *rows, int l, std::vector<uint32_t> &ent, uint32_t *base, uint8_t *lg) {
    if (l > kPolarMaxTrellisKernel) return pfail(BCHK_EINVAL, "no trellis for a kernel of size %d (> %d)", l, kPolarMaxTrellisKernel), 0;
    int most = 1;
    const unsigned N = (unsigned)l + 1u;
    for (int ph = 0; ph < l; ++ph) {
        const unsigned K = (unsigned)(l - ph);
        uint64_t M[kPolarMaxKernel];
        for (unsigned i = 0; i < K; ++i) M[i] = rows[ph + (int)i];
        M[0] |= 1ull << l;
        unsigned start[kPolarMaxKernel + 1], end[kPolarMaxKernel + 1];
        for (unsigned c = 0; c < N; ++c) start[c] = end[c] = ~0u;
        unsigned C = 0;  // MinimumSpan (:7-67)
        for (unsigned i = 0; i < K; ++i) {
            bool found = false;
            for (; C < N; ++C) {
                if (!((M[i] >> C) & 1ull)) {
                    for (unsigned j = i + 1; j < K; ++j)
                        if ((M[j] >> C) & 1ull) {
                            M[i] ^= M[j];
                            found = true;
                            break;
                        }
                    if (found) {
                        start[C] = i;
                        break;
                    }
                } else {
                    start[C] = i;
                    found = true;
                    break;
                }
            }
            if (!found) return pfail(BCHK_EINVAL, "Matrix is not full rank"), 0;
            for (unsigned j = i + 1; j < K; ++j)
                if ((M[j] >> C) & 1ull) M[j] ^= M[i];
        }
        for (int i = (int)K - 1; i >= 0; --i)
            for (int j = (int)N - 1; j >= 0; --j)
                if ((M[i] >> j) & 1ull) {
                    end[j] = (unsigned)i;
                    for (int q = 0; q < i; ++q)
                        if ((M[q] >> j) & 1ull) M[q] ^= M[i];
                    break;
                }
        base[ph] = (uint32_t)ent.size();
        uint8_t *lgp = lg + (size_t)ph * (kPolarMaxKernel + 1);
        lgp[0] = 0;
        std::vector<uint64_t> cw0(1, 0ull), cw1;
        unsigned active[kPolarMaxKernel + 1], na = 0;
        for (int j = 0; j < l; ++j) {  // :107-158, depths 0..l-1 (GetLLRs never reads depth l's edges)
            unsigned B = na;
            for (unsigned q = 0; q < na; ++q)
                if (active[q] == end[j]) { B = q; break; }
            const uint64_t emask = (end[j] == ~0u) ? ~0ull : ((1ull << B) - 1ull);
            const uint64_t ns = 1ull << na;
            const unsigned na1 = na + (start[j] != ~0u ? 1u : 0u) - (end[j] != ~0u ? 1u : 0u);
            if (na1 > (unsigned)kPolarTrellisMaxBits || na + 1 > (unsigned)kPolarTrellisMaxBits + 1)
                return pfail(BCHK_EINVAL, "kernel of size %d: its trellis needs 2^%u states (GPU limit 2^%d)", l,
                             std::max(na1, na), kPolarTrellisMaxBits), 0;
            const uint64_t ns1 = 1ull << na1;
            cw1.assign(ns1, 0ull);
            const size_t e0 = ent.size();
            ent.resize(e0 + ns1, 0u);
            auto link = [&](uint64_t S, uint64_t S1, uint32_t z) {
                uint32_t &e = ent[e0 + S1];
                const uint32_t h = (uint32_t)S | (z ? kTrellisZ : 0u) | kTrellisValid;
                if (!(e & kTrellisValid)) e |= h;
                else e |= h << 16;
            };
            if (start[j] == ~0u) {
                for (uint64_t S = 0; S < ns; ++S) {
                    const uint32_t bit = (uint32_t)((cw0[S] >> j) & 1ull);
                    const uint64_t nx = (S & emask) | ((S >> 1) & ~emask);
                    cw1[nx] = cw0[S];
                    link(S, nx, bit);
                }
            } else {
                for (uint64_t S = 0; S < ns; ++S) {
                    uint64_t n0 = S, n1 = S ^ (1ull << na);
                    n0 = (n0 & emask) | ((n0 >> 1) & ~emask);
                    n1 = (n1 & emask) | ((n1 >> 1) & ~emask);
                    const uint64_t c1 = cw0[S] ^ M[start[j]];
                    cw1[n0] = cw0[S];
                    cw1[n1] = c1;
                    link(S, n0, (uint32_t)((cw0[S] >> j) & 1ull));
                    link(S, n1, (uint32_t)((c1 >> j) & 1ull));
                }
                active[na++] = start[j];
            }
            cw0.swap(cw1);
            if (end[j] != ~0u) {
                memmove(active + B, active + B + 1, sizeof(unsigned) * (na - B - 1));
                --na;
            }
            if (na != na1) return pfail(BCHK_EINVAL, "trellis construction inconsistent"), 0;
            lgp[j + 1] = (uint8_t)na;
            most = std::max(most, 1 << na);
        }
    }
    return most;
}

int parse_spec(bchk_polar *c, const char *spec, const char *kdir) {
    std::istringstream in(spec);
    int N, K, dmin, layers, nsh, npu;
    if (!(in >> N >> K >> dmin >> layers >> nsh >> npu)) return pfail(BCHK_EINVAL, "Error reading file header");
    if (K > N || K < 0 || N <= 0) return pfail(BCHK_EINVAL, "Code dimension cannot exceed code length");
    if (layers < 1 || layers > kPolarMaxLayers) return pfail(BCHK_EINVAL, "%d layers unsupported", layers);
    c->ksize.assign(layers, 2);
    c->arikan.assign(layers, 1);
    c->krows.assign((size_t)layers * kPolarMaxKernel, 0ull);
    long Ul = 1;
    for (int i = 0; i < layers; ++i) {
        std::string name;
        if (!(in >> name)) return pfail(BCHK_EINVAL, "missing kernel name %d", i);
        bool ar = false;
        if (int rc = read_kernel(name, kdir, &c->ksize[i], &c->krows[(size_t)i * kPolarMaxKernel], &ar)) return rc;
        c->arikan[i] = ar ? 1 : 0;
        c->mixed = c->mixed || !ar;
        Ul *= c->ksize[i];
        if (Ul > 16384) return pfail(BCHK_EINVAL, "length %ld exceeds 16384", Ul);
    }
    const int U = (int)Ul;
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
    return bchk_polar_create_kdir(spec, nullptr, list_size, device, out);
}

int bchk_polar_create_kdir(const char *spec, const char *kdir, int list_size, int device, bchk_polar **out) {
    if (!out || !spec) return pfail(BCHK_EINVAL, "NULL argument");
    *out = nullptr;
    if (list_size < 1 || list_size > kPolarMaxList)
        return pfail(BCHK_EINVAL, "list size %d unsupported (1..%d)", list_size, kPolarMaxList);
    // the specification is checked first, so malformed codes are reported with or without a GPU
    bchk_polar *c = new bchk_polar();
    c->L = list_size;
    c->device = device;
    if (int rc = parse_spec(c, spec, kdir)) {
        delete c;
        return rc;
    }
    if (c->mixed) {  // the mixed layout (oracle/polar_oracle.c plr_decode's offsets)
        PolarMixedParams &m = c->mp;
        const int nl = c->n;
        m.nl = nl;
        m.outer[0] = c->U;
        for (int j = 0; j < nl; ++j) {
            m.ksize[j] = c->ksize[j];
            m.arikan[j] = c->arikan[j];
            m.outer[j + 1] = m.outer[j] / c->ksize[j];
        }
        int so = 0, co = 0, oo = 0;
        for (int lam = 1; lam <= nl; ++lam) { m.soff[lam] = so; so += m.outer[lam]; }
        for (int lam = 0; lam <= nl; ++lam) { m.coff[lam] = co; co += lam ? m.outer[lam] * c->ksize[lam - 1] : m.outer[0]; }
        for (int j = 0; j < nl; ++j) { m.ooff[j] = oo; if (!c->arikan[j]) oo += c->ksize[j] * m.outer[j + 1]; }
        m.soff[0] = 0;
        m.ssize = (so + 3) & ~3;
        m.csize = (co + 15) & ~15;
        m.osize = (oo + 15) & ~15;
        // matrix layers from the trellis threshold up take their LLRs from the trellis; those
        // larger than the trellis limit (or from BCHK_POLAR_ML up) from the exact
        // ordered-statistics search
        int tmin = 16, mlmin = kPolarMaxTrellisKernel + 1;
        if (const char *e = getenv("BCHK_POLAR_TRELLIS")) tmin = std::max(2, atoi(e));
        if (const char *e = getenv("BCHK_POLAR_ML")) mlmin = std::max(2, atoi(e));
        m.any_ml = 0;
        m.tstates = 0;
        c->tbase.assign((size_t)nl * kPolarMaxKernel, 0u);
        c->tlog.assign((size_t)nl * kPolarMaxKernel * (kPolarMaxKernel + 1), 0u);
        c->tent.clear();
        for (int j = 0; j < nl; ++j) {
            m.ml[j] = (!c->arikan[j] && c->ksize[j] >= std::min(mlmin, kPolarMaxTrellisKernel + 1)) ? 1 : 0;
            m.any_ml |= m.ml[j];
            m.trellis[j] = (!c->arikan[j] && !m.ml[j] && c->ksize[j] >= tmin) ? 1 : 0;
            if (!m.trellis[j]) continue;
            const int most = build_trellis(&c->krows[(size_t)j * kPolarMaxKernel], c->ksize[j], c->tent,
                                           &c->tbase[(size_t)j * kPolarMaxKernel],
                                           &c->tlog[(size_t)j * kPolarMaxKernel * (kPolarMaxKernel + 1)]);
            if (!most) {
                delete c;
                return BCHK_EINVAL;  // build_trellis set the message
            }
            m.tstates = std::max(m.tstates, std::max(64, most));
        }
        if (c->tent.empty()) c->tent.push_back(0u);
        c->lds = polar_mixed_lds_bytes(c->U, c->L, c->K, m.ssize, m.csize, m.osize, nl, m.tstates, m.any_ml != 0);
    } else {
        c->lds = polar_lds_bytes(c->U, c->L, c->K);
    }
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
    c->off_krows = o; o = al(o + 8 * c->krows.size());
    c->off_tent = o; o = al(o + 4 * c->tent.size());
    c->off_tbase = o; o = al(o + 4 * c->tbase.size());
    c->off_tlog = o; o = al(o + c->tlog.size());
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
    memcpy(blob.data() + c->off_krows, c->krows.data(), 8 * c->krows.size());
    if (!c->tent.empty()) memcpy(blob.data() + c->off_tent, c->tent.data(), 4 * c->tent.size());
    if (!c->tbase.empty()) memcpy(blob.data() + c->off_tbase, c->tbase.data(), 4 * c->tbase.size());
    if (!c->tlog.empty()) memcpy(blob.data() + c->off_tlog, c->tlog.data(), c->tlog.size());
    if (hipMalloc(&c->d_tab, o) != hipSuccess ||
        hipMemcpy(c->d_tab, blob.data(), o, hipMemcpyHostToDevice) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        bchk_polar_destroy(c);
        return pfail(BCHK_EHIP, "device setup failed");
    }
    const void *fn = c->mixed ? polar_mixed_kernel_ptr() : polar_kernel_ptr();
    if (c->lds > 65536) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, c->lds) != hipSuccess || per_cu <= 0) {
        per_cu = 1;
        (void)hipGetLastError();
    }
    c->grid = per_cu * prop.multiProcessorCount;
    if (const char *g = getenv("BCHK_POLAR_GRID")) c->grid = std::max(1, atoi(g));
    // codes with search layers: launches of at most ~50 ms (BCHK_POLAR_BUDGET_MS, 0 = one
    // launch per call), so no launch holds the GPU for seconds
    if (c->mixed && c->mp.any_ml) {
        double ms = 50.0;
        if (const char *b = getenv("BCHK_POLAR_BUDGET_MS")) ms = std::max(0.0, atof(b));
        c->budget_ticks = (uint64_t)(ms * 1e5);  // s_memrealtime: 100 MHz
    }
    if (getenv("BCHK_POLAR_DEBUG"))
        fprintf(stderr, "bchk_polar: U=%d L=%d lds=%zu per_cu=%d CUs=%d grid=%d\n", c->U, c->L, c->lds, per_cu,
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
    c->rstate.release();
    c->rsave.release();
    c->unfinished.release();
    if (c->d_tab) (void)hipFree(c->d_tab);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int bchk_polar_last_launches(const bchk_polar *c, uint64_t *launches) {
    if (!c || !launches) return pfail(BCHK_EINVAL, "NULL argument");
    *launches = c->budget_ticks ? c->launches_last : 1;
    return 0;
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
    p.pathCw = polar_cw_layout(c->U, p.cwoff);
    p.n = c->n;
    p.U = c->U;
    p.N = c->N;
    p.K = c->K;
    p.L = c->L;
    const int grid = (int)std::min<size_t>((size_t)c->grid, B);
    if (c->mixed) {
        PolarMixedParams m = c->mp;
        m.llr = p.llr;
        m.info = p.info;
        m.cw = p.cw;
        m.metric = p.metric;
        m.count = p.count;
        m.symmap = p.symmap;
        m.phase = p.phase;
        m.dfcorr = p.dfcorr;
        m.cwpos = p.cwpos;
        m.krows = reinterpret_cast<const uint64_t *>(c->d_tab + c->off_krows);
        m.tent = reinterpret_cast<const uint32_t *>(c->d_tab + c->off_tent);
        m.tbase = reinterpret_cast<const uint32_t *>(c->d_tab + c->off_tbase);
        m.tlog = c->d_tab + c->off_tlog;
        m.B = p.B;
        m.U = c->U;
        m.N = c->N;
        m.K = c->K;
        m.L = c->L;
        hipStream_t s = stream ? (hipStream_t)stream : c->stream;
        if (!(m.any_ml && c->budget_ticks)) {
            PHIP_TRY(launch_polar_mixed(m, grid, c->lds, s));
            return 0;
        }
        // Codes with search layers: one codeword's list decode can run for seconds (every
        // phase's search items in one wave), so the call is a series of launches of at most
        // ~budget each (plus one search item): a wave suspends its codeword between two items
        // past the budget and the next launch resumes it (same results, bit for bit: the
        // state saved is the whole list state). The call returns when every codeword is done.
        const PolarMixedLayout ol = polar_mixed_layout(c->U, c->L, m.ssize, m.csize, m.osize, m.nl, polar_rec_words(c->K));
        const uint32_t stride = polar_mixed_save_bytes(ol);
        int rc;
        if ((rc = c->rstate.ensure(B * 4)) || (rc = c->rsave.ensure(B * (size_t)stride)) ||
            (rc = c->unfinished.ensure(4)))
            return rc;
        PHIP_TRY(hipMemsetAsync(c->rstate.p, 0, B * 4, s));
        m.rstate = (uint32_t *)c->rstate.p;
        m.rsave = (uint8_t *)c->rsave.p;
        m.rstride = stride;
        m.unfinished = (uint32_t *)c->unfinished.p;
        m.budget = c->budget_ticks;
        m.no_mid = getenv("BCHK_POLAR_NO_MID") ? 1 : 0;
        for (uint64_t launch = 0;; ++launch) {
            PHIP_TRY(hipMemsetAsync(c->unfinished.p, 0, 4, s));
            PHIP_TRY(launch_polar_mixed(m, grid, c->lds, s));
            uint32_t left = 0;
            PHIP_TRY(hipMemcpyAsync(&left, c->unfinished.p, 4, hipMemcpyDeviceToHost, s));
            PHIP_TRY(hipStreamSynchronize(s));
            c->launches_last = launch + 1;
            if (left == 0) break;
        }
        return 0;
    }
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
        // the transform, innermost layer first (MixedKernelEncoder.cpp:159-170): each block of
        // `next` symbols, viewed as l rows of `stride`, becomes (rows) x K
        std::vector<uint8_t> t(c->U);
        for (int L = c->n - 1, stride = 1; L >= 0; --L) {
            const int l = c->ksize[L], next = stride * l;
            const uint64_t *kr = &c->krows[(size_t)L * kPolarMaxKernel];
            for (int b0 = 0; b0 < c->U; b0 += next)
                for (int i = 0; i < l; ++i)
                    for (int s2 = 0; s2 < stride; ++s2) {
                        uint8_t acc = 0;
                        for (int j = 0; j < l; ++j) acc ^= (uint8_t)(u[b0 + j * stride + s2] & ((kr[j] >> i) & 1ull));
                        t[b0 + i * stride + s2] = acc;
                    }
            u.swap(t);
            stride = next;
        }
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
