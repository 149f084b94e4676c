// bchk_host.cpp -- host runtime of libbchk.so: code construction, device tables, kernel
// dispatch and the batched Monte-Carlo sweep behind the C ABI in include/bchk.h.
//
// Reference behaviour it reproduces (paths relative to the reference repo root):
//   GF(2^m) tables and g(x)       src/main.cpp:59-93, src/bchCoder.cpp:25-226
//   input stream / channel        src/bchCoder.cpp:19-22, 228-250 (std::default_random_engine)
//   FER sweep fun()               src/dataForPlot.cpp:16-116
// All decoding runs on the GPU; there is no CPU decode path in this library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <chrono>
#include <sstream>
#include <string>
#include <vector>

#include "bchk.h"
#include "bchk_device.h"
#include "bchk_launch.h"
#include "bchk_stream.h"


using namespace bchk;

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(BCHK_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),      \
                        __FILE__, __LINE__);                                            \
    } while (0)

const unsigned kPrim[16] = {3, 7, 11, 19, 37, 67, 137, 285, 529, 1033,
                            2053, 4179, 8219, 17475, 32771, 69643};  // main.cpp:14-15

struct Field {
    int m = 0, n = 0;
    std::vector<unsigned> alog;  // alpha^i
    std::vector<int> log;        // log(v), log(0) = -1
    unsigned mul(unsigned a, unsigned b) const {
        if (!a || !b) return 0;
        int s = log[a] + log[b];
        return alog[s >= n ? s - n : s];
    }
};

Field make_field(int m) {
    Field f;
    f.m = m;
    f.n = (1 << m) - 1;
    f.alog.resize(f.n);
    f.log.assign(f.n + 1, -1);
    f.alog[0] = 1;
    for (int i = 1; i < f.n; ++i) {
        unsigned v = f.alog[i - 1] << 1;
        if (v >> m) v ^= kPrim[m - 1];
        f.alog[i] = v;
    }
    for (int i = 0; i < f.n; ++i) f.log[f.alog[i]] = i;
    return f;
}

// g(x) = product of the distinct minimal polynomials of alpha^1 .. alpha^(2t-1)
// (= their lcm, main.cpp:84-92), binary coefficients low -> high.
std::vector<uint8_t> make_generator(const Field &f, int t) {
    std::vector<uint8_t> g{1};
    std::vector<bool> done(f.n, false);
    for (int i = 1; i < 2 * t; ++i) {
        const int i0 = i % f.n;
        if (done[i0]) continue;
        std::vector<unsigned> mp{1};
        int e = i0;
        do {
            done[e] = true;
            const unsigned root = f.alog[e];
            std::vector<unsigned> nx(mp.size() + 1, 0);
            for (size_t d = 0; d < mp.size(); ++d) {
                nx[d + 1] ^= mp[d];
                nx[d] ^= f.mul(mp[d], root);
            }
            mp.swap(nx);
            e = (2 * e) % f.n;
        } while (e != i0);
        std::vector<uint8_t> prod(g.size() + mp.size() - 1, 0);
        for (size_t a = 0; a < g.size(); ++a)
            if (g[a])
                for (size_t b = 0; b < mp.size(); ++b) prod[a + b] ^= (uint8_t)(mp[b] & 1u);
        g.swap(prod);
    }
    return g;
}

// Device table blob (see TableDesc in bchk_device.h). The syndrome columns are laid out
// with the word count of the kernel instantiation (tmax, the TMAX bucket >= t): kernels
// index them with a compile-time stride.
std::vector<uint8_t> make_tables(const Field &f, int t, TableDesc *td, int tmax = 0) {
    const int n = f.n, m = f.m;
    const int W = (std::max(std::max(t, tmax), 1) + 3) / 4;
    const int EW = (m + 1) & ~1;
    auto align16 = [](size_t v) { return (v + 15) & ~size_t(15); };
    size_t off = 0;
    td->off_exp = (uint32_t)off;
    off = align16(off + (m >= 7 ? 4 : 2) * size_t(n));  // m >= 7: zeros past 2n-1 (gf_exp2)
    td->off_log = (uint32_t)off;
    off = align16(off + 2 * (size_t(1) << m));
    td->off_col = (uint32_t)off;
    off = align16(off + 4 * size_t(n) * W);
    td->off_chien = (uint32_t)off;
    if (m <= 6) off = align16(off + 8 * size_t(t + 1) * 2 * size_t(m) * 8);
    td->bytes = (uint32_t)off;
    td->W = W;
    td->EW = EW;
    std::vector<uint8_t> blob(off, 0);
    uint8_t *ex = blob.data() + td->off_exp;
    for (int i = 0; i < 2 * n - 1; ++i) ex[i] = (uint8_t)f.alog[i % n];  // ex[2n-1] = 0
    uint16_t *lg = reinterpret_cast<uint16_t *>(blob.data() + td->off_log);
    lg[0] = (uint16_t)(2 * n - 1);
    for (int v = 1; v <= n; ++v) lg[v] = (uint16_t)f.log[v];
    uint32_t *col = reinterpret_cast<uint32_t *>(blob.data() + td->off_col);
    for (int p = 0; p < n; ++p)
        for (int j = 0; j < t; ++j) {
            const unsigned s = f.alog[(size_t(2 * j + 1) * p) % n];
            col[p * W + j / 4] |= s << (8 * (j % 4));
        }
    if (m <= 6) {
        // [j][half][b][8]: half 0 holds lo * alpha^(jk), half 1 holds (8 hi) * alpha^(jk)
        uint64_t *ch = reinterpret_cast<uint64_t *>(blob.data() + td->off_chien);
        for (int j = 0; j <= t; ++j)
            for (int half = 0; half < 2; ++half)
                for (unsigned x = 0; x < 8; ++x) {
                    const unsigned v = half ? (x << 3) : x;
                    if (v >= (1u << m)) continue;
                    for (int k = 0; k < n; ++k) {
                        const unsigned val = f.mul(v, f.alog[(size_t(j) * k) % n]);
                        for (int b = 0; b < m; ++b)
                            if ((val >> b) & 1u)
                                ch[((size_t(j) * 2 + half) * m + b) * 8 + x] |= 1ull << k;
                    }
                }
    }
    return blob;
}

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, bytes) != hipSuccess) return fail(BCHK_ENOMEM, "hipMalloc(%zu) failed", bytes);
        cap = bytes;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// ------------------------------------------------------ syndrome decoding table
// Host build of the table described in bchk_syndtab.h. Every error pattern of weight 1..t
// that contains position 0 is enumerated (incremental odd-syndrome XOR over the position
// columns); its normalised key maps to the pattern shifted by the normalising shift (the
// same entry for every member of a shift orbit: inserted once). Keys in the raw region
// (all coprime syndromes zero, no normalisation) are inserted for all n cyclic shifts.
typedef SyndKey (*SyndKeyFn)(const uint32_t *, int, const uint16_t *);
constexpr int kTabTmax = 8;  // t <= 7 whenever syndtab_feasible(m, t)

SyndKeyFn synd_key_fn(int m) {
    switch (m) {
        case 2: return &synd_key<2, kTabTmax>;
        case 3: return &synd_key<3, kTabTmax>;
        case 4: return &synd_key<4, kTabTmax>;
        case 5: return &synd_key<5, kTabTmax>;
        case 6: return &synd_key<6, kTabTmax>;
        default: return nullptr;
    }
}

struct HostTable {
    int m = 0, t = 0;
    uint32_t bbits = 0, max_probe = 0, kbits = 0, tbits = 0;
    size_t keys = 0;
    std::vector<uint64_t> slots;  // [nbuckets][kTabSlots]
};

// Packed position fields (m bits each, ascending, unused fields all ones) of the pattern
// 2^kf (e + s): e shifted by s, then every position multiplied by 2^kf mod n.
uint64_t pack_leader(uint64_t e, int s, int kf, int m, int n, int t) {
    std::vector<int> pos;
    for (int p = 0; p < n; ++p)
        if ((e >> p) & 1ull) {
            const int p1 = (p + s) % n;
            pos.push_back(kf ? (((p1 << kf) | (p1 >> (m - kf))) & n) : p1);
        }
    std::sort(pos.begin(), pos.end());
    uint64_t v = 0;
    for (int f = t - 1; f >= 0; --f) v = (v << m) | (uint64_t)(f < (int)pos.size() ? pos[f] : n);
    return v;
}

// Insert (key, positions) unless the key is present (then they must agree: the coset
// leader is unique). Returns 0, 1 on a disagreement (a logic error), 2 when the key would
// sit 2^kTabDistBits buckets or more past its home (the caller grows the table).
int tab_insert(HostTable &h, uint64_t key, uint64_t fields) {
    const SyndTable T{nullptr, h.bbits, 0, h.kbits, h.tbits};
    const TabHome H = tab_home(key, T);
    const uint64_t tm = (1ull << h.tbits) - 1ull;
    const uint32_t bm = (1u << h.bbits) - 1u;
    uint32_t b = H.b;
    for (uint32_t p = 0; p < (1u << kTabDistBits); ++p, b = (b + 1u) & bm) {
        const uint64_t tag = H.tag | p;
        uint64_t *bk = h.slots.data() + (size_t)b * kTabSlots;
        for (int j = 0; j < kTabSlots; ++j) {
            if ((bk[j] & tm) == tag) return (bk[j] >> h.tbits) == fields ? 0 : 1;
            if (bk[j] == 0) {
                bk[j] = (fields << h.tbits) | tag;
                h.max_probe = std::max(h.max_probe, p + 1);
                ++h.keys;
                return 0;
            }
        }
    }
    return 2;
}

int build_table(const Field &f, int t, HostTable &h) {
    const int m = f.m, n = f.n;
    h.m = m;
    h.t = t;
    TableDesc td{};
    const std::vector<uint8_t> blob = make_tables(f, t, &td);
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(blob.data() + td.off_log);
    std::vector<uint64_t> col(n, 0);  // packed odd-syndrome column of each position
    for (int p = 0; p < n; ++p)
        for (int q = 0; q < t; ++q)
            col[p] |= uint64_t(f.alog[(size_t(2 * q + 1) * p) % n]) << (8 * q);
    const SyndKeyFn keyf = synd_key_fn(m);
    // raw-region keys: every coprime syndrome zero (the key's region is the last one)
    int K = 0;
    for (int q = 0; q < t; ++q) K += f_coprime(q, n) ? 1 : 0;
    // table size: at most half of the slots used (orbits ~ C(n, <=t) / (n m), plus raw
    // keys); BCHK_TAB_MAXLOAD (experiments) sets another bound
    double est = 0.0, c = 1.0;
    for (int w = 1; w <= t; ++w) {
        c = c * (n - w + 1) / w;
        est += c;
    }
    est = est / ((double)n * m) * 1.05 + 64;
    double maxload = 0.5;
    if (const char *ml = getenv("BCHK_TAB_MAXLOAD")) maxload = std::min(0.95, std::max(0.05, atof(ml)));
    h.bbits = 1;
    while ((double)(kTabSlots << h.bbits) * maxload < est) ++h.bbits;
    h.kbits = (uint32_t)tab_kbits(m, t);
    h.bbits = std::min(h.bbits, h.kbits);  // tiny key spaces: one bucket per key
    while (!tab_fits(m, t, (int)h.bbits) && (int)h.bbits < (int)h.kbits) ++h.bbits;  // a 32-bit tag
    // enumerate in parallel (threads own second positions), insert serially
    const int hw = (int)std::thread::hardware_concurrency();
    const int nth = std::max(1, std::min(16, hw > 0 ? hw : 1));
    std::vector<std::vector<uint64_t>> found(nth);  // (key, mask) pairs
    auto emit = [&](std::vector<uint64_t> &out, uint64_t S, uint64_t pat) {
        const uint32_t Sw[2] = {(uint32_t)S, (uint32_t)(S >> 32)};
        const SyndKey k = keyf(Sw, t, lg);
        if ((k.key >> tab_vbits(m, t)) < (uint64_t)K) {  // a normalised region
            out.push_back(k.key);
            out.push_back(pack_leader(pat, k.s, k.kf, m, n, t));
            return;
        }
        for (int u = 0; u < n; ++u) {  // raw region: each shift is its own key
            uint64_t Su = 0;
            for (int q = 0; q < t; ++q) {
                const unsigned v = (S >> (8 * q)) & 0xFFu;
                const unsigned w = v ? f.alog[(f.log[v] + size_t(2 * q + 1) * u) % n] : 0u;
                Su |= uint64_t(w) << (8 * q);
            }
            const uint32_t Swu[2] = {(uint32_t)Su, (uint32_t)(Su >> 32)};
            const SyndKey ku = keyf(Swu, t, lg);
            out.push_back(ku.key);
            out.push_back(pack_leader(pat, u + ku.s, ku.kf, m, n, t));  // ku.s == 0
        }
    };
    struct Rec {
        const std::vector<uint64_t> &col;
        int n;
        const decltype(emit) &put;
        void go(std::vector<uint64_t> &out, int from, int left, uint64_t S, uint64_t pat) const {
            for (int p = from; p < n; ++p) {
                const uint64_t Sp = S ^ col[p], pp = pat | (1ull << p);
                put(out, Sp, pp);
                if (left > 1) go(out, p + 1, left - 1, Sp, pp);
            }
        }
    };
    const Rec rec{col, n, emit};
    std::vector<std::thread> th;
    for (int w = 0; w < nth; ++w)
        th.emplace_back([&, w] {
            if (w == 0) emit(found[0], col[0], 1ull);  // weight 1: {0}
            for (int p1 = 1 + w; p1 < n && t >= 2; p1 += nth) {
                const uint64_t S1 = col[0] ^ col[p1], pat = 1ull | (1ull << p1);
                emit(found[w], S1, pat);
                if (t > 2) rec.go(found[w], p1 + 1, t - 2, S1, pat);
            }
        });
    for (auto &x : th) x.join();
    // insert; a key too far from its home grows the table (a larger bbits also leaves fewer
    // quotient bits, so the slot always fits: syndtab_feasible checked bbits = 1)
    for (;; ++h.bbits) {
        if (h.bbits > h.kbits || !tab_fits(m, t, (int)h.bbits))
            return fail(BCHK_EINVAL, "syndrome table: no layout (m=%d t=%d)", m, t);
        h.tbits = (uint32_t)tab_tbits(m, t, (int)h.bbits);
        h.slots.assign(size_t(kTabSlots) << h.bbits, 0);
        h.keys = 0;
        h.max_probe = 0;
        int rc = 0;
        for (auto &v : found) {
            for (size_t i = 0; i < v.size() && !rc; i += 2) rc = tab_insert(h, v[i], v[i + 1]);
            if (rc) break;
        }
        if (rc == 1) return fail(BCHK_EINVAL, "syndrome table: two leaders for one key (m=%d t=%d)", m, t);
        if (rc == 0) break;
    }
    for (auto &v : found) std::vector<uint64_t>().swap(v);
    return 0;
}

// Process-wide cache: one host table per (m, t), one device copy per (device, m, t).
struct TableCache {
    std::mutex mu;
    std::vector<HostTable *> host;
    struct Dev { int device, m, t; uint64_t *slots; };
    std::vector<Dev> dev;
};
TableCache &table_cache() {
    static TableCache *c = new TableCache();  // never destroyed (outlives static dtors)
    return *c;
}

int host_table(const Field &f, int t, const HostTable **out) {
    TableCache &tc = table_cache();
    std::lock_guard<std::mutex> g(tc.mu);
    for (auto *h : tc.host)
        if (h->m == f.m && h->t == t) {
            *out = h;
            return 0;
        }
    auto *h = new HostTable();
    if (int rc = build_table(f, t, *h)) {
        delete h;
        return rc;
    }
    tc.host.push_back(h);
    *out = h;
    return 0;
}

}  // namespace

struct bchk_ctx {
    int m = 0, t = 0, n = 0, k = 0, J = -1, device = 0;
    double decoder_snr_db = 0.5, s2 = 0.0;
    Field field;
    std::vector<uint8_t> g;
    std::vector<uint8_t> tables_host;
    TableDesc td{};
    KernelSet ks{};
    FastFn fast = nullptr;
    bool use_fast = true;
    size_t lds_fast = 0, lds_coop = 0;
    int grid_coop = 0, grid_coop_tab = 0;
    int32_t long_rec = 2;      // cooperative kernel (m >= 7): candidate records per ring slot
    uint64_t last_coop_stats[2] = {0, 0};
    uint32_t chunk_limit = 8;  // exact steps before a hand-off (measured best over 4-6 dB, J = 15 / inf)
    DevBuf diag;
    // One decode pipeline per sub-batch: its work queues, control words (one 128-B line
    // each) and streams. A call splits a large batch over npipes pipelines, each on its own
    // stream, with every fast kernel after the one before it: one sub-batch's fast kernel
    // (HBM-bound, the whole chip) runs while the sub-batches before it drain their
    // latency-bound search / tail kernels.
    struct Pipe {
        DevBuf queue, heavy, ctrl, l1q, l1rec;  // l1q / l1rec: first pass -> analytic tail
        DevBuf pre;                             // m >= 7: the lane pre-pass's finished rows
        DevBuf jobctl, jobs;                    // m >= 7: cooperative-kernel jobs (help)
        hipStream_t s = nullptr, aux = nullptr;  // s unused for pipe 0 (the caller's stream)
        hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_done = nullptr, ev_fast = nullptr;
    };
    std::vector<Pipe> pipes;
    int npipes = 1;              // BCHK_PIPES (sub-batch pipelines; 1 = off)
    int last_pipes = 0;          // pipelines the last call used
    size_t pipe_min = 1u << 17;  // codewords per sub-batch at least
    hipEvent_t ev_start = nullptr;
    uint8_t *d_tables = nullptr;
    hipStream_t stream = nullptr;
    size_t lds = 0, lds_alg = 0, lds_tail = 0;
    size_t lds_tab = 0;  // the first pass with the syndrome table: no Chien rows in LDS
    int grid = 0, grid_tab = 0, grid_tail = 0, grid_tail_tab = 0;
    uint64_t max_decodes = 0;
    DevBuf y, res, l0, st, words, synd, ok;
    bool coop_concurrent = false;  // BCHK_COOP_CONCURRENT=1: measured neutral at 5 dB
    bool analytic = true;          // analytic tail of heavy codewords (BCHK_NO_ANALYTIC=1: off)
    uint64_t last_tail = 0;        // codewords the last call handed to the tail kernel
    uint64_t last_tail_stats[6] = {0, 0, 0, 0, 0, 0};
    bool tail_diag_on = false;     // BCHK_TAIL_DIAG=1: per-codeword tail timing records
    bool tail_concurrent = false;  // BCHK_TAIL_CONCURRENT=1: the tail kernel beside the first pass
    // BCHK_TAIL_INLINE=1: the first pass IS the analytic-tail kernel instance -- a codeword
    // past the chunk limit is finished by the same wave at once, no second kernel
    bool tail_inline = false;
    // idle waves of the tail kernel help a sibling's split codeword decode its exact chunks
    // (BCHK_AN_HELP=0: off; results identical either way)
    bool an_help = true;
    // fast ring kernel: waves per workgroup (BCHK_FAST_RING_WAVES, 0 = 16) and experiment
    // mode (BCHK_FAST_MODE)
    uint32_t fast_waves = 0, fast_mode = 0;
    uint32_t heavy_t = 0;  // BCHK_HEAVY_T (experiments; 0: the kernel's kHeavyT)
    uint32_t heavy_tmax = 0;  // BCHK_HEAVY_TMAX (experiments; 0: no upper limit)
    // m >= 7: the lane-per-codeword pre-pass of the first kernel (BCHK_LANE_PRE=0: off)
    FastFn lane = nullptr;
    bool lane_pre = true;
    // m >= 7: idle cooperative workgroups help the running long codewords (BCHK_LONG_HELP=0: off)
    bool long_help = true;
    uint32_t long_help_max = 0, long_share_min = 0;
    uint32_t long_epoch = 0;  // cooperative launches with jobs (tag generations)  // BCHK_LONG_HELP_MAX / BCHK_LONG_SHARE_MIN (0: defaults)
    DevBuf syn8;  // its hard-decision syndrome table (SearchParams::syn8)
    DevBuf gfmul; // m >= 7: GF(2^m) products and inverses (SearchParams::gfmul)
    int tail_conc_blocks = 64;     // blocks of the concurrent tail kernel (BCHK_TAIL_BLOCKS)
    bool heavy_first = true;       // fast path queues likely heavy codewords first (BCHK_HEAVY_FIRST)
    // hybrid tail: a first-pass hand-off whose loop bound is below this goes to a cooperative
    // kernel running beside the tail kernel instead (0: every hand-off to the tail kernel)
    uint64_t tail_min_bound = 0;
    DevBuf tdiag;
    DevBuf cnt;  // fused FER/op counters: kCntSlots partial slots
    DevBuf fault;  // sticky fault word (SearchParams::fault), checked by bchk_sync
    DevBuf gtx, gy, gres, gst, gcnt, gflags;  // bchk_sweep_device's batch buffers
    bool profile = false;
    // syndrome decoding table (bchk_syndtab.h): built on first use, shared across contexts
    bool use_table = true;
    SyndTable tab{};
    struct Ev {  // [fast, exact, coop, tail] x [start, end] of one pipeline of one call
        hipEvent_t e[8];
        bool first;  // the call's first pipeline
    };
    std::vector<Ev> events;
    double prof_ms[4] = {0.0, 0.0, 0.0, 0.0};
    uint64_t prof_launches = 0;
};

namespace {

int sigma_s2(int k, int n, double snr_db, double *sd) {
    // KanekoKernelProcessor ctor, src/KanekoKernelProcessor.cpp:20 (k, n are long there)
    const long K = k, Nn = n;
    *sd = sqrt(1 / (pow(10, snr_db / 10) * 2 * K / Nn));
    return 0;
}

// control block: fast-path queue tail (line 0), 8 per-XCD heads (lines 1-8), heavy front
// tail / head (lines 9, 10), back tail / head (11, 12), 8 per-XCD counts of codewords the
// exact kernel has finished (13-20), diagnostic record count (21), the first pass's
// hand-offs to the analytic tail kernel (22), its 8 per-XCD heads (23-30) and finished
// counts (31-38), its outcome counters (39), an always-empty queue tail and head (40, 41),
// the hybrid tail's back-queue tail and head (42, 43), the fast path's front / back queue
// counts (44, 45); zeroed by one memset per decode call
constexpr size_t kCtrlBytes = 46 * 128;
constexpr int kHeavyTail = 32 * 9, kHeavyHead = 32 * 10, kHeavyTail2 = 32 * 11,
              kHeavyHead2 = 32 * 12, kExactDone = 32 * 13, kL1Tail = 32 * 22, kTailHeads = 32 * 23,
              kTailDone = 32 * 31, kTailStats = 32 * 39, kNoneTail = 32 * 40, kNoneHead = 32 * 41,
              kL1Back = 32 * 42, kL1BackHead = 32 * 43, kQFront = 32 * 44, kQBack = 32 * 45,
              kCoopStats = kTailStats + 8;  // line 39, words 8-9: cooperative-kernel counters
#ifdef BCHK_DIAG
constexpr int kDiagCount = 32 * 21;
#endif
// a codeword handed to the cooperative kernel with a loop bound >= this goes to the front
// queue (2^12 - 1: T >= 12 patterns left)
constexpr uint64_t kHeavyBig = 4095;

int ensure_heavy(bchk_ctx::Pipe &P, size_t B, hipStream_t s) {
    if (B <= P.heavy.cap / sizeof(uint32_t)) return 0;
    int rc = P.heavy.ensure(B * sizeof(uint32_t));
    if (rc) return rc;
    // empty slots (consumers restore them after every read); ordered before the pipeline's
    // kernels on its stream (a null-stream memset is not, for non-blocking streams)
    HIP_TRY(hipMemsetAsync(P.heavy.p, 0xFF, P.heavy.cap, s));
    return 0;
}

int ensure_pipes(bchk_ctx *c, int K) {
    if (!c->ev_start) HIP_TRY(hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming));
    while ((int)c->pipes.size() < K) {
        c->pipes.emplace_back();
        bchk_ctx::Pipe &P = c->pipes.back();
        if (c->pipes.size() > 1) HIP_TRY(hipStreamCreateWithFlags(&P.s, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&P.aux, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&P.ev_fork, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&P.ev_join, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&P.ev_done, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&P.ev_fast, hipEventDisableTiming));
    }
    return 0;
}

void release_pipes(bchk_ctx *c) {
    for (auto &P : c->pipes) {
        P.queue.release();
        P.heavy.release();
        P.ctrl.release();
        P.l1q.release();
        P.l1rec.release();
        P.pre.release();
        P.jobctl.release();
        P.jobs.release();
        if (P.s) (void)hipStreamDestroy(P.s);
        if (P.aux) (void)hipStreamDestroy(P.aux);
        for (hipEvent_t e : {P.ev_fork, P.ev_join, P.ev_done, P.ev_fast})
            if (e) (void)hipEventDestroy(e);
    }
    c->pipes.clear();
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    c->ev_start = nullptr;
}

// The context's device copy of the syndrome decoding table (first decode call; no-op when
// (m, t) has none or it is disabled).
int ensure_table(bchk_ctx *c) {
    if (!c->use_table || c->tab.slots || !syndtab_feasible(c->m, c->t)) return 0;
    const HostTable *h = nullptr;
    if (int rc = host_table(c->field, c->t, &h)) return rc;
    TableCache &tc = table_cache();
    std::lock_guard<std::mutex> g(tc.mu);
    uint64_t *d = nullptr;
    for (auto &e : tc.dev)
        if (e.device == c->device && e.m == c->m && e.t == c->t) d = e.slots;
    if (!d) {
        const size_t bytes = h->slots.size() * sizeof(uint64_t);
        if (hipMalloc(&d, bytes) != hipSuccess) return fail(BCHK_ENOMEM, "hipMalloc(%zu) for the syndrome table", bytes);
        if (hipMemcpy(d, h->slots.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            return fail(BCHK_EHIP, "syndrome table upload failed");
        }
        tc.dev.push_back({c->device, c->m, c->t, d});
    }
    c->tab.slots = d;
    c->tab.bbits = h->bbits;
    c->tab.max_probe = h->max_probe;
    c->tab.kbits = h->kbits;
    c->tab.tbits = h->tbits;
    return 0;
}

// One decode call: the fast kernel on the launch stream, then the exact wave kernel on it
// and -- concurrently, on the auxiliary stream -- the cooperative kernel, which takes heavy
// codewords as soon as the exact kernel hands them off (longest first). The launch stream
// waits for the cooperative kernel before the call's work counts as done.
int launch_pipe(bchk_ctx *c, bchk_ctx::Pipe &P, bool first, int variant, const double *d_y, size_t B,
                uint8_t *d_res, double *d_l0, bchk_stats *d_st, hipStream_t s, const uint8_t *d_tx,
                hipEvent_t wait_fast, hipEvent_t after_fast) {
    int rc;
    if ((rc = P.ctrl.ensure(kCtrlBytes)) || (rc = ensure_heavy(P, B, s))) return rc;
    const bool fast = c->fast && c->use_fast;
    if (fast && (rc = P.queue.ensure(B * sizeof(uint32_t)))) return rc;
    // the pre-pass decides rows without a stats record (the first kernel writes those)
    const bool lane = fast && c->lane && c->lane_pre && !d_st;
    if (lane && (rc = P.pre.ensure((B + 63) / 64 * sizeof(uint64_t)))) return rc;
    uint32_t *ctrl = (uint32_t *)P.ctrl.p;
    SearchParams p{};
    p.y = d_y;
    p.res = d_res;
    p.l0 = d_l0;
    p.st = d_st;
    p.tables = c->d_tables;
    p.td = c->td;
    p.s2 = c->s2;
    p.max_decodes = c->max_decodes;
    p.count = (uint32_t)B;
    p.t = c->t;
    p.J = c->J;
    p.variant = variant;
    p.fault = (uint32_t *)c->fault.p;
    p.gfmul = (const uint8_t *)c->gfmul.p;  // null for m <= 6
    if (d_tx) {  // fused counters (zeroed by launch_search at allocation, then by every reduction)
        p.tx = d_tx;
        p.cnt = (unsigned long long *)c->cnt.p;
    }
    p.heavy_queue = (uint32_t *)P.heavy.p;
    p.heavy_tail = c->chunk_limit ? ctrl + kHeavyTail : nullptr;
    p.heavy_tail2 = ctrl + kHeavyTail2;
    p.heavy_head = ctrl + kHeavyHead;
    p.heavy_head2 = ctrl + kHeavyHead2;
    p.exact_done = ctrl + kExactDone;
    p.exact_total = fast ? ctrl : nullptr;  // the fast path's queue length
    p.heavy_big = kHeavyBig;
    p.chunk_limit = c->chunk_limit;
    p.long_rec = c->long_rec;
    p.coop_stats = ctrl + kCoopStats;
    p.analytic = 0;
    if (c->use_table) p.tab = c->tab;
#ifdef BCHK_DIAG
    if (!c->diag.p) (void)c->diag.ensure(size_t(1) << 24);
    (void)hipMemsetAsync(c->diag.p, 0, size_t(1) << 24, s);
    p.diag = (unsigned long long *)c->diag.p;
    p.diag_count = ctrl + kDiagCount;
#endif
    // kernel variant and its persistent grid: the syndrome-table kernels when the table is on
    const bool tabk = p.tab.slots && c->ks.search_tab;
    const int grid = tabk ? c->grid_tab : c->grid;
    const int grid_coop = tabk ? c->grid_coop_tab : c->grid_coop;
    // analytic tail: the first pass hands its heavy codewords to the tail kernel (queue
    // l1q), which finishes most of them and hands the rest to the cooperative kernel
    // (n <= 31 without a pattern cap below n: every position is a flip position, and the
    // analytic tail lists the improving codewords by an ordered-statistics search, an_osd)
    const bool tail_any = c->analytic && c->ks.tail && p.heavy_tail && variant == BCHK_VARIANT_ANSWER;
    const bool inl = tail_any && c->tail_inline && !c->tail_diag_on;  // the first pass finishes its tails
    const bool tail = tail_any && !inl;
    if (tail && (rc = P.l1rec.ensure(B * sizeof(TailRec)))) return rc;
    if (tail && B > P.l1q.cap / sizeof(uint32_t)) {
        if ((rc = P.l1q.ensure(B * sizeof(uint32_t)))) return rc;
        HIP_TRY(hipMemsetAsync(P.l1q.p, 0xFF, P.l1q.cap, s));  // empty slots (consumers restore them)
    }
    // the tail kernel runs on the auxiliary stream, concurrently with the first pass
    const bool tconc = tail && c->tail_concurrent;
    // hybrid: the short hand-offs to a cooperative kernel on s while the tail kernel (aux)
    // takes the long ones; the tail's own hand-offs to a second cooperative kernel on aux
    const bool hybrid = tail && !tconc && c->tail_min_bound > 0;
    const bool conc = c->coop_concurrent && p.heavy_tail && !tail;
    hipStream_t cs = conc ? P.aux : s;  // the cooperative kernel's stream
    bchk_ctx::Ev ev{};
    if (c->profile) {
        for (auto &e : ev.e) HIP_TRY(hipEventCreate(&e));
        ev.first = first;
        HIP_TRY(hipEventRecord(ev.e[0], s));
    }
    HIP_TRY(hipMemsetAsync(ctrl, 0, kCtrlBytes, s));
    if (wait_fast) HIP_TRY(hipStreamWaitEvent(s, wait_fast, 0));
    if (fast) {
        SearchParams f = p;
#ifdef BCHK_DIAG
        f.diag = p.diag + (size_t(1) << 20);  // fast-kernel stamps: second half of the buffer
#endif
        f.qtail = ctrl;
        f.queue_out = (uint32_t *)P.queue.p;
        if (c->heavy_first && c->m <= 6) {  // the lane fast kernel (m >= 7: the first kernel)
            f.qfront = ctrl + kQFront;
            f.qback = ctrl + kQBack;
        }
        if (c->m <= 6) {
            f.fast_waves = c->fast_waves;
            f.fast_mode = c->fast_mode;
            f.heavy_t = c->heavy_t;
            f.heavy_tmax = c->heavy_tmax;
            f.syn8 = (const uint32_t *)c->syn8.p;  // null unless built
        }
        if (lane) {
            f.pre_mask = (uint64_t *)P.pre.p;
            f.syn8 = (const uint32_t *)c->syn8.p;
            HIP_TRY(c->lane(f, 0, s));
        }
        HIP_TRY(c->fast(f, c->lds_fast, s));
    }
    if (after_fast) HIP_TRY(hipEventRecord(after_fast, s));
    if (c->profile) HIP_TRY(hipEventRecord(ev.e[1], s));
    if (conc || tconc) {
        HIP_TRY(hipEventRecord(P.ev_fork, s));
        HIP_TRY(hipStreamWaitEvent(P.aux, P.ev_fork, 0));
    }
    if (c->profile) HIP_TRY(hipEventRecord(ev.e[2], s));
    {
        SearchParams q = p;
        if (tail) {  // hand-offs (all to the front) into the tail kernel's queue
            q.heavy_queue = (uint32_t *)P.l1q.p;
            q.heavy_tail = ctrl + kL1Tail;
            q.heavy_tail2 = ctrl + kL1Back;  // hybrid: loop bounds below heavy_big
            q.heavy_big = hybrid ? c->tail_min_bound : 0;
            q.tail_rec = (TailRec *)P.l1rec.p;
        }
        if (c->tail_diag_on && !inl) {  // experiment builds (BCHK_AN_PROF): first-pass phase cycles
            if (!c->tdiag.p && (rc = c->tdiag.ensure(size_t(1) << 22))) return rc;
            HIP_TRY(hipMemsetAsync(c->tdiag.p, 0, c->tdiag.cap, s));
            q.tail_diag = (unsigned long long *)c->tdiag.p;
            q.tail_diag_cap = (uint32_t)(c->tdiag.cap / 128);
#ifdef BCHK_FP_TRACE
            q.tail_diag_count = ctrl + kTailStats + 16;  // first-pass timeline records first
#endif
        }
        if (inl) {  // the analytic tail inside the first pass; failures to the cooperative kernel
            q.analytic = 1;
            q.tail_stats = ctrl + kTailStats;
        }
        const int igrid = tabk ? c->grid_tail_tab : c->grid_tail;
        if (fast) {
            q.queue = (const uint32_t *)P.queue.p;
            q.qcount = ctrl;
            q.heads = ctrl + 32;
            if (c->heavy_first && c->m <= 6) q.qfront_n = ctrl + kQFront;
            // every resident wave may take work; waves beyond the queue length exit at once
            HIP_TRY(inl ? launch_tail(c->ks, q, igrid, c->lds_tail, s)
                        : launch_search(c->ks, q, grid, tabk ? c->lds_tab : c->lds, s));
        } else {
            const int need = (int)((B + kWavesPerBlock - 1) / kWavesPerBlock);
            HIP_TRY(inl ? launch_tail(c->ks, q, std::max(1, std::min(igrid, need)), c->lds_tail, s)
                        : launch_search(c->ks, q, std::max(1, std::min(grid, need)), tabk ? c->lds_tab : c->lds, s));
        }
    }
    if (c->profile) HIP_TRY(hipEventRecord(ev.e[3], s));
    SearchParams pc = p;  // the cooperative kernel's view of its producer
    hipStream_t ts = (tconc || hybrid) ? P.aux : s;  // the tail kernel's stream
    if (hybrid) {
        HIP_TRY(hipEventRecord(P.ev_fork, s));
        HIP_TRY(hipStreamWaitEvent(P.aux, P.ev_fork, 0));
    }
    if (c->profile) HIP_TRY(hipEventRecord(ev.e[6], ts));
    if (tail) {
        SearchParams q = p;
        q.queue = (const uint32_t *)P.l1q.p;
        q.qcount = ctrl + kL1Tail;
        q.heads = ctrl + kTailHeads;
        q.exact_done = ctrl + kTailDone;
        q.analytic = 1;
        q.tail_stats = ctrl + kTailStats;
        q.tail_rec = (TailRec *)P.l1rec.p;
        q.an_help = (c->an_help && !tconc) ? 1 : 0;
        if (tconc) {  // take the first pass's hand-offs as they come, with their state
            q.in_queue = (uint32_t *)P.l1q.p;
            q.in_tail = ctrl + kL1Tail;
            q.in_head = ctrl + kTailHeads;
            q.in_done = ctrl + kExactDone;
            q.in_total = fast ? ctrl : nullptr;
        }
        if (c->tail_diag_on) {
            if (!c->tdiag.p && (rc = c->tdiag.ensure(size_t(1) << 22))) return rc;
            if (inl)  // (otherwise zeroed before the first pass)
                HIP_TRY(hipMemsetAsync(c->tdiag.p, 0, c->tdiag.cap, s));
            q.tail_diag = (unsigned long long *)c->tdiag.p;
            q.tail_diag_count = ctrl + kTailStats + 16;
            q.tail_diag_cap = (uint32_t)(c->tdiag.cap / 128);  // second half: bchk_tail_prof_read
        }
        int tgrid = tabk ? c->grid_tail_tab : c->grid_tail;
        if (tconc || hybrid) tgrid = std::min(tgrid, c->tail_conc_blocks);  // CUs for the others
        HIP_TRY(launch_tail(c->ks, q, tgrid, c->lds_tail, ts));
        pc.exact_done = ctrl + kTailDone;
        pc.exact_total = ctrl + kL1Tail;
    }
    if (c->profile) HIP_TRY(hipEventRecord(ev.e[7], ts));
    if (hybrid) {
        SearchParams ph = p;  // the first pass's short hand-offs: the back of l1q
        ph.heavy_queue = (uint32_t *)P.l1q.p;
        ph.heavy_tail = ctrl + kNoneTail;
        ph.heavy_head = ctrl + kNoneHead;
        ph.heavy_tail2 = ctrl + kL1Back;
        ph.heavy_head2 = ctrl + kL1BackHead;
        if (c->profile) HIP_TRY(hipEventRecord(ev.e[4], s));
        HIP_TRY(launch_coop(c->ks, ph, grid_coop, c->lds_coop, s));
        if (c->profile) HIP_TRY(hipEventRecord(ev.e[5], s));
        // the tail kernel's hand-offs (rare) after it on aux, then s waits for aux
        HIP_TRY(launch_coop(c->ks, pc, grid_coop, c->lds_coop, P.aux));
        HIP_TRY(hipEventRecord(P.ev_join, P.aux));
        HIP_TRY(hipStreamWaitEvent(s, P.ev_join, 0));
        if (c->profile) c->events.push_back(ev);
        return 0;
    }
    if (tconc) {  // the cooperative kernel (stream s) follows both
        HIP_TRY(hipEventRecord(P.ev_join, P.aux));
        HIP_TRY(hipStreamWaitEvent(s, P.ev_join, 0));
    }
    if (p.heavy_tail) {
        if (c->m >= 7 && c->long_help && c->ks.long_job_bytes) {  // jobs of the cooperative workgroups
            // A chunk record is taken as delivered when its tag equals (generation << 32 |
            // chunk + 1), the generation built from this context's 20-bit launch epoch. Tags
            // must therefore never hold a value from another context (memory hipMalloc hands
            // back) or from the launch 2^20 epochs ago: the jobs memory is zeroed whenever it
            // is (re)allocated and whenever the epoch's low 20 bits wrap. A zero tag matches
            // no chunk (chunk + 1 >= 1).
            const size_t jobs_cap_before = P.jobs.cap;  // ensure() only grows it
            if ((rc = P.jobctl.ensure((size_t)(grid_coop + 1) * 128)) ||
                (rc = P.jobs.ensure((size_t)grid_coop * c->ks.long_job_bytes)))
                return rc;
            HIP_TRY(hipMemsetAsync(P.jobctl.p, 0, (size_t)(grid_coop + 1) * 128, cs));
            const uint32_t epoch = ++c->long_epoch;
            if (P.jobs.cap != jobs_cap_before || (epoch & 0xFFFFFu) == 0u)
                HIP_TRY(hipMemsetAsync(P.jobs.p, 0, P.jobs.cap, cs));
            pc.long_jobctl = P.jobctl.p;
            pc.long_jobs = P.jobs.p;
            pc.long_help_max = c->long_help_max;
            pc.long_epoch = epoch;
            pc.long_share_min = c->long_share_min;
        }
        if (c->profile) HIP_TRY(hipEventRecord(ev.e[4], cs));
        HIP_TRY(launch_coop(c->ks, pc, grid_coop, c->lds_coop, cs));
        if (c->profile) HIP_TRY(hipEventRecord(ev.e[5], cs));
    } else if (c->profile) {
        HIP_TRY(hipEventRecord(ev.e[4], s));
        HIP_TRY(hipEventRecord(ev.e[5], s));
    }
    if (conc) {
        HIP_TRY(hipEventRecord(P.ev_join, cs));
        HIP_TRY(hipStreamWaitEvent(s, P.ev_join, 0));
    }
    if (c->profile) c->events.push_back(ev);
    return 0;
}

int launch_search(bchk_ctx *c, int variant, const double *d_y, size_t B, uint8_t *d_res,
                  double *d_l0, bchk_stats *d_st, hipStream_t s, const uint8_t *d_tx = nullptr) {
    if (B == 0) return 0;
    if (B > 0xFFFFFFFFull) return fail(BCHK_EINVAL, "batch too large");
    int rc;
    if ((rc = ensure_table(c))) return rc;
    int K = c->tail_diag_on ? 1 : std::max(1, c->npipes);
    K = (int)std::min<size_t>((size_t)K, std::max<size_t>(1, B / c->pipe_min));
    if ((rc = ensure_pipes(c, K))) return rc;
    if (d_tx && !c->cnt.p) {  // fused counters: zeroed before any pipeline starts
        if ((rc = c->cnt.ensure(size_t(kCntSlots) * kCntStride * 8))) return rc;
        HIP_TRY(hipMemsetAsync(c->cnt.p, 0, c->cnt.cap, s));
    }
    c->last_pipes = K;
    if (K == 1)
        return launch_pipe(c, c->pipes[0], true, variant, d_y, B, d_res, d_l0, d_st, s, d_tx, nullptr, nullptr);
    // sub-batches of whole 64-codeword chunks; pipe 0 on the caller's stream
    const size_t n = (size_t)c->n;
    const size_t chunk = ((B + K - 1) / K + 63) / 64 * 64;
    HIP_TRY(hipEventRecord(c->ev_start, s));
    hipEvent_t prev_fast = nullptr;
    for (int k = 0; k < K; ++k) {
        const size_t off = (size_t)k * chunk;
        if (off >= B) break;
        const size_t nb = std::min(chunk, B - off);
        bchk_ctx::Pipe &P = c->pipes[k];
        const hipStream_t ps = k ? P.s : s;
        if (k) HIP_TRY(hipStreamWaitEvent(ps, c->ev_start, 0));
        if ((rc = launch_pipe(c, P, k == 0, variant, d_y + off * n, nb, d_res + off * n, d_l0 ? d_l0 + off : nullptr,
                              d_st ? d_st + off : nullptr, ps, d_tx ? d_tx + off * n : nullptr, prev_fast,
                              k + 1 < K ? P.ev_fast : nullptr)))
            return rc;
        prev_fast = P.ev_fast;
        if (k) {
            HIP_TRY(hipEventRecord(P.ev_done, ps));
            HIP_TRY(hipStreamWaitEvent(s, P.ev_done, 0));
        }
    }
    return 0;
}

}  // namespace

namespace bchk {
void set_last_error(const char *msg) { g_err = msg; }  // for polar_host.cpp
}  // namespace bchk

extern "C" {

const char *bchk_last_error(void) { return g_err.c_str(); }
const char *bchk_version(void) { return "bchk 0.1 (gfx950)"; }

int bchk_create(int m, int t, int J, double decoder_snr_db, int device, bchk_ctx **out) {
    if (!out) return fail(BCHK_EINVAL, "out is NULL");
    *out = nullptr;
    if (m < 2 || m > kMaxM) return fail(BCHK_EINVAL, "m=%d unsupported (2..%d)", m, kMaxM);
    if (t <= 0 || t >= (1 << (m - 1)) || t > kMaxT)
        return fail(BCHK_EINVAL, "t=%d invalid for m=%d (1 <= t < 2^(m-1), t <= %d)", t, m, kMaxT);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(BCHK_ENODEV, "no HIP device visible (libbchk has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(BCHK_EINVAL, "device %d out of range", device);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(BCHK_ENODEV, "device %d is %s; libbchk is built for gfx950 only", device,
                    prop.gcnArchName);
    HIP_TRY(hipSetDevice(device));
    bchk_ctx *c = new bchk_ctx();
    c->m = m;
    c->t = t;
    c->J = J < 0 ? -1 : J;
    c->device = device;
    c->decoder_snr_db = decoder_snr_db;
    c->field = make_field(m);
    c->n = c->field.n;
    c->g = make_generator(c->field, t);
    c->k = c->n - (int)c->g.size() + 1;
    double sd0;
    sigma_s2(c->k, c->n, decoder_snr_db, &sd0);
    c->s2 = pow(sd0, 2);  // src/KanekoKernelProcessor.cpp:337 `pow(sd, 2)`
    if (!select_kernels(m, t, &c->ks)) {
        delete c;
        return fail(BCHK_EINVAL, "no kernel instantiated for m=%d t=%d", m, t);
    }
    c->tables_host = make_tables(c->field, t, &c->td, c->ks.tmax);
    int rc = 0;
    if (hipMalloc(&c->d_tables, c->td.bytes) != hipSuccess ||
        hipMemcpy(c->d_tables, c->tables_host.data(), c->td.bytes, hipMemcpyHostToDevice) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        ensure_pipes(c, 1) != 0 || c->fault.ensure(128) != 0 ||
        hipMemset(c->fault.p, 0, 128) != hipSuccess) {
        bchk_destroy(c);
        return fail(BCHK_EHIP, "device setup failed: %s", hipGetErrorString(hipGetLastError()));
    }
    const size_t tb = (c->td.bytes + 15) & ~size_t(15);
    c->lds = tb + kWavesPerBlock * c->ks.wave_bytes;
    c->lds_tab = ((c->td.off_chien + 15) & ~size_t(15)) + kWavesPerBlock * c->ks.wave_bytes;
    c->lds_tail = tb + kWavesPerBlock * c->ks.tail_wave_bytes + c->ks.tail_block_bytes;
    c->lds_alg = tb;
    if (select_fast(m, t, &c->fast))  // m >= 7: kaneko_first_kernel, the search kernel's layout
        c->lds_fast = m >= 7 ? c->lds : tb + fast_block_waves() * fast_wave_bytes();
    if (m >= 7 && !select_lane(m, t, &c->lane)) c->lane = nullptr;
    if (c->lane || (m <= 6 && c->fast)) {
        // the byte syndrome table of the lane kernels (m >= 7 pre-pass, n <= 63 ring kernel)
        // from the column table (same word stride W)
        const int n = c->field.n, W = (int)c->td.W, NB = (n + 7) / 8;
        const uint32_t *colh = reinterpret_cast<const uint32_t *>(c->tables_host.data() + c->td.off_col);
        std::vector<uint32_t> syn((size_t)NB * 256 * W, 0u);
        for (int j = 0; j < NB; ++j)
            for (int v = 0; v < 256; ++v)
                for (int b = 0; b < 8; ++b)
                    if (((v >> b) & 1) && 8 * j + b < n)
                        for (int w = 0; w < W; ++w) syn[((size_t)j * 256 + v) * W + w] ^= colh[(8 * j + b) * W + w];
        if (c->syn8.ensure(syn.size() * 4) != 0 ||
            hipMemcpy(c->syn8.p, syn.data(), syn.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            bchk_destroy(c);
            return fail(BCHK_EHIP, "device setup failed: %s", hipGetErrorString(hipGetLastError()));
        }
    }
    if (c->ks.gfmul) {
        // the cooperative decoders' product table: [a][b] = a b, then [a] = 1 / a (0 for 0)
        const int q = 1 << m, n = c->field.n;
        std::vector<uint8_t> mt((size_t)q * q + q, 0);
        for (int a = 1; a < q; ++a)
            for (int b = 1; b < q; ++b)
                mt[(size_t)a * q + b] = (uint8_t)c->field.alog[(c->field.log[a] + c->field.log[b]) % n];
        for (int a = 1; a < q; ++a) mt[(size_t)q * q + a] = (uint8_t)c->field.alog[(n - c->field.log[a]) % n];
        if (c->gfmul.ensure(mt.size()) != 0 ||
            hipMemcpy(c->gfmul.p, mt.data(), mt.size(), hipMemcpyHostToDevice) != hipSuccess) {
            bchk_destroy(c);
            return fail(BCHK_EHIP, "device setup failed: %s", hipGetErrorString(hipGetLastError()));
        }
    }
    if (const char *lp = getenv("BCHK_LANE_PRE")) c->lane_pre = atoi(lp) != 0;
    if (const char *lh = getenv("BCHK_LONG_HELP")) c->long_help = atoi(lh) != 0;
    if (const char *hm = getenv("BCHK_LONG_HELP_MAX")) c->long_help_max = (uint32_t)std::max(1, atoi(hm));
    if (const char *sm = getenv("BCHK_LONG_SHARE_MIN")) c->long_share_min = (uint32_t)std::max(8, atoi(sm));
    if (getenv("BCHK_NO_FAST")) c->use_fast = false;
    if (getenv("BCHK_NO_TABLE")) c->use_table = false;
    if (const char *cl = getenv("BCHK_CHUNK_LIMIT")) c->chunk_limit = (uint32_t)atoi(cl);
    if (const char *lr = getenv("BCHK_LONG_REC")) c->long_rec = std::max(0, std::min(2, atoi(lr)));
    if (const char *cc = getenv("BCHK_COOP_CONCURRENT")) c->coop_concurrent = atoi(cc) != 0;
    if (getenv("BCHK_NO_ANALYTIC")) c->analytic = false;
    if (getenv("BCHK_TAIL_DIAG")) c->tail_diag_on = true;
    if (const char *tc = getenv("BCHK_TAIL_CONCURRENT")) c->tail_concurrent = atoi(tc) != 0;
    if (const char *ti = getenv("BCHK_TAIL_INLINE")) c->tail_inline = atoi(ti) != 0;
    if (const char *ah = getenv("BCHK_AN_HELP")) c->an_help = atoi(ah) != 0;
    if (const char *fw = getenv("BCHK_FAST_RING_WAVES")) c->fast_waves = (uint32_t)std::max(2, std::min(16, atoi(fw)));
    if (const char *ht = getenv("BCHK_HEAVY_T")) c->heavy_t = (uint32_t)std::max(0, atoi(ht));
    if (const char *hx = getenv("BCHK_HEAVY_TMAX")) c->heavy_tmax = (uint32_t)std::max(0, atoi(hx));
    if (const char *fm = getenv("BCHK_FAST_MODE")) {
        c->fast_mode = (uint32_t)std::max(0, atoi(fm));
#ifndef BCHK_EXPERIMENT_MODES
        // modes 1 and 2 time parts of the ring kernel and give wrong results: experiment
        // builds only, never the product library (a leftover variable must not yield a
        // plausible-looking record)
        if (c->fast_mode == 1u || c->fast_mode == 2u) c->fast_mode = 0;
#endif
    }
    if (const char *tb = getenv("BCHK_TAIL_BLOCKS")) c->tail_conc_blocks = std::max(1, atoi(tb));
    if (const char *tm = getenv("BCHK_TAIL_MIN_BOUND")) c->tail_min_bound = strtoull(tm, nullptr, 10);
    if (const char *hf = getenv("BCHK_HEAVY_FIRST")) c->heavy_first = atoi(hf) != 0;
    if (const char *np = getenv("BCHK_PIPES")) c->npipes = std::max(1, std::min(8, atoi(np)));
    if (const char *pm = getenv("BCHK_PIPE_MIN")) c->pipe_min = std::max<size_t>(64, strtoull(pm, nullptr, 10));
    c->lds_coop = tb + c->ks.coop_bytes;
    // one cooperative workgroup per CU by default (LDS sized past half the CU's 160 KB):
    // a heavy codeword's 16 waves then own the CU's four SIMDs, which shortens the longest
    // searches -- the critical path of a decode call -- and leaves the remaining wave slots
    // to the concurrent exact kernel
    int coop_target = 1;
    if (const char *cp = getenv("BCHK_COOP_PER_CU")) coop_target = std::max(1, atoi(cp));
    if (coop_target == 1) c->lds_coop = std::max<size_t>(c->lds_coop, 82 * 1024);
    // resident workgroups per CU of a kernel (its own registers; LDS as given)
    auto grid_of = [&](const void *fn, int threads, size_t lds) {
        if (lds > 65536) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, lds) != hipSuccess || per_cu <= 0) {
            per_cu = 1;
            (void)hipGetLastError();
        }
        return per_cu * prop.multiProcessorCount;
    };
    c->grid_coop = grid_of(c->ks.coop_ptr(), c->ks.coop_threads, c->lds_coop);
    c->grid = grid_of(c->ks.search_ptr(), kWaveSize * kWavesPerBlock, c->lds);
    if (c->ks.search_tab) {
        c->grid_coop_tab = grid_of(c->ks.coop_tab_ptr(), c->ks.coop_threads, c->lds_coop);
        c->grid_tab = grid_of(c->ks.search_tab_ptr(), kWaveSize * kWavesPerBlock, c->lds_tab);
    }
    if (c->ks.tail) c->grid_tail = grid_of(c->ks.tail_ptr(), kWaveSize * kWavesPerBlock, c->lds_tail);
    if (c->ks.tail_tab) c->grid_tail_tab = grid_of(c->ks.tail_tab_ptr(), kWaveSize * kWavesPerBlock, c->lds_tail);
    if (const char *fp = getenv("BCHK_FIRST_PER_CU")) {  // experiment: the first pass's workgroups per CU
        const int per = std::max(1, atoi(fp));
        c->grid = per * prop.multiProcessorCount;
        if (c->ks.search_tab) c->grid_tab = per * prop.multiProcessorCount;
    }
    if (getenv("BCHK_VERBOSE"))  // persistent grids (workgroups) and their LDS bytes
        fprintf(stderr, "bchk m=%d t=%d cus=%d grid %d (lds %zu) tab %d (lds %zu) tail %d tail_tab %d (lds %zu) coop %d coop_tab %d (lds %zu)\n",
                m, t, prop.multiProcessorCount, c->grid, c->lds, c->grid_tab, c->lds_tab, c->grid_tail,
                c->grid_tail_tab, c->lds_tail, c->grid_coop, c->grid_coop_tab, c->lds_coop);
    (void)rc;
    *out = c;
    return 0;
}

void bchk_destroy(bchk_ctx *c) {
    if (!c) return;
    for (auto &e : c->events)
        for (auto &x : e.e) (void)hipEventDestroy(x);
    release_pipes(c);
    c->tdiag.release();
    c->cnt.release();
    c->fault.release();
    c->diag.release();
    for (DevBuf *b : {&c->gtx, &c->gy, &c->gres, &c->gst, &c->gcnt, &c->gflags}) b->release();
    c->y.release();
    c->res.release();
    c->l0.release();
    c->st.release();
    c->words.release();
    c->synd.release();
    c->ok.release();
    c->syn8.release();
    c->gfmul.release();
    if (c->d_tables) (void)hipFree(c->d_tables);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int bchk_code_params(const bchk_ctx *c, int *n, int *k, int *gsize) {
    if (!c) return fail(BCHK_EINVAL, "ctx is NULL");
    if (n) *n = c->n;
    if (k) *k = c->k;
    if (gsize) *gsize = (int)c->g.size();
    return 0;
}

int bchk_generator(const bchk_ctx *c, uint8_t *g) {
    if (!c || !g) return fail(BCHK_EINVAL, "NULL argument");
    memcpy(g, c->g.data(), c->g.size());
    return 0;
}

int bchk_set_max_decodes(bchk_ctx *c, uint64_t md) {
    if (!c) return fail(BCHK_EINVAL, "ctx is NULL");
    c->max_decodes = md;
    return 0;
}

void *bchk_stream(bchk_ctx *c) { return c ? (void *)c->stream : nullptr; }

// After the context's stream has drained: a bounded queue wait that ran out in a kernel
// (SearchParams::fault) means codewords were left unfinished -- an error, cleared once read.
static int check_fault(bchk_ctx *c) {
    if (!c->fault.p) return 0;
    uint32_t f = 0;
    HIP_TRY(hipMemcpyAsync(&f, c->fault.p, sizeof f, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (!f) return 0;
    HIP_TRY(hipMemsetAsync(c->fault.p, 0, sizeof f, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return fail(BCHK_EHIP, "a work-queue wait timed out in a decode kernel (fault bits %#x): codewords "
                "were left unfinished", f);
}

int bchk_sync(bchk_ctx *c) {
    if (!c) return fail(BCHK_EINVAL, "ctx is NULL");
    HIP_TRY(hipStreamSynchronize(c->stream));
    return check_fault(c);
}

int bchk_decode_device(bchk_ctx *c, const double *d_y, size_t B, uint8_t *d_res, double *d_l0,
                       bchk_stats *d_st, void *stream) {
    if (!c || (B && (!d_y || !d_res))) return fail(BCHK_EINVAL, "NULL argument");
    return launch_search(c, BCHK_VARIANT_ANSWER, d_y, B, d_res, d_l0, d_st,
                         stream ? (hipStream_t)stream : c->stream);
}

int bchk_decode_variant_host(bchk_ctx *c, int variant, const double *y, size_t B, uint8_t *res,
                             double *l0, bchk_stats *st) {
    if (!c || (B && (!y || !res))) return fail(BCHK_EINVAL, "NULL argument");
    if (variant != BCHK_VARIANT_ANSWER && variant != BCHK_VARIANT_WORD)
        return fail(BCHK_EINVAL, "unknown variant %d", variant);
    if (B == 0) return 0;
    const size_t n = c->n;
    int rc;
    if ((rc = c->y.ensure(B * n * sizeof(double))) || (rc = c->res.ensure(B * n)) ||
        (rc = c->l0.ensure(B * sizeof(double))) || (rc = c->st.ensure(B * sizeof(bchk_stats))))
        return rc;
    HIP_TRY(hipMemcpyAsync(c->y.p, y, B * n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    // rows that are never accepted must come back untouched
    HIP_TRY(hipMemcpyAsync(c->res.p, res, B * n, hipMemcpyHostToDevice, c->stream));
    if ((rc = launch_search(c, variant, (const double *)c->y.p, B, (uint8_t *)c->res.p,
                            (double *)c->l0.p, (bchk_stats *)c->st.p, c->stream)))
        return rc;
    HIP_TRY(hipMemcpyAsync(res, c->res.p, B * n, hipMemcpyDeviceToHost, c->stream));
    if (l0) HIP_TRY(hipMemcpyAsync(l0, c->l0.p, B * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (st) HIP_TRY(hipMemcpyAsync(st, c->st.p, B * sizeof(bchk_stats), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return check_fault(c);
}

int bchk_decode_host(bchk_ctx *c, const double *y, size_t B, uint8_t *res, double *l0, bchk_stats *st) {
    return bchk_decode_variant_host(c, BCHK_VARIANT_ANSWER, y, B, res, l0, st);
}

int bchk_alg_decode_host(bchk_ctx *c, const uint8_t *words, const uint32_t *synd, size_t N,
                         uint8_t *answers, uint8_t *ok) {
    if (!c || (N && (!words || !answers || !ok))) return fail(BCHK_EINVAL, "NULL argument");
    if (N == 0) return 0;
    if (N > 0xFFFFFFFFull) return fail(BCHK_EINVAL, "too many words");
    const size_t n = c->n;
    int rc;
    if ((rc = c->words.ensure(N * n)) || (rc = c->res.ensure(N * n)) || (rc = c->ok.ensure(N)))
        return rc;
    if (synd && (rc = c->synd.ensure(N * c->t * sizeof(uint32_t)))) return rc;
    HIP_TRY(hipMemcpyAsync(c->words.p, words, N * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->res.p, answers, N * n, hipMemcpyHostToDevice, c->stream));
    if (synd)
        HIP_TRY(hipMemcpyAsync(c->synd.p, synd, N * c->t * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    AlgParams p{};
    p.words = (const uint8_t *)c->words.p;
    p.synd = synd ? (const uint32_t *)c->synd.p : nullptr;
    p.answers = (uint8_t *)c->res.p;
    p.ok = (uint8_t *)c->ok.p;
    p.tables = c->d_tables;
    p.td = c->td;
    p.count = (uint32_t)N;
    p.t = c->t;
    HIP_TRY(launch_alg(c->ks, p, c->lds_alg, c->stream));
    HIP_TRY(hipMemcpyAsync(answers, c->res.p, N * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(ok, c->ok.p, N, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int bchk_decode_count_device(bchk_ctx *c, const double *d_y, const uint8_t *d_tx, size_t B, uint8_t *d_res,
                             double *d_l0, bchk_stats *d_st, uint64_t *d_out6, void *stream) {
    if (!c || (B && (!d_y || !d_tx || !d_res || !d_out6))) return fail(BCHK_EINVAL, "NULL argument");
    if (B == 0) return 0;
    const hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (int rc = launch_search(c, BCHK_VARIANT_ANSWER, d_y, B, d_res, d_l0, d_st, s, d_tx)) return rc;
    HIP_TRY(launch_cnt_reduce((unsigned long long *)c->cnt.p, (unsigned long long *)d_out6, s));
    return 0;
}

int bchk_count_device(bchk_ctx *c, const uint8_t *d_tx, const uint8_t *d_res, const bchk_stats *d_st,
                      size_t B, uint64_t *d_out6, void *stream) {
    if (!c || (B && (!d_tx || !d_res || !d_out6))) return fail(BCHK_EINVAL, "NULL argument");
    if (B == 0) return 0;
    HIP_TRY(launch_count(c->n, d_tx, d_res, d_st, (uint32_t)B, d_out6,
                         stream ? (hipStream_t)stream : c->stream));
    return 0;
}

// The reference's stream: std::default_random_engine (seed 1 unless RANDOM is defined,
// src/bchCoder.cpp:14-22), uniform_int_distribution<unsigned short>(0, 1) for the
// information bits and a fresh normal_distribution(0, sd) per addNoise call -- drawn from
// Minstd0 (bchk_stream.h), the same engine with its state readable.
}  // extern "C"

template <class Eng>
static void gen_word(Eng &eng, const bchk_ctx *c, double sd, uint8_t *tx, double *y,
                     std::vector<uint8_t> &info) {
    std::uniform_int_distribution<unsigned short> bit(0, 1);
    for (int i = 0; i < c->k; ++i) info[i] = (uint8_t)bit(eng);
    memset(tx, 0, c->n);
    for (int i = 0; i < c->k; ++i)  // c(x) = info(x) g(x), bchCoder.cpp:120-132
        if (info[i])
            for (size_t j = 0; j < c->g.size(); ++j) tx[i + j] ^= c->g[j];
    std::normal_distribution<double> noise(0.0, sd);
    for (int i = 0; i < c->n; ++i) y[i] = (tx[i] ? 1 : -1) + noise(eng);
}

// host threads for generating words: the job's CPU share (OMP_NUM_THREADS on the GPU box),
// at most 16
static int gen_threads() {
    int t = (int)std::thread::hardware_concurrency();
    if (const char *e = getenv("OMP_NUM_THREADS")) t = std::min(t > 0 ? t : 1, std::max(1, atoi(e)));
    if (const char *e = getenv("BCHK_GEN_THREADS")) t = std::max(1, atoi(e));
    return std::max(1, std::min(t, 16));
}

// `start` holds B + 1 word-start states (start[b] = engine state before word b, from the
// sample-free parse); the B words are generated by up to gen_threads() threads, each from its
// words' own start states, so the rows are the sequential stream's.
static int gen_from_starts(const bchk_ctx *c, double sd, const std::vector<uint64_t> &start, size_t B, uint8_t *tx,
                           double *y) {
    const size_t n = (size_t)c->n;
    const int T = (int)std::min<size_t>((size_t)gen_threads(), std::max<size_t>(1, B / 1024));
    std::vector<int> bad(T, 0);
    auto work = [&](int q) {
        std::vector<uint8_t> info(c->k);
        for (size_t b = B * q / T; b < B * (q + 1) / T; ++b) {
            Minstd0 e(start[b]);
            gen_word(e, c, sd, tx + b * n, y + b * n, info);
            bad[q] |= e.x != start[b + 1];  // the parse and the distributions agree on every word
        }
    };
    std::vector<std::thread> th;
    for (int q = 1; q < T; ++q) th.emplace_back(work, q);
    work(0);
    for (auto &t : th) t.join();
    for (int q = 0; q < T; ++q)
        if (bad[q]) return fail(BCHK_EINVAL, "stream parse and generator disagree (internal error)");
    return 0;
}

// B words from engine state *x (advanced past them); after[b] (may be NULL) = the state after
// word b; *draws (may be NULL) = the engine draws the words consumed.
static int gen_words(const bchk_ctx *c, double sd, uint64_t *x, size_t B, uint8_t *tx, double *y, uint64_t *after,
                     uint64_t *draws) {
    const int pairs = (c->n + 1) / 2;
    std::vector<uint64_t> start(B + 1);
    start[0] = Minstd0(*x).x;
    uint64_t d = 0;
    for (size_t b = 0; b < B; ++b) {
        uint64_t xx = start[b];
        d += stream_skip_word(xx, c->k, pairs);
        start[b + 1] = xx;
    }
    if (int rc = gen_from_starts(c, sd, start, B, tx, y)) return rc;
    if (after)
        for (size_t b = 0; b < B; ++b) after[b] = start[b + 1];
    *x = start[B];
    if (draws) *draws = d;
    return 0;
}

extern "C" {

static double sweep_sigma(const bchk_ctx *c, double stnr) {
    // src/dataForPlot.cpp:45 (getK()/getN() return long)
    const long K = c->k, Nn = c->n;
    return sqrt(1 / (pow(10, stnr / 10) * 2 * K / Nn));
}

// minstd_rand0: x <- 16807 x mod (2^31 - 1); jumping d draws ahead multiplies by 16807^d.
static constexpr uint64_t kMinstdM = 2147483647ull, kMinstdA = 16807ull;
static uint64_t minstd_state(uint64_t s) {  // the state std::minstd_rand0(s) starts from
    s %= kMinstdM;
    return s ? s : 1ull;
}

uint64_t bchk_rng_jump(uint64_t state, uint64_t draws) {
    uint64_t r = minstd_state(state), a = kMinstdA;
    for (uint64_t e = draws % (kMinstdM - 1); e; e >>= 1) {  // period 2^31 - 2
        if (e & 1) r = r * a % kMinstdM;
        a = a * a % kMinstdM;
    }
    return r;
}

int bchk_generate_host_draws(const bchk_ctx *c, double snr_db, size_t B, uint64_t *rng_state, uint64_t seed,
                             uint8_t *tx, double *y, uint64_t *draws) {
    if (!c || (B && (!tx || !y))) return fail(BCHK_EINVAL, "NULL argument");
    uint64_t x = minstd_state(rng_state && *rng_state ? *rng_state : seed);
    if (int rc = gen_words(c, sweep_sigma(c, snr_db), &x, B, tx, y, nullptr, draws)) return rc;
    if (rng_state) *rng_state = x;
    return 0;
}

// decode B generated words on the GPU: res rows zeroed, then written on acceptance
static int sweep_decode(bchk_ctx *c, const double *y, size_t B, uint8_t *res, uint8_t *accepted, uint64_t *ops) {
    if (B == 0) return 0;
    std::vector<bchk_stats> st(B);
    memset(res, 0, B * c->n);
    if (int rc = bchk_decode_host(c, y, B, res, nullptr, st.data())) return rc;
    for (size_t b = 0; b < B; ++b) {
        accepted[b] = (st[b].flags & BCHK_F_ACCEPTED) ? 1 : 0;
        ops[3 * b] = st[b].decodes;
        ops[3 * b + 1] = st[b].comparisons;
        ops[3 * b + 2] = st[b].sums;
    }
    return 0;
}

int bchk_sweep_block(bchk_ctx *c, double snr_db, uint64_t *rng_state, size_t skip, size_t B, uint8_t *tx,
                     uint8_t *res, uint8_t *accepted, uint64_t *ops, uint64_t *states) {
    if (!c || !rng_state || (B && (!tx || !res || !accepted || !ops || !states)))
        return fail(BCHK_EINVAL, "NULL argument");
    uint64_t x = minstd_state(*rng_state);
    const int pairs = (c->n + 1) / 2;
    for (size_t b = 0; b < skip; ++b) stream_skip_word(x, c->k, pairs);  // other ranks' words: draws only
    std::vector<double> y(B * c->n);
    if (int rc = gen_words(c, sweep_sigma(c, snr_db), &x, B, tx, y.data(), states, nullptr)) return rc;
    *rng_state = x;
    return sweep_decode(c, y.data(), B, res, accepted, ops);
}

int bchk_sweep_range(bchk_ctx *c, double snr_db, uint64_t *rng_state, uint64_t draws, size_t max_words,
                     uint8_t *tx, uint8_t *res, uint8_t *accepted, uint64_t *ops, uint64_t *states, size_t *words) {
    if (!c || !rng_state || !words || (max_words && (!tx || !res || !accepted || !ops || !states)))
        return fail(BCHK_EINVAL, "NULL argument");
    const int pairs = (c->n + 1) / 2;
    std::vector<uint64_t> start(1, minstd_state(*rng_state));
    uint64_t d = 0;
    while (d < draws) {  // the words of the range, found by the sample-free parse
        if (start.size() > max_words) return fail(BCHK_EINVAL, "range holds more than %zu words", max_words);
        uint64_t xx = start.back();
        d += stream_skip_word(xx, c->k, pairs);
        start.push_back(xx);
    }
    if (d != draws) return fail(BCHK_EINVAL, "the range does not end on a word boundary (%llu != %llu draws)",
                                (unsigned long long)d, (unsigned long long)draws);
    const size_t B = start.size() - 1;
    std::vector<double> y(B * c->n);
    if (int rc = gen_from_starts(c, sweep_sigma(c, snr_db), start, B, tx, y.data())) return rc;
    for (size_t b = 0; b < B; ++b) states[b] = start[b + 1];
    *rng_state = start[B];
    *words = B;
    return sweep_decode(c, y.data(), B, res, accepted, ops);
}

int bchk_generate_host(const bchk_ctx *c, double snr_db, size_t B, uint64_t *rng_state, uint64_t seed,
                       uint8_t *tx, double *y) {
    return bchk_generate_host_draws(c, snr_db, B, rng_state, seed, tx, y, nullptr);
}

// On-GPU channel (bchk_channel.hip): words [word0, word0 + B) of the counter-based stream
// `seed` at Eb/N0 snr_db (sd as src/dataForPlot.cpp:45), tx and y written on device.
int bchk_generate_device(bchk_ctx *c, double snr_db, size_t B, uint64_t seed, uint64_t word0, uint8_t *d_tx,
                         double *d_y, void *stream) {
    if (!c || (B && (!d_tx || !d_y))) return fail(BCHK_EINVAL, "NULL argument");
    if (B > 0xFFFFFFFFull) return fail(BCHK_EINVAL, "batch too large");
    if (B == 0) return 0;
    ChanParams cp{};
    cp.tx = d_tx;
    cp.y = d_y;
    cp.word0 = word0;
    cp.count = (uint32_t)B;
    cp.n = c->n;
    cp.k = c->k;
    cp.seed_lo = (uint32_t)seed;
    cp.seed_hi = (uint32_t)(seed >> 32);
    cp.sd = sweep_sigma(c, snr_db);
    for (size_t j = 0; j < c->g.size(); ++j)
        if (c->g[j]) cp.g[j >> 6] |= 1ull << (j & 63);
    HIP_TRY(launch_channel(cp, stream ? (hipStream_t)stream : c->stream));
    return 0;
}

// fun() (src/dataForPlot.cpp:16-74) with the words generated on the GPU (statistically the
// reference's stream, not bit-exactly) and the counters fused into the decode: Eb/N0 from 0
// to max_snr in steps of 0.5, each point until p words or e frame errors -- the e-th error
// cut exactly in word order (the batch that reaches it is decoded again with per-word
// stats and counted up to that word). CSV as bchk_sweep; seconds = wall time of the sweep,
// words = words decoded (including the re-decoded tail batches once).
int bchk_sweep_device(bchk_ctx *c, long p, long e, double max_snr, uint64_t seed, size_t batch, char *csv,
                      size_t cap, double *seconds, uint64_t *words) {
    if (!c || !csv || cap == 0) return fail(BCHK_EINVAL, "NULL argument");
    if (p <= 0 || e <= 0) return fail(BCHK_EINVAL, "p and e must be positive");
    const size_t n = c->n;
    const size_t B = batch ? batch : (size_t(1) << 20);
    int rc;
    if ((rc = c->gtx.ensure(B * n)) || (rc = c->gy.ensure(B * n * sizeof(double))) || (rc = c->gres.ensure(B * n)) ||
        (rc = c->gst.ensure(B * sizeof(bchk_stats))) || (rc = c->gcnt.ensure(16 * sizeof(uint64_t))) ||
        (rc = c->gflags.ensure(B)))
        return rc;
    const hipStream_t s = c->stream;
    HIP_TRY(hipMemsetAsync(c->gres.p, 0, B * n, s));
    const auto t0 = std::chrono::steady_clock::now();
    std::ostringstream out;
    long count = 0, countErr = 0;
    long long countE = 0;  // never reset between points, as src/dataForPlot.cpp:20,61
    unsigned long D = 0, Cc = 0, Ss = 0, wordCount = 0;
    uint64_t word = 0, decoded = 0;
    std::vector<uint8_t> flags;
    uint64_t h[6];
    uint64_t *d6 = (uint64_t *)c->gcnt.p;
    for (double stnr = 0.0; stnr <= max_snr; stnr += 0.5) {
        while (count < p && countErr < e) {
            const size_t nb = std::min<size_t>(B, (size_t)(p - count));
            if ((rc = bchk_generate_device(c, stnr, nb, seed, word, (uint8_t *)c->gtx.p, (double *)c->gy.p, s)))
                return rc;
            HIP_TRY(hipMemsetAsync(d6, 0, 6 * sizeof(uint64_t), s));
            if ((rc = bchk_decode_count_device(c, (const double *)c->gy.p, (const uint8_t *)c->gtx.p, nb,
                                               (uint8_t *)c->gres.p, nullptr, nullptr, d6, s)))
                return rc;
            HIP_TRY(hipMemcpyAsync(h, d6, sizeof h, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            if ((rc = check_fault(c))) return rc;
            if (h[5] != nb)  // every word of the batch must have been finished and counted
                return fail(BCHK_EHIP, "fused counters saw %llu of %zu words", (unsigned long long)h[5], nb);
            decoded += nb;
            size_t used = nb;
            if (countErr + (long)h[0] >= e) {  // the e-th error falls in this batch: cut there
                if ((rc = launch_search(c, BCHK_VARIANT_ANSWER, (const double *)c->gy.p, nb, (uint8_t *)c->gres.p,
                                        nullptr, (bchk_stats *)c->gst.p, s)))
                    return rc;
                HIP_TRY(launch_frame_errors((const uint8_t *)c->gtx.p, (const uint8_t *)c->gres.p, (uint32_t)nb,
                                            (int)n, (uint8_t *)c->gflags.p, s));
                flags.resize(nb);
                HIP_TRY(hipMemcpyAsync(flags.data(), c->gflags.p, nb, hipMemcpyDeviceToHost, s));
                HIP_TRY(hipStreamSynchronize(s));
                long need = e - countErr;
                used = nb;
                for (size_t w = 0; w < nb; ++w)
                    if (flags[w] && --need == 0) {
                        used = w + 1;
                        break;
                    }
                HIP_TRY(hipMemsetAsync(d6, 0, 6 * sizeof(uint64_t), s));
                HIP_TRY(launch_count(c->n, (const uint8_t *)c->gtx.p, (const uint8_t *)c->gres.p,
                                     (const bchk_stats *)c->gst.p, (uint32_t)used, d6, s));
                HIP_TRY(hipMemcpyAsync(h, d6, sizeof h, hipMemcpyDeviceToHost, s));
                HIP_TRY(hipStreamSynchronize(s));
                decoded += nb;
            }
            countErr += (long)h[0];
            countE += (long long)h[1];
            D += h[2];
            Cc += h[3];
            Ss += h[4];
            count += (long)used;
            wordCount += used;
            word += used;
        }
        out << stnr << "," << ((double)countErr) / count << "," << ((double)countE) / count / (long)n << ","
            << ((double)D) / wordCount << "," << ((double)Cc) / wordCount << "," << ((double)Ss) / wordCount
            << "\n";
        D = Cc = Ss = 0;
        wordCount = 0;
        count = 0, countErr = 0;
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (seconds) *seconds = secs;
    if (words) *words = decoded;
    const std::string str = out.str();
    if (str.size() + 1 > cap) return fail(BCHK_EINVAL, "csv buffer too small (%zu needed)", str.size() + 1);
    memcpy(csv, str.c_str(), str.size() + 1);
    return 0;
}

int bchk_sweep(bchk_ctx *c, long p, long e, double max_snr, uint64_t *rng_state, uint64_t seed,
               size_t batch, char *csv, size_t cap) {
    if (!c || !csv || cap == 0) return fail(BCHK_EINVAL, "NULL argument");
    if (p <= 0 || e <= 0) return fail(BCHK_EINVAL, "p and e must be positive");
    const size_t n = c->n;
    const size_t max_batch = batch ? batch : (size_t(1) << 18);
    uint64_t x = minstd_state(rng_state && *rng_state ? *rng_state : seed);
    std::vector<uint8_t> tx, res, dec(n, 0);
    std::vector<double> y;
    std::vector<bchk_stats> st;
    std::vector<uint64_t> after;  // engine state after each word of the batch
    std::ostringstream out;
    int count = 0, countErr = 0, countE = 0;  // int, as src/dataForPlot.cpp:20
    unsigned long D = 0, Cc = 0, Ss = 0, wordCount = 0;
    double fer_est = 0.5;
    for (double stnr = 0.0; stnr <= max_snr; stnr += 0.5) {
        const double sd = sweep_sigma(c, stnr);
        while (count < p && countErr < e) {
            // batch size: enough words to reach e errors at the current estimate
            const double want = 2.0 * (double)(e - countErr) / std::max(fer_est, 1e-7);
            size_t nb = (size_t)std::min<double>(want, (double)max_batch);
            nb = std::max<size_t>(nb, 256);
            nb = std::min<size_t>(nb, (size_t)(p - count));
            tx.resize(nb * n);
            y.resize(nb * n);
            res.assign(nb * n, 0);
            st.resize(nb);
            after.resize(nb);
            const uint64_t x0 = x;
            if (int rc = gen_words(c, sd, &x, nb, tx.data(), y.data(), after.data(), nullptr)) return rc;
            int rc = bchk_decode_host(c, y.data(), nb, res.data(), nullptr, st.data());
            if (rc) return rc;
            size_t used = 0;
            int errs_batch = 0;
            for (size_t b = 0; b < nb; ++b) {
                if (!(count < p && countErr < e)) break;
                if (st[b].flags & BCHK_F_ACCEPTED) memcpy(dec.data(), &res[b * n], n);
                // else: the caller's buffer keeps the previous word's result (:25,52)
                bool differ = memcmp(&tx[b * n], dec.data(), n) != 0;
                if (differ) ++countErr, ++errs_batch;
                for (size_t i = 0; i < n; ++i) countE += tx[b * n + i] != dec[i];
                ++count;
                ++wordCount;
                D += st[b].decodes;
                Cc += st[b].comparisons;
                Ss += st[b].sums;
                used = b + 1;
            }
            x = used ? after[used - 1] : x0;  // rewind the stream to the first word not consumed
            fer_est = std::max(1e-7, (double)(errs_batch + 1) / (double)(used + 1));
        }
        out << stnr << "," << ((double)countErr) / count << "," << ((double)countE) / count / (long)n << ","
            << ((double)D) / wordCount << "," << ((double)Cc) / wordCount << "," << ((double)Ss) / wordCount
            << "\n";
        D = Cc = Ss = 0;
        wordCount = 0;
        count = 0, countErr = 0;
    }
    if (rng_state) *rng_state = x;
    const std::string s = out.str();
    if (s.size() + 1 > cap) return fail(BCHK_EINVAL, "csv buffer too small (%zu needed)", s.size() + 1);
    memcpy(csv, s.c_str(), s.size() + 1);
    return 0;
}

int bchk_profile(bchk_ctx *c, int enable) {
    if (!c) return fail(BCHK_EINVAL, "ctx is NULL");
    c->profile = enable != 0;
    return 0;
}

int bchk_profile_read_stages(bchk_ctx *c, double *ms4, uint64_t *launches) {
    if (!c) return fail(BCHK_EINVAL, "ctx is NULL");
    for (auto &e : c->events) {
        HIP_TRY(hipEventSynchronize(e.e[5]));
        HIP_TRY(hipEventSynchronize(e.e[7]));
        for (int k = 0; k < 4; ++k) {
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, e.e[2 * k], e.e[2 * k + 1]));
            c->prof_ms[k] += ms;
        }
        c->prof_launches += e.first ? 1 : 0;  // per call: a call's pipelines add up
        for (auto &x : e.e) (void)hipEventDestroy(x);
    }
    c->events.clear();
    if (ms4)
        for (int k = 0; k < 4; ++k) ms4[k] = c->prof_ms[k];
    if (launches) *launches = c->prof_launches;
    for (int k = 0; k < 4; ++k) c->prof_ms[k] = 0.0;
    c->prof_launches = 0;
    return 0;
}

int bchk_profile_read(bchk_ctx *c, double *ms3, uint64_t *launches) {
    double ms4[4];
    if (int rc = bchk_profile_read_stages(c, ms4, launches)) return rc;
    if (ms3) {  // the exact stage includes the analytic tail kernel
        ms3[0] = ms4[0];
        ms3[1] = ms4[1] + ms4[3];
        ms3[2] = ms4[2];
    }
    return 0;
}

int bchk_tail_count(bchk_ctx *c, uint64_t *to_tail) {
    if (!c || !to_tail) return fail(BCHK_EINVAL, "NULL argument");
    uint64_t a = 0, b = 0;
    if (int rc = bchk_path_counts(c, &a, &b)) return rc;
    *to_tail = c->last_tail;
    return 0;
}

// diagnostics (BCHK_TAIL_DIAG=1): the last call's per-codeword tail records, 8 u64 each
int bchk_tail_diag_read(bchk_ctx *c, uint64_t *out, size_t items, uint64_t *count) {
    if (!c || !out || !count) return fail(BCHK_EINVAL, "NULL argument");
    *count = 0;
    if (!c->tdiag.p) return 0;
    uint32_t n = 0;
    if (c->pipes.empty() || !c->pipes[0].ctrl.p) return 0;
    HIP_TRY(hipMemcpy(&n, (uint32_t *)c->pipes[0].ctrl.p + kTailStats + 16, 4, hipMemcpyDeviceToHost));
    const size_t m = std::min<size_t>({items, (size_t)n, c->tdiag.cap / 128});
    HIP_TRY(hipMemcpy(out, c->tdiag.p, m * 64, hipMemcpyDeviceToHost));
    *count = n;
    return 0;
}

int bchk_tail_prof_read(bchk_ctx *c, uint64_t *out, size_t items) {
    if (!c || !out) return fail(BCHK_EINVAL, "NULL argument");
    if (!c->tdiag.p) return 0;
    const size_t cap = c->tdiag.cap / 128, m = std::min(items, cap);
    HIP_TRY(hipMemcpy(out, (const uint8_t *)c->tdiag.p + cap * 64, m * 64, hipMemcpyDeviceToHost));
    return 0;
}

int bchk_tail_stats(bchk_ctx *c, uint64_t *out6) {
    if (!c || !out6) return fail(BCHK_EINVAL, "NULL argument");
    uint64_t a = 0, b = 0;
    if (int rc = bchk_path_counts(c, &a, &b)) return rc;
    for (int k = 0; k < 6; ++k) out6[k] = c->last_tail_stats[k];
    return 0;
}

int bchk_coop_stats(bchk_ctx *c, uint64_t *out2) {
    if (!c || !out2) return fail(BCHK_EINVAL, "NULL argument");
    uint64_t a = 0, b = 0;
    if (int rc = bchk_path_counts(c, &a, &b)) return rc;
    for (int k = 0; k < 2; ++k) out2[k] = c->last_coop_stats[k];
    return 0;
}

int bchk_path_counts(bchk_ctx *c, uint64_t *to_exact, uint64_t *to_coop) {
    if (!c) return fail(BCHK_EINVAL, "ctx is NULL");
    // the last call's counts, summed over its pipelines (a pipeline the call did not use
    // still holds an earlier call's: only the first npipes_used are read)
    uint64_t v[2] = {0, 0};
    c->last_tail = 0;
    for (auto &x : c->last_tail_stats) x = 0;
    for (auto &x : c->last_coop_stats) x = 0;
    for (int k = 0; k < c->last_pipes && k < (int)c->pipes.size(); ++k) {
        const bchk_ctx::Pipe &P = c->pipes[k];
        if (!P.ctrl.p) continue;
        std::vector<uint32_t> h(kCtrlBytes / 4);
        HIP_TRY(hipMemcpyAsync(h.data(), P.ctrl.p, kCtrlBytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        v[0] += h[0];
        v[1] += (uint64_t)h[kHeavyTail] + h[kHeavyTail2];
        c->last_tail += h[kL1Tail];
        for (int q = 0; q < 2; ++q) c->last_coop_stats[q] += h[kCoopStats + q];
        for (int q = 0; q < 6; ++q)
            c->last_tail_stats[q] = q == 5 ? std::max<uint64_t>(c->last_tail_stats[q], h[kTailStats + q])
                                           : c->last_tail_stats[q] + h[kTailStats + q];
    }
    if (to_exact) *to_exact = v[0];
    if (to_coop) *to_coop = v[1];
    return 0;
}

#ifdef BCHK_DIAG
// diagnostic builds: copy the cooperative kernel's per-item stamps (8 u64 each)
int bchk_diag_read(bchk_ctx *c, uint64_t *out, size_t items) {
    if (!c || !out) return fail(BCHK_EINVAL, "NULL argument");
    if (!c->diag.p) return fail(BCHK_EINVAL, "not a diagnostic build");
    const size_t bytes = std::min(items * 64, c->diag.cap);
    HIP_TRY(hipMemcpy(out, c->diag.p, bytes, hipMemcpyDeviceToHost));
    return 0;
}
#endif

int bchk_set_syndrome_table(bchk_ctx *c, int enable) {
    if (!c) return fail(BCHK_EINVAL, "ctx is NULL");
    c->use_table = enable != 0;
    return 0;
}

int bchk_syndrome_table_query(int m, int t, const uint32_t *synd, size_t N, uint8_t *ok,
                              uint64_t *err) {
    if (N && (!synd || !ok)) return fail(BCHK_EINVAL, "NULL argument");
    if (m < 2 || m > kMaxM || t < 1 || t >= (1 << (m - 1))) return fail(BCHK_EINVAL, "bad m/t");
    if (!syndtab_feasible(m, t)) return fail(BCHK_EINVAL, "no syndrome table for m=%d t=%d", m, t);
    const Field f = make_field(m);
    const HostTable *h = nullptr;
    if (int rc = host_table(f, t, &h)) return rc;
    TableDesc td{};
    const std::vector<uint8_t> blob = make_tables(f, t, &td);
    const uint16_t *lg = reinterpret_cast<const uint16_t *>(blob.data() + td.off_log);
    SyndTable T{h->slots.data(), h->bbits, h->max_probe, h->kbits, h->tbits};
    for (size_t i = 0; i < N; ++i) {
        uint32_t Sw[2] = {0, 0};
        for (int q = 0; q < t; ++q) Sw[q >> 2] |= (synd[i * t + q] & 0xFFu) << (8 * (q & 3));
        uint64_t E = 0;
        bool hit = false;
        switch (m) {
            case 2: hit = tab_decode<2, kTabTmax>(T, Sw, t, lg, E); break;
            case 3: hit = tab_decode<3, kTabTmax>(T, Sw, t, lg, E); break;
            case 4: hit = tab_decode<4, kTabTmax>(T, Sw, t, lg, E); break;
            case 5: hit = tab_decode<5, kTabTmax>(T, Sw, t, lg, E); break;
            default: hit = tab_decode<6, kTabTmax>(T, Sw, t, lg, E); break;
        }
        ok[i] = hit ? 1 : 0;
        if (err) err[i] = E;
    }
    return 0;
}

int bchk_syndrome_table_info(int m, int t, uint64_t *keys, uint64_t *bytes, uint32_t *max_probe) {
    if (!syndtab_feasible(m, t) || t >= (1 << (m - 1)))
        return fail(BCHK_EINVAL, "no syndrome table for m=%d t=%d", m, t);
    const Field f = make_field(m);
    const HostTable *h = nullptr;
    if (int rc = host_table(f, t, &h)) return rc;
    if (keys) *keys = h->keys;
    if (bytes) *bytes = h->slots.size() * sizeof(uint64_t);
    if (max_probe) *max_probe = h->max_probe;
    return 0;
}

int bchk_set_analytic(bchk_ctx *c, int enable) {
    if (!c) return fail(BCHK_EINVAL, "ctx is NULL");
    c->analytic = enable != 0;
    return 0;
}

int bchk_set_chunk_limit(bchk_ctx *c, uint32_t chunks) {
    if (!c) return fail(BCHK_EINVAL, "ctx is NULL");
    c->chunk_limit = chunks;
    return 0;
}

int bchk_set_fast_path(bchk_ctx *c, int enable) {
    if (!c) return fail(BCHK_EINVAL, "ctx is NULL");
    c->use_fast = enable != 0;
    return 0;
}

}  // extern "C"
