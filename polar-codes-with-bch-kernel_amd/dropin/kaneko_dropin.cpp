// Drop-in KanekoKernelProcessor and Decoder (include/bchk_dropin/) over the C ABI.
// Reference semantics cited per member; the decoding itself runs on the GPU.
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "KanekoKernelProcessor.h"
#include "bchk.h"

namespace {

int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

// The reference reports bad setups by throwing const char* (src/main.cpp:52,56,152),
// which its main() catches and prints; keep that contract.
[[noreturn]] void raise(const std::string &what) {
    static thread_local std::string keep;
    keep = what;
    throw keep.c_str();
}

bchk_ctx *open_ctx(long pw, long n, long t, long k, int J, double snr) {
    bchk_ctx *c = nullptr;
    if (bchk_create((int)pw, (int)t, J, snr, env_int("BCHK_DEVICE", 0), &c) != 0)
        raise(std::string("bchk: ") + bchk_last_error() + "\n");
    int nn = 0, kk = 0;
    bchk_code_params(c, &nn, &kk, nullptr);
    if (nn != n || kk != k) {
        bchk_destroy(c);
        raise("bchk: (n, k) does not match the code built for (m, t)\n");
    }
    return c;
}

}  // namespace

// ------------------------------------------------------------- KanekoKernelProcessor
// src/KanekoKernelProcessor.cpp:17-26
KanekoKernelProcessor::KanekoKernelProcessor(long pw, long n, long t, long k, unsigned long *,
                                             unsigned long *, double signalToNoiseRatio)
    : n_(n), t_(t), k_(k) {
    ctx_ = open_ctx(pw, n, t, k, env_int("BCHK_J", -1), signalToNoiseRatio);
    const double sd = sqrt(1 / (pow(10, signalToNoiseRatio / 10) * 2 * k / n));
    s2_ = pow(sd, 2);
    absAlpha_.assign(n, 0.0);
    hard_.assign(n, 0);
}

KanekoKernelProcessor::~KanekoKernelProcessor() { bchk_destroy(ctx_); }

// alpha = 2 y / pow(sd, 2), yH, |alpha| (:150-159); kept for calcL(word).
void KanekoKernelProcessor::stage(const double *word) const {
    for (long i = 0; i < n_; ++i) {
        const double a = 2 * word[i] / s2_;
        hard_[i] = (a <= 0.0) ? 0 : 1;
        absAlpha_[i] = fabs(a);
    }
}

void KanekoKernelProcessor::set(const double *word) const { stage(word); }

void KanekoKernelProcessor::decode(unsigned char *) {
    throw std::logic_error(
        "KanekoKernelProcessor::decode(res): the reference never calls the algebraic decoder "
        "here (src/KanekoKernelProcessor.cpp:161-210 reads `success` uninitialised)");
}

void KanekoKernelProcessor::decode(const double *word, unsigned char *res) {
    bchk_stats st;
    if (bchk_decode_variant_host(ctx_, BCHK_VARIANT_WORD, word, 1, res, nullptr, &st) != 0)
        raise(std::string("bchk: ") + bchk_last_error() + "\n");
    stage(word);
    addCounters(st.decodes, st.comparisons, st.sums);
}

void KanekoKernelProcessor::decode(const unsigned char *, const double *word, unsigned char *res) {
    bchk_stats st;
    if (bchk_decode_host(ctx_, word, 1, res, nullptr, &st) != 0)
        raise(std::string("bchk: ") + bchk_last_error() + "\n");
    stage(word);
    addCounters(st.decodes, st.comparisons, st.sums);
}

void KanekoKernelProcessor::decodeBatch(const double *words, std::size_t count, unsigned char *res,
                                        double *l0, bchk_stats *stats) {
    std::vector<bchk_stats> tmp;
    if (!stats) {
        tmp.resize(count);
        stats = tmp.data();
    }
    if (bchk_decode_host(ctx_, words, count, res, l0, stats) != 0)
        raise(std::string("bchk: ") + bchk_last_error() + "\n");
    for (std::size_t b = 0; b < count; ++b)
        addCounters(stats[b].decodes, stats[b].comparisons, stats[b].sums);
    if (count) stage(words + (count - 1) * n_);
}

void KanekoKernelProcessor::addCounters(unsigned long d, unsigned long c, unsigned long s) {
    decodes_ += d;
    comparisons_ += c;
    sums_ += s;
}

// calcL(word), :79-87: sum of |alpha_i| where yH_i != word_i, in index order.
double KanekoKernelProcessor::calcL(const unsigned char *word) const {
    double l = 0;
    for (long i = 0; i < n_; ++i)
        if (hard_[i] != word[i]) l += absAlpha_[i];
    return l;
}

long KanekoKernelProcessor::getN() const { return n_; }
long KanekoKernelProcessor::getT() const { return t_; }
long KanekoKernelProcessor::getK() const { return k_; }
unsigned long KanekoKernelProcessor::getComparisonCount() const { return comparisons_; }
unsigned long KanekoKernelProcessor::getSummCount() const { return sums_; }
unsigned long KanekoKernelProcessor::getDecodingCount() const { return decodes_; }
void KanekoKernelProcessor::setDecodingCount(unsigned long c) { decodes_ = c; }
void KanekoKernelProcessor::setComparisonCount(unsigned long c) { comparisons_ = c; }
void KanekoKernelProcessor::setSummCount(unsigned long c) { sums_ = c; }

// ----------------------------------------------------------------------------- Decoder
// src/Decoder.cpp:12-38
Decoder::Decoder(long pw, long n, long t, long k, unsigned long *antilogarithms, unsigned long *)
    : syndromPoly(new unsigned long[2 * t]), syndromPolySize(0), power_(pw), n_(n), t_(t),
      k_(k), alog_(antilogarithms), last_(n, 0), odd_(t, 0) {
    ctx_ = open_ctx(pw, n, t, k, -1, 0.5);
    for (long j = 0; j < 2 * t; ++j) syndromPoly[j] = 0;
}

Decoder::~Decoder() {
    delete[] syndromPoly;
    bchk_destroy(ctx_);
}

void Decoder::refreshSize() {
    syndromPolySize = 0;
    for (long j = 2 * t_; j >= 1; --j)
        if (syndromPoly[j - 1]) {
            syndromPolySize = j;
            break;
        }
}

// S_j = sum_i w_i alpha^(i j), j = 1..2t (:184-207)
void Decoder::findSyndromPoly(const unsigned char *word) {
    for (long j = 1; j <= 2 * t_; ++j) {
        unsigned long s = 0;
        for (long i = 0; i < n_; ++i)
            if (word[i]) s ^= alog_[(i * j) % n_];
        syndromPoly[j - 1] = s;
    }
    refreshSize();
    std::memcpy(last_.data(), word, n_);
}

// incremental update over the positions that changed since the last call (:210-230)
void Decoder::alterSyndromPoly(const unsigned char *word) {
    for (long i = 0; i < n_; ++i)
        if (last_[i] != word[i])
            for (long j = 1; j <= 2 * t_; ++j) syndromPoly[j - 1] ^= alog_[(i * j) % n_];
    refreshSize();
    std::memcpy(last_.data(), word, n_);
}

// :298-321 on the GPU from the stored syndromes; answer is written only on success.
bool Decoder::decode(const unsigned char *word, unsigned char *answer) {
    for (long j = 0; j < t_; ++j) odd_[j] = (unsigned int)syndromPoly[2 * j];
    uint8_t ok = 0;
    if (bchk_alg_decode_host(ctx_, word, odd_.data(), 1, answer, &ok) != 0)
        raise(std::string("bchk: ") + bchk_last_error() + "\n");
    return ok != 0;
}

long Decoder::getN() const { return n_; }
long Decoder::getT() const { return t_; }
long Decoder::getK() const { return k_; }
