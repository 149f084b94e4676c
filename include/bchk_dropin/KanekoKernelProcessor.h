// bchk drop-in for the reference's headers/KanekoKernelProcessor.h.
//
// Same public interface (headers/KanekoKernelProcessor.h:47-68), so src/main.cpp and
// src/dataForPlot.cpp of the reference compile against it unchanged. Every decode runs on
// the MI355X through the C ABI (include/bchk.h); there is no CPU decode path.
//   J cap: the reference's compiled-in choice (src/KanekoKernelProcessor.cpp:392-393) is
//   read from the environment: BCHK_J unset/negative = shipped (uncapped), else the cap.
//   Device: BCHK_DEVICE (default 0).
#ifndef BCHK_DROPIN_KANEKO_H
#define BCHK_DROPIN_KANEKO_H

#include <cstddef>
#include <vector>

#include "Decoder.h"

struct bchk_ctx;
struct bchk_stats;

class KanekoKernelProcessor {
public:
    KanekoKernelProcessor(long pw, long n, long t, long k, unsigned long *antilogarithms,
                          unsigned long *logarithms, double signalToNoiseRatio);
    virtual ~KanekoKernelProcessor();
    KanekoKernelProcessor(const KanekoKernelProcessor &) = delete;
    KanekoKernelProcessor &operator=(const KanekoKernelProcessor &) = delete;

    // src/KanekoKernelProcessor.cpp:161 -- never runs the algebraic decoder in the
    // reference (`success` is read uninitialised); throws std::logic_error here.
    void decode(unsigned char *res);
    // :212-276, the file-mode variant (src/main.cpp:158)
    void decode(const double *word, unsigned char *res);
    // :335-407, the variant the FER sweep uses (src/dataForPlot.cpp:52)
    void decode(const unsigned char *answer, const double *word, unsigned char *res);
    // :150-159: stages a word for calcL / decode(res)
    void set(const double *word) const;

    long getN() const;
    long getT() const;
    long getK() const;
    // :79-87 against the last decoded (or set) word
    double calcL(const unsigned char *word) const;

    unsigned long getComparisonCount() const;
    unsigned long getSummCount() const;
    unsigned long getDecodingCount() const;
    void setDecodingCount(unsigned long c = 0);
    void setComparisonCount(unsigned long comparisonCount = 0);
    void setSummCount(unsigned long summCount = 0);

    // ---- batched extension (not in the reference) ------------------------------------
    // count words y[count][n]; res rows written only where accepted (as the reference).
    void decodeBatch(const double *words, std::size_t count, unsigned char *res,
                     double *l0 = nullptr, bchk_stats *stats = nullptr);
    bchk_ctx *context() const { return ctx_; }
    void addCounters(unsigned long decodes, unsigned long comparisons, unsigned long sums);

private:
    void stage(const double *word) const;

    bchk_ctx *ctx_ = nullptr;
    long n_, t_, k_;
    double s2_;
    mutable std::vector<double> absAlpha_;
    mutable std::vector<unsigned char> hard_;
    unsigned long comparisons_ = 0, sums_ = 0, decodes_ = 0;
};

#endif
