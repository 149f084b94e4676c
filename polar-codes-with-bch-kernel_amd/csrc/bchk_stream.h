// bchk_stream.h -- the reference's input stream as draws of its engine (host side).
//
// fun() (src/dataForPlot.cpp:47-50) draws each word from ONE std::default_random_engine
// (minstd_rand0, src/bchCoder.cpp:14-22): k information bits from
// uniform_int_distribution<unsigned short>(0, 1) (generateRandomPoly, :236-240), then n noise
// samples from a fresh normal_distribution (addNoise, :243-250: Marsaglia's polar method,
// ceil(n/2) accepted pairs, each attempt two generate_canonical<double, 53> = four draws).
// Minstd0 is that engine with its state readable (the distributions see the same result_type,
// min, max and values, so the words are unchanged); the draw structure below restates
// libstdc++ 11's acceptance tests without computing a sample, which is what lets a rank find
// word boundaries in the stream without generating the words before them.
#pragma once
#include <stdint.h>

#include <random>

namespace bchk {

constexpr uint64_t kMinstdMod = 2147483647ull, kMinstdMul = 16807ull;

inline uint64_t minstd_mulmod(uint64_t a, uint64_t b) {  // a, b < 2^31 - 1 (Mersenne reduction)
    const uint64_t p = a * b;
    uint64_t t = (p & kMinstdMod) + (p >> 31);
    return t >= kMinstdMod ? t - kMinstdMod : t;
}

struct Minstd0 {
    using result_type = std::minstd_rand0::result_type;
    static constexpr result_type min() { return std::minstd_rand0::min(); }
    static constexpr result_type max() { return std::minstd_rand0::max(); }
    uint64_t x;
    // the state std::minstd_rand0(s) starts from (linear_congruential_engine::seed)
    explicit Minstd0(uint64_t s = 1) : x(s % kMinstdMod ? s % kMinstdMod : 1ull) {}
    result_type operator()() {
        x = minstd_mulmod(x, kMinstdMul);
        return (result_type)x;
    }
};

// uniform_int_distribution<unsigned short>(0, 1) on minstd_rand0 (libstdc++ downscaling): a
// draw v is used iff v - 1 < 2 * ((2^31 - 3) / 2); only v = 2^31 - 2 and 2^31 - 3 are
// redrawn, at two positions of the whole period.
inline bool info_draw_ok(uint64_t v) { return v - 1u < 2147483644ull; }

// generate_canonical<double, 53>(minstd_rand0): two draws, base R = 2^31 - 2. libstdc++ forms
// sum += double(v - min) * tmp; tmp = double(long double(tmp) * R) (from tmp = 1): the two
// factors are the constants below (R and R^2 rounded to double), so no long double remains.
constexpr double kCanonT1 = (double)(1.0L * 2147483646.0L);
constexpr double kCanonT2 = (double)((long double)kCanonT1 * 2147483646.0L);
inline double canonical2(uint64_t v1, uint64_t v2) {
    double sum = 0.0;
    sum += (double)(v1 - 1u) * 1.0;
    sum += (double)(v2 - 1u) * kCanonT1;
    double r = sum / kCanonT2;
    if (r >= 1.0) r = __builtin_nextafter(1.0, 0.0);
    return r;
}

// one polar-method attempt from its four draws: accepted iff 0 < x^2 + y^2 <= 1
inline bool polar_pair_ok(uint64_t v1, uint64_t v2, uint64_t v3, uint64_t v4) {
    const double x = 2.0 * canonical2(v1, v2) - 1.0, y = 2.0 * canonical2(v3, v4) - 1.0;
    const double r2 = x * x + y * y;
    return !(r2 > 1.0 || r2 == 0.0);
}

// The draws of one word from engine state x (advanced past it): k information draws (with
// redraws), then polar attempts until `pairs` are accepted. Returns the draws consumed.
uint64_t stream_skip_word(uint64_t &x, int k, int pairs);

}  // namespace bchk
