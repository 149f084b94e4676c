// oracle/ref_golden.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Golden-vector driver for the REFERENCE implementation. It is our own code; it is
// linked (by oracle/Makefile) against the reference's unmodified translation units
//   /root/reference/src/{bchCoder,Decoder,KanekoKernelProcessor}.cpp
// and includes the reference's headers from /root/reference/headers. Its output is
// written as small text fixtures under tests/golden/ by oracle/make_golden.py.
//
// Modes
//   vectors <m> <t> <seed> <count> <snr_db>
//       Reproduces the per-word body of fun() (src/dataForPlot.cpp:43-52):
//       generateRandomPoly -> multiplyPolynomials -> addNoise -> decode(answer,y,res)
//       and prints, per word, the input, the output and the counter deltas read from
//       the getters (headers/KanekoKernelProcessor.h:63-68).
//   file <m> <t> <path>
//       The known-answer word of in/infile.txt, decoded with decode(answer, y, res).
//   bench <m> <t> <seed> <count> <snr_db>
//       CPU-baseline timing of decode(answer, word, res) over `count` stream words.
//   algdec <m> <t> exhaustive
//       Decoder::decode (src/Decoder.cpp:298) on every coset representative of the
//       cyclic code (every word supported on positions 0..n-k-1).
//   algdec <m> <t> random <count> <seed>
//       Decoder::decode on codeword + random low-weight error patterns.
//
// Number format: doubles as C99 hex-float (%a), exact.
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <random>
#include <string>
#include <vector>

#include "KanekoKernelProcessor.h"
#include "Decoder.h"
#include "bchCoder.h"

// The reference's global engine (src/bchCoder.cpp:20) -- reseeded per run.
extern std::default_random_engine generator;

static const unsigned long kPrim[16] = {3, 7, 11, 19, 37, 67, 137, 285, 529, 1033,
                                        2053, 4179, 8219, 17475, 32771, 69643};

struct Code {
    long m, t, n, k;
    int gSize;
    unsigned long *alog, *log;
    unsigned char *g;
};

// Same construction sequence as src/main.cpp:59-93, calling the reference's own
// findMinimalPolynomial / lcm.
static Code make_code(long m, long t) {
    Code c;
    c.m = m; c.t = t;
    c.n = (1L << m) - 1;
    long n = c.n;
    c.alog = new unsigned long[n];
    c.log = new unsigned long[n + 1];
    c.alog[0] = 1; c.alog[1] = 2;
    c.log[0] = LONG_MAX; c.log[1] = 0; c.log[2] = 1;
    for (unsigned long i = 2; i < (unsigned long)n; ++i) {
        c.alog[i] = c.alog[i - 1] << 1;
        if (c.alog[i] >> m == 1) c.alog[i] ^= kPrim[m - 1];
        c.log[c.alog[i]] = i;
    }
    c.g = new unsigned char[n];
    findMinimalPolynomial(1, (int)m, c.alog, &c.gSize, c.g);
    unsigned char mp[64];
    int mpSize;
    for (unsigned long i = 2; i < (unsigned long)(2 * t); ++i) {
        findMinimalPolynomial((int)i, (int)m, c.alog, &mpSize, mp);
        unsigned char *tmp = lcm(c.g, c.gSize, mp, mpSize, &c.gSize);
        delete[] c.g;
        c.g = tmp;
    }
    c.k = n - c.gSize + 1;
    return c;
}

static void print_bits(const unsigned char *w, long n) {
    for (long i = 0; i < n; ++i) putchar(w[i] ? '1' : '0');
}

static int mode_vectors(long m, long t, unsigned long seed, long count, double snr) {
    Code c = make_code(m, t);
    const long n = c.n, k = c.k;
    generator.seed(seed);
    KanekoKernelProcessor dec(m, n, t, k, c.alog, c.log, 0.5);
    std::vector<unsigned char> info(k), tx(n), out(n);
    std::vector<double> y(n);
    // sigma exactly as src/dataForPlot.cpp:45
    double sd = sqrt(1 / (pow(10, snr / 10) * 2 * dec.getK() / dec.getN()));
    printf("# code %ld %ld %ld %ld gsize %d seed %lu snr %a count %ld\n", n, k, t, m,
           c.gSize, seed, snr, count);
    printf("# g ");
    print_bits(c.g, c.gSize);
    printf("\n");
    for (long w = 0; w < count; ++w) {
        generateRandomPoly(info.data(), k);
        multiplyPolynomials(info.data(), (int)k, c.g, c.gSize, tx.data());
        addNoise(sd, tx.data(), y.data(), n);
        memset(out.data(), 0xFF, n);  // sentinel: res is written only on acceptance
        unsigned long d0 = dec.getDecodingCount(), c0 = dec.getComparisonCount(),
                      s0 = dec.getSummCount();
        dec.decode(tx.data(), y.data(), out.data());
        unsigned long d1 = dec.getDecodingCount(), c1 = dec.getComparisonCount(),
                      s1 = dec.getSummCount();
        int accepted = out[0] != 0xFF;
        double l0 = accepted ? dec.calcL(out.data()) : HUGE_VAL;
        // line: W tx y[0..n-1] res l0 ddec dcmp dsum accepted
        printf("W ");
        print_bits(tx.data(), n);
        for (long i = 0; i < n; ++i) printf(" %a", y[i]);
        printf(" ");
        if (accepted) print_bits(out.data(), n); else printf("-");
        printf(" %a %lu %lu %lu %d\n", l0, d1 - d0, c1 - c0, s1 - s0, accepted);
    }
    return 0;
}

// file <m> <t> <path>: the in/infile.txt format read by src/main.cpp:136-149
// (n chars 0/1, then n doubles), decoded with decode(answer, word, res).
static int mode_file(long m, long t, const char *path) {
    Code c = make_code(m, t);
    const long n = c.n, k = c.k;
    FILE *f = fopen(path, "r");
    if (!f) { fprintf(stderr, "cannot open %s\n", path); return 1; }
    std::vector<unsigned char> tx(n), out(n);
    std::vector<double> y(n);
    for (long i = 0; i < n; ++i) {
        int ch;
        do ch = fgetc(f); while (ch == ' ' || ch == '\n' || ch == '\r' || ch == '\t');
        tx[i] = ch == '1';
    }
    for (long i = 0; i < n; ++i)
        if (fscanf(f, "%lf", &y[i]) != 1) { fprintf(stderr, "short file\n"); return 1; }
    fclose(f);
    KanekoKernelProcessor dec(m, n, t, k, c.alog, c.log, 0.5);
    printf("# code %ld %ld %ld %ld gsize %d file %s\n", n, k, t, m, c.gSize, path);
    memset(out.data(), 0xFF, n);
    dec.decode(tx.data(), y.data(), out.data());
    int accepted = out[0] != 0xFF;
    double l0 = accepted ? dec.calcL(out.data()) : HUGE_VAL;
    printf("W ");
    print_bits(tx.data(), n);
    for (long i = 0; i < n; ++i) printf(" %a", y[i]);
    printf(" ");
    if (accepted) print_bits(out.data(), n); else printf("-");
    printf(" %a %lu %lu %lu %d\n", l0, dec.getDecodingCount(), dec.getComparisonCount(),
           dec.getSummCount(), accepted);
    return 0;
}

// bench <m> <t> <seed> <count> <snr_db>: CPU baseline timing. Generates `count` words of
// the stream first, then times only the decode(answer, word, res) calls (one core).
static int mode_bench(long m, long t, unsigned long seed, long count, double snr) {
    Code c = make_code(m, t);
    const long n = c.n, k = c.k;
    generator.seed(seed);
    KanekoKernelProcessor dec(m, n, t, k, c.alog, c.log, 0.5);
    std::vector<unsigned char> info(k), tx(n * count), out(n);
    std::vector<double> y(n * count);
    double sd = sqrt(1 / (pow(10, snr / 10) * 2 * dec.getK() / dec.getN()));
    for (long w = 0; w < count; ++w) {
        generateRandomPoly(info.data(), k);
        multiplyPolynomials(info.data(), (int)k, c.g, c.gSize, &tx[w * n]);
        addNoise(sd, &tx[w * n], &y[w * n], n);
    }
    long errs = 0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (long w = 0; w < count; ++w) {
        dec.decode(&tx[w * n], &y[w * n], out.data());
        errs += memcmp(out.data(), &tx[w * n], n) != 0;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double el = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    printf("{\"words\": %ld, \"seconds\": %.6f, \"codewords_per_s\": %.3f, \"decodes\": %lu, "
           "\"frame_errors\": %ld}\n", count, el, count / el, dec.getDecodingCount(), errs);
    return 0;
}

static uint64_t splitmix(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static int mode_algdec(long m, long t, const char *what, long count, uint64_t seed) {
    Code c = make_code(m, t);
    const long n = c.n, k = c.k, r = n - k;
    Decoder dec(m, n, t, k, c.alog, c.log);
    std::vector<unsigned char> w(n), ans(n), info(k);
    printf("# algdec %ld %ld %ld %s\n", n, k, t, what);
    auto run = [&]() {
        dec.findSyndromPoly(w.data());
        memset(ans.data(), 0, n);
        bool ok = dec.decode(w.data(), ans.data());
        printf("A ");
        print_bits(w.data(), n);
        printf(" %d ", ok ? 1 : 0);
        if (ok) print_bits(ans.data(), n); else printf("-");
        printf("\n");
    };
    if (!strcmp(what, "exhaustive")) {
        for (uint64_t s = 0; s < (1ULL << r); ++s) {
            for (long i = 0; i < n; ++i) w[i] = (i < r) ? (s >> i) & 1 : 0;
            run();
        }
    } else {
        uint64_t st = seed;
        for (long it = 0; it < count; ++it) {
            for (long i = 0; i < k; ++i) info[i] = splitmix(st) & 1;
            multiplyPolynomials(info.data(), (int)k, c.g, c.gSize, w.data());
            long wt = (long)(splitmix(st) % (uint64_t)(t + 4));
            for (long e = 0; e < wt; ++e) w[splitmix(st) % (uint64_t)n] ^= 1;
            run();
        }
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 7 && !strcmp(argv[1], "vectors"))
        return mode_vectors(atol(argv[2]), atol(argv[3]), strtoul(argv[4], 0, 10),
                            atol(argv[5]), atof(argv[6]));
    if (argc >= 7 && !strcmp(argv[1], "bench"))
        return mode_bench(atol(argv[2]), atol(argv[3]), strtoul(argv[4], 0, 10), atol(argv[5]),
                          atof(argv[6]));
    if (argc >= 5 && !strcmp(argv[1], "file"))
        return mode_file(atol(argv[2]), atol(argv[3]), argv[4]);
    if (argc >= 5 && !strcmp(argv[1], "algdec"))
        return mode_algdec(atol(argv[2]), atol(argv[3]), argv[4],
                           argc > 5 ? atol(argv[5]) : 0,
                           argc > 6 ? strtoull(argv[6], 0, 10) : 1);
    fprintf(stderr, "usage: ref_golden vectors m t seed count snr | algdec m t exhaustive|random count seed\n");
    return 2;
}
