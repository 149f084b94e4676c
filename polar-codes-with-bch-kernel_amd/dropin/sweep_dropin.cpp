// Drop-in fun() (include/bchk_dropin/dataForPlot.h): the reference's Monte-Carlo FER sweep
// (src/dataForPlot.cpp:16-116) run batched on the GPU through bchk_sweep. It consumes the
// shared global stream exactly as the reference loop would, writes `file`.csv with the
// same rows, prints the same progress lines, and leaves the counters reset.
#include <clocale>
#include <ctime>
#include <fstream>
#include <iostream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "KanekoKernelProcessor.h"
#include "bchk.h"
#include "dataForPlot.h"

extern std::default_random_engine generator;  // bchcoder_dropin.cpp

void fun(const std::string &file, KanekoKernelProcessor &decoder, const unsigned char *,
         unsigned long, long p, long e, double maxSTNR) {
    setlocale(LC_ALL, "Russian");
    std::ofstream fout(file + ".csv");
    const clock_t start = clock();
    uint64_t state = 0;
    {
        std::stringstream ss;
        ss << generator;
        ss >> state;
    }
    std::vector<char> csv(1 << 16);
    if (bchk_sweep(decoder.context(), p, e, maxSTNR, &state, 1, 0, csv.data(), csv.size()) != 0)
        throw bchk_last_error();
    {
        std::stringstream ss;
        ss << state;
        ss >> generator;
    }
    fout << csv.data();
    for (double stnr = 0.0; stnr <= maxSTNR; stnr += 0.5) std::cout << stnr << "\n";
    decoder.setDecodingCount();
    decoder.setComparisonCount();
    decoder.setSummCount();
    const clock_t end = clock();
    std::cout << "Общее время: " << ((double)end - start) / (double)CLOCKS_PER_SEC << " секунд\n";
    fout.close();
}
