// bchk drop-in for the reference's headers/dataForPlot.h: the Monte-Carlo FER sweep,
// batched on the GPU (bchk_sweep) with the reference's stream, stopping rule, quirks and
// CSV format (src/dataForPlot.cpp:16-116).
#ifndef BCHK_DROPIN_DATAFORPLOT_H
#define BCHK_DROPIN_DATAFORPLOT_H

#include <string>

class KanekoKernelProcessor;

void fun(const std::string &file, KanekoKernelProcessor &decoder, const unsigned char *g,
         unsigned long gSize, long p, long e, double maxSTNR = 5.0);

#endif
