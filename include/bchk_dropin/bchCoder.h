// bchk drop-in for the reference's headers/bchCoder.h: binary polynomial algebra, code
// construction, the random word / AWGN stream, and printing helpers. Declarations follow
// headers/bchCoder.h:10-48; the stream uses the same standard-library engine and
// distributions (src/bchCoder.cpp:14-22), so words and noise are identical.
#ifndef BCHK_DROPIN_BCHCODER_H
#define BCHK_DROPIN_BCHCODER_H

#include <algorithm>
#include <fstream>

void findMinimalPolynomial(int i, int power, const unsigned long *fieldElements, int *size,
                           unsigned char *res);

bool comparePoly(const unsigned char *poly1, int size1, const unsigned char *poly2, int size2);

unsigned char *multiplyPolynomials(const unsigned char *first, int size1,
                                   const unsigned char *second, int size2,
                                   int *sizeRes = nullptr);

void multiplyPolynomials(const unsigned char *first, int size1, const unsigned char *second,
                         int size2, unsigned char *res, int *sizeRes = nullptr);

unsigned char *dividePolynomial(const unsigned char *first, int size1,
                                const unsigned char *second, int size2, int *size,
                                bool needRemainder);

unsigned char *lcm(const unsigned char *first, int size1, const unsigned char *second,
                   int size2, int *sizeRes);

unsigned char *generateRandomPoly(long k);

void generateRandomPoly(unsigned char *res, long k);

void addNoise(double standartDeviation, const unsigned char *codeword, double *wordWithNoise,
              unsigned long n);

void printVec(const unsigned char *poly, int size);

void printVec(const unsigned long *poly, int size);

void printVec(const double *poly, int size);

void printVec(std::ofstream &out, const unsigned char *poly, int size);

void printVec(std::ofstream &out, const double *poly, int size);

void printMatrix(unsigned char **const matrix, int sizeI, int sizeJ = -1);

void printMatrix(std::ofstream &out, unsigned char **const matrix, int sizeI, int sizeJ = -1);

void makeMatrix(int power, const unsigned long *fieldElements, unsigned char **matrix);

#endif
