// Drop-in bchCoder functions (include/bchk_dropin/bchCoder.h): binary polynomial algebra
// over GF(2), minimal polynomials over GF(2^m), the reference's random stream, printing.
// Host-side set-up and I/O only; nothing here is on the decode path.
#include <cstring>
#include <iostream>
#include <random>
#include <vector>

#include "bchCoder.h"

// The reference's stream objects, same names and types (src/bchCoder.cpp:19-22): a
// default-seeded std::default_random_engine and a 0/1 uniform_int_distribution.
std::default_random_engine generator;
std::uniform_int_distribution<unsigned short> distribution(0, 1);

namespace {

int degree(const unsigned char *p, int size) {
    for (int d = size - 1; d >= 0; --d)
        if (p[d]) return d;
    return -1;
}

// long division over GF(2): quotient q (size s1-s2+1) and remainder r (size s1) of a / b
void divmod2(const unsigned char *a, int s1, const unsigned char *b, int s2,
             std::vector<unsigned char> &q, std::vector<unsigned char> &r) {
    r.assign(a, a + s1);
    q.assign(s1 >= s2 ? s1 - s2 + 1 : 1, 0);
    const int db = degree(b, s2);
    if (db < 0) return;
    for (int d = degree(r.data(), s1); d >= db; d = degree(r.data(), s1)) {
        q[d - db] = 1;
        for (int i = 0; i <= db; ++i) r[d - db + i] ^= b[i];
    }
}

}  // namespace

// Minimal polynomial of alpha^i (src/bchCoder.cpp:25-91): prod over the conjugates
// alpha^(i 2^j) of (x + alpha^(i 2^j)), computed in GF(2^power) from the antilog table.
void findMinimalPolynomial(int i, int power, const unsigned long *fieldElements, int *size,
                           unsigned char *res) {
    const int n = (1 << power) - 1;
    std::vector<int> lg(n + 1, -1);
    for (int e = 0; e < n; ++e) lg[fieldElements[e]] = e;
    auto mul = [&](unsigned long a, unsigned long b) -> unsigned long {
        if (!a || !b) return 0;
        return fieldElements[(lg[a] + lg[b]) % n];
    };
    std::vector<unsigned long> mp{1};
    int e = i % n;
    do {
        const unsigned long root = fieldElements[e];
        std::vector<unsigned long> nx(mp.size() + 1, 0);
        for (size_t d = 0; d < mp.size(); ++d) {
            nx[d + 1] ^= mp[d];
            nx[d] ^= mul(mp[d], root);
        }
        mp.swap(nx);
        e = (2 * e) % n;
    } while (e != i % n);
    *size = (int)mp.size();
    for (size_t d = 0; d < mp.size(); ++d) res[d] = (unsigned char)(mp[d] % 2);
}

bool comparePoly(const unsigned char *a, int s1, const unsigned char *b, int s2) {
    return s1 == s2 && std::memcmp(a, b, (size_t)s1) == 0;
}

void multiplyPolynomials(const unsigned char *a, int s1, const unsigned char *b, int s2,
                         unsigned char *res, int *sizeRes) {
    std::memset(res, 0, (size_t)(s1 + s2 - 1));
    for (int i = 0; i < s1; ++i)
        if (a[i])
            for (int j = 0; j < s2; ++j) res[i + j] ^= b[j];
    if (sizeRes) *sizeRes = s1 + s2 - 1;
}

unsigned char *multiplyPolynomials(const unsigned char *a, int s1, const unsigned char *b, int s2,
                                   int *sizeRes) {
    unsigned char *res = new unsigned char[s1 + s2 - 1];
    multiplyPolynomials(a, s1, b, s2, res, sizeRes);
    return res;
}

// src/bchCoder.cpp:134-184: remainder trimmed to its degree (size >= 1), or the quotient
// of size s1 - s2 + 1.
unsigned char *dividePolynomial(const unsigned char *a, int s1, const unsigned char *b, int s2,
                                int *size, bool needRemainder) {
    std::vector<unsigned char> q, r;
    divmod2(a, s1, b, s2, q, r);
    if (needRemainder) {
        const int d = degree(r.data(), s1);
        *size = d < 0 ? 1 : d + 1;
        unsigned char *out = new unsigned char[*size];
        for (int i = 0; i < *size; ++i) out[i] = r[i];
        return out;
    }
    *size = s1 - s2 + 1;
    unsigned char *out = new unsigned char[*size];
    for (int i = 0; i < *size; ++i) out[i] = q[i];
    return out;
}

// lcm(a, b) = a b / gcd(a, b) (src/bchCoder.cpp:186-226)
unsigned char *lcm(const unsigned char *a, int s1, const unsigned char *b, int s2, int *sizeRes) {
    std::vector<unsigned char> x(a, a + s1), y(b, b + s2), q, r;
    while (degree(y.data(), (int)y.size()) >= 0) {
        divmod2(x.data(), (int)x.size(), y.data(), (int)y.size(), q, r);
        const int d = degree(r.data(), (int)r.size());
        x.swap(y);
        y.assign(r.begin(), r.begin() + (d < 0 ? 1 : d + 1));
    }
    const int dg = degree(x.data(), (int)x.size());
    std::vector<unsigned char> prod(s1 + s2 - 1, 0);
    multiplyPolynomials(a, s1, b, s2, prod.data());
    divmod2(prod.data(), (int)prod.size(), x.data(), dg + 1, q, r);
    *sizeRes = (int)prod.size() - dg;
    unsigned char *out = new unsigned char[*sizeRes];
    for (int i = 0; i < *sizeRes; ++i) out[i] = q[i];
    return out;
}

unsigned char *generateRandomPoly(long k) {
    unsigned char *res = new unsigned char[k];
    generateRandomPoly(res, k);
    return res;
}

void generateRandomPoly(unsigned char *res, long k) {
    for (long i = 0; i < k; ++i) res[i] = (unsigned char)distribution(generator);
}

// y_i = (c_i ? 1 : -1) + N(0, sd^2), a fresh normal_distribution per call (:243-250)
void addNoise(double sd, const unsigned char *codeword, double *y, unsigned long n) {
    std::normal_distribution<double> noise(0.0, sd);
    for (unsigned long i = 0; i < n; ++i) y[i] = (codeword[i] ? 1 : -1) + noise(generator);
}

void printVec(const unsigned char *p, int size) {
    for (int i = 0; i < size; ++i) std::cout << (p[i] ? 1 : 0) << ' ';
    std::cout << std::endl;
}
void printVec(const unsigned long *p, int size) {
    for (int i = 0; i < size; ++i) std::cout << p[i] << ' ';
    std::cout << std::endl;
}
void printVec(const double *p, int size) {
    for (int i = 0; i < size; ++i) std::cout << p[i] << ' ';
    std::cout << std::endl;
}
void printVec(std::ofstream &out, const unsigned char *p, int size) {
    for (int i = 0; i < size; ++i) out << (p[i] ? 1 : 0) << ' ';
    out << std::endl;
}
void printVec(std::ofstream &out, const double *p, int size) {
    for (int i = 0; i < size; ++i) out << p[i] << ' ';
    out << std::endl;
}

template <class Out>
static void print_matrix(Out &out, unsigned char **const m, int rows, int cols) {
    if (cols == -1) cols = rows;
    for (int i = 0; i < rows; ++i) {
        for (int j = 0; j < cols; ++j) out << (m[i][j] ? 1 : 0) << ' ';
        out << std::endl;
    }
    out << std::endl;
}
void printMatrix(unsigned char **const m, int rows, int cols) { print_matrix(std::cout, m, rows, cols); }
void printMatrix(std::ofstream &out, unsigned char **const m, int rows, int cols) {
    print_matrix(out, m, rows, cols);
}

// The nested-BCH kernel matrix of src/bchCoder.cpp:317-345 (used by the un-built
// src/matrixMain.cpp): row deg(g)-1 of each growing generator g = lcm(M_2, ..., M_i) holds
// g, the rows in between hold shifts of the previous generator; row 0 is [1, 0, ...].
void makeMatrix(int power, const unsigned long *fieldElements, unsigned char **matrix) {
    const int len = (1 << power) - 1;
    const int amount = ((1 << power) - 2) / 2;
    for (int i = 0; i < len; ++i) std::memset(matrix[i], 0, (size_t)len);
    matrix[0][0] = 1;
    std::vector<unsigned char> g(len, 0), poly(power + 2);
    g[0] = 1;
    int gOld = 1;
    for (int i = 2; i <= amount; ++i) {
        int ps = 0;
        findMinimalPolynomial(i, power, fieldElements, &ps, poly.data());
        if (gOld >= ps) {
            int rs = 0;
            unsigned char *rem = dividePolynomial(g.data(), gOld, poly.data(), ps, &rs, true);
            const bool divides = !rem[0] && rs == 1;
            delete[] rem;
            if (divides) continue;
        }
        const int gNew = ps + gOld - 1;
        multiplyPolynomials(poly.data(), ps, g.data(), gOld, matrix[gNew - 1]);
        for (int j = gOld, shift = 1; j < gNew - 1; ++j, ++shift)
            for (int kk = shift; kk < shift + gOld; ++kk) matrix[j][kk] = g[kk - shift];
        std::memcpy(g.data(), matrix[gNew - 1], (size_t)gNew);
        gOld = gNew;
    }
}
