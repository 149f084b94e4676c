// bchk drop-in for the reference's headers/Decoder.h (algebraic BCH decoder).
//
// Public interface of headers/Decoder.h:67-78. Syndromes are kept on the host exactly as
// the reference keeps them (findSyndromPoly / alterSyndromPoly, src/Decoder.cpp:184-230);
// decode() hands the stored syndromes and the word to the GPU (bchk_alg_decode_host),
// which solves the key equation and searches the roots (src/Decoder.cpp:233-321).
#ifndef BCHK_DROPIN_DECODER_H
#define BCHK_DROPIN_DECODER_H

#include <vector>

struct bchk_ctx;

class Decoder {
public:
    Decoder(long pw, long n, long t, long k, unsigned long *antilogarithms,
            unsigned long *logarithms);
    ~Decoder();
    Decoder(const Decoder &) = delete;
    Decoder &operator=(const Decoder &) = delete;

    void findSyndromPoly(const unsigned char *word);
    void alterSyndromPoly(const unsigned char *word);
    bool decode(const unsigned char *word, unsigned char *answer);
    long getN() const;
    long getT() const;
    long getK() const;

    // S_1 .. S_2t (index j-1), and one past the last nonzero entry, as the reference.
    unsigned long *syndromPoly;
    long syndromPolySize;

private:
    void refreshSize();

    bchk_ctx *ctx_ = nullptr;
    long power_, n_, t_, k_;
    const unsigned long *alog_;
    std::vector<unsigned char> last_;
    std::vector<unsigned int> odd_;
};

#endif
