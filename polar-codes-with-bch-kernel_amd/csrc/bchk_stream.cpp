// bchk_stream.cpp -- word boundaries of the reference's input stream without its samples
// (bchk_stream.h), so that a rank of a sharded fun() sweep (src/dataForPlot.cpp:41-95) starts
// its block where the sequential stream would be, without generating the blocks before it.
//
// The stream is one minstd_rand0 sequence; a word is k information draws (src/bchCoder.cpp:
// 236-240) then polar attempts of four draws until ceil(n/2) are accepted (:243-250). Where a
// word starts inside a long stretch of draws is decided by the whole stretch before it -- but
// only through which hypothesis holds at the stretch's end: "j information draws of the current
// word done" or "in an attempt, a pairs accepted, o draws into it". Every hypothesis determines
// where its word ends; following all of them word by word, they merge (two hypotheses that
// reach the same word start are the same from there on). Once one is left, it is the true
// word start, whatever the stretch before held. Two facts keep the set small: word starts
// advance by k + 4 (attempts), so their residue mod 4 moves through the subgroup generated
// by k -- hypotheses outside it are impossible and never merge with the true one -- unless an
// information draw is redrawn, which only the two largest engine values cause, at two
// positions of the whole period, found by a discrete logarithm (Pohlig-Hellman, 2^31 - 2 is
// smooth). A prefix holding one of them is reported unresolved (the caller then parses it).
#include "bchk_stream.h"

#include <algorithm>
#include <set>
#include <vector>

#include "bchk.h"

namespace bchk {

namespace {

uint64_t powmod(uint64_t b, uint64_t e) {
    uint64_t r = 1;
    for (; e; e >>= 1) {
        if (e & 1) r = minstd_mulmod(r, b);
        b = minstd_mulmod(b, b);
    }
    return r;
}

constexpr uint64_t kOrder = kMinstdMod - 1;  // 2 * 3^2 * 7 * 11 * 31 * 151 * 331

// d with 16807^d = h (mod 2^31 - 1); 16807 = 7^5 generates the group (gcd(5, 2^31 - 2) = 1)
uint64_t dlog16807(uint64_t h) {
    static const uint64_t pf[][2] = {{2, 2}, {3, 9}, {7, 7}, {11, 11}, {31, 31}, {151, 151}, {331, 331}};
    uint64_t x = 0, mod = 1;
    for (const auto &f : pf) {
        const uint64_t qe = f[1];
        const uint64_t gq = powmod(kMinstdMul, kOrder / qe), hq = powmod(h, kOrder / qe);
        uint64_t t = 0, acc = 1;
        while (acc != hq && t < qe) {
            acc = minstd_mulmod(acc, gq);
            ++t;
        }
        uint64_t j = 0;  // CRT: x + j mod == t (mod qe)
        while ((x + j * mod) % qe != t % qe) ++j;
        x += j * mod;
        mod *= qe;
    }
    return x % kOrder;
}

}  // namespace

uint64_t stream_skip_word(uint64_t &x, int k, int pairs) {
    static const uint64_t g2 = minstd_mulmod(kMinstdMul, kMinstdMul), g3 = minstd_mulmod(g2, kMinstdMul),
                          g4 = minstd_mulmod(g3, kMinstdMul);
    uint64_t d = 0;
    for (int i = 0; i < k; ++i) {
        do {
            x = minstd_mulmod(x, kMinstdMul);
            ++d;
        } while (!info_draw_ok(x));
    }
    for (int acc = 0; acc < pairs;) {  // the four draws of an attempt, independently from x
        const uint64_t v1 = minstd_mulmod(x, kMinstdMul), v2 = minstd_mulmod(x, g2), v3 = minstd_mulmod(x, g3),
                       v4 = minstd_mulmod(x, g4);
        x = v4;
        d += 4;
        acc += polar_pair_ok(v1, v2, v3, v4) ? 1 : 0;
    }
    return d;
}

}  // namespace bchk

using namespace bchk;

extern "C" {

int bchk_stream_skip(int k, int n, uint64_t state, uint64_t words, uint64_t *state_out, uint64_t *draws) {
    if (k < 1 || n < 1 || n > 4096) return BCHK_EINVAL;
    uint64_t x = Minstd0(state).x, d = 0;
    const int pairs = (n + 1) / 2;
    for (uint64_t w = 0; w < words; ++w) d += stream_skip_word(x, k, pairs);
    if (state_out) *state_out = x;
    if (draws) *draws = d;
    return BCHK_OK;
}

int bchk_stream_sync(int k, int n, uint64_t state, uint64_t offset, uint64_t limit, uint64_t *word_offset,
                     uint64_t *word_state) {
    if (k < 1 || n < 1 || n > 4096 || !word_offset || !word_state) return BCHK_EINVAL;
    const uint64_t x0 = Minstd0(state).x;
    if (offset == 0) {
        *word_offset = 0;
        *word_state = x0;
        return BCHK_OK;
    }
    if (offset >= kOrder / 2 || limit >= kOrder / 2) return BCHK_EINVAL;
    // a redrawn information bit in draws 1..offset would shift the residues: unresolved
    const uint64_t l0 = dlog16807(x0);
    for (uint64_t v : {2147483645ull, 2147483646ull}) {
        uint64_t p = (dlog16807(v) + kOrder - l0) % kOrder;
        if (p == 0) p = kOrder;
        if (p <= offset) return 1;
    }
    const int pairs = (n + 1) / 2;
    const uint64_t step = (k % 4 == 0) ? 4 : ((k % 2 == 0) ? 2 : 1);  // <k> in Z_4
    auto at = [&](uint64_t pos) { return minstd_mulmod(x0, powmod(kMinstdMul, pos % kOrder)); };
    std::set<uint64_t> cand;  // word starts of the hypotheses still apart
    for (int j = 0; j < k; ++j) {  // j information draws of the current word done
        if (offset < (uint64_t)j) break;
        const uint64_t s = offset - (uint64_t)j;
        if ((s % 4) % step) continue;
        uint64_t x = at(s);
        cand.insert(s + stream_skip_word(x, k, pairs));
    }
    for (uint64_t o = 0; o < 4 && o <= offset; ++o) {  // o draws into an attempt; any count so far
        const uint64_t q = offset - o;
        if (q < (uint64_t)k || ((q + 4 - (uint64_t)(k % 4)) % 4) % step) continue;
        uint64_t x = at(q), pos = q;
        static const uint64_t g2 = minstd_mulmod(kMinstdMul, kMinstdMul), g3 = minstd_mulmod(g2, kMinstdMul),
                              g4 = minstd_mulmod(g3, kMinstdMul);
        for (int acc = 0; acc < pairs;) {
            const uint64_t v1 = minstd_mulmod(x, kMinstdMul), v2 = minstd_mulmod(x, g2),
                           v3 = minstd_mulmod(x, g3), v4 = minstd_mulmod(x, g4);
            x = v4;
            pos += 4;
            if (polar_pair_ok(v1, v2, v3, v4)) {
                ++acc;
                cand.insert(pos);  // the word's end if this was its last pair
            }
        }
    }
    while (cand.size() > 1) {  // advance the earliest hypothesis by one word until one is left
        const uint64_t s = *cand.begin();
        if (s >= offset + limit) return 1;
        cand.erase(cand.begin());
        uint64_t x = at(s);
        cand.insert(s + stream_skip_word(x, k, pairs));
    }
    const uint64_t c = *cand.begin();
    if (c >= offset + limit) return 1;
    *word_offset = c;
    *word_state = at(c);
    return BCHK_OK;
}

}  // extern "C"
