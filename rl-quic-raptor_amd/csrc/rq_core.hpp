// rq_core.hpp -- RaptorQ parameters, Rand, LT tuples and GF(256) for the rqhip engine.
//
// Behaviour follows github.com/xssnick/raptorq v1.1.0 as used by go/fec/raptorq_wrap.go
// (SURVEY.md Appendix A):
//   calcParams      RQ/params.go:31-61, RQ/raw-params.go:14-19, isPrime RQ/params.go:193-207
//                   (P1 = smallest prime STRICTLY greater than P -- the library's quirk)
//   Rand            RQ/rand.go:25-31
//   getDegree       RQ/params.go:71-80
//   calcEncodingRow RQ/params.go:83-112
//   LT columns      RQ/params.go:140-160 (matrix rows) == RQ/params.go:162-182 (encodeGen)
//   GF(256)         RQ/discmath/oct.go:41-66 (poly 0x11D, alpha = 2)
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

#include "rfc6330_tables.h"

namespace rq {

struct Params {
    uint32_t K, Kp, J, S, H, W, L, P, P1, U, B;
};

enum Err : int {
    ERR_OK = 0,
    ERR_SYMBOL_SIZE_ZERO = -1,      // "symbol size cannot be zero"
    ERR_K_TOO_BIG = -2,             // "k is too big"
};

inline bool is_prime(uint32_t n) {
    if (n <= 3) return true;
    if (n % 2 == 0 || n % 3 == 0) return false;
    for (uint64_t i = 5; i * i <= n; i += 6)
        if (n % i == 0 || n % (i + 2) == 0) return false;
    return true;
}

// Parameters for the smallest table row with K' >= K (K = ceil(size / T)).
inline int params_for_K(uint64_t K, Params* p) {
    const uint32_t* row = nullptr;
    for (int i = 0; i < RQ_NUM_SYSTEMATIC; ++i)
        if (RQ_SYSTEMATIC[i][0] >= K) { row = RQ_SYSTEMATIC[i]; break; }
    if (!row) return ERR_K_TOO_BIG;
    p->K = (uint32_t)K;
    p->Kp = row[0]; p->J = row[1]; p->S = row[2]; p->H = row[3]; p->W = row[4];
    p->L = p->Kp + p->S + p->H;
    p->B = p->W - p->S;
    p->P = p->L - p->W;
    p->U = p->P - p->H;
    p->P1 = p->P + 1;
    while (!is_prime(p->P1)) ++p->P1;
    return ERR_OK;
}

inline int calc_params(uint64_t size, uint32_t T, Params* p) {
    if (T == 0) return ERR_SYMBOL_SIZE_ZERO;
    return params_for_K((size + T - 1) / T, p);
}

inline uint32_t rand_(uint32_t y, uint32_t i, uint32_t m) {
    return (RQ_V0[(y + i) & 255u] ^ RQ_V1[((y >> 8) + i) & 255u] ^
            RQ_V2[((y >> 16) + i) & 255u] ^ RQ_V3[((y >> 24) + i) & 255u]) % m;
}

struct Tuple { uint32_t d, a, b, d1, a1, b1; };

inline Tuple tuple_of(const Params& p, uint32_t X) {
    uint32_t A = 53591u + 997u * p.J;
    if ((A & 1u) == 0) ++A;
    const uint32_t y = 10267u * (p.J + 1u) + X * A;
    const uint32_t v = rand_(y, 0, 1u << 20);
    uint32_t d = 0;
    for (uint32_t i = 0; i < 31; ++i)
        if (v < RQ_DEGREE_F[i]) { d = i; break; }
    if (d > p.W - 2) d = p.W - 2;
    Tuple t;
    t.d = d;
    t.a = 1 + rand_(y, 1, p.W - 1);
    t.b = rand_(y, 2, p.W);
    t.d1 = d < 4 ? 2 + rand_(X, 3, 2) : 2;
    t.a1 = 1 + rand_(X, 4, p.P1 - 1);
    t.b1 = rand_(X, 5, p.P1);
    return t;
}

// Columns of the intermediate-symbol vector combined for ISI X.  Returns the count (<= 64).
inline int lt_cols(const Params& p, uint32_t X, uint32_t* cols) {
    const Tuple t = tuple_of(p, X);
    uint32_t b = t.b, b1 = t.b1;
    int n = 0;
    cols[n++] = b;
    for (uint32_t j = 1; j < t.d; ++j) { b = (b + t.a) % p.W; cols[n++] = b; }
    while (b1 >= p.P) b1 = (b1 + t.a1) % p.P1;
    cols[n++] = p.W + b1;
    for (uint32_t j = 1; j < t.d1; ++j) {
        b1 = (b1 + t.a1) % p.P1;
        while (b1 >= p.P) b1 = (b1 + t.a1) % p.P1;
        cols[n++] = p.W + b1;
    }
    return n;
}

// ---------------------------------- GF(256) -------------------------------------------
struct GF {
    uint8_t exp[512];
    uint8_t log[256];
    GF() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)x; log[x] = (uint8_t)i;
            x <<= 1; if (x & 0x100) x ^= 0x11D;
        }
        for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
        log[0] = 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
    uint8_t inv(uint8_t a) const { return exp[255 - log[a]]; }
    uint8_t pow_alpha(uint32_t e) const { return exp[e % 255]; }
};
const GF& gf();

}  // namespace rq
