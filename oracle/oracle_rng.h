/*
 * TEST INFRASTRUCTURE ONLY — part of the CPU oracle (see oracle/README.md).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * the oracle.  The product never includes or links anything under oracle/.
 *
 * Counter-based RNG of the parity mode: Philox4x32-10 (Salmon et al., SC'11,
 * "Parallel random numbers: as easy as 1, 2, 3"), pinned by the Random123
 * known-answer vectors in tests/test_oracle_primitives.py.  Key derivation,
 * counter layout and the truncated-normal sampler are specified in DESIGN.md
 * §RNG and re-implemented independently in the HIP kernel.
 */
#ifndef FKS_ORACLE_RNG_H
#define FKS_ORACLE_RNG_H

#include <stdint.h>

namespace oracle {

struct Philox4 {
    uint32_t v[4];
};

inline void mulhilo32(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
    const uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    *lo = (uint32_t)p;
}

/* Philox4x32 with 10 rounds */
inline Philox4 philox4x32_10(Philox4 ctr, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    for (int round = 0; round < 10; ++round) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo32(M0, ctr.v[0], &hi0, &lo0);
        mulhilo32(M1, ctr.v[2], &hi1, &lo1);
        Philox4 next;
        next.v[0] = hi1 ^ ctr.v[1] ^ k0;
        next.v[1] = lo1;
        next.v[2] = hi0 ^ ctr.v[3] ^ k1;
        next.v[3] = lo0;
        ctr = next;
        k0 += W0;
        k1 += W1;
    }
    return ctr;
}

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

/* stream key of one forward-simulation call */
inline uint64_t call_key(uint64_t seed, uint64_t call_index) {
    return splitmix64(seed ^ splitmix64(call_index));
}

/* [0,1) double from two 32-bit words (53 random bits) */
inline double u53(uint32_t a, uint32_t b) {
    const uint64_t bits = (((uint64_t)a << 32) | (uint64_t)b) >> 11;
    return (double)bits * (1.0 / 9007199254740992.0);
}

}  // namespace oracle

#endif
