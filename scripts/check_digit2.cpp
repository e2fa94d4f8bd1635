// Exhaustive check of Digit2 (tfhe-rs-odd_amd/csrc/pbs_common.h): for every 32-bit hi word and
// beta = 1..15 the two int16 digits of the short form equal decomp_state32<2> + two decomp_digit32
// (the SignedDecomposer's digits, decomposer.rs:99-119 / iter.rs:134-141); and DigitL1, the one-level
// 3-op digit, against decomp_state32<1> + decomp_digit32 for beta = 1..30.
//   g++ -O3 -fopenmp scripts/check_digit2.cpp -o /tmp/check_digit2 && /tmp/check_digit2   (~30 s on 8 cores)
//   /tmp/check_digit2 24   : 2^24 evenly spread hi words per beta instead (tests/test_digit2.py)
#include <cstdint>
#include <cstdlib>
#include <cstdio>
static inline int32_t dig(uint32_t &state, int beta, uint32_t mask) {
    uint32_t res = state & mask; state >>= beta;
    uint32_t carry = ((res - 1) | state) & res; carry >>= beta - 1; state += carry;
    return (int32_t)(res - (carry << beta));
}
int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 32;  // 2^lg hi words per beta
    long bad = 0;
    for (int beta = 1; beta <= 15; beta++) {
        const uint32_t mask = (1u << beta) - 1, hm1 = (1u << (beta - 1)) - 1, k1 = 1u << (31 - 2 * beta);
        const int s0 = 32 - 2 * beta, s1 = 32 - beta;
        long bb = 0;
        #pragma omp parallel for reduction(+:bb)
        for (long xl = 0; xl < (1l << lg); xl++) {
            const uint32_t xh = (uint32_t)((xl << (32 - lg)) | (xl & ((1l << (32 - lg)) - 1)));
            uint32_t st = ((xh >> (31 - 2 * beta)) + 1) >> 1;
            int32_t r0 = dig(st, beta, mask), r1 = dig(st, beta, mask);
            uint32_t y = xh + k1;
            uint32_t a = (y >> s0) & mask, t = y >> 31, z0 = a + t + hm1, c = (z0 >> beta) & 1;
            int32_t d0 = (int32_t)a - (int32_t)(c << beta);
            uint32_t z1 = (y >> s1) + c + hm1;
            int32_t d1 = (int32_t)(z1 & mask) - (int32_t)hm1;
            if ((uint16_t)d0 != (uint16_t)r0 || (uint16_t)d1 != (uint16_t)r1) bb++;
        }
        printf("beta %d mismatches %ld\n", beta, bb); fflush(stdout);
        bad += bb;
    }
    // DigitL1 (one level, beta = 1..30): ((x_hi + ((2^beta - 1) << (31 - beta))) >> (32 - beta)) - (2^(beta-1) - 1)
    for (int beta = 1; beta <= 30; beta++) {
        const uint32_t mask = (1u << beta) - 1, ck = ((1u << beta) - 1) << (31 - beta);
        const int sh = 32 - beta;
        const int32_t h = (int32_t)(1u << (beta - 1)) - 1;
        long bb = 0;
        #pragma omp parallel for reduction(+:bb)
        for (long xl = 0; xl < (1l << lg); xl++) {
            const uint32_t xh = (uint32_t)((xl << (32 - lg)) | (xl & ((1l << (32 - lg)) - 1)));
            uint32_t st = ((xh >> (31 - beta)) + 1) >> 1;
            const int32_t r0 = dig(st, beta, mask);
            if ((int32_t)((xh + ck) >> sh) - h != r0) bb++;
        }
        printf("L1 beta %d mismatches %ld\n", beta, bb); fflush(stdout);
        bad += bb;
    }
    return bad != 0;
}
