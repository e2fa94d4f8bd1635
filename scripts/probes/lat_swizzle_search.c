// Exhaustive search for an XOR swizzle of the latency kernel's exchange buffers (pbs_latency.hip,
// LAT_MAP = 1 lane mapping): slot(P) = P ^ f(P >> 4) with f a linear map of bits 4..9 onto bits
// 0..3 (4 x 6 GF(2) matrix, 2^24 candidates).  A candidate is accepted when every access pattern
// of a wave is free of bank conflicts for both ds_read_b128's 16-lane groups (16-byte slot =
// P' mod 16) and ds_write_b128's 8-lane groups (P' mod 8):
//   (i)   stage 1:  P = w + 4 col + 64 lrow + 256 q
//   (ii)  stage 2:  P = 64 col + w + 4 lrow + 16 q
//   (iii) MAC / inverse stage 3 blocks: P = 256 w + 64 (col & 3) + 4 lrow + 16 (col >> 2) + e
// (lane = 16 lrow + col; w = wave quarter, q and e the per-instruction constant).
// Build: gcc -O2 -o /tmp/lat_swz lat_swizzle_search.c
#include <stdio.h>

static const int rd_groups[4][16] = {
    {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
    {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
    {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
    {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};

static int pos(int pat, int lane, int w, int k) {
    const int lrow = lane >> 4, col = lane & 15;
    if (pat == 0) return w + 4 * col + 64 * lrow + 256 * k;
    if (pat == 1) return 64 * col + w + 4 * lrow + 16 * k;
    return 256 * w + 64 * (col & 3) + 4 * lrow + 16 * (col >> 2) + k;
}

// bits 0..2 ^= G (bits 3..9), bit 3 ^= H (bits 4..9): a bijection (each XOR reads only bits above
// the ones it changes)
static unsigned gcol[7], hrow;
static int swz(int P) {
    int f = 0;
    for (int j = 0; j < 7; j++)
        if ((P >> (3 + j)) & 1) f ^= gcol[j];
    f |= (__builtin_popcount((unsigned)(P >> 4) & hrow) & 1) << 3;
    return P ^ f;
}

static int ok(void) {
    for (int pat = 0; pat < 3; pat++)
        for (int w = 0; w < 4; w++)
            for (int k = 0; k < 4; k++) {
                int s[64];
                for (int l = 0; l < 64; l++) s[l] = swz(pos(pat, l, w, k));
                for (int g = 0; g < 4; g++) {  // reads: 16 distinct slots mod 16
                    int used = 0;
                    for (int t = 0; t < 16; t++) {
                        const int b = 1 << (s[rd_groups[g][t]] & 15);
                        if (used & b) return 0;
                        used |= b;
                    }
                }
                for (int g = 0; g < 8; g++) {  // writes: 8 contiguous lanes, distinct mod 8
                    int used = 0;
                    for (int t = 0; t < 8; t++) {
                        const int b = 1 << (s[8 * g + t] & 7);
                        if (used & b) return 0;
                        used |= b;
                    }
                }
            }
    return 1;
}

int main(void) {
    long found = 0;
    for (unsigned long m = 0; m < (1ul << 27); m++) {
        for (int j = 0; j < 7; j++) gcol[j] = (m >> (3 * j)) & 7;
        hrow = (m >> 21) & 63;
        if (ok()) {
            if (found < 40) {
                printf("found:");
                for (int j = 0; j < 7; j++) printf(" b%d->%x", 3 + j, gcol[j]);
                printf(" h=%02x (bits 4..9)\n", hrow);
            }
            found++;
        }
    }
    printf("total %ld\n", found);
    return 0;
}
