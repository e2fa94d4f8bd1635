/*
 * pbs_oracle.c -- CPU restatement of the tfhe-rs-odd (tfhe 0.5.0 fork) classic PBS hot path.
 *
 *   *** TEST INFRASTRUCTURE ONLY ***
 *   Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 *   library, and only as the checker / the timed CPU baseline.  The product
 *   (tfhe-rs-odd_amd/, libtfhe_mi355.so) never links, loads or calls it.
 *
 * Parity status (see DESIGN.md section "Oracle"):
 *   - integer paths (decomposer, keyswitch, modulus switch, rotations, sample extract, LUT)
 *     restate the reference exactly and are pinned by the reference's own known-answer
 *     tests (decomposer.rs:95-96, term.rs:48,144, fft/tests.rs:244-300);
 *   - the FFT butterflies live in the absent third-party crate concrete-fft 0.3.0 whose plan
 *     is picked at run time (fft/mod.rs:159-162), so ciphertext bits are "parity unpinned"
 *     against the reference at the FFT boundary; the restatement pins itself to the
 *     reference's FFT tolerance test (fft/tests.rs:82-222) and to decryption round trips
 *     (test/lwe_programmable_bootstrapping.rs:70-166).  The GPU engine is required to be
 *     bit-exact against THIS restatement (same butterfly DAG, see DESIGN.md "FFT spec").
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off; every fused multiply-add is an
 * explicit fma()).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    double re, im;
} cplx;

/* ------------------------------------------------------------------------------------ */
/* PRNG (harness only; the reference uses concrete-csprng AES-CTR, which is not needed:  */
/* key/ciphertext values never need to match the reference's bits).                      */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    uint64_t s[4];
} orc_rng;

static uint64_t splitmix64(uint64_t *x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void rng_seed(orc_rng *r, uint64_t seed, uint64_t stream) {
    uint64_t x = seed ^ (stream * 0xD1B54A32D192ED03ULL);
    for (int i = 0; i < 4; i++) r->s[i] = splitmix64(&x);
}

static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

static uint64_t rng_next(orc_rng *r) { /* xoshiro256** */
    uint64_t *s = r->s;
    uint64_t result = rotl64(s[1] * 5, 7) * 9;
    uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl64(s[3], 45);
    return result;
}

/* f64 -> i64 by bit twiddling, fft/math/fft/tests.rs:244-300 and x86.rs:28-81
 * (mm256_cvtpd_epi64).  Exact (truncating) for |x| < 2^64, wraps 2^63 to -2^63. */
int64_t orc_f64_to_i64(double x) {
    uint64_t bits;
    memcpy(&bits, &x, 8);
    uint64_t mant = (bits & 0xFFFFFFFFFFFFFULL) | 0x10000000000000ULL;
    uint64_t biased_exp = (bits >> 52) & 0x7FF;
    uint64_t sign = bits >> 63;
    uint64_t lshift = mant << 11;
    uint64_t rs = 1086 - biased_exp;
    uint64_t v = rs < 64 ? (lshift >> rs) : 0;
    if (biased_exp == 0) v = 0;
    return sign ? (int64_t)(0 - v) : (int64_t)v;
}

/* Torus <-> f64, commons/math/torus/mod.rs:71-78 (from_torus; F::round = half away). */
static uint64_t from_torus(double x) {
    double fract = x - round(x);
    fract *= 18446744073709551616.0;
    fract = round(fract);
    return (uint64_t)orc_f64_to_i64(fract);
}

/* Gaussian by Marsaglia polar, commons/math/random/gaussian.rs:15-52. */
static void gaussian_pair(orc_rng *r, double std, double *a, double *b) {
    for (;;) {
        double u = (double)(int64_t)rng_next(r) * 0x1p-63;
        double v = (double)(int64_t)rng_next(r) * 0x1p-63;
        double s = u * u + v * v;
        if (s > 0.0 && s < 1.0) {
            double cst = std * sqrt(-2.0 * log(s) / s);
            *a = u * cst;
            *b = v * cst;
            return;
        }
    }
}

static uint64_t gaussian_torus(orc_rng *r, double std) {
    double a, b;
    gaussian_pair(r, std, &a, &b);
    return from_torus(a);
}

/* ------------------------------------------------------------------------------------ */
/* Decomposer: commons/math/decomposition/decomposer.rs:99-119 (closest_representable),   */
/* iter.rs:134-141 (decompose_one_level), fft64/math/decomposition.rs:79-86.              */
/* ------------------------------------------------------------------------------------ */
uint64_t orc_closest_representable(uint64_t x, int base_log, int level) {
    int non_rep = 64 - base_log * level;
    int shift = non_rep - 1;
    uint64_t res = x >> shift;
    res += 1;
    res &= ~(uint64_t)1;
    return res << shift;
}

static inline uint64_t decompose_one_level(int base_log, uint64_t *state, uint64_t mask) {
    uint64_t res = *state & mask;
    *state >>= base_log;
    uint64_t carry = ((res - 1) | *state) & res;
    carry >>= base_log - 1;
    *state += carry;
    return res - (carry << base_log);
}

/* Writes the signed digits (as wrapping u64) in iterator order: out[0] is the term of level
 * `level` (least significant), out[level-1] the term of level 1 (decomposer.rs:145-153). */
void orc_decompose(uint64_t x, int base_log, int level, uint64_t *out) {
    uint64_t state = orc_closest_representable(x, base_log, level) >> (64 - base_log * level);
    uint64_t mask = (1ULL << base_log) - 1;
    for (int l = 0; l < level; l++) out[l] = decompose_one_level(base_log, &state, mask);
}

/* ------------------------------------------------------------------------------------ */
/* FFT spec (DESIGN.md "FFT spec"): negacyclic real FFT of size N as a complex FFT of      */
/* M = N/2 points on x[j] + i x[j+M] twisted by w_j = exp(i pi j / N)                    */
/* (fft/mod.rs:30-70, 197-326).  The complex FFT is an in-place mixed-radix DIF whose     */
/* output stays in "position" order (like concrete-fft's unordered plan); the inverse is  */
/* the mirrored DIT.  Every butterfly below is written op-for-op as the GPU kernels do.   */
/* ------------------------------------------------------------------------------------ */
#define C16_1 0x1.d906bcf328d46p-1 /* cos(pi/8) */
#define S16_1 0x1.87de2a6aea963p-2 /* sin(pi/8) */
#define SQH 0x1.6a09e667f3bcdp-1   /* sqrt(1/2) */

static inline cplx cadd(cplx a, cplx b) { return (cplx){a.re + b.re, a.im + b.im}; }
static inline cplx csub(cplx a, cplx b) { return (cplx){a.re - b.re, a.im - b.im}; }
/* general twiddle product: (fma(xr,wr,-(xi*wi)), fma(xr,wi,xi*wr)) */
static inline cplx cmulw(cplx x, double wr, double wi) {
    return (cplx){fma(x.re, wr, -(x.im * wi)), fma(x.re, wi, x.im * wr)};
}
/* x * exp(-i pi/4) */
static inline cplx mul_w8(cplx x) { return (cplx){(x.re + x.im) * SQH, (x.im - x.re) * SQH}; }
/* x * exp(-3 i pi/4) */
static inline cplx mul_w8_3(cplx x) { return (cplx){(x.im - x.re) * SQH, -((x.re + x.im) * SQH)}; }
/* x * exp(+i pi/4) */
static inline cplx mul_w8c(cplx x) { return (cplx){(x.re - x.im) * SQH, (x.re + x.im) * SQH}; }
/* x * exp(+3 i pi/4) */
static inline cplx mul_w8_3c(cplx x) { return (cplx){-((x.re + x.im) * SQH), (x.re - x.im) * SQH}; }
static inline cplx mul_mi(cplx x) { return (cplx){x.im, -x.re}; } /* * (-i) */
static inline cplx mul_pi(cplx x) { return (cplx){-x.im, x.re}; } /* * (+i) */

static inline void r4_fwd(cplx *x0, cplx *x1, cplx *x2, cplx *x3) {
    cplx t0 = cadd(*x0, *x2), t1 = csub(*x0, *x2), t2 = cadd(*x1, *x3), t3 = csub(*x1, *x3);
    *x0 = cadd(t0, t2);
    *x2 = csub(t0, t2);
    *x1 = (cplx){t1.re + t3.im, t1.im - t3.re};
    *x3 = (cplx){t1.re - t3.im, t1.im + t3.re};
}
static inline void r4_inv(cplx *x0, cplx *x1, cplx *x2, cplx *x3) {
    cplx t0 = cadd(*x0, *x2), t1 = csub(*x0, *x2), t2 = cadd(*x1, *x3), t3 = csub(*x1, *x3);
    *x0 = cadd(t0, t2);
    *x2 = csub(t0, t2);
    *x1 = (cplx){t1.re - t3.im, t1.im + t3.re};
    *x3 = (cplx){t1.re + t3.im, t1.im - t3.re};
}

/* internal twiddle omega_16^e, e in {0,1,2,3,4,6,9} */
static inline cplx tw16_fwd(cplx x, int e) {
    switch (e) {
    case 0: return x;
    case 1: return cmulw(x, C16_1, -S16_1);
    case 2: return mul_w8(x);
    case 3: return cmulw(x, S16_1, -C16_1);
    case 4: return mul_mi(x);
    case 6: return mul_w8_3(x);
    case 9: return cmulw(x, -C16_1, S16_1);
    }
    abort();
}
static inline cplx tw16_inv(cplx x, int e) {
    switch (e) {
    case 0: return x;
    case 1: return cmulw(x, C16_1, S16_1);
    case 2: return mul_w8c(x);
    case 3: return cmulw(x, S16_1, C16_1);
    case 4: return mul_pi(x);
    case 6: return mul_w8_3c(x);
    case 9: return cmulw(x, -C16_1, -S16_1);
    }
    abort();
}
static inline cplx tw8_fwd(cplx x, int e) {
    switch (e) {
    case 0: return x;
    case 1: return mul_w8(x);
    case 2: return mul_mi(x);
    case 3: return mul_w8_3(x);
    }
    abort();
}
static inline cplx tw8_inv(cplx x, int e) {
    switch (e) {
    case 0: return x;
    case 1: return mul_w8c(x);
    case 2: return mul_pi(x);
    case 3: return mul_w8_3c(x);
    }
    abort();
}

/* radix-R DFTs on v[0..R) producing natural order output (forward: omega = exp(-2 pi i/R)) */
static void dft_fwd(cplx *v, int R) {
    if (R == 2) {
        cplx a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    } else if (R == 4) {
        r4_fwd(&v[0], &v[1], &v[2], &v[3]);
    } else if (R == 8) {
        cplx u[2][4];
        for (int a = 0; a < 2; a++) {
            cplx y0 = v[a], y1 = v[a + 2], y2 = v[a + 4], y3 = v[a + 6];
            r4_fwd(&y0, &y1, &y2, &y3);
            u[a][0] = y0;
            u[a][1] = tw8_fwd(y1, a * 1);
            u[a][2] = tw8_fwd(y2, a * 2);
            u[a][3] = tw8_fwd(y3, a * 3);
        }
        for (int c = 0; c < 4; c++) {
            v[c] = cadd(u[0][c], u[1][c]);
            v[c + 4] = csub(u[0][c], u[1][c]);
        }
    } else if (R == 16) {
        cplx u[4][4];
        for (int a = 0; a < 4; a++) {
            cplx y0 = v[a], y1 = v[a + 4], y2 = v[a + 8], y3 = v[a + 12];
            r4_fwd(&y0, &y1, &y2, &y3);
            u[a][0] = y0;
            u[a][1] = tw16_fwd(y1, a * 1);
            u[a][2] = tw16_fwd(y2, a * 2);
            u[a][3] = tw16_fwd(y3, a * 3);
        }
        for (int c = 0; c < 4; c++) {
            cplx y0 = u[0][c], y1 = u[1][c], y2 = u[2][c], y3 = u[3][c];
            r4_fwd(&y0, &y1, &y2, &y3);
            v[c] = y0;
            v[c + 4] = y1;
            v[c + 8] = y2;
            v[c + 12] = y3;
        }
    } else {
        abort();
    }
}

static void dft_inv(cplx *v, int R) {
    if (R == 2) {
        cplx a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    } else if (R == 4) {
        r4_inv(&v[0], &v[1], &v[2], &v[3]);
    } else if (R == 8) {
        cplx u[2][4];
        for (int c = 0; c < 4; c++) {
            u[0][c] = cadd(v[c], v[c + 4]);
            u[1][c] = csub(v[c], v[c + 4]);
        }
        for (int a = 0; a < 2; a++) {
            cplx y0 = u[a][0], y1 = tw8_inv(u[a][1], a * 1), y2 = tw8_inv(u[a][2], a * 2),
                 y3 = tw8_inv(u[a][3], a * 3);
            r4_inv(&y0, &y1, &y2, &y3);
            v[a] = y0;
            v[a + 2] = y1;
            v[a + 4] = y2;
            v[a + 6] = y3;
        }
    } else if (R == 16) {
        cplx u[4][4];
        for (int c = 0; c < 4; c++) {
            cplx y0 = v[c], y1 = v[c + 4], y2 = v[c + 8], y3 = v[c + 12];
            r4_inv(&y0, &y1, &y2, &y3);
            u[0][c] = y0;
            u[1][c] = y1;
            u[2][c] = y2;
            u[3][c] = y3;
        }
        for (int a = 0; a < 4; a++) {
            cplx y0 = u[a][0], y1 = tw16_inv(u[a][1], a * 1), y2 = tw16_inv(u[a][2], a * 2),
                 y3 = tw16_inv(u[a][3], a * 3);
            r4_inv(&y0, &y1, &y2, &y3);
            v[a] = y0;
            v[a + 4] = y1;
            v[a + 8] = y2;
            v[a + 12] = y3;
        }
    } else {
        abort();
    }
}

typedef struct {
    int N, M, nrad;
    int rad[8];
    cplx *W;     /* W[t] = exp(-2 pi i t / M), t < M */
    cplx *twist; /* w_j = exp(i pi j / N), j < M (fft/mod.rs:58-69) */
} orc_fft;

static int radix_plan(int M, int *rad) {
    switch (M) {
    case 512: rad[0] = 8; rad[1] = 8; rad[2] = 8; return 3;
    case 1024: rad[0] = 16; rad[1] = 16; rad[2] = 4; return 3;
    /* N = 4096 / 8192 / 16384: top radix R = M / 1024, then the 1024-point [16, 16, 4] plan of
     * each sub-block -- the engine's split CMUX (pbs_large.hip) runs this DAG */
    case 2048: rad[0] = 2; rad[1] = 16; rad[2] = 16; rad[3] = 4; return 4;
    case 4096: rad[0] = 4; rad[1] = 16; rad[2] = 16; rad[3] = 4; return 4;
    case 8192: rad[0] = 8; rad[1] = 16; rad[2] = 16; rad[3] = 4; return 4;
    case 16384: rad[0] = 16; rad[1] = 16; rad[2] = 16; rad[3] = 4; return 4;
    case 256: rad[0] = 16; rad[1] = 16; return 2;
    case 128: rad[0] = 16; rad[1] = 8; return 2;
    case 64: rad[0] = 16; rad[1] = 4; return 2;
    case 32: rad[0] = 16; rad[1] = 2; return 2;
    case 16: rad[0] = 16; return 1;
    default: return 0;
    }
}

/* cos and sin are called separately through opaque pointers: a compiler may otherwise fuse the
 * pair into sincos(), whose last bits can differ; the engine builds its tables the same way
 * (capi.cpp build_tables), so both sides see identical twiddles. */
static double (*volatile orc_cos)(double) = cos;
static double (*volatile orc_sin)(double) = sin;

static int fft_init(orc_fft *f, int N) {
    f->N = N;
    f->M = N / 2;
    f->nrad = radix_plan(f->M, f->rad);
    if (!f->nrad) return -1;
    int M = f->M;
    f->W = (cplx *)malloc(sizeof(cplx) * M);
    f->twist = (cplx *)malloc(sizeof(cplx) * M);
    for (int t = 0; t < M; t++) {
        double ang = 2.0 * M_PI * (double)t / (double)M;
        f->W[t].re = orc_cos(ang);
        f->W[t].im = -orc_sin(ang);
    }
    double unit = M_PI / (2.0 * (double)M);
    for (int j = 0; j < M; j++) {
        double a = (double)j * unit;
        f->twist[j].re = orc_cos(a);
        f->twist[j].im = orc_sin(a);
    }
    return 0;
}

static void fft_free(orc_fft *f) {
    free(f->W);
    free(f->twist);
}

static void dif_rec(const orc_fft *f, cplx *z, int off, int L, int stage) {
    int R = f->rad[stage];
    int m = L / R;
    int tstride = f->M / L;
    cplx v[16];
    for (int a = 0; a < m; a++) {
        for (int b = 0; b < R; b++) v[b] = z[off + a + m * b];
        dft_fwd(v, R);
        for (int c = 0; c < R; c++) {
            int t = a * c;
            cplx y = v[c];
            if (t) y = cmulw(y, f->W[t * tstride].re, f->W[t * tstride].im);
            z[off + a + m * c] = y;
        }
    }
    if (m > 1)
        for (int c = 0; c < R; c++) dif_rec(f, z, off + m * c, m, stage + 1);
}

static void dit_rec(const orc_fft *f, cplx *z, int off, int L, int stage) {
    int R = f->rad[stage];
    int m = L / R;
    int tstride = f->M / L;
    cplx v[16];
    if (m > 1)
        for (int c = 0; c < R; c++) dit_rec(f, z, off + m * c, m, stage + 1);
    for (int a = 0; a < m; a++) {
        for (int c = 0; c < R; c++) {
            int t = a * c;
            cplx y = z[off + a + m * c];
            if (t) y = cmulw(y, f->W[t * tstride].re, -f->W[t * tstride].im);
            v[c] = y;
        }
        dft_inv(v, R);
        for (int b = 0; b < R; b++) z[off + a + m * b] = v[b];
    }
}

static void fft_fwd(const orc_fft *f, cplx *z) { dif_rec(f, z, 0, f->M, 0); }
static void fft_inv(const orc_fft *f, cplx *z) { dit_rec(f, z, 0, f->M, 0); }

/* convert_forward_integer (fft/mod.rs:242-261; AVX2 form x86.rs:505-596):
 *   re = fma(xr, wr, -(xi*wi)), im = fma(xr, wi, xi*wr) with xr = (f64)(i64)x[j], xi = x[j+M] */
static void forward_integer(const orc_fft *f, const uint64_t *x, cplx *out) {
    int M = f->M;
    for (int j = 0; j < M; j++) {
        cplx in = {(double)(int64_t)x[j], (double)(int64_t)x[j + M]};
        out[j] = cmulw(in, f->twist[j].re, f->twist[j].im);
    }
    fft_fwd(f, out);
}

/* convert_forward_torus (fft/mod.rs:197-218): scalar c64 product, no fma. */
static void forward_torus(const orc_fft *f, const uint64_t *x, cplx *out) {
    int M = f->M;
    for (int j = 0; j < M; j++) {
        double xr = (double)(int64_t)x[j] * 0x1p-64;
        double xi = (double)(int64_t)x[j + M] * 0x1p-64;
        double wr = f->twist[j].re, wi = f->twist[j].im;
        out[j].re = xr * wr - xi * wi;
        out[j].im = xr * wi + xi * wr;
    }
    fft_fwd(f, out);
}

/* add_backward_in_place_as_torus (fft/mod.rs:487-557) with the AVX2 conversion
 * (x86.rs:823-874, 961-1044): t = z * conj(w)/M via fma; fract = t - rint(t);
 * out += (i64)rint(fract * 2^64).  `z` is destroyed. `add` = 0 overwrites instead. */
static void backward_torus(const orc_fft *f, cplx *z, uint64_t *out, int add) {
    int M = f->M;
    fft_inv(f, z);
    double norm = 1.0 / (double)M;
    for (int j = 0; j < M; j++) {
        double wr = norm * f->twist[j].re, wi = norm * f->twist[j].im;
        double mr = fma(z[j].re, wr, z[j].im * wi);
        double mi = fma(-z[j].re, wi, z[j].im * wr);
        double fr = mr - rint(mr);
        double fi = mi - rint(mi);
        uint64_t vr = (uint64_t)orc_f64_to_i64(rint(fr * 18446744073709551616.0));
        uint64_t vi = (uint64_t)orc_f64_to_i64(rint(fi * 18446744073709551616.0));
        if (add) {
            out[j] += vr;
            out[j + M] += vi;
        } else {
            out[j] = vr;
            out[j + M] = vi;
        }
    }
}

/* ---- exported FFT test hooks ---- */
int orc_fft_supported(int N) {
    int rad[8];
    return N >= 32 && (N & (N - 1)) == 0 && radix_plan(N / 2, rad) > 0;
}

/* out = backward( forward_torus(a) * forward_integer(b) )  (fft/tests.rs:82-222 product) */
int orc_fft_product(int N, const uint64_t *a_torus, const uint64_t *b_int, uint64_t *out) {
    orc_fft f;
    if (fft_init(&f, N)) return -1;
    int M = N / 2;
    cplx *fa = malloc(sizeof(cplx) * M), *fb = malloc(sizeof(cplx) * M);
    forward_torus(&f, a_torus, fa);
    forward_integer(&f, b_int, fb);
    for (int j = 0; j < M; j++) {
        double re = fa[j].re * fb[j].re - fa[j].im * fb[j].im;
        double im = fa[j].re * fb[j].im + fa[j].im * fb[j].re;
        fa[j].re = re;
        fa[j].im = im;
    }
    backward_torus(&f, fa, out, 0);
    free(fa);
    free(fb);
    fft_free(&f);
    return 0;
}

/* out = backward(forward_torus(a))  (fft/tests.rs:9-80 round trip) */
int orc_fft_roundtrip(int N, const uint64_t *a, uint64_t *out) {
    orc_fft f;
    if (fft_init(&f, N)) return -1;
    cplx *fa = malloc(sizeof(cplx) * (N / 2));
    forward_torus(&f, a, fa);
    backward_torus(&f, fa, out, 0);
    free(fa);
    fft_free(&f);
    return 0;
}

/* raw complex FFT in position order (for FFT-vs-DFT checks) */
int orc_fft_complex(int M, const double *in_reim, double *out_reim, int inverse) {
    orc_fft f;
    if (fft_init(&f, 2 * M)) return -1;
    memcpy(out_reim, in_reim, sizeof(double) * 2 * M);
    if (inverse)
        fft_inv(&f, (cplx *)out_reim);
    else
        fft_fwd(&f, (cplx *)out_reim);
    fft_free(&f);
    return 0;
}

/* exact wrapping negacyclic product (fft/tests.rs:86-103 convolution_naive) */
void orc_negacyclic_mul_u64(int N, const uint64_t *a, const uint64_t *b, uint64_t *out) {
    for (int i = 0; i < N; i++) out[i] = 0;
    for (int i = 0; i < N; i++) {
        for (int j = 0; j < N; j++) {
            uint64_t p = a[i] * b[j];
            int k = i + j;
            if (k < N)
                out[k] += p;
            else
                out[k - N] -= p;
        }
    }
}

/* ------------------------------------------------------------------------------------ */
/* Polynomial helpers: algorithms/polynomial_algorithms.rs:219-260, 425-490.              */
/* ------------------------------------------------------------------------------------ */
/* fast_pbs_modulus_switch (fft_impl/common.rs:26-43), offset 0, lut_count_log 0 */
uint64_t orc_pbs_modulus_switch(uint64_t x, int log2N) {
    uint64_t o = x >> (64 - log2N - 2);
    o += 1;
    o >>= 1;
    return o;
}

/* out = in / X^d  (polynomial_wrapping_monic_monomial_div), d in [0, 2N] */
static void monomial_div(uint64_t *out, const uint64_t *in, int N, uint64_t d) {
    uint64_t full = d / N, rem = d % N;
    int neg = (full & 1);
    for (int j = 0; j < N; j++) {
        uint64_t src = j + rem;
        uint64_t v;
        if (src < (uint64_t)N)
            v = in[src];
        else
            v = 0 - in[src - N];
        out[j] = neg ? 0 - v : v;
    }
}

/* out = in * X^d - in  (polynomial_wrapping_monic_monomial_mul_and_subtract) */
static void monomial_mul_sub(uint64_t *out, const uint64_t *in, int N, uint64_t d) {
    uint64_t full = d / N, rem = d % N;
    for (uint64_t j = 0; j < rem; j++) {
        uint64_t src = in[N - rem + j];
        out[j] = ((full & 1) ? src : 0 - src) - in[j];
    }
    for (uint64_t j = rem; j < (uint64_t)N; j++) {
        uint64_t src = in[j - rem];
        out[j] = ((full & 1) ? 0 - src : src) - in[j];
    }
}

/* extract_lwe_sample_from_glwe_ciphertext at degree 0 (glwe_sample_extraction.rs:91-147) */
static void sample_extract0(const uint64_t *glwe, uint64_t *lwe, int k, int N) {
    for (int p = 0; p < k; p++) {
        const uint64_t *a = glwe + (size_t)p * N;
        uint64_t *o = lwe + (size_t)p * N;
        o[0] = a[0];
        for (int j = 1; j < N; j++) o[j] = 0 - a[N - j];
    }
    lwe[(size_t)k * N] = glwe[(size_t)k * N];
}

/* ------------------------------------------------------------------------------------ */
/* Keys and encryption (client side; harness).                                            */
/* ------------------------------------------------------------------------------------ */
void orc_gen_binary_key(uint64_t seed, uint64_t stream, size_t len, uint64_t *key) {
    orc_rng r;
    rng_seed(&r, seed, stream);
    for (size_t i = 0; i < len; i++) key[i] = rng_next(&r) >> 63;
}

/* body += sum_p a_p * s_p (negacyclic, binary key) */
static void glwe_mask_key_product_add(uint64_t *body, const uint64_t *mask, const uint64_t *key,
                                      int k, int N) {
    for (int p = 0; p < k; p++) {
        const uint64_t *a = mask + (size_t)p * N;
        const uint64_t *s = key + (size_t)p * N;
        for (int i = 0; i < N; i++) {
            if (!s[i]) continue;
            /* body[j] += a[j - i] for j >= i, -= a[j - i + N] for j < i */
            for (int j = 0; j < i; j++) body[j] -= a[j - i + N];
            for (int j = i; j < N; j++) body[j] += a[j - i];
        }
    }
}

/* GLWE encryption of (already placed) body message (glwe_encryption.rs) */
static void glwe_encrypt_assign(orc_rng *r, uint64_t *glwe, const uint64_t *glwe_key, int k, int N,
                                double std) {
    uint64_t *body = glwe + (size_t)k * N;
    for (size_t i = 0; i < (size_t)k * N; i++) glwe[i] = rng_next(r);
    for (int j = 0; j < N; j++) body[j] += gaussian_torus(r, std);
    glwe_mask_key_product_add(body, glwe, glwe_key, k, N);
}

typedef struct {
    uint64_t seed;
    const uint64_t *lwe_sk;
    int n;
    const uint64_t *glwe_sk;
    int k, N, base_log, level;
    double std;
    uint64_t *bsk;
    int g;      /* 0: classic BSK; > 0: multi-bit grouping factor */
    int items;  /* GGSWs to generate */
    int next;
    pthread_mutex_t mu;
} bsk_job;

/* encrypt_constant_ggsw_ciphertext (ggsw_encryption.rs:116-150,300-331) of the plaintext m;
 * layout [L][k+1][k+1][N], level lvl stored at lvl-1 */
static void ggsw_encrypt_constant(const bsk_job *J, orc_rng *r, uint64_t *ggsw, uint64_t m) {
    int k = J->k, N = J->N, L = J->level;
    size_t glwe_len = (size_t)(k + 1) * N;
    for (int lvl = 1; lvl <= L; lvl++) {
        uint64_t factor = (0 - m) * (1ULL << (64 - J->base_log * lvl));
        for (int row = 0; row <= k; row++) {
            uint64_t *g = ggsw + ((size_t)(lvl - 1) * (k + 1) + row) * glwe_len;
            uint64_t *body = g + (size_t)k * N;
            if (row < k) {
                const uint64_t *s = J->glwe_sk + (size_t)row * N;
                for (int j = 0; j < N; j++) body[j] = s[j] * factor;
            } else {
                for (int j = 0; j < N; j++) body[j] = 0;
                body[0] = 0 - factor;
            }
            glwe_encrypt_assign(r, g, J->glwe_sk, k, N, J->std);
        }
    }
}

/* combine_key_bits (lwe_multi_bit_bootstrap_key_generation.rs:401-427): GGSW number `sel` of a
 * group encrypts prod_i (bit_{g-1-i}(sel) ? s_i : 1 - s_i), so GGSW 0 is the constant term. */
static uint64_t combine_key_bits(int sel, const uint64_t *key, int g) {
    uint64_t p = 1;
    for (int i = 0; i < g; i++) {
        uint64_t inv = (uint64_t)(((sel >> (g - 1 - i)) & 1) ^ 1);
        p *= key[i] ^ inv;
    }
    return p;
}

/* classic: BSK = GGSW_i(s_i), [n][L][k+1][k+1][N] (lwe_bootstrap_key_generation.rs);
 * multi-bit: [n/g][2^g][L][k+1][k+1][N], GGSW (j, sel) = GGSW(combine_key_bits(sel, s_{gj..}))
 * (lwe_multi_bit_bootstrap_key_generation.rs:87-173).  RNG stream per GGSW. */
static void gen_one_ggsw(bsk_job *J, int i) {
    int k = J->k, N = J->N, L = J->level;
    size_t ggsw_len = (size_t)L * (k + 1) * (k + 1) * N;
    orc_rng r;
    uint64_t m;
    if (J->g == 0) {
        rng_seed(&r, J->seed, 0x1000000ULL + (uint64_t)i);
        m = J->lwe_sk[i];
    } else {
        int per = 1 << J->g;
        rng_seed(&r, J->seed, 0x4000000ULL + (uint64_t)i);
        m = combine_key_bits(i % per, J->lwe_sk + (size_t)(i / per) * J->g, J->g);
    }
    ggsw_encrypt_constant(J, &r, J->bsk + (size_t)i * ggsw_len, m);
}

static void *bsk_worker(void *arg) {
    bsk_job *J = (bsk_job *)arg;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        int i = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (i >= J->items) break;
        gen_one_ggsw(J, i);
    }
    return NULL;
}

static void run_bsk_job(bsk_job *J, int threads) {
    pthread_mutex_init(&J->mu, NULL);
    if (threads < 1) threads = 1;
    pthread_t th[64];
    if (threads > 64) threads = 64;
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, bsk_worker, J);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&J->mu);
}

void orc_gen_bsk(uint64_t seed, const uint64_t *lwe_sk, int n, const uint64_t *glwe_sk, int k, int N,
                 int base_log, int level, double std, uint64_t *bsk, int threads) {
    bsk_job J = {seed, lwe_sk, n, glwe_sk, k, N, base_log, level, std, bsk, 0, n, 0};
    run_bsk_job(&J, threads);
}

void orc_gen_mb_bsk(uint64_t seed, const uint64_t *lwe_sk, int n, const uint64_t *glwe_sk, int k, int N,
                    int base_log, int level, int g, double std, uint64_t *bsk, int threads) {
    bsk_job J = {seed, lwe_sk, n, glwe_sk, k, N, base_log, level, std, bsk, g, (n / g) << g, 0};
    run_bsk_job(&J, threads);
}

static void lwe_encrypt_one(orc_rng *r, const uint64_t *sk, int n, uint64_t pt, double std,
                            uint64_t *ct) {
    uint64_t b = pt + gaussian_torus(r, std);
    for (int i = 0; i < n; i++) {
        ct[i] = rng_next(r);
        b += ct[i] * sk[i];
    }
    ct[n] = b;
}

/* KSK: lwe_keyswitch_key_generation.rs:60-135 (levels stored L..1); layout [in][L][out+1] */
void orc_gen_ksk(uint64_t seed, const uint64_t *in_sk, int in_dim, const uint64_t *out_sk, int out_dim,
                 int base_log, int level, double std, uint64_t *ksk) {
    orc_rng r;
    rng_seed(&r, seed, 0x2000000ULL);
    for (int i = 0; i < in_dim; i++) {
        for (int l = 0; l < level; l++) {
            int lvl = level - l;
            uint64_t msg = in_sk[i] << (64 - base_log * lvl);
            lwe_encrypt_one(&r, out_sk, out_dim, msg, std,
                            ksk + ((size_t)i * level + l) * (size_t)(out_dim + 1));
        }
    }
}

/* LWE -> GLWE packing KSK (lwe_packing_keyswitch_key_generation.rs:74-149): block i, level
 * lvl = L..1 is a GLWE encryption of the constant polynomial in_sk[i] * 2^(64 - base_log*lvl);
 * layout [in][L][(k+1)N]; input coefficient i draws from RNG stream 0x5000000 + i. */
void orc_gen_pksk(uint64_t seed, const uint64_t *in_sk, int in_dim, const uint64_t *glwe_sk, int k, int N,
                  int base_log, int level, double std, uint64_t *pksk) {
    size_t glwe_len = (size_t)(k + 1) * N;
    for (int i = 0; i < in_dim; i++) {
        orc_rng r;
        rng_seed(&r, seed, 0x5000000ULL + (uint64_t)i);
        for (int l = 0; l < level; l++) {
            int lvl = level - l;
            uint64_t *g = pksk + ((size_t)i * level + l) * glwe_len;
            memset(g + (size_t)k * N, 0, sizeof(uint64_t) * N);
            g[(size_t)k * N] = in_sk[i] << (64 - base_log * lvl);
            glwe_encrypt_assign(&r, g, glwe_sk, k, N, std);
        }
    }
}

/* keyswitch_lwe_ciphertext_into_glwe_ciphertext (lwe_packing_keyswitch.rs:102-186): output
 * zeroed, GLWE body[0] = LWE body, then minus sum of signed digits times the key GLWEs. */
void orc_packing_keyswitch_batch(const uint64_t *pksk, int in_dim, int k, int N, int base_log, int level,
                                 const uint64_t *in, uint64_t *out, size_t count) {
    uint64_t mask = (1ULL << base_log) - 1;
    size_t glwe_len = (size_t)(k + 1) * N;
    for (size_t c = 0; c < count; c++) {
        const uint64_t *x = in + c * (size_t)(in_dim + 1);
        uint64_t *o = out + c * glwe_len;
        memset(o, 0, sizeof(uint64_t) * glwe_len);
        o[(size_t)k * N] = x[in_dim];
        for (int i = 0; i < in_dim; i++) {
            uint64_t state = orc_closest_representable(x[i], base_log, level) >> (64 - base_log * level);
            for (int l = 0; l < level; l++) {
                uint64_t d = decompose_one_level(base_log, &state, mask);
                if (!d) continue;
                const uint64_t *row = pksk + ((size_t)i * level + l) * glwe_len;
                for (size_t j = 0; j < glwe_len; j++) o[j] -= d * row[j];
            }
        }
    }
}

/* out[c][i] = sum_j glwe_in[c][j] * polys[i][j] per GLWE polynomial (schoolbook negacyclic
 * product, polynomial_wrapping_add_mul_assign semantics), then optionally
 * extract_lwe_sample_from_glwe_ciphertext at degree 0. */
void orc_glwe_poly_mul(int k, int N, const uint64_t *glwe_in, size_t J, const uint64_t *polys, size_t npoly,
                       size_t count, int extract, uint64_t *out) {
    size_t glwe_len = (size_t)(k + 1) * N;
    size_t out_len = extract ? (size_t)k * N + 1 : glwe_len;
    uint64_t *acc = malloc(sizeof(uint64_t) * glwe_len);
    for (size_t c = 0; c < count; c++)
        for (size_t i = 0; i < npoly; i++) {
            memset(acc, 0, sizeof(uint64_t) * glwe_len);
            for (size_t j = 0; j < J; j++) {
                const uint64_t *g = glwe_in + (c * J + j) * glwe_len;
                const uint64_t *v = polys + (i * J + j) * (size_t)N;
                for (int t = 0; t < N; t++) {
                    if (!v[t]) continue;
                    for (int p = 0; p <= k; p++) {
                        const uint64_t *a = g + (size_t)p * N;
                        uint64_t *o = acc + (size_t)p * N;
                        for (int m = 0; m < t; m++) o[m] -= v[t] * a[m - t + N];
                        for (int m = t; m < N; m++) o[m] += v[t] * a[m - t];
                    }
                }
            }
            uint64_t *dst = out + (c * npoly + i) * out_len;
            if (extract)
                sample_extract0(acc, dst, k, N);
            else
                memcpy(dst, acc, sizeof(uint64_t) * glwe_len);
        }
    free(acc);
}

void orc_lwe_encrypt_batch(uint64_t seed, const uint64_t *sk, int n, const uint64_t *pts, size_t count,
                           double std, uint64_t *cts) {
    orc_rng r;
    rng_seed(&r, seed, 0x3000000ULL);
    for (size_t c = 0; c < count; c++) lwe_encrypt_one(&r, sk, n, pts[c], std, cts + c * (n + 1));
}

void orc_lwe_decrypt_batch(const uint64_t *sk, int n, const uint64_t *cts, size_t count, uint64_t *pts) {
    for (size_t c = 0; c < count; c++) {
        const uint64_t *ct = cts + c * (n + 1);
        uint64_t b = ct[n];
        for (int i = 0; i < n; i++) b -= ct[i] * sk[i];
        pts[c] = b;
    }
}

/* shortint fill_accumulator (shortint/engine/mod.rs:72-128): f_values[i] = f(i) for
 * i < message_modulus*carry_modulus.  Mask polys zero, body = boxes of f(i)*delta, first
 * half box negated, rotated left by half a box. */
void orc_fill_accumulator(int N, int k, int msg_mod, int carry_mod, const uint64_t *f_values,
                          uint64_t *acc) {
    int p = msg_mod * carry_mod;
    int box = N / p;
    uint64_t delta = (1ULL << 63) / (uint64_t)p;
    memset(acc, 0, sizeof(uint64_t) * (size_t)k * N);
    uint64_t *body = acc + (size_t)k * N;
    uint64_t *tmp = malloc(sizeof(uint64_t) * N);
    for (int i = 0; i < p; i++)
        for (int j = 0; j < box; j++) tmp[i * box + j] = f_values[i] * delta;
    int half = box / 2;
    for (int j = 0; j < half; j++) tmp[j] = 0 - tmp[j];
    for (int j = 0; j < N; j++) body[j] = tmp[(j + half) % N];
    free(tmp);
}

/* ------------------------------------------------------------------------------------ */
/* Fourier BSK + classic PBS (fft64/crypto/bootstrap.rs:243-380, ggsw.rs:477-697).        */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    int n, k, N, base_log, level;
    orc_fft fft;
    cplx *fourier; /* [n][L][k+1][k+1][M] in position order */
} orc_fbsk;

void *orc_fbsk_create(const uint64_t *bsk, int n, int k, int N, int base_log, int level) {
    orc_fbsk *b = calloc(1, sizeof(orc_fbsk));
    b->n = n;
    b->k = k;
    b->N = N;
    b->base_log = base_log;
    b->level = level;
    if (fft_init(&b->fft, N)) {
        free(b);
        return NULL;
    }
    int M = N / 2;
    size_t npoly = (size_t)n * level * (k + 1) * (k + 1);
    b->fourier = malloc(sizeof(cplx) * npoly * M);
    for (size_t p = 0; p < npoly; p++) forward_torus(&b->fft, bsk + p * N, b->fourier + p * M);
    return b;
}

void orc_fbsk_destroy(void *h) {
    orc_fbsk *b = h;
    if (!b) return;
    fft_free(&b->fft);
    free(b->fourier);
    free(b);
}

/* Copies the Fourier BSK (position order) out, for layout tests. */
void orc_fbsk_copy(const void *h, double *out) {
    const orc_fbsk *b = h;
    size_t npoly = (size_t)b->n * b->level * (b->k + 1) * (b->k + 1);
    memcpy(out, b->fourier, sizeof(cplx) * npoly * (b->N / 2));
}

typedef struct {
    uint64_t *ct1, *state, *digits;
    cplx *fd, *facc;
} pbs_scratch;

static void scratch_alloc(pbs_scratch *s, int k, int N) {
    size_t gl = (size_t)(k + 1) * N;
    s->ct1 = malloc(sizeof(uint64_t) * gl);
    s->state = malloc(sizeof(uint64_t) * gl);
    s->digits = malloc(sizeof(uint64_t) * N);
    s->fd = malloc(sizeof(cplx) * (N / 2));
    s->facc = malloc(sizeof(cplx) * (size_t)(k + 1) * (N / 2));
}

static void scratch_free(pbs_scratch *s) {
    free(s->ct1);
    free(s->state);
    free(s->digits);
    free(s->fd);
    free(s->facc);
}

/* add_external_product_assign (ggsw.rs:477-598): out += ggsw (x) glwe.
 * MAC (update_with_fmadd, ggsw.rs:616-697), product g*d:
 *   first: (fma(gr,dr,-(gi*di)), fma(gr,di,gi*dr));
 *   next : (fma(gr,dr,fma(-gi,di,acc_r)), fma(gr,di,fma(gi,dr,acc_i))). */
static void external_product_add(const orc_fbsk *b, const cplx *ggsw, uint64_t *out, const uint64_t *glwe,
                                 pbs_scratch *s) {
    int k = b->k, N = b->N, M = N / 2, L = b->level, beta = b->base_log;
    size_t gl = (size_t)(k + 1) * N;
    uint64_t mask = (1ULL << beta) - 1;
    for (size_t j = 0; j < gl; j++)
        s->state[j] = orc_closest_representable(glwe[j], beta, L) >> (64 - beta * L);
    int first = 1;
    for (int lvl = L; lvl >= 1; lvl--) {
        /* ggsw level matrix for `lvl` is stored at index lvl-1 (ggsw.rs:524 .rev()) */
        const cplx *lm = ggsw + (size_t)(lvl - 1) * (k + 1) * (k + 1) * M;
        for (int row = 0; row <= k; row++) {
            uint64_t *st = s->state + (size_t)row * N;
            for (int j = 0; j < N; j++) s->digits[j] = decompose_one_level(beta, &st[j], mask);
            forward_integer(&b->fft, s->digits, s->fd);
            for (int col = 0; col <= k; col++) {
                const cplx *g = lm + ((size_t)row * (k + 1) + col) * M;
                cplx *acc = s->facc + (size_t)col * M;
                if (first) {
                    for (int f = 0; f < M; f++) {
                        double gr = g[f].re, gi = g[f].im, dr = s->fd[f].re, di = s->fd[f].im;
                        acc[f].re = fma(gr, dr, -(gi * di));
                        acc[f].im = fma(gr, di, gi * dr);
                    }
                } else {
                    for (int f = 0; f < M; f++) {
                        double gr = g[f].re, gi = g[f].im, dr = s->fd[f].re, di = s->fd[f].im;
                        acc[f].re = fma(gr, dr, fma(-gi, di, acc[f].re));
                        acc[f].im = fma(gr, di, fma(gi, dr, acc[f].im));
                    }
                }
            }
            first = 0;
        }
    }
    for (int col = 0; col <= k; col++)
        backward_torus(&b->fft, s->facc + (size_t)col * M, out + (size_t)col * N, 1);
}

/* programmable_bootstrap_lwe_ciphertext (lwe_programmable_bootstrapping.rs:1017-1111) =
 * bootstrap (bootstrap.rs:346-380) = blind_rotate_assign (bootstrap.rs:243-344, without the
 * fork's PATTERN noise dump) + sample extract at degree 0. */
static void pbs_one(const orc_fbsk *b, const uint64_t *lwe_in, uint64_t *lwe_out, const uint64_t *lut,
                    uint64_t *acc, pbs_scratch *s, int glwe_out) {
    int n = b->n, k = b->k, N = b->N, M = N / 2;
    int log2N = 0;
    while ((1 << log2N) < N) log2N++;
    size_t ggsw_len = (size_t)b->level * (k + 1) * (k + 1) * M;
    uint64_t bt = orc_pbs_modulus_switch(lwe_in[n], log2N);
    for (int p = 0; p <= k; p++) monomial_div(acc + (size_t)p * N, lut + (size_t)p * N, N, bt);
    for (int i = 0; i < n; i++) {
        if (lwe_in[i] == 0) continue;
        uint64_t at = orc_pbs_modulus_switch(lwe_in[i], log2N);
        for (int p = 0; p <= k; p++)
            monomial_mul_sub(s->ct1 + (size_t)p * N, acc + (size_t)p * N, N, at);
        external_product_add(b, b->fourier + (size_t)i * ggsw_len, acc, s->ct1, s);
    }
    if (glwe_out) /* bootstrap_without_sample_extract (fork, bootstrap.rs:383-412) */
        memcpy(lwe_out, acc, sizeof(uint64_t) * (size_t)(k + 1) * N);
    else
        sample_extract0(acc, lwe_out, k, N);
}

typedef struct {
    const orc_fbsk *b;
    const uint64_t *in, *luts;
    const uint32_t *lut_idx;
    uint64_t *out;
    size_t count;
    size_t next;
    pthread_mutex_t mu;
    int glwe_out;
} pbs_job;

static void *pbs_worker(void *arg) {
    pbs_job *J = arg;
    const orc_fbsk *b = J->b;
    int k = b->k, N = b->N;
    pbs_scratch s;
    scratch_alloc(&s, k, N);
    uint64_t *acc = malloc(sizeof(uint64_t) * (size_t)(k + 1) * N);
    for (;;) {
        pthread_mutex_lock(&J->mu);
        size_t c = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (c >= J->count) break;
        size_t li = J->lut_idx ? J->lut_idx[c] : 0;
        const size_t out_len = J->glwe_out ? (size_t)(k + 1) * N : (size_t)(k * N + 1);
        pbs_one(b, J->in + c * (size_t)(b->n + 1), J->out + c * out_len, J->luts + li * (size_t)(k + 1) * N, acc, &s,
                J->glwe_out);
    }
    free(acc);
    scratch_free(&s);
    return NULL;
}

/* Batched PBS, one ciphertext per thread (mirrors pbs_bench.rs:430-549 par_iter). */
static void pbs_batch(const void *fbsk, const uint64_t *in, uint64_t *out, const uint64_t *luts,
                      const uint32_t *lut_idx, size_t count, int threads, int glwe_out) {
    pbs_job J = {fbsk, in, luts, lut_idx, out, count, 0};
    J.glwe_out = glwe_out;
    pthread_mutex_init(&J.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, pbs_worker, &J);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&J.mu);
}

void orc_pbs_batch(const void *fbsk, const uint64_t *in, uint64_t *out, const uint64_t *luts,
                   const uint32_t *lut_idx, size_t count, int threads) {
    pbs_batch(fbsk, in, out, luts, lut_idx, count, threads, 0);
}

/* blind rotation without sample extraction: out = [count][(k+1)N] */
void orc_blind_rotate_batch(const void *fbsk, const uint64_t *in, uint64_t *out, const uint64_t *luts,
                            const uint32_t *lut_idx, size_t count, int threads) {
    pbs_batch(fbsk, in, out, luts, lut_idx, count, threads, 1);
}

/* ------------------------------------------------------------------------------------ */
/* Multi-bit PBS, deterministic group order                                               */
/* (lwe_multi_bit_programmable_bootstrapping.rs:548-828, 18-84; ggsw.rs:699-754).          */
/* ------------------------------------------------------------------------------------ */
/* Frequency index of FFT output position P (the DIF butterflies leave the spectrum in
 * digit-reversed order): P = c0 (M/R0) + c1 (M/(R0 R1)) + ...  ->  f = c0 + R0 c1 + R0 R1 c2 ... */
static int pos_freq(const orc_fft *f, int P) {
    int fr = 0, mult = 1, L = f->M;
    for (int st = 0; st < f->nrad; st++) {
        int m = L / f->rad[st];
        fr += mult * (P / m);
        P %= m;
        mult *= f->rad[st];
        L = m;
    }
    return fr;
}

/* Spectrum of the monomial X^d, d in [0, 2N], at frequency fr.  The reference builds it as
 * factor * fwd_monomial(d mod M) (fft/mod.rs:407-445: unit 1 or i, twist[d mod M], sign of
 * X^N = -1).  In closed form it is the 2N-th root of unity exp(i pi d (1 - 4 fr) / N) =
 * i^q twist[r] with t = d (1 - 4 fr) mod 2N, q = t / M, r = t mod M: one table read and exact
 * sign/swap operations, no rounding. */
static cplx mono_spectrum(const orc_fft *f, uint32_t d, int fr) {
    uint32_t t = (d - 4u * d * (uint32_t)fr) & (uint32_t)(2 * f->N - 1);
    uint32_t q = t / (uint32_t)f->M, r = t % (uint32_t)f->M;
    cplx w = f->twist[r];
    switch (q) {
    case 0: return w;
    case 1: return (cplx){-w.im, w.re};
    case 2: return (cplx){-w.re, -w.im};
    default: return (cplx){w.im, -w.re};
    }
}

/* test hooks: the closed form against the transform of X^d */
int orc_mono_spectrum(int N, uint32_t d, double *out_reim) {
    orc_fft f;
    if (fft_init(&f, N)) return -1;
    for (int P = 0; P < N / 2; P++) ((cplx *)out_reim)[P] = mono_spectrum(&f, d, pos_freq(&f, P));
    fft_free(&f);
    return 0;
}
int orc_fft_forward_integer(int N, const uint64_t *x, double *out_reim) {
    orc_fft f;
    if (fft_init(&f, N)) return -1;
    forward_integer(&f, x, (cplx *)out_reim);
    fft_free(&f);
    return 0;
}
int orc_pos_freq(int N, int P) {
    orc_fft f;
    if (fft_init(&f, N)) return -1;
    int r = pos_freq(&f, P);
    fft_free(&f);
    return r;
}

typedef struct {
    orc_fbsk b;  /* b.fourier: [n/g][2^g][L][k+1][k+1][M] in position order */
    int g;
    int *freq;   /* frequency of each position */
} orc_mb_fbsk;

void *orc_mb_fbsk_create(const uint64_t *bsk, int n, int k, int N, int base_log, int level, int g) {
    if (g < 1 || n % g) return NULL;
    orc_mb_fbsk *mb = calloc(1, sizeof(orc_mb_fbsk));
    orc_fbsk *b = &mb->b;
    b->n = n;
    b->k = k;
    b->N = N;
    b->base_log = base_log;
    b->level = level;
    mb->g = g;
    if (fft_init(&b->fft, N)) {
        free(mb);
        return NULL;
    }
    int M = N / 2;
    size_t npoly = (size_t)(n / g) * (1u << g) * level * (k + 1) * (k + 1);
    b->fourier = malloc(sizeof(cplx) * npoly * M);
    for (size_t p = 0; p < npoly; p++) forward_torus(&b->fft, bsk + p * N, b->fourier + p * M);
    mb->freq = malloc(sizeof(int) * M);
    for (int P = 0; P < M; P++) mb->freq[P] = pos_freq(&b->fft, P);
    return mb;
}

/* Copies the multi-bit Fourier BSK ([n/g][2^g][L][k+1][k+1][M], position order) out. */
void orc_mb_fbsk_copy(const void *h, double *out) {
    const orc_mb_fbsk *mb = h;
    const orc_fbsk *b = &mb->b;
    size_t npoly = (size_t)(b->n / mb->g) * (1u << mb->g) * b->level * (b->k + 1) * (b->k + 1);
    memcpy(out, b->fourier, sizeof(cplx) * npoly * (b->N / 2));
}

void orc_mb_fbsk_destroy(void *h) {
    orc_mb_fbsk *mb = h;
    if (!mb) return;
    fft_free(&mb->b.fft);
    free(mb->b.fourier);
    free(mb->freq);
    free(mb);
}

/* keybundle (prepare_multi_bit_ggsw_mem_optimized, :18-84):
 *   KB = GGSW_0 + sum_{sel=1}^{2^g-1} X^{deg_sel} GGSW_sel,
 *   deg_sel = modswitch(sum_i bit_{g-1-i}(sel) a_i), accumulated in sel order per element:
 *   kb.re = fma(g.re, m.re, fma(-g.im, m.im, kb.re)); kb.im = fma(g.re, m.im, fma(g.im, m.re, kb.im))
 * (update_with_fmadd_factor computes factor*(ggsw*mono) + kb; here the factor is folded into the
 * exact monomial spectrum, see mono_spectrum). */
static void mb_keybundle(const orc_mb_fbsk *mb, const cplx *group, const uint64_t *a, cplx *kb, cplx *mono,
                         int log2N) {
    const orc_fbsk *b = &mb->b;
    int g = mb->g, M = b->N / 2;
    size_t npoly = (size_t)b->level * (b->k + 1) * (b->k + 1);
    size_t ggsw_len = npoly * M;
    memcpy(kb, group, sizeof(cplx) * ggsw_len);
    for (int sel = 1; sel < (1 << g); sel++) {
        uint64_t deg = 0;
        for (int i = 0; i < g; i++)
            if ((sel >> (g - 1 - i)) & 1) deg += a[i];
        uint32_t d = (uint32_t)orc_pbs_modulus_switch(deg, log2N);
        for (int P = 0; P < M; P++) mono[P] = mono_spectrum(&b->fft, d, mb->freq[P]);
        const cplx *G = group + (size_t)sel * ggsw_len;
        for (size_t q = 0; q < npoly; q++) {
            for (int P = 0; P < M; P++) {
                cplx gg = G[q * M + P], m = mono[P], *o = &kb[q * M + P];
                o->re = fma(gg.re, m.re, fma(-gg.im, m.im, o->re));
                o->im = fma(gg.re, m.im, fma(gg.im, m.re, o->im));
            }
        }
    }
}

/* multi_bit_programmable_bootstrap_lwe_ciphertext (:1035-1128) with the deterministic blind
 * rotation (:548-828): acc = LUT / X^{b~}; for each group j in order: acc <- ExtProd(KB_j, acc)
 * into a zeroed GLWE (ping-pong buffers, :782-800); sample extract at degree 0. */
static void mb_pbs_one(const orc_mb_fbsk *mb, const uint64_t *lwe_in, uint64_t *lwe_out, const uint64_t *lut,
                       uint64_t *acc, uint64_t *tmp, cplx *kb, cplx *mono, pbs_scratch *s) {
    const orc_fbsk *b = &mb->b;
    int n = b->n, k = b->k, N = b->N, M = N / 2, g = mb->g;
    int log2N = 0;
    while ((1 << log2N) < N) log2N++;
    size_t ggsw_len = (size_t)b->level * (k + 1) * (k + 1) * M;
    size_t gl = (size_t)(k + 1) * N;
    uint64_t bt = orc_pbs_modulus_switch(lwe_in[n], log2N);
    for (int p = 0; p <= k; p++) monomial_div(acc + (size_t)p * N, lut + (size_t)p * N, N, bt);
    for (int j = 0; j < n / g; j++) {
        mb_keybundle(mb, b->fourier + (size_t)j * ((size_t)1 << g) * ggsw_len, lwe_in + (size_t)j * g, kb,
                     mono, log2N);
        memset(tmp, 0, sizeof(uint64_t) * gl);
        external_product_add(b, kb, tmp, acc, s);
        memcpy(acc, tmp, sizeof(uint64_t) * gl);
    }
    sample_extract0(acc, lwe_out, k, N);
}

typedef struct {
    const orc_mb_fbsk *mb;
    const uint64_t *in, *luts;
    const uint32_t *lut_idx;
    uint64_t *out;
    size_t count;
    size_t next;
    pthread_mutex_t mu;
} mb_pbs_job;

static void *mb_pbs_worker(void *arg) {
    mb_pbs_job *J = arg;
    const orc_fbsk *b = &J->mb->b;
    int k = b->k, N = b->N, M = N / 2;
    pbs_scratch s;
    scratch_alloc(&s, k, N);
    size_t gl = (size_t)(k + 1) * N;
    uint64_t *acc = malloc(sizeof(uint64_t) * gl), *tmp = malloc(sizeof(uint64_t) * gl);
    cplx *kb = malloc(sizeof(cplx) * (size_t)b->level * (k + 1) * (k + 1) * M);
    cplx *mono = malloc(sizeof(cplx) * M);
    for (;;) {
        pthread_mutex_lock(&J->mu);
        size_t c = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (c >= J->count) break;
        size_t li = J->lut_idx ? J->lut_idx[c] : 0;
        mb_pbs_one(J->mb, J->in + c * (size_t)(b->n + 1), J->out + c * (size_t)(k * N + 1),
                   J->luts + li * gl, acc, tmp, kb, mono, &s);
    }
    free(acc);
    free(tmp);
    free(kb);
    free(mono);
    scratch_free(&s);
    return NULL;
}

void orc_mb_pbs_batch(const void *h, const uint64_t *in, uint64_t *out, const uint64_t *luts,
                      const uint32_t *lut_idx, size_t count, int threads) {
    mb_pbs_job J = {h, in, luts, lut_idx, out, count, 0};
    pthread_mutex_init(&J.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, mb_pbs_worker, &J);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&J.mu);
}

/* ------------------------------------------------------------------------------------ */
/* Keyswitch: lwe_keyswitch.rs:96-170.                                                    */
/* ------------------------------------------------------------------------------------ */
void orc_keyswitch_batch(const uint64_t *ksk, int in_dim, int out_dim, int base_log, int level,
                         const uint64_t *in, uint64_t *out, size_t count) {
    uint64_t mask = (1ULL << base_log) - 1;
    for (size_t c = 0; c < count; c++) {
        const uint64_t *x = in + c * (size_t)(in_dim + 1);
        uint64_t *o = out + c * (size_t)(out_dim + 1);
        memset(o, 0, sizeof(uint64_t) * (out_dim + 1));
        o[out_dim] = x[in_dim];
        for (int i = 0; i < in_dim; i++) {
            uint64_t state = orc_closest_representable(x[i], base_log, level) >> (64 - base_log * level);
            for (int l = 0; l < level; l++) {
                uint64_t d = decompose_one_level(base_log, &state, mask);
                const uint64_t *row = ksk + ((size_t)i * level + l) * (size_t)(out_dim + 1);
                for (int j = 0; j <= out_dim; j++) o[j] -= d * row[j];
            }
        }
    }
}

/* ------------------------------------------------------------------------------------ */
/* FFT-free exact PBS (second oracle).                                                    */
/* The same blind rotation (bootstrap.rs:243-344) and external product (ggsw.rs:477-598)  */
/* with every negacyclic product computed exactly in (Z/2^64)[X]/(X^N+1) from the          */
/* STANDARD-domain BSK: Karatsuba over wrapping u64 (ring operations only, so exact mod    */
/* 2^64 whatever the split), checked against the schoolbook orc_negacyclic_mul_u64.       */
/* The reference's own tests pin its FFT only to a tolerance (fft/tests.rs:166-172); this  */
/* oracle is what the GPU's FFT-based PBS is bounded against (tests/test_exact_pbs_gpu.py).*/
/* ------------------------------------------------------------------------------------ */
/* r[0 .. 2n-1) = a * b (full product, wrapping); n a power of two; t: >= 8n words */
static void kara_mul(uint64_t *r, const uint64_t *a, const uint64_t *b, int n, uint64_t *t) {
    if (n <= 32) {
        for (int i = 0; i < 2 * n - 1; i++) r[i] = 0;
        for (int i = 0; i < n; i++) {
            const uint64_t ai = a[i];
            for (int j = 0; j < n; j++) r[i + j] += ai * b[j];
        }
        return;
    }
    const int h = n / 2;
    uint64_t *sa = t, *sb = t + h, *z1 = t + 2 * h, *tt = t + 4 * h;
    for (int i = 0; i < h; i++) {
        sa[i] = a[i] + a[i + h];
        sb[i] = b[i] + b[i + h];
    }
    kara_mul(z1, sa, sb, h, tt);              /* (a0 + a1)(b0 + b1) */
    kara_mul(r, a, b, h, tt);                 /* z0 -> r[0, 2h-1)   */
    r[2 * h - 1] = 0;
    kara_mul(r + 2 * h, a + h, b + h, h, tt); /* z2 -> r[2h, 4h-1)  */
    for (int i = 0; i < 2 * h - 1; i++) z1[i] -= r[i] + r[2 * h + i];
    for (int i = 0; i < 2 * h - 1; i++) r[h + i] += z1[i];
}

/* out += a * b  mod (X^N + 1), exact over Z/2^64.  t: >= 10 N words */
static void negacyclic_mul_add_exact(uint64_t *out, const uint64_t *a, const uint64_t *b, int N, uint64_t *t) {
    uint64_t *full = t, *tt = t + 2 * N;
    kara_mul(full, a, b, N, tt);
    for (int i = 0; i < N - 1; i++) out[i] += full[i] - full[i + N];
    out[N - 1] += full[N - 1];
}

void orc_negacyclic_mul_add_exact(int N, const uint64_t *a, const uint64_t *b, uint64_t *out) {
    uint64_t *t = malloc(sizeof(uint64_t) * 10 * (size_t)N);
    negacyclic_mul_add_exact(out, a, b, N, t);
    free(t);
}

typedef struct {
    const uint64_t *bsk; /* standard [n][L][k+1][k+1][N], borrowed from the caller */
    int n, k, N, base_log, level;
} exact_bsk;

typedef struct {
    uint64_t *ct1, *state, *digits, *t;
} exact_scratch;

/* out += GGSW (x) glwe, exact (ggsw.rs:477-598 with every FFT product replaced by the exact
 * negacyclic product; same decomposition, level order L..1 and rows 0..k) */
static void exact_external_product_add(const exact_bsk *b, const uint64_t *ggsw, uint64_t *out,
                                       const uint64_t *glwe, exact_scratch *s) {
    int k = b->k, N = b->N, L = b->level, beta = b->base_log;
    size_t gl = (size_t)(k + 1) * N;
    uint64_t mask = (1ULL << beta) - 1;
    for (size_t j = 0; j < gl; j++)
        s->state[j] = orc_closest_representable(glwe[j], beta, L) >> (64 - beta * L);
    for (int lvl = L; lvl >= 1; lvl--) {
        const uint64_t *lm = ggsw + (size_t)(lvl - 1) * (k + 1) * (k + 1) * N;
        for (int row = 0; row <= k; row++) {
            uint64_t *st = s->state + (size_t)row * N;
            for (int j = 0; j < N; j++) s->digits[j] = decompose_one_level(beta, &st[j], mask);
            for (int col = 0; col <= k; col++)
                negacyclic_mul_add_exact(out + (size_t)col * N, s->digits, lm + ((size_t)row * (k + 1) + col) * N, N,
                                         s->t);
        }
    }
}

static void exact_pbs_one(const exact_bsk *b, const uint64_t *lwe_in, uint64_t *lwe_out, const uint64_t *lut,
                          uint64_t *acc, exact_scratch *s, int glwe_out) {
    int n = b->n, k = b->k, N = b->N;
    int log2N = 0;
    while ((1 << log2N) < N) log2N++;
    size_t ggsw_len = (size_t)b->level * (k + 1) * (k + 1) * N;
    uint64_t bt = orc_pbs_modulus_switch(lwe_in[n], log2N);
    for (int p = 0; p <= k; p++) monomial_div(acc + (size_t)p * N, lut + (size_t)p * N, N, bt);
    for (int i = 0; i < n; i++) {
        if (lwe_in[i] == 0) continue;
        uint64_t at = orc_pbs_modulus_switch(lwe_in[i], log2N);
        for (int p = 0; p <= k; p++) monomial_mul_sub(s->ct1 + (size_t)p * N, acc + (size_t)p * N, N, at);
        exact_external_product_add(b, b->bsk + (size_t)i * ggsw_len, acc, s->ct1, s);
    }
    if (glwe_out)
        memcpy(lwe_out, acc, sizeof(uint64_t) * (size_t)(k + 1) * N);
    else
        sample_extract0(acc, lwe_out, k, N);
}

typedef struct {
    const exact_bsk *b;
    const uint64_t *in, *luts;
    const uint32_t *lut_idx;
    uint64_t *out;
    size_t count, next;
    pthread_mutex_t mu;
    int glwe_out;
} exact_job;

static void *exact_worker(void *arg) {
    exact_job *J = arg;
    const exact_bsk *b = J->b;
    int k = b->k, N = b->N;
    size_t gl = (size_t)(k + 1) * N;
    exact_scratch s;
    s.ct1 = malloc(sizeof(uint64_t) * gl);
    s.state = malloc(sizeof(uint64_t) * gl);
    s.digits = malloc(sizeof(uint64_t) * N);
    s.t = malloc(sizeof(uint64_t) * 10 * (size_t)N);
    uint64_t *acc = malloc(sizeof(uint64_t) * gl);
    for (;;) {
        pthread_mutex_lock(&J->mu);
        size_t c = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (c >= J->count) break;
        size_t li = J->lut_idx ? J->lut_idx[c] : 0;
        const size_t out_len = J->glwe_out ? gl : (size_t)(k * N + 1);
        exact_pbs_one(b, J->in + c * (size_t)(b->n + 1), J->out + c * out_len, J->luts + li * gl, acc, &s,
                      J->glwe_out);
    }
    free(acc);
    free(s.ct1);
    free(s.state);
    free(s.digits);
    free(s.t);
    return NULL;
}

/* Exact PBS (glwe_out = 0: sample-extracted LWE [count][kN+1]; 1: accumulators [count][(k+1)N]) */
void orc_exact_pbs_batch(const uint64_t *bsk, int n, int k, int N, int base_log, int level, const uint64_t *in,
                         uint64_t *out, const uint64_t *luts, const uint32_t *lut_idx, size_t count, int threads,
                         int glwe_out) {
    exact_bsk b = {bsk, n, k, N, base_log, level};
    exact_job J = {&b, in, luts, lut_idx, out, count, 0};
    J.glwe_out = glwe_out;
    pthread_mutex_init(&J.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, exact_worker, &J);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&J.mu);
}

/* ---- exact multi-bit PBS ---------------------------------------------------------------- */
/* out = X^d p  (d in [0, 2N]; negacyclic: a full N flips the sign) */
static void monomial_mul(uint64_t *out, const uint64_t *p, int N, uint64_t d) {
    uint64_t full = d / N, rem = d % N;
    for (int j = 0; j < N; j++) {
        uint64_t v = (uint64_t)j >= rem ? p[j - rem] : 0 - p[j - rem + N];
        out[j] = (full & 1) ? 0 - v : v;
    }
}

/* FFT-free counterpart of mb_pbs_one (lwe_multi_bit_programmable_bootstrapping.rs:548-828,
 * 18-84): per group j in order, the keybundle KB = GGSW_{j,0} + sum_sel X^{deg_sel} GGSW_{j,sel}
 * exactly in the standard domain (a monomial product is a signed rotation; the sum is ring
 * arithmetic, so its order is immaterial), then acc <- ExtProd(KB, acc) exactly into a zeroed
 * GLWE.  Standard multi-bit BSK [n/g][2^g][L][k+1][k+1][N]. */
static void exact_mb_pbs_one(const exact_bsk *b, int g, const uint64_t *lwe_in, uint64_t *lwe_out, const uint64_t *lut,
                             uint64_t *acc, uint64_t *tmp, uint64_t *kb, uint64_t *rot, exact_scratch *s, int glwe_out) {
    int n = b->n, k = b->k, N = b->N;
    int log2N = 0;
    while ((1 << log2N) < N) log2N++;
    const size_t npoly = (size_t)b->level * (k + 1) * (k + 1);
    const size_t ggsw_len = npoly * N;
    const size_t gl = (size_t)(k + 1) * N;
    uint64_t bt = orc_pbs_modulus_switch(lwe_in[n], log2N);
    for (int p = 0; p <= k; p++) monomial_div(acc + (size_t)p * N, lut + (size_t)p * N, N, bt);
    for (int j = 0; j < n / g; j++) {
        const uint64_t *grp = b->bsk + (size_t)j * ((size_t)1 << g) * ggsw_len;
        memcpy(kb, grp, sizeof(uint64_t) * ggsw_len);
        for (int sel = 1; sel < (1 << g); sel++) {
            uint64_t deg = 0;
            for (int i = 0; i < g; i++)
                if ((sel >> (g - 1 - i)) & 1) deg += lwe_in[(size_t)j * g + i];
            const uint64_t d = orc_pbs_modulus_switch(deg, log2N);
            const uint64_t *G = grp + (size_t)sel * ggsw_len;
            for (size_t q = 0; q < npoly; q++) {
                monomial_mul(rot, G + q * N, N, d);
                for (int t = 0; t < N; t++) kb[q * N + t] += rot[t];
            }
        }
        memset(tmp, 0, sizeof(uint64_t) * gl);
        exact_external_product_add(b, kb, tmp, acc, s);
        memcpy(acc, tmp, sizeof(uint64_t) * gl);
    }
    if (glwe_out)
        memcpy(lwe_out, acc, sizeof(uint64_t) * gl);
    else
        sample_extract0(acc, lwe_out, k, N);
}

typedef struct {
    const exact_bsk *b;
    int g;
    const uint64_t *in, *luts;
    const uint32_t *lut_idx;
    uint64_t *out;
    size_t count, next;
    pthread_mutex_t mu;
    int glwe_out;
} exact_mb_job;

static void *exact_mb_worker(void *arg) {
    exact_mb_job *J = arg;
    const exact_bsk *b = J->b;
    int k = b->k, N = b->N;
    size_t gl = (size_t)(k + 1) * N;
    exact_scratch s;
    s.ct1 = NULL;
    s.state = malloc(sizeof(uint64_t) * gl);
    s.digits = malloc(sizeof(uint64_t) * N);
    s.t = malloc(sizeof(uint64_t) * 10 * (size_t)N);
    uint64_t *acc = malloc(sizeof(uint64_t) * gl), *tmp = malloc(sizeof(uint64_t) * gl);
    uint64_t *kb = malloc(sizeof(uint64_t) * (size_t)b->level * (k + 1) * (k + 1) * N);
    uint64_t *rot = malloc(sizeof(uint64_t) * N);
    for (;;) {
        pthread_mutex_lock(&J->mu);
        size_t c = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (c >= J->count) break;
        size_t li = J->lut_idx ? J->lut_idx[c] : 0;
        const size_t out_len = J->glwe_out ? gl : (size_t)(k * N + 1);
        exact_mb_pbs_one(b, J->g, J->in + c * (size_t)(b->n + 1), J->out + c * out_len, J->luts + li * gl, acc, tmp,
                         kb, rot, &s, J->glwe_out);
    }
    free(acc);
    free(tmp);
    free(kb);
    free(rot);
    free(s.state);
    free(s.digits);
    free(s.t);
    return NULL;
}

void orc_exact_mb_pbs_batch(const uint64_t *bsk, int n, int k, int N, int base_log, int level, int g,
                            const uint64_t *in, uint64_t *out, const uint64_t *luts, const uint32_t *lut_idx,
                            size_t count, int threads, int glwe_out) {
    exact_bsk b = {bsk, n, k, N, base_log, level};
    exact_mb_job J = {&b, g, in, luts, lut_idx, out, count, 0};
    J.glwe_out = glwe_out;
    pthread_mutex_init(&J.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, exact_mb_worker, &J);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&J.mu);
}
