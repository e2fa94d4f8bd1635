/* pbs_simd.c -- CPU BASELINE ONLY (bench.py's cpu_baseline leg), checked bit for bit against
 * pbs_oracle.c by tests/test_oracle_simd.py.  Never linked or loaded by the product.
 *
 * The oracle's classic PBS (pbs_oracle.c pbs_one / external_product_add, restating
 * bootstrap.rs:243-380 and ggsw.rs:477-697 with the engine's fixed FFT DAG) with W independent
 * ciphertexts in the W lanes of one SIMD register (AVX-512: W = 8, AVX2: W = 4).  Every lane runs
 * exactly the oracle's scalar operation sequence -- the same adds, multiplies, explicit fmas,
 * sign flips and roundings in the same order, no contraction (-ffp-contract=off) -- so outputs are
 * bit-identical to the oracle; only the throughput differs.  This is the reference bench's
 * par_iter throughput form (benches/core_crypto/pbs_bench.rs:430-549) on the host cores, with each
 * core's vector unit filled by W ciphertexts instead of by one FFT (concrete-fft's choice).
 *
 * A zero mask element is executed as a rotation by 0 instead of skipped: X^0 acc - acc = 0, whose
 * digits, spectra and backward increments are all (signed) zeros that add 0, the same result.
 */
#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#if defined(__AVX512F__) && defined(__AVX512DQ__)
#define W 8
typedef __m512d vd;
#define vset1 _mm512_set1_pd
#define vzero _mm512_setzero_pd
#define vadd _mm512_add_pd
#define vsub _mm512_sub_pd
#define vmul _mm512_mul_pd
#define vfma _mm512_fmadd_pd
#define vxor _mm512_xor_pd
#define vrint(x) _mm512_roundscale_pd((x), _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC)
#define vload _mm512_load_pd
#define vstore _mm512_store_pd
static inline vd vcvt_i64(const int64_t *p) { return _mm512_cvtepi64_pd(_mm512_loadu_si512((const void *)p)); }
#elif defined(__AVX2__) && defined(__FMA__)
#define W 4
typedef __m256d vd;
#define vset1 _mm256_set1_pd
#define vzero _mm256_setzero_pd
#define vadd _mm256_add_pd
#define vsub _mm256_sub_pd
#define vmul _mm256_mul_pd
#define vfma _mm256_fmadd_pd
#define vxor _mm256_xor_pd
#define vrint(x) _mm256_round_pd((x), _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC)
#define vload _mm256_load_pd
#define vstore _mm256_store_pd
static inline vd vcvt_i64(const int64_t *p) {
    return _mm256_set_pd((double)p[3], (double)p[2], (double)p[1], (double)p[0]);
}
#else
#error "pbs_simd.c needs AVX2+FMA or AVX-512F/DQ"
#endif

#define ALIGN 64
/* -(x): sign flip, as the oracle's unary minus (differs from 0 - x on zeros) */
static inline vd vneg(vd x) { return vxor(x, vset1(-0.0)); }

typedef struct {
    vd re, im;
} vcx;

static inline vcx cadd(vcx a, vcx b) { return (vcx){vadd(a.re, b.re), vadd(a.im, b.im)}; }
static inline vcx csub(vcx a, vcx b) { return (vcx){vsub(a.re, b.re), vsub(a.im, b.im)}; }
/* (fma(xr,wr,-(xi*wi)), fma(xr,wi,xi*wr)) */
static inline vcx cmulw(vcx x, double wr, double wi) {
    const vd r = vset1(wr), i = vset1(wi);
    return (vcx){vfma(x.re, r, vneg(vmul(x.im, i))), vfma(x.re, i, vmul(x.im, r))};
}

#define C16_1 0x1.d906bcf328d46p-1 /* cos(pi/8) */
#define S16_1 0x1.87de2a6aea963p-2 /* sin(pi/8) */
#define SQH 0x1.6a09e667f3bcdp-1   /* sqrt(1/2) */
static inline vcx mul_w8(vcx x) { return (vcx){vmul(vadd(x.re, x.im), vset1(SQH)), vmul(vsub(x.im, x.re), vset1(SQH))}; }
static inline vcx mul_w8_3(vcx x) {
    return (vcx){vmul(vsub(x.im, x.re), vset1(SQH)), vneg(vmul(vadd(x.re, x.im), vset1(SQH)))};
}
static inline vcx mul_w8c(vcx x) { return (vcx){vmul(vsub(x.re, x.im), vset1(SQH)), vmul(vadd(x.re, x.im), vset1(SQH))}; }
static inline vcx mul_w8_3c(vcx x) {
    return (vcx){vneg(vmul(vadd(x.re, x.im), vset1(SQH))), vmul(vsub(x.re, x.im), vset1(SQH))};
}
static inline vcx mul_mi(vcx x) { return (vcx){x.im, vneg(x.re)}; }
static inline vcx mul_pi(vcx x) { return (vcx){vneg(x.im), x.re}; }

static inline void r4_fwd(vcx *x0, vcx *x1, vcx *x2, vcx *x3) {
    vcx t0 = cadd(*x0, *x2), t1 = csub(*x0, *x2), t2 = cadd(*x1, *x3), t3 = csub(*x1, *x3);
    *x0 = cadd(t0, t2);
    *x2 = csub(t0, t2);
    *x1 = (vcx){vadd(t1.re, t3.im), vsub(t1.im, t3.re)};
    *x3 = (vcx){vsub(t1.re, t3.im), vadd(t1.im, t3.re)};
}
static inline void r4_inv(vcx *x0, vcx *x1, vcx *x2, vcx *x3) {
    vcx t0 = cadd(*x0, *x2), t1 = csub(*x0, *x2), t2 = cadd(*x1, *x3), t3 = csub(*x1, *x3);
    *x0 = cadd(t0, t2);
    *x2 = csub(t0, t2);
    *x1 = (vcx){vsub(t1.re, t3.im), vadd(t1.im, t3.re)};
    *x3 = (vcx){vadd(t1.re, t3.im), vsub(t1.im, t3.re)};
}
static inline vcx tw16_fwd(vcx x, int e) {
    switch (e) {
    case 0: return x;
    case 1: return cmulw(x, C16_1, -S16_1);
    case 2: return mul_w8(x);
    case 3: return cmulw(x, S16_1, -C16_1);
    case 4: return mul_mi(x);
    case 6: return mul_w8_3(x);
    default: return cmulw(x, -C16_1, S16_1); /* 9 */
    }
}
static inline vcx tw16_inv(vcx x, int e) {
    switch (e) {
    case 0: return x;
    case 1: return cmulw(x, C16_1, S16_1);
    case 2: return mul_w8c(x);
    case 3: return cmulw(x, S16_1, C16_1);
    case 4: return mul_pi(x);
    case 6: return mul_w8_3c(x);
    default: return cmulw(x, -C16_1, -S16_1); /* 9 */
    }
}
static inline vcx tw8_fwd(vcx x, int e) {
    switch (e) {
    case 0: return x;
    case 1: return mul_w8(x);
    case 2: return mul_mi(x);
    default: return mul_w8_3(x);
    }
}
static inline vcx tw8_inv(vcx x, int e) {
    switch (e) {
    case 0: return x;
    case 1: return mul_w8c(x);
    case 2: return mul_pi(x);
    default: return mul_w8_3c(x);
    }
}

/* pbs_oracle.c dft_fwd / dft_inv, lane-parallel */
static void dft_fwd(vcx *v, int R) {
    if (R == 2) {
        vcx a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    } else if (R == 4) {
        r4_fwd(&v[0], &v[1], &v[2], &v[3]);
    } else if (R == 8) {
        vcx u[2][4];
        for (int a = 0; a < 2; a++) {
            vcx y0 = v[a], y1 = v[a + 2], y2 = v[a + 4], y3 = v[a + 6];
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
    } else {
        vcx u[4][4];
        for (int a = 0; a < 4; a++) {
            vcx y0 = v[a], y1 = v[a + 4], y2 = v[a + 8], y3 = v[a + 12];
            r4_fwd(&y0, &y1, &y2, &y3);
            u[a][0] = y0;
            u[a][1] = tw16_fwd(y1, a * 1);
            u[a][2] = tw16_fwd(y2, a * 2);
            u[a][3] = tw16_fwd(y3, a * 3);
        }
        for (int c = 0; c < 4; c++) {
            vcx y0 = u[0][c], y1 = u[1][c], y2 = u[2][c], y3 = u[3][c];
            r4_fwd(&y0, &y1, &y2, &y3);
            v[c] = y0;
            v[c + 4] = y1;
            v[c + 8] = y2;
            v[c + 12] = y3;
        }
    }
}
static void dft_inv(vcx *v, int R) {
    if (R == 2) {
        vcx a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    } else if (R == 4) {
        r4_inv(&v[0], &v[1], &v[2], &v[3]);
    } else if (R == 8) {
        vcx u[2][4];
        for (int c = 0; c < 4; c++) {
            u[0][c] = cadd(v[c], v[c + 4]);
            u[1][c] = csub(v[c], v[c + 4]);
        }
        for (int a = 0; a < 2; a++) {
            vcx y0 = u[a][0], y1 = tw8_inv(u[a][1], a * 1), y2 = tw8_inv(u[a][2], a * 2), y3 = tw8_inv(u[a][3], a * 3);
            r4_inv(&y0, &y1, &y2, &y3);
            v[a] = y0;
            v[a + 2] = y1;
            v[a + 4] = y2;
            v[a + 6] = y3;
        }
    } else {
        vcx u[4][4];
        for (int c = 0; c < 4; c++) {
            vcx y0 = v[c], y1 = v[c + 4], y2 = v[c + 8], y3 = v[c + 12];
            r4_inv(&y0, &y1, &y2, &y3);
            u[0][c] = y0;
            u[1][c] = y1;
            u[2][c] = y2;
            u[3][c] = y3;
        }
        for (int a = 0; a < 4; a++) {
            vcx y0 = u[a][0], y1 = tw16_inv(u[a][1], a * 1), y2 = tw16_inv(u[a][2], a * 2),
                y3 = tw16_inv(u[a][3], a * 3);
            r4_inv(&y0, &y1, &y2, &y3);
            v[a] = y0;
            v[a + 4] = y1;
            v[a + 8] = y2;
            v[a + 12] = y3;
        }
    }
}

typedef struct {
    int N, M, nrad, rad[8];
    double *Wre, *Wim, *twre, *twim;
} sfft;

/* the oracle's radix plans (pbs_oracle.c radix_plan) */
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
    default: return 0;
    }
}
/* same tables as the oracle: cos and sin through opaque pointers (never fused into sincos) */
static double (*volatile s_cos)(double) = cos;
static double (*volatile s_sin)(double) = sin;
static int sfft_init(sfft *f, int N) {
    f->N = N;
    f->M = N / 2;
    f->nrad = radix_plan(f->M, f->rad);
    if (!f->nrad) return -1;
    const int M = f->M;
    f->Wre = malloc(sizeof(double) * M);
    f->Wim = malloc(sizeof(double) * M);
    f->twre = malloc(sizeof(double) * M);
    f->twim = malloc(sizeof(double) * M);
    for (int t = 0; t < M; t++) {
        double ang = 2.0 * M_PI * (double)t / (double)M;
        f->Wre[t] = s_cos(ang);
        f->Wim[t] = -s_sin(ang);
    }
    double unit = M_PI / (2.0 * (double)M);
    for (int j = 0; j < M; j++) {
        double a = (double)j * unit;
        f->twre[j] = s_cos(a);
        f->twim[j] = s_sin(a);
    }
    return 0;
}
static void sfft_free(sfft *f) {
    free(f->Wre);
    free(f->Wim);
    free(f->twre);
    free(f->twim);
}

static void dif_rec(const sfft *f, vcx *z, int off, int L, int stage) {
    const int R = f->rad[stage], m = L / R, tstride = f->M / L;
    vcx v[16];
    for (int a = 0; a < m; a++) {
        for (int b = 0; b < R; b++) v[b] = z[off + a + m * b];
        dft_fwd(v, R);
        for (int c = 0; c < R; c++) {
            const int t = a * c;
            vcx y = v[c];
            if (t) y = cmulw(y, f->Wre[t * tstride], f->Wim[t * tstride]);
            z[off + a + m * c] = y;
        }
    }
    if (m > 1)
        for (int c = 0; c < R; c++) dif_rec(f, z, off + m * c, m, stage + 1);
}
static void dit_rec(const sfft *f, vcx *z, int off, int L, int stage) {
    const int R = f->rad[stage], m = L / R, tstride = f->M / L;
    vcx v[16];
    if (m > 1)
        for (int c = 0; c < R; c++) dit_rec(f, z, off + m * c, m, stage + 1);
    for (int a = 0; a < m; a++) {
        for (int c = 0; c < R; c++) {
            const int t = a * c;
            vcx y = z[off + a + m * c];
            if (t) y = cmulw(y, f->Wre[t * tstride], -f->Wim[t * tstride]);
            v[c] = y;
        }
        dft_inv(v, R);
        for (int b = 0; b < R; b++) z[off + a + m * b] = v[b];
    }
}

/* the oracle's f64 -> i64 bit twiddle (pbs_oracle.c orc_f64_to_i64) */
static inline int64_t f64_to_i64(double x) {
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

/* forward_integer: digits [N][W] (signed, as i64) -> spectrum z[M] */
static void forward_integer(const sfft *f, const int64_t *dig, vcx *z) {
    const int M = f->M;
    for (int j = 0; j < M; j++) {
        vcx in = {vcvt_i64(dig + (size_t)j * W), vcvt_i64(dig + (size_t)(j + M) * W)};
        z[j] = cmulw(in, f->twre[j], f->twim[j]);
    }
    dif_rec(f, z, 0, M, 0);
}

/* backward_torus with add: out[N][W] += rounded torus values of z (destroyed) */
static void backward_torus_add(const sfft *f, vcx *z, uint64_t *out) {
    const int M = f->M;
    dit_rec(f, z, 0, M, 0);
    const double norm = 1.0 / (double)M;
    const vd two64 = vset1(18446744073709551616.0);
    double __attribute__((aligned(ALIGN))) br[W], bi[W];
    for (int j = 0; j < M; j++) {
        const vd wr = vset1(norm * f->twre[j]), wi = vset1(norm * f->twim[j]);
        const vd mr = vfma(z[j].re, wr, vmul(z[j].im, wi));
        const vd mi = vfma(vneg(z[j].re), wi, vmul(z[j].im, wr));
        const vd fr = vsub(mr, vrint(mr)), fi = vsub(mi, vrint(mi));
        uint64_t *o0 = out + (size_t)j * W, *o1 = out + (size_t)(j + M) * W;
#if W == 8
        /* |rint(fract * 2^64)| <= 2^63 and integral: the packed conversion gives the bit twiddle's
         * value (2^63 and -2^63 both map to 0x8000000000000000, as the twiddle's wrap does) */
        const __m512i vr = _mm512_cvtpd_epi64(vrint(vmul(fr, two64)));
        const __m512i vi = _mm512_cvtpd_epi64(vrint(vmul(fi, two64)));
        _mm512_storeu_si512((void *)o0, _mm512_add_epi64(_mm512_loadu_si512((const void *)o0), vr));
        _mm512_storeu_si512((void *)o1, _mm512_add_epi64(_mm512_loadu_si512((const void *)o1), vi));
        (void)br;
        (void)bi;
#else
        vstore(br, vrint(vmul(fr, two64)));
        vstore(bi, vrint(vmul(fi, two64)));
        for (int l = 0; l < W; l++) {
            o0[l] += (uint64_t)f64_to_i64(br[l]);
            o1[l] += (uint64_t)f64_to_i64(bi[l]);
        }
#endif
    }
}

static inline uint64_t closest_representable(uint64_t x, int base_log, int level) {
    const int shift = 64 - base_log * level - 1;
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

typedef struct {
    int n, k, N, base_log, level, log2N;
    sfft fft;
    const double *fourier; /* [n][L][k+1][k+1][M] complex, position order (oracle FourierBsk) */
} simd_bsk;

typedef struct {
    uint64_t *acc, *ct1, *state;
    int64_t *dig;
    vcx *fd, *facc;
} lanes_scratch;

/* external_product_add of W ciphertexts: acc[(k+1)N][W] += GGSW (x) ct1 */
static void external_product_add(const simd_bsk *b, const double *ggsw, lanes_scratch *s) {
    const int k = b->k, N = b->N, M = N / 2, L = b->level, beta = b->base_log;
    const size_t gl = (size_t)(k + 1) * N * W;
    const uint64_t mask = (1ULL << beta) - 1;
    for (size_t e = 0; e < gl; e++) s->state[e] = closest_representable(s->ct1[e], beta, L) >> (64 - beta * L);
    int first = 1;
    for (int lvl = L; lvl >= 1; lvl--) {
        const double *lm = ggsw + (size_t)(lvl - 1) * (k + 1) * (k + 1) * M * 2;
        for (int row = 0; row <= k; row++) {
            uint64_t *st = s->state + (size_t)row * N * W;
            for (size_t e = 0; e < (size_t)N * W; e++) s->dig[e] = (int64_t)decompose_one_level(beta, &st[e], mask);
            forward_integer(&b->fft, s->dig, s->fd);
            for (int col = 0; col <= k; col++) {
                const double *g = lm + ((size_t)row * (k + 1) + col) * M * 2;
                vcx *acc = s->facc + (size_t)col * M;
                if (first) {
                    for (int f = 0; f < M; f++) {
                        const vd gr = vset1(g[2 * f]), gi = vset1(g[2 * f + 1]);
                        const vd dr = s->fd[f].re, di = s->fd[f].im;
                        acc[f].re = vfma(gr, dr, vneg(vmul(gi, di)));
                        acc[f].im = vfma(gr, di, vmul(gi, dr));
                    }
                } else {
                    for (int f = 0; f < M; f++) {
                        const vd gr = vset1(g[2 * f]), gi = vset1(g[2 * f + 1]);
                        const vd dr = s->fd[f].re, di = s->fd[f].im;
                        acc[f].re = vfma(gr, dr, vfma(vneg(gi), di, acc[f].re));
                        acc[f].im = vfma(gr, di, vfma(gi, dr, acc[f].im));
                    }
                }
            }
            first = 0;
        }
    }
    for (int col = 0; col <= k; col++) backward_torus_add(&b->fft, s->facc + (size_t)col * M, s->acc + (size_t)col * N * W);
}

static inline uint64_t modulus_switch(uint64_t x, int log2N) {
    uint64_t o = x >> (64 - log2N - 2);
    o += 1;
    o >>= 1;
    return o;
}

/* W ciphertexts (rows of `in`, `nct` <= W real, the rest padded with the last) */
static void pbs_lanes(const simd_bsk *b, const uint64_t *const *in, const uint64_t *const *lut, lanes_scratch *s) {
    const int n = b->n, k = b->k, N = b->N, M = N / 2;
    const size_t ggsw_len = (size_t)b->level * (k + 1) * (k + 1) * M * 2;
    /* acc = LUT / X^{b~}  (monomial_div) */
    for (int l = 0; l < W; l++) {
        const uint64_t d = modulus_switch(in[l][n], b->log2N);
        const uint64_t full = d / N, rem = d % N;
        for (int p = 0; p <= k; p++)
            for (int j = 0; j < N; j++) {
                const uint64_t src = j + rem;
                uint64_t v = src < (uint64_t)N ? lut[l][(size_t)p * N + src] : 0 - lut[l][(size_t)p * N + src - N];
                s->acc[((size_t)p * N + j) * W + l] = (full & 1) ? 0 - v : v;
            }
    }
    for (int i = 0; i < n; i++) {
        /* ct1 = X^{a~} acc - acc  (monomial_mul_sub) */
        for (int l = 0; l < W; l++) {
            const uint64_t d = modulus_switch(in[l][i], b->log2N);
            const uint64_t full = d / N, rem = d % N;
            for (int p = 0; p <= k; p++) {
                const uint64_t *a = s->acc + (size_t)p * N * W + l;
                uint64_t *o = s->ct1 + (size_t)p * N * W + l;
                for (uint64_t j = 0; j < rem; j++) {
                    const uint64_t src = a[(N - rem + j) * W];
                    o[j * W] = ((full & 1) ? src : 0 - src) - a[j * W];
                }
                for (uint64_t j = rem; j < (uint64_t)N; j++) {
                    const uint64_t src = a[(j - rem) * W];
                    o[j * W] = ((full & 1) ? 0 - src : src) - a[j * W];
                }
            }
        }
        external_product_add(b, b->fourier + (size_t)i * ggsw_len, s);
    }
    (void)M;
}

typedef struct {
    const simd_bsk *b;
    const uint64_t *in, *luts;
    const uint32_t *lut_idx;
    uint64_t *out;
    size_t count, next;
    pthread_mutex_t mu;
} simd_job;

static void *simd_worker(void *arg) {
    simd_job *J = arg;
    const simd_bsk *b = J->b;
    const int k = b->k, N = b->N, M = N / 2;
    lanes_scratch s;
    const size_t gl = (size_t)(k + 1) * N * W;
    s.acc = aligned_alloc(ALIGN, sizeof(uint64_t) * gl);
    s.ct1 = aligned_alloc(ALIGN, sizeof(uint64_t) * gl);
    s.state = aligned_alloc(ALIGN, sizeof(uint64_t) * gl);
    s.dig = aligned_alloc(ALIGN, sizeof(int64_t) * (size_t)N * W);
    s.fd = aligned_alloc(ALIGN, sizeof(vcx) * M);
    s.facc = aligned_alloc(ALIGN, sizeof(vcx) * (size_t)(k + 1) * M);
    const size_t out_len = (size_t)k * N + 1;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        const size_t c0 = J->next;
        J->next += W;
        pthread_mutex_unlock(&J->mu);
        if (c0 >= J->count) break;
        const uint64_t *in[W], *lut[W];
        for (int l = 0; l < W; l++) {
            const size_t c = c0 + l < J->count ? c0 + l : J->count - 1;
            in[l] = J->in + c * (size_t)(b->n + 1);
            lut[l] = J->luts + (J->lut_idx ? J->lut_idx[c] : 0) * (size_t)(k + 1) * N;
        }
        pbs_lanes(b, in, lut, &s);
        /* sample extract at degree 0 */
        for (int l = 0; l < W && c0 + l < J->count; l++) {
            uint64_t *o = J->out + (c0 + l) * out_len;
            for (int p = 0; p < k; p++) {
                const uint64_t *a = s.acc + (size_t)p * N * W + l;
                o[(size_t)p * N] = a[0];
                for (int j = 1; j < N; j++) o[(size_t)p * N + j] = 0 - a[(size_t)(N - j) * W];
            }
            o[(size_t)k * N] = s.acc[(size_t)k * N * W + l];
        }
    }
    free(s.acc);
    free(s.ct1);
    free(s.state);
    free(s.dig);
    free(s.fd);
    free(s.facc);
    return NULL;
}

int simd_width(void) { return W; }

/* Classic PBS of `count` ciphertexts, W per thread step; fourier = the oracle's Fourier BSK. */
int simd_pbs_batch(const double *fourier, int n, int k, int N, int base_log, int level, const uint64_t *in,
                   uint64_t *out, const uint64_t *luts, const uint32_t *lut_idx, size_t count, int threads) {
    simd_bsk b = {n, k, N, base_log, level, 0};
    while ((1 << b.log2N) < N) b.log2N++;
    if (sfft_init(&b.fft, N)) return -1;
    b.fourier = fourier;
    simd_job J = {&b, in, luts, lut_idx, out, count, 0};
    pthread_mutex_init(&J.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, simd_worker, &J);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&J.mu);
    sfft_free(&b.fft);
    return 0;
}

/* The oracle's keyswitch (pbs_oracle.c orc_keyswitch_batch, lwe_keyswitch.rs:96-170), compiled
 * here with the SIMD build's flags: the per-level AXPY over the output row vectorises (u64
 * multiply-subtract, exact), so it is bit-identical by construction. */
void simd_keyswitch_batch(const uint64_t *ksk, int in_dim, int out_dim, int base_log, int level, const uint64_t *in,
                          uint64_t *out, size_t count) {
    const uint64_t mask = (1ULL << base_log) - 1;
    for (size_t c = 0; c < count; c++) {
        const uint64_t *x = in + c * (size_t)(in_dim + 1);
        uint64_t *o = out + c * (size_t)(out_dim + 1);
        memset(o, 0, sizeof(uint64_t) * (out_dim + 1));
        o[out_dim] = x[in_dim];
        for (int i = 0; i < in_dim; i++) {
            uint64_t state = closest_representable(x[i], base_log, level) >> (64 - base_log * level);
            for (int l = 0; l < level; l++) {
                const uint64_t d = decompose_one_level(base_log, &state, mask);
                const uint64_t *row = ksk + ((size_t)i * level + l) * (size_t)(out_dim + 1);
                for (int j = 0; j <= out_dim; j++) o[j] -= d * row[j];
            }
        }
    }
}

/* ---- multi-bit PBS, W ciphertexts per register (pbs_oracle.c mb_pbs_one / mb_keybundle) ---- */
/* frequency of FFT output position P (pbs_oracle.c pos_freq) */
static int pos_freq(const sfft *f, int P) {
    int fr = 0, mult = 1, L = f->M;
    for (int st = 0; st < f->nrad; st++) {
        const int m = L / f->rad[st];
        fr += mult * (P / m);
        P %= m;
        mult *= f->rad[st];
        L = m;
    }
    return fr;
}
/* spectrum of X^d at frequency fr (pbs_oracle.c mono_spectrum): exact i^q twist[r] */
static inline void mono_spectrum(const sfft *f, uint32_t d, int fr, double *re, double *im) {
    const uint32_t t = (d - 4u * d * (uint32_t)fr) & (uint32_t)(2 * f->N - 1);
    const uint32_t q = t / (uint32_t)f->M, r = t % (uint32_t)f->M;
    const double wr = f->twre[r], wi = f->twim[r];
    switch (q) {
    case 0: *re = wr; *im = wi; break;
    case 1: *re = -wi; *im = wr; break;
    case 2: *re = -wr; *im = -wi; break;
    default: *re = wi; *im = -wr; break;
    }
}

typedef struct {
    simd_bsk b;  /* b.fourier: [n/g][2^g][L][k+1][k+1][M] complex, position order */
    int g;
    int *freq;
} simd_mb_bsk;

typedef struct {
    lanes_scratch s;
    uint64_t *tmp;
    vcx *kb, *mono;
} mb_scratch;

/* external_product_add with a per-lane GGSW (the keybundles): out[(k+1)N][W] += KB (x) glwe[...] */
static void external_product_add_v(const simd_bsk *b, const vcx *kb, const uint64_t *glwe, uint64_t *out,
                                   lanes_scratch *s) {
    const int k = b->k, N = b->N, M = N / 2, L = b->level, beta = b->base_log;
    const size_t gl = (size_t)(k + 1) * N * W;
    const uint64_t mask = (1ULL << beta) - 1;
    for (size_t e = 0; e < gl; e++) s->state[e] = closest_representable(glwe[e], beta, L) >> (64 - beta * L);
    int first = 1;
    for (int lvl = L; lvl >= 1; lvl--) {
        const vcx *lm = kb + (size_t)(lvl - 1) * (k + 1) * (k + 1) * M;
        for (int row = 0; row <= k; row++) {
            uint64_t *st = s->state + (size_t)row * N * W;
            for (size_t e = 0; e < (size_t)N * W; e++) s->dig[e] = (int64_t)decompose_one_level(beta, &st[e], mask);
            forward_integer(&b->fft, s->dig, s->fd);
            for (int col = 0; col <= k; col++) {
                const vcx *g = lm + ((size_t)row * (k + 1) + col) * M;
                vcx *acc = s->facc + (size_t)col * M;
                for (int f = 0; f < M; f++) {
                    const vd gr = g[f].re, gi = g[f].im, dr = s->fd[f].re, di = s->fd[f].im;
                    if (first) {
                        acc[f].re = vfma(gr, dr, vneg(vmul(gi, di)));
                        acc[f].im = vfma(gr, di, vmul(gi, dr));
                    } else {
                        acc[f].re = vfma(gr, dr, vfma(vneg(gi), di, acc[f].re));
                        acc[f].im = vfma(gr, di, vfma(gi, dr, acc[f].im));
                    }
                }
            }
            first = 0;
        }
    }
    for (int col = 0; col <= k; col++) backward_torus_add(&b->fft, s->facc + (size_t)col * M, out + (size_t)col * N * W);
}

static void mb_pbs_lanes(const simd_mb_bsk *mb, const uint64_t *const *in, const uint64_t *const *lut, mb_scratch *ms) {
    const simd_bsk *b = &mb->b;
    lanes_scratch *s = &ms->s;
    const int n = b->n, k = b->k, N = b->N, M = N / 2, g = mb->g;
    const size_t npoly = (size_t)b->level * (k + 1) * (k + 1);
    const size_t ggsw_len = npoly * M * 2;  /* doubles */
    const size_t gl = (size_t)(k + 1) * N * W;
    for (int l = 0; l < W; l++) {  /* acc = LUT / X^{b~} */
        const uint64_t d = modulus_switch(in[l][n], b->log2N);
        const uint64_t full = d / N, rem = d % N;
        for (int p = 0; p <= k; p++)
            for (int j = 0; j < N; j++) {
                const uint64_t src = j + rem;
                uint64_t v = src < (uint64_t)N ? lut[l][(size_t)p * N + src] : 0 - lut[l][(size_t)p * N + src - N];
                s->acc[((size_t)p * N + j) * W + l] = (full & 1) ? 0 - v : v;
            }
    }
    double __attribute__((aligned(ALIGN))) mr[W], mi[W];
    for (int j = 0; j < n / g; j++) {
        const double *grp = b->fourier + (size_t)j * ((size_t)1 << g) * ggsw_len;
        /* keybundle, per lane, in the oracle's order: GGSW_0, then sel = 1 .. 2^g - 1 */
        for (size_t e = 0; e < npoly * M; e++) ms->kb[e] = (vcx){vset1(grp[2 * e]), vset1(grp[2 * e + 1])};
        for (int sel = 1; sel < (1 << g); sel++) {
            uint32_t d[W];
            for (int l = 0; l < W; l++) {
                uint64_t deg = 0;
                for (int i = 0; i < g; i++)
                    if ((sel >> (g - 1 - i)) & 1) deg += in[l][(size_t)j * g + i];
                d[l] = (uint32_t)modulus_switch(deg, b->log2N);
            }
            for (int P = 0; P < M; P++) {
                for (int l = 0; l < W; l++) mono_spectrum(&b->fft, d[l], mb->freq[P], &mr[l], &mi[l]);
                ms->mono[P] = (vcx){vload(mr), vload(mi)};
            }
            const double *G = grp + (size_t)sel * ggsw_len;
            for (size_t q = 0; q < npoly; q++)
                for (int P = 0; P < M; P++) {
                    const vd gr = vset1(G[2 * (q * M + P)]), gi = vset1(G[2 * (q * M + P) + 1]);
                    const vcx m = ms->mono[P];
                    vcx *o = &ms->kb[q * M + P];
                    o->re = vfma(gr, m.re, vfma(vneg(gi), m.im, o->re));
                    o->im = vfma(gr, m.im, vfma(gi, m.re, o->im));
                }
        }
        /* acc <- ExtProd(KB, acc) into a zeroed GLWE (ping-pong) */
        memset(ms->tmp, 0, sizeof(uint64_t) * gl);
        external_product_add_v(b, ms->kb, s->acc, ms->tmp, s);
        memcpy(s->acc, ms->tmp, sizeof(uint64_t) * gl);
    }
}

typedef struct {
    const simd_mb_bsk *mb;
    const uint64_t *in, *luts;
    const uint32_t *lut_idx;
    uint64_t *out;
    size_t count, next;
    pthread_mutex_t mu;
} simd_mb_job;

static void *simd_mb_worker(void *arg) {
    simd_mb_job *J = arg;
    const simd_bsk *b = &J->mb->b;
    const int k = b->k, N = b->N, M = N / 2;
    const size_t gl = (size_t)(k + 1) * N * W;
    mb_scratch ms;
    lanes_scratch *s = &ms.s;
    s->acc = aligned_alloc(ALIGN, sizeof(uint64_t) * gl);
    s->ct1 = NULL;
    s->state = aligned_alloc(ALIGN, sizeof(uint64_t) * gl);
    s->dig = aligned_alloc(ALIGN, sizeof(int64_t) * (size_t)N * W);
    s->fd = aligned_alloc(ALIGN, sizeof(vcx) * M);
    s->facc = aligned_alloc(ALIGN, sizeof(vcx) * (size_t)(k + 1) * M);
    ms.tmp = aligned_alloc(ALIGN, sizeof(uint64_t) * gl);
    ms.kb = aligned_alloc(ALIGN, sizeof(vcx) * (size_t)b->level * (k + 1) * (k + 1) * M);
    ms.mono = aligned_alloc(ALIGN, sizeof(vcx) * M);
    const size_t out_len = (size_t)k * N + 1;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        const size_t c0 = J->next;
        J->next += W;
        pthread_mutex_unlock(&J->mu);
        if (c0 >= J->count) break;
        const uint64_t *in[W], *lut[W];
        for (int l = 0; l < W; l++) {
            const size_t c = c0 + l < J->count ? c0 + l : J->count - 1;
            in[l] = J->in + c * (size_t)(b->n + 1);
            lut[l] = J->luts + (J->lut_idx ? J->lut_idx[c] : 0) * (size_t)(k + 1) * N;
        }
        mb_pbs_lanes(J->mb, in, lut, &ms);
        for (int l = 0; l < W && c0 + l < J->count; l++) {  /* sample extract at degree 0 */
            uint64_t *o = J->out + (c0 + l) * out_len;
            for (int p = 0; p < k; p++) {
                const uint64_t *a = s->acc + (size_t)p * N * W + l;
                o[(size_t)p * N] = a[0];
                for (int j = 1; j < N; j++) o[(size_t)p * N + j] = 0 - a[(size_t)(N - j) * W];
            }
            o[(size_t)k * N] = s->acc[(size_t)k * N * W + l];
        }
    }
    free(s->acc);
    free(s->state);
    free(s->dig);
    free(s->fd);
    free(s->facc);
    free(ms.tmp);
    free(ms.kb);
    free(ms.mono);
    return NULL;
}

/* Multi-bit PBS (deterministic group order) of `count` ciphertexts, W per thread step;
 * fourier = the oracle's multi-bit Fourier BSK (orc_mb_fbsk_copy). */
int simd_mb_pbs_batch(const double *fourier, int n, int k, int N, int base_log, int level, int g, const uint64_t *in,
                      uint64_t *out, const uint64_t *luts, const uint32_t *lut_idx, size_t count, int threads) {
    if (g < 1 || n % g) return -1;
    simd_mb_bsk mb = {{n, k, N, base_log, level, 0}, g, NULL};
    while ((1 << mb.b.log2N) < N) mb.b.log2N++;
    if (sfft_init(&mb.b.fft, N)) return -1;
    mb.b.fourier = fourier;
    mb.freq = malloc(sizeof(int) * (N / 2));
    for (int P = 0; P < N / 2; P++) mb.freq[P] = pos_freq(&mb.b.fft, P);
    simd_mb_job J = {&mb, in, luts, lut_idx, out, count, 0};
    pthread_mutex_init(&J.mu, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, simd_mb_worker, &J);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&J.mu);
    free(mb.freq);
    sfft_free(&mb.b.fft);
    return 0;
}
