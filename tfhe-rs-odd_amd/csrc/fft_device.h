// fft_device.h -- negacyclic f64 FFT building blocks for CDNA4 (gfx950), one wavefront per
// polynomial.  The butterfly DAG is the one fixed in DESIGN.md "FFT spec" (the CPU oracle
// oracle/pbs_oracle.c computes the same DAG op for op, which is what makes the PBS outputs
// bit-exact).  Reference semantics being replaced: concrete-fft Plan::{fwd,inv} behind
// tfhe/src/core_crypto/fft_impl/fft64/math/fft/mod.rs:496-557 plus the twist/convert helpers
// at mod.rs:197-326 and x86.rs:505-596, 823-874, 961-1044.
//
// Compiled with -ffp-contract=off: every fused multiply-add below is an explicit fma().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tfhe_mi355 {

struct cx {
    double re, im;
};

#define TM_C16_1 0x1.d906bcf328d46p-1 /* cos(pi/8) */
#define TM_S16_1 0x1.87de2a6aea963p-2 /* sin(pi/8) */
#define TM_SQH 0x1.6a09e667f3bcdp-1   /* sqrt(1/2) */

__device__ __forceinline__ cx cadd(cx a, cx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cx csub(cx a, cx b) { return {a.re - b.re, a.im - b.im}; }
// general twiddle product (fma(xr,wr,-(xi*wi)), fma(xr,wi,xi*wr))
__device__ __forceinline__ cx cmulw(cx x, double wr, double wi) {
    return {fma(x.re, wr, -(x.im * wi)), fma(x.re, wi, x.im * wr)};
}
__device__ __forceinline__ cx mul_w8(cx x) { return {(x.re + x.im) * TM_SQH, (x.im - x.re) * TM_SQH}; }
__device__ __forceinline__ cx mul_w8_3(cx x) { return {(x.im - x.re) * TM_SQH, -((x.re + x.im) * TM_SQH)}; }
__device__ __forceinline__ cx mul_w8c(cx x) { return {(x.re - x.im) * TM_SQH, (x.re + x.im) * TM_SQH}; }
__device__ __forceinline__ cx mul_w8_3c(cx x) { return {-((x.re + x.im) * TM_SQH), (x.re - x.im) * TM_SQH}; }
__device__ __forceinline__ cx mul_mi(cx x) { return {x.im, -x.re}; }
__device__ __forceinline__ cx mul_pi(cx x) { return {-x.im, x.re}; }

__device__ __forceinline__ void r4_fwd(cx &x0, cx &x1, cx &x2, cx &x3) {
    cx t0 = cadd(x0, x2), t1 = csub(x0, x2), t2 = cadd(x1, x3), t3 = csub(x1, x3);
    x0 = cadd(t0, t2);
    x2 = csub(t0, t2);
    x1 = {t1.re + t3.im, t1.im - t3.re};
    x3 = {t1.re - t3.im, t1.im + t3.re};
}
__device__ __forceinline__ void r4_inv(cx &x0, cx &x1, cx &x2, cx &x3) {
    cx t0 = cadd(x0, x2), t1 = csub(x0, x2), t2 = cadd(x1, x3), t3 = csub(x1, x3);
    x0 = cadd(t0, t2);
    x2 = csub(t0, t2);
    x1 = {t1.re - t3.im, t1.im + t3.re};
    x3 = {t1.re + t3.im, t1.im - t3.re};
}

template <int E>
__device__ __forceinline__ cx tw16_fwd(cx x) {
    if constexpr (E == 0) return x;
    else if constexpr (E == 1) return cmulw(x, TM_C16_1, -TM_S16_1);
    else if constexpr (E == 2) return mul_w8(x);
    else if constexpr (E == 3) return cmulw(x, TM_S16_1, -TM_C16_1);
    else if constexpr (E == 4) return mul_mi(x);
    else if constexpr (E == 6) return mul_w8_3(x);
    else return cmulw(x, -TM_C16_1, TM_S16_1);  // E == 9
}
template <int E>
__device__ __forceinline__ cx tw16_inv(cx x) {
    if constexpr (E == 0) return x;
    else if constexpr (E == 1) return cmulw(x, TM_C16_1, TM_S16_1);
    else if constexpr (E == 2) return mul_w8c(x);
    else if constexpr (E == 3) return cmulw(x, TM_S16_1, TM_C16_1);
    else if constexpr (E == 4) return mul_pi(x);
    else if constexpr (E == 6) return mul_w8_3c(x);
    else return cmulw(x, -TM_C16_1, -TM_S16_1);  // E == 9
}
template <int E>
__device__ __forceinline__ cx tw8_fwd(cx x) {
    if constexpr (E == 0) return x;
    else if constexpr (E == 1) return mul_w8(x);
    else if constexpr (E == 2) return mul_mi(x);
    else return mul_w8_3(x);
}
template <int E>
__device__ __forceinline__ cx tw8_inv(cx x) {
    if constexpr (E == 0) return x;
    else if constexpr (E == 1) return mul_w8c(x);
    else if constexpr (E == 2) return mul_pi(x);
    else return mul_w8_3c(x);
}

// 16-point DFT, natural order in/out: first radix 4 over stride-4 elements (DIF), internal
// twiddles omega_16^{a c}, then radix 4.  v[m] on exit = X[m].
template <int A>
__device__ __forceinline__ void dft16_fwd_col(cx *v, cx (&u)[4][4]) {
    cx y0 = v[A], y1 = v[A + 4], y2 = v[A + 8], y3 = v[A + 12];
    r4_fwd(y0, y1, y2, y3);
    u[A][0] = y0;
    u[A][1] = tw16_fwd<A * 1>(y1);
    u[A][2] = tw16_fwd<A * 2>(y2);
    u[A][3] = tw16_fwd<A * 3>(y3);
}
__device__ __forceinline__ void dft16_fwd(cx *v) {
    cx u[4][4];
    dft16_fwd_col<0>(v, u);
    dft16_fwd_col<1>(v, u);
    dft16_fwd_col<2>(v, u);
    dft16_fwd_col<3>(v, u);
#pragma unroll
    for (int c = 0; c < 4; c++) {
        cx y0 = u[0][c], y1 = u[1][c], y2 = u[2][c], y3 = u[3][c];
        r4_fwd(y0, y1, y2, y3);
        v[c] = y0;
        v[c + 4] = y1;
        v[c + 8] = y2;
        v[c + 12] = y3;
    }
}
template <int A>
__device__ __forceinline__ void dft16_inv_row(cx *v, cx (&u)[4][4]) {
    cx y0 = u[A][0], y1 = tw16_inv<A * 1>(u[A][1]), y2 = tw16_inv<A * 2>(u[A][2]),
       y3 = tw16_inv<A * 3>(u[A][3]);
    r4_inv(y0, y1, y2, y3);
    v[A] = y0;
    v[A + 4] = y1;
    v[A + 8] = y2;
    v[A + 12] = y3;
}
__device__ __forceinline__ void dft16_inv(cx *v) {
    cx u[4][4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        cx y0 = v[c], y1 = v[c + 4], y2 = v[c + 8], y3 = v[c + 12];
        r4_inv(y0, y1, y2, y3);
        u[0][c] = y0;
        u[1][c] = y1;
        u[2][c] = y2;
        u[3][c] = y3;
    }
    dft16_inv_row<0>(v, u);
    dft16_inv_row<1>(v, u);
    dft16_inv_row<2>(v, u);
    dft16_inv_row<3>(v, u);
}

// 8-point DFT: radix 4 over stride-2 elements, twiddles omega_8^{a c}, then radix 2.
template <int A>
__device__ __forceinline__ void dft8_fwd_col(cx *v, cx (&u)[2][4]) {
    cx y0 = v[A], y1 = v[A + 2], y2 = v[A + 4], y3 = v[A + 6];
    r4_fwd(y0, y1, y2, y3);
    u[A][0] = y0;
    u[A][1] = tw8_fwd<A * 1>(y1);
    u[A][2] = tw8_fwd<A * 2>(y2);
    u[A][3] = tw8_fwd<A * 3>(y3);
}
__device__ __forceinline__ void dft8_fwd(cx *v) {
    cx u[2][4];
    dft8_fwd_col<0>(v, u);
    dft8_fwd_col<1>(v, u);
#pragma unroll
    for (int c = 0; c < 4; c++) {
        v[c] = cadd(u[0][c], u[1][c]);
        v[c + 4] = csub(u[0][c], u[1][c]);
    }
}
template <int A>
__device__ __forceinline__ void dft8_inv_row(cx *v, cx (&u)[2][4]) {
    cx y0 = u[A][0], y1 = tw8_inv<A * 1>(u[A][1]), y2 = tw8_inv<A * 2>(u[A][2]),
       y3 = tw8_inv<A * 3>(u[A][3]);
    r4_inv(y0, y1, y2, y3);
    v[A] = y0;
    v[A + 2] = y1;
    v[A + 4] = y2;
    v[A + 6] = y3;
}
__device__ __forceinline__ void dft8_inv(cx *v) {
    cx u[2][4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        u[0][c] = cadd(v[c], v[c + 4]);
        u[1][c] = csub(v[c], v[c + 4]);
    }
    dft8_inv_row<0>(v, u);
    dft8_inv_row<1>(v, u);
}

// LDS exchange buffer addressing: one 16-B pad slot per 64 positions.
__device__ __forceinline__ int xpad(int p) { return p + (p >> 6); }
constexpr int xbuf_len(int M) { return M + M / 64; }

__device__ __forceinline__ void lds_st(cx *xb, int p, cx v) {
    reinterpret_cast<double2 *>(xb)[xpad(p)] = make_double2(v.re, v.im);
}
__device__ __forceinline__ cx lds_ld(const cx *xb, int p) {
    double2 t = reinterpret_cast<const double2 *>(xb)[xpad(p)];
    return {t.x, t.y};
}
__device__ __forceinline__ cx gld(const double2 *__restrict__ p) {
    double2 t = *p;
    return {t.x, t.y};
}

template <int M>
struct WaveFft;

// ---------------------------------------------------------------------------------------
// M = 1024 (N = 2048): radices [16, 16, 4]; 64 lanes x 16 values.
//   natural layout  : lane a, slot b  <->  position a + 64 b
//   fourier layout  : lane L, slot s  <->  position 64 (L & 15) + 16 (L >> 4) + s
// W = exp(-2 pi i t / 1024) table (t < 1024).  `sync()` orders the wave's LDS accesses.
// ---------------------------------------------------------------------------------------
template <>
struct WaveFft<1024> {
    static constexpr int M = 1024;
    static constexpr int V = 16;

    template <class Sync>
    __device__ __forceinline__ static void forward(cx *v, cx *xb, const double2 *__restrict__ W,
                                                   int lane, Sync sync) {
        // stage 1: L=1024, R=16, m=64, a = lane
        dft16_fwd(v);
#pragma unroll
        for (int c = 1; c < 16; c++) {
            int t = lane * c;
            if (t) {
                cx w = gld(W + t);
                v[c] = cmulw(v[c], w.re, w.im);
            }
        }
#pragma unroll
        for (int c = 0; c < 16; c++) lds_st(xb, lane + 64 * c, v[c]);
        sync();
        // stage 2: blocks of 64 (cc), R=16, m=4 (a1)
        const int cc = lane & 15, a1 = lane >> 4;
#pragma unroll
        for (int b = 0; b < 16; b++) v[b] = lds_ld(xb, 64 * cc + a1 + 4 * b);
        dft16_fwd(v);
#pragma unroll
        for (int c2 = 1; c2 < 16; c2++) {
            int t = a1 * c2;
            if (t) {
                cx w = gld(W + 16 * t);
                v[c2] = cmulw(v[c2], w.re, w.im);
            }
        }
        sync();
#pragma unroll
        for (int c2 = 0; c2 < 16; c2++) lds_st(xb, 64 * cc + a1 + 4 * c2, v[c2]);
        sync();
        // stage 3: blocks of 4, R=4, m=1 -- lane (cc, j) takes positions 64cc + 16j + [0,16)
        const int j = lane >> 4;
#pragma unroll
        for (int s = 0; s < 16; s++) v[s] = lds_ld(xb, 64 * cc + 16 * j + s);
#pragma unroll
        for (int q = 0; q < 4; q++) r4_fwd(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        sync();  // xb free again
    }

    template <class Sync>
    __device__ __forceinline__ static void inverse(cx *v, cx *xb, const double2 *__restrict__ W,
                                                   int lane, Sync sync) {
        const int cc = lane & 15, j = lane >> 4, a1 = lane >> 4;
#pragma unroll
        for (int q = 0; q < 4; q++) r4_inv(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
#pragma unroll
        for (int s = 0; s < 16; s++) lds_st(xb, 64 * cc + 16 * j + s, v[s]);
        sync();
#pragma unroll
        for (int c2 = 0; c2 < 16; c2++) {
            cx y = lds_ld(xb, 64 * cc + a1 + 4 * c2);
            int t = a1 * c2;
            if (t) {
                cx w = gld(W + 16 * t);
                y = cmulw(y, w.re, -w.im);
            }
            v[c2] = y;
        }
        dft16_inv(v);
        sync();
#pragma unroll
        for (int b = 0; b < 16; b++) lds_st(xb, 64 * cc + a1 + 4 * b, v[b]);
        sync();
#pragma unroll
        for (int c = 0; c < 16; c++) {
            cx y = lds_ld(xb, lane + 64 * c);
            int t = lane * c;
            if (t) {
                cx w = gld(W + t);
                y = cmulw(y, w.re, -w.im);
            }
            v[c] = y;
        }
        dft16_inv(v);
        sync();  // xb free again
    }
};

// ---------------------------------------------------------------------------------------
// M = 512 (N = 1024): radices [8, 8, 8]; 64 lanes x 8 values.
//   natural layout  : lane a, slot b  <->  position a + 64 b
//   fourier layout  : lane L, slot s  <->  position 64 (L & 7) + 8 (L >> 3) + s
// ---------------------------------------------------------------------------------------
template <>
struct WaveFft<512> {
    static constexpr int M = 512;
    static constexpr int V = 8;

    template <class Sync>
    __device__ __forceinline__ static void forward(cx *v, cx *xb, const double2 *__restrict__ W,
                                                   int lane, Sync sync) {
        dft8_fwd(v);
#pragma unroll
        for (int c = 1; c < 8; c++) {
            int t = lane * c;
            if (t) {
                cx w = gld(W + t);
                v[c] = cmulw(v[c], w.re, w.im);
            }
        }
#pragma unroll
        for (int c = 0; c < 8; c++) lds_st(xb, lane + 64 * c, v[c]);
        sync();
        const int cc = lane & 7, a1 = lane >> 3;
#pragma unroll
        for (int b = 0; b < 8; b++) v[b] = lds_ld(xb, 64 * cc + a1 + 8 * b);
        dft8_fwd(v);
#pragma unroll
        for (int c2 = 1; c2 < 8; c2++) {
            int t = a1 * c2;
            if (t) {
                cx w = gld(W + 8 * t);
                v[c2] = cmulw(v[c2], w.re, w.im);
            }
        }
        sync();
#pragma unroll
        for (int c2 = 0; c2 < 8; c2++) lds_st(xb, 64 * cc + a1 + 8 * c2, v[c2]);
        sync();
        const int j = lane >> 3;
#pragma unroll
        for (int s = 0; s < 8; s++) v[s] = lds_ld(xb, 64 * cc + 8 * j + s);
        dft8_fwd(v);
        sync();
    }

    template <class Sync>
    __device__ __forceinline__ static void inverse(cx *v, cx *xb, const double2 *__restrict__ W,
                                                   int lane, Sync sync) {
        const int cc = lane & 7, j = lane >> 3, a1 = lane >> 3;
        dft8_inv(v);
#pragma unroll
        for (int s = 0; s < 8; s++) lds_st(xb, 64 * cc + 8 * j + s, v[s]);
        sync();
#pragma unroll
        for (int c2 = 0; c2 < 8; c2++) {
            cx y = lds_ld(xb, 64 * cc + a1 + 8 * c2);
            int t = a1 * c2;
            if (t) {
                cx w = gld(W + 8 * t);
                y = cmulw(y, w.re, -w.im);
            }
            v[c2] = y;
        }
        dft8_inv(v);
        sync();
#pragma unroll
        for (int b = 0; b < 8; b++) lds_st(xb, 64 * cc + a1 + 8 * b, v[b]);
        sync();
#pragma unroll
        for (int c = 0; c < 8; c++) {
            cx y = lds_ld(xb, lane + 64 * c);
            int t = lane * c;
            if (t) {
                cx w = gld(W + t);
                y = cmulw(y, w.re, -w.im);
            }
            v[c] = y;
        }
        dft8_inv(v);
        sync();
    }
};

// f64 -> i64 by bit twiddling (exact for integral |x| < 2^64; 2^63 wraps), as
// fft/math/fft/x86.rs:28-81.
__device__ __forceinline__ uint64_t f64_to_u64_wrap(double x) {
    uint64_t bits = __double_as_longlong(x);
    uint64_t mant = (bits & 0xFFFFFFFFFFFFFULL) | 0x10000000000000ULL;
    uint64_t biased_exp = (bits >> 52) & 0x7FF;
    uint64_t lshift = mant << 11;
    uint64_t rs = 1086 - biased_exp;
    uint64_t v = rs < 64 ? (lshift >> rs) : 0;
    v = biased_exp == 0 ? 0 : v;
    return (bits >> 63) ? (0 - v) : v;
}

// backward conversion of one complex value (x86.rs:823-874 + 961-1044): returns the two
// torus increments for coefficients j (re) and j+M (im).
__device__ __forceinline__ void backward_convert(cx z, cx w_scaled, uint64_t &dre, uint64_t &dim) {
    double mr = fma(z.re, w_scaled.re, z.im * w_scaled.im);
    double mi = fma(-z.re, w_scaled.im, z.im * w_scaled.re);
    double fr = mr - rint(mr);
    double fi = mi - rint(mi);
    dre = f64_to_u64_wrap(rint(fr * 18446744073709551616.0));
    dim = f64_to_u64_wrap(rint(fi * 18446744073709551616.0));
}

}  // namespace tfhe_mi355
