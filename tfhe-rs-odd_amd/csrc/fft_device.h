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
// M = 1024 exchange addressing.  Default: one pad slot per 64 positions (p + p/64): both access
// patterns (lane + 64 c, and 64 cc + a1 + 4 b) become a per-lane base + compile-time immediate
// offsets.  TM_XCHG_XOR=1: unpadded buffer with an XOR swizzle of the 16-B slot,
// p ^ ((p >> 6) & 15) (saves 256 B per buffer, costs per-access address math).
#ifndef TM_TW_SB
#define TM_TW_SB 16 // twiddle multiplies per scheduling region (16 = one region)
#endif
#ifndef TM_XCHG_XOR
#define TM_XCHG_XOR 1
#endif
__device__ __forceinline__ int xswz(int p) { return TM_XCHG_XOR ? (p ^ ((p >> 6) & 15)) : xpad(p); }
constexpr int xbuf_len_1024() { return TM_XCHG_XOR ? 1024 : xbuf_len(1024); }
__device__ __forceinline__ void lds_stx(cx *xb, int p, cx v) {
    reinterpret_cast<double2 *>(xb)[xswz(p)] = make_double2(v.re, v.im);
}
__device__ __forceinline__ cx lds_ldx(const cx *xb, int p) {
    double2 t = reinterpret_cast<const double2 *>(xb)[xswz(p)];
    return {t.x, t.y};
}
// M = 1024 XOR-swizzled exchange on byte addresses: for a buffer at a 1 KiB-aligned LDS address
// X, 16 xswz(p) + X is
//   p = lane + 64 c        : ((X + 16 lane) ^ 16 c) + 1024 c   (one v_xor; 1024 c is the ds offset)
//   p = 64 cc + a1 + 4 b   : (X + 1024 cc + 16 (a1 ^ cc)) ^ 64 b (one v_xor)
// since X has no bits in 4..9 and (a1 + 4 b) ^ cc = (a1 ^ cc) ^ 4 b (a1 < 4).
// Sync types may carry `static constexpr int launder` (WaveLocalSyncL, pbs_common.h): bit 1
// recomputes the lane base la, bit 2 the stage-2 base qa, at every transform, so that their 15
// XOR images are not hoisted out of the caller's loop (where a kernel at its register limit
// spills them).  Same addresses, same values.
template <class S, class = void>
struct SyncLaunder {
    static constexpr int value = 0;
};
template <class S>
struct SyncLaunder<S, decltype((void)S::launder)> {
    static constexpr int value = S::launder;
};
template <class S, int Bit>
__device__ __forceinline__ uint32_t launder_addr(uint32_t a) {
    if constexpr ((SyncLaunder<S>::value & Bit) != 0) asm volatile("" : "+v"(a));
    return a;
}
typedef double lds_d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) lds_d2v lds_d2;
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)p;
}
__device__ __forceinline__ void lds_st_at(uint32_t a, cx v) { *(lds_d2 *)(uintptr_t)a = lds_d2v{v.re, v.im}; }
__device__ __forceinline__ cx lds_ld_at(uint32_t a) {
    const lds_d2v t = *(const lds_d2 *)(uintptr_t)a;
    return {t.x, t.y};
}
// The resident Fourier BSK is the reference's forward_as_torus transform (fft/mod.rs:197-218)
// scaled by 1/M: the torus input is read as (i64)x * 2^-64 / M.  A power-of-two scale commutes
// with every rounding of the FFT, the MAC and the inverse FFT (no value comes near the subnormal
// or overflow range), so the inverse spectrum arrives already divided by M and the backward
// conversion (x86.rs:823-874) multiplies by the plain twist, bit-identically to the reference's
// twist / M -- without a second twist table or a per-element scale in the CMUX loop.
__host__ __device__ constexpr double fourier_key_scale(int M) { return 0x1p-64 / (double)M; }

__device__ __forceinline__ double lds_ld_f64(uint32_t a) { return *(const __attribute__((address_space(3))) double *)(uintptr_t)a; }
// -x when bit 31 of m is set, else x (one XOR into the high word)
__device__ __forceinline__ double flip_sign(double x, uint32_t m) {
    return __hiloint2double(__double2hiint(x) ^ (int)(m & 0x80000000u), __double2loint(x));
}
// Buffer-resource loads: SGPR base (the V#) + a per-lane VGPR byte offset + an SGPR byte offset +
// an immediate, so a wave-uniform stream costs no VALU address arithmetic.  dword3 0x00020000:
// raw dwords on gfx9 (CDNA); num_records = 2^31 - 1 bytes.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ double2 buffer_ld_d2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u t = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
    return make_double2(__hiloint2double((int)t.y, (int)t.x), __hiloint2double((int)t.w, (int)t.z));
}
// 16-byte store through a buffer resource with cache-policy bits aux (gfx950: 16 = sc1, a
// write-through store whose line leaves the XCD's L2 at once)
template <int AUX>
__device__ __forceinline__ void buffer_st_d2p(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double2 x) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u t = {(unsigned)__double2loint(x.x), (unsigned)__double2hiint(x.x), (unsigned)__double2loint(x.y),
                   (unsigned)__double2hiint(x.y)};
    __builtin_amdgcn_raw_buffer_store_b128(t, r, voff, soff, AUX);
}
__device__ __forceinline__ cx gld(const double2 *__restrict__ p) {
    double2 t = *p;
    return {t.x, t.y};
}

// ---- twiddle sources ---------------------------------------------------------------------
// Stage-1 twiddle of lane a, output c:   W_M[a c]           (c = 1..R1-1)
// Stage-2 twiddle of row a1, output c2:  W_M[(M/64) a1 c2]  (c2 = 1..R2-1)
// with W_M[t] = exp(-2 pi i t / M).  t == 0 multiplies by W[0] = (1, -0): value-identical to
// skipping it (only the sign of a zero can change, which no later rounding observes), so the
// multiply is unconditional (branch-free).
template <int M>
struct GlobalTwiddles {  // straight from the M-entry table in global memory (L1/L2)
    const double2 *__restrict__ W;
    __device__ __forceinline__ cx s1(int c, int lane) const { return gld(W + lane * c); }
    __device__ __forceinline__ cx s2(int c2, int a1) const { return gld(W + (M / 64) * a1 * c2); }
};
// LDS copies laid out for conflict-free reads: s1 table [c-1][lane] (R1-1 x 64 entries),
// s2 table [c2-1][a1] (R2-1 x A1 entries).
template <int R1, int R2, int A1>
struct LdsTwiddles {
    const double2 *t1, *t2;
    __device__ __forceinline__ cx s1(int c, int lane) const {
        double2 t = t1[(c - 1) * 64 + lane];
        return {t.x, t.y};
    }
    // stage-2 twiddle W[(M/64) a1 c2] = W[lane' c2] with lane' = (64/A1) a1 < 64: an s1 entry
    __device__ __forceinline__ cx s2(int c2, int a1) const {
        static_assert(R2 <= R1, "stage-2 twiddles are read from the stage-1 table");
        double2 t = t1[(c2 - 1) * 64 + (64 / A1) * a1];
        return {t.x, t.y};
    }
    static constexpr int s1_len = (R1 - 1) * 64;
    static constexpr int s2_len = 0;
    // cooperative fill from the global W table by `nthreads` threads
    template <int M>
    __device__ static void fill(double2 *t1, double2 *, const double2 *__restrict__ W, int tid,
                                int nthreads) {
        for (int e = tid; e < s1_len; e += nthreads) t1[e] = W[(e & 63) * ((e >> 6) + 1)];
    }
};

template <int M>
struct WaveFft;

// ---- cross-lane 4x4 transposes on gfx950 (v_permlane32_swap / v_permlane16_swap) --------
// permlane32_swap(A, B): A <- [A.lo32, B.lo32], B <- [A.hi32, B.hi32]   (lanes 0-31 / 32-63)
// permlane16_swap(A, B): A <- [A.r0, B.r0, A.r2, B.r2], B <- [A.r1, B.r1, A.r3, B.r3]
__device__ __forceinline__ void pl32_swap(double &a, double &b) {
    uint64_t ua = __double_as_longlong(a), ub = __double_as_longlong(b);
    auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)ua, (uint32_t)ub, false, false);
    auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
    a = __longlong_as_double(((uint64_t)hi[0] << 32) | lo[0]);
    b = __longlong_as_double(((uint64_t)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ void pl16_swap(double &a, double &b) {
    uint64_t ua = __double_as_longlong(a), ub = __double_as_longlong(b);
    auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)ua, (uint32_t)ub, false, false);
    auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
    a = __longlong_as_double(((uint64_t)hi[0] << 32) | lo[0]);
    b = __longlong_as_double(((uint64_t)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ void pl32_swap(cx &a, cx &b) {
    pl32_swap(a.re, b.re);
    pl32_swap(a.im, b.im);
}
__device__ __forceinline__ void pl16_swap(cx &a, cx &b) {
    pl16_swap(a.re, b.re);
    pl16_swap(a.im, b.im);
}
// (register r, row-of-16 w) 4x4 transpose: R_r[w] <- R_w[r]
__device__ __forceinline__ void transpose_rows4(cx &r0, cx &r1, cx &r2, cx &r3) {
    pl32_swap(r0, r2);
    pl32_swap(r1, r3);
    pl16_swap(r0, r1);
    pl16_swap(r2, r3);
}

// ---------------------------------------------------------------------------------------
// M = 1024 (N = 2048): radices [16, 16, 4]; 64 lanes x 16 values.
//   natural layout  : lane a, slot b  <->  position a + 64 b
//   fourier layout  : lane L, slot s  <->  position 64 (L & 15) + 16 (L >> 4) + s
// stage 1 -> stage 2 goes through the wave's LDS buffer; stage 2 -> stage 3 is a register
// transpose across the four 16-lane rows (lanes L, L+16, L+32, L+48 share cc = L & 15).
// `sync()` orders the wave's LDS accesses.
// ---------------------------------------------------------------------------------------
template <>
struct WaveFft<1024> {
    static constexpr int M = 1024;
    static constexpr int V = 16;
    static constexpr int XL = xbuf_len_1024();  // exchange buffer entries
    using Lds = LdsTwiddles<16, 16, 4>;
    // Spectrum element (slot s, lane) sits at FFT position P = 64 (lane & 15) + 16 (lane >> 4) + s;
    // the DIF output is digit reversed (P = 64 c0 + 4 c1 + c2 -> f = c0 + 16 c1 + 256 c2), so its
    // frequency is freq_lane(lane) + freq_slot(s) (oracle pos_freq).
    __device__ __forceinline__ static uint32_t freq_lane(int lane) { return (lane & 15) + 64 * (lane >> 4); }
    static constexpr uint32_t freq_slot(int s) { return 16 * (s >> 2) + 256 * (s & 3); }

    template <class TW, class Sync>
    __device__ __forceinline__ static void forward(cx *v, cx *xb, const TW &tw, int lane, Sync sync) {
        // stage 1: L=1024, R=16, m=64, a = lane
        dft16_fwd(v);
#pragma unroll
        for (int c = 1; c < 16; c++) {
            if (c % TM_TW_SB == 1) __builtin_amdgcn_sched_barrier(0);  // bound twiddle loads in flight
            cx w = tw.s1(c, lane);
            v[c] = cmulw(v[c], w.re, w.im);
        }
        sync();  // previous readers of xb done
        const int cc = lane & 15, a1 = lane >> 4;
        if constexpr (TM_XCHG_XOR) {
            const uint32_t xa = lds_addr(xb), la = launder_addr<Sync, 1>(xa + 16u * lane);
#pragma unroll
            for (int c = 0; c < 16; c++) lds_st_at((la ^ (16u * c)) + 1024u * c, v[c]);
            sync();
            // stage 2: blocks of 64 (cc), R=16, m=4 (a1 = row)
            const uint32_t qa = launder_addr<Sync, 2>(xa + 1024u * cc + 16u * (a1 ^ cc));
#pragma unroll
            for (int b = 0; b < 16; b++) v[b] = lds_ld_at(qa ^ (64u * b));
        } else {
#pragma unroll
            for (int c = 0; c < 16; c++) lds_stx(xb, lane + 64 * c, v[c]);
            sync();
#pragma unroll
            for (int b = 0; b < 16; b++) v[b] = lds_ldx(xb, 64 * cc + a1 + 4 * b);
        }
        dft16_fwd(v);
#pragma unroll
        for (int c2 = 1; c2 < 16; c2++) {
            if (c2 % TM_TW_SB == 1) __builtin_amdgcn_sched_barrier(0);
            cx w = tw.s2(c2, a1);
            v[c2] = cmulw(v[c2], w.re, w.im);
        }
        // lane (cc, a1) holds positions 64cc + a1 + 4 c2 -> lane (cc, j) slot 4q+b holds
        // 64cc + 16j + 4q + b (from row b, register 4j + q)
#pragma unroll
        for (int q = 0; q < 4; q++) transpose_rows4(v[q], v[4 + q], v[8 + q], v[12 + q]);
        cx t[16];
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int b = 0; b < 4; b++) t[4 * q + b] = v[4 * b + q];
        // stage 3: blocks of 4, R=4, m=1
#pragma unroll
        for (int q = 0; q < 4; q++) {
            r4_fwd(t[4 * q], t[4 * q + 1], t[4 * q + 2], t[4 * q + 3]);
#pragma unroll
            for (int b = 0; b < 4; b++) v[4 * q + b] = t[4 * q + b];
        }
    }

    template <class TW, class Sync>
    __device__ __forceinline__ static void inverse(cx *v, cx *xb, const TW &tw, int lane, Sync sync) {
        const int cc = lane & 15, a1 = lane >> 4;
        cx t[16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            r4_inv(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
#pragma unroll
            for (int b = 0; b < 4; b++) t[4 * b + q] = v[4 * q + b];
        }
        // inverse of the row transpose: register 4j+q of row a1 <- slot 4q+a1 of row j
#pragma unroll
        for (int q = 0; q < 4; q++) transpose_rows4(t[q], t[4 + q], t[8 + q], t[12 + q]);
        v[0] = t[0];
#pragma unroll
        for (int c2 = 1; c2 < 16; c2++) {
            cx w = tw.s2(c2, a1);
            v[c2] = cmulw(t[c2], w.re, -w.im);
        }
        dft16_inv(v);
        sync();  // previous readers of xb done
        if constexpr (TM_XCHG_XOR) {
            const uint32_t xa = lds_addr(xb);
            const uint32_t qa = launder_addr<Sync, 2>(xa + 1024u * cc + 16u * (a1 ^ cc));
#pragma unroll
            for (int b = 0; b < 16; b++) lds_st_at(qa ^ (64u * b), v[b]);
            sync();
            const uint32_t la = launder_addr<Sync, 1>(xa + 16u * lane);
            v[0] = lds_ld_at(la);
#pragma unroll
            for (int c = 1; c < 16; c++) {
                cx y = lds_ld_at((la ^ (16u * c)) + 1024u * c);
                cx w = tw.s1(c, lane);
                v[c] = cmulw(y, w.re, -w.im);
            }
        } else {
#pragma unroll
            for (int b = 0; b < 16; b++) lds_stx(xb, 64 * cc + a1 + 4 * b, v[b]);
            sync();
            v[0] = lds_ldx(xb, lane);
#pragma unroll
            for (int c = 1; c < 16; c++) {
                cx y = lds_ldx(xb, lane + 64 * c);
                cx w = tw.s1(c, lane);
                v[c] = cmulw(y, w.re, -w.im);
            }
        }
        dft16_inv(v);
    }
};

// ---------------------------------------------------------------------------------------
// M = 512 (N = 1024): radices [8, 8, 8]; 64 lanes x 8 values, both exchanges through LDS.
//   natural layout  : lane a, slot b  <->  position a + 64 b
//   fourier layout  : lane L, slot s  <->  position 64 (L & 7) + 8 (L >> 3) + s
// ---------------------------------------------------------------------------------------
template <>
struct WaveFft<512> {
    static constexpr int M = 512;
    static constexpr int V = 8;
    static constexpr int XL = xbuf_len(512);  // exchange buffer entries (padded)
    using Lds = LdsTwiddles<8, 8, 8>;

    template <class TW, class Sync>
    __device__ __forceinline__ static void forward(cx *v, cx *xb, const TW &tw, int lane, Sync sync) {
        dft8_fwd(v);
#pragma unroll
        for (int c = 1; c < 8; c++) {
            cx w = tw.s1(c, lane);
            v[c] = cmulw(v[c], w.re, w.im);
        }
        sync();
#pragma unroll
        for (int c = 0; c < 8; c++) lds_st(xb, lane + 64 * c, v[c]);
        sync();
        const int cc = lane & 7, a1 = lane >> 3;
#pragma unroll
        for (int b = 0; b < 8; b++) v[b] = lds_ld(xb, 64 * cc + a1 + 8 * b);
        dft8_fwd(v);
#pragma unroll
        for (int c2 = 1; c2 < 8; c2++) {
            cx w = tw.s2(c2, a1);
            v[c2] = cmulw(v[c2], w.re, w.im);
        }
        sync();
#pragma unroll
        for (int c2 = 0; c2 < 8; c2++) lds_st(xb, 64 * cc + a1 + 8 * c2, v[c2]);
        sync();
        const int j = lane >> 3;
#pragma unroll
        for (int s = 0; s < 8; s++) v[s] = lds_ld(xb, 64 * cc + 8 * j + s);
        dft8_fwd(v);
    }

    template <class TW, class Sync>
    __device__ __forceinline__ static void inverse(cx *v, cx *xb, const TW &tw, int lane, Sync sync) {
        const int cc = lane & 7, j = lane >> 3, a1 = lane >> 3;
        dft8_inv(v);
        sync();
#pragma unroll
        for (int s = 0; s < 8; s++) lds_st(xb, 64 * cc + 8 * j + s, v[s]);
        sync();
        v[0] = lds_ld(xb, 64 * cc + a1);
#pragma unroll
        for (int c2 = 1; c2 < 8; c2++) {
            cx y = lds_ld(xb, 64 * cc + a1 + 8 * c2);
            cx w = tw.s2(c2, a1);
            v[c2] = cmulw(y, w.re, -w.im);
        }
        dft8_inv(v);
        sync();
#pragma unroll
        for (int b = 0; b < 8; b++) lds_st(xb, 64 * cc + a1 + 8 * b, v[b]);
        sync();
        v[0] = lds_ld(xb, lane);
#pragma unroll
        for (int c = 1; c < 8; c++) {
            cx y = lds_ld(xb, lane + 64 * c);
            cx w = tw.s1(c, lane);
            v[c] = cmulw(y, w.re, -w.im);
        }
        dft8_inv(v);
    }
};

// ---------------------------------------------------------------------------------------
// M = 256 (N = 512): radices [16, 16]; 64 lanes x 4 values.  A 16-point DFT is spread over the
// four 16-lane rows: row A holds its column (v[A], v[A+4], v[A+8], v[A+12]), runs the first
// radix-4 and the internal twiddles omega_16^{A q} (A is per row, so selected at run time), a
// cross-row register transpose hands row c the values u[0..3][c], and the second radix-4 leaves
// X[c + 4q] in slot q.  Same operations as dft16_fwd/inv, distributed.
//   natural layout  : lane a, slot b  <->  position a + 64 b
//   stage 1 (a' = lane & 15 = butterfly, row i): position a' + 16 (i + 4 b): column A = i
//   fourier layout  : lane L, slot q  <->  position 16 (L & 15) + (L >> 4) + 4 q
// One LDS exchange per transform (between the two stages).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void tw16_fwd_row(int A, cx &y1, cx &y2, cx &y3) {
    if (A == 1) {
        y1 = tw16_fwd<1>(y1);
        y2 = tw16_fwd<2>(y2);
        y3 = tw16_fwd<3>(y3);
    } else if (A == 2) {
        y1 = tw16_fwd<2>(y1);
        y2 = tw16_fwd<4>(y2);
        y3 = tw16_fwd<6>(y3);
    } else if (A == 3) {
        y1 = tw16_fwd<3>(y1);
        y2 = tw16_fwd<6>(y2);
        y3 = tw16_fwd<9>(y3);
    }
}
__device__ __forceinline__ void tw16_inv_row(int A, cx &y1, cx &y2, cx &y3) {
    if (A == 1) {
        y1 = tw16_inv<1>(y1);
        y2 = tw16_inv<2>(y2);
        y3 = tw16_inv<3>(y3);
    } else if (A == 2) {
        y1 = tw16_inv<2>(y1);
        y2 = tw16_inv<4>(y2);
        y3 = tw16_inv<6>(y3);
    } else if (A == 3) {
        y1 = tw16_inv<3>(y1);
        y2 = tw16_inv<6>(y2);
        y3 = tw16_inv<9>(y3);
    }
}
// dft16_fwd across rows: in  row A slot j = v[A + 4j];  out  row c slot q = X[c + 4q]
__device__ __forceinline__ void dft16_fwd_rows(cx *v, int row) {
    r4_fwd(v[0], v[1], v[2], v[3]);
    tw16_fwd_row(row, v[1], v[2], v[3]);
    transpose_rows4(v[0], v[1], v[2], v[3]);
    r4_fwd(v[0], v[1], v[2], v[3]);
}
// dft16_inv across rows: in  row c slot q = X[c + 4q];  out  row A slot j = v[A + 4j]
__device__ __forceinline__ void dft16_inv_rows(cx *v, int row) {
    r4_inv(v[0], v[1], v[2], v[3]);
    transpose_rows4(v[0], v[1], v[2], v[3]);
    tw16_inv_row(row, v[1], v[2], v[3]);
    r4_inv(v[0], v[1], v[2], v[3]);
}
// stage-1 twiddles W[a' C] (a' < 16, C = 1..15): LDS table [C-1][a']
struct LdsTwiddles256 {
    const double2 *t1, *t2;
    __device__ __forceinline__ cx s1(int c, int a) const {
        double2 t = t1[(c - 1) * 16 + a];
        return {t.x, t.y};
    }
    static constexpr int s1_len = 15 * 16;
    static constexpr int s2_len = 0;
    template <int M>
    __device__ static void fill(double2 *t1, double2 *, const double2 *__restrict__ W, int tid, int nthreads) {
        for (int e = tid; e < s1_len; e += nthreads) t1[e] = W[(e & 15) * ((e >> 4) + 1)];
    }
};

template <>
struct WaveFft<256> {
    static constexpr int M = 256;
    static constexpr int V = 4;
    static constexpr int XL = xbuf_len(256);
    using Lds = LdsTwiddles256;
    // Spectrum element (slot q, lane) is output c1 = (lane >> 4) + 4 q of the stage-2 block
    // C = lane & 15 (FFT position 16 C + c1), so its frequency is C + 16 c1 (oracle pos_freq of the
    // [16, 16] plan).
    __device__ __forceinline__ static uint32_t freq_lane(int lane) { return (lane & 15) + 16 * (lane >> 4); }
    static constexpr uint32_t freq_slot(int q) { return 64 * q; }

    template <class TW, class Sync>
    __device__ __forceinline__ static void forward(cx *v, cx *xb, const TW &tw, int lane, Sync sync) {
        // stage 1: L = 256, R = 16, m = 16; butterfly a' = lane & 15
        const int ap = lane & 15, row = lane >> 4;
        dft16_fwd_rows(v, row);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int C = row + 4 * q;
            if (C) {
                cx w = tw.s1(C, ap);
                v[q] = cmulw(v[q], w.re, w.im);
            }
        }
        sync();
#pragma unroll
        for (int q = 0; q < 4; q++) lds_st(xb, ap + 16 * (row + 4 * q), v[q]);  // position a' + 16C
        sync();
        // stage 2: blocks of 16 (C = lane & 15), R = 16, m = 1, no twiddles; column A = row
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = lds_ld(xb, 16 * ap + row + 4 * j);
        dft16_fwd_rows(v, row);
    }

    template <class TW, class Sync>
    __device__ __forceinline__ static void inverse(cx *v, cx *xb, const TW &tw, int lane, Sync sync) {
        const int ap = lane & 15, row = lane >> 4;
        // block DFTs (stage 2 of the forward), lane (c2, C) slot q = X_C[c2 + 4q]
        dft16_inv_rows(v, row);
        sync();
#pragma unroll
        for (int j = 0; j < 4; j++) lds_st(xb, 16 * ap + row + 4 * j, v[j]);
        sync();
        // stage 1: butterfly a' = lane & 15, column c = row: z[a' + 16 (c + 4q)] * conj(W[a' (c + 4q)])
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int C = row + 4 * q;
            cx y = lds_ld(xb, ap + 16 * C);
            if (C) {
                cx w = tw.s1(C, ap);
                y = cmulw(y, w.re, -w.im);
            }
            v[q] = y;
        }
        dft16_inv_rows(v, row);
    }
};

// ---------------------------------------------------------------------------------------
// M = 128 (N = 256, GADGET_SHA3_PARAMETERS_40): radices [16, 8]; 64 lanes x 2 values.
//   natural layout = fourier layout : lane a, slot b  <->  position a + 64 b
// Stage 1 (8 butterflies of 16 points, z[a' + 8 b]) is spread over the four 16-lane rows as in
// WaveFft<256>, on the lanes with (lane & 15) < 8 (the other half computes a duplicate and does
// not store); stage 2 (16 blocks of 8 points, no twiddles) runs one block per lane on lanes
// 0-15.  Both stages exchange through the wave's LDS buffer.  N = 256 is a small niche shape:
// this favours reusing the verified radix-16/8 kernels over lane efficiency.
// ---------------------------------------------------------------------------------------
struct LdsTwiddles128 {  // stage-1 twiddles W_128[a' C] (a' < 8, C = 1..15): table [C-1][a']
    const double2 *t1, *t2;
    __device__ __forceinline__ cx s1(int c, int a) const {
        double2 t = t1[(c - 1) * 8 + a];
        return {t.x, t.y};
    }
    static constexpr int s1_len = 15 * 8;
    static constexpr int s2_len = 0;
    template <int M>
    __device__ static void fill(double2 *t1, double2 *, const double2 *__restrict__ W, int tid, int nthreads) {
        for (int e = tid; e < s1_len; e += nthreads) t1[e] = W[(e & 7) * ((e >> 3) + 1)];
    }
};

template <>
struct WaveFft<128> {
    static constexpr int M = 128;
    static constexpr int V = 2;
    static constexpr int XL = xbuf_len(128);
    using Lds = LdsTwiddles128;

    template <class TW, class Sync>
    __device__ __forceinline__ static void forward(cx *v, cx *xb, const TW &tw, int lane, Sync sync) {
        const int ap = lane & 7, row = (lane >> 4) & 3;
        const bool st1 = (lane & 15) < 8;
        sync();
        lds_st(xb, lane, v[0]);
        lds_st(xb, lane + 64, v[1]);
        sync();
        // stage 1: L = 128, R = 16, m = 8; column A = row holds z[a' + 8 (A + 4 j)]
        cx u[4];
#pragma unroll
        for (int j = 0; j < 4; j++) u[j] = lds_ld(xb, ap + 8 * (row + 4 * j));
        dft16_fwd_rows(u, row);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int C = row + 4 * q;
            if (C) {
                cx w = tw.s1(C, ap);
                u[q] = cmulw(u[q], w.re, w.im);
            }
        }
        sync();
        if (st1) {
#pragma unroll
            for (int q = 0; q < 4; q++) lds_st(xb, ap + 8 * (row + 4 * q), u[q]);
        }
        sync();
        // stage 2: blocks of 8 (lane = block), R = 8, m = 1
        if (lane < 16) {
            cx b[8];
#pragma unroll
            for (int t = 0; t < 8; t++) b[t] = lds_ld(xb, 8 * lane + t);
            dft8_fwd(b);
#pragma unroll
            for (int t = 0; t < 8; t++) lds_st(xb, 8 * lane + t, b[t]);
        }
        sync();
        v[0] = lds_ld(xb, lane);
        v[1] = lds_ld(xb, lane + 64);
    }

    template <class TW, class Sync>
    __device__ __forceinline__ static void inverse(cx *v, cx *xb, const TW &tw, int lane, Sync sync) {
        const int ap = lane & 7, row = (lane >> 4) & 3;
        const bool st1 = (lane & 15) < 8;
        sync();
        lds_st(xb, lane, v[0]);
        lds_st(xb, lane + 64, v[1]);
        sync();
        if (lane < 16) {
            cx b[8];
#pragma unroll
            for (int t = 0; t < 8; t++) b[t] = lds_ld(xb, 8 * lane + t);
            dft8_inv(b);
#pragma unroll
            for (int t = 0; t < 8; t++) lds_st(xb, 8 * lane + t, b[t]);
        }
        sync();
        // stage 1: z[a' + 8C] * conj(W[a' C]), C = row + 4 q; out row A slot j -> z[a' + 8 (A + 4 j)]
        cx u[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int C = row + 4 * q;
            cx y = lds_ld(xb, ap + 8 * C);
            if (C) {
                cx w = tw.s1(C, ap);
                y = cmulw(y, w.re, -w.im);
            }
            u[q] = y;
        }
        dft16_inv_rows(u, row);
        sync();
        if (st1) {
#pragma unroll
            for (int j = 0; j < 4; j++) lds_st(xb, ap + 8 * (row + 4 * j), u[j]);
        }
        sync();
        v[0] = lds_ld(xb, lane);
        v[1] = lds_ld(xb, lane + 64);
    }
};

// Torus increment of a fractional part (x86.rs:823-874 + 961-1044): X = rint(fr * 2^64) mod 2^64
// for fr in [-1/2, 1/2], with four f64 ops, one integer add and no f64->int conversion.
// For an even integer C in [2^52 + 2^31, 2^53 - 2^31], fma(t, 1, C) with |t| <= 2^31 is
// C + rint_half_even(t) (ulp 1 there; C even keeps the tie parity) and its bit pattern is
// bits(C) + rint(t) as a 64-bit integer.  With MB = 1.5 * 2^52 (bits 0x4338000000000000) and
// MA = MB - 0x43380000:
//   a = fma(fr, 2^32, MA):  h = a - MA = rint(fr 2^32) exactly, lo32(a) = h - 0x43380000
//   f = fma(fr, 2^32, -h) = fr 2^32 - h in [-1/2, 1/2] (exact)
//   b = fma(f, 2^32, MB):   bits(b) = 0x4338000000000000 + l, l = rint(f 2^32) in [-2^31, 2^31]
// fr 2^64 = h 2^32 + f 2^32 with h 2^32 even, so rint(fr 2^64) = h 2^32 + l (ties included)
// = bits(b) + (lo32(a) << 32) mod 2^64.  fr = +-1/2 gives h = +-2^31 -> X = 2^63, as the
// reference's wrapping conversion.  Checked against a long-double rint on 2e8 inputs + edges.
// X is never built as an integer: X = bits(b) + (lo32(a) << 32) mod 2^64.  The f64 part is one
// asm block: 2^32 lives in a VGPR and the magics in SGPRs (one constant-bus operand per VOP3 on
// gfx9; as plain fma() the compiler picks v_fmac with the magic copied into the destination
// first), and the hazard recognizer, which pads every inline-asm block with an s_nop, sees one
// block per coefficient.  (v_lshl_add_u64 shifts by at most 4: the high-word add is separate.)
constexpr double TORUS_MB = 0x1.8p52;
constexpr double TORUS_MA = 0x1.8p52 - 1127743488.0;  // MB - 0x43380000
// 2^32 in a VGPR, hoisted by the caller out of its loops
__device__ __forceinline__ double torus_k32() {
    double k = 0x1p32;
    asm volatile("" : "+v"(k));
    return k;
}
__device__ __forceinline__ void frac_to_torus(double fr, double k32, double &a, double &b) {
    asm("v_fma_f64 %[a], %[fr], %[k], %[ma]\n\t"
        "v_add_f64 %[t], %[a], -%[ma]\n\t"
        "v_fma_f64 %[t], %[fr], %[k], -%[t]\n\t"
        "v_fma_f64 %[t], %[t], %[k], %[mb]"
        : [a] "=&v"(a), [t] "=&v"(b)
        : [fr] "v"(fr), [k] "v"(k32), [ma] "s"(TORUS_MA), [mb] "s"(TORUS_MB));
}
// c += X (mod 2^64)
__device__ __forceinline__ void torus_add_frac(uint64_t &c, double fr, double k32) {
    double a, b;
    frac_to_torus(fr, k32, a, b);
    // one 64-bit add of bits(b), then a 32-bit add into the high word; the opaque copy keeps the
    // compiler from re-associating the latter into a 64-bit add of the pair (0, lo32(a)), which
    // costs a v_mov per coefficient to build
    c += (uint64_t)__double_as_longlong(b);
    uint32_t hi = (uint32_t)(c >> 32) + (uint32_t)__double2loint(a);
    asm("" : "+v"(hi));
    c = ((uint64_t)hi << 32) | (uint32_t)c;
}
// c = X
__device__ __forceinline__ uint64_t torus_from_frac(double fr, double k32) {
    double a, b;
    frac_to_torus(fr, k32, a, b);
    const uint32_t hi = (uint32_t)__double2hiint(b) + (uint32_t)__double2loint(a);
    return ((uint64_t)hi << 32) | (uint32_t)__double2loint(b);
}

// backward conversion (x86.rs:823-874 + 961-1044): with ws = twist / M,
// torus increments for coefficient j (re) and j + M (im).
__device__ __forceinline__ void backward_convert(cx z, cx ws, uint64_t &dre, uint64_t &dim, double k32) {
    double mr = fma(z.re, ws.re, z.im * ws.im);
    double mi = fma(-z.re, ws.im, z.im * ws.re);
    dre = torus_from_frac(mr - rint(mr), k32);
    dim = torus_from_frac(mi - rint(mi), k32);
}
// same, added in place: c_re += increment(j), c_im += increment(j + M)
__device__ __forceinline__ void backward_add(cx z, cx ws, uint64_t &c_re, uint64_t &c_im, double k32) {
    double mr = fma(z.re, ws.re, z.im * ws.im);
    double mi = fma(-z.re, ws.im, z.im * ws.re);
    torus_add_frac(c_re, mr - rint(mr), k32);
    torus_add_frac(c_im, mi - rint(mi), k32);
}

}  // namespace tfhe_mi355
