// pbs_large.hip -- classic PBS for N = 32768 (PARAM_MESSAGE_4_CARRY_4_KS_PBS: n=996, k=1, L=2,
// base 2^15) on gfx950.
//
// Replaces the same reference functions as pbs_classic.hip (bootstrap.rs:243-380,
// ggsw.rs:477-697, polynomial_algorithms.rs:219-490, glwe_sample_extraction.rs:91-147,
// fft/mod.rs:197-557) at the 4_4 shapes.
//
// Why a different structure (DESIGN.md "Kernels"): at N = 32768 one ciphertext's accumulator is
// (k+1) N u64 = 512 KiB and one spectrum M = 16384 c64 = 256 KiB -- neither fits a CU (160 KiB
// LDS), so the accumulator lives in HBM scratch.  The M = 16384 FFT is the oracle's
// [16, 16, 16, 4] DAG; after its top radix-16 stage the 16 sub-blocks of 1024 positions are
// independent, and so are the MAC and the inverse up to its own top stage.  A CMUX is three
// batch-wide launches (below), each streaming at full occupancy.  Twiddles: top stage W_M[a c]
// from a [c-1][a] copy of the table (coalesced); sub-blocks W_M[16 x] through an LDS table (the
// oracle's tstride-16 reads of the same table, so bit-identical).
#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "engine.h"
#include "pbs_common.h"

namespace tfhe_mi355 {

namespace {
constexpr int LN = 32768;
constexpr int LM = LN / 2;
constexpr int LT = 512;                    // threads per workgroup (8 waves)
constexpr int LW = LT / 64;
using SubFft = WaveFft<1024>;
constexpr int XCH_DOUBLES = LM;            // 128 KiB exchange region
constexpr int S1_OFF = XCH_DOUBLES / 2;    // in double2 units
constexpr size_t LARGE_LDS = sizeof(double2) * (S1_OFF + SubFft::Lds::s1_len);
static_assert(LW * SubFft::XL * 2 <= XCH_DOUBLES, "wave buffers fit the exchange region");

struct LargeCtx {
    double *xch;        // exchange region (doubles)
    cx *wxb;            // this wave's 1024-entry buffer inside it
    SubFft::Lds tw;     // sub-block twiddles (LDS)
    const double2 *W;   // W_M, global
    const double2 *wtop;  // top-stage twiddles [c-1][a] = W[a c], global
    int t, lane, wave;
};

__device__ __forceinline__ LargeCtx large_setup(const double2 *W, const double2 *wtop) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    LargeCtx c;
    c.t = threadIdx.x;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.xch = reinterpret_cast<double *>(smem);
    c.wxb = reinterpret_cast<cx *>(smem) + c.wave * SubFft::XL;
    double2 *s1 = lds + S1_OFF;
    // sub-block stage twiddles W_1024[lane c] = W_M[16 lane c]  (oracle dif_rec tstride 16)
    for (int e = threadIdx.x; e < SubFft::Lds::s1_len; e += LT) s1[e] = W[16 * (e & 63) * ((e >> 6) + 1)];
    c.tw = SubFft::Lds{s1, s1};
    c.W = W;
    c.wtop = wtop;
    __syncthreads();
    return c;
}

// top stage butterflies of thread t: a = t + 512 h (h = 0, 1), values at positions a + 1024 b.
// After it, wave w owns sub-blocks 2w + h' (positions 1024 (2w+h') + [0, 1024)).
__device__ __forceinline__ void large_exchange_to_blocks(const LargeCtx &c, cx (&u)[2][16]) {
#pragma unroll
    for (int part = 0; part < 2; part++) {
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int q = 0; q < 16; q++) c.xch[c.t + 512 * h + 1024 * q] = part ? u[h][q].im : u[h][q].re;
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int b = 0; b < 16; b++) {
                const double x = c.xch[1024 * (2 * c.wave + h) + c.lane + 64 * b];
                if (part) u[h][b].im = x;
                else u[h][b].re = x;
            }
    }
    __syncthreads();  // the region now serves as the per-wave buffers
}
// forward: u[h][b] = twisted input at position (t + 512 h) + 1024 b; on exit u[h] holds
// sub-block 2 wave + h in the WaveFft<1024> Fourier layout.
__device__ __forceinline__ void large_forward(const LargeCtx &c, cx (&u)[2][16]) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int a = c.t + 512 * h;
        dft16_fwd(u[h]);
#pragma unroll
        for (int q = 1; q < 16; q++) {
            if (q % 4 == 1) __builtin_amdgcn_sched_barrier(0);  // bound twiddle loads in flight
            const cx w = gld(c.wtop + (q - 1) * 1024 + a);  // = W[a q]
            u[h][q] = cmulw(u[h][q], w.re, w.im);
        }
    }
    large_exchange_to_blocks(c, u);
    WaveLocalSync wsync;
#pragma unroll
    for (int h = 0; h < 2; h++) SubFft::forward(u[h], c.wxb, c.tw, c.lane, wsync);
}

// spectrum element (h, slot s) of thread (wave, lane) <-> offset in a poly's engine layout
__device__ __forceinline__ size_t spec_off(int wave, int h, int s, int lane) {
    return ((size_t)(2 * wave + h) * 16 + s) * 64 + lane;
}

}  // namespace

// Cache policy of the stores of f64 spectra that a later launch reads, mostly on other XCDs
// (gfx950 aux bits: 16 = sc1, write-through -- the line leaves the XCD's L2 at once instead of in
// the end-of-kernel L2 writeback; 0 = plain): large_top_fwd's top-stage spectra here (-1:
// write-through for the multi-bit path only -- its paired sub-block kernel reads them on other
// XCDs: g3 8969 -> 9089 KS+PBS/s, while 2_5 lost 2260 -> 2241), the sub-block outputs
// (LARGE_SUB_AUX, LARGE_U_AUX) below.
#ifndef LARGE_TOPF_AUX
#define LARGE_TOPF_AUX (-1)
#endif

// Shapes of the split CMUX (N = 4096 ... 32768, k = 1): M = N / 2 = R x 1024 -- a top radix-R
// stage and R independent 1024-point sub-blocks ([R | 16, 16, 4], the oracle's radix_plan).
template <int N>
struct Split {
    static constexpr int M = N / 2;
    static constexpr int R = M / 1024;
    static constexpr int LOGN = ilog2(N);
    static constexpr int LOGM = LOGN - 1;
    static_assert(R == 2 || R == 4 || R == 8 || R == 16, "top radix 2, 4, 8 or 16");
};

// Accumulator row layout: position p at u64 index 2 (p mod M) + (p div M), so the pair (j, j + M)
// that one folded complex coefficient is made of sits in one 16-byte word (one load / store in
// top_inv, one self and one rotated load per row in the digits / top stage).
template <int M>
__device__ __forceinline__ int accx_m(int p) { return 2 * (p & (M - 1)) + (p >> ilog2(M)); }
__device__ __forceinline__ int accx(int p) { return accx_m<LM>(p); }
typedef unsigned long long acc_pair __attribute__((ext_vector_type(2)));
// ct1 = X^{a~} acc - acc at positions j and j + M of one row (rem = a~ mod N, full_odd = a~ >= N):
// the rotated sources j - rem and j + M - rem lie in ONE pair word, q = (j - rem) mod M, with its
// halves swapped when only the first one wraps
template <int M>
__device__ __forceinline__ void ct1_pair_m(const uint64_t *acc, int j, int rem, bool full_odd, uint64_t &d0,
                                           uint64_t &d1) {
    const acc_pair self = *reinterpret_cast<const acc_pair *>(acc + 2 * j);
    const int jj0 = j - rem;  // in (-N, M)
    const acc_pair rot = *reinterpret_cast<const acc_pair *>(acc + 2 * (jj0 & (M - 1)));
    const bool swap = jj0 < 0 && jj0 >= -M;
    const uint64_t x0 = swap ? rot.y : rot.x, x1 = swap ? rot.x : rot.y;
    const bool neg0 = (jj0 < 0) != full_odd, neg1 = (jj0 + M < 0) != full_odd;
    d0 = (neg0 ? 0 - x0 : x0) - self.x;
    d1 = (neg1 ? 0 - x1 : x1) - self.y;
}
__device__ __forceinline__ void ct1_pair(const uint64_t *acc, int j, int rem, bool full_odd, uint64_t &d0,
                                         uint64_t &d1) {
    ct1_pair_m<LM>(acc, j, rem, full_odd, d0, d1);
}

// acc[ct] = LUT[idx] / X^{b~}  (bootstrap.rs:255-275)
template <int N, int K>
__global__ void __launch_bounds__(256) large_init_kernel(LargePbsLaunch a, int ct0, int cnt) {
    using S = Split<N>;
    const size_t per = (size_t)(K + 1) * N;
    const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= per * cnt) return;
    const int cl = (int)(e / per);
    const int p = (int)((e % per) / N), j = (int)(e % N);
    const int ct = ct0 + cl;
    const uint64_t *in = a.lwe_in + (size_t)ct * (a.n + 1);
    const uint32_t bt = pbs_modulus_switch<S::LOGN>(in[a.n]);
    const uint32_t li = a.lut_indexes ? min(a.lut_indexes[ct], a.lut_count - 1u) : 0u;
    const uint64_t *lut = a.luts + (size_t)li * (K + 1) * N + (size_t)p * N;
    const int full = bt / N, rem = bt % N;
    const int src = j + rem;
    const bool wrap = src >= N;
    const uint64_t v = lut[wrap ? src - N : src];
    a.acc[(e / N) * N + accx_m<S::M>(j)] = (wrap != (bool)(full & 1)) ? 0 - v : v;
}

// radix-R DFTs of the top stage, natural order in and out (the oracle's dft_fwd / dft_inv)
template <int R>
__device__ __forceinline__ void dftR_fwd(cx *v) {
    if constexpr (R == 2) {
        const cx x = v[0], y = v[1];
        v[0] = cadd(x, y);
        v[1] = csub(x, y);
    } else if constexpr (R == 4) {
        r4_fwd(v[0], v[1], v[2], v[3]);
    } else if constexpr (R == 8) {
        dft8_fwd(v);
    } else {
        dft16_fwd(v);
    }
}
template <int R>
__device__ __forceinline__ void dftR_inv(cx *v) {
    if constexpr (R == 2) {
        const cx x = v[0], y = v[1];
        v[0] = cadd(x, y);
        v[1] = csub(x, y);
    } else if constexpr (R == 4) {
        r4_inv(v[0], v[1], v[2], v[3]);
    } else if constexpr (R == 8) {
        dft8_inv(v);
    } else {
        dft16_inv(v);
    }
}

// all L signed digits of x, level L (least significant) first -- SignedDecomposer::decompose
// (decomposer.rs:99-153, iter.rs:134-141) in 64-bit arithmetic: any base_log * L <= 63 (the
// shortint sets go up to 11 x 3 = 33 bits).  A rounding that overflows 2^(base_log L) leaves
// every digit 0, as in the reference (whose discarded final state differs only there).
template <int L>
__device__ __forceinline__ void decompose64(uint64_t x, int beta, int32_t (&d)[L]) {
    const int nonrep = 64 - beta * L;
    uint64_t st = ((x >> (nonrep - 1)) + 1) >> 1;
    const uint64_t mask = (1ull << beta) - 1;
#pragma unroll
    for (int l = 0; l < L; l++) {
        const uint64_t res = st & mask;
        st >>= beta;
        uint64_t carry = ((res - 1) | st) & res;
        carry >>= beta - 1;
        st += carry;
        d[l] = (int32_t)(int64_t)(res - (carry << beta));
    }
}

// ---------------------------------------------------------------------------------------
// Split CMUX (N = 4096 ... 32768): the accumulator (k+1) N u64 lives in device scratch and the
// M-point FFT is [R | 16, 16, 4]; after its top radix-R stage the R sub-blocks of 1024 positions
// are independent, and so are the MAC (per frequency) and the inverse up to its own top stage.
// Three batch-wide launches per CMUX:
//   large_top_fwd : per (ct, row, butterfly a < 1024): rotate, decompose (all L levels), twist,
//                   top DIF radix-R per level -> T[ct][lvl][row][a + 1024 c]           (no LDS)
//   large_sub     : per (ct, sub-block q): (k+1) L waves run the 1024-point WaveFft of their
//                   polynomial's sub-block, publish to LDS; wave c: MAC with GGSW sub-block q of
//                   column c, inverse sub-FFT -> T[ct][lvl 1][row c][q-block]
//   large_top_inv : per (ct, column, butterfly a): top DIT radix-R, backward conversion,
//                   acc += increments                                                  (no LDS)
// Same DAG as the oracle (dif_rec / dit_rec stage 0 = top, stages 1-3 = WaveFft<1024> with
// tstride R), so the outputs are bit-exact.  At N = 32768, L = 2 the grouped CMUX below replaces
// it.  Scratch per ciphertext: acc + T.
// ---------------------------------------------------------------------------------------
#ifndef LARGE_TOPT
#define LARGE_TOPT 256
#endif
#ifndef LARGE_MAC_SB
#define LARGE_MAC_SB 4  // MAC slots per scheduling region of large_sub (GGSW loads in flight)
#endif
constexpr int TOPT = LARGE_TOPT;  // threads per top-stage workgroup

#ifndef LARGE_DIGIT2
#define LARGE_DIGIT2 1  // split / grouped digit kernels: Digit2 (pbs_common.h) when 2 base_log <= 30 (0: A/B)
#endif
// rotate, decompose, twist and top DIF radix-R of butterfly t of row r, CMUX i -> T.
// G > 0 (multi-bit, step i = group i): the external product's input is the accumulator itself
// (acc <- ExtProd(KB_i, acc), lwe_multi_bit_programmable_bootstrapping.rs:548-828): no rotation.
template <int N, int K, int L, int G>
__device__ __forceinline__ void top_fwd_body(const LargePbsLaunch &a, int ct0, int i, int cl, int r, int t) {
    using S = Split<N>;
    constexpr int R = S::R, M = S::M;
    static_assert(L >= 1 && L <= 3, "levels 1..3");
    const uint64_t *in = a.lwe_in + (size_t)(ct0 + cl) * (a.n + 1);
    const uint32_t at = G ? 0u : pbs_modulus_switch<S::LOGN>(in[i]);
    const bool full_odd = (at / N) & 1;
    const int rem = at % N;
    const uint64_t *acc = a.acc + ((size_t)cl * (K + 1) + r) * N;
    const int beta = a.base_log;
    cx u[R];
    uint64_t pk[L > 1 ? R : 1];  // levels L-1 .. 1 of both halves as int16 fields, for the later passes
#pragma unroll
    for (int b = 0; b < R; b++) {
        const int j = t + 1024 * b;
        uint64_t dd[2];  // ct1 = X^{a~} acc - acc  (polynomial_wrapping_monic_monomial_mul_and_subtract)
        if constexpr (G > 0) {
            const acc_pair self = *reinterpret_cast<const acc_pair *>(acc + 2 * j);
            dd[0] = self.x;
            dd[1] = self.y;
        } else {
            ct1_pair_m<M>(acc, j, rem, full_odd, dd[0], dd[1]);
        }
        int32_t d0[L], d1[L];
        if (LARGE_DIGIT2 && L == 2 && N <= 16384 && beta * 2 <= 30) {  // Digit2 (at N = 32768 it spilled)
            uint32_t lv0, lv1;
            Digit2(beta).pair((uint32_t)(dd[0] >> 32), (uint32_t)(dd[1] >> 32), lv0, lv1);
            d0[0] = (int32_t)(int16_t)(lv0 & 0xffffu);
            d1[0] = (int32_t)(int16_t)(lv0 >> 16);
            d0[L - 1] = (int32_t)(int16_t)(lv1 & 0xffffu);
            d1[L - 1] = (int32_t)(int16_t)(lv1 >> 16);
        } else if (LARGE_DIGIT2 && L == 1 && beta <= 30) {  // DigitL1
            const DigitL1 dl1(beta);
            d0[0] = dl1((uint32_t)(dd[0] >> 32));
            d1[0] = dl1((uint32_t)(dd[1] >> 32));
        } else {
            decompose64<L>(dd[0], beta, d0);
            decompose64<L>(dd[1], beta, d1);
        }
        if constexpr (L > 1) {
            uint64_t w = 0;
#pragma unroll
            for (int l = 1; l < L; l++)
                w |= ((uint64_t)((uint32_t)d0[l] & 0xffffu) << (32 * (l - 1))) |
                     ((uint64_t)((uint32_t)d1[l] & 0xffffu) << (32 * (l - 1) + 16));
            pk[b] = w;
        }
        const cx tw = gld(a.twist + j);
        u[b] = cmulw(cx{(double)d0[0], (double)d1[0]}, tw.re, tw.im);
    }
    auto top_and_store = [&](int lvl) {
        dftR_fwd<R>(u);
        double2 *T = a.spectra + (((size_t)cl * L + (lvl - 1)) * (K + 1) + r) * M + t;
        // read by the sub-block workgroups, mostly on other XCDs
        auto st = [&](int c, double2 x) {
            constexpr int AUX = LARGE_TOPF_AUX < 0 ? (G > 0 ? 16 : 0) : LARGE_TOPF_AUX;
            if (AUX) buffer_st_d2p<AUX>(make_rsrc(T - t), 16u * (t + 1024 * c), 0, x);
            else T[1024 * c] = x;
        };
        st(0, make_double2(u[0].re, u[0].im));
#pragma unroll
        for (int c = 1; c < R; c++) {
            const cx w = gld(a.wtop + (c - 1) * 1024 + t);  // = W[t c]
            const cx y = cmulw(u[c], w.re, w.im);
            st(c, make_double2(y.re, y.im));
        }
    };
    top_and_store(L);
#pragma unroll
    for (int l = 1; l < L; l++) {
#pragma unroll
        for (int b = 0; b < R; b++) {
            const int32_t e0 = (int32_t)(int16_t)((pk[b] >> (32 * (l - 1))) & 0xffffu);
            const int32_t e1 = (int32_t)(int16_t)((pk[b] >> (32 * (l - 1) + 16)) & 0xffffu);
            const cx tw = gld(a.twist + t + 1024 * b);
            u[b] = cmulw(cx{(double)e0, (double)e1}, tw.re, tw.im);
        }
        top_and_store(L - l);
    }
}

// waves per SIMD the top stage's register budget allows: 4 (128 VGPRs) except the radix-16 stage
// with one or three levels, which spills at 128 (the compiler keeps more of it live)
template <int N, int L>
constexpr int top_fwd_wpe() { return Split<N>::R == 16 && L != 2 ? 2 : 4; }

template <int N, int K, int L, int G>
__global__ void __launch_bounds__(TOPT, (top_fwd_wpe<N, L>())) large_top_fwd_kernel(LargePbsLaunch a, int ct0, int i) {
    constexpr int BPP = 1024 / TOPT;  // workgroups per polynomial
    // XCD-aware: workgroup w runs on XCD w % 8; all (K+1) BPP workgroups of a ciphertext share
    // one XCD, so the rotated gather re-reads the accumulator rows from that XCD's L2
    const int x = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int sub = m % ((K + 1) * BPP);
    const int cl = x + 8 * (m / ((K + 1) * BPP));
    if (cl >= a.chunk_count) return;  // whole workgroup
    top_fwd_body<N, K, L, G>(a, ct0, i, cl, sub / BPP, (sub % BPP) * TOPT + threadIdx.x);
}

#ifndef LARGE_U_AUX
#define LARGE_U_AUX 16  // cache policy of the group kernel's U stores: 16 = sc1 (write-through), 0 = plain
#endif
#ifndef LARGE_SUB_AUX
#define LARGE_SUB_AUX 16  // the same for the split path's sub-block outputs (large_sub / dsub / pair_sub)
#endif
// sub-block output of one wave: 16 x 16 B per lane, cache policy AUX (16: write-through)
template <int AUX>
__device__ __forceinline__ void store_sub_out(double2 *dst, const cx (&v)[16], int lane) {
#pragma unroll
    for (int b = 0; b < 16; b++) {
        if (AUX) buffer_st_d2p<AUX>(make_rsrc(dst - lane), 16u * (lane + 64 * b), 0, make_double2(v[b].re, v[b].im));
        else dst[64 * b] = make_double2(v[b].re, v[b].im);
    }
}

// (k+1) L waves; LDS: one 1024-entry buffer per wave + the sub-block twiddle table
template <int K, int L>
struct LargeSubCfg {
    static constexpr int WAVES = (K + 1) * L;
    static constexpr int THREADS = 64 * WAVES;
    static constexpr int S1 = WAVES * SubFft::XL;  // table offset (double2 units)
    static constexpr size_t LDS = sizeof(double2) * (S1 + SubFft::Lds::s1_len);
};

// workgroup -> (sub-block q, chunk ciphertext cl): at R >= 8 consecutive workgroups land on
// consecutive XCDs (8), so XCD x only ever sees sub-blocks q = x (mod 8) -- their GGSW slices stay
// in its L2
template <int R>
__device__ __forceinline__ void sub_block_of(int b, int &q, int &cl) {
    if constexpr (R >= 8) {
        const int x = b & 7, y = b >> 3;
        q = x + 8 * (y % (R / 8));
        cl = y / (R / 8);
    } else {
        q = b % R;
        cl = b / R;
    }
}

// multi-bit: spectrum of X^d at frequency f, i^q twist[r] with t = d (1 - 4 f) mod 2N = q M + r
// (exact; the oracle's mono_spectrum, the same sign/swap per quadrant)
template <int N>
__device__ __forceinline__ cx mono_spectrum(const double2 *__restrict__ twist, uint32_t d, uint32_t f) {
    constexpr int M = N / 2;
    const uint32_t t = (d - 4u * d * f) & (uint32_t)(2 * N - 1);
    const uint32_t q = t / (uint32_t)M, r = t % (uint32_t)M;
    const cx w = gld(twist + r);
    switch (q) {
        case 0: return w;
        case 1: return cx{-w.im, w.re};
        case 2: return cx{-w.re, -w.im};
        default: return cx{w.im, -w.re};
    }
}

// the sub-block CMUX of one (ciphertext, sub-block q) after this wave's input v (polynomial
// (lvl - 1)(K+1) + r = wave, sub-block q, natural layout) is in registers and the twiddle table
// is visible: forward sub-FFT, publish, MAC of column c = wave, inverse -> T[lvl 1][row c][q]
template <int N, int K, int L>
__device__ __forceinline__ void sub_cmux_body(const LargePbsLaunch &a, int i, int q, double2 *T, double2 *lds, cx (&v)[16],
                                              const SubFft::Lds &tw, int wave, int lane) {
    constexpr int M = Split<N>::M;
    cx *xb = reinterpret_cast<cx *>(lds) + wave * SubFft::XL;
    WaveLocalSync wsync;
    SubFft::forward(v, xb, tw, lane, wsync);
    wsync();
#pragma unroll
    for (int s = 0; s < 16; s++) reinterpret_cast<double2 *>(xb)[s * 64 + lane] = make_double2(v[s].re, v[s].im);
    __syncthreads();
    const bool mac = wave <= K;  // wave c computes output column c
    if (mac) {
        // column c: sum over levels L..1 and rows 0..k (ggsw.rs:524-567), oracle order
        constexpr size_t ggsw_len = (size_t)L * (K + 1) * (K + 1) * M;
        const double2 *Gp = a.fbsk + (size_t)i * ggsw_len + (size_t)wave * M + 1024 * q + lane;
#pragma unroll
        for (int s = 0; s < 16; s++) {
            if (s % LARGE_MAC_SB == 0) __builtin_amdgcn_sched_barrier(0);  // bound the loads in flight
            cx o{0.0, 0.0};
#pragma unroll
            for (int lvl = L; lvl >= 1; lvl--) {
#pragma unroll
                for (int r = 0; r <= K; r++) {
                    const int p = (lvl - 1) * (K + 1) + r;
                    const double2 gg = Gp[(size_t)p * (K + 1) * M + s * 64];
                    const double2 ff = reinterpret_cast<const double2 *>(lds)[p * SubFft::XL + s * 64 + lane];
                    if (lvl == L && r == 0) {
                        o.re = fma(gg.x, ff.x, -(gg.y * ff.y));
                        o.im = fma(gg.x, ff.y, gg.y * ff.x);
                    } else {
                        o.re = fma(gg.x, ff.x, fma(-gg.y, ff.y, o.re));
                        o.im = fma(gg.x, ff.y, fma(gg.y, ff.x, o.im));
                    }
                }
            }
            v[s] = o;
        }
    }
    __syncthreads();  // every column's MAC has read the published spectra
    if (!mac) return;
    SubFft::inverse(v, xb, tw, lane, wsync);
    double2 *dst = T + (size_t)wave * M + 1024 * q + lane;  // (lvl 1, row c) slot: read by this WG only
    store_sub_out<LARGE_SUB_AUX>(dst, v, lane);
}

// classic CMUX sub-blocks from large_top_fwd's spectra (the multi-bit sets run
// large_pair_sub_kernel below)
template <int N, int K, int L>
__global__ void __launch_bounds__((LargeSubCfg<K, L>::THREADS), 2) large_sub_kernel(LargePbsLaunch a, int ct0, int i) {
    using Cfg = LargeSubCfg<K, L>;
    using S = Split<N>;
    constexpr int M = S::M, R = S::R;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int q, cl;
    sub_block_of<R>(blockIdx.x, q, cl);
    double2 *s1 = lds + Cfg::S1;
    // sub-block stage twiddles W_1024[lane c] = W_M[R lane c]  (oracle dif_rec tstride R)
    for (int e = threadIdx.x; e < SubFft::Lds::s1_len; e += Cfg::THREADS) s1[e] = a.W[R * (e & 63) * ((e >> 6) + 1)];
    const SubFft::Lds tw{s1, s1};
    double2 *T = a.spectra + (size_t)cl * L * (K + 1) * M;
    cx v[16];
    {
        const double2 *src = T + (size_t)wave * M + 1024 * q + lane;
#pragma unroll
        for (int b = 0; b < 16; b++) v[b] = gld(src + 64 * b);
    }
    __syncthreads();  // twiddle table
    sub_cmux_body<N, K, L>(a, i, q, T, lds, v, tw, wave, lane);
}

// ---------------------------------------------------------------------------------------
// Digits-fed split CMUX (L = 2, k = 1, N = 4096 and 8192).  As the grouped CMUX
// at N = 32768 does, large_top_fwd's f64 spectra (4 polynomials x M x 16 B per ciphertext written,
// then read back) are replaced by packed int16 digits (M x 16 B) and the twist + top radix-R
// share of each sub-block is computed where it is consumed:
//   split_digits_kernel : per (ct, j < M), both rows: ct1 = X^{a~} acc - acc at j and j + M,
//                         decompose64<2> (the top stage's own decomposition), four int16 digits
//                         per row word (level L at j, j + M; level L-1 at j, j + M)
//   large_dsub_kernel   : per (ct, sub-block q): for every butterfly a < 1024 and polynomial
//                         (level, row): twist, the top DIF radix-R (dftR_fwd, every output as the
//                         top stage computes them), output q times W[a q] -> the wave's LDS buffer
//                         in the WaveFft<1024> natural layout; then the sub-block CMUX as above.
// The R workgroups of a ciphertext run on one XCD (digits from the Infinity Cache once, then L2;
// the CMUX's GGSW, 0.25-0.5 MiB, fits that L2).  Same operations in the same order as
// large_top_fwd + large_sub_kernel, so the outputs are bit-identical.  Digits live in the
// ciphertext's level-2 spectra slots, which this path does not otherwise use.
// ---------------------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ acc_pair *split_digits(const LargePbsLaunch &a, int cl) {
    constexpr int M = Split<N>::M;
    return reinterpret_cast<acc_pair *>(a.spectra + ((size_t)cl * 2 * 2 + 2) * M);
}

template <int N>
__global__ void __launch_bounds__(256) split_digits_kernel(LargePbsLaunch a, int ct0, int i) {
    using S = Split<N>;
    constexpr int M = S::M, PER = M / 256;
    const int x = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int cl = x + 8 * (m / PER), sub = m % PER;
    if (cl >= a.chunk_count) return;
    const uint64_t *in = a.lwe_in + (size_t)(ct0 + cl) * (a.n + 1);
    const uint32_t at = pbs_modulus_switch<S::LOGN>(in[i]);
    const bool full_odd = (at / N) & 1;
    const int rem = at % N;
    const int j = sub * 256 + threadIdx.x;
    uint64_t w[2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        uint64_t dd[2];
        ct1_pair_m<M>(a.acc + ((size_t)cl * 2 + r) * N, j, rem, full_odd, dd[0], dd[1]);
        if (LARGE_DIGIT2 && a.base_log * 2 <= 30) {  // Digit2: the same words, 32-bit
            uint32_t lv0, lv1;
            Digit2(a.base_log).pair((uint32_t)(dd[0] >> 32), (uint32_t)(dd[1] >> 32), lv0, lv1);
            w[r] = (uint64_t)lv0 | ((uint64_t)lv1 << 32);
            continue;
        }
        int32_t d0[2], d1[2];
        decompose64<2>(dd[0], a.base_log, d0);
        decompose64<2>(dd[1], a.base_log, d1);
        w[r] = ((uint64_t)((uint32_t)d0[0] & 0xffffu)) | ((uint64_t)((uint32_t)d1[0] & 0xffffu) << 16) |
               ((uint64_t)((uint32_t)d0[1] & 0xffffu) << 32) | ((uint64_t)((uint32_t)d1[1] & 0xffffu) << 48);
    }
    split_digits<N>(a, cl)[j] = acc_pair{w[0], w[1]};
}

// phase 1 of large_dsub_kernel for sub-block Q: butterflies a0 = tid + 256 t -> the LDS buffer of
// polynomial p = (lvl - 1)(K+1) + r at a0 (twist, top DIF radix-R, output Q times W[a0 Q])
template <int N, int Q>
__device__ __forceinline__ void dsub_phase1(const LargePbsLaunch &a, const acc_pair *dig, double2 *lds) {
    constexpr int K = 1, R = Split<N>::R;
    using Cfg = LargeSubCfg<K, 2>;
    for (int a0 = threadIdx.x; a0 < 1024; a0 += Cfg::THREADS) {
        acc_pair dw[R];
        cx tv[R];
#pragma unroll
        for (int b = 0; b < R; b++) {
            dw[b] = dig[a0 + 1024 * b];
            tv[b] = gld(a.twist + a0 + 1024 * b);
        }
        const cx wq = Q ? gld(a.wtop + (Q - 1) * 1024 + a0) : cx{1.0, 0.0};  // = W[a0 Q]
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int li = 0; li < 2; li++) {  // li = 0: level L (the top stage's first pass), 1: level L-1
                cx u[R];
#pragma unroll
                for (int b = 0; b < R; b++) {
                    const uint64_t wr = r ? dw[b].y : dw[b].x;
                    const int32_t e0 = (int32_t)(int16_t)((wr >> (32 * li)) & 0xffffu);
                    const int32_t e1 = (int32_t)(int16_t)((wr >> (32 * li + 16)) & 0xffffu);
                    u[b] = cmulw(cx{(double)e0, (double)e1}, tv[b].re, tv[b].im);
                }
                dftR_fwd<R>(u);
                const cx y = Q ? cmulw(u[Q], wq.re, wq.im) : u[0];
                const int p = (1 - li) * (K + 1) + r;  // level L -> polys 2, 3; level L-1 -> 0, 1
                lds[p * SubFft::XL + a0] = make_double2(y.re, y.im);
            }
    }
}

template <int N>
__global__ void __launch_bounds__((LargeSubCfg<1, 2>::THREADS), 2) large_dsub_kernel(LargePbsLaunch a, int ct0, int i) {
    constexpr int K = 1, L = 2;
    using Cfg = LargeSubCfg<K, L>;
    using S = Split<N>;
    constexpr int M = S::M, R = S::R;
    static_assert(R <= 4, "N <= 8192 (the top stage's R-fold recomputation loses at R = 8)");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // the R sub-block workgroups of ciphertext cl: blocks 8 m + x with the same x (one XCD)
    const int x = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int cl = x + 8 * (m / R), q = m % R;
    if (cl >= a.chunk_count) return;  // whole workgroup
    (void)ct0;
    double2 *s1 = lds + Cfg::S1;
    for (int e = threadIdx.x; e < SubFft::Lds::s1_len; e += Cfg::THREADS) s1[e] = a.W[R * (e & 63) * ((e >> 6) + 1)];
    const SubFft::Lds tw{s1, s1};
    const acc_pair *dig = split_digits<N>(a, cl);
    // phase 1 with the sub-block index a compile-time constant, so that only output q of each top
    // radix-R butterfly is computed (the compiler drops the other outputs' adds)
    switch (q) {
        case 0: dsub_phase1<N, 0>(a, dig, lds); break;
        case 1: dsub_phase1<N, 1>(a, dig, lds); break;
        case 2: if constexpr (R > 2) dsub_phase1<N, 2>(a, dig, lds); break;
        default: if constexpr (R > 3) dsub_phase1<N, 3>(a, dig, lds); break;
    }
    __syncthreads();  // phase-1 outputs and the twiddle table
    cx v[16];
#pragma unroll
    for (int b = 0; b < 16; b++) {
        const double2 t = lds[wave * SubFft::XL + lane + 64 * b];
        v[b] = cx{t.x, t.y};
    }
    double2 *T = a.spectra + (size_t)cl * L * (K + 1) * M;
    sub_cmux_body<N, K, L>(a, i, q, T, lds, v, tw, wave, lane);
}

// ---------------------------------------------------------------------------------------
// Paired sub-block kernel (split CMUX, L <= 2).  The MAC needs the GGSW operands of
// every (level, row, column, frequency) -- for multi-bit the 2^g GGSWs of the group, 1 MiB per
// sub-block at g = 3, k = 1, L = 2.  One workgroup per sub-block q and PAIR of ciphertexts,
// 2 (k+1) L waves:
//   phase 1  wave (c, p): forward sub-FFT of polynomial p of ciphertext c, published to LDS;
//   phase 2  wave w owns spectrum slots SPW w .. SPW w + SPW - 1 of BOTH ciphertexts and all
//            columns: per (slot, level, column) it loads the (k+1) (x 2^g) operands once (so each
//            GGSW byte is read once per pair of ciphertexts), builds each ciphertext's keybundle
//            entries with its own monomials (multi-bit) and MACs them into registers; the slot's outputs go
//            over the (level 1, row = column) spectra, which no other wave reads;
//   phase 3  wave (c, column), c < 2: inverse sub-FFT, store to the spectra scratch.
// Every wave of the 2 (k+1) L works in phases 1 and 2 (the single-ciphertext kernel above leaves
// L - 1 of every L waves idle in its MAC), the operands of the next (level, column) are in flight
// while the current one is consumed, and at R <= 8 all workgroups of sub-block q run on the XCDs
// x = q (mod R), so a group's GGSW slice stays in their L2.  Per (ciphertext, column, frequency)
// the arithmetic and its order are those of large_sub_kernel (keybundle in selector order, MAC
// over levels L..1 and rows 0..k), so the outputs are bit-identical.
// ---------------------------------------------------------------------------------------
template <int K, int L>
struct PairSubCfg {
    static constexpr int CPW = 2;                    // ciphertexts per workgroup
    static constexpr int PW = (K + 1) * L;           // polynomials per ciphertext
    static constexpr int WAVES = CPW * PW;
    static constexpr int THREADS = 64 * WAVES;
    static constexpr int SPW = 16 / WAVES;           // phase-2 slots per wave
    static_assert(16 % WAVES == 0, "slots split evenly over the waves");
    static constexpr int S1 = WAVES * SubFft::XL;    // twiddle table offset (double2 units)
    static constexpr size_t LDS = sizeof(double2) * (S1 + SubFft::Lds::s1_len);
    static_assert(LDS <= 160 * 1024, "LDS per workgroup exceeds a CU");
};

// workgroup -> (sub-block q, ciphertext pair cp): at R <= 8 XCD x = b % 8 serves q = x % R only
template <int R>
__device__ __forceinline__ void pair_sub_block_of(int b, int &q, int &cp) {
    const int x = b & 7, y = b >> 3;
    if constexpr (R >= 8) {
        q = x + 8 * (y % (R / 8));
        cp = y / (R / 8);
    } else {
        q = x % R;
        cp = y * (8 / R) + x / R;
    }
}
template <int R>
constexpr unsigned pair_sub_blocks(int pairs) {
    return R >= 8 ? (unsigned)pairs * R : (unsigned)((pairs + 8 / R - 1) / (8 / R)) * 8u;
}

// SB: (level, column) operand batches per scheduling region (loads of SB batches in flight)
template <int N, int K, int L, int G, int SB>
__global__ void __launch_bounds__((PairSubCfg<K, L>::THREADS), 2) large_pair_sub_kernel(LargePbsLaunch a, int ct0, int i) {
    using Cfg = PairSubCfg<K, L>;
    using S = Split<N>;
    constexpr int M = S::M, R = S::R;
    constexpr int NSEL = G ? 1 << G : 1;
    constexpr int CPW = Cfg::CPW, PW = Cfg::PW, SPW = Cfg::SPW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int q, cp;
    pair_sub_block_of<R>(blockIdx.x, q, cp);
    const int cnt = a.chunk_count;
    if (2 * cp >= cnt) return;  // whole workgroup
    double2 *s1 = lds + Cfg::S1;
    for (int e = threadIdx.x; e < SubFft::Lds::s1_len; e += Cfg::THREADS) s1[e] = a.W[R * (e & 63) * ((e >> 6) + 1)];
    const SubFft::Lds tw{s1, s1};
    WaveLocalSync wsync;
    auto buf = [&](int c, int p) { return reinterpret_cast<cx *>(lds) + (c * PW + p) * SubFft::XL; };
    auto ct_of = [&](int c) { return min(2 * cp + c, cnt - 1); };  // idle slot: a valid ciphertext
    auto spectra = [&](int c) { return a.spectra + (size_t)ct_of(c) * L * (K + 1) * M; };

    // ---- phase 1: forward sub-FFT of polynomial p of ciphertext c ----
    {
        const int c = wave / PW, p = wave % PW;
        cx v[16];
        const double2 *src = spectra(c) + (size_t)p * M + 1024 * q + lane;
#pragma unroll
        for (int b = 0; b < 16; b++) v[b] = gld(src + 64 * b);
        __syncthreads();  // twiddle table
        cx *xb = buf(c, p);
        SubFft::forward(v, xb, tw, lane, wsync);
        wsync();
#pragma unroll
        for (int s = 0; s < 16; s++) reinterpret_cast<double2 *>(xb)[s * 64 + lane] = make_double2(v[s].re, v[s].im);
    }
    // monomial degrees of each ciphertext's 2^g - 1 non-constant GGSWs (wave-uniform)
    uint32_t deg[CPW][NSEL];
#pragma unroll
    for (int c = 0; c < (G ? CPW : 0); c++) {
        const uint64_t *in = a.lwe_in + (size_t)(ct0 + ct_of(c)) * (a.n + 1) + (size_t)i * G;
#pragma unroll
        for (int sel = 1; sel < NSEL; sel++) {
            uint64_t d = 0;
#pragma unroll
            for (int b = 0; b < G; b++)
                if ((sel >> (G - 1 - b)) & 1) d += in[b];
            deg[c][sel] = pbs_modulus_switch<S::LOGN>(d);
        }
    }
    // the group's 2^g GGSWs through a buffer resource: element (sel, lvl, r, col, position) at
    // ((sel L + lvl - 1) (K+1) + r) (K+1) M + col M + position
    constexpr size_t ggsw_len = (size_t)L * (K + 1) * (K + 1) * M;
    constexpr uint32_t rowb = 16u * (uint32_t)((K + 1) * M);
    const __amdgpu_buffer_rsrc_t grs = make_rsrc(a.fbsk + (size_t)i * NSEL * ggsw_len);
    const uint32_t gvo = 16u * (uint32_t)(1024 * q + lane);
    const uint32_t fl = (uint32_t)q + (uint32_t)R * SubFft::freq_lane(lane);
    __syncthreads();  // spectra published

    // ---- phase 2: keybundle + MAC of this wave's slots for both ciphertexts ----
#pragma unroll
    for (int si = 0; si < SPW; si++) {
        const int s = wave * SPW + si;  // wave-uniform
        const uint32_t f = fl + (uint32_t)R * SubFft::freq_slot(s);
        cx mono[CPW][NSEL];
#pragma unroll
        for (int c = 0; c < CPW; c++)
#pragma unroll
            for (int sel = 1; sel < NSEL; sel++) mono[c][sel] = mono_spectrum<N>(a.twist, deg[c][sel], f);
        cx o[CPW][K + 1];
#pragma unroll
        for (int lvl = L; lvl >= 1; lvl--) {
            cx ff[CPW][K + 1];
#pragma unroll
            for (int c = 0; c < CPW; c++)
#pragma unroll
                for (int r = 0; r <= K; r++) {
                    const double2 t = reinterpret_cast<const double2 *>(buf(c, (lvl - 1) * (K + 1) + r))[s * 64 + lane];
                    ff[c][r] = cx{t.x, t.y};
                }
#pragma unroll
            for (int col = 0; col <= K; col++) {
                if (((L - lvl) * (K + 1) + col) % SB == 0) __builtin_amdgcn_sched_barrier(0);
                double2 g[K + 1][NSEL];
#pragma unroll
                for (int r = 0; r <= K; r++)
#pragma unroll
                    for (int sel = 0; sel < NSEL; sel++)
                        g[r][sel] = buffer_ld_d2(grs, gvo,
                                                 (uint32_t)(16u * sel * ggsw_len) + (uint32_t)((lvl - 1) * (K + 1) + r) * rowb +
                                                     16u * (uint32_t)(col * M) + 1024u * (uint32_t)s);
#pragma unroll
                for (int c = 0; c < CPW; c++) {
#pragma unroll
                    for (int r = 0; r <= K; r++) {
                        double2 kb = g[r][0];
#pragma unroll
                        for (int sel = 1; sel < NSEL; sel++) {
                            kb.x = fma(g[r][sel].x, mono[c][sel].re, fma(-g[r][sel].y, mono[c][sel].im, kb.x));
                            kb.y = fma(g[r][sel].x, mono[c][sel].im, fma(g[r][sel].y, mono[c][sel].re, kb.y));
                        }
                        cx &oc = o[c][col];
                        if (lvl == L && r == 0) {
                            oc.re = fma(kb.x, ff[c][r].re, -(kb.y * ff[c][r].im));
                            oc.im = fma(kb.x, ff[c][r].im, kb.y * ff[c][r].re);
                        } else {
                            oc.re = fma(kb.x, ff[c][r].re, fma(-kb.y, ff[c][r].im, oc.re));
                            oc.im = fma(kb.x, ff[c][r].im, fma(kb.y, ff[c][r].re, oc.im));
                        }
                    }
                }
            }
        }
        // outputs over the (level 1, row = column) spectra of slot s: read only by this wave, and
        // every read of slot s is above
#pragma unroll
        for (int c = 0; c < CPW; c++)
#pragma unroll
            for (int col = 0; col <= K; col++)
                reinterpret_cast<double2 *>(buf(c, col))[s * 64 + lane] = make_double2(o[c][col].re, o[c][col].im);
    }
    __syncthreads();
    // ---- phase 3: inverse sub-FFT of column col of ciphertext c ----
    if (wave >= CPW * (K + 1)) return;
    const int c = wave / (K + 1), col = wave % (K + 1);
    cx *xb = buf(c, col);
    cx v[16];
#pragma unroll
    for (int s = 0; s < 16; s++) {
        const double2 t = reinterpret_cast<const double2 *>(xb)[s * 64 + lane];
        v[s] = cx{t.x, t.y};
    }
    wsync();
    SubFft::inverse(v, xb, tw, lane, wsync);
    if (2 * cp + c >= cnt) return;
    double2 *dst = spectra(c) + (size_t)col * M + 1024 * q + lane;  // (lvl 1, row col) slot: this WG only
    store_sub_out<LARGE_SUB_AUX>(dst, v, lane);
}

// ---------------------------------------------------------------------------------------
// Multi-bit paired sub-block kernel with the monomials from LDS (N = 8192, k = 1, L = 2, g = 2 / 3:
// the PARAM_MULTI_BIT_MESSAGE_3_CARRY_3 sets, multi_bit.rs:134,192).  The kernel
// above reads every monomial spectrum i^q twist[r] from the global twist table: 2^g - 1 gathers per
// (ciphertext, slot), 64 lanes on scattered 16-byte entries, which with the GGSW operand loads make
// up ~half of its time (timing-only builds).  Here the table lives in LDS as two
// swizzled double planes (TwistLds<4096>, 64 KiB, the address-free form of pbs_multibit.hip), which
// fits once the spectra no longer occupy the whole 128 KiB exchange region during the MAC:
//   phase 1  wave (c, p): forward sub-FFT of polynomial p of ciphertext c (its 16 KiB exchange block
//            of the region), spectrum kept in registers; then the region becomes [twist planes |
//            half buffer];
//   phase 2  two rounds h = 0, 1: every wave publishes slots 8h .. 8h + 7 of its spectrum into the
//            half buffer (8 polynomials x 8 slots, 64 KiB), then wave w builds the keybundle and MAC
//            of slot 8h + w for both ciphertexts and both columns (GGSW operands loaded once per
//            pair, as above; monomials from LDS);
//   phase 3  the MAC outputs (2 ciphertexts x 2 columns x 16 slots) go to the half buffer, and wave
//            (c, col) inverse-transforms its column in it.
// Per (ciphertext, column, frequency) the keybundle (selector order) and MAC (levels L..1, rows
// 0..k) are those of the kernel above, so the outputs are bit-identical.  TFHE_MI355_MB_PAIR2=0
// selects the kernel above (A/B).
// ---------------------------------------------------------------------------------------
#ifndef MB_DIGITS_MIN
#define MB_DIGITS_MIN 128  // smallest chunk fed packed digits (TFHE_MI355_MB_DIGITS_MIN overrides; profiles/r06_mb_digits_min.txt)
#endif
#ifndef MB2_PIPE
#define MB2_PIPE 1  // phase 2's GGSW operand batches software pipelined (0: one (level, column) batch at a time)
#endif
#ifndef MB2_DEPTH
#define MB2_DEPTH 2  // MB2_PIPE: operand batches issued ahead of the one being consumed (1: 11.83k / 10.16-10.28k, 2: 11.88k / 10.40-10.43k KS+PBS/s at g = 3 / 2, profiles/r05_ab_mb_depth.log)
#endif
#ifndef MB2_SROT
#define MB2_SROT 1  // MAC slot of wave w rotated per workgroup (0: slot 8 h + w everywhere)
#endif
#ifndef MB2_TSKIP
#define MB2_TSKIP 0  // timing-only builds (wrong outputs): 1 no GGSW loads, 2 no forward sub-FFTs, 4 no
                     // inverse sub-FFTs, 8 no keybundle sums (PBS_MB_TSKIP_MONO=1: conflict-free monomials)
#endif
// top DIF output Q of butterfly a0 for both rows and levels -> spectra buffers p = (lvl - 1) 2 + r
// (tv[h][b] = twist[a0 + 1024 b], wq[h] = W[a0 Q], loaded by the caller ahead of the barrier)
// (L = 1: one level, the digits of j and j + M as two int32 fields -> buffers p = r)
template <int N, int Q, int H, int L = 2>
__device__ __forceinline__ void quad_top(double2 *lds, const uint64_t (&pk)[2][H][Split<N>::R],
                                         const cx (&tvh)[H][Split<N>::R], const cx (&wqh)[H], int t) {
    constexpr int R = Split<N>::R, BUF = SubFft::XL;
    static_assert(L == 1 || L == 2, "one or two levels");
#pragma unroll
    for (int h = 0; h < H; h++) {
        const int a0 = t + 512 * h;
        const cx *tv = tvh[h];
        const cx wq = wqh[h];
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int li = 0; li < L; li++) {  // li = 0: level L, 1: level L-1
                cx u[R];
#pragma unroll
                for (int b = 0; b < R; b++) {
                    int32_t d0, d1;
                    if constexpr (L == 2) {
                        const uint64_t w = pk[r][h][b] >> (32 * li);
                        d0 = (int32_t)(int16_t)(w & 0xffffu);
                        d1 = (int32_t)(int16_t)((w >> 16) & 0xffffu);
                    } else {
                        d0 = (int32_t)(uint32_t)pk[r][h][b];
                        d1 = (int32_t)(uint32_t)(pk[r][h][b] >> 32);
                    }
                    u[b] = cmulw(cx{(double)d0, (double)d1}, tv[b].re, tv[b].im);
                }
                dftR_fwd<R>(u);
                const cx y = Q ? cmulw(u[Q], wq.re, wq.im) : u[0];
                const int p = (L - 1 - li) * 2 + r;  // level L -> 2, 3 (L = 2) or 0, 1 (L = 1); level L-1 -> 0, 1
                lds[p * BUF + a0] = make_double2(y.re, y.im);
            }
    }
}

// MB2_DIGITS: the multi-bit step's input as packed int16 digits (the quad / on-chip word: level L at
// j, j + M in the low dword, level L-1 in the high dword), row r at [r M + j], in the level-2
// spectra slots of the ciphertext (the pair kernel's outputs go to the level-1 slots)
template <int N>
__device__ __forceinline__ uint64_t *mb_digits(const LargePbsLaunch &a, int cl) {
    constexpr int M = Split<N>::M;
    return reinterpret_cast<uint64_t *>(a.spectra + ((size_t)cl * 4 + 2) * M);
}

// digits of group 0 (the initial accumulator; multi-bit: no rotation), thread per (ct, row, t < 1024)
template <int N>
__global__ void __launch_bounds__(256) mb_digits_init_kernel(LargePbsLaunch a, int ct0) {
    constexpr int M = Split<N>::M, R = Split<N>::R;
    (void)ct0;
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int cl = e / 2048, r = (e >> 10) & 1, t = e & 1023;
    if (cl >= a.chunk_count) return;
    const Digit2 dg2(a.base_log);
    const uint64_t *acc = a.acc + ((size_t)cl * 2 + r) * N;
    uint64_t *dg = mb_digits<N>(a, cl) + (size_t)r * M;
#pragma unroll
    for (int b = 0; b < R; b++) {
        const int j = t + 1024 * b;
        const acc_pair self = *reinterpret_cast<const acc_pair *>(acc + 2 * j);
        uint32_t lv0, lv1;
        dg2.pair((uint32_t)(self.x >> 32), (uint32_t)(self.y >> 32), lv0, lv1);
        dg[j] = (uint64_t)lv0 | ((uint64_t)lv1 << 32);
    }
}

template <int N, int G>
struct MbPair2Cfg {
    static constexpr int K = 1, L = 2, CPW = 2, PW = (K + 1) * L, WAVES = CPW * PW, THREADS = 64 * WAVES;
    static constexpr int M = N / 2;
    static constexpr int REGION = WAVES * SubFft::XL;      // double2: phase-1 exchange blocks
    static constexpr int TWIST = 0;                        // phase 2: twist planes (2 M doubles) at byte 0
    static constexpr int HALF = M;                         // then the half buffer [poly][8 slots][64]
    static constexpr int S1 = REGION;                      // sub-FFT twiddle table
    static constexpr size_t LDS = sizeof(double2) * (S1 + SubFft::Lds::s1_len);
    static_assert(M + WAVES * 8 * 64 <= REGION, "twist planes + half buffer fit the exchange region");
    static_assert(LDS <= 160 * 1024, "LDS per workgroup exceeds a CU");
};

template <int N, int G, bool DIG>
__global__ void __launch_bounds__((MbPair2Cfg<N, G>::THREADS), 2) large_mb_pair2_kernel(LargePbsLaunch a, int ct0, int i) {
    using Cfg = MbPair2Cfg<N, G>;
    using S = Split<N>;
    using Tw = TwistLds<Cfg::M>;
    constexpr int K = 1, L = 2, M = S::M, R = S::R, NSEL = 1 << G;
    constexpr int CPW = Cfg::CPW, PW = Cfg::PW;
    static_assert(M == Cfg::M, "split shape");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int q, cp;
    pair_sub_block_of<R>(blockIdx.x, q, cp);
    const int cnt = a.chunk_count;
    if (2 * cp >= cnt) return;  // whole workgroup
    // the slot of wave w in each MAC round: 8 h + ws, rotated by the workgroup's index among those
    // of its XCD (MB2_SROT) so that its CUs do not all stream the same GGSW slot at once
    const int ws = (wave + (MB2_SROT ? (int)(blockIdx.x >> 3) : 0)) & 7;
    double2 *s1 = lds + Cfg::S1;
    for (int e = threadIdx.x; e < SubFft::Lds::s1_len; e += Cfg::THREADS) s1[e] = a.W[R * (e & 63) * ((e >> 6) + 1)];
    const SubFft::Lds tw{s1, s1};
    WaveLocalSync wsync;
    auto ct_of = [&](int c) { return min(2 * cp + c, cnt - 1); };  // idle slot: a valid ciphertext
    auto spectra = [&](int c) { return a.spectra + (size_t)ct_of(c) * L * (K + 1) * M; };

    // ---- phase 1: forward sub-FFT of polynomial p of ciphertext c (spectrum stays in registers) ----
    const int c1 = wave / PW, p1 = wave % PW;
    cx v[16];
    if constexpr (DIG) {
        // the top DIF output q of both ciphertexts' four polynomials, from their packed digits
        // (quad_top: twist, dftR_fwd, times W[a0 q] -- top_fwd_body's operations), thread t serving
        // butterflies a0 = t + 512 h -> the waves' exchange blocks in the natural layout
        const int t = threadIdx.x;
        cx tvh[2][R], wqh[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
#pragma unroll
            for (int b = 0; b < R; b++) tvh[h][b] = gld(a.twist + t + 512 * h + 1024 * b);
            wqh[h] = q ? gld(a.wtop + (q - 1) * 1024 + t + 512 * h) : cx{1.0, 0.0};
        }
#pragma unroll
        for (int c = 0; c < CPW; c++) {
            const uint64_t *dg = mb_digits<N>(a, ct_of(c));
            uint64_t pk[2][2][R];
#pragma unroll
            for (int r = 0; r < 2; r++)
#pragma unroll
                for (int h = 0; h < 2; h++)
#pragma unroll
                    for (int b = 0; b < R; b++) pk[r][h][b] = dg[r * M + t + 512 * h + 1024 * b];
            double2 *blk = lds + c * PW * SubFft::XL;
            switch (q) {
                case 0: quad_top<N, 0, 2>(blk, pk, tvh, wqh, t); break;
                case 1: quad_top<N, 1, 2>(blk, pk, tvh, wqh, t); break;
                case 2: quad_top<N, 2, 2>(blk, pk, tvh, wqh, t); break;
                default: quad_top<N, 3, 2>(blk, pk, tvh, wqh, t); break;
            }
        }
        __syncthreads();  // twiddle table, every exchange block filled
        cx *xb = reinterpret_cast<cx *>(lds) + wave * SubFft::XL;
#pragma unroll
        for (int b = 0; b < 16; b++) {
            const double2 y = reinterpret_cast<const double2 *>(xb)[lane + 64 * b];
            v[b] = cx{y.x, y.y};
        }
        wsync();
        if (!(MB2_TSKIP & 2)) SubFft::forward(v, xb, tw, lane, wsync);
    } else {
        const double2 *src = spectra(c1) + (size_t)p1 * M + 1024 * q + lane;
#pragma unroll
        for (int b = 0; b < 16; b++) v[b] = gld(src + 64 * b);
        __syncthreads();  // twiddle table
        cx *xb = reinterpret_cast<cx *>(lds) + wave * SubFft::XL;
        if (!(MB2_TSKIP & 2)) SubFft::forward(v, xb, tw, lane, wsync);
    }
    // monomial degrees of each ciphertext's 2^g - 1 non-constant GGSWs (wave-uniform)
    uint32_t deg[CPW][NSEL];
#pragma unroll
    for (int c = 0; c < CPW; c++) {
        const uint64_t *in = a.lwe_in + (size_t)(ct0 + ct_of(c)) * (a.n + 1) + (size_t)i * G;
#pragma unroll
        for (int sel = 1; sel < NSEL; sel++) {
            uint64_t d = 0;
#pragma unroll
            for (int b = 0; b < G; b++)
                if ((sel >> (G - 1 - b)) & 1) d += in[b];
            deg[c][sel] = pbs_modulus_switch<S::LOGN>(d);
        }
    }
    __syncthreads();  // every wave's exchange block is free: the region becomes twist | half buffer
    Tw::fill(reinterpret_cast<double *>(lds + Cfg::TWIST), a.twist, threadIdx.x, Cfg::THREADS);
    double2 *half = lds + Cfg::HALF;
    auto hslot = [&](int c, int p, int sl) { return half + ((c * PW + p) * 8 + sl) * 64 + lane; };

    constexpr size_t ggsw_len = (size_t)L * (K + 1) * (K + 1) * M;
    constexpr uint32_t rowb = 16u * (uint32_t)((K + 1) * M);
    const __amdgpu_buffer_rsrc_t grs = make_rsrc(a.fbsk + (size_t)i * NSEL * ggsw_len);
    const uint32_t gvo = 16u * (uint32_t)(1024 * q + lane);
    // t = d (1 - 4 f) mod 2N with f = fl + R freq_slot(s): per lane and ciphertext-selector the
    // slot-independent part, t(s) = tl - 4 d R freq_slot(s)  (mod 2^32; the low bits are exact)
    const uint32_t fl = (uint32_t)q + (uint32_t)R * SubFft::freq_lane(lane);
    cx o[2][CPW][K + 1];  // MAC outputs of the wave's slot in round 0 and round 1

#pragma unroll
    for (int h = 0; h < 2; h++) {
        // ---- publish slots 8h .. 8h + 7 of this wave's spectrum ----
#pragma unroll
        for (int sl = 0; sl < 8; sl++) *hslot(c1, p1, sl) = make_double2(v[8 * h + sl].re, v[8 * h + sl].im);
        const int s = 8 * h + ws;  // this wave's slot in round h (wave-uniform)
#if MB2_PIPE
        // the round's 8 operand batches (level, column, row) of 2^g GGSW values each, software
        // pipelined: batch k + 1 in flight while batch k is consumed (the same registers as one
        // (level, column) batch); batch 0 is issued before the barrier
        auto gload = [&](int st, double2 (&g)[NSEL]) {
            const int lv = L - (st >> 2), cl = (st >> 1) & 1, rr = st & 1;
#pragma unroll
            for (int sel = 0; sel < NSEL; sel++)
                g[sel] = (MB2_TSKIP & 1) ? make_double2(1.0 + sel, 0.5 * rr)
                                         : buffer_ld_d2(grs, gvo, (uint32_t)(16u * sel * ggsw_len) +
                                                                      (uint32_t)((lv - 1) * (K + 1) + rr) * rowb +
                                                                      16u * (uint32_t)(cl * M) + 1024u * (uint32_t)s);
        };
        constexpr int NB = MB2_DEPTH + 1;  // operand batches in flight + the one consumed
        double2 gb[NB][NSEL];
#pragma unroll
        for (int st = 0; st < MB2_DEPTH; st++) gload(st, gb[st]);
#endif
        __syncthreads();  // (h = 0: also the twist planes)
        const uint32_t f = fl + (uint32_t)R * SubFft::freq_slot(s);
        cx mono[CPW][NSEL];
#pragma unroll
        for (int c = 0; c < CPW; c++)
#pragma unroll
            for (int sel = 1; sel < NSEL; sel++) mono[c][sel] = Tw::mono(deg[c][sel] - 4u * deg[c][sel] * f);
#if MB2_PIPE
        cx ff[CPW][K + 1];
#pragma unroll
        for (int st = 0; st < 8; st++) {
            const int lvl = L - (st >> 2), col = (st >> 1) & 1, r = st & 1;
            __builtin_amdgcn_sched_barrier(0);
            if (st + MB2_DEPTH < 8) gload(st + MB2_DEPTH, gb[(st + MB2_DEPTH) % NB]);
            if (st % 4 == 0) {
#pragma unroll
                for (int c = 0; c < CPW; c++)
#pragma unroll
                    for (int rr = 0; rr <= K; rr++) {
                        const double2 t = *hslot(c, (lvl - 1) * (K + 1) + rr, ws);
                        ff[c][rr] = cx{t.x, t.y};
                    }
            }
            const double2 (&g)[NSEL] = gb[st % NB];
#pragma unroll
            for (int c = 0; c < CPW; c++) {
                double2 kb = g[0];
#pragma unroll
                for (int sel = 1; sel < ((MB2_TSKIP & 8) ? 1 : NSEL); sel++) {
                    kb.x = fma(g[sel].x, mono[c][sel].re, fma(-g[sel].y, mono[c][sel].im, kb.x));
                    kb.y = fma(g[sel].x, mono[c][sel].im, fma(g[sel].y, mono[c][sel].re, kb.y));
                }
                cx &oc = o[h][c][col];
                if (lvl == L && r == 0) {
                    oc.re = fma(kb.x, ff[c][r].re, -(kb.y * ff[c][r].im));
                    oc.im = fma(kb.x, ff[c][r].im, kb.y * ff[c][r].re);
                } else {
                    oc.re = fma(kb.x, ff[c][r].re, fma(-kb.y, ff[c][r].im, oc.re));
                    oc.im = fma(kb.x, ff[c][r].im, fma(kb.y, ff[c][r].re, oc.im));
                }
            }
        }
#else
#pragma unroll
        for (int lvl = L; lvl >= 1; lvl--) {
            cx ff[CPW][K + 1];
#pragma unroll
            for (int c = 0; c < CPW; c++)
#pragma unroll
                for (int r = 0; r <= K; r++) {
                    const double2 t = *hslot(c, (lvl - 1) * (K + 1) + r, ws);
                    ff[c][r] = cx{t.x, t.y};
                }
#pragma unroll
            for (int col = 0; col <= K; col++) {
                __builtin_amdgcn_sched_barrier(0);  // one (level, column) operand batch in flight
                double2 g[K + 1][NSEL];
#pragma unroll
                for (int r = 0; r <= K; r++)
#pragma unroll
                    for (int sel = 0; sel < NSEL; sel++)
                        g[r][sel] = (MB2_TSKIP & 1) ? make_double2(1.0 + sel, 0.5 * r) : buffer_ld_d2(grs, gvo,
                                                 (uint32_t)(16u * sel * ggsw_len) + (uint32_t)((lvl - 1) * (K + 1) + r) * rowb +
                                                     16u * (uint32_t)(col * M) + 1024u * (uint32_t)s);
#pragma unroll
                for (int c = 0; c < CPW; c++) {
#pragma unroll
                    for (int r = 0; r <= K; r++) {
                        double2 kb = g[r][0];
#pragma unroll
                        for (int sel = 1; sel < ((MB2_TSKIP & 8) ? 1 : NSEL); sel++) {
                            kb.x = fma(g[r][sel].x, mono[c][sel].re, fma(-g[r][sel].y, mono[c][sel].im, kb.x));
                            kb.y = fma(g[r][sel].x, mono[c][sel].im, fma(g[r][sel].y, mono[c][sel].re, kb.y));
                        }
                        cx &oc = o[h][c][col];
                        if (lvl == L && r == 0) {
                            oc.re = fma(kb.x, ff[c][r].re, -(kb.y * ff[c][r].im));
                            oc.im = fma(kb.x, ff[c][r].im, kb.y * ff[c][r].re);
                        } else {
                            oc.re = fma(kb.x, ff[c][r].re, fma(-kb.y, ff[c][r].im, oc.re));
                            oc.im = fma(kb.x, ff[c][r].im, fma(kb.y, ff[c][r].re, oc.im));
                        }
                    }
                }
            }
        }
#endif
        __syncthreads();  // every wave has read round h's half buffer
    }
    // ---- phase 3: outputs -> the half buffer as [c][col][16 slots][64], inverse sub-FFTs ----
    auto oslot = [&](int c, int col, int sl) { return half + ((c * (K + 1) + col) * 16 + sl) * 64 + lane; };
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int c = 0; c < CPW; c++)
#pragma unroll
            for (int col = 0; col <= K; col++)
                *oslot(c, col, 8 * h + ws) = make_double2(o[h][c][col].re, o[h][c][col].im);
    __syncthreads();
    if (wave >= CPW * (K + 1)) return;
    const int c = wave / (K + 1), col = wave % (K + 1);
#pragma unroll
    for (int sl = 0; sl < 16; sl++) {
        const double2 t = *oslot(c, col, sl);
        v[sl] = cx{t.x, t.y};
    }
    cx *xb = reinterpret_cast<cx *>(oslot(c, col, 0) - lane);  // this column's 16 KiB: its exchange block
    wsync();
    if (!(MB2_TSKIP & 4)) SubFft::inverse(v, xb, tw, lane, wsync);
    if (2 * cp + c >= cnt) return;
    double2 *dst = spectra(c) + (size_t)col * M + 1024 * q + lane;  // (lvl 1, row col) slot: this WG only
    store_sub_out<LARGE_SUB_AUX>(dst, v, lane);
}

// TFHE_MI355_MB_DIGITS=0: the multi-bit pair kernel reads f64 spectra from large_top_fwd /
// large_mb_inv_fwd instead of packed digits (A/B)
// Chunks below TFHE_MI355_MB_DIGITS_MIN ciphertexts keep the spectra path: there the inverse kernel is
// not bandwidth-bound and the pair kernel's top DIF sits on the critical path of every group
static bool mb_digits_enabled(int cnt) {
    static const int v = [] {
        const char *e = std::getenv("TFHE_MI355_MB_DIGITS");
        if (e && e[0] == '0') return -1;
        const char *m = std::getenv("TFHE_MI355_MB_DIGITS_MIN");
        return m ? std::atoi(m) : MB_DIGITS_MIN;
    }();
    return v >= 0 && cnt >= v;
}

static bool mb_pair2_enabled() {
    static const bool v = [] {
        const char *e = std::getenv("TFHE_MI355_MB_PAIR2");
        return !(e && e[0] == '0');
    }();
    return v;
}

// ---------------------------------------------------------------------------------------
// Grouped CMUX (k = 1, L = 2).  The top DIF radix-16 is R4 over stride 4, twiddles
// omega_16^{A c}, R4 (dft16_fwd): its outputs c = G, G+4, G+8, G+12 come from ONE second-layer
// R4, which needs only output G of each first-layer R4.  So a workgroup per (ciphertext, group G,
// part) builds KW of the group's sub-blocks straight from the CMUX's packed digits (twist + its
// share of every radix-16 butterfly), and no f64 spectra cross a launch boundary.  Per CMUX:
//   large_digits_kernel     rotation + both decomposition levels -> packed int16 digits, both rows
//                           of a position in one 16-byte word
//   large_group_cmux_kernel per (ct, G, part), 2 KW waves = level li x sub-block s = G + 4 k:
//     1. per half h of the butterflies a: digits -> twist -> the group's radix-16 share for both
//        rows and levels -> top twiddle W[a c] -> LDS [w][row][a - 512 h]; wave w picks up slots
//        8h..8h+7 of both rows (WaveFft<1024> natural layout);
//     2. wave w: forward sub-FFTs of both rows (spectra in registers);
//     3. MAC split by slots: wave (li, k) computes both columns for slots 8 li .. 8 li + 7, rows and
//        levels in the oracle's order; the partner level's spectra and the column halves go
//        through the pair's own exchange blocks, ordered by pair flags (no workgroup barrier);
//     4. wave (li, k): inverse sub-FFT of column 1 - li -> U[col][1024 s + position].
//   large_top_inv_kernel    top DIT radix-16, backward conversion, accumulator update.
// The operations are the oracle's, in its order, so the outputs stay bit-exact.  LDS: 2 KW blocks
// of 16 KiB (phase-1 staging, per-wave FFT exchange, MAC exchange) + the sub-FFT twiddle table.
// KW = 4: 512 threads, 143 KiB, one workgroup per CU; KW = 2: 256 threads, 79 KiB, two per CU
// (the digits are read by twice as many workgroups; measured slower: 1016 vs 1116 KS+PBS/s).
// ---------------------------------------------------------------------------------------
#ifndef LARGE_GROUP_SUB
#define LARGE_GROUP_SUB 1
#endif
#ifndef LARGE_GROUP_KW
#define LARGE_GROUP_KW 4  // sub-blocks per level per group workgroup (4: all of group G; 2: half)
#endif

// output G of r4_fwd(x0, x1, x2, x3), same expressions
template <int G>
__device__ __forceinline__ cx r4_out(cx x0, cx x1, cx x2, cx x3) {
    if constexpr (G == 0 || G == 2) {
        const cx t0 = cadd(x0, x2), t2 = cadd(x1, x3);
        return G == 0 ? cadd(t0, t2) : csub(t0, t2);
    } else {
        const cx t1 = csub(x0, x2), t3 = csub(x1, x3);
        return G == 1 ? cx{t1.re + t3.im, t1.im - t3.re} : cx{t1.re - t3.im, t1.im + t3.re};
    }
}

// Wave of (level li, sub-block k) in a group workgroup.  1: w = 2k + li -- the two waves of a
// pair (which sync with each other in the MAC) are adjacent, so they run on different SIMDs and
// each SIMD holds waves of two different pairs; 0: w = li KW + k (the pair on one SIMD).
#ifndef LARGE_TSKIP
#define LARGE_TSKIP 0  // timing-only builds (wrong outputs): 1 no phase 1, 2 no GGSW loads, 4 no U stores
#endif
#ifndef LARGE_ACC_AUX
#define LARGE_ACC_AUX 0  // cache policy of top_inv's accumulator stores (16 = sc1)
#endif
#ifndef LARGE_GRP_WMAP
#define LARGE_GRP_WMAP 1
#endif
#ifndef LARGE_GRP_QROT
#define LARGE_GRP_QROT 1  // group kernel: wave pair -> sub-block rotated per ciphertext (0: pair k on G + 4k)
#endif
template <int KW>
__device__ __forceinline__ constexpr int grp_wave(int li, int k) { return LARGE_GRP_WMAP ? 2 * k + li : li * KW + k; }

template <int KW>
struct LargeGroupCfg {
    static_assert(KW == 2 || KW == 4, "2 or 4 sub-blocks per level per workgroup");
    static constexpr int WAVES = 2 * KW;
    static constexpr int THREADS = 64 * WAVES;
    static constexpr int PARTS = 4 / KW;     // workgroups per (ciphertext, group)
    static constexpr int REGION = WAVES * 1024;  // double2 entries: one 16 KiB block per wave
    static constexpr int FLAGS = REGION + SubFft::Lds::s1_len;  // double2 offset of the pair-sync flags
    static constexpr size_t LDS = sizeof(double2) * FLAGS + 8 * KW;  // + one 8-byte flag pair per k
};

__device__ __forceinline__ uint64_t buffer_ld_u64(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    typedef unsigned v2u __attribute__((ext_vector_type(2)));
    const v2u t = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    return ((uint64_t)t.y << 32) | t.x;
}

// Packed digits of one position pair (j, j + M) of a row: int16 fields (level L at j, level L at
// j + M, level L-1 at j, level L-1 at j + M); |digit| <= 2^(beta-1) = 2^14.  They live in the
// chunk's spectra scratch behind U: [ct][poly 2..3 region] as [j][row] u64 -- both rows of a
// position in one 16-byte word, written by one store and read by one phase-1 load (the [row][j]
// layout with 8-byte loads measured 1152 vs 1203 KS+PBS/s).
__device__ __forceinline__ uint64_t *group_digits(const LargePbsLaunch &a, int cl) {
    return reinterpret_cast<uint64_t *>(a.spectra + ((size_t)cl * 2 * 2 + 2) * LM);
}

// Phase 1 step = (row r, column A) of butterfly ap: the inputs b = A + 4m (m = 0..3).  All of a
// step's loads are issued together and the next step's before this one's arithmetic (a
// sched_barrier after each load group), so ~20 loads per wave are in flight.
struct GroupDg {
    uint64_t dg[4];
    cx tv[4];  // twist at a + 1024 b
};
template <int A>
__device__ __forceinline__ void group_load_dg(GroupDg &d, __amdgpu_buffer_rsrc_t dig, __amdgpu_buffer_rsrc_t twist,
                                              int ap, int r) {
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const int b = A + 4 * m;
        d.dg[m] = buffer_ld_u64(dig, 16u * ap, 16u * 1024u * b + 8u * r);
        const double2 t = buffer_ld_d2(twist, 16u * ap, 16u * 1024u * b);
        d.tv[m] = cx{t.x, t.y};
    }
}
// twist of both levels' digits, first-layer R4 output G of column A, omega_16^{A G}
template <int A, int G>
__device__ __forceinline__ void group_compute_dg(const GroupDg &d, cx (&y)[2][4]) {
    cx z[2][4];  // [li][m]
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const uint64_t w = d.dg[m];
        const double g0 = (double)(int16_t)(w & 0xffffu), g1 = (double)(int16_t)((w >> 16) & 0xffffu);
        const double l0 = (double)(int16_t)((w >> 32) & 0xffffu), l1 = (double)(int16_t)(w >> 48);
        z[0][m] = cmulw(cx{g0, g1}, d.tv[m].re, d.tv[m].im);
        z[1][m] = cmulw(cx{l0, l1}, d.tv[m].re, d.tv[m].im);
    }
#pragma unroll
    for (int l = 0; l < 2; l++) y[l][A] = tw16_fwd<A * G>(r4_out<G>(z[l][0], z[l][1], z[l][2], z[l][3]));
}

// phase 1 for butterfly ap of half h: both rows -> LDS staging [w][row][ap - 512 h]
#ifndef LARGE_GRP_TW_SHARED
#define LARGE_GRP_TW_SHARED 1  // 1: a phase-1 step is a column A for both rows (twist loaded once per a, not per row)
#endif
// both rows of column A: the twist is shared
struct GroupDg2 {
    uint64_t dg[2][4];
    cx tv[4];
};
template <int A>
__device__ __forceinline__ void group_load_dg2(GroupDg2 &d, __amdgpu_buffer_rsrc_t dig, __amdgpu_buffer_rsrc_t twist,
                                               int ap) {
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const int b = A + 4 * m;
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v4u q = __builtin_amdgcn_raw_buffer_load_b128(dig, 16u * ap, 16u * 1024u * b, 0);
        d.dg[0][m] = ((uint64_t)q.y << 32) | q.x;
        d.dg[1][m] = ((uint64_t)q.w << 32) | q.z;
        const double2 t = buffer_ld_d2(twist, 16u * ap, 16u * 1024u * b);
        d.tv[m] = cx{t.x, t.y};
    }
}
template <int A, int G>
__device__ __forceinline__ void group_compute_dg2(const GroupDg2 &d, cx (&y)[2][2][4]) {
#pragma unroll
    for (int r = 0; r < 2; r++) {
        GroupDg e;
#pragma unroll
        for (int m = 0; m < 4; m++) {
            e.dg[m] = d.dg[r][m];
            e.tv[m] = d.tv[m];
        }
        group_compute_dg<A, G>(e, y[r]);
    }
}

template <int KW, int G>
__device__ __forceinline__ void group_phase1(const LargePbsLaunch &a, int cl, int part, int ap, int h, double2 *lds,
                                             int rot) {
    const __amdgpu_buffer_rsrc_t rdig = make_rsrc(group_digits(a, cl)), rtw = make_rsrc(a.twist);
#if LARGE_GRP_TW_SHARED
    cx yy[2][2][4];  // [row][li][A]
    {
        GroupDg2 e0, e1;
        group_load_dg2<0>(e0, rdig, rtw, ap);
        __builtin_amdgcn_sched_barrier(0);
        group_load_dg2<1>(e1, rdig, rtw, ap);
        __builtin_amdgcn_sched_barrier(0);  // issue the step's loads here, not at their uses
        group_compute_dg2<0, G>(e0, yy);
        group_load_dg2<2>(e0, rdig, rtw, ap);
        __builtin_amdgcn_sched_barrier(0);
        group_compute_dg2<1, G>(e1, yy);
        group_load_dg2<3>(e1, rdig, rtw, ap);
        __builtin_amdgcn_sched_barrier(0);
        group_compute_dg2<2, G>(e0, yy);
        group_compute_dg2<3, G>(e1, yy);
    }
#pragma unroll
    for (int r = 0; r < 2; r++) {
        cx (&y)[2][4] = yy[r];
#else
    GroupDg e0, e1;
    group_load_dg<0>(e0, rdig, rtw, ap, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < 2; r++) {
        cx y[2][4];  // [li][A]: first-layer outputs, then X[G + 4k]
        group_load_dg<1>(e1, rdig, rtw, ap, r);
        __builtin_amdgcn_sched_barrier(0);  // issue the step's loads here, not at their uses
        group_compute_dg<0, G>(e0, y);
        group_load_dg<2>(e0, rdig, rtw, ap, r);
        __builtin_amdgcn_sched_barrier(0);
        group_compute_dg<1, G>(e1, y);
        group_load_dg<3>(e1, rdig, rtw, ap, r);
        __builtin_amdgcn_sched_barrier(0);
        group_compute_dg<2, G>(e0, y);
        if (r == 0) group_load_dg<0>(e0, rdig, rtw, ap, 1);  // next row's first step
        __builtin_amdgcn_sched_barrier(0);
        group_compute_dg<3, G>(e1, y);
#endif
        cx wt[KW];
#pragma unroll
        for (int k = 0; k < KW; k++) {
            const int c = G + 4 * (KW * part + k);
            wt[k] = c ? gld(a.wtop + (c - 1) * 1024 + ap) : cx{1.0, 0.0};  // = W[a c]
        }
#pragma unroll
        for (int l = 0; l < 2; l++) {
            r4_fwd(y[l][0], y[l][1], y[l][2], y[l][3]);  // y[l][k] = X[G + 4k]
#pragma unroll
            for (int k = 0; k < KW; k++) {
                const int kg = KW * part + k;  // uniform: part is per workgroup
                const cx x = KW == 4 ? y[l][k] : (part ? y[l][2 + k] : y[l][k]);
                const cx v = (G + 4 * kg) ? cmulw(x, wt[k].re, wt[k].im) : x;
                // sub-block k goes to wave pair (k - rot) mod KW (LARGE_GRP_QROT)
                lds[(grp_wave<KW>(l, (k - rot) & (KW - 1)) * 2 + r) * 512 + (ap - 512 * h)] = make_double2(v.re, v.im);
            }
        }
    }
}

// Slot-split MAC with the exchange in the pair's own two exchange blocks, ordered by the pair's
// LDS flags (GroupSync<2>): wave (LI, k) writes the half of its spectra that the partner needs into
// its own block, the pair syncs, each reads the other's block; then the same for the column
// halves.  The four pairs of a workgroup drift independently (no workgroup barrier).
template <int KW, int LI>
__device__ __forceinline__ void group_mac_pair(cx (&f)[2][16], cx (&v)[16], double2 *lds, int lane, int k,
                                               const double2 *Gb, GroupSync<2> &ps) {
    constexpr int K = 1, L = 2;
    double2 *own = lds + grp_wave<KW>(LI, k) * 1024 + lane;          // this wave's block
    const double2 *oth = lds + grp_wave<KW>(1 - LI, k) * 1024 + lane;  // the partner's block
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
        for (int sp = 0; sp < 8; sp++) {
            const cx t = f[r][8 * (1 - LI) + sp];
            own[r * 512 + sp * 64] = make_double2(t.re, t.im);
        }
    ps();  // both halves published
    cx o[2][8];
#pragma unroll
    for (int sp = 0; sp < 8; sp++) {
        __builtin_amdgcn_sched_barrier(0);  // bound loads in flight
        const int s = 8 * LI + sp;
        cx fl[2], fm[2];  // level L / level L-1 spectra of rows 0, 1 at slot s
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const cx mine = f[r][8 * LI + sp];
            const cx other = gld(oth + r * 512 + sp * 64);
            fl[r] = LI ? other : mine;
            fm[r] = LI ? mine : other;
        }
#pragma unroll
        for (int c = 0; c < 2; c++) {
            // ggsw.rs:524-567: p = (lvl - 1)(k + 1) + r, lvl = L..1, r = 0..k; GGSW poly p (k+1) + c
#if LARGE_TSKIP & 2  // timing only: no GGSW loads
            const double2 g0 = make_double2(1.0 + lane, 2.0), g1 = make_double2(3.0, 1.0 + c), g2 = make_double2(sp, 0.5), g3 = g0;
#else
            const double2 g0 = Gb[(size_t)((L - 1) * (K + 1) * (K + 1) + c) * LM + s * 64];
            const double2 g1 = Gb[(size_t)(((L - 1) * (K + 1) + 1) * (K + 1) + c) * LM + s * 64];
            const double2 g2 = Gb[(size_t)c * LM + s * 64];
            const double2 g3 = Gb[(size_t)((K + 1) + c) * LM + s * 64];
#endif
            cx t;
            t.re = fma(g0.x, fl[0].re, -(g0.y * fl[0].im));
            t.im = fma(g0.x, fl[0].im, g0.y * fl[0].re);
            t.re = fma(g1.x, fl[1].re, fma(-g1.y, fl[1].im, t.re));
            t.im = fma(g1.x, fl[1].im, fma(g1.y, fl[1].re, t.im));
            t.re = fma(g2.x, fm[0].re, fma(-g2.y, fm[0].im, t.re));
            t.im = fma(g2.x, fm[0].im, fma(g2.y, fm[0].re, t.im));
            t.re = fma(g3.x, fm[1].re, fma(-g3.y, fm[1].im, t.re));
            t.im = fma(g3.x, fm[1].im, fma(g3.y, fm[1].re, t.im));
            o[c][sp] = t;
        }
    }
    ps();  // both have read the other's spectra: the blocks are free for the column halves
    // column 1 - LI is this wave's inverse; the partner gets column LI of this half
#pragma unroll
    for (int sp = 0; sp < 8; sp++) own[sp * 64] = make_double2(o[LI][sp].re, o[LI][sp].im);
    ps();
#pragma unroll
    for (int sp = 0; sp < 8; sp++) {
        v[8 * LI + sp] = o[1 - LI][sp];
        v[8 * (1 - LI) + sp] = gld(oth + sp * 64);
    }
    ps();  // the partner has read this block: it is this wave's FFT exchange buffer again
}

template <int KW, int G>
__device__ __forceinline__ void group_cmux_body(const LargePbsLaunch &a, int i, int cl, int part, double2 *lds, int rot) {
    constexpr int K = 1, L = 2;
    using Cfg = LargeGroupCfg<KW>;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = LARGE_GRP_WMAP ? wave & 1 : wave / KW, k = LARGE_GRP_WMAP ? wave >> 1 : wave % KW;
    const int sblk = G + 4 * (KW * part + ((k + rot) & (KW - 1)));  // wave pair k runs sub-block k + rot
    double2 *s1 = lds + Cfg::REGION;
    // sub-block stage twiddles W_1024[lane c] = W_M[16 lane c]  (oracle dif_rec tstride 16)
    for (int e = tid; e < SubFft::Lds::s1_len; e += Cfg::THREADS) s1[e] = a.W[16 * (e & 63) * ((e >> 6) + 1)];
    if (tid < 2 * KW) reinterpret_cast<uint32_t *>(lds + Cfg::FLAGS)[tid] = 0;  // pair-sync flags
    const SubFft::Lds tw{s1, s1};
    cx *xb = reinterpret_cast<cx *>(lds) + wave * 1024;
    WaveLocalSync wsync;

    cx f[2][16];  // per row: this wave's sub-block input (natural layout), then its spectrum
#pragma unroll
    for (int h = 0; h < 2; h++) {
        if (h) __syncthreads();  // every wave has picked up half 0
#pragma unroll
        for (int q = 0; q < 512 / Cfg::THREADS; q++)
            if (!(LARGE_TSKIP & 1)) group_phase1<KW, G>(a, cl, part, 512 * h + Cfg::THREADS * q + tid, h, lds, rot);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int b = 0; b < 8; b++) f[r][8 * h + b] = gld(lds + (wave * 2 + r) * 512 + lane + 64 * b);
    }
    __syncthreads();  // the region now serves as the per-wave exchange buffers
#pragma unroll
    for (int r = 0; r < 2; r++) SubFft::forward(f[r], xb, tw, lane, wsync);

    const double2 *Gb = a.fbsk + (size_t)i * L * (K + 1) * (K + 1) * LM + 1024 * sblk + lane;
    cx v[16];
    // pair flags instead of workgroup barriers (A/B with two barriers around a region-wide
    // exchange: 64.4 -> 61.4 us per chunk)
    GroupSync<2> ps;
    ps.mine = lds_addr(lds + Cfg::FLAGS) + 8u * k + 4u * li;
    if (li) group_mac_pair<KW, 1>(f, v, lds, lane, k, Gb, ps);
    else group_mac_pair<KW, 0>(f, v, lds, lane, k, Gb, ps);
    SubFft::inverse(v, xb, tw, lane, wsync);
    const int col = 1 - li;
    double2 *dst = a.spectra + ((size_t)cl * L * (K + 1) + col) * LM + 1024 * sblk + lane;
    if (!(LARGE_TSKIP & 4) || a.n == 12345) store_sub_out<LARGE_U_AUX>(dst, v, lane);
}

// rotation + decomposition of CMUX i for the grouped path at positions j and j + M of row r
__device__ __forceinline__ uint64_t group_digit_word(const LargePbsLaunch &a, int cl, int r, int j, bool full_odd,
                                                     int rem) {
    constexpr int L = 2;
    const int beta = a.base_log;
    const uint32_t dmask = (1u << beta) - 1;
    const uint64_t *acc = a.acc + ((size_t)cl * 2 + r) * LN;
    uint64_t w = 0, dd[2];
    ct1_pair(acc, j, rem, full_odd, dd[0], dd[1]);  // ct1 = X^{a~} acc - acc
    if (LARGE_DIGIT2) {  // Digit2 (pbs_common.h): the same int16 words in 9 VALU per value
        uint32_t lv0, lv1;
        Digit2(beta).pair((uint32_t)(dd[0] >> 32), (uint32_t)(dd[1] >> 32), lv0, lv1);
        return (uint64_t)lv0 | ((uint64_t)lv1 << 32);
    }
#pragma unroll
    for (int half = 0; half < 2; half++) {
        const uint64_t d = dd[half];
        uint32_t st = decomp_state32_hi<L>((uint32_t)(d >> 32), beta);
        const int32_t dg = decomp_digit32(st, beta, dmask);  // level L
        const int32_t dl = decomp_digit32(st, beta, dmask);  // level L-1
        w |= ((uint64_t)((uint32_t)dg & 0xffffu) << (16 * half)) | ((uint64_t)((uint32_t)dl & 0xffffu) << (32 + 16 * half));
    }
    return w;
}

// digits of CMUX i: one thread per (ciphertext, j < M), both rows in one 16-byte store
#ifndef LARGE_DIGT
#define LARGE_DIGT 256  // digits-kernel workgroup size
#endif
__global__ void __launch_bounds__(LARGE_DIGT) large_digits_kernel(LargePbsLaunch a, int ct0, int i) {
    constexpr int PER = LM / LARGE_DIGT;  // workgroups per ciphertext
    // XCD-aware: ciphertext cl on XCD group cl % 8, as its grouped-CMUX workgroups
    const int x = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int cl = x + 8 * (m / PER), sub = m % PER;
    if (cl >= a.chunk_count) return;
    const uint64_t *in = a.lwe_in + (size_t)(ct0 + cl) * (a.n + 1);
    const uint32_t at = pbs_modulus_switch<15>(in[i]);
    const bool full_odd = (at / LN) & 1;
    const int rem = at % LN;
    const int j = sub * LARGE_DIGT + threadIdx.x;
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    const u64x2 w = {group_digit_word(a, cl, 0, j, full_odd, rem), group_digit_word(a, cl, 1, j, full_odd, rem)};
    reinterpret_cast<u64x2 *>(group_digits(a, cl))[j] = w;
}

using GroupCfg = LargeGroupCfg<LARGE_GROUP_KW>;
__global__ void __launch_bounds__(GroupCfg::THREADS, 2) large_group_cmux_kernel(LargePbsLaunch a, int ct0, int i) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    constexpr int KW = LARGE_GROUP_KW, PARTS = GroupCfg::PARTS;
    // XCD-aware: the 4 PARTS workgroups of a ciphertext are blocks 8 m + x with the same x (one
    // XCD), so the digits they all read come from the Infinity Cache once
    const int x = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int cl = x + 8 * (m / (4 * PARTS));
    if (cl >= a.chunk_count) return;  // whole workgroup
    const int part = (m >> 2) % PARTS;
    (void)ct0;
    // wave pair -> sub-block rotated per ciphertext (LARGE_GRP_QROT, as ONCHIP_QROT)
    const int rot = (LARGE_GRP_QROT && KW == 4) ? (m >> 2) & 3 : 0;
    switch (m & 3) {
        case 0: group_cmux_body<KW, 0>(a, i, cl, part, lds, rot); break;
        case 1: group_cmux_body<KW, 1>(a, i, cl, part, lds, rot); break;
        case 2: group_cmux_body<KW, 2>(a, i, cl, part, lds, rot); break;
        default: group_cmux_body<KW, 3>(a, i, cl, part, lds, rot); break;
    }
}

// top DIT radix-R of butterfly t of column col, backward conversion, acc += increments (G > 0,
// multi-bit: acc = the external product, the reference's zeroed ping-pong destination)
template <int N, int K, int G = 0>
__device__ __forceinline__ void top_inv_body(const LargePbsLaunch &a, int cl, int col, int t) {
    using S = Split<N>;
    constexpr int R = S::R, M = S::M;
    const double2 *U = a.spectra + ((size_t)cl * a.levels * (K + 1) + col) * M + t;
    cx u[R];
    u[0] = gld(U);
#pragma unroll
    for (int c = 1; c < R; c++) {
        const cx w = gld(a.wtop + (c - 1) * 1024 + t);  // = W[t c]
        u[c] = cmulw(gld(U + 1024 * c), w.re, -w.im);
    }
    dftR_inv<R>(u);
    uint64_t *acc = a.acc + ((size_t)cl * (K + 1) + col) * N;
    const double k32 = torus_k32();
#pragma unroll
    for (int b = 0; b < R; b++) {
        const int j = t + 1024 * b;
        const cx w = gld(a.twist + j);
        acc_pair pr;
        uint64_t lo, hi;
        if constexpr (G > 0) {
            backward_convert(u[b], w, lo, hi, k32);
        } else {
            pr = *reinterpret_cast<const acc_pair *>(acc + 2 * j);
            lo = pr.x;
            hi = pr.y;
            backward_add(u[b], w, lo, hi, k32);  // the resident key carries the 1/M
        }
        if (LARGE_ACC_AUX) {
            const double2 w2 = make_double2(__longlong_as_double((long long)lo), __longlong_as_double((long long)hi));
            buffer_st_d2p<LARGE_ACC_AUX>(make_rsrc(acc), 16u * j, 0, w2);
        } else {
            pr.x = lo;
            pr.y = hi;
            *reinterpret_cast<acc_pair *>(acc + 2 * j) = pr;
        }
    }
}

// Multi-bit split CMUX (G > 0): large_top_inv of group i fused with large_top_fwd of group i + 1.
// Without a rotation (ct1 = acc) the new accumulator pair at positions j = t + 1024 b, b < R, that
// butterfly t of column r produces is exactly what butterfly t of row r decomposes next, so one
// thread runs both: top DIT radix-R of U, backward conversion (the reference's zeroed ping-pong
// destination, lwe_multi_bit_programmable_bootstrapping.rs:782-800), decompose64 of the pairs,
// twist, top DIF radix-R per level -> the next group's top-stage spectra.  The accumulator stays in
// registers: it is written to scratch only by the last group's plain large_top_inv (for the
// extraction).  Per ciphertext and group: 384 KiB (U in, spectra out) instead of 640 KiB (top_inv's
// accumulator write and top_fwd's read), and one launch fewer.  Same operations on the same values
// as the two kernels, so bit-identical.  TFHE_MI355_MB_FUSED=0: the separate launches (A/B).
template <int N, int K, int L, int G, bool DIG>
__global__ void __launch_bounds__(TOPT, (top_fwd_wpe<N, L>())) large_mb_inv_fwd_kernel(LargePbsLaunch a, int ct0, int i) {
    static_assert(G > 0, "multi-bit only (the classic CMUX rotates between the two)");
    using S = Split<N>;
    constexpr int R = S::R, M = S::M, BPP = 1024 / TOPT;
    const int x = blockIdx.x & 7, m = blockIdx.x >> 3;  // XCD-aware as large_top_fwd_kernel
    const int sub = m % ((K + 1) * BPP);
    const int cl = x + 8 * (m / ((K + 1) * BPP));
    if (cl >= a.chunk_count) return;  // whole workgroup
    (void)ct0;
    (void)i;
    const int r = sub / BPP, t = (sub % BPP) * TOPT + threadIdx.x;  // column r of group i = row r of i + 1
    // ---- large_top_inv of group i, column r, butterfly t ----
    const double2 *U = a.spectra + ((size_t)cl * L * (K + 1) + r) * M + t;
    cx wt[R], tw[R], u[R];
    wt[0] = cx{1.0, 0.0};
#pragma unroll
    for (int c = 1; c < R; c++) wt[c] = gld(a.wtop + (c - 1) * 1024 + t);  // = W[t c]
#pragma unroll
    for (int b = 0; b < R; b++) tw[b] = gld(a.twist + t + 1024 * b);
    u[0] = gld(U);
#pragma unroll
    for (int c = 1; c < R; c++) u[c] = cmulw(gld(U + 1024 * c), wt[c].re, -wt[c].im);
    dftR_inv<R>(u);
    const double k32 = torus_k32();
    uint64_t lo[R], hi[R];
#pragma unroll
    for (int b = 0; b < R; b++) backward_convert(u[b], tw[b], lo[b], hi[b], k32);
    if constexpr (DIG) {
        // MB2_DIGITS: group i + 1's packed digits; the pair kernel does the twist + top DIF
        static_assert(N == 8192 && K == 1 && L == 2, "pair kernel shape");
        const Digit2 dg2(a.base_log);
        uint64_t *dg = mb_digits<N>(a, cl) + (size_t)r * M;
#pragma unroll
        for (int b = 0; b < R; b++) {
            uint32_t lv0, lv1;
            dg2.pair((uint32_t)(lo[b] >> 32), (uint32_t)(hi[b] >> 32), lv0, lv1);
            dg[t + 1024 * b] = (uint64_t)lv0 | ((uint64_t)lv1 << 32);
        }
        return;
    }
    // ---- large_top_fwd of group i + 1, row r, butterfly t (top_fwd_body, G > 0) ----
    const int beta = a.base_log;
    uint64_t pk[L > 1 ? R : 1];
#pragma unroll
    for (int b = 0; b < R; b++) {
        int32_t d0[L], d1[L];
        decompose64<L>(lo[b], beta, d0);
        decompose64<L>(hi[b], beta, d1);
        if constexpr (L > 1) {
            uint64_t w = 0;
#pragma unroll
            for (int l = 1; l < L; l++)
                w |= ((uint64_t)((uint32_t)d0[l] & 0xffffu) << (32 * (l - 1))) |
                     ((uint64_t)((uint32_t)d1[l] & 0xffffu) << (32 * (l - 1) + 16));
            pk[b] = w;
        }
        u[b] = cmulw(cx{(double)d0[0], (double)d1[0]}, tw[b].re, tw[b].im);
    }
    auto top_and_store = [&](int lvl) {
        dftR_fwd<R>(u);
        double2 *T = a.spectra + (((size_t)cl * L + (lvl - 1)) * (K + 1) + r) * M;
        constexpr int AUX = LARGE_TOPF_AUX < 0 ? 16 : LARGE_TOPF_AUX;
        auto st = [&](int c, cx y) {
            const double2 v2 = make_double2(y.re, y.im);
            if (AUX) buffer_st_d2p<AUX>(make_rsrc(T), 16u * (t + 1024 * c), 0, v2);
            else T[t + 1024 * c] = v2;
        };
        st(0, u[0]);
#pragma unroll
        for (int c = 1; c < R; c++) st(c, cmulw(u[c], wt[c].re, wt[c].im));
    };
    top_and_store(L);
#pragma unroll
    for (int l = 1; l < L; l++) {
#pragma unroll
        for (int b = 0; b < R; b++) {
            const int32_t e0 = (int32_t)(int16_t)((pk[b] >> (32 * (l - 1))) & 0xffffu);
            const int32_t e1 = (int32_t)(int16_t)((pk[b] >> (32 * (l - 1) + 16)) & 0xffffu);
            u[b] = cmulw(cx{(double)e0, (double)e1}, tw[b].re, tw[b].im);
        }
        top_and_store(L - l);
    }
}

static bool mb_fused_enabled() {
    static const bool v = [] {
        const char *e = std::getenv("TFHE_MI355_MB_FUSED");
        return !(e && e[0] == '0');
    }();
    return v;
}

template <int N, int K, int G = 0>
__global__ void __launch_bounds__(TOPT) large_top_inv_kernel(LargePbsLaunch a, int ct0, int i) {
    constexpr int BPP = 1024 / TOPT;
    const int col = (blockIdx.x / BPP) % (K + 1);
    top_inv_body<N, K, G>(a, blockIdx.x / (BPP * (K + 1)), col, (blockIdx.x % BPP) * TOPT + threadIdx.x);
}

// Digits-fed CMUX (N = 4096 / 8192, L = 2): large_top_inv of CMUX i fused with split_digits of
// CMUX i + 1.  One 1024-thread workgroup per (ciphertext, row): thread t runs top_inv_body's
// butterfly t of column `row` (positions j = t + 1024 b), keeps the updated accumulator pairs in
// registers, writes them to HBM (the extraction and the final CMUX read them there) and to LDS (one
// row is M pairs, 32 / 64 KiB); after one barrier it gathers X^{a~_(i+1)} acc - acc at its own
// positions from LDS and writes the row's half of the next CMUX's digit words.  Saves
// split_digits' re-read of the accumulator from HBM (self + rotated pair per position) and one
// launch per CMUX.  Same operations as top_inv_body + split_digits_kernel, so bit-identical.
template <int N>
__global__ void __launch_bounds__(1024) split_inv_digits_kernel(LargePbsLaunch a, int ct0, int i) {
    using S = Split<N>;
    constexpr int K = 1, R = S::R, M = S::M;
    static_assert(M == 1024 * R, "one butterfly per thread");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    acc_pair *row_acc = reinterpret_cast<acc_pair *>(smem);
    // XCD-aware as split_digits / large_dsub: ciphertext cl on XCD cl % 8
    const int x = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int cl = x + 8 * (m >> 1), row = m & 1;
    if (cl >= a.chunk_count) return;  // whole workgroup
    const int t = threadIdx.x;
    // ---- top DIT radix-R of butterfly t of column `row`, backward conversion, acc += ----
    const double2 *U = a.spectra + ((size_t)cl * a.levels * (K + 1) + row) * M + t;
    cx u[R];
    u[0] = gld(U);
#pragma unroll
    for (int c = 1; c < R; c++) {
        const cx w = gld(a.wtop + (c - 1) * 1024 + t);  // = W[t c]
        u[c] = cmulw(gld(U + 1024 * c), w.re, -w.im);
    }
    dftR_inv<R>(u);
    uint64_t *acc = a.acc + ((size_t)cl * (K + 1) + row) * N;
    const double k32 = torus_k32();
    uint64_t lo[R], hi[R];
#pragma unroll
    for (int b = 0; b < R; b++) {
        const int j = t + 1024 * b;
        const cx w = gld(a.twist + j);
        const acc_pair pr = *reinterpret_cast<const acc_pair *>(acc + 2 * j);
        lo[b] = pr.x;
        hi[b] = pr.y;
        backward_add(u[b], w, lo[b], hi[b], k32);  // the resident key carries the 1/M
        const acc_pair nw = {lo[b], hi[b]};
        *reinterpret_cast<acc_pair *>(acc + 2 * j) = nw;
        row_acc[j] = nw;
    }
    __syncthreads();
    // ---- split_digits of CMUX i + 1 for this row ----
    const uint64_t *in = a.lwe_in + (size_t)(ct0 + cl) * (a.n + 1);
    const uint32_t at = pbs_modulus_switch<S::LOGN>(in[i + 1]);
    const bool full_odd = (at / N) & 1;
    const int rem = at % N;
    uint64_t *dig = reinterpret_cast<uint64_t *>(split_digits<N>(a, cl));
#pragma unroll
    for (int b = 0; b < R; b++) {
        const int j = t + 1024 * b;
        // ct1_pair_m with the self pair from registers and the rotated one from LDS
        const int jj0 = j - rem;  // in (-N, M)
        const acc_pair rot = row_acc[jj0 & (M - 1)];
        const bool swap = jj0 < 0 && jj0 >= -M;
        const uint64_t x0 = swap ? rot.y : rot.x, x1 = swap ? rot.x : rot.y;
        const bool neg0 = (jj0 < 0) != full_odd, neg1 = (jj0 + M < 0) != full_odd;
        const uint64_t d0 = (neg0 ? 0 - x0 : x0) - lo[b];
        const uint64_t d1 = (neg1 ? 0 - x1 : x1) - hi[b];
        if (LARGE_DIGIT2 && a.base_log * 2 <= 30) {  // Digit2: the same words, 32-bit
            uint32_t lv0, lv1;
            Digit2(a.base_log).pair((uint32_t)(d0 >> 32), (uint32_t)(d1 >> 32), lv0, lv1);
            dig[2 * j + row] = (uint64_t)lv0 | ((uint64_t)lv1 << 32);
            continue;
        }
        int32_t e0[2], e1[2];
        decompose64<2>(d0, a.base_log, e0);
        decompose64<2>(d1, a.base_log, e1);
        dig[2 * j + row] = ((uint64_t)((uint32_t)e0[0] & 0xffffu)) | ((uint64_t)((uint32_t)e1[0] & 0xffffu) << 16) |
                           ((uint64_t)((uint32_t)e0[1] & 0xffffu) << 32) | ((uint64_t)((uint32_t)e1[1] & 0xffffu) << 48);
    }
}

// ---------------------------------------------------------------------------------------
// On-chip CMUX (N = 8192, k = 1, L = 2, classic).  One 512-thread workgroup per
// ciphertext runs the WHOLE blind rotation: the accumulator (2 rows x 8192 u64 = 128 KiB) lives in
// registers (thread t owns the pairs (j, j + M), j = t + 512 h + 1024 b, h < 2, b < 4, of both
// rows: 64 VGPRs) and every intermediate in the 128 KiB LDS region -- no accumulator, digit or
// spectrum traffic to HBM, one launch per batch instead of 2 per CMUX.  Per CMUX:
//   rotation   : both rows' pairs -> LDS, ct1 = X^{a~} acc - acc gathered (ct1_pair_m's rules),
//                decompose64<2>, 4 int16 digits per (row, pair) kept in registers
//   level L, then level L-1 (the MAC's order):
//     top      : every thread: twist, top DIF radix-4 of its butterflies of both rows, output c
//                times W[a c] -> wave buffer (2 c + row) at a (natural layout)
//     sub-FFT  : wave (q, row) = buffer 2 q + row: WaveFft<1024>::forward, spectrum published in
//                place
//     MAC      : wave (q, col = its row index) adds G[lvl][0][col] F_0 + G[lvl][1][col] F_1 of
//                sub-block q (F_own from registers, F_partner from the partner's buffer) into o
//   inverse    : wave (q, col): WaveFft<1024>::inverse(o) -> its buffer (natural layout)
//   top inverse: every thread: top DIT radix-4 of its butterflies of both columns, backward_add
//                into the registers
// Then the sample extraction from registers (through LDS).  The same operations in the same order
// as large_top_fwd + large_sub_kernel + large_top_inv (and the digits-fed path), so the outputs
// are bit-identical.  LDS: 8 x 16 KiB wave buffers (= the rotation's 2 x M pairs) + the sub-block
// twiddle table: 143 KiB, one workgroup (8 waves, 2 per SIMD) per CU.
// TFHE_MI355_ONCHIP=0: the digits-fed split CMUX instead (A/B).
// ---------------------------------------------------------------------------------------
#ifndef ONCHIP_TSKIP
#define ONCHIP_TSKIP 0  // timing-only builds (wrong outputs): 1 no GGSW loads, 2 no forward sub-FFTs,
                        // 4 no inverse sub-FFTs, 8 no top-stage arithmetic, 16 no rotation gather
#endif
#ifndef ONCHIP_MAC_SB
#define ONCHIP_MAC_SB 4  // MAC slots per scheduling region (GGSW loads in flight)
#endif
#ifndef ONCHIP_QROT
#define ONCHIP_QROT 1  // wave pair -> sub-block rotated per workgroup (0: pair p on sub-block p)
#endif
// L = 2: WaveFft exchange bases recomputed per transform (bit 1 la, bit 2 qa).  Hoisted out of the
// CMUX loop, their 32 XOR images were spilled to scratch inside it (<8192, true, 2>: 132 B private,
// 15 scratch stores + 33 loads per CMUX, vmcnt(0) waits on the GGSW prefetch; <4096, true, 2>: 84 B).
// The bits per N are the smallest that leave every L = 2 instantiation with no private segment
// (8192: 3 -> 246 VGPRs, +66 VALU per CMUX; 4096: 1 -> 249-253 VGPRs, +21 VALU; 4096 with both bits
// spilled again in the 64-bit-digit instantiation)
#ifndef ONCHIP_LAUNDER_8192
#define ONCHIP_LAUNDER_8192 3
#endif
#ifndef ONCHIP_LAUNDER_4096
#define ONCHIP_LAUNDER_4096 1
#endif
#ifndef ONCHIP_4096_CPW
#define ONCHIP_4096_CPW 1  // N = 4096: 1 = one ciphertext per 256-thread workgroup (two workgroups per CU,
                           // independent barriers); 2 = two ciphertexts per 512-thread workgroup
#endif
template <int N>
struct OnchipCfg {
    static constexpr int M = N / 2, R = M / 1024;
    static constexpr int CPW = R == 4 ? 1 : ONCHIP_4096_CPW;  // ciphertexts per workgroup
    static constexpr int THREADS = 256 * R / 2 * CPW;         // 2 R waves per ciphertext
    static constexpr int WAVES = THREADS / 64;
    static constexpr int WPS = THREADS / 256;                 // waves per SIMD of one workgroup
    static constexpr int MIN_WPS = 2;                         // 2 waves per SIMD per CU: 256 VGPRs
    static constexpr int TPC = THREADS / CPW;  // threads per ciphertext
    static constexpr int H = 1024 / TPC;       // top-stage butterflies per thread
    static constexpr int BUF = SubFft::XL;    // double2 per wave buffer
    static constexpr int S1 = WAVES * BUF;    // twiddle table offset (double2 units)
    static constexpr int FLAGS = S1 + SubFft::Lds::s1_len;  // pair-sync flags (double2 offset), one word per wave
    static constexpr size_t LDS = sizeof(double2) * FLAGS + 4 * WAVES;
    static_assert(R == 4 || R == 2, "CPW ciphertexts x R sub-blocks x 2 rows of waves");
    static_assert(WAVES * BUF * sizeof(double2) == CPW * 2 * M * sizeof(acc_pair), "the rotation's pairs fill the wave buffers");
    static_assert(LDS <= 160 * 1024 / (MIN_WPS / WPS), "LDS of the workgroups one CU holds");
};

// MAC of level L - LI for one sub-block: both rows' spectra from their buffers F (row r at
// F + r BUF; the own one too, so its registers are free here); o accumulates over levels L..1
// and rows 0..k in the oracle's order (sub_cmux_body's forms)
#ifndef ONCHIP_PAIRSYNC
#define ONCHIP_PAIRSYNC 1  // the publish -> MAC sync through the pair's LDS flags instead of a barrier
#endif
#ifndef ONCHIP_TPF
#define ONCHIP_TPF 1  // top-stage twist / twiddle loads issued before the barrier preceding their use
#endif
#ifndef ONCHIP_PF
#define ONCHIP_PF 4  // MAC slots whose GGSW operands are issued before the publish barrier (0: none)
#endif
// N = 8192, L = 2 (3_3): 6 slots before the barrier, then regions of 4 -- round 5 (with the spilling
// build) measured 5 / 3 best (10.75-10.78k -> 11.34-11.37k KS+PBS/s against 4 / 4,
// profiles/r05_ab_onchip_pfsb*.log); re-swept after the exchange addresses stopped spilling (round 6,
// profiles/r06_ab_onchip_pfsb.txt): 5 / 3 12.02-12.03k, 6 / 4 12.27k, 6 / 3 12.26k, 8 / 4 12.20k,
// 7 / 3 12.18k, 5 / 4 12.10-12.11k, 4 / 4 12.08k (the other shapes measured best at 4 / 4)
#ifndef ONCHIP_PF_8192_L2
#define ONCHIP_PF_8192_L2 6
#endif
#ifndef ONCHIP_MAC_SB_8192_L2
#define ONCHIP_MAC_SB_8192_L2 4
#endif
template <int M, int L>
constexpr int onchip_pf() { return M == 4096 && L == 2 ? ONCHIP_PF_8192_L2 : ONCHIP_PF; }
template <int M, int L>
constexpr int onchip_sb() { return M == 4096 && L == 2 ? ONCHIP_MAC_SB_8192_L2 : ONCHIP_MAC_SB; }
template <int M, int L>
constexpr int onchip_pfs() { return onchip_pf<M, L>() > 0 ? onchip_pf<M, L>() : 1; }
// GGSW operands (rows 0 and 1 of level L - LI, column of rg) of MAC slot s
template <int M, int LI, int L = 2>
__device__ __forceinline__ void onchip_ggsw(__amdgpu_buffer_rsrc_t rg, uint32_t gvo, int s, double2 &g0, double2 &g1) {
    constexpr int P0 = (L - 1 - LI) * 2;  // polynomial (lvl - 1)(k + 1) of row 0, lvl = L - LI
    g0 = buffer_ld_d2(rg, gvo, 16u * (uint32_t)(P0 * 2 * M + s * 64));
    g1 = buffer_ld_d2(rg, gvo, 16u * (uint32_t)((P0 + 1) * 2 * M + s * 64));
}
template <int M, int BUF, int LI, int L = 2>
__device__ __forceinline__ void onchip_mac(__amdgpu_buffer_rsrc_t rg, uint32_t gvo, const double2 *F, cx (&o)[16],
                                           const double2 (&pf)[onchip_pfs<M, L>()][2]) {
    constexpr int PF = onchip_pf<M, L>(), PFS = onchip_pfs<M, L>(), SB = onchip_sb<M, L>();
#pragma unroll
    for (int s = 0; s < 16; s++) {
        if (s >= PF && (s - PF) % SB == 0) __builtin_amdgcn_sched_barrier(0);
        const double2 f0 = F[s * 64], f1 = F[BUF + s * 64];
        double2 g0, g1;
        if (s < PF) {
            g0 = pf[s < PFS ? s : 0][0];
            g1 = pf[s < PFS ? s : 0][1];
        } else {
            onchip_ggsw<M, LI, L>(rg, gvo, s, g0, g1);
        }
        if (ONCHIP_TSKIP & 1) {
            g0 = f1;
            g1 = f0;
        }
        cx x = o[s];
        if constexpr (LI == 0) {
            x.re = fma(g0.x, f0.x, -(g0.y * f0.y));
            x.im = fma(g0.x, f0.y, g0.y * f0.x);
        } else {
            x.re = fma(g0.x, f0.x, fma(-g0.y, f0.y, x.re));
            x.im = fma(g0.x, f0.y, fma(g0.y, f0.x, x.im));
        }
        x.re = fma(g1.x, f1.x, fma(-g1.y, f1.y, x.re));
        x.im = fma(g1.x, f1.y, fma(g1.y, f1.x, x.im));
        o[s] = x;
    }
}

// decompose64<2> in 32-bit registers when base_log * 2 <= 30 (pbs_common.h decomp_state32: the
// same digits)
template <bool D32>
__device__ __forceinline__ void onchip_decompose(uint64_t x, int beta, int32_t (&d)[2]) {
    if constexpr (D32) {
        uint32_t st = decomp_state32<2>(x, beta);
        const uint32_t mask = (1u << beta) - 1;
        d[0] = decomp_digit32(st, beta, mask);
        d[1] = decomp_digit32(st, beta, mask);
    } else {
        decompose64<2>(x, beta, d);
    }
}

#ifndef ONCHIP_DIGIT2
#define ONCHIP_DIGIT2 1  // 0: two decomp_digit32 per value (A/B of Digit2, pbs_common.h)
#endif
// both levels of the values at j and j + M as the int16 quad the top DIF reads: level L at j, j + M
// in the low dword, level L-1 in the high dword
template <bool D32>
__device__ __forceinline__ uint64_t onchip_pack2(uint64_t v0, uint64_t v1, int beta, const Digit2 &dg2) {
    if constexpr (D32 && ONCHIP_DIGIT2) {
        uint32_t lv0, lv1;
        dg2.pair((uint32_t)(v0 >> 32), (uint32_t)(v1 >> 32), lv0, lv1);
        return (uint64_t)lv0 | ((uint64_t)lv1 << 32);
    } else {
        int32_t e0[2], e1[2];
        onchip_decompose<D32>(v0, beta, e0);
        onchip_decompose<D32>(v1, beta, e1);
        return ((uint64_t)((uint32_t)e0[0] & 0xffffu)) | ((uint64_t)((uint32_t)e1[0] & 0xffffu) << 16) |
               ((uint64_t)((uint32_t)e0[1] & 0xffffu) << 32) | ((uint64_t)((uint32_t)e1[1] & 0xffffu) << 48);
    }
}

// L = 1: the one signed digit (decompose64<1>; 32-bit when base_log <= 30)
template <bool D32>
__device__ __forceinline__ int32_t onchip_decompose1(uint64_t x, int beta) {
    if constexpr (D32) {
        uint32_t st = decomp_state32<1>(x, beta);
        return decomp_digit32(st, beta, (1u << beta) - 1);
    } else {
        int32_t d[1];
        decompose64<1>(x, beta, d);
        return d[0];
    }
}

// a zero the compiler cannot see through: table pointers offset by it (the twist, the top-stage
// twiddles, the CMUX's GGSW) are not provably loop-invariant, so their loads stay where they are
// used instead of being hoisted out of the CMUX loop into registers held for good (an opaque
// pointer instead would lose its address space: flat loads, counted against the LDS waits too)
__device__ __forceinline__ int opaque_zero() {
    int z = 0;
    asm volatile("" : "+s"(z));
    return z;
}

template <int N, bool D32, int L = 2>
__global__ void __launch_bounds__(OnchipCfg<N>::THREADS, OnchipCfg<N>::MIN_WPS / OnchipCfg<N>::WPS) onchip_cmux_kernel(LargePbsLaunch a) {
    using S = Split<N>;
    using Cfg = OnchipCfg<N>;
    static_assert(L == 1 || L == 2, "one or two decomposition levels");
    constexpr int K = 1, M = S::M, R = S::R, H = Cfg::H, BUF = Cfg::BUF, CPW = Cfg::CPW, TPC = Cfg::TPC;
    constexpr size_t ggsw_len = (size_t)L * (K + 1) * (K + 1) * M;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    acc_pair *pairs = reinterpret_cast<acc_pair *>(smem);  // rotation view: [row][M] pairs
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    // wave = 2 R c + 2 q + wr: ciphertext c of the workgroup, sub-block q, row (forward) = column
    // (MAC, inverse) wr; thread t works for ciphertext ctl = t / TPC as thread tc = t mod TPC
    // sub-block of the wave pair, rotated by the workgroup's index among those of its XCD
    // (ONCHIP_QROT) so that the CUs of an XCD do not all stream the same GGSW slice at once
    const int q = ((wave >> 1) + (ONCHIP_QROT ? (int)(blockIdx.x >> 3) : 0)) & (R - 1), wr = wave & 1;
    const int ctl = CPW == 1 ? 0 : t / TPC, tc = CPW == 1 ? t : t % TPC;
    const int cb = 2 * R * ctl;  // this thread's ciphertext's first wave buffer
    const int wbuf = cb + 2 * q + wr;  // this wave's buffer: sub-block q, row / column wr
    const int ct_raw = CPW == 1 ? (int)blockIdx.x : (int)blockIdx.x * CPW + ctl;
    const int ct = CPW == 1 ? ct_raw : min(ct_raw, a.count - 1);  // a padding slot repeats the last ciphertext
    double2 *s1 = lds + Cfg::S1;
    // sub-block stage twiddles W_1024[lane c] = W_M[R lane c]  (oracle dif_rec tstride R)
    for (int e = t; e < SubFft::Lds::s1_len; e += Cfg::THREADS) s1[e] = a.W[R * (e & 63) * ((e >> 6) + 1)];
    if (t < Cfg::WAVES) reinterpret_cast<uint32_t *>(lds + Cfg::FLAGS)[t] = 0;
    GroupSync<2> ps;  // the two waves of sub-block q (flag words 2 q, 2 q + 1)
    ps.mine = lds_addr(lds + Cfg::FLAGS) + 4u * wave;
    const SubFft::Lds tw{s1, s1};
    cx *xb = reinterpret_cast<cx *>(lds) + wbuf * BUF;
    double2 *own = lds + wbuf * BUF;
    WaveLocalSyncL<L == 2 ? (N == 8192 ? ONCHIP_LAUNDER_8192 : ONCHIP_LAUNDER_4096) : 0> wsync;
    const uint64_t *in = a.lwe_in + (size_t)ct * (a.n + 1);
    // twist and top-stage twiddles through buffer loads: one VGPR offset, the rest in SGPRs
    const __amdgpu_buffer_rsrc_t rtw = make_rsrc(a.twist), rwt = make_rsrc(a.wtop);
    const uint32_t tvo = 16u * tc;
    auto ld_cx = [](__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
        const double2 x = buffer_ld_d2(r, vo, so);
        return cx{x.x, x.y};
    };

    // acc = LUT / X^{b~} (large_init_kernel)
    uint64_t lo[2][H][R], hi[2][H][R];
    {
        const uint32_t bt = pbs_modulus_switch<S::LOGN>(in[a.n]);
        const uint32_t li = a.lut_indexes ? min(a.lut_indexes[ct], a.lut_count - 1u) : 0u;
        const uint64_t *lut = a.luts + (size_t)li * (K + 1) * N;
        const int full = bt / N, rem = bt % N;
        auto init = [&](int r, int p) -> uint64_t {
            const int src = p + rem;
            const bool wrap = src >= N;
            const uint64_t v = lut[(size_t)r * N + (wrap ? src - N : src)];
            return (wrap != (bool)(full & 1)) ? 0 - v : v;
        };
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int h = 0; h < H; h++)
#pragma unroll
                for (int b = 0; b < R; b++) {
                    const int j = tc + TPC * h + 1024 * b;
                    lo[r][h][b] = init(r, j);
                    hi[r][h][b] = init(r, j + M);
                }
    }
    const double k32 = torus_k32();
    const int beta = a.base_log;
    const Digit2 dg2(D32 ? beta : 2);  // (unused unless D32)
    const DigitL1 dl1(D32 ? beta : 2);
    // accumulator pair (row r, j) <-> LDS slot (2 (j >> 10) + r) BUF + (j & 1023): the slots thread t
    // owns, (2 b + r) BUF + t + 512 h, are exactly the top-stage / top-inverse slots of its butterflies,
    // so the top inverse writes the updated pairs in place (no barrier between its reads and them)
    auto pslot = [&](int r, int j) { return (cb + 2 * (j >> 10) + r) * BUF + (j & 1023); };
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
        for (int h = 0; h < H; h++)
#pragma unroll
            for (int b = 0; b < R; b++) pairs[(cb + 2 * b + r) * BUF + tc + TPC * h] = acc_pair{lo[r][h][b], hi[r][h][b]};

    uint64_t a_next = in[0];
    for (int i = 0; i < a.n; i++) {
        const uint32_t at = pbs_modulus_switch<S::LOGN>(a_next);
        a_next = in[i + 1 < a.n ? i + 1 : i];  // next mask element: its load latency hides behind this CMUX
        const bool full_odd = (at / N) & 1;
        const int rem = at % N;
        // ---- rotation + decomposition (split_digits through LDS) ----
        __syncthreads();  // every pair written (and, at i = 0, the twiddle table)
        uint64_t pk[2][H][R];  // int16 digits: level L at j, j + M; level L-1 at j, j + M
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int h = 0; h < H; h++)
#pragma unroll
                for (int b = 0; b < R; b++) {
                    const int j = tc + TPC * h + 1024 * b;
                    const int jj0 = j - rem;  // in (-N, M)
                    const acc_pair rot = (ONCHIP_TSKIP & 16) ? acc_pair{lo[r][h][b] * 3, hi[r][h][b]} : pairs[pslot(r, jj0 & (M - 1))];
                    const bool swap = jj0 < 0 && jj0 >= -M;
                    const uint64_t x0 = swap ? rot.y : rot.x, x1 = swap ? rot.x : rot.y;
                    const bool neg0 = (jj0 < 0) != full_odd, neg1 = (jj0 + M < 0) != full_odd;
                    if constexpr (L == 2) {
                        pk[r][h][b] = onchip_pack2<D32>((neg0 ? 0 - x0 : x0) - lo[r][h][b], (neg1 ? 0 - x1 : x1) - hi[r][h][b],
                                                        beta, dg2);
                    } else {  // one level: |digit| <= 2^(beta - 1) (2^21 at base 2^22) -- two int32 fields
                        const uint64_t v0 = (neg0 ? 0 - x0 : x0) - lo[r][h][b], v1 = (neg1 ? 0 - x1 : x1) - hi[r][h][b];
                        int32_t e0, e1;
                        if constexpr (D32 && ONCHIP_DIGIT2) {  // the classic kernel's 3-op digit (DigitL1)
                            e0 = dl1((uint32_t)(v0 >> 32));
                            e1 = dl1((uint32_t)(v1 >> 32));
                        } else {
                            e0 = onchip_decompose1<D32>(v0, beta);
                            e1 = onchip_decompose1<D32>(v1, beta);
                        }
                        pk[r][h][b] = (uint64_t)(uint32_t)e0 | ((uint64_t)(uint32_t)e1 << 32);
                    }
                }
        // the top stage's twist and twiddles (tv[h][b] = twist[a + 1024 b], wq[h][c] = W[a c] of
        // butterfly a = t + 512 h): issued before the barrier that precedes their use
        cx tv[H][R], wq[H][R];
        auto top_loads_h = [&](int h) {
            const uint32_t z = (uint32_t)opaque_zero();
#pragma unroll
            for (int b = 0; b < R; b++) tv[h][b] = ld_cx(rtw, tvo, z + 16u * (TPC * h + 1024 * b));
#pragma unroll
            for (int c = 1; c < R; c++) wq[h][c] = ld_cx(rwt, tvo, z + 16u * ((c - 1) * 1024 + TPC * h));
        };
        auto top_loads = [&]() {
#pragma unroll
            for (int h = 0; h < H; h++) top_loads_h(h);
        };
        if (ONCHIP_TPF) top_loads();
        __syncthreads();  // the pairs are read: the region becomes the wave buffers
        const __amdgpu_buffer_rsrc_t rg = make_rsrc(a.fbsk + (size_t)i * ggsw_len + (size_t)wr * M + 1024 * q);
        cx o[16];
        auto level = [&](auto LIc) {
            constexpr int LI = decltype(LIc)::value;  // 0: level L, 1: level L-1
            // ---- twist + top DIF radix-4 of both rows -> wave buffers (large_top_fwd) ----
            // (level L-1: per butterfly half, where they are used -- the MAC outputs are live)
#pragma unroll
            for (int h = 0; h < H; h++) {
                const int a0 = tc + TPC * h;
                if (!ONCHIP_TPF || LI == 1) top_loads_h(h);
#pragma unroll
                for (int r = 0; r < 2; r++) {
                    cx u[R];
#pragma unroll
                    for (int b = 0; b < R; b++) {
                        int32_t d0, d1;
                        if constexpr (L == 2) {
                            const uint64_t w = pk[r][h][b] >> (32 * LI);
                            d0 = (int32_t)(int16_t)(w & 0xffffu);
                            d1 = (int32_t)(int16_t)((w >> 16) & 0xffffu);
                        } else {
                            d0 = (int32_t)(uint32_t)pk[r][h][b];
                            d1 = (int32_t)(uint32_t)(pk[r][h][b] >> 32);
                        }
                        u[b] = cmulw(cx{(double)d0, (double)d1}, tv[h][b].re, tv[h][b].im);
                    }
                    if (!(ONCHIP_TSKIP & 8)) dftR_fwd<R>(u);
                    lds[(cb + r) * BUF + a0] = make_double2(u[0].re, u[0].im);
#pragma unroll
                    for (int c = 1; c < R; c++) {
                        const cx y = cmulw(u[c], wq[h][c].re, wq[h][c].im);
                        lds[(cb + 2 * c + r) * BUF + a0] = make_double2(y.re, y.im);
                    }
                }
            }
            __syncthreads();
            // ---- sub-block forward FFT of (q, row wr), published in place ----
            cx v[16];
#pragma unroll
            for (int b = 0; b < 16; b++) {
                const double2 x = own[lane + 64 * b];
                v[b] = cx{x.x, x.y};
            }
            if (!(ONCHIP_TSKIP & 2)) SubFft::forward(v, xb, tw, lane, wsync);
            wsync();
#pragma unroll
            for (int s = 0; s < 16; s++) own[s * 64 + lane] = make_double2(v[s].re, v[s].im);
            // the first slots' GGSW operands are in flight during the barrier
            double2 pf[onchip_pfs<M, L>()][2];
#pragma unroll
            for (int s = 0; s < onchip_pf<M, L>(); s++) onchip_ggsw<M, LI, L>(rg, 16u * lane, s, pf[s][0], pf[s][1]);
            if (ONCHIP_PAIRSYNC) ps();  // only the partner reads this spectrum
            else __syncthreads();
            // ---- MAC of this level, column wr ----
            onchip_mac<M, BUF, LI, L>(rg, 16u * lane, lds + (wbuf & ~1) * BUF + lane, o, pf);
            __syncthreads();  // the partner has read this wave's spectrum
        };
        level(std::integral_constant<int, 0>{});
        if constexpr (L == 2) level(std::integral_constant<int, 1>{});
        // ---- inverse sub-FFT of (q, column wr) -> its buffer, natural layout ----
        if (!(ONCHIP_TSKIP & 4)) SubFft::inverse(o, xb, tw, lane, wsync);
        wsync();
#pragma unroll
        for (int b = 0; b < 16; b++) own[lane + 64 * b] = make_double2(o[b].re, o[b].im);
        if (ONCHIP_TPF) top_loads();
        __syncthreads();
        // ---- top DIT radix-4, backward conversion, acc += (large_top_inv) ----
        if (!ONCHIP_TPF) top_loads();
#pragma unroll
        for (int h = 0; h < H; h++) {
            const int a0 = tc + TPC * h;
#pragma unroll
            for (int col = 0; col < 2; col++) {
                cx u[R];
                {
                    const double2 x = lds[(cb + col) * BUF + a0];
                    u[0] = cx{x.x, x.y};
                }
#pragma unroll
                for (int c = 1; c < R; c++) {
                    const double2 x = lds[(cb + 2 * c + col) * BUF + a0];
                    u[c] = cmulw(cx{x.x, x.y}, wq[h][c].re, -wq[h][c].im);
                }
                if (!(ONCHIP_TSKIP & 8)) dftR_inv<R>(u);
#pragma unroll
                for (int b = 0; b < R; b++) {
                    backward_add(u[b], tv[h][b], lo[col][h][b], hi[col][h][b], k32);
                    pairs[(cb + 2 * b + col) * BUF + a0] = acc_pair{lo[col][h][b], hi[col][h][b]};  // = slot read above
                }
            }
        }
    }
    // ---- sample extract at degree 0 (large_extract_kernel) from the pairs ----
    __syncthreads();
    uint64_t *out = a.lwe_out + (size_t)ct * ((size_t)K * N + 1);
    if (CPW > 1 && ct_raw >= a.count) return;  // padding slot: nothing to store (no barrier follows)
    for (int e = tc; e < N; e += TPC) {
        const int p = e == 0 ? 0 : N - e;
        const acc_pair pr = pairs[pslot(0, p & (M - 1))];
        const uint64_t x = p >= M ? pr.y : pr.x;
        out[e] = e == 0 ? x : 0 - x;
    }
    if (tc == 0) out[N] = lo[1][0][0];  // row 1 position 0: the body
}

static bool onchip_enabled() {
    static const bool v = [] {
        const char *e = std::getenv("TFHE_MI355_ONCHIP");
        return !(e && e[0] == '0');
    }();
    return v;
}

// ---------------------------------------------------------------------------------------
// Quad CMUX (N = 8192, k = 1, L = 2, classic; small batches).  The
// on-chip CMUX runs a ciphertext's whole blind rotation on ONE CU (25 us per CMUX: 22-25 ms per
// call whatever the count), the split CMUX spreads it over several launches per CMUX (16.3 ms for
// one ciphertext).  Here the R = 4 sub-blocks of one ciphertext run on R CUs of one XCD at once, in
// one launch for the whole blind rotation.  Every workgroup keeps the FULL accumulator (registers
// as in the on-chip kernel, thread t owning the pairs (j, j + M), j = t + 512 h + 1024 b) and does
// the cheap full-width work itself -- rotation, decomposition, the top DIT inverse + backward
// conversion -- but the expensive part only for its sub-block q:
//   rotation     : pairs -> LDS, ct1 = X^{a~} acc - acc gathered, digits (as the on-chip kernel)
//   top DIF      : output q of every top radix-4 butterfly, both levels and rows -> 4 LDS buffers
//   sub-FFTs     : waves 0-3, one polynomial (level, row) each, spectra published in place;
//                  meanwhile waves 4-7 load the CMUX's GGSW operands of sub-block q (4 slots each)
//   MAC          : waves 4-7, slots 4 w' .. 4 w' + 3, both columns, the oracle's level/row order
//   inverse      : waves 0-1 (column c) -> U_q[c], stored write-through to the ciphertext's
//                  exchange buffer (double-buffered by CMUX parity), then a flag
//   exchange     : every workgroup waits for the R flags of CMUX i, loads U_0..U_{R-1} at its
//                  butterflies (sc1 loads: L2 / Infinity Cache, never a stale L1 line) and runs the
//                  top DIT radix-4 + backward_add of both columns into its registers
// One exchange per CMUX (U: 32 KiB out, 96 KiB in per workgroup); the hand-off is the guide's
// "sc1 payload + drained flag" form (MI355X_MICROARCH.md, inter-workgroup visibility).  Same
// operations on the same values as the on-chip / split paths (the redundant full-width parts
// compute identical values in every workgroup), so the outputs are bit-identical.
// Co-residency: the R workgroups of a ciphertext wait on each other, so a launch holds at most one
// workgroup per CU (143 KiB of LDS each) and at most CUs / R ciphertexts, and quad launches of one
// device are serialised (launch_quad below); every flag wait is bounded (QUAD_SPIN_MAX polls).
// ---------------------------------------------------------------------------------------
#ifndef QUAD_SPIN_MAX
#define QUAD_SPIN_MAX (1u << 24)
#endif
#ifndef QUAD_STAMPS
#define QUAD_STAMPS 0  // diagnostic builds: s_memtime at the phase boundaries of CMUX 200 (waves 0 and 4 of
                       // ciphertext 0's workgroup q = 0), written over that ciphertext's output words 1..26
#endif
#ifndef QUAD_TPF
#define QUAD_TPF 1  // the top stages' twist / W loads issued ahead of the barrier before their use
#endif
#ifndef QUAD_OWNU
#define QUAD_OWNU 0  // 1: the workgroup's own U_q read back from LDS, not from the exchange buffer -- the
                     // per-sub-block branch serialises the U loads: 13.07-13.68 vs 12.63 ms per call
                     // (profiles/r06_quad_ab.txt)
#endif
#ifndef QUAD_PPOLL
#define QUAD_PPOLL 1  // the R exchange flags polled by R lanes at once (0: lane 0 polls them in turn)
#endif
#ifndef QUAD_WPOLL
#define QUAD_WPOLL 0  // 1: every wave polls the flags itself instead of wave 0 + a workgroup barrier
#endif
#ifndef QUAD_PKFENCE
#define QUAD_PKFENCE 1  // the digits computed before the barrier that ends the rotation
#endif
#ifndef QUAD_TSKIP
#define QUAD_TSKIP 0  // timing-only builds (wrong outputs): 1 no flag wait, 2 no forward sub-FFTs, 4 no inverse
                      // sub-FFTs, 8 no GGSW loads, 16 no U loads, 32 no U stores
#endif
template <int N>
struct QuadCfg {
    static constexpr int M = N / 2, R = M / 1024;
    static constexpr int THREADS = 512, TPC = THREADS, H = 1024 / THREADS;
    static constexpr int BUF = SubFft::XL;
    // the rotation's 2 x M pairs; then 4 spectra + 2 columns (N = 4096: the six buffers are the larger)
    static constexpr int REGION = (2 * R > 6 ? 2 * R : 6) * BUF;
    static constexpr int S1 = REGION;
    static constexpr size_t LDS = sizeof(double2) * (S1 + SubFft::Lds::s1_len);
    static_assert(LDS > 80 * 1024 && LDS <= 160 * 1024, "one workgroup per CU");
    // device scratch of a launch: flags [ct][R] (one 128-B line each), then per ciphertext the
    // exchange U [parity 2][sub-block R][column 2][1024] double2
    static constexpr size_t FLAG_BYTES = 128;
    static constexpr size_t U_BYTES = (size_t)2 * R * 2 * 1024 * sizeof(double2);
};

template <int N>
__device__ __forceinline__ double2 *quad_u(const LargePbsLaunch &a, int cnt, int ct, int par, int q, int c) {
    using Cfg = QuadCfg<N>;
    char *base = reinterpret_cast<char *>(a.scratch) + (size_t)cnt * Cfg::R * Cfg::FLAG_BYTES;
    return reinterpret_cast<double2 *>(base + (size_t)ct * Cfg::U_BYTES) + ((size_t)(par * Cfg::R + q) * 2 + c) * 1024;
}

template <int N, bool D32, int L>
__global__ void __launch_bounds__(512, 1) quad_cmux_kernel(LargePbsLaunch a, int ct0, int cnt) {
    using S = Split<N>;
    using Cfg = QuadCfg<N>;
    constexpr int K = 1, M = S::M, R = S::R, H = Cfg::H, BUF = Cfg::BUF, TPC = Cfg::TPC, P = 2 * L;
    static_assert(L == 1 || L == 2, "one or two levels (2 L spectra per sub-block)");
    static_assert(R == 4 || R == 2, "N = 8192 (quad) or 4096 (duo)");
    constexpr size_t ggsw_len = (size_t)L * (K + 1) * (K + 1) * M;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    acc_pair *pairs = reinterpret_cast<acc_pair *>(smem);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    // the R workgroups of ciphertext cl: blocks 8 m + x with the same x (one XCD), q = m mod R
    const int x = blockIdx.x & 7, mm = blockIdx.x >> 3;
    const int cl = x + 8 * (mm / R), q = mm % R;
    if (cl >= cnt) return;  // all R workgroups of a padding slot
    const int ct = ct0 + cl;
    uint32_t *flags = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(a.scratch) + (size_t)cl * R * Cfg::FLAG_BYTES);
    double2 *s1 = lds + Cfg::S1;
    for (int e = t; e < SubFft::Lds::s1_len; e += TPC) s1[e] = a.W[R * (e & 63) * ((e >> 6) + 1)];
    const SubFft::Lds tw{s1, s1};
    const uint64_t *in = a.lwe_in + (size_t)ct * (a.n + 1);

    // acc = LUT / X^{b~} (large_init_kernel), full width in every workgroup
    uint64_t lo[2][H][R], hi[2][H][R];
    {
        const uint32_t bt = pbs_modulus_switch<S::LOGN>(in[a.n]);
        const uint32_t li = a.lut_indexes ? min(a.lut_indexes[ct], a.lut_count - 1u) : 0u;
        const uint64_t *lut = a.luts + (size_t)li * (K + 1) * N;
        const int full = bt / N, rem = bt % N;
        auto init = [&](int r, int p) -> uint64_t {
            const int src = p + rem;
            const bool wrap = src >= N;
            const uint64_t v = lut[(size_t)r * N + (wrap ? src - N : src)];
            return (wrap != (bool)(full & 1)) ? 0 - v : v;
        };
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int h = 0; h < H; h++)
#pragma unroll
                for (int b = 0; b < R; b++) {
                    const int j = t + TPC * h + 1024 * b;
                    lo[r][h][b] = init(r, j);
                    hi[r][h][b] = init(r, j + M);
                }
    }
    const double k32 = torus_k32();
    const int beta = a.base_log;
    const Digit2 dg2(D32 ? beta : 2);  // (unused unless D32)
    const DigitL1 dl1(D32 ? beta : 2);
    auto pslot = [&](int r, int j) { return (2 * (j >> 10) + r) * BUF + (j & 1023); };
    auto store_pairs = [&]() {
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int h = 0; h < H; h++)
#pragma unroll
                for (int b = 0; b < R; b++) pairs[(2 * b + r) * BUF + t + TPC * h] = acc_pair{lo[r][h][b], hi[r][h][b]};
    };
    store_pairs();
    WaveLocalSyncL<3> wsync;
    const __amdgpu_buffer_rsrc_t rtw = make_rsrc(a.twist), rwt = make_rsrc(a.wtop);
    uint64_t st[QUAD_STAMPS ? 13 : 1];
    auto stamp = [&](int i, int k) {
        if constexpr (QUAD_STAMPS) {
            if (i == 200) st[k] = __builtin_amdgcn_s_memtime();
        }
    };

    uint64_t a_next = in[0];
    for (int i = 0; i < a.n; i++) {
        stamp(i, 0);
        const uint32_t at = pbs_modulus_switch<S::LOGN>(a_next);
        a_next = in[i + 1 < a.n ? i + 1 : i];
        const bool full_odd = (at / N) & 1;
        const int rem = at % N;
        const int par = i & 1;
        // the top stage's twist and W[a0 q], issued ahead of the barrier (QUAD_TPF)
        cx tvh[H][R], wqh[H];
        auto top_tables = [&]() {
            const uint32_t z = (uint32_t)opaque_zero();
#pragma unroll
            for (int h = 0; h < H; h++) {
#pragma unroll
                for (int b = 0; b < R; b++) {
                    const double2 y = buffer_ld_d2(rtw, 16u * (t + TPC * h + 1024 * b), z);
                    tvh[h][b] = cx{y.x, y.y};
                }
                const double2 y = q ? buffer_ld_d2(rwt, 16u * ((q - 1) * 1024 + t + TPC * h), z) : make_double2(1.0, 0.0);
                wqh[h] = cx{y.x, y.y};
            }
        };
        if (QUAD_TPF) top_tables();
        __syncthreads();  // every pair written (and, at i = 0, the twiddle table)
        stamp(i, 1);
        // ---- rotation + decomposition (the on-chip kernel's) ----
        uint64_t pk[2][H][R];
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int h = 0; h < H; h++)
#pragma unroll
                for (int b = 0; b < R; b++) {
                    const int j = t + TPC * h + 1024 * b;
                    const int jj0 = j - rem;
                    const acc_pair rot = pairs[pslot(r, jj0 & (M - 1))];
                    const bool swap = jj0 < 0 && jj0 >= -M;
                    const uint64_t x0 = swap ? rot.y : rot.x, x1 = swap ? rot.x : rot.y;
                    const bool neg0 = (jj0 < 0) != full_odd, neg1 = (jj0 + M < 0) != full_odd;
                    const uint64_t v0 = (neg0 ? 0 - x0 : x0) - lo[r][h][b], v1 = (neg1 ? 0 - x1 : x1) - hi[r][h][b];
                    if constexpr (L == 2) {
                        pk[r][h][b] = onchip_pack2<D32>(v0, v1, beta, dg2);
                    } else {  // |digit| <= 2^(beta - 1): two int32 fields
                        int32_t e0, e1;
                        if constexpr (D32) {
                            e0 = dl1((uint32_t)(v0 >> 32));
                            e1 = dl1((uint32_t)(v1 >> 32));
                        } else {
                            e0 = onchip_decompose1<D32>(v0, beta);
                            e1 = onchip_decompose1<D32>(v1, beta);
                        }
                        pk[r][h][b] = (uint64_t)(uint32_t)e0 | ((uint64_t)(uint32_t)e1 << 32);
                    }
                    if (QUAD_PKFENCE) asm volatile("" : "+v"(pk[r][h][b]));  // digits before the barrier: 32
                                                                            // registers live across it, not 64
                }
        stamp(i, 2);
        __syncthreads();  // the pairs are read: the region becomes the spectra
        stamp(i, 3);
        // ---- top DIF output q of both rows and levels ----
        if (!QUAD_TPF) top_tables();
        if constexpr (R == 4) {
            switch (q) {
                case 0: quad_top<N, 0, H, L>(lds, pk, tvh, wqh, t); break;
                case 1: quad_top<N, 1, H, L>(lds, pk, tvh, wqh, t); break;
                case 2: quad_top<N, 2, H, L>(lds, pk, tvh, wqh, t); break;
                default: quad_top<N, 3, H, L>(lds, pk, tvh, wqh, t); break;
            }
        } else {
            if (q == 0) quad_top<N, 0, H, L>(lds, pk, tvh, wqh, t);
            else quad_top<N, 1, H, L>(lds, pk, tvh, wqh, t);
        }
        stamp(i, 4);
        __syncthreads();
        stamp(i, 5);
        const __amdgpu_buffer_rsrc_t rg = make_rsrc(a.fbsk + (size_t)i * ggsw_len + 1024 * q);
        if (wave < 4) {
            cx v[16];
            if (wave < P) {
                // ---- sub-block forward FFT of polynomial p = wave, published in place ----
                double2 *own = lds + wave * BUF;
#pragma unroll
                for (int b = 0; b < 16; b++) {
                    const double2 y = own[lane + 64 * b];
                    v[b] = cx{y.x, y.y};
                }
                if (!(QUAD_TSKIP & 2)) SubFft::forward(v, reinterpret_cast<cx *>(own), tw, lane, wsync);
                wsync();
#pragma unroll
                for (int sl = 0; sl < 16; sl++) own[sl * 64 + lane] = make_double2(v[sl].re, v[sl].im);
            }
            __syncthreads();  // spectra published
            stamp(i, 6);
            __syncthreads();  // MAC outputs in the column buffers
            stamp(i, 7);
            if (wave < 2) {
                // ---- inverse sub-FFT of column c = wave -> U_q[c] (write-through) ----
                double2 *colb = lds + (4 + wave) * BUF;
#pragma unroll
                for (int sl = 0; sl < 16; sl++) {
                    const double2 y = colb[sl * 64 + lane];
                    v[sl] = cx{y.x, y.y};
                }
                if (!(QUAD_TSKIP & 4)) SubFft::inverse(v, reinterpret_cast<cx *>(colb), tw, lane, wsync);
                if (QUAD_OWNU) {
                    wsync();  // the inverse's own exchange reads of colb are done
#pragma unroll
                    for (int b = 0; b < 16; b++) colb[lane + 64 * b] = make_double2(v[b].re, v[b].im);  // own U_q[c]
                }
                double2 *dst = quad_u<N>(a, cnt, cl, par, q, wave);
                const __amdgpu_buffer_rsrc_t ru = make_rsrc(dst);
                if (!(QUAD_TSKIP & 32))
#pragma unroll
                    for (int b = 0; b < 16; b++)
                        buffer_st_d2p<16>(ru, 16u * (lane + 64 * b), 0, make_double2(v[b].re, v[b].im));
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            stamp(i, 8);
        } else {
            // ---- GGSW operands of slots 4 w' .. 4 w' + 3, both columns (in flight during the FFTs) ----
            const int w4 = wave - 4;
            double2 g[4][2][P];  // [slot][column][polynomial p]
#pragma unroll
            for (int k = 0; k < 4; k++)
#pragma unroll
                for (int c = 0; c < 2; c++)
#pragma unroll
                    for (int p = 0; p < P; p++)
                        g[k][c][p] = (QUAD_TSKIP & 8) ? make_double2(p + c, k)
                                                      : buffer_ld_d2(rg, 16u * lane, 16u * (uint32_t)((p * 2 + c) * M + (4 * w4 + k) * 64));
            __syncthreads();  // spectra published
            stamp(i, 6);
            // ---- MAC: levels L..1, rows 0..k (p = 2, 3, 0, 1 at L = 2; 0, 1 at L = 1), the oracle's forms ----
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int sl = 4 * w4 + k;
                double2 f[P];
#pragma unroll
                for (int p = 0; p < P; p++) f[p] = lds[p * BUF + sl * 64 + lane];
                constexpr int first = 2 * (L - 1);  // level L, row 0; then row 1, then level L-1 (L = 2)
#pragma unroll
                for (int c = 0; c < 2; c++) {
                    cx o;
                    {
                        const double2 gg = g[k][c][first], ff = f[first];
                        o.re = fma(gg.x, ff.x, -(gg.y * ff.y));
                        o.im = fma(gg.x, ff.y, gg.y * ff.x);
                    }
#pragma unroll
                    for (int u = 1; u < P; u++) {
                        const int pp = (first + u) % P;
                        const double2 gg = g[k][c][pp], ff = f[pp];
                        o.re = fma(gg.x, ff.x, fma(-gg.y, ff.y, o.re));
                        o.im = fma(gg.x, ff.y, fma(gg.y, ff.x, o.im));
                    }
                    lds[(4 + c) * BUF + sl * 64 + lane] = make_double2(o.re, o.im);
                }
            }
            stamp(i, 7);
            __syncthreads();  // MAC outputs in the column buffers
            stamp(i, 8);
        }
        // the top inverse's twist and W[a0 c], issued ahead of the exchange wait
        cx tvd[H][R], wqd[H][R];
        auto dit_tables = [&]() {
            const uint32_t z = (uint32_t)opaque_zero();
#pragma unroll
            for (int h = 0; h < H; h++) {
#pragma unroll
                for (int b = 0; b < R; b++) {
                    const double2 y = buffer_ld_d2(rtw, 16u * (t + TPC * h + 1024 * b), z);
                    tvd[h][b] = cx{y.x, y.y};
                }
#pragma unroll
                for (int c = 1; c < R; c++) {
                    const double2 y = buffer_ld_d2(rwt, 16u * ((c - 1) * 1024 + t + TPC * h), z);
                    wqd[h][c] = cx{y.x, y.y};
                }
            }
        };
        if (QUAD_TPF) dit_tables();
        __syncthreads();  // U_q stored and drained by both storing waves
        stamp(i, 9);
        // ---- exchange: the R workgroups' U of CMUX i ----
        if (QUAD_PPOLL && (QUAD_WPOLL || wave == 0)) {
            // lanes 0..R-1 poll the R flags together: one L2 round trip per poll instead of R in turn
            // (QUAD_WPOLL: every wave polls for itself, so no workgroup barrier follows the wait)
            if (wave == 0 && lane == 0)
                __hip_atomic_store(flags + q * (Cfg::FLAG_BYTES / 4), (uint32_t)(i + 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t *f = flags + (lane < R ? lane : 0) * (Cfg::FLAG_BYTES / 4);
            uint32_t spin = 0;
            for (; spin < ((QUAD_TSKIP & 1) ? 0u : QUAD_SPIN_MAX); spin++) {
                const uint32_t v = lane < R ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0u;
                if (__all(v >= (uint32_t)(i + 1))) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (spin == QUAD_SPIN_MAX && lane == 0 && a.quad_fail)
                __hip_atomic_store(a.quad_fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (!QUAD_PPOLL && t == 0) {
            __hip_atomic_store(flags + q * (Cfg::FLAG_BYTES / 4), (uint32_t)(i + 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            for (int p = 0; p < ((QUAD_TSKIP & 1) ? 0 : R); p++) {
                const uint32_t *f = flags + p * (Cfg::FLAG_BYTES / 4);
                uint32_t spin = 0;
                for (; spin < QUAD_SPIN_MAX; spin++) {
                    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (uint32_t)(i + 1)) break;
                    __builtin_amdgcn_s_sleep(1);
                }
                // a partner that never arrived (the device's CUs held by another process's quad grid):
                // the outputs are invalid -- recorded for the host (tfhe_mi355 fails the call), no hang
                if (spin == QUAD_SPIN_MAX && a.quad_fail)
                    __hip_atomic_store(a.quad_fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (!(QUAD_PPOLL && QUAD_WPOLL)) __syncthreads();
        stamp(i, 10);
        // ---- top DIT radix-4 of both columns, backward_add (large_top_inv), full width ----
        if (!QUAD_TPF) dit_tables();
#pragma unroll
        for (int h = 0; h < H; h++) {
            const int a0 = t + TPC * h;
            const cx *tv = tvd[h], *wq = wqd[h];
#pragma unroll
            for (int col = 0; col < 2; col++) {
                cx u[R];
#pragma unroll
                for (int c = 0; c < R; c++) {
                    typedef unsigned v4u __attribute__((ext_vector_type(4)));
                    cx y;
                    if (QUAD_OWNU && c == q) {  // this workgroup's own sub-block: kept in LDS by the inverse wave
                        const double2 z = lds[(4 + col) * BUF + a0];
                        y = cx{z.x, z.y};
                    } else if (QUAD_TSKIP & 16) {
                        const double2 z = lds[(c * 2 + col) * BUF + a0];
                        y = cx{z.x, z.y};
                    } else {
                        const v4u w = __builtin_amdgcn_raw_buffer_load_b128(make_rsrc(quad_u<N>(a, cnt, cl, par, c, col)),
                                                                             16u * a0, 0, 16);  // sc1: L2, not L1
                        y = cx{__hiloint2double((int)w.y, (int)w.x), __hiloint2double((int)w.w, (int)w.z)};
                    }
                    u[c] = c == 0 ? y : cmulw(y, wq[c].re, -wq[c].im);
                }
                dftR_inv<R>(u);
#pragma unroll
                for (int b = 0; b < R; b++) backward_add(u[b], tv[b], lo[col][h][b], hi[col][h][b], k32);
            }
        }
        stamp(i, 11);
        store_pairs();  // every LDS reader of this CMUX passed the barrier above
        stamp(i, 12);
    }
    // ---- sample extract at degree 0 (large_extract_kernel), workgroup 0 of the ciphertext ----
    __syncthreads();
    if (q != 0) return;
    uint64_t *out = a.lwe_out + (size_t)ct * ((size_t)K * N + 1);
    for (int e = t; e < N; e += TPC) {
        const int p = e == 0 ? 0 : N - e;
        const acc_pair pr = pairs[pslot(0, p & (M - 1))];
        const uint64_t xv = p >= M ? pr.y : pr.x;
        out[e] = e == 0 ? xv : 0 - xv;
    }
    if (t == 0) out[N] = lo[1][0][0];  // row 1 position 0: the body
    if constexpr (QUAD_STAMPS) {
        __syncthreads();
        if (cl == 0 && lane == 0 && (wave == 0 || wave == 4))
            for (int k = 1; k < 13; k++) out[(wave ? 14 : 1) + k] = st[k] - st[0];
    }
}

// TFHE_MI355_QUAD=0: never the quad CMUX (A/B)
static bool quad_enabled() {
    static const bool v = [] {
        const char *e = std::getenv("TFHE_MI355_QUAD");
        return !(e && e[0] == '0');
    }();
    return v;
}

// sample extract at degree 0 (glwe_sample_extraction.rs:91-147)
template <int N, int K>
__global__ void __launch_bounds__(256) large_extract_kernel(LargePbsLaunch a, int ct0, int cnt) {
    using S = Split<N>;
    const size_t per = (size_t)K * N + 1;
    const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= per * cnt) return;
    const int cl = (int)(e / per);
    const size_t q = e % per;
    const uint64_t *acc = a.acc + (size_t)cl * (K + 1) * N;
    uint64_t v;
    if (q == (size_t)K * N) {
        v = acc[(size_t)K * N];  // accx(0) = 0
    } else {
        const int p = (int)(q / N), j = (int)(q % N);
        v = j == 0 ? acc[(size_t)p * N] : 0 - acc[(size_t)p * N + accx_m<S::M>(N - j)];
    }
    a.lwe_out[(size_t)(ct0 + cl) * per + q] = v;
}


// standard -> Fourier BSK at N = 32768 (forward_as_torus, fft/mod.rs:197-218): one workgroup per poly
__global__ void __launch_bounds__(LT) large_bsk_to_fourier_kernel(const uint64_t *__restrict__ polys,
                                                                  double2 *__restrict__ out,
                                                                  const double2 *__restrict__ W,
                                                                  const double2 *__restrict__ wtop,
                                                                  const double2 *__restrict__ twist) {
    const LargeCtx c = large_setup(W, wtop);
    const uint64_t *x = polys + (size_t)blockIdx.x * LN;
    cx u[2][16];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int b = 0; b < 16; b++) {
            const int j = c.t + 512 * h + 1024 * b;
            const double xr = (double)(int64_t)x[j] * fourier_key_scale(LM);
            const double xi = (double)(int64_t)x[j + LM] * fourier_key_scale(LM);
            const cx w = gld(twist + j);
            u[h][b].re = xr * w.re - xi * w.im;
            u[h][b].im = xr * w.im + xi * w.re;
        }
    large_forward(c, u);
    double2 *o = out + (size_t)blockIdx.x * LM;
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int s = 0; s < 16; s++) o[spec_off(c.wave, h, s, c.lane)] = make_double2(u[h][s].re, u[h][s].im);
}

// standard -> Fourier BSK at N = 4096 ... 16384 (forward_as_torus, fft/mod.rs:197-218), in place in
// two launches: the top DIF radix-R of every polynomial into the natural sub-block order, then the
// 1024-point WaveFft of each sub-block (one wave each, read whole before it is overwritten in the
// engine layout: element (q 16 + s) 64 + lane = position 1024 q + 64 (lane & 15) + 16 (lane >> 4) + s)
template <int N>
__global__ void __launch_bounds__(256) mid_bsk_top_kernel(const uint64_t *__restrict__ polys, double2 *__restrict__ out,
                                                          const double2 *__restrict__ wtop,
                                                          const double2 *__restrict__ twist, size_t npoly) {
    using S = Split<N>;
    constexpr int R = S::R, M = S::M;
    const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= npoly * 1024) return;
    const size_t poly = e / 1024;
    const int t = (int)(e % 1024);
    const uint64_t *x = polys + poly * N;
    cx u[R];
#pragma unroll
    for (int b = 0; b < R; b++) {
        const int j = t + 1024 * b;
        const double xr = (double)(int64_t)x[j] * fourier_key_scale(M);
        const double xi = (double)(int64_t)x[j + M] * fourier_key_scale(M);
        const cx w = gld(twist + j);
        u[b].re = xr * w.re - xi * w.im;
        u[b].im = xr * w.im + xi * w.re;
    }
    dftR_fwd<R>(u);
    double2 *o = out + poly * M + t;
    o[0] = make_double2(u[0].re, u[0].im);
#pragma unroll
    for (int c = 1; c < R; c++) {
        const cx w = gld(wtop + (c - 1) * 1024 + t);  // = W[t c]
        const cx y = cmulw(u[c], w.re, w.im);
        o[1024 * c] = make_double2(y.re, y.im);
    }
}

template <int N>
__global__ void __launch_bounds__(256) mid_bsk_sub_kernel(double2 *__restrict__ out, const double2 *__restrict__ W,
                                                          size_t nblocks) {
    constexpr int R = Split<N>::R;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double2 *s1 = lds + 4 * SubFft::XL;
    for (int e = threadIdx.x; e < SubFft::Lds::s1_len; e += 256) s1[e] = W[R * (e & 63) * ((e >> 6) + 1)];
    __syncthreads();
    const size_t blk = (size_t)blockIdx.x * 4 + wave;  // (poly, q) = sub-block blk of the key
    if (blk >= nblocks) return;
    const SubFft::Lds tw{s1, s1};
    cx *xb = reinterpret_cast<cx *>(lds) + wave * SubFft::XL;
    WaveLocalSync wsync;
    double2 *o = out + blk * 1024;
    cx v[16];
#pragma unroll
    for (int b = 0; b < 16; b++) v[b] = gld(o + lane + 64 * b);
    SubFft::forward(v, xb, tw, lane, wsync);
#pragma unroll
    for (int sl = 0; sl < 16; sl++) o[sl * 64 + lane] = make_double2(v[sl].re, v[sl].im);
}

bool large_pbs_supported(int N, int k, int L) {
    return (N == 4096 || N == 8192 || N == 16384 || N == 32768) && k == 1 && L >= 1 && L <= 3;
}

size_t large_pbs_scratch_per_ct(int N, int k, int L) {
    const size_t split = (size_t)(k + 1) * N * sizeof(uint64_t) + (size_t)L * (k + 1) * (N / 2) * sizeof(double2);
    // the quad / duo CMUX's flags + exchange buffers per ciphertext (more than the split CMUX's
    // accumulator + spectra at L = 1)
    size_t quad = 0;
    if (k == 1 && L <= 2 && N == 8192) quad = QuadCfg<8192>::R * QuadCfg<8192>::FLAG_BYTES + QuadCfg<8192>::U_BYTES;
    if (k == 1 && L <= 2 && N == 4096) quad = QuadCfg<4096>::R * QuadCfg<4096>::FLAG_BYTES + QuadCfg<4096>::U_BYTES;
    return std::max(split, quad);
}

// TFHE_MI355_LARGE_SPLIT=1: the N = 32768, L = 2 CMUX through the split path (top_fwd / sub /
// top_inv) instead of the grouped one -- same Fourier key layout, same outputs (A/B switch)
static bool large_grouped_enabled() {
    static const bool v = [] {
        const char *e = std::getenv("TFHE_MI355_LARGE_SPLIT");
        return !(e && e[0] && e[0] != '0');
    }();
    return v;
}

// TFHE_MI355_DSUB=0: the classic L = 2 split CMUX at N <= 8192 through large_top_fwd +
// large_sub_kernel instead of the digits-fed path (A/B switch)
static bool large_dsub_enabled() {
    static const bool v = [] {
        const char *e = std::getenv("TFHE_MI355_DSUB");
        return !(e && e[0] == '0');
    }();
    return v;
}

// TFHE_MI355_SPLIT_FUSED=0: the digits-fed CMUX with separate large_top_inv and split_digits
// launches instead of split_inv_digits_kernel (A/B switch)
static bool split_fused_enabled() {
    static const bool v = [] {
        const char *e = std::getenv("TFHE_MI355_SPLIT_FUSED");
        return !(e && e[0] == '0');
    }();
    return v;
}

// TFHE_MI355_PAIR_SUB=1: the classic split CMUX (L <= 2) through large_pair_sub_kernel too (A/B)
static bool large_pair_sub_classic() {
    static const bool v = [] {
        const char *e = std::getenv("TFHE_MI355_PAIR_SUB");
        return e && e[0] && e[0] != '0';
    }();
    return v;
}

// The grouped N = 32768 CMUX on two CU-masked lanes (round 6).  Per chunk-CMUX the group kernel
// is FP64-bound (VALU busy 0.42) and the two streaming kernels (large_top_inv, large_digits: 43 % of
// the time) run at the Infinity-Cache streaming ceiling, one after the other on every CU.  Here two
// chunks A and B alternate: lane_c (most CUs) runs group(A, i) while lane_m (the other CUs) runs
// top_inv(B, i - 1) + digits(B, i), then the roles swap; cross-lane order by events.  Per lane the
// kernel sequence and its arguments are those of the one-stream path, so outputs are identical.
//   lane_m: init(A) digits(A,0) [dA]  init(B) digits(B,0) [dB]
//   per CMUX i:  lane_c: <dA> group(A,i) [gA]  <dB> group(B,i) [gB]
//                lane_m: <gA> top_inv(A,i) digits(A,i+1) [dA]  <gB> top_inv(B,i) digits(B,i+1) [dB]
//   lane_m: extract(A) extract(B); the launch stream waits for both lanes
static hipError_t launch_grouped_lanes(const LargePbsLaunch &a0, hipStream_t s, size_t per_ct) {
    constexpr int N = LN, K = 1;
    const int lchunk = (int)std::min<size_t>((size_t)a0.count, a0.scratch_bytes / per_ct / 2);
    if (lchunk <= 0) return hipErrorInvalidValue;
    hipStream_t C = a0.lane_c, Mst = a0.lane_m;
    hipEvent_t ev[5] = {};
    hipError_t e = hipSuccess;
    for (auto &x : ev)
        if ((e = hipEventCreateWithFlags(&x, hipEventDisableTiming)) != hipSuccess) return e;
    hipEvent_t &start = ev[0], &dA = ev[1], &dB = ev[2], &gA = ev[3], &gB = ev[4];
    (void)hipEventRecord(start, s);  // the caller's prior work (inputs, LUTs) before either lane
    (void)hipStreamWaitEvent(C, start, 0);
    (void)hipStreamWaitEvent(Mst, start, 0);
    LargePbsLaunch la[2] = {a0, a0};
    for (int l = 0; l < 2; l++) {
        la[l].levels = 2;
        la[l].acc = reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(a0.scratch) + (size_t)l * lchunk * per_ct);
        la[l].spectra = reinterpret_cast<double2 *>(reinterpret_cast<char *>(la[l].acc) +
                                                    (size_t)lchunk * (K + 1) * N * sizeof(uint64_t));
    }
    hipEvent_t *dev[2] = {&dA, &dB}, *gev[2] = {&gA, &gB};
    for (int ct0 = 0; ct0 < a0.count; ct0 += 2 * lchunk) {
        int c0[2], cnt[2];
        for (int l = 0; l < 2; l++) {
            c0[l] = ct0 + l * lchunk;
            cnt[l] = std::max(0, std::min(lchunk, a0.count - c0[l]));
            la[l].chunk_count = cnt[l];
        }
        const int lanes = cnt[1] > 0 ? 2 : 1;
        auto grp_blocks = [&](int l) { return (unsigned)((cnt[l] + 7) / 8) * 8 * 4 * GroupCfg::PARTS; };
        auto dig_blocks = [&](int l) { return (unsigned)((cnt[l] + 7) / 8) * 8 * (LM / LARGE_DIGT); };
        auto top_blocks = [&](int l) { return (unsigned)cnt[l] * (K + 1) * (1024 / TOPT); };
        for (int l = 0; l < lanes; l++) {
            const size_t init_elems = (size_t)cnt[l] * (K + 1) * N;
            hipLaunchKernelGGL((large_init_kernel<N, K>), dim3((unsigned)((init_elems + 255) / 256)), dim3(256), 0, Mst,
                               la[l], c0[l], cnt[l]);
            {
                TimedLaunch tl(a0.timer, "large_digits_kernel", Mst);
                hipLaunchKernelGGL(large_digits_kernel, dim3(dig_blocks(l)), dim3(LARGE_DIGT), 0, Mst, la[l], c0[l], 0);
            }
            (void)hipEventRecord(*dev[l], Mst);
        }
        for (int i = 0; i < a0.n; i++) {
            for (int l = 0; l < lanes; l++) {
                (void)hipStreamWaitEvent(C, *dev[l], 0);
                {
                    TimedLaunch tl(a0.timer, "large_group_cmux_kernel", C);
                    hipLaunchKernelGGL(large_group_cmux_kernel, dim3(grp_blocks(l)), dim3(GroupCfg::THREADS), GroupCfg::LDS, C,
                                       la[l], c0[l], i);
                }
                (void)hipEventRecord(*gev[l], C);
            }
            for (int l = 0; l < lanes; l++) {
                (void)hipStreamWaitEvent(Mst, *gev[l], 0);
                {
                    TimedLaunch tl(a0.timer, "large_top_inv_kernel", Mst);
                    hipLaunchKernelGGL((large_top_inv_kernel<N, K>), dim3(top_blocks(l)), dim3(TOPT), 0, Mst, la[l], c0[l], i);
                }
                if (i + 1 < a0.n) {
                    TimedLaunch tl(a0.timer, "large_digits_kernel", Mst);
                    hipLaunchKernelGGL(large_digits_kernel, dim3(dig_blocks(l)), dim3(LARGE_DIGT), 0, Mst, la[l], c0[l],
                                       i + 1);
                    (void)hipEventRecord(*dev[l], Mst);
                }
            }
        }
        for (int l = 0; l < lanes; l++) {
            const size_t out_elems = (size_t)cnt[l] * (K * N + 1);
            hipLaunchKernelGGL((large_extract_kernel<N, K>), dim3((unsigned)((out_elems + 255) / 256)), dim3(256), 0, Mst,
                               la[l], c0[l], cnt[l]);
        }
        // the next pair reuses both lanes' scratch: its init (lane_m) must follow this pair's last
        // group kernels (lane_c) -- lane_m already ran top_inv after them (gA / gB waits above)
    }
    (void)hipEventRecord(gA, C);
    (void)hipEventRecord(dA, Mst);
    (void)hipStreamWaitEvent(s, gA, 0);
    (void)hipStreamWaitEvent(s, dA, 0);
    e = hipGetLastError();
    for (auto &x : ev) (void)hipEventDestroy(x);
    return e;
}

// The quad CMUX over the batch in passes of quad_pass ciphertexts.  Its workgroups wait on each
// other, so two quad launches must never share the device's CUs: every launch of a device waits
// for the previous one (an event chained across streams under a process-wide lock).
template <int N, int L>
static hipError_t launch_quad(const LargePbsLaunch &a0, hipStream_t s) {
    using Cfg = QuadCfg<N>;
    static std::mutex mu;
    static hipEvent_t last[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(s, &cs);
    const bool capturing = cs != hipStreamCaptureStatusNone;
    // passes of at most quad_pass ciphertexts (one per R CUs) and of what the caller's scratch holds
    const int pass = (int)std::min<size_t>((size_t)a0.quad_pass, a0.scratch_bytes / (Cfg::R * Cfg::FLAG_BYTES + Cfg::U_BYTES));
    if (pass <= 0) return hipErrorInvalidValue;
    std::lock_guard<std::mutex> g(mu);
    if (!capturing && last[dev]) (void)hipStreamWaitEvent(s, last[dev], 0);
    for (int c0 = 0; c0 < a0.count; c0 += pass) {
        const int cnt = std::min(pass, a0.count - c0);
        hipError_t e = hipMemsetAsync(a0.scratch, 0, (size_t)cnt * Cfg::R * Cfg::FLAG_BYTES, s);  // the flags
        if (e != hipSuccess) return e;
        TimedLaunch tl(a0.timer, "quad_cmux_kernel", s);
        const dim3 grid((unsigned)((cnt + 7) / 8) * 8 * Cfg::R), block(Cfg::THREADS);
        if (a0.base_log * L <= 30)
            hipLaunchKernelGGL((quad_cmux_kernel<N, true, L>), grid, block, Cfg::LDS, s, a0, c0, cnt);
        else
            hipLaunchKernelGGL((quad_cmux_kernel<N, false, L>), grid, block, Cfg::LDS, s, a0, c0, cnt);
    }
    if (!capturing) {
        if (!last[dev]) (void)hipEventCreateWithFlags(&last[dev], hipEventDisableTiming);
        (void)hipEventRecord(last[dev], s);
    }
    return hipGetLastError();
}

template <int N, int K, int L, int G = 0>
static hipError_t launch_large_t(const LargePbsLaunch &a0, hipStream_t s) {
    using S = Split<N>;
    if (a0.count == 0) return hipSuccess;
    if constexpr (G == 0 && K == 1 && (L == 2 || L == 1) && (S::R == 4 || S::R == 2)) {  // quad (8192) / duo (4096)
        if (quad_enabled() && a0.count <= a0.quad_max_count) return launch_quad<N, L>(a0, s);
    }
    if constexpr (G == 0 && K == 1 && (L == 2 || L == 1) && (S::R == 4 || S::R == 2)) {
        if (onchip_enabled() && a0.count >= a0.onchip_min_count) {  // the whole blind rotation on chip, no scratch
            TimedLaunch tl(a0.timer, "onchip_cmux_kernel", s);
            const dim3 grid((unsigned)((a0.count + OnchipCfg<N>::CPW - 1) / OnchipCfg<N>::CPW)), block(OnchipCfg<N>::THREADS);
            if (a0.base_log * L <= 30)  // 32-bit digit extraction (every shortint set at these shapes)
                hipLaunchKernelGGL((onchip_cmux_kernel<N, true, L>), grid, block, OnchipCfg<N>::LDS, s, a0);
            else
                hipLaunchKernelGGL((onchip_cmux_kernel<N, false, L>), grid, block, OnchipCfg<N>::LDS, s, a0);
            return hipGetLastError();
        }
    }
    const size_t per_ct = large_pbs_scratch_per_ct(N, K, L);
    if constexpr (N == LN && K == 1 && L == 2 && G == 0) {
        if (LARGE_GROUP_SUB && large_grouped_enabled() && a0.lane_c && a0.lane_m)
            return launch_grouped_lanes(a0, s, per_ct);
    }
    const int chunk = (int)std::min<size_t>((size_t)a0.count, a0.scratch_bytes / per_ct);
    if (chunk <= 0) return hipErrorInvalidValue;
    LargePbsLaunch a = a0;
    a.levels = L;
    a.acc = reinterpret_cast<uint64_t *>(a0.scratch);
    a.spectra = reinterpret_cast<double2 *>(reinterpret_cast<char *>(a0.scratch) +
                                            (size_t)chunk * (K + 1) * N * sizeof(uint64_t));
    for (int ct0 = 0; ct0 < a.count; ct0 += chunk) {
        const int cnt = std::min(chunk, a.count - ct0);
        a.chunk_count = cnt;
        const size_t init_elems = (size_t)cnt * (K + 1) * N;
        hipLaunchKernelGGL((large_init_kernel<N, K>), dim3((unsigned)((init_elems + 255) / 256)), dim3(256), 0, s, a,
                           ct0, cnt);
        using Sub = LargeSubCfg<K, L>;
        const unsigned top_blocks = (unsigned)cnt * (K + 1) * (1024 / TOPT);
        const unsigned fwd_blocks = (unsigned)((cnt + 7) / 8) * 8 * (K + 1) * (1024 / TOPT);
        const size_t out_elems = (size_t)cnt * (K * N + 1);
        if constexpr (N == LN && K == 1 && L == 2 && G == 0) {
            if (LARGE_GROUP_SUB && large_grouped_enabled()) {
                const unsigned grp_blocks = (unsigned)((cnt + 7) / 8) * 8 * 4 * GroupCfg::PARTS;
                const unsigned dig_blocks = (unsigned)((cnt + 7) / 8) * 8 * (LM / LARGE_DIGT);
                for (int i = 0; i < a.n; i++) {
                    {
                        TimedLaunch tl(a.timer, "large_digits_kernel", s);
                        hipLaunchKernelGGL(large_digits_kernel, dim3(dig_blocks), dim3(LARGE_DIGT), 0, s, a, ct0, i);
                    }
                    {
                        TimedLaunch tl(a.timer, "large_group_cmux_kernel", s);
                        hipLaunchKernelGGL(large_group_cmux_kernel, dim3(grp_blocks), dim3(GroupCfg::THREADS),
                                           GroupCfg::LDS, s, a, ct0, i);
                    }
                    TimedLaunch tl(a.timer, "large_top_inv_kernel", s);
                    hipLaunchKernelGGL((large_top_inv_kernel<N, K>), dim3(top_blocks), dim3(TOPT), 0, s, a, ct0, i);
                }
                hipLaunchKernelGGL((large_extract_kernel<N, K>), dim3((unsigned)((out_elems + 255) / 256)), dim3(256),
                                   0, s, a, ct0, cnt);
                continue;
            }
        }
        // N = 4096 / 8192 only: at R = 8 the R-fold recomputation of the top stage in each
        // sub-block workgroup costs more than the spectra it saves (2_5: 2005 vs 2191 KS+PBS/s)
        if constexpr (G == 0 && K == 1 && L == 2 && S::R <= 4) {
            if (large_dsub_enabled()) {  // digits-fed CMUX: digits, sub-blocks from digits, top_inv
                constexpr int DPER = S::M / 256;
                const unsigned dig_blocks = (unsigned)((cnt + 7) / 8) * 8 * DPER;
                const unsigned dsub_blocks = (unsigned)((cnt + 7) / 8) * 8 * S::R;
                const unsigned fused_blocks = (unsigned)((cnt + 7) / 8) * 8 * 2;  // (ct, row)
                const bool fused = split_fused_enabled();
                for (int i = 0; i < a.n; i++) {
                    if (i == 0 || !fused) {
                        TimedLaunch tl(a.timer, "split_digits_kernel", s);
                        hipLaunchKernelGGL((split_digits_kernel<N>), dim3(dig_blocks), dim3(256), 0, s, a, ct0, i);
                    }
                    {
                        TimedLaunch tl(a.timer, "large_dsub_kernel", s);
                        hipLaunchKernelGGL((large_dsub_kernel<N>), dim3(dsub_blocks), dim3(Sub::THREADS), Sub::LDS, s,
                                           a, ct0, i);
                    }
                    if (fused && i + 1 < a.n) {  // top_inv of CMUX i + digits of CMUX i + 1
                        TimedLaunch tl(a.timer, "split_inv_digits_kernel", s);
                        hipLaunchKernelGGL((split_inv_digits_kernel<N>), dim3(fused_blocks), dim3(1024),
                                           sizeof(acc_pair) * S::M, s, a, ct0, i);
                        continue;
                    }
                    TimedLaunch tl(a.timer, "large_top_inv_kernel", s);
                    hipLaunchKernelGGL((large_top_inv_kernel<N, K, G>), dim3(top_blocks), dim3(TOPT), 0, s, a, ct0, i);
                }
                hipLaunchKernelGGL((large_extract_kernel<N, K>), dim3((unsigned)((out_elems + 255) / 256)), dim3(256),
                                   0, s, a, ct0, cnt);
                continue;
            }
        }
        const unsigned sub_blocks = (unsigned)cnt * S::R;
        const int steps = G ? a.n / G : a.n;  // CMUXes, or multi-bit groups
        const bool mb_fused = G > 0 && mb_fused_enabled();  // top_inv of group i + top_fwd of i + 1
        // packed digits between the fused inverse and the pair kernel (MB2_DIGITS)
        const bool mb_dig = N == 8192 && K == 1 && L == 2 && mb_fused && mb_pair2_enabled() && mb_digits_enabled(cnt) &&
                            a.base_log * 2 <= 30;
        for (int i = 0; i < steps; i++) {
            if (i == 0 && mb_dig) {
                TimedLaunch tl(a.timer, "mb_digits_init_kernel", s);
                hipLaunchKernelGGL((mb_digits_init_kernel<N>), dim3((unsigned)cnt * 8), dim3(256), 0, s, a, ct0);
            } else if (i == 0 || !mb_fused) {
                TimedLaunch tl(a.timer, "large_top_fwd_kernel", s);
                hipLaunchKernelGGL((large_top_fwd_kernel<N, K, L, G>), dim3(fwd_blocks), dim3(TOPT), 0, s, a, ct0, i);
            }
            if constexpr (G > 0) {
                // multi-bit: the paired kernel (3283 -> 8921 KS+PBS/s at
                // PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3; for the classic sets it measured slower
                // than large_sub_kernel: 4640 vs 4895 KS+PBS/s at 3_3, 939 vs 1036 at 4_4 split)
                using PairSub = PairSubCfg<K, L>;
                bool pair2 = false;
                if constexpr (N == 8192 && K == 1 && L == 2) {  // monomials from LDS (large_mb_pair2_kernel)
                    if (mb_pair2_enabled()) {
                        using P2 = MbPair2Cfg<N, G>;
                        TimedLaunch tl(a.timer, "large_mb_pair2_kernel", s);
                        if (mb_dig)
                            hipLaunchKernelGGL((large_mb_pair2_kernel<N, G, true>), dim3(pair_sub_blocks<S::R>((cnt + 1) / 2)),
                                               dim3(P2::THREADS), P2::LDS, s, a, ct0, i);
                        else
                            hipLaunchKernelGGL((large_mb_pair2_kernel<N, G, false>), dim3(pair_sub_blocks<S::R>((cnt + 1) / 2)),
                                               dim3(P2::THREADS), P2::LDS, s, a, ct0, i);
                        pair2 = true;
                    }
                }
                if (!pair2) {
                    TimedLaunch tl(a.timer, "large_pair_sub_kernel", s);
                    hipLaunchKernelGGL((large_pair_sub_kernel<N, K, L, G, 1>), dim3(pair_sub_blocks<S::R>((cnt + 1) / 2)),
                                       dim3(PairSub::THREADS), PairSub::LDS, s, a, ct0, i);
                }
            } else {
                bool paired = false;
                if constexpr (16 % (2 * (K + 1) * L) == 0) {  // L <= 2 at k = 1
                    if (large_pair_sub_classic()) {
                        using PairSub = PairSubCfg<K, L>;
                        TimedLaunch tl(a.timer, "large_pair_sub_kernel", s);
                        hipLaunchKernelGGL((large_pair_sub_kernel<N, K, L, G, 1>),
                                           dim3(pair_sub_blocks<S::R>((cnt + 1) / 2)), dim3(PairSub::THREADS),
                                           PairSub::LDS, s, a, ct0, i);
                        paired = true;
                    }
                }
                if (!paired) {
                    TimedLaunch tl(a.timer, "large_sub_kernel", s);
                    hipLaunchKernelGGL((large_sub_kernel<N, K, L>), dim3(sub_blocks), dim3(Sub::THREADS), Sub::LDS, s,
                                       a, ct0, i);
                }
            }
            if constexpr (G > 0) {
                if (mb_fused && i + 1 < steps) {
                    TimedLaunch tl(a.timer, "large_mb_inv_fwd_kernel", s);
                    bool dig_done = false;
                    if constexpr (N == 8192 && K == 1 && L == 2) {
                        if (mb_dig) {
                            hipLaunchKernelGGL((large_mb_inv_fwd_kernel<N, K, L, G, true>), dim3(fwd_blocks), dim3(TOPT), 0,
                                               s, a, ct0, i);
                            dig_done = true;
                        }
                    }
                    if (!dig_done)
                        hipLaunchKernelGGL((large_mb_inv_fwd_kernel<N, K, L, G, false>), dim3(fwd_blocks), dim3(TOPT), 0,
                                           s, a, ct0, i);
                    continue;
                }
            }
            TimedLaunch tl(a.timer, "large_top_inv_kernel", s);
            hipLaunchKernelGGL((large_top_inv_kernel<N, K, G>), dim3(top_blocks), dim3(TOPT), 0, s, a, ct0, i);
        }
        hipLaunchKernelGGL((large_extract_kernel<N, K>), dim3((unsigned)((out_elems + 255) / 256)), dim3(256), 0, s, a,
                           ct0, cnt);
    }
    return hipGetLastError();
}

template <int N>
static hipError_t launch_large_n(int L, const LargePbsLaunch &a, hipStream_t s) {
    switch (L) {
        case 1: return launch_large_t<N, 1, 1>(a, s);
        case 2: return launch_large_t<N, 1, 2>(a, s);
        case 3: return launch_large_t<N, 1, 3>(a, s);
        default: return hipErrorInvalidValue;
    }
}

// multi-bit through the split CMUX: the reference's multi-bit sets above N = 2048
// (PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_{2,3}_KS_PBS: N = 8192, L = 2, shortint/parameters/
// multi_bit.rs:134-153, 192-210)
bool large_multibit_supported(int N, int k, int L, int g) { return N == 8192 && k == 1 && L == 2 && (g == 2 || g == 3); }

hipError_t launch_large_pbs(int N, int k, int L, const LargePbsLaunch &a, hipStream_t s) {
    if (a.grouping) {
        if (!large_multibit_supported(N, k, L, a.grouping) || a.n % a.grouping) return hipErrorInvalidValue;
        return a.grouping == 2 ? launch_large_t<8192, 1, 2, 2>(a, s) : launch_large_t<8192, 1, 2, 3>(a, s);
    }
    if (!large_pbs_supported(N, k, L)) return hipErrorInvalidValue;
    switch (N) {
        case 4096: return launch_large_n<4096>(L, a, s);
        case 8192: return launch_large_n<8192>(L, a, s);
        case 16384: return launch_large_n<16384>(L, a, s);
        default: return launch_large_n<32768>(L, a, s);
    }
}

template <int N>
static hipError_t launch_mid_bsk(const uint64_t *std_polys, double2 *fourier, size_t npoly, const FftTables &t,
                                 hipStream_t s) {
    hipLaunchKernelGGL((mid_bsk_top_kernel<N>), dim3((unsigned)((npoly * 1024 + 255) / 256)), dim3(256), 0, s,
                       std_polys, fourier, t.wtop, t.twist, npoly);
    const size_t nblocks = npoly * Split<N>::R;
    const size_t lds = sizeof(double2) * (4 * SubFft::XL + SubFft::Lds::s1_len);
    hipLaunchKernelGGL((mid_bsk_sub_kernel<N>), dim3((unsigned)((nblocks + 3) / 4)), dim3(256), lds, s, fourier, t.W,
                       nblocks);
    return hipGetLastError();
}

hipError_t launch_large_bsk_to_fourier(const uint64_t *std_polys, double2 *fourier, size_t npoly,
                                       const FftTables &t, hipStream_t s) {
    if (npoly == 0) return hipSuccess;
    if (t.N == 4096) return launch_mid_bsk<4096>(std_polys, fourier, npoly, t, s);
    if (t.N == 8192) return launch_mid_bsk<8192>(std_polys, fourier, npoly, t, s);
    if (t.N == 16384) return launch_mid_bsk<16384>(std_polys, fourier, npoly, t, s);
    hipLaunchKernelGGL(large_bsk_to_fourier_kernel, dim3((unsigned)npoly), dim3(LT), LARGE_LDS, s, std_polys,
                       fourier, t.W, t.wtop, t.twist);
    return hipGetLastError();
}

}  // namespace tfhe_mi355
