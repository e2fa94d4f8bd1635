// pbs_classic.hip -- batched classic programmable bootstrap on gfx950.
//
// Replaces (reference tfhe-rs-odd, CPU Rust):
//   FourierLweBootstrapKeyView::blind_rotate_assign   fft64/crypto/bootstrap.rs:243-344
//   FourierLweBootstrapKeyView::bootstrap             fft64/crypto/bootstrap.rs:346-380
//   add_external_product_assign / update_with_fmadd   fft64/crypto/ggsw.rs:477-697
//   polynomial_wrapping_monic_monomial_{div,mul_and_subtract}
//                                                     algorithms/polynomial_algorithms.rs:219-490
//   fast_pbs_modulus_switch                           fft_impl/common.rs:26-43
//   extract_lwe_sample_from_glwe_ciphertext (deg 0)   algorithms/glwe_sample_extraction.rs:91-147
//   par_convert_polynomials_list_to_fourier           fft64/math/fft/mod.rs:719-764
// The fork's PATTERN msgpack dump (bootstrap.rs:340-342) is deliberately not reproduced.
//
// Design (DESIGN.md "Kernels"): one workgroup per ciphertext, one wavefront per GLWE
// polynomial (k+1 waves).  Each wave keeps its accumulator polynomial in registers (u64),
// rotates it through its LDS buffer, decomposes and forward-FFTs it (row r = wave); the (k+1)
// spectra are exchanged through LDS and wave c computes output column c = sum_r F_r * GGSW[r][c]
// (GGSW streamed from L2/HBM, 16 B per lane, coalesced, prefetched at the top of the CMUX),
// inverse-FFTs it and adds it back.  FFT twiddles and the twist live in LDS.
#include "engine.h"
#include "fft_device.h"

#ifndef PBS_WAVES_PER_EU
#define PBS_WAVES_PER_EU 1
#endif
#ifndef PBS_PREFETCH_GGSW
#define PBS_PREFETCH_GGSW 1
#endif

namespace tfhe_mi355 {

template <int LOG2N>
__device__ __forceinline__ uint32_t pbs_modulus_switch(uint64_t x) {
    uint64_t o = x >> (64 - LOG2N - 2);
    o += 1;
    o >>= 1;
    return (uint32_t)o;  // in [0, 2N]
}

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }

struct BlockSync {
    __device__ __forceinline__ void operator()() const { __syncthreads(); }
};

// digit extraction in 32-bit registers: valid when base_log * level <= 30 (all supported
// parameter sets).  Bit-identical digits to the 64-bit SignedDecomposer (decomposer.rs:99-119,
// iter.rs:134-141): the only divergence is the discarded final state when the rounding
// overflows, where every digit is 0 in both.
template <int L>
__device__ __forceinline__ uint32_t decomp_state32(uint64_t x, int beta) {
    const int shift = 63 - beta * L;  // >= 33
    uint32_t s = (uint32_t)((x >> 32) >> (shift - 32));
    return (s + 1) >> 1;
}
__device__ __forceinline__ int32_t decomp_digit32(uint32_t &state, int beta, uint32_t mask) {
    uint32_t res = state & mask;
    state >>= beta;
    uint32_t carry = ((res - 1) | state) & res;
    carry >>= beta - 1;
    state += carry;
    return (int32_t)(res - (carry << beta));
}

template <int M>
struct PbsLds {
    using Tw = typename WaveFft<M>::Lds;
    static constexpr int XL = xbuf_len(M);
    // layout (double2 units): [twist M][s1 table][s2 table][exchange (k+1) x XL]
    static constexpr int twist_off = 0;
    static constexpr int s1_off = M;
    static constexpr int s2_off = s1_off + Tw::s1_len;
    static constexpr int xbuf_off = ((s2_off + Tw::s2_len + 3) / 4) * 4;
    static constexpr size_t bytes(int waves) { return sizeof(double2) * (size_t)(xbuf_off + waves * XL); }
};

template <int N, int K, int L>
__global__ void __launch_bounds__(64 * (K + 1), PBS_WAVES_PER_EU) pbs_classic_kernel(ClassicPbsLaunch a) {
    constexpr int M = N / 2;
    constexpr int V = M / 64;
    constexpr int LOG2N = ilog2(N);
    using Fft = WaveFft<M>;
    using Lay = PbsLds<M>;
    constexpr int XL = Lay::XL;
    static_assert(sizeof(cx) * XL >= sizeof(uint64_t) * N, "exchange buffer holds one polynomial");

    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    double2 *s_twist = lds + Lay::twist_off;
    cx *xbuf = reinterpret_cast<cx *>(lds + Lay::xbuf_off);  // (K+1) * XL, one per wave

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int ct = blockIdx.x;
    const int n = a.n;
    const int beta = a.base_log;
    const uint32_t dmask = (1u << beta) - 1;
    const double norm = 1.0 / (double)M;
    BlockSync sync;

    // twiddles and twist -> LDS (once per workgroup)
    for (int e = threadIdx.x; e < M; e += blockDim.x) s_twist[e] = a.twist[e];
    Fft::Lds::template fill<M>(lds + Lay::s1_off, lds + Lay::s2_off, a.W, threadIdx.x, blockDim.x);
    const typename Fft::Lds tw{lds + Lay::s1_off, lds + Lay::s2_off};

    cx *xb = xbuf + wave * XL;
    uint64_t *xb64 = reinterpret_cast<uint64_t *>(xb);
    const uint64_t *in = a.lwe_in + (size_t)ct * (n + 1);
    const uint32_t li = a.lut_indexes ? a.lut_indexes[ct] : 0u;
    const uint64_t *lut = a.luts + (size_t)li * (K + 1) * N + (size_t)wave * N;

    // this wave's accumulator polynomial, in registers: c0[h] = position lane + 64 h
    // (h < V: j < M; h >= V: j = M + lane + 64 (h - V)).  ct0 = LUT / X^{b~}
    // (bootstrap.rs:255-275, polynomial_wrapping_monic_monomial_div)
    uint64_t c0[2 * V];
    {
        const uint32_t bt = pbs_modulus_switch<LOG2N>(in[n]);
        const int full = bt / N, rem = bt % N;
#pragma unroll
        for (int h = 0; h < 2 * V; h++) {
            const int src = lane + 64 * h + rem;
            const bool wrap = src >= N;
            uint64_t v = lut[wrap ? src - N : src];
            c0[h] = (wrap != (bool)(full & 1)) ? 0 - v : v;
        }
    }

    constexpr size_t ggsw_stride = (size_t)L * (K + 1) * (K + 1) * M;
    const double2 *gcol = a.fbsk + (size_t)wave * M + lane;  // column c = wave, this lane

    for (int i = 0; i < n; i++) {
        const uint64_t ai = in[i];
        if (ai == 0) continue;  // bootstrap.rs:285 (uniform across the workgroup)
        const uint32_t at = pbs_modulus_switch<LOG2N>(ai);
        const bool full_odd = (at / N) & 1;
        const int rem = at % N;

        // prefetch this CMUX's GGSW column (level L first, rows 0..k) -- 16 B per lane per slot
        const double2 *ggsw = gcol + (size_t)i * ggsw_stride;
        double2 g[K + 1][V];
        if (PBS_PREFETCH_GGSW)
#pragma unroll
        for (int r = 0; r <= K; r++)
#pragma unroll
            for (int s = 0; s < V; s++)
                g[r][s] = ggsw[((size_t)(L - 1) * (K + 1) * (K + 1) + (size_t)r * (K + 1)) * M + s * 64];

        // ct1 = X^{a~} ct0 - ct0 (polynomial_algorithms.rs:425-490) through the LDS buffer
        sync();
#pragma unroll
        for (int h = 0; h < 2 * V; h++) xb64[lane + 64 * h] = c0[h];
        sync();
        uint32_t st[2 * V];
#pragma unroll
        for (int h = 0; h < 2 * V; h++) {
            const int j = lane + 64 * h;
            const bool wrap = j < rem;  // (X^d p)[j] = -p[N-d+j] (j < d), p[j-d] otherwise
            uint64_t r = xb64[wrap ? N - rem + j : j - rem];
            r = (wrap != full_odd) ? 0 - r : r;
            st[h] = decomp_state32<L>(r - c0[h], beta);
        }

        cx acc[L > 1 ? V : 1];
#pragma unroll
        for (int lvl = L; lvl >= 1; lvl--) {
            if (lvl != L || !PBS_PREFETCH_GGSW) {  // (next level's) GGSW column
#pragma unroll
                for (int r = 0; r <= K; r++)
#pragma unroll
                    for (int s = 0; s < V; s++)
                        g[r][s] = ggsw[((size_t)(lvl - 1) * (K + 1) * (K + 1) + (size_t)r * (K + 1)) * M + s * 64];
            }
            cx v[V];
#pragma unroll
            for (int b = 0; b < V; b++) {
                const int32_t d0 = decomp_digit32(st[b], beta, dmask);
                const int32_t d1 = decomp_digit32(st[V + b], beta, dmask);
                const cx z = {(double)d0, (double)d1};
                const double2 w = s_twist[lane + 64 * b];
                v[b] = cmulw(z, w.x, w.y);  // convert_forward_integer (x86.rs:505-596)
            }
            Fft::forward(v, xb, tw, lane, sync);
            // publish this row's spectrum to the other waves
            sync();
#pragma unroll
            for (int s = 0; s < V; s++)
                reinterpret_cast<double2 *>(xb)[s * 64 + lane] = make_double2(v[s].re, v[s].im);
            sync();
            // output column c = wave: sum_r F_r * G[lvl][r][c]   (ggsw.rs:524-567, update_with_fmadd)
#pragma unroll
            for (int s = 0; s < V; s++) {
                cx o = (L > 1 && lvl != L) ? acc[L > 1 ? s : 0] : cx{0.0, 0.0};
#pragma unroll
                for (int r = 0; r <= K; r++) {
                    const double2 gg = g[r][s];
                    double2 ff;
                    if (r == wave) {
                        ff = make_double2(v[s].re, v[s].im);
                    } else {
                        ff = reinterpret_cast<const double2 *>(xbuf + r * XL)[s * 64 + lane];
                    }
                    if (lvl == L && r == 0) {
                        o.re = fma(gg.x, ff.x, -(gg.y * ff.y));
                        o.im = fma(gg.x, ff.y, gg.y * ff.x);
                    } else {
                        o.re = fma(gg.x, ff.x, fma(-gg.y, ff.y, o.re));
                        o.im = fma(gg.x, ff.y, fma(gg.y, ff.x, o.im));
                    }
                }
                if constexpr (L > 1) acc[s] = o;
                else v[s] = o;
            }
            if constexpr (L == 1) {
                Fft::inverse(v, xb, tw, lane, sync);
#pragma unroll
                for (int b = 0; b < V; b++) {
                    uint64_t dre, dim;
                    const double2 w = s_twist[lane + 64 * b];
                    backward_convert(v[b], cx{norm * w.x, norm * w.y}, dre, dim);
                    c0[b] += dre;
                    c0[V + b] += dim;
                }
            }
        }
        if constexpr (L > 1) {
            Fft::inverse(acc, xb, tw, lane, sync);
#pragma unroll
            for (int b = 0; b < V; b++) {
                uint64_t dre, dim;
                const double2 w = s_twist[lane + 64 * b];
                backward_convert(acc[b], cx{norm * w.x, norm * w.y}, dre, dim);
                c0[b] += dre;
                c0[V + b] += dim;
            }
        }
    }

    // sample extract at degree 0 (glwe_sample_extraction.rs:91-147)
    uint64_t *out = a.lwe_out + (size_t)ct * (K * N + 1);
    sync();
#pragma unroll
    for (int h = 0; h < 2 * V; h++) xb64[lane + 64 * h] = c0[h];
    sync();
    if (wave < K) {
        for (int j = lane; j < N; j += 64) out[wave * N + j] = j == 0 ? xb64[0] : 0 - xb64[N - j];
    } else if (lane == 0) {
        out[K * N] = c0[0];
    }
}

template <int N, int K, int L>
static hipError_t launch_pbs_t(const ClassicPbsLaunch &a, hipStream_t s) {
    constexpr int M = N / 2;
    const size_t lds = PbsLds<M>::bytes(K + 1);
    if (a.count == 0) return hipSuccess;
    hipLaunchKernelGGL((pbs_classic_kernel<N, K, L>), dim3(a.count), dim3(64 * (K + 1)), lds, s, a);
    return hipGetLastError();
}

bool classic_pbs_supported(int N, int k, int L) {
    if (k != 1) return false;
    if (N == 2048) return L == 1 || L == 2;
    if (N == 1024) return L == 1 || L == 2;
    return false;
}

hipError_t launch_classic_pbs(int N, int k, int L, const ClassicPbsLaunch &a, hipStream_t s) {
    if (k == 1 && N == 2048 && L == 1) return launch_pbs_t<2048, 1, 1>(a, s);
    if (k == 1 && N == 2048 && L == 2) return launch_pbs_t<2048, 1, 2>(a, s);
    if (k == 1 && N == 1024 && L == 1) return launch_pbs_t<1024, 1, 1>(a, s);
    if (k == 1 && N == 1024 && L == 2) return launch_pbs_t<1024, 1, 2>(a, s);
    return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------
// standard -> Fourier BSK (forward_as_torus, fft/mod.rs:197-218 + 378-385): one wave per
// polynomial; output in the engine layout [poly][slot*64 + lane].
// ---------------------------------------------------------------------------------------
template <int N>
__global__ void __launch_bounds__(64) bsk_to_fourier_kernel(const uint64_t *__restrict__ polys,
                                                            double2 *__restrict__ out, size_t npoly,
                                                            const double2 *__restrict__ W,
                                                            const double2 *__restrict__ twist) {
    constexpr int M = N / 2;
    constexpr int V = M / 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cx *xb = reinterpret_cast<cx *>(smem);
    const int lane = threadIdx.x;
    const size_t p = blockIdx.x;
    if (p >= npoly) return;  // whole (single-wave) block exits together
    const uint64_t *x = polys + p * N;
    cx v[V];
#pragma unroll
    for (int b = 0; b < V; b++) {
        const int j = lane + 64 * b;
        double xr = (double)(int64_t)x[j] * 0x1p-64;
        double xi = (double)(int64_t)x[j + M] * 0x1p-64;
        cx w = gld(twist + j);
        v[b].re = xr * w.re - xi * w.im;
        v[b].im = xr * w.im + xi * w.re;
    }
    WaveFft<M>::forward(v, xb, GlobalTwiddles<M>{W}, lane, BlockSync{});
    double2 *o = out + p * M + lane;
#pragma unroll
    for (int s = 0; s < V; s++) o[s * 64] = make_double2(v[s].re, v[s].im);
}

hipError_t launch_bsk_to_fourier(int N, const uint64_t *std_polys, double2 *fourier, size_t npoly,
                                 const FftTables &t, hipStream_t s) {
    if (npoly == 0) return hipSuccess;
    if (N == 2048) {
        hipLaunchKernelGGL(bsk_to_fourier_kernel<2048>, dim3(npoly), dim3(64),
                           sizeof(cx) * xbuf_len(1024), s, std_polys, fourier, npoly, t.W, t.twist);
    } else if (N == 1024) {
        hipLaunchKernelGGL(bsk_to_fourier_kernel<1024>, dim3(npoly), dim3(64),
                           sizeof(cx) * xbuf_len(512), s, std_polys, fourier, npoly, t.W, t.twist);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace tfhe_mi355
