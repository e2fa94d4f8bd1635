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
// polynomial (k+1 waves).  The accumulator GLWE lives in LDS as u64; each wave rotates,
// decomposes and forward-FFTs its own polynomial (row r = wave), the (k+1) spectra are
// exchanged through LDS, and wave c computes output column c = sum_r F_r * GGSW[r][c]
// (GGSW streamed from HBM/L2, 16 B per lane, coalesced), inverse-FFTs it and adds it back.
#include "engine.h"
#include "fft_device.h"

namespace tfhe_mi355 {

__device__ __forceinline__ uint64_t closest_representable(uint64_t x, int base_log, int level) {
    int shift = 64 - base_log * level - 1;
    uint64_t res = x >> shift;
    res += 1;
    res &= ~(uint64_t)1;
    return res << shift;
}

__device__ __forceinline__ uint64_t decompose_one_level(int base_log, uint64_t &state, uint64_t mask) {
    uint64_t res = state & mask;
    state >>= base_log;
    uint64_t carry = ((res - 1) | state) & res;
    carry >>= base_log - 1;
    state += carry;
    return res - (carry << base_log);
}

template <int LOG2N>
__device__ __forceinline__ uint32_t pbs_modulus_switch(uint64_t x) {
    uint64_t o = x >> (64 - LOG2N - 2);
    o += 1;
    o >>= 1;
    return (uint32_t)o;  // in [0, 2N]
}

// (X^d * p)[j] for d = full*N + rem, full in {0,1,2}
__device__ __forceinline__ uint64_t rotated_coeff(const uint64_t *p, int N, int j, int rem, int full_odd) {
    uint64_t v;
    if (j < rem) {
        v = p[N - rem + j];
        v = full_odd ? v : 0 - v;
    } else {
        v = p[j - rem];
        v = full_odd ? 0 - v : v;
    }
    return v;
}

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }

struct BlockSync {
    __device__ __forceinline__ void operator()() const { __syncthreads(); }
};

template <int N, int K, int L>
__global__ void __launch_bounds__(64 * (K + 1)) pbs_classic_kernel(ClassicPbsLaunch a) {
    constexpr int M = N / 2;
    constexpr int V = M / 64;
    constexpr int LOG2N = ilog2(N);
    constexpr int XL = xbuf_len(M);
    using Fft = WaveFft<M>;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    cx *xbuf = reinterpret_cast<cx *>(smem);                              // (K+1) * XL
    uint64_t *ct0 = reinterpret_cast<uint64_t *>(smem + sizeof(cx) * (K + 1) * XL);  // (K+1) * N

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int ct = blockIdx.x;
    const int n = a.n;
    const int beta = a.base_log;
    const uint64_t dmask = (1ULL << beta) - 1;
    BlockSync sync;

    uint64_t *my = ct0 + wave * N;
    cx *xb = xbuf + wave * XL;
    const uint64_t *in = a.lwe_in + (size_t)ct * (n + 1);
    const uint32_t li = a.lut_indexes ? a.lut_indexes[ct] : 0u;
    const uint64_t *lut = a.luts + (size_t)li * (K + 1) * N + (size_t)wave * N;

    // ct0 = LUT / X^{b~}  (bootstrap.rs:255-275)
    {
        const uint32_t bt = pbs_modulus_switch<LOG2N>(in[n]);
        const int full = bt / N, rem = bt % N;
        for (int j = lane; j < N; j += 64) {
            int src = j + rem;
            uint64_t v = src < N ? lut[src] : 0 - lut[src - N];
            my[j] = (full & 1) ? 0 - v : v;
        }
    }
    sync();

    // twist factors for this lane's positions j = lane + 64 b
    const double2 *__restrict__ fbsk = a.fbsk;
    constexpr size_t ggsw_stride = (size_t)L * (K + 1) * (K + 1) * M;

    for (int i = 0; i < n; i++) {
        const uint64_t ai = in[i];
        if (ai == 0) continue;  // bootstrap.rs:285 (uniform across the workgroup)
        const uint32_t at = pbs_modulus_switch<LOG2N>(ai);
        const int full_odd = (at / N) & 1;
        const int rem = at % N;

        // ct1 = X^{a~} ct0 - ct0 for this wave's polynomial, rounded + decomposition states
        uint64_t st[2 * V];
#pragma unroll
        for (int b = 0; b < V; b++) {
            const int j0 = lane + 64 * b, j1 = j0 + M;
            uint64_t x0 = rotated_coeff(my, N, j0, rem, full_odd) - my[j0];
            uint64_t x1 = rotated_coeff(my, N, j1, rem, full_odd) - my[j1];
            st[2 * b] = closest_representable(x0, beta, L) >> (64 - beta * L);
            st[2 * b + 1] = closest_representable(x1, beta, L) >> (64 - beta * L);
        }

        cx acc[V];
        const double2 *ggsw = fbsk + (size_t)i * ggsw_stride;
#pragma unroll
        for (int lvl = L; lvl >= 1; lvl--) {
            cx v[V];
#pragma unroll
            for (int b = 0; b < V; b++) {
                const int j0 = lane + 64 * b;
                uint64_t d0 = decompose_one_level(beta, st[2 * b], dmask);
                uint64_t d1 = decompose_one_level(beta, st[2 * b + 1], dmask);
                cx z = {(double)(int64_t)d0, (double)(int64_t)d1};
                cx w = gld(a.twist + j0);
                v[b] = cmulw(z, w.re, w.im);
            }
            Fft::forward(v, xb, a.W, lane, sync);
            // publish this row's spectrum
#pragma unroll
            for (int s = 0; s < V; s++) {
                reinterpret_cast<double2 *>(xb)[s * 64 + lane] = make_double2(v[s].re, v[s].im);
            }
            sync();
            // output column c = wave: acc += sum_r F_r * G[lvl][r][c]   (ggsw.rs:524-567)
            const double2 *lm = ggsw + (size_t)(lvl - 1) * (K + 1) * (K + 1) * M;
#pragma unroll
            for (int r = 0; r <= K; r++) {
                const double2 *g = lm + ((size_t)r * (K + 1) + wave) * M + lane;
                const double2 *fr = reinterpret_cast<const double2 *>(xbuf + r * XL) + lane;
                const bool first = (lvl == L) && (r == 0);
#pragma unroll
                for (int s = 0; s < V; s++) {
                    double2 gg = g[s * 64];
                    double2 ff = fr[s * 64];
                    if (first) {
                        acc[s].re = fma(gg.x, ff.x, -(gg.y * ff.y));
                        acc[s].im = fma(gg.x, ff.y, gg.y * ff.x);
                    } else {
                        acc[s].re = fma(gg.x, ff.x, fma(-gg.y, ff.y, acc[s].re));
                        acc[s].im = fma(gg.x, ff.y, fma(gg.y, ff.x, acc[s].im));
                    }
                }
            }
            sync();
        }

        Fft::inverse(acc, xb, a.W, lane, sync);
        // acc[b] = position lane + 64 b; add back as torus (fft/mod.rs:487-494)
#pragma unroll
        for (int b = 0; b < V; b++) {
            const int j0 = lane + 64 * b;
            uint64_t dre, dim;
            backward_convert(acc[b], gld(a.twist_inv + j0), dre, dim);
            my[j0] += dre;
            my[j0 + M] += dim;
        }
        sync();
    }

    // sample extract at degree 0 (glwe_sample_extraction.rs:91-147)
    uint64_t *out = a.lwe_out + (size_t)ct * (K * N + 1);
    if (wave < K) {
        for (int j = lane; j < N; j += 64) out[wave * N + j] = j == 0 ? my[0] : 0 - my[N - j];
    } else if (lane == 0) {
        out[K * N] = my[0];
    }
}

template <int N, int K, int L>
static hipError_t launch_pbs_t(const ClassicPbsLaunch &a, hipStream_t s) {
    constexpr int M = N / 2;
    size_t lds = sizeof(cx) * (K + 1) * xbuf_len(M) + sizeof(uint64_t) * (K + 1) * N;
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
struct WaveSync {
    __device__ __forceinline__ void operator()() const { __syncthreads(); }
};

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
    WaveFft<M>::forward(v, xb, W, lane, WaveSync{});
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
