// pbs_latency.hip -- latency form of the classic PBS at N = 2048, k = 1, L = 1 (the 2_2 shape):
// ONE ciphertext per workgroup of 8 wavefronts, each GLWE polynomial's 1024-point FFT spread over
// four of them.
//
// Replaces the same reference functions as pbs_classic.hip (FourierLweBootstrapKeyView::
// bootstrap, fft64/crypto/bootstrap.rs:243-380; add_external_product_assign, ggsw.rs:477-697;
// fast_pbs_modulus_switch, fft_impl/common.rs:26-43; extract_lwe_sample_from_glwe_ciphertext,
// glwe_sample_extraction.rs:91-147) for the calling pattern of the reference itself: a handful
// of ciphertexts per call (keyswitch_programmable_bootstrap_assign bootstraps ONE ciphertext,
// shortint/server_key/mod.rs:783-857, from each rayon worker, radix_parallel/mul.rs:347-407).
// The throughput kernel puts a ciphertext on 2 waves (one per GLWE row) and needs four of them
// per CU to fill its SIMDs; alone on a CU its 742 dependent CMUXes take ~5.9 ms.  Here the 8 waves
// of a CU all work on one ciphertext, so a batch of up to 256 ciphertexts (one per CU) finishes
// in the time of one CMUX chain at 4x the per-CMUX parallelism.
//
// Same FFT DAG as WaveFft<1024> and the oracle ([16, 16, 4] DIF forward / mirrored DIT inverse,
// same twiddle products and fma forms, same MAC order), so outputs are bit-identical to the
// throughput kernel and to oracle/pbs_oracle.c.  Work split of one row's transform (waves
// w = 0..3 of that row; lane = 16 lrow + col):
//   stage 1 (R16, stride 64): butterfly a = 16 w + col, split over the four 16-lane rows as in
//     WaveFft<256> (in-row radix 4, row twiddles, v_permlane transpose, radix 4): lane holds
//     z[a + 64 (lrow + 4 j)], j < 4, and leaves output C = lrow + 4 q -> LDS X[a + 64 C];
//   stage 2 (R16 on blocks of 64, stride 4): block cc = 4 w + (col >> 2), a1 = col & 3, same
//     row split -> LDS Y[64 cc + a1 + 4 C2];
//   stage 3 (R4 on blocks of 4) is computed by the MAC lane that owns the block, for both rows
//     (the MAC needs both rows' spectra anyway): block t = 16 cc' + C2', cc' = 4 w + (col & 3),
//     C2' = lrow + 4 (col >> 2), positions 4 t + e, e < 4;
//   the inverse mirrors it; the stage-3 inverse output goes back to stage-2 lanes through this
//     wave's own quarter of X (wave-private, no barrier).
// Four workgroup barriers per CMUX: accumulator -> rotation gather, stage 1 -> 2, stage 2 -> MAC,
// inverse stage 2 -> 1.
#include "engine.h"
#include "pbs_common.h"

namespace tfhe_mi355 {

namespace {

constexpr int LAT_N = 2048, LAT_M = 1024;
// LDS layout in double2 units: stage-1 twiddles W[a C] as [C][a] (C, a < 16 x 64), stage-2
// twiddles W[16 a1 C2] as [C2][a1], the twist, per GLWE row an exchange buffer X (stages 1/2) and
// a buffer Y (stage-2 outputs, and the accumulator pairs of the rotation).
struct LatLds {
    static constexpr int twf = 0;
    static constexpr int tw2 = twf + 16 * 64;
    static constexpr int twist = tw2 + 16 * 4;
    static constexpr int X = twist + LAT_M;
    static constexpr int Y = X + 2 * LAT_M;
    static constexpr int end = Y + 2 * LAT_M;
    static constexpr size_t bytes = sizeof(double2) * end;
};
static_assert(LatLds::bytes <= 160 * 1024, "latency PBS LDS exceeds a CU");

__device__ __forceinline__ cx ld2(const double2 *p) {
    const double2 t = *p;
    return {t.x, t.y};
}
__device__ __forceinline__ void st2(double2 *p, cx v) { *p = make_double2(v.re, v.im); }

}  // namespace

__global__ void __launch_bounds__(512, 2) pbs_latency_kernel(ClassicPbsLaunch a) {
    constexpr int N = LAT_N, M = LAT_M, K = 1, LOG2N = 11;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *lds = reinterpret_cast<double2 *>(smem);
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int row = wid >> 2;     // GLWE polynomial this wave transforms (and MAC output column)
    const int w = wid & 3;        // quarter of that polynomial's transform
    const int lane0 = tid & 63;

    // tables: W[a C] (C = 0 row = W[0] = (1, -0): value-identical to the oracle's skipped multiply)
    for (int e = tid; e < 16 * 64; e += 512) lds[LatLds::twf + e] = a.W[(e & 63) * (e >> 6)];
    if (tid < 64) lds[LatLds::tw2 + tid] = a.W[16 * (tid & 3) * (tid >> 2)];
    for (int e = tid; e < M; e += 512) lds[LatLds::twist + e] = a.twist[e];

    const int ct = blockIdx.x;
    const int n = a.n;
    const uint64_t *in = a.lwe_in + (size_t)ct * (n + 1);
    const __attribute__((address_space(4))) uint64_t *in_s = (const __attribute__((address_space(4))) uint64_t *)(
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)in >> 32)) << 32) |
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)in));
    const uint32_t li = a.lut_indexes ? min(a.lut_indexes[ct], a.lut_count - 1u) : 0u;
    const uint64_t *lut = a.luts + (size_t)li * (K + 1) * N + (size_t)row * N;
    const DigitL1 digit_l1(a.base_log);

    // this lane's accumulator coefficients: j_q = a1 + 64 (lrow + 4 q) (a1 = 16 w + col) and j_q + M
    // (the stage-1 input positions and the backward conversion's output positions)
    uint64_t lo[4], hi[4];
    {
        const uint32_t bt = pbs_modulus_switch<LOG2N>(in[n]);
        const int full = bt / N, rem = bt % N;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int j = 16 * w + (lane0 & 15) + 64 * (lane0 >> 4) + 256 * q;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int src = j + h * M + rem;
                const bool wrap = src >= N;
                const uint64_t v = lut[wrap ? src - N : src];
                const uint64_t c = (wrap != (bool)(full & 1)) ? 0 - v : v;
                (h ? hi : lo)[q] = c;
            }
        }
    }
    __syncthreads();  // tables

    const double2 *twf = lds + LatLds::twf;
    const double2 *tw2 = lds + LatLds::tw2;
    const double2 *s_twist = lds + LatLds::twist;
    double2 *X = lds + LatLds::X + row * M;
    double2 *Y = lds + LatLds::Y + row * M;
    // accumulator pairs (acc[p], acc[p + M]) in Y between CMUXes (Y's stage-2 outputs are dead then)
    uint64_t *A64 = reinterpret_cast<uint64_t *>(Y);
    constexpr size_t ggsw_stride = (size_t)(K + 1) * (K + 1) * M;
    const double k32 = torus_k32();

    for (int i = 0; i < n; i++) {
        int lane = lane0;  // opaque per-iteration copy: lane-derived addresses are not hoisted
        asm volatile("" : "+v"(lane));
        const int lrow = lane >> 4, col = lane & 15;
        const uint32_t at = pbs_modulus_switch<LOG2N>(in_s[i]);
        const bool full_odd = (at / N) & 1;
        const int rem = at % N;

        // ---- accumulator -> LDS pairs, rotation gather, ct1 = X^at acc - acc, digits, twist ----
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int j = 16 * w + col + 64 * lrow + 256 * q;
            A64[2 * j] = lo[q];
            A64[2 * j + 1] = hi[q];
        }
        __syncthreads();  // (A) every wave's pairs written
        cx v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int j = 16 * w + col + 64 * lrow + 256 * q;
            // (X^rem p) at j and j + M from ONE pair: u = j - rem, s = u mod M; u >= 0: (lo, hi);
            // -M <= u < 0: (-hi, lo) (X^M acts as i on the fold); u < -M: (-lo, -hi)
            const int u = j - rem;
            const int s = u & (M - 1);
            const uint64_t plo = A64[2 * s], phi = A64[2 * s + 1];
            const bool swap = u < 0 && u >= -M;
            const bool n0 = (u < 0) != full_odd, n1 = (u < -M) != full_odd;
            const uint64_t x0 = swap ? phi : plo, x1 = swap ? plo : phi;
            const uint64_t r0 = n0 ? 0 - x0 : x0, r1 = n1 ? 0 - x1 : x1;
            const int32_t d0 = digit_l1((uint32_t)((r0 - lo[q]) >> 32));
            const int32_t d1 = digit_l1((uint32_t)((r1 - hi[q]) >> 32));
            const double2 tw = s_twist[j];
            v[q] = cmulw(cx{(double)d0, (double)d1}, tw.x, tw.y);  // convert_forward_integer (x86.rs:505-596)
        }

        // ---- forward stage 1: butterfly a1 = 16 w + col, column lrow ----
        dft16_fwd_rows(v, lrow);
        {
            const int a1 = 16 * w + col;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int C = lrow + 4 * q;
                const double2 t = twf[C * 64 + a1];
                st2(X + a1 + 64 * C, cmulw(v[q], t.x, t.y));
            }
        }
        __syncthreads();  // (B)
        // ---- forward stage 2: block cc = 4 w + (col >> 2), butterfly a2 = col & 3 ----
        {
            const int cc = 4 * w + (col >> 2), a2 = col & 3;
#pragma unroll
            for (int q = 0; q < 4; q++) v[q] = ld2(X + 64 * cc + a2 + 4 * (lrow + 4 * q));
            dft16_fwd_rows(v, lrow);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int C2 = lrow + 4 * q;
                const double2 t = tw2[C2 * 4 + a2];
                st2(Y + 64 * cc + a2 + 4 * C2, cmulw(v[q], t.x, t.y));
            }
        }
        __syncthreads();  // (C) both rows' stage-2 outputs
        // ---- stage 3 of both rows + MAC of output column `row` on block t ----
        const int ccm = 4 * w + (col & 3), xm = col >> 2;
        const int tb = 64 * ccm + 4 * (lrow + 4 * xm);  // first position of block t
        cx o[4];
        {
            // GGSW elements of positions tb + e in the engine layout (element s*64 + L <-> position
            // 64 (L & 15) + 16 (L >> 4) + s): (4 lrow + e) 64 + 16 xm + ccm
            const double2 *g = a.fbsk + (size_t)i * ggsw_stride + (size_t)row * M + 256 * lrow + 16 * xm + ccm;
#pragma unroll
            for (int rr = 0; rr <= K; rr++) {
                const double2 *Yr = lds + LatLds::Y + rr * M + tb;
                cx f0 = ld2(Yr), f1 = ld2(Yr + 1), f2 = ld2(Yr + 2), f3 = ld2(Yr + 3);
                r4_fwd(f0, f1, f2, f3);
                const cx f[4] = {f0, f1, f2, f3};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const double2 gg = g[(size_t)rr * (K + 1) * M + 64 * e];
                    const double2 ff = make_double2(f[e].re, f[e].im);
                    if (rr == 0) {  // update_with_fmadd (ggsw.rs:524-567), the throughput kernel's form
                        o[e].re = fma(gg.x, ff.x, -(gg.y * ff.y));
                        o[e].im = fma(gg.x, ff.y, gg.y * ff.x);
                    } else {
                        o[e].re = fma(gg.x, ff.x, fma(-gg.y, ff.y, o[e].re));
                        o[e].im = fma(gg.x, ff.y, fma(gg.y, ff.x, o[e].im));
                    }
                }
            }
        }
        // ---- inverse stage 3 (R4 on the block), back to the stage-2 lanes through this wave's
        //      own quarter of X (positions 256 w .. 256 w + 255: written and read by this wave only)
        r4_inv(o[0], o[1], o[2], o[3]);
#pragma unroll
        for (int e = 0; e < 4; e++) st2(X + tb + e, o[e]);
        WaveLocalSync{}();
        {
            const int cc = 4 * w + (col >> 2), a2 = col & 3;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int C2 = lrow + 4 * q;
                const double2 t = tw2[C2 * 4 + a2];
                v[q] = cmulw(ld2(X + 64 * cc + a2 + 4 * C2), t.x, -t.y);
            }
            dft16_inv_rows(v, lrow);
            WaveLocalSync{}();
#pragma unroll
            for (int q = 0; q < 4; q++) st2(X + 64 * cc + a2 + 4 * (lrow + 4 * q), v[q]);
        }
        __syncthreads();  // (D)
        // ---- inverse stage 1 + backward conversion into the accumulator ----
        {
            const int a1 = 16 * w + col;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int C = lrow + 4 * q;
                const double2 t = twf[C * 64 + a1];
                v[q] = cmulw(ld2(X + a1 + 64 * C), t.x, -t.y);
            }
            dft16_inv_rows(v, lrow);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int j = a1 + 64 * lrow + 256 * q;
                const double2 tw = s_twist[j];  // the resident key carries the 1/M
                backward_add(v[q], cx{tw.x, tw.y}, lo[q], hi[q], k32);
            }
        }
    }

    // ---- output ----
    const int lrow = lane0 >> 4, col = lane0 & 15;
    if (a.glwe_out) {  // bootstrap_without_sample_extract (fork, bootstrap.rs:383-412)
        uint64_t *g = a.lwe_out + ((size_t)ct * (K + 1) + row) * N;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int j = 16 * w + col + 64 * lrow + 256 * q;
            g[j] = lo[q];
            g[j + M] = hi[q];
        }
        return;
    }
    // sample extract at degree 0 (glwe_sample_extraction.rs:91-147): mask j = -acc0[N - j] (j > 0)
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int j = 16 * w + col + 64 * lrow + 256 * q;
        A64[2 * j] = lo[q];
        A64[2 * j + 1] = hi[q];
    }
    __syncthreads();
    uint64_t *out = a.lwe_out + (size_t)ct * (K * N + 1);
    if (row < K) {
        const uint64_t *A0 = reinterpret_cast<const uint64_t *>(lds + LatLds::Y + row * M);
        for (int j = tid & 255; j < N; j += 256) {
            uint64_t x;
            if (j == 0) {
                x = A0[0];
            } else {
                const int src = N - j;  // acc0[src]: pair (src mod M), lo below M, hi above
                x = 0 - A0[2 * (src & (M - 1)) + (src >= M)];
            }
            out[(size_t)row * N + j] = x;
        }
    } else if (tid == 256 * K) {
        out[K * N] = lo[0];  // body = acc_k[0]: j = 0 lives in lane 0 of wave 0 of row k (q = 0)
    }
}

bool latency_pbs_supported(int N, int k, int L) { return N == 2048 && k == 1 && L == 1; }

hipError_t launch_latency_pbs(const ClassicPbsLaunch &a, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    hipLaunchKernelGGL(pbs_latency_kernel, dim3(a.count), dim3(512), LatLds::bytes, s, a);
    return hipGetLastError();
}

}  // namespace tfhe_mi355
