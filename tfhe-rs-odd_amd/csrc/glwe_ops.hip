// glwe_ops.hip -- GLWE x plaintext-polynomial products for the fork's gadget layer.
//
//   out[c][i] = sum_{j<J} glwe_in[c][j] * polys[i][j]      (Z/2^64)[X]/(X^N+1), per GLWE polynomial
//
// with an optional degree-0 sample extraction of each product.  Replaces, bit for bit:
//   MVB:  accu_i = v0 * v_i by polynomial_karatsuba_wrapping_mul, then
//         extract_lwe_sample_from_glwe_ciphertext(.., MonomialDegree(0))
//         (gadget/engine/bootstrapping.rs:567-620; polynomial_algorithms.rs:683-742)
//   tree packing: sum over the Z_p windows of monomial-shifted packed GLWEs,
//         polynomial_wrapping_monic_monomial_mul_assign + slice_wrapping_add_assign
//         (bootstrapping.rs:690-773): the window sums are products with 0/1/-1 polynomials.
// Products over Z/2^64 are exact whatever the algorithm, so a direct sum over the nonzero
// coefficients of polys[i] (p of them for an MVB v_i, N for a window set) equals the Karatsuba
// result.  One workgroup per (ciphertext, output): the nonzeros of polys[i] are compacted into LDS
// window by window (atomic slots: the order of a wrapping sum does not matter), then every thread
// accumulates 8 output words per tile, reading the input GLWE coalesced from L2.
#include "engine.h"

namespace tfhe_mi355 {

namespace {
constexpr int GPM_THREADS = 256;
constexpr int GPM_R = 8;      // output words per thread per tile
constexpr int GPM_CH = 2048;  // polynomial coefficients scanned per LDS compaction window
}  // namespace

__global__ void __launch_bounds__(GPM_THREADS) glwe_poly_mul_kernel(GlwePolyMulLaunch a) {
    __shared__ uint32_t nz_pos[GPM_CH];
    __shared__ uint64_t nz_val[GPM_CH];
    __shared__ int nz_count;
    const int tid = threadIdx.x;
    const size_t item = blockIdx.x;  // c * npoly + i
    const size_t c = item / (size_t)a.npoly;
    const int i = (int)(item % (size_t)a.npoly);
    const int N = a.N, k = a.k, log2N = __builtin_ctz((unsigned)N);
    const size_t glwe = (size_t)(k + 1) * N;
    const uint64_t *in = a.glwe_in + c * (size_t)a.J * glwe;
    const uint64_t *poly = a.polys + (size_t)i * a.J * N;
    const size_t total = (size_t)a.J * N;
    const int out_len = a.extract ? k * N + 1 : (k + 1) * N;
    uint64_t *out = a.out + item * (size_t)out_len;

    for (int tile = 0; tile < out_len; tile += GPM_THREADS * GPM_R) {
        // output word e -> (GLWE polynomial, coefficient m, negate?)
        int src_off[GPM_R], m[GPM_R];
        bool neg_out[GPM_R];
#pragma unroll
        for (int r = 0; r < GPM_R; r++) {
            const int e = tile + r * GPM_THREADS + tid;
            const int ee = e < out_len ? e : 0;
            const int p = ee >> log2N, ii = ee & (N - 1);
            if (a.extract && ee < k * N) {
                // extract_lwe_sample_from_glwe_ciphertext (degree 0): mask_p[0] = a_p[0],
                // mask_p[i] = -a_p[N - i] (glwe_sample_extraction.rs)
                src_off[r] = p * N;
                m[r] = ii == 0 ? 0 : N - ii;
                neg_out[r] = ii != 0;
            } else {
                src_off[r] = p * N;
                m[r] = a.extract ? 0 : ii;
                neg_out[r] = false;
            }
        }
        uint64_t acc[GPM_R];
#pragma unroll
        for (int r = 0; r < GPM_R; r++) acc[r] = 0;

        for (size_t w0 = 0; w0 < total; w0 += GPM_CH) {
            if (tid == 0) nz_count = 0;
            __syncthreads();
            for (int q = tid; q < GPM_CH && w0 + q < total; q += GPM_THREADS) {
                const uint64_t v = poly[w0 + q];
                if (v) {
                    const int slot = atomicAdd(&nz_count, 1);
                    nz_pos[slot] = (uint32_t)(w0 + q);
                    nz_val[slot] = v;
                }
            }
            __syncthreads();
            const int nnz = nz_count;
            for (int z = 0; z < nnz; z++) {
                const uint32_t pos = nz_pos[z];
                const uint64_t v = nz_val[z];
                const int j = (int)(pos >> log2N), t = (int)(pos & (uint32_t)(N - 1));
                const uint64_t *src = in + (size_t)j * glwe;
#pragma unroll
                for (int r = 0; r < GPM_R; r++) {
                    // coefficient m of (a * v X^t): a[m - t], negated when it wraps past X^N
                    int idx = m[r] - t;
                    const bool wrap = idx < 0;
                    idx += wrap ? N : 0;
                    const uint64_t prod = v * src[src_off[r] + idx];
                    acc[r] += wrap ? (0 - prod) : prod;
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < GPM_R; r++) {
            const int e = tile + r * GPM_THREADS + tid;
            if (e < out_len) out[e] = neg_out[r] ? (0 - acc[r]) : acc[r];
        }
    }
}

hipError_t launch_glwe_poly_mul(const GlwePolyMulLaunch &a, hipStream_t s) {
    if (a.count == 0 || a.npoly == 0) return hipSuccess;
    if (a.N < 64 || (a.N & (a.N - 1)) || a.k < 1 || a.J < 1 || (size_t)a.J * a.N > 0xffffffffull)
        return hipErrorInvalidValue;
    const size_t items = a.count * (size_t)a.npoly;
    if (items > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(glwe_poly_mul_kernel, dim3((unsigned)items), dim3(GPM_THREADS), 0, s, a);
    return hipGetLastError();
}

}  // namespace tfhe_mi355
