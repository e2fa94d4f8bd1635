// keyswitch.hip -- batched LWE keyswitch on gfx950 (u64 wrapping integer arithmetic).
//
// Replaces keyswitch_lwe_ciphertext (tfhe/src/core_crypto/algorithms/lwe_keyswitch.rs:96-170)
// with the signed decomposer (commons/math/decomposition/decomposer.rs:99-153, iter.rs:134-141)
// and slice_wrapping_sub_scalar_mul_assign (algorithms/slice_algorithms.rs:363).
//
// Shape: out[c][j] = (j == out_dim ? in[c][in_dim] : 0) - sum_{i,l} d[c][i][l] * KSK[i][l][j]
// i.e. a [count x in_dim*L] x [in_dim*L x (out_dim+1)] product over Z/2^64 with tiny signed
// digits.  A workgroup owns a 64-ciphertext x 64-column tile; every KSK row segment it loads
// (512 B, coalesced) is reused by its 64 ciphertexts, the digits are staged in LDS per chunk
// of input coefficients and broadcast to the wave.
#include "engine.h"

namespace tfhe_mi355 {

namespace {
constexpr int KS_TJ = 64;     // output columns per workgroup
constexpr int KS_TC = 64;     // ciphertexts per workgroup
constexpr int KS_CPT = 16;    // ciphertexts per thread
constexpr int KS_IC = 8;      // input coefficients per LDS chunk
constexpr int KS_MAXL = 16;   // max decomposition levels

__device__ __forceinline__ uint64_t closest_repr(uint64_t x, int base_log, int level) {
    int shift = 64 - base_log * level - 1;
    uint64_t res = x >> shift;
    res += 1;
    res &= ~(uint64_t)1;
    return res << shift;
}
}  // namespace

__global__ void __launch_bounds__(256) keyswitch_kernel(KeyswitchLaunch a) {
    __shared__ int8_t dig[KS_IC][KS_MAXL][KS_TC];
    const int tid = threadIdx.x;
    const int tj = tid & 63, tg = tid >> 6;
    const int j = blockIdx.x * KS_TJ + tj;
    const int c0 = blockIdx.y * KS_TC;
    const int in_dim = a.in_dim, out_dim = a.out_dim, L = a.level, beta = a.base_log;
    const uint64_t mask = (1ULL << beta) - 1;
    const size_t in_stride = (size_t)in_dim + 1, out_stride = (size_t)out_dim + 1;
    const bool jok = j <= out_dim;

    uint64_t acc[KS_CPT];
#pragma unroll
    for (int t = 0; t < KS_CPT; t++) acc[t] = 0;

    for (int i0 = 0; i0 < in_dim; i0 += KS_IC) {
        __syncthreads();
        // decompose KS_IC coefficients of KS_TC ciphertexts: 512 (ct, i) pairs, 2 per thread
        for (int q = tid; q < KS_IC * KS_TC; q += 256) {
            const int ci = q % KS_TC, ii = q / KS_TC;
            const int c = c0 + ci, i = i0 + ii;
            uint64_t state = 0;
            if (c < a.count && i < in_dim)
                state = closest_repr(a.lwe_in[(size_t)c * in_stride + i], beta, L) >> (64 - beta * L);
            for (int l = 0; l < L; l++) {
                uint64_t res = state & mask;
                state >>= beta;
                uint64_t carry = ((res - 1) | state) & res;
                carry >>= beta - 1;
                state += carry;
                dig[ii][l][ci] = (int8_t)(int64_t)(res - (carry << beta));
            }
        }
        __syncthreads();
        const int ni = min(KS_IC, in_dim - i0);
        for (int ii = 0; ii < ni; ii++) {
            for (int l = 0; l < L; l++) {
                const uint64_t k = jok ? a.ksk[((size_t)(i0 + ii) * L + l) * out_stride + j] : 0;
#pragma unroll
                for (int t = 0; t < KS_CPT; t++) {
                    const int64_t d = dig[ii][l][tg * KS_CPT + t];
                    acc[t] -= (uint64_t)(d * (int64_t)k);
                }
            }
        }
    }
    if (!jok) return;
#pragma unroll
    for (int t = 0; t < KS_CPT; t++) {
        const int c = c0 + tg * KS_CPT + t;
        if (c >= a.count) break;
        uint64_t body = (j == out_dim) ? a.lwe_in[(size_t)c * in_stride + in_dim] : 0;
        a.lwe_out[(size_t)c * out_stride + j] = body + acc[t];
    }
}

hipError_t launch_keyswitch(const KeyswitchLaunch &a, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    if (a.level > KS_MAXL || a.base_log * a.level >= 64 || a.base_log > 7) return hipErrorInvalidValue;
    dim3 grid((a.out_dim + 1 + KS_TJ - 1) / KS_TJ, (a.count + KS_TC - 1) / KS_TC);
    hipLaunchKernelGGL(keyswitch_kernel, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace tfhe_mi355
