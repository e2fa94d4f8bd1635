// lwe_ops.hip -- batched LWE linear algebra and trivial PBS on device, for the integer layer
// (tfhe_mi355/integer.py) keeping radix ciphertexts resident in HBM between PBS layers.
//
// Replaces, batched over rows of u64 words:
//   shortint unchecked_add_assign / unchecked_scalar_mul_assign
//       (core_crypto/algorithms/lwe_linear_algebra.rs: lwe_ciphertext_add_assign,
//        lwe_ciphertext_cleartext_mul_assign; shortint/server_key/add.rs, scalar_mul.rs)
//   the bivariate packing  left = left * factor + right  (shortint/server_key/bivariate_pbs.rs:167-182)
//   trivial_pbs_assign     (shortint/server_key/mod.rs:763-781)
// All arithmetic is wrapping mod 2^64, as the reference's.
#include "engine.h"
#include "fft_device.h"

namespace tfhe_mi355 {

// y[r][w] = y[r][w] * scalar + (x ? x[r][w] : 0)
__global__ void __launch_bounds__(256) lwe_scalar_mul_add_kernel(uint64_t *__restrict__ y, const uint64_t *__restrict__ x,
                                                                 uint64_t scalar, size_t rows, size_t words,
                                                                 size_t y_stride, size_t x_stride) {
    const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= rows * words) return;
    const size_t r = e / words, w = e % words;
    uint64_t v = y[r * y_stride + w] * scalar;
    if (x) v += x[r * x_stride + w];
    y[r * y_stride + w] = v;
}

// trivial ciphertexts (zero mask): body <- LUT body at the box of body / delta (negated past the
// padding bit); the mask stays zero
__global__ void __launch_bounds__(256) trivial_pbs_kernel(uint64_t *__restrict__ body, size_t rows, size_t stride,
                                                          const uint64_t *__restrict__ lut_body, uint64_t delta,
                                                          uint64_t modulus_sup, uint64_t box) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    const uint64_t value = body[r * stride] / delta;
    const uint64_t entry = lut_body[(value % modulus_sup) * box];
    body[r * stride] = value >= modulus_sup ? 0 - entry : entry;
}

// Diagnostic: the PBS kernels' backward torus conversion (fft_device.h frac_to_torus) applied to
// given fractions: acc[i] += X(fr[i]) and set[i] = X(fr[i]), X = rint(fr * 2^64) mod 2^64.
__global__ void __launch_bounds__(256) torus_from_fraction_kernel(const double *__restrict__ fr,
                                                                  uint64_t *__restrict__ acc,
                                                                  uint64_t *__restrict__ set, size_t n) {
    const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
    const double k32 = torus_k32();
    if (e >= n) return;
    uint64_t c = acc[e];
    torus_add_frac(c, fr[e], k32);
    acc[e] = c;
    set[e] = torus_from_frac(fr[e], k32);
}

hipError_t launch_torus_from_fraction(const double *fr, uint64_t *acc, uint64_t *set, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(torus_from_fraction_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, fr, acc, set, n);
    return hipGetLastError();
}

hipError_t launch_lwe_scalar_mul_add(uint64_t *y, const uint64_t *x, uint64_t scalar, size_t rows, size_t words,
                                     size_t y_stride, size_t x_stride, hipStream_t s) {
    const size_t n = rows * words;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(lwe_scalar_mul_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, y, x, scalar,
                       rows, words, y_stride, x_stride);
    return hipGetLastError();
}

hipError_t launch_trivial_pbs(uint64_t *body, size_t rows, size_t stride, const uint64_t *lut_body, uint64_t delta,
                              uint64_t modulus_sup, uint64_t box, hipStream_t s) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(trivial_pbs_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, body, rows, stride,
                       lut_body, delta, modulus_sup, box);
    return hipGetLastError();
}

}  // namespace tfhe_mi355
