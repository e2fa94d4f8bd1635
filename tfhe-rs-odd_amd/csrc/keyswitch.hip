// keyswitch.hip -- batched LWE keyswitch on gfx950 (u64 wrapping integer arithmetic).
//
// Replaces keyswitch_lwe_ciphertext (tfhe/src/core_crypto/algorithms/lwe_keyswitch.rs:96-170)
// with the signed decomposer (commons/math/decomposition/decomposer.rs:99-153, iter.rs:134-141)
// and slice_wrapping_sub_scalar_mul_assign (algorithms/slice_algorithms.rs:363).
//
// Shape: out[c][j] = (j == body ? in[c][in_dim] : 0) - sum_{i,l} d[c][i][l] * KSK[i][l][j]
// (body = out_dim for an LWE output; k*N for the LWE -> GLWE packing keyswitch,
// lwe_packing_keyswitch.rs:102-186, whose rows are (k+1)N-word GLWEs)
// i.e. a [count x in_dim*L] x [in_dim*L x (out_dim+1)] product over Z/2^64 with tiny signed
// digits.  A workgroup owns a 64-ciphertext x 64-column tile; every KSK row segment it loads
// (512 B, coalesced) is reused by its 64 ciphertexts, the digits are staged in LDS per chunk
// of input coefficients and broadcast to the wave.
#include <cstdlib>

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
        uint64_t body = (j == a.body()) ? a.lwe_in[(size_t)c * in_stride + in_dim] : 0;
        a.lwe_out[(size_t)c * out_stride + j] = body + acc[t];
    }
}

// ---------------------------------------------------------------------------------------
// Keyswitch as int8 MFMA GEMMs.  With D[c][m] the signed digits (|d| <= 2^(beta-1) <= 64) and
// the KSK split into byte planes K[m][j] = sum_b 2^(8b) K_b[m][j], K_b in [0, 256):
//   sum_m D K = sum_b 2^(8b) (D (K_b - 128) + 128 rowsum(D))          (mod 2^64)
// so each plane is an exact int8 x int8 -> int32 product (v_mfma_i32_32x32x32_i8; |partial| <
// M 2^(beta-1) 128 < 2^31 is checked), and the u64 result is recombined in the epilogue.
// KSK planes are repacked once at upload: Kt[b][j][m] = (int8)(byte_b(K[m][j]) - 128), column-
// major so a lane's 16 consecutive k of one column are one 16-B load.  Layout of the MFMA
// operands (probed on gfx950, scripts/probes/mfma_i8_probe.hip): lane l, r = l & 31, h = l >> 5
// holds A[r][16h + j] and B[16h + j][r] (j = 0..15); C/D col = r, row = (reg&3) + 8(reg>>2) + 4h.
// ---------------------------------------------------------------------------------------
typedef int ks_v4i __attribute__((ext_vector_type(4)));
typedef int ks_v16i __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256) ksk_repack_kernel(const uint64_t *__restrict__ ksk, int8_t *__restrict__ kt,
                                                         size_t rows, size_t cols, size_t mpad, size_t jpad) {
    const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= rows * cols) return;
    const size_t m = e / cols, j = e % cols;
    const uint64_t v = ksk[e];
#pragma unroll
    for (int b = 0; b < 8; b++) kt[((size_t)b * jpad + j) * mpad + m] = (int8_t)(uint8_t)(((v >> (8 * b)) & 0xff) ^ 0x80);
}

// KS_DPARTS workgroups per ciphertext: digits D[c][i*L + l] (levels L..1 as the KSK rows) of an
// eighth of the inputs each, and that part's digit sum (rowsum[c][part]: the GEMM adds the parts,
// so no reduction across workgroups and no zeroing is needed)
constexpr int KS_DPARTS = 8;
__global__ void __launch_bounds__(256) ks_digits_kernel(KeyswitchLaunch a, int8_t *__restrict__ dig,
                                                        int *__restrict__ rowsum, size_t mpad, int zero_out) {
    __shared__ int red[256];
    const int c = blockIdx.x / KS_DPARTS, part = blockIdx.x % KS_DPARTS;
    if (zero_out && part == 0) {  // split-K: the GEMM's workgroups add their partial products into a zeroed row
        uint64_t *o = a.lwe_out + (size_t)c * ((size_t)a.out_dim + 1);
        for (int j = threadIdx.x; j <= a.out_dim; j += 256) o[j] = 0;
    }
    const int in_dim = a.in_dim, L = a.level, beta = a.base_log;
    const uint64_t mask = (1ULL << beta) - 1;
    const uint64_t *x = a.lwe_in + (size_t)c * (in_dim + 1);
    int8_t *d = dig + (size_t)c * mpad;
    const int per = (in_dim + KS_DPARTS - 1) / KS_DPARTS, i0 = part * per, i1 = min(in_dim, i0 + per);
    int sum = 0;
    for (int i = i0 + threadIdx.x; i < i1; i += 256) {
        uint64_t state = closest_repr(x[i], beta, L) >> (64 - beta * L);
        for (int l = 0; l < L; l++) {
            uint64_t res = state & mask;
            state >>= beta;
            uint64_t carry = ((res - 1) | state) & res;
            carry >>= beta - 1;
            state += carry;
            const int v = (int)(int64_t)(res - (carry << beta));
            d[(size_t)i * L + l] = (int8_t)v;
            sum += v;
        }
    }
    if (part == KS_DPARTS - 1)
        for (size_t m = (size_t)in_dim * L + threadIdx.x; m < mpad; m += 256) d[m] = 0;
    red[threadIdx.x] = sum;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) rowsum[(size_t)c * KS_DPARTS + part] = red[0];
}

// workgroup tile: 64 ciphertexts x 64 output columns, 4 waves of 32 x 32, 8 byte planes each
__global__ void __launch_bounds__(256) ks_mfma_kernel(KeyswitchLaunch a, const int8_t *__restrict__ dig,
                                                      const int *__restrict__ rowsum,
                                                      const int8_t *__restrict__ kt, size_t mpad, size_t jpad,
                                                      int cpad) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int c0 = blockIdx.y * 64 + 32 * (wave >> 1);
    const int j0 = blockIdx.x * 64 + 32 * (wave & 1);
    const int8_t *pa = dig + (size_t)(c0 + r) * mpad + 16 * h;
    const int8_t *pb = kt + (size_t)(j0 + r) * mpad + 16 * h;
    const size_t plane = jpad * mpad;
    ks_v16i acc[8];
#pragma unroll
    for (int b = 0; b < 8; b++)
#pragma unroll
        for (int q = 0; q < 16; q++) acc[b][q] = 0;
    // split K (gridDim.z > 1, small batches): slice z of the rows, the partial products combined by
    // 64-bit atomic adds into an output zeroed beforehand (sums mod 2^64: order-independent, exact)
    // whole 32-row steps spread evenly (slices differ by at most one step: the critical path is the
    // longest slice)
    const size_t steps = mpad / 32;
    const size_t kbeg = 32 * (steps * blockIdx.z / gridDim.z), kend = 32 * (steps * (blockIdx.z + 1) / gridDim.z);
    // digit rows past the batch (the tile's padding) read as zero: no memset of the scratch
    const bool arow = c0 + r < a.count;
    for (size_t k = kbeg; k < kend; k += 32) {
        const ks_v4i av = arow ? *reinterpret_cast<const ks_v4i *>(pa + k) : ks_v4i{0, 0, 0, 0};
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const ks_v4i bv = *reinterpret_cast<const ks_v4i *>(pb + (size_t)b * plane + k);
            acc[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc[b], 0, 0, 0);
        }
    }
    const int j = j0 + r;
    if (j > a.out_dim) return;
    const size_t in_stride = (size_t)a.in_dim + 1, out_stride = (size_t)a.out_dim + 1;
    // sum_b 2^(8b) * 128 = 128 * 0x0101010101010101 (mod 2^64)
    constexpr uint64_t kOffset = 0x8080808080808080ULL;
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int c = c0 + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (c >= a.count) continue;
        const bool first = blockIdx.z == 0;
        int rs = 0;
        if (first)
#pragma unroll
            for (int p = 0; p < KS_DPARTS; p++) rs += rowsum[(size_t)c * KS_DPARTS + p];
        uint64_t v = (uint64_t)(int64_t)rs * kOffset;
#pragma unroll
        for (int b = 0; b < 8; b++) v += (uint64_t)(int64_t)acc[b][q] << (8 * b);
        const uint64_t body = (first && j == a.body()) ? a.lwe_in[(size_t)c * in_stride + a.in_dim] : 0;
        uint64_t *o = a.lwe_out + (size_t)c * out_stride + j;
        if (gridDim.z == 1) *o = body - v;
        else atomicAdd(reinterpret_cast<unsigned long long *>(o), (unsigned long long)(body - v));
    }
    (void)cpad;
}

size_t ks_mfma_rows(int in_dim, int level) { return ((size_t)in_dim * level + 31) / 32 * 32; }
size_t ks_mfma_cols(int out_dim) { return ((size_t)out_dim + 1 + 63) / 64 * 64; }

bool ks_mfma_supported(int in_dim, int level, int base_log) {
    // |partial| <= M * 2^(beta-1) * 128 must stay below 2^31
    return base_log <= 7 && (double)ks_mfma_rows(in_dim, level) * (double)(1 << (base_log - 1)) * 128.0 < 2147483648.0;
}

size_t ks_mfma_scratch_bytes(int in_dim, int level, int count) {
    const size_t cp = ((size_t)count + 63) / 64 * 64;
    return cp * ks_mfma_rows(in_dim, level) + cp * KS_DPARTS * sizeof(int) + 256;
}

hipError_t launch_ksk_repack(const uint64_t *ksk, int8_t *kt, int in_dim, int level, int out_dim, hipStream_t s) {
    const size_t rows = (size_t)in_dim * level, cols = (size_t)out_dim + 1;
    const size_t mpad = ks_mfma_rows(in_dim, level), jpad = ks_mfma_cols(out_dim);
    hipError_t e = hipMemsetAsync(kt, 0, 8 * mpad * jpad, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ksk_repack_kernel, dim3((unsigned)((rows * cols + 255) / 256)), dim3(256), 0, s, ksk, kt, rows,
                       cols, mpad, jpad);
    return hipGetLastError();
}

hipError_t launch_keyswitch_mfma(const KeyswitchLaunch &a, const int8_t *kt, void *scratch, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    if (!ks_mfma_supported(a.in_dim, a.level, a.base_log)) return hipErrorInvalidValue;
    const size_t mpad = ks_mfma_rows(a.in_dim, a.level), jpad = ks_mfma_cols(a.out_dim);
    const int cpad = (a.count + 63) / 64 * 64;
    int8_t *dig = reinterpret_cast<int8_t *>(scratch);
    int *rowsum = reinterpret_cast<int *>(reinterpret_cast<char *>(scratch) + (((size_t)cpad * mpad + 255) / 256) * 256);
    // few output tiles (small batches: 12 at 2_2 for up to 64 ciphertexts, each streaming 5 MiB of
    // KSK planes through one CU, latency-bound at one k-step per load round trip): split K over up
    // to ~1024 workgroups (4 per CU; more slices cost more in atomics on the same words than they
    // gain), >= 2 k-steps each; ks_digits_kernel zeroes the output rows
    // that the slices' 64-bit atomics accumulate into
    const unsigned tiles = (unsigned)(jpad / 64) * (unsigned)(cpad / 64);
    unsigned split = 1;
    static const unsigned target = [] {  // TFHE_MI355_KS_SPLIT_WG: workgroups aimed at (A/B)
        const char *e = std::getenv("TFHE_MI355_KS_SPLIT_WG");
        const long v = e ? std::atol(e) : 0;
        return v > 0 ? (unsigned)v : 1024u;
    }();
    // (mpad is a multiple of 32: mpad / 64 slices keep >= 2 k-steps each)
    if (tiles < 128) split = (unsigned)std::min<size_t>((target + tiles - 1) / tiles, mpad / 64);
    if (split < 2) split = 1;
    hipLaunchKernelGGL(ks_digits_kernel, dim3((unsigned)a.count * KS_DPARTS), dim3(256), 0, s, a, dig, rowsum, mpad,
                       split > 1 ? 1 : 0);
    hipLaunchKernelGGL(ks_mfma_kernel, dim3((unsigned)(jpad / 64), (unsigned)(cpad / 64), split), dim3(256), 0, s, a,
                       dig, rowsum, kt, mpad, jpad, cpad);
    return hipGetLastError();
}

hipError_t launch_keyswitch(const KeyswitchLaunch &a, hipStream_t s) {
    if (a.count == 0) return hipSuccess;
    if (a.level > KS_MAXL || a.base_log * a.level >= 64 || a.base_log > 7) return hipErrorInvalidValue;
    dim3 grid((a.out_dim + 1 + KS_TJ - 1) / KS_TJ, (a.count + KS_TC - 1) / KS_TC);
    hipLaunchKernelGGL(keyswitch_kernel, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace tfhe_mi355
