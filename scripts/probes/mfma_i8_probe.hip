// Probe of the gfx950 v_mfma_i32_32x32x32_i8 operand layout with exact integer data (asymmetric B).
// Assumed map: lane l, r = l & 31, h = l >> 5: A[r][16h + j], B[16h + j][r] for byte j = 0..15;
// C/D: col = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void probe(const int8_t *A, const int8_t *B, int *C) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; j++) {
        a[j] = A[r * 32 + 16 * h + j];
        b[j] = B[(16 * h + j) * 32 + r];
    }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v16i c = {0};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
    for (int reg = 0; reg < 16; reg++) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h, col = r;
        C[row * 32 + col] = c[reg];
    }
}

int main() {
    int8_t A[1024], B[1024];
    int ref[1024], C[1024];
    for (int i = 0; i < 32; i++)
        for (int k = 0; k < 32; k++) {
            A[i * 32 + k] = (int8_t)((i * 7 + k * 3) % 23 - 11);
            B[i * 32 + k] = (int8_t)((i * 5 + k * 11) % 19 - 9);  // B[k=i][col=k]
        }
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++) {
            int s = 0;
            for (int k = 0; k < 32; k++) s += A[i * 32 + k] * B[k * 32 + j];
            ref[i * 32 + j] = s;
        }
    int8_t *dA, *dB;
    int *dC;
    hipMalloc(&dA, 1024);
    hipMalloc(&dB, 1024);
    hipMalloc(&dC, 4096);
    hipMemcpy(dA, A, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(C, dC, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; i++) bad += C[i] != ref[i];
    printf("mfma_i32_32x32x32_i8 assumed layout: %d of 1024 wrong (C[0]=%d ref %d, C[33]=%d ref %d)\n", bad, C[0],
           ref[0], C[33], ref[33]);
    return bad != 0;
}
