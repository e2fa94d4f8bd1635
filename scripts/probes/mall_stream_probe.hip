// Streaming rate of data that stays in the 256 MiB Infinity Cache (MALL) on MI355X: the ceiling
// for large_top_inv / large_digits, whose per-chunk working set (~192 MiB) is
// sized to stay resident.  Kernel: out[i] = in[i] + in2[i] over S bytes of input, S/2 output,
// repeated; reports read+write bytes / time.  hipcc --offload-arch=gfx950 -O3 -o mall_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void __launch_bounds__(256) stream_kernel(const ulonglong2 *__restrict__ a, const ulonglong2 *__restrict__ b,
                                                     ulonglong2 *__restrict__ o, size_t n, int unroll) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const ulonglong2 x = a[i], y = b[i];
        o[i] = make_ulonglong2(x.x + y.x, x.y + y.y);
    }
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? (size_t)atol(argv[1]) : 64;  // per array
    const size_t n = mib * (1u << 20) / 16;
    ulonglong2 *a, *b, *o;
    if (hipMalloc(&a, n * 16) || hipMalloc(&b, n * 16) || hipMalloc(&o, n * 16)) return 1;
    (void)hipMemset(a, 1, n * 16);
    (void)hipMemset(b, 2, n * 16);
    (void)hipMemset(o, 0, n * 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int blocks : {1024, 2048, 4096, 8192}) {
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(stream_kernel, dim3(blocks), dim3(256), 0, 0, a, b, o, n, 1);
        const int reps = 50;
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(stream_kernel, dim3(blocks), dim3(256), 0, 0, a, b, o, n, 1);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double bytes = 3.0 * n * 16 * reps;
        printf("arrays %zu MiB x3 (working set %zu MiB), blocks %d: %.2f TB/s (%.1f us per pass)\n", mib, 3 * mib, blocks,
               bytes / (ms * 1e-3) / 1e12, ms * 1e3 / reps);
    }
    return 0;
}
