// Development microbenchmark: sustained fp64 / fp32 VALU FMA rate on the
// whole chip (independent chains, full occupancy) -- the practical ceiling
// the particle-filter fused kernel is compared with.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <typename T, int CH>
__global__ __launch_bounds__(256) void fma_kernel(T* out, int iters, T a, T b) {
    T acc[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = (T)(threadIdx.x + k);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < CH; ++k) acc[k] = fma(acc[k], a, b);
    }
    T s = 0;
#pragma unroll
    for (int k = 0; k < CH; ++k) s += acc[k];
    if (s == (T)12345.678) out[blockIdx.x] = s;
}

template <typename T, int CH>
void run(const char* name, int blocks) {
    T* out;
    hipMalloc(&out, sizeof(T) * blocks);
    const int iters = 4096;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    fma_kernel<T, CH><<<blocks, 256>>>(out, iters, (T)0.999, (T)0.001);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) fma_kernel<T, CH><<<blocks, 256>>>(out, iters, (T)0.999, (T)0.001);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * CH * (double)iters * blocks * 256 * 5;
    const double winst = (double)CH * iters * blocks * 4 * 5;   // wave-instructions
    printf("%s chains=%d blocks=%d: %.2f TFLOP/s, %.3f wave-FMA/clk/SIMD at 2.4 GHz\n", name, CH, blocks,
           flops / (ms * 1e-3) / 1e12, winst / (ms * 1e-3) / 2.4e9 / 1024);
    hipFree(out);
}

int main() {
    run<double, 4>("f64", 2048);
    run<double, 8>("f64", 2048);
    run<double, 8>("f64", 8192);
    run<float, 8>("f32", 2048);
    run<float, 8>("f32", 8192);
    return 0;
}
