// Development microbenchmark: fp64 VALU vs fp64 MFMA (v_mfma_f64_16x16x4_f64)
// rates on gfx950 and whether the two pipes overlap -- (a) across the waves of
// one SIMD (split roles) and (b) inside one wave (MFMA + VALU interleaved).
// Decides whether the particle-filter residuals (a K = 4 affine map per
// particle-landmark pair) are worth moving onto the matrix cores.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int CH>
__device__ __forceinline__ void valu_body(double* acc, double a, double b) {
#pragma unroll
    for (int k = 0; k < CH; ++k) acc[k] = fma(acc[k], a, b);
}

__device__ __forceinline__ void mfma_body(d4* c, double a, double b) {
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
}

// mode 0: VALU only (8 chains); 1: MFMA only (4 accumulators);
// 2: odd waves MFMA, even waves VALU (split roles, 2 waves per SIMD at 512 threads);
// 3: every wave: per iteration 4 MFMA + M VALU fma (interleaved in one wave)
template <int MODE, int M>
__global__ __launch_bounds__(512) void probe(double* out, int iters, double a, double b) {
    double acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = (double)(threadIdx.x + k);
    d4 c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = d4{acc[k], acc[k + 1], acc[k + 2], acc[k + 3]};
    const int wave = threadIdx.x >> 6;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
            valu_body<8>(acc, a, b);
        } else if (MODE == 1) {
            mfma_body(c, a, b);
        } else if (MODE == 2) {
            if (wave & 1) mfma_body(c, a, b);
            else {
                valu_body<8>(acc, a, b);
                valu_body<8>(acc, a, b);
            }
        } else {
            mfma_body(c, a, b);
            valu_body<M>(acc, a, b);
        }
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += acc[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) s += c[k].x + c[k].y + c[k].z + c[k].w;
    if (s == 12345.678) out[blockIdx.x] = s;
}

template <int MODE, int M>
void run(const char* name, int blocks, int iters) {
    double* out;
    hipMalloc(&out, sizeof(double) * blocks);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    probe<MODE, M><<<blocks, 512>>>(out, iters, 0.999, 0.001);
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) probe<MODE, M><<<blocks, 512>>>(out, iters, 0.999, 0.001);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double s = ms * 1e-3 / reps;
    // per SIMD: blocks * 8 waves / (256 CU * 4 SIMD) waves, each iters iterations
    const double waves_per_simd = (double)blocks * 8 / 1024.0;
    const double cyc = s * 2.4e9 / (waves_per_simd * iters);   // cycles per wave-iteration per SIMD (at 2.4 GHz)
    printf("%-34s blocks=%5d iters=%d: %.3f ms, %.1f cyc (2.4 GHz) per wave-iteration per SIMD\n", name, blocks,
           iters, s * 1e3, cyc);
    hipFree(out);
}

int main() {
    const int it = 2048;
    run<0, 0>("valu 8 fma", 1024, it);
    run<0, 0>("valu 8 fma", 2048, it);
    run<1, 0>("mfma 4x16x16x4f64", 1024, it);
    run<1, 0>("mfma 4x16x16x4f64", 2048, it);
    run<2, 0>("split: mfma(4) | valu(16)", 1024, it);
    run<2, 0>("split: mfma(4) | valu(16)", 2048, it);
    run<3, 4>("same wave: mfma(4)+valu(4)", 1024, it);
    run<3, 8>("same wave: mfma(4)+valu(8)", 1024, it);
    run<3, 16>("same wave: mfma(4)+valu(16)", 1024, it);
    run<3, 16>("same wave: mfma(4)+valu(16)", 2048, it);
    return 0;
}
