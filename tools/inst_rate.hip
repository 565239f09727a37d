// Development microbenchmark: issue cost of single VALU instructions on gfx950
// (cycles per wave-instruction per SIMD, 8 independent chains per lane,
// 8 waves per SIMD), relative to v_fma_f64.  Guides the fused PF kernel's
// instruction choices (RNG integer multiplies, fp64 transcendentals).
//   hipcc --offload-arch=gfx950 -O3 -o tools/inst_rate tools/inst_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CH 8
#define ITERS 2048

#define K64(NAME, ASM)                                                                 \
    __global__ __launch_bounds__(256) void k_##NAME(double* out, double a, double b) {   \
        double acc[CH];                                                                \
        for (int k = 0; k < CH; ++k) acc[k] = (double)(threadIdx.x + k) * 1e-3 + 1.0;   \
        for (int i = 0; i < ITERS; ++i) {                                              \
            _Pragma("unroll") for (int k = 0; k < CH; ++k) asm volatile(ASM : "+v"(acc[k]) : "v"(a), "v"(b)); \
        }                                                                              \
        double s = 0;                                                                  \
        for (int k = 0; k < CH; ++k) s += acc[k];                                      \
        if (s == 12345.678) out[blockIdx.x] = s;                                       \
    }
#define K32(NAME, ASM)                                                                 \
    __global__ __launch_bounds__(256) void k_##NAME(double* out, double a, double b) {   \
        uint32_t acc[CH];                                                              \
        uint32_t x = (uint32_t)(a * 1000.0) | 1u, y = (uint32_t)(b * 1000.0) | 3u;      \
        for (int k = 0; k < CH; ++k) acc[k] = threadIdx.x * 2654435761u + k;            \
        for (int i = 0; i < ITERS; ++i) {                                              \
            _Pragma("unroll") for (int k = 0; k < CH; ++k) asm volatile(ASM : "+v"(acc[k]) : "v"(x), "v"(y)); \
        }                                                                              \
        uint32_t s = 0;                                                                \
        for (int k = 0; k < CH; ++k) s ^= acc[k];                                      \
        if (s == 12345u) out[blockIdx.x] = s;                                          \
    }

K64(fma_f64, "v_fma_f64 %0, %0, %1, %2")
K64(add_f64, "v_add_f64 %0, %0, %1")
K64(mul_f64, "v_mul_f64 %0, %0, %1")
K64(rcp_f64, "v_rcp_f64 %0, %0")
K64(rsq_f64, "v_rsq_f64 %0, %0")
K64(sqrt_f64, "v_sqrt_f64 %0, %0")
K64(ldexp_f64, "v_ldexp_f64 %0, %0, 1")
K64(frexp_mant_f64, "v_frexp_mant_f64 %0, %0")
K64(rndne_f64, "v_rndne_f64 %0, %0")
K64(max_f64, "v_max_f64 %0, %0, %1")
K32(mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
K32(mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
K32(xor_b32, "v_xor_b32 %0, %0, %1")

K32(add_u32, "v_add_u32 %0, %0, %1")
K32(alignbit_b32, "v_alignbit_b32 %0, %0, %0, 13")
K32(fma_f32, "v_fma_f32 %0, %0, %1, %2")
K32(log_f32, "v_log_f32 %0, %0")
K32(cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
K32(mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
K32(mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %0, %1")
K32(cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
K32(sin_f32, "v_sin_f32 %0, %0")
K32(exp_f32, "v_exp_f32 %0, %0")
K32(sqrt_f32, "v_sqrt_f32 %0, %0")
K32(mul_f32, "v_mul_f32 %0, %0, %1")
K64(fract_f64, "v_fract_f64 %0, %0")

// v_mad_u64_u32 needs a 64-bit destination: 4 chains of 64-bit state
__global__ __launch_bounds__(256) void k_mad_u64_u32(double* out, double a, double b) {
    uint64_t acc[CH];
    uint32_t x = (uint32_t)(a * 1000.0) | 1u;
    for (int k = 0; k < CH; ++k) acc[k] = threadIdx.x * 2654435761ull + k;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            uint64_t cc;
            asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cc) : "v"((uint32_t)acc[k]), "v"(x));
        }
    }
    uint64_t s = 0;
    for (int k = 0; k < CH; ++k) s ^= acc[k];
    if (s == 12345u) out[blockIdx.x] = (double)s;
}

typedef void (*kfn)(double*, double, double);

static void run(const char* name, kfn f, double ref_ms) {
    double* out;
    hipMalloc(&out, sizeof(double) * 8192);
    const int blocks = 8192;   // 8 waves per SIMD at 256 CUs
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, 0.999, 0.001);
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, 0.999, 0.001);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 3;
    const double winst = (double)CH * ITERS * blocks * 4;   // wave-instructions
    const double cyc = (ms * 1e-3) * 2.4e9 * 1024 / winst;  // per SIMD at nominal clock
    printf("%-16s %8.3f ms  %6.2f cyc/wave-inst @2.4GHz  %5.2fx fma_f64\n", name, ms, cyc,
           ref_ms > 0 ? ms / ref_ms : 1.0);
    hipFree(out);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    double* out;
    hipMalloc(&out, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_fma_f64, dim3(8192), dim3(256), 0, 0, out, 0.999, 0.001);
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_fma_f64, dim3(8192), dim3(256), 0, 0, out, 0.999, 0.001);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ref;
    hipEventElapsedTime(&ref, e0, e1);
    ref /= 3;
#define R(n) run(#n, k_##n, ref)
    R(fma_f64); R(add_f64); R(mul_f64); R(rcp_f64); R(rsq_f64); R(sqrt_f64); R(ldexp_f64);
    R(frexp_mant_f64); R(rndne_f64); R(max_f64); R(mul_lo_u32); R(mul_hi_u32); R(mad_u64_u32);
    R(xor_b32); R(add_u32); R(alignbit_b32); R(fma_f32); R(log_f32); R(cvt_f32_u32);
    R(mul_u32_u24); R(mul_hi_u32_u24); R(cndmask); R(sin_f32); R(exp_f32); R(sqrt_f32);
    R(mul_f32); R(fract_f64);
    return 0;
}
