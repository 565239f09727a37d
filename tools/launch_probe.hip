// Per-launch cost of a kernel that exits at once, replayed in a hipGraph
// (development probe): 200 launches of grid G x 256 lanes per graph, for a
// few G; prints us per launch.  hipcc --offload-arch=gfx950 -O3 -o /tmp/lp tools/launch_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void idle_kernel(const int* flag) {
    if (*flag != 1) return;
}

// the same early exit in a kernel with the exact-cumsum launch's footprint
// (static LDS, many VGPRs): does the dispatch of big waves cost more?
__global__ __launch_bounds__(256) void idle_heavy_kernel(const int* flag, double* out) {
    __shared__ double sh[4096];
    if (*flag != 1) return;
    double v[96];
#pragma unroll
    for (int k = 0; k < 96; ++k) v[k] = out[threadIdx.x + 256 * k];
    sh[threadIdx.x] = v[0];
    __syncthreads();
    double a = sh[(threadIdx.x + 1) & 4095];
#pragma unroll
    for (int k = 0; k < 96; ++k) a = a * v[k] + v[(k + 7) % 96];
    out[threadIdx.x] = a;
}

int main() {
    int* flag;
    (void)hipMalloc(&flag, 4);
    (void)hipMemset(flag, 0, 4);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    double* buf;
    (void)hipMalloc(&buf, sizeof(double) * 256 * 96);
    const int grids[] = {1, 8, 64, 256, 512, 2048};
    for (int heavy = 0; heavy < 2; ++heavy)
    for (int g : grids) {
        hipGraph_t gr;
        hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int k = 0; k < 200; ++k) {
            if (heavy) idle_heavy_kernel<<<g, 256, 0, s>>>(flag, buf);
            else idle_kernel<<<g, 256, 0, s>>>(flag);
        }
        (void)hipStreamEndCapture(s, &gr);
        (void)hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
        for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, s);
        (void)hipStreamSynchronize(s);
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < 10; ++r) (void)hipGraphLaunch(ge, s);
        (void)hipStreamSynchronize(s);
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        printf("%s grid %5d: %.2f us per launch\n", heavy ? "heavy" : "light", g, us / 2000.0);
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(gr);
    }
    return 0;
}
