// Per-launch cost of a kernel that exits at once, replayed in a hipGraph
// (development probe): 200 launches of grid G x 256 lanes per graph, for a
// few G; prints us per launch.  hipcc --offload-arch=gfx950 -O3 -o /tmp/lp tools/launch_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void idle_kernel(const int* flag) {
    if (*flag != 1) return;
}

int main() {
    int* flag;
    (void)hipMalloc(&flag, 4);
    (void)hipMemset(flag, 0, 4);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    const int grids[] = {1, 8, 64, 256, 512, 2048};
    for (int g : grids) {
        hipGraph_t gr;
        hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int k = 0; k < 200; ++k) idle_kernel<<<g, 256, 0, s>>>(flag);
        (void)hipStreamEndCapture(s, &gr);
        (void)hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
        for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, s);
        (void)hipStreamSynchronize(s);
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < 10; ++r) (void)hipGraphLaunch(ge, s);
        (void)hipStreamSynchronize(s);
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        printf("grid %5d: %.2f us per launch\n", g, us / 2000.0);
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(gr);
    }
    return 0;
}
