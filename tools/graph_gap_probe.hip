// Probe: cost of a kernel node in a replayed hipGraph (empty kernels, a
// 1-block kernel, a 2048-block early-exit kernel), and of a plain stream launch.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void empty_k(int* f) { if (f[0] == 12345) f[1] = 1; }

int main() {
    int* f;
    hipMalloc(&f, 64);
    hipMemset(f, 0, 64);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int grid : {1, 256, 2048}) {
        for (int nodes : {1, 4, 16}) {
            hipGraph_t g;
            hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
            for (int k = 0; k < nodes; ++k) empty_k<<<grid, 256, 0, s>>>(f);
            hipStreamEndCapture(s, &g);
            hipGraphExec_t ge;
            hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            for (int w = 0; w < 20; ++w) hipGraphLaunch(ge, s);
            hipStreamSynchronize(s);
            const int reps = 200;
            auto t0 = std::chrono::steady_clock::now();
            for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, s);
            hipStreamSynchronize(s);
            double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
            printf("graph grid %5d nodes %2d: %7.2f us per replay, %6.2f us per node\n", grid, nodes, us, us / nodes);
            hipGraphExecDestroy(ge);
            hipGraphDestroy(g);
        }
        const int reps = 400;
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) empty_k<<<grid, 256, 0, s>>>(f);
        hipStreamSynchronize(s);
        double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
        printf("stream grid %5d: %6.2f us per launch\n", grid, us);
    }
    return 0;
}
