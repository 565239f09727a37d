// Development probe: do independent branches of a captured hipGraph run
// concurrently on gfx950?  Kernel A is one workgroup that spins ~40 us (like
// the PF step end); kernel B is a full-chip ALU kernel of similar length (like
// the next step's noise draw).  Times: A alone, B alone, A then B on one
// stream, A || B on two streams (fork / join by events), and the same fork /
// join captured into a graph and replayed.
//   hipcc --offload-arch=gfx950 -O3 -o tools/graph_concurrency tools/graph_concurrency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void spin_one(long long cycles, int* out) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0) out[0] = 1;
}

__global__ __launch_bounds__(256) void busy_many(int iters, double* out) {
    double a = threadIdx.x * 1e-3 + 1.0, b = 0.999;
    for (int i = 0; i < iters; ++i) a = fma(a, b, 1e-7);
    if (a == 12345.0) out[blockIdx.x] = a;
}

int main() {
    int* flag;
    double* out;
    CK(hipMalloc(&flag, 64));
    CK(hipMalloc(&out, 8192 * sizeof(double)));
    int clk_khz = 100000;
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0);
    const long long spin = (long long)(40e-6 * clk_khz * 1e3);   // 40 us of wall clock
    const int iters = 6000;
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e0, e1, f1, f2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreateWithFlags(&f1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&f2, hipEventDisableTiming));
    auto A = [&](hipStream_t st) { hipLaunchKernelGGL(spin_one, dim3(1), dim3(64), 0, st, spin, flag); };
    auto B = [&](hipStream_t st) { hipLaunchKernelGGL(busy_many, dim3(4096), dim3(256), 0, st, iters, out); };
    auto fork = [&]() {
        A(s);
        CK(hipEventRecord(f1, s));   // fork point before A would be better; A first keeps block 0 early
        return 0;
    };
    (void)fork;
    auto time = [&](const char* name, auto body) {
        for (int w = 0; w < 3; ++w) body();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        const int reps = 20;
        for (int r = 0; r < reps; ++r) body();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-34s %8.1f us per rep\n", name, ms * 1e3 / reps);
        return 0;
    };
    time("A alone (1 WG spin)", [&]() { A(s); });
    time("B alone (4096 WG ALU)", [&]() { B(s); });
    time("A then B, one stream", [&]() { A(s); B(s); });
    auto forkjoin = [&]() {
        (void)hipEventRecord(f1, s);
        (void)hipStreamWaitEvent(s2, f1, 0);
        A(s);
        B(s2);
        (void)hipEventRecord(f2, s2);
        (void)hipStreamWaitEvent(s, f2, 0);
    };
    time("A || B, two streams", forkjoin);
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < 4; ++k) forkjoin();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    time("graph: 4 x (A || B), per A||B", [&]() { (void)hipGraphLaunch(ge, s); });
    printf("(graph line is per 4 fork/joins: divide by 4)\n");
    hipGraph_t g2;
    hipGraphExec_t ge2;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < 4; ++k) { A(s); B(s); }
    CK(hipStreamEndCapture(s, &g2));
    CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
    time("graph: 4 x (A then B)", [&]() { (void)hipGraphLaunch(ge2, s); });
    return 0;
}
